"""Minimal GGUF v3 writer for tests (the repo's own code, independent of the reference's gguf-py): KV metadata
(u32 / i32 / f32 / string scalars, string / int32 arrays) and f32 / q8_0 tensors, 32-byte aligned data section.
Layout per gguf/constants.py:10-12 and gguf_reader.py:132-182 of the reference's vendored gguf-py."""
import struct

import numpy as np

GGML_F32, GGML_Q8_0 = 0, 8


def _s(b):
    b = b.encode("utf-8") if isinstance(b, str) else b
    return struct.pack("<Q", len(b)) + b


def _kv(key, val):
    out = _s(key)
    if isinstance(val, str):
        return out + struct.pack("<I", 8) + _s(val)
    if isinstance(val, float):
        return out + struct.pack("<If", 6, val)
    if isinstance(val, int):
        return out + struct.pack("<Ii", 5, val)
    if isinstance(val, list) and (not val or isinstance(val[0], str)):
        return out + struct.pack("<IIQ", 9, 8, len(val)) + b"".join(_s(v) for v in val)
    if isinstance(val, list):
        return out + struct.pack("<IIQ", 9, 5, len(val)) + struct.pack(f"<{len(val)}i", *val)
    raise TypeError(key)


def write_gguf(path, kv, tensors, arch="qwen3"):
    """tensors: list of (name, array f32 [rows, cols] or [n], type); q8_0 tensors given as (d f16, q int8) blocks."""
    from oracle import q8
    kv = dict({"general.architecture": arch, "general.alignment": 32}, **kv)
    infos, blobs, off = [], [], 0
    for name, arr, ty in tensors:
        a = np.asarray(arr, np.float32)
        dims = list(a.shape[::-1])  # ggml order: ne[0] = innermost
        if ty == GGML_Q8_0:
            d, q = q8.quantize_q8_0(a)
            blob = q8.pack_q8_0(d, q).tobytes()
        else:
            blob = a.tobytes()
        infos.append(_s(name) + struct.pack("<I", len(dims)) + struct.pack(f"<{len(dims)}Q", *dims) +
                     struct.pack("<IQ", ty, off))
        blobs.append(blob)
        off += (len(blob) + 31) // 32 * 32
    head = b"GGUF" + struct.pack("<IQQ", 3, len(tensors), len(kv))
    head += b"".join(_kv(k, v) for k, v in kv.items()) + b"".join(infos)
    head += b"\0" * ((32 - len(head) % 32) % 32)
    with open(path, "wb") as f:
        f.write(head)
        for b in blobs:
            f.write(b)
            f.write(b"\0" * ((32 - len(b) % 32) % 32))
