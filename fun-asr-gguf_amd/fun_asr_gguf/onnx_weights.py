"""Encoder / CTC weights from the reference's ONNX files (nano_onnx.load_onnx_models, /root/reference/fun_asr_gguf/
nano_onnx.py:21-46): Fun-ASR-Nano-Encoder-Adaptor.{fp32,fp16,int8}.onnx and Fun-ASR-Nano-CTC.{fp32,fp16,int8}.onnx as
exported by 01-Export-Encoder-Adaptor-CTC.py:107-135 (torch.onnx.export dynamo=True) and converted by
02-Quantize-ONNX.py:13-48.

The `onnx` package is absent, so the protobuf wire format is read directly: ModelProto.graph (field 7) ->
GraphProto.initializer (field 5, TensorProto: dims 1, data_type 2, float_data 4, int32_data 5, int64_data 7,
name 8, raw_data 9) and GraphProto.node (field 1, NodeProto: input 1, output 2, op_type 4, attribute 5) to tell
how each weight is consumed. Initializers map back to HybridSenseVoice state_dict names (model_definition.py):
the dynamo exporter names them by module path from the export wrapper (`hybrid_model.` prefix for the encoder
graph, EncoderExportWrapperPaddable; none for CTCHeadExportWrapper). A weight consumed by MatMul is stored
[in, out] and is transposed back to nn.Linear's [out, in]; Gemm honours transB. fp16 initializers are widened;
ORT dynamic-quant weights (`<w>_quantized` uint8 + `<w>_scale` + `<w>_zero_point`, per output channel) are
dequantised to f32 by state_dict_from_onnx, and handed over as they are by u8dq_from_onnx: the CTC graph runs them with
the quantized graph's own arithmetic (DynamicQuantizeLinear + MatMulInteger on the GPU, fa_set_tensor_u8dq).
Parity unpinned: no ONNX file ships in the reference (weights absent) and `onnx` is not installed; the reader is
tested on files written by the repo's own encoder of the same wire format (tests/test_weights_io.py).
"""
import struct

import numpy as np

_DT = {1: np.float32, 2: np.uint8, 3: np.int8, 5: np.int16, 6: np.int32, 7: np.int64, 10: np.float16, 11: np.float64}


def _varint(b, i):
    r = s = 0
    while True:
        c = b[i]
        i += 1
        r |= (c & 0x7F) << s
        if c < 0x80:
            return r, i
        s += 7


def _fields(b):
    """Yield (field number, wire type, value) of one protobuf message (value: int or memoryview)."""
    i, n = 0, len(b)
    while i < n:
        key, i = _varint(b, i)
        f, wt = key >> 3, key & 7
        if wt == 0:
            v, i = _varint(b, i)
        elif wt == 1:
            v, i = b[i:i + 8], i + 8
        elif wt == 2:
            ln, i = _varint(b, i)
            v, i = b[i:i + ln], i + ln
        elif wt == 5:
            v, i = b[i:i + 4], i + 4
        else:
            raise ValueError(f"unsupported protobuf wire type {wt}")
        yield f, wt, v


def _packed_ints(v, wt):
    if wt == 0:
        return [v]
    out, i, b = [], 0, bytes(v)
    while i < len(b):
        x, i = _varint(b, i)
        out.append(x)
    return out


def _tensor(b):
    dims, dt, name, raw, fl, i32, i64 = [], 1, "", None, [], [], []
    for f, wt, v in _fields(b):
        if f == 1:
            dims += _packed_ints(v, wt)
        elif f == 2:
            dt = v
        elif f == 4:
            fl += list(np.frombuffer(bytes(v), "<f4")) if wt == 2 else [struct.unpack("<f", bytes(v))[0]]
        elif f == 5:
            i32 += _packed_ints(v, wt)
        elif f == 7:
            i64 += _packed_ints(v, wt)
        elif f == 8:
            name = bytes(v).decode()
        elif f == 9:
            raw = bytes(v)
        elif f == 13:
            raise ValueError(f"initializer {name or '?'} uses external data: unsupported")
    if raw is not None:
        a = np.frombuffer(raw, np.dtype(_DT[dt]).newbyteorder("<")).copy()
    elif dt == 1:
        a = np.array(fl, np.float32)
    elif dt == 10:  # float16 in int32_data (low 16 bits)
        a = np.array(i32, np.uint16).view(np.float16)
    elif dt in (2, 3, 5, 6):
        a = np.array(i32, _DT[dt])
    else:
        a = np.array(i64, _DT.get(dt, np.int64))
    return name, a.reshape(dims) if dims else a


def _node(b):
    ins, outs, op, attrs = [], [], "", {}
    for f, wt, v in _fields(b):
        if f == 1:
            ins.append(bytes(v).decode())
        elif f == 2:
            outs.append(bytes(v).decode())
        elif f == 4:
            op = bytes(v).decode()
        elif f == 5:
            an, ai = "", None
            for g, _, x in _fields(v):
                if g == 1:
                    an = bytes(x).decode()
                elif g == 3:
                    ai = x
            attrs[an] = ai
    return op, ins, outs, attrs


def read_onnx(path):
    """-> (initializers {name: ndarray}, nodes [(op_type, inputs, outputs, attrs)])."""
    data = memoryview(open(path, "rb").read())
    inits, nodes = {}, []
    for f, _, v in _fields(data):
        if f != 7:
            continue
        for g, _, x in _fields(v):
            if g == 5:
                n, a = _tensor(x)
                inits[n] = a
            elif g == 1:
                nodes.append(_node(x))
    return inits, nodes


def _key(name):
    return name[len("hybrid_model."):] if name.startswith("hybrid_model.") else name


def u8dq_from_onnx(path, inits=None):
    """ORT dynamic-quant MatMul weights of an ONNX file, as stored: {state_dict weight name: (q [out][in] uint8,
    scale [out] f32, zero_point [out] uint8)} (the `<w>_quantized` initializer is the MatMul B [in][out]; per output
    channel scale / zero point, 02-Quantize-ONNX.py:38-46 per_channel=True, QUInt8)."""
    if inits is None:
        inits, _ = read_onnx(path)
    out = {}
    for name, a in inits.items():
        if not name.endswith("_quantized"):
            continue
        base = name[: -len("_quantized")]
        scale, zp = inits.get(base + "_scale"), inits.get(base + "_zero_point")
        key = _key(base)
        if scale is None or a.ndim != 2 or not key.endswith(".weight"):
            continue
        n_out = a.shape[1]
        scale = np.asarray(scale, np.float32).ravel()
        zp = np.zeros(n_out, np.uint8) if zp is None else np.asarray(zp).astype(np.uint8).ravel()
        if scale.size == 1:  # per-tensor quantisation: one scale / zero point for every channel
            scale, zp = np.repeat(scale, n_out), np.repeat(zp, n_out)
        if scale.size != n_out or zp.size != n_out:
            raise ValueError(f"{path}: {base}: scale / zero point do not match the {n_out} output channels")
        out[key] = (np.ascontiguousarray(np.asarray(a, np.uint8).T), scale, zp)
    return out


def state_dict_from_onnx(path):
    """HybridSenseVoice state_dict entries (f32, nn.Linear [out, in]) held by an encoder or CTC ONNX file."""
    inits, nodes = read_onnx(path)
    consumers = {}
    for op, ins, _, attrs in nodes:
        for k, nm in enumerate(ins):
            consumers.setdefault(nm, []).append((op, k, attrs))
    out = {}
    for name, a in inits.items():
        base = name
        if name.endswith("_quantized"):
            base = name[: -len("_quantized")]
            scale = inits.get(base + "_scale")
            zp = inits.get(base + "_zero_point")
            if scale is None:
                continue
            zp = np.zeros_like(scale) if zp is None else zp.astype(np.float32)
            a = (a.astype(np.float32) - zp) * scale.astype(np.float32)  # [in, out] with per-out-channel scales
            uses = [("MatMul", 1, {})]
        elif any(name.endswith(sfx) and name[: -len(sfx)] + "_quantized" in inits for sfx in ("_scale", "_zero_point")):
            continue
        else:
            uses = consumers.get(name, [])
        key = _key(base)
        if not key.startswith(("audio_encoder.", "audio_adaptor.", "ctc_decoder.", "ctc_proj.")):
            continue
        w = np.asarray(a, np.float32)
        if w.ndim == 2 and key.endswith(".weight"):
            for op, k, attrs in uses:
                if op == "MatMul" and k == 1:
                    w = w.T
                    break
                if op == "Gemm" and k == 1:
                    if not attrs.get("transB"):
                        w = w.T
                    break
        out[key] = np.ascontiguousarray(w)
    return out
