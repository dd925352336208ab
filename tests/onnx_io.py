"""Minimal ONNX (protobuf wire format) writer for tests — the repo's own encoder of the ModelProto fields the
reader (fun_asr_gguf.onnx_weights) consumes: graph.initializer (TensorProto dims / data_type / name / raw_data)
and graph.node (MatMul / Gemm consumers). Files are shaped as 01-Export-Encoder-Adaptor-CTC.py's dynamo export
names its initializers (module paths under the export wrapper) and as 02-Quantize-ONNX.py converts them (fp16
initializers; ORT dynamic-quant `<w>_quantized` uint8 + `_scale` + `_zero_point`, per output channel)."""
import struct

import numpy as np

FLOAT, UINT8, FLOAT16 = 1, 2, 10


def _varint(x):
    out = bytearray()
    while True:
        b = x & 0x7F
        x >>= 7
        if x:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _key(f, wt):
    return _varint((f << 3) | wt)


def _ld(f, payload):
    return _key(f, 2) + _varint(len(payload)) + payload


def _str(f, s):
    return _ld(f, s.encode())


def tensor_proto(name, a, dtype):
    b = b"".join(_key(1, 0) + _varint(int(d)) for d in a.shape)
    b += _key(2, 0) + _varint(dtype) + _str(8, name)
    npdt = {FLOAT: "<f4", UINT8: "u1", FLOAT16: "<f2"}[dtype]
    return b + _ld(9, np.ascontiguousarray(a).astype(npdt).tobytes())


def node_proto(op, inputs, outputs, trans_b=None):
    b = b"".join(_str(1, i) for i in inputs) + b"".join(_str(2, o) for o in outputs) + _str(4, op)
    if trans_b is not None:
        b += _ld(5, _str(1, "transB") + _key(3, 0) + _varint(trans_b) + _key(20, 0) + _varint(2))
    return b


def write_onnx(path, state_dict, prefix="", dtype="fp32", gemm_every=3):
    """state_dict: name -> f32 array (nn.Linear [out, in]). 2-D weights: every `gemm_every`-th one consumed by
    Gemm(transB=1) as [out, in], the others stored transposed [in, out] for MatMul (dynamo's aten.linear
    lowering). dtype: fp32 | fp16 | int8 (2-D weights dynamic-quantised per output channel, like ORT's
    quantize_dynamic(MatMul, per_channel=True, QUInt8))."""
    inits, nodes = [], []
    for i, (k, w) in enumerate(sorted(state_dict.items())):
        name = prefix + k
        w = np.asarray(w, np.float32)
        if w.ndim == 2 and k.endswith(".weight"):
            gemm = dtype != "int8" and i % gemm_every == 0
            if gemm:
                nodes.append(node_proto("Gemm", ["x%d" % i, name], ["y%d" % i], trans_b=1))
                stored = w
            else:
                stored = w.T.copy()
                if dtype == "int8":
                    lo = np.minimum(stored.min(0), 0.0)
                    hi = np.maximum(stored.max(0), 0.0)
                    scale = ((hi - lo) / 255.0).astype(np.float32)
                    scale[scale == 0] = 1.0
                    zp = np.clip(np.round(-lo / scale), 0, 255).astype(np.uint8)
                    q = np.clip(np.round(stored / scale) + zp, 0, 255).astype(np.uint8)
                    inits += [tensor_proto(name + "_quantized", q, UINT8), tensor_proto(name + "_scale", scale, FLOAT),
                              tensor_proto(name + "_zero_point", zp, UINT8)]
                    nodes.append(node_proto("MatMulInteger", ["xq%d" % i, name + "_quantized"], ["y%d" % i]))
                    continue
                nodes.append(node_proto("MatMul", ["x%d" % i, name], ["y%d" % i]))
            inits.append(tensor_proto(name, stored, FLOAT16 if dtype == "fp16" else FLOAT))
        else:
            inits.append(tensor_proto(name, w, FLOAT16 if dtype == "fp16" else FLOAT))
    graph = b"".join(_ld(1, n) for n in nodes) + _str(2, "main_graph") + b"".join(_ld(5, t) for t in inits)
    model = _key(1, 0) + _varint(8) + _ld(7, graph)  # ir_version 8, graph
    with open(path, "wb") as f:
        f.write(model)
