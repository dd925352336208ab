"""int8-dynamic CTC graph restatement (numpy) — TEST INFRASTRUCTURE ONLY.

The reference's default CTC model is Fun-ASR-Nano-CTC.int8.onnx (README.md:71-72, 153-154, 480-481), made by
02-Quantize-ONNX.py:38-46: onnxruntime.quantization.quantize_dynamic(op_types_to_quantize=["MatMul"],
per_channel=True, reduce_range=False, weight_type=QuantType.QUInt8). Restated from the published algorithms:

* offline weight quantisation (onnxruntime quantization/quant_utils.py compute_scale_zp + quantize_nparray, asymmetric
  uint8 [0, 255] per output channel): rmin = min(0, min w), rmax = max(0, max w), scale = f32((rmax - rmin) / 255)
  (computed in float64), zp = round_half_even(-rmin / scale), q = clip(round_half_even(f32(w) / scale) + zp, 0, 255).
  Only MatMuls whose B input is a constant are quantised (quantize_dynamic's MatMulConstBOnly default): the attention's
  q.k^T and p.v stay f32.
* at run time every quantised MatMul is DynamicQuantizeLinear(x) -> MatMulInteger(xq, wq, xzp, wzp) -> Cast(float) ->
  Mul(x_scale * w_scale) (the ONNX operator definitions; onnxruntime may fuse them into DynamicQuantizeMatMul with the
  same arithmetic), then the exporter's bias Add:
    DynamicQuantizeLinear (per TENSOR, uint8): x_min = min(0, min x), x_max = max(0, max x), xs = (x_max - x_min) / 255,
    xzp = round_half_even(clamp(-x_min / xs, 0, 255)), xq = clip(round_half_even(x / xs) + xzp, 0, 255);
    MatMulInteger: y_int = sum_k (xq - xzp)(wq - wzp) in int32 (exact);
    y = f32(y_int) * f32(xs * ws) + bias.
  The CTC graph's input tensor is one clip's unpadded encoder output [1, T, 512] (nano_onnx CPU-EP policy), so the
  activation scale of every MatMul is taken over that clip's T rows.

PARITY UNPINNED against onnxruntime itself (absent here; no int8 fixture ships): the ONNX operator semantics are pinned by
the ONNX specification's own DynamicQuantizeLinear / MatMulInteger examples (tests/test_ctc_int8.py); the rest of the
graph is oracle/encoder.py's (model_definition.py:114-185, 331-337).
"""
import numpy as np

from . import encoder as e32

# the CTC graph's linears quantised by quantize_dynamic (MatMul with a constant weight): model_definition.py:165-185, 216-219
def ctc_linear_names(cfg):
    names = ["ctc_decoder.linear1", "ctc_decoder.linear2"]
    for b in range(cfg["ctc_blocks"]):
        q = f"ctc_decoder.blocks.{b}"
        names += [q + ".self_attn.linear_q", q + ".self_attn.linear_k", q + ".self_attn.linear_v",
                  q + ".self_attn.linear_out", q + ".feed_forward.w_1", q + ".feed_forward.w_2"]
    return names + ["ctc_proj.ctc_lo"]


def quantize_weight(w):
    """nn.Linear weight [out][in] f32 -> (q [out][in] uint8, scale [out] f32, zero_point [out] uint8): per output channel
    (the ONNX MatMul B = w^T [in][out], channel axis 1), asymmetric QUInt8, reduce_range off."""
    w = np.asarray(w, np.float32)
    rmin = np.minimum(w.min(1), np.float32(0))
    rmax = np.maximum(w.max(1), np.float32(0))
    dr = (rmax.astype(np.float64) - rmin.astype(np.float64))
    scale64 = dr / 255.0
    tiny = scale64 < np.finfo(np.float32).tiny
    zp = np.where(tiny, 0.0, np.round(0.0 - rmin.astype(np.float64) / np.where(tiny, 1.0, scale64)))
    scale = np.where(tiny, np.float32(1.0), scale64.astype(np.float32)).astype(np.float32)
    q = np.clip(np.round(w / scale[:, None]) + zp[:, None], 0, 255).astype(np.uint8)
    return q, scale, zp.astype(np.uint8)


def dynamic_quantize_linear(x):
    """ONNX DynamicQuantizeLinear (uint8) of the whole tensor -> (xq uint8, scale f32, zero_point uint8)."""
    x = np.asarray(x, np.float32)
    mn = np.float32(min(float(x.min()), 0.0))
    mx = np.float32(max(float(x.max()), 0.0))
    xs = np.float32(1.0) if mx == mn else np.float32((mx - mn) / np.float32(255.0))
    zp = np.float32(np.round(np.clip(np.float32(0.0) - mn / xs, 0.0, 255.0)))  # np.round: half to even
    xq = np.clip(np.round(x / xs) + zp, 0, 255).astype(np.uint8)
    return xq, xs, np.uint8(zp)


def matmul_integer(a, b, a_zp, b_zp):
    """ONNX MatMulInteger: (a - a_zp) @ (b - b_zp) in int32 (b: [K][N], b_zp per column or scalar). Evaluated as a
    float64 product: every term is an integer below 2^16 and every sum below 255^2 K < 2^53, so it is exact."""
    d = (a.astype(np.float64) - float(a_zp)) @ (b.astype(np.float64) - np.asarray(b_zp, np.float64))
    return d.astype(np.int64)


def linear_int8(x, Q, W, p):
    """y = f32(MatMulInteger(DQL(x), wq^T)) * f32(xs * ws) + bias for the quantised linear `p`."""
    q, ws, wzp = Q[p]
    xq, xs, xzp = dynamic_quantize_linear(x)
    acc = matmul_integer(xq, q.T, xzp, wzp[None, :])
    y = acc.astype(np.float32) * (np.float32(xs) * ws)
    b = W.get(p + ".bias")
    return (y + b).astype(np.float32) if b is not None else y.astype(np.float32)


def quantize_ctc(W, cfg):
    """Every CTC-graph linear of a state_dict through quantize_weight -> {prefix: (q, scale, zp)}."""
    return {p: quantize_weight(W[p + ".weight"]) for p in ctc_linear_names(cfg)}


def ctc_logits_int8(enc, W, Q, cfg):
    """CTCHeadExportWrapper (model_definition.py:331-337) of the int8 graph on one clip's unpadded encoder output:
    ctc_decoder (CorrectTransformerAdaptor, mask=None) with int8-dynamic linears, f32 attention / LayerNorm, ctc_lo."""
    p = "ctc_decoder"
    x = linear_int8(np.maximum(linear_int8(enc, Q, W, p + ".linear1"), 0), Q, W, p + ".linear2")
    for b in range(cfg["ctc_blocks"]):
        q = f"{p}.blocks.{b}"
        h = e32.layer_norm(x, W[q + ".norm1.weight"], W[q + ".norm1.bias"], 1e-12)
        att = e32.attention(linear_int8(h, Q, W, q + ".self_attn.linear_q"), linear_int8(h, Q, W, q + ".self_attn.linear_k"),
                            linear_int8(h, Q, W, q + ".self_attn.linear_v"), cfg["ctc_heads"], None)
        x = (x + linear_int8(att, Q, W, q + ".self_attn.linear_out")).astype(np.float32)
        h = e32.layer_norm(x, W[q + ".norm2.weight"], W[q + ".norm2.bias"], 1e-12)
        f = linear_int8(np.maximum(linear_int8(h, Q, W, q + ".feed_forward.w_1"), 0), Q, W, q + ".feed_forward.w_2")
        x = (x + f).astype(np.float32)
    return linear_int8(x, Q, W, "ctc_proj.ctc_lo")


def ctc_ids_int8(enc, W, Q, cfg):
    lg = ctc_logits_int8(enc, W, Q, cfg)
    return np.argmax(lg, -1).astype(np.int32), lg
