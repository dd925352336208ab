"""q8_0 block quantisation — TEST INFRASTRUCTURE ONLY.

quantize_q8_0 restates the ggml reference quantiser that the vendored gguf-py declares bit-exact
(/root/reference/fun_asr_gguf/gguf/quants.py:378-393): per 32-wide block d = amax/127,
id = d ? 1/d : 0, q = roundf(x*id) (round half away from zero), d stored as fp16 (RNE).
Byte layout of one block (34 B): fp16 d, then 32 x int8 (ggml block_q8_0).
"""
import numpy as np

QK = 32


def np_roundf(n):
    a = np.abs(n)
    fl = np.floor(a)
    return np.sign(n) * (fl + np.floor(np.float32(2) * (a - fl)))


def quantize_q8_0(x):
    """x [..., K] f32 (K % 32 == 0) -> (d f16 [..., K/32], q int8 [..., K/32, 32])."""
    x = np.asarray(x, dtype=np.float32)
    shp = x.shape[:-1]
    blk = x.reshape(*shp, x.shape[-1] // QK, QK)
    d = (np.abs(blk).max(-1, keepdims=True) / np.float32(127)).astype(np.float32)
    with np.errstate(divide="ignore"):
        inv = np.where(d == 0, np.float32(0), np.float32(1) / d).astype(np.float32)
    q = np_roundf((blk * inv).astype(np.float32)).astype(np.int8)
    return d[..., 0].astype(np.float16), q


def pack_q8_0(d, q):
    """-> uint8 [..., K/32*34] in ggml block order."""
    shp = q.shape[:-2]
    nb = q.shape[-2]
    out = np.empty((*shp, nb, 34), np.uint8)
    out[..., :2] = d.reshape(*shp, nb, 1).view(np.uint8).reshape(*shp, nb, 2)
    out[..., 2:] = q.view(np.uint8)
    return out.reshape(*shp, nb * 34)


def dequant_f32(d, q):
    """ggml dequantize_row_q8_0: y = f32(d) * q, in f32."""
    return (d.astype(np.float32)[..., None] * q.astype(np.float32)).reshape(*q.shape[:-2], -1)


def dequant_numpy_f16(d, q):
    """llama.py:778-784 (get_token_embeddings_gguf): numpy f16 x int8 -> f16 product -> f32."""
    return (d[..., None] * q).astype(np.float32).reshape(*q.shape[:-2], -1)


def matmul_q8(wd, wq, x):
    """ggml q8_0 x q8_0: y[o] = sum_b f32(int_dot(qw[o,b], qx[b])) * (f32(dw[o,b]) * f32(dx[b])).
    wd [O, nb] f16, wq [O, nb, 32] i8, x [N, K] f32 -> y [N, O] f32. Activations are quantised
    per row with the reference q8_0 quantiser (ggml vec_dot_type of q8_0 is q8_0)."""
    xd, xq = quantize_q8_0(x)                                   # [N, nb], [N, nb, 32]
    # per-block integer dots: |sum| <= 32*127*127 < 2^24, so an f32 batched matmul is exact
    wqf = wq.astype(np.float32).transpose(1, 2, 0)              # [nb, 32, O]
    xqf = xq.astype(np.float32).transpose(1, 0, 2)              # [nb, N, 32]
    sumi = np.matmul(xqf, wqf).transpose(1, 2, 0)               # [N, O, nb] exact ints
    scale = wd.astype(np.float32)[None, :, :] * xd.astype(np.float32)[:, None, :]
    return (sumi * scale).sum(-1, dtype=np.float32)
