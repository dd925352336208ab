"""fp16 encoder graph restatement (numpy) — TEST INFRASTRUCTURE ONLY.

The reference's fp16 models are its fp32 ONNX graphs converted by onnxruntime.transformers.float16
(02-Quantize-ONNX.py:13-27: keep_io_types=False, min_positive_val=1e-7, max_finite_val=65504,
op_block_list=['LayerNormalization']) and fed float16 audio (nano_onnx.py:84,101). Restated here as: every
initializer converted like the converter does (magnitudes clamped into [1e-7, 65504], round to nearest
even); every op computes in f32 from its fp16 inputs and rounds its output to fp16; LayerNormalization
computes in f32 and only its output is fp16. The math is model_definition.py's, as in oracle/encoder.py.

PARITY UNPINNED against onnxruntime's fp16 kernels (onnxruntime is absent here, and no reference test holds
fp16 outputs): this is the contract the GPU fp16 path is checked against; the fp32 oracle bounds it loosely.
"""
import numpy as np

from . import encoder as e32
from . import frontend as fe


def h(x):
    """op output -> fp16 value (held in float32)."""
    return np.asarray(x, np.float32).astype(np.float16).astype(np.float32)


def init16(w):
    """float16 converter on an initializer (onnxruntime.transformers.float16.convert_np_to_float16)."""
    w = np.asarray(w, np.float32)
    a = np.abs(w)
    w = np.where((a > 0) & (a < 1e-7), np.sign(w) * np.float32(1e-7), w)
    w = np.where(a > 65504, np.sign(w) * np.float32(65504), w)
    return w.astype(np.float16).astype(np.float32)


def weights16(W):
    """All initializers through the converter, except LayerNorm's (op_block_list keeps them fp32)."""
    out = {}
    for k, v in W.items():
        is_ln = ".norm" in k or "after_norm" in k or "tp_norm" in k
        out[k] = np.asarray(v, np.float32) if is_ln else init16(v)
    return out


def linear(x, W, p, relu=False, add2=None, add1=None):
    y = h(x @ W[p + ".weight"].T + (W[p + ".bias"] if p + ".bias" in W else np.float32(0)))
    if relu:
        y = np.maximum(y, 0)
    if add2 is not None:
        y = h(y + add2)
    if add1 is not None:
        y = h(add1 + y)
    return y


def layer_norm(x, w, b, eps):
    return h(e32.layer_norm(x, w, b, eps))


def attention(q, k, v, n_heads, key_mask):
    return h(e32.attention(q, k, v, n_heads, key_mask))


def fsmn(v, W, p, m, ksize):
    vm = v * m[:, None] if m is not None else v
    w = W[p + ".self_attn.fsmn_block.weight"][:, 0, :]
    T = v.shape[0]
    lp = (ksize - 1) // 2
    xp = np.pad(vm, ((lp, ksize - 1 - lp), (0, 0)))
    acc = np.zeros_like(vm)
    for j in range(ksize):
        acc += xp[j:j + T] * w[:, j][None, :]
    return h(h(acc) + vm)


def sanm_block(x, W, p, m, cfg, first=False):
    d = cfg["d_model"]
    hn = layer_norm(x, W[p + ".norm1.weight"], W[p + ".norm1.bias"], 1e-5)
    qkv = linear(hn, W, p + ".self_attn.linear_q_k_v")
    q, k, v = qkv[:, :d], qkv[:, d:2 * d], qkv[:, 2 * d:]
    mem = fsmn(v, W, p, m, cfg["fsmn_k"])
    att = attention(q, k, v, cfg["n_heads"], m)
    if first:
        return linear(att, W, p + ".self_attn.linear_out", add2=mem)
    x = linear(att, W, p + ".self_attn.linear_out", add2=mem, add1=x)
    hn = layer_norm(x, W[p + ".norm2.weight"], W[p + ".norm2.bias"], 1e-5)
    f = linear(hn, W, p + ".feed_forward.w_1", relu=True)
    return linear(f, W, p + ".feed_forward.w_2", add1=x)


def adaptor(x, W, p, n_blocks, n_heads, mask):
    x = linear(linear(x, W, p + ".linear1", relu=True), W, p + ".linear2")
    for b in range(n_blocks):
        q = f"{p}.blocks.{b}"
        hn = layer_norm(x, W[q + ".norm1.weight"], W[q + ".norm1.bias"], 1e-12)
        att = attention(linear(hn, W, q + ".self_attn.linear_q"), linear(hn, W, q + ".self_attn.linear_k"),
                        linear(hn, W, q + ".self_attn.linear_v"), n_heads, mask)
        x = linear(att, W, q + ".self_attn.linear_out", add1=x)
        hn = layer_norm(x, W[q + ".norm2.weight"], W[q + ".norm2.bias"], 1e-12)
        x = linear(linear(hn, W, q + ".feed_forward.w_1", relu=True), W, q + ".feed_forward.w_2", add1=x)
    return x


def frontend(audio, valid=None):
    """F1-F4 on float16 audio (model_definition.py:269-311 with fp16 op outputs)."""
    a = h(audio)
    if valid is None:
        valid = a.shape[0]
    c = fe.frame_counts(valid, a.shape[0])
    msk = (np.arange(a.shape[0]) < valid).astype(np.float32)
    mean = h(np.float32(np.sum((a * msk).astype(np.float64)) / valid))
    ac = h(a - mean) * msk
    pre = ac.copy()
    pre[1:] = h(ac[1:] - h(np.float32(fe.PRE_EMPH) * ac[:-1]))
    pre = pre * msk
    cos_k, sin_k = fe.stft_basis()
    cos_k, sin_k = init16(cos_k), init16(sin_k)
    fb = init16(fe.mel_fbank())
    xp = np.pad(pre, (fe.N_FFT // 2, fe.N_FFT // 2))
    t_phys = pre.shape[0] // fe.HOP + 1
    idx = np.arange(t_phys)[:, None] * fe.HOP + np.arange(fe.N_FFT)[None, :]
    frames = xp[idx].astype(np.float32)
    re, im = h(frames @ cos_k.T), h(frames @ sin_k.T)
    power = h(h(re * re) + h(im * im))
    mel = h(np.log(h(h(power @ fb.T) + h(np.float32(1e-7)))))
    x, m = fe.lfr(mel, c["t_mel_valid"])
    pe = fe.sinusoidal_pe(x.shape[0], x.shape[1])
    x = h(h(x * h(np.float32(512 ** 0.5))) + h(pe))
    return x, m, c


def encode(audio, W32, cfg, valid=None):
    """Encoder + adaptor + CTC head of the fp16 graphs for one clip (CPU-EP policy, as oracle/encoder.encode)."""
    W = weights16(W32)
    x, m, c = frontend(audio, valid)
    x = sanm_block(x, W, "audio_encoder.encoders0.0", m, cfg, first=True)
    for i in range(cfg["n_blocks"] - 1):
        x = sanm_block(x, W, f"audio_encoder.encoders.{i}", m, cfg)
    x = layer_norm(x, W["audio_encoder.after_norm.weight"], W["audio_encoder.after_norm.bias"], 1e-5) * m[:, None]
    for i in range(cfg["n_tp_blocks"]):
        x = sanm_block(x, W, f"audio_encoder.tp_encoders.{i}", m, cfg)
    enc = layer_norm(x, W["audio_encoder.tp_norm.weight"], W["audio_encoder.tp_norm.bias"], 1e-5) * m[:, None]
    ad = adaptor(enc, W, "audio_adaptor", cfg["adaptor_blocks"], cfg["adaptor_heads"], m)
    tl = c["target_len"]
    logits = linear(adaptor(enc, W, "ctc_decoder", cfg["ctc_blocks"], cfg["ctc_heads"], None), W, "ctc_proj.ctc_lo")
    return dict(enc=enc, audio_embd=ad[:tl].astype(np.float32), ctc_ids=np.argmax(logits, -1).astype(np.int32),
                ctc_logits=logits, counts=c)
