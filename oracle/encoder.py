"""Encoder / adaptor / CTC-head restatement (numpy fp32) — TEST INFRASTRUCTURE ONLY.

Follows /root/reference/fun_asr_gguf/model_definition.py:
  SenseVoiceEncoderSmall.forward :205-214, EncoderLayerSANM :92-116, MultiHeadedAttentionSANM :50-90,
  PositionwiseFeedForward :30-40, LayerNorm :42-44 (eps 1e-5), CorrectTransformerAdaptor :165-185,
  EncoderLayer :147-163 (eps 1e-12), MultiHeadedAttention :122-145, length control :316-321,
  CTCHeadExportWrapper :335-337 (ctc_decoder run with mask=None, then argmax -> int32).
`W` is a dict keyed by the reference's state_dict names (oracle/synth.py).
"""
import numpy as np
from . import frontend as fe


def layer_norm(x, w, b, eps):
    x64 = x.astype(np.float64)
    mu = x64.mean(-1, keepdims=True)
    var = ((x64 - mu) ** 2).mean(-1, keepdims=True)
    return (((x64 - mu) / np.sqrt(var + eps)) * w + b).astype(np.float32)


def linear(x, W, p):
    y = x @ W[p + ".weight"].T
    b = W.get(p + ".bias")
    if b is not None:
        y = y + b
    return y.astype(np.float32)


def softmax(s):
    s = s - s.max(-1, keepdims=True)
    e = np.exp(s)
    return (e / e.sum(-1, keepdims=True)).astype(np.float32)


def attention(q, k, v, n_heads, key_mask):
    """softmax(q*d^-0.5 @ k^T + (m-1)*1e4) @ v over heads; q,k,v [T, H*dk]."""
    T, HD = q.shape
    dk = HD // n_heads
    out = np.empty((T, HD), np.float32)
    add = None if key_mask is None else ((key_mask - 1.0) * 10000.0).astype(np.float32)
    scale = np.float32(dk ** -0.5)
    for h in range(n_heads):
        sl = slice(h * dk, (h + 1) * dk)
        s = (q[:, sl] * scale) @ k[:, sl].T
        if add is not None:
            s = s + add[None, :]
        out[:, sl] = softmax(s) @ v[:, sl]
    return out


def fsmn(v, W, p, m, ksize):
    """forward_fsmn (:60-66): depthwise conv1d (zero pad (k-1)/2 both sides, no bias) of v*m, + v*m."""
    vm = v * m[:, None] if m is not None else v
    w = W[p + ".self_attn.fsmn_block.weight"][:, 0, :]  # [C, k]
    T = v.shape[0]
    lp = (ksize - 1) // 2
    xp = np.pad(vm, ((lp, ksize - 1 - lp), (0, 0)))
    out = np.zeros_like(vm)
    for j in range(ksize):
        out += xp[j:j + T] * w[:, j][None, :]
    return (out + vm).astype(np.float32)


def sanm_block(x, W, p, m, cfg, first=False):
    d = cfg["d_model"]
    res = x
    h = layer_norm(x, W[p + ".norm1.weight"], W[p + ".norm1.bias"], 1e-5)
    qkv = linear(h, W, p + ".self_attn.linear_q_k_v")
    q, k, v = qkv[:, :d], qkv[:, d:2 * d], qkv[:, 2 * d:]
    mem = fsmn(v, W, p, m, cfg["fsmn_k"])
    att = attention(q, k, v, cfg["n_heads"], m)
    y = linear(att, W, p + ".self_attn.linear_out") + mem
    if first:  # encoders0: in_size != size -> no residual, no FFN (:105-107)
        return y.astype(np.float32)
    x = (res + y).astype(np.float32)
    h = layer_norm(x, W[p + ".norm2.weight"], W[p + ".norm2.bias"], 1e-5)
    f = linear(np.maximum(linear(h, W, p + ".feed_forward.w_1"), 0), W, p + ".feed_forward.w_2")
    return (x + f).astype(np.float32)


def sense_voice_encoder(x, m, W, cfg, taps=None):
    """x: LFR features [T, 560] (already masked); m: [T] mask. Returns enc [T, 512]."""
    x = (x * np.float32(512 ** 0.5)).astype(np.float32) + fe.sinusoidal_pe(x.shape[0], x.shape[1])
    x = sanm_block(x, W, "audio_encoder.encoders0.0", m, cfg, first=True)
    if taps is not None:
        taps["block0"] = x.copy()
    for i in range(cfg["n_blocks"] - 1):
        x = sanm_block(x, W, f"audio_encoder.encoders.{i}", m, cfg)
    x = layer_norm(x, W["audio_encoder.after_norm.weight"], W["audio_encoder.after_norm.bias"], 1e-5)
    x = x * m[:, None]
    if taps is not None:
        taps["after_norm"] = x.copy()
    for i in range(cfg["n_tp_blocks"]):
        x = sanm_block(x, W, f"audio_encoder.tp_encoders.{i}", m, cfg)
    x = layer_norm(x, W["audio_encoder.tp_norm.weight"], W["audio_encoder.tp_norm.bias"], 1e-5)
    return (x * m[:, None]).astype(np.float32)


def adaptor(x, W, p, n_blocks, n_heads, mask):
    """CorrectTransformerAdaptor.forward with k=1 (:179-185); EncoderLayer pre-norm, eps 1e-12."""
    x = linear(np.maximum(linear(x, W, p + ".linear1"), 0), W, p + ".linear2")
    for b in range(n_blocks):
        q = f"{p}.blocks.{b}"
        h = layer_norm(x, W[q + ".norm1.weight"], W[q + ".norm1.bias"], 1e-12)
        att = attention(linear(h, W, q + ".self_attn.linear_q"), linear(h, W, q + ".self_attn.linear_k"),
                        linear(h, W, q + ".self_attn.linear_v"), n_heads, mask)
        x = (x + linear(att, W, q + ".self_attn.linear_out")).astype(np.float32)
        h = layer_norm(x, W[q + ".norm2.weight"], W[q + ".norm2.bias"], 1e-12)
        f = linear(np.maximum(linear(h, W, q + ".feed_forward.w_1"), 0), W, q + ".feed_forward.w_2")
        x = (x + f).astype(np.float32)
    return x


def ctc_logits(enc, W, cfg, mask=None):
    h = adaptor(enc, W, "ctc_decoder", cfg["ctc_blocks"], cfg["ctc_heads"], mask)
    return linear(h, W, "ctc_proj.ctc_lo")


def encode(audio, W, cfg, valid=None, taps=None):
    """The whole encoder ORT graph + CTC ORT graph for one clip (nano_onnx.encode_audio:78-133 with
    the CPU-EP policy: no padding beyond the clip). Returns dict(enc, adaptor, audio_embd, ctc_ids, counts)."""
    x, m, c = fe.frontend(audio, valid)
    if taps is not None:
        taps["lfr"] = x.copy()
    enc = sense_voice_encoder(x, m, W, cfg, taps)
    ad = adaptor(enc, W, "audio_adaptor", cfg["adaptor_blocks"], cfg["adaptor_heads"], m)
    tl = c["target_len"]
    ad = ad * (np.arange(ad.shape[0]) < tl)[:, None]
    logits = ctc_logits(enc, W, cfg, None)  # reference runs the CTC head unmasked (:336)
    ids = np.argmax(logits, -1).astype(np.int32)
    return dict(enc=enc, adaptor=ad.astype(np.float32), audio_embd=ad[:tl].astype(np.float32),
                ctc_ids=ids, ctc_logits=logits, counts=c)
