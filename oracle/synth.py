"""Deterministic synthetic weights (oracle side) — TEST INFRASTRUCTURE ONLY.

The real Fun-ASR-Nano-2512 weights are absent, so parity and benchmarks run on
weights produced by a counter-based hash that the HIP engine reproduces bit-for-bit on device
(fun-asr-gguf_amd/csrc/synth.hip). Spec (shared contract, restated independently here):

  key(name, seed) = lowbias32(fnv1a32(name) ^ (seed * 0x9E3779B9 mod 2^32))
  h_i             = lowbias32(i ^ key)                (i = flat element index, uint32)
  u_i             = float32((h_i >> 8)) * 2^-24 * 2 - 1   in [-1, 1), exact in f32
  w_i             = fl32(fl32(u_i * scale) + offset)     (two IEEE roundings, no fma)

Tensor names follow the reference's state_dict (model_definition.py) for the encoder side and
the GGUF tensor names (gguf/constants.py:1696-1712, arch qwen3) for the decoder side.
"""
import math
import numpy as np

M32 = 0xFFFFFFFF


def fnv1a32(s: str) -> int:
    h = 0x811C9DC5
    for b in s.encode("utf-8"):
        h ^= b
        h = (h * 0x01000193) & M32
    return h


def lowbias32(x: np.ndarray) -> np.ndarray:
    x = x.astype(np.uint32, copy=True)
    x ^= x >> np.uint32(16)
    x *= np.uint32(0x7FEB352D)
    x ^= x >> np.uint32(15)
    x *= np.uint32(0x846CA68B)
    x ^= x >> np.uint32(16)
    return x


def tensor_key(name: str, seed: int) -> int:
    k = np.array([fnv1a32(name) ^ ((seed * 0x9E3779B9) & M32)], dtype=np.uint32)
    return int(lowbias32(k)[0])


def gen(name: str, n: int, scale: float, offset: float = 0.0, seed: int = 0) -> np.ndarray:
    key = np.uint32(tensor_key(name, seed))
    idx = np.arange(n, dtype=np.uint32)
    h = lowbias32(idx ^ key)
    u = (h >> np.uint32(8)).astype(np.float32) * np.float32(2.0 ** -24) * np.float32(2.0) - np.float32(1.0)
    w = u * np.float32(scale)
    if offset != 0.0:
        w = w + np.float32(offset)
    return w.astype(np.float32)


# ---------------------------------------------------------------------------------------
# Model configurations. "full" = the reference's dims (model_definition.py:191-229; Qwen3-0.6B).
# "tiny" shrinks only the layer counts / vocab so CPU tests stay fast; all widths are kept.
# ---------------------------------------------------------------------------------------
ENC_FULL = dict(n_mels=80, lfr_m=7, lfr_n=6, d_in=560, d_model=512, n_heads=4, d_ffn=2048,
                n_blocks=50, n_tp_blocks=20, fsmn_k=11,
                d_llm=1024, adaptor_ffn=2048, adaptor_blocks=2, adaptor_heads=8,
                ctc_blocks=5, ctc_heads=8, ctc_ffn=2048, ctc_vocab=60515)
ENC_TINY = dict(ENC_FULL, n_blocks=3, n_tp_blocks=2, adaptor_blocks=1, ctc_blocks=1, ctc_vocab=3001)

LLM_FULL = dict(n_layer=28, n_embd=1024, n_head=16, n_head_kv=8, head_dim=128, n_ff=3072,
                n_vocab=151936, rope_theta=1000000.0, rms_eps=1e-6)
LLM_TINY = dict(LLM_FULL, n_layer=2, n_vocab=4096)


def _lin(names, prefix, n_in, n_out, bias=True):
    names.append((prefix + ".weight", (n_out, n_in), math.sqrt(3.0 / n_in), 0.0))
    if bias:
        names.append((prefix + ".bias", (n_out,), 0.02, 0.0))


def _ln(names, prefix, d):
    names.append((prefix + ".weight", (d,), 0.1, 1.0))
    names.append((prefix + ".bias", (d,), 0.02, 0.0))


def _sanm_block(names, p, d_in, d, d_ffn, k):
    _ln(names, p + ".norm1", d_in)
    _ln(names, p + ".norm2", d)
    _lin(names, p + ".self_attn.linear_q_k_v", d_in, 3 * d)
    _lin(names, p + ".self_attn.linear_out", d, d)
    names.append((p + ".self_attn.fsmn_block.weight", (d, 1, k), math.sqrt(3.0 / k) * 0.5, 0.0))
    _lin(names, p + ".feed_forward.w_1", d, d_ffn)
    _lin(names, p + ".feed_forward.w_2", d_ffn, d)


def _adaptor(names, p, d_enc, d_out, d_ffn, n_blocks):
    _lin(names, p + ".linear1", d_enc, d_ffn)
    _lin(names, p + ".linear2", d_ffn, d_out)
    for b in range(n_blocks):
        q = f"{p}.blocks.{b}"
        for nm in ("linear_q", "linear_k", "linear_v", "linear_out"):
            _lin(names, f"{q}.self_attn.{nm}", d_out, d_out)
        _lin(names, q + ".feed_forward.w_1", d_out, d_out // 4)
        _lin(names, q + ".feed_forward.w_2", d_out // 4, d_out)
        _ln(names, q + ".norm1", d_out)
        _ln(names, q + ".norm2", d_out)


def encoder_tensors(cfg):
    """(name, shape, scale, offset) for every encoder/adaptor/CTC parameter (HybridSenseVoice
    state_dict names, model_definition.py:191-229)."""
    names = []
    d, f, k = cfg["d_model"], cfg["d_ffn"], cfg["fsmn_k"]
    _sanm_block(names, "audio_encoder.encoders0.0", cfg["d_in"], d, f, k)
    for i in range(cfg["n_blocks"] - 1):
        _sanm_block(names, f"audio_encoder.encoders.{i}", d, d, f, k)
    for i in range(cfg["n_tp_blocks"]):
        _sanm_block(names, f"audio_encoder.tp_encoders.{i}", d, d, f, k)
    _ln(names, "audio_encoder.after_norm", d)
    _ln(names, "audio_encoder.tp_norm", d)
    _adaptor(names, "audio_adaptor", d, cfg["d_llm"], cfg["adaptor_ffn"], cfg["adaptor_blocks"])
    _adaptor(names, "ctc_decoder", d, d, cfg["ctc_ffn"], cfg["ctc_blocks"])
    _lin(names, "ctc_proj.ctc_lo", d, cfg["ctc_vocab"])
    return names


def llm_tensors(cfg):
    """(name, shape[out,in], scale, offset) in GGUF naming (qwen3 arch). Norms stay F32; every
    2-D tensor is stored q8_0 (convert_hf_to_gguf.py:564-565, 622-623)."""
    E, H, KV, D, F = cfg["n_embd"], cfg["n_head"], cfg["n_head_kv"], cfg["head_dim"], cfg["n_ff"]
    s = lambda n_in: math.sqrt(3.0 / n_in)
    names = [("token_embd.weight", (cfg["n_vocab"], E), 0.05, 0.0)]
    for l in range(cfg["n_layer"]):
        b = f"blk.{l}."
        names += [
            (b + "attn_norm.weight", (E,), 0.1, 1.0),
            (b + "attn_q.weight", (H * D, E), s(E), 0.0),
            (b + "attn_k.weight", (KV * D, E), s(E), 0.0),
            (b + "attn_v.weight", (KV * D, E), s(E), 0.0),
            (b + "attn_q_norm.weight", (D,), 0.1, 1.0),
            (b + "attn_k_norm.weight", (D,), 0.1, 1.0),
            (b + "attn_output.weight", (E, H * D), s(H * D), 0.0),
            (b + "ffn_norm.weight", (E,), 0.1, 1.0),
            (b + "ffn_gate.weight", (F, E), s(E), 0.0),
            (b + "ffn_up.weight", (F, E), s(E), 0.0),
            (b + "ffn_down.weight", (E, F), s(F), 0.0),
        ]
    names.append(("output_norm.weight", (E,), 0.1, 1.0))
    return names


def make_weights(table, seed=0, only=None):
    out = {}
    for name, shape, scale, offset in table:
        if only is not None and not only(name):
            continue
        n = int(np.prod(shape))
        out[name] = gen(name, n, scale, offset, seed).reshape(shape)
    return out
