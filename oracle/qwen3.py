"""Qwen3 decoder restatement with ggml q8_0 numerics — TEST INFRASTRUCTURE ONLY.

The reference runs this model inside llama.cpp b7798 (Windows DLLs only, no source in the tree;
call sites fun_asr_gguf/llama.py:257-260, 490-510, 536-570, 609-644), so the restatement follows the
published llama.cpp/ggml algorithm for arch `qwen3` (tensor set gguf/constants.py:1696-1712):

  per layer: h = rms_norm(x)*attn_norm; q,k,v = W{q,k,v} . h      (q8_0 x q8_0 integer dot)
             q,k = rms_norm_per_head(.)*{q,k}_norm; NEOX RoPE (theta 1e6, iterative f32 theta)
             K/V cache stored fp16 (llama.cpp default cache type)
             o = Wo . softmax(q.k/sqrt(128), causal) v ;  x += o
             h = rms_norm(x)*ffn_norm; x += Wdown . (silu(Wgate.h) * (Wup.h))
  logits = token_embd(q8_0, tied) . (rms_norm(x)*output_norm)

ggml rms_norm accumulates sum(x*x) in double and scales by 1/sqrtf(mean+eps) (f32). Matmul inputs
are quantised per 32-block with the reference q8_0 quantiser (q8.py). Embedding rows: prompt rows are
fp16(d*q) as produced by numpy in llama.py:778-784; generated-token rows are f32(d)*q (ggml get_rows).
"Parity unpinned" w.r.t. llama.cpp itself (absent); anchored on HF Qwen3 in tests.

Attention arithmetic. The reference creates its context with flash_attn_type = 1 (llama.py:404, 475), so llama.cpp
runs flash_attn_ext; its CPU kernel (ggml-cpu ops.cpp, ggml_compute_forward_flash_attn_ext_f16 on an f16 cache)
rounds Q to f16 for the K dot and accumulates P.V in f16 with an online softmax (y = f16(f32(y) * ms) on a new
max, y = f16(f32(y) + f32(v) * vs) per key, S in f32), while GPU backends differ again. attn="f32" (default, what
the HIP engine computes: f32 Q, f32 softmax and P.V over the fp16 cache) is the backend-neutral form;
attn="ggml_cpu_fa" restates the CPU kernel; tests/test_oracle_golden.py::test_attention_mode_below_q8_noise_floor
shows the two differ by less than the q8_0 activation noise floor the GPU tolerances are set on.
"""
import numpy as np
from . import q8


def rms_norm(x, w, eps):
    ss = (x.astype(np.float32) * x.astype(np.float32)).astype(np.float64).sum(-1, keepdims=True)
    mean = (ss / x.shape[-1]).astype(np.float32)
    scale = (np.float32(1.0) / np.sqrt(mean + np.float32(eps))).astype(np.float32)
    return ((x * scale).astype(np.float32) * w).astype(np.float32)


def rope_table(n_pos, head_dim, theta_base):
    """cos/sin [n_pos, head_dim/2] with ggml's iterative f32 theta (ggml_rope_cache_init)."""
    ts = np.float32(np.power(np.float32(theta_base), np.float32(-2.0 / head_dim)))
    cos = np.empty((n_pos, head_dim // 2), np.float32)
    sin = np.empty((n_pos, head_dim // 2), np.float32)
    theta = np.arange(n_pos, dtype=np.float32)
    for i in range(head_dim // 2):
        cos[:, i] = np.cos(theta.astype(np.float64)).astype(np.float32)
        sin[:, i] = np.sin(theta.astype(np.float64)).astype(np.float32)
        theta = (theta * ts).astype(np.float32)
    return cos, sin


def rope_neox(x, pos, cos, sin):
    """x [N, H, D]; NEOX pairs (i, i + D/2)."""
    h = x.shape[-1] // 2
    c = cos[pos][:, None, :]
    s = sin[pos][:, None, :]
    x0, x1 = x[..., :h], x[..., h:]
    return np.concatenate([x0 * c - x1 * s, x0 * s + x1 * c], -1).astype(np.float32)


def silu(x):
    return (x / (np.float32(1.0) + np.exp(-x))).astype(np.float32)


def attn_ggml_cpu_fa(q, k16, v16, scale, pos):
    """ggml-cpu flash_attn_ext over an f16 cache (see the module docstring): q [N, H, D] f32, k16 / v16 [T, KV, D]
    f16, query row n attends keys 0..pos[n]."""
    N, H, D = q.shape
    g = H // k16.shape[1]
    q16 = q.astype(np.float16).astype(np.float32)
    o = np.empty((N, H, D), np.float32)
    for n in range(N):
        T = int(pos[n]) + 1
        for hh in range(H):
            kk = k16[:T, hh // g].astype(np.float32)
            vv = v16[:T, hh // g].astype(np.float32)
            s = ((kk @ q16[n, hh]).astype(np.float32) * scale).astype(np.float32)
            M, S = np.float32(-np.inf), np.float32(0.0)
            acc = np.zeros(D, np.float16)
            for t in range(T):
                if s[t] > M:
                    ms = np.float32(np.exp(np.float32(M - s[t]))) if M != -np.inf else np.float32(0.0)
                    M, vs = s[t], np.float32(1.0)
                    acc = (acc.astype(np.float32) * ms).astype(np.float16)
                else:
                    ms, vs = np.float32(1.0), np.float32(np.exp(np.float32(s[t] - M)))
                acc = (acc.astype(np.float32) + vv[t] * vs).astype(np.float16)
                S = np.float32(S * ms + vs)
            o[n, hh] = acc.astype(np.float32) * np.float32(1.0 / S)
    return o


class Qwen3Q8:
    def __init__(self, weights, cfg, n_ctx=2048, attn="f32"):
        """weights: name -> f32 array (GGUF names); 2-D tensors are q8_0-quantised here, exactly as
        the GGUF converter does (convert_hf_to_gguf.py:622-623 -> gguf/quants.py:378-393)."""
        self.cfg = cfg
        self.q = {}
        self.f = {}
        for k, v in weights.items():
            if v.ndim == 2:
                self.q[k] = q8.quantize_q8_0(v)
            else:
                self.f[k] = v.astype(np.float32)
        self.cos, self.sin = rope_table(n_ctx, cfg["head_dim"], cfg["rope_theta"])
        self.n_ctx = n_ctx
        assert attn in ("f32", "ggml_cpu_fa")
        self.attn = attn
        self.reset()

    def reset(self):
        c = self.cfg
        kvd = c["n_head_kv"] * c["head_dim"]
        self.kc = [np.zeros((self.n_ctx, kvd), np.float16) for _ in range(c["n_layer"])]
        self.vc = [np.zeros((self.n_ctx, kvd), np.float16) for _ in range(c["n_layer"])]

    def mm(self, name, x):
        d, q = self.q[name]
        return q8.matmul_q8(d, q, x)

    def embed_prompt(self, ids):
        d, q = self.q["token_embd.weight"]
        return q8.dequant_numpy_f16(d[ids], q[ids])

    def embed_tokens(self, ids):
        d, q = self.q["token_embd.weight"]
        return q8.dequant_f32(d[ids], q[ids])

    def forward(self, x, pos0, all_logits=False):
        """x: input embeddings [N, E] at positions pos0..pos0+N-1 -> logits [V] of the last row
        (llama.py:556 sets logits only on the last batch row) or [N, V]."""
        c = self.cfg
        N = x.shape[0]
        H, KV, D, eps = c["n_head"], c["n_head_kv"], c["head_dim"], c["rms_eps"]
        pos = np.arange(pos0, pos0 + N)
        scale = np.float32(1.0 / np.sqrt(np.float32(D)))
        x = x.astype(np.float32)
        for l in range(c["n_layer"]):
            b = f"blk.{l}."
            h = rms_norm(x, self.f[b + "attn_norm.weight"], eps)
            q = self.mm(b + "attn_q.weight", h).reshape(N, H, D)
            k = self.mm(b + "attn_k.weight", h).reshape(N, KV, D)
            v = self.mm(b + "attn_v.weight", h).reshape(N, KV, D)
            q = rope_neox(rms_norm(q, self.f[b + "attn_q_norm.weight"], eps), pos, self.cos, self.sin)
            k = rope_neox(rms_norm(k, self.f[b + "attn_k_norm.weight"], eps), pos, self.cos, self.sin)
            self.kc[l][pos] = k.reshape(N, KV * D).astype(np.float16)
            self.vc[l][pos] = v.reshape(N, KV * D).astype(np.float16)
            T = pos0 + N
            K = self.kc[l][:T].astype(np.float32).reshape(T, KV, D)
            V = self.vc[l][:T].astype(np.float32).reshape(T, KV, D)
            o = np.empty((N, H, D), np.float32)
            causal = np.where(np.arange(T)[None, :] <= pos[:, None], 0.0, -np.inf).astype(np.float32)
            g = H // KV
            if self.attn == "ggml_cpu_fa":
                o = attn_ggml_cpu_fa(q, self.kc[l][:T].reshape(T, KV, D), self.vc[l][:T].reshape(T, KV, D), scale,
                                     pos)
            else:
                for hh in range(H):
                    s = (q[:, hh, :] @ K[:, hh // g, :].T) * scale + causal
                    s = s - s.max(-1, keepdims=True)
                    e = np.exp(s)
                    o[:, hh, :] = (e / e.sum(-1, keepdims=True)) @ V[:, hh // g, :]
            x = (x + self.mm(b + "attn_output.weight", o.reshape(N, H * D))).astype(np.float32)
            h = rms_norm(x, self.f[b + "ffn_norm.weight"], eps)
            a = (silu(self.mm(b + "ffn_gate.weight", h)) * self.mm(b + "ffn_up.weight", h)).astype(np.float32)
            x = (x + self.mm(b + "ffn_down.weight", a)).astype(np.float32)
        rows = x if all_logits else x[-1:]
        h = rms_norm(rows, self.f["output_norm.weight"], eps)
        lg = self.mm("token_embd.weight", h)
        return lg if all_logits else lg[0]

    def greedy(self, prompt_embd, n_steps, stop_ids=()):
        """Prefill + greedy loop (decoder.py:70-123 at temperature 0, llama.py:604-605)."""
        self.reset()
        lg = self.forward(prompt_embd, 0)
        pos = prompt_embd.shape[0]
        out = []
        for _ in range(n_steps):
            t = int(np.argmax(lg))
            out.append(t)
            lg = self.forward(self.embed_tokens([t]), pos)
            pos += 1
            if t in stop_ids:
                break
        return out
