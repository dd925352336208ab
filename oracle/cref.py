"""ctypes wrapper of oracle/_build/libcref.so (oracle/cref/cref.cpp) — TEST INFRASTRUCTURE ONLY.

The C++/OpenMP restatement of the encoder (oracle/encoder.py) and of the q8_0 Qwen3 decoder (oracle/qwen3.py) on
synthetic weights (oracle/synth.py): fast enough to serve as the full-size oracle of the GPU parity tests (60 s
clips, 28 layers / 151936 vocab) and as bench.py's CPU baseline. Pinned against the numpy oracle and the
reference goldens in tests/test_cref.py. Built by `make -C oracle` (__graft_entry__.build()).
"""
import ctypes
import os

import numpy as np

from . import synth

LIB = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_build", "libcref.so")
ENC_FIELDS = ["n_mels", "lfr_m", "lfr_n", "d_in", "d_model", "n_heads", "d_ffn", "n_blocks", "n_tp_blocks", "fsmn_k",
              "d_llm", "adaptor_ffn", "adaptor_blocks", "adaptor_heads", "ctc_blocks", "ctc_heads", "ctc_ffn", "ctc_vocab"]
_lib = None


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            raise RuntimeError(f"{LIB} missing: run `make -C oracle` (or __graft_entry__.build())")
        lib = ctypes.CDLL(LIB)
        P, I32, I64, F32 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_float
        lib.cref_enc_create.restype = P
        lib.cref_enc_create.argtypes = [P, ctypes.c_uint32]
        lib.cref_enc_destroy.argtypes = [P]
        lib.cref_enc_forward.argtypes = [P, P, I64, I64, P, P, P, P, P]
        lib.cref_llm_create.restype = P
        lib.cref_llm_create.argtypes = [P, F32, F32, I32, I32, ctypes.c_uint32]
        lib.cref_llm_destroy.argtypes = [P]
        lib.cref_llm_embed.argtypes = [P, P, I32, I32, P]
        lib.cref_llm_forward.argtypes = [P, I32, P, I32, I32, I32, P]
        lib.cref_llm_tensor_q8.argtypes = [P, ctypes.c_char_p, P, I64]
        _lib = lib
    return _lib


def threads():
    return int(load().cref_threads())


def _p(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


class CEncoder:
    """oracle.encoder.encode() for one clip (CPU-EP policy: no padding beyond the clip)."""

    def __init__(self, cfg, seed=0):
        self.cfg = dict(cfg)
        self._cfg = np.array([cfg[k] for k in ENC_FIELDS], np.int32)
        self.h = load().cref_enc_create(_p(self._cfg), seed)

    def close(self):
        if self.h:
            _lib.cref_enc_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def encode(self, audio, valid=None, want_ctc=True):
        a = np.ascontiguousarray(audio, np.float32)
        valid = a.shape[0] if valid is None else int(valid)
        T = ((a.shape[0] // 160 + 1) + 5) // 6
        enc = np.empty((T, self.cfg["d_model"]), np.float32)
        ad = np.empty((T, self.cfg["d_llm"]), np.float32)
        ids = np.empty(T, np.int32) if want_ctc else None
        mg = np.empty(T, np.float32) if want_ctc else None
        tgt = np.zeros(1, np.int32)
        t = _lib.cref_enc_forward(self.h, _p(a), a.shape[0], valid, _p(enc), _p(ad), _p(ids), _p(mg), _p(tgt))
        assert t == T
        tl = int(tgt[0])
        return dict(enc=enc, adaptor=ad, audio_embd=ad[:tl], ctc_ids=ids, ctc_margin=mg, target_len=tl)


class CQwen3:
    """oracle.qwen3.Qwen3Q8 on the synthetic weights of `cfg` (seed), one KV cache per sequence slot."""

    def __init__(self, cfg, n_ctx=2048, max_seqs=1, seed=0):
        self.cfg = dict(cfg)
        self.n_ctx = n_ctx
        c = np.array([cfg["n_layer"], cfg["n_embd"], cfg["n_head"], cfg["n_head_kv"], cfg["head_dim"], cfg["n_ff"],
                      cfg["n_vocab"]], np.int32)
        self.h = load().cref_llm_create(_p(c), cfg["rope_theta"], cfg["rms_eps"], n_ctx, max_seqs, seed)

    def close(self):
        if self.h:
            _lib.cref_llm_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _embed(self, ids, fp16):
        ids = np.ascontiguousarray(ids, np.int32)
        out = np.empty((ids.size, self.cfg["n_embd"]), np.float32)
        _lib.cref_llm_embed(self.h, _p(ids), ids.size, 1 if fp16 else 0, _p(out))
        return out

    def embed_prompt(self, ids):
        return self._embed(ids, True)

    def embed_tokens(self, ids):
        return self._embed(ids, False)

    def forward(self, x, pos0, seq=0, all_logits=False):
        x = np.ascontiguousarray(x, np.float32)
        n = x.shape[0]
        out = np.empty((n if all_logits else 1, self.cfg["n_vocab"]), np.float32)
        rc = _lib.cref_llm_forward(self.h, seq, _p(x), n, pos0, 1 if all_logits else 0, _p(out))
        assert rc == 0, "cref_llm_forward: bad seq / position"
        return out if all_logits else out[0]

    def tensor_q8(self, name, n_elements):
        out = np.empty(n_elements // 32 * 34, np.uint8)
        assert _lib.cref_llm_tensor_q8(self.h, name.encode(), _p(out), out.size) == 0, name
        return out

    def greedy(self, prompt_embd, n_steps, seq=0):
        lg = self.forward(prompt_embd, 0, seq)
        pos, out = prompt_embd.shape[0], []
        for _ in range(n_steps):
            t = int(np.argmax(lg))
            out.append(t)
            lg = self.forward(self.embed_tokens([t]), pos, seq)
            pos += 1
        return out


def encoder_tiny():
    return CEncoder(synth.ENC_TINY)
