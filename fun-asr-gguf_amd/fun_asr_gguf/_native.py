"""ctypes binding of libfunasr_hip.so (include/funasr_hip.h).

This is the product's only compute path: if the library (built in-tree by __graft_entry__.build())
is missing, every call raises — there is no CPU fallback.
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("FUNASR_HIP_LIB", os.path.join(os.path.dirname(_HERE), "lib", "libfunasr_hip.so"))

EXPORTS = [
    "fa_engine_create", "fa_engine_destroy", "fa_last_error", "fa_set_log_callback", "fa_weights_synthetic",
    "fa_set_tensor_f32", "fa_set_tensor_q8_0", "fa_load_gguf", "fa_get_tensor_q8_0", "fa_encode",
    "fa_encode_device", "fa_encode_fetch", "fa_ctc_collapse", "fa_set_debug", "fa_encode_tap", "fa_embd_rows",
    "fa_llm_reset", "fa_llm_prefill", "fa_llm_prefill_batch", "fa_llm_generate", "fa_llm_generate_begin",
    "fa_llm_generate_end", "fa_llm_logits", "fa_llm_n_past", "fa_profile_enable",
    "fa_profile_read", "fa_synchronize", "fa_align_timestamps", "fa_pcm_upload", "fa_set_encoder_fp16",
    "fa_get_tensor_f32", "fa_fuzzy_substring_distance", "fa_set_decode_fused", "fa_set_encoder_gemm",
    "fa_vocab_load_gguf", "fa_vocab_free", "fa_vocab_info", "fa_tokenize", "fa_token_piece", "fa_gguf_read_tensor",
    "fa_weights_mark_unset", "fa_tensor_names", "fa_llm_set_token",
    "fa_llm_invariant_width", "fa_set_encode_mode", "fa_ctc_head", "fa_set_tensor_u8dq", "fa_set_ctc_int8",
    "fa_ctc_int8_active", "fa_comm_unique_id", "fa_comm_init", "fa_comm_allgather_sizes", "fa_comm_allgather_bytes",
    "fa_comm_destroy", "fa_llm_prefill_rows", "fa_encode_generation", "fa_llm_decode_recoveries",
]


class EncoderConfig(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in (
        "n_mels", "lfr_m", "lfr_n", "d_in", "d_model", "n_heads", "d_ffn", "n_blocks", "n_tp_blocks", "fsmn_k",
        "d_llm", "adaptor_ffn", "adaptor_blocks", "adaptor_heads", "ctc_blocks", "ctc_heads", "ctc_ffn", "ctc_vocab")]


class LlmConfig(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in (
        "n_layer", "n_embd", "n_head", "n_head_kv", "head_dim", "n_ff", "n_vocab", "n_ctx", "max_seqs")] + [
        ("rope_theta", ctypes.c_float), ("rms_eps", ctypes.c_float)]


class Sampling(ctypes.Structure):
    _fields_ = [("temperature", ctypes.c_float), ("top_p", ctypes.c_float), ("top_k", ctypes.c_int32),
                ("seed", ctypes.c_uint32)]


_lib = None
LOG_CB = ctypes.CFUNCTYPE(None, ctypes.c_int32, ctypes.c_char_p, ctypes.c_void_p)


def load():
    """Load the engine library; raises if it is absent or does not export the full C-ABI."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"libfunasr_hip.so not found at {LIB_PATH}: run __graft_entry__.build() first")
    lib = ctypes.CDLL(LIB_PATH)
    missing = [s for s in EXPORTS if not hasattr(lib, s)]
    if missing:
        raise RuntimeError(f"libfunasr_hip.so lacks symbols {missing}")
    P, I32, I64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64
    lib.fa_last_error.restype = ctypes.c_char_p
    lib.fa_engine_create.argtypes = [I32, ctypes.POINTER(EncoderConfig), ctypes.POINTER(LlmConfig), I32, I64,
                                     ctypes.POINTER(P)]
    lib.fa_engine_destroy.argtypes = [P]
    lib.fa_set_log_callback.argtypes = [LOG_CB, P]
    lib.fa_weights_synthetic.argtypes = [P, ctypes.c_uint32]
    lib.fa_set_tensor_f32.argtypes = [P, ctypes.c_char_p, P, I64]
    lib.fa_set_tensor_q8_0.argtypes = [P, ctypes.c_char_p, P, I64]
    lib.fa_set_tensor_u8dq.argtypes = [P, ctypes.c_char_p, P, P, P, I64, I64]
    lib.fa_set_ctc_int8.argtypes = [P, I32]
    lib.fa_ctc_int8_active.argtypes = [P, P]
    lib.fa_comm_unique_id.argtypes = [P]
    lib.fa_comm_init.argtypes = [P, I32, I32, P]
    lib.fa_comm_allgather_sizes.argtypes = [P, I64, P]
    lib.fa_comm_allgather_bytes.argtypes = [P, P, I64, I64, P]
    lib.fa_comm_destroy.argtypes = [P]
    lib.fa_get_tensor_q8_0.argtypes = [P, ctypes.c_char_p, P, I64]
    lib.fa_get_tensor_f32.argtypes = [P, ctypes.c_char_p, P, I64]
    lib.fa_weights_mark_unset.argtypes = [P, ctypes.c_char_p]
    lib.fa_tensor_names.argtypes = [P, ctypes.c_char_p, I32, P, I64, ctypes.POINTER(I64)]
    lib.fa_load_gguf.argtypes = [P, ctypes.c_char_p]
    lib.fa_encode.argtypes = [P, P, P, I32, I64, P, I64, P, I64, P, P, P]
    lib.fa_encode_device.argtypes = [P, P, P, I32, I64]
    lib.fa_encode_fetch.argtypes = [P, P, I64, P, I64, P, P, P]
    lib.fa_ctc_collapse.argtypes = [P, I32, P, P, I64, P]
    lib.fa_ctc_head.argtypes = [P, P, I32, P]
    lib.fa_set_debug.argtypes = [P, I32]
    lib.fa_set_encoder_fp16.argtypes = [P, I32]
    lib.fa_set_decode_fused.argtypes = [P, I32]
    lib.fa_set_encoder_gemm.argtypes = [P, I32]
    lib.fa_set_encode_mode.argtypes = [P, I32]
    lib.fa_encode_tap.argtypes = [P, I32, P, I64]
    lib.fa_embd_rows.argtypes = [P, P, I32, I32, P]
    lib.fa_llm_reset.argtypes = [P, I32]
    lib.fa_llm_prefill.argtypes = [P, I32, P, I32, ctypes.POINTER(Sampling), P, P]
    lib.fa_llm_generate.argtypes = [P, P, I32, I32, ctypes.POINTER(Sampling), P]
    lib.fa_llm_generate_begin.argtypes = [P, P, I32, I32, ctypes.POINTER(Sampling)]
    lib.fa_llm_generate_end.argtypes = [P, P]
    lib.fa_llm_prefill_batch.argtypes = [P, P, I32, P, P, ctypes.POINTER(Sampling), P]
    lib.fa_llm_prefill_rows.argtypes = [P, P, I32, P, I32, P, P, I64, ctypes.POINTER(Sampling), P]
    lib.fa_encode_generation.argtypes = [P, P]
    lib.fa_llm_logits.argtypes = [P, I32, P]
    lib.fa_llm_set_token.argtypes = [P, I32, I32]
    lib.fa_llm_invariant_width.argtypes = [P, ctypes.c_void_p]
    lib.fa_llm_decode_recoveries.argtypes = [P, P, P]
    lib.fa_llm_n_past.argtypes = [P, I32, P]
    lib.fa_profile_enable.argtypes = [P, I32]
    lib.fa_profile_read.argtypes = [P, I32, P, P, P, P]
    lib.fa_synchronize.argtypes = [P]
    lib.fa_align_timestamps.argtypes = [P, P, I32, P, I32, P, P]
    lib.fa_pcm_upload.argtypes = [P, P, I64]
    lib.fa_vocab_load_gguf.argtypes = [ctypes.c_char_p, ctypes.POINTER(P)]
    lib.fa_vocab_free.argtypes = [P]
    lib.fa_vocab_info.argtypes = [P, P, P]
    lib.fa_tokenize.argtypes = [P, ctypes.c_char_p, I32, I32, P, I32, P]
    lib.fa_token_piece.argtypes = [P, I32, ctypes.c_char_p, I32, P]
    lib.fa_gguf_read_tensor.argtypes = [ctypes.c_char_p, ctypes.c_char_p, I32, P, I64]
    lib.fa_fuzzy_substring_distance.argtypes = [P, I32, P, I32, P]
    _lib = lib
    return lib


def _ptr(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def _check(rc, what):
    if rc != 0:
        raise RuntimeError(f"{what} failed ({rc}): {_lib.fa_last_error().decode(errors='replace')}")


ENC_FIELDS = [f for f, _ in EncoderConfig._fields_]
LLM_INT_FIELDS = ["n_layer", "n_embd", "n_head", "n_head_kv", "head_dim", "n_ff", "n_vocab", "n_ctx", "max_seqs"]


class Engine:
    """One device-bound engine (one per GPU). Owns all device memory; explicit close()."""

    def __init__(self, enc_cfg, llm_cfg, max_batch=1, max_samples=16000 * 62, device=0):
        lib = load()
        self.enc_cfg = dict(enc_cfg)
        self.llm_cfg = dict(llm_cfg)
        self.llm_cfg.setdefault("n_ctx", 2048)
        self.llm_cfg.setdefault("max_seqs", 1)
        ec = EncoderConfig(**{k: int(self.enc_cfg[k]) for k in ENC_FIELDS})
        lc = LlmConfig(**{k: int(self.llm_cfg[k]) for k in LLM_INT_FIELDS}, rope_theta=float(self.llm_cfg["rope_theta"]),
                       rms_eps=float(self.llm_cfg["rms_eps"]))
        h = ctypes.c_void_p()
        _check(lib.fa_engine_create(device, ctypes.byref(ec), ctypes.byref(lc), max_batch, max_samples, ctypes.byref(h)),
               "fa_engine_create")
        self.h = h
        self.max_batch = max_batch
        self.max_samples = max_samples
        self.lib = lib
        self.weights_gen = 0  # bumped by every weight change (host-side caches of weight-derived rows key on it)

    def close(self):
        if getattr(self, "h", None):
            if getattr(self, "comm_world", 0):
                self.lib.fa_comm_destroy(self.h)
                self.comm_world = 0
            self.lib.fa_engine_destroy(self.h)
            self.h = None

    # ---- result gather over RCCL (fa_comm_*)
    @staticmethod
    def comm_unique_id():
        """128-byte RCCL id, created on rank 0 and handed to every rank (fa_comm_unique_id)."""
        lib = load()
        buf = np.zeros(128, np.uint8)
        _check(lib.fa_comm_unique_id(_ptr(buf)), "fa_comm_unique_id")
        return buf.tobytes()

    def comm_init(self, rank, world, uid):
        """Join this engine to an RCCL communicator of `world` ranks (fa_comm_init)."""
        b = np.frombuffer(bytes(uid), np.uint8).copy()
        assert b.size == 128
        _check(self.lib.fa_comm_init(self.h, rank, world, _ptr(b)), "fa_comm_init")
        self.comm_rank, self.comm_world = rank, world

    def comm_allgather(self, payload):
        """Every rank's bytes, in rank order (two RCCL all-gathers: the sizes, then the padded payloads)."""
        data = np.frombuffer(bytes(payload), np.uint8).copy() if payload else np.zeros(1, np.uint8)
        n = len(payload)
        sizes = np.zeros(self.comm_world, np.int64)
        _check(self.lib.fa_comm_allgather_sizes(self.h, n, _ptr(sizes)), "fa_comm_allgather_sizes")
        slot = max(1, int(sizes.max()))
        out = np.zeros(slot * self.comm_world, np.uint8)
        _check(self.lib.fa_comm_allgather_bytes(self.h, _ptr(data), n, slot, _ptr(out)), "fa_comm_allgather_bytes")
        return [out[r * slot: r * slot + int(sizes[r])].tobytes() for r in range(self.comm_world)]

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- weights
    def set_encoder_fp16(self, on=True):
        """fp16 encoder graph (the reference's *.fp16.onnx, 02-Quantize-ONNX.py:13-27); fp32 when off."""
        _check(self.lib.fa_set_encoder_fp16(self.h, 1 if on else 0), "fa_set_encoder_fp16")

    def set_encoder_gemm(self, mode="bf16x3"):
        """fp32-graph GEMM arithmetic: "bf16x3" (default, split operands on the bf16 matrix cores) or "f32"."""
        _check(self.lib.fa_set_encoder_gemm(self.h, {"f32": 0, "bf16x3": 1}[mode]), "fa_set_encoder_gemm")

    def set_decode_fused(self, on=True):
        """Batch-1 decode layer: True / 1 the two-launch fused layer (default), 2 the three-launch fused layer,
        False / 0 the 5-launch layer."""
        mode = int(on) if not isinstance(on, bool) else (1 if on else 0)
        _check(self.lib.fa_set_decode_fused(self.h, mode), "fa_set_decode_fused")

    def synthetic_weights(self, seed=0):
        _check(self.lib.fa_weights_synthetic(self.h, seed), "fa_weights_synthetic")
        self.weights_gen += 1

    def set_tensor(self, name, arr):
        a = np.ascontiguousarray(arr, dtype=np.float32)
        _check(self.lib.fa_set_tensor_f32(self.h, name.encode(), _ptr(a), a.size), f"fa_set_tensor_f32({name})")
        self.weights_gen += 1

    def set_tensor_q8_0(self, name, blocks):
        b = np.ascontiguousarray(blocks, dtype=np.uint8)
        _check(self.lib.fa_set_tensor_q8_0(self.h, name.encode(), _ptr(b), b.size), f"fa_set_tensor_q8_0({name})")
        self.weights_gen += 1

    def set_tensor_u8dq(self, name, q, scale, zero_point):
        """One CTC-graph linear in onnxruntime dynamic-quant form (Fun-ASR-Nano-CTC.int8.onnx): q [out][in] uint8,
        scale [out] f32, zero_point [out] uint8 (fa_set_tensor_u8dq). With every CTC linear set, the CTC head runs the
        int8-dynamic graph."""
        q = np.ascontiguousarray(q, dtype=np.uint8)
        sc = np.ascontiguousarray(scale, dtype=np.float32).ravel()
        zp = np.ascontiguousarray(zero_point, dtype=np.uint8).ravel()
        assert q.ndim == 2 and sc.size == zp.size == q.shape[0]
        _check(self.lib.fa_set_tensor_u8dq(self.h, name.encode(), _ptr(q), _ptr(sc), _ptr(zp), q.shape[0], q.shape[1]),
               f"fa_set_tensor_u8dq({name})")
        self.weights_gen += 1

    def set_ctc_int8(self, on=True):
        """Run the int8-dynamic CTC graph once its weights are set (default), or the f32 / fp16 graph."""
        _check(self.lib.fa_set_ctc_int8(self.h, 1 if on else 0), "fa_set_ctc_int8")

    def ctc_int8_active(self):
        v = ctypes.c_int32()
        _check(self.lib.fa_ctc_int8_active(self.h, ctypes.byref(v)), "fa_ctc_int8_active")
        return bool(v.value)

    def get_tensor_q8_0(self, name, n_elements):
        out = np.empty(n_elements // 32 * 34, np.uint8)
        _check(self.lib.fa_get_tensor_q8_0(self.h, name.encode(), _ptr(out), out.size), "fa_get_tensor_q8_0")
        return out

    def get_tensor_f32(self, name, n_elements):
        out = np.empty(n_elements, np.float32)
        _check(self.lib.fa_get_tensor_f32(self.h, name.encode(), _ptr(out), out.size), "fa_get_tensor_f32")
        return out

    def mark_unset(self, prefix=""):
        """Clear the loaded mark of every tensor under `prefix` (fa_weights_mark_unset)."""
        _check(self.lib.fa_weights_mark_unset(self.h, prefix.encode()), "fa_weights_mark_unset")

    def tensor_names(self, prefix="", only_unset=False):
        """Engine tensor names under `prefix` in registration order; only those not loaded since the last
        mark_unset() when only_unset (fa_tensor_names)."""
        need = ctypes.c_int64()
        _check(self.lib.fa_tensor_names(self.h, prefix.encode(), int(only_unset), None, 0, ctypes.byref(need)),
               "fa_tensor_names")
        buf = ctypes.create_string_buffer(need.value)
        _check(self.lib.fa_tensor_names(self.h, prefix.encode(), int(only_unset), buf, need.value, ctypes.byref(need)),
               "fa_tensor_names")
        s = buf.value.decode()
        return s.split("\n") if s else []

    def load_gguf(self, path):
        _check(self.lib.fa_load_gguf(self.h, os.fspath(path).encode()), "fa_load_gguf")
        self.weights_gen += 1

    # ---- encoder
    @staticmethod
    def frame_counts(n):
        t_mel = n // 160 + 1
        t_lfr = (t_mel + 5) // 6
        o1 = 1 + (t_lfr - 3 + 2) // 2
        tgt = (1 + (o1 - 3 + 2) // 2 - 1) // 2 + 1
        ctc_len = ((max(n, 16000) // 160 + 1) + 5) // 6
        return t_lfr, tgt, ctc_len

    @staticmethod
    def _pack(clips):
        B = len(clips)
        stride = max(max(len(c) for c in clips), 1)
        pcm = np.zeros((B, stride), np.float32)
        for i, c in enumerate(clips):
            pcm[i, :len(c)] = c
        return pcm, np.array([len(c) for c in clips], np.int64)

    def upload(self, clips):
        """Make clips resident in the engine's HBM PCM buffer; -> handle for encode(resident=handle)."""
        pcm, ns = self._pack(clips)
        _check(self.lib.fa_pcm_upload(self.h, _ptr(pcm), pcm.size), "fa_pcm_upload")
        return dict(ns=ns, stride=pcm.shape[1])

    def encode(self, clips, want_enc=False, debug_lfr=False, resident=None, independent=False):
        """clips: list of 1-D float32 arrays (or resident=upload() handle, clips = their lengths only).
        independent: every clip gets its single-clip encode (concurrent lanes, fa_set_encode_mode(1)) instead of one
        padded batch. Returns dict(audio_embd=[...], ctc_ids=[...], t_lfr, target_len[, enc, lfr_embedded])."""
        if independent:
            _check(self.lib.fa_set_encode_mode(self.h, 1), "fa_set_encode_mode")
            try:
                return self.encode(clips, want_enc, debug_lfr, resident)
            finally:
                _check(self.lib.fa_set_encode_mode(self.h, 0), "fa_set_encode_mode")
        if resident is not None:
            ns, stride, pcm = resident["ns"], resident["stride"], None
        else:
            pcm, ns = self._pack(clips)
            stride = pcm.shape[1]
        B = len(ns)
        assert 1 <= B <= self.max_batch
        counts = [self.frame_counts(int(n)) for n in ns]
        tgt_stride = max(c[1] for c in counts)
        ids_stride = max(c[2] for c in counts)
        d_llm, d = self.enc_cfg["d_llm"], self.enc_cfg["d_model"]
        emb = np.empty((B, tgt_stride, d_llm), np.float32)
        ids = np.empty((B, ids_stride), np.int32)
        tl = np.zeros(B, np.int32)
        tg = np.zeros(B, np.int32)
        enc = np.zeros((B, ids_stride, d), np.float32) if want_enc else None
        if debug_lfr:
            _check(self.lib.fa_set_debug(self.h, 1), "fa_set_debug")
        if pcm is None:
            _check(self.lib.fa_encode_device(self.h, None, _ptr(ns), B, stride), "fa_encode_device")
            _check(self.lib.fa_encode_fetch(self.h, _ptr(emb), tgt_stride, _ptr(ids), ids_stride, _ptr(tl), _ptr(tg),
                                            _ptr(enc)), "fa_encode_fetch")
        else:
            _check(self.lib.fa_encode(self.h, _ptr(pcm), _ptr(ns), B, stride, _ptr(emb), tgt_stride, _ptr(ids),
                                      ids_stride, _ptr(tl), _ptr(tg), _ptr(enc)), "fa_encode")
        out = dict(audio_embd=[emb[b, :tg[b]] for b in range(B)], ctc_ids=[ids[b, :tl[b]] for b in range(B)],
                   t_lfr=tl, target_len=tg, enc_gen=self.encode_generation())
        if want_enc:
            out["enc"] = [enc[b, :tl[b]] for b in range(B)]
        if debug_lfr:
            t0 = counts[0][2]
            lfr = np.zeros((max(c[2] for c in counts), self.enc_cfg["d_in"]), np.float32)
            _check(self.lib.fa_encode_tap(self.h, 0, _ptr(lfr), lfr.size), "fa_encode_tap")
            out["lfr_embedded"] = lfr[:t0]
            _check(self.lib.fa_set_debug(self.h, 0), "fa_set_debug")
        return out

    def encode_generation(self):
        """Generation of the adaptor rows the last encode left in HBM (-1: none held); fa_encode_generation."""
        g = ctypes.c_int64()
        _check(self.lib.fa_encode_generation(self.h, ctypes.byref(g)), "fa_encode_generation")
        return g.value

    def ctc_head(self, enc):
        """The CTC graph alone over encoder rows enc [T, d_model] -> argmax ids [T] int32 (fa_ctc_head)."""
        enc = np.ascontiguousarray(enc, np.float32)
        ids = np.zeros(enc.shape[0], np.int32)
        _check(self.lib.fa_ctc_head(self.h, _ptr(enc), enc.shape[0], _ptr(ids)), "fa_ctc_head")
        return ids

    def ctc_collapse(self, blank_id, n_clips):
        stride = self.frame_counts(self.max_samples)[2] + 1
        ids = np.zeros((n_clips, stride), np.int32)
        fr = np.zeros((n_clips, stride), np.int32)
        n = np.zeros(n_clips, np.int32)
        _check(self.lib.fa_ctc_collapse(self.h, blank_id, _ptr(ids), _ptr(fr), stride, _ptr(n)), "fa_ctc_collapse")
        return [(ids[b, :n[b]], fr[b, :n[b]]) for b in range(n_clips)]

    # ---- decoder
    def embd_rows(self, ids, fp16_round=True):
        ids = np.ascontiguousarray(ids, dtype=np.int32)
        out = np.empty((ids.size, self.llm_cfg["n_embd"]), np.float32)
        _check(self.lib.fa_embd_rows(self.h, _ptr(ids), ids.size, 1 if fp16_round else 0, _ptr(out)), "fa_embd_rows")
        return out

    def llm_reset(self, seq=0):
        _check(self.lib.fa_llm_reset(self.h, seq), "fa_llm_reset")

    @staticmethod
    def _sampling(temperature=0.0, top_k=50, top_p=1.0, seed=0):
        return Sampling(temperature=float(temperature), top_p=float(top_p), top_k=int(top_k), seed=int(seed) & 0xFFFFFFFF)

    def llm_prefill(self, seq, embd, want_logits=False, **samp):
        e = np.ascontiguousarray(embd, dtype=np.float32)
        tok = ctypes.c_int32()
        lg = np.empty(self.llm_cfg["n_vocab"], np.float32) if want_logits else None
        s = self._sampling(**samp)
        _check(self.lib.fa_llm_prefill(self.h, seq, _ptr(e), e.shape[0], ctypes.byref(s), ctypes.byref(tok), _ptr(lg)),
               "fa_llm_prefill")
        return (tok.value, lg) if want_logits else tok.value

    def llm_prefill_batch(self, seqs, embds, **samp):
        """Prefill several sequences in shared forwards (fa_llm_prefill_batch); -> first tokens, one per sequence."""
        seqs = np.ascontiguousarray(seqs, dtype=np.int32)
        n = np.array([e.shape[0] for e in embds], np.int32)
        e = np.ascontiguousarray(np.concatenate(embds, 0), dtype=np.float32)
        tok = np.zeros(len(seqs), np.int32)
        s = self._sampling(**samp)
        _check(self.lib.fa_llm_prefill_batch(self.h, _ptr(seqs), len(seqs), _ptr(e), _ptr(n), ctypes.byref(s), _ptr(tok)),
               "fa_llm_prefill_batch")
        return tok.tolist()

    def llm_prefill_rows(self, seqs, prompts, **samp):
        """llm_prefill (one prompt) / llm_prefill_batch with every prompt's audio rows read where the last encode
        left them (fa_llm_prefill_rows). prompts: objects with .pre / .suf (host rows [n, n_embd]), .clip (the clip's
        index in that encode), .n_audio and .enc_gen (core/decoder.PromptRows). The distinct prefix / suffix arrays
        are uploaded once. -> first tokens, one per sequence."""
        seqs = np.ascontiguousarray(seqs, dtype=np.int32)
        blocks, offs, codes = [], {}, []
        gen = None
        for p in prompts:
            part = []
            for arr in (p.pre, None, p.suf):
                if arr is None:
                    part.append(-1 - ((p.clip << 16) | np.arange(p.n_audio, dtype=np.int32)))
                    continue
                if len(arr) == 0:
                    continue
                k = id(arr)
                if k not in offs:
                    offs[k] = sum(len(b) for b in blocks)
                    blocks.append(arr)
                part.append(offs[k] + np.arange(len(arr), dtype=np.int32))
            codes.append(np.concatenate(part).astype(np.int32))
            gen = p.enc_gen if gen is None else gen
            assert p.enc_gen == gen, "prompts of different encodes"
        n = np.array([len(c) for c in codes], np.int32)
        rs = np.ascontiguousarray(np.concatenate(codes))
        host = np.ascontiguousarray(np.concatenate(blocks, 0), np.float32) if blocks else None
        tok = np.zeros(len(seqs), np.int32)
        s = self._sampling(**samp)
        _check(self.lib.fa_llm_prefill_rows(self.h, _ptr(seqs), len(seqs), _ptr(host), 0 if host is None else len(host),
                                            _ptr(rs), _ptr(n), int(gen), ctypes.byref(s), _ptr(tok)),
               "fa_llm_prefill_rows")
        return tok.tolist()

    def llm_generate(self, seqs, n_steps, **samp):
        sq = np.ascontiguousarray(seqs, dtype=np.int32)
        out = np.empty((sq.size, n_steps), np.int32)
        s = self._sampling(**samp)
        _check(self.lib.fa_llm_generate(self.h, _ptr(sq), sq.size, n_steps, ctypes.byref(s), _ptr(out)),
               "fa_llm_generate")
        return out

    def llm_generate_begin(self, seqs, n_steps, **samp):
        """Enqueue n_steps decode steps for `seqs` and return at once (fa_llm_generate_begin); the tokens come from
        llm_generate_end(). The host may process earlier tokens in between."""
        sq = np.ascontiguousarray(seqs, dtype=np.int32)
        s = self._sampling(**samp)
        _check(self.lib.fa_llm_generate_begin(self.h, _ptr(sq), sq.size, n_steps, ctypes.byref(s)), "fa_llm_generate_begin")
        self._gen_shape = (sq.size, n_steps)
        return self._gen_shape

    def llm_generate_end(self):
        out = np.empty(self._gen_shape, np.int32)
        _check(self.lib.fa_llm_generate_end(self.h, _ptr(out)), "fa_llm_generate_end")
        return out

    def llm_invariant_width(self):
        """Largest decode batch width with single-sequence arithmetic per token (fa_llm_invariant_width)."""
        v = ctypes.c_int32()
        _check(self.lib.fa_llm_invariant_width(self.h, ctypes.byref(v)), "fa_llm_invariant_width")
        return v.value

    def llm_decode_recoveries(self):
        """(retries, fallbacks): decode chunks re-run on the fused layer after an in-launch timeout (results unchanged)
        and chunks that ran on the 5-launch layer instead (noise-floor agreement only); fa_llm_decode_recoveries."""
        r, f = ctypes.c_int32(), ctypes.c_int32()
        _check(self.lib.fa_llm_decode_recoveries(self.h, ctypes.byref(r), ctypes.byref(f)), "fa_llm_decode_recoveries")
        return r.value, f.value

    def llm_set_token(self, seq, token):
        """Feed `token` as the sequence's next generate input instead of its own last draw (teacher forcing)."""
        _check(self.lib.fa_llm_set_token(self.h, seq, int(token)), "fa_llm_set_token")

    def llm_logits(self, seq=0):
        """Logits of `seq`'s row in the most recent forward (prefill or generate step) that included it."""
        out = np.empty(self.llm_cfg["n_vocab"], np.float32)
        _check(self.lib.fa_llm_logits(self.h, seq, _ptr(out)), "fa_llm_logits")
        return out

    def llm_n_past(self, seq=0):
        v = ctypes.c_int32()
        _check(self.lib.fa_llm_n_past(self.h, seq, ctypes.byref(v)), "fa_llm_n_past")
        return v.value

    # ---- profiling
    def profile_enable(self, on=True):
        _check(self.lib.fa_profile_enable(self.h, 1 if on else 0), "fa_profile_enable")

    def profile_read(self, cls):
        ms, n, b, f = ctypes.c_double(), ctypes.c_int64(), ctypes.c_double(), ctypes.c_double()
        _check(self.lib.fa_profile_read(self.h, cls, ctypes.byref(ms), ctypes.byref(n), ctypes.byref(b), ctypes.byref(f)),
               "fa_profile_read")
        return dict(ms=ms.value, launches=n.value, bytes=b.value, flops=f.value)

    def synchronize(self):
        _check(self.lib.fa_synchronize(self.h), "fa_synchronize")


class Vocab:
    """Native GGUF tokenizer (fa_vocab): llama_tokenize(add_special=False, parse_special=True) and
    llama_token_to_piece(special=True) of the reference (llama.py:738-748)."""

    def __init__(self, gguf_path):
        lib = load()
        h = ctypes.c_void_p()
        _check(lib.fa_vocab_load_gguf(os.fspath(gguf_path).encode(), ctypes.byref(h)), "fa_vocab_load_gguf")
        self.h, self.lib = h, lib
        n, eos = ctypes.c_int32(), ctypes.c_int32()
        _check(lib.fa_vocab_info(h, ctypes.byref(n), ctypes.byref(eos)), "fa_vocab_info")
        self.n_vocab, self.eos = n.value, eos.value

    def close(self):
        if getattr(self, "h", None):
            self.lib.fa_vocab_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def tokenize(self, text, parse_special=True):
        b = text.encode("utf-8")
        cap = len(b) + 32
        out = np.empty(cap, np.int32)
        n = ctypes.c_int32()
        _check(self.lib.fa_tokenize(self.h, b, len(b), 1 if parse_special else 0, _ptr(out), cap, ctypes.byref(n)),
               "fa_tokenize")
        return [int(t) for t in out[:n.value]]

    def token_to_bytes(self, tid):
        buf = ctypes.create_string_buffer(256)
        n = ctypes.c_int32()
        rc = self.lib.fa_token_piece(self.h, int(tid), buf, 256, ctypes.byref(n))
        if rc != 0 and n.value > 256:
            buf = ctypes.create_string_buffer(n.value)
            rc = self.lib.fa_token_piece(self.h, int(tid), buf, n.value, ctypes.byref(n))
        _check(rc, "fa_token_piece")
        return buf.raw[:n.value]


def gguf_read_tensor(path, name, n_elements, fp16_product=False):
    """Dequantised GGUF tensor (q8_0 / f16 / f32) as f32 (get_token_embeddings_gguf, llama.py:751-796)."""
    lib = load()
    out = np.empty(n_elements, np.float32)
    _check(lib.fa_gguf_read_tensor(os.fspath(path).encode(), name.encode(), 1 if fp16_product else 0, _ptr(out),
                                   n_elements), "fa_gguf_read_tensor")
    return out


def fuzzy_substring_distance(main_codes, sub_codes):
    """FastRAG coarse distance (rag_fast.py:35-77) on int32 phoneme codes."""
    lib = load()
    a = np.ascontiguousarray(main_codes, np.int32)
    b = np.ascontiguousarray(sub_codes, np.int32)
    d = ctypes.c_float()
    _check(lib.fa_fuzzy_substring_distance(_ptr(a), a.size, _ptr(b), b.size, ctypes.byref(d)),
           "fa_fuzzy_substring_distance")
    return d.value
