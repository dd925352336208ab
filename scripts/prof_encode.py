"""Encoder-only runs (full Fun-ASR-Nano encoder/adaptor/CTC dims, synthetic weights) for kernel profiling:
  rocprofv3 --kernel-trace --stats -d gpurun_out/pe -o run -- python scripts/prof_encode.py [batch] [reps] [fp16|f32|bf16x3]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "fun-asr-gguf_amd")]
from oracle import synth  # noqa: E402  (config dicts only)
from fun_asr_gguf import _native  # noqa: E402
from fun_asr_gguf.synthetic import synth_audio  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
fp16 = len(sys.argv) > 3 and sys.argv[3] == "fp16"
gemm = sys.argv[3] if len(sys.argv) > 3 and sys.argv[3] in ("f32", "bf16x3") else "bf16x3"
eng = _native.Engine(synth.ENC_FULL, dict(synth.LLM_TINY, n_ctx=256, max_seqs=1), max_batch=B, max_samples=16000 * 60)
eng.synthetic_weights(0)
eng.set_encoder_fp16(fp16)
eng.set_encoder_gemm(gemm)
clips = [synth_audio(16000 * 60, i) for i in range(B)]
h = eng.upload(clips)
eng.encode(clips, resident=h)
eng.synchronize()
t = time.perf_counter()
for _ in range(reps):
    eng.encode(clips, resident=h)
eng.synchronize()
dt = (time.perf_counter() - t) / reps
print(f"encode batch {B} x 60 s ({'fp16' if fp16 else 'fp32 ' + gemm}): {dt * 1e3:.2f} ms per call, {dt * 1e3 / B:.2f} ms per clip")
if os.environ.get("ENC_HASH"):  # bit-identity check across builds / settings: hash of every clip's encoder rows
    import hashlib
    import numpy as np
    out = eng.encode(clips, resident=h, want_enc=True)
    hs = hashlib.sha256()
    for e in out["enc"]:
        hs.update(np.ascontiguousarray(e).tobytes())
    print(f"encoder rows hash: {hs.hexdigest()[:16]}")
eng.close()
