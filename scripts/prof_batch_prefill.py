"""Multi-sequence prefill (fa_llm_prefill_batch) on the full Qwen3-0.6B q8_0 shape, for kernel profiling:
  rocprofv3 --kernel-trace -d gpurun_out/pp -o run -- python scripts/prof_batch_prefill.py 32 204"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "fun-asr-gguf_amd")]
import numpy as np  # noqa: E402
from oracle import synth  # noqa: E402  (config dicts only)
from fun_asr_gguf import _native  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
T = int(sys.argv[2]) if len(sys.argv) > 2 else 204
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
eng = _native.Engine(synth.ENC_TINY, dict(synth.LLM_FULL, n_ctx=512, max_seqs=B), max_batch=1, max_samples=16000)
eng.synthetic_weights(0)
rng = np.random.default_rng(0)
prompts = [(rng.standard_normal((T, 1024)) * 0.05).astype(np.float32) for _ in range(B)]
for r in range(reps + 1):
    for s in range(B):
        eng.llm_reset(s)
    eng.synchronize()
    t = time.perf_counter()
    eng.llm_prefill_batch(list(range(B)), prompts, temperature=0.0)
    eng.synchronize()
    if r:
        print(f"prefill batch {B} x {T} rows: {(time.perf_counter() - t) * 1e3:.2f} ms", flush=True)
import hashlib  # noqa: E402
h = hashlib.sha256(b"".join(eng.llm_logits(s).tobytes() for s in sorted({0, B // 2, B - 1}))).hexdigest()[:16]
print(f"logits hash (sequences 0, {B // 2}, {B - 1}): {h}")
eng.close()
