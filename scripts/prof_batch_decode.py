"""Batch-B decode steps on the full Qwen3-0.6B q8_0 shape (synthetic weights), for kernel-level profiling:
  rocprofv3 --kernel-trace --stats -d gpurun_out/pb -o run -- python scripts/prof_batch_decode.py 32
(FUNASR_GRAPHS=0 is set by the caller's environment so every launch is traced individually)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "fun-asr-gguf_amd")]
import numpy as np  # noqa: E402
from oracle import synth  # noqa: E402  (config dicts only)
from fun_asr_gguf import _native  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 32
eng = _native.Engine(synth.ENC_TINY, dict(synth.LLM_FULL, n_ctx=512, max_seqs=B), max_batch=1, max_samples=16000)
eng.synthetic_weights(0)
rng = np.random.default_rng(0)
for s in range(B):
    eng.llm_reset(s)
    eng.llm_prefill(s, (rng.standard_normal((204, 1024)) * 0.05).astype(np.float32))
eng.llm_generate(list(range(B)), 4)
eng.synchronize()
t = time.perf_counter()
eng.llm_generate(list(range(B)), steps)
eng.synchronize()
dt = time.perf_counter() - t
print(f"batch {B}: {dt / steps * 1e3:.3f} ms/step ({'graphs' if os.environ.get('FUNASR_GRAPHS', '1') != '0' else 'eager'})")
eng.close()
