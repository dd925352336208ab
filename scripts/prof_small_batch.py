"""Decode step time of small batches (M = 1..8) on the full Qwen3-0.6B q8_0 shape (synthetic weights), for the
two-launch fused layer (mode 1) and the 5-launch layer (mode 0): python scripts/prof_small_batch.py [steps]."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "fun-asr-gguf_amd")]
import numpy as np  # noqa: E402
from oracle import synth  # noqa: E402  (config dicts only)
from fun_asr_gguf import _native  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 32
eng = _native.Engine(synth.ENC_TINY, dict(synth.LLM_FULL, n_ctx=512, max_seqs=8), max_batch=1, max_samples=16000)
eng.synthetic_weights(0)
rng = np.random.default_rng(0)
for M in (1, 2, 3, 4, 5, 6, 7, 8):
    line = []
    for mode in (1, 0):
        eng.set_decode_fused(mode)
        for s in range(M):
            eng.llm_reset(s)
            eng.llm_prefill(s, (rng.standard_normal((204, 1024)) * 0.05).astype(np.float32))
        eng.llm_generate(list(range(M)), 4)
        eng.synchronize()
        t = time.perf_counter()
        eng.llm_generate(list(range(M)), steps)
        eng.synchronize()
        line.append(f"mode {mode}: {(time.perf_counter() - t) / steps * 1e3:.3f} ms/step")
    print(f"batch {M}: " + ", ".join(line), flush=True)
eng.close()
