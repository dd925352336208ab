"""Single-prompt prefill (fa_llm_prefill) time vs prompt length on the full Qwen3-0.6B q8_0 shape:
  [FUNASR_PF_ROW_LOCAL_MAX=n] python scripts/prof_prefill_long.py 204 512 1024 2000
(row-local forward -- the arithmetic a prompt gets inside a row-local batch -- vs the tiled forward above n rows)"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "fun-asr-gguf_amd")]
import numpy as np  # noqa: E402
from oracle import synth  # noqa: E402  (config dicts only)
from fun_asr_gguf import _native  # noqa: E402

lens = [int(x) for x in sys.argv[1:]] or [204, 512, 1024]
eng = _native.Engine(synth.ENC_TINY, dict(synth.LLM_FULL, n_ctx=max(lens) + 8, max_seqs=1), max_batch=1,
                     max_samples=16000)
eng.synthetic_weights(0)
rng = np.random.default_rng(0)
for T in lens:
    p = (rng.standard_normal((T, 1024)) * 0.05).astype(np.float32)
    ts = []
    for r in range(4):
        eng.llm_reset(0)
        eng.synchronize()
        t = time.perf_counter()
        eng.llm_prefill(0, p, temperature=0.0)
        eng.synchronize()
        ts.append(time.perf_counter() - t)
    print(f"prefill 1 x {T} rows (row-local max {os.environ.get('FUNASR_PF_ROW_LOCAL_MAX', 'inf')}): "
          f"{min(ts[1:]) * 1e3:.2f} ms")
eng.close()
