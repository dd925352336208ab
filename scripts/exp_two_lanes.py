"""Experiment: does a 32-stream decode step run faster as two concurrent 16-stream lanes (two engines, two host
threads, two HIP streams) than as one batch-32 graph? Full Qwen3-0.6B shape, synthetic weights.
  python scripts/exp_two_lanes.py [B] [steps]"""
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "fun-asr-gguf_amd")]
import numpy as np  # noqa: E402
from oracle import synth  # noqa: E402  (config dicts only)
from fun_asr_gguf import _native  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 64


def make(b):
    e = _native.Engine(synth.ENC_TINY, dict(synth.LLM_FULL, n_ctx=512, max_seqs=b), max_batch=1, max_samples=16000)
    e.synthetic_weights(0)
    rng = np.random.default_rng(0)
    embd = [(rng.standard_normal((204, 1024)) * 0.05).astype(np.float32) for _ in range(b)]
    for s in range(b):
        e.llm_reset(s)
    e.llm_prefill_batch(list(range(b)), embd, temperature=0.0)
    e.llm_generate(list(range(b)), 4)
    e.synchronize()
    return e


one = make(B)
t = time.perf_counter()
one.llm_generate(list(range(B)), steps)
one.synchronize()
print(f"one lane  x{B}: {(time.perf_counter() - t) / steps * 1e3:.3f} ms/step", flush=True)
one.close()
for nl in (2, 4):
    lanes = [make(B // nl) for _ in range(nl)]
    for e in lanes:  # warm the graphs of this width
        e.llm_generate(list(range(B // nl)), 2)
        e.synchronize()

    def run(e):
        e.llm_generate(list(range(B // nl)), steps)
        e.synchronize()

    th = [threading.Thread(target=run, args=(e,)) for e in lanes]
    t = time.perf_counter()
    for x in th:
        x.start()
    for x in th:
        x.join()
    print(f"{nl} lanes x{B // nl}: {(time.perf_counter() - t) / steps * 1e3:.3f} ms/step (all {B} streams)", flush=True)
    t = time.perf_counter()
    run(lanes[0])
    print(f"  one of them alone: {(time.perf_counter() - t) / steps * 1e3:.3f} ms/step", flush=True)
    for e in lanes:
        e.close()
