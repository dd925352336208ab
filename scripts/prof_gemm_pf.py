"""Batched decode step (batch B, default 32) with and without the split-K GEMMs' L2 prefetch slabs (FUNASR_GEMM_PF
mask, FUNASR_GEMM_PF_SLABS, FUNASR_GEMM_PF_DELAY): full Qwen3-0.6B q8_0 shape, synthetic weights, 204-row prefills,
graph-replayed steps. python scripts/prof_gemm_pf.py [steps] [mask:slabs:delay ...]; B from PF_B.
Prints ms per step per setting (interleaved) and checks every setting's tokens against the first one's."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "fun-asr-gguf_amd")]
import numpy as np  # noqa: E402
from oracle import synth  # noqa: E402  (config dicts only)
from fun_asr_gguf import _native  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 64
settings = [tuple(int(v) for v in a.split(":")) for a in sys.argv[2:]] or [(0, 1, 100), (7, 1, 100)]
B = int(os.environ.get("PF_B", "32"))
rng = np.random.default_rng(0)
prompts = [(rng.standard_normal((204, 1024)) * 0.05).astype(np.float32) for _ in range(B)]
ref = None
for mask, slabs, delay in settings:
    os.environ["FUNASR_GEMM_PF"] = str(mask)
    os.environ["FUNASR_GEMM_PF_SLABS"] = str(slabs)
    os.environ["FUNASR_GEMM_PF_DELAY"] = str(delay)
    eng = _native.Engine(synth.ENC_TINY, dict(synth.LLM_FULL, n_ctx=512, max_seqs=B), max_batch=1, max_samples=16000)
    eng.synthetic_weights(0)
    ms = []
    for rep in range(3):
        for q in range(B):
            eng.llm_reset(q)
            eng.llm_prefill(q, prompts[q])
        eng.llm_generate(list(range(B)), 4)
        eng.synchronize()
        t = time.perf_counter()
        toks = eng.llm_generate(list(range(B)), steps)
        eng.synchronize()
        ms.append((time.perf_counter() - t) / steps * 1e3)
    if ref is None:
        ref = toks
    same = bool(np.array_equal(toks, ref))
    print(f"B={B} gemm_pf={mask} slabs={slabs} delay={delay}: {' '.join(f'{m:.4f}' for m in ms)} ms/step "
          f"(min {min(ms):.4f}); tokens {'equal' if same else 'DIFFER'}", flush=True)
    eng.close()
    if not same:
        sys.exit(1)
