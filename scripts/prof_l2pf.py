"""Batch-1 decode step with and without the attention launch's L2 prefetch blocks (FUNASR_L2PF blocks per kv head,
FUNASR_L2PF_DELAY ticks): full Qwen3-0.6B q8_0 shape, synthetic weights, 204-row prefill, graph-replayed steps.
python scripts/prof_l2pf.py [steps] [pf:delay[:mask] ...]   (default: 0:0 16:150 0:0 16:150)
Prints ms per step per setting, interleaved, and checks every setting's tokens against the first one's.
L2PF_M=<M> decodes M sequences per step (FUNASR_L2PF_MAX_M is set to M)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "fun-asr-gguf_amd")]
import numpy as np  # noqa: E402
from oracle import synth  # noqa: E402  (config dicts only)
from fun_asr_gguf import _native  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 256
settings = [tuple(int(v) for v in a.split(":")) for a in sys.argv[2:]] or [(0, 0), (16, 150), (0, 0), (16, 150)]
settings = [(s + (7,))[:3] for s in settings]
M = int(os.environ.get("L2PF_M", "1"))
rng = np.random.default_rng(0)
prompts = [(rng.standard_normal((204, 1024)) * 0.05).astype(np.float32) for _ in range(M)]
ref = None
for pf, delay, mask in settings:
    os.environ["FUNASR_L2PF"] = str(pf)
    os.environ["FUNASR_L2PF_DELAY"] = str(delay)
    os.environ["FUNASR_L2PF_MASK"] = str(mask)
    os.environ["FUNASR_L2PF_MAX_M"] = str(M)
    eng = _native.Engine(synth.ENC_TINY, dict(synth.LLM_FULL, n_ctx=512, max_seqs=M), max_batch=1, max_samples=16000)
    eng.synthetic_weights(0)
    eng.set_decode_fused(1)
    ms = []
    for rep in range(3):
        for q in range(M):
            eng.llm_reset(q)
            eng.llm_prefill(q, prompts[q])
        eng.llm_generate(list(range(M)), 4)
        eng.synchronize()
        t = time.perf_counter()
        toks = eng.llm_generate(list(range(M)), steps)
        eng.synchronize()
        ms.append((time.perf_counter() - t) / steps * 1e3)
    if ref is None:
        ref = toks
    same = bool(np.array_equal(toks, ref))
    print(f"M={M} l2pf={pf} delay={delay} mask={mask}: {' '.join(f'{m:.4f}' for m in ms)} ms/step (min {min(ms):.4f}); "
          f"tokens {'equal' if same else 'DIFFER'}", flush=True)
    eng.close()
    if not same:
        sys.exit(1)
