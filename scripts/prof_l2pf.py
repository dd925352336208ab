"""Batch-1 decode step with and without the attention launch's L2 prefetch blocks (FUNASR_L2PF blocks per kv head,
FUNASR_L2PF_DELAY ticks): full Qwen3-0.6B q8_0 shape, synthetic weights, 204-row prefill, graph-replayed steps.
python scripts/prof_l2pf.py [steps] [pf:delay[:mask] ...]   (default: 0:0 16:150 0:0 16:150)
Prints ms per step per setting, interleaved, and checks every setting's tokens against the first one's."""
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
rng = np.random.default_rng(0)
prompt = (rng.standard_normal((204, 1024)) * 0.05).astype(np.float32)
ref = None
for pf, delay, mask in settings:
    os.environ["FUNASR_L2PF"] = str(pf)
    os.environ["FUNASR_L2PF_DELAY"] = str(delay)
    os.environ["FUNASR_L2PF_MASK"] = str(mask)
    eng = _native.Engine(synth.ENC_TINY, dict(synth.LLM_FULL, n_ctx=512, max_seqs=1), max_batch=1, max_samples=16000)
    eng.synthetic_weights(0)
    eng.set_decode_fused(1)
    ms = []
    for rep in range(3):
        eng.llm_reset(0)
        eng.llm_prefill(0, prompt)
        eng.llm_generate([0], 4)
        eng.synchronize()
        t = time.perf_counter()
        toks = eng.llm_generate([0], steps)
        eng.synchronize()
        ms.append((time.perf_counter() - t) / steps * 1e3)
    if ref is None:
        ref = toks
    same = bool(np.array_equal(toks, ref))
    print(f"l2pf={pf} delay={delay} mask={mask}: {' '.join(f'{m:.4f}' for m in ms)} ms/step (min {min(ms):.4f}); "
          f"tokens {'equal' if same else 'DIFFER'}", flush=True)
    eng.close()
    if not same:
        sys.exit(1)
