"""Graph-replayed decode step under several engine settings, interleaved (full Qwen3-0.6B q8_0 shape, synthetic weights,
a 204-row prefill per sequence, then `steps` greedy steps from n_past 204).
python scripts/prof_decode_ab.py [steps] SETTING [SETTING ...]
SETTING = comma-separated ENV=VALUE assignments applied before the engine is created ('-' = defaults), e.g.
  FUNASR_AB_FULL=0  FUNASR_AB_FULL=1024
AB_M=<M> decodes M sequences per step; AB_REPS=<r> timed repetitions per setting (default 3); AB_PREFILL=<rows>.
Prints ms per step per setting, whether its tokens equal the first setting's (settings that change the f32
summation order may legitimately differ) and a hash of the tokens and the last logits row (library A/B across processes)."""
import hashlib
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "fun-asr-gguf_amd")]
import numpy as np  # noqa: E402
from oracle import synth  # noqa: E402  (config dicts only)
from fun_asr_gguf import _native  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 256
settings = sys.argv[2:] or ["-"]
M = int(os.environ.get("AB_M", "1"))
reps = int(os.environ.get("AB_REPS", "3"))
n_pre = int(os.environ.get("AB_PREFILL", "204"))
rng = np.random.default_rng(0)
prompts = [(rng.standard_normal((n_pre, 1024)) * 0.05).astype(np.float32) for _ in range(M)]
base = dict(os.environ)
ref = None
for st in settings:
    os.environ.clear()
    os.environ.update(base)
    if st != "-":
        for kv in st.split(","):
            k, v = kv.split("=", 1)
            os.environ[k] = v
    eng = _native.Engine(synth.ENC_TINY, dict(synth.LLM_FULL, n_ctx=n_pre + steps + 64, max_seqs=max(M, 1)),
                         max_batch=1, max_samples=16000)
    eng.synthetic_weights(0)
    ms = []
    for rep in range(reps):
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
    th = hashlib.sha256(np.ascontiguousarray(toks).tobytes() + eng.llm_logits(0).tobytes()).hexdigest()[:12]
    print(f"M={M} [{st}]: {' '.join(f'{m:.4f}' for m in ms)} ms/step (min {min(ms):.4f}); tokens "
          f"{'equal' if same else 'differ'}; invariant width {eng.llm_invariant_width()}; tokens+logits {th}", flush=True)
    eng.close()
