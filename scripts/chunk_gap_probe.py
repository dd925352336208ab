"""Decode-loop overhead probe: 253 greedy steps of one sequence (configs[1] shape: 204-row prompt) as one
fa_llm_generate call vs 8 chunks of 32 through generate_begin / _end (decode_many's loop, host token work between
chunks). The difference is the GPU idle time at the chunk seams."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "fun-asr-gguf_amd")]
import numpy as np  # noqa: E402
from oracle import synth  # noqa: E402
from fun_asr_gguf import _native  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1
eng = _native.Engine(synth.ENC_TINY, dict(synth.LLM_FULL, n_ctx=512, max_seqs=B), max_batch=1, max_samples=16000)
eng.synthetic_weights(0)
rng = np.random.default_rng(0)
prompt = [(rng.standard_normal((204, 1024)) * 0.05).astype(np.float32) for _ in range(B)]
seqs = list(range(B))


def prefill():
    for s in seqs:
        eng.llm_reset(s)
        eng.llm_prefill(s, prompt[s])


for rep in range(3):
    prefill()
    eng.synchronize()
    t = time.perf_counter()
    one = eng.llm_generate(seqs, 253)
    t_one = time.perf_counter() - t
    prefill()
    eng.synchronize()
    t = time.perf_counter()
    toks, left = [], 253
    eng.llm_generate_begin(seqs, 32)
    left -= 32
    while True:
        tk = eng.llm_generate_end()
        nxt = min(32, left)
        if nxt:
            eng.llm_generate_begin(seqs, nxt)
            left -= nxt
        toks.append(tk)
        if not nxt:
            break
    t_ch = time.perf_counter() - t
    same = (np.concatenate(toks, 1) == one).all()
    print(f"batch {B}: one call {t_one / 253 * 1e6:.1f} us/step, 32-step chunks {t_ch / 253 * 1e6:.1f} us/step "
          f"(seam {(t_ch - t_one) / 7 * 1e6:.0f} us per seam), tokens equal {bool(same)}")
eng.close()
