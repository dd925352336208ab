"""Diagnostic: teacher-forced per-step decode logits, GPU vs oracle (tiny config)."""
import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "fun-asr-gguf_amd")]
import numpy as np
from fun_asr_gguf import _native
from oracle import synth, qwen3 as oqw
cfg = synth.LLM_TINY
eng = _native.Engine(synth.ENC_TINY, dict(cfg, n_ctx=512, max_seqs=4), max_batch=1, max_samples=16000)
eng.synthetic_weights(0)
m = oqw.Qwen3Q8(synth.make_weights(synth.llm_tensors(cfg)), cfg, n_ctx=512)
rng = np.random.default_rng(3)
prompt = np.concatenate([m.embed_prompt(rng.integers(0, 4096, 30)), (rng.standard_normal((21, 1024)) * 0.5).astype(np.float32)], 0)
eng.llm_reset(0)
tok, lg = eng.llm_prefill(0, prompt, want_logits=True)
m.reset()
ref = m.forward(prompt, 0)
pos = prompt.shape[0]
def cmp(a, b, t):
    cos = float(a @ b / np.linalg.norm(a) / np.linalg.norm(b))
    s = np.sort(b)
    print(f"step {t}: cos {cos:.7f} maxabs {np.abs(a-b).max():.4g} gpu_arg {a.argmax()} ref_arg {b.argmax()} ref_margin {s[-1]-s[-2]:.4g}")
cmp(lg, ref, 0)
for t in range(1, 8):
    nxt = int(lg.argmax())
    g = eng.llm_generate([0], 1)[0]
    lg = eng.llm_logits(0)
    ref = m.forward(m.embed_tokens([nxt]), pos)
    pos += 1
    cmp(lg, ref, t)
