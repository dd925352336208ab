"""Experiment: the chip partitioned between a batch-32 decode (engine A) and the next batch's 32-clip encode (engine B)
by CU-masked streams (FUNASR_CU_MASK -> hipExtStreamCreateWithCUMask), each alone and overlapped from two host
threads. python scripts/exp_cu_partition.py <decode mask words> <encode mask words> (comma-separated hex, 8 words =
256 CUs; "-" = no mask)."""
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "fun-asr-gguf_amd")]
import numpy as np  # noqa: E402
from oracle import synth  # noqa: E402  (config dicts only)
from fun_asr_gguf import _native  # noqa: E402

dmask, emask = sys.argv[1], sys.argv[2]
B, steps = 32, 96


def make(mask, *a, **k):
    if mask != "-":
        os.environ["FUNASR_CU_MASK"] = mask
    try:
        return _native.Engine(*a, **k)
    finally:
        os.environ.pop("FUNASR_CU_MASK", None)


dec = make(dmask, synth.ENC_TINY, dict(synth.LLM_FULL, n_ctx=512, max_seqs=B), max_batch=1, max_samples=16000)
dec.synthetic_weights(0)
rng = np.random.default_rng(0)
embd = [(rng.standard_normal((204, 1024)) * 0.05).astype(np.float32) for _ in range(B)]
for s in range(B):
    dec.llm_reset(s)
dec.llm_prefill_batch(list(range(B)), embd, temperature=0.0)
dec.llm_generate(list(range(B)), 4)
dec.synchronize()
enc = make(emask, synth.ENC_FULL, synth.LLM_TINY, max_batch=B, max_samples=16000 * 60)
enc.synthetic_weights(1)
clips = [(np.sin(np.arange(960000) * (0.01 + 0.001 * i)) * 0.1).astype(np.float32) for i in range(B)]
h = enc.upload(clips)
enc.encode(None, resident=h)


def run_dec(res):
    t = time.perf_counter()
    dec.llm_generate(list(range(B)), steps)
    dec.synchronize()
    res.append((time.perf_counter() - t) / steps * 1e3)


def run_enc(res, n):
    t = time.perf_counter()
    for _ in range(n):
        enc.encode(None, resident=h)
    res.append((time.perf_counter() - t) / n * 1e3)


r = []
run_dec(r)
run_enc(r, 3)
rd, re_ = [], []
td = threading.Thread(target=run_dec, args=(rd,))
te = threading.Thread(target=run_enc, args=(re_, 1))
t0 = time.perf_counter()
td.start(); te.start(); te.join(); t_enc = time.perf_counter() - t0; td.join()
tot = (time.perf_counter() - t0) * 1e3
print(f"masks dec={dmask[:17]} enc={emask[:17]}: alone decode {r[0]:.3f} ms/step, encode {r[1]:.1f} ms; overlapped decode "
      f"{rd[-1]:.3f} ms/step, encode {re_[-1]:.1f} ms; total {tot:.0f} ms vs serial {r[0] * steps + r[1]:.0f} ms",
      flush=True)
