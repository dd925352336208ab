"""A/B of the FSMN kernels on the batch-32 encode (FUNASR_FSMN_VEC=1: 16-B lanes, 0: 4-B lanes): outputs must be
bit-identical; prints the encode time of each."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "fun-asr-gguf_amd")]
import numpy as np  # noqa: E402
from oracle import synth  # noqa: E402
from fun_asr_gguf import _native  # noqa: E402
from fun_asr_gguf.synthetic import synth_audio  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
clips = [synth_audio(16000 * 60 - 977 * i, 100 + i) for i in range(B)]
outs = {}
for vec in ("0", "1", "0", "1"):
    os.environ["FUNASR_FSMN_VEC"] = vec
    e = _native.Engine(synth.ENC_FULL, dict(synth.LLM_TINY, n_ctx=64, max_seqs=1), max_batch=B, max_samples=16000 * 61)
    e.synthetic_weights(0)
    h = e.upload(clips)
    e.encode(clips, resident=h)
    e.synchronize()
    t = time.perf_counter()
    for _ in range(3):
        r = e.encode(clips, resident=h, want_enc=True)
    e.synchronize()
    dt = (time.perf_counter() - t) / 3
    outs[vec] = r
    print(f"FSMN_VEC={vec}: encode batch {B} {dt * 1e3:.2f} ms")
    e.close()
same = all((a == b).all() for a, b in zip(outs["0"]["enc"], outs["1"]["enc"])) and \
    all((a == b).all() for a, b in zip(outs["0"]["audio_embd"], outs["1"]["audio_embd"])) and \
    all((a == b).all() for a, b in zip(outs["0"]["ctc_ids"], outs["1"]["ctc_ids"]))
print("bit-identical:", same)
