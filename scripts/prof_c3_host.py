"""Host-side profile of one C3 step (bench.py c3_leg's workload: 32 x 60 s clips, encoder batch + decoder batch of 32):
cProfile of decode_streams after a warmup step, plus the wall time not covered by the per-stage timings.
  python scripts/prof_c3_host.py [batch]"""
import cProfile
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "fun-asr-gguf_amd")]
import numpy as np  # noqa: E402
import bench  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
from fun_asr_gguf import FunASREngine  # noqa: E402
from fun_asr_gguf.nano_dataclass import RecognitionStream  # noqa: E402
from fun_asr_gguf.synthetic import synth_audio  # noqa: E402

eng = FunASREngine("synthetic", "synthetic", "synthetic", "synthetic", n_predict=bench.N_GEN, device=0, model="full",
                   ignore_eos=True, max_batch=B, n_ctx=512)
assert eng.initialize(verbose=False)
m = eng.models
rng = np.random.default_rng(1234)
m.prompt_builder.fixed_ids = (list(rng.integers(0, m.llm_cfg["n_vocab"] - 3, bench.N_PREFIX)),
                              list(rng.integers(0, m.llm_cfg["n_vocab"] - 3, bench.N_SUFFIX)))
clips = [synth_audio(int(bench.CLIP_S * bench.SR), 1000 + i) for i in range(B)]
streams = []
for c in clips:
    st = RecognitionStream()
    st.accept_waveform(bench.SR, c)
    streams.append(st)
handle = m.engine.upload(clips)
dec = eng.orchestrator.decoder
dec.decode_streams(streams, verbose=False, temperature=0.0, resident=handle)
m.engine.synchronize()
pr = cProfile.Profile()
t0 = time.perf_counter()
pr.enable()
rs = dec.decode_streams(streams, verbose=False, temperature=0.0, resident=handle)
pr.disable()
dt = time.perf_counter() - t0
tm = rs[0].timings
covered = tm.encode + tm.ctc * B + tm.prepare * B + tm.inject * B + tm.llm_generate + tm.align * B
print(f"C3 step {dt * 1e3:.1f} ms: encode {tm.encode * 1e3:.1f}, ctc {tm.ctc * B * 1e3:.1f}, prompt {tm.prepare * B * 1e3:.1f}, "
      f"prefill(host) {tm.inject * B * 1e3:.1f}, generate {tm.llm_generate * 1e3:.1f}, align {tm.align * B * 1e3:.1f}; "
      f"not covered {(dt - covered) * 1e3:.1f} ms")
pstats.Stats(pr).sort_stats("cumulative").print_stats(28)
eng.cleanup()
