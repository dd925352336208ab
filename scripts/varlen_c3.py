"""configs[2] variable-length leg alone (bench.py c3_varlen_leg), with the scheduler's timing stats: continuous batching
vs static groups. python scripts/varlen_c3.py [n_clips] [slots] [admit_min]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "fun-asr-gguf_amd")]
import numpy as np  # noqa: E402

from fun_asr_gguf import FunASREngine  # noqa: E402
from fun_asr_gguf.core.scheduler import ContinuousBatcher  # noqa: E402
from fun_asr_gguf.nano_dataclass import RecognitionStream  # noqa: E402
from fun_asr_gguf.synthetic import synth_audio  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 64
S = int(sys.argv[2]) if len(sys.argv) > 2 else 32
admit = int(sys.argv[3]) if len(sys.argv) > 3 else None
eng = FunASREngine("synthetic", "synthetic", "synthetic", "synthetic", n_predict=384, ignore_eos=True, max_batch=S,
                   n_ctx=640)
assert eng.initialize(verbose=False)
m = eng.models
rng = np.random.default_rng(1234)
m.prompt_builder.fixed_ids = (list(rng.integers(0, 151933, 73)), list(rng.integers(0, 151933, 5)))
clips = [synth_audio(960000, 3000 + i) for i in range(n)]
lens = [int(x) for x in np.random.default_rng(77).integers(128, 385, n)]
dec = eng.orchestrator.decoder
for it in range(2):
    cb = ContinuousBatcher(dec, admit_min=admit)
    t = time.perf_counter()
    rs = cb.run(clips, None, None, 0.0, 1.0, 50, n_predicts=lens)
    m.engine.synchronize()
    dt = time.perf_counter() - t
    assert [r.n_gen for r in rs] == lens
    print(f"continuous (admit_min {admit}): {dt * 1e3:.1f} ms = {60 * n / dt:.1f} audio-s/s  {cb.stats}", flush=True)
t = time.perf_counter()
for i in range(0, n, S):
    sts = []
    for c in clips[i:i + S]:
        st = RecognitionStream()
        st.accept_waveform(16000, c)
        sts.append(st)
    dec.decode_streams(sts, verbose=False, temperature=0.0, n_predicts=lens[i:i + S])
m.engine.synchronize()
dt = time.perf_counter() - t
print(f"static groups of {S}: {dt * 1e3:.1f} ms = {60 * n / dt:.1f} audio-s/s; token-steps {sum(lens)}, "
      f"mean len {np.mean(lens):.0f}, max per group {[max(lens[i:i + S]) for i in range(0, n, S)]}")
eng.cleanup()
