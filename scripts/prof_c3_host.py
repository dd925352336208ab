"""Host-side profile of one C3 step (32 x 60 s clips through StreamDecoder.decode_streams): per-stage timings of the
result and the top cumulative Python functions: python scripts/prof_c3_host.py [batch]."""
import cProfile
import os
import pstats
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "fun-asr-gguf_amd")]
import bench  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
pr = cProfile.Profile()
pr.enable()
out = bench.c3_leg(B, 2, 1, 0, "full", lambda: None, None)
pr.disable()
print(out)
pstats.Stats(pr).sort_stats("cumulative").print_stats(40)
