#!/bin/bash
# Greedy batch-1 sampling inside the LM head launch (FUNASR_LM_GREEDY_TAIL): the GPU suite, then the graph-replayed
# batch-1 step with and without it (interleaved), then the C2 bench leg.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 240 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/greedy_tests.log 2>&1 || { tail -40 gpurun_out/greedy_tests.log; exit 1; }
tail -2 gpurun_out/greedy_tests.log
timeout -k 10 300 python -u scripts/prof_decode_ab.py 128 FUNASR_LM_GREEDY_TAIL=0 FUNASR_LM_GREEDY_TAIL=1 \
  FUNASR_LM_GREEDY_TAIL=0 FUNASR_LM_GREEDY_TAIL=1 2>&1 | tee gpurun_out/greedy_ab.log
timeout -k 10 600 python -u bench.py --steps 3 --warmup 1 > gpurun_out/greedy_bench.json 2> gpurun_out/greedy_bench.err \
  || { tail -20 gpurun_out/greedy_bench.err; exit 1; }
cat gpurun_out/greedy_bench.json | cut -c1-600
