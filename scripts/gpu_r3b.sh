#!/bin/bash
# round-3 re-entry: GPU tests + bench on the rebuilt tree, then the batch-32 attention MALL experiment
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
true
true
timeout -k 10 180 scripts/ubench/gemm_batch 32 > gpurun_out/gemm_batch8.txt 2>&1 || { tail -5 gpurun_out/gemm_batch8.txt; exit 1; }
cat gpurun_out/gemm_batch8.txt
for w in 4 8 4 8; do FUNASR_SK_WAVES=$w timeout -k 10 120 python scripts/prof_batch_decode.py 32 64 2>&1 | sed "s/^/waves $w: /" | tee -a gpurun_out/batch_step_waves.txt || exit 1; done
if [ -z "$NOTESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
  tail -2 gpurun_out/gpu_tests.log
fi
timeout -k 10 900 python -u bench.py ${BENCH_ARGS} > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
