#!/bin/bash
# quick GPU loop: parity tests (stop at first failure) -> decode-step ablation microbenchmark
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/gpu_tests.log | tail -25
if [ $rc -ne 0 ]; then grep -E "Error|assert" gpurun_out/gpu_tests.log | head -30; exit $rc; fi
timeout -k 5 120 ./scripts/ubench/decode_step
