#!/bin/bash
# encoder loop: encoder parity tests at tiny + full size, then encode timing per GEMM mode (B=1 and B=32)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -k "${K:-encoder}" -x -v -s -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_enc_tests.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed|max-abs" gpurun_out/gpu_enc_tests.log | tail -30
if [ $rc -ne 0 ]; then grep -E "Error|assert" gpurun_out/gpu_enc_tests.log | head -30; exit $rc; fi
for m in f32 bf16x3; do
  timeout -k 10 120 python scripts/prof_encode.py 1 10 $m || exit 1
  timeout -k 10 200 python scripts/prof_encode.py 32 3 $m || exit 1
done
