#!/bin/bash
# GPU parity tests only (stop at the first failure); optional TESTS="tests/x.py" to select
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -x -v -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/gpu_tests.log | tail -40
if [ $rc -ne 0 ]; then grep -E "Error|assert" gpurun_out/gpu_tests.log | head -30; fi
exit $rc
