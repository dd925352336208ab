#!/bin/bash
# Round 5: fused-decode parity tests, then a graph-replayed decode-step A/B of engine settings (scripts/prof_decode_ab.py).
# AB_TESTS: pytest -k expression (empty: skip the tests); AB_SETTINGS: the settings (prof_decode_ab.py syntax).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
if [ -n "${AB_TESTS}" ]; then
  timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -v \
    --timeout 120 --timeout-method thread -k "${AB_TESTS}" 2>&1 | tee gpurun_out/ab_tests.log
  rc=$?
  # assertion failures (1) still allow the timing runs; anything else (a fault, an abort, a timeout) ends the call
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
fi
timeout -k 10 400 python -u scripts/prof_decode_ab.py ${AB_STEPS:-256} ${AB_SETTINGS:--} \
  2>&1 | tee gpurun_out/ab.log
