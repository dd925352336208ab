#!/bin/bash
# Round-3 GPU session: GPU tests (optional filter in $TESTS) then a bench line (skipped with NOBENCH=1).
# Each GPU step has its own time limit; the script stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
if [ -z "$NOTESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider \
    ${TESTS} > gpurun_out/gpu_tests.log 2>&1
  rc=$?
  tail -15 gpurun_out/gpu_tests.log
  [ $rc -eq 0 ] || { echo "tests rc=$rc"; exit $rc; }
fi
if [ -z "$NOBENCH" ]; then
  timeout -k 10 600 python -u bench.py ${BENCH_ARGS} > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
  cat gpurun_out/bench.json
fi
