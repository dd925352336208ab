#!/bin/bash
# Round-4 GPU session: GPU tests -> bench line (optionally then the kernel-trace and PMC passes of scripts/gpu_round3.sh).
# Each GPU step has its own limit; stop at the first failure.
#   TESTS="tests/x.py::y" limits the tests; NOTESTS=1 skips them; BENCH_ARGS passes bench flags; NOBENCH=1 skips it.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
if [ -z "$NOTESTS" ]; then
  timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -x -v -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
  tail -3 gpurun_out/gpu_tests.log
fi
if [ -z "$NOBENCH" ]; then
  timeout -k 10 900 python -u bench.py ${BENCH_ARGS} > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
  cat gpurun_out/bench.json
fi
