#!/bin/bash
# Round-end evidence: parity tests -> smoke -> bench (JSON line) -> rocprofv3 kernel trace of the bench workload
# -> PMC FETCH_SIZE pass on the decode-step replica (see profiles/README.md). Stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1 || { grep -E "FAILED|Error" gpurun_out/gpu_tests.log | head; exit 1; }
grep -E "passed|failed" gpurun_out/gpu_tests.log | tail -1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
rm -rf gpurun_out/prof
FUNASR_GRAPHS=0 timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof.log 2>&1 || { echo "rocprof failed"; tail -20 gpurun_out/prof.log; exit 1; }
python scripts/prof_summary.py gpurun_out/prof/run_results.db 45 > gpurun_out/prof_summary.txt
cp gpurun_out/prof/run_kernel_stats.csv gpurun_out/prof_kernel_stats.csv 2>/dev/null
rm -rf gpurun_out/prof gpurun_out/pmc
timeout -k 5 120 ./scripts/ubench/decode_step > gpurun_out/decode_step.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc -o pmc -- ./scripts/ubench/decode_step eager 2 > gpurun_out/pmc.log 2>&1 || { tail -5 gpurun_out/pmc.log; exit 1; }
python scripts/pmc_traffic.py gpurun_out/pmc/pmc_results.db gpurun_out/pmc_gemv.json | tail -12
rm -rf gpurun_out/pmc
