#!/bin/bash
# Round-2 evidence: bench (JSON line) -> rocprofv3 kernel-trace stats of the bench workload -> a PMC FETCH_SIZE
# pass on bench.py itself (eager decode, short run). Each GPU step has its own limit; stop at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python bench.py ${BENCH_ARGS} > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
if [ -n "$NOPROF" ]; then exit 0; fi
rm -rf gpurun_out/prof
FUNASR_GRAPHS=0 timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof.log 2>&1 || { echo "rocprof failed"; tail -20 gpurun_out/prof.log; exit 1; }
python scripts/prof_summary.py gpurun_out/prof/run_results.db 45 > gpurun_out/prof_summary.txt
find gpurun_out/prof -name "*kernel_stats.csv" -exec cp {} gpurun_out/prof_kernel_stats.csv \;
rm -rf gpurun_out/prof
FUNASR_GRAPHS=0 timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc -o pmc -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --c3-batch 0 --no-c4 > gpurun_out/pmc.log 2>&1 || { echo "pmc pass failed rc=$?"; tail -30 gpurun_out/pmc.log; exit 0; }
python scripts/pmc_traffic.py gpurun_out/pmc/pmc_results.db gpurun_out/pmc_gemv_bench.json | tail -12
rm -rf gpurun_out/pmc
