#!/bin/bash
# PMC FETCH_SIZE pass on bench.py itself (eager decode, one step) -> per-launch traffic summary of the decode launches
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
rm -rf gpurun_out/pmc
FUNASR_GRAPHS=0 timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc -o pmc -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --c3-batch 0 --no-c4 > gpurun_out/pmc.log 2>&1 || { echo "pmc pass failed rc=$?"; tail -30 gpurun_out/pmc.log; exit 1; }
python3 scripts/pmc_traffic.py gpurun_out/pmc/pmc_results.db gpurun_out/pmc_gemv_bench.json
rm -rf gpurun_out/pmc
