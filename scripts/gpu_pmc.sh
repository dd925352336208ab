#!/bin/bash
# PMC pass (FETCH_SIZE) over a short bench run, eager decode (graphs off: rocprof replays graphs very slowly)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
FUNASR_GRAPHS=0 timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc -o pmc -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/pmc.log 2>&1 || { echo "pmc failed"; tail -20 gpurun_out/pmc.log; exit 1; }
python scripts/pmc_traffic.py gpurun_out/pmc/pmc_results.db gpurun_out/pmc_gemv.json
