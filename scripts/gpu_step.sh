#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 5 120 ./scripts/ubench/decode_step || exit 1
if [ -n "$PMC" ]; then
  rm -rf gpurun_out/pmc
  timeout -k 5 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc -o pmc -- ./scripts/ubench/decode_step eager 2 > gpurun_out/pmc.log 2>&1 || { tail -5 gpurun_out/pmc.log; exit 1; }
  python scripts/pmc_traffic.py gpurun_out/pmc/pmc_results.db gpurun_out/pmc_gemv.json | tail -30
fi
