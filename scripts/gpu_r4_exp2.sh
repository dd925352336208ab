#!/bin/bash
# long-prompt prefill test + graph/PMC repro (kernel-trace and PMC, graph and eager); the PMC graph runs go last
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_fullsize.py -k "long_prompt or slot_reuse" -x -v -m gpu --timeout 240 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/t_long.log 2>&1 || { tail -30 gpurun_out/t_long.log; exit 1; }
tail -3 gpurun_out/t_long.log
timeout -k 10 120 python -u scripts/prof_prefill_long.py 204 1024 1536 2000 || exit 1
rm -rf gpurun_out/gr
timeout -s KILL 60 rocprofv3 --kernel-trace --stats -d gpurun_out/gr -o kt -- scripts/ubench/graph_pmc_repro > gpurun_out/repro_kt.log 2>&1
echo "kernel-trace + graph rc=$?"; tail -2 gpurun_out/repro_kt.log
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/gr -o pe -- scripts/ubench/graph_pmc_repro eager > gpurun_out/repro_pe.log 2>&1
echo "pmc + eager rc=$?"; tail -2 gpurun_out/repro_pe.log
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/gr -o pg -- scripts/ubench/graph_pmc_repro > gpurun_out/repro_pg.log 2>&1
echo "pmc + graph rc=$?"; grep -v "^    @" gpurun_out/repro_pg.log | tail -6
