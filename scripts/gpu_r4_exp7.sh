#!/bin/bash
# one-clip GEMMs with 128-deep stages (force 9 / 10) vs the default policy; FETCH_SIZE pass on the graph-replayed
# production decode (HIP graph packet capture off under the profiler)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 200 scripts/ubench/gemm_f32_bench kscan > gpurun_out/kscan2.txt 2>&1 || { tail -5 gpurun_out/kscan2.txt; exit 1; }
grep -E "variant (9|10)|M=1001 [a-z]" gpurun_out/kscan2.txt
rm -rf gpurun_out/pmcg
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -s KILL 170 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmcg -o pmc -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --c3-batch 0 --no-c4 --c3-varlen 0 > gpurun_out/pmcg.log 2>&1
echo "pmc graph pass rc=$?"; tail -3 gpurun_out/pmcg.log
db=$(find gpurun_out/pmcg -name "*results.db" | head -1)
[ -n "$db" ] && python3 scripts/pmc_traffic.py "$db" gpurun_out/pmc_gemv_graph.json | tail -14
rm -rf gpurun_out/pmcg
