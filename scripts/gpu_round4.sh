#!/bin/bash
# Round-4 evidence: GPU tests -> bench (JSON line) -> rocprofv3 kernel-trace stats of the bench workload on the
# graph-replayed production path -> PMC passes on bench.py itself, graphs on (FETCH_SIZE for the decode-layer traffic;
# MFMA busy for the encoder in bf16x3 and fp16). Graph packet capture off under the profiler. Each GPU step
# has its own limit; stop at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
if [ -z "$NOTESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
  tail -2 gpurun_out/gpu_tests.log
fi
timeout -k 10 900 python -u bench.py ${BENCH_ARGS} > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
if [ -n "$NOPROF" ]; then exit 0; fi
export DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
rm -rf gpurun_out/prof
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --c3-varlen 0 > gpurun_out/prof.log 2>&1 || { echo "rocprof failed"; tail -20 gpurun_out/prof.log; exit 1; }
python3 scripts/prof_summary.py gpurun_out/prof/run_results.db 45 > gpurun_out/prof_summary.txt
rm -rf gpurun_out/prof
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc -o pmc -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --c3-batch 0 --no-c4 --c3-varlen 0 > gpurun_out/pmc.log 2>&1 || { echo "pmc pass failed rc=$?"; tail -30 gpurun_out/pmc.log; exit 1; }
python3 scripts/pmc_traffic.py gpurun_out/pmc/pmc_results.db gpurun_out/pmc_gemv_bench.json | tail -12
rm -rf gpurun_out/pmc
for mode in bf16x3 fp16; do
  rm -rf gpurun_out/pmcm
  if [ $mode = fp16 ]; then cmd="scripts/prof_encode.py 32 2 fp16"; else cmd="bench.py --steps 1 --warmup 0 --no-cpu-baseline --c3-batch 32 --c3-steps 1 --no-c4 --c3-varlen 0"; fi
  timeout -s KILL 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE \
    -d gpurun_out/pmcm -o pmc -- python3 $cmd > gpurun_out/pmcm_$mode.log 2>&1 || { echo "pmc mfma pass failed rc=$?"; tail -30 gpurun_out/pmcm_$mode.log; exit 1; }
  db=$(find gpurun_out/pmcm -name "*results.db" | head -1)
  python3 scripts/pmc_mfma.py "$db" gpurun_out/pmc_mfma_$mode.json | head -40
  rm -rf gpurun_out/pmcm
done
