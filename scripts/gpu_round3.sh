#!/bin/bash
# Round-3 evidence: GPU tests -> bench (JSON line) -> rocprofv3 kernel-trace stats of the bench workload -> PMC passes on
# bench.py itself (FETCH_SIZE for the decode layer traffic; SQ_VALU_MFMA_BUSY_CYCLES / SQ_BUSY_CU_CYCLES / GRBM_GUI_ACTIVE
# for the encoder's MFMA utilisation). Each GPU step has its own limit; stop at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
if [ -z "$NOTESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
  tail -2 gpurun_out/gpu_tests.log
fi
timeout -k 10 900 python -u bench.py ${BENCH_ARGS} > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
if [ -n "$NOPROF" ]; then exit 0; fi
rm -rf gpurun_out/prof
FUNASR_GRAPHS=0 timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --c3-varlen 0 > gpurun_out/prof.log 2>&1 || { echo "rocprof failed"; tail -20 gpurun_out/prof.log; exit 1; }
python3 scripts/prof_summary.py gpurun_out/prof/run_results.db 45 > gpurun_out/prof_summary.txt
find gpurun_out/prof -name "*kernel_stats.csv" -exec cp {} gpurun_out/prof_kernel_stats.csv \;
rm -rf gpurun_out/prof
FUNASR_GRAPHS=0 timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc -o pmc -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --c3-batch 0 --no-c4 --c3-varlen 0 > gpurun_out/pmc.log 2>&1 || { echo "pmc pass failed rc=$?"; tail -30 gpurun_out/pmc.log; exit 1; }
python3 scripts/pmc_traffic.py gpurun_out/pmc/pmc_results.db gpurun_out/pmc_gemv_bench.json | tail -12
rm -rf gpurun_out/pmc
for mode in bf16x3 f32; do
  rm -rf gpurun_out/pmcm
  FUNASR_GRAPHS=0 FUNASR_ENC_GEMM=$mode timeout -s KILL 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE \
    -d gpurun_out/pmcm -o pmc -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --c3-batch 32 --c3-steps 1 --no-c4 --c3-varlen 0 \
    > gpurun_out/pmcm_$mode.log 2>&1 || { echo "pmc mfma pass failed rc=$?"; tail -30 gpurun_out/pmcm_$mode.log; exit 1; }
  db=$(find gpurun_out/pmcm -name "*results.db" | head -1)
  python3 scripts/pmc_mfma.py "$db" gpurun_out/pmc_mfma_$mode.json
  rm -rf gpurun_out/pmcm
done
