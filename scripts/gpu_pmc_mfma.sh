#!/bin/bash
# PMC pass on bench.py itself for the matrix-core kernels: SQ_VALU_MFMA_BUSY_CYCLES + SQ_BUSY_CU_CYCLES (2 SQ slots) +
# GRBM_GUI_ACTIVE (1 GRBM slot) in one pass -> per-class MFMA utilisation (scripts/pmc_mfma.py). C2 leg (one clip,
# f32 graph on bf16x3, fp16 graph) and the C3 leg (32-clip encoder batch). Then the same for the exact-f32 GEMM mode.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for mode in bf16x3 f32; do
  rm -rf gpurun_out/pmcm
  FUNASR_GRAPHS=0 FUNASR_ENC_GEMM=$mode timeout -s KILL 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE \
    -d gpurun_out/pmcm -o pmc -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --c3-batch 32 --c3-steps 1 --no-c4 \
    > gpurun_out/pmcm_$mode.log 2>&1 || { echo "pmc pass failed rc=$?"; tail -30 gpurun_out/pmcm_$mode.log; exit 1; }
  db=$(find gpurun_out/pmcm -name "*results.db" | head -1)
  python3 scripts/pmc_mfma.py "$db" gpurun_out/pmc_mfma_$mode.json
  rm -rf gpurun_out/pmcm
done
