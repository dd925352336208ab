#!/bin/bash
# split-K GEMM L2 prefetch slabs in batched decode (FUNASR_GEMM_PF mask:slabs:delay), graph-replayed step A/B at
# batches $PF_BS (default 32)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for b in ${PF_BS:-32}; do
  PF_B=$b timeout -k 10 500 python -u scripts/prof_gemm_pf.py 64 ${PF_SETTINGS:-0:1:100 7:1:100 15:1:100 7:2:100 7:1:50 7:1:150 1:1:100 2:1:100 4:1:100 0:1:100 7:2:50} \
    2>&1 | tee -a gpurun_out/gemm_pf2.log || exit 1
done
