#!/bin/bash
# 256x256 bf16x3 GEMM variants (B3B_VARIANT 0 / 1 / 2) + 16-wave batch-32 decode attention
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
U=scripts/ubench
timeout -k 10 120 $U/attn_batch 1024 > gpurun_out/attn_wide.txt 2>&1 || { cat gpurun_out/attn_wide.txt; exit 1; }
cat gpurun_out/attn_wide.txt
for v in "" _v1 _v2; do
  timeout -k 10 300 $U/gemm_f32_bench$v > gpurun_out/g256$v.txt 2>&1 || { tail -5 gpurun_out/g256$v.txt; exit 1; }
  echo "== variant$v"; grep -E "variant 6|256x256 vs|M=32032" gpurun_out/g256$v.txt | sed 's/.*engine default *[0-9.]* us *[0-9.]* TF\/s//'
done
