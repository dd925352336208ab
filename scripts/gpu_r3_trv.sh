#!/bin/bash
# bf16x3 encoder attention: transposed-read V (FA_ATTN_TRV=1) vs f32 V tile (v0): correctness + hashes, timings
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
U=scripts/ubench
for v in "" _v0; do
  timeout -k 10 200 $U/attn_f32_check$v > gpurun_out/trv_check$v.txt 2>&1 || { tail -5 gpurun_out/trv_check$v.txt; exit 1; }
  echo "== check$v"; grep -v "^split" gpurun_out/trv_check$v.txt | tail -16
  timeout -k 10 200 $U/attn_f32_bench$v > gpurun_out/trv_bench$v.txt 2>&1 || { tail -5 gpurun_out/trv_bench$v.txt; exit 1; }
  echo "== bench$v"; grep "bf16x3" gpurun_out/trv_bench$v.txt
done
