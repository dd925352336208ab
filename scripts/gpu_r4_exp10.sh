#!/bin/bash
# (binaries: scripts/ubench/build_diag.sh) encoder attention ablations (FA_ATTN_DIAG 1-4: no K/V staging / no S MFMAs / no PV MFMAs / no softmax) vs the full
# kernel, graph-replayed, one clip and batch 32
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for v in "" _d1 _d2 _d3 _d4; do
  timeout -k 10 120 scripts/ubench/attn_f32_bench$v > gpurun_out/attn_diag$v.txt 2>&1 || { tail -5 gpurun_out/attn_diag$v.txt; exit 1; }
  echo "== attn_f32_bench$v"; grep -E "bf16x3 batch  1 splits 8 \(|bf16x3 batch 32 splits 1 \(" gpurun_out/attn_diag$v.txt
done
