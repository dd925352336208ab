#!/bin/bash
# A/B of FA_KV_EARLY (0 / 1 / 2) on the graph-replayed decode step + the AB timeline of variant 2
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
U=scripts/ubench; o=gpurun_out/kv_ab.txt; : > $o
for i in 1 2 3; do
  for v in "" _e1 _e2; do
    timeout -k 10 60 $U/decode_step$v fused2 3 2>&1 | grep -E "decode step|B attn" | sed "s/^/[E$v] /" >> $o || exit 1
  done
done
cat $o
timeout -k 10 60 $U/attn_stamps_e2 1 a > gpurun_out/kv_stamps_e2.txt 2>&1 || exit 1
timeout -k 10 60 $U/attn_stamps 1 a > gpurun_out/kv_stamps_e0.txt 2>&1 || exit 1
grep -A16 "n_past 330" gpurun_out/kv_stamps_e0.txt; grep -A16 "n_past 330" gpurun_out/kv_stamps_e2.txt
