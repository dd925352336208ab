#!/bin/bash
# timelines: batch-32 decode attention blocks, the fused C launch; bare K/V stream rates
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
U=scripts/ubench
timeout -k 10 60 $U/attn_stamps 32 > gpurun_out/st_attn32.txt 2>&1 || { tail -5 gpurun_out/st_attn32.txt; exit 1; }
cat gpurun_out/st_attn32.txt
timeout -k 10 60 $U/attn_stamps 1 c > gpurun_out/st_c.txt 2>&1 || { tail -5 gpurun_out/st_c.txt; exit 1; }
cat gpurun_out/st_c.txt
timeout -k 10 60 $U/kv_stream > gpurun_out/st_kv.txt 2>&1 || { tail -5 gpurun_out/st_kv.txt; exit 1; }
cat gpurun_out/st_kv.txt
