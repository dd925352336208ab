#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 120 scripts/ubench/gemm_batch 32 > gpurun_out/gemm_batch32.txt 2>&1 || { tail -5 gpurun_out/gemm_batch32.txt; exit 1; }
cat gpurun_out/gemm_batch32.txt
timeout -k 10 120 scripts/ubench/gemm_batch_stamps 32 > gpurun_out/gemm_batch32_stamps.txt 2>&1 || { tail -5 gpurun_out/gemm_batch32_stamps.txt; exit 1; }
grep -v "kw" gpurun_out/gemm_batch32_stamps.txt | head -60
timeout -k 10 120 scripts/ubench/attn_batch 1024 > gpurun_out/attn_batch.txt 2>&1 || { tail -5 gpurun_out/attn_batch.txt; exit 1; }
cat gpurun_out/attn_batch.txt
bash scripts/gpu_trace_decode.sh
