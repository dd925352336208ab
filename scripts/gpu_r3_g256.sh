#!/bin/bash
# 256x256 bf16x3 encoder GEMM: correctness spot checks, bit-identity vs 128x128, timings at M = 1001 / 32032
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 scripts/ubench/gemm_f32_bench > gpurun_out/g256.txt 2>&1; rc=$?
cat gpurun_out/g256.txt; exit $rc
