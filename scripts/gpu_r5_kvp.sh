#!/bin/bash
# bf16x3 encoder attention staging K/V from bf16 planes written by the q|k|v GEMM's epilogue (FUNASR_ENC_KV_PLANES=1)
# vs splitting the f32 K/V rows in every block (=0): encoder-row hashes (bit-identity) and encode times, batch 32 / 6 /
# 1, interleaved; then the encoder GPU tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
en() { env FUNASR_ENC_KV_PLANES=$1 ENC_HASH=1 timeout -k 10 200 python -u scripts/prof_encode.py $2 5 bf16x3 2>&1 | sed "s/^/kvp=$1 B=$2 /" | tee -a gpurun_out/kvp.log; }
for r in 1 2; do
  en 1 32 && en 0 32 && en 1 6 && en 0 6 && en 1 1 && en 0 1 || exit 1
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py -x -v -m gpu -k "encoder" --timeout 300 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/kvp_tests.log 2>&1 || { tail -30 gpurun_out/kvp_tests.log; exit 1; }
tail -2 gpurun_out/kvp_tests.log
