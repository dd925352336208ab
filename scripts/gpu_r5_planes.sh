#!/bin/bash
# bf16x3 encoder activation planes (FUNASR_ENC_PLANES): bit-identity test, then encode timings interleaved 0/1
# (batch 32 and one clip, 60 s clips, full encoder dims, synthetic weights).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_fullsize.py -x -v -m gpu -k "planes_bit_identical or encoder_batch32_vs_oracle" \
  --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/planes_tests.log 2>&1 || { tail -30 gpurun_out/planes_tests.log; exit 1; }
tail -3 gpurun_out/planes_tests.log
IFS=, read -ra MODE_LIST <<< "${MODES:-0 1 0,1 0 0,1 1 0,0 1 1,1 0 1,1 1 1}"
for r in 1 2; do
  for mode in "${MODE_LIST[@]}"; do
    set -- $mode
    for b in ${BATCHES:-32 1}; do
      FUNASR_ENC_PLANES=$1 FUNASR_BF3_DMA=$2 FUNASR_BF3_PERSIST=$3 timeout -k 10 200 python3 -u scripts/prof_encode.py $b 5 2>&1 | \
        sed "s/^/planes=$1 dma=$2 persist=$3 /" | tee -a gpurun_out/planes_ab.log || exit 1
    done
  done
done
