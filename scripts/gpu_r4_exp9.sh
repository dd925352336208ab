#!/bin/bash
# write-after-barrier staging: GEMM 256/128 tiles (now default) and the encoder attention (A/B), encodes, encoder parity
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 200 scripts/ubench/gemm_f32_bench sched > gpurun_out/sched2.txt 2>&1 || { tail -5 gpurun_out/sched2.txt; exit 1; }
grep "M=32032" gpurun_out/sched2.txt
timeout -k 10 200 scripts/ubench/attn_f32_bench wab > gpurun_out/wab.txt 2>&1 || { tail -5 gpurun_out/wab.txt; exit 1; }
cat gpurun_out/wab.txt
for w in 0 1 0 1; do
  FUNASR_ATTN_WAB=$w timeout -k 10 120 python -u scripts/prof_encode.py 32 3 bf16x3 2>&1 | tail -1 | sed "s/^/wab=$w /" || exit 1
  FUNASR_ATTN_WAB=$w timeout -k 10 120 python -u scripts/prof_encode.py 1 10 bf16x3 2>&1 | tail -1 | sed "s/^/wab=$w /" || exit 1
  FUNASR_ATTN_WAB=$w timeout -k 10 120 python -u scripts/prof_encode.py 1 10 fp16 2>&1 | tail -1 | sed "s/^/wab=$w /" || exit 1
done
FUNASR_ATTN_WAB=1 timeout -k 10 500 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_parity.py -k "encoder or encode or f16 or c4" -x -q -m gpu --timeout 300 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/t_wab.log 2>&1 || { tail -30 gpurun_out/t_wab.log; exit 1; }
tail -2 gpurun_out/t_wab.log
