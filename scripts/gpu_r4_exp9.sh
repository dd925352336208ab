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
for w in 0 1 0 1; do
  FUNASR_GEMM_T_WAB=$w timeout -k 10 120 python -u scripts/prof_batch_prefill.py 32 204 3 2>&1 | tail -1 | sed "s/^/gemm_t_wab=$w /" || exit 1
done
FUNASR_GEMM_T_WAB=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_fullsize.py -k "c3_bench_shape or batch32_vs_single" -x -q -m gpu --timeout 280 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/t_twab.log 2>&1 || { tail -30 gpurun_out/t_twab.log; exit 1; }
tail -2 gpurun_out/t_twab.log
for w in 0 1 0 1; do
  FUNASR_F32_WAB=$w timeout -k 10 120 python -u scripts/prof_encode.py 32 2 f32 2>&1 | tail -1 | sed "s/^/f32_wab=$w /" || exit 1
  FUNASR_F32_WAB=$w timeout -k 10 120 python -u scripts/prof_encode.py 1 10 f32 2>&1 | tail -1 | sed "s/^/f32_wab=$w /" || exit 1
done
timeout -k 10 180 python -u scripts/prof_c3_host.py 32 > gpurun_out/c3_host.txt 2>&1 || { tail -20 gpurun_out/c3_host.txt; exit 1; }
head -45 gpurun_out/c3_host.txt
