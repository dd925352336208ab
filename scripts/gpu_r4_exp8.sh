#!/bin/bash
# 256x256 staging schedule A/B (write-after-barrier) + batch-32 encode; fp16 128-deep one-clip stages: parity + encode A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 200 scripts/ubench/gemm_f32_bench sched > gpurun_out/sched.txt 2>&1 || { tail -5 gpurun_out/sched.txt; exit 1; }
grep "M=32032" gpurun_out/sched.txt
for s in 0 1 0 1; do
  FUNASR_BF3_256_S=$s timeout -k 10 120 python -u scripts/prof_encode.py 32 3 bf16x3 2>&1 | tail -1 | sed "s/^/sched=$s /" || exit 1
done
timeout -k 10 400 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_parity.py -k "f16 or fp16 or batch32" -x -q -m gpu --timeout 240 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/t_f16deep.log 2>&1 || { tail -30 gpurun_out/t_f16deep.log; exit 1; }
tail -2 gpurun_out/t_f16deep.log
for d in 0 1 0 1; do
  FUNASR_F16_DEEP=$d timeout -k 10 120 python -u scripts/prof_encode.py 1 10 fp16 2>&1 | tail -1 | sed "s/^/f16deep=$d /" || exit 1
done
