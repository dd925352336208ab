#!/bin/bash
# four K groups per block for one clip's K = 2048 GEMMs (ffn2): microbenchmark + checks, encoder parity with the knob
# on, one-clip encode A/B in both graphs; then the graph kernarg repro bare / under the profiler
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 200 scripts/ubench/gemm_f32_bench > gpurun_out/kw4_bench.txt 2>&1 || { tail -20 gpurun_out/kw4_bench.txt; exit 1; }
grep -E "check|M= 1001" gpurun_out/kw4_bench.txt
FUNASR_BF3_KW4=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_parity.py -k "encoder or encode or f16" -x -q -m gpu --timeout 240 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/t_kw4.log 2>&1 || { tail -30 gpurun_out/t_kw4.log; exit 1; }
tail -2 gpurun_out/t_kw4.log
for mode in bf16x3 fp16; do for kw in 0 1 0 1; do
  FUNASR_BF3_KW4=$kw timeout -k 10 120 python -u scripts/prof_encode.py 1 10 $mode 2>&1 | tail -1 | sed "s/^/$mode kw4=$kw /" || exit 1
done; done
bash scripts/gpu_r4_exp4.sh
