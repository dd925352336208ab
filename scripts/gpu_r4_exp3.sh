#!/bin/bash
# 128x64 one-clip GEMM tiles A/B + encoder parity; production-path (graph) kernel trace of a short bench; then the
# decode_step replica's graph under PMC (last: it may crash the profiler)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_parity.py tests/test_gpu_dist.py tests/test_gpu_ort_compat.py -k "encoder or dist or rccl or int8" -x -q -m gpu --timeout 240 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/t_enc.log 2>&1 || { tail -30 gpurun_out/t_enc.log; exit 1; }
tail -2 gpurun_out/t_enc.log
for mode in bf16x3 fp16; do for mid in 0 1 0 1; do
  FUNASR_BF3_MID=$mid timeout -k 10 120 python -u scripts/prof_encode.py 1 10 $mode 2>&1 | tail -1 | sed "s/^/mid=$mid /" || exit 1
done; done
rm -rf gpurun_out/ktg
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ktg -o kt -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --c3-batch 0 --c3-varlen 0 --no-c4 > gpurun_out/ktg.log 2>&1
echo "kernel-trace bench (graphs on) rc=$?"
python3 scripts/prof_summary.py gpurun_out/ktg/kt_results.db 16 > gpurun_out/ktg_summary.txt 2>&1; head -18 gpurun_out/ktg_summary.txt
rm -rf gpurun_out/ktg
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pds -o p -- scripts/ubench/decode_step fused2 > gpurun_out/pmc_ds_graph.log 2>&1
echo "pmc decode_step graph rc=$?"; grep -v "^    @" gpurun_out/pmc_ds_graph.log | tail -8
