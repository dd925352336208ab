#!/bin/bash
# int8-dynamic CTC head GPU tests + the whole GPU suite + kernel trace of the one-clip fp16 encode
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_ctc_int8.py -x -v -s -m gpu --timeout 240 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/i8_tests.log 2>&1 || { tail -40 gpurun_out/i8_tests.log; exit 1; }
grep -E "differ|passed|failed" gpurun_out/i8_tests.log
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
rm -rf gpurun_out/pe
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pe -o run -- python3 scripts/prof_encode.py 1 3 fp16 > gpurun_out/pe.log 2>&1 || { tail -20 gpurun_out/pe.log; exit 1; }
python3 scripts/prof_summary.py gpurun_out/pe/run_results.db 14 > gpurun_out/enc_f16_b1_kernels.txt 2>&1; head -16 gpurun_out/enc_f16_b1_kernels.txt
rm -rf gpurun_out/pe
