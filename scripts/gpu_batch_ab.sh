#!/bin/bash
# batched-decode A/B: decoder parity tests (stop at the first failure), then batch-32 step time per knob setting
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -k "${K:-llm}" -x -v -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_batch_tests.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/gpu_batch_tests.log | tail -20
if [ $rc -ne 0 ]; then grep -E "Error|assert" gpurun_out/gpu_batch_tests.log | head -30; exit $rc; fi
for v in ${AB:-0 1}; do
  echo "${KNOB:-FUNASR_DECODE_NRM}=$v"; env ${KNOB:-FUNASR_DECODE_NRM}=$v timeout -k 10 200 python3 scripts/prof_batch_decode.py ${B:-32} 64 || exit 1
done
