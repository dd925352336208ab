#!/bin/bash
# the reference-ABI drop-ins on the GPU: onnxruntime-compatible sessions and the llama.cpp-compatible library
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_ort_compat.py tests/test_gpu_llama_compat.py tests/test_gpu_compat_pipeline.py -x -v -m gpu \
  --timeout 180 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_compat.log 2>&1; rc=$?
tail -30 gpurun_out/gpu_compat.log; exit $rc
