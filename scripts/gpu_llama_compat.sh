#!/bin/bash
# the llama.cpp-compatible library on the GPU (tests/test_gpu_llama_compat.py)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_llama_compat.py -x -v -m gpu --timeout 120 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/gpu_llama_compat.log 2>&1; rc=$?
tail -25 gpurun_out/gpu_llama_compat.log; exit $rc
