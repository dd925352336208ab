#!/bin/bash
# round-3 experiments: split-K shape sweep at batch 32, variable-length continuous batching, recovery test,
# diagnostics tests with output
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for mb in 256 192 128 96; do
  echo -n "SK_MIN_BLOCKS=$mb B=32: "; FUNASR_SK_MIN_BLOCKS=$mb timeout -k 10 120 python3 scripts/prof_batch_decode.py 32 64 || exit 1
  echo -n "SK_MIN_BLOCKS=$mb B=16: "; FUNASR_SK_MIN_BLOCKS=$mb timeout -k 10 120 python3 scripts/prof_batch_decode.py 16 64 || exit 1
done
timeout -k 10 300 python -u -m pytest -x -q tests/test_gpu_parity.py -k "recovers" --timeout 120 -p no:cacheprovider 2>&1 | tail -3 || exit 1
timeout -k 10 300 python3 scripts/varlen_c3.py 64 32 8 2>&1 | tail -4 || exit 1
timeout -k 10 300 python3 scripts/varlen_c3.py 64 32 16 2>&1 | tail -3 || exit 1
timeout -k 10 300 python -u -m pytest -s -q tests/test_gpu_fullsize.py -k "hf_anchor or bound or batch_vs_alone" --timeout 300 -p no:cacheprovider 2>&1 | grep -v "^$" | tail -12
