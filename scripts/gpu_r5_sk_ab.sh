#!/bin/bash
# Split-K decode GEMM scaling A/B, same box, interleaved: this tree (block scales converted once per wave into LDS,
# packed f32 scaling, in k_gemm_q8_sk and k_gemm_q8_kw) vs lib/diag/kw_old.so (the previous commit's llm.hip):
# graph-replayed batch-32 and batch-1 steps with token + logits hashes, the row-local prefill, then the GPU suite.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
L=fun-asr-gguf_amd/lib/libfunasr_hip.so; O=fun-asr-gguf_amd/lib/diag/kw_old.so
dec() { FUNASR_HIP_LIB=$2 AB_M=$3 timeout -k 10 200 python -u scripts/prof_decode_ab.py 128 - 2>&1 | sed "s/^/$1 /" | tee -a gpurun_out/sk_ab.log; }
for r in 1 2; do
  dec new $L 32 && dec old $O 32 || exit 1
done
dec new $L 12 && dec old $O 12 && dec new $L 1 && dec old $O 1 || exit 1
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 240 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/sk_tests.log 2>&1 || { tail -40 gpurun_out/sk_tests.log; exit 1; }
tail -2 gpurun_out/sk_tests.log
