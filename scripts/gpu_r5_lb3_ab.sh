#!/bin/bash
# k_gemm_q8_t EPI 0 / 1 (q|k|v, o, down of the batched prefill) at three blocks per CU (lib/diag/lb3.so: 168 VGPRs, a
# 12-20 B spill) vs two (this tree), interleaved, 32-prompt prefill with logits hashes
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
L=fun-asr-gguf_amd/lib/libfunasr_hip.so; O=fun-asr-gguf_amd/lib/diag/lb3.so
pf() { FUNASR_HIP_LIB=$2 timeout -k 10 200 python -u scripts/prof_batch_prefill.py 32 204 4 2>&1 | sed "s/^/$1 /" | tee -a gpurun_out/lb3_ab.log; }
for r in 1 2; do pf two $L && pf three $O || exit 1; done
