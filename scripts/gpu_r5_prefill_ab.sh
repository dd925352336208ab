#!/bin/bash
# same-box A/B of the 32-prompt prefill batch (scripts/prof_batch_prefill.py 32 204) and the one-prompt C2 prefill:
# current library vs fun-asr-gguf_amd/lib/diag/$OLD.so; prints ms per batch and a logits hash (bit-identity check)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
L=fun-asr-gguf_amd/lib/libfunasr_hip.so; O=fun-asr-gguf_amd/lib/diag/${OLD:-qt_old}.so
run() { FUNASR_HIP_LIB=$2 timeout -k 10 200 python -u scripts/prof_batch_prefill.py $3 204 4 2>&1 | sed "s/^/$1 B=$3 /" | tee -a gpurun_out/prefill_ab.log; }
for b in 32 1; do run new $L $b && run old $O $b && run new $L $b && run old $O $b || exit 1; done
