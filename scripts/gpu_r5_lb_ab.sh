#!/bin/bash
# Occupancy A/B (same box, interleaved): this tree (k_gemm_q8_t and the prefill / encoder attention bounded to two
# blocks per CU) vs fun-asr-gguf_amd/lib/diag/lb_old.so (the unbounded kernels): 32-prompt and one-prompt prefill with
# logits hashes, batch-32 and one-clip encode with encoder-row hashes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
L=fun-asr-gguf_amd/lib/libfunasr_hip.so; O=fun-asr-gguf_amd/lib/diag/lb_old.so
pf() { FUNASR_HIP_LIB=$2 timeout -k 10 200 python -u scripts/prof_batch_prefill.py $3 204 4 2>&1 | sed "s/^/$1 B=$3 /" | tee -a gpurun_out/lb_ab.log; }
en() { FUNASR_HIP_LIB=$2 ENC_HASH=1 timeout -k 10 200 python -u scripts/prof_encode.py $3 5 $4 2>&1 | sed "s/^/$1 B=$3 $4 /" | tee -a gpurun_out/lb_ab.log; }
for r in 1 2; do
  pf new $L 32 && pf old $O 32 || exit 1
  en new $L 32 bf16x3 && en old $O 32 bf16x3 && en new $L 1 bf16x3 && en old $O 1 bf16x3 || exit 1
  en new $L 1 fp16 && en old $O 1 fp16 || exit 1
done
pf new $L 1 && pf old $O 1
