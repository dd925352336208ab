#!/bin/bash
# Encoder attention: tiles of valid keys only skip the mask and the -inf checks (this tree) vs lib/diag/attn_old.so
# (previous commit); batch-32 and one-clip encodes (bf16x3, fp16), interleaved, encoder-row hashes (bit-identity).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
L=fun-asr-gguf_amd/lib/libfunasr_hip.so; O=fun-asr-gguf_amd/lib/diag/attn_old.so
en() { FUNASR_HIP_LIB=$2 ENC_HASH=1 timeout -k 10 200 python -u scripts/prof_encode.py $3 5 $4 2>&1 | sed "s/^/$1 B=$3 $4 /" | tee -a gpurun_out/amask.log; }
for r in 1 2; do
  en new $L 32 bf16x3 && en old $O 32 bf16x3 && en new $L 32 fp16 && en old $O 32 fp16 || exit 1
  en new $L 1 bf16x3 && en old $O 1 bf16x3 && en new $L 1 fp16 && en old $O 1 fp16 || exit 1
done
