#!/bin/bash
# Encoder attention with the query tiles of one (head, clip) on one XCD (FUNASR_ATTN_XCD=1) vs dispatch order (=0):
# batch-32 encode (bf16x3 and fp16 graphs), batch 6 and one clip (key-split launches), interleaved, with encoder-row
# hashes (bit-identity).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
en() { env FUNASR_ATTN_XCD=$1 ENC_HASH=1 timeout -k 10 200 python -u scripts/prof_encode.py $2 5 $3 2>&1 | sed "s/^/xcd=$1 B=$2 $3 /" | tee -a gpurun_out/axcd.log; }
for r in 1 2; do
  en 1 32 bf16x3 && en 0 32 bf16x3 && en 1 32 fp16 && en 0 32 fp16 && en 1 6 bf16x3 && en 0 6 bf16x3 || exit 1
  en 1 1 bf16x3 && en 0 1 bf16x3 && en 1 1 fp16 && en 0 1 fp16 || exit 1
done
