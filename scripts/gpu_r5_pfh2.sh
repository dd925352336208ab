#!/bin/bash
# Decode kernels back to the previous commit's code (only the tiled prefill GEMM keeps the 1.5 * 2^23 start): batch-32
# step vs lib/diag/mg_old.so with the per-row prefill (FUNASR_ATTN_PF_RL=0: same tokens) and with the default; then
# the one-prompt prefill's attention launches per kind under the kernel tracer (tiles vs per-row).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
L=fun-asr-gguf_amd/lib/libfunasr_hip.so; O=fun-asr-gguf_amd/lib/diag/mg_old.so
dec() { env $4 FUNASR_HIP_LIB=$2 AB_M=$3 timeout -k 10 200 python -u scripts/prof_decode_ab.py 128 - 2>&1 | sed "s/^/$1 /" | tee -a gpurun_out/pfh2_ab.log; }
dec rl0 $L 32 FUNASR_ATTN_PF_RL=0 && dec old $O 32 X=0 && dec new $L 32 X=0 && dec rl0 $L 32 FUNASR_ATTN_PF_RL=0 && dec old $O 32 X=0 && dec new $L 32 X=0 || exit 1
for v in 1 0; do
  d=gpurun_out/pft$v
  FUNASR_ATTN_PF_RL=$v timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $d -o run -- python3 -u scripts/prof_batch_prefill.py 1 204 6 > $d.log 2>&1 || { tail -5 $d.log; exit 1; }
  f=$(find $d -name "*results.db" | head -1)
  python3 scripts/prof_summary.py $f 12 > gpurun_out/pft${v}_summary.txt; rm -rf $d
done
cat gpurun_out/pft1_summary.txt gpurun_out/pft0_summary.txt
