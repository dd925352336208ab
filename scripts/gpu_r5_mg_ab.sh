#!/bin/bash
# (1) int8 MFMA with a 1.5 * 2^23 accumulator start (exact f32 conversion by v_pk_add_f32 instead of v_cvt_f32_i32):
#     this tree with FUNASR_ATTN_PF_F16=0 vs lib/diag/mg_old.so (the previous commit), interleaved: row-local prefill
#     (1 and 6 prompts), the 32-prompt tiled prefill, the graph-replayed batch-32 step, logits / token hashes equal.
# (2) the query-tiled prefill attention on f16 MFMAs (default; row-local forwards of >= 64 rows take it too) vs (1).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
L=fun-asr-gguf_amd/lib/libfunasr_hip.so; O=fun-asr-gguf_amd/lib/diag/mg_old.so
pf() { env $4 FUNASR_HIP_LIB=$2 timeout -k 10 200 python -u scripts/prof_batch_prefill.py $3 204 5 2>&1 | sed "s/^/$1 B=$3 /" | tee -a gpurun_out/mg_ab.log; }
dec() { env $4 FUNASR_HIP_LIB=$2 AB_M=$3 timeout -k 10 200 python -u scripts/prof_decode_ab.py 128 - 2>&1 | sed "s/^/$1 /" | tee -a gpurun_out/mg_ab.log; }
for r in 1 2; do
  for b in 1 6 32; do
    pf mg $L $b FUNASR_ATTN_PF_F16=0 && pf old $O $b X=0 && pf f16 $L $b X=0 || exit 1
  done
  dec mg $L 32 FUNASR_ATTN_PF_F16=0 && dec old $O 32 X=0 || exit 1
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_parity.py -x -v -m gpu --timeout 240 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/mg_tests.log 2>&1 || { tail -40 gpurun_out/mg_tests.log; exit 1; }
tail -2 gpurun_out/mg_tests.log
