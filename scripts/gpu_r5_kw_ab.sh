#!/bin/bash
# Row-local prefill GEMM (k_gemm_q8_kw) scaling A/B, same box, interleaved: this tree (block scales converted once per
# wave into LDS, packed f32 scaling) vs lib/diag/kw_old.so (each lane converting its 16 rows' fp16 scales per block)
# and lib/diag/kw_b6.so (this tree with the NBW = 4 form bounded to 6 waves per SIMD); one-prompt (C2) and 6-prompt
# row-local prefill with logits hashes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
L=fun-asr-gguf_amd/lib/libfunasr_hip.so; D=fun-asr-gguf_amd/lib/diag
pf() { FUNASR_HIP_LIB=$2 timeout -k 10 200 python -u scripts/prof_batch_prefill.py $3 204 6 2>&1 | sed "s/^/$1 B=$3 /" | tee -a gpurun_out/kw_ab.log; }
for r in 1 2; do
  pf new $L 1 && pf old $D/kw_old.so 1 && pf b6 $D/kw_b6.so 1 || exit 1
  pf new $L 6 && pf old $D/kw_old.so 6 && pf b6 $D/kw_b6.so 6 || exit 1
done
