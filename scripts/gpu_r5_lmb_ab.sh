#!/bin/bash
# Batched LM head packed scaling A/B (this tree vs lib/diag/lmb_old.so = this tree with the scalar k_lm_head_b),
# graph-replayed batch-32 step, interleaved, old first; the batch-1 step in both orders (process-order check); then
# the bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
L=fun-asr-gguf_amd/lib/libfunasr_hip.so; O=fun-asr-gguf_amd/lib/diag/lmb_old.so
dec() { FUNASR_HIP_LIB=$2 AB_M=$3 timeout -k 10 200 python -u scripts/prof_decode_ab.py 128 - 2>&1 | sed "s/^/$1 /" | tee -a gpurun_out/lmb_ab.log; }
dec old $O 32 && dec new $L 32 && dec old $O 32 && dec new $L 32 || exit 1
dec old $O 1 && dec new $L 1 && dec new $L 1 && dec old $O 1 || exit 1
timeout -k 10 600 python -u bench.py > gpurun_out/bench_lmb.json 2> gpurun_out/bench_lmb.err || { tail -20 gpurun_out/bench_lmb.err; exit 1; }
cut -c1-400 gpurun_out/bench_lmb.json
