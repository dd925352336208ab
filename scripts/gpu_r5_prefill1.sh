#!/bin/bash
# One-prompt (C2) prefill, 204 rows, full Qwen3-0.6B q8_0 shape: the tiled GEMM / query-tiled attention thresholds
# lowered below 204 rows vs the defaults (interleaved, logits hash = bit-identity check), then a kernel trace of the
# default with the launch-gap summary (scripts/prof_gaps.py).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
run() { env $2 timeout -k 10 200 python -u scripts/prof_batch_prefill.py 1 204 6 2>&1 | sed "s/^/$1 /" | tee -a gpurun_out/prefill1_ab.log; }
for r in 1 2; do
  run default "X=0" && run gemm_t "FUNASR_GEMM_T_MIN_M=128" && run attn_pf "FUNASR_ATTN_PREFILL_MIN_M=128" && \
    run both "FUNASR_GEMM_T_MIN_M=128 FUNASR_ATTN_PREFILL_MIN_M=128" || exit 1
done
d=gpurun_out/pf1
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $d -o run -- python3 -u scripts/prof_batch_prefill.py 1 204 6 > $d.log 2>&1 || { tail -5 $d.log; exit 1; }
f=$(find $d -name "*results.db" | head -1)
python3 scripts/prof_gaps.py $f 1400 | tee gpurun_out/pf1_gaps.txt; python3 scripts/prof_summary.py $f 20 > gpurun_out/pf1_summary.txt; rm -rf $d
