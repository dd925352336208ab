#!/bin/bash
# Small-batch MFMA LM head (k_lm_head_s, FUNASR_LM_HEAD_S): the GPU suite, then graph-replayed decode steps at batches
# 2, 3, 6 with it off / on (interleaved; the tokens+logits hash must not change), then the batch-6 step's launches.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 240 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/lms_tests.log 2>&1 || { tail -40 gpurun_out/lms_tests.log; exit 1; }
tail -2 gpurun_out/lms_tests.log
for m in 2 3 6; do
  AB_M=$m timeout -k 10 300 python -u scripts/prof_decode_ab.py 128 FUNASR_LM_HEAD_S=0 FUNASR_LM_HEAD_S=1 \
    FUNASR_LM_HEAD_S=2 FUNASR_LM_HEAD_S=0 FUNASR_LM_HEAD_S=1 FUNASR_LM_HEAD_S=2 2>&1 | tee -a gpurun_out/lms_ab.log || exit 1
done
AB_M=1 timeout -k 10 300 python -u scripts/prof_decode_ab.py 128 FUNASR_LM_HEAD_S1=0 FUNASR_LM_HEAD_S1=1 \
  FUNASR_LM_HEAD_S1=2 FUNASR_LM_HEAD_S1=0 FUNASR_LM_HEAD_S1=1 FUNASR_LM_HEAD_S1=2 2>&1 | tee -a gpurun_out/lms_ab.log || exit 1
for v in 1 2; do
d=gpurun_out/trs6_$v
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 FUNASR_LM_HEAD_S=$v AB_M=6 AB_REPS=1 timeout -s KILL 180 rocprofv3 --kernel-trace --stats -d $d -o run -- \
  python3 -u scripts/prof_decode_ab.py 64 - > $d.log 2>&1 || { tail -5 $d.log; exit 1; }
python3 scripts/prof_summary.py $(find $d -name "*results.db" | head -1) 12 > gpurun_out/trs6_${v}_summary.txt; rm -rf $d
cat gpurun_out/trs6_${v}_summary.txt
done
