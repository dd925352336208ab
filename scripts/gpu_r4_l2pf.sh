#!/bin/bash
# L2 prefetch blocks in the batch-1 attention launch (FUNASR_L2PF / _DELAY / _MASK): graph-replayed step A/B;
# LMT=1 also runs the default-policy LM-head build (lib/diag/libfunasr_hip_lmt.so, FA_LM_HEAD_NT=0)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
S="${L2PF_SETTINGS:-0:0 16:50}"
timeout -k 10 300 python -u scripts/prof_l2pf.py 256 $S 2>&1 | sed 's/^/nt  /' | tee gpurun_out/l2pf4.log || exit 1
if [ "${LMT:-0}" = 1 ]; then
  FUNASR_HIP_LIB=fun-asr-gguf_amd/lib/diag/libfunasr_hip_lmt.so timeout -k 10 300 python -u scripts/prof_l2pf.py 256 $S \
    2>&1 | sed 's/^/lmt /' | tee -a gpurun_out/l2pf4.log || exit 1
  timeout -k 10 300 python -u scripts/prof_l2pf.py 256 $S 2>&1 | sed 's/^/nt  /' | tee -a gpurun_out/l2pf4.log
fi
