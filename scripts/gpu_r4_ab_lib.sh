#!/bin/bash
# same-box A/B of the batch-1 graph-replayed step: current library vs lib/diag/libfunasr_hip_old.so (an earlier commit, built by hand from git show)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
run() { FUNASR_HIP_LIB=$2 timeout -k 10 200 python -u scripts/prof_l2pf.py 256 16:50 2>&1 | sed "s/^/$1 /" | tee -a gpurun_out/ab_lib.log; }
L=fun-asr-gguf_amd/lib/libfunasr_hip.so; O=fun-asr-gguf_amd/lib/diag/libfunasr_hip_old.so
run new $L && run old $O && run new $L && run old $O
