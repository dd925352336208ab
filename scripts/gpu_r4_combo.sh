#!/bin/bash
# one box: the staging-schedule A/Bs (scripts/gpu_r4_exp9.sh), then the round-4 evidence set (scripts/gpu_round4.sh)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash scripts/gpu_r4_exp9.sh > gpurun_out/exp9.log 2>&1 || { tail -30 gpurun_out/exp9.log; exit 1; }
grep -v "^ *[0-9]* *[0-9.]* *[0-9.]* *[0-9.]* *[0-9.]* .*(" gpurun_out/exp9.log | head -60
bash scripts/gpu_round4.sh
