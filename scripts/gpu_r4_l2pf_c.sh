#!/bin/bash
# batch-1 prefetch split: the attention launch's slab pulls only the FFN weights and the FFN launch's trailing slab
# (FUNASR_L2PF_C blocks per XCD) pulls the next layer's attention weights and K/V rows; 0 = all from the attention launch
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for c in 0 8 16 32 0 16 4; do
  FUNASR_L2PF_C=$c timeout -k 10 200 python -u scripts/prof_l2pf.py 256 16:50 2>&1 | sed "s/^/c=$c /" | tee -a gpurun_out/l2pf_c.log || exit 1
done
