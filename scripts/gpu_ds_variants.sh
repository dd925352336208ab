#!/bin/bash
# decode_step microbenchmark: the default build and the variants given in VARS (binaries scripts/ubench/decode_step_*)
# in mode MODE (default fused2), then the fused-layer parity tests. Each GPU step has its own limit.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for rep in $(seq ${REPS:-1}); do
  for b in decode_step ${VARS}; do
    echo "== $b"
    timeout -k 5 120 ./scripts/ubench/$b ${MODE:-fused2} > gpurun_out/ds_$b.txt 2>&1 || { cat gpurun_out/ds_$b.txt; exit 1; }
    grep -v "^weights" gpurun_out/ds_$b.txt | head -${LINES_PER:-20}
  done
done
if [ -n "$STAMPS" ]; then
  for m in $STAMPS; do timeout -k 5 60 ./scripts/ubench/attn_stamps 1 $m | head -12 || exit 1; done
fi
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "fused or continuous" --timeout 120 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/t_fused.log 2>&1 || { tail -30 gpurun_out/t_fused.log; exit 1; }
tail -2 gpurun_out/t_fused.log
