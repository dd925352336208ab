#!/bin/bash
# Two-launch batch-1 decode layer: microbenchmark (three- vs two-launch), its parity tests, then (FULL=1) the whole
# GPU suite and the bench line. Each GPU step has its own limit; stop at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for m in ${MODES:-fused fused2}; do
  timeout -k 5 120 ./scripts/ubench/decode_step $m > gpurun_out/ds_$m.txt 2>&1 || { cat gpurun_out/ds_$m.txt; exit 1; }
  cat gpurun_out/ds_$m.txt
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "fused or continuous" --timeout 120 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/t_fused.log 2>&1 || { tail -30 gpurun_out/t_fused.log; exit 1; }
tail -3 gpurun_out/t_fused.log
if [ -z "$FULL" ]; then exit 0; fi
bash scripts/gpu_tests.sh && NOPROF=1 bash scripts/gpu_round2.sh
