#!/bin/bash
# C3 leg of bench.py with the batched-decode GEMM L2 prefetch off / on (FUNASR_GEMM_PF 0 / 7), interleaved on one box
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for pf in 0 7 0 7; do
  FUNASR_GEMM_PF=$pf timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --c3-batch 32 --c3-steps 2 --no-c4 --c3-varlen 0 \
    > gpurun_out/c3pf_$pf.json 2> gpurun_out/c3pf_$pf.err || { tail -20 gpurun_out/c3pf_$pf.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/c3pf_$pf.json').read().strip().splitlines()[-1])
print('gemm_pf=$pf C3', d['c3']['value'], d['c3']['stage_ms'], 'C2', d['value'], 'roof', d['roofline']['frac'], d['roofline']['avg_launch_us'])" | tee -a gpurun_out/c3pf.log
done
