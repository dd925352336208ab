#!/bin/bash
# device-assembled prompt rows: parity tests (new + the decode / scheduler / C4 exactness tests that now take that
# path), then bench legs C2 + C3 for the host-overhead change
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py -k "prefill_rows or c4_batch_of_6 or slot_reuse_equals or invariant_width_batch" -x -v -m gpu --timeout 300 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/t_rows.log 2>&1 || { tail -40 gpurun_out/t_rows.log; exit 1; }
grep -E "PASS|FAIL|passed|failed" gpurun_out/t_rows.log | tail -8
timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --c3-varlen 0 --no-c4 > gpurun_out/b_rows.json 2> gpurun_out/b_rows.err || { tail -20 gpurun_out/b_rows.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/b_rows.json').read().strip().splitlines()[-1])
print('C2', d['value'], d.get('stage_ms')); c3=d.get('c3', {}); print('C3', c3.get('value'), c3.get('ms_per_step'), c3.get('stage_ms'))"
# 256x256 bf16x3 tile diagnostics at M = 32032: default / no global loads / no MFMAs
for v in "" _v3 _v4; do
  timeout -k 10 300 scripts/ubench/gemm_f32_bench$v > gpurun_out/g256diag$v.txt 2>&1 || { tail -5 gpurun_out/g256diag$v.txt; exit 1; }
  echo "== gemm$v"; grep -E "M=32032" gpurun_out/g256diag$v.txt | sed 's/.*bf3 128x128x32/bf3 128x128x32/'
done
timeout -k 10 120 scripts/ubench/gemm_f32_bench kscan > gpurun_out/kscan.txt 2>&1 || { tail -5 gpurun_out/kscan.txt; exit 1; }
cat gpurun_out/kscan.txt
bash scripts/gpu_r4_exp6.sh
