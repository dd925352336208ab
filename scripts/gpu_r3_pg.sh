#!/bin/bash
# A/B of the attention-partial granule exchange (FA_PART_GRANULE) on the graph-replayed decode step, its AB
# timeline, the fused-layer GPU tests and a C2 bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
U=scripts/ubench; o=gpurun_out/pg_ab.txt; : > $o
for i in 1 2 3; do
  timeout -k 10 60 $U/decode_step fused2 3 >> $o 2>&1 || exit 1
  timeout -k 10 60 $U/decode_step_v fused2 3 | sed 's/^/[PG0] /' >> $o 2>&1 || exit 1
done
cat $o
timeout -k 10 60 $U/attn_stamps 1 a > gpurun_out/pg_stamps.txt 2>&1 || exit 1
cat gpurun_out/pg_stamps.txt | head -40
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pg_tests.log 2>&1; rc=$?
tail -3 gpurun_out/pg_tests.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u bench.py --no-cpu-baseline --c3-batch 0 --c3-varlen 0 --no-c4 > gpurun_out/pg_bench.json 2> gpurun_out/pg_bench.err || { tail -5 gpurun_out/pg_bench.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/pg_bench.json'));print(d['value'],d['stage_ms'],d['roofline']['avg_launch_us'],d['roofline']['frac'])"
