#!/bin/bash
# final tree: full GPU suite + the bench line (no profiler passes; those are in scripts/gpu_round4.sh)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/gpu_tests_final.log 2>&1 || { tail -30 gpurun_out/gpu_tests_final.log; exit 1; }
tail -2 gpurun_out/gpu_tests_final.log
timeout -k 10 900 python -u bench.py > gpurun_out/bench_final.json 2> gpurun_out/bench_final.err || { tail -20 gpurun_out/bench_final.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/bench_final.json').read().strip().splitlines()[-1])
print('C2', d['value'], d['stage_ms']); print('C3', d['c3']['value'], d['c3']['stage_ms']); print('C4', d['c4']['value'], 'C5', d['c5']['value'], 'c5_long', d['c5_long']['value'])"
