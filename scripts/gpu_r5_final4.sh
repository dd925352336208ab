#!/bin/bash
# End-of-round evidence on the final tree: GPU suite, then the bench line twice (run-to-run spread on one box).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
STEPS="tests bench" bash scripts/gpu_r5_round.sh || exit 1
cp gpurun_out/bench.json gpurun_out/bench_a.json
timeout -k 10 900 python -u bench.py > gpurun_out/bench_b.json 2> gpurun_out/bench_b.err || { tail -20 gpurun_out/bench_b.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/bench_b.json').read().strip().splitlines()[-1])
print('B: C2', d['value'], 'step1', d.get('decode_step_ms_graph'), 'C3', d['c3']['value'], 'C4', d['c4']['value'], 'C5', d['c5']['value'], 'c5_long', d['c5_long']['value'])"
