#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/c4_repeat.py 5 2>&1 | grep -v "^$" | tail -8
timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --c3-batch 0 --c3-varlen 0 > gpurun_out/bench_c4.json 2>gpurun_out/bench_c4.err || { tail gpurun_out/bench_c4.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_c4.json')); print('C2', d['value'], d['stage_ms'], 'C4', d['c4']['value'], d['c4']['ms_per_step'])"
timeout -k 10 300 python3 scripts/varlen_c3.py 192 32 4 2>&1 | tail -3 || exit 1
