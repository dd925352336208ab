#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q -s tests/test_gpu_fullsize.py -k "batch_vs_alone or c4_batch_of_6 or invariant_width" --timeout 300 -p no:cacheprovider 2>&1 | grep -v "^$" | tail -4 || exit 1
timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --c3-batch 0 --c3-varlen 0 > gpurun_out/bench_c4.json 2>gpurun_out/bench_c4.err || { tail gpurun_out/bench_c4.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_c4.json')); print('C2', d['value'], 'C4', d['c4']['value'], d['c4']['ms_per_step'])"
timeout -k 10 300 python3 scripts/varlen_c3.py 192 32 4 2>&1 | tail -3 || exit 1
timeout -k 10 300 python3 scripts/varlen_c3.py 192 32 8 2>&1 | tail -2 || exit 1
