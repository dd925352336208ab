#!/bin/bash
# round-4 experiments: AB split granularity (AMIN_G), long single-prompt prefill row-local vs tiled, PMC on graph replay
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for v in base g4 g16 base; do
  echo "== decode_step_$v"; timeout -k 10 120 scripts/ubench/decode_step_$v fused2 | grep -E "decode step|AB|A\+B|C ffn|lm_head|TIMEOUT" || exit 1
done
timeout -k 10 180 python -u scripts/prof_prefill_long.py 204 512 1024 2000 || exit 1
FUNASR_PF_ROW_LOCAL_MAX=511 timeout -k 10 180 python -u scripts/prof_prefill_long.py 204 512 1024 2000 || exit 1
rm -rf gpurun_out/pmcg
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmcg -o pmc -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --c3-batch 0 --no-c4 --c3-varlen 0 > gpurun_out/pmc_graph.log 2>&1
echo "pmc graph pass rc=$?"; tail -25 gpurun_out/pmc_graph.log
