#!/bin/bash
# Evidence set on one GPU box (the one reusable wrapper; the single-use round-3..5 wrappers were removed in round 6,
# their outputs are under profiles/ and the scripts in git history before commit "Hygiene: ...").
# STEPS selects the parts (default "tests bench"); every GPU step has its own time limit and the chain stops at the
# first failure:
#   tests   the GPU suite                         -> gpurun_out/gpu_tests.log
#   smoke   __graft_entry__.smoke()               -> gpurun_out/smoke.log
#   bench   python bench.py (defaults)            -> gpurun_out/bench.json
#   trace   kernel trace of the bench workload (graph-replayed decode, packet capture off) -> gpurun_out/prof_summary.txt
#   trace32 kernel trace of the graph-replayed batch-32 step                              -> gpurun_out/tr32_summary.txt
#   pmc     FETCH_SIZE of the bench's decode launches with the batch-1 prefetch slabs off / on, TCC hit rates
# TESTS: pytest selection for the tests step (default: the whole -m gpu suite)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
STEPS=${STEPS:-"tests bench"}
if [[ " $STEPS " == *" tests "* ]]; then
  timeout -k 10 1000 python -u -m pytest ${TESTS:-tests} -x -v -m gpu --timeout 300 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
  tail -2 gpurun_out/gpu_tests.log
fi
if [[ " $STEPS " == *" smoke "* ]]; then
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
  tail -1 gpurun_out/smoke.log
fi
if [[ " $STEPS " == *" bench "* ]]; then
  timeout -k 10 900 python -u bench.py ${BENCH_ARGS} > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/bench.json').read().strip().splitlines()[-1])
print('C2', d['value'], d['stage_ms'], 'step1', d.get('decode_step_ms_graph')); print('roof', d['roofline']['frac'], d['roofline']['avg_launch_us'])
for k in ('c3', 'c4', 'c5', 'c5_long'):
    if k in d: print(k, d[k].get('value'), d[k].get('stage_ms'), 'step', d[k].get('decode_step_ms_graph'))"
fi
if [[ " $STEPS " == *" trace "* ]]; then  # per-kernel device time of the bench workload, graph-replayed decode
  d=gpurun_out/prof
  DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $d -o run -- python3 bench.py \
    --steps 3 --warmup 1 --no-cpu-baseline --c3-varlen 0 > gpurun_out/prof.log 2>&1 || { tail -20 gpurun_out/prof.log; exit 1; }
  python3 scripts/prof_summary.py $(find $d -name "*results.db" | head -1) 45 > gpurun_out/prof_summary.txt; rm -rf $d
  echo "trace ok"
fi
if [[ " $STEPS " == *" trace32 "* ]]; then  # the graph-replayed batch-32 step's launches
  d=gpurun_out/tr32
  DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 AB_M=32 AB_REPS=1 timeout -s KILL 180 rocprofv3 --kernel-trace --stats -d $d -o run -- \
    python3 -u scripts/prof_decode_ab.py 64 - > $d.log 2>&1 || { tail -5 $d.log; exit 1; }
  python3 scripts/prof_summary.py $(find $d -name "*results.db" | head -1) 30 > gpurun_out/tr32_summary.txt; rm -rf $d
  head -14 gpurun_out/tr32_summary.txt
fi
if [[ " $STEPS " == *" pmc "* ]]; then
  export DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
  B="python3 -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --c2-only"
  for pf in 0 16; do
    d=gpurun_out/pmc_fetch_pf$pf
    FUNASR_L2PF=$pf timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $d -o run -- $B > $d.log 2>&1 || { tail -5 $d.log; exit 1; }
    f=$(find $d -name "*results.db" | head -1)
    python3 scripts/pmc_traffic.py $f gpurun_out/pmc_gemv_pf$pf.json > gpurun_out/pmc_gemv_pf$pf.txt && echo "fetch pf$pf ok"
    rm -rf $d
  done
  for pf in 0 16; do
    d=gpurun_out/pmc_hit_pf$pf
    FUNASR_L2PF=$pf AB_REPS=1 timeout -s KILL 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $d -o run -- \
      python3 -u scripts/prof_decode_ab.py 32 - > $d.log 2>&1 || { tail -5 $d.log; exit 1; }
    f=$(find $d -name "*results.db" | head -1)
    python3 scripts/pmc_l2hit.py $f gpurun_out/pmc_l2hit_pf$pf.json "FUNASR_L2PF=$pf" > gpurun_out/pmc_l2hit_pf$pf.txt && echo "l2hit pf$pf ok"
    rm -rf $d
  done
fi
