#!/bin/bash
# Round 5 evidence set on one box: the GPU suite, the bench line, then the counter passes behind roofline.traffic:
#   FETCH_SIZE of the bench's decode launches with the batch-1 prefetch slabs OFF (the HBM bytes the layer launches
#   need: the slabs' pulls would otherwise be counted as well as the consumers' reads) and ON, and TCC hit / miss per
#   decode launch with the slabs on and off (does C hit the L2 lines AB's slab pulled?).
# STEPS: which parts to run (default "abw tests bench"; "pmc" separately); every GPU step has its own time limit and the chain stops at
# the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
STEPS=${STEPS:-"abw tests bench"}
if [[ " $STEPS " == *" abw "* ]]; then  # batch-32 graph-replayed decode step: lean VALU vs one-round-trip MFMA attention
  AB_M=32 timeout -k 10 300 python -u scripts/prof_decode_ab.py 128 FUNASR_ATTN_MFMA=0 FUNASR_ATTN_MFMA=1 \
    FUNASR_ATTN_MFMA=0 FUNASR_ATTN_MFMA=1 2>&1 | tee gpurun_out/ab_wide.log || exit 1
fi
if [[ " $STEPS " == *" tests "* ]]; then
  timeout -k 10 1000 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
  tail -2 gpurun_out/gpu_tests.log
fi
if [[ " $STEPS " == *" bench "* ]]; then
  timeout -k 10 900 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/bench.json').read().strip().splitlines()[-1])
print('C2', d['value'], d['stage_ms'], 'step1', d.get('decode_step_ms_graph')); print('roof', d['roofline']['frac'], d['roofline']['avg_launch_us'])
print('C3', d['c3']['value'], d['c3'].get('stage_ms'), 'step32', d['c3'].get('decode_step_ms_graph')); print('C4', d['c4']['value'], 'C5', d['c5']['value'], 'c5_long', d['c5_long']['value'])"
fi
if [[ " $STEPS " == *" trace "* ]]; then  # per-kernel device time of the bench workload, graph-replayed decode
  d=gpurun_out/prof
  DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $d -o run -- python3 bench.py \
    --steps 3 --warmup 1 --no-cpu-baseline --c3-varlen 0 > gpurun_out/prof.log 2>&1 || { tail -20 gpurun_out/prof.log; exit 1; }
  python3 scripts/prof_summary.py $(find $d -name "*results.db" | head -1) 45 > gpurun_out/prof_summary.txt; rm -rf $d
  echo "trace ok"
fi
if [[ " $STEPS " == *" pmc "* ]]; then
  export DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
  B="python3 -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --c3-batch 0 --c3-varlen 0 --no-c4"
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
