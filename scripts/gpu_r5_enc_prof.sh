#!/bin/bash
# Kernel classes of a batch-32 encode (60 s clips, full encoder dims) per activation mode: f32 rows (FUNASR_ENC_PLANES=0),
# bf16 planes with register staging (FUNASR_BF3_DMA=0) and with LDS-DMA staging; then (last: it may fail) the round-4
# graph-profiler repro, bench.py's C2 leg under --kernel-trace with HIP's graph packet capture ON.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for mode in "0 1" "1 0" "1 1"; do
  set -- $mode
  d=gpurun_out/pe_p$1_d$2
  FUNASR_ENC_PLANES=$1 FUNASR_BF3_DMA=$2 timeout -s KILL 180 rocprofv3 --kernel-trace --stats -d $d -o run -- \
    python3 -u scripts/prof_encode.py 32 2 > $d.log 2>&1 || { tail -5 $d.log; exit 1; }
  python3 scripts/prof_summary.py $(find $d -name "*results.db" | head -1) 25 > $d.summary.txt; rm -rf $d
  echo "planes=$1 dma=$2 ok"
done
if [ -n "$GRAPH_REPRO" ]; then
  unset DEBUG_CLR_GRAPH_PACKET_CAPTURE
  d=gpurun_out/ktg_pc_on
  timeout -s KILL 150 rocprofv3 --kernel-trace --stats -d $d -o run -- python3 bench.py --steps 2 --warmup 1 \
    --no-cpu-baseline --c3-batch 0 --c3-varlen 0 --no-c4 > $d.log 2>&1
  rc=$?
  echo "bench under kernel-trace, packet capture on: exit $rc"; tail -4 $d.log
  f=$(find $d -name "*results.db" | head -1); [ -n "$f" ] && python3 scripts/prof_summary.py $f 20 > $d.summary.txt
  rm -rf $d
fi
