#!/bin/bash
# Round-5 counter passes (each its own rocprofv3 --pmc run): MFMA-pipe busy of the encoder kernels (bf16x3 at batch 32 via
# the bench's C3 leg, and the fp16 graph at batch 32), and FETCH_SIZE of the batch-6 decode step (k_lm_head_s traffic).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
for mode in bf16x3 fp16; do
  d=gpurun_out/pmcm_$mode
  if [ $mode = fp16 ]; then cmd="scripts/prof_encode.py 32 2 fp16"; else cmd="scripts/prof_encode.py 32 2 bf16x3"; fi
  timeout -s KILL 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE -d $d -o pmc -- \
    python3 $cmd > $d.log 2>&1 || { echo "pmc mfma pass failed"; tail -20 $d.log; exit 1; }
  db=$(find $d -name "*results.db" | head -1)
  python3 scripts/pmc_mfma.py "$db" gpurun_out/r05_pmc_mfma_$mode.json | head -20
  rm -rf $d
done
d=gpurun_out/pmcf6
AB_M=6 AB_REPS=1 timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $d -o pmc -- python3 -u scripts/prof_decode_ab.py 32 - \
  > $d.log 2>&1 || { echo "fetch pass failed"; tail -20 $d.log; exit 1; }
db=$(find $d -name "*results.db" | head -1)
python3 - "$db" <<'PY' | tee gpurun_out/r05_pmc_fetch_lm_head_s.txt
import sqlite3, sys
from collections import defaultdict
c = sqlite3.connect(sys.argv[1])
cols = [r[1] for r in c.execute("pragma table_info(pmc_events)").fetchall()]
disp = "dispatch_id" if "dispatch_id" in cols else "correlation_id"
tot = defaultdict(float); n = defaultdict(set)
for name, cn, v, d in c.execute(f"select name, counter_name, counter_value, {disp} from pmc_events"):
    if cn.startswith("FETCH_SIZE"):
        tot[name] += v; n[name].add(d)
print("# FETCH_SIZE x 2 per launch (MI355X_MICROARCH.md: gfx950 reports half the bytes of a wide streaming read), batch-6 decode step")
for name in sorted(tot, key=lambda k: -tot[k])[:8]:
    k = len(n[name]) or 1
    print(f"{2 * tot[name] * 1024 / k / 1e6:10.2f} MB per launch  {k:6d} launches  {name[:110]}")
PY
rm -rf $d
