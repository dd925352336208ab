#!/bin/bash
# quick GPU loop: selected parity tests (stop at first failure) -> C2-only bench (no CPU leg)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest ${TESTS:-tests} -x -v -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/gpu_tests.log | tail -40
if [ $rc -ne 0 ]; then grep -E "Error|assert" gpurun_out/gpu_tests.log | head -30; exit $rc; fi
timeout -k 10 400 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --c3-batch ${C3:-0} ${BENCH_EXTRA:---no-c4} > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
python - <<'PY'
import json; d = json.load(open("gpurun_out/bench.json"))
print("C2", d["value"], "ms/step", d["ms_per_step"], d["stage_ms"])
print("roofline", {k: d["roofline"].get(k) for k in ("kernel", "achieved", "frac", "avg_launch_us")}, d["kernel_class_avg_us"])
for k in ("c2_sampled", "c5", "c3", "c4"):
    if k in d: print(k, d[k].get("value"), d[k].get("ms_per_step"), d[k].get("stage_ms", d[k].get("generate_ms")))
PY
