#!/bin/bash
# GPU: parity tests (stop at first failure) -> bench (no CPU leg) ; extra env passes through (e.g. FUNASR_GEMM_KW=0)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1; rc=$?
grep -E "passed|failed" gpurun_out/gpu_tests.log | tail -3
if [ $rc -ne 0 ]; then grep -E "Error|assert|FAILED" gpurun_out/gpu_tests.log | head -30; exit $rc; fi
timeout -k 10 600 python bench.py --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
python - <<'PY'
import json; d = json.load(open("gpurun_out/bench.json"))
print("C2 value", d["value"], "ms/step", d["ms_per_step"], d["stage_ms"])
print("roofline", {k: d["roofline"][k] for k in ("kernel", "achieved", "frac", "avg_launch_us")}, d["kernel_class_avg_us"])
print("C3", d["c3"].get("value"), d["c3"].get("ms_per_step"), d["c3"].get("stage_ms"))
print("C5", d["c5"].get("value"), d["c5"].get("ms_per_step"), d["c5"].get("stage_ms"))
print("C4", d.get("c4"))
PY
