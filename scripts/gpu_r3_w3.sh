#!/bin/bash
# separate MFMA accumulators in the q8_0 MFMA GEMMs + early K/V in the two-launch layer: microbenchmarks, GPU tests, bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
U=scripts/ubench
timeout -k 10 120 $U/gemm_batch 32 > gpurun_out/w3_gemm_batch32.txt 2>&1 || { tail -5 gpurun_out/w3_gemm_batch32.txt; exit 1; }
cat gpurun_out/w3_gemm_batch32.txt
timeout -k 10 60 $U/decode_step fused2 3 2>&1 | grep -E "decode step|B attn|C ffn|lm_head" || exit 1
timeout -k 10 300 python -u scripts/prof_batch_decode.py 32 64 > gpurun_out/w3_batch_decode.txt 2>&1 || { tail -5 gpurun_out/w3_batch_decode.txt; exit 1; }
tail -5 gpurun_out/w3_batch_decode.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/w3_tests.log 2>&1; rc=$?
tail -3 gpurun_out/w3_tests.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 600 python -u bench.py --no-cpu-baseline > gpurun_out/w3_bench.json 2> gpurun_out/w3_bench.err || { tail -5 gpurun_out/w3_bench.err; exit 1; }
python3 -c "
import json;d=json.load(open('gpurun_out/w3_bench.json'));print('C2',d['value'],d['stage_ms'],d['roofline']['avg_launch_us'],d['roofline']['frac'])
for k in ['c2_exact_f32','c3','c3_varlen','c4','c5']:
  v=d.get(k,{}); print(k, v.get('value', v.get('continuous')), v.get('stage_ms'))"
