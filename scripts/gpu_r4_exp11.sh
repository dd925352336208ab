#!/bin/bash
# LM head of 2-8 tokens with the transposed row x token reduction (FUNASR_LM_TR=1, default) vs wave_sum per value:
# batch invariance tests (M = 6 logits bit-identical to M = 1), small-batch decode steps, C4 / c5_long bench legs
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_parity.py -k "invariant_width or c4_batch_of_6 or slot_reuse_equals or batch or continuous" -x -q -m gpu --timeout 300 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/t_lmtr.log 2>&1 || { tail -30 gpurun_out/t_lmtr.log; exit 1; }
tail -2 gpurun_out/t_lmtr.log
for tr in 0 1 0 1; do
  FUNASR_LM_TR=$tr timeout -k 10 200 python -u scripts/prof_small_batch.py 32 2>&1 | sed "s/^/lm_tr=$tr /" || exit 1
done
for tr in 0 1; do
  FUNASR_LM_TR=$tr timeout -k 10 400 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --c3-batch 0 --c3-varlen 0 > gpurun_out/b_lmtr$tr.json 2> gpurun_out/b_lmtr$tr.err || { tail -20 gpurun_out/b_lmtr$tr.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/b_lmtr$tr.json').read().strip().splitlines()[-1])
print('lm_tr=$tr C2', d['value'], 'C4', d['c4']['value'], 'c5_long', d['c5_long']['value'])"
done
