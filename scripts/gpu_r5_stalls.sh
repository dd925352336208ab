#!/bin/bash
# SQ stall breakdown (one --pmc pass of 8 SQ counters each) of the batch-32 encoder GEMM / attention (planes on) and of
# the 32-prompt prefill GEMMs and attention: where do the waves of these kernels spend their cycles?
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS"
d=gpurun_out/st_enc
timeout -s KILL 120 rocprofv3 --pmc $C -d $d -o run -- python3 -u scripts/prof_encode.py 32 1 > $d.log 2>&1 || { tail -5 $d.log; exit 1; }
python3 scripts/pmc_kernels.py $(find $d -name "*results.db" | head -1) k_gemm_bf3_256 k_attn_bf3 k_layernorm k_fsmn > gpurun_out/stalls_enc.txt; rm -rf $d
d=gpurun_out/st_pf
timeout -s KILL 120 rocprofv3 --pmc $C -d $d -o run -- python3 -u scripts/prof_batch_prefill.py 32 204 1 > $d.log 2>&1 || { tail -5 $d.log; exit 1; }
python3 scripts/pmc_kernels.py $(find $d -name "*results.db" | head -1) k_gemm_q8_t k_attn_prefill k_qk_rope k_prep_q8 > gpurun_out/stalls_prefill.txt; rm -rf $d
head -40 gpurun_out/stalls_enc.txt; head -30 gpurun_out/stalls_prefill.txt
