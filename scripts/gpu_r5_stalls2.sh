#!/bin/bash
# SQ stall breakdown (one --pmc pass of 8 SQ counters each) of the graph-replayed batch-32 decode step's launches and
# of the one-clip encoder (attention with key splits, the few-tile GEMMs).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS"
d=gpurun_out/st_dec
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 AB_M=32 AB_REPS=1 timeout -s KILL 150 rocprofv3 --pmc $C -d $d -o run -- \
  python3 -u scripts/prof_decode_ab.py 32 - > $d.log 2>&1 || { tail -5 $d.log; exit 1; }
python3 scripts/pmc_kernels.py $(find $d -name "*results.db" | head -1) k_lm_head_b k_attn_block k_gemm_q8_sk k_sample \
  > gpurun_out/stalls_dec32.txt; rm -rf $d
d=gpurun_out/st_enc1
timeout -s KILL 120 rocprofv3 --pmc $C -d $d -o run -- python3 -u scripts/prof_encode.py 1 2 > $d.log 2>&1 || { tail -5 $d.log; exit 1; }
python3 scripts/pmc_kernels.py $(find $d -name "*results.db" | head -1) k_gemm_bf3 k_attn_bf3 k_layernorm k_fsmn \
  > gpurun_out/stalls_enc1.txt; rm -rf $d
cat gpurun_out/stalls_dec32.txt gpurun_out/stalls_enc1.txt
