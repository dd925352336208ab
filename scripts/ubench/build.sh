#!/bin/bash
# Build the microbenchmarks against the engine's kernel objects (run from the repo root after build()).
# VARIANT="-DNAME=value ..." builds decode_step_v / attn_stamps_v from llm.hip with those extra defines.
set -e
B=fun-asr-gguf_amd/build; U=scripts/ubench; F="-O3 -std=c++17 --offload-arch=gfx950 -Iinclude"
hipcc $F -c $U/decode_step.hip -o /tmp/ds.o && hipcc --offload-arch=gfx950 /tmp/ds.o $B/llm.hip.o $B/synth.hip.o -o $U/decode_step
hipcc $F $U/edge_chain.hip -o $U/edge_chain
hipcc $F $U/kv_stream.hip -o $U/kv_stream
hipcc $F -c $U/attn_f32_check.hip -o /tmp/afc.o && hipcc --offload-arch=gfx950 /tmp/afc.o $B/attn_f32.hip.o $B/synth.hip.o -o $U/attn_f32_check
hipcc $F -c $U/attn_f32_bench.hip -o /tmp/af.o && hipcc --offload-arch=gfx950 /tmp/af.o $B/attn_f32.hip.o $B/synth.hip.o -o $U/attn_f32_bench
hipcc $F -c $U/gemm_f32_bench.hip -o /tmp/gf.o && hipcc --offload-arch=gfx950 /tmp/gf.o $B/gemm_f32.hip.o $B/synth.hip.o -o $U/gemm_f32_bench
hipcc $F -c $U/gemm_batch.hip -o /tmp/gb.o && hipcc --offload-arch=gfx950 /tmp/gb.o $B/llm.hip.o $B/synth.hip.o -o $U/gemm_batch
hipcc $F -c $U/attn_batch.hip -o /tmp/ab.o && hipcc --offload-arch=gfx950 /tmp/ab.o $B/llm.hip.o $B/synth.hip.o -o $U/attn_batch
hipcc $F -DFA_GEMV_STAMPS -x hip -c fun-asr-gguf_amd/csrc/llm.hip -o /tmp/llm_gstamps.o
hipcc $F -c $U/gemv_stamps.hip -o /tmp/gs.o && hipcc --offload-arch=gfx950 /tmp/gs.o /tmp/llm_gstamps.o $B/synth.hip.o -o $U/gemv_stamps
hipcc $F -DFA_GEMV_STAMPS -c $U/gemm_batch.hip -o /tmp/gbs.o && hipcc --offload-arch=gfx950 /tmp/gbs.o /tmp/llm_gstamps.o $B/synth.hip.o -o $U/gemm_batch_stamps
hipcc $F -DFA_ATTN_STAMPS -x hip -c fun-asr-gguf_amd/csrc/llm.hip -o /tmp/llm_astamps.o
hipcc $F -c $U/attn_stamps.hip -o /tmp/as.o && hipcc --offload-arch=gfx950 /tmp/as.o /tmp/llm_astamps.o $B/synth.hip.o -o $U/attn_stamps
if [ -n "$VARIANT" ]; then
  hipcc $F $VARIANT -x hip -c fun-asr-gguf_amd/csrc/llm.hip -o /tmp/llm_v.o
  hipcc --offload-arch=gfx950 /tmp/ds.o /tmp/llm_v.o $B/synth.hip.o -o $U/decode_step_v
  hipcc $F $VARIANT -DFA_ATTN_STAMPS -x hip -c fun-asr-gguf_amd/csrc/llm.hip -o /tmp/llm_vastamps.o
  hipcc --offload-arch=gfx950 /tmp/as.o /tmp/llm_vastamps.o $B/synth.hip.o -o $U/attn_stamps_v
fi
