#!/bin/bash
# Ablation builds of the encoder GEMM / attention microbenchmarks (run from the repo root after build(); results are
# wrong by construction): gemm_f32_bench_v{3,4} (B3B_VARIANT: no global loads / no MFMAs in the 256x256 tile) and
# attn_f32_bench_d{1..4} (FA_ATTN_DIAG: no K/V staging / no S MFMAs / no PV MFMAs / no softmax). They are
# gpurun-ignored: drop them from .gpurunignore before a run that needs them.
set -e
B=fun-asr-gguf_amd/build; U=scripts/ubench; F="-O3 -std=c++17 --offload-arch=gfx950 -Iinclude"
hipcc $F -c $U/gemm_f32_bench.hip -o /tmp/gf.o
for v in 3 4; do
  hipcc $F -DB3B_VARIANT=$v -x hip -c fun-asr-gguf_amd/csrc/gemm_f32.hip -o /tmp/gemm_v$v.o
  hipcc --offload-arch=gfx950 /tmp/gf.o /tmp/gemm_v$v.o $B/synth.hip.o -o $U/gemm_f32_bench_v$v
done
hipcc $F -c $U/attn_f32_bench.hip -o /tmp/af.o
for d in 1 2 3 4; do
  hipcc $F -DFA_ATTN_DIAG=$d -x hip -c fun-asr-gguf_amd/csrc/attn_f32.hip -o /tmp/attn_d$d.o
  hipcc --offload-arch=gfx950 /tmp/af.o /tmp/attn_d$d.o $B/synth.hip.o -o $U/attn_f32_bench_d$d
done
