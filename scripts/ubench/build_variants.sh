#!/bin/bash
# decode_step replicas of llm.hip compile-time variants (run from the repo root after build()):
#   scripts/ubench/build_variants.sh NAME "-DDEFINE=value ..." [NAME "..."]...  -> scripts/ubench/decode_step_NAME
set -e
B=fun-asr-gguf_amd/build; U=scripts/ubench; F="-O3 -std=c++17 --offload-arch=gfx950 -Iinclude"
hipcc $F -c $U/decode_step.hip -o /tmp/ds.o
while [ $# -ge 2 ]; do
  hipcc $F $2 -x hip -c fun-asr-gguf_amd/csrc/llm.hip -o /tmp/llm_$1.o
  hipcc --offload-arch=gfx950 /tmp/ds.o /tmp/llm_$1.o $B/llm_aux.o $B/synth.hip.o -o $U/decode_step_$1 2>/dev/null || \
    hipcc --offload-arch=gfx950 /tmp/ds.o /tmp/llm_$1.o $B/synth.hip.o -o $U/decode_step_$1
  shift 2
done
