#!/bin/bash
# decode_step (and, with VARIANT="-DNAME=value ...", decode_step_v from llm.hip with those defines) only
set -e
B=fun-asr-gguf_amd/build; U=scripts/ubench; F="-O3 -std=c++17 --offload-arch=gfx950 -Iinclude"
hipcc $F -c $U/decode_step.hip -o /tmp/ds.o && hipcc --offload-arch=gfx950 /tmp/ds.o $B/llm.hip.o $B/synth.hip.o -o $U/decode_step
if [ -n "$VARIANT" ]; then
  hipcc $F $VARIANT -x hip -c fun-asr-gguf_amd/csrc/llm.hip -o /tmp/llm_v.o
  hipcc --offload-arch=gfx950 /tmp/ds.o /tmp/llm_v.o $B/synth.hip.o -o $U/decode_step_v
fi
