#!/bin/bash
# attn_stamps only (llm.hip with -DFA_ATTN_STAMPS; the driver recompiled every time: it shares kernels.h structs)
set -e
B=fun-asr-gguf_amd/build; U=scripts/ubench; F="-O3 -std=c++17 --offload-arch=gfx950 -Iinclude"
hipcc $F -DFA_ATTN_STAMPS $VARIANT -x hip -c fun-asr-gguf_amd/csrc/llm.hip -o /tmp/llm_astamps.o
hipcc $F -c $U/attn_stamps.hip -o /tmp/as.o && hipcc --offload-arch=gfx950 /tmp/as.o /tmp/llm_astamps.o $B/synth.hip.o -o $U/attn_stamps
