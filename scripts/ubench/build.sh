#!/bin/bash
# Build the microbenchmarks against the engine's kernel objects (run from the repo root after build()).
set -e
B=fun-asr-gguf_amd/build; U=scripts/ubench; F="-O3 -std=c++17 --offload-arch=gfx950 -Iinclude"
hipcc $F -c $U/decode_step.hip -o /tmp/ds.o && hipcc --offload-arch=gfx950 /tmp/ds.o $B/llm.hip.o $B/synth.hip.o -o $U/decode_step
hipcc $F $U/edge_chain.hip -o $U/edge_chain
