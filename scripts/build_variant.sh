#!/bin/bash
# A/B library variant: llm.hip compiled with extra -D flags, linked with the in-tree objects into
# fun-asr-gguf_amd/lib/var/<name>.so (select it with FUNASR_HIP_LIB=...). Usage: scripts/build_variant.sh name -DX=1 ...
set -e
cd "$(dirname "$0")/.."
name=$1; shift
B=fun-asr-gguf_amd/build; mkdir -p fun-asr-gguf_amd/lib/var
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-result "$@" -x hip -I include \
  -c fun-asr-gguf_amd/csrc/llm.hip -o $B/llm_$name.o
objs=$(ls $B/*.o | grep -v "llm\.hip\.o\|llm_" )
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o fun-asr-gguf_amd/lib/var/$name.so $B/llm_$name.o $objs
echo fun-asr-gguf_amd/lib/var/$name.so
