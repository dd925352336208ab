#!/bin/bash
# Build an A/B variant of libfunasr_hip.so (CPU side, before a gpurun call): the current objects with llm.hip replaced
# by the file given (e.g. a git show of an earlier revision, or a copy with a -D switch):
#   scripts/build_ab_lib.sh <llm.hip> <name> [extra hipcc flags]  ->  fun-asr-gguf_amd/lib/diag/<name>.so
set -e
cd "$(dirname "$0")/.."
src=$1; name=$2; shift 2
mkdir -p fun-asr-gguf_amd/lib/diag /tmp/ab_build
cp "$src" fun-asr-gguf_amd/csrc/_ab_llm.hip
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-result "$@" -x hip -I include \
  -c fun-asr-gguf_amd/csrc/_ab_llm.hip -o /tmp/ab_build/llm_$name.o
rm -f fun-asr-gguf_amd/csrc/_ab_llm.hip
objs=$(ls fun-asr-gguf_amd/build/*.o | grep -v llm.hip.o)
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o fun-asr-gguf_amd/lib/diag/$name.so $objs /tmp/ab_build/llm_$name.o
echo "built fun-asr-gguf_amd/lib/diag/$name.so"
