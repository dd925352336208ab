#!/bin/bash
# Like build_ab_lib.sh for any one source file: the current objects with <unit>.hip replaced by the file given
#   scripts/build_ab_lib2.sh <unit> <src.hip> <name> [extra hipcc flags]  ->  fun-asr-gguf_amd/lib/diag/<name>.so
# (e.g. scripts/build_ab_lib2.sh attn_f32 /tmp/attn_f32_head.hip attn_old)
set -e
cd "$(dirname "$0")/.."
unit=$1; src=$2; name=$3; shift 3
mkdir -p fun-asr-gguf_amd/lib/diag /tmp/ab_build
cp "$src" fun-asr-gguf_amd/csrc/_ab_$unit.hip
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-result "$@" -x hip -I include \
  -c fun-asr-gguf_amd/csrc/_ab_$unit.hip -o /tmp/ab_build/${unit}_$name.o
rm -f fun-asr-gguf_amd/csrc/_ab_$unit.hip
objs=$(ls fun-asr-gguf_amd/build/*.o | grep -v "/$unit.hip.o")
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o fun-asr-gguf_amd/lib/diag/$name.so $objs /tmp/ab_build/${unit}_$name.o
echo "built fun-asr-gguf_amd/lib/diag/$name.so"
