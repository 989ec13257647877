#!/bin/bash
# A variant build of libttmi in which one source file gets extra compile-time flags, for A/B
# runs (tools/lib_ab.sh swaps it in on the GPU box).
#   usage: tools/lib_variant.sh NAME SRC "-DKNOB=V ..."    (SRC: e.g. ttmi_gemm)
set -e
cd "$(dirname "$0")/.."
name=$1; src=$2; flags=$3
make -s >/dev/null
mkdir -p build/var music-recommendation-multimodal_amd/lib/var
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -Iinclude $flags \
  -c music-recommendation-multimodal_amd/csrc/$src.hip -o build/var/${src}_$name.o
objs=$(ls build/*.o | grep -v "/$src.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $objs build/var/${src}_$name.o \
  -o music-recommendation-multimodal_amd/lib/var/libttmi_$name.so
echo music-recommendation-multimodal_amd/lib/var/libttmi_$name.so
