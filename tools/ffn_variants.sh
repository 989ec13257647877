#!/bin/bash
# Variant builds of libttmi differing only in ttmi_ffn.hip's compile-time knobs, for A/B timing
# with tools/ffn_time.py (TTMI_LIB=...).  usage: tools/ffn_variants.sh NAME "-DKNOB=V ..." [NAME FLAGS]...
set -e
cd "$(dirname "$0")/.."
make -s >/dev/null
mkdir -p build/var music-recommendation-multimodal_amd/lib/var
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -Iinclude $flags \
    -c music-recommendation-multimodal_amd/csrc/ttmi_ffn.hip -o build/var/ttmi_ffn_$name.o
  objs=$(ls build/*.o | grep -v ttmi_ffn.o)
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $objs build/var/ttmi_ffn_$name.o \
    -o music-recommendation-multimodal_amd/lib/var/libttmi_$name.so
  echo music-recommendation-multimodal_amd/lib/var/libttmi_$name.so
done
