#!/bin/bash
# Diagnostic build of libttmi with per-wave phase stamps (-DTTMI_STAMP, ttmi_common.h) into
# build/stamp/libttmi_stamp.so; the shipped library is untouched.  Run on the CPU container
# (hipcc cross-compiles); tools/stamp_phases.py loads it on the GPU box via TTMI_LIB.
set -e
cd "$(dirname "$0")/.."
mkdir -p build/stamp music-recommendation-multimodal_amd/lib/diag
for f in music-recommendation-multimodal_amd/csrc/*.hip; do
  b=$(basename "$f" .hip)
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -DTTMI_STAMP -Iinclude -c "$f" -o build/stamp/$b.o &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC build/stamp/*.o -o music-recommendation-multimodal_amd/lib/diag/libttmi_stamp.so
echo music-recommendation-multimodal_amd/lib/diag/libttmi_stamp.so
