#!/bin/bash
# On the GPU box: alternate library builds under the default 200-step cfg-2 bench.
#   usage: tools/lib_ab.sh PAIRS LIB_A LIB_B [-- bench args]   ("-" = the in-tree lib)
# The in-tree lib/libttmi.so is saved first and restored at the end (the box is a scratch copy).
set -o pipefail
mkdir -p gpurun_out
pairs=$1; shift
libs=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do libs+=("$1"); shift; done
[ "$1" = "--" ] && shift
L=music-recommendation-multimodal_amd/lib/libttmi.so
cp $L gpurun_out/.lib_default.so
rc=0
for i in $(seq 1 "$pairs"); do
  for v in "${libs[@]}"; do
    if [ "$v" = "-" ]; then cp gpurun_out/.lib_default.so $L; else cp "$v" $L; fi
    tag=$(basename "$v" .so | tr -c 'A-Za-z0-9_' '_')
    timeout -k 10 300 python bench.py --skip-cpu --steps 200 --warmup 20 "$@" > gpurun_out/lab_$tag.json \
      2> gpurun_out/lab_$tag.err || { tail -20 gpurun_out/lab_$tag.err; rc=1; break 2; }
    python3 -c "import json;d=json.loads(open('gpurun_out/lab_$tag.json').read().strip().splitlines()[-1]);print('$v', d['value'], d['ms_per_step'])"
  done
done
cp gpurun_out/.lib_default.so $L
rm -f gpurun_out/.lib_default.so
exit $rc
