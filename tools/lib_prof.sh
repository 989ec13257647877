#!/bin/bash
# On the GPU box: per-kernel mean durations (rocprofv3 --kernel-trace, 20-step cfg-2 bench) of
# several library builds.   usage: tools/lib_prof.sh FILTER LIB... [-- bench args]  ("-" = in-tree)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
flt=$1; shift
libs=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do libs+=("$1"); shift; done
[ "$1" = "--" ] && shift
L=music-recommendation-multimodal_amd/lib/libttmi.so
cp $L gpurun_out/.lib_default.so
rc=0
for v in "${libs[@]}"; do
  if [ "$v" = "-" ]; then cp gpurun_out/.lib_default.so $L; else cp "$v" $L; fi
  tag=$(basename "$v" .so | tr -c 'A-Za-z0-9_' '_')
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/lp_$tag -o run \
    -- python3 $R/bench.py --steps 20 --warmup 5 --skip-cpu "$@") > gpurun_out/lp_$tag.log 2>&1 \
    || { tail -20 gpurun_out/lp_$tag.log; rc=1; break; }
  f=$(ls gpurun_out/lp_$tag/*/run_kernel_trace.csv 2>/dev/null || ls gpurun_out/lp_$tag/run_kernel_trace.csv)
  python3 - "$f" "$flt" "$v" <<'PY'
import csv, statistics, sys
f, flt, v = sys.argv[1:4]
by = {}
for x in csv.DictReader(open(f)):
    if flt in x['Kernel_Name']:
        by.setdefault(x['Kernel_Name'][:60], []).append((int(x['End_Timestamp']) - int(x['Start_Timestamp'])) / 1000)
for k, d in sorted(by.items()):
    print(v, k, len(d), 'mean %.2f median %.2f min %.2f' % (statistics.mean(d), statistics.median(d), min(d)))
PY
done
cp gpurun_out/.lib_default.so $L
rm -f gpurun_out/.lib_default.so
exit $rc
