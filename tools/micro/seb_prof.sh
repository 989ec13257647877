#!/bin/bash
# rocprofv3 kernel stats of tools/micro/seb_time.py against the shipped library and the
# -DTTMI_DIAG_NOATOM diagnostic build (lib/diag/libttmi_noatom.so).  GPU box, repo root.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
for v in ship noatom; do
  if [ $v = noatom ]; then export TTMI_LIB=$R/music-recommendation-multimodal_amd/lib/diag/libttmi_noatom.so; fi
  (cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/seb_$v -o run \
    -- python3 $R/tools/micro/seb_time.py) > $R/gpurun_out/seb_$v.log 2>&1 || exit 1
  f=$(ls $R/gpurun_out/seb_$v/*/run_kernel_stats.csv $R/gpurun_out/seb_$v/run_kernel_stats.csv 2>/dev/null | head -1)
  python3 - "$f" $v <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "seq_embed_bwd" in r["Name"]:
        print(sys.argv[2], "seq_embed_bwd", r["Calls"], round(float(r["AverageNs"]) / 1000, 2), "us")
PY
done
