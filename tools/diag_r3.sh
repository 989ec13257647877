#!/bin/bash
# Panel row-count scaling and a grouped-wgrad split sweep (chunked order) on the cfg-2 step.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python tools/panel_scale.py > gpurun_out/panel_scale.txt 2>&1 || { tail -20 gpurun_out/panel_scale.txt; exit 1; }
cat gpurun_out/panel_scale.txt
for g in 128:8 128:12 128:16 128:24 64:0; do
  TTMI_WGRAD_GROUP=$g timeout -k 10 300 python bench.py --skip-cpu --steps 200 --warmup 20 > gpurun_out/sw_$g.json 2> gpurun_out/sw_$g.err \
    || { tail -20 gpurun_out/sw_$g.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/sw_$g.json').read().strip().splitlines()[-1]);r=d['roofline'];print('group=$g', d['value'], d['ms_per_step'], r['avg_us'], r['frac'])"
done
