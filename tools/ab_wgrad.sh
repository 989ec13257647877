#!/bin/bash
# wgrad group ring depth A/B on the cfg-2 step: 4-deep (default) vs 5-deep, three alternating pairs.
set -o pipefail
mkdir -p gpurun_out
for i in 1 2 3; do
  for ns in 4 5; do
    TTMI_WGRAD_NS=$ns timeout -k 10 300 python bench.py --skip-cpu --steps 200 --warmup 20 > gpurun_out/abw_$ns.json 2> gpurun_out/abw_$ns.err \
      || { tail -20 gpurun_out/abw_$ns.err; exit 1; }
    python -c "import json;d=json.loads(open('gpurun_out/abw_$ns.json').read().strip().splitlines()[-1]);r=d['roofline'];print('ns=$ns', d['value'], d['ms_per_step'], r['avg_us'], r['frac'])"
  done
done
