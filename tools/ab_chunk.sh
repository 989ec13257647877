#!/bin/bash
# Grouped wgrad block order A/B on the cfg-2 step: XCD-chunked (default) vs tile-major
# (TTMI_WGRAD_CHUNK=0), three alternating pairs, then the chunked launch's PMC traffic.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -q -m gpu -k "wgrad or bitexact or fold" --timeout 120 --timeout-method thread \
  > gpurun_out/abc_tests.log 2>&1 || { tail -30 gpurun_out/abc_tests.log; exit 1; }
tail -2 gpurun_out/abc_tests.log
for i in 1 2 3; do
  for c in 1 0; do
    TTMI_WGRAD_CHUNK=$c timeout -k 10 300 python bench.py --skip-cpu --steps 200 --warmup 20 > gpurun_out/abc_$c.json 2> gpurun_out/abc_$c.err \
      || { tail -20 gpurun_out/abc_$c.err; exit 1; }
    python -c "import json;d=json.loads(open('gpurun_out/abc_$c.json').read().strip().splitlines()[-1]);r=d['roofline'];print('chunk=$c', d['value'], d['ms_per_step'], r['avg_us'], r['frac'])"
  done
done
bash tools/pmc_traffic.sh chunk 2 && python3 -c "import json;d=json.load(open('gpurun_out/traffic_chunk.json'));[print(k,v) for k,v in d.items() if 'wgrad' in k]"
