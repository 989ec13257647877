#!/bin/bash
# Segment lookup check: weight-gradient / fold / bit-exact tests, then three cfg-2 runs
# (roofline avg_us = the grouped wgrad + fold launches per GEMM; 4.15 us before).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -q -m gpu -x -k "wgrad or bitexact or fold or trainstep" --timeout 200 --timeout-method thread \
  > gpurun_out/seg_tests.log 2>&1 || { tail -30 gpurun_out/seg_tests.log; exit 1; }
tail -2 gpurun_out/seg_tests.log
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --skip-cpu --steps 200 --warmup 20 > gpurun_out/seg_$i.json 2> gpurun_out/seg_$i.err \
    || { tail -20 gpurun_out/seg_$i.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/seg_$i.json').read().strip().splitlines()[-1]);r=d['roofline'];print('run $i', d['value'], d['ms_per_step'], r['avg_us'], r['frac'])"
done
