#!/bin/bash
# cfg-2 bench under several grouped weight-gradient tilings (TTMI_WGRAD_GROUP="tile:splits"):
# step time and the wgrad family's per-GEMM time (roofline.avg_us).
set -o pipefail
mkdir -p gpurun_out
for cfg in "${@:-64:0 128:16 128:12 128:8 128:24}"; do
  TTMI_WGRAD_GROUP=$cfg timeout -k 10 300 python bench.py --skip-cpu --steps 100 --warmup 20 \
    > gpurun_out/sweep_$cfg.log 2>&1 || { tail -20 gpurun_out/sweep_$cfg.log; exit 1; }
  python -c "import json,sys;d=json.loads(open('gpurun_out/sweep_$cfg.log').read().strip().splitlines()[-1]);print('$cfg', d['value'], d['ms_per_step'], d['roofline']['avg_us'], d['roofline']['frac'])"
done
