#!/bin/bash
# Panel-kernel W staging A/B: parity tests, then cfg-2 step with VGPR staging vs LDS-DMA staging
# (three alternating pairs) and the per-kernel device times of one profiled run each.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -q -m gpu -x \
  -k "row_panel or linear_ln_bwd or linear_res_ln or seq_embed_fwd_norm1" --timeout 120 --timeout-method thread \
  > gpurun_out/ab_tests.log 2>&1 || { tail -30 gpurun_out/ab_tests.log; exit 1; }
tail -2 gpurun_out/ab_tests.log
for i in 1 2 3; do
  for w in 0 1; do
    TTMI_PANEL_WDMA=$w timeout -k 10 300 python bench.py --skip-cpu --steps 200 --warmup 20 > gpurun_out/ab_$w.json 2> gpurun_out/ab_$w.err \
      || { tail -20 gpurun_out/ab_$w.err; exit 1; }
    python -c "import json;d=json.loads(open('gpurun_out/ab_$w.json').read().strip().splitlines()[-1]);print('wdma=$w', d['value'], d['ms_per_step'])"
  done
done
