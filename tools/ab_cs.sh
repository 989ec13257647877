#!/bin/bash
# Panel column split A/B: row-panel tests, then the cfg-2 step with CS=1 vs CS=2 (three pairs)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -q -m gpu -x \
  -k "row_panel or linear_ln_bwd or linear_res_ln or gemm_layouts or gemm_epilogue" --timeout 120 --timeout-method thread \
  > gpurun_out/cs_tests.log 2>&1 || { tail -30 gpurun_out/cs_tests.log; exit 1; }
tail -2 gpurun_out/cs_tests.log
for i in 1 2 3; do
  for c in 1 2; do
    TTMI_PANEL_CS=$c timeout -k 10 300 python bench.py --skip-cpu --steps 200 --warmup 20 > gpurun_out/cs_$c.json 2> gpurun_out/cs_$c.err \
      || { tail -20 gpurun_out/cs_$c.err; exit 1; }
    python -c "import json;d=json.loads(open('gpurun_out/cs_$c.json').read().strip().splitlines()[-1]);print('cs=$c', d['value'], d['ms_per_step'])"
  done
done
bash tools/prof_step.sh r03c && head -20 gpurun_out/prof_r03c_step.txt
