#!/bin/bash
# weight-gradient / fold tests + determinism tests, fold segment timings, cfg-2 step profile
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -q -m gpu -x \
  -k "weight_grad or wgrad or bitexact or layernorm or seq_embed or linear_ln_bwd or trainstep_vs_oracle" \
  --timeout 120 --timeout-method thread > gpurun_out/fold_tests.log 2>&1 || { tail -30 gpurun_out/fold_tests.log; exit 1; }
tail -2 gpurun_out/fold_tests.log
timeout -k 10 300 python tools/fold_segments.py > gpurun_out/fold_segments.txt 2>&1 || { tail -20 gpurun_out/fold_segments.txt; exit 1; }
head -4 gpurun_out/fold_segments.txt
bash tools/prof_step.sh r03f && head -20 gpurun_out/prof_r03f_step.txt
