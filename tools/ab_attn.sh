#!/bin/bash
# attention kernel tests + fold segment timings + cfg-2 step profile
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -q -m gpu -x -k "mha or dropout" --timeout 120 --timeout-method thread \
  > gpurun_out/attn_tests.log 2>&1 || { tail -30 gpurun_out/attn_tests.log; exit 1; }
tail -2 gpurun_out/attn_tests.log
timeout -k 10 300 python tools/fold_segments.py > gpurun_out/fold_segments.txt 2>&1 || { tail -20 gpurun_out/fold_segments.txt; exit 1; }
bash tools/prof_step.sh r03a && head -30 gpurun_out/prof_r03a_step.txt
