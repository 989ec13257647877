#!/bin/bash
# Longest-first order of the grouped weight gradients: tests, D = 256 and cfg-2 A/B, step profile.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_colaunch.py tests/test_gpu_model.py -x -q \
  --timeout 120 --timeout-method thread -k "wgrad or fold or trainstep or cfg2 or deferred" > gpurun_out/lpt_tests.log 2>&1
rc=$?; tail -2 gpurun_out/lpt_tests.log; [ $rc -eq 0 ] || exit $rc
TTMI_LIB=music-recommendation-multimodal_amd/lib/diag/libttmi_stamp.so timeout -k 10 120 python tools/stamp_wgrad.py --dim 256 2>&1 | grep -v amdgpu.ids || exit 1
bash tools/ab.sh 2 - -- --dim 256 || exit 1
bash tools/ab.sh 2 - || exit 1
bash tools/prof_step.sh lpt_d256 --dim 256 && head -4 gpurun_out/prof_lpt_d256_step.txt
