#!/bin/bash
# Software-pipelined weight-gradient loop: tests, stamps, encoder-shape group timing, cfg-2 A/B.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_colaunch.py tests/test_gpu_model.py -x -q \
  --timeout 120 --timeout-method thread > gpurun_out/pipe_tests.log 2>&1
rc=$?; tail -3 gpurun_out/pipe_tests.log; [ $rc -eq 0 ] || exit $rc
for d in 128 256; do
  TTMI_LIB=music-recommendation-multimodal_amd/lib/diag/libttmi_stamp.so timeout -k 10 120 python tools/stamp_wgrad.py --dim $d 2>&1 | grep -v amdgpu.ids || exit 1
done
cd /tmp
for d in 128 256; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/pipe_d$d -o run -- python3 $R/tools/wgrad_shapes.py --dim $d --blas 0 > $R/gpurun_out/pipe_d$d.log 2>&1 || { tail -5 $R/gpurun_out/pipe_d$d.log; exit 1; }
  echo "== D=$d $(grep err $R/gpurun_out/pipe_d$d.log)"; grep -E "wgrad_group" $R/gpurun_out/pipe_d$d/run_kernel_stats.csv | cut -d, -f1,4
done
cd $R
bash tools/ab.sh 2 - || exit 1
bash tools/ab.sh 1 - -- --dim 256 || exit 1
bash tools/prof_step.sh pipe && head -26 gpurun_out/prof_pipe_step.txt
