#!/bin/bash
# 256 x 256 weight-gradient tiles (D = 256): the wgrad / model tests, the encoder-shape group
# per split count, and the D = 256 bench A/B against 128 x 128 tiles.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_colaunch.py tests/test_gpu_model.py -x -q \
  --timeout 120 --timeout-method thread -k "wgrad or fold or trainstep or cfg2 or deferred" > gpurun_out/wide_tests.log 2>&1
rc=$?; tail -3 gpurun_out/wide_tests.log; [ $rc -eq 0 ] || exit $rc
cd /tmp
for s in "-" "TTMI_WGRAD_WIDE=0" "TTMI_WGRAD_WIDE=12" "TTMI_WGRAD_WIDE=24"; do
  envs=(); [ "$s" != "-" ] && envs=("$s")
  tag=wide_$(echo "$s" | tr -c 'A-Za-z0-9_' '_')
  env "${envs[@]}" timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/$tag -o run -- python3 $R/tools/wgrad_shapes.py --dim 256 --blas 0 > $R/gpurun_out/$tag.log 2>&1 || { tail -5 $R/gpurun_out/$tag.log; exit 1; }
  echo "== $s $(grep err $R/gpurun_out/$tag.log)"; grep -E "wgrad_group" $R/gpurun_out/$tag/run_kernel_stats.csv | cut -d, -f1,4 | sed 's/(anonymous namespace):://g'
done
cd $R
bash tools/ab.sh 2 - TTMI_WGRAD_WIDE=0 -- --dim 256 || exit 1
bash tools/prof_step.sh wide_d256 --dim 256 && head -20 gpurun_out/prof_wide_d256_step.txt
