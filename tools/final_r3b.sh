#!/bin/bash
# Closing GPU session after the row-kernel and big-GEMM epilogue changes: GPU tests + smoke +
# default bench, the D = 256 bench line and its step profile.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_tests.sh || exit 1
bash tools/bench_all.sh r03s3 2d256 || exit 1
bash tools/prof_step.sh d256b --dim 256 || exit 1
head -24 gpurun_out/prof_d256b_step.txt
