#!/bin/bash
# Round-4 GPU check: the changed kernels' tests, the model tests, the cfg-2 bench at D = 128 and
# D = 256 with their step profiles, and the panel phase stamps.  usage: tools/r4_check.sh TAG
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=$1
timeout -k 10 700 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_colaunch.py tests/test_gpu_model.py \
  tests/test_gpu_dist.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1
rc=$?
tail -5 gpurun_out/${tag}_tests.log
[ $rc -eq 0 ] || exit $rc
bash tools/ab.sh 1 TTMI_PANEL_WROT=0 TTMI_FOLD_IN_UPDATE=0 TTMI_SEQ_VEC=0 - || exit 1
bash tools/ab.sh 1 - -- --dim 256 || exit 1
bash tools/prof_step.sh ${tag} && cat gpurun_out/prof_${tag}_step.txt | head -30 || exit 1
bash tools/prof_step.sh ${tag}_d256 --dim 256 && cat gpurun_out/prof_${tag}_d256_step.txt | head -40 || exit 1
TTMI_LIB=music-recommendation-multimodal_amd/lib/diag/libttmi_stamp.so timeout -k 10 120 python tools/stamp_phases.py \
  > gpurun_out/${tag}_stamps.txt 2>&1
cat gpurun_out/${tag}_stamps.txt
