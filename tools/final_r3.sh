#!/bin/bash
# Round-3 closing GPU session: GPU tests + smoke + default bench (tools/gpu_tests.sh), the cfg-2
# kernel-trace step profile (tools/prof_step.sh) and the cfg-2 PMC traffic (tools/pmc_traffic.sh).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_tests.sh || exit 1
bash tools/prof_step.sh r03s3 || exit 1
tail -40 gpurun_out/prof_r03s3_step.txt
bash tools/pmc_traffic.sh r03s3 2 || exit 1
python3 -c "import json;d=json.load(open('gpurun_out/traffic_r03s3.json'));[print(k,v) for k,v in d.items() if 'wgrad' in k or 'panel' in k]"
