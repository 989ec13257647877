#!/bin/bash
# Row-kernel grids A/B: LayerNorm / seq-embed parity tests, then the cfg-2 step with the
# seq-embed grid capped at 2,048 blocks (round 2) vs one row per wave, and the D = 256 step.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -q -m gpu -x -k "layernorm or ln_ or seq_embed or bitexact or d256 or full_size" \
  --timeout 200 --timeout-method thread > gpurun_out/rows_tests.log 2>&1 || { tail -30 gpurun_out/rows_tests.log; exit 1; }
tail -2 gpurun_out/rows_tests.log
for i in 1 2 3; do
  for c in 2048 0; do
    if [ $c = 0 ]; then unset TTMI_SEQ_GRID; else export TTMI_SEQ_GRID=$c; fi
    timeout -k 10 300 python bench.py --skip-cpu --steps 200 --warmup 20 > gpurun_out/rows_$c.json 2> gpurun_out/rows_$c.err \
      || { tail -20 gpurun_out/rows_$c.err; exit 1; }
    python -c "import json;d=json.loads(open('gpurun_out/rows_$c.json').read().strip().splitlines()[-1]);print('seqgrid=$c', d['value'], d['ms_per_step'])"
  done
done
unset TTMI_SEQ_GRID
timeout -k 10 300 python bench.py --skip-cpu --dim 256 --steps 50 --warmup 10 > gpurun_out/rows_d256.json 2> gpurun_out/rows_d256.err \
  || { tail -20 gpurun_out/rows_d256.err; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/rows_d256.json').read().strip().splitlines()[-1]);print('d256', d['value'], d['ms_per_step'])"
