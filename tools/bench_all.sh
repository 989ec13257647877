#!/bin/bash
# Refresh every bench line: cfg 2 (metric), cfg 2 at D = 256, cfg 3, cfg 4, cfg 5, eval, prep.
# Usage: tools/bench_all.sh TAG [configs...]; lines go to gpurun_out/bench_TAG_<cfg>.jsonl
set -o pipefail
mkdir -p gpurun_out
tag=$1; shift
cfgs="$*"
[ -z "$cfgs" ] && cfgs="2 2d256 3 4 5 eval prep"
for c in $cfgs; do
  case $c in
    2d256) args="--config 2 --dim 256 --steps 50 --warmup 10" ;;
    3) args="--config 3 --steps 20 --warmup 5" ;;
    4) args="--config 4 --steps 10 --warmup 3" ;;
    *) args="--config $c" ;;
  esac
  timeout -k 10 600 python bench.py $args > gpurun_out/bench_${tag}_$c.jsonl 2> gpurun_out/bench_${tag}_$c.err \
    || { tail -20 gpurun_out/bench_${tag}_$c.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/bench_${tag}_$c.jsonl').read().strip().splitlines()[-1]);r=d.get('roofline') or {};print('$c', d['value'], d.get('ms_per_step'), r.get('frac'), (d.get('cpu_baseline') or {}).get('value'))"
done
