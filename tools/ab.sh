#!/bin/bash
# Generic A/B of environment settings on the cfg-2 bench (the documented replacement of the
# round-3 one-off ab_*.sh / diag_r3.sh scripts).  Each setting is "NAME=VALUE[,NAME=VALUE...]"
# ("-" = no override); the settings alternate for PAIRS rounds, each a 200-step default bench.
#   usage: tools/ab.sh PAIRS SETTING_A SETTING_B [...]  [-- extra bench.py args]
#   e.g.   tools/ab.sh 3 TTMI_WGRAD_CHUNK=1 TTMI_WGRAD_CHUNK=0
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
pairs=$1; shift
sets=(); extra=()
while [ $# -gt 0 ]; do
  if [ "$1" = "--" ]; then shift; extra=("$@"); break; fi
  sets+=("$1"); shift
done
for i in $(seq 1 "$pairs"); do
  for s in "${sets[@]}"; do
    envs=()
    [ "$s" != "-" ] && IFS=',' read -r -a envs <<< "$s"
    tag=$(echo "$s" | tr -c 'A-Za-z0-9_' '_')
    env "${envs[@]}" timeout -k 10 300 python bench.py --skip-cpu --steps 200 --warmup 20 "${extra[@]}" \
      > gpurun_out/ab_$tag.json 2> gpurun_out/ab_$tag.err || { tail -20 gpurun_out/ab_$tag.err; exit 1; }
    python3 -c "import json;d=json.loads(open('gpurun_out/ab_$tag.json').read().strip().splitlines()[-1]);r=d.get('roofline') or {};print('$s', d['value'], d['ms_per_step'], r.get('avg_us'), r.get('frac'))"
  done
done
