set -o pipefail
mkdir -p gpurun_out
for c in "5" "3" "4"; do
  case $c in
    3) a="--config 3 --steps 20 --warmup 5" ;;
    4) a="--config 4 --steps 10 --warmup 3" ;;
    *) a="--config $c" ;;
  esac
  for v in single ddp; do
    x=""; [ $v = ddp ] && x="--ddp-schedule"
    timeout -k 10 400 python bench.py --skip-cpu $a $x > gpurun_out/ddpcfg_${c}_$v.json 2> gpurun_out/ddpcfg_${c}_$v.err || { tail -20 gpurun_out/ddpcfg_${c}_$v.err; exit 1; }
    python3 -c "import json;d=json.loads(open('gpurun_out/ddpcfg_${c}_$v.json').read().strip().splitlines()[-1]);print('$c $v', d['value'], d['ms_per_step'], d['config'].get('schedule'))"
  done
done
