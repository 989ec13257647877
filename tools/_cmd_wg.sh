set -o pipefail
for wg in 320 192 256 448 640 320; do
  TTMI_WGRAD_WG=$wg timeout -k 10 200 python bench.py --steps 100 --warmup 10 --skip-cpu | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('wg $wg', d['value'], d['roofline']['avg_us'])" || exit 1
done
