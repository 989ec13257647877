# wgrad split sweep on the whole cfg-2 bench: TTMI_WGRAD_WG (workgroup target) x
# TTMI_WGRAD_MIN_STAGES; prints pairs/s and the graph-replayed wgrad mix avg_us.
set -o pipefail
mkdir -p gpurun_out
for wg in 256 320 512 640; do
  for ms in 6 12; do
    TTMI_WGRAD_WG=$wg TTMI_WGRAD_MIN_STAGES=$ms timeout -k 10 120 python bench.py --skip-cpu --steps 100 > gpurun_out/sw.log 2>&1 || { tail -5 gpurun_out/sw.log; exit 1; }
    python3 -c "import json,sys; d=json.loads([l for l in open('gpurun_out/sw.log') if l.startswith('{')][0]); print('$wg', '$ms', d['value'], d['roofline']['avg_us'])"
  done
done
