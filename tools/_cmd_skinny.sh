set -o pipefail
mkdir -p gpurun_out
for cfg in 4,4,256 8,4,256 10,4,256 10,8,256 8,4,384 4,4,384 8,8,128 10,4,128 8,8,192; do
  TTMI_SKINNY=$cfg timeout -k 10 120 python tools/skinny_sweep.py || exit 1
done
