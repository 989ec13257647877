# Tuning sweep for the weight-gradient GEMM (GPU): tile/ring configs x split counts.
for c in ${CFGS:-64x64x4 64x64x8 128x128x4}; do
  echo "== $c"; TTMI_WGRAD=$c timeout -k 10 120 python tools/gemm_profile.py --sweep --wgrad 2>&1 | grep -v amdgpu.ids || exit 1
done
