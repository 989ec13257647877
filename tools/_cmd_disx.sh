# Time the dis-attention forward of each experiment build (build_exp/libttmi_*.so).
set -o pipefail
for f in $GRAFT_REPO_ROOT/build_exp/libttmi_*.so; do
  echo "== $f"
  TTMI_LIB=$f ATTN_FWD_ONLY=1 timeout -k 10 100 python3 -u tools/attn_bench.py 2>&1 | grep dis_attn || exit 1
done
