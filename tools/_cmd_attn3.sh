set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/profa -o run -- python3 $GRAFT_REPO_ROOT/tools/attn_bench.py) > gpurun_out/profa.log 2>&1 || { tail -30 gpurun_out/profa.log; exit 1; }
(cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof4 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config 4 --steps 3 --warmup 1 --skip-cpu) > gpurun_out/prof4.log 2>&1 || { tail -30 gpurun_out/prof4.log; exit 1; }
grep '"metric"' gpurun_out/prof4.log | cut -c1-250
