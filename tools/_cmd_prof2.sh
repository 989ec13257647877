set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof2 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --skip-cpu) > gpurun_out/prof2.log 2>&1 || { tail -30 gpurun_out/prof2.log; exit 1; }
grep '"metric"' gpurun_out/prof2.log | cut -c1-200
