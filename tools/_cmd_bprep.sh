set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --config prep --steps 20 --warmup 3 > gpurun_out/bprep.log 2>&1 || { tail -30 gpurun_out/bprep.log; exit 1; }
tail -1 gpurun_out/bprep.log
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/profp -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config prep --steps 5 --warmup 2 --skip-cpu) > gpurun_out/profp.log 2>&1 || { tail -30 gpurun_out/profp.log; exit 1; }
