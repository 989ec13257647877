set -o pipefail
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_fb -o run -- python3 $GRAFT_REPO_ROOT/tools/fold_bench.py) > gpurun_out/prof_fb.log 2>&1 || { tail -30 gpurun_out/prof_fb.log; exit 1; }
f=$(ls gpurun_out/prof_fb/*/run_kernel_stats.csv 2>/dev/null || ls gpurun_out/prof_fb/run_kernel_stats.csv)
cut -d, -f1-8 $f | head -20
