set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --config 4 --steps 10 --warmup 3 --skip-cpu > gpurun_out/b4_$1.log 2>&1 || { tail -20 gpurun_out/b4_$1.log; exit 1; }
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof4_$1 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config 4 --steps 5 --warmup 2 --skip-cpu) > gpurun_out/prof4_$1.log 2>&1 || { tail -30 gpurun_out/prof4_$1.log; exit 1; }
f=$(ls gpurun_out/prof4_$1/*/run_kernel_trace.csv 2>/dev/null || ls gpurun_out/prof4_$1/run_kernel_trace.csv)
python3 tools/step_profile.py $f adamw_kernel 40 > gpurun_out/prof4_$1_step.txt
echo DONE
