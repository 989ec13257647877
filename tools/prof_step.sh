set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_$1 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --skip-cpu ${@:2}) > gpurun_out/prof_$1.log 2>&1 || { tail -30 gpurun_out/prof_$1.log; exit 1; }
f=$(ls gpurun_out/prof_$1/*/run_kernel_trace.csv 2>/dev/null || ls gpurun_out/prof_$1/run_kernel_trace.csv)
python3 tools/step_profile.py $f adamw 40 seq > gpurun_out/prof_$1_step.txt
echo DONE
