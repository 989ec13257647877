set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-s3d}
timeout -k 10 300 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_kernels.py -x -q -m gpu --timeout 120 --timeout-method thread -k "head or train or step or seq_embed or wgrad or infonce or nce" > gpurun_out/${T}_tk.log 2>&1 || { tail -60 gpurun_out/${T}_tk.log; exit 1; }
tail -2 gpurun_out/${T}_tk.log
timeout -k 10 300 python bench.py --steps 50 --warmup 10 --skip-cpu > gpurun_out/${T}_b.log 2>&1 || { tail -30 gpurun_out/${T}_b.log; exit 1; }
grep '"metric"' gpurun_out/${T}_b.log | cut -c1-250
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_${T} -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --skip-cpu) > gpurun_out/prof_${T}.log 2>&1 || { tail -30 gpurun_out/prof_${T}.log; exit 1; }
f=$(ls gpurun_out/prof_${T}/*/run_kernel_trace.csv 2>/dev/null || ls gpurun_out/prof_${T}/run_kernel_trace.csv)
python3 tools/step_profile.py $f adamw_kernel 40 seq > gpurun_out/prof_${T}_step.txt
head -3 gpurun_out/prof_${T}_step.txt
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/${T}_t.log 2>&1 || { tail -40 gpurun_out/${T}_t.log; exit 1; }
tail -2 gpurun_out/${T}_t.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || { tail -30 gpurun_out/${T}_smoke.log; exit 1; }
tail -1 gpurun_out/${T}_smoke.log
echo DONE
