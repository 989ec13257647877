set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r18_t.log 2>&1 || { tail -40 gpurun_out/r18_t.log; exit 1; }
tail -2 gpurun_out/r18_t.log
timeout -k 10 300 python bench.py --steps 50 --warmup 10 --skip-cpu > gpurun_out/r18_b.log 2>&1 || { tail -30 gpurun_out/r18_b.log; exit 1; }
grep '"metric"' gpurun_out/r18_b.log | cut -c1-250
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/profr18 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --skip-cpu) > gpurun_out/profr18.log 2>&1 || { tail -30 gpurun_out/profr18.log; exit 1; }
echo DONE
