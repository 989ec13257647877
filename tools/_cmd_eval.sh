set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_retrieval.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/ev_t.log 2>&1 || { tail -40 gpurun_out/ev_t.log; exit 1; }
tail -2 gpurun_out/ev_t.log
timeout -k 10 300 python bench.py --config eval --steps 50 --warmup 10 > gpurun_out/ev_b.log 2>&1 || { tail -30 gpurun_out/ev_b.log; exit 1; }
grep '"metric"' gpurun_out/ev_b.log
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/profev -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config eval --steps 20 --warmup 5 --skip-cpu) > gpurun_out/profev.log 2>&1 || { tail -30 gpurun_out/profev.log; exit 1; }
echo DONE
