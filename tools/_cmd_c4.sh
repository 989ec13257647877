set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/c19_t.log 2>&1 || { tail -40 gpurun_out/c19_t.log; exit 1; }
tail -2 gpurun_out/c19_t.log
timeout -k 10 300 python bench.py --steps 50 --warmup 10 --skip-cpu > gpurun_out/c19_b2.log 2>&1 || { tail -30 gpurun_out/c19_b2.log; exit 1; }
grep '"metric"' gpurun_out/c19_b2.log | cut -c1-200
timeout -k 10 400 python bench.py --config 4 --steps 5 --warmup 2 --skip-cpu > gpurun_out/c19_b4.log 2>&1 || { tail -30 gpurun_out/c19_b4.log; exit 1; }
grep '"metric"' gpurun_out/c19_b4.log | cut -c1-200
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/profc19 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config 4 --steps 3 --warmup 1 --skip-cpu) > gpurun_out/profc19.log 2>&1 || { tail -30 gpurun_out/profc19.log; exit 1; }
echo DONE
