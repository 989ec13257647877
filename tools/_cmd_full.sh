set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/fin5_t.log 2>&1 || { tail -40 gpurun_out/fin5_t.log; exit 1; }
tail -2 gpurun_out/fin5_t.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/fin5_smoke.log 2>&1 || { tail -30 gpurun_out/fin5_smoke.log; exit 1; }
tail -2 gpurun_out/fin5_smoke.log
timeout -k 10 400 python bench.py > gpurun_out/fin5_bench.log 2>&1 || { tail -30 gpurun_out/fin5_bench.log; exit 1; }
grep '"metric"' gpurun_out/fin5_bench.log | cut -c1-300
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/proffin5 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --skip-cpu) > gpurun_out/proffin5.log 2>&1 || { tail -30 gpurun_out/proffin5.log; exit 1; }
echo DONE
