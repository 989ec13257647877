set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/last_t.log 2>&1 || { tail -40 gpurun_out/last_t.log; exit 1; }
tail -1 gpurun_out/last_t.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/last_smoke.log 2>&1 || { tail -20 gpurun_out/last_smoke.log; exit 1; }
tail -1 gpurun_out/last_smoke.log
timeout -k 10 400 python bench.py > gpurun_out/last_b2.log 2>&1 || { tail -20 gpurun_out/last_b2.log; exit 1; }
grep '"metric"' gpurun_out/last_b2.log | cut -c1-200
echo DONE
