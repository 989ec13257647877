set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/s3a_t.log 2>&1 || { tail -40 gpurun_out/s3a_t.log; exit 1; }
tail -2 gpurun_out/s3a_t.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s3a_smoke.log 2>&1 || { tail -30 gpurun_out/s3a_smoke.log; exit 1; }
tail -2 gpurun_out/s3a_smoke.log
timeout -k 10 400 python bench.py > gpurun_out/s3a_bench.log 2>&1 || { tail -30 gpurun_out/s3a_bench.log; exit 1; }
grep '"metric"' gpurun_out/s3a_bench.log | cut -c1-300
echo DONE
