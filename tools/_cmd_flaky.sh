set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/fl_t.log 2>&1; tail -5 gpurun_out/fl_t.log
for i in 1 2; do timeout -k 10 200 python -u -m pytest tests/test_gpu_cnn.py -q -k graph_equals --timeout 120 --timeout-method thread > gpurun_out/fl_$i.log 2>&1; grep -E "passed|failed|AssertionError: \(" gpurun_out/fl_$i.log | head -3; done
echo DONE
