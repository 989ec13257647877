set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_prep.py tests/test_gpu_cnn.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t5.log 2>&1 || { tail -60 gpurun_out/t5.log; exit 1; }
tail -3 gpurun_out/t5.log
