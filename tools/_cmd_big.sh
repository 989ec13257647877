set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "gemm" --timeout 120 --timeout-method thread > gpurun_out/t_big.log 2>&1 || { tail -40 gpurun_out/t_big.log; exit 1; }
tail -3 gpurun_out/t_big.log
timeout -k 10 300 python tools/bigemm_bench.py > gpurun_out/bigemm.log 2>&1 || { cat gpurun_out/bigemm.log; exit 1; }
cat gpurun_out/bigemm.log
