set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "gemm" --timeout 120 --timeout-method thread > gpurun_out/t_big.log 2>&1 || { tail -40 gpurun_out/t_big.log; exit 1; }
tail -2 gpurun_out/t_big.log
timeout -k 10 200 python tools/attn_bench.py > gpurun_out/attn.log 2>&1 || { cat gpurun_out/attn.log; exit 1; }
cat gpurun_out/attn.log
timeout -k 10 300 python tools/bigemm_bench.py > gpurun_out/bigemm.log 2>&1 || { cat gpurun_out/bigemm.log; exit 1; }
cat gpurun_out/bigemm.log
timeout -k 10 300 python bench.py --config 4 --steps 5 --warmup 2 --skip-cpu > gpurun_out/b4.log 2>&1 || { tail -20 gpurun_out/b4.log; exit 1; }
tail -1 gpurun_out/b4.log | cut -c1-400
