set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_text.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t3.log 2>&1 || { tail -40 gpurun_out/t3.log; exit 1; }
tail -2 gpurun_out/t3.log
timeout -k 10 200 python tools/attn_bench.py > gpurun_out/attn.log 2>&1 || { cat gpurun_out/attn.log; exit 1; }
cat gpurun_out/attn.log
