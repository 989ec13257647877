set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_text.py tests/test_gpu_kernels.py -x -q -k "text or dis_attn or skinny or lora" --timeout 200 --timeout-method thread > gpurun_out/t4.log 2>&1 || { tail -40 gpurun_out/t4.log; exit 1; }
tail -2 gpurun_out/t4.log
(cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof4 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config 4 --steps 3 --warmup 1 --skip-cpu) > gpurun_out/prof4.log 2>&1 || { tail -30 gpurun_out/prof4.log; exit 1; }
grep '"metric"' gpurun_out/prof4.log | cut -c1-250
