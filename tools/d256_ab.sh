# FFN block A/B on one box: the fused-block tests, the D = 256 model tests, cfg 2 (D = 128) and
# cfg 2 --dim 256 bench lines with and without the blocks, per-launch device times
# (tools/ffn_time.py) and kernel traces.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-d256}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_ffn_block.py > $O/ffn_tests.txt 2>&1 && \
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_model.py -k "256" > $O/model_tests.txt 2>&1 && \
timeout -k 10 120 python tools/ffn_time.py > $O/ffn_time.txt 2>&1 && \
timeout -k 10 200 python bench.py --config 2 --dim 256 --steps 50 --warmup 10 > $O/bench_d256.txt 2>&1 && \
TTMI_NO_FFN=1 timeout -k 10 200 python bench.py --config 2 --dim 256 --steps 50 --warmup 10 > $O/bench_d256_noffn.txt 2>&1 && \
timeout -k 10 200 python bench.py --config 2 --dim 256 --steps 50 --warmup 10 > $O/bench_d256b.txt 2>&1 && \
timeout -k 10 200 python bench.py --steps 50 --warmup 10 > $O/bench_cfg2.txt 2>&1 && \
cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof256 -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --config 2 --dim 256 --steps 20 --warmup 5 > $GRAFT_REPO_ROOT/$O/prof256.log 2>&1
