set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_model.py -x -q -m gpu --timeout 120 --timeout-method thread -k "train_step" > gpurun_out/ab_t.log 2>&1 || { tail -30 gpurun_out/ab_t.log; exit 1; }
TTMI_ITEM_SIDE=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_model.py -x -q -m gpu --timeout 120 --timeout-method thread -k "train_step" >> gpurun_out/ab_t.log 2>&1 || { tail -30 gpurun_out/ab_t.log; exit 1; }
grep passed gpurun_out/ab_t.log
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --steps 100 --warmup 10 --skip-cpu | python -c "import json,sys; print('base', json.loads(sys.stdin.read().strip().splitlines()[-1])['value'])" || exit 1
  TTMI_ITEM_SIDE=1 timeout -k 10 200 python bench.py --steps 100 --warmup 10 --skip-cpu | python -c "import json,sys; print('side', json.loads(sys.stdin.read().strip().splitlines()[-1])['value'])" || exit 1
done
