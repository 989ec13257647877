set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-s3i}
timeout -k 10 300 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_kernels.py -x -q -m gpu --timeout 120 --timeout-method thread -k "adamw or train" > gpurun_out/${T}_tk.log 2>&1 || { tail -60 gpurun_out/${T}_tk.log; exit 1; }
tail -1 gpurun_out/${T}_tk.log
timeout -k 10 300 python bench.py --steps 50 --warmup 10 --skip-cpu > gpurun_out/${T}_b.log 2>&1 || { tail -30 gpurun_out/${T}_b.log; exit 1; }
grep '"metric"' gpurun_out/${T}_b.log | cut -c1-250
bash tools/_cmd_prof2.sh ${T}
grep -E "adamw|step:" gpurun_out/prof_${T}_step.txt | head -3
echo DONE
