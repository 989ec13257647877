# Grouped weight-gradient A/B at the cfg-2 encoder shapes (tools/wgrad_shapes.py, D = 128 and 256):
# kernel durations per setting, then FETCH_SIZE and TCC hit/miss passes at D = 256.
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 200 python -u -m pytest tests/test_gpu_colaunch.py -q --timeout 120 --timeout-method thread -k "infonce" > gpurun_out/wg_tests.log 2>&1; tail -3 gpurun_out/wg_tests.log
cd /tmp && export TMPDIR=/tmp
for d in 128 256; do
 for s in "-" "TTMI_WGRAD_SWZ=0" "TTMI_WGRAD_GROUP=128:16"; do
  envs=(); [ "$s" != "-" ] && envs=("$s")
  tag=d${d}_$(echo "$s" | tr -c 'A-Za-z0-9_' '_')
  env "${envs[@]}" timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/wg_$tag -o run -- python3 $R/tools/wgrad_shapes.py --dim $d --blas $([ "$s" = "-" ] && echo 1 || echo 0) > $R/gpurun_out/wg_$tag.log 2>&1 || { tail -5 $R/gpurun_out/wg_$tag.log; exit 1; }
  echo "== $tag"; grep -E "wgrad|Cijk|gemm" $R/gpurun_out/wg_$tag/run_kernel_stats.csv | cut -d, -f1-5 | cut -c1-150
 done
done
for d in 128 256; do
  timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/wg_pmcF$d -o run -- python3 $R/tools/wgrad_shapes.py --dim $d --blas 0 --reps 3 > $R/gpurun_out/wg_pmcF$d.log 2>&1 || exit 1
  timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $R/gpurun_out/wg_pmcH$d -o run -- python3 $R/tools/wgrad_shapes.py --dim $d --blas 0 --reps 3 > $R/gpurun_out/wg_pmcH$d.log 2>&1 || exit 1
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_BUSY_CYCLES --output-format csv -d $R/gpurun_out/wg_pmcS$d -o run -- python3 $R/tools/wgrad_shapes.py --dim $d --blas 0 --reps 3 > $R/gpurun_out/wg_pmcS$d.log 2>&1 || exit 1
done
echo DONE
