# Kernel-trace stats of tools/attn_bench.py (cfg-4 attention shapes).
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd /tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/disprof -o run -- python3 $R/tools/attn_bench.py > $R/gpurun_out/disprof.log 2>&1 || { tail -20 $R/gpurun_out/disprof.log; exit 1; }
F=$(ls $R/gpurun_out/disprof/*/run_kernel_stats.csv 2>/dev/null || ls $R/gpurun_out/disprof/run_kernel_stats.csv)
python3 $R/tools/prof_summary.py $F 1 12
