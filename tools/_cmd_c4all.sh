# cfg-4: bench line, kernel-trace step profile, and the PMC traffic passes (gemm_big_kernel).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
bash $R/tools/_cmd_pmc2.sh $1_c4 4 || exit 1
cp $R/gpurun_out/traffic_$1_c4.json $R/gpurun_out/cfg4_traffic.json
bash $R/tools/_cmd_c4p.sh $1 || exit 1
grep '"metric"' $R/gpurun_out/b4_$1.log | cut -c1-400
head -12 $R/gpurun_out/prof4_$1_step.txt
