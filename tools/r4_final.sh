#!/bin/bash
# Round-4 closing measurements: the full GPU suite, the default bench (with cpu_baseline) under
# rocprofv3 --stats, D = 256 / cfg 3 / cfg 4 / cfg 5 benches, cfg-3 and cfg-4 step profiles,
# the cfg-2 PMC traffic passes and the disentangled-attention counters.  usage: tools/r4_final.sh
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
step() { echo "[$(date +%T)] $*" | tee -a gpurun_out/r4f_progress.txt; }
step tests
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread \
  > gpurun_out/r4f_tests.log 2>&1
rc=$?; tail -4 gpurun_out/r4f_tests.log; [ $rc -eq 0 ] || exit $rc
step bench
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r4f_bench_prof -o run \
  -- python3 $R/bench.py) > gpurun_out/r4f_bench.json 2> gpurun_out/r4f_bench.err || { tail -20 gpurun_out/r4f_bench.err; exit 1; }
tail -1 gpurun_out/r4f_bench.json
for c in "--dim 256" "--config 5" "--config 3" "--config 4"; do
  tag=$(echo "$c" | tr -c 'A-Za-z0-9' '_')
  step "bench $c"
  timeout -k 10 400 python3 bench.py $c > gpurun_out/r4f_bench$tag.json 2> gpurun_out/r4f_bench$tag.err \
    || { tail -20 gpurun_out/r4f_bench$tag.err; exit 1; }
  tail -1 gpurun_out/r4f_bench$tag.json
done
step "profiles cfg 3 / 4"
bash tools/prof_step.sh r4f_cfg3 --config 3 && head -30 gpurun_out/prof_r4f_cfg3_step.txt || exit 1
bash tools/prof_step.sh r4f_cfg4 --config 4 && head -30 gpurun_out/prof_r4f_cfg4_step.txt || exit 1
step "pmc traffic"
bash tools/pmc_traffic.sh r4f 2 && cat gpurun_out/traffic_r4f.txt | head -20 || exit 1
step "disattn counters"
bash tools/dis_counters.sh > gpurun_out/r4f_dis.txt 2>&1 && tail -30 gpurun_out/r4f_dis.txt || exit 1
step done
