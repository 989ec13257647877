# PMC HBM traffic of one bench config: FETCH_SIZE and WRITE_SIZE in separate passes
# (MI355X_MICROARCH.md §HBM), then tools/traffic.py.  Usage: bash tools/pmc_traffic.sh TAG CONFIG
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd /tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 150 rocprofv3 --pmc $c --output-format csv -d $R/gpurun_out/pmc_$1_$c -o run -- python3 $R/bench.py --config $2 --steps 5 --warmup 2 --skip-cpu > $R/gpurun_out/pmc_$1_$c.log 2>&1 || { tail -20 $R/gpurun_out/pmc_$1_$c.log; exit 1; }
done
F=$(ls $R/gpurun_out/pmc_$1_FETCH_SIZE/*/run_counter_collection.csv 2>/dev/null || ls $R/gpurun_out/pmc_$1_FETCH_SIZE/run_counter_collection.csv)
W=$(ls $R/gpurun_out/pmc_$1_WRITE_SIZE/*/run_counter_collection.csv 2>/dev/null || ls $R/gpurun_out/pmc_$1_WRITE_SIZE/run_counter_collection.csv)
python3 $R/tools/traffic.py $F $W $R/gpurun_out/traffic_$1.json > $R/gpurun_out/traffic_$1.txt
echo DONE
