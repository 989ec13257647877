set -o pipefail
mkdir -p gpurun_out
cd /tmp
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmc_ev_f -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config eval --steps 5 --warmup 2 --skip-cpu > $GRAFT_REPO_ROOT/gpurun_out/pmc_ev_f.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/pmc_ev_f.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmc_ev_w -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config eval --steps 5 --warmup 2 --skip-cpu > $GRAFT_REPO_ROOT/gpurun_out/pmc_ev_w.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/pmc_ev_w.log; exit 1; }
echo DONE
