# Round-end style validation: full GPU suite, smoke, default bench (cfg 2 incl. CPU baseline),
# cfg 5 bench, cfg-2 kernel profile.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/full_t.log 2>&1; echo "pytest rc=$?" >> gpurun_out/full_t.log; tail -2 gpurun_out/full_t.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/full_smoke.log 2>&1 || { tail -20 gpurun_out/full_smoke.log; exit 1; }
tail -1 gpurun_out/full_smoke.log
timeout -k 10 300 python bench.py > gpurun_out/full_b2.log 2>&1 || { tail -20 gpurun_out/full_b2.log; exit 1; }
timeout -k 10 300 python bench.py --config 5 --skip-cpu > gpurun_out/full_b5.log 2>&1 || { tail -20 gpurun_out/full_b5.log; exit 1; }
bash tools/_cmd_prof2.sh full
