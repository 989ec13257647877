# Session-3 state: full GPU suite, smoke, default bench (cfg 2 incl. CPU baseline), cfg 5 and
# cfg 3 bench lines, cfg-2 kernel profile + step timeline.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/fin2_t.log 2>&1 || { tail -40 gpurun_out/fin2_t.log; exit 1; }
tail -1 gpurun_out/fin2_t.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/fin2_smoke.log 2>&1 || { tail -20 gpurun_out/fin2_smoke.log; exit 1; }
tail -1 gpurun_out/fin2_smoke.log
timeout -k 10 400 python bench.py > gpurun_out/fin2_b2.log 2>&1 || { tail -20 gpurun_out/fin2_b2.log; exit 1; }
grep '"metric"' gpurun_out/fin2_b2.log | cut -c1-200
timeout -k 10 300 python bench.py --config 5 --skip-cpu > gpurun_out/fin2_b5.log 2>&1 || { tail -20 gpurun_out/fin2_b5.log; exit 1; }
grep '"metric"' gpurun_out/fin2_b5.log | cut -c1-200
timeout -k 10 300 python bench.py --config 3 --skip-cpu > gpurun_out/fin2_b3.log 2>&1 || { tail -20 gpurun_out/fin2_b3.log; exit 1; }
grep '"metric"' gpurun_out/fin2_b3.log | cut -c1-200
bash tools/_cmd_prof2.sh fin2
head -3 gpurun_out/prof_fin2_step.txt
echo DONE
