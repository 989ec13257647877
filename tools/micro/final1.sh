set -o pipefail
R=$(pwd); export TMPDIR=/tmp; mkdir -p gpurun_out
tag=r05f
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 || { tail -30 gpurun_out/${tag}_tests.log; exit 1; }
tail -2 gpurun_out/${tag}_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${tag}_smoke.log 2>&1 || { tail -20 gpurun_out/${tag}_smoke.log; exit 1; }
tail -1 gpurun_out/${tag}_smoke.log
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${tag}_bench_prof -o run -- python3 $R/bench.py) > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err || { tail -20 gpurun_out/${tag}_bench.err; exit 1; }
tail -1 gpurun_out/${tag}_bench.json
timeout -k 10 300 python3 bench.py > gpurun_out/${tag}_bench_plain.json 2> gpurun_out/${tag}_bench_plain.err || { tail -20 gpurun_out/${tag}_bench_plain.err; exit 1; }
tail -1 gpurun_out/${tag}_bench_plain.json
for c in "--dim 256" "--config 5"; do
  t=$(echo "$c" | tr -c 'A-Za-z0-9' '_')
  timeout -k 10 400 python3 bench.py $c > gpurun_out/${tag}_bench$t.json 2> gpurun_out/${tag}_bench$t.err || { tail -20 gpurun_out/${tag}_bench$t.err; exit 1; }
  tail -1 gpurun_out/${tag}_bench$t.json
done
