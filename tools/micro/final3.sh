set -o pipefail
tag=r05g
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 || { tail -30 gpurun_out/${tag}_tests.log; exit 1; }
tail -2 gpurun_out/${tag}_tests.log
timeout -k 10 300 python3 bench.py > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err || { tail -20 gpurun_out/${tag}_bench.err; exit 1; }
tail -1 gpurun_out/${tag}_bench.json | cut -c1-400
timeout -k 10 400 python3 bench.py --dim 256 > gpurun_out/${tag}_bench_d256.json 2> gpurun_out/${tag}_bench_d256.err || { tail -20 gpurun_out/${tag}_bench_d256.err; exit 1; }
tail -1 gpurun_out/${tag}_bench_d256.json | cut -c1-300
tools/gpu.sh profile ${tag}_cfg2 > /dev/null || exit 1
head -1 gpurun_out/prof_${tag}_cfg2_step.txt
tools/gpu.sh pmc ${tag} 2 > gpurun_out/${tag}_pmc.out 2>&1 || { tail -20 gpurun_out/${tag}_pmc.out; exit 1; }
grep -A4 '"wgrad_group_kernel"' gpurun_out/traffic_${tag}.json
