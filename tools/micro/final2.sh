set -o pipefail
tag=r05f
for c in "--config 3" "--config 4"; do
  t=$(echo "$c" | tr -c 'A-Za-z0-9' '_')
  timeout -k 10 400 python3 bench.py $c > gpurun_out/${tag}_bench$t.json 2> gpurun_out/${tag}_bench$t.err || { tail -20 gpurun_out/${tag}_bench$t.err; exit 1; }
  tail -1 gpurun_out/${tag}_bench$t.json | cut -c1-300
done
tools/gpu.sh profile ${tag}_cfg2 > /dev/null || exit 1
tools/gpu.sh profile ${tag}_d256 --dim 256 > /dev/null || exit 1
tools/gpu.sh profile ${tag}_cfg3 --config 3 > /dev/null || exit 1
tools/gpu.sh profile ${tag}_cfg4 --config 4 > /dev/null || exit 1
head -1 gpurun_out/prof_${tag}_cfg2_step.txt gpurun_out/prof_${tag}_d256_step.txt gpurun_out/prof_${tag}_cfg3_step.txt gpurun_out/prof_${tag}_cfg4_step.txt
