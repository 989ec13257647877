set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python bench.py --config 4 --skip-cpu > gpurun_out/fin2_b4.log 2>&1 || { tail -20 gpurun_out/fin2_b4.log; exit 1; }
grep '"metric"' gpurun_out/fin2_b4.log | cut -c1-200
echo DONE
