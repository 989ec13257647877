set -o pipefail
timeout -k 10 200 python bench.py --skip-cpu --steps 100 > gpurun_out/e1.log 2>&1 && bash tools/_cmd_prof2.sh e1 && TTMI_EXP_NO_LNSUM=1 timeout -k 10 200 python bench.py --skip-cpu --steps 100 > gpurun_out/e2.log 2>&1 && TTMI_EXP_NO_LNSUM=1 bash tools/_cmd_prof2.sh e2
