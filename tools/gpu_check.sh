#!/bin/bash
# One GPU session: tests, smoke, short bench, kernel-trace profile.  Each GPU step has its
# own time limit; the chain stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS=${STEPS:-all}
run() { echo "== $*"; }
if [[ "$STEPS" == *tests* || "$STEPS" == all ]]; then
  run tests
  timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1 || { tail -50 gpurun_out/pytest_gpu.log; exit 1; }
  tail -3 gpurun_out/pytest_gpu.log
fi
if [[ "$STEPS" == *smoke* || "$STEPS" == all ]]; then
  run smoke
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -30 gpurun_out/smoke.log; exit 1; }
  tail -2 gpurun_out/smoke.log
fi
if [[ "$STEPS" == *bench* || "$STEPS" == all ]]; then
  run bench
  timeout -k 10 600 python bench.py --steps 50 --warmup 10 > gpurun_out/bench.log 2>&1 || { tail -30 gpurun_out/bench.log; exit 1; }
  tail -1 gpurun_out/bench.log
fi
if [[ "$STEPS" == *prof* || "$STEPS" == all ]]; then
  run prof
  (cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --skip-cpu) > gpurun_out/prof.log 2>&1 || { tail -30 gpurun_out/prof.log; exit 1; }
  find gpurun_out/prof -name "*stats*" | head
fi
if [[ "$STEPS" == *traffic* ]]; then
  run traffic
  for c in FETCH_SIZE WRITE_SIZE; do
    (cd /tmp && timeout -k 10 600 rocprofv3 --pmc $c --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmc_$c -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --skip-cpu) > gpurun_out/pmc_$c.log 2>&1 || { tail -30 gpurun_out/pmc_$c.log; exit 1; }
  done
  find gpurun_out/pmc_* -name "*counter_collection*"
fi
echo DONE
