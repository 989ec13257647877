#!/bin/bash
# The one GPU-box runner (run it through gpurun from the repo root).  Every GPU step has its own
# time limit; a failing step ends the command (no retries).  Output goes to gpurun_out/.
#
#   tools/gpu.sh tests [pytest args]     GPU suite (per-test timeout), smoke, default bench
#   tools/gpu.sh serial                  GPU suite with kernels serialised, -x -v: names the
#                                        faulting launch / test in one run
#   tools/gpu.sh profile TAG [bench args]  rocprofv3 --kernel-trace --stats of a 20-step bench,
#                                        -> gpurun_out/prof_TAG_step.txt (tools/step_profile.py)
#   tools/gpu.sh pmc TAG CONFIG          FETCH_SIZE / WRITE_SIZE passes of `bench.py --config
#                                        CONFIG` -> gpurun_out/traffic_TAG.json (tools/traffic.py)
#   tools/gpu.sh bench-all TAG [cfgs]    bench lines of 2, 2d256, 3, 4, 5, eval, prep
#   tools/gpu.sh ab PAIRS A B [...] [-- bench args]   alternate env settings ("N=V[,N=V]" or
#                                        "-"), 200-step cfg-2 benches
#   tools/gpu.sh ddp TAG [bench args]   RCCL world-1 tests, then cfg-2 bench lines: single-process,
#                                        forced DDP schedule with captured RCCL collectives, and
#                                        with host cuts (-> gpurun_out/ddp_TAG_*.json)
#   tools/gpu.sh dis-counters            disentangled-attention timing + SQ counters (cfg 4)
#   tools/gpu.sh final TAG               closing measurements: suite, default bench under
#                                        rocprofv3, the other configs, cfg-2/3/4 step profiles,
#                                        cfg-2 PMC traffic, disentangled-attention counters
# The diagnostic phase-stamp build is CPU-side: tools/stamp_build.sh.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
note() { echo "[$(date +%T)] $*" | tee -a gpurun_out/progress.txt; }

tests() {
  timeout -k 10 900 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread "$@" \
    > gpurun_out/pytest_gpu.log 2>&1
  local rc=$?
  tail -40 gpurun_out/pytest_gpu.log
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || return $rc     # 1 = test failures: still smoke and bench
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 \
    || { tail -30 gpurun_out/smoke.log; return 1; }
  tail -2 gpurun_out/smoke.log
  timeout -k 10 600 python bench.py > gpurun_out/bench.log 2>&1 || { tail -30 gpurun_out/bench.log; return 1; }
  tail -1 gpurun_out/bench.log
  return $rc
}

serial() {
  AMD_SERIALIZE_KERNEL=3 timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 200 \
    --timeout-method thread "$@" > gpurun_out/serial.log 2>&1
  local rc=$?
  grep -E "FAILED|PASSED|ERROR" gpurun_out/serial.log | tail -5
  return $rc
}

profile() {
  local tag=$1; shift
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$tag \
    -o run -- python3 $R/bench.py --steps 20 --warmup 5 --skip-cpu "$@") > gpurun_out/prof_$tag.log 2>&1 \
    || { tail -30 gpurun_out/prof_$tag.log; return 1; }
  local f
  f=$(ls gpurun_out/prof_$tag/*/run_kernel_trace.csv 2>/dev/null || ls gpurun_out/prof_$tag/run_kernel_trace.csv)
  python3 tools/step_profile.py $f adamw 40 seq > gpurun_out/prof_${tag}_step.txt
  head -30 gpurun_out/prof_${tag}_step.txt
}

pmc() {
  local tag=$1 cfg=$2 c
  for c in FETCH_SIZE WRITE_SIZE; do
    (cd /tmp && timeout -s KILL 60 rocprofv3 --pmc $c --output-format csv -d $R/gpurun_out/pmc_${tag}_$c -o run \
      -- python3 $R/bench.py --config $cfg --steps 5 --warmup 2 --skip-cpu) > gpurun_out/pmc_${tag}_$c.log 2>&1 \
      || { tail -20 gpurun_out/pmc_${tag}_$c.log; return 1; }
  done
  local F W
  F=$(ls gpurun_out/pmc_${tag}_FETCH_SIZE/*/run_counter_collection.csv 2>/dev/null || ls gpurun_out/pmc_${tag}_FETCH_SIZE/run_counter_collection.csv)
  W=$(ls gpurun_out/pmc_${tag}_WRITE_SIZE/*/run_counter_collection.csv 2>/dev/null || ls gpurun_out/pmc_${tag}_WRITE_SIZE/run_counter_collection.csv)
  python3 tools/traffic.py $F $W gpurun_out/traffic_$tag.json > gpurun_out/traffic_$tag.txt && head -20 gpurun_out/traffic_$tag.txt
}

bench_all() {
  local tag=$1; shift
  local cfgs="$*" c args
  [ -z "$cfgs" ] && cfgs="2 2d256 3 4 5 eval prep"
  for c in $cfgs; do
    case $c in
      2d256) args="--config 2 --dim 256 --steps 50 --warmup 10" ;;
      3) args="--config 3 --steps 20 --warmup 5" ;;
      4) args="--config 4 --steps 10 --warmup 3" ;;
      *) args="--config $c" ;;
    esac
    timeout -k 10 600 python bench.py $args > gpurun_out/bench_${tag}_$c.jsonl 2> gpurun_out/bench_${tag}_$c.err \
      || { tail -20 gpurun_out/bench_${tag}_$c.err; return 1; }
    python -c "import json;d=json.loads(open('gpurun_out/bench_${tag}_$c.jsonl').read().strip().splitlines()[-1]);r=d.get('roofline') or {};print('$c', d['value'], d.get('ms_per_step'), r.get('frac'), (d.get('cpu_baseline') or {}).get('value'))"
  done
}

ab() {
  local pairs=$1; shift
  local sets=() extra=() i s tag envs
  while [ $# -gt 0 ]; do
    if [ "$1" = "--" ]; then shift; extra=("$@"); break; fi
    sets+=("$1"); shift
  done
  for i in $(seq 1 "$pairs"); do
    for s in "${sets[@]}"; do
      envs=()
      [ "$s" != "-" ] && IFS=',' read -r -a envs <<< "$s"
      tag=$(echo "$s" | tr -c 'A-Za-z0-9_' '_')
      env "${envs[@]}" timeout -k 10 300 python bench.py --skip-cpu --steps 200 --warmup 20 "${extra[@]}" \
        > gpurun_out/ab_$tag.json 2> gpurun_out/ab_$tag.err || { tail -20 gpurun_out/ab_$tag.err; return 1; }
      python3 -c "import json;d=json.loads(open('gpurun_out/ab_$tag.json').read().strip().splitlines()[-1]);r=d.get('roofline') or {};print('$s', d['value'], d['ms_per_step'], r.get('avg_us'), r.get('frac'))"
    done
  done
}

ddp() {
  local tag=$1; shift
  timeout -k 10 400 python -u -m pytest tests/test_gpu_rccl.py -v --timeout 300 --timeout-method thread \
    > gpurun_out/ddp_${tag}_tests.log 2>&1
  local rc=$?
  tail -8 gpurun_out/ddp_${tag}_tests.log
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || return $rc
  local v args
  for v in single captured overlap segmented; do
    case $v in
      single) args="" ;;
      captured) args="--ddp-schedule" ;;
      overlap) args="--ddp-schedule --overlap-grad-sync" ;;
      segmented) args="--ddp-schedule --overlap-grad-sync --no-capture-collectives" ;;
    esac
    timeout -k 10 300 python bench.py --skip-cpu --steps 200 --warmup 20 $args "$@" > gpurun_out/ddp_${tag}_$v.json \
      2> gpurun_out/ddp_${tag}_$v.err || { tail -20 gpurun_out/ddp_${tag}_$v.err; return 1; }
    python3 -c "import json;d=json.loads(open('gpurun_out/ddp_${tag}_$v.json').read().strip().splitlines()[-1]);print('$v', d['value'], d['ms_per_step'], d['config'].get('schedule'))"
  done
  return $rc
}

dis_counters() {
  timeout -k 10 120 python3 -u tools/attn_bench.py > gpurun_out/dis_time.log 2>&1 || { tail -20 gpurun_out/dis_time.log; return 1; }
  cat gpurun_out/dis_time.log
  local P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES"
  local P2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_INSTS_VMEM SQ_WAVES GRBM_GUI_ACTIVE"
  local i=0 P
  for P in "$P1" "$P2"; do
    i=$((i+1))
    (cd /tmp && timeout -s KILL 60 rocprofv3 --pmc $P --output-format csv -d $R/gpurun_out/dis_pmc$i -o run \
      -- python3 $R/tools/attn_bench.py) > gpurun_out/dis_pmc$i.log 2>&1 || { tail -20 gpurun_out/dis_pmc$i.log; return 1; }
  done
  python3 tools/pmc_kernels.py dis_ $(ls gpurun_out/dis_pmc*/*/run_counter_collection.csv gpurun_out/dis_pmc*/run_counter_collection.csv 2>/dev/null)
}

# kcounters SCRIPT FILTER: two SQ counter passes over SCRIPT's launches, per-kernel means of the
# kernels whose name contains FILTER
kcounters() {
  local script=$1 flt=$2 i=0 P
  local P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES"
  local P2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_INSTS_VMEM SQ_WAVES GRBM_GUI_ACTIVE"
  timeout -k 10 120 python3 -u $script > gpurun_out/kc_time.log 2>&1 || { tail -20 gpurun_out/kc_time.log; return 1; }
  cat gpurun_out/kc_time.log
  for P in "$P1" "$P2"; do
    i=$((i+1))
    (cd /tmp && timeout -s KILL 60 rocprofv3 --pmc $P --output-format csv -d $R/gpurun_out/kc_pmc$i -o run \
      -- python3 $R/$script) > gpurun_out/kc_pmc$i.log 2>&1 || { tail -20 gpurun_out/kc_pmc$i.log; return 1; }
  done
  python3 tools/pmc_kernels.py $flt $(ls gpurun_out/kc_pmc*/*/run_counter_collection.csv gpurun_out/kc_pmc*/run_counter_collection.csv 2>/dev/null)
}

final() {
  local tag=$1 c t
  note tests
  timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread \
    > gpurun_out/${tag}_tests.log 2>&1 || { tail -30 gpurun_out/${tag}_tests.log; return 1; }
  tail -2 gpurun_out/${tag}_tests.log
  note "default bench under rocprofv3"
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${tag}_bench_prof \
    -o run -- python3 $R/bench.py) > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err \
    || { tail -20 gpurun_out/${tag}_bench.err; return 1; }
  tail -1 gpurun_out/${tag}_bench.json
  for c in "--dim 256" "--config 5" "--config 3" "--config 4"; do
    t=$(echo "$c" | tr -c 'A-Za-z0-9' '_')
    note "bench $c"
    timeout -k 10 400 python3 bench.py $c > gpurun_out/${tag}_bench$t.json 2> gpurun_out/${tag}_bench$t.err \
      || { tail -20 gpurun_out/${tag}_bench$t.err; return 1; }
    tail -1 gpurun_out/${tag}_bench$t.json
  done
  note profiles
  profile ${tag}_cfg2 && profile ${tag}_cfg3 --config 3 && profile ${tag}_cfg4 --config 4 || return 1
  note "pmc traffic"
  pmc $tag 2 || return 1
  note "disentangled-attention counters"
  dis_counters > gpurun_out/${tag}_dis.txt 2>&1 && tail -30 gpurun_out/${tag}_dis.txt || return 1
  note done
}

cmd=$1; shift
case $cmd in
  tests) tests "$@" ;;
  serial) serial "$@" ;;
  profile) profile "$@" ;;
  pmc) pmc "$@" ;;
  kcounters) kcounters "$@" ;;
  bench-all) bench_all "$@" ;;
  ab) ab "$@" ;;
  dis-counters) dis_counters "$@" ;;
  ddp) ddp "$@" ;;
  final) final "$@" ;;
  *) sed -n 2,22p "$0"; exit 2 ;;
esac
