set -o pipefail
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_wb -o run -- python3 $GRAFT_REPO_ROOT/tools/wgrad_vs_blas.py) > gpurun_out/prof_wb.log 2>&1 || { tail -30 gpurun_out/prof_wb.log; exit 1; }
f=$(ls gpurun_out/prof_wb/*/run_kernel_trace.csv 2>/dev/null || ls gpurun_out/prof_wb/run_kernel_trace.csv)
python3 - "$f" <<'PY'
import csv, sys, collections
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
seq = [(r["Kernel_Name"][:60], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3) for r in rows]
for n, t in seq[-12:]:
    print(f"{t:8.2f}  {n}")
agg = collections.defaultdict(list)
for n, t in seq:
    agg[n].append(t)
for n, v in agg.items():
    print(f"{len(v):5d} {sorted(v)[len(v)//2]:8.2f} median  {n}")
PY
