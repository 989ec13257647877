#!/usr/bin/env python3
"""Per-step kernel breakdown from a rocprofv3 kernel trace: the step is delimited by a marker
kernel (default: the AdamW launch that ends every train step); the last complete step
before the final marker is summarised."""
import collections
import csv
import sys

path = sys.argv[1]
marker = sys.argv[2] if len(sys.argv) > 2 else "adamw"
top = int(sys.argv[3]) if len(sys.argv) > 3 else 30
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
if len(idx) < 2:
    sys.exit(f"fewer than two '{marker}' dispatches")
a, b = idx[-2] + 1, idx[-1] + 1
step = rows[a:b]
wall = (int(step[-1]["End_Timestamp"]) - int(step[0]["Start_Timestamp"])) / 1e3
tot = collections.defaultdict(float)
cnt = collections.Counter()
for r in step:
    n = r["Kernel_Name"].replace("(anonymous namespace)::", "")
    n = n.split("(")[0] if not n.startswith("void ") else n[5:].split("(")[0]
    tot[n] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    cnt[n] += 1
busy = sum(tot.values())
print(f"step: {len(step)} dispatches, wall {wall:.1f} us, kernel busy {busy:.1f} us")
for n, t in sorted(tot.items(), key=lambda x: -x[1])[:top]:
    print(f"{t:10.1f} us {100 * t / busy:5.1f}% {cnt[n]:5d}x {t / cnt[n]:9.2f} us  {n[:90]}")
if len(sys.argv) > 4 and sys.argv[4] == "seq":          # the step's dispatches in order
    t0 = int(step[0]["Start_Timestamp"])
    for r in step:
        n = r["Kernel_Name"].replace("(anonymous namespace)::", "")
        n = n.split("(")[0] if not n.startswith("void ") else n[5:].split("(")[0]
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.2f}  {n[:80]}")
