#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel-stats CSV: per-kernel total/avg/calls and per-step share."""
import csv
import sys

path = sys.argv[1]
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 1
rows = list(csv.DictReader(open(path)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total kernel time {tot/1e3:.1f} us over {steps} steps = {tot/1e3/steps:.1f} us/step")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:int(sys.argv[3]) if len(sys.argv) > 3 else 30]:
    name = r["Name"].replace("(anonymous namespace)::", "")
    print(f"{float(r['TotalDurationNs'])/1e3/steps:9.1f} us/step {int(r['Calls'])/steps:5.1f}x "
          f"{float(r['AverageNs'])/1e3:8.2f} us {100*float(r['TotalDurationNs'])/tot:5.1f}%  {name[:100]}")
