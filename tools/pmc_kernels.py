#!/usr/bin/env python3
"""Per-kernel mean of every counter in one or more rocprofv3 counter_collection.csv files.
Usage: pmc_kernels.py FILTER csv [csv ...]  (FILTER: substring of the kernel name)"""
import collections
import csv
import sys

flt, paths = sys.argv[1], sys.argv[2:]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for p in paths:
    for r in csv.DictReader(open(p)):
        name = r["Kernel_Name"]
        if flt not in name:
            continue
        key = name.replace("(anonymous namespace)::", "")[:60]
        acc[key][(r["Dispatch_Id"], r["Counter_Name"])].append(float(r["Counter_Value"]))
for k, d in acc.items():
    per = collections.defaultdict(list)
    for (disp, cn), vals in d.items():
        per[cn].append(sum(vals))
    print(k)
    for cn in sorted(per):
        v = per[cn]
        print(f"   {cn:28s} {sum(v) / len(v):16.0f}  (n={len(v)})")
