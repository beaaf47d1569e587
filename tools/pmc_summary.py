#!/usr/bin/env python3
"""Average rocprofv3 --pmc counter values per dispatch of one kernel (skipping the first
dispatch = warmup).  Usage: pmc_summary.py <counter_collection.csv> [kernel-substring]"""
import csv
import collections
import sys

path = sys.argv[1]
kern = sys.argv[2] if len(sys.argv) > 2 else "k_rollout"
per = collections.defaultdict(dict)
for r in csv.DictReader(open(path)):
    if kern not in r["Kernel_Name"]:
        continue
    per[int(r["Dispatch_Id"])][r["Counter_Name"]] = per[int(r["Dispatch_Id"])].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
ids = sorted(per)[1:] or sorted(per)
names = sorted({k for d in ids for k in per[d]})
for n in names:
    vals = [per[d].get(n, 0.0) for d in ids]
    print(f"{n:28s} {sum(vals) / len(vals):16.1f}   ({len(vals)} dispatches)")
