#!/usr/bin/env python3
"""Per-XCD L2 -> HBM read traffic of the split rollout kernel.

Reads rocprofv3 counter CSVs of the derived counters in tools/xcd_counters.yaml (XCDk_RDREQ:
TCC_EA0_RDREQ of XCD k summed over its 16 TCC instances; XCDk_RDREQ128: the 128-B requests) and
prints, per dispatch of k_rollout1s, the read requests per XCD, their bytes (128 B each, the
request-size counters show ~98 % are 128 B) and the excess over the launch's algorithmic reads
(one action byte per env-step, split evenly over the XCDs: workgroups go round-robin).

    python tools/pmc_xcd.py <run_counter_collection.csv> --envs 4096 --steps 2000
"""
import argparse
import collections
import csv

ap = argparse.ArgumentParser()
ap.add_argument("csv")
ap.add_argument("--envs", type=int, required=True)
ap.add_argument("--steps", type=int, required=True)
ap.add_argument("--kernel", default="k_rollout1s")
a = ap.parse_args()
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(a.csv)):
    if a.kernel in r["Kernel_Name"]:
        agg[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
alg_xcd = a.envs * a.steps / 8 / 1e6
print(f"algorithmic reads per XCD {alg_xcd:.3f} MB (actions: {a.envs} envs x {a.steps} steps / 8 XCDs)")
for d in sorted(agg):
    v = agg[d]
    mb = [v.get(f"XCD{k}_RDREQ", v.get(f"XCD{k}_RDREQ128", 0.0)) * 128 / 1e6 for k in range(8)]
    ex = [m - alg_xcd for m in mb]
    print(f"dispatch {d}: MB per XCD " + " ".join(f"{m:.3f}" for m in mb) +
          f" | excess per XCD min {min(ex):.3f} max {max(ex):.3f} total {sum(ex):.2f} MB")
