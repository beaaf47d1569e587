#!/usr/bin/env python3
"""Fold rocprofv3 --pmc passes into profiles/pmc_traffic.json for bench.py's `roofline.traffic`.

Usage: pmc_traffic.py <workload-key> <kernel> <fetch.csv> <write.csv> [sq.csv ...]

traffic per launch = 2 * FETCH_SIZE + WRITE_SIZE (KB -> B), each the mean over dispatches
of <kernel> after the first (warmup).  FETCH_SIZE is doubled per MI355X_MICROARCH.md's HBM
section: gfx950 reports half of a 16-B/lane streaming read (the kernel's action tiles);
WRITE_SIZE is exact for 16-B/lane streaming stores (its reward/flag tiles).  Extra csv files
(SQ_* passes) are averaged the same way and recorded with the entry, together with the hash of
the kernel sources (bench.csrc_hash): bench.py uses an entry only for the same sources."""
import collections
import csv
import json
import os
import sys


def per_dispatch(path, kern):
    per = collections.defaultdict(dict)
    for r in csv.DictReader(open(path)):
        if kern not in r["Kernel_Name"]:
            continue
        d = per[int(r["Dispatch_Id"])]
        d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    ids = sorted(per)[1:] or sorted(per)
    names = sorted({k for i in ids for k in per[i]})
    return {n: sum(per[i].get(n, 0.0) for i in ids) / len(ids) for n in names}, len(ids)


def main():
    key, kern, fetch, write, *extra = sys.argv[1:]
    f, nf = per_dispatch(fetch, kern)
    w, nw = per_dispatch(write, kern)
    counters = {**f, **w}
    for p in extra:
        counters.update(per_dispatch(p, kern)[0])
    traffic = int(round((2 * f["FETCH_SIZE"] + w["WRITE_SIZE"]) * 1024))
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, repo)
    import bench   # csrc_hash: the kernel sources these counters were collected on
    out = os.path.join(repo, "profiles", "pmc_traffic.json")
    d = json.load(open(out)) if os.path.exists(out) else {}
    d.setdefault(key, {})[kern] = {
        "bytes": traffic,
        "csrc_hash": bench.csrc_hash(),
        "dispatches_averaged": min(nf, nw),
        "fetch_size_kb_raw": round(f["FETCH_SIZE"], 1),
        "write_size_kb": round(w["WRITE_SIZE"], 1),
        "counters": {k: round(v, 1) for k, v in counters.items()},
        "source": [os.path.relpath(os.path.abspath(x), repo) for x in (fetch, write, *extra)],
    }
    json.dump(d, open(out, "w"), indent=1)
    print(key, kern, traffic)


if __name__ == "__main__":
    main()
