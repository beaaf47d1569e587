#!/usr/bin/env python3
"""Fold rocprofv3 --pmc passes into profiles/pmc_traffic.json for bench.py's `roofline.traffic`.

Usage: pmc_traffic.py <workload-key> <kernel> <fetch.csv> <write.csv> [sq.csv ...]

traffic per launch = read bytes + WRITE_SIZE (KB -> B), each the mean over dispatches of <kernel>
after the first (warmup).  Read bytes come from the read-request counters by size when their
pass (TCC_EA0_RDREQ{,_32B,_64B,_128B}_sum) is given: tools/pmc_calib measured that these give
the bytes of every access width the kernels use, while FETCH_SIZE counts a 128-B request as 64 B
(MI355X_MICROARCH.md's HBM section); without that pass, 2 x FETCH_SIZE (exact only for 16-B/lane
streaming reads).  WRITE_SIZE is exact for 16-B/lane streaming stores (the reward/flag tiles).  Extra csv files
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
    # read bytes: from the read requests by size when that pass was collected (tools/pmc_calib:
    # 128-B requests are what FETCH_SIZE undercounts on gfx950, so the request counters give the
    # bytes for every access width), else the guide's 2 x FETCH_SIZE for 16-B streaming reads
    if "TCC_EA0_RDREQ_sum" in counters and "TCC_EA0_RDREQ_128B_sum" in counters:
        n, n32, n128 = (counters["TCC_EA0_RDREQ_sum"], counters.get("TCC_EA0_RDREQ_32B_sum", 0.0),
                        counters["TCC_EA0_RDREQ_128B_sum"])
        read_b = 128 * n128 + 64 * (n - n128 - n32) + 32 * n32
        read_model = "128 x RDREQ_128B + 64 x RDREQ_64B + 32 x RDREQ_32B (request counters)"
    else:
        read_b = 2 * f["FETCH_SIZE"] * 1024
        read_model = "2 x FETCH_SIZE"
    traffic = int(round(read_b + w["WRITE_SIZE"] * 1024))
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
        "read_bytes": int(round(read_b)),
        "read_model": read_model,
        "write_size_kb": round(w["WRITE_SIZE"], 1),
        "counters": {k: round(v, 1) for k, v in counters.items()},
        "source": [os.path.relpath(os.path.abspath(x), repo) for x in (fetch, write, *extra)],
    }
    json.dump(d, open(out, "w"), indent=1)
    print(key, kern, traffic)


if __name__ == "__main__":
    main()
