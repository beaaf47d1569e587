#!/usr/bin/env python3
"""Join tools/pmc_calib/pmc_calib.hip's expected byte counts with its rocprofv3 counter passes.

    analyze.py <calib stdout> <counter_collection.csv> [more csv ...] > calib.json

For every calibration dispatch (kernel, grid) it reports the known read / write bytes beside
  fetch_kb        FETCH_SIZE (KB as rocprofv3 derives it)
  req_bytes       128 * RDREQ_128B + 64 * (RDREQ - RDREQ_128B - RDREQ_32B) + 32 * RDREQ_32B:
                  the read requests by size (gfx950 has a 128-B request counter; FETCH_SIZE's
                  formula takes 128-B requests from TCC_BUBBLE instead)
  write_kb        WRITE_SIZE
and the ratios measured / known.  The traffic model of tools/pmc_traffic.py takes its read
bytes from the request counters when they were collected (the ratio column shows why)."""
import collections
import csv
import json
import sys


def main():
    expect = [json.loads(ln) for ln in open(sys.argv[1]) if ln.startswith("{")]
    per = collections.defaultdict(dict)   # (kernel, grid) -> counter -> value
    for path in sys.argv[2:]:
        for r in csv.DictReader(open(path)):
            name = r["Kernel_Name"].split("(")[0].strip()
            grid = int(r.get("Grid_Size", r.get("Grid_Size_X", 0)) or 0) // 256
            d = per[(name, grid)]
            d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    rows = []
    for e in expect:
        c = per.get((e["kernel"], e["grid"]), {})
        row = dict(e)
        if "FETCH_SIZE" in c:
            row["fetch_bytes"] = c["FETCH_SIZE"] * 1024
        if "TCC_EA0_RDREQ_sum" in c:
            n = c["TCC_EA0_RDREQ_sum"]
            n32 = c.get("TCC_EA0_RDREQ_32B_sum", 0.0)
            n128 = c.get("TCC_EA0_RDREQ_128B_sum", 0.0)
            n64c = c.get("TCC_EA0_RDREQ_64B_sum")
            row["rdreq"] = {"all": n, "32B": n32, "64B": n64c, "128B": n128}
            row["req_bytes"] = 128 * n128 + 64 * (n - n128 - n32) + 32 * n32
        if "WRITE_SIZE" in c:
            row["write_size_bytes"] = c["WRITE_SIZE"] * 1024
        if e["read_bytes"]:
            for k in ("fetch_bytes", "req_bytes"):
                if k in row:
                    row[k.replace("bytes", "ratio")] = round(row[k] / e["read_bytes"], 4)
        if e["write_bytes"] and "write_size_bytes" in row:
            row["write_ratio"] = round(row["write_size_bytes"] / e["write_bytes"], 4)
        rows.append(row)
    json.dump(rows, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
