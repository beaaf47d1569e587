#!/usr/bin/env python3
"""Load time of the rule table on a large pool: sparc_load_rules builds the
region-code table on the GPU (k_region_table: every region cell mask of every puzzle with at most
12 cells, one exact-fit search per mask whose area check passes) up to the 2^28-entry budget.

    python tools/prof_load_rules.py [--puzzles 100000] [--distinct 2000] [--grid 3 4]

`--distinct` synthetic puzzles of the given cell grid (3 x 4 cells: 12 cells, 4,096 masks each),
with the full property set and with base planes only, are repeated up to `--full` and
`--puzzles` (the table build does the same work per puzzle whether or not two are equal).  Prints one JSON line: host packing time, the
sparc_load_rules wall time, the puzzles that got a table (the rest: past the budget) and the
entries built."""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "sparc-gym_amd"))

import torch  # noqa: E402

from sparc_gym_amd import synthetic  # noqa: E402
from sparc_gym_amd.core import SparcCore  # noqa: E402
from sparc_gym_amd.puzzles import pack_rules, pack_table, process_puzzles  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--puzzles", type=int, default=100000)
ap.add_argument("--distinct", type=int, default=1000)
ap.add_argument("--full", type=int, default=100000,
                help="puzzles with the full property set (the rest: base planes); the rule table has no "
                     "pool-wide limit (32-bit instance offsets, 21-bit shape ids)")
ap.add_argument("--grid", type=int, nargs=2, default=(3, 4))
a = ap.parse_args()
t0 = time.perf_counter()
full = process_puzzles(synthetic.make_puzzles(a.distinct, seed=0, sizes=(tuple(a.grid),), full_properties=True))
base = process_puzzles(synthetic.make_puzzles(a.distinct, seed=1, sizes=(tuple(a.grid),), full_properties=False))
proc = [full[k % len(full)] for k in range(min(a.full, a.puzzles))]
proc += [base[k % len(base)] for k in range(a.puzzles - len(proc))]
t1 = time.perf_counter()
table = pack_table(proc)
rules = pack_rules(proc, table)
t2 = time.perf_counter()
torch.cuda.init()
core = SparcCore(table, 256, True, 2000, "next_step", 0)
torch.cuda.synchronize()
t3 = time.perf_counter()
core.load_rules(rules)
core.sync()
t4 = time.perf_counter()
cells = a.grid[0] * a.grid[1]
per = 8 * (1 if cells <= 3 else 1 << (cells - 3))
tabled = min(a.puzzles, (1 << 28) // per)
print(json.dumps({"puzzles": a.puzzles, "full_property_puzzles": min(a.full, a.puzzles), "distinct": a.distinct,
                  "cells": cells, "words": table.words, "instances": int(len(rules.inst)),
                  "generate_s": round(t1 - t0, 2), "pack_s": round(t2 - t1, 2),
                  "load_rules_s": round(t4 - t3, 3), "puzzles_with_table": tabled,
                  "table_entries": tabled * per, "table_mb": round(tabled * per / 2 / 2**20, 1)}))
