"""Readers for the golden vectors in tests/golden/*.json.gz (see tests/golden/make_golden.py)."""
import glob
import gzip
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
POOLS = sorted(os.path.basename(p)[:-8] for p in glob.glob(os.path.join(GOLDEN, "pool*.json.gz")))


def load(name):
    with gzip.open(os.path.join(GOLDEN, name + ".json.gz"), "rt") as f:
        return json.load(f)


def dense(plane, dtype=np.int64):
    a = np.zeros(plane["shape"], dtype)
    for i, v in plane["nz"]:
        a.flat[i] = v
    return a


def oracle_puzzles(golden):
    """processed reference puzzles -> oracle pool format."""
    out = []
    for p in golden["processed"]:
        out.append({"x_size": p["x_size"], "y_size": p["y_size"], "start": p["start"],
                    "target": p["target"], "solution_count": p["solution_count"],
                    "solution_paths": p["solution_paths"], "gaps": dense(p["base"]["gaps"])})
    return out


def rows_as_ndarray(grid):
    """list of rows -> 1-D object ndarray of per-row string ndarrays: the form a parquet export
    of the dataset gives puzzle_array (make_golden.text_episodes(ndarray_rows=True))."""
    out = np.empty(len(grid), dtype=object)
    for k, r in enumerate(grid):
        out[k] = np.array(r, dtype=object)
    return out


def text_dataframe(golden):
    """The DataFrame a text-obs fixture was generated from (puzzle_array in its recorded form)."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(GOLDEN), os.pardir, "sparc-gym_amd"))
    from sparc_gym_amd import synthetic
    df = synthetic.records_to_dataframe(golden["records"])
    if golden.get("ndarray_rows"):
        df["puzzle_array"] = [rows_as_ndarray(g) for g in df["puzzle_array"]]
    return df
