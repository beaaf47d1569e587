"""CPU check of the kernel ALGORITHM (tests/kernel_model.py mirrors csrc/sparc_env.hpp) against the
C oracle, including launches that split an episode at arbitrary points (state round trip)."""
import numpy as np
import pytest

import golden_io
from kernel_model import KernelModel
from oracle import COracle
from sparc_gym_amd import synthetic
from sparc_gym_amd.puzzles import pack_table, process_puzzles


def _pool(proc):
    return [{"x_size": p["x_size"], "y_size": p["y_size"], "start": list(p["start_location"]),
             "target": list(p["target_location"]), "solution_count": p["solution_count"],
             "solution_paths": p["solution_paths"], "gaps": p["obs_array"]["gaps"]} for p in proc]


CASES = [
    ("7x7", ((3, 3),), True), ("7x7_base", ((3, 3),), False),
    ("mixed", ((2, 2), (3, 3), (4, 4), (5, 5), (2, 4)), True), ("15x15", ((7, 7),), True),
]


@pytest.mark.parametrize("name,sizes,full", CASES)
@pytest.mark.parametrize("tb", [False, True])
@pytest.mark.parametrize("autoreset", [0, 1])
def test_model_matches_oracle_with_chunked_launches(name, sizes, full, tb, autoreset):
    proc = process_puzzles(synthetic.make_puzzles(12, seed=len(name) + 7 * tb, sizes=sizes, full_properties=full))
    table = pack_table(proc)
    n, T = 24, 160
    rng = np.random.default_rng(autoreset * 10 + tb)
    pids = rng.integers(len(proc), size=n)
    acts = rng.choice(np.array([0, 1, 2, 3, 0, 1, 2, 3, 4, 255], np.uint8), size=(T, n))
    max_steps = 2000 if autoreset else 90
    m = KernelModel(table, n, tb, max_steps, autoreset)
    m.reset(pids)
    cuts = [0, 1, 2, 5, 13, 40, 41, 100, T]   # launches of 1, 1, 3, 8, 27, 1, 59, 60 steps
    parts = [m.rollout(acts[a:b]) for a, b in zip(cuts[:-1], cuts[1:])]
    rm = np.concatenate([p[0] for p in parts])
    fm = np.concatenate([p[1] for p in parts])
    o = COracle(_pool(proc), n, tb, max_steps, autoreset)
    o.reset(pids)
    ro, fo = o.rollout(T, acts)
    assert not m.guard_fired
    assert np.array_equal(rm, ro)
    assert np.array_equal(fm, fo)


@pytest.mark.parametrize("pool", ["poolA_tb1", "poolD_tb1", "poolE_tb1"])
def test_model_matches_golden_one_step_launches(pool):
    """Every golden episode with one launch per step (the k_step path)."""
    g = golden_io.load(pool)
    proc = process_puzzles(g["records"])
    table = pack_table(proc)
    for ep in g["episodes"]:
        m = KernelModel(table, 1, g["traceback"], g["max_steps"], 0)
        m.reset([ep["puzzle_index"]])
        for a, st in zip(ep["actions"], ep["steps"]):
            r, f = m.rollout(np.array([[a if a < 256 else 255]], np.uint8))
            assert r[0, 0] == int(round(st["reward"]["value"] * 100))
            assert bool(f[0, 0] & 1) == st["terminated"] and bool(f[0, 0] & 2) == st["truncated"]
            assert [k for k in range(4) if f[0, 0] >> (2 + k) & 1] == st["info"]["legal_actions"]
    assert not m.guard_fired
