"""Host-side parity of the 'SPaRC' text observation and of the reset index choice (CPU).

* The text grid a reset shows (SPaRC_Gym.py:153-164 parsing the puzzle's puzzle_array, 988-992
  serialising it) equals the reference's reset observation for every episode of both text
  fixtures (list rows and parquet-style ndarray rows).  The per-step 'V' / 'L' / '+' edits need
  the device path and are checked in tests/test_gpu_text_resets.py.
* The seeded puzzle choice (SPaRC_Gym.py:1084-1085) equals the reference's for every seed of
  tests/golden/resets.json.gz, through the gymnasium fallback's seeding restatement.
"""
import pytest

import golden_io
from sparc_gym_amd.env import text_grid_rows, text_obs
from sparc_gym_amd.puzzles import process_puzzles
from sparc_gym_amd.spaces import Env

TEXT = ("text_tb1", "text_tb0_nd")


@pytest.mark.parametrize("name", TEXT)
def test_reset_text_grid_matches_reference(name):
    g = golden_io.load(name)
    proc = process_puzzles(golden_io.text_dataframe(g), "SPaRC")
    for ep in g["episodes"]:
        p = proc[ep["puzzle_index"]]
        assert str(p["id"]) == ep["puzzle_id"]
        assert text_obs(text_grid_rows(p["observ"])) == ep["reset_obs"]


def test_text_grid_forms_and_errors():
    rows = [["+", "S"], [".", "E"]]
    import numpy as np
    assert text_grid_rows(rows) == rows
    assert text_grid_rows(np.array(rows)) == rows
    assert text_grid_rows(golden_io.rows_as_ndarray(rows)) == rows
    fresh = text_grid_rows(rows)
    fresh[0][0] = "V"
    assert rows[0][0] == "+"                      # a fresh grid per load: edits never alias
    with pytest.raises(ValueError):
        text_grid_rows([["+", "+"], ["+"]])       # 162-163


def test_seeded_reset_index_matches_reference():
    r = golden_io.load("resets")
    env = Env()
    for seed, idx in r["seeded"]:
        Env.reset(env, seed=seed)
        assert int(env.np_random.integers(r["n"])) == idx, seed


def test_alias_fixtures_hold_stale_resets():
    """The aliasing fixtures (make_alias_golden.py) re-load puzzles in one reference env: most
    resets start with the previous episode's visited bits (more than the start point), and some
    start with fewer legal moves than a fresh load would give."""
    from golden_io import load
    for name in ("alias_tb1", "alias_tb0", "alias_rules", "alias_mixed"):
        g = load(name)
        stale = sum(len(ep["reset"]["visited"]["nz"]) > 1 for ep in g["episodes"])
        assert stale >= len(g["episodes"]) // 2, name
