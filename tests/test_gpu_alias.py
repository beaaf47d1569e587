"""SPaRC_Gym(alias_compat=True) against the reference's plane aliasing (SPaRC_Gym.py:149-151).

The fixtures (tests/golden/make_alias_golden.py) come from ONE reference env object playing
many episodes over a few puzzles without restoring them, so most resets start from the planes
the previous episode on that puzzle left behind, and the stale `visited` bits change the legal
moves (1040, 1141) and the dots rule (529).  Every reset and step must match: reward value and
type, flags, info, both planes and the whole rule_status dict."""
import numpy as np
import pytest

import golden_io
from oracle import rules_ref

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

ALIAS = ["alias_tb1", "alias_tb0", "alias_rules", "alias_mixed"]


def _check_snapshot(obs, info, ref, where):
    assert np.array_equal(obs["base"]["visited"], golden_io.dense(ref["visited"])), where
    assert np.array_equal(obs["base"]["agent_location"], golden_io.dense(ref["agent_plane"])), where
    for k in ("legal_actions", "current_step", "solution_count", "difficulty", "grid_x_size", "grid_y_size"):
        assert info[k] == ref["info"][k], (where, k)
    assert [int(v) for v in info["agent_location"]] == ref["info"]["agent_location"], where
    assert repr(info["Rewards"]["normal_reward"]) == ref["info"]["normal_reward"]["repr"], where
    assert repr(info["Rewards"]["outcome_reward"]) == ref["info"]["outcome_reward"]["repr"], where
    assert rules_ref.normalize(info["rule_status"]) == ref["rule_status"], where


@pytest.mark.parametrize("name", ALIAS)
def test_alias_compat_matches_reference(on_gpu, name):
    from sparc_gym_amd import SPaRC_Gym
    g = golden_io.load(name)
    env = SPaRC_Gym(puzzles=g["records"], traceback=g["traceback"], max_steps=g["max_steps"], alias_compat=True)
    for e, ep in enumerate(g["episodes"]):
        obs, info = env.reset(options={"puzzle_id": ep["puzzle_id"]})
        assert env.current_puzzle_index == ep["puzzle_index"]
        _check_snapshot(obs, info, ep["reset"], (name, e, "reset"))
        for t, (a, st) in enumerate(zip(ep["actions"], ep["steps"])):
            obs, r, term, trunc, info = env.step(a)
            assert repr(r) == st["reward"]["repr"] and type(r).__name__ == st["reward"]["type"], (name, e, t)
            assert (term, trunc) == (st["terminated"], st["truncated"]), (name, e, t)
            _check_snapshot(obs, info, st, (name, e, t))


def test_alias_fixture_needs_the_compat_mode(on_gpu):
    """The default (pristine re-load) mode departs from these fixtures: the quirk is exercised."""
    from sparc_gym_amd import SPaRC_Gym
    g = golden_io.load("alias_tb1")
    env = SPaRC_Gym(puzzles=g["records"], traceback=g["traceback"], max_steps=g["max_steps"])
    diffs = 0
    for ep in g["episodes"]:
        obs, info = env.reset(options={"puzzle_id": ep["puzzle_id"]})
        diffs += info["legal_actions"] != ep["reset"]["info"]["legal_actions"]
        diffs += not np.array_equal(obs["base"]["visited"], golden_io.dense(ep["reset"]["visited"]))
    assert diffs > 10
