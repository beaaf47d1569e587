"""Pin both oracle restatements (pure Python and C) to the reference's own golden vectors."""
import numpy as np
import pytest

import golden_io
from oracle import COracle
from oracle.cpu_ref import CpuRefEnv


def _code(r):
    return int(round(float(r) * 100))


@pytest.mark.parametrize("pool", golden_io.POOLS)
def test_cpu_ref_matches_reference(pool):
    g = golden_io.load(pool)
    puzzles = golden_io.oracle_puzzles(g)
    for ep in g["episodes"]:
        env = CpuRefEnv(puzzles[ep["puzzle_index"]], g["traceback"], g["max_steps"])
        assert env.legal_actions() == ep["reset"]["info"]["legal_actions"]
        for a, st in zip(ep["actions"], ep["steps"]):
            r, term, trunc = env.step(a)
            # value AND Python type (0 int, +-0.01 float, +-1 int; SPaRC_Gym.py:1133-1223)
            assert repr(r) == st["reward"]["repr"] and type(r).__name__ == st["reward"]["type"]
            assert term == st["terminated"] and trunc == st["truncated"]
            assert env.legal_actions() == st["info"]["legal_actions"]
            assert env.loc == st["info"]["agent_location"]
            assert env.current_step == st["info"]["current_step"]
            assert repr(env.outcome_reward) == st["info"]["outcome_reward"]["repr"]
            assert np.array_equal(env.visited, golden_io.dense(st["visited"]))


@pytest.mark.parametrize("pool", golden_io.POOLS)
def test_c_oracle_matches_reference(pool):
    g = golden_io.load(pool)
    puzzles = golden_io.oracle_puzzles(g)
    eps = g["episodes"]
    T = max(len(e["actions"]) for e in eps)
    # all episodes of the pool as one batch; shorter ones padded with steps we do not check
    o = COracle(puzzles, len(eps), g["traceback"], g["max_steps"], autoreset=0)
    o.reset([e["puzzle_index"] for e in eps])
    acts = np.zeros((T, len(eps)), np.uint8)
    for i, e in enumerate(eps):
        acts[:len(e["actions"]), i] = e["actions"]
    # step one at a time so that the per-step state can be checked
    for t in range(T):
        rew, flags = o.rollout(1, acts[t:t + 1])
        s = o.state()
        for i, e in enumerate(eps):
            if t >= len(e["steps"]):
                continue
            st = e["steps"][t]
            assert rew[0, i] == _code(st["reward"]["value"]), (pool, i, t)
            assert bool(flags[0, i] & 1) == st["terminated"]
            assert bool(flags[0, i] & 2) == st["truncated"]
            legal = [a for a in range(4) if (flags[0, i] >> (2 + a)) & 1]
            assert legal == st["info"]["legal_actions"]
            assert [s["x"][i], s["y"][i]] == st["info"]["agent_location"]
            assert s["step"][i] == st["info"]["current_step"]
            X, Y = st["visited"]["shape"]
            assert np.array_equal(s["visited"][i, :X, :Y], golden_io.dense(st["visited"]))


def test_rand_action_distribution():
    g = golden_io.load("poolA_tb0")
    o = COracle(golden_io.oracle_puzzles(g), 1, False, 2000)
    a = np.array([o.rand_action(7, e, t) for e in range(64) for t in range(64)])
    assert set(np.unique(a)) == {0, 1, 2, 3}
    assert abs(np.bincount(a).min() - len(a) / 4) < 0.1 * len(a)


@pytest.mark.parametrize("pool", golden_io.POOLS)
def test_c_oracle_obs_planes_match_reference(pool):
    """oracle_rollout_obs's per-step visited / agent_location planes == the reference's
    obs['base'] planes after every step (SPaRC_Gym.py:956-979), padded to 16x16."""
    g = golden_io.load(pool)
    puzzles = golden_io.oracle_puzzles(g)
    eps = g["episodes"]
    T = max(len(e["actions"]) for e in eps)
    o = COracle(puzzles, len(eps), g["traceback"], g["max_steps"], autoreset=0)
    o.reset([e["puzzle_index"] for e in eps])
    acts = np.zeros((T, len(eps)), np.uint8)
    for i, e in enumerate(eps):
        acts[:len(e["actions"]), i] = e["actions"]
    _, _, vis, agent = o.rollout_obs(T, 16, 16, acts)
    for i, e in enumerate(eps):
        for t, st in enumerate(e["steps"]):
            X, Y = st["visited"]["shape"]
            assert np.array_equal(vis[t, i, :X, :Y], golden_io.dense(st["visited"])), (pool, i, t)
            assert np.array_equal(agent[t, i, :X, :Y], golden_io.dense(st["agent_plane"])), (pool, i, t)
            assert vis[t, i].sum() == vis[t, i, :X, :Y].sum() and agent[t, i].sum() == 1
