"""Edge cases of the multi-word split kernel (k_rolloutWs) against the C oracle.

Gap-free 9x9 and 15x15 lattices (no cell centres marked as gaps: a table the C ABI accepts,
though _process_puzzles never makes one, SPaRC_Gym.py:345-351), traceback on, autoreset 'none':
half of the envs walk a snake through EVERY point (len reaches the lattice's point count) and
keep stepping after the episode ended, so the move wave writes its stack slot len - 1 = points
- 1 on every later step.  The stack must hold that slot (a one-byte-short stack wrote into the
next pair's action tile); the other envs step randomly and would see such corruption.
Compared with the C oracle: reward codes, flags, stats, final state (SPaRC_Gym.py:1111-1238).
"""
import copy

import numpy as np
import pytest

from oracle import COracle
from sparc_gym_amd import synthetic
from sparc_gym_amd.puzzles import pack_table, process_puzzles

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


def _snake(X, Y):
    """Actions of a path from (0, 0) through every point: down a column, right, up the next..."""
    acts = []
    for x in range(X):
        acts += [3 if x % 2 == 0 else 1] * (Y - 1)
        if x + 1 < X:
            acts.append(0)
    return acts


def _gap_free_pool(cells):
    proc = process_puzzles(synthetic.make_puzzles(4, seed=5, sizes=((cells, cells),), full_properties=False))
    out = []
    for k, p in enumerate(proc):
        q = copy.deepcopy(p)
        X, Y = q["x_size"], q["y_size"]
        q["obs_array"]["gaps"] = np.zeros_like(np.asarray(q["obs_array"]["gaps"]))
        q["start_location"] = [0, 0]
        q["target_location"] = [X - 1, Y - 1] if k % 2 == 0 else [X - 1, 0]
        # one solution: the snake itself
        path, x, y = [[0, 0]], 0, 0
        for a in _snake(X, Y):
            x, y = x + (1 if a == 0 else -1 if a == 2 else 0), y + (-1 if a == 1 else 1 if a == 3 else 0)
            path.append([x, y])
        q["solution_paths"] = [path]
        q["solution_count"] = 1
        out.append(q)
    return out


@pytest.mark.parametrize("cells", [4, 7])   # 9x9 (2 words), 15x15 (4 words)
def test_gap_free_full_path_snake_vs_oracle(on_gpu, cells):
    from sparc_gym_amd import SPaRCVecEnv
    proc = _gap_free_pool(cells)
    table = pack_table(proc)
    X = proc[0]["x_size"]
    assert table.words == (2 if cells == 4 else 4)
    n = 512
    snake = _snake(X, X)
    T = len(snake) + 32
    T -= T % 16                                    # whole tiles: k_rolloutWs only
    rng = np.random.default_rng(cells)
    acts = rng.integers(0, 4, (T, n)).astype(np.uint8)
    for i in range(0, n, 2):                       # even envs: the snake, then "right" (illegal)
        acts[:len(snake), i] = snake
        acts[len(snake):, i] = 0
    pids = np.arange(n) % len(proc)
    v = SPaRCVecEnv(n, processed=proc, table=table, traceback=True, max_steps=100000, autoreset="none",
                    observation="compact")
    v.reset(options={"puzzle_index": pids})
    stats = torch.zeros((n, 4), dtype=torch.int32, device="cuda")
    out = v.rollout(T, torch.from_numpy(acts).cuda(), stats=stats)
    pool = [{"x_size": p["x_size"], "y_size": p["y_size"], "start": list(p["start_location"]),
             "target": list(p["target_location"]), "solution_count": p["solution_count"],
             "solution_paths": p["solution_paths"], "gaps": p["obs_array"]["gaps"]} for p in proc]
    o = COracle(pool, n, True, 100000, autoreset=0)
    o.reset(pids)
    ost = np.zeros((n, 4), np.int32)
    ro, fo = o.rollout(T, acts, stats=ost)
    assert np.array_equal(out["reward_code"].cpu().numpy(), ro)
    assert np.array_equal(out["flags"].cpu().numpy(), fo)
    assert np.array_equal(stats.cpu().numpy(), ost)
    s, so = v.state(), o.state()
    assert np.array_equal(s["path_len"].astype(np.int64), so["path_len"])
    assert int(so["path_len"][0]) == X * X            # the snake covered every point
    assert (ro[len(snake) - 1, 0::4] == 100).all()    # and solved the puzzles whose target is its end
