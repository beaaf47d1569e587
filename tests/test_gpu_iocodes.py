"""k_rollout1s with the reward codes and episode counters derived by the I/O waves (IOR, the
default under next-step autoreset): the trie wave hands over a class byte per env-step and the
I/O waves compute the codes four envs per dword (io_codes4) and count per env in bytes, flushed
to LDS at least every 128 tiles.  Checked bit-exact against the C oracle:

* the W = 1 kernel and the multi-word kernel (k_rolloutWs<4>, k_rolloutWs<2>: 16-bit words,
  io_codes4w);
* many 16-step launches (every launch end is a chance for a done last step: the stored
  outcome, i.e. Oneg after the launch, comes from TrieLane::finish_oneg), with and without
  traceback, so that both solved and failed done steps end launches;
* one 4,160-step launch (260 tiles: two mid-launch counter flushes), stats and state;
* the same launches with the codes on the trie wave (sparc_set_variant SPARC_VARIANT_IO_CODES_OFF)
  give identical outputs.
"""

import numpy as np
import pytest

from oracle import COracle
from sparc_gym_amd import synthetic
from sparc_gym_amd.puzzles import pack_table, process_puzzles

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


# W = 1 (k_rollout1s), 15 x 15 points (k_rolloutWs<4>), mixed 5 x 5 - 11 x 11 (k_rolloutWs<2>)
POOLS = {"w1": ((3, 3),), "w4": ((7, 7),), "mixed": ((2, 2), (3, 3), (4, 4), (5, 5))}


def _pool(sizes):
    proc = process_puzzles(synthetic.make_puzzles(1024, seed=0, sizes=sizes, full_properties=True))
    opool = [{"x_size": p["x_size"], "y_size": p["y_size"], "start": list(p["start_location"]),
              "target": list(p["target_location"]), "solution_count": p["solution_count"],
              "solution_paths": p["solution_paths"], "gaps": p["obs_array"]["gaps"]} for p in proc]
    return proc, pack_table(proc), opool


def _pids(n):
    return (np.arange(n, dtype=np.uint64) * 2654435761 % 1024).astype(np.int64)


def _state(v):
    s = v.state()
    return {k: np.asarray(s[k]) for k in ("x", "y", "step", "path_len", "puzzle", "outcome")}


def _ostate(o):
    s = o.state()
    return {"x": s["x"], "y": s["y"], "step": s["step"], "path_len": s["path_len"], "puzzle": s["pid"],
            "outcome": s["outcome"]}


def _run(pool, tb, launches, T, io_off):
    from sparc_gym_amd import SPaRCVecEnv
    proc, table, opool = _pool(POOLS[pool])
    n = 1024
    v = SPaRCVecEnv(n, processed=proc, table=table, traceback=tb, max_steps=2000, observation="compact")
    if io_off:
        v.core.set_variant(v.core.VARIANT_IO_CODES_OFF, 1)
    v.reset(options={"puzzle_index": _pids(n)})
    st = torch.zeros((n, 4), dtype=torch.int32, device="cuda")
    g = torch.Generator(device="cuda")
    g.manual_seed(5)
    outs = []
    for _ in range(launches):
        acts = torch.randint(0, 4, (T, n), dtype=torch.uint8, device="cuda", generator=g)
        out = v.rollout(T, acts, stats=st)
        outs.append((acts.cpu().numpy(), out["reward_code"].cpu().numpy(), out["flags"].cpu().numpy(), _state(v),
                     st.cpu().numpy().copy()))
    return outs, opool


@pytest.mark.parametrize("pool", list(POOLS))
@pytest.mark.parametrize("tb", [True, False])
def test_io_codes_short_launches_vs_oracle(on_gpu, pool, tb):
    outs, opool = _run(pool, tb, 48, 16, False)
    n = 1024
    o = COracle(opool, n, tb, 2000, autoreset=1)
    o.reset(_pids(n))
    ost = np.zeros((n, 4), np.int32)
    ends = {1: 0, -1: 0}
    for acts, r, f, s, st in outs:
        ro, fo = o.rollout(16, acts, stats=ost)
        assert np.array_equal(r, ro) and np.array_equal(f, fo)
        assert np.array_equal(st, ost)
        so = _ostate(o)
        for k in s:
            assert np.array_equal(s[k], so[k]), k
        for k in ends:
            ends[k] += int((so["outcome"] == k).sum())
    # launches did end on solved and on failed done steps (outcome 1 / -1 in the stored state)
    # (15 x 15 with traceback: random walks rarely solve, ~1 launch end in 48)
    assert ends[-1] > 0 and (ends[1] > 0 or (pool == "w4" and tb)), ends
    # and the trie-wave path gives the same outputs
    outs_off, _ = _run(pool, tb, 48, 16, True)
    for a, b in zip(outs, outs_off):
        for x, y in zip(a[1:3] + (a[4],), b[1:3] + (b[4],)):
            assert np.array_equal(x, y)


@pytest.mark.parametrize("pool", ["w1", "w4"])
def test_io_codes_long_launch_flushes_vs_oracle(on_gpu, pool):
    T = 4160   # 260 tiles: the byte counters flush after tiles 127 and 255 and at the end
    outs, opool = _run(pool, True, 1, T, False)
    acts, r, f, s, st = outs[0]
    n = 1024
    o = COracle(opool, n, True, 2000, autoreset=1)
    o.reset(_pids(n))
    ost = np.zeros((n, 4), np.int32)
    ro, fo = o.rollout(T, acts, stats=ost)
    assert np.array_equal(r, ro) and np.array_equal(f, fo)
    assert np.array_equal(st, ost)
    so = _ostate(o)
    for k in s:
        assert np.array_equal(s[k], so[k]), k
    assert ost[:, 1].max() > 0 and np.abs(ost[:, 0]).max() > 255   # counters past one byte
