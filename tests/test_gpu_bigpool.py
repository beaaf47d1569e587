"""Puzzle pools past the LDS row budget (the reference takes any dataset of the SPaRC structure,
/root/reference/README.md:37; reset() walks it sequentially, SPaRC_Gym.py:1087).

The split W = 1 rollout (k_rollout1s) stages every puzzle's move and trie rows in LDS while
they fit beside its rings (pools of at most 1,024 puzzles).  Larger pools run the same kernel with
the rows read from the L2: the move wave reads both rows of the next puzzle at the previous
reset and hands the trie row to the trie wave through per-env LDS slots, or, when two resets
of one env fall within two tiles, the trie wave reads the row itself (sparc_move1.hpp,
row_slots).  These tests compare that path with the C oracle directly:

* c3 at full size on a 4,096-puzzle pool: 65,536 envs, two back-to-back 2,000-step launches
  through the bench's C-ABI call, every env's reward codes, flags, stats and final state;
* the slot rule's fallback: max_steps 1, 2, 3 and 7 (an autoreset every 2-8 steps) on a
  2,048-puzzle pool with many solved episodes, chunked launches, traceback on and off, and the
  in-kernel random actions;
* autoreset 'none' on the same pool (the trie wave's slot path without resets).
"""
import os

import numpy as np
import pytest

from oracle import COracle
from sparc_gym_amd import synthetic
from sparc_gym_amd.puzzles import pack_table, process_puzzles

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

LDS_ROW_LIMIT = 1024   # k_rollout1s stages the rows in LDS up to this many puzzles


def _oracle_pool(proc):
    return [{"x_size": p["x_size"], "y_size": p["y_size"], "start": list(p["start_location"]),
             "target": list(p["target_location"]), "solution_count": p["solution_count"],
             "solution_paths": p["solution_paths"], "gaps": p["obs_array"]["gaps"]} for p in proc]


def _state_equal(s, so, table):
    from sparc_gym_amd.core import visited_planes
    for k, ko in (("x", "x"), ("y", "y"), ("step", "step"), ("path_len", "path_len"), ("puzzle", "pid"),
                  ("outcome", "outcome")):
        assert np.array_equal(s[k], so[ko]), k
    assert np.array_equal(visited_planes(s["visited"], table, 16, 16), so["visited"].astype(np.int32))


def _sharded_oracle(proc, pids, acts_list, tb, ms, shards=16):
    """The C oracle over column shards in threads; per launch (codes, flags), stats, state."""
    from concurrent.futures import ThreadPoolExecutor
    from oracle import OraclePool
    n = len(pids)
    bounds = np.linspace(0, n, shards + 1).astype(int)
    opool = OraclePool(_oracle_pool(proc))
    oracles = [COracle(opool, int(b - a), tb, ms, autoreset=1) for a, b in zip(bounds[:-1], bounds[1:])]
    stats = [np.zeros((int(b - a), 4), np.int32) for a, b in zip(bounds[:-1], bounds[1:])]
    for o, a in zip(oracles, bounds[:-1]):
        o.reset(pids[a:a + o.n])
    outs = []
    with ThreadPoolExecutor(shards) as ex:
        for acts in acts_list:
            futs = [ex.submit(o.rollout, acts.shape[0], np.ascontiguousarray(acts[:, a:a + o.n]), 0, 0, 0, st)
                    for o, a, st in zip(oracles, bounds[:-1], stats)]
            res = [f.result() for f in futs]
            outs.append((np.concatenate([r[0] for r in res], 1), np.concatenate([r[1] for r in res], 1)))
    states = [o.state() for o in oracles]
    return outs, np.concatenate(stats), {k: np.concatenate([s[k] for s in states]) for k in states[0]}


@pytest.mark.parametrize("P,placement", [(4096, "hash"), (16384, "hash"), (16384, "xcd")])
def test_c3_full_size_big_puzzle_pool_vs_oracle(on_gpu, P, placement):
    """c3 (65,536 envs, 7x7 full property set, traceback, max_steps 2,000, next-step autoreset)
    on a 4,096- and a 16,384-puzzle pool (bench.make_pool: the bench's 1,024-puzzle pool and more
    blocks; 16,384 is the pool of the bench line whose trie records outgrow an XCD's L2), env i ->
    puzzle i * 2654435761 mod P ('hash': the mixed 4-/8-B trie records) or the bench's XCD-local
    first puzzles ('xcd', bench.initial_puzzles: one eighth of the pool per XCD, so the reset keeps
    the 8-B records, xcd_hot_bytes), actions drawn as the bench's, two back-to-back 2,000-step
    launches through the bench's C-ABI call: every env bit-exact against the C oracle
    (SPaRC_Gym.py:1111-1238, reset 1087)."""
    import bench
    from sparc_gym_amd import SPaRCVecEnv
    os.environ["SPARC_POOL_WORKERS"] = "1"   # no worker processes from a process that drives the GPU
    proc = bench.make_pool(P, ((3, 3),), True)
    table = pack_table(proc)
    assert len(proc) == P > LDS_ROW_LIMIT and table.words == 1
    n, T, L = 65536, 2000, 2
    pids, used = bench.initial_puzzles(np.arange(n, dtype=np.uint64), len(proc), placement)
    assert used == placement
    v = SPaRCVecEnv(n, processed=proc, table=table, traceback=True, max_steps=2000, autoreset="next_step",
                    observation="compact")
    v.reset(options={"puzzle_index": pids})
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev)
    g.manual_seed(1234)
    acts = torch.randint(0, 4, (L, T, n), dtype=torch.uint8, device=dev, generator=g)
    rew = torch.empty((L, T, n), dtype=torch.int8, device=dev)
    flg = torch.empty((L, T, n), dtype=torch.uint8, device=dev)
    stats = torch.zeros((n, 4), dtype=torch.int32, device=dev)
    v._stream()
    for k in range(L):
        v.core.rollout_device(T, acts[k].data_ptr(), rew[k].data_ptr(), flg[k].data_ptr(), stats.data_ptr())
    torch.cuda.synchronize()
    v.core.sync()
    outs, ost, so = _sharded_oracle(proc, pids, list(acts.cpu().numpy()), True, 2000)
    r_np, f_np = rew.cpu().numpy(), flg.cpu().numpy()
    for k in range(L):
        assert np.array_equal(r_np[k], outs[k][0]), f"reward codes differ in launch {k}"
        assert np.array_equal(f_np[k], outs[k][1]), f"flags differ in launch {k}"
    assert np.array_equal(stats.cpu().numpy(), ost)
    _state_equal(v.state(), so, table)
    # the pool's far end is reached and episodes end both ways, with autoresets after them
    assert int(so["pid"].max()) >= 3 * P // 4
    f_all = f_np.reshape(-1, n)
    assert ((f_all & 1) != 0).sum() > 0 and ((f_all & 2) != 0).sum() > 0 and ((f_all & 64) != 0).sum() > 0


@pytest.fixture(scope="module")
def pool2048():
    recs = synthetic.make_puzzles(2048, seed=5, sizes=((3, 3), (2, 2)), n_solutions=8, shared_prefix_prob=0.9,
                                  full_properties=True)
    proc = process_puzzles(recs)
    return proc, pack_table(proc)


@pytest.mark.parametrize("max_steps", [1, 2, 3, 7, 2000])
@pytest.mark.parametrize("tb", [True, False])
@pytest.mark.parametrize("mixed", [0, 1])
def test_slot_fallback_short_episodes_vs_oracle(on_gpu, pool2048, max_steps, tb, mixed):
    """Autoresets every 2-8 steps: two resets of an env within two tiles make the move wave
    write its spare slot and the trie wave read the row from the L2 (the slot rule); launches of
    64 + 48 + 37 steps (the last one's 5-step tail through k_rollout1), the state round-tripping
    through HBM: reward codes, flags, stats and state against the C oracle.  mixed = 1 forces the
    mixed trie tables (SPARC_VARIANT_MIXED_TRIE: 4-B records for tries of <= 127 nodes, 8-B ones
    for the larger tries of this pool; by default only pools past 4 MB of records take them)."""
    from sparc_gym_amd import SPaRCVecEnv
    proc, table = pool2048
    assert len(proc) > LDS_ROW_LIMIT and table.words == 1
    if mixed:
        cnt = table.info[:, 3] & 0xFFFF
        assert (cnt > 127).any() and (cnt <= 127).any()   # both record formats in one pool
    n = 4096
    rng = np.random.default_rng(max_steps + 100 * tb)
    pids = rng.integers(len(proc), size=n)
    v = SPaRCVecEnv(n, processed=proc, table=table, traceback=tb, max_steps=max_steps, autoreset="next_step",
                    observation="compact")
    v.core.set_variant(v.core.VARIANT_MIXED_TRIE, 1 if mixed else 2)
    v.reset(options={"puzzle_index": pids})
    o = COracle(_oracle_pool(proc), n, tb, max_steps, autoreset=1)
    o.reset(pids)
    st = torch.zeros((n, 4), dtype=torch.int32, device="cuda")
    ost = np.zeros((n, 4), np.int32)
    solved = 0
    for T in (64, 48, 37):
        acts = rng.integers(0, 4, size=(T, n)).astype(np.uint8)
        out = v.rollout(T, torch.from_numpy(acts).cuda(), stats=st)
        ro, fo = o.rollout(T, acts, stats=ost)
        r = out["reward_code"].cpu().numpy()
        assert np.array_equal(r, ro), f"reward codes differ (T={T})"
        assert np.array_equal(out["flags"].cpu().numpy(), fo), f"flags differ (T={T})"
        solved += int((r == 100).sum())
    assert np.array_equal(st.cpu().numpy(), ost)
    _state_equal(v.state(), o.state(), table)
    if max_steps <= 7:
        assert ost[:, 3].sum() > 10 * n    # many autoresets per env
    if max_steps >= 3:
        assert solved > 0


def test_slot_path_random_actions_and_no_autoreset(on_gpu, pool2048):
    """The in-kernel random actions (k_rollout1s<…, RAND, global rows>) with short episodes, and
    autoreset 'none' (no resets: the trie wave's slot path never reads a slot)."""
    from sparc_gym_amd import SPaRCVecEnv
    proc, table = pool2048
    n = 4096
    pids = (np.arange(n) * 7 + 3) % len(proc)
    for autoreset, ms in (("next_step", 5), ("none", 40)):
        v = SPaRCVecEnv(n, processed=proc, table=table, traceback=True, max_steps=ms, autoreset=autoreset,
                        observation="compact")
        v.reset(options={"puzzle_index": pids})
        o = COracle(_oracle_pool(proc), n, True, ms, autoreset=1 if autoreset == "next_step" else 0)
        o.reset(pids)
        st = torch.zeros((n, 4), dtype=torch.int32, device="cuda")
        ost = np.zeros((n, 4), np.int32)
        out = v.rollout(96, None, seed=31, t0=5, stats=st)
        ro, fo = o.rollout(96, None, seed=31, t0=5, stats=ost)
        assert np.array_equal(out["reward_code"].cpu().numpy(), ro), autoreset
        assert np.array_equal(out["flags"].cpu().numpy(), fo), autoreset
        assert np.array_equal(st.cpu().numpy(), ost), autoreset
        _state_equal(v.state(), o.state(), table)
