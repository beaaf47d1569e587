"""GPU parity: the HIP step path (through the C ABI) against the reference's golden vectors and
against the C oracle at batch sizes up to the benchmark's 65,536 envs.  Bit-exact throughout:
reward codes, flags, positions, step counters and visited bitboards are integers."""
import zlib

import numpy as np
import pytest

import golden_io
from oracle import COracle
from sparc_gym_amd import synthetic
from sparc_gym_amd.puzzles import pack_table, process_puzzles

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


def _code(v):
    return int(round(float(v) * 100))


def oracle_pool_from_processed(proc):
    return [{"x_size": p["x_size"], "y_size": p["y_size"], "start": list(p["start_location"]),
             "target": list(p["target_location"]), "solution_count": p["solution_count"],
             "solution_paths": p["solution_paths"], "gaps": p["obs_array"]["gaps"]} for p in proc]


# ----------------------------------------------------------------------------- golden vectors
@pytest.mark.parametrize("pool", golden_io.POOLS)
def test_single_env_matches_reference(on_gpu, pool):
    """SPaRC_Gym (batch of one on the GPU) reproduces the reference's reset/step outputs."""
    from sparc_gym_amd import SPaRC_Gym
    g = golden_io.load(pool)
    env = SPaRC_Gym(puzzles=g["records"], traceback=g["traceback"], max_steps=g["max_steps"])
    for ep in g["episodes"]:
        obs, info = env.reset(options={"puzzle_id": ep["puzzle_id"]})
        assert env.current_puzzle_index == ep["puzzle_index"]
        ref = ep["reset"]
        assert list(obs["base"].keys()) == ref["obs"]["base_keys"]
        for k, plane in ref["obs"]["base"].items():
            assert np.array_equal(obs["base"][k], golden_io.dense(plane)), k
        assert np.array_equal(obs["color"], golden_io.dense(ref["obs"]["color"]))
        assert np.array_equal(obs["additional_info"], golden_io.dense(ref["obs"]["additional_info"]))
        assert info["legal_actions"] == ref["info"]["legal_actions"]
        for a, st in zip(ep["actions"], ep["steps"]):
            obs, r, term, trunc, info = env.step(a)
            assert repr(r) == st["reward"]["repr"] and type(r).__name__ == st["reward"]["type"]
            assert (term, trunc) == (st["terminated"], st["truncated"])
            for k in ("legal_actions", "current_step", "solution_count", "difficulty",
                      "grid_x_size", "grid_y_size"):
                assert info[k] == st["info"][k], k
            assert [int(v) for v in info["agent_location"]] == st["info"]["agent_location"]
            assert repr(info["Rewards"]["normal_reward"]) == st["info"]["normal_reward"]["repr"]
            assert repr(info["Rewards"]["outcome_reward"]) == st["info"]["outcome_reward"]["repr"]
            assert np.array_equal(obs["base"]["visited"], golden_io.dense(st["visited"]))
            assert np.array_equal(obs["base"]["agent_location"], golden_io.dense(st["agent_plane"]))


@pytest.mark.parametrize("pool", golden_io.POOLS)
def test_vec_env_matches_reference(on_gpu, pool):
    """All episodes of a pool as one batch through the step kernel (autoreset='none')."""
    from sparc_gym_amd import SPaRCVecEnv
    g = golden_io.load(pool)
    eps = g["episodes"]
    n, T = len(eps), max(len(e["actions"]) for e in eps)
    vec = SPaRCVecEnv(n, puzzles=g["records"], traceback=g["traceback"], max_steps=g["max_steps"],
                      autoreset="none")
    obs, info = vec.reset(options={"puzzle_index": [e["puzzle_index"] for e in eps]})
    legal0 = info["legal_mask"].cpu().numpy()
    for i, e in enumerate(eps):
        assert [a for a in range(4) if legal0[i] >> a & 1] == e["reset"]["info"]["legal_actions"]
    acts = np.zeros((T, n), np.int64)
    for i, e in enumerate(eps):
        acts[:len(e["actions"]), i] = e["actions"]
    for t in range(T):
        obs, rew, term, trunc, info = vec.step(torch.from_numpy(acts[t]).cuda())
        rew, term, trunc = rew.cpu().numpy(), term.cpu().numpy(), trunc.cpu().numpy()
        legal = info["legal_mask"].cpu().numpy()
        vis, agent = obs["visited"].cpu().numpy(), obs["agent_location"].cpu().numpy()
        for i, e in enumerate(eps):
            if t >= len(e["steps"]):
                continue
            st = e["steps"][t]
            assert rew[i] == st["reward"]["value"], (pool, i, t)   # float64, bit-exact
            assert (bool(term[i]), bool(trunc[i])) == (st["terminated"], st["truncated"])
            assert [a for a in range(4) if legal[i] >> a & 1] == st["info"]["legal_actions"]
            X, Y = st["visited"]["shape"]
            assert np.array_equal(vis[i, :X, :Y], golden_io.dense(st["visited"]))
            assert np.array_equal(agent[i, :X, :Y], golden_io.dense(st["agent_plane"]))
            assert vis[i, X:].sum() == 0 and vis[i, :, Y:].sum() == 0


# ----------------------------------------------------------------------------- vs C oracle
POOLS = {
    "7x7_full": dict(sizes=((3, 3),), full_properties=True),
    "7x7_base": dict(sizes=((3, 3),), full_properties=False),
    "mixed_5_11": dict(sizes=((2, 2), (3, 3), (4, 4), (5, 5), (2, 5), (5, 3)), full_properties=True),
    "15x15": dict(sizes=((7, 7), (6, 7)), full_properties=True),
}


def _make(name, n_puzzles=64, seed=0):
    recs = synthetic.make_puzzles(n_puzzles, seed=seed, **POOLS[name])
    proc = process_puzzles(recs)
    return proc, pack_table(proc)


def _run_three_ways(proc, table, n, T, tb, max_steps, autoreset, seed):
    """rollout kernel (one launch) vs T step kernels vs the C oracle, same inputs."""
    from sparc_gym_amd import SPaRCVecEnv
    rng = np.random.default_rng(seed)
    pids = rng.integers(len(proc), size=n)
    acts = rng.choice(np.array([0, 1, 2, 3, 0, 1, 2, 3, 4, 255], np.uint8), size=(T, n))
    kw = dict(processed=proc, table=table, traceback=tb, max_steps=max_steps, autoreset=autoreset,
              observation="compact")
    a = SPaRCVecEnv(n, **kw)
    a.reset(options={"puzzle_index": pids})
    stats = torch.zeros((n, 4), dtype=torch.int32, device="cuda")
    out = a.rollout(T, torch.from_numpy(acts).cuda(), stats=stats)
    ra, fa = out["reward_code"].cpu().numpy(), out["flags"].cpu().numpy()
    sa = a.state()

    b = SPaRCVecEnv(n, **kw)
    b.reset(options={"puzzle_index": pids})
    rb, fb = np.zeros((T, n), np.int8), np.zeros((T, n), np.uint8)
    for t in range(T):
        _, _, _, _, info = b.step(torch.from_numpy(acts[t]).cuda())
        rb[t] = info["reward_code"].cpu().numpy()
        fb[t] = b._flags.cpu().numpy()
    sb = b.state()

    o = COracle(oracle_pool_from_processed(proc), n, tb, max_steps, autoreset={"none": 0, "next_step": 1}[autoreset])
    o.reset(pids)
    ostats = np.zeros((n, 4), np.int32)
    ro, fo = o.rollout(T, acts, stats=ostats)
    so = o.state()
    return (ra, fa, sa, stats.cpu().numpy()), (rb, fb, sb), (ro, fo, so, ostats), table


def _assert_states_equal(s_gpu, s_or, table):
    assert np.array_equal(s_gpu["x"], s_or["x"]) and np.array_equal(s_gpu["y"], s_or["y"])
    assert np.array_equal(s_gpu["step"], s_or["step"])
    assert np.array_equal(s_gpu["path_len"], s_or["path_len"])
    assert np.array_equal(s_gpu["puzzle"], s_or["pid"])
    assert np.array_equal(s_gpu["outcome"], s_or["outcome"])
    from sparc_gym_amd.core import visited_planes
    planes = visited_planes(s_gpu["visited"], table, 16, 16)
    assert np.array_equal(planes, s_or["visited"].astype(np.int32))


@pytest.mark.parametrize("name", list(POOLS))
@pytest.mark.parametrize("tb", [False, True])
@pytest.mark.parametrize("autoreset", ["next_step", "none"])
def test_rollout_step_oracle_agree(on_gpu, name, tb, autoreset):
    proc, table = _make(name, seed=len(name))
    max_steps = 2000 if autoreset == "next_step" else 150
    (ra, fa, sa, st_a), (rb, fb, sb), (ro, fo, so, st_o), table = _run_three_ways(
        proc, table, 2048, 257, tb, max_steps, autoreset, seed=zlib.crc32(f"{name}{tb}".encode()))
    assert np.array_equal(ra, ro) and np.array_equal(fa, fo)
    assert np.array_equal(rb, ro) and np.array_equal(fb, fo)
    assert np.array_equal(st_a, st_o)
    _assert_states_equal(sa, so, table)
    _assert_states_equal(sb, so, table)


def test_random_action_rollout_matches_oracle(on_gpu):
    """Device counter-based actions == oracle's restatement of the same hash."""
    from sparc_gym_amd import SPaRCVecEnv
    proc, table = _make("7x7_full", seed=5)
    n, T = 4096, 300
    pids = np.arange(n) % len(proc)
    v = SPaRCVecEnv(n, processed=proc, table=table, traceback=True, observation="compact", env_offset=12345)
    v.reset(options={"puzzle_index": pids})
    out = v.rollout(T, None, seed=99, t0=7)
    o = COracle(oracle_pool_from_processed(proc), n, True, 2000, autoreset=1)
    o.reset(pids)
    ro, fo = o.rollout(T, None, seed=99, env_offset=12345, t0=7)
    assert np.array_equal(out["reward_code"].cpu().numpy(), ro)
    assert np.array_equal(out["flags"].cpu().numpy(), fo)


def test_chunked_rollouts_equal_one_launch(on_gpu):
    """State round-trips HBM between launches bit-exactly (T=100 + 57 + 1 == T=158)."""
    from sparc_gym_amd import SPaRCVecEnv
    proc, table = _make("mixed_5_11", seed=2)
    n = 3000
    pids = np.arange(n) % len(proc)
    acts = torch.randint(0, 4, (158, n), dtype=torch.uint8, device="cuda")
    kw = dict(processed=proc, table=table, traceback=True, observation="compact")
    a = SPaRCVecEnv(n, **kw)
    a.reset(options={"puzzle_index": pids})
    full = a.rollout(158, acts)
    b = SPaRCVecEnv(n, **kw)
    b.reset(options={"puzzle_index": pids})
    parts = [b.rollout(100, acts[:100].contiguous()), b.rollout(57, acts[100:157].contiguous()),
             b.rollout(1, acts[157:].contiguous())]
    for key in ("reward_code", "flags"):
        assert torch.equal(full[key], torch.cat([p[key] for p in parts]))


# ----------------------------------------------------------------------------- full size
def test_full_size_65536_bit_exact_and_invariants(on_gpu):
    """BASELINE config C3 shape: 65,536 envs, 7x7 full property set, traceback=True."""
    from sparc_gym_amd import SPaRCVecEnv
    proc, table = _make("7x7_full", n_puzzles=1024, seed=0)
    n, T = 65536, 400
    pids = (np.arange(n, dtype=np.uint64) * 2654435761 % 1024).astype(np.int64)
    v = SPaRCVecEnv(n, processed=proc, table=table, traceback=True, observation="compact")
    v.reset(options={"puzzle_index": pids})
    stats = torch.zeros((n, 4), dtype=torch.int32, device="cuda")
    out = v.rollout(T, None, seed=2024, stats=stats)
    r, f = out["reward_code"].cpu().numpy(), out["flags"].cpu().numpy()
    s = v.state()
    # size-independent properties
    assert set(np.unique(r)) <= {-100, -1, 0, 1, 100}
    assert not np.any((f & 3) == 3)                     # terminated and truncated exclusive
    st = stats.cpu().numpy()
    assert np.array_equal(st[:, 0], r.astype(np.int64).sum(0))
    assert np.array_equal(st[:, 1], ((f & 3) != 0).sum(0))
    done_prev = np.vstack([np.zeros((1, n), bool), (f[:-1] & 3) != 0])
    assert np.array_equal((f & 64) != 0, done_prev)     # next-step autoreset exactly after done
    assert np.all(r[(f & 64) != 0] == 0)
    pop = np.zeros(n, np.int64)
    for w in range(table.words):
        pop += np.array([bin(int(b)).count("1") for b in s["visited"][w]])
    assert np.array_equal(pop, s["path_len"].astype(np.int64))   # visited == path nodes
    # and bit-exact against the C oracle at full size
    o = COracle(oracle_pool_from_processed(proc), n, True, 2000, autoreset=1)
    o.reset(pids)
    ro, fo = o.rollout(T, None, seed=2024)
    assert np.array_equal(r, ro) and np.array_equal(f, fo)


def test_obs_pack_matches_state(on_gpu):
    from sparc_gym_amd import SPaRCVecEnv
    from sparc_gym_amd.core import visited_planes
    proc, table = _make("mixed_5_11", seed=8)
    n = 1000
    v = SPaRCVecEnv(n, processed=proc, table=table, traceback=True)
    v.reset(seed=3)
    v.rollout(37, None, seed=1)
    obs, *_ = v.step(torch.randint(0, 4, (n,), device="cuda"))
    s = v.state()
    vis = obs["visited"].cpu().numpy()
    assert np.array_equal(vis, visited_planes(s["visited"], table))
    ag = obs["agent_location"].cpu().numpy()
    assert np.array_equal(ag.reshape(n, -1).sum(1), np.ones(n))
    assert np.all(ag[np.arange(n), s["x"], s["y"]] == 1)
    pidx = obs["puzzle_index"].cpu().numpy()
    assert np.array_equal(pidx, s["puzzle"].astype(np.int32))


def test_device_reset_rejects_bad_index(on_gpu):
    from sparc_gym_amd import SPaRCVecEnv
    proc, table = _make("7x7_base", seed=1)
    v = SPaRCVecEnv(64, processed=proc, table=table, observation="compact")
    with pytest.raises(ValueError):
        v.reset(options={"puzzle_index": np.full(64, len(proc))})
    q = torch.full((64,), len(proc) + 5, dtype=torch.int32, device="cuda")
    v.reset(options={"puzzle_index": np.zeros(64, np.int64)})
    v.core.reset_device(q.data_ptr())
    with pytest.raises(ValueError):
        v.core.sync()


@pytest.mark.parametrize("n", [2560, 2624, 3000])
def test_w1_chunked_partial_workgroups(on_gpu, n):
    """W = 1 rollouts: n = 2560 (a multiple of 256) runs the full tiles through the split move /
    trie kernel k_rollout1s and the T % 16 tail through k_rollout1; n = 2624 (n % 16 == 0,
    tiled) runs k_rollout1's full workgroups through the I/O wave next to a partial last
    workgroup; n = 3000 runs every workgroup on the direct path (untiled).  Launches of
    100 + 57 + 1 + 32 steps (tails, single steps, exact tiles) equal one launch of 190 steps,
    reward codes, flags and per-env stats alike, and equal the oracle."""
    from sparc_gym_amd import SPaRCVecEnv
    proc, table = _make("7x7_full", seed=9)
    assert table.words == 1
    pids = (np.arange(n) * 7) % len(proc)
    acts = torch.randint(0, 5, (190, n), dtype=torch.uint8, device="cuda")
    kw = dict(processed=proc, table=table, traceback=True, observation="compact", max_steps=60)
    a = SPaRCVecEnv(n, **kw)
    a.reset(options={"puzzle_index": pids})
    sa = torch.zeros((n, 4), dtype=torch.int32, device="cuda")
    full = a.rollout(190, acts, stats=sa)
    b = SPaRCVecEnv(n, **kw)
    b.reset(options={"puzzle_index": pids})
    sb = torch.zeros((n, 4), dtype=torch.int32, device="cuda")
    parts, t = [], 0
    for T in (100, 57, 1, 32):
        parts.append(b.rollout(T, acts[t:t + T].contiguous(), stats=sb))
        t += T
    for key in ("reward_code", "flags"):
        assert torch.equal(full[key], torch.cat([p[key] for p in parts]))
    assert torch.equal(sa, sb)
    o = COracle(oracle_pool_from_processed(proc), n, True, 60, autoreset=1)
    o.reset(pids)
    ost = np.zeros((n, 4), np.int32)
    ro, fo = o.rollout(190, acts.cpu().numpy(), stats=ost)
    assert np.array_equal(full["reward_code"].cpu().numpy(), ro)
    assert np.array_equal(full["flags"].cpu().numpy(), fo)
    assert np.array_equal(sa.cpu().numpy(), ost)
    _assert_states_equal(b.state(), o.state(), table)


@pytest.mark.parametrize("name", ["mixed_5_11", "15x15"])
@pytest.mark.parametrize("tb", [False, True])
@pytest.mark.parametrize("max_steps", [12, 2000])
def test_multiword_split_chunked_vs_oracle(on_gpu, name, tb, max_steps):
    """W = 2 / 4 rollouts at n = 2560 (whole 256-env workgroups): the full tiles run through the
    multi-word split kernel k_rolloutWs (free board in LDS, TrieLane trie wave), the T % 16
    tails through the generic k_rollout.  Launches of 100 + 57 + 1 + 32 steps equal one launch
    of 190 (reward codes, flags, stats) and the oracle, also with many autoresets per launch
    (max_steps 12) and illegal actions."""
    from sparc_gym_amd import SPaRCVecEnv
    proc, table = _make(name, seed=31 + max_steps)
    assert table.words > 1
    n = 2560
    pids = (np.arange(n) * 7) % len(proc)
    rng = np.random.default_rng(max_steps + 17 * tb)
    acts_np = rng.choice(np.array([0, 1, 2, 3, 0, 1, 2, 3, 4, 255], np.uint8), size=(190, n))
    acts = torch.from_numpy(acts_np).cuda()
    kw = dict(processed=proc, table=table, traceback=tb, observation="compact", max_steps=max_steps)
    a = SPaRCVecEnv(n, **kw)
    a.reset(options={"puzzle_index": pids})
    sa = torch.zeros((n, 4), dtype=torch.int32, device="cuda")
    full = a.rollout(190, acts, stats=sa)
    b = SPaRCVecEnv(n, **kw)
    b.reset(options={"puzzle_index": pids})
    sb = torch.zeros((n, 4), dtype=torch.int32, device="cuda")
    parts, t = [], 0
    for T in (100, 57, 1, 32):
        parts.append(b.rollout(T, acts[t:t + T].contiguous(), stats=sb))
        t += T
    for key in ("reward_code", "flags"):
        assert torch.equal(full[key], torch.cat([p[key] for p in parts]))
    assert torch.equal(sa, sb)
    o = COracle(oracle_pool_from_processed(proc), n, tb, max_steps, autoreset=1)
    o.reset(pids)
    ost = np.zeros((n, 4), np.int32)
    ro, fo = o.rollout(190, acts_np, stats=ost)
    assert np.array_equal(full["reward_code"].cpu().numpy(), ro)
    assert np.array_equal(full["flags"].cpu().numpy(), fo)
    assert np.array_equal(sa.cpu().numpy(), ost)
    _assert_states_equal(a.state(), o.state(), table)
    _assert_states_equal(b.state(), o.state(), table)
    if max_steps == 12:
        assert ost[:, 3].sum() > n       # autoresets inside the launches


def test_multiword_full_size_15x15_vs_oracle(on_gpu):
    """The second reading of '7x7' (SPaRC_Gym.py:243-248): a 7x7 cell grid = 15x15 lattice on
    4-word boards, 65,536 envs, traceback, full property set (bench config c3g7): bit-exact
    against the C oracle and the size-independent invariants."""
    from sparc_gym_amd import SPaRCVecEnv
    recs = synthetic.make_puzzles(1024, seed=0, sizes=((7, 7),), full_properties=True)
    proc = process_puzzles(recs)
    table = pack_table(proc)
    assert table.words == 4
    n, T = 65536, 208
    pids = (np.arange(n, dtype=np.uint64) * 2654435761 % 1024).astype(np.int64)
    v = SPaRCVecEnv(n, processed=proc, table=table, traceback=True, observation="compact")
    v.reset(options={"puzzle_index": pids})
    stats = torch.zeros((n, 4), dtype=torch.int32, device="cuda")
    out = v.rollout(T, None, seed=77, stats=stats)
    r, f = out["reward_code"].cpu().numpy(), out["flags"].cpu().numpy()
    st = stats.cpu().numpy()
    assert np.array_equal(st[:, 0], r.astype(np.int64).sum(0))
    assert np.array_equal(st[:, 1], ((f & 3) != 0).sum(0))
    s = v.state()
    pop = np.zeros(n, np.int64)
    for w in range(table.words):
        pop += np.array([bin(int(b)).count("1") for b in s["visited"][w]])
    assert np.array_equal(pop, s["path_len"].astype(np.int64))
    o = COracle(oracle_pool_from_processed(proc), n, True, 2000, autoreset=1)
    o.reset(pids)
    ost = np.zeros((n, 4), np.int32)
    ro, fo = o.rollout(T, None, seed=77, stats=ost)
    assert np.array_equal(r, ro) and np.array_equal(f, fo)
    assert np.array_equal(st, ost)


def test_w1_rollout_without_outputs_keeps_state_and_stats(on_gpu):
    """record=False (no reward / flag tensors) and in-kernel random actions: same state and
    stats as the recorded run."""
    from sparc_gym_amd import SPaRCVecEnv
    proc, table = _make("7x7_full", seed=10)
    n = 4096
    pids = np.arange(n) % len(proc)
    kw = dict(processed=proc, table=table, traceback=True, observation="compact")
    runs = []
    for record in (True, False):
        v = SPaRCVecEnv(n, **kw)
        v.reset(options={"puzzle_index": pids})
        st = torch.zeros((n, 4), dtype=torch.int32, device="cuda")
        v.rollout(96, None, seed=3, stats=st, record=record)
        runs.append((st.cpu().numpy(), v.state()))
    assert np.array_equal(runs[0][0], runs[1][0])
    for k in ("x", "y", "step", "path_len", "puzzle", "outcome", "pending"):
        assert np.array_equal(runs[0][1][k], runs[1][1][k]), k
    assert np.array_equal(runs[0][1]["visited"], runs[1][1]["visited"])


@pytest.mark.parametrize("max_steps,sizes", [(3, ((3, 3),)), (9, ((3, 3),)), (25, ((3, 3),)),
                                             (9, ((7, 7),)), (25, ((4, 4), (5, 5)))])
def test_many_short_episodes_vs_oracle(on_gpu, max_steps, sizes):
    """Thousands of autoresets per launch (short max_steps, puzzles with many solutions sharing
    prefixes, mostly-legal actions): every done step's reward and the step after it are where
    the pipelined rollout hands the trie state over to the reset, so compare them all."""
    from sparc_gym_amd import SPaRCVecEnv
    recs = synthetic.make_puzzles(256, seed=max_steps, sizes=sizes, n_solutions=8,
                                  shared_prefix_prob=0.9, full_properties=False)
    proc = process_puzzles(recs)
    table = pack_table(proc)
    n, T = 16384, 240
    rng = np.random.default_rng(max_steps)
    pids = rng.integers(len(proc), size=n)
    acts = rng.integers(0, 4, size=(T, n)).astype(np.uint8)
    v = SPaRCVecEnv(n, processed=proc, table=table, traceback=True, max_steps=max_steps, observation="compact")
    v.reset(options={"puzzle_index": pids})
    st = torch.zeros((n, 4), dtype=torch.int32, device="cuda")
    out = v.rollout(T, torch.from_numpy(acts).cuda(), stats=st)
    o = COracle(oracle_pool_from_processed(proc), n, True, max_steps, autoreset=1)
    o.reset(pids)
    ost = np.zeros((n, 4), np.int32)
    ro, fo = o.rollout(T, acts, stats=ost)
    r = out["reward_code"].cpu().numpy()
    assert np.array_equal(r, ro) and np.array_equal(out["flags"].cpu().numpy(), fo)
    assert np.array_equal(st.cpu().numpy(), ost)
    assert (r == 100).sum() > 100        # the case needs solved episodes, and many of them


# ----------------------------------------------------------------------------- 'new' obs traces
@pytest.mark.parametrize("name", ["7x7_full", "mixed_5_11", "15x15"])
@pytest.mark.parametrize("tb", [False, True])
@pytest.mark.parametrize("n", [1001, 2048])
def test_rollout_obs_and_step_obs_match_oracle(on_gpu, name, tb, n):
    """rollout(obs=True) records the visited / agent_location planes after every step
    (k_rollout OBS, cooperative 16-B stores); step() returns the same planes from k_step_obs.
    Both bit-exact vs the oracle's planes, with autoresets inside the launch (max_steps 25)
    and n = 1001 (partial last wave; n * x_dim * y_dim odd for 7x7 / 15x15, so odd steps take
    the unaligned store path)."""
    from sparc_gym_amd import SPaRCVecEnv
    proc, table = _make(name, seed=11 + len(name))
    T, ms = 48, 25
    rng = np.random.default_rng(n + tb)
    pids = rng.integers(len(proc), size=n)
    acts = rng.choice(np.array([0, 1, 2, 3, 0, 1, 2, 3, 9], np.uint8), size=(T, n))
    kw = dict(processed=proc, table=table, traceback=tb, max_steps=ms, observation="new")
    a = SPaRCVecEnv(n, **kw)
    a.reset(options={"puzzle_index": pids})
    out = a.rollout(T, torch.from_numpy(acts).cuda(), obs=True)
    X, Y = a.x_dim, a.y_dim
    o = COracle(oracle_pool_from_processed(proc), n, tb, ms, autoreset=1)
    o.reset(pids)
    ro, fo, vo, ao = o.rollout_obs(T, X, Y, acts)
    assert np.array_equal(out["reward_code"].cpu().numpy(), ro)
    assert np.array_equal(out["flags"].cpu().numpy(), fo)
    assert np.any(fo & 64)                                       # autoresets happened
    assert np.array_equal(out["visited"].cpu().numpy(), vo)
    assert np.array_equal(out["agent_location"].cpu().numpy(), ao)
    b = SPaRCVecEnv(n, **kw)
    b.reset(options={"puzzle_index": pids})
    b_t = 0                                                      # steps b has taken
    for t in range(0, T, 7 if n > 1500 else 1):
        if t > b_t:
            b.rollout(t - b_t, torch.from_numpy(acts[b_t:t]).cuda().contiguous())
        obs, rew, term, trunc, info = b.step(torch.from_numpy(acts[t]).cuda())
        b_t = t + 1
        assert np.array_equal(info["reward_code"].cpu().numpy(), ro[t])
        assert np.array_equal(obs["visited"].cpu().numpy(), vo[t]), t
        assert np.array_equal(obs["agent_location"].cpu().numpy(), ao[t]), t
        xy = obs["agent_xy"].cpu().numpy()
        assert np.all(ao[t][np.arange(n), xy[:, 0], xy[:, 1]] == 1)


def test_rollout_obs_only_one_plane_and_chunks(on_gpu):
    """Either trace may be omitted; chunked obs rollouts equal one launch."""
    from sparc_gym_amd import SPaRCVecEnv
    proc, table = _make("mixed_5_11", seed=4)
    n, T = 4096, 40
    acts = torch.randint(0, 4, (T, n), dtype=torch.uint8, device="cuda")
    kw = dict(processed=proc, table=table, traceback=True, observation="new")
    a = SPaRCVecEnv(n, **kw)
    a.reset(seed=1)
    full = a.rollout(T, acts, obs=True)
    b = SPaRCVecEnv(n, **kw)
    b.reset(seed=1)
    X, Y = b.x_dim, b.y_dim
    vis1 = torch.full((16, n, X, Y), -7, dtype=torch.int32, device="cuda")
    p1 = b.rollout(16, acts[:16].contiguous(), obs_out=(vis1, None))
    p2 = b.rollout(T - 16, acts[16:].contiguous(), obs=True)
    assert p1["agent_location"] is None
    assert torch.equal(full["visited"][:16], vis1)
    assert torch.equal(full["visited"][16:], p2["visited"])
    assert torch.equal(full["agent_location"][16:], p2["agent_location"])
    assert torch.equal(full["flags"], torch.cat([p1["flags"], p2["flags"]]))


def test_obs_entry_points_validate_plane_dims(on_gpu):
    """x_dim * y_dim > 256 (the plane writer's cell LUT) and x_dim < 1 are rejected with
    ValueError before any launch; a valid call still works afterwards."""
    from sparc_gym_amd import SPaRCVecEnv
    proc, table = _make("7x7_full", seed=12)
    n = 128
    v = SPaRCVecEnv(n, processed=proc, table=table, observation="compact")
    v.reset(seed=0)
    a = torch.zeros(n, dtype=torch.uint8, device="cuda")
    r = torch.empty(n, dtype=torch.int8, device="cuda")
    f = torch.empty(n, dtype=torch.uint8, device="cuda")
    planes = torch.empty(n * 17 * 17, dtype=torch.int32, device="cuda")
    for xd, yd in ((17, 17), (0, 7)):
        with pytest.raises(ValueError):
            v.core.step_obs_device(a.data_ptr(), r.data_ptr(), f.data_ptr(), planes.data_ptr(), None, xd, yd)
        with pytest.raises(ValueError):
            v.core.rollout_obs_device(1, a.data_ptr(), r.data_ptr(), f.data_ptr(), None, planes.data_ptr(), None, xd, yd)
    v.core.step_obs_device(a.data_ptr(), r.data_ptr(), f.data_ptr(), planes.data_ptr(), None, 7, 7)
    torch.cuda.synchronize()
    vis = planes[:n * 49].view(n, 7, 7).cpu().numpy()
    assert vis.reshape(n, -1).sum(1).min() >= 1          # the start (and any move) is visited


def test_step_gym_action_types_and_outputs(on_gpu):
    """SPaRCVecEnv.step's one-launch gym outputs (sparc_step_gym_device): int64, int32 and uint8
    actions with out-of-range values give identical steps (< 0 or >= 4 is illegal for the
    integer types, >= 4 for uint8); reward == reward_code / 100 in float64, terminated /
    truncated / legal_mask / autoreset equal the flag bits; agent_xy equals the reset path's
    (x, y); compact and 'new' observations agree.  Also checks the ABI's argument validation."""
    from sparc_gym_amd import SPaRCVecEnv
    proc, table = _make("7x7_full", seed=21)
    n, T = 1000, 60
    rng = np.random.default_rng(5)
    acts = rng.integers(-3, 7, size=(T, n)).astype(np.int64)
    envs = {k: SPaRCVecEnv(n, processed=proc, table=table, traceback=True, max_steps=25,
                           observation="new" if k != "compact" else "compact")
            for k in ("i64", "i32", "u8", "compact")}
    for v in envs.values():
        v.reset(seed=3)
    for t in range(T):
        a64 = torch.from_numpy(acts[t]).cuda()
        outs = {"i64": envs["i64"].step(a64), "i32": envs["i32"].step(a64.to(torch.int32)),
                "u8": envs["u8"].step(torch.where((a64 >= 0) & (a64 < 4), a64, 255).to(torch.uint8)),
                "compact": envs["compact"].step(acts[t])}                      # numpy int64
        ref_obs, ref_r, ref_te, ref_tr, ref_info = outs["i64"]
        code = ref_info["reward_code"].to(torch.float64) / 100.0
        assert torch.equal(ref_r, code)
        assert ref_r.dtype == torch.float64 and ref_te.dtype == torch.bool and ref_tr.dtype == torch.bool
        for k, (obs, r, te, tr, info) in outs.items():
            assert torch.equal(r, ref_r) and torch.equal(te, ref_te) and torch.equal(tr, ref_tr), (k, t)
            assert torch.equal(info["legal_mask"], ref_info["legal_mask"]), (k, t)
            assert torch.equal(info["autoreset"], ref_info["autoreset"]), (k, t)
            assert torch.equal(obs["puzzle_index"], ref_obs["puzzle_index"]), (k, t)
            loc = obs["agent_location"] if k == "compact" else obs["agent_xy"]
            assert torch.equal(loc, ref_obs["agent_xy"]), (k, t)
            if k != "compact":
                assert torch.equal(obs["visited"], ref_obs["visited"]), (k, t)
        f = envs["i64"]._flags
        assert torch.equal(ref_te, (f & 1).bool()) and torch.equal(ref_tr, (f & 2).bool())
        assert torch.equal(ref_info["legal_mask"], (f >> 2) & 0xF)
        assert torch.equal(ref_info["autoreset"], (f & 64).bool())
    # the step path's (x, y) equals the observation-pack path's (reset's _obs)
    v = envs["compact"]
    step_xy = v._loc.clone()
    assert torch.equal(v._obs()["agent_location"], step_xy)
    with pytest.raises(ValueError):
        v.step(torch.zeros(n, dtype=torch.float32))
    with pytest.raises(ValueError):
        v.core.step_gym_device(torch.zeros(n, dtype=torch.int16, device="cuda").data_ptr(), 2)


@pytest.mark.parametrize("name,tb,n", [("mixed_5_11", True, 4096), ("7x7_full", False, 1001), ("15x15", True, 300)])
def test_rollout_obs_writer_waves_equal_inline(on_gpu, name, tb, n):
    """rollout(obs=True) runs k_rollout_obsw (compute waves stage the boards, four writer waves
    per 256 envs stream the planes: bit streams on the multi-word pools, the LUT on 7x7); the
    per-wave kernel that writes its own planes
    (sparc_set_variant SPARC_VARIANT_OBS_INLINE) gives identical planes, codes, flags, stats and
    state, with file actions and with the in-kernel random actions, over two launches."""
    from sparc_gym_amd import SPaRCVecEnv
    proc, table = _make(name, seed=23 + n)
    rng = np.random.default_rng(n)
    pids = rng.integers(len(proc), size=n)
    acts = torch.from_numpy(rng.integers(0, 5, size=(40, n)).astype(np.uint8)).cuda()
    runs = []
    for inline in (False, True):
        v = SPaRCVecEnv(n, processed=proc, table=table, traceback=tb, max_steps=30, observation="new")
        if inline:
            v.core.set_variant(v.core.VARIANT_OBS_INLINE, 1)
        v.reset(options={"puzzle_index": pids})
        st = torch.zeros((n, 4), dtype=torch.int32, device="cuda")
        r1 = v.rollout(24, acts[:24].contiguous(), obs=True, stats=st)
        r2 = v.rollout(16, None, seed=5, t0=24, obs=True, stats=st)
        runs.append(([r[k].cpu().numpy() for r in (r1, r2) for k in ("reward_code", "flags", "visited",
                                                                        "agent_location")],
                     st.cpu().numpy(), v.state()))
    (a, sa, xa), (b, sb, xb) = runs
    for u, w in zip(a, b):
        assert np.array_equal(u, w)
    assert np.array_equal(sa, sb)
    for k in ("x", "y", "step", "path_len", "puzzle", "outcome", "visited"):
        assert np.array_equal(np.asarray(xa[k]), np.asarray(xb[k])), k


@pytest.mark.parametrize("pad", [0, 2])
def test_rollout_obs_writer_waves_padded_x_dim(on_gpu, pad):
    """the bit-stream staging holds 64 envs x 64 W bits, so a multi-word pool
    whose planes are padded past its largest lattice (x_dim > x_max: 13 x 11 = 143 cells > 128
    board bits at W = 2) must take the LUT staging.  The writer-wave planes equal the inline
    kernel's and, inside the lattice, the unpadded planes; the padding rows are zero."""
    from sparc_gym_amd import SPaRCVecEnv
    proc, table = _make("mixed_5_11", seed=41)
    assert table.words == 2
    n, T = 1280, 40
    rng = np.random.default_rng(7)
    pids = rng.integers(len(proc), size=n)
    acts = torch.from_numpy(rng.integers(0, 5, size=(T, n)).astype(np.uint8)).cuda()
    runs = []
    for x_pad, inline in ((0, False), (pad, False), (pad, True)):
        v = SPaRCVecEnv(n, processed=proc, table=table, traceback=True, max_steps=30, observation="new")
        v.x_dim = table.x_max + x_pad
        if inline:
            v.core.set_variant(v.core.VARIANT_OBS_INLINE, 1)
        v.reset(options={"puzzle_index": pids})
        r = v.rollout(T, acts, obs=True)
        runs.append({k: r[k].cpu().numpy() for k in ("reward_code", "flags", "visited", "agent_location")})
    base, stream, inl = runs
    for k in base:
        assert np.array_equal(stream[k], inl[k]), k
    X = table.x_max
    for k in ("visited", "agent_location"):
        assert np.array_equal(stream[k][:, :, :X], base[k]), k
        assert not stream[k][:, :, X:].any(), k
    for k in ("reward_code", "flags"):
        assert np.array_equal(stream[k], base[k]), k
