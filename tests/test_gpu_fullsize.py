"""GPU parity at BASELINE.json's full sizes (configs c2, c3, c4).

* c2: exactly 4,096 envs, 7x7 base planes, traceback off, 2,000 steps in one launch, bit-exact
  against the C oracle over every env (reward codes, flags, state, stats).
* c3: 65,536 envs, 7x7 full property set, traceback on, max_steps = 37 so that truncation by
  step count (SPaRC_Gym.py:1134) happens at full size, bit-exact against the oracle.
* c4: 262,144 envs, mixed 5x5-11x11 lattices padded to 11x11, 'new' planes after every step
  (the [T][N][11][11] int32 traces, 2 x 127 MB per step), autoresets inside the launch.  The
  oracle replays ~2,000 sampled env columns (their puzzles and action columns; the envs are
  independent) and every output of those columns must match; every env is checked with
  size-independent invariants on the GPU: the agent plane is one-hot and inside the visited
  plane, nothing lies outside the env's own lattice, the visited count moves by one per
  moving step and restarts at 1 on a reset step, and at the end it equals path_len.
* c4c: the same 262,144-env mixed pool without planes, through the multi-word split kernel
  (k_rolloutWs), 256 steps with autoresets: sampled oracle columns (reward codes, flags, final
  state, stats) and, for every env, the stats against the output traces.
* c4 and c4c at the bench's exact launch shape, EVERY env against the C
  oracle run in column shards on threads: c4 through the bench's own call
  (sparc_rollout_obs_device -> k_rollout_obsw, 262,144 envs x 50 steps, max_steps 2,000, the
  bench's action tiles), two back-to-back launches into the same [50][262,144][11][11] int32
  traces (6.3 GB per plane, past 4 GiB: the size_t addressing of the writer waves), reward codes,
  flags, stats, final state and every env's visited / agent_location planes at every step
  (bit-packed losslessly on both sides after checking that every entry is 0 or 1); c4c through
  sparc_rollout_device (k_rolloutWs, 262,144 envs x 2,000 steps, two launches).
"""
import numpy as np
import pytest

from oracle import COracle
from sparc_gym_amd import synthetic
from sparc_gym_amd.puzzles import pack_table, process_puzzles

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


def _oracle_pool(proc):
    return [{"x_size": p["x_size"], "y_size": p["y_size"], "start": list(p["start_location"]),
             "target": list(p["target_location"]), "solution_count": p["solution_count"],
             "solution_paths": p["solution_paths"], "gaps": p["obs_array"]["gaps"]} for p in proc]


def _bench_pool(sizes, full):
    proc = process_puzzles(synthetic.make_puzzles(1024, seed=0, sizes=sizes, full_properties=full))
    return proc, pack_table(proc)


def _bench_pids(n):
    return (np.arange(n, dtype=np.uint64) * 2654435761 % 1024).astype(np.int64)


def _state_equal(s, so, table):
    from sparc_gym_amd.core import visited_planes
    for k, ko in (("x", "x"), ("y", "y"), ("step", "step"), ("path_len", "path_len"), ("puzzle", "pid"),
                  ("outcome", "outcome")):
        assert np.array_equal(s[k], so[ko]), k
    assert np.array_equal(visited_planes(s["visited"], table, 16, 16), so["visited"].astype(np.int32))


def test_c2_4096_envs_2000_steps_bit_exact(on_gpu):
    from sparc_gym_amd import SPaRCVecEnv
    proc, table = _bench_pool(((3, 3),), False)
    n, T = 4096, 2000
    pids = _bench_pids(n)
    g = torch.Generator(device="cuda")
    g.manual_seed(42)
    acts = torch.randint(0, 4, (T, n), dtype=torch.uint8, device="cuda", generator=g)
    v = SPaRCVecEnv(n, processed=proc, table=table, traceback=False, observation="compact")
    v.reset(options={"puzzle_index": pids})
    st = torch.zeros((n, 4), dtype=torch.int32, device="cuda")
    out = v.rollout(T, acts, stats=st)
    o = COracle(_oracle_pool(proc), n, False, 2000, autoreset=1)
    o.reset(pids)
    ost = np.zeros((n, 4), np.int32)
    ro, fo = o.rollout(T, acts.cpu().numpy(), stats=ost)
    assert np.array_equal(out["reward_code"].cpu().numpy(), ro)
    assert np.array_equal(out["flags"].cpu().numpy(), fo)
    assert np.array_equal(st.cpu().numpy(), ost)
    _state_equal(v.state(), o.state(), table)
    # and the in-kernel random actions at the same size
    v.reset(options={"puzzle_index": pids})
    out = v.rollout(T, None, seed=9)
    o.reset(pids)
    ro, fo = o.rollout(T, None, seed=9)
    assert np.array_equal(out["reward_code"].cpu().numpy(), ro)
    assert np.array_equal(out["flags"].cpu().numpy(), fo)


def test_c3_65536_envs_step_count_truncation(on_gpu):
    from sparc_gym_amd import SPaRCVecEnv
    proc, table = _bench_pool(((3, 3),), True)
    n, T, ms = 65536, 400, 37
    pids = _bench_pids(n)
    v = SPaRCVecEnv(n, processed=proc, table=table, traceback=True, max_steps=ms, observation="compact")
    v.reset(options={"puzzle_index": pids})
    st = torch.zeros((n, 4), dtype=torch.int32, device="cuda")
    out = v.rollout(T, None, seed=77, stats=st)
    r, f = out["reward_code"].cpu().numpy(), out["flags"].cpu().numpy()
    o = COracle(_oracle_pool(proc), n, True, ms, autoreset=1)
    o.reset(pids)
    ost = np.zeros((n, 4), np.int32)
    ro, fo = o.rollout(T, None, seed=77, stats=ost)
    assert np.array_equal(r, ro) and np.array_equal(f, fo)
    assert np.array_equal(st.cpu().numpy(), ost)
    _state_equal(v.state(), o.state(), table)
    # truncation by step count did happen: a truncated step whose legal mask is not empty
    trunc_steps = ((f & 2) != 0) & (((f >> 2) & 15) != 0)
    assert trunc_steps.sum() > 1000


def test_c4_262144_envs_new_planes_sampled_oracle_and_invariants(on_gpu):
    from sparc_gym_amd import SPaRCVecEnv
    proc, table = _bench_pool(((2, 2), (3, 3), (4, 4), (5, 5)), True)
    n, T, ms = 262144, 12, 7                      # max_steps 7: autoresets inside the launch
    pids = _bench_pids(n)
    v = SPaRCVecEnv(n, processed=proc, table=table, traceback=True, max_steps=ms, observation="new")
    v.reset(options={"puzzle_index": pids})
    X, Y = v.x_dim, v.y_dim
    assert (X, Y) == (11, 11) and table.words == 2
    g = torch.Generator(device="cuda")
    g.manual_seed(7)
    acts = torch.randint(0, 4, (T, n), dtype=torch.uint8, device="cuda", generator=g)
    out = v.rollout(T, acts, obs=True)
    vis, ag = out["visited"], out["agent_location"]
    f = out["flags"]
    # --- sampled oracle columns (including the last envs: large-offset indexing)
    rng = np.random.default_rng(0)
    idx = np.unique(np.concatenate([rng.choice(n, 2000, replace=False), np.arange(n - 64, n), np.arange(64)]))
    ti = torch.from_numpy(idx).cuda()
    o = COracle(_oracle_pool(proc), len(idx), True, ms, autoreset=1)
    o.reset(pids[idx])
    ro, fo, vo, ao = o.rollout_obs(T, X, Y, np.ascontiguousarray(acts[:, ti].cpu().numpy()))
    assert np.array_equal(out["reward_code"][:, ti].cpu().numpy(), ro)
    assert np.array_equal(f[:, ti].cpu().numpy(), fo)
    assert np.array_equal(vis[:, ti].cpu().numpy(), vo)
    assert np.array_equal(ag[:, ti].cpu().numpy(), ao)
    assert (fo & 64).any()
    # --- every env: invariants on the GPU
    xs = torch.tensor([p["x_size"] for p in proc], device="cuda")
    ys = torch.tensor([p["y_size"] for p in proc], device="cuda")
    resets = ((f & 64) != 0).to(torch.int64)
    pid_t = (torch.from_numpy(pids).cuda()[None, :] + torch.cumsum(resets, 0)) % len(proc)   # [T, N]
    cx = torch.arange(X, device="cuda").view(1, 1, X, 1)
    cy = torch.arange(Y, device="cuda").view(1, 1, 1, Y)
    outside = (cx >= xs[pid_t][..., None, None]) | (cy >= ys[pid_t][..., None, None])      # [T, N, X, Y]
    assert not bool(((vis != 0) & outside).any())
    assert not bool(((ag != 0) & outside).any())
    assert bool((ag.sum((2, 3)) == 1).all())                       # one-hot agent plane
    assert bool(((ag == 1) <= (vis == 1)).all())                   # the agent's point is visited
    assert bool(((vis == 0) | (vis == 1)).all())
    cnt = vis.sum((2, 3)).to(torch.int64)                          # [T, N] path lengths
    prev = torch.cat([torch.ones((1, n), dtype=torch.int64, device="cuda"), cnt[:-1]])
    d = cnt - prev
    rs = resets.bool()
    assert bool((cnt[rs] == 1).all())
    assert bool((d[~rs].abs() <= 1).all())
    s = v.state()
    assert np.array_equal(cnt[-1].cpu().numpy(), s["path_len"].astype(np.int64))
    assert np.array_equal(pid_t[-1].cpu().numpy(), s["puzzle"].astype(np.int64))


def test_c4c_262144_envs_split_kernel_sampled_oracle(on_gpu):
    from sparc_gym_amd import SPaRCVecEnv
    from sparc_gym_amd.core import visited_planes
    proc, table = _bench_pool(((2, 2), (3, 3), (4, 4), (5, 5)), True)
    n, T, ms = 262144, 256, 60                    # max_steps 60: many autoresets inside the launch
    pids = _bench_pids(n)
    v = SPaRCVecEnv(n, processed=proc, table=table, traceback=True, max_steps=ms, observation="compact")
    v.reset(options={"puzzle_index": pids})
    assert table.words == 2
    g = torch.Generator(device="cuda")
    g.manual_seed(11)
    acts = torch.randint(0, 4, (T, n), dtype=torch.uint8, device="cuda", generator=g)
    stats = torch.zeros((n, 4), dtype=torch.int32, device="cuda")
    out = v.rollout(T, acts, stats=stats)
    r, f = out["reward_code"], out["flags"]
    # every env: the stats are the sums of its own trace
    st = stats.cpu().numpy()
    assert np.array_equal(st[:, 0], r.to(torch.int64).sum(0).cpu().numpy())
    assert np.array_equal(st[:, 1], ((f & 3) != 0).sum(0).cpu().numpy())
    assert np.array_equal(st[:, 2], (((f & 3) != 0) & (r == 100)).sum(0).cpu().numpy())
    assert np.array_equal(st[:, 3], ((f & 64) != 0).sum(0).cpu().numpy())
    assert not bool(((f & 3) == 3).any())
    # sampled oracle columns, the first and last envs included (large-offset indexing)
    rng = np.random.default_rng(1)
    idx = np.unique(np.concatenate([rng.choice(n, 2000, replace=False), np.arange(n - 256, n), np.arange(256)]))
    ti = torch.from_numpy(idx).cuda()
    o = COracle(_oracle_pool(proc), len(idx), True, ms, autoreset=1)
    o.reset(pids[idx])
    ost = np.zeros((len(idx), 4), np.int32)
    ro, fo = o.rollout(T, np.ascontiguousarray(acts[:, ti].cpu().numpy()), stats=ost)
    assert np.array_equal(r[:, ti].cpu().numpy(), ro)
    assert np.array_equal(f[:, ti].cpu().numpy(), fo)
    assert np.array_equal(st[idx], ost)
    assert (fo & 64).sum() > len(idx)
    s, so = v.state(), o.state()
    for k, ko in (("x", "x"), ("y", "y"), ("step", "step"), ("path_len", "path_len"), ("puzzle", "pid"),
                  ("outcome", "outcome")):
        assert np.array_equal(s[k][idx], so[ko]), k
    assert np.array_equal(visited_planes(s["visited"][:, idx], table, 16, 16), so["visited"].astype(np.int32))


def _sharded_oracle_rollouts(proc, pids, acts_list, tb, ms, shards=16):
    """The C oracle over column shards in threads (ctypes releases the GIL in the call): for
    each launch's actions [T, n] (numpy), (reward codes, flags) [T, n]; returns them, the
    accumulated stats [n, 4] and the concatenated final state."""
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
            T = acts.shape[0]
            futs = [ex.submit(o.rollout, T, np.ascontiguousarray(acts[:, a:a + o.n]), 0, 0, 0, st)
                    for o, a, st in zip(oracles, bounds[:-1], stats)]
            res = [f.result() for f in futs]
            outs.append((np.concatenate([r[0] for r in res], 1), np.concatenate([r[1] for r in res], 1)))
    states = [o.state() for o in oracles]
    state = {k: np.concatenate([s[k] for s in states]) for k in states[0]}
    return outs, np.concatenate(stats), state


def test_c3_bench_kernel_exact_instantiation_full_size(on_gpu):
    """The bench's headline workload exactly (bench.py defaults, config c3): the c3 pool (1,024
    puzzles, seed 0, full property set), 65,536 envs, env i -> puzzle i * 2654435761 mod 1024,
    traceback, max_steps 2,000, next-step autoreset, uint8 actions drawn with torch.randint into
    HBM by the bench's generator seed, and THREE back-to-back 2,000-step launches through the
    same C-ABI call the bench times (sparc_rollout_device -> k_rollout1s<TB=1, RAND=0, LDS=1>:
    65,536 = 256 whole 256-env workgroups, T % 16 == 0, the 1,024 puzzle rows staged in LDS),
    the state round-tripping through HBM between launches.  Every env's reward codes, flags,
    stats and final state must equal the C oracle (SPaRC_Gym.py:1111-1238)."""
    from sparc_gym_amd import SPaRCVecEnv
    proc, table = _bench_pool(((3, 3),), True)
    n, T, L = 65536, 2000, 3
    pids = _bench_pids(n)
    v = SPaRCVecEnv(n, processed=proc, table=table, traceback=True, max_steps=2000, autoreset="next_step",
                    observation="compact")
    v.reset(options={"puzzle_index": pids})
    assert table.words == 1 and len(proc) == 1024
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev)
    g.manual_seed(1234)                                   # bench.py rank 0
    acts = torch.randint(0, 4, (L, T, n), dtype=torch.uint8, device=dev, generator=g)
    rew = torch.empty((L, T, n), dtype=torch.int8, device=dev)
    flg = torch.empty((L, T, n), dtype=torch.uint8, device=dev)
    stats = torch.zeros((n, 4), dtype=torch.int32, device=dev)
    v._stream()
    for k in range(L):                                    # as bench.run(): raw C-ABI calls, back to back
        v.core.rollout_device(T, acts[k].data_ptr(), rew[k].data_ptr(), flg[k].data_ptr(), stats.data_ptr())
    torch.cuda.synchronize()
    v.core.sync()
    acts_np = acts.cpu().numpy()
    outs, ost, so = _sharded_oracle_rollouts(proc, pids, list(acts_np), True, 2000)
    r_np, f_np = rew.cpu().numpy(), flg.cpu().numpy()
    for k in range(L):
        assert np.array_equal(r_np[k], outs[k][0]), f"reward codes differ in launch {k}"
        assert np.array_equal(f_np[k], outs[k][1]), f"flags differ in launch {k}"
    assert np.array_equal(stats.cpu().numpy(), ost)
    _state_equal(v.state(), so, table)
    # the workload exercised what the bench measures: episodes end at the target and by
    # truncation, autoresets follow, and some episodes are solved
    f_all = f_np.reshape(-1, n)
    assert ((f_all & 1) != 0).sum() > 0 and ((f_all & 2) != 0).sum() > 0 and ((f_all & 64) != 0).sum() > 0
    assert int(ost[:, 2].sum()) > 0


def _pack_planes_gpu(p):
    """[T, N, X, Y] int32 planes on the GPU -> [T, N, ceil(X*Y/8)] uint8 on the host, bit c of a
    row = entry c (np.packbits(..., bitorder='little') of the flattened plane); asserts that every
    entry is 0 or 1, so the packing is lossless."""
    T, N = p.shape[:2]
    XY = p.shape[2] * p.shape[3]
    nb = (XY + 7) // 8
    w = (1 << torch.arange(8, device=p.device, dtype=torch.int32))
    out = torch.empty((T, N, nb), dtype=torch.uint8, device=p.device)
    for t in range(T):
        f = p[t].reshape(N, XY)
        assert bool(((f == 0) | (f == 1)).all())
        f = torch.nn.functional.pad(f, (0, nb * 8 - XY)).view(N, nb, 8)
        out[t] = (f * w).sum(-1).to(torch.uint8)
    return out.cpu().numpy()


def _pack_planes_np(v):
    T, n = v.shape[:2]
    return np.packbits(v.reshape(T, n, -1) != 0, axis=-1, bitorder="little")


class _ShardedOracle:
    """The C oracle over column shards of n envs in threads (ctypes and np.packbits release the
    GIL), drawing the bench's counter-based actions (sparc_rand_action(seed, env, t)) itself."""

    def __init__(self, proc, pids, tb, ms, shards=16):
        from concurrent.futures import ThreadPoolExecutor
        from oracle import OraclePool
        self.n = len(pids)
        self.bounds = np.linspace(0, self.n, shards + 1).astype(int)
        opool = OraclePool(_oracle_pool(proc))
        self.oracles = [COracle(opool, int(b - a), tb, ms, autoreset=1)
                        for a, b in zip(self.bounds[:-1], self.bounds[1:])]
        self.stats = [np.zeros((o.n, 4), np.int32) for o in self.oracles]
        for o, a in zip(self.oracles, self.bounds[:-1]):
            o.reset(pids[a:a + o.n])
        self.ex = ThreadPoolExecutor(shards)

    def launch(self, T, seed, t0, obs=None):
        """One launch of T steps: (codes, flags) [T, n], and with obs = (X, Y) the packed planes."""
        def one(k):
            o, a, st = self.oracles[k], int(self.bounds[k]), self.stats[k]
            if obs is None:
                return o.rollout(T, None, seed, a, t0, st)
            r, f, vo, ao = o.rollout_obs(T, obs[0], obs[1], None, seed, a, t0, st)
            return r, f, _pack_planes_np(vo), _pack_planes_np(ao)
        res = list(self.ex.map(one, range(len(self.oracles))))
        return [np.concatenate([r[j] for r in res], 1) for j in range(len(res[0]))]

    def final(self):
        self.ex.shutdown()
        states = [o.state() for o in self.oracles]
        return np.concatenate(self.stats), {k: np.concatenate([s[k] for s in states]) for k in states[0]}


@pytest.mark.parametrize("config", ["c4", "c4c"])
def test_c4_bench_launch_shape_every_env(on_gpu, config):
    """c4 / c4c exactly as bench.py runs them (262,144 envs of the mixed 5x5-11x11 pool, 1,024
    puzzles, traceback, max_steps 2,000, next-step autoreset, the bench's action tiles
    sparc_rand_action(ACTION_SEED, env, j * T + t) in HBM, T = 50 with planes / 2,000 without),
    two back-to-back launches through the bench's C-ABI call with the state carried through HBM.
    Every env's reward codes, flags, stats and final state, and with c4 every env's planes at
    every step, equal the C oracle (SPaRC_Gym.py:956-979, 1111-1238)."""
    import bench
    from sparc_gym_amd import SPaRCVecEnv
    sizes, full, tb, obs = bench.CONFIGS[config]
    proc, table = _bench_pool(sizes, full)
    n, L = 262144, 2
    T = 50 if obs else 2000
    pids = _bench_pids(n)
    v = SPaRCVecEnv(n, processed=proc, table=table, traceback=tb, max_steps=2000, autoreset="next_step",
                    observation="compact")
    v.reset(options={"puzzle_index": pids})
    X, Y = v.x_dim, v.y_dim
    assert (X, Y) == (11, 11) and table.words == 2
    dev = torch.device("cuda", 0)
    acts = torch.empty((L, T, n), dtype=torch.uint8, device=dev)
    for j in range(L):
        v.random_actions(T, seed=bench.ACTION_SEED, t0=j * T, out=acts[j])
    rew = torch.empty((L, T, n), dtype=torch.int8, device=dev)
    flg = torch.empty((L, T, n), dtype=torch.uint8, device=dev)
    stats = torch.zeros((n, 4), dtype=torch.int32, device=dev)
    if obs:   # the bench's traces, reused by both launches: 6.3 GB per plane
        ovis = torch.empty((T, n, X, Y), dtype=torch.int32, device=dev)
        oag = torch.empty_like(ovis)
        assert ovis.numel() * 4 > 4 * 2**30
    ora = _ShardedOracle(proc, pids, tb, 2000)
    v._stream()
    for k in range(L):
        if obs:
            v.core.rollout_obs_device(T, acts[k].data_ptr(), rew[k].data_ptr(), flg[k].data_ptr(), stats.data_ptr(),
                                      ovis.data_ptr(), oag.data_ptr(), X, Y)
        else:
            v.core.rollout_device(T, acts[k].data_ptr(), rew[k].data_ptr(), flg[k].data_ptr(), stats.data_ptr())
        torch.cuda.synchronize()
        out = ora.launch(T, bench.ACTION_SEED, k * T, (X, Y) if obs else None)
        assert np.array_equal(rew[k].cpu().numpy(), out[0]), f"reward codes differ in launch {k}"
        assert np.array_equal(flg[k].cpu().numpy(), out[1]), f"flags differ in launch {k}"
        if obs:
            assert np.array_equal(_pack_planes_gpu(ovis), out[2]), f"visited planes differ in launch {k}"
            assert np.array_equal(_pack_planes_gpu(oag), out[3]), f"agent planes differ in launch {k}"
    ost, so = ora.final()
    assert np.array_equal(stats.cpu().numpy(), ost)
    _state_equal(v.state(), so, table)
    # the workload exercised what the bench measures: episodes end at the target and autoresets
    # follow (truncation needs max_steps 2,000 steps or a dead end, which traceback rules out: c4's
    # 100 steps have none)
    f_all = flg.cpu().numpy().reshape(-1, n)
    assert ((f_all & 1) != 0).sum() > 0 and ((f_all & 64) != 0).sum() > 0
