"""BASELINE config c5 end to end on the one GPU: 524,288 envs in 8 ranks of 65,536.

``bench.py --gpus 8 --rehearsal --backend gloo`` starts its own 8 rank processes (the box has one
GPU, so they share it: a rehearsal, never a measurement), each stepping its shard of the c3 pool
through the bench's own C-ABI rollout launches on action tiles drawn from the global env id, then
one all_gather of the per-env stats.  The gathered stats must equal ONE process stepping all
524,288 envs (env_offset 0) through the same launches, and the columns on both sides of every
shard boundary (global ids 65,536·r − 1 and 65,536·r) must equal the C oracle run on those ids
alone — which pins the env_offset-keyed random actions (sparc_rand_action) and the puzzle
assignment of each shard.  The reference has no counterpart: it is one env per process
(llm_testing/llm_host.py:257-264); SURVEY §8e."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
RANKS, PER_RANK, T, K, W = 8, 65536, 64, 2, 1


def _bench_single_process(proc, table, n_total):
    """The bench's launch sequence (bench.py run()) in one process over every env."""
    import bench
    from sparc_gym_amd import SPaRCVecEnv
    vec = SPaRCVecEnv(n_total, processed=proc, table=table, traceback=True, max_steps=2000,
                      autoreset="next_step", observation="compact")
    gid = np.arange(n_total, dtype=np.uint64)
    vec.reset(options={"puzzle_index": (gid * 2654435761 % len(proc)).astype(np.int64)})
    RA = min(max(K, W), 8)
    acts = torch.empty((RA, T, n_total), dtype=torch.uint8, device="cuda")
    for j in range(RA):
        vec.random_actions(T, seed=bench.ACTION_SEED, t0=j * T, out=acts[j])
    stats = torch.zeros((n_total, 4), dtype=torch.int32, device="cuda")
    for k in range(W + K):
        if k == W:
            stats.zero_()
        vec.rollout(T, acts[k % RA], stats=stats, record=False)
    torch.cuda.synchronize()
    return stats.cpu().numpy(), RA


def test_c5_eight_rank_rehearsal_equals_one_process_and_oracle(on_gpu, tmp_path):
    out = str(tmp_path / "stats.npy")
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--gpus", str(RANKS), "--rehearsal", "--backend", "gloo",
           "--envs", str(PER_RANK), "--env-steps", str(T), "--steps", str(K), "--warmup", str(W),
           "--no-cpu-baseline", "--stats-out", out]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1                                          # rank 0 prints one line
    o = json.loads(lines[0])
    w = o["world_observed"]
    assert o["n_gpus"] == RANKS and w["world_size"] == RANKS and w["backend"] == "gloo"
    assert w["launcher"] == "bench.py (child per rank)" and w["rehearsal"] is True
    assert len(w["per_rank_kernel_ms"]) == RANKS and all(t > 0 for t in w["per_rank_kernel_ms"])
    assert o["config"]["envs_per_gpu"] == PER_RANK
    n_total = RANKS * PER_RANK
    got = np.load(out)
    assert got.shape == (n_total, 4) and got.dtype == np.int32

    # one process over all 524,288 envs through the same launches
    sys.path.insert(0, REPO)
    from sparc_gym_amd import synthetic
    from sparc_gym_amd.puzzles import pack_table, process_puzzles
    proc = process_puzzles(synthetic.make_puzzles(1024, seed=0, sizes=((3, 3),), full_properties=True))
    table = pack_table(proc)
    want, RA = _bench_single_process(proc, table, n_total)
    assert np.array_equal(got, want)
    tot = want.astype(np.int64).sum(0)
    assert o["episodes"] == {"reward_code_sum": int(tot[0]), "done": int(tot[1]), "solved": int(tot[2]),
                             "autoresets": int(tot[3])}
    assert tot[1] > 0 and tot[3] > 0
    for r_ in range(RANKS):                                          # every shard ended episodes
        assert want[r_ * PER_RANK:(r_ + 1) * PER_RANK, 1].sum() > 0

    # the C oracle on the columns either side of every shard boundary, each on its own
    import bench
    from oracle import COracle
    pool = [{"x_size": p["x_size"], "y_size": p["y_size"], "start": list(p["start_location"]),
             "target": list(p["target_location"]), "solution_count": p["solution_count"],
             "solution_paths": p["solution_paths"], "gaps": p["obs_array"]["gaps"]} for p in proc]
    ids = sorted({0, n_total - 1} | {PER_RANK * r_ + d for r_ in range(1, RANKS) for d in (-1, 0)})
    for g_ in ids:
        oc = COracle(pool, 1, True, 2000, autoreset=1)
        oc.reset([int(np.uint64(g_) * np.uint64(2654435761) % np.uint64(len(proc)))])
        st = np.zeros((1, 4), np.int32)
        for k in range(W + K):
            if k == W:
                st[:] = 0
            oc.rollout(T, None, seed=bench.ACTION_SEED, env_offset=g_, t0=(k % RA) * T, stats=st)
        assert np.array_equal(got[g_], st[0]), (g_, got[g_], st[0])


@pytest.mark.parametrize("n,offset", [(1001, 0), (4096, 65536 * 3 - 7)])
def test_random_actions_are_the_rand_rollout_actions(on_gpu, n, offset):
    """sparc_random_actions_device writes exactly the actions a NULL-action rollout draws
    (sparc_rand_action(seed, env_offset + i, t0 + t)), also for a batch that is not a multiple of
    4 envs (the unaligned row tails)."""
    from oracle import COracle
    from sparc_gym_amd import SPaRCVecEnv, synthetic
    from sparc_gym_amd.puzzles import process_puzzles
    proc = process_puzzles(synthetic.make_puzzles(64, seed=2, sizes=((3, 3),), full_properties=True))
    kw = dict(processed=proc, traceback=True, autoreset="next_step", observation="compact", env_offset=offset)
    T, seed, t0 = 40, 99, 17
    a = SPaRCVecEnv(n, **kw)
    acts = a.random_actions(T, seed=seed, t0=t0).cpu().numpy()
    oc = COracle([{"x_size": 7, "y_size": 7, "start": [0, 0], "target": [6, 6], "solution_count": 0,
                   "solution_paths": [], "gaps": np.zeros((7, 7), np.int64)}], 1, True, 2000)
    rng = np.random.default_rng(0)
    for t, i in zip(rng.integers(0, T, 300), rng.integers(0, n, 300)):
        assert acts[t, i] == oc.rand_action(seed, offset + int(i), t0 + int(t))
    assert set(np.unique(acts)) == {0, 1, 2, 3}
    pids = np.arange(n) % len(proc)
    a.reset(options={"puzzle_index": pids})
    ra = a.rollout(T, torch.from_numpy(acts).cuda())
    b = SPaRCVecEnv(n, **kw)
    b.reset(options={"puzzle_index": pids})
    rb = b.rollout(T, None, seed=seed, t0=t0)
    assert torch.equal(ra["reward_code"], rb["reward_code"]) and torch.equal(ra["flags"], rb["flags"])
