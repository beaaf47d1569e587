"""World-size-2 gloo run of the sharded rollout + end-of-batch gather on CPU.

Each rank runs its env shard (the C oracle stands in for the GPU step path here: this tests
the sharding and the collective, the step itself is covered by the parity tests) and the
gathered per-env stats must equal one process running every env."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import COracle
from sparc_gym_amd import dist as sdist
from sparc_gym_amd import synthetic
from sparc_gym_amd.puzzles import process_puzzles

N_PER_RANK, T, SEED = 96, 120, 5


def _pool():
    proc = process_puzzles(synthetic.make_puzzles(16, seed=11))
    return [{"x_size": p["x_size"], "y_size": p["y_size"], "start": list(p["start_location"]),
             "target": list(p["target_location"]), "solution_count": p["solution_count"],
             "solution_paths": p["solution_paths"], "gaps": p["obs_array"]["gaps"]} for p in proc]


def _run_shard(pool, offset, n):
    o = COracle(pool, n, True, 2000, autoreset=1)
    gid = np.arange(offset, offset + n, dtype=np.uint64)
    o.reset((gid * 2654435761 % len(pool)).astype(np.int64))
    stats = np.zeros((n, 4), np.int32)
    o.rollout(T, None, seed=SEED, env_offset=offset, stats=stats)
    return stats


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    r, w, _ = sdist.init_from_env("gloo")
    offset, n = sdist.env_shard(N_PER_RANK, r)
    stats = torch.from_numpy(_run_shard(_pool(), offset, n))
    gathered = sdist.gather_stats(stats)
    t = sdist.max_over_ranks(0.1 * (r + 1))
    vals = sdist.gather_values([r, 2.5 * r, 7])
    if r == 0:
        q.put((gathered.numpy(), sdist.summarize(gathered), t, vals))
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_two_rank_gather_equals_single_process():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    gathered, summary, t, vals = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ref = _run_shard(_pool(), 0, 2 * N_PER_RANK)
    assert np.array_equal(gathered, ref)
    assert summary["done"] == int(ref[:, 1].sum())
    assert t == pytest.approx(0.2)
    assert vals == [[0.0, 0.0, 7.0], [1.0, 2.5, 7.0]]   # bench.py's per-rank records


def test_shards_are_contiguous_and_disjoint():
    spans = [sdist.env_shard(1000, r) for r in range(8)]
    assert spans[0] == (0, 1000) and spans[7] == (7000, 1000)
    assert all(a[0] + a[1] == b[0] for a, b in zip(spans, spans[1:]))
