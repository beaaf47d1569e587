"""One rank of the sharded HIP rollout (tests/test_gpu_dist.py launches it with torchrun).

Each rank owns the contiguous global env ids [rank * N, (rank + 1) * N) (sparc_gym_amd.dist),
steps them on the GPU through the C ABI with the counter-based random actions of those global
ids, and the end-of-batch all_gather collects the per-env stats (plus, for the test, the
reward-code and flag traces).  Rank 0 writes everything to an .npz file.

    torchrun --nproc-per-node 2 tests/gpu_dist_worker.py OUT.npz --envs 65536 --steps 96
"""
import argparse
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "sparc-gym_amd"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from sparc_gym_amd import SPaRCVecEnv, synthetic  # noqa: E402
from sparc_gym_amd import dist as sdist  # noqa: E402
from sparc_gym_amd.puzzles import pack_table, process_puzzles  # noqa: E402


def pool():
    proc = process_puzzles(synthetic.make_puzzles(1024, seed=0, sizes=((3, 3),), full_properties=True))
    return proc, pack_table(proc)


def run_envs(proc, table, offset, n, T, seed, device=0):
    """The rollout of global envs [offset, offset + n) on one GPU: (stats [n,4], reward [T,n],
    flags [T,n]) as tensors on the GPU."""
    v = SPaRCVecEnv(n, processed=proc, table=table, traceback=True, observation="compact", device=device,
                    env_offset=offset)
    gid = np.arange(offset, offset + n, dtype=np.uint64)
    v.reset(options={"puzzle_index": (gid * 2654435761 % len(proc)).astype(np.int64)})
    stats = torch.zeros((n, 4), dtype=torch.int32, device=v.device)
    out = v.rollout(T, None, seed=seed, stats=stats)
    return stats, out["reward_code"], out["flags"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--steps", type=int, default=96)
    ap.add_argument("--seed", type=int, default=31)
    a = ap.parse_args()
    rank, world, local = sdist.init_from_env("gloo")
    proc, table = pool()
    offset, n = sdist.env_shard(a.envs, rank)
    stats, rew, flg = run_envs(proc, table, offset, n, a.steps, a.seed, device=0)
    gathered = sdist.gather_stats(stats).cpu()
    traces = []
    for t in (rew, flg):
        src = t.t().contiguous().cpu()                              # [n, T]: env-major for the gather
        dst = torch.empty((world * n, a.steps), dtype=src.dtype)
        dist.all_gather_into_tensor(dst, src)
        traces.append(dst.t().contiguous().numpy())
    elapsed = sdist.max_over_ranks(0.5 + rank)
    if rank == 0:
        np.savez(a.out, stats=gathered.numpy(), reward=traces[0], flags=traces[1], world=world,
                 backend=dist.get_backend(), elapsed=elapsed)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
