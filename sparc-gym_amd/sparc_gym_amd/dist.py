"""Multi-GPU data parallelism over independent env shards.

The reference is one env per process (SPaRC_Gym.py:44; llm_host.py:257-264 runs independent
envs concurrently).  Here each rank (one process per GPU) owns a contiguous range of global env
ids, steps it with no communication, and at the end of a rollout batch the per-env summaries
(reward-code sum, done steps, solved steps, autoresets: the ``stats`` [N, 4] int32 of
``SPaRCVecEnv.rollout``) are gathered with ONE all_gather (RCCL over xGMI with backend "nccl";
gloo in the CPU tests).  Global env id = rank * envs_per_rank + local id, which also seeds the
counter-based random actions, so a sharded run reproduces the single-process run of all envs.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist


def env_shard(envs_per_rank: int, rank: int):
    """(env_offset, count) of this rank's contiguous shard (weak scaling: fixed per rank)."""
    return rank * envs_per_rank, envs_per_rank


def init_from_env(backend="nccl", device=None):
    """Initialise torch.distributed from torchrun's environment; returns (rank, world, local).
    ``device``: this rank's GPU (default LOCAL_RANK, one process per GPU)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and not dist.is_initialized():
        if backend == "nccl":
            dev = local if device is None else device
            torch.cuda.set_device(dev)
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:
            dist.init_process_group(backend)
    return rank, world, local


def gather_stats(stats: torch.Tensor, group=None) -> torch.Tensor:
    """End-of-batch gather: [N, 4] int32 per rank -> [world * N, 4] on every rank, ordered by
    global env id.  A single all_gather (one RCCL call per batch, never per step); it runs
    whenever a process group exists, world size 1 included (a copy)."""
    if not dist.is_initialized():
        return stats
    world = dist.get_world_size(group)
    src = stats.contiguous()
    if dist.get_backend(group) != "nccl":   # gloo (CPU tests / rehearsals): stage through host
        src = src.cpu()
    out = torch.empty((world * src.shape[0],) + tuple(src.shape[1:]), dtype=src.dtype, device=src.device)
    dist.all_gather_into_tensor(out, src, group=group)
    return out.to(stats.device)


def summarize(gathered: torch.Tensor) -> dict:
    """Totals over every env of every rank."""
    t = gathered.to(torch.int64).sum(0).cpu().tolist()
    return {"reward_code_sum": t[0], "done": t[1], "solved": t[2], "autoresets": t[3]}


def gather_values(values, device=None):
    """Every rank's list of numbers (same length on every rank) -> [[rank 0's], [rank 1's], ...]
    (float64; one small all_gather).  Without a process group: [values]."""
    if not dist.is_initialized():
        return [list(map(float, values))]
    if dist.get_backend() != "nccl":
        device = "cpu"
    t = torch.tensor([float(v) for v in values], dtype=torch.float64, device=device)
    out = torch.empty(dist.get_world_size() * t.numel(), dtype=torch.float64, device=device)
    dist.all_gather_into_tensor(out, t)   # flat output: gloo takes no [world, n] shape
    return out.view(dist.get_world_size(), t.numel()).cpu().tolist()


def max_over_ranks(seconds: float, device=None) -> float:
    """The slowest rank's time (the job's time)."""
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return seconds
    if dist.get_backend() != "nccl":
        device = "cpu"
    t = torch.tensor([seconds], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
