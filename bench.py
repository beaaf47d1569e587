#!/usr/bin/env python3
"""Benchmark: env-steps/s of the batched SPaRC step path on MI355X (BASELINE.json metric).

Workload (default, BASELINE.json configs[2]): 65,536 concurrent 7x7 SPaRC instances per GPU,
full property set, traceback=True, max_steps=2000, gymnasium next-step autoreset onto the next
puzzle, 1,024 synthetic puzzles (seed 0), env i -> puzzle (i * 2654435761) mod 1024.
One bench "step" = every env advanced by one env.step().  Actions are uniform random in
{0,1,2,3}, generated on the GPU before the timed region ([K, N] uint8 resident in HBM, like a
policy's output).  The timed region runs K steps as ceil(K / chunk) launches of the fused
rollout kernel (state in VGPRs, per-step reward codes + flags streamed to HBM), then the
end-of-batch gather of per-env (reward sum, dones, solved, resets) to rank 0 over RCCL.
``--mode step`` instead times one k_step launch per env-step (the gym one-call-per-step contract).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--envs 65536] [--chunk 500]
    torchrun --nproc-per-node N bench.py --gpus N ...      (one process per GPU)
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import subprocess
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "sparc-gym_amd"))

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)

CONFIGS = {
    # name: (grid sizes, full property set, traceback, 'new' observation planes every step)
    "c2": (((3, 3),), False, False, False),
    "c3": (((3, 3),), True, True, False),
    # BASELINE configs[3]: 262,144 mixed 5x5-11x11 puzzles, observation='new' dict pack
    "c4": (((2, 2), (3, 3), (4, 4), (5, 5)), True, True, True),
}
DEFAULT_ENVS = {"c2": 4096, "c3": 65536, "c4": 262144}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--warmup", type=int, default=200)
    ap.add_argument("--envs", type=int, default=0, help="envs per GPU (0 = the config's: c2 4,096, c3 65,536, "
                                                         "c4 262,144)")
    ap.add_argument("--chunk", type=int, default=0,
                    help="env-steps per rollout launch (0 = all timed steps in one launch; with observation "
                         "traces (c4) 0 = 50)")
    ap.add_argument("--backend", default="nccl", help="torch.distributed backend for N > 1 (nccl = RCCL)")
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--mode", default="rollout", choices=["rollout", "step"])
    ap.add_argument("--puzzles", type=int, default=1024)
    ap.add_argument("--max-steps", type=int, default=2000)
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="bounded CPU-baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    return ap.parse_args()


def state_bytes_per_env(words, traceback):
    """HBM bytes one launch loads AND stores per env for its state (k_rollout / k_step):
    visited 8*words + dir stack 16*words (traceback) + pos/aux/step/pid 16."""
    return 8 * words + (16 * words if traceback else 0) + 16


def cpu_baseline(proc, tb, max_steps, seconds, obs_dims=None, config="c3"):
    """C oracle (sparc_oracle.c, 1 thread) on a bounded sample of the same workload (with
    obs_dims = (x_dim, y_dim): also writing the 'new' observation planes of every step)."""
    from oracle import COracle
    pool = [{"x_size": p["x_size"], "y_size": p["y_size"], "start": list(p["start_location"]),
             "target": list(p["target_location"]), "solution_count": p["solution_count"],
             "solution_paths": p["solution_paths"], "gaps": p["obs_array"]["gaps"]} for p in proc]
    n = 1024
    o = COracle(pool, n, tb, max_steps, autoreset=1)
    o.reset((np.arange(n, dtype=np.uint64) * 2654435761 % len(proc)).astype(np.int64))
    steps, T = 0, 64
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        if obs_dims:
            o.rollout_obs(T, obs_dims[0], obs_dims[1], None, seed=1, t0=steps)
        else:
            o.rollout(T, None, seed=1, t0=steps)
        steps += T
    dt = time.perf_counter() - t0
    c_rate = n * steps / dt
    # pure-Python restatement: the reference-speed step() core (no rule audit)
    from oracle.cpu_ref import CpuRefEnv
    rng = np.random.default_rng(0)
    env = CpuRefEnv(pool[0], tb, max_steps)
    k, t1 = 0, time.perf_counter()
    while time.perf_counter() - t1 < min(3.0, seconds):
        _, term, trunc = env.step(int(rng.integers(4)))
        k += 1
        if term or trunc:
            env.p = pool[k % len(pool)]
            env.reset()
    py_rate = k / (time.perf_counter() - t1)
    out = {"value": round(c_rate, 1), "unit": "env-steps/s", "cores": 1, "kind": "port",
           "sample": f"oracle/sparc_oracle.c, {n} envs x {steps} steps, random actions, next-step autoreset, "
                     f"{'visited + agent_location planes written every step, ' if obs_dims else ''}"
                     f"1 thread, {dt:.1f} s; CPU {platform.processor() or platform.machine()}, "
                     f"os.cpu_count()={os.cpu_count()}",
           "value_1core": round(c_rate, 1),
           "python_port_value": round(py_rate, 1),
           "python_port_sample": "oracle/cpu_ref.py (reference step() restated in pure Python, no rule "
                                 f"audit), 1 env, {k} steps, 1 thread"}
    # the same oracle, one process per core (BASELINE.md CPU-baseline plan), in a child process
    # that never touches the GPU; up to 16 cores (one GPU's share of the box)
    cmd = [sys.executable, "-m", "oracle.cpu_bench", "--config", config, "--seconds", str(seconds),
           "--max-steps", str(max_steps)] + (["--obs", str(obs_dims[0]), str(obs_dims[1])] if obs_dims else [])
    try:
        r = subprocess.run(cmd, cwd=REPO, capture_output=True, text=True, timeout=seconds * 4 + 120)
        mc = json.loads(r.stdout.strip().splitlines()[-1])
        out.update(value=mc["value"], cores=mc["procs"],
                   sample=out["sample"] +
                   f"; all-cores value: {mc['procs']} processes x {n} envs (oracle/cpu_bench.py), "
                   f"{mc['seconds']:.0f} s, {mc['usable_cores']} usable cores")
    except (subprocess.SubprocessError, ValueError, KeyError, IndexError) as exc:   # keep the 1-core number
        out["multi_core_error"] = repr(exc)[:200]
    return out


def load_traffic(workload, kernel):
    """HBM bytes per launch from a committed rocprofv3 --pmc summary (profiles/pmc_traffic.json),
    produced by tools/pmc_traffic.py; None when absent."""
    path = os.path.join(REPO, "profiles", "pmc_traffic.json")
    if not os.path.exists(path):
        return None
    try:
        d = json.load(open(path))
        return d.get(workload, {}).get(kernel)
    except (OSError, ValueError):
        return None


def main():
    args = parse()
    import torch
    import torch.distributed as dist
    from sparc_gym_amd import SPaRCVecEnv, synthetic
    from sparc_gym_amd import dist as sdist
    from sparc_gym_amd.puzzles import pack_table, process_puzzles

    rank, world, local = sdist.init_from_env(args.backend)
    local = local % max(1, torch.cuda.device_count())   # (rehearsals: several ranks on one GPU)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    sizes, full, tb, obs = CONFIGS[args.config]
    if args.envs <= 0:
        args.envs = DEFAULT_ENVS[args.config]
    recs = synthetic.make_puzzles(args.puzzles, seed=0, sizes=sizes, full_properties=full)
    proc = process_puzzles(recs)
    table = pack_table(proc)
    offset, n = sdist.env_shard(args.envs, rank)
    vec = SPaRCVecEnv(n, processed=proc, table=table, traceback=tb, max_steps=args.max_steps,
                      autoreset="next_step", device=local, env_offset=offset, observation="compact")
    gid = np.arange(offset, offset + n, dtype=np.uint64)
    vec.reset(options={"puzzle_index": (gid * 2654435761 % len(proc)).astype(np.int64)})

    K, W = args.steps, args.warmup
    if args.chunk <= 0:
        args.chunk = 50 if obs else K
    chunk = max(1, min(args.chunk, K))
    # observation traces [chunk, N, x_dim, y_dim] int32 (visited, agent_location), reused by
    # every launch (one launch = one chunk of steps; a consumer reads them between launches)
    X, Y = vec.x_dim, vec.y_dim
    plane_bytes = X * Y * 4
    ovis = oag = None
    if obs:
        ovis = torch.empty((chunk, n, X, Y), dtype=torch.int32, device=dev)
        oag = torch.empty_like(ovis)
    g = torch.Generator(device=dev)
    g.manual_seed(1234 + rank)
    actions = torch.randint(0, 4, (K, n), dtype=torch.uint8, device=dev, generator=g)
    warm_actions = torch.randint(0, 4, (max(W, 1), n), dtype=torch.uint8, device=dev, generator=g)
    rew = torch.empty((K, n), dtype=torch.int8, device=dev)
    flags = torch.empty((K, n), dtype=torch.uint8, device=dev)
    stats = torch.zeros((n, 4), dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream(dev)

    vec._stream()                       # bind the context to this (torch's current) stream
    core = vec.core
    s_ptr = stats.data_ptr()

    def run(lo, hi, acts, rew_out, flag_out, events=None):
        if args.mode == "rollout":
            # direct C-ABI calls on pre-validated buffers (vec.rollout() checks shapes per call)
            ap, rp, fp = acts.data_ptr(), rew_out.data_ptr(), flag_out.data_ptr()
            t = lo
            while t < hi:
                c = min(chunk, hi - t)
                ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) if events is not None else None
                if ev:
                    ev[0].record(stream)
                if obs:
                    core.rollout_obs_device(c, ap + t * n, rp + t * n, fp + t * n, s_ptr, ovis.data_ptr(),
                                            oag.data_ptr(), X, Y)
                else:
                    core.rollout_device(c, ap + t * n, rp + t * n, fp + t * n, s_ptr)
                if ev:
                    ev[1].record(stream)
                    events.append((ev, c))
                t += c
        else:
            for t in range(lo, hi):
                ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) if events is not None else None
                if ev:
                    ev[0].record(stream)
                core.step_device(acts.data_ptr() + t * n, rew_out.data_ptr() + t * n, flag_out.data_ptr() + t * n)
                if ev:
                    ev[1].record(stream)
                    events.append((ev, 1))

    # warmup (untimed)
    if W > 0:
        wr = torch.empty((W, n), dtype=torch.int8, device=dev)
        wf = torch.empty((W, n), dtype=torch.uint8, device=dev)
        run(0, W, warm_actions, wr, wf)
    torch.cuda.synchronize(dev)
    stats.zero_()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    events = []
    t0 = time.perf_counter()
    run(0, K, actions, rew, flags, events)
    # end-of-batch gather of per-env summaries (reward sum, dones, solved, resets): one RCCL call
    gathered = sdist.gather_stats(stats)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = sdist.max_over_ranks(t1 - t0, dev)
    summary = sdist.summarize(gathered)

    kern_ms = [a.elapsed_time(b) for (a, b), _ in events]
    steps_per_launch = [c for _, c in events]
    avg_ms = float(np.mean(kern_ms))
    avg_T = float(np.mean(steps_per_launch))
    value = world * n * K / elapsed
    # algorithmic HBM bytes per launch: per env-step action 1 + reward 1 + flags 1; per env and
    # launch the state (load + store) and, for rollouts, the stats record (load + store)
    sb = state_bytes_per_env(table.words, tb)
    per_env_launch = 2 * sb + (32 if args.mode == "rollout" else 0)
    per_step = 3 + (2 * plane_bytes if obs and args.mode == "rollout" else 0)
    bytes_launch = n * (per_step * avg_T + per_env_launch)
    achieved = bytes_launch / (avg_ms * 1e-3) / 1e9
    if args.mode != "rollout":
        kernel = "k_step"
    elif table.words == 1 and not obs:
        # batches of whole 256-env workgroups: the split move / trie kernel
        kernel = "k_rollout1s" if n % 256 == 0 and chunk >= 16 else "k_rollout1"
    else:
        kernel = "k_rollout"
    workload = f"{args.config}_{args.mode}_n{n}_chunk{chunk if args.mode == 'rollout' else 1}"
    traffic = load_traffic(workload, kernel)
    out = {
        "metric": "env-steps/sec at 65,536 envs, 7x7 grid (HBM roofline fraction in 'roofline')",
        "value": round(value, 1),
        "unit": "env-steps/s",
        "n_gpus": world,
        "steps": K,
        "warmup": W,
        "ms_per_step": round(elapsed * 1e3 / K, 6),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8/u64 (integer bitboards)",
        "data": "synthetic SPaRC-schema puzzles (sparc_gym_amd.synthetic, seed 0); uniform random actions in HBM",
        "config": {"workload": f"{args.config}: {n} envs/GPU, lattices {['%dx%d' % (2*w+1, 2*h+1) for w, h in sizes]}, "
                               f"{'full property set' if full else 'base planes'}, traceback={tb}, "
                               f"max_steps={args.max_steps}, next-step autoreset, {args.puzzles} puzzles"
                               + (f", observation='new': visited + agent_location int32 planes "
                                  f"[N, {X}, {Y}] written every step" if obs else ""),
                   "mode": args.mode, "envs_per_gpu": n, "env_steps_per_launch": chunk if args.mode == "rollout" else 1,
                   "parallelism": f"dp{world} (env shards, {'RCCL' if args.backend == 'nccl' else args.backend} "
                                  f"all_gather of per-env stats at end of batch)"},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 6), "traffic": traffic,
                     "kernel": kernel, "kernel_avg_ms": round(avg_ms, 4), "launches": len(kern_ms),
                     "algorithmic_bytes_per_launch": int(bytes_launch),
                     "bytes_model": f"per env-step {per_step} B (action, reward code, flags"
                                    f"{f', visited + agent_location planes 2 x {plane_bytes} B' if obs else ''}"
                                    f"); per env per launch "
                                    f"{per_env_launch} B (state {sb} B load+store"
                                    f"{', stats 16 B load+store' if args.mode == 'rollout' else ''})"},
        "episodes": summary,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cb = cpu_baseline(proc, tb, args.max_steps, args.cpu_seconds, (X, Y) if obs else None, args.config)
        out["cpu_baseline"] = cb
        out["gpu_vs_cpu"] = round(value / cb["value"], 1)
    elif rank == 0:
        out["cpu_baseline"] = None
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
