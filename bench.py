#!/usr/bin/env python3
"""Benchmark: env-steps/s of the batched SPaRC step path on MI355X (BASELINE.json metric).

Workload (default, BASELINE.json configs[2]): 65,536 concurrent 7x7 SPaRC instances per GPU,
full property set, traceback=True, max_steps=2000, gymnasium next-step autoreset onto the next
puzzle, 1,024 synthetic puzzles (seed 0; ``--puzzles P`` extends the pool by blocks of 1,024, block b
drawn with seed b), env i -> puzzle (i * 2654435761) mod P.
Actions are uniform random in {0,1,2,3}, generated on the GPU before the timed region (uint8
tiles resident in HBM, like a policy's output) by the counter-based generator keyed by the
global env id (sparc_random_actions_device), so N ranks hold the tiles of one process over all
N x envs and a sharded run equals the single-process one env for env.

One bench "step" is one pass of the hot path over the batch: one rollout launch that advances
every env by ``--env-steps`` T env.step()s (default 2,000; 50 for c4, whose launch also writes
the 'new' planes of every step), state in VGPRs, per-step reward codes + flags streamed to HBM.
The timed region runs K such launches back to back, then the end-of-batch gather of per-env
(reward sum, dones, solved, resets) to every rank over RCCL.  ``value`` = all env-steps of all
ranks / the slowest rank's time.  ``--mode step`` instead times one k_step launch per bench
step (T = 1, the gym one-call-per-step contract).

Buffers: K launches cycle through up to 8 distinct action tiles [T, N] and 2 output tiles (a
consumer reads each launch's outputs before the next one but one), so any K fits in HBM.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--envs 65536] [--env-steps 2000]
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
# VALU issue peak: 256 CUs x 4 SIMDs, one wave64 VALU instruction per 2 cycles per SIMD
# (MI355X_MICROARCH.md, Wave scheduling), at the 2.4 GHz peak engine clock
VALU_PEAK_WAVE_INSTS = 1024 * 2.4e9 / 2


def csrc_files():
    """Every kernel source (all of csrc/, so a new header can never be left out), the ABI
    header and the Makefile, repo-relative and sorted."""
    import glob
    srcs = sorted(os.path.relpath(f, REPO) for f in glob.glob(os.path.join(REPO, "sparc-gym_amd", "csrc", "*"))
                  if f.endswith((".hip", ".hpp", ".h", ".cpp")))
    return tuple(srcs) + ("include/sparc_gym_amd.h", "sparc-gym_amd/Makefile")

CONFIGS = {
    # name: (grid sizes, full property set, traceback, 'new' observation planes every step)
    "c2": (((3, 3),), False, False, False),
    "c3": (((3, 3),), True, True, False),
    # BASELINE configs[3]: 262,144 mixed 5x5-11x11 puzzles, observation='new' dict pack
    "c4": (((2, 2), (3, 3), (4, 4), (5, 5)), True, True, True),
    # c4's pool without the observation planes (the step compute of the mixed pool alone)
    "c4c": (((2, 2), (3, 3), (4, 4), (5, 5)), True, True, False),
    # the other reading of "7x7": a 7x7 cell grid, i.e. a 15x15 lattice (SPaRC_Gym.py:243-248)
    "c3g7": (((7, 7),), True, True, False),
    # c3 with the rule audit after every step, as the reference's full step() runs it
    # (_validate_rules at SPaRC_Gym.py:1227 and 1011 -> info['rule_status'], 941-950)
    "c3r": (((3, 3),), True, True, False),
}
RULE_CONFIGS = ("c3r",)
ACTION_SEED = 1234   # seed of the bench's random action tiles (sparc_rand_action)
DEFAULT_ENVS = {"c2": 4096, "c3": 65536, "c4": 262144, "c4c": 262144, "c3g7": 65536, "c3r": 65536}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20, help="timed bench steps (rollout launches of T env-steps)")
    ap.add_argument("--warmup", type=int, default=3, help="untimed bench steps")
    ap.add_argument("--envs", type=int, default=0, help="envs per GPU (0 = the config's: c2 4,096, c3 65,536, "
                                                         "c4 262,144)")
    ap.add_argument("--env-steps", "--chunk", dest="chunk", type=int, default=0,
                    help="env-steps per env in one bench step = one rollout launch (0 = 2,000; with "
                         "observation traces (c4) 50)")
    ap.add_argument("--backend", default="nccl", help="torch.distributed backend for N > 1 (nccl = RCCL)")
    ap.add_argument("--rehearsal", action="store_true",
                    help="allow more ranks than GPUs (ranks share GPUs: a rehearsal, never a measurement)")
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--mode", default="rollout", choices=["rollout", "step"])
    ap.add_argument("--puzzles", type=int, default=1024)
    ap.add_argument("--placement", default="auto", choices=["auto", "hash", "xcd"],
                    help="first puzzle of each env (initial_puzzles): auto = xcd past 1,024 puzzles")
    ap.add_argument("--max-steps", type=int, default=2000)
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="bounded CPU-baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--stats-out", default="",
                    help="rank 0 saves the gathered per-env stats [world*N, 4] int32 here (.npy; tests)")
    a = ap.parse_args()
    if a.mode == "step" and a.config in RULE_CONFIGS:
        ap.error(f"--mode step runs no rule audit: {a.config} needs --mode rollout")
    return a


def initial_puzzles(gid, P, placement):
    """Each env's first puzzle (the rest follow by next-step autoreset, pid + 1 mod P); gid: this
    rank's global env ids.  'hash': env g -> (g * 2654435761) mod P.  'xcd':
    sparc_gym_amd.vec_env.xcd_local_puzzle_index, the same hash within one eighth of the pool per
    XCD group of workgroups, so an XCD's L2 holds the records of about P / 8 puzzles; every puzzle
    still starts 65,536 / P envs, only the env slot that plays it changes.  'auto': 'xcd' for
    pools past the 1,024 LDS-staged rows (P % 8 == 0), else 'hash'."""
    from sparc_gym_amd.vec_env import xcd_local_puzzle_index
    gid = np.asarray(gid, dtype=np.uint64)
    if placement == "auto":
        placement = "xcd" if P > 1024 and P % 8 == 0 else "hash"
    if placement == "hash" or P < 8 or P % 8:
        return (gid * np.uint64(2654435761) % np.uint64(P)).astype(np.int64), "hash"
    off = int(gid[0]) if len(gid) else 0
    return xcd_local_puzzle_index(len(gid), P, off), "xcd"


def rule_rollout_kernel(proc, table):
    """The kernel sparc_rollout_rules_device runs on this pool (csrc rollout_impl): k_rollout1r
    when the boards are one word, fit its ring word (x_size * pitch <= 57) and every puzzle has a
    region-code table (at most 12 cells, 2^(cells) entries each within the 2^28-entry budget);
    else the generic k_rollout<..., RULES>."""
    if table.words != 1:
        return "k_rollout"
    entries = 0
    for p in proc:
        cells = ((p["x_size"] - 1) // 2) * ((p["y_size"] - 1) // 2)
        if cells > 12 or p["x_size"] * table.pitch > 57:
            return "k_rollout"
        entries += 8 * (1 if cells <= 3 else 1 << (cells - 3))
    return "k_rollout1r" if entries <= 1 << 28 else "k_rollout"


def _pool_block(args):
    b, cnt, sizes, full = args
    from sparc_gym_amd import synthetic
    from sparc_gym_amd.puzzles import process_puzzles
    return process_puzzles(synthetic.make_puzzles(cnt, seed=b, sizes=sizes, full_properties=full))


def make_pool(P, sizes, full, workers=8):
    """The bench's synthetic pool of P processed puzzles: blocks of 1,024 records, block b drawn
    by synthetic.make_puzzles(seed=b), so the default 1,024-puzzle pool is block 0 and a larger
    pool extends it.  Blocks are generated in worker processes (fork, before any GPU call;
    SPARC_POOL_WORKERS=1: in this process, e.g. under a profiler that initialises the GPU
    first).  SPARC_POOL_CACHE=<dir>: the pool is kept there as a pickle this function wrote."""
    import pickle
    cache = os.environ.get("SPARC_POOL_CACHE")
    path = os.path.join(cache, f"pool_{P}_{'_'.join('%dx%d' % s for s in sizes)}_{int(bool(full))}.pkl") if cache else None
    if path and os.path.exists(path):
        with open(path, "rb") as f:
            return pickle.load(f)
    workers = int(os.environ.get("SPARC_POOL_WORKERS", workers))
    blocks = [(b, min(1024, P - 1024 * b), sizes, full) for b in range((P + 1023) // 1024)]
    if len(blocks) == 1 or workers <= 1:
        pool = [p for blk in map(_pool_block, blocks) for p in blk]
    else:
        import concurrent.futures as cf
        import multiprocessing as mp
        with cf.ProcessPoolExecutor(min(workers, len(blocks)), mp_context=mp.get_context("fork")) as ex:
            pool = [p for blk in ex.map(_pool_block, blocks) for p in blk]
    if path:
        os.makedirs(cache, exist_ok=True)
        with open(path, "wb") as f:
            pickle.dump(pool, f)
    return pool


def state_bytes_per_env(words, traceback):
    """HBM bytes one launch loads AND stores per env for its state (k_rollout / k_step):
    visited 8*words + dir stack 16*words (traceback) + pos/aux/step/pid 16."""
    return 8 * words + (16 * words if traceback else 0) + 16


def cpu_procs(world, usable=None):
    """CPU-baseline processes for a job of `world` GPUs: the host cores available to the job, one
    GPU's 16-core share per rank (the GPU box's process rules), at most the cores this process may
    run on."""
    if usable is None:
        usable = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    return max(1, min(16 * max(1, int(world)), int(usable)))


def cpu_baseline_rules(proc, tb, max_steps, seconds, procs=0):
    """The reference's full step() including its rule audit, on the CPU: oracle/sparc_oracle.c's
    step + oracle/sparc_rules_oracle.c's port of _validate_rules TWICE per step, as the reference
    runs it (SPaRC_Gym.py:1227 with the step's flags, and 1011 in _get_info with both False), one
    env per thread, counter-hash random actions (the C port, as every other config's baseline),
    and beside it the pure-Python restatements (oracle/cpu_ref.py + oracle/rules_ref.py, the
    reference's own speed).  Next-step autoreset as the GPU kernel counts it: the step after a
    done step is the reset (reset() -> _load_puzzle 182 and _get_info 1011: two audits), one
    env-step."""
    from oracle import COracle, RulesCOracle
    from oracle.cpu_ref import CpuRefEnv
    from oracle import rules_ref
    pool = [{"x_size": p["x_size"], "y_size": p["y_size"], "start": list(p["start_location"]),
             "target": list(p["target_location"]), "solution_count": p["solution_count"],
             "solution_paths": p["solution_paths"], "gaps": p["obs_array"]["gaps"]} for p in proc]
    refp = [dict(p) for p in proc]

    def run_c(secs):
        o = COracle(pool, 1, tb, max_steps, autoreset=1)
        o.reset([0])
        ro = RulesCOracle(proc)
        k, t1 = 0, time.perf_counter()
        while time.perf_counter() - t1 < secs:
            k += ro.rollout(o.pool, o.envs[0], 2000, seed=1, traceback=tb, max_steps=max_steps, audits=2)
        return k, time.perf_counter() - t1

    def run_py(audits, secs):
        rng = np.random.default_rng(0)
        q = 0
        env = CpuRefEnv(pool[q], tb, max_steps)
        pending = False
        k, t1 = 0, time.perf_counter()
        while time.perf_counter() - t1 < secs:
            if pending:                  # the autoreset step (its action is ignored)
                q = (q + 1) % len(pool)
                env.p = pool[q]
                env.reset()
                term = trunc = pending = False
            else:
                _, term, trunc = env.step(int(rng.integers(4)))
                pending = term or trunc
            rules_ref.audit(refp[q], env.path, env.loc, term, trunc)
            if audits == 2:
                rules_ref.audit(refp[q], env.path, env.loc, False, False)
            k += 1
        return k, time.perf_counter() - t1

    kc, dtc = run_c(min(seconds, 5.0))
    k, dt = run_py(2, min(seconds, 5.0))
    k1, dt1 = run_py(1, min(seconds, 3.0))
    cpu = f"CPU {platform.processor() or platform.machine()}, os.cpu_count()={os.cpu_count()}"
    out = {"value": round(kc / dtc, 1), "unit": "env-steps/s", "cores": 1, "kind": "port",
           "sample": f"oracle/sparc_oracle.c step() + oracle/sparc_rules_oracle.c rule audit twice per step as the "
                     f"reference (SPaRC_Gym.py:1227, 1011), 1 env, {kc} steps incl. next-step autoreset steps, "
                     f"random actions, {dtc:.1f} s, 1 thread; {cpu}",
           "value_1core": round(kc / dtc, 1),
           "python_port_value": round(k / dt, 1),
           "python_port_sample": f"oracle/cpu_ref.py step() + oracle/rules_ref.py audit twice per step (pure Python, "
                                 f"the reference's algorithms), 1 env, {k} steps, {dt:.1f} s, 1 thread",
           "python_port_value_audit_once": round(k1 / dt1, 1)}
    # the same on one process per core of this GPU's share of the host (BASELINE.md's plan)
    mc = _cpu_bench_multi("c3r", "c_rules", max_steps, seconds, procs)
    if mc:
        out.update(value=mc["value"], cores=mc["procs"],
                   sample=out["sample"] + f"; value: {mc['procs']} processes x 1 env, {mc['seconds']:.0f} s "
                                          f"(oracle/cpu_bench.py --impl c_rules, two audits per step)")
    mp_ = _cpu_bench_multi("c3r", "py_rules", max_steps, min(seconds, 5.0), procs)
    if mp_:
        out["python_port_multicore"] = {"value": mp_["value"], "procs": mp_["procs"],
                                        "sample": "oracle/cpu_bench.py --impl py_rules, two audits per step"}
    return out


def cpu_baseline(proc, tb, max_steps, seconds, obs_dims=None, config="c3", procs=0):
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
    q, pending = 0, False
    k, t1 = 0, time.perf_counter()
    while time.perf_counter() - t1 < min(3.0, seconds):
        if pending:          # next-step autoreset: one env-step, as the GPU kernel counts it
            q = (q + 1) % len(pool)
            env.p = pool[q]
            env.reset()
            pending = False
        else:
            _, term, trunc = env.step(int(rng.integers(4)))
            pending = term or trunc
        k += 1
    py_rate = k / (time.perf_counter() - t1)
    out = {"value": round(c_rate, 1), "unit": "env-steps/s", "cores": 1, "kind": "port",
           "sample": f"oracle/sparc_oracle.c, {n} envs x {steps} steps, random actions, next-step autoreset, "
                     f"{'visited + agent_location planes written every step, ' if obs_dims else ''}"
                     f"1 thread, {dt:.1f} s; CPU {platform.processor() or platform.machine()}, "
                     f"os.cpu_count()={os.cpu_count()}",
           "value_1core": round(c_rate, 1),
           "python_port_value": round(py_rate, 1),
           "python_port_sample": "oracle/cpu_ref.py (reference step() restated in pure Python, no rule "
                                 f"audit), 1 env, {k} steps incl. next-step autoreset steps, 1 thread"}
    # the same oracle, one process per core (BASELINE.md CPU-baseline plan), in a child process
    # that never touches the GPU; up to 16 cores (one GPU's share of the box)
    cmd = [sys.executable, "-m", "oracle.cpu_bench", "--config", config, "--seconds", str(seconds),
           "--max-steps", str(max_steps), "--procs", str(procs)] + \
        (["--obs", str(obs_dims[0]), str(obs_dims[1])] if obs_dims else [])
    try:
        r = subprocess.run(cmd, cwd=REPO, capture_output=True, text=True, timeout=seconds * 4 + 120)
        mc = json.loads(r.stdout.strip().splitlines()[-1])
        phys, logical, aff, quota = physical_cores()
        out.update(value=mc["value"], cores=mc["procs"],
                   sample=out["sample"] +
                   f"; value: {mc['procs']} processes x {n} envs (oracle/cpu_bench.py), "
                   f"{mc['seconds']:.0f} s, one per core of the job's share of the host",
                   per_core=round(mc["value"] / mc["procs"], 1),
                   host={"physical_cores": phys, "logical_cpus": logical, "affinity_cpus": aff,
                         "cgroup_cpu_quota": quota,
                         "note": "the GPU box gives a job a 16-core share per GPU (its process rules); "
                                 "whole_host_estimate = per_core x physical_cores is a linear estimate, "
                                 "not a measurement"})
        if phys:
            out["whole_host_estimate"] = round(mc["value"] / mc["procs"] * phys, 1)
    except (subprocess.SubprocessError, ValueError, KeyError, IndexError) as exc:   # keep the 1-core number
        out["multi_core_error"] = repr(exc)[:200]
    if not obs_dims:   # the pure-Python port on the same cores (one process per core)
        mp_ = _cpu_bench_multi(config, "py", max_steps, seconds, procs)
        if mp_:
            out["python_port_multicore"] = {"value": mp_["value"], "procs": mp_["procs"],
                                            "sample": f"oracle/cpu_ref.py, {mp_['procs']} processes x 1 env, "
                                                      f"{mp_['seconds']:.0f} s (oracle/cpu_bench.py --impl py)"}
    return out


def _cpu_bench_multi(config, impl, max_steps, seconds, procs=0):
    """oracle/cpu_bench.py in a child process (never touches the GPU); its JSON or None."""
    cmd = [sys.executable, "-m", "oracle.cpu_bench", "--config", config, "--seconds", str(seconds),
           "--max-steps", str(max_steps), "--impl", impl, "--procs", str(procs)]
    try:
        r = subprocess.run(cmd, cwd=REPO, capture_output=True, text=True, timeout=seconds * 4 + 120)
        return json.loads(r.stdout.strip().splitlines()[-1])
    except (subprocess.SubprocessError, ValueError, IndexError):
        return None


def achievable_bw(dev, gib=2, reps=10):
    """Achievable HBM bandwidth on THIS box, measured in the same run as the bench line (SURVEY
    §8d): torch's fill_ (pure stores, the c4 plane writer's traffic) and copy_ (read + write) over
    a `gib` GiB buffer, `reps` launches after two warm-ups, HIP events; GB/s = 1e9 B/s."""
    import torch
    n = gib << 30
    a = torch.empty(n, dtype=torch.uint8, device=dev)
    b = torch.empty(n, dtype=torch.uint8, device=dev)
    out = {}
    for name, fn, moved in (("store", lambda k: a.fill_(k & 0xFF), n), ("copy", lambda k: b.copy_(a), 2 * n)):
        fn(1)
        fn(2)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for k in range(reps):
            fn(k)
        e1.record()
        e1.synchronize()
        out[f"{name}_gbs"] = round(moved * reps / (e0.elapsed_time(e1) * 1e-3) / 1e9, 1)
    del a, b
    torch.cuda.empty_cache()
    return out


def csrc_hash():
    """sha256 (16 hex) of the kernel sources + ABI header + Makefile: the build a committed
    counter summary belongs to."""
    import hashlib
    h = hashlib.sha256()
    for f in csrc_files():
        h.update(f.encode())
        h.update(open(os.path.join(REPO, f), "rb").read())
    return h.hexdigest()[:16]


def load_traffic(workload, kernel):
    """The committed rocprofv3 --pmc summary of this workload's kernel (profiles/pmc_traffic.json,
    written by tools/pmc_traffic.py): {"bytes": HBM bytes per launch, "counters": SQ counters
    per launch, "csrc_hash": ...}, or None when absent or recorded for other kernel sources
    (then bench reports traffic: null rather than another build's counters)."""
    path = os.path.join(REPO, "profiles", "pmc_traffic.json")
    if not os.path.exists(path):
        return None
    try:
        e = json.load(open(path)).get(workload, {}).get(kernel)
    except (OSError, ValueError):
        return None
    if not isinstance(e, dict) or e.get("csrc_hash") != csrc_hash():
        return None
    return e


def physical_cores():
    """(physical cores, logical CPUs) of the host from /proc/cpuinfo, and the CPUs this process
    may use: its affinity set and its cgroup CPU quota (cpu.max), as (affinity, quota)."""
    phys, logical = set(), 0
    try:
        cur = {}
        for line in open("/proc/cpuinfo"):
            if not line.strip():
                if cur:
                    logical += 1
                    phys.add((cur.get("physical id"), cur.get("core id")))
                cur = {}
                continue
            k, _, v = line.partition(":")
            cur[k.strip()] = v.strip()
        if cur:
            logical += 1
            phys.add((cur.get("physical id"), cur.get("core id")))
    except OSError:
        pass
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        quota = None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    return len(phys) or None, logical or os.cpu_count(), aff, quota


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n, argv, extra_env=None, poll_s=0.2):
    """Start n rank processes of ``argv`` (one per GPU: LOCAL_RANK = RANK = r, WORLD_SIZE = n,
    rendezvous on 127.0.0.1) as children of a parent that never touches the GPU, and wait for
    them.  Returns the exit code: 0 when every rank succeeded, else the first failing rank's code
    (the other ranks are then terminated by PID, so none is left waiting in a collective)."""
    port = free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), GROUP_RANK="0")
        env.update(extra_env or {})
        procs.append(subprocess.Popen(argv, env=env))
    rc = 0
    live = list(procs)
    while live:
        time.sleep(poll_s)
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 128 - code
                for q in live:
                    q.terminate()
    for p in procs:
        try:
            p.wait(timeout=30)
        except subprocess.TimeoutExpired:
            p.kill()
            p.wait()
    return rc


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # `python bench.py --gpus N` (no torchrun): one rank process per GPU, started before
        # this process imports torch or makes any GPU call
        return launch_ranks(args.gpus, [sys.executable, os.path.abspath(__file__)] + sys.argv[1:],
                            {"SPARC_BENCH_LAUNCHER": "1"})
    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    if world_env != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world_env}: the job would not measure "
                         f"{args.gpus} GPUs")
    sizes, full, tb, obs = CONFIGS[args.config]
    proc = make_pool(args.puzzles, sizes, full)   # before torch / any GPU call (worker processes fork)
    import torch
    import torch.distributed as dist
    from sparc_gym_amd import SPaRCVecEnv
    from sparc_gym_amd import dist as sdist
    from sparc_gym_amd.puzzles import pack_table

    ndev = torch.cuda.device_count()
    local_env = int(os.environ.get("LOCAL_RANK", "0"))
    if local_env >= ndev and not args.rehearsal:
        raise SystemExit(f"LOCAL_RANK {local_env} but only {ndev} GPU(s) visible: one rank per GPU "
                         f"(--rehearsal lets ranks share GPUs, for tests only)")
    rank, world, local = sdist.init_from_env(args.backend, device=local_env % max(1, ndev))
    local = local_env % max(1, ndev)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    # which physical GPU each rank drives (PCI domain / bus / device): distinct unless rehearsing
    props = torch.cuda.get_device_properties(dev)
    ident = sdist.gather_values([rank, local, props.pci_domain_id, props.pci_bus_id, props.pci_device_id], dev)
    pci = [tuple(int(v) for v in r[2:]) for r in ident]
    if world != args.gpus or (len(set(pci)) != len(pci) and not args.rehearsal):
        raise SystemExit(f"rank {rank}: world {world} (asked {args.gpus}), GPUs per rank {pci}: need one "
                         f"distinct GPU per rank (--rehearsal lets ranks share GPUs, for tests only)")

    if args.envs <= 0:
        args.envs = DEFAULT_ENVS[args.config]
    table = pack_table(proc)
    offset, n = sdist.env_shard(args.envs, rank)
    vec = SPaRCVecEnv(n, processed=proc, table=table, traceback=tb, max_steps=args.max_steps,
                      autoreset="next_step", device=local, env_offset=offset, observation="compact")
    gid = np.arange(offset, offset + n, dtype=np.uint64)
    pidx, placement = initial_puzzles(gid, len(proc), args.placement)
    vec.reset(options={"puzzle_index": pidx})

    K, W = max(1, args.steps), max(0, args.warmup)
    # env-steps per env in one bench step (one launch)
    rules = args.config in RULE_CONFIGS
    # env-steps per launch: 2,000 (as c3; c3r too: its step + audit waves fill a pipeline of
    # 10-step tiles per launch), 50 with observation traces (c4: 12.7 GB of planes per launch)
    T = 1 if args.mode == "step" else (args.chunk if args.chunk > 0 else (50 if obs else 2000))
    chunk = T
    # observation traces [T, N, x_dim, y_dim] int32 (visited, agent_location), reused by every
    # launch (a consumer reads them between launches)
    X, Y = vec.x_dim, vec.y_dim
    plane_bytes = X * Y * 4
    ovis = oag = None
    if obs:
        ovis = torch.empty((T, n, X, Y), dtype=torch.int32, device=dev)
        oag = torch.empty_like(ovis)
    RA, RO = min(max(K, W), 8), min(max(K, W), 2)   # distinct action tiles / output tiles
    # action tile j = env.action_space.sample() for every env and step, drawn on the GPU by the
    # counter-based generator keyed by the GLOBAL env id (sparc_rand_action(ACTION_SEED,
    # env_offset + i, j * T + t)): the ranks' shards together hold exactly the tiles of one
    # process over all world * n envs
    actions = torch.empty((RA, T, n), dtype=torch.uint8, device=dev)
    for j in range(RA):
        vec.random_actions(T, seed=ACTION_SEED, t0=j * T, out=actions[j])
    rew = torch.empty((RO, T, n), dtype=torch.int8, device=dev)
    flags = torch.empty((RO, T, n), dtype=torch.uint8, device=dev)
    stats = torch.zeros((n, 4), dtype=torch.int32, device=dev)
    rbits = None
    if rules:   # rule bits of every step [T, N] int16, as rollout(rules=True)
        vec._load_rules()
        rbits = torch.empty((RO, T, n), dtype=torch.int16, device=dev)
    stream = torch.cuda.current_stream(dev)

    vec._stream()                       # bind the context to this (torch's current) stream
    core = vec.core
    s_ptr = stats.data_ptr()

    def run(k0, k1, events=None):
        """Bench steps k0..k1-1: direct C-ABI calls on pre-validated buffers (vec.rollout()
        checks shapes per call), each bracketed by HIP events on the launch stream."""
        for k in range(k0, k1):
            ap, rp, fp = actions[k % RA].data_ptr(), rew[k % RO].data_ptr(), flags[k % RO].data_ptr()
            ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) if events is not None else None
            if ev:
                ev[0].record(stream)
            if args.mode == "step":
                core.step_device(ap, rp, fp)
            elif obs:
                core.rollout_obs_device(T, ap, rp, fp, s_ptr, ovis.data_ptr(), oag.data_ptr(), X, Y)
            elif rules:
                core.rollout_rules_device(T, ap, rp, fp, s_ptr, rbits[k % RO].data_ptr())
            else:
                core.rollout_device(T, ap, rp, fp, s_ptr)
            if ev:
                ev[1].record(stream)
                events.append((ev, T))

    # warmup (untimed), and one untimed end-of-batch gather so that RCCL's first-call setup is
    # not inside the timed region
    run(0, W)
    torch.cuda.synchronize(dev)
    sdist.gather_stats(stats)
    torch.cuda.synchronize(dev)
    stats.zero_()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    events = []
    t0 = time.perf_counter()
    run(W, W + K, events)
    # end-of-batch gather of per-env summaries (reward sum, dones, solved, resets): one RCCL call
    gathered = sdist.gather_stats(stats)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = sdist.max_over_ranks(t1 - t0, dev)
    summary = sdist.summarize(gathered)

    if rank == 0 and args.stats_out:
        np.save(args.stats_out, gathered.cpu().numpy())
    kern_ms = [a.elapsed_time(b) for (a, b), _ in events]
    steps_per_launch = [c for _, c in events]
    avg_ms = float(np.mean(kern_ms))
    rank_ms = sdist.gather_values([avg_ms, t1 - t0], dev)   # per rank: kernel ms, wall s
    avg_T = float(np.mean(steps_per_launch))
    value = world * n * T * K / elapsed
    # algorithmic HBM bytes per launch: per env-step action 1 + reward 1 + flags 1; per env and
    # launch the state (load + store) and, for rollouts, the stats record (load + store)
    sb = state_bytes_per_env(table.words, tb)
    # rule rollouts: k_rollout1r (every puzzle in the region-code table: no exact-fit memo) or the
    # generic k_rollout<..., RULES> (the per-env memo loaded and stored, 48 B each way)
    rule_kernel = rule_rollout_kernel(proc, table) if rules else None
    memo_bytes = 96 if rule_kernel == "k_rollout" else 0
    per_env_launch = 2 * sb + (32 if args.mode == "rollout" else 0) + memo_bytes
    per_step = 3 + (2 * plane_bytes if obs and args.mode == "rollout" else 0) + (2 if rules else 0)
    bytes_launch = n * (per_step * avg_T + per_env_launch)
    achieved = bytes_launch / (avg_ms * 1e-3) / 1e9
    if args.mode != "rollout":
        kernel = "k_step"
    elif rules:
        kernel = rule_kernel     # the audit after every step
    elif table.words == 1 and not obs:
        # batches of whole 256-env workgroups: the split move / trie kernel
        kernel = "k_rollout1s" if n % 256 == 0 and chunk >= 16 else "k_rollout1"
    elif not obs and n % 256 == 0 and chunk >= 16:
        kernel = "k_rolloutWs"   # the multi-word split kernel (when the pool fits its LDS layout)
    elif obs:
        kernel = "k_rollout_obsw"   # the 'new' planes by writer waves (256-env workgroups)
    else:
        kernel = "k_rollout"
    workload = f"{args.config}_{args.mode}_n{n}_chunk{chunk if args.mode == 'rollout' else 1}"
    if args.puzzles != 1024:   # the counters of another pool size are recorded under their own key
        workload += f"_p{args.puzzles}"
    if placement == "xcd":
        workload += "_xcd"
    pmc = load_traffic(workload, kernel)
    traffic = pmc["bytes"] if pmc else None
    issue = None
    if pmc and "SQ_INSTS_VALU" in pmc.get("counters", {}):
        valu = pmc["counters"]["SQ_INSTS_VALU"]
        wave_steps = n / 64.0 * avg_T
        issue = {"valu_wave_insts_per_launch": int(valu),
                 "valu_per_wave_step": round(valu / wave_steps, 2),
                 "salu_per_wave_step": round(pmc["counters"].get("SQ_INSTS_SALU", 0) / wave_steps, 2),
                 "lds_per_wave_step": round(pmc["counters"].get("SQ_INSTS_LDS", 0) / wave_steps, 2),
                 "peak_wave_insts_per_s": VALU_PEAK_WAVE_INSTS,
                 "frac": round(valu / (avg_ms * 1e-3) / VALU_PEAK_WAVE_INSTS, 4),
                 "note": "VALU issue roofline: SQ_INSTS_VALU of the committed PMC pass / the live kernel time / "
                         "(1,024 SIMDs x one wave64 VALU per 2 cycles x 2.4 GHz)"}
    # the HBM-bound configuration (observation planes: ~99 % of its bytes are plane stores) gets
    # this box's achievable store bandwidth beside the 8 TB/s peak
    ach = achievable_bw(dev) if obs and args.mode == "rollout" else None
    backend = dist.get_backend() if dist.is_initialized() else None
    observed_world = dist.get_world_size() if dist.is_initialized() else 1
    out = {
        "metric": "env-steps/sec at 65,536 envs, 7x7 grid (HBM roofline fraction in 'roofline')",
        "value": round(value, 1),
        "unit": "env-steps/s",
        "n_gpus": world,
        "world_observed": {"world_size": observed_world, "backend": backend, "gpus_visible": ndev,
                           "rehearsal": bool(args.rehearsal),
                           "distinct_gpus": len(set(pci)),
                           "rank_gpu_pci": [list(p) for p in pci],
                           "per_rank_kernel_ms": [round(r[0], 4) for r in rank_ms],
                           "per_rank_wall_s": [round(r[1], 6) for r in rank_ms],
                           "launcher": ("bench.py (child per rank)" if os.environ.get("SPARC_BENCH_LAUNCHER")
                                        else "torchrun" if "TORCHELASTIC_RUN_ID" in os.environ
                                        else "external" if world > 1 else "none")},
        "steps": K,
        "warmup": W,
        "ms_per_step": round(elapsed * 1e3 / K, 6),   # per bench step: T env-steps of every env
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8/u64 (integer bitboards)",
        "data": "synthetic SPaRC-schema puzzles (sparc_gym_amd.synthetic, seed 0); uniform random actions in HBM "
                "(sparc_rand_action of the global env id, drawn before the timed region)",
        "config": {"workload": f"{args.config}: {n} envs/GPU, lattices {['%dx%d' % (2*w+1, 2*h+1) for w, h in sizes]}, "
                               f"{'full property set' if full else 'base planes'}, traceback={tb}, "
                               f"max_steps={args.max_steps}, next-step autoreset, {args.puzzles} puzzles"
                               + (", XCD-local first puzzles (bench.initial_puzzles)" if placement == "xcd" else "")
                               + (f", observation='new': visited + agent_location int32 planes "
                                  f"[N, {X}, {Y}] written every step" if obs else "")
                               + (", rule audit (info['rule_status'] bits, SPaRC_Gym.py:941-950) after "
                                  "every step" if rules else ""),
                   "mode": args.mode, "envs_per_gpu": n, "env_steps_per_bench_step": T,
                   "env_steps_per_launch": T,
                   "parallelism": f"dp{world} (env shards, "
                                  f"{'RCCL' if backend == 'nccl' else (backend or 'no')} "
                                  f"all_gather of per-env stats at end of batch)"},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 6), "traffic": traffic,
                     "traffic_source": (f"profiles/pmc_traffic.json [{workload}][{kernel}], csrc {csrc_hash()}"
                                        if pmc else f"none recorded for csrc {csrc_hash()}"),
                     "issue": issue,
                     **({"achievable_gbs": ach["store_gbs"], "frac_of_achievable": round(achieved / ach["store_gbs"], 4),
                         "achievable": dict(ach, source="torch fill_ (stores) / copy_ (read + write) over 2 GiB, 10 "
                                                        "launches, this box, this run")} if ach else {}),
                     "kernel": kernel, "kernel_avg_ms": round(avg_ms, 4), "launches": len(kern_ms),
                     "algorithmic_bytes_per_launch": int(bytes_launch),
                     "bytes_model": f"per env-step {per_step} B (action, reward code, flags"
                                    f"{f', visited + agent_location planes 2 x {plane_bytes} B' if obs else ''}"
                                    f"{', rule bits 2 B' if rules else ''}"
                                    f"); per env per launch "
                                    f"{per_env_launch} B (state {sb} B load+store"
                                    f"{', stats 16 B load+store' if args.mode == 'rollout' else ''}"
                                    f"{', exact-fit memo 48 B load+store' if memo_bytes else ''})"},
        "episodes": summary,
    }
    if world > 1:
        dist.destroy_process_group()
    # the CPU step() beside the GPU number at EVERY world size (north_star: "next to the reference
    # Python CPU step() timed on the host cores of the same box in the same run"): rank 0, after
    # the timed region and the final barrier, on the host cores the job has (cpu_procs)
    if rank == 0 and not args.no_cpu_baseline:
        procs = cpu_procs(len(set(pci)))   # the GPUs the job drives (a rehearsal shares one)
        if rules:
            cb = cpu_baseline_rules(proc, tb, args.max_steps, args.cpu_seconds, procs)
        else:
            cb = cpu_baseline(proc, tb, args.max_steps, args.cpu_seconds, (X, Y) if obs else None, args.config,
                              procs)
        out["cpu_baseline"] = cb
        out["gpu_vs_cpu"] = round(value / cb["value"], 1)
    elif rank == 0:
        out["cpu_baseline"] = None
    if rank == 0:
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    sys.exit(main() or 0)
