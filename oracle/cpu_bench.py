"""Multi-process CPU baseline: the C oracle (sparc_oracle.c) on every core it is given, one
process per core.  TEST / BENCHMARK INFRASTRUCTURE ONLY: bench.py's cpu_baseline leg runs this
as a child process (it never touches the GPU) and reports its aggregate rate next to the
single-thread one, as BASELINE.md's CPU-baseline plan asks (one process per host core, core
count stated).

    python -m oracle.cpu_bench --config c3 --procs 16 --seconds 10 [--obs X Y] [--impl c|py|py_rules]

Each process runs 1,024 envs of the bench pool (synthetic seed 0, the same puzzle assignment as
bench.py) with counter-based random actions and next-step autoreset, for `seconds`; with
--obs it also writes the visited / agent_location planes of every step (config c4).  Prints
one JSON line: {"value": env-steps/s summed over processes, "procs": P, ...}.

--impl c_rules runs one env per process through sparc_oracle.c's step plus the C port of the rule
audit (sparc_rules_oracle.c) twice per step: the c3r baseline at C speed.
--impl py runs the pure-Python restatement instead (oracle/cpu_ref.py: the reference's step()
core at reference speed, one env at a time), --impl py_rules the same plus the rule audit of
oracle/rules_ref.py twice per step, as the reference's full step() runs _validate_rules (941-950) at
1227 and again in _get_info (1011).  Autoreset steps count as env-steps, as on the GPU.
"""
from __future__ import annotations

import argparse
import json
import multiprocessing as mp
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CONFIGS = {   # name: (grid sizes, full property set, traceback) — as bench.CONFIGS
    "c2": (((3, 3),), False, False),
    "c3": (((3, 3),), True, True),
    "c3r": (((3, 3),), True, True),
    "c4": (((2, 2), (3, 3), (4, 4), (5, 5)), True, True),
    "c4c": (((2, 2), (3, 3), (4, 4), (5, 5)), True, True),
    "c3g7": (((7, 7),), True, True),
}


def make_proc(config, n_puzzles):
    sys.path.insert(0, os.path.join(REPO, "sparc-gym_amd"))
    from sparc_gym_amd import synthetic                      # host-side only: no HIP library
    from sparc_gym_amd.puzzles import process_puzzles
    sizes, full, _ = CONFIGS[config]
    return process_puzzles(synthetic.make_puzzles(n_puzzles, seed=0, sizes=sizes, full_properties=full))


def make_pool(config, n_puzzles):
    sys.path.insert(0, os.path.join(REPO, "sparc-gym_amd"))
    from sparc_gym_amd import synthetic                      # host-side only: no HIP library
    from sparc_gym_amd.puzzles import process_puzzles
    sizes, full, _ = CONFIGS[config]
    proc = process_puzzles(synthetic.make_puzzles(n_puzzles, seed=0, sizes=sizes, full_properties=full))
    return [{"x_size": p["x_size"], "y_size": p["y_size"], "start": list(p["start_location"]),
             "target": list(p["target_location"]), "solution_count": p["solution_count"],
             "solution_paths": p["solution_paths"], "gaps": p["obs_array"]["gaps"]} for p in proc]


def _worker(args):
    pool, tb, max_steps, seconds, obs, rank = args
    from oracle import COracle
    n, T = 1024, 64
    o = COracle(pool, n, tb, max_steps, autoreset=1)
    gid = np.arange(rank * n, (rank + 1) * n, dtype=np.uint64)
    o.reset((gid * 2654435761 % len(pool)).astype(np.int64))
    steps = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        if obs:
            o.rollout_obs(T, obs[0], obs[1], None, seed=1, env_offset=rank * n, t0=steps)
        else:
            o.rollout(T, None, seed=1, env_offset=rank * n, t0=steps)
        steps += T
    return n * steps, time.perf_counter() - t0


def _worker_c_rules(args):
    """One env through oracle/sparc_rules_oracle.c's oracle_rules_rollout: sparc_oracle.c's step
    plus the C port of the rule audit twice per step (SPaRC_Gym.py:1227 and 1011), next-step
    autoreset onto the next puzzle (the reset step audits twice too: 182, 1011), counter-hash
    random actions."""
    proc, tb, max_steps, seconds, rank = args
    from oracle import COracle, RulesCOracle
    pool = [{"x_size": p["x_size"], "y_size": p["y_size"], "start": list(p["start_location"]),
             "target": list(p["target_location"]), "solution_count": p["solution_count"],
             "solution_paths": p["solution_paths"], "gaps": p["obs_array"]["gaps"]} for p in proc]
    o = COracle(pool, 1, tb, max_steps, autoreset=1)
    o.reset([(rank * 2654435761) % len(pool)])
    ro = RulesCOracle(proc)
    k, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        k += ro.rollout(o.pool, o.envs[0], 2000, seed=1 + rank, traceback=tb, max_steps=max_steps, audits=2)
    return k, time.perf_counter() - t0


def _worker_py(args):
    """One env at a time through oracle/cpu_ref.py (+ oracle/rules_ref.py's audit twice per step,
    SPaRC_Gym.py:1227 and 1011).  Next-step autoreset counted as the GPU kernel and the C oracle
    count it: the step after a done step is the reset (reset() audits twice too: 182, 1011), one
    env-step."""
    proc, tb, max_steps, seconds, rules, rank = args
    from oracle.cpu_ref import CpuRefEnv
    from oracle import rules_ref
    pool = [{"x_size": p["x_size"], "y_size": p["y_size"], "start": list(p["start_location"]),
             "target": list(p["target_location"]), "solution_count": p["solution_count"],
             "solution_paths": p["solution_paths"], "gaps": p["obs_array"]["gaps"]} for p in proc]
    rng = np.random.default_rng(rank)
    q = (rank * 2654435761) % len(pool)
    env = CpuRefEnv(pool[q], tb, max_steps)
    pending = False
    k, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        if pending:
            q = (q + 1) % len(pool)
            env.p = pool[q]
            env.reset()
            term = trunc = pending = False
        else:
            _, term, trunc = env.step(int(rng.integers(4)))
            pending = term or trunc
        if rules:
            rules_ref.audit(proc[q], env.path, env.loc, term, trunc)
            rules_ref.audit(proc[q], env.path, env.loc, False, False)
        k += 1
    return k, time.perf_counter() - t0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--procs", type=int, default=0, help="0 = min(16, usable cores)")
    ap.add_argument("--seconds", type=float, default=10.0)
    ap.add_argument("--puzzles", type=int, default=1024)
    ap.add_argument("--max-steps", type=int, default=2000)
    ap.add_argument("--obs", type=int, nargs=2, default=None, metavar=("X", "Y"))
    ap.add_argument("--impl", default="c", choices=["c", "py", "py_rules", "c_rules"])
    a = ap.parse_args()
    usable = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    procs = a.procs if a.procs > 0 else max(1, min(16, usable))
    tb = CONFIGS[a.config][2]
    if a.impl == "c":
        pool = make_pool(a.config, a.puzzles)
        from oracle import build
        build()                                                  # compile once, before forking
        with mp.get_context("fork").Pool(procs) as p:
            res = p.map(_worker, [(pool, tb, a.max_steps, a.seconds, a.obs, r) for r in range(procs)])
    elif a.impl == "c_rules":
        proc = make_proc(a.config, a.puzzles)
        from oracle import build
        build()
        with mp.get_context("fork").Pool(procs) as p:
            res = p.map(_worker_c_rules, [(proc, tb, a.max_steps, a.seconds, r) for r in range(procs)])
    else:
        proc = make_proc(a.config, a.puzzles)
        with mp.get_context("fork").Pool(procs) as p:
            res = p.map(_worker_py, [(proc, tb, a.max_steps, a.seconds, a.impl == "py_rules", r)
                                     for r in range(procs)])
    value = sum(s / dt for s, dt in res)
    print(json.dumps({"value": round(value, 1), "procs": procs, "usable_cores": usable,
                      "os_cpu_count": os.cpu_count(), "config": a.config, "seconds": a.seconds,
                      "env_steps": int(sum(s for s, _ in res)), "obs": a.obs, "impl": a.impl}))


if __name__ == "__main__":
    main()
