#!/usr/bin/env python3
"""Latency of the drop-in single env: microseconds per SPaRC_Gym.step() and
reset() call on the GPU box, the way the reference's callers drive it (human_play.py:34-64,
llm_host.py:182-242, Final_Product.py:26-38: one env, env.step(a) -> info).

For the 7 x 7 (c3 pool) and 15 x 15 (c3g7 pool) puzzles, observation 'new' and 'SPaRC', and
rule_status True / False, it runs random-action episodes (reset on done) and reports the mean
wall time of step() and of reset().  Beside it: the bare C calls of one step (sparc_env_step with
and without the audit, one stream synchronisation each) against the previous composition
(sparc_step_host + sparc_read_state + sparc_rules_host: four or more synchronisations).  One JSON
line per measurement.  (The CPU side of the comparison is bench.py's cpu_baseline leg: the c3r
line times the reference-speed restatement of step() with its two audits per step.)"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "sparc-gym_amd"))

import numpy as np  # noqa: E402

from sparc_gym_amd import SPaRC_Gym, synthetic  # noqa: E402

POOLS = {"7x7": ((3, 3),), "15x15": ((7, 7),)}

ap = argparse.ArgumentParser()
ap.add_argument("--steps", type=int, default=2000)
ap.add_argument("--puzzles", type=int, default=256)
a = ap.parse_args()


def emit(**kw):
    print(json.dumps(kw), flush=True)


for pool, sizes in POOLS.items():
    recs = synthetic.make_puzzles(a.puzzles, seed=0, sizes=sizes, full_properties=True)
    for rule_status in (True, False):
        for observation in ("new", "SPaRC"):
            env = SPaRC_Gym(puzzles=recs, observation=observation, traceback=True, rule_status=rule_status)
            rng = np.random.default_rng(0)
            env.reset(seed=0)
            for _ in range(50):                                        # warm-up
                _, _, term, trunc, _ = env.step(int(rng.integers(4)))
                if term or trunc:
                    env.reset()
            t_step = t_reset = 0.0
            n_reset = 0
            for _ in range(a.steps):
                t0 = time.perf_counter()
                _, _, term, trunc, _ = env.step(int(rng.integers(4)))
                t_step += time.perf_counter() - t0
                if term or trunc:
                    t0 = time.perf_counter()
                    env.reset()
                    t_reset += time.perf_counter() - t0
                    n_reset += 1
            emit(kind="SPaRC_Gym", pool=pool, observation=observation, rule_status=rule_status,
                 step_us=round(t_step / a.steps * 1e6, 1), reset_us=round(t_reset / max(1, n_reset) * 1e6, 1),
                 steps=a.steps, resets=n_reset, steps_per_s=round(a.steps / t_step, 1))

    # the bare C calls of one step: the one-record entry point against the previous composition
    env = SPaRC_Gym(puzzles=recs, observation="new", traceback=True, rule_status=True)
    core = env._core
    rng = np.random.default_rng(1)
    q = 0
    for audit in (True, False):
        for legacy in (False, True):
            core.env_reset(q, audit=False)
            t = 0.0
            for k in range(a.steps):
                act = int(rng.integers(4))
                t0 = time.perf_counter()
                if legacy:
                    _, fl = core.step_host(np.array([act], np.uint8))
                    core.read_state()
                    if audit:
                        core.rules_host(region=True, fit=True)
                    f = int(fl[0])
                else:
                    f = core.env_step(act, audit=audit).flags
                t += time.perf_counter() - t0
                if f & 3:
                    q = (q + 1) % len(recs)
                    core.env_reset(q, audit=False)
            emit(kind="c_abi", pool=pool, audit=audit,
                 calls="step_host+read_state" + ("+rules_host" if audit else "") if legacy else "env_step",
                 us=round(t / a.steps * 1e6, 1))
