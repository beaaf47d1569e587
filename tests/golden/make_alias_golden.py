"""Generate tests/golden/alias_*.json.gz: the reference's plane aliasing across re-loads.

`_load_puzzle` binds the puzzle's observation planes without copying (SPaRC_Gym.py:149-151),
and `step()` edits them in place (1141-1188), so a puzzle loaded again by the same env object
starts from the previous episode's `visited` / `agent_location` planes.  The stale `visited`
bits are not cosmetic: `_get_legal_actions` (1040) and `step` (1141) read that plane, so they
change which moves are legal, and `_rule_all_dots_collected` (529) reads it too.

Unlike make_golden.py, the episodes here do NOT restore pristine puzzles: one env object plays
many episodes over a few puzzles (re-loads on purpose), and every reset and step is recorded
(the reward, flags, legal actions, both planes and the full rule_status), so the drop-in's
`alias_compat=True` mode is pinned to the reference itself.  Same recipe as make_golden.py
(unmodified reference, stubbed gymnasium / pygame, patched load_dataset).

Usage:  python tests/golden/make_alias_golden.py
"""
from __future__ import annotations

import gzip
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
sys.path.insert(0, REPO)
import make_golden as mg  # noqa: E402
from oracle.rules_ref import normalize  # noqa: E402
from sparc_gym_amd import synthetic  # noqa: E402


def snapshot(obs, info):
    return {"visited": mg.plane(obs["base"]["visited"]), "agent_plane": mg.plane(obs["base"]["agent_location"]),
            "info": mg.info_dict(info), "rule_status": normalize(info["rule_status"])}


def alias_episodes(records, tb, max_steps, n_eps, seed, tag, n_puzzles=3, max_len=60):
    env = mg.make_env(records, traceback=tb, max_steps=max_steps)
    rng = np.random.default_rng(seed)
    strategies = ["random", "legal", "solution", "solution_detour"]
    eps = []
    for e in range(n_eps):
        idx = int(rng.integers(min(n_puzzles, len(env.puzzles))))
        pid = env.puzzles[idx]["id"]
        obs, info = env.reset(options={"puzzle_id": pid})
        rec = {"puzzle_index": idx, "puzzle_id": str(pid), "strategy": strategies[e % 4],
               "reset": snapshot(obs, info), "actions": [], "steps": []}
        sols = env.solution_paths[:env.solution_count]
        plan = []
        if rec["strategy"].startswith("solution") and sols:
            plan = mg.sol_actions(sols[int(rng.integers(len(sols)))])
            if rec["strategy"] == "solution_detour" and len(plan) > 3:
                k = int(rng.integers(1, len(plan) - 1))
                d = int(rng.integers(4))
                plan = plan[:k] + [d, (d + 2) % 4] + plan[k:]
        for t in range(int(rng.integers(5, max_len))):
            if plan:
                a = plan.pop(0)
            elif rec["strategy"] == "legal":
                la = info["legal_actions"]
                a = int(la[int(rng.integers(len(la)))]) if la else 0
            else:
                a = int(rng.integers(4))
            obs, r, term, trunc, info = env.step(a)
            rec["actions"].append(a)
            rec["steps"].append({"reward": mg.reward_repr(r), "terminated": bool(term), "truncated": bool(trunc),
                                 **snapshot(obs, info)})
            if term or trunc:
                break
        eps.append(rec)
    return {"tag": tag, "traceback": tb, "max_steps": max_steps, "records": records, "episodes": eps}


def main():
    mg.REFMOD = mg.import_reference()
    out = {}
    poolA = synthetic.make_puzzles(6, seed=41, sizes=((3, 3),), full_properties=True)
    poolR = synthetic.make_rule_puzzles(4, seed=42, sizes=((2, 2), (3, 3)), break_prob=0.2)
    poolC = synthetic.make_puzzles(4, seed=43, sizes=((4, 4), (5, 5)), full_properties=True, max_shaped=3)
    out["alias_tb1"] = alias_episodes(poolA, True, 2000, 30, 1, "7x7 full, traceback, 3 puzzles re-loaded")
    out["alias_tb0"] = alias_episodes(poolA, False, 40, 24, 2, "7x7 full, no traceback, max_steps=40")
    out["alias_rules"] = alias_episodes(poolR, True, 2000, 24, 3, "rule-consistent 5x5 / 7x7, traceback", 2)
    out["alias_mixed"] = alias_episodes(poolC, True, 2000, 16, 4, "9x9 / 11x11 lattices, traceback", 2)
    for k, v in out.items():
        path = os.path.join(HERE, f"{k}.json.gz")
        with open(path, "wb") as f:  # mtime=0: byte-identical output on every run
            with gzip.GzipFile(fileobj=f, mode="wb", mtime=0) as g:
                g.write(json.dumps(v, separators=(",", ":"), sort_keys=True).encode())
        print(k, len(v["episodes"]), "episodes,", sum(len(e["steps"]) for e in v["episodes"]), "steps ->", path)


if __name__ == "__main__":
    main()
