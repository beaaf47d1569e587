"""Generate tests/golden/rules_*.json.gz: the reference's `info['rule_status']` per step.

Same recipe as make_golden.py: the unmodified reference is imported with gymnasium / pygame
stubbed and `datasets.load_dataset` patched to a synthetic DataFrame.  Every episode
restores a pristine copy of the puzzles first (the reference aliases planes across
re-loads, SPaRC_Gym.py:149-151).  The rule audit is SPaRC_Gym.py:372-950; `_get_info`
re-runs it with terminated = truncated = False (1011), which is what the records hold.

Per episode the file stores the puzzle index, the actions, and after reset and after
every step: the agent location, the path (env.path), and rule_status normalised to JSON
(oracle.rules_ref.normalize: tuple keys -> "[x, y]", numpy scalars -> int).

Usage:  python tests/golden/make_rules_golden.py
"""
from __future__ import annotations

import copy
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

import yaml  # noqa: E402


def processed_full(env):
    out = mg.processed(env)
    for o, p in zip(out, env.puzzles):
        ps = p["polyshapes"]
        # [key, key type, shape]: the audit matches str(additional_info) against the keys (727)
        o["polyshapes"] = [[str(k), type(k).__name__, v] for k, v in ps.items()] if isinstance(ps, dict) else None
        o["difficulty"] = int(p["difficulty"])
    return out


def snapshot(env, info):
    return {"agent": [int(v) for v in env._agent_location],
            "path": [[int(a), int(b)] for a, b in env.path],
            "rule_status": normalize(info["rule_status"])}


def run_episode(env, pristine, idx, strategy, rng, max_len):
    env.puzzles = copy.deepcopy(pristine)
    pid = env.puzzles[idx]["id"]
    obs, info = env.reset(options={"puzzle_id": pid})
    rec = {"puzzle_index": idx, "strategy": strategy, "reset": snapshot(env, info), "actions": [], "steps": []}
    sols = env.solution_paths[:env.solution_count]
    plan = []
    if strategy == "solution0" and sols:
        plan = mg.sol_actions(sols[0])
    elif strategy == "solution_any" and sols:
        plan = mg.sol_actions(sols[int(rng.integers(len(sols)))])
    elif strategy == "solution_detour" and sols:
        plan = mg.sol_actions(sols[0])
        if len(plan) > 3:
            k = int(rng.integers(1, len(plan) - 1))
            d = int(rng.integers(4))
            plan = plan[:k] + [d, (d + 2) % 4] + plan[k:]
    for _ in range(max_len):
        if plan:
            a = plan.pop(0)
        elif strategy in ("legal", "solution0", "solution_any", "solution_detour"):
            la = info["legal_actions"]
            a = int(la[int(rng.integers(len(la)))]) if la else 0
        else:
            a = int(rng.integers(4))
        obs, r, term, trunc, info = env.step(a)
        rec["actions"].append(a)
        rec["steps"].append(snapshot(env, info))
        if (term or trunc) and not plan:
            break
    return rec


def episodes(records, tb, strategies, n_eps, seed, tag, max_len=40, first_each=True):
    env = mg.make_env(records, traceback=tb, max_steps=2000)
    pristine = copy.deepcopy(env.puzzles)
    rng = np.random.default_rng(seed)
    eps = []
    for e in range(n_eps):
        strat = strategies[e % len(strategies)]
        idx = e % len(pristine) if first_each and e < len(pristine) else int(rng.integers(len(pristine)))
        eps.append(run_episode(env, pristine, idx, strat, rng, max_len))
    return {"tag": tag, "traceback": tb, "records": records,
            "processed": processed_full(mg.make_env(records, traceback=tb, max_steps=2000)), "episodes": eps}


def crafted_records():
    """Edge cases of the audit: a triangle whose count names a polyshape (720-731), a start on
    a gap property (no_gap_violations, 505-515), a region with two stacked ylops, a star
    without colour (star_pairing 592-595), and int-keyed polyshapes (never matched, 727)."""
    rng = np.random.default_rng(99)
    out = []
    r = synthetic.make_rule_puzzle(rng, 3, 3, break_prob=0.0, triangle_shape_clash=True)
    out.append(r)
    r = synthetic.make_rule_puzzle(rng, 3, 3, break_prob=0.0)
    t = yaml.safe_load(r["text_visualization"])
    s = t["puzzle"]["start"]
    t["puzzle"]["cells"].append({"position": {"x": s["x"], "y": s["y"]}, "properties": {"gap": True}})
    r["text_visualization"] = yaml.safe_dump(t, sort_keys=False)
    out.append(r)
    r = synthetic.make_rule_puzzle(rng, 2, 2, break_prob=0.0)
    t = yaml.safe_load(r["text_visualization"])
    t["puzzle"]["cells"] = [{"position": {"x": 1, "y": 1}, "properties": {"type": "poly", "color": "red", "polyshape": 7}},
                            {"position": {"x": 1, "y": 3}, "properties": {"type": "ylop", "color": "red", "polyshape": 8}},
                            {"position": {"x": 3, "y": 1}, "properties": {"type": "ylop", "color": "red", "polyshape": 8}},
                            {"position": {"x": 3, "y": 3}, "properties": {"type": "star"}}]
    r["text_visualization"] = yaml.safe_dump(t, sort_keys=False)
    r["polyshapes"] = yaml.safe_dump({"7": [[1, 1, 1], [1, 1, 1]], "8": [[1]]}, sort_keys=False)
    out.append(r)
    r = synthetic.make_rule_puzzle(rng, 3, 3, break_prob=0.0)
    shapes = yaml.safe_load(r["polyshapes"]) or {}
    r["polyshapes"] = yaml.safe_dump({int(k): v for k, v in shapes.items()}, sort_keys=False)
    out.append(r)
    return out


def main():
    mg.REFMOD = mg.import_reference()
    out = {}
    strat = ["solution0", "legal", "solution_detour", "random", "solution_any"]
    r7 = synthetic.make_rule_puzzles(16, seed=21, sizes=((3, 3),), break_prob=0.3)
    rmix = synthetic.make_rule_puzzles(14, seed=22, sizes=((2, 2), (4, 4), (5, 5), (2, 3), (4, 2), (7, 7)),
                                       break_prob=0.3)
    rand7 = synthetic.make_puzzles(10, seed=23, sizes=((3, 3),), full_properties=True)
    out["rules_7x7_tb1"] = episodes(r7, True, strat, 32, 31, "rule-consistent 7x7, traceback")
    out["rules_mixed_tb0"] = episodes(rmix, False, strat, 28, 32, "rule-consistent mixed lattices")
    out["rules_random_tb1"] = episodes(rand7, True, strat, 20, 33, "random full-property 7x7")
    out["rules_crafted_tb1"] = episodes(crafted_records(), True, strat, 12, 34, "crafted audit edge cases")
    for k, v in out.items():
        path = os.path.join(HERE, f"{k}.json.gz")
        raw = json.dumps(v, separators=(",", ":")).encode()
        with open(path, "wb") as f:
            with gzip.GzipFile(fileobj=f, mode="wb", mtime=0) as g:
                g.write(raw)
        print(k, os.path.getsize(path))


if __name__ == "__main__":
    main()
