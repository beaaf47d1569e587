"""Generate the golden vectors in tests/golden/*.json from the REFERENCE env.

Runs only in the build container (the reference lives at /root/reference and never travels).
The reference `SPaRC_Gym/SPaRC_Gym.py` is imported unmodified; three blockers are stubbed:
  * gymnasium (not installed)  -> tests/golden/stubs/gymnasium (seeding restated from
    gymnasium.utils.seeding.np_random: Generator(PCG64(SeedSequence(seed))));
  * pygame (not installed, imported by SPaRC_Gym/render/__init__.py) -> empty module;
  * datasets.load_dataset (network, SPaRC_Gym.py:77) -> monkey-patched to return a synthetic
    DataFrame in the SPaRC schema built by sparc_gym_amd.synthetic.

Aliasing (SURVEY §8a trap 1): `_load_puzzle` binds the puzzle's planes without copying
(SPaRC_Gym.py:149-151), so a re-loaded puzzle keeps the previous episode's `visited` bits.
Every episode below therefore restores a pristine deep copy of `env.puzzles` before
`reset()`: the vectors record the reference's first-load semantics.

Usage:  python tests/golden/make_golden.py        (writes tests/golden/*.json.gz)
"""
from __future__ import annotations

import copy
import gzip
import json
import os
import sys
from types import SimpleNamespace

import numpy as np
import yaml

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, os.path.join(REPO, "sparc-gym_amd"))
from sparc_gym_amd import synthetic  # noqa: E402
sys.path.insert(0, os.path.dirname(HERE))
from golden_io import rows_as_ndarray  # noqa: E402


def import_reference():
    sys.dont_write_bytecode = True
    sys.path.insert(0, os.path.join(HERE, "stubs"))
    sys.path.insert(1, REF)
    import SPaRC_Gym  # noqa: F401  (package __init__ imports the class + registration)
    return sys.modules["SPaRC_Gym.SPaRC_Gym"]


REFMOD = None


def make_env(records, **kw):
    df = synthetic.records_to_dataframe(records)
    REFMOD.load_dataset = lambda *a, **k: SimpleNamespace(to_pandas=lambda: df)
    return REFMOD.SPaRC_Gym(**kw)


# ---------------------------------------------------------------- serialisation helpers
def plane(a):
    a = np.asarray(a)
    nz = np.flatnonzero(a)
    return {"shape": list(a.shape), "nz": [[int(i), int(a.flat[i])] for i in nz]}


def reward_repr(r):
    return {"value": float(r), "type": type(r).__name__, "repr": repr(r)}


def obs_dict(obs):
    return {"base_keys": list(obs["base"].keys()),
            "base": {k: plane(v) for k, v in obs["base"].items()},
            "color": plane(obs["color"]),
            "additional_info": plane(obs["additional_info"])}


def info_dict(info):
    return {"solution_count": int(info["solution_count"]),
            "difficulty": int(info["difficulty"]),
            "grid_x_size": int(info["grid_x_size"]),
            "grid_y_size": int(info["grid_y_size"]),
            "legal_actions": [int(a) for a in info["legal_actions"]],
            "current_step": int(info["current_step"]),
            "agent_location": [int(v) for v in info["agent_location"]],
            "normal_reward": reward_repr(info["Rewards"]["normal_reward"]),
            "outcome_reward": reward_repr(info["Rewards"]["outcome_reward"])}


def processed(env):
    out = []
    for p in env.puzzles:
        out.append({"id": str(p["id"]),
                    "x_size": int(p["x_size"]), "y_size": int(p["y_size"]),
                    "start": [int(v) for v in p["start_location"]],
                    "target": [int(v) for v in p["target_location"]],
                    "solution_count": int(p["solution_count"]),
                    "solution_paths": [[[int(a), int(b)] for a, b in s] for s in p["solution_paths"]],
                    "base_keys": list(p["obs_array"].keys()),
                    "base": {k: plane(v) for k, v in p["obs_array"].items()},
                    "color": plane(p["color_array"]),
                    "additional_info": plane(p["additional_info"])})
    return out


# ---------------------------------------------------------------- action strategies
DIRS = {(1, 0): 0, (0, -1): 1, (-1, 0): 2, (0, 1): 3}


def sol_actions(path):
    return [DIRS[(b[0] - a[0], b[1] - a[1])] for a, b in zip(path[:-1], path[1:])
            if (b[0] - a[0], b[1] - a[1]) in DIRS]


def run_episode(env, pristine, idx, strategy, rng, max_len=400, post_done=3):
    env.puzzles = copy.deepcopy(pristine)
    pid = env.puzzles[idx]["id"]
    obs, info = env.reset(options={"puzzle_id": pid})
    rec = {"puzzle_index": idx, "puzzle_id": str(pid), "strategy": strategy,
           "reset": {"obs": obs_dict(obs), "info": info_dict(info)}, "actions": [], "steps": []}
    sols = env.solution_paths[:env.solution_count]
    plan = []
    if strategy.startswith("solution") and sols:
        s = sols[int(rng.integers(len(sols)))]
        plan = sol_actions(s)
        if strategy == "solution_detour" and len(plan) > 3:
            k = int(rng.integers(1, len(plan) - 1))
            d = int(rng.integers(4))
            plan = plan[:k] + [d, (d + 2) % 4] + plan[k:]
        elif strategy == "solution_wrong_end" and len(plan) > 2:
            plan = plan[:-1] + [int(rng.integers(4))] * 3
    done_at = None
    t = 0
    while t < max_len:
        if plan:
            a = plan.pop(0)
        elif strategy == "legal":
            la = info["legal_actions"]
            a = int(la[int(rng.integers(len(la)))]) if la else 0
        elif strategy == "illegal_mix":
            a = int(rng.choice([0, 1, 2, 3, 4, 5, 7, 255]))
        else:
            a = int(rng.integers(4))
        obs, r, term, trunc, info = env.step(a)
        rec["actions"].append(a)
        vis = np.asarray(obs["base"]["visited"])
        agent = np.asarray(obs["base"]["agent_location"])
        rec["steps"].append({"reward": reward_repr(r), "terminated": bool(term), "truncated": bool(trunc),
                             "info": info_dict(info), "visited": plane(vis), "agent_plane": plane(agent)})
        t += 1
        if (term or trunc) and done_at is None:
            done_at = t
        if done_at is not None and t >= done_at + post_done:
            break
    rec["done_at"] = done_at
    return rec


def run_text_episode(env, pristine, idx, strategy, rng, max_len=120, post_done=2):
    """One observation='SPaRC' episode: the JSON text grid after reset and every step
    (SPaRC_Gym.py:153-164, 988-992, 1150-1184)."""
    env.puzzles = copy.deepcopy(pristine)
    pid = env.puzzles[idx]["id"]
    obs, info = env.reset(options={"puzzle_id": pid})
    rec = {"puzzle_index": idx, "puzzle_id": str(pid), "strategy": strategy, "reset_obs": obs,
           "reset_legal": [int(a) for a in info["legal_actions"]], "actions": [], "steps": []}
    sols = env.solution_paths[:env.solution_count]
    plan = sol_actions(sols[int(rng.integers(len(sols)))]) if strategy == "solution" and sols else []
    if strategy == "detour" and sols:
        plan = sol_actions(sols[0])
        if len(plan) > 2:
            k = int(rng.integers(1, len(plan) - 1))
            d = int(rng.integers(4))
            plan = plan[:k] + [d, (d + 2) % 4, d, (d + 2) % 4] + plan[k:]
    done_at, t = None, 0
    while t < max_len:
        if plan:
            a = plan.pop(0)
        elif strategy == "legal":
            la = info["legal_actions"]
            a = int(la[int(rng.integers(len(la)))]) if la else 0
        else:
            a = int(rng.choice([0, 1, 2, 3, 0, 1, 2, 3, 5]))
        obs, r, term, trunc, info = env.step(a)
        rec["actions"].append(a)
        rec["steps"].append({"obs": obs, "reward": reward_repr(r), "terminated": bool(term),
                             "truncated": bool(trunc), "legal_actions": [int(x) for x in info["legal_actions"]],
                             "agent_location": [int(v) for v in info["agent_location"]]})
        t += 1
        if (term or trunc) and done_at is None:
            done_at = t
        if done_at is not None and t >= done_at + post_done:
            break
    return rec


def text_episodes(records, tb, max_steps, n_eps, seed, tag, ndarray_rows=False):
    """observation='SPaRC' episodes.  ndarray_rows: puzzle_array as a 1-D object array of
    per-row string arrays, the form a parquet export of the dataset hands to the reference
    (its first branch at SPaRC_Gym.py:155-156); otherwise lists of rows (the third branch)."""
    df = synthetic.records_to_dataframe(records)
    if ndarray_rows:
        df["puzzle_array"] = [rows_as_ndarray(g) for g in df["puzzle_array"]]
    REFMOD.load_dataset = lambda *a, **k: SimpleNamespace(to_pandas=lambda: df)
    env = REFMOD.SPaRC_Gym(observation="SPaRC", traceback=tb, max_steps=max_steps)
    pristine = copy.deepcopy(env.puzzles)
    rng = np.random.default_rng(seed)
    strategies = ["solution", "legal", "random", "detour"]
    eps = [run_text_episode(env, pristine, int(rng.integers(len(pristine))), strategies[e % 4], rng)
           for e in range(n_eps)]
    return {"tag": tag, "traceback": tb, "max_steps": max_steps, "records": records,
            "ndarray_rows": ndarray_rows, "episodes": eps}


def episodes(records, tb, max_steps, strategies, n_eps, seed, tag):
    env = make_env(records, traceback=tb, max_steps=max_steps)
    pristine = copy.deepcopy(env.puzzles)
    rng = np.random.default_rng(seed)
    eps = []
    for e in range(n_eps):
        strat = strategies[e % len(strategies)]
        idx = int(rng.integers(len(pristine)))
        eps.append(run_episode(env, pristine, idx, strat, rng))
    return {"tag": tag, "traceback": tb, "max_steps": max_steps, "records": records,
            "processed": processed(make_env(records, traceback=tb, max_steps=max_steps)),
            "episodes": eps}


# ---------------------------------------------------------------- stale-symbol crafted pool
def stale_symbol_records():
    rng = np.random.default_rng(77)
    recs = [synthetic.make_puzzle(rng, 3, 3, n_solutions=2, full_properties=True) for _ in range(6)]

    def set_cells(r, cells):
        t = yaml.safe_load(r["text_visualization"])
        t["puzzle"]["cells"] = cells
        r["text_visualization"] = yaml.safe_dump(t, sort_keys=False)

    # puzzle 0 ends on a triangle cell, puzzle 1 STARTS with a gap-only cell -> the gap key
    # re-uses the stale `symbol` ('triangle') from puzzle 0 (SPaRC_Gym.py:304-306, 339-343)
    set_cells(recs[0], [{"position": {"x": 1, "y": 1}, "properties": {"type": "star", "color": "red"}},
                        {"position": {"x": 3, "y": 3}, "properties": {"type": "triangle", "color": "blue", "count": 2}}])
    set_cells(recs[1], [{"position": {"x": 0, "y": 1}, "properties": {"gap": True}},
                        {"position": {"x": 1, "y": 3}, "properties": {"type": "square", "color": "green"}}])
    # colour key before type key; unknown colour name; type 'gap' (not the 'gap' key)
    set_cells(recs[2], [{"position": {"x": 5, "y": 5}, "properties": {"color": "blue", "type": "square"}},
                        {"position": {"x": 1, "y": 5}, "properties": {"type": "star", "color": "magenta"}},
                        {"position": {"x": 2, "y": 1}, "properties": {"type": "gap"}}])
    # a colour-only cell and a dot cell with a colour
    set_cells(recs[3], [{"position": {"x": 3, "y": 1}, "properties": {"type": "poly", "color": "white", "polyshape": 4242}},
                        {"position": {"x": 5, "y": 1}, "properties": {"color": "red"}},
                        {"position": {"x": 4, "y": 4}, "properties": {"dot": True, "color": "black"}}])
    # no cells at all
    set_cells(recs[4], [])
    # triangle count 0 and poly without polyshape
    set_cells(recs[5], [{"position": {"x": 1, "y": 1}, "properties": {"type": "triangle", "color": "yellow", "count": 0}},
                        {"position": {"x": 3, "y": 3}, "properties": {"type": "ylop", "color": "purple"}}])
    return recs


def unbound_records():
    rng = np.random.default_rng(5)
    r = synthetic.make_puzzle(rng, 2, 2, n_solutions=1)
    t = yaml.safe_load(r["text_visualization"])
    t["puzzle"]["cells"] = [{"position": {"x": 1, "y": 1}, "properties": {"color": "red", "type": "star"}}]
    r["text_visualization"] = yaml.safe_dump(t, sort_keys=False)
    return [r]


def main():
    global REFMOD
    REFMOD = import_reference()
    out = {}
    rs = ["random", "legal", "solution", "solution_detour", "illegal_mix", "solution_wrong_end"]

    poolA = synthetic.make_puzzles(12, seed=1, sizes=((3, 3),), full_properties=True)
    poolB = synthetic.make_puzzles(6, seed=2, sizes=((3, 3),), full_properties=False)
    poolC = synthetic.make_puzzles(10, seed=3, sizes=((2, 2), (3, 3), (4, 4), (5, 5), (2, 3), (4, 2)),
                                   full_properties=True)
    rngD = np.random.default_rng(4)
    poolD = [synthetic.make_puzzle(rngD, 3, 3, n_solutions=0),
             synthetic.make_puzzle(rngD, 1, 1, n_solutions=1),
             synthetic.make_puzzle(rngD, 1, 2, n_solutions=3),
             synthetic.make_puzzle(rngD, 3, 3, n_solutions=8, shared_prefix_prob=0.9),
             synthetic.make_puzzle(rngD, 3, 2, n_solutions=1, n_gaps=0),
             synthetic.make_puzzle(rngD, 7, 7, n_solutions=4)]
    poolE = stale_symbol_records()

    out["poolA_tb0"] = episodes(poolA, False, 2000, rs, 36, 10, "7x7 full, traceback off")
    out["poolA_tb1"] = episodes(poolA, True, 2000, rs, 36, 11, "7x7 full, traceback on")
    out["poolB_tb0_ms17"] = episodes(poolB, False, 17, rs, 12, 12, "7x7 base, max_steps=17")
    out["poolB_tb1_ms5"] = episodes(poolB, True, 5, rs, 12, 13, "7x7 base, traceback, max_steps=5")
    out["poolC_tb0"] = episodes(poolC, False, 2000, rs, 24, 14, "mixed 5..11 lattices, traceback off")
    out["poolC_tb1"] = episodes(poolC, True, 300, rs, 24, 15, "mixed 5..11 lattices, traceback, max_steps=300")
    out["poolD_tb1"] = episodes(poolD, True, 2000, rs, 24, 16, "edge puzzles (0 solutions, 3x3, 15x15, ...)")
    out["poolD_tb0"] = episodes(poolD, False, 2000, rs, 12, 17, "edge puzzles, traceback off")
    out["poolE_tb1"] = episodes(poolE, True, 2000, rs, 12, 18, "stale-symbol crafted cells")
    # observation='SPaRC' (the text grid), both puzzle_array forms, traceback on / off
    out["text_tb1"] = text_episodes(poolC, True, 300, 24, 19, "SPaRC text obs, mixed lattices, traceback")
    out["text_tb0_nd"] = text_episodes(poolA, False, 40, 16, 20, "SPaRC text obs, 7x7, ndarray rows, max_steps=40",
                                       ndarray_rows=True)

    # seeded / sequential / option resets (SPaRC_Gym.py:1075-1087)
    env = make_env(poolA, traceback=False, max_steps=2000)
    seeded = []
    for s in list(range(40)) + [12345, 2**31 - 1, 2**40 + 7]:
        env.reset(seed=s)
        seeded.append([s, int(env.current_puzzle_index)])
    env2 = make_env(poolA, traceback=False, max_steps=2000)
    seq = [int(env2.current_puzzle_index)]
    for _ in range(15):
        env2.reset()
        seq.append(int(env2.current_puzzle_index))
    env2.reset(options={})
    seq_opt_empty = int(env2.current_puzzle_index)
    env2.reset(options={"puzzle_id": "not-a-puzzle"})
    seq_opt_missing = int(env2.current_puzzle_index)
    env2.reset(seed=3)
    after_seed = int(env2.current_puzzle_index)
    env2.reset()
    after_seed_next = int(env2.current_puzzle_index)
    out["resets"] = {"pool": "poolA", "n": len(poolA), "seeded": seeded, "sequential": seq,
                     "options_empty": seq_opt_empty, "options_missing": seq_opt_missing,
                     "seed3": after_seed, "seed3_then_plain": after_seed_next}

    try:
        make_env(unbound_records())
        unb = {"raises": None}
    except Exception as e:  # noqa: BLE001
        unb = {"raises": type(e).__name__}
    out["unbound_symbol"] = {"records": unbound_records(), **unb}

    for k, v in out.items():
        path = os.path.join(HERE, f"{k}.json.gz")
        raw = json.dumps(v, separators=(",", ":")).encode()
        with open(path, "wb") as f:  # mtime=0: byte-identical output on every run
            with gzip.GzipFile(fileobj=f, mode="wb", mtime=0) as g:
                g.write(raw)
        print(k, os.path.getsize(path))


if __name__ == "__main__":
    main()
