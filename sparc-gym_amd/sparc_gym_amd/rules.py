"""info['rule_status'] for the single-env drop-in, assembled from the GPU rule audit.

The reference rebuilds a nested dict on every step (`_validate_rules`, SPaRC_Gym.py:941-950).
Here the k_rules kernel does the audit itself — region flood fill, the eight checks and the
poly/ylop exact-fit search — and returns the pass bits, the region id of every cell and the
per-region fit results.  This module only lays those results out in the reference's dict
shape, filling the `detail` lists from the region map and the static planes with the same
iteration orders as the reference (x-major scans, layer order of obs_array, region ids).
"""
from __future__ import annotations

from collections import Counter

import numpy as np

RULE_NAMES = ("reached_target", "path_not_crossing", "no_gap_violations", "all_dots_collected",
              "square_color_separation", "star_pairing_exact", "triangles_edge_count", "poly_ylop_area",
              "all_rules_satisfied")
SKIP_LAYERS = ("visited", "gaps", "agent_location", "target_location")
RULE_SEARCH_EXHAUSTED = 1 << 9   # SPARC_RULE_SEARCH_EXHAUSTED: an exact fit still pending on the host


def region_map_of(region_bits, x_size, y_size, pitch):
    """Device region ids per bit -> the reference's region_map [x, y] (-1 off cells)."""
    xs, ys = np.meshgrid(np.arange(x_size), np.arange(y_size), indexing="ij")
    r = np.asarray(region_bits)[xs * pitch + ys].astype(np.int32)
    return np.where(r == 255, -1, r)


class RuleStatic:
    """What rule_status reads of a puzzle that no step changes, as plain Python lists (numpy
    scalar indexing per cell cost most of a call): the symbol cells of each layer in the
    reference's iteration order (obs_array layer order, x-major), the colour grid, the
    triangle cells with their required counts, the dot cells, the gap grid and the poly / ylop
    instances (_extract_poly_instances, SPaRC_Gym.py:714-734)."""

    def __init__(self, puzzle, obs_array):
        self.color = np.asarray(puzzle["color_array"]).tolist()
        add = np.asarray(puzzle["additional_info"])
        self.layers = []
        for layer, arr in obs_array.items():
            if layer in SKIP_LAYERS:
                continue
            xs, ys = np.where(np.asarray(arr) == 1)
            self.layers.append((layer, list(zip(xs.tolist(), ys.tolist()))))
        self.keys = set(obs_array.keys())
        self.gaps = np.asarray(obs_array["gaps"]).tolist()
        self.dots = None
        if "dot" in obs_array:
            xs, ys = np.where(np.asarray(obs_array["dot"]) == 1)
            self.dots = list(zip(xs.tolist(), ys.tolist()))
        self.tri = None
        if "triangle" in obs_array:
            tri = np.asarray(obs_array["triangle"])
            h, w = tri.shape
            self.tri = [(x, y, int(add[x, y])) for x in range(1, h - 1) for y in range(1, w - 1)
                        if tri[x, y] == 1 and int(add[x, y]) > 0]
        self.inst = _poly_instances(puzzle, obs_array, add)


def rule_status(puzzle, obs_array, path, agent, target, bits, region_map, fit, terminated=False,
                truncated=False, static=None):
    """The reference's rule_status dict (structure of SPaRC_Gym.py:896-950).

    The GPU caps each exact-fit search; the C ABI finishes any search past the cap on the host
    without a cap (sparc_rules_finish, run by sparc_rules_host), so `bits` always carry the
    reference's answer.  Bits that still mark a pending search are a caller error.  static: the
    puzzle's RuleStatic (built here when not given; SPaRC_Gym keeps one per puzzle)."""
    if int(bits) & RULE_SEARCH_EXHAUSTED:
        raise RuntimeError("rule bits with a pending exact-fit search: call sparc_rules_finish first")
    st = static if static is not None else RuleStatic(puzzle, obs_array)
    color = st.color
    passed = {n: bool((int(bits) >> k) & 1) for k, n in enumerate(RULE_NAMES)}
    rm = np.asarray(region_map)
    rml = rm.tolist()
    nreg = int(rm.max()) + 1 if rm.size and rm.max() >= 0 else 0
    # _collect_region_symbols (456-481): per region, layer -> coords and colour -> count
    symbols = [dict() for _ in range(nreg)]
    colors = [dict() for _ in range(nreg)]
    for layer, cells in st.layers:
        for x, y in cells:
            rid = rml[x][y]
            if rid == -1:
                continue
            symbols[rid].setdefault(layer, []).append((x, y))
            c = color[x][y]
            if c:
                colors[rid][c] = colors[rid].get(c, 0) + 1
    area = np.bincount(rm[rm >= 0], minlength=nreg).tolist() if nreg else []
    res = {}

    def add_rule(name, detail):
        res[name] = {"passed": passed[name], "detail": detail}

    add_rule("reached_target", {"agent_loc": np.asarray(agent).tolist(), "target_loc": np.asarray(target).tolist()})
    counts = Counter(tuple(p) for p in path)
    add_rule("path_not_crossing", {"duplicates": {k: v for k, v in counts.items() if v > 1}})
    gaps = st.gaps
    add_rule("no_gap_violations", {"violations": [(x, y) for x, y in path if gaps[x][y] == 1]})
    if st.dots is None:
        add_rule("all_dots_collected", {"total": 0, "collected": 0})
    else:
        vis = obs_array["visited"]
        add_rule("all_dots_collected", {"total": len(st.dots),
                                        "collected": sum(1 for x, y in st.dots if vis[x, y] == 1)})
    if "square" not in st.keys:
        add_rule("square_color_separation", {"regions": []})
    else:
        bad, det = [], []
        for r in range(nreg):
            sq = symbols[r].get("square", [])
            if not sq:
                continue
            cs = set(color[x][y] for x, y in sq if color[x][y] != 0)
            if len(cs) > 1:
                bad.append(r)
            det.append({"region": r, "square_count": len(sq), "colors": list(cs)})
        add_rule("square_color_separation", {"violating_regions": bad, "region_square_details": det})
    if "star" not in st.keys:
        add_rule("star_pairing_exact", {"regions": []})
    else:
        viol, per = [], []
        for r in range(nreg):
            stars = symbols[r].get("star", [])
            if not stars:
                continue
            allc = {}
            for coords in symbols[r].values():
                for x, y in coords:
                    c = color[x][y]
                    if c != 0:
                        allc[c] = allc.get(c, 0) + 1
            sc = {}
            for x, y in stars:
                c = color[x][y]
                if c == 0:
                    viol.append({"region": r, "color": 0, "found_total": 1})
                    continue
                sc[c] = sc.get(c, 0) + 1
            ok_all, det = True, []
            for c, n in sc.items():
                tot = allc.get(c, 0)
                ok = tot == 2
                if not ok:
                    ok_all = False
                    viol.append({"region": r, "color": c, "found_total": tot, "star_cells": n})
                det.append({"color": c, "total_symbols_of_color": tot, "star_cells": n, "ok": ok})
            per.append({"region": r, "details": det, "all_ok": ok_all})
        add_rule("star_pairing_exact", {"violations": viol, "per_region": per})
    if st.tri is None:
        add_rule("triangles_edge_count", {"mismatches": []})
    else:
        nodes = {(p[0], p[1]) for p in path}
        mism = []
        for x, y, req in st.tri:
            t = ((x + 1, y) in nodes) + ((x - 1, y) in nodes) + ((x, y - 1) in nodes) + ((x, y + 1) in nodes)
            if t != req:
                mism.append({"x": x, "y": y, "required": req, "touches": t})
        add_rule("triangles_edge_count", {"mismatches": mism})
    add_rule("poly_ylop_area", _poly_detail(st.inst, rml, area, fit))
    core = [k for k in res]
    add_rule("all_rules_satisfied", {"rules_checked": core})
    res["_terminated"] = {"passed": True, "detail": terminated}
    res["_truncated"] = {"passed": True, "detail": truncated}
    res["_regions"] = {r: {"id": r, "area": area[r], "symbol_counts": {k: len(v) for k, v in symbols[r].items()},
                           "colors": colors[r]} for r in range(nreg)}
    return res


def _poly_instances(puzzle, obs_array, add):
    """The poly / ylop instances of _rule_poly_ylop_balance (714-734): name, cell, area, kind."""
    shapes = puzzle["polyshapes"]
    inst = []
    if isinstance(shapes, dict):
        h, w = add.shape
        for x in range(h):
            for y in range(w):
                val = add[x, y]
                if val != 0 and f"{val}" in shapes:
                    name = f"{val}"
                    a = int(np.array(shapes[name]).sum())
                    kind = "poly" if obs_array["poly"][x, y] == 1 else "ylop"
                    inst.append({"name": name, "x": x, "y": y, "area": a, "kind": kind})
    return inst


def _poly_detail(inst, rml, area, fit):
    """_rule_poly_ylop_balance (648-709) detail; the area check and exact fit come from the GPU."""
    if not inst:
        return {"regions": []}
    by_region = {}
    for it in inst:
        rid = rml[it["x"]][it["y"]]
        if rid != -1:
            by_region.setdefault(int(rid), []).append(it)
    details = []
    for rid, lst in by_region.items():
        pa = sum(i["area"] for i in lst if i["kind"] == "poly")
        ya = sum(i["area"] for i in lst if i["kind"] == "ylop")
        net = pa - ya
        area_ok = area[rid] == net
        d = {"region": rid, "area_check": {"region_area": area[rid], "poly_area": pa, "ylop_area": ya,
                                           "net": net, "ok": area_ok}}
        if area_ok:
            ok = bool((int(fit) >> rid) & 1)
            d["exact_fit"] = {"ok": ok, "region_id": rid, "region_area": area[rid], "poly_area": pa,
                              "ylop_area": ya, "net": net}
        else:
            d["exact_fit"] = {"ok": False, "skipped": True}
        d["ok"] = area_ok and d["exact_fit"]["ok"]
        details.append(d)
    return {"violations": [d["region"] for d in details if not d["ok"]], "region_details": details}
