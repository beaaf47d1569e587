"""Host-side puzzle loading and packing.

``process_puzzles`` restates the reference's one-time preprocessing
``SPaRC_Gym._process_puzzles`` (SPaRC_Gym/SPaRC_Gym.py:219-368) exactly, including its quirks:

* the loop variable ``symbol`` is never reset per cell or per puzzle, so a property key that
  is not ``type``/``dot`` (``gap``, ``color``, ...) re-uses the previous cell's (or previous
  puzzle's) symbol and may add a zero plane of that name (283-306, 334-343);
* a pool whose first property key is neither ``type`` nor ``dot`` raises UnboundLocalError;
* every cell centre (odd, odd) is marked in ``gaps`` (345-351).

``pack_table`` turns processed puzzles into the device table of include/sparc_gym_amd.h:
an ``open`` bitboard (in lattice and not a gap), start/target, and a solution-prefix trie
over the first ``solution_count`` solutions (the ones ``range(self.solution_count)`` visits at
SPaRC_Gym.py:1205 and 1217).
"""
from __future__ import annotations

from collections import OrderedDict
from dataclasses import dataclass

import numpy as np
import yaml

COLOR_TO_NUMBER = {"red": 1, "blue": 2, "yellow": 3, "green": 4, "black": 5, "purple": 6,
                   "orange": 7, "white": 8}   # SPaRC_Gym.py:310
BASE_KEYS = ("visited", "gaps", "agent_location", "target_location")
_NONE = 0xFFFF
_DIRS = ((1, 0), (0, -1), (-1, 0), (0, 1))   # right, up, left, down (SPaRC_Gym.py:212-217)
_UNBOUND = object()
# yaml.safe_load (SPaRC_Gym.py:261, 266) through libyaml when PyYAML has it: the same
# SafeConstructor and resolver, only the scanner / parser in C (~9x faster on dataset rows;
# equality with the pure-Python loader on the golden pools: tests/test_puzzles.py)
_SAFE_LOADER = getattr(yaml, "CSafeLoader", yaml.SafeLoader)


def safe_load(text):
    """``yaml.safe_load`` semantics (libyaml parser when available)."""
    return yaml.load(text, Loader=_SAFE_LOADER)


def _rows(df):
    """Per-row column access for a pandas DataFrame (df[col][i], as the reference) or records."""
    if hasattr(df, "columns"):
        n = len(df)
        cols = list(df.columns)
        return n, (lambda c, i: df[c][i]), cols
    recs = list(df)
    cols = list(recs[0].keys()) if recs else []
    return len(recs), (lambda c, i: recs[i][c]), cols


def process_puzzles(df, observation="new"):
    """Restatement of SPaRC_Gym._process_puzzles (SPaRC_Gym.py:219-368).

    Returns a list of dicts with the reference's keys: difficulty, x_size, y_size,
    solution_count, solution_paths, polyshapes, start_location, target_location, obs_array
    (ordered planes), color_array, additional_info, id (+ observ for observation='SPaRC').
    """
    n, get, _ = _rows(df)
    puzzles = []
    symbol = _UNBOUND

    def sym():
        if symbol is _UNBOUND:
            raise UnboundLocalError("local variable 'symbol' referenced before assignment")
        return symbol

    for i in range(n):
        puzzle = {}
        puzzle["difficulty"] = get("difficulty_level", i)                          # 239-240
        grid_size = get("grid_size", i)                                             # 243-248
        x_size = grid_size["width"] * 2 + 1
        y_size = grid_size["height"] * 2 + 1
        puzzle["x_size"], puzzle["y_size"] = x_size, y_size
        solution_count = get("solution_count", i)                                   # 251-257
        solution_paths = [[[pt["x"], pt["y"]] for pt in item["path"]] for item in get("solutions", i)]
        puzzle["solution_count"], puzzle["solution_paths"] = solution_count, solution_paths
        puzzle["polyshapes"] = safe_load(get("polyshapes", i))                 # 260-262
        text_yaml = safe_load(get("text_visualization", i))                    # 265-269
        puzzle["start_location"] = (text_yaml["puzzle"]["start"]["x"], text_yaml["puzzle"]["start"]["y"])
        puzzle["target_location"] = (text_yaml["puzzle"]["end"]["x"], text_yaml["puzzle"]["end"]["y"])

        obs_array = OrderedDict((k, np.zeros((x_size, y_size), dtype=np.int32)) for k in BASE_KEYS)
        color_array = np.zeros((x_size, y_size), dtype=np.int32)                    # 279-280
        additional_info = np.zeros((x_size, y_size), dtype=np.int64)

        for cell in text_yaml["puzzle"]["cells"]:                                   # 283-325
            properties = cell.get("properties", {})
            count = shape = color = None
            for key, value in properties.items():
                if key == "type":
                    symbol = f"{value}"
                    color = properties.get("color", "")
                    if value == "triangle":
                        count = properties.get("count", "")
                    elif value not in ("star", "square"):
                        shape = properties.get("polyshape", "")
                elif key == "dot":
                    symbol = "dot"
                if sym() not in obs_array:
                    obs_array[symbol] = np.zeros((x_size, y_size), dtype=np.int32)
                if color:
                    position = cell.get("position", {})
                    x, y = position.get("x"), position.get("y")
                    for color_ in COLOR_TO_NUMBER:
                        if color_ == color:
                            color_array[x][y] = COLOR_TO_NUMBER[color_]
                if count:
                    position = cell.get("position", {})
                    additional_info[position.get("x")][position.get("y")] = count
                elif shape:
                    position = cell.get("position", {})
                    additional_info[position.get("x")][position.get("y")] = shape

        for cell in text_yaml["puzzle"]["cells"]:                                   # 329-343
            position = cell.get("position", {})
            properties = cell.get("properties", {})
            x, y = position.get("x"), position.get("y")
            for key, value in properties.items():
                if key == "type":
                    symbol = f"{value}"
                elif key == "dot":
                    symbol = "dot"
                elif key == "gap":
                    symbol = "gaps"
                if sym() in obs_array:
                    obs_array[symbol][x, y] = 1

        for k in range(x_size - 1):                                                 # 345-351
            for j in range(y_size - 1):
                if k % 2 == 1 and j % 2 == 1:
                    obs_array["gaps"][k, j] = 1

        puzzle["obs_array"] = obs_array
        puzzle["color_array"] = color_array
        puzzle["additional_info"] = additional_info
        if observation == "SPaRC":                                                  # 358-360
            puzzle["observ"] = get("puzzle_array", i)
        puzzle["id"] = get("id", i)                                                 # 362-363
        puzzles.append(puzzle)
    return puzzles


# ----------------------------------------------------------------------------------- packing
@dataclass
class PuzzleTable:
    """Device puzzle table (layout documented in include/sparc_gym_amd.h)."""
    open: np.ndarray        # uint64 [P][words]
    info: np.ndarray        # uint32 [P][4]
    trie: np.ndarray        # uint32 [nodes][4]
    pitch: int
    words: int
    x_max: int
    y_max: int

    @property
    def num_puzzles(self):
        return len(self.info)


def lattice_geometry(puzzles, pitch=None, words=None):
    """Bitboard geometry (pitch, words, x_max, y_max) for a pool.

    words == 1 is the PADDED 64-bit layout of the kernel's fast path: pitch > y_max (a blocked
    column) and (x_max + 1) * pitch <= 64 (a blocked row), pitch <= 15 — every 7x7 or 5x5
    pool.  Larger lattices use 2 or 4 words with pitch >= y_max and explicit bounds checks.
    """
    x_max = max(int(p["x_size"]) for p in puzzles)
    y_max = max(int(p["y_size"]) for p in puzzles)
    if x_max > 255 or y_max > 255:
        raise ValueError("lattice too large")
    padded_ok = lambda pt: y_max < pt <= 15 and (x_max + 1) * pt <= 64  # noqa: E731
    if words is None:
        if pitch is None and padded_ok(y_max + 1):
            return y_max + 1, 1, x_max, y_max
        if pitch is not None and padded_ok(int(pitch)):
            return int(pitch), 1, x_max, y_max
    pitch = (y_max + 1 if words == 1 else y_max) if pitch is None else int(pitch)
    if pitch < y_max:
        raise ValueError(f"pitch {pitch} < max y_size {y_max}")
    if words == 1:
        if not padded_ok(pitch):
            raise ValueError(f"words=1 needs a padded geometry: {y_max} < pitch <= 15 and "
                             f"(x_max + 1) * pitch <= 64 (x_max={x_max}, pitch={pitch})")
        return pitch, 1, x_max, y_max
    bits = (x_max - 1) * pitch + y_max
    need = 2 if bits <= 128 else 4 if bits <= 256 else None
    if need is None:
        raise ValueError(f"lattice {x_max}x{y_max} exceeds the 256-bit bitboard (15x15 lattices max)")
    words = need if words is None else int(words)
    if words not in (2, 4) or words < need:
        raise ValueError(f"words={words} cannot hold a {x_max}x{pitch} lattice")
    return pitch, words, x_max, y_max


def _int_coord(v):
    f = float(v)
    if f != int(f):
        return None
    return int(f)


def build_trie(start, solutions):
    """Solution-prefix trie.  Node 0 is the one-point path [start].  Returns
    (nodes list of [c0, c1, c2, c3, parent, terminal, depth], root_valid)."""
    nodes = [[_NONE, _NONE, _NONE, _NONE, _NONE, 0, 0]]
    root_valid = False
    for sol in solutions:
        pts = [(_int_coord(a), _int_coord(b)) for a, b in sol]
        if not pts or pts[0] != tuple(start) or None in pts[0]:
            continue                          # never equal to / extended by [start, ...]
        root_valid = True
        cur, complete = 0, True
        for (ax, ay), (bx, by) in zip(pts[:-1], pts[1:]):
            if ax is None or bx is None or ay is None or by is None:
                complete = False
                break
            d = _DIRS.index((bx - ax, by - ay)) if (bx - ax, by - ay) in _DIRS else None
            if d is None:                     # the agent only moves to a neighbour: this
                complete = False              # solution's remaining points are unreachable
                break
            nxt = nodes[cur][d]
            if nxt == _NONE:
                nxt = len(nodes)
                nodes.append([_NONE, _NONE, _NONE, _NONE, cur, 0, nodes[cur][6] + 1])
                nodes[cur][d] = nxt
            cur = nxt
        if complete:
            nodes[cur][5] = 1
    if len(nodes) > _NONE:
        raise ValueError("solution trie exceeds 65535 nodes for one puzzle")
    return _bfs_order(nodes), root_valid


def _bfs_order(nodes):
    """The trie renumbered breadth-first (root 0, then depth 1, ...).  A random walk is on the
    trie mostly near the root, so the records the GPU gathers (8 B each, 16 per 128-B line) sit in
    the puzzle's first lines: fewer L2 lines per puzzle when a large pool's tries outgrow the L2."""
    order, head = [0], 0
    while head < len(order):
        order.extend(c for c in nodes[order[head]][:4] if c != _NONE)
        head += 1
    new = {old: k for k, old in enumerate(order)}
    out = []
    for old in order:
        c0, c1, c2, c3, par, term, depth = nodes[old]
        out.append([new.get(c, _NONE) for c in (c0, c1, c2, c3)] + [new.get(par, _NONE), term, depth])
    return out


def pack_table(puzzles, pitch=None, words=None):
    """Processed puzzles -> PuzzleTable (numpy, host)."""
    pitch, words, x_max, y_max = lattice_geometry(puzzles, pitch, words)
    P = len(puzzles)
    open_ = np.zeros((P, words), np.uint64)
    info = np.zeros((P, 4), np.uint32)
    tries = []
    base = 0
    for q, p in enumerate(puzzles):
        X, Y = int(p["x_size"]), int(p["y_size"])
        sx, sy = (int(v) for v in p["start_location"])
        tx, ty = (int(v) for v in p["target_location"])
        if not (0 <= sx < X and 0 <= sy < Y and 0 <= tx < X and 0 <= ty < Y):
            raise ValueError(f"puzzle {q}: start/target outside the {X}x{Y} lattice")
        gaps = np.asarray(p["obs_array"]["gaps"])
        xs, ys = np.nonzero(gaps[:X, :Y] == 0)
        bits = xs.astype(np.int64) * pitch + ys
        words_arr = np.zeros(words, np.uint64)
        for w in range(words):
            sel = bits[(bits >> 6) == w] & 63
            words_arr[w] = np.bitwise_or.reduce(np.left_shift(np.uint64(1), sel.astype(np.uint64)),
                                                initial=np.uint64(0))
        open_[q] = words_arr
        nsol = int(p["solution_count"])
        sols = p["solution_paths"]
        if nsol > len(sols):
            # the reference raises IndexError lazily at SPaRC_Gym.py:1206/1218; refuse up front
            raise ValueError(f"puzzle {q}: solution_count {nsol} > {len(sols)} stored solutions")
        nodes, root_valid = build_trie((sx, sy), sols[:max(nsol, 0)])
        start_closed = gaps[sx, sy] != 0
        flags = (1 if nsol > 0 else 0) | (2 if root_valid else 0) | (4 if start_closed else 0)
        info[q, 0] = X | (Y << 8) | (sx << 16) | (sy << 24)
        info[q, 1] = tx | (ty << 8) | (flags << 16)
        if root_valid:
            info[q, 2], info[q, 3] = base, len(nodes)
            arr = np.asarray(nodes, np.int64)
            term = arr[:, 5]
            # terminal bits of the 4 children and of the parent, so that the kernel knows a
            # new node's terminal flag without waiting for that node's record
            kid_term = np.zeros(len(nodes), np.int64)
            for d in range(4):
                has = arr[:, d] != _NONE
                kid_term |= np.where(has, term[np.where(has, arr[:, d], 0)], 0) << d
            par = arr[:, 4]
            par_term = np.where(par != _NONE, term[np.where(par != _NONE, par, 0)], 0)
            rec = np.zeros((len(nodes), 4), np.uint32)
            rec[:, 0] = arr[:, 0] | (arr[:, 1] << 16)
            rec[:, 1] = arr[:, 2] | (arr[:, 3] << 16)
            rec[:, 2] = par | (term << 16) | (kid_term << 17) | (par_term << 21)
            rec[:, 3] = arr[:, 6]
            tries.append(rec)
            base += len(nodes)
    trie = np.concatenate(tries) if tries else np.zeros((0, 4), np.uint32)
    return PuzzleTable(open_, info, np.ascontiguousarray(trie), pitch, words, x_max, y_max)


# ----------------------------------------------------------------------------------- rule audit
RULE_PLANES = 25   # SPARC_RULE_PLANES
(RP_CELLS, RP_LATTICE, RP_GAPS, RP_DOTS, RP_TRI, RP_TRI0, RP_TRI1, RP_TRI2, RP_STAR, RP_SQUARE,
 RP_COLORED) = range(11)
RP_COL1, RP_M0, RP_M1, RP_M2, RP_NOTFIRST, RP_NOTLAST, RP_INST = 11, 19, 20, 21, 22, 23, 24
RULE_SKIP_LAYERS = ("visited", "gaps", "agent_location", "target_location")   # SPaRC_Gym.py:466


@dataclass
class RulesTable:
    """Rule-audit table (layout: include/sparc_gym_amd.h, sparc_rules_table)."""
    planes: np.ndarray       # uint64 [P][RULE_PLANES][words]
    inst_first: np.ndarray   # uint32 [P + 1] offsets into inst
    inst: np.ndarray         # uint32 [I]: bit | ylop << 10 | shape << 11
    shape_first: np.ndarray  # uint32 [S + 1] offsets into shape_off
    shape_area: np.ndarray   # int32 [S]
    shape_off: np.ndarray    # int8 [O][2]

    def inst_range(self, q):
        """(first, count) of puzzle q's instances."""
        return int(self.inst_first[q]), int(self.inst_first[q + 1]) - int(self.inst_first[q])

    def shape_offsets(self, s):
        return [(int(dx), int(dy)) for dx, dy in self.shape_off[int(self.shape_first[s]):int(self.shape_first[s + 1])]]


def _pack_planes(masks, pitch, words):
    """Boolean [K][X][Y] planes -> uint64 [K][words] bitboards (bit x*pitch + y), all at once."""
    K, X, Y = masks.shape
    bi = (np.arange(X, dtype=np.uint64)[:, None] * np.uint64(pitch) + np.arange(Y, dtype=np.uint64)[None, :]).reshape(-1)
    v = np.uint64(1) << (bi & np.uint64(63))
    wid = bi >> np.uint64(6)
    flat = masks.reshape(K, -1)
    out = np.zeros((K, words), np.uint64)
    for k in range(words):   # distinct bits: their sum is their OR
        out[:, k] = (flat * np.where(wid == k, v, np.uint64(0))).sum(axis=1, dtype=np.uint64)
    return out


def shape_offsets(shape_arr):
    """_get_offsets (SPaRC_Gym.py:840-855) in cell units: the anchor is the first 1 of the
    shape's first row that has one."""
    s = np.array(shape_arr, dtype=np.int32)
    xs, ys = np.where(s == 1)
    if len(xs) == 0:
        return []
    ax = xs.min()
    ay = ys[np.where(xs == ax)[0]].min()
    return [(int(x - ax), int(y - ay)) for x, y in zip(xs, ys)]


def pack_rules(puzzles, table: PuzzleTable) -> RulesTable:
    """Processed puzzles -> the rule-audit table, on ``table``'s geometry.

    Restates what `_validate_rules` reads from a puzzle (SPaRC_Gym.py:372-838) as bit-planes:
    the symbol layers of `_collect_region_symbols` (456-481) only count at cell centres (the
    only points with a region id), triangles only at x in 1..x_size-2 / y in 1..y_size-2 with
    count > 0 (630-636), poly/ylop instances are the cells whose additional_info names a
    polyshape key (714-734).  Like the reference (734), a pool with a shaped instance and no
    'poly' layer raises KeyError('poly').
    """
    pitch, W = table.pitch, table.words
    P = len(puzzles)
    planes = np.zeros((P, RULE_PLANES, W), np.uint64)
    inst_first = np.zeros(P + 1, np.uint64)
    inst, shapes, shape_ids = [], [], {}
    for q, p in enumerate(puzzles):
        X, Y = int(p["x_size"]), int(p["y_size"])
        obs = p["obs_array"]
        color = np.asarray(p["color_array"])[:X, :Y]
        add = np.asarray(p["additional_info"])[:X, :Y]
        xs, ys = np.meshgrid(np.arange(X), np.arange(Y), indexing="ij")
        cells = (xs % 2 == 1) & (ys % 2 == 1)
        layer = lambda k: (np.asarray(obs[k])[:X, :Y] == 1) if k in obs else np.zeros((X, Y), bool)  # noqa: E731
        m = np.zeros((RULE_PLANES, X, Y), bool)
        m[RP_CELLS] = cells
        m[RP_LATTICE] = True
        m[RP_GAPS] = layer("gaps")
        m[RP_DOTS] = layer("dot")
        inner = (xs >= 1) & (xs <= X - 2) & (ys >= 1) & (ys <= Y - 2)
        tri = layer("triangle") & inner & (add > 0)
        cnt = np.clip(add, 0, 7)
        m[RP_TRI] = tri
        for k in range(3):
            m[RP_TRI0 + k] = tri & (((cnt >> k) & 1) == 1)
        m[RP_STAR] = layer("star") & cells
        m[RP_SQUARE] = layer("square") & cells
        m[RP_COLORED] = (color != 0) & cells
        for c in range(1, 9):
            m[RP_COL1 + c - 1] = (color == c) & cells
        mult = np.zeros((X, Y), np.int64)
        for k in obs:
            if k not in RULE_SKIP_LAYERS:
                mult += layer(k)
        mult = np.where(cells, mult, 0)
        if mult.max(initial=0) > 7:
            raise ValueError(f"puzzle {q}: more than 7 symbol layers on one cell")
        for k in range(3):
            m[RP_M0 + k] = ((mult >> k) & 1) == 1
        m[RP_NOTFIRST] = ys != 0
        m[RP_NOTLAST] = ys != Y - 1
        planes[q] = _pack_planes(m, pitch, W)   # RP_INST stays 0 here: set per instance below
        first = len(inst)
        poly = p["polyshapes"]
        if isinstance(poly, dict):
            for x in range(X):                                        # _extract_poly_instances
                for y in range(Y):
                    val = add[x, y]
                    if val == 0 or f"{val}" not in poly:
                        continue
                    name = f"{val}"
                    ylop = not (np.asarray(obs["poly"])[x, y] == 1)   # KeyError('poly') as at 734
                    if not cells[x, y]:
                        continue                                      # region id -1 (687-690)
                    arr = poly[name]
                    offs = shape_offsets(arr)
                    key = (tuple(offs), int(np.array(arr).sum()))
                    if key not in shape_ids:
                        shape_ids[key] = len(shapes)
                        shapes.append(key)
                    b = x * pitch + y
                    planes[q, RP_INST, b >> 6] |= np.uint64(1) << np.uint64(b & 63)
                    inst.append(b | (int(ylop) << 10) | (shape_ids[key] << 11))
        inst_first[q + 1] = len(inst)
    offs, sfirst, sarea = [], [0], []
    for o, area in shapes:
        sarea.append(area)
        offs.extend(o)
        sfirst.append(len(offs))
    if len(shapes) >= 1 << 21 or len(inst) >= 1 << 32 or len(offs) >= 1 << 32:
        raise ValueError("rule table past 2^21 distinct polyshapes or 2^32 entries")
    if any(not -128 <= v <= 127 for o, _ in shapes for d in o for v in d):
        raise ValueError("polyshape wider than 127 cells")
    return RulesTable(planes, inst_first.astype(np.uint32), np.asarray(inst, np.uint32),
                      np.asarray(sfirst, np.uint32), np.asarray(sarea, np.int32),
                      np.asarray(offs, np.int8).reshape(-1, 2))
