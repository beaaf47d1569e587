"""SPaRC_Gym: drop-in for the reference's single-puzzle ``gymnasium.Env``.

Same constructor kwargs, ``reset/step/render/close``, ``Discrete(4)`` actions, ``'new'`` dict
and ``'SPaRC'`` text observations, and the same ``info`` keys as
/root/reference/SPaRC_Gym/SPaRC_Gym.py (class at 44-1315).  The step itself runs on the GPU
through the C ABI (a batch of one env); host code only mirrors the observation planes from
the device state.

Differences (documented in DESIGN.md):
* ``puzzles=`` accepts a local DataFrame / list of records in the SPaRC schema, because the
  hub dataset (``load_dataset``, SPaRC_Gym.py:77) needs the network; ``df_name`` etc. are
  still honoured when ``puzzles`` is None.
* By default every reset restores pristine planes (the reference's first load of a puzzle).
  The reference aliases the planes across re-loads (SPaRC_Gym.py:149-151): a puzzle loaded
  again keeps the previous episode's ``visited`` and ``agent_location`` bits, and the stale
  ``visited`` bits block moves (_get_legal_actions reads that plane, 1040).  ``alias_compat=True``
  reproduces that exactly (pinned by tests/golden/alias_*.json.gz from the reference): the
  puzzle's planes persist in ``self.puzzles``, the device board starts from them, and the
  rule audit takes its path-based rules from the path and ``all_dots_collected`` from the
  plane, as the reference does (400, 529).
* ``info['rule_status']`` (the rule audit, 941-950) is computed by the k_rules kernel and laid
  out in the reference's dict shape by ``rules.rule_status``; ``rule_status=False`` skips it
  (then ``{}``).  After ``__init__`` (before any reset) it describes the loaded state with the
  start point visited; the reference audits once before marking it (182-185).
* ``render_mode='human'/'llm'`` needs pygame, which is not available: raises.
"""
from __future__ import annotations

import json
import os
from collections import OrderedDict

import numpy as np

from .core import SparcCore
from .puzzles import pack_rules, pack_table, process_puzzles
from .rules import RuleStatic, region_map_of, rule_status as _rule_status
from .spaces import Box, Dict, Discrete, Env, Text

_REWARD = {0: 0, 1: 0.01, -1: -0.01, 100: 1, -100: -1}   # code -> the reference's Python value


def reward_value(code):
    """int8 reward code -> the reference's value and type (SPaRC_Gym.py:1133, 1207-1223)."""
    return _REWARD[int(code)]


def text_grid_rows(raw):
    """The 'SPaRC' text grid (rows of one-character strings, row = y) from a puzzle's
    ``puzzle_array`` in any of the three forms _load_puzzle accepts (SPaRC_Gym.py:153-164):
    a 1-D object array of row arrays (parquet), a 2-D array, or nested sequences.  Always a
    fresh list of lists, which step() edits in place."""
    if isinstance(raw, np.ndarray) and raw.dtype == object and raw.ndim == 1:
        grid_rows = [r.astype(str).tolist() for r in raw]
    elif isinstance(raw, np.ndarray) and raw.ndim == 2:
        grid_rows = raw.astype(str).tolist()
    else:
        grid_rows = [[str(c) for c in row] for row in raw]
    w = len(grid_rows[0])
    if any(len(r) != w for r in grid_rows):
        raise ValueError("Non-rectangular SPaRC grid")
    return grid_rows


def text_obs(grid_rows):
    """_build_json_obs (SPaRC_Gym.py:988-992)."""
    return json.dumps(grid_rows, separators=(",", ":"))


def action_code(action):
    """Map a caller's action to 0..3, or 255 if `action in legal_actions` can never hold."""
    for k in range(4):
        try:
            if action == k:
                return k
        except Exception:  # noqa: BLE001
            return 255
    return 255


def load_puzzle_source(puzzles, df_name, df_split, df_set):
    """The puzzle DataFrame of SPaRC_Gym.__init__ (77-78).

    ``puzzles`` may be a DataFrame, a list of records, or a local path: a ``.parquet`` file, a
    directory of parquet files (a local export of the ``lkaesberg/SPaRC`` split, read in sorted
    file order), or a ``.json`` / ``.jsonl`` file of records.  Without ``puzzles`` the hub
    dataset is loaded as the reference does (needs the network, or a local HF cache)."""
    if puzzles is None:
        from datasets import load_dataset   # SPaRC_Gym.py:77-78
        return load_dataset(df_name, df_split, split=df_set).to_pandas()
    if isinstance(puzzles, (str, os.PathLike)):
        return load_local(os.fspath(puzzles))
    return puzzles


def load_local(path):
    """DataFrame of SPaRC records from a local parquet file / directory or json(l) file."""
    import pandas as pd
    if os.path.isdir(path):
        files = sorted(os.path.join(path, f) for f in os.listdir(path) if f.endswith(".parquet"))
        if not files:
            raise ValueError(f"no .parquet files in {path}")
        return pd.concat([pd.read_parquet(f) for f in files], ignore_index=True)
    if path.endswith(".parquet"):
        return pd.read_parquet(path)
    if path.endswith(".jsonl"):
        return pd.read_json(path, lines=True, dtype=False)
    if path.endswith(".json"):
        return pd.read_json(path, dtype=False)
    raise ValueError(f"unsupported puzzle file {path!r} (.parquet, a parquet directory, .json or .jsonl)")


class SPaRC_Gym(Env):
    metadata = {"render_modes": ["human", "llm"], "render_fps": 30}

    def __init__(self, df_name="lkaesberg/SPaRC", df_split="all", df_set="test", render_mode=None,
                 observation="new", traceback=False, max_steps=2000, puzzles=None, device=0, rule_status=True,
                 alias_compat=False, fit_cap=None):
        self.render_mode = render_mode
        self.alias_compat = bool(alias_compat)
        self.observation = observation
        self.traceback = traceback
        self.max_steps = max_steps
        if render_mode in ("human", "llm"):
            raise NotImplementedError("pygame renderers are not part of this build (render_mode must be None)")
        df = load_puzzle_source(puzzles, df_name, df_split, df_set)
        self.current_puzzle_index = 0
        self.current_step = 0
        self.rule_status = {}
        if df is None or isinstance(df, Exception):
            raise ValueError("No valid dataframe provided")                          # 86-87
        self.puzzles = process_puzzles(df, observation)
        self._core = SparcCore(pack_table(self.puzzles), 1, traceback, max_steps, "none", device)
        self._audit = bool(rule_status)
        if fit_cap is not None:   # GPU node cap of one exact fit (the host finishes longer searches)
            self._core.set_rule_limits(fit_cap, 0)
        if self._audit:
            self._core.load_rules(pack_rules(self.puzzles, self._core.table))
        self._legal = 0
        self._rec = None          # the last one-env record (sparc_env_*), its audit for _validate_rules
        self._bit_index = {}      # (x_size, y_size) -> visited-board word / bit of every plane cell
        self._rstatic = {}        # puzzle index -> rules.RuleStatic (what rule_status reads of the puzzle)
        self._load_puzzle(self.current_puzzle_index)
        self._validate_rules()                                                       # 182

    # ------------------------------------------------------------------ loading
    def _load_puzzle(self, index):
        """SPaRC_Gym.py:95-217 (fresh planes; see module docstring)."""
        puzzle = self.puzzles[index]
        self.difficulty = puzzle["difficulty"]
        self.polyshapes = puzzle["polyshapes"]
        self.x_size, self.y_size = puzzle["x_size"], puzzle["y_size"]
        if self.alias_compat:   # the puzzle's own planes, aliased across re-loads (149-151)
            self.obs_array = puzzle["obs_array"]
        else:
            self.obs_array = OrderedDict((k, v.copy()) for k, v in puzzle["obs_array"].items())
        self.color_array = puzzle["color_array"]
        self.additional_info = puzzle["additional_info"]
        if self.observation == "SPaRC":                                              # 153-164
            self.observ = text_grid_rows(puzzle["observ"])
        self.start_location = puzzle["start_location"]
        self.target_location = puzzle["target_location"]
        self.solution_paths = puzzle["solution_paths"]
        self.solution_count = puzzle["solution_count"]
        self.path = [[self.start_location[0], self.start_location[1]]]
        self.normal_reward = 0
        self.outcome_reward = 0
        self.rule_status = {}
        self._agent_location = np.array([self.start_location[0], self.start_location[1]], dtype=np.int32)
        self._target_location = np.array([self.target_location[0], self.target_location[1]], dtype=np.int32)

        if self.alias_compat:
            self._rec = None
            flags = self._core.reset_host(np.array([index], np.uint32))
            self._legal = int(flags[0] >> 2) & 0xF
            sx, sy = int(self.start_location[0]), int(self.start_location[1])
            vis = self.obs_array["visited"]
            vis[sx, sy] = 1                                                          # 185
            self._core.set_visited_host(self._plane_words(vis))
            self._legal = self._start_legal_mask()
            self.obs_array["agent_location"][sx, sy] = 1                             # 186
            st = self._core.read_state()
            self.current_step = int(st["step"][0])
            self.outcome_reward = int(st["outcome"][0])
        else:
            # reset, the new state and its rule audit in one round trip (sparc_env_reset)
            rec = self._core.env_reset(index, audit=self._audit)
            self._apply_record(rec)
            self._legal = (rec.flags >> 2) & 0xF
        self.obs_array["target_location"][self._target_location[0], self._target_location[1]] = 1

        if self.observation == "new":                                                # 190-196
            keys = list(self.obs_array.keys())
            self.observation_space = Dict({
                "base": Dict({k: Box(low=0, high=1, shape=(self.x_size, self.y_size), dtype=np.int32) for k in keys}),
                "color": Box(low=0, high=8, shape=(self.x_size, self.y_size), dtype=np.int32),
                "additional_info": Box(low=0, high=143632, shape=(self.x_size, self.y_size), dtype=np.int64),
            })
        elif self.observation == "SPaRC":                                            # 198-204
            init_json = self._build_json_obs()
            charset = "".join(sorted(set(init_json) | set("LV.")))
            self._json_charset = charset
            self.observation_space = Text(max_length=int(len(init_json) * 2), charset=charset)
        else:
            raise ValueError("Invalid observation type. Choose 'new' or 'SPaRC'.")
        self.action_space = Discrete(4)                                              # 210
        self._action_to_direction = {0: np.array([1, 0]), 1: np.array([0, -1]),
                                     2: np.array([-1, 0]), 3: np.array([0, 1])}

    def _apply_record(self, rec):
        """The device state of a one-env record -> visited / agent_location planes, step, outcome
        (fresh planes: the agent plane holds the agent alone).  Keeps the record for the audit."""
        X, Y = self.x_size, self.y_size
        idx = self._bit_index.get((X, Y))
        if idx is None:
            pitch = self._core.table.pitch
            xs, ys = np.meshgrid(np.arange(X), np.arange(Y), indexing="ij")
            b = (xs * pitch + ys).astype(np.uint64)
            idx = self._bit_index[(X, Y)] = ((b >> np.uint64(6)).astype(np.int64), b & np.uint64(63))
        words = np.frombuffer(rec.visited, dtype=np.uint64)
        self.obs_array["visited"][...] = ((words[idx[0]] >> idx[1]) & np.uint64(1)).astype(np.int32)
        agent = self.obs_array["agent_location"]
        agent[...] = 0
        agent[rec.x, rec.y] = 1
        self.current_step = int(rec.step)
        self.outcome_reward = int(rec.outcome)
        self._rec = rec
        return rec.x, rec.y, rec.path_len

    def _sync_planes(self, old=None):
        """Mirror visited / agent_location planes from the device state.  alias_compat: the
        agent plane is edited as the reference edits it (the point left -> 0, the new point
        -> 1, 1145-1157 / 1170-1179), so stale bits of an earlier episode stay."""
        st = self._core.read_state()
        X, Y, pitch = self.x_size, self.y_size, self._core.table.pitch
        bits = st["visited"][:, 0]
        xs, ys = np.meshgrid(np.arange(X), np.arange(Y), indexing="ij")
        b = (xs * pitch + ys).astype(np.uint64)
        vis = ((bits[(b >> np.uint64(6)).astype(np.int64)] >> (b & np.uint64(63))) & np.uint64(1)).astype(np.int32)
        self.obs_array["visited"][...] = vis
        agent = self.obs_array["agent_location"]
        x, y = int(st["x"][0]), int(st["y"][0])
        if not self.alias_compat:
            agent[...] = 0
        elif old is not None and old != (x, y):
            agent[old[0], old[1]] = 0
        agent[x, y] = 1
        self.current_step = int(st["step"][0])
        self.outcome_reward = int(st["outcome"][0])
        return x, y, int(st["path_len"][0])

    def _plane_words(self, plane):
        """[X][Y] 0/1 plane -> the device's visited board [words][1] (bit x * pitch + y)."""
        W, pitch = self._core.table.words, self._core.table.pitch
        words = np.zeros((W, 1), np.uint64)
        for x, y in zip(*np.nonzero(np.asarray(plane))):
            b = int(x) * pitch + int(y)
            words[b >> 6, 0] |= np.uint64(1) << np.uint64(b & 63)
        return words

    def _start_legal_mask(self):
        """_get_legal_actions (1024-1051) at a fresh start (path of one point): in bounds, not a
        gap, not visited (the aliased plane may hold stale bits)."""
        m = 0
        sx, sy = int(self.start_location[0]), int(self.start_location[1])
        for a, (dx, dy) in enumerate(((1, 0), (0, -1), (-1, 0), (0, 1))):
            nx, ny = sx + dx, sy + dy
            if 0 <= nx < self.x_size and 0 <= ny < self.y_size and self.obs_array["gaps"][nx, ny] == 0 \
                    and self.obs_array["visited"][nx, ny] == 0:
                m |= 1 << a
        return m

    # ------------------------------------------------------------------ gym API
    def reset(self, seed=None, options=None):
        """SPaRC_Gym.py:1057-1108."""
        super().reset(seed=seed)
        if options is not None:
            puzzle_id = options.get("puzzle_id", None)
            for idx, puzzle in enumerate(self.puzzles):
                if puzzle["id"] == puzzle_id:
                    self.current_puzzle_index = idx
                    break
        elif seed is not None:
            self.current_puzzle_index = int(self.np_random.integers(len(self.puzzles)))
        else:
            self.current_puzzle_index = (self.current_puzzle_index + 1) % len(self.puzzles)
        self.current_step = 0
        self._load_puzzle(self.current_puzzle_index)
        return self._get_obs(), self._get_info()

    def step(self, action):
        """SPaRC_Gym.py:1111-1238; the transition runs in the HIP step kernel.  Without
        alias_compat the step, the new state and the rule audit of _get_info come back in ONE
        round trip (sparc_env_step: one stream synchronisation)."""
        old = (int(self._agent_location[0]), int(self._agent_location[1]))
        if self.alias_compat:
            codes, flags = self._core.step_host(np.array([action_code(action)], np.uint8))
            x, y, plen = self._sync_planes(old)
            code, f = int(codes[0]), int(flags[0])
        else:
            rec = self._core.env_step(action_code(action), audit=self._audit)
            x, y, plen = self._apply_record(rec)
            code, f = int(rec.reward_code), int(rec.flags)
        if (x, y) != old:
            if plen < len(self.path):                                                # traceback pop
                if self.observation == "SPaRC":
                    self.observ[old[1]][old[0]] = "." if self.obs_array["gaps"][old[0], old[1]] == 1 else "+"
                del self.path[-1]
            else:
                if self.observation == "SPaRC":
                    self.observ[old[1]][old[0]] = "V"
                self.path.append([x, y])
            if self.observation == "SPaRC":
                self.observ[y][x] = "L"
            self._agent_location = np.array([x, y], dtype=np.int64)
        terminated, truncated = bool(f & 1), bool(f & 2)
        self._legal = (f >> 2) & 0xF
        self.normal_reward = reward_value(code)
        return self._get_obs(), self.normal_reward, terminated, truncated, self._get_info()

    def _get_obs(self):
        if self.observation == "new":                                                # 978-979
            return {"base": self.obs_array, "color": self.color_array, "additional_info": self.additional_info}
        if self.observation == "SPaRC":
            return self._build_json_obs()
        raise ValueError("Invalid observation type. Choose 'new' or 'SPaRC'.")

    def _build_json_obs(self):
        return text_obs(self.observ)

    def _validate_rules(self, terminated=False, truncated=False):
        """_validate_rules (SPaRC_Gym.py:941-950): the audit runs in the k_rules kernel."""
        if not self._audit:
            self.rule_status = {}
            return self.rule_status
        if not self.alias_compat:
            # the audit of the current state: from the last step / reset record, else one read
            rec = self._rec if self._rec is not None and self._rec.audited else self._core.env_read(audit=True)
            self._rec = rec
            W = self._core.table.words
            r = {"bits": [rec.rule_bits], "region": [np.frombuffer(rec.region, np.uint8)[:64 * W]],
                 "fit": [rec.fit]}
        else:
            r = self._core.rules_host(region=True, fit=True)
        if self.alias_compat:
            # the path-based rules and the regions read self.path (400, 503-515, 639), the dots
            # rule the visited plane (529): with stale plane bits the audit runs on the path's
            # points, and the dots bit comes from the audit of the plane
            path_plane = np.zeros_like(self.obs_array["visited"])
            for px, py in self.path:
                path_plane[px, py] = 1
            if (path_plane != self.obs_array["visited"]).any():
                self._core.set_visited_host(self._plane_words(path_plane))
                rp = self._core.rules_host(region=True, fit=True)
                self._core.set_visited_host(self._plane_words(self.obs_array["visited"]))
                dots = 1 << 3   # all_dots_collected (RULE_NAMES order)
                bits = (int(rp["bits"][0]) & ~dots & ~(1 << 8)) | (int(r["bits"][0]) & dots)
                if (bits & 0xFF) == 0xFF:
                    bits |= 1 << 8   # all_rules_satisfied: every core rule (931-934)
                rp["bits"][0] = bits
                r = rp
        rmap = region_map_of(r["region"][0], self.x_size, self.y_size, self._core.table.pitch)
        q = self.current_puzzle_index
        st = self._rstatic.get(q)
        if st is None:
            st = self._rstatic[q] = RuleStatic(self.puzzles[q], self.obs_array)
        self.rule_status = _rule_status(self.puzzles[q], self.obs_array, self.path, self._agent_location,
                                        self._target_location, r["bits"][0], rmap, r["fit"][0], terminated,
                                        truncated, static=st)
        return self.rule_status

    def _get_legal_actions(self):
        return [a for a in range(4) if (self._legal >> a) & 1]

    def _get_info(self):
        """SPaRC_Gym.py:994-1022."""
        self._validate_rules(terminated=False, truncated=False)
        return {"solution_count": self.solution_count,
                "difficulty": self.difficulty,
                "grid_x_size": self.x_size,
                "grid_y_size": self.y_size,
                "legal_actions": self._get_legal_actions(),
                "current_step": self.current_step,
                "agent_location": self._agent_location,
                "rule_status": self.rule_status,
                "Rewards": {"normal_reward": self.normal_reward, "outcome_reward": self.outcome_reward}}

    def render(self):
        return None

    def close(self):
        """SPaRC_Gym.py:1301-1311 closes only the renderers; the env stays usable."""
        return None
