"""SparcCore: owns one C-ABI context (one GPU, one batch of envs) and its calls.

Thin, typed wrapper over include/sparc_gym_amd.h used by SPaRCVecEnv (batched) and SPaRC_Gym
(batch of one).  Device pointers are plain ints (e.g. torch ``tensor.data_ptr()``).
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from .puzzles import PuzzleTable, RulesTable

INT32_MAX = 2**31 - 1


def _ptr(a):
    return None if a is None else a.ctypes.data


class SparcCore:
    def __init__(self, table: PuzzleTable, num_envs: int, traceback=False, max_steps=2000,
                 autoreset="none", device=0, env_offset=0):
        self.lib = _lib.load()
        if autoreset not in _lib.AUTORESET:
            raise ValueError(f"autoreset must be one of {sorted(_lib.AUTORESET)}")
        self.table = table
        self.num_envs = int(num_envs)
        self.traceback = bool(traceback)
        self.max_steps = int(max(min(int(max_steps), INT32_MAX), -INT32_MAX - 1))
        self.device = int(device)
        cfg = _lib.SparcConfig(self.num_envs, int(self.traceback), self.max_steps, _lib.AUTORESET[autoreset],
                               table.pitch, table.words, int(env_offset))
        ctx = ctypes.c_void_p()
        _lib.check(self.lib.sparc_create(self.device, ctypes.byref(cfg), ctypes.byref(ctx)))
        self.ctx = ctx
        self.load_table(table)

    # ---------------------------------------------------------------- lifecycle
    def load_table(self, table: PuzzleTable):
        open_ = np.ascontiguousarray(table.open, np.uint64)
        info = np.ascontiguousarray(table.info, np.uint32)
        trie = np.ascontiguousarray(table.trie, np.uint32)
        t = _lib.SparcPuzzleTable(len(info), len(trie), open_.ctypes.data, info.ctypes.data,
                                  trie.ctypes.data if len(trie) else None)
        self._check(self.lib.sparc_load_puzzles(self.ctx, ctypes.byref(t)))
        self.table = table
        self.has_state = False   # as the context: the old state may name puzzles that are gone

    def load_rules(self, rt: RulesTable):
        """Upload the rule-audit table (puzzles.pack_rules) for the loaded puzzles."""
        planes = np.ascontiguousarray(rt.planes, np.uint64)
        first = np.ascontiguousarray(rt.inst_first, np.uint32)
        inst = np.ascontiguousarray(rt.inst, np.uint32)
        sf = np.ascontiguousarray(rt.shape_first, np.uint32)
        sa = np.ascontiguousarray(rt.shape_area, np.int32)
        so = np.ascontiguousarray(rt.shape_off, np.int8)
        t = _lib.SparcRulesTable(len(first) - 1, len(inst), len(sa), len(so), planes.ctypes.data, first.ctypes.data,
                                 inst.ctypes.data if len(inst) else None, sf.ctypes.data,
                                 sa.ctypes.data if len(sa) else None, so.ctypes.data if len(so) else None)
        self._check(self.lib.sparc_load_rules(self.ctx, ctypes.byref(t)))
        self.rules = rt

    def rules_host(self, region=False, fit=False):
        """Rule audit of every env's current state: dict of bits [N] uint16 (+ region
        [N][64*words] uint8, fit [N] uint64 when asked)."""
        n, W = self.num_envs, self.table.words
        out = {"bits": np.empty(n, np.uint16)}
        if region:
            out["region"] = np.empty((n, 64 * W), np.uint8)
        if fit:
            out["fit"] = np.empty(n, np.uint64)
        self._check(self.lib.sparc_rules_host(self.ctx, _ptr(out["bits"]), _ptr(out.get("region")),
                                              _ptr(out.get("fit"))))
        return out

    def rules_device(self, d_bits, d_region=None, d_fit=None):
        self._check(self.lib.sparc_rules_device(self.ctx, d_bits, d_region, d_fit))

    def rules_finish(self, d_bits, d_fit=None):
        """Finish, on the host and without a node cap, the exact-fit searches of the last audit
        call that passed the GPU's cap, and patch its bits (and fit) in place (synchronous)."""
        self._check(self.lib.sparc_rules_finish(self.ctx, d_bits, d_fit))

    def rules_queue_stats(self):
        """The exact-fit queue: capacity, searches the last rules_finish ran on the host, calls
        run again after a queue overflow."""
        out = np.zeros(3, np.uint64)
        self._check(self.lib.sparc_rules_queue_stats(self.ctx, out.ctypes.data))
        return {"capacity": int(out[0]), "last_searches": int(out[1]), "reruns": int(out[2])}

    def set_rule_limits(self, fit_cap=0, table_entries=0):
        """GPU node cap of one exact-fit search (0: 2^26) and the region-code table budget in
        entries (0: 2^28); the budget applies at the next load_rules."""
        self._check(self.lib.sparc_set_rule_limits(self.ctx, int(fit_cap or 0), int(table_entries or 0)))

    # sparc_set_variant (include/sparc_gym_amd.h): kernel variants with identical results
    VARIANT_IO_CODES_OFF, VARIANT_RULE_ROLLOUT_GENERIC, VARIANT_R1R_SHAPE, VARIANT_OBS_INLINE = 1, 2, 3, 4
    VARIANT_MIXED_TRIE, VARIANT_HOST_FITS = 5, 6

    def set_variant(self, which, value):
        """Debug: select a kernel variant of identical results for this context (A/B, tests)."""
        self._check(self.lib.sparc_set_variant(self.ctx, int(which), int(value)))

    def close(self):
        if getattr(self, "ctx", None) is not None and self.ctx.value:
            self.lib.sparc_destroy(self.ctx)
        self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass

    def _check(self, rc):
        _lib.check(rc, self.ctx)

    def set_stream(self, stream_handle):
        """Order all calls on this HIP stream (int handle; 0 = the null stream, e.g. torch's
        default stream)."""
        self._check(self.lib.sparc_set_stream(self.ctx, stream_handle or None))

    def use_own_stream(self):
        self._check(self.lib.sparc_use_own_stream(self.ctx))

    def sync(self):
        self._check(self.lib.sparc_sync(self.ctx))

    # ---------------------------------------------------------------- host-pointer calls
    def reset_host(self, puzzle_index, mask=None):
        q = np.ascontiguousarray(puzzle_index, np.uint32)
        if q.shape != (self.num_envs,):
            raise ValueError(f"puzzle_index must have shape ({self.num_envs},)")
        m = None if mask is None else np.ascontiguousarray(mask, np.uint8)
        if m is not None and m.shape != (self.num_envs,):
            raise ValueError("mask shape mismatch")
        flags = np.zeros(self.num_envs, np.uint8)
        self._check(self.lib.sparc_reset_host(self.ctx, _ptr(q), _ptr(m), _ptr(flags)))
        self.has_state = True
        return flags

    def step_host(self, actions):
        a = np.ascontiguousarray(actions, np.uint8)
        if a.shape != (self.num_envs,):
            raise ValueError(f"actions must have shape ({self.num_envs},)")
        rew = np.empty(self.num_envs, np.int8)
        flags = np.empty(self.num_envs, np.uint8)
        self._check(self.lib.sparc_step_host(self.ctx, _ptr(a), _ptr(rew), _ptr(flags)))
        return rew, flags

    def read_state(self):
        n, W = self.num_envs, self.table.words
        out = {"x": np.empty(n, np.uint8), "y": np.empty(n, np.uint8), "path_len": np.empty(n, np.uint16),
               "step": np.empty(n, np.uint32), "puzzle": np.empty(n, np.uint32), "outcome": np.empty(n, np.int8),
               "pending": np.empty(n, np.uint8), "visited": np.empty((W, n), np.uint64)}
        s = _lib.SparcStateHost(*(out[k].ctypes.data for k in
                                  ("x", "y", "path_len", "step", "puzzle", "outcome", "pending", "visited")))
        self._check(self.lib.sparc_read_state(self.ctx, ctypes.byref(s)))
        return out

    # ---------------------------------------------------------------- one env, one round trip
    def env_step(self, action, audit=False, env=0):
        """sparc_env_step: step env `env` and return its record (state, reward code, flags and,
        with ``audit``, the rule audit of the new state) after ONE stream synchronisation."""
        rec = self._rec()
        self._check(self.lib.sparc_env_step(self.ctx, int(env), int(action), int(bool(audit)), ctypes.byref(rec)))
        return rec

    def env_reset(self, puzzle_index, audit=False, env=0):
        rec = self._rec()
        self._check(self.lib.sparc_env_reset(self.ctx, int(env), int(puzzle_index), int(bool(audit)),
                                             ctypes.byref(rec)))
        self.has_state = True
        return rec

    def env_read(self, audit=False, env=0):
        rec = self._rec()
        self._check(self.lib.sparc_env_read(self.ctx, int(env), int(bool(audit)), ctypes.byref(rec)))
        return rec

    def _rec(self):
        # a fresh record per call: a caller may keep the previous one
        return _lib.SparcEnvRecord()

    def set_visited_host(self, words):
        """Overwrite the visited boards [words][N] uint64 of the current state."""
        v = np.ascontiguousarray(words, np.uint64)
        if v.shape != (self.table.words, self.num_envs):
            raise ValueError(f"visited must have shape ({self.table.words}, {self.num_envs})")
        self._check(self.lib.sparc_set_visited_host(self.ctx, _ptr(v)))

    # ---------------------------------------------------------------- device-pointer calls (async)
    def reset_device(self, d_puzzle_index, d_mask=None, d_flags=None):
        self._check(self.lib.sparc_reset_device(self.ctx, d_puzzle_index, d_mask, d_flags))
        self.has_state = True

    def step_device(self, d_actions, d_reward, d_flags):
        self._check(self.lib.sparc_step_device(self.ctx, d_actions, d_reward, d_flags))

    def rollout_device(self, T, d_actions, d_reward, d_flags, d_stats=None, seed=0, t0=0):
        self._check(self.lib.sparc_rollout_device(self.ctx, int(T), d_actions, int(seed) & (2**64 - 1),
                                                  int(t0), d_reward, d_flags, d_stats))

    def random_actions_device(self, T, d_actions, seed=0, t0=0):
        """[T, N] uint8 counter-based random actions (global env ids) into device memory."""
        self._check(self.lib.sparc_random_actions_device(self.ctx, int(T), int(seed) & (2**64 - 1), int(t0),
                                                         d_actions))

    def step_obs_device(self, d_actions, d_reward, d_flags, d_visited, d_agent, x_dim, y_dim, d_puzzle=None,
                        d_xy=None):
        self._check(self.lib.sparc_step_obs_device(self.ctx, d_actions, d_reward, d_flags, d_visited, d_agent,
                                                   int(x_dim), int(y_dim), d_puzzle, d_xy))

    def step_gym_device(self, d_actions, action_bytes, d_reward=None, d_terminated=None, d_truncated=None,
                        d_legal=None, d_autoreset=None, d_reward_code=None, d_flags=None, d_visited=None,
                        d_agent=None, x_dim=1, y_dim=1, d_puzzle=None, d_loc=None):
        self._check(self.lib.sparc_step_gym_device(self.ctx, d_actions, int(action_bytes), d_reward, d_terminated,
                                                   d_truncated, d_legal, d_autoreset, d_reward_code, d_flags,
                                                   d_visited, d_agent, int(x_dim), int(y_dim), d_puzzle, d_loc))

    def rollout_obs_device(self, T, d_actions, d_reward, d_flags, d_stats, d_visited, d_agent, x_dim, y_dim,
                           seed=0, t0=0):
        self._check(self.lib.sparc_rollout_obs_device(self.ctx, int(T), d_actions, int(seed) & (2**64 - 1),
                                                      int(t0), d_reward, d_flags, d_stats, d_visited, d_agent,
                                                      int(x_dim), int(y_dim)))

    def rollout_rules_device(self, T, d_actions, d_reward, d_flags, d_stats, d_rule_bits, seed=0, t0=0):
        self._check(self.lib.sparc_rollout_rules_device(self.ctx, int(T), d_actions, int(seed) & (2**64 - 1),
                                                        int(t0), d_reward, d_flags, d_stats, d_rule_bits))

    def copy_state_device(self, which, d_out):
        self._check(self.lib.sparc_copy_state_device(self.ctx, int(which), d_out))

    def obs_pack_device(self, d_visited, d_agent, x_dim, y_dim):
        self._check(self.lib.sparc_obs_pack_device(self.ctx, d_visited, d_agent, int(x_dim), int(y_dim)))


def visited_planes(bits, table: PuzzleTable, x_dim=None, y_dim=None):
    """Decode visited bitboards [words][N] into int32 planes [N][x_dim][y_dim] (host)."""
    W, n = bits.shape
    x_dim = table.x_max if x_dim is None else x_dim
    y_dim = table.y_max if y_dim is None else y_dim
    xs, ys = np.meshgrid(np.arange(x_dim), np.arange(y_dim), indexing="ij")
    b = xs * table.pitch + ys
    valid = (ys < table.pitch) & (b < 64 * W)
    b = np.where(valid, b, 0)
    words = bits[(b >> 6), :]                                   # [x, y, N]
    v = (words >> (b & 63).astype(np.uint64)[..., None]) & np.uint64(1)
    v = np.where(valid[..., None], v, 0).astype(np.int32)
    return np.ascontiguousarray(np.moveaxis(v, -1, 0))
