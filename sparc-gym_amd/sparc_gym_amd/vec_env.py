"""SPaRCVecEnv: thousands of SPaRC envs stepped together on one MI355X.

The batched form of the reference's ``reset()/step()`` (SPaRC_Gym.py:1057-1238).  State lives in
HBM as a structure of arrays owned by the C context; every call is one HIP launch on the
caller's torch stream, and results stay on the GPU as torch tensors (no host round trip).

    vec = SPaRCVecEnv(65536, puzzles=records, traceback=True)
    obs, info = vec.reset(seed=0)
    obs, reward, terminated, truncated, info = vec.step(actions)   # actions: [N] on the GPU
    out = vec.rollout(T, actions=None, seed=1)                      # T steps in one launch

Autoreset follows gymnasium's next-step convention by default: the step after an env
terminates/truncates resets it onto the next puzzle ((index + 1) % P, the reference's plain
``reset()`` at SPaRC_Gym.py:1087) and ignores that step's action.  ``autoreset='none'``
reproduces the reference exactly (stepping past the end keeps the finished state).

Observations (``observation='new'``): ``visited`` and ``agent_location`` as int32 planes
[N, x_dim, y_dim] (padded lattice) written by the obs-pack kernel, plus ``puzzle_index``; the
static planes (gaps, target, symbols, color, additional_info) of every puzzle are in
``static_planes`` and ``static_keys`` (``static_planes[puzzle_index]`` gives an env's).
``observation='compact'`` returns only ``puzzle_index`` and the agent location.

Rule audit (``rules=True``, or ``rule_audit()`` on demand): the reference's
``info['rule_status']`` (SPaRC_Gym.py:941-950) evaluated by the k_rules kernel for every env,
as ``info['rule_bits']`` [N] int16 with bit k = ``RULE_NAMES[k]`` passed.  An exact-fit search
that passes the GPU's node cap (``fit_cap``, default 2^26) is finished on the host without a
cap, as the reference's unbounded search (sparc_rules_finish): the bits are always final.
"""
from __future__ import annotations

import numpy as np
import torch

from .core import SparcCore
from .env import load_puzzle_source
from .puzzles import pack_rules, pack_table, process_puzzles

RULE_NAMES = ("reached_target", "path_not_crossing", "no_gap_violations", "all_dots_collected",
              "square_color_separation", "star_pairing_exact", "triangles_edge_count", "poly_ylop_area",
              "all_rules_satisfied")   # _run_rule_validators order, SPaRC_Gym.py:908-936

# reward code -> float64 value; code/100 in float64 is exactly the reference's 0.01/-0.01 double
REWARD_SCALE = 100.0


def xcd_local_puzzle_index(num_envs, num_puzzles, env_offset=0):
    """First puzzles for a batched reset (``reset(options={'puzzle_index': ...})``) that keep each
    XCD's L2 on one eighth of a large pool.  The split rollout kernel runs 256 envs per workgroup
    and the MI355X deals workgroups round-robin over its 8 XCDs (workgroups b, b + 8, ... share
    one XCD and its 4 MB L2), so env slot s belongs to XCD group g = (s // 256) % 8; it gets a
    puzzle of block g of the pool, [g * P/8, (g+1) * P/8), by a multiplicative hash of its index
    within the group (plus env_offset, so shards differ).  Every puzzle starts equally many envs
    (num_envs a multiple of 2,048 and P of 8); next-step autoresets walk on from the start
    puzzle (reset(), SPaRC_Gym.py:1087).  With env i on puzzle i * 2654435761 mod P every XCD
    touches the whole pool instead (MI355X, c3 at 16,384 puzzles: 0.353 against 0.404 ms per
    2,000-step launch; the library then also keeps the shorter 8-B trie records,
    sparc_reset_host).  P < 8 or P % 8 != 0: the plain hash."""
    P = int(num_puzzles)
    slot = np.arange(int(num_envs), dtype=np.uint64)
    if P < 8 or P % 8:
        return ((slot + np.uint64(env_offset)) * np.uint64(2654435761) % np.uint64(P)).astype(np.int64)
    span = np.uint64(P // 8)
    grp = (slot // np.uint64(256)) % np.uint64(8)
    k = (slot // np.uint64(2048)) * np.uint64(256) + slot % np.uint64(256) + np.uint64(env_offset)
    return (grp * span + k * np.uint64(2654435761) % span).astype(np.int64)


class SPaRCVecEnv:
    def __init__(self, num_envs, puzzles=None, df_name="lkaesberg/SPaRC", df_split="all", df_set="test",
                 observation="new", traceback=False, max_steps=2000, autoreset="next_step", device=0,
                 env_offset=0, pitch=None, words=None, processed=None, table=None, rules=False, copy=True,
                 fit_cap=None, rule_table_entries=None):
        if observation not in ("new", "compact"):
            raise ValueError("observation must be 'new' or 'compact' for the vector env")
        self.num_envs = int(num_envs)
        self.observation = observation
        # copy=True (gymnasium's vector-env default): every step() returns observation tensors
        # of its own, so an (obs, next_obs) pair kept by the caller stays intact; copy=False
        # returns the env's buffers, overwritten in place by the next step (the reference's
        # by-reference planes, SPaRC_Gym.py:979)
        self.copy = bool(copy)
        self.traceback = bool(traceback)
        self.max_steps = max_steps
        self.autoreset = autoreset
        self.device = torch.device("cuda", device)
        if processed is None:
            processed = process_puzzles(load_puzzle_source(puzzles, df_name, df_split, df_set))
        self.puzzles = processed
        self.table = table if table is not None else pack_table(processed, pitch, words)
        self.num_puzzles = self.table.num_puzzles
        self.core = SparcCore(self.table, self.num_envs, traceback, max_steps, autoreset, device, env_offset)
        # rule-audit limits (tests force the host fallback of the exact fit with a tiny cap)
        if fit_cap is not None or rule_table_entries is not None:
            self.core.set_rule_limits(fit_cap or 0, rule_table_entries or 0)
        self.x_dim, self.y_dim = self.table.x_max, self.table.y_max
        n, dev = self.num_envs, self.device
        self._act = torch.empty(n, dtype=torch.uint8, device=dev)
        self._rew = torch.empty(n, dtype=torch.int8, device=dev)
        self._flags = torch.empty(n, dtype=torch.uint8, device=dev)
        self._pidx = torch.empty(n, dtype=torch.int32, device=dev)
        self._pos = torch.empty(n, dtype=torch.int32, device=dev)
        self._loc = torch.empty((n, 2), dtype=torch.int32, device=dev)
        if observation == "new":
            self._vis = torch.empty((n, self.x_dim, self.y_dim), dtype=torch.int32, device=dev)
            self._agent = torch.empty_like(self._vis)
            self._build_static()
        self._cursor = np.arange(n, dtype=np.int64) % self.num_puzzles   # "__init__ loads" env i -> i mod P
        self.rules = bool(rules)
        self._rbits = None
        if self.rules:
            self._load_rules()
        self._np_random = None
        self._bound_stream = None

    # ------------------------------------------------------------------ helpers
    def _stream(self):
        s = torch.cuda.current_stream(self.device)
        if self._bound_stream != s.cuda_stream:
            self.core.set_stream(s.cuda_stream)
            self._bound_stream = s.cuda_stream
        return s

    def _build_static(self):
        keys = []
        for p in self.puzzles:
            for k in p["obs_array"]:
                if k not in keys and k not in ("visited", "agent_location"):
                    keys.append(k)
        self.static_keys = keys + ["color", "additional_info"]
        P, X, Y = self.num_puzzles, self.x_dim, self.y_dim
        st = np.zeros((P, len(self.static_keys), X, Y), np.int64)
        for q, p in enumerate(self.puzzles):
            px, py = p["x_size"], p["y_size"]
            for j, k in enumerate(keys):
                if k in p["obs_array"]:
                    st[q, j, :px, :py] = p["obs_array"][k]
            tx, ty = p["target_location"]
            st[q, keys.index("target_location"), :, :] = 0
            st[q, keys.index("target_location"), tx, ty] = 1
            st[q, -2, :px, :py] = p["color_array"]
            st[q, -1, :px, :py] = p["additional_info"]
        self.static_planes = torch.from_numpy(st).to(self.device)

    def _obs(self):
        """Observation of the current state (after reset): separate copy / obs-pack launches."""
        self.core.copy_state_device(4, self._pidx.data_ptr())
        self.core.copy_state_device(1, self._pos.data_ptr())
        if self.observation == "new":
            self.core.obs_pack_device(self._vis.data_ptr(), self._agent.data_ptr(), self.x_dim, self.y_dim)
        return self._obs_dict()

    def _stage_host_actions(self, actions, stream):
        """numpy integer actions -> the device through pinned int64 staging buffers (two, used
        alternately) and an asynchronous copy on the step's stream (torch.as_tensor of a
        pageable array is a synchronous copy; tools/prof_vec_step.py).  A buffer's event,
        recorded on the stream that runs its copy, keeps a later call from overwriting it before
        the copy has read it.  The device copy is a fresh allocation on that stream (the caching
        allocator orders its reuse on the stream), so a caller that switches streams between
        steps cannot overwrite actions a previous step's kernel is still reading."""
        n = self.num_envs
        if getattr(self, "_pin", None) is None:
            self._pin = [torch.empty(n, dtype=torch.int64, pin_memory=True) for _ in range(2)]
            self._pin_done = [None, None]
            self._pin_k = 0
        k = self._pin_k = self._pin_k ^ 1
        if self._pin_done[k] is not None:
            self._pin_done[k].synchronize()
        np.copyto(self._pin[k].numpy(), actions, casting="unsafe")   # integer widening only
        act = torch.empty(n, dtype=torch.int64, device=self.device)
        act.copy_(self._pin[k], non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(stream)
        self._pin_done[k] = ev
        return act

    def _step_obs_dict(self, bufs):
        """_obs_dict after step_gym_device, which wrote the agent's (x, y) into loc itself."""
        vis, agent, pidx, loc = bufs
        if self.observation == "compact":
            return {"puzzle_index": pidx, "agent_location": loc}
        return {"visited": vis, "agent_location": agent, "puzzle_index": pidx, "agent_xy": loc}

    def _step_obs_buffers(self):
        """(visited, agent_location, puzzle_index, agent_xy) targets of one step: fresh tensors
        with copy=True, else the env's own buffers."""
        if not self.copy:
            new = self.observation == "new"
            return (self._vis if new else None, self._agent if new else None, self._pidx, self._loc)
        n, dev = self.num_envs, self.device
        vis = agent = None
        if self.observation == "new":
            vis = torch.empty((n, self.x_dim, self.y_dim), dtype=torch.int32, device=dev)
            agent = torch.empty_like(vis)
        return (vis, agent, torch.empty(n, dtype=torch.int32, device=dev),
                torch.empty((n, 2), dtype=torch.int32, device=dev))

    def _obs_dict(self):
        loc = torch.stack([self._pos & 0xFF, (self._pos >> 8) & 0xFF], dim=1)
        pidx = self._pidx.clone() if self.copy else self._pidx
        if self.observation == "compact":
            return {"puzzle_index": pidx, "agent_location": loc}
        if self.copy:
            return {"visited": self._vis.clone(), "agent_location": self._agent.clone(), "puzzle_index": pidx,
                    "agent_xy": loc}
        return {"visited": self._vis, "agent_location": self._agent, "puzzle_index": pidx, "agent_xy": loc}

    def _load_rules(self):
        if self._rbits is None:
            self.core.load_rules(pack_rules(self.puzzles, self.table))
            self._rbits = torch.empty(self.num_envs, dtype=torch.int16, device=self.device)

    def rule_audit(self, region=False, fit=False):
        """The rule audit of every env's current state on the GPU (k_rules): dict with ``bits``
        [N] int16 (bit k = RULE_NAMES[k] passed), optionally ``region`` [N, 64*words] uint8
        (region id per cell bit, the reference's numbering; 255 elsewhere) and ``fit`` [N]
        int64 (bit r: region r passed the poly/ylop area check and exact fit)."""
        self._stream()
        self._load_rules()
        n = self.num_envs
        out = {"bits": self._rbits}
        if region:
            out["region"] = torch.empty((n, 64 * self.table.words), dtype=torch.uint8, device=self.device)
        if fit:
            out["fit"] = torch.empty(n, dtype=torch.int64, device=self.device)
        self.core.rules_device(self._rbits.data_ptr(), out["region"].data_ptr() if region else None,
                               out["fit"].data_ptr() if fit else None)
        # exact fits that passed the GPU's node cap: finished on the host.  This synchronises the
        # stream (a 4-byte read of the queue count when nothing was queued), so rule_audit() and
        # step() with rules=True return final bits and are synchronous
        self.core.rules_finish(self._rbits.data_ptr(), out["fit"].data_ptr() if fit else None)
        return out

    @property
    def np_random(self):
        if self._np_random is None:
            self._np_random = np.random.Generator(np.random.PCG64(np.random.SeedSequence()))
        return self._np_random

    # ------------------------------------------------------------------ API
    def current_puzzle_indices(self):
        """[N] int64: each env's current puzzle index (the reference's current_puzzle_index),
        read from the device, so it follows the device's autoresets.  Before the first
        reset: env i -> i mod P (the vector form of __init__ loading puzzle 0, SPaRC_Gym.py:90)."""
        if not self.core.has_state:
            return self._cursor.copy()
        cur = torch.empty(self.num_envs, dtype=torch.int32, device=self.device)
        self.core.copy_state_device(4, cur.data_ptr())
        return cur.cpu().numpy().astype(np.int64)

    def reset(self, seed=None, options=None):
        """Per-env puzzle choice as SPaRC_Gym.reset (SPaRC_Gym.py:1075-1087), vectorised:
        * options given: options['puzzle_index'] ([N] ints, this build's extension) or
          options['puzzle_id'] (one id or [N] ids); an env whose id is missing (or any options
          without either key, e.g. {}) keeps its current puzzle (1076-1082);
        * else seed: Generator(PCG64(SeedSequence(seed))).integers(P, size=N) (1084-1085; env
          0 gets the reference's index);
        * else sequential: current index + 1 mod P (1087).
        "Current" is the device's puzzle index, which next-step autoresets advance."""
        self._stream()
        P = self.num_puzzles
        if options is not None and "puzzle_index" in options:
            q = np.asarray(options["puzzle_index"], np.int64)
        elif options is not None:
            cur = self.current_puzzle_indices()
            want = options.get("puzzle_id", None)
            if want is None:
                q = cur
            else:
                ids = {p["id"]: i for i, p in reversed(list(enumerate(self.puzzles)))}
                want = [want] * self.num_envs if isinstance(want, str) or not hasattr(want, "__len__") else list(want)
                if len(want) != self.num_envs:
                    raise ValueError(f"options['puzzle_id'] must be one id or {self.num_envs} ids")
                q = np.array([ids.get(w, c) for w, c in zip(want, cur)], np.int64)
        elif seed is not None:
            self._np_random = np.random.Generator(np.random.PCG64(np.random.SeedSequence(seed)))
            q = self._np_random.integers(P, size=self.num_envs)
        else:
            q = (self.current_puzzle_indices() + 1) % P
        if q.shape != (self.num_envs,) or q.min() < 0 or q.max() >= P:
            raise ValueError("puzzle indices must be [num_envs] in [0, num_puzzles)")
        self._cursor = q.copy()
        flags = self.core.reset_host(q.astype(np.uint32))
        info = {"legal_mask": torch.from_numpy(((flags >> 2) & 0xF).astype(np.uint8)).to(self.device)}
        if self.rules:
            info["rule_bits"] = self.rule_audit()["bits"]
        return self._obs(), info

    def step(self, actions):
        """One step() of every env: actions [N] (uint8: >= 4 is illegal = no move; other integer
        types: < 0 or >= 4 is illegal).  ONE launch (sparc_step_gym_device) writes the step, the
        post-step observation and the gym outputs: reward [N] float64 (the reference's exact
        values), terminated / truncated [N] bool, and info's legal_mask, autoreset and
        reward_code.  Every returned tensor is fresh per call (copy=True, the default); with
        copy=False the observation tensors and reward_code are the env's buffers, overwritten
        by the next step (the reference returns its planes by reference, SPaRC_Gym.py:979)."""
        self._stream()
        n = self.num_envs
        if isinstance(actions, np.ndarray) and actions.shape == (n,) and actions.dtype.kind in "iu":
            a = self._stage_host_actions(actions, torch.cuda.current_stream(self.device))
        else:
            a = torch.as_tensor(actions, device=self.device)
        if a.shape != (n,):
            raise ValueError(f"actions must have shape ({n},)")
        if a.dtype not in (torch.uint8, torch.int32, torch.int64):
            if a.dtype.is_floating_point or a.dtype == torch.bool:
                raise ValueError("actions must be integers")
            a = a.to(torch.int64)
        a = a.contiguous()
        # one allocation for the fresh outputs: reward f64 [N] | terminated | truncated | legal | autoreset
        buf = torch.empty(12 * n, dtype=torch.uint8, device=self.device)
        reward = buf[:8 * n].view(torch.float64)
        terminated = buf[8 * n:9 * n].view(torch.bool)
        truncated = buf[9 * n:10 * n].view(torch.bool)
        legal = buf[10 * n:11 * n]
        autoreset = buf[11 * n:].view(torch.bool)
        new = self.observation == "new"
        bufs = self._step_obs_buffers()
        vis, agent, pidx, loc = bufs
        self.core.step_gym_device(a.data_ptr(), a.element_size(), reward.data_ptr(), terminated.data_ptr(),
                                  truncated.data_ptr(), legal.data_ptr(), autoreset.data_ptr(), self._rew.data_ptr(),
                                  self._flags.data_ptr(), vis.data_ptr() if new else None,
                                  agent.data_ptr() if new else None, self.x_dim if new else 1,
                                  self.y_dim if new else 1, pidx.data_ptr(), loc.data_ptr())
        if self.copy:
            self._loc = loc   # the latest agent (x, y), as the step path wrote it
        info = {"legal_mask": legal, "autoreset": autoreset,
                "reward_code": self._rew.clone() if self.copy else self._rew}
        if self.rules:
            bits = self.rule_audit()["bits"]
            info["rule_bits"] = bits.clone() if self.copy else bits
        return self._step_obs_dict(bufs), reward, terminated, truncated, info

    def rollout(self, T, actions=None, seed=0, t0=0, stats=None, record=True, out=None, obs=False, obs_out=None,
                rules=False):
        """T steps of every env in ONE kernel launch.  actions: [T, N] uint8 on the GPU or None
        (counter-based random actions, sparc_rand_action(seed, env_offset + i, t0 + t)).
        Returns reward codes and flags [T, N] (int8 / uint8) if ``record`` (written into
        ``out=(reward_code, flags)`` when given).  With ``obs`` (or ``obs_out=(visited,
        agent_location)``) the 'new' observation after every step is recorded too: int32
        traces [T, N, x_dim, y_dim] under "visited" / "agent_location" (8 * x_dim * y_dim
        bytes per env-step of HBM writes).  With ``rules`` the rule audit runs after every step
        as in the reference's step() (SPaRC_Gym.py:1227): "rule_bits" [T, N] int16 (bit k =
        RULE_NAMES[k] passed), step t's bits equal rule_audit() after t + 1 single steps."""
        self._stream()
        n = self.num_envs
        if actions is not None:
            actions = torch.as_tensor(actions, device=self.device)
            if actions.shape != (T, n) or actions.dtype != torch.uint8 or not actions.is_contiguous():
                raise ValueError(f"actions must be a contiguous uint8 tensor of shape ({T}, {n})")
        rew = flags = None
        if out is not None:
            rew, flags = out
            for t_, dt in ((rew, torch.int8), (flags, torch.uint8)):
                if t_.shape != (T, n) or t_.dtype != dt or not t_.is_contiguous() or t_.device != self.device:
                    raise ValueError(f"out tensors must be contiguous [{T}, {n}] int8 / uint8 on {self.device}")
        elif record:
            rew = torch.empty((T, n), dtype=torch.int8, device=self.device)
            flags = torch.empty((T, n), dtype=torch.uint8, device=self.device)
        if stats is not None and (stats.shape != (n, 4) or stats.dtype != torch.int32 or not stats.is_contiguous()):
            raise ValueError("stats must be a contiguous int32 tensor [N, 4]")
        args = (None if actions is None else actions.data_ptr(), None if rew is None else rew.data_ptr(),
                None if flags is None else flags.data_ptr(), None if stats is None else stats.data_ptr())
        if rules:
            if obs or obs_out is not None:
                raise ValueError("rules=True records the rule bits only (no observation traces)")
            self._load_rules()
            bits = torch.empty((T, n), dtype=torch.int16, device=self.device)
            self.core.rollout_rules_device(T, *args, bits.data_ptr(), seed, t0)
            self.core.rules_finish(bits.data_ptr())   # searches past the GPU's node cap (a sync)
            return {"reward_code": rew, "flags": flags, "rule_bits": bits}
        if not obs and obs_out is None:
            self.core.rollout_device(T, *args, seed, t0)
            return {"reward_code": rew, "flags": flags}
        X, Y = self.x_dim, self.y_dim
        if obs_out is not None:
            vis, agent = obs_out
            for t_ in (vis, agent):
                if t_ is not None and (t_.shape != (T, n, X, Y) or t_.dtype != torch.int32 or
                                       not t_.is_contiguous() or t_.device != self.device):
                    raise ValueError(f"obs_out tensors must be contiguous int32 [{T}, {n}, {X}, {Y}] on {self.device}")
        else:
            vis = torch.empty((T, n, X, Y), dtype=torch.int32, device=self.device)
            agent = torch.empty_like(vis)
        self.core.rollout_obs_device(T, *args, None if vis is None else vis.data_ptr(),
                                     None if agent is None else agent.data_ptr(), X, Y, seed, t0)
        return {"reward_code": rew, "flags": flags, "visited": vis, "agent_location": agent}

    def random_actions(self, T, seed=0, t0=0, out=None):
        """[T, N] uint8 uniform random actions written on the GPU: ``action_space.sample()``
        (Final_Product.py:29) for every env and step, entry (t, i) = sparc_rand_action(seed,
        env_offset + i, t0 + t) — the actions ``rollout(T, None, seed, t0)`` draws, keyed by the
        global env id (a rank's shard holds the columns of one process over all envs)."""
        self._stream()
        n = self.num_envs
        if out is None:
            out = torch.empty((T, n), dtype=torch.uint8, device=self.device)
        elif out.shape != (T, n) or out.dtype != torch.uint8 or not out.is_contiguous() or out.device != self.device:
            raise ValueError(f"out must be a contiguous uint8 tensor [{T}, {n}] on {self.device}")
        self.core.random_actions_device(T, out.data_ptr(), seed, t0)
        return out

    def state(self):
        """Host snapshot of the per-env state (x, y, path_len, step, puzzle, outcome, visited bits)."""
        torch.cuda.current_stream(self.device).synchronize()
        return self.core.read_state()

    def close(self):
        self.core.close()
