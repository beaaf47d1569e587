"""Line-by-line Python model of sparc-gym_amd/csrc/sparc_env.hpp + k_rollout (TEST ONLY).

It executes the device algorithm (bitboards, 2-bit direction stack, trie node + off-trie depth,
the `rec` register and its invariant, node_term from the parent's child-terminal bits,
the carried legal mask, per-launch SoA load/store with the same bit packing) on
the host, so design errors in the kernel logic show up in the CPU suite instead of as GPU
faults.  It reads the packed PuzzleTable exactly as the kernel does, including the bounds
guard on trie indices (which must never fire).
"""
from __future__ import annotations

import numpy as np

NONE = 0xFFFF
SENTINEL = (0xFFFFFFFF, 0xFFFFFFFF, NONE, 0)
DX = (1, 0, -1, 0)
DY = (0, -1, 0, 1)


class KernelModel:
    def __init__(self, table, n, traceback, max_steps, autoreset):
        self.t = table
        self.n, self.tb, self.max_steps, self.autoreset = n, bool(traceback), int(max_steps), int(autoreset)
        W = table.words
        self.vis = np.zeros((W, n), np.uint64)
        self.dirs = np.zeros((2 * W, n), np.uint64)
        self.pos = np.zeros(n, np.uint32)
        self.aux = np.zeros(n, np.uint32)
        self.step_ = np.zeros(n, np.uint32)
        self.pid = np.zeros(n, np.uint32)
        self.guard_fired = False

    # ---------------------------------------------------------------- per-lane env (registers)
    def _puzzle(self, e, q):
        inf = [int(v) for v in self.t.info[q]]
        e["X"], e["Y"] = inf[0] & 0xFF, (inf[0] >> 8) & 0xFF
        sx, sy = (inf[0] >> 16) & 0xFF, inf[0] >> 24
        e["tx"], e["ty"], e["pflags"] = inf[1] & 0xFF, (inf[1] >> 8) & 0xFF, inf[1] >> 16
        e["trie_base"], e["trie_cnt"] = inf[2], inf[3]
        e["open"] = int(sum(int(w) << (64 * k) for k, w in enumerate(self.t.open[q])))
        return sx, sy

    def _load_rec(self, e):
        if e["node"] >= e["trie_cnt"]:
            self.guard_fired = True
            e["node"] = 0
        e["rec"] = tuple(int(v) for v in self.t.trie[e["trie_base"] + e["node"]])

    def _root(self, e, q):
        if e["pflags"] & 2:
            return tuple(int(v) for v in self.t.trie[e["trie_base"]])
        return SENTINEL

    def _reset(self, e, q):
        sx, sy = self._puzzle(e, q)
        e.update(pid=q, x=sx, y=sy, len=1, node=0, off=0 if e["pflags"] & 2 else 1, outcome=0,
                 pending=0, step=0, dirs=0, last=0, vis=1 << (sx * self.t.pitch + sy))
        e["rec"] = self._root(e, q)
        e["node_term"] = (e["rec"][2] >> 16) & 1
        e["legal"] = self._legal(e)

    def _dir_at(self, e, k):
        return (e["dirs"] >> (2 * k)) & 3

    def _legal(self, e):
        if self.t.words == 1:
            return self._legal_w1(e)
        back = (e["last"] ^ 2) if (self.tb and e["len"] >= 2) else 8
        m = 0
        for d in range(4):
            nx, ny = e["x"] + DX[d], e["y"] + DY[d]
            if not (0 <= nx < e["X"] and 0 <= ny < e["Y"]):
                continue
            b = nx * self.t.pitch + ny
            if (e["open"] >> b) & 1 and (not (e["vis"] >> b) & 1 or d == back):
                m |= 1 << d
        return m

    def _legal_w1(self, e):
        """Env<1, TB>::legal_mask: the free board (open, unvisited) stored one row up, shifted
        right by the agent's bit; out-of-lattice neighbours read 0 (empty bottom row, padding
        column, top row / bits shifted out of the 64-bit word)."""
        P, M = self.t.pitch, (1 << 64) - 1
        b = e["x"] * P + e["y"]
        fr = ((e["open"] & ~e["vis"]) << P) & M
        w = (fr >> b) & 0xFFFFFFFF
        m = ((w >> (2 * P)) & 1) | (((w >> (P - 1)) & 1) << 1) | ((w & 1) << 2) | (((w >> (P + 1)) & 1) << 3)
        if self.tb:
            bk = 0x7FFFFFFD + (0 if e["pflags"] & 4 else 1)   # (len + bk) >> 31: the traceback rule
            m |= (((e["len"] + bk) & 0xFFFFFFFF) >> 31) << (e["last"] ^ 2)
        return m

    def _advance(self, e, a):
        if self.autoreset == 1 and e["pending"]:
            q = 0 if e["pid"] + 1 == self.t.num_puzzles else e["pid"] + 1
            self._reset(e, q)
            return 0, (e["legal"] << 2) | 64
        legal = e["legal"]
        e["step"] = e["step"] + 1 if e["step"] < 0x7FFFFFFF else e["step"]
        trunc = e["step"] >= self.max_steps
        moved = a < 4 and (legal >> a) & 1
        if moved:
            nx, ny = e["x"] + DX[a], e["y"] + DY[a]
            b = nx * self.t.pitch + ny
            if self.t.words == 1:
                is_pop = self.tb and (a ^ 2) == e["last"] and e["len"] >= 2
            else:
                is_pop = self.tb and (e["vis"] >> b) & 1
            if is_pop:
                e["vis"] &= ~(1 << (e["x"] * self.t.pitch + e["y"]))
                e["len"] -= 1
                e["last"] = self._dir_at(e, e["len"] - 2 if e["len"] >= 2 else 0)
                if e["off"] > 0:
                    e["off"] -= 1
                else:
                    e["node_term"] = (e["rec"][2] >> 21) & 1
                    e["node"] = e["rec"][2] & 0xFFFF
                    self._load_rec(e)
            else:
                e["vis"] |= 1 << b
                k = e["len"] - 1
                e["dirs"] = (e["dirs"] & ~(3 << (2 * k))) | (a << (2 * k))
                e["last"] = a
                e["len"] += 1
                if e["off"] > 0:
                    e["off"] += 1
                else:
                    cw = e["rec"][0] if a < 2 else e["rec"][1]
                    c = (cw >> 16) if a & 1 else (cw & 0xFFFF)
                    if c != NONE:
                        e["node_term"] = (e["rec"][2] >> (17 + a)) & 1
                        e["node"] = c
                        self._load_rec(e)
                    else:
                        e["off"] = 1
            e["x"], e["y"] = nx, ny
            e["legal"] = self._legal(e)
        term = e["x"] == e["tx"] and e["y"] == e["ty"]
        legal2 = e["legal"]
        if legal2 == 0:
            trunc = True
        if term:
            trunc = False
        if term or trunc:
            if e["off"] == 0 and e["node_term"]:
                e["outcome"], code = 1, 100
            elif e["outcome"] != 1:
                e["outcome"], code = 2, -100
            else:
                code = 0
        else:
            e["outcome"] = 0
            code = 0 if (not moved or not e["pflags"] & 1) else (1 if e["off"] == 0 else -1)
        e["pending"] = 1 if (term or trunc) else 0
        return code, int(term) | (int(trunc) << 1) | (legal2 << 2)

    # ---------------------------------------------------------------- SoA <-> registers
    def _load(self, i):
        W = self.t.words
        e = {"vis": int(sum(int(self.vis[k, i]) << (64 * k) for k in range(W))),
             "dirs": int(sum(int(self.dirs[k, i]) << (64 * k) for k in range(2 * W))) if self.tb else 0}
        ps, ax = int(self.pos[i]), int(self.aux[i])
        e.update(x=ps & 0xFF, y=(ps >> 8) & 0xFF, len=(ps >> 16) & 0xFF, off=ps >> 24,
                 node=ax & 0xFFFF, outcome=(ax >> 16) & 3, pending=(ax >> 18) & 1, node_term=(ax >> 19) & 1,
                 step=int(self.step_[i]), pid=int(self.pid[i]))
        self._puzzle(e, e["pid"])
        if e["pflags"] & 2:
            self._load_rec(e)
        else:
            e["rec"] = SENTINEL
        e["last"] = self._dir_at(e, e["len"] - 2) if (self.tb and e["len"] >= 2) else 0
        e["legal"] = self._legal(e)
        return e

    def _store(self, i, e):
        W = self.t.words
        for k in range(W):
            self.vis[k, i] = (e["vis"] >> (64 * k)) & (2**64 - 1)
        if self.tb:
            for k in range(2 * W):
                self.dirs[k, i] = (e["dirs"] >> (64 * k)) & (2**64 - 1)
        self.pos[i] = e["x"] | (e["y"] << 8) | (e["len"] << 16) | (e["off"] << 24)
        self.aux[i] = e["node"] | (e["outcome"] << 16) | (e["pending"] << 18) | (e["node_term"] << 19)
        self.step_[i] = e["step"]
        self.pid[i] = e["pid"]

    # ---------------------------------------------------------------- kernels
    def reset(self, pids):
        for i, q in enumerate(pids):
            e = {}
            self._reset(e, int(q))
            self._store(i, e)

    def rollout(self, actions):
        T = actions.shape[0]
        rew = np.zeros((T, self.n), np.int8)
        flags = np.zeros((T, self.n), np.uint8)
        for i in range(self.n):
            e = self._load(i)
            for t in range(T):
                c, f = self._advance(e, int(actions[t, i]))
                rew[t, i], flags[t, i] = c, f
            self._store(i, e)
        return rew, flags
