// sparc_env.hpp — per-lane SPaRC env state machine for gfx950 (device code).
//
// One lane = one env.  The whole per-env state fits in VGPRs:
//   vis[W]      visited bitboard (bit x*pitch+y)          obs['base']['visited']
//   dirs[2W]    2-bit direction stack of the path moves    self.path (SPaRC_Gym.py:173, 1166, 1188)
//   x, y        agent location                             self._agent_location
//   len         len(self.path)
//   node, off   solution-trie node + off-trie depth        prefix/equality vs solution_paths
//   rec         trie record of `node` (children, parent, terminal)
//   step, outcome, pending, pid
// plus the puzzle's static row (open bitboard, sizes, start/target, trie base).
//
// Reference semantics restated (SPaRC_Gym.py):
//   legal mask  = _get_legal_actions 1024-1051: in bounds, gaps==0, and unvisited or (traceback,
//                 len>=2, n == path[-2]); path[-2] == pos - dir(last move), so the only legal
//                 revisit is the reverse of the last move.
//   advance()   = step 1131-1223: move or traceback-pop, terminated, truncated (max_steps or no
//                 legal move, cleared when terminated), reward code (x100).
//   prefix test = _is_on_solution_path 1244-1265 and np.array_equal 1206 via the trie: the path
//                 is a prefix of some solution iff off == 0; it equals one iff additionally the
//                 trie node is terminal.  O(1) per step instead of O(S*L).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace sparc {

constexpr uint32_t kNone = 0xFFFFu;

struct Table {
    const uint64_t* __restrict__ open;  // [P][W]
    const uint4* __restrict__ info;     // [P]
    const uint4* __restrict__ trie;     // [nodes]
    uint32_t num_puzzles;
};

struct State {                 // SoA, N = num_envs
    uint64_t* __restrict__ vis;   // [W][N]
    uint64_t* __restrict__ dirs;  // [2W][N] (traceback only)
    uint32_t* __restrict__ pos;   // x | y<<8 | len<<16 | off<<24
    uint32_t* __restrict__ aux;   // node | outcome<<16 (0: 0, 1: +1, 2: -1) | pending<<18
    uint32_t* __restrict__ step;
    uint32_t* __restrict__ pid;
};

struct Params {
    Table tab;
    State st;
    uint32_t n;
    uint32_t pitch;
    int32_t max_steps;
    int32_t autoreset;
    uint64_t env_offset;
    int32_t* __restrict__ err;
};

__device__ __forceinline__ int dir_dx(uint32_t d) { return d == 0 ? 1 : (d == 2 ? -1 : 0); }
__device__ __forceinline__ int dir_dy(uint32_t d) { return d == 1 ? -1 : (d == 3 ? 1 : 0); }

// ---- W-word bitboards held in registers.  Words are combined with masks, never selected
// between (a select of two array elements is folded into a dynamically indexed load, which
// demotes the whole Env to scratch memory).
template <int W>
__device__ __forceinline__ uint64_t bb_word(const uint64_t (&v)[W], uint32_t wi) {
    uint64_t r = 0;
#pragma unroll
    for (int k = 0; k < W; ++k) r |= v[k] & (wi == (uint32_t)k ? ~0ull : 0ull);
    return r;
}
template <int W>
__device__ __forceinline__ bool bb_test(const uint64_t (&v)[W], uint32_t b) {
    return (bb_word<W>(v, b >> 6) >> (b & 63)) & 1ull;
}
template <int W>
__device__ __forceinline__ void bb_set(uint64_t (&v)[W], uint32_t b) {
    const uint64_t m = 1ull << (b & 63);
#pragma unroll
    for (int k = 0; k < W; ++k) v[k] |= ((b >> 6) == (uint32_t)k) ? m : 0ull;
}
template <int W>
__device__ __forceinline__ void bb_clear(uint64_t (&v)[W], uint32_t b) {
    const uint64_t m = 1ull << (b & 63);
#pragma unroll
    for (int k = 0; k < W; ++k) v[k] &= ((b >> 6) == (uint32_t)k) ? ~m : ~0ull;
}

__device__ __forceinline__ uint32_t uint_rand_action(uint64_t seed, uint64_t env, uint64_t t) {
    uint64_t z = seed + env * 0x9E3779B97F4A7C15ull + t * 0xD1B54A32D192ED03ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    return (uint32_t)(z >> 62);
}

template <int W, bool TB>
struct Env {
    static constexpr int D = TB ? 2 * W : 1;   // direction-stack words (32 moves per word)
    uint64_t vis[W];
    uint64_t dirs[D];
    uint64_t open[W];
    uint32_t x, y, len, off, node, outcome, pending, step, pid;
    uint32_t X, Y, tx, ty, pflags, trie_base, trie_cnt;
    uint4 rec;   // invariant: the trie record of `node` whenever the puzzle's root is valid

    __device__ __forceinline__ void load_puzzle(const Params& p, uint32_t q, uint32_t& sx, uint32_t& sy) {
        const uint4 inf = p.tab.info[q];
        X = inf.x & 0xFFu;
        Y = (inf.x >> 8) & 0xFFu;
        sx = (inf.x >> 16) & 0xFFu;
        sy = inf.x >> 24;
        tx = inf.y & 0xFFu;
        ty = (inf.y >> 8) & 0xFFu;
        pflags = inf.y >> 16;
        trie_base = inf.z;
        trie_cnt = inf.w;
#pragma unroll
        for (int k = 0; k < W; ++k) open[k] = p.tab.open[(size_t)q * W + k];
    }

    // node < trie_cnt always holds (host-validated tables); the guard turns a broken invariant
    // into a reported error (sparc_sync) instead of an out-of-bounds read
    __device__ __forceinline__ void load_rec(const Params& p) {
        if (node >= trie_cnt) {
            atomicOr(p.err, 2);
            node = 0;
        }
        rec = p.tab.trie[trie_base + node];
    }

    // _load_puzzle (SPaRC_Gym.py:166-187) with fresh planes
    __device__ __forceinline__ void reset(const Params& p, uint32_t q) {
        uint32_t sx, sy;
        pid = q;
        load_puzzle(p, q, sx, sy);
        x = sx;
        y = sy;
        len = 1;
        node = 0;
        off = (pflags & 2u) ? 0u : 1u;  // [start] is a prefix iff some solution begins at start
        outcome = 0;
        pending = 0;
        step = 0;
#pragma unroll
        for (int k = 0; k < W; ++k) vis[k] = 0;
#pragma unroll
        for (int k = 0; k < D; ++k) dirs[k] = 0;
        bb_set<W>(vis, x * p.pitch + y);
        if (off == 0) load_rec(p);
        else rec = make_uint4(0xFFFFFFFFu, 0xFFFFFFFFu, kNone, 0u);
    }

    __device__ __forceinline__ uint32_t dir_at(uint32_t k) const {
        if constexpr (TB) {
            uint64_t w = 0;
#pragma unroll
            for (int j = 0; j < D; ++j) w |= dirs[j] & ((k >> 5) == (uint32_t)j ? ~0ull : 0ull);
            return (uint32_t)(w >> ((k & 31) * 2)) & 3u;
        } else {
            return 0;
        }
    }
    __device__ __forceinline__ void push_dir(uint32_t k, uint32_t d) {
        if constexpr (TB) {
            const uint32_t sh = (k & 31) * 2;
            const uint64_t clr = ~(3ull << sh), val = (uint64_t)d << sh;
#pragma unroll
            for (int j = 0; j < D; ++j) {
                const uint64_t sel = (k >> 5) == (uint32_t)j ? ~0ull : 0ull;
                dirs[j] = (dirs[j] & (clr | ~sel)) | (val & sel);
            }
        }
    }

    // _get_legal_actions (SPaRC_Gym.py:1024-1051) as a 4-bit mask in action order
    __device__ __forceinline__ uint32_t legal_mask(uint32_t pitch) const {
        uint32_t back = 8;  // direction of path[-2] from the agent, if traceback may use it
        if constexpr (TB) {
            if (len >= 2) back = dir_at(len - 2) ^ 2u;
        }
        uint32_t m = 0;
#pragma unroll
        for (uint32_t d = 0; d < 4; ++d) {
            const uint32_t nx = x + dir_dx(d), ny = y + dir_dy(d);   // wraps to huge when < 0
            const bool inb = nx < X && ny < Y;
            const uint32_t b = inb ? nx * pitch + ny : 0u;
            const bool ok = inb && bb_test<W>(open, b) && (!bb_test<W>(vis, b) || d == back);
            m |= (uint32_t)ok << d;
        }
        return m;
    }

    // one step() (SPaRC_Gym.py:1131-1223); returns reward code, writes flags
    __device__ __forceinline__ int advance(const Params& p, uint32_t a, uint32_t& flags) {
        if (p.autoreset == 1 && pending) {   // gymnasium next-step autoreset: reset(), 1087
            const uint32_t q = pid + 1 == p.tab.num_puzzles ? 0u : pid + 1;
            reset(p, q);
            flags = (legal_mask(p.pitch) << 2) | 64u;
            return 0;
        }
        const uint32_t legal = legal_mask(p.pitch);
        step = step < 0x7FFFFFFFu ? step + 1 : step;                     // 1132
        bool trunc = (int32_t)step >= p.max_steps;                       // 1134
        const bool moved = a < 4 && ((legal >> a) & 1u);                 // 1137
        if (moved) {
            const uint32_t nx = x + dir_dx(a), ny = y + dir_dy(a);
            const uint32_t b = nx * p.pitch + ny;
            if (TB && bb_test<W>(vis, b)) {                              // traceback pop 1141-1166
                bb_clear<W>(vis, x * p.pitch + y);
                len -= 1;
                if (off > 0) {
                    off -= 1;
                } else {
                    node = rec.z & 0xFFFFu;
                    load_rec(p);
                }
            } else {                                                     // forward 1167-1188
                bb_set<W>(vis, b);
                push_dir(len - 1, a);
                len += 1;
                if (off > 0) {
                    off += 1;
                } else {
                    const uint32_t cw = (a < 2) ? rec.x : rec.y;
                    const uint32_t c = (a & 1) ? (cw >> 16) : (cw & 0xFFFFu);
                    if (c != kNone) {
                        node = c;
                        load_rec(p);
                    } else {
                        off = 1;
                    }
                }
            }
            x = nx;
            y = ny;
        }
        const bool term = (x == tx) && (y == ty);                        // 1192
        const uint32_t legal2 = legal_mask(p.pitch);
        if (legal2 == 0) trunc = true;                                   // 1195-1196
        if (term) trunc = false;                                         // 1198-1199
        int code;
        if (term || trunc) {                                             // 1204-1213
            const bool match = off == 0 && ((rec.z >> 16) & 1u);
            if (match) {
                outcome = 1;
                code = 100;
            } else if (outcome != 1) {
                outcome = 2;
                code = -100;
            } else {
                code = 0;   // outcome_reward still 1 from the previous done step (1211)
            }
        } else {                                                         // 1214-1223
            outcome = 0;
            code = (!moved || !(pflags & 1u)) ? 0 : (off == 0 ? 1 : -1);
        }
        pending = (term || trunc) ? 1u : 0u;
        flags = (uint32_t)term | ((uint32_t)trunc << 1) | (legal2 << 2);
        return code;
    }

    // ---- SoA <-> registers
    __device__ __forceinline__ void load(const Params& p, uint32_t i) {
        const State& s = p.st;
#pragma unroll
        for (int k = 0; k < W; ++k) vis[k] = s.vis[(size_t)k * p.n + i];
        if constexpr (TB) {
#pragma unroll
            for (int k = 0; k < D; ++k) dirs[k] = s.dirs[(size_t)k * p.n + i];
        } else {
            dirs[0] = 0;
        }
        const uint32_t ps = s.pos[i], ax = s.aux[i];
        x = ps & 0xFFu;
        y = (ps >> 8) & 0xFFu;
        len = (ps >> 16) & 0xFFu;
        off = ps >> 24;
        node = ax & 0xFFFFu;
        outcome = (ax >> 16) & 3u;
        pending = (ax >> 18) & 1u;
        step = s.step[i];
        pid = s.pid[i];
        uint32_t sx, sy;
        load_puzzle(p, pid, sx, sy);
        // keep the invariant: pops can bring `off` back to 0 at any later step of a launch.
        // Puzzles whose root is not a prefix (flags bit1 clear) have off >= 1 forever and may
        // have no trie nodes at all.
        if (pflags & 2u) load_rec(p);
        else rec = make_uint4(0xFFFFFFFFu, 0xFFFFFFFFu, kNone, 0u);
    }

    __device__ __forceinline__ void store(const Params& p, uint32_t i) const {
        const State& s = p.st;
#pragma unroll
        for (int k = 0; k < W; ++k) s.vis[(size_t)k * p.n + i] = vis[k];
        if constexpr (TB) {
#pragma unroll
            for (int k = 0; k < D; ++k) s.dirs[(size_t)k * p.n + i] = dirs[k];
        }
        s.pos[i] = x | (y << 8) | (len << 16) | (off << 24);
        s.aux[i] = node | (outcome << 16) | (pending << 18);
        s.step[i] = step;
        s.pid[i] = pid;
    }
};

}  // namespace sparc
