// sparc_env.hpp — per-lane SPaRC env state machine for gfx950 (device code).
//
// One lane = one env.  The whole per-env state fits in VGPRs:
//   vis[W]      visited bitboard (bit x*pitch+y)          obs['base']['visited']
//   dirs[2W]    2-bit direction stack of the path moves    self.path (SPaRC_Gym.py:173, 1166, 1188)
//   x, y        agent location                             self._agent_location
//   len         len(self.path)
//   node, off   solution-trie node + off-trie depth        prefix/equality vs solution_paths
//   node_term   node is a complete solution (valid when off == 0)
//   rec         trie record of `node`; only read at the NEXT on-trie transition, so the load
//               issued at a transition overlaps the rest of that step
//   legal       legal-action mask of the current state (carried from the previous step)
//   last        direction of the last move (traceback: the only legal revisit is its reverse)
//   step, outcome, pending, pid
// plus the puzzle's static row (open bitboard, sizes, start/target, trie base) read from a
// PuzzleSrc: the global table (k_step) or an LDS copy of it (k_rollout).
//
// Reference semantics restated (SPaRC_Gym.py):
//   legal_mask  = _get_legal_actions 1024-1051: in bounds, gaps==0, and unvisited or (traceback,
//                 len>=2, n == path[-2]); path[-2] == pos - dir(last move).
//   advance()   = step 1131-1223: move or traceback-pop, terminated, truncated (max_steps or no
//                 legal move, cleared when terminated), reward code (x100).
//   prefix test = _is_on_solution_path 1244-1265 and np.array_equal 1206 via the trie: the path
//                 is a prefix of some solution iff off == 0; it equals one iff additionally the
//                 node is terminal.  O(1) per step instead of O(S*L).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace sparc {

constexpr uint32_t kNone = 0xFFFFu;
constexpr uint32_t kErrPuzzle = 1, kErrTrie = 2;

// trie record w2 fields
__device__ __forceinline__ uint32_t rec_parent(const uint4& r) { return r.z & 0xFFFFu; }
__device__ __forceinline__ uint32_t rec_term(const uint4& r) { return (r.z >> 16) & 1u; }
__device__ __forceinline__ uint32_t rec_child_term(const uint4& r, uint32_t d) { return (r.z >> (17 + d)) & 1u; }
__device__ __forceinline__ uint32_t rec_parent_term(const uint4& r) { return (r.z >> 21) & 1u; }
__device__ __forceinline__ uint32_t rec_child(const uint4& r, uint32_t d) {
    const uint32_t w = d < 2 ? r.x : r.y;
    return (d & 1) ? (w >> 16) : (w & 0xFFFFu);
}

struct Table {
    const uint64_t* __restrict__ open;  // [P][W]
    const uint4* __restrict__ info;     // [P]
    const uint4* __restrict__ root;     // [P] trie record of each puzzle's root (sentinel if none)
    const uint4* __restrict__ trie;     // [nodes]
    const uint64_t* __restrict__ init;  // [P] padded W = 1 layout: blocked board at reset
    const uint4* __restrict__ row1;     // [P] padded W = 1 layout: compact puzzle row
    const uint2* __restrict__ trie8;    // [nodes] split-kernel trie records (sparc_trie.hpp)
    const uint2* __restrict__ trieg;    // [nodes][4] record of each node's field-d node (TrieLane::step1la)
    const uint4* __restrict__ trow;     // [P] split-kernel trie rows (sparc_trie.hpp)
    const uint4* __restrict__ mrow;     // [P] W = 1 split move wave: {row1.x, reset board lo, hi, 0}
    uint32_t num_puzzles;
};

struct State {                 // SoA, N = num_envs
    uint64_t* __restrict__ vis;   // [W][N]
    uint64_t* __restrict__ dirs;  // [2W][N] (traceback only)
    uint32_t* __restrict__ pos;   // x | y<<8 | len<<16 | off<<24
    uint32_t* __restrict__ aux;   // node | outcome<<16 (0: 0, 1: +1, 2: -1) | pending<<18 | node_term<<19
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
    uint32_t nbr_pos;   // W = 1: window bit of each direction's neighbour, one byte per direction
    uint32_t nbm;       // W = 1 split move wave: mask of the four neighbour bits of the window
    uint32_t lmagic;    // W = 1 split move wave: legal-bit gather constant (sparc_move1.hpp)
};

// Static puzzle rows, from global memory or from an LDS copy (same layout).  info.w holds the
// trie node count (low 16 bits) and the legal mask of the freshly reset puzzle (bits 16-19);
// init[q] is the blocked board at reset (~open | start) of the padded W = 1 layout.
template <int W>
struct PuzzleSrc {
    const uint4* info;
    const uint4* root;
    const uint64_t* open;
    const uint64_t* init;
    const uint4* row1;     // W = 1: {start_bit | target_bit<<8 | flags<<16, trie_base,
                           //         trie_max | legal0<<16, 0}; init: free board at reset
    __device__ __forceinline__ uint4 get_row1(uint32_t q) const { return row1[q]; }
    __device__ __forceinline__ uint4 get_info(uint32_t q) const { return info[q]; }
    __device__ __forceinline__ uint4 get_root(uint32_t q) const { return root[q]; }
    __device__ __forceinline__ uint64_t get_open(uint32_t q, int k) const { return open[(size_t)q * W + k]; }
    __device__ __forceinline__ uint64_t get_init(uint32_t q) const { return init[q]; }
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

// element of a global table at a 32-bit byte offset: the load takes the table base in SGPRs and
// the offset in one VGPR (global_load v, vOff, s[base:base+1]) instead of a 64-bit VGPR address
// (tables are < 4 GiB: sparc_load_puzzles)
template <class T>
__device__ __forceinline__ T ld_off(const T* __restrict__ base, uint32_t byte_off) {
    return *reinterpret_cast<const T*>(reinterpret_cast<const char*>(base) + byte_off);
}

__device__ __forceinline__ uint32_t uint_rand_action(uint64_t seed, uint64_t env, uint64_t t) {
    uint64_t z = seed + env * 0x9E3779B97F4A7C15ull + t * 0xD1B54A32D192ED03ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    return (uint32_t)(z >> 62);
}

struct RegStack;

template <int W, bool TB, class Stack = RegStack>
struct Env {
    static constexpr int D = TB ? 2 * W : 1;   // direction-stack words (32 moves per word)
    uint64_t vis[W];
    uint64_t dirs[D];
    uint64_t open[W];
    uint32_t x, y, len, off, node, node_term, outcome, pending, step, pid, legal, last;
    uint32_t X, Y, tx, ty, pflags, trie_base, trie_cnt;
    uint4 rec;

    template <class Src>
    __device__ __forceinline__ void load_puzzle(const Src& src, uint32_t q, uint32_t& sx, uint32_t& sy) {
        const uint4 inf = src.get_info(q);
        X = inf.x & 0xFFu;
        Y = (inf.x >> 8) & 0xFFu;
        sx = (inf.x >> 16) & 0xFFu;
        sy = inf.x >> 24;
        tx = inf.y & 0xFFu;
        ty = (inf.y >> 8) & 0xFFu;
        pflags = inf.y >> 16;
        trie_base = inf.z;
        trie_cnt = inf.w & 0xFFFFu;
#pragma unroll
        for (int k = 0; k < W; ++k) open[k] = src.get_open(q, k);
    }

    // node < trie_cnt always holds (host-validated tables); the guard turns a broken invariant
    // into a reported error (sparc_sync) instead of an out-of-bounds read
    __device__ __forceinline__ void load_rec(const Params& p) {
        if (node >= trie_cnt) {
            atomicOr(p.err, (int)kErrTrie);
            node = 0;
        }
        rec = p.tab.trie[trie_base + node];
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
        const uint32_t back = (TB && len >= 2) ? (last ^ 2u) : 8u;  // direction of path[-2]
        const uint32_t b = x * pitch + y;
        uint32_t m = 0;
#pragma unroll
        for (uint32_t d = 0; d < 4; ++d) {
            const bool inb = d == 0 ? x + 1 < X : d == 1 ? y > 0 : d == 2 ? x > 0 : y + 1 < Y;
            const uint32_t nb = d == 0 ? b + pitch : d == 1 ? b - 1 : d == 2 ? b - pitch : b + 1;
            const uint32_t bb = inb ? nb : 0u;
            const bool ok = inb && bb_test<W>(open, bb) && (!bb_test<W>(vis, bb) || d == back);
            m |= (uint32_t)ok << d;
        }
        return m;
    }

    // _load_puzzle (SPaRC_Gym.py:166-187) with fresh planes; no global load on this path
    template <class Src>
    __device__ __forceinline__ void reset(const Params& p, const Src& src, uint32_t q) {
        reset(src, p.pitch, q);
    }
    template <class Src>
    __device__ __forceinline__ void reset(const Src& src, uint32_t pitch, uint32_t q) {
        uint32_t sx, sy;
        pid = q;
        load_puzzle(src, q, sx, sy);
        x = sx;
        y = sy;
        len = 1;
        node = 0;
        off = (pflags & 2u) ? 0u : 1u;  // [start] is a prefix iff some solution begins at start
        rec = src.get_root(q);          // sentinel (terminal bits 0) when there is no root
        node_term = rec_term(rec);
        outcome = 0;
        pending = 0;
        step = 0;
        last = 0;
#pragma unroll
        for (int k = 0; k < W; ++k) vis[k] = 0;
#pragma unroll
        for (int k = 0; k < D; ++k) dirs[k] = 0;
        bb_set<W>(vis, x * pitch + y);
        legal = legal_mask(pitch);
    }

    // one step() (SPaRC_Gym.py:1131-1223); returns reward code, writes flags
    template <class Src>
    __device__ __forceinline__ int advance(const Params& p, const Src& src, uint32_t a, uint32_t& flags) {
        if (p.autoreset == 1 && pending) {   // gymnasium next-step autoreset: reset(), 1087
            const uint32_t q = pid + 1 == p.tab.num_puzzles ? 0u : pid + 1;
            reset(src, p.pitch, q);
            flags = (legal << 2) | 64u;
            return 0;
        }
        step = step < 0x7FFFFFFFu ? step + 1 : step;                     // 1132
        bool trunc = (int32_t)step >= p.max_steps;                       // 1134
        const bool moved = a < 4 && ((legal >> a) & 1u);                 // 1137
        if (moved) {
            const uint32_t nx = x + dir_dx(a), ny = y + dir_dy(a);
            const uint32_t b = nx * p.pitch + ny;
            if (TB && bb_test<W>(vis, b)) {                              // traceback pop 1141-1166
                bb_clear<W>(vis, x * p.pitch + y);
                len -= 1;
                last = dir_at(len >= 2 ? len - 2 : 0);
                if (off > 0) {
                    off -= 1;
                } else {
                    node_term = rec_parent_term(rec);
                    node = rec_parent(rec);
                    load_rec(p);
                }
            } else {                                                     // forward 1167-1188
                bb_set<W>(vis, b);
                push_dir(len - 1, a);
                last = a;
                len += 1;
                if (off > 0) {
                    off += 1;
                } else {
                    const uint32_t c = rec_child(rec, a);
                    if (c != kNone) {
                        node_term = rec_child_term(rec, a);
                        node = c;
                        load_rec(p);
                    } else {
                        off = 1;
                    }
                }
            }
            x = nx;
            y = ny;
            legal = legal_mask(p.pitch);
        }
        const bool term = (x == tx) && (y == ty);                        // 1192
        if (legal == 0) trunc = true;                                    // 1195-1196
        if (term) trunc = false;                                         // 1198-1199
        int code;
        if (term || trunc) {                                             // 1204-1213
            if (off == 0 && node_term) {
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
        flags = (uint32_t)term | ((uint32_t)trunc << 1) | (legal << 2);
        return code;
    }

    // obs['base']['visited'] bits and the agent's bit index (SPaRC_Gym.py:956-979)
    template <class Src>
    __device__ __forceinline__ void obs_words(const Params& p, const Src&, uint64_t (&v)[W], uint32_t& ab) const {
#pragma unroll
        for (int k = 0; k < W; ++k) v[k] = vis[k];
        ab = x * p.pitch + y;
    }
    __device__ __forceinline__ uint32_t agent_xy(const Params&) const { return x | (y << 8); }

    // ---- SoA <-> registers
    template <class Src>
    __device__ __forceinline__ void load(const Params& p, const Src& src, uint32_t i) {
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
        node_term = (ax >> 19) & 1u;
        step = s.step[i];
        pid = s.pid[i];
        uint32_t sx, sy;
        load_puzzle(src, pid, sx, sy);
        // invariant: rec is node's record whenever the root is valid (pops can bring `off`
        // back to 0 at any later step).  Rootless puzzles (flags bit1 clear) keep off >= 1.
        if (pflags & 2u) load_rec(p);
        else rec = make_uint4(0xFFFFFFFFu, 0xFFFFFFFFu, kNone, 0u);
        last = (TB && len >= 2) ? dir_at(len - 2) : 0u;
        legal = legal_mask(p.pitch);
    }

    template <class Src>
    __device__ __forceinline__ void store(const Params& p, const Src&, uint32_t i) const {
        const State& s = p.st;
#pragma unroll
        for (int k = 0; k < W; ++k) s.vis[(size_t)k * p.n + i] = vis[k];
        if constexpr (TB) {
#pragma unroll
            for (int k = 0; k < D; ++k) s.dirs[(size_t)k * p.n + i] = dirs[k];
        }
        s.pos[i] = x | (y << 8) | (len << 16) | (off << 24);
        s.aux[i] = node | (outcome << 16) | (pending << 18) | (node_term << 19);
        s.step[i] = step;
        s.pid[i] = pid;
    }
};

// ---------------------------------------------------------------------------------------------
// Direction stacks of the W = 1 path (2 bits of information per move, <= 63 moves on a 64-bit
// board).  Registers / LDS hold the REVERSED moves (move k ^ 2 = the direction from path[k+1]
// back to path[k]), which is what the traceback rule and the pop need; in HBM both are stored
// as the moves themselves, two u64 words [2][N] (move k at bits 2(k%32) of word k/32), only
// the path's len-1 moves set.  Writes are unconditional: a step writes slot len-1, which is
// the new top after a forward move and lies above the top otherwise.
constexpr uint64_t kRev2 = 0xAAAAAAAAAAAAAAAAull;   // XOR: move <-> reversed move, every field
__device__ __forceinline__ uint64_t low_moves(uint32_t moves, uint32_t word) {
    // mask of the fields of `moves` moves that live in word `word` (0: moves 0-31)
    const uint32_t m = word ? (moves > 32u ? moves - 32u : 0u) : (moves < 32u ? moves : 32u);
    return m >= 32u ? ~0ull : ((1ull << (2u * m)) - 1ull);
}

struct RegStack {            // k_step / k_reset: two u64 registers
    uint64_t lo = 0, hi = 0;
    __device__ __forceinline__ void clear() { lo = hi = 0; }
    __device__ __forceinline__ uint32_t read(uint32_t k) const {
        return (uint32_t)((k < 32 ? lo : hi) >> ((k & 31u) * 2u)) & 3u;
    }
    __device__ __forceinline__ void write(uint32_t k, uint32_t d) {
        const uint32_t sh = (k & 31u) * 2u;
        const bool hiw = k >= 32;
        const uint64_t w = hiw ? hi : lo;
        const uint64_t upd = (w & ~(3ull << sh)) | ((uint64_t)(d & 3u) << sh);
        lo = hiw ? lo : upd;
        hi = hiw ? upd : hi;
    }
    __device__ __forceinline__ void load(const uint64_t* d, size_t n, uint32_t i, uint32_t) {
        lo = d[i] ^ kRev2;
        hi = d[n + i] ^ kRev2;
    }
    __device__ __forceinline__ void store(uint64_t* d, size_t n, uint32_t i, uint32_t moves) const {
        d[i] = (lo ^ kRev2) & low_moves(moves, 0);
        d[n + i] = (hi ^ kRev2) & low_moves(moves, 1);
    }
};

template <uint32_t S>         // k_rollout: one byte per move in this lane's column of a per-wave
struct LdsStack {            // [64 moves][S lanes] LDS array
    uint8_t* col;
    __device__ __forceinline__ void clear() {}
    __device__ __forceinline__ uint32_t read(uint32_t k) const { return col[k * S]; }
    __device__ __forceinline__ void write(uint32_t k, uint32_t d) { col[k * S] = (uint8_t)d; }
    __device__ __forceinline__ void load(const uint64_t* d, size_t n, uint32_t i, uint32_t moves) {
        const uint64_t lo = d[i] ^ kRev2, hi = d[n + i] ^ kRev2;
        for (uint32_t k = 0; k < moves; ++k)
            col[k * S] = (uint8_t)(((k < 32 ? lo : hi) >> ((k & 31u) * 2u)) & 3u);
    }
    __device__ __forceinline__ void store(uint64_t* d, size_t n, uint32_t i, uint32_t moves) const {
        uint64_t lo = 0, hi = 0;
        for (uint32_t k = 0; k < moves; ++k) {
            const uint64_t v = (uint64_t)((col[k * S] ^ 2u) & 3u) << ((k & 31u) * 2u);
            lo |= k < 32 ? v : 0ull;
            hi |= k < 32 ? 0ull : v;
        }
        d[i] = lo;
        d[n + i] = hi;
    }
};

// ---------------------------------------------------------------------------------------------
// W = 1 specialisation: lattices that fit a 64-bit board PADDED by one column (pitch > y_size)
// and one row, (x_size + 1) * pitch <= 64 (every 7x7 and 5x5 pool; the host packer picks this
// geometry).  The agent is the bit index e = x*pitch + y.  The only bitboard in registers is
// the FREE board `fr` (in the lattice, not a gap, unvisited) stored one row up: bit e + pitch
// is point e.  So the four neighbour tests of _get_legal_actions are one 64-bit shift,
//     w = (uint32_t)(fr >> e):  bit 0 left (x-1), pitch-1 up (y-1), pitch+1 down (y+1),
//                               2*pitch right (x+1)
// and every out-of-lattice neighbour reads 0: below row 0 is the empty bottom row, beyond
// y_size-1 the empty padding column, beyond the last row either the empty top row or bits
// shifted out of the word.  No bounds compares, no rotate.  The step is branch-free except
// for the autoreset and is ordered so that the trie record gathered at the end of one step is
// first read in the next step's trie phase.
template <bool TB, class Stack>
struct Env<1, TB, Stack> {
    uint64_t fr;         // free board, one row up (bit e + pitch = point e)
    Stack stk;           // reversed moves of self.path (traceback only)
    uint32_t e, len, off, outcome, pending, pid, legal, rl;
    uint32_t nn;         // trie node | node_term << 15 (a "packed node", as in the W = 1 records)
    int32_t step;
    uint32_t tgt, pflags, trie_base, trie_max;
    uint32_t bk;         // traceback rule bias: (len + bk) >> 31 = len >= 3 or (len == 2, open start)
    uint32_t w = 0;      // window of fr at e (see above), valid between steps
    uint32_t pnr = 0;    // traceback: reversed move before the last one, read one step ahead
    uint32_t solved = 0, was_reset = 0;   // this step: a +1 outcome / an autoreset (for stats)
    uint32_t rs = 0;     // the coming step is an autoreset step (its state already loaded)
    // phase_move -> phase_trie hand-over: action, forward / pop, moved on a puzzle with
    // solutions, done, reset step
    uint32_t s_a = 0, s_fwd = 0, s_pop = 0, s_mv = 0, s_done = 0, s_rs = 0;
    uint2 rec;

    // all arms are computed unconditionally and merged with masks: a C++ ?: whose arms are
    // 64-bit shifts is otherwise lowered to exec-masked if/else blocks
    __device__ __forceinline__ static uint32_t pick(bool c, uint32_t a, uint32_t b) {
        const uint32_t m = 0u - (uint32_t)c;
        return (a & m) | (b & ~m);
    }

    // _get_legal_actions (1024-1051): bit d = direction d is legal; sets the window w
    __device__ __forceinline__ uint32_t legal_mask(uint32_t P) {
        w = (uint32_t)(fr >> (e & 63u));
        // bits P-2..P+1 of w: (-, up, self, down); up and down land on their action bits 1, 3
        const uint32_t ud = __builtin_amdgcn_ubfe(w, P - 2u, 4u);
        uint32_t m = (ud & 10u) | (((w << 2) & 4u) | __builtin_amdgcn_ubfe(w, 2u * P, 1u));
        // traceback: path[-2] (the reverse of the last move) is visited but legal
        if constexpr (TB) m |= ((len + bk) >> 31) << rl;
        return m;
    }

    // row: {start | target<<8 | flags<<16, trie_base, trie_max | legal0<<16, 0}; flags bit0
    // solutions, bit1 root valid, bit2 start closed, bit3 root terminal
    template <class Src>
    __device__ __forceinline__ uint32_t load_puzzle(const Src& src, uint32_t q) {
        return apply_row(src.get_row1(q));
    }
    __device__ __forceinline__ uint32_t apply_row(const uint4 r) {
        tgt = (r.x >> 8) & 0xFFu;
        pflags = r.x >> 16;
        trie_base = r.y;
        trie_max = r.z & 0xFFFFu;
        bk = 0x7FFFFFFDu + ((~pflags >> 2) & 1u);
        return r.x & 0xFFu;   // start
    }

    // the current node's record, loaded unconditionally (L2-resident table): the split
    // kernels' 8-B records (trie8, sparc_trie.hpp): field d = the child in direction d as a packed
    // node (index | terminal << 15, 0xFFFF = none), and the PARENT in the field of the direction
    // back to it, which is exactly the direction a traceback pop moves, so a forward move and a
    // pop read the same field[action].  node <= trie_max holds on validated tables; the clamp
    // keeps a broken state from reading out of bounds.
    __device__ __forceinline__ void load_rec(const Params& p) {
        const uint32_t node = nn & 0x7FFFu;
        rec = p.tab.trie8[trie_base + (node < trie_max ? node : trie_max)];
    }

    // _load_puzzle (SPaRC_Gym.py:166-187) with fresh planes: the puzzle rows and the board,
    // not the trie state (inside a rollout the done step's phase_trie runs after this).  The
    // step that resets recomputes pending, outcome and legal itself, and rl is unused until
    // the first move.
    template <class Src>
    __device__ __forceinline__ void reset_rows(const Src& src, uint32_t q) {
        pid = q;
        e = load_puzzle(src, q);
        fr = src.get_init(q);
    }
    template <class Src>
    __device__ __forceinline__ void reset(const Params& p, const Src& src, uint32_t q) {
        reset_rows(src, q);
        off = ((pflags >> 1) & 1u) ^ 1u;
        len = 1;
        nn = ((pflags >> 3) & 1u) << 15;   // node 0 (the root); it is a solution iff [start] is one
        step = 0;
        rs = 0;
        outcome = 0;
        pending = 0;
        rl = 0;
        stk.clear();
        legal = legal_mask(p.pitch);
        load_rec(p);
    }

    // ---- the step in two phases.  phase_move (legality, move, path, flags) needs no trie
    // record; phase_trie (solution trie, reward) of step t needs the record gathered by
    // phase_trie of step t-1.  k_rollout runs phase_trie(t-1) next to phase_move(t): two
    // independent dependency chains per iteration, and a whole iteration for the gather.
    // A step is: reset_next (if the previous step ended an episode) -> phase_move -> phase_trie.

    // gymnasium next-step autoreset (reset(), SPaRC_Gym.py:1087): the step after a done step
    // loads the next puzzle (index + 1 mod P), ignores its action and returns reward 0, flag
    // 64.  Only the puzzle rows, the board and the counters are set here; the trie state (nn,
    // off) is set to the root by that step's phase_trie: in k_rollout1 the done step's
    // phase_trie runs after this call and still needs it.
    template <class Src>
    __device__ __forceinline__ void reset_next(const Params& p, const Src& src) {
        if (pending & (uint32_t)(p.autoreset == 1)) {
            reset_rows(src, pid + 1 == p.tab.num_puzzles ? 0u : pid + 1);
            len = 1;
            step = -1;   // this step's increment brings it to 0
            rs = 1;
        }
    }

    __device__ __forceinline__ uint32_t phase_move(const Params& p, uint32_t a) {
        const uint32_t P = p.pitch;
        step = __builtin_elementwise_add_sat(step, 1);                              // 1132
        const bool trunc0 = step >= p.max_steps;                                    // 1134
        // `action in legal` (1137): bit a of the legal mask; actions >= 4 read bit 4 (0); a
        // reset step does not move
        const uint32_t moved = (legal >> (a < 4u ? a : 4u)) & (rs ^ 1u) & 1u;
        // neighbour's bit in the window: right 2P, up P-1, left 0, down P+1 (bytes of one
        // constant; the bfe offset keeps 5 bits, so a<<3 selects byte a&3)
        const uint32_t pos = __builtin_amdgcn_ubfe(p.nbr_pos, a << 3, 8u);
        // the only legal move onto a non-free point is the traceback pop (1141-1166)
        const uint32_t pop = TB ? moved & ~__builtin_amdgcn_ubfe(w, pos, 1u) : 0u;
        const uint32_t fwd = moved ^ pop;                                            // 1167-1188
        const int32_t d = (int32_t)pos - (int32_t)P;  // the neighbour's offset from e
        // free board: a forward move takes the target (bit e + d + P), a pop frees the point
        // it leaves (bit e + P)
        const uint32_t tog = e + (fwd ? pos : P);
        fr ^= (uint64_t)moved << (tog & 63u);
        if constexpr (TB) {
            const uint32_t ar = a ^ 2u;
            stk.write(len - 1u, ar);                 // the new top if fwd, above the top otherwise
            rl = fwd ? ar : (pop ? pnr : rl);
        }
        len = len + fwd - pop;
        e = (uint32_t)((int32_t)e + __mul24((int32_t)moved, d));   // one v_mad_i32_i24
        legal = legal_mask(P);
        const uint32_t live = rs ^ 1u;                                               // 0 on a reset step
        const uint32_t term = e == tgt ? live : 0u;                                  // 1192
        const uint32_t trunc = (trunc0 | (legal == 0)) ? live ^ term : 0u;          // 1195-1199
        const uint32_t done = term | trunc;
        pending = done;
        if constexpr (TB) pnr = stk.read(__builtin_elementwise_sub_sat(len, 3u));   // next step's pop
        s_a = a;
        s_fwd = fwd;
        s_pop = pop;
        s_mv = moved & pflags & 1u;   // moved, and the puzzle has solutions (1205, 1217)
        s_done = done;
        s_rs = rs;
        const uint32_t f = (legal << 2) | (rs << 6) | term | (trunc << 1);
        rs = 0;
        return f;
    }

    __device__ __forceinline__ int phase_trie(const Params& p) {
        // a reset step starts the new puzzle's trie at its root
        nn = pick(s_rs != 0u, ((pflags >> 3) & 1u) << 15, nn);
        off = pick(s_rs != 0u, ((pflags >> 1) & 1u) ^ 1u, off);
        // solution trie (first read of the record loaded at the previous step): a forward move
        // on the trie goes to the child field[a] (or leaves the trie), a pop on the trie to the
        // parent, which is field[a] as well; off the trie they count the depth off it
        const bool on = off == 0;
        const uint32_t c = (uint32_t)((((uint64_t)rec.y << 32) | rec.x) >> ((s_a << 4) & 63u)) & 0xFFFFu;
        const bool has = c != 0xFFFFu;
        const bool down = (s_fwd != 0u) & on & has;
        const bool up = (s_pop != 0u) & on;
        nn = pick(down | up, c, nn);
        off = pick(on, s_fwd & (uint32_t)!has, off + s_fwd - s_pop);
        // the record changes only with the node (a random walk is off the trie on most steps)
        load_rec(p);
        // reward code (1204-1223): done: +100 on a solution, else -100 unless the previous
        // done step already set outcome_reward = 1 (then 0); otherwise +-1 when moved (0 if the
        // puzzle has no solutions); a reset step returns 0 (no move, not done)
        const bool match = (off == 0) & (nn >= 0x8000u);
        const bool done = s_done != 0u;
        const int c_done = match ? 100 : (outcome != 1 ? -100 : 0);
        const int c_move = s_mv ? (off == 0 ? 1 : -1) : 0;
        outcome = done ? ((match | (outcome == 1)) ? 1u : 2u) : 0u;
        solved = (uint32_t)(done & match);
        return done ? c_done : c_move;
    }

    // one whole step (k_step, and the generic-width interface)
    template <class Src>
    __device__ __forceinline__ int advance(const Params& p, const Src& src, uint32_t a, uint32_t& flags) {
        reset_next(p, src);
        flags = phase_move(p, a);
        was_reset = s_rs;
        return phase_trie(p);
    }

    // the code and solved flag that phase_trie would report again for the last step of the
    // previous launch (k_rollout runs one phase_trie before its first step, on the stored
    // state, which leaves the state unchanged; its outputs are subtracted from the stats)
    __device__ __forceinline__ void replay_outputs(int& code, uint32_t& sol) const {
        const bool match = (off == 0) & (nn >= 0x8000u);
        code = pending ? (match ? 100 : (outcome != 1 ? -100 : 0)) : 0;
        sol = (uint32_t)(pending & match);
    }

    // obs['base']['visited'] bits (visited = in the puzzle and not free, plus the start, as
    // store() writes them) and the agent's bit index
    template <class Src>
    __device__ __forceinline__ void obs_words(const Params& p, const Src& src, uint64_t (&v)[1], uint32_t& ab) const {
        v[0] = ((src.get_init(pid) & ~fr) >> p.pitch) | (1ull << (src.get_row1(pid).x & 0xFFu));
        ab = e;
    }
    __device__ __forceinline__ uint32_t agent_xy(const Params& p) const {
        const uint32_t x = e / p.pitch;
        return x | ((e - x * p.pitch) << 8);
    }

    template <class Src>
    __device__ __forceinline__ void load(const Params& p, const Src& src, uint32_t i) {
        const State& s = p.st;
        const uint32_t P = p.pitch;
        const uint64_t vis = s.vis[i];
        const uint32_t ps = s.pos[i], ax = s.aux[i];
        e = (ps & 0xFFu) * P + ((ps >> 8) & 0xFFu);
        len = (ps >> 16) & 0xFFu;
        off = ps >> 24;
        nn = (ax & 0x7FFFu) | (((ax >> 19) & 1u) << 15);
        outcome = (ax >> 16) & 3u;
        pending = (ax >> 18) & 1u;
        step = (int32_t)s.step[i];
        pid = s.pid[i];
        load_puzzle(src, pid);
        fr = (p.tab.open[pid] & ~vis) << P;
        load_rec(p);
        if constexpr (TB) {
            stk.load(s.dirs, p.n, i, len >= 1 ? len - 1 : 0u);
            rl = len >= 2 ? stk.read(len - 2) : 0u;
            pnr = stk.read(__builtin_elementwise_sub_sat(len, 3u));
        } else {
            rl = 0;
        }
        legal = legal_mask(P);
        // a hand-over that replays the stored step's trie phase: no move, same done flag
        rs = 0;
        s_a = s_fwd = s_pop = s_mv = s_rs = 0;
        s_done = pending;
    }

    template <class Src>
    __device__ __forceinline__ void store(const Params& p, const Src& src, uint32_t i) const {
        const State& s = p.st;
        const uint32_t P = p.pitch;
        const uint32_t sb = src.get_row1(pid).x & 0xFFu;
        // visited = in the puzzle and not free, plus the start (always on the path, even when
        // it is a gap)
        s.vis[i] = ((~fr) >> P & p.tab.open[pid]) | (1ull << sb);
        if constexpr (TB) stk.store(s.dirs, p.n, i, len >= 1 ? len - 1 : 0u);
        const uint32_t x = e / P, y = e - x * P;
        s.pos[i] = x | (y << 8) | (len << 16) | (off << 24);
        s.aux[i] = (nn & 0x7FFFu) | (outcome << 16) | (pending << 18) | ((nn >> 15) << 19);
        s.step[i] = (uint32_t)step;
        s.pid[i] = pid;
    }
};

}  // namespace sparc
