// sparc_split.hpp — the W = 1 env step cut into three wave roles (device code, k_rollout1r).
//
// At 65,536 envs an MI355X has exactly 64 envs per SIMD, and one wave alone issues an
// instruction only every ~4-5 cycles while its SIMD accepts one every 2.  So the step of each
// 64-env group runs on three waves of the same SIMD, cut where the data flow is one-way:
//
//   MOVE   (MoveLane)   reset_next + legality + move + path stack + terminated / truncated.
//                       Its loop-carried chain is the only serial part of step() that feeds
//                       itself (SPaRC_Gym.py:1131-1199).  Per env-step it writes one 16-bit
//                       hand-over word: the flag byte | pop << 8 | forward << 9 | action << 10.
//   TRIE   (TrieLane)   the solution-trie walk (_is_on_solution_path 1244-1265 and the
//                       np.array_equal test of 1206, as a trie), the reward code and the
//                       outcome_reward chain (1201-1223) and the episode counters, two tiles
//                       behind.  Per env-step it writes the reward code byte.
//   I/O                 streams the actions in (decoding them for the move wave) and the
//                       reward / flag tiles out, three tiles behind.
//
// Nothing flows back: the reward never feeds the trie, the trie never feeds the move.
//
// Move window.  The padded W = 1 board (Env<1> in sparc_env.hpp) keeps the FREE board `fr`
// one row up, bit e + P = point e, so w = (uint32)(fr >> e) holds the neighbours of the agent
// e at bits 0 (left), P-1 (up), P+1 (down), 2P (right) and the agent itself at bit P (always 0).
// With traceback, path[-2] is legal although visited: w2 = w | tb_ok << rlp, where rlp is
// path[-2]'s window bit.  So `action in legal` (1137) is one bit test of w2, and a pop is a
// legal move onto a point that is not free.  The move stack (LDS, one byte per move) holds, for
// each move, the window bit of the point it left behind (2P - pos); only its low 5 bits are
// meaningful (the stored byte also carries -64*action).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "sparc_env.hpp"

namespace sparc {

// Decoded actions (decode_actions4, on the I/O wave): one u32 per action,
//   pos | (d & 0xFF) << 8 | action << 26,   d = pos - P (signed byte)
// pos = the neighbour's window bit (action 0..3), or P for an action >= 4 (never legal); then
// (ac & 31) = pos for the bit tests, bfe_i32(ac, 8, 8) = the agent's move on the board and
// ac >> 16 = action << 10, its place in the hand-over word.
struct ActionLuts {
    uint32_t pos, d, a, prep;   // v_perm byte tables for actions 0..3; prep: bytes 4..7 (= P)
};
__device__ __forceinline__ ActionLuts action_luts(uint32_t nbr_pos, uint32_t P) {
    ActionLuts l;
    l.pos = nbr_pos;
    l.d = 0;
#pragma unroll
    for (int a = 0; a < 4; ++a) l.d |= (((nbr_pos >> (8 * a)) - P) & 0xFFu) << (8 * a);
    l.a = 0x0C080400u;   // action << 2: byte 3 of the decoded word
    l.prep = P * 0x01010101u;
    return l;
}
// four action bytes -> four decoded words (o[j] for byte j); bytes 4..255 decode to P
__device__ __forceinline__ void decode_actions4(uint32_t x, const ActionLuts& l, uint32_t (&o)[4]) {
    // bit 7 of each byte of `big`: that action byte is >= 8 ((b >> 3) * 4 + 124 carries into bit 7)
    const uint32_t big = (((x >> 1) & 0x7C7C7C7Cu) + 0x7C7C7C7Cu) & 0x80808080u;
    const uint32_t sel = (x & 0x07070707u) | (big >> 5);   // 0..3: table byte; 4..7: invalid
    const uint32_t pos = __builtin_amdgcn_perm(l.prep, l.pos, sel);   // invalid: P
    const uint32_t d = __builtin_amdgcn_perm(0u, l.d, sel);           // invalid: 0
    const uint32_t a = __builtin_amdgcn_perm(0u, l.a, sel);           // invalid: 0
#pragma unroll
    for (uint32_t j = 0; j < 4; ++j) {
        // {pos_j, d_j, 0, 0} then byte 3 = a_j
        const uint32_t pd = __builtin_amdgcn_perm(d, pos, 0x0C0C0400u + j * 0x0101u);
        o[j] = __builtin_amdgcn_perm(a, pd, 0x04020100u + j * 0x01000000u);
    }
}

// rows of the split kernel (sparc_load_puzzles, words == 1), per puzzle q:
//   mrow[2q]     = {start_bit, target_bit, bk, next(q)}   bk: see MoveLane::bk
//   mrow[2q + 1] = {reset free board lo, hi, 0, 0}
//   trow[q]      = {trie_base, trie_max | flags << 16, root children right | up << 16, left | down << 16}
// flags: bit0 solution_count > 0, bit1 some solution starts at start (root valid), bit2 the
// start is a gap, bit3 [start] itself is a solution.  Children are packed nodes
// (index | terminal << 15, 0xFFFF = none), as in the W = 1 trie records.

__device__ __forceinline__ uint32_t next_puzzle(uint32_t q, uint32_t num_puzzles) {
    return q + 1 == num_puzzles ? 0u : q + 1;   // reset() without options, SPaRC_Gym.py:1087
}

template <bool TB>
struct MoveLane {
    uint64_t fr;         // free board, one row up
    uint32_t w = 0;      // window of fr at e
    uint32_t w2 = 0;     // w | traceback-legal bit
    uint32_t e, tgt, len, npid, pend = 0, live = 1;
    uint32_t bk;         // (len + bk) >> 31 = len >= 3, or len == 2 with an open start (1041-1046)
    uint32_t rlp = 0;    // window bit of path[-2] (traceback)
    uint32_t pnr = 0;    // the stack entry below the top: the next pop's rlp (read one step ahead)
    int32_t step;
    uint4 nm;            // mrow[2 * npid] of the next puzzle, prefetched: a reset needs no LDS wait
    uint2 ni;            // its reset board
    uint8_t* stk = nullptr;   // this lane's column of the [64 moves][64 lanes] LDS stack

    __device__ __forceinline__ void window() {
        w = (uint32_t)(fr >> (e & 63u));
        const uint32_t ok = TB ? (len + bk) >> 31 : 0u;
        w2 = w | (ok << rlp);
    }
    // _get_legal_actions (1024-1051) in action order, from the window
    __device__ __forceinline__ uint32_t legal4(uint32_t P) const {
        const uint32_t ud = __builtin_amdgcn_ubfe(w2, P - 2u, 4u);   // up, down at bits 1, 3
        return (ud & 10u) | ((w2 << 2) & 4u) | __builtin_amdgcn_ubfe(w2, 2u * P, 1u);
    }
    __device__ __forceinline__ void prefetch(const uint4* mrow) {
        nm = mrow[2 * npid];
        const uint4 b = mrow[2 * npid + 1];
        ni = make_uint2(b.x, b.y);
    }

    __device__ __forceinline__ void load(const Params& p, const uint4* mrow, uint32_t i) {
        const State& s = p.st;
        const uint32_t P = p.pitch;
        const uint64_t vis = s.vis[i];
        const uint32_t ps = s.pos[i], ax = s.aux[i];
        e = (ps & 0xFFu) * P + ((ps >> 8) & 0xFFu);
        len = (ps >> 16) & 0xFFu;
        pend = (ax >> 18) & 1u;
        step = (int32_t)s.step[i];
        const uint32_t pid = s.pid[i];
        const uint4 r = mrow[2 * pid];
        tgt = r.y;
        bk = r.z;
        npid = r.w;
        fr = (p.tab.open[pid] & ~vis) << P;
        if constexpr (TB) {
            // HBM holds the moves themselves (move k at bits 2(k % 32) of word k / 32)
            const uint32_t moves = len >= 1 ? len - 1 : 0u;
            const uint64_t lo = s.dirs[i], hi = s.dirs[p.n + i];
            for (uint32_t k = 0; k < moves; ++k) {
                const uint32_t a = (uint32_t)(((k < 32 ? lo : hi) >> ((k & 31u) * 2u)) & 3u);
                stk[k * 64] = (uint8_t)__builtin_amdgcn_ubfe(p.nbr_pos, (a ^ 2u) << 3, 8u);
            }
            rlp = len >= 2 ? stk[(len - 2) * 64] : 0u;
            pnr = stk[__builtin_elementwise_sub_sat(len, 3u) * 64];
        }
        window();
        live = 1;
        prefetch(mrow);
    }

    // reset_next + phase_move of Env<1> (sparc_env.hpp) on the window; returns the hand-over word
    __device__ __forceinline__ uint32_t step_hw(const Params& p, const uint4* mrow, uint32_t ac) {
        const uint32_t P = p.pitch;
        // gymnasium next-step autoreset (reset(), 1087): the step after a done step loads the
        // next puzzle, does not move and returns reward 0 / flag 64.  Branch-free: the row was
        // prefetched, so a reset is a few selects.
        const bool r = (pend & (uint32_t)p.autoreset) != 0u;
        e = r ? nm.x : e;
        tgt = r ? nm.y : tgt;
        bk = r ? nm.z : bk;
        npid = r ? nm.w : npid;
        fr = r ? (((uint64_t)ni.y << 32) | ni.x) : fr;
        len = r ? 1u : len;
        step = r ? 0 : __builtin_elementwise_add_sat(step, 1);                    // 1132
        live = r ? 0u : 1u;
        prefetch(mrow);   // unchanged unless this lane reset
        const uint32_t b2 = __builtin_amdgcn_ubfe(w2, ac, 1u), bw = __builtin_amdgcn_ubfe(w, ac, 1u);
        const uint32_t moved = b2 & live;                                           // 1137
        const uint32_t pop = TB ? moved & ~bw : 0u;                                 // 1141-1166
        const uint32_t fwd = TB ? moved & bw : moved;                               // 1167-1188
        const int32_t d = __builtin_amdgcn_sbfe((int32_t)ac, 8u, 8u);
        // free board: a forward move takes its target (bit e + P + d), a pop frees e (bit e + P)
        fr ^= (uint64_t)moved << ((e + P + (uint32_t)__mul24((int32_t)fwd, d)) & 63u);
        if constexpr (TB) {
            const uint32_t rp = 2u * P - ac;      // low 5 bits: window bit of the point left behind
            stk[(len - 1u) * 64] = (uint8_t)rp;   // the new top if forward, above the top otherwise
            rlp = fwd ? rp : (pop ? pnr : rlp);
        }
        len = len + fwd - pop;
        e = (uint32_t)((int32_t)e + __mul24((int32_t)moved, d));
        window();
        const uint32_t legal = legal4(P);
        const uint32_t term = e == tgt ? live : 0u;                                 // 1192
        const uint32_t trunc = ((step >= p.max_steps) | (legal == 0u)) ? live ^ term : 0u;   // 1134, 1195-1199
        pend = term | trunc;
        if constexpr (TB) pnr = stk[(len - 3u) * 64];   // next step's pop (any value while len < 3)
        return term | (trunc << 1) | (legal << 2) | ((live ^ 1u) << 6) | (pop << 8) | (fwd << 9) | (ac >> 16);
    }

    // state -> HBM (Env<1>::store's layout); nn / off / pid from the trie wave, outcome from
    // the reward wave
    __device__ __forceinline__ void store(const Params& p, const uint4* mrow, uint32_t i, uint32_t pid, uint32_t nn,
                                          uint32_t off, uint32_t outcome) const {
        const State& s = p.st;
        const uint32_t P = p.pitch;
        const uint32_t sb = mrow[2 * pid].x;
        // visited = in the puzzle and not free, plus the start (on the path even when a gap)
        s.vis[i] = ((~fr) >> P & p.tab.open[pid]) | (1ull << sb);
        if constexpr (TB) {
            const uint32_t moves = len >= 1 ? len - 1 : 0u;
            uint64_t lo = 0, hi = 0;
            for (uint32_t k = 0; k < moves; ++k) {
                const uint32_t q = stk[k * 64] & 31u;   // window bit of path[k] seen from path[k+1]
                const uint32_t rev = q == 2u * P ? 0u : (q == P - 1u ? 1u : (q == 0u ? 2u : 3u));
                const uint64_t v = (uint64_t)(rev ^ 2u) << ((k & 31u) * 2u);
                lo |= k < 32 ? v : 0ull;
                hi |= k < 32 ? 0ull : v;
            }
            s.dirs[i] = lo;
            s.dirs[p.n + i] = hi;
        }
        const uint32_t x = e / P, y = e - x * P;
        s.pos[i] = x | (y << 8) | (len << 16) | (off << 24);
        s.aux[i] = (nn & 0x7FFFu) | (outcome << 16) | (pend << 18) | ((nn >> 15) << 19);
        s.step[i] = (uint32_t)step;
        s.pid[i] = pid;
    }
};

// ---- the trie wave.  Its state is one packed word per env, S = global node | terminal << 21 |
// off << 22 | has-solutions << 28: the deepest node of the solution trie on the path, whether
// that node is a complete solution, the path's depth beyond it (0: the path is a solution
// prefix), and the puzzle's solution_count > 0 flag.  The walk S_t -> S_t+1 is a pointer chase
// (a node's children are in memory), so one gather per step would expose the whole gather
// latency every step.  Instead the trie wave takes two steps per iteration: ONE gather from a
// table of 2-move transitions per node (tab2, sparc_load_puzzles) returns both S_t+1 and S_t+2
// from S_t and the two moves, and it is consumed one iteration later, so each gather has two
// steps of work to arrive.  Move classes: forward a -> a, pop -> 4, none -> 5.
constexpr uint32_t kTsTermBit = 21, kTsOffShift = 22, kTsSolBit = 28, kTsNode = (1u << 21) - 1u;
constexpr uint32_t kClsB = 4, kClsN = 5, kClasses = 6, kTab2Row = kClasses * kClasses;
constexpr uint32_t kDeltaLut = 0x4AAu;   // depth change + 1 per class, 2 bits each: 2, 2, 2, 2, 0, 1

__device__ __forceinline__ uint32_t move_class(uint32_t hw) {
    const uint32_t a = (hw >> 10) & 3u;
    return (hw & 0x100u) ? kClsB : ((hw & 0x200u) ? a : kClsN);
}

template <bool TB>
struct TrieLane {
    uint32_t npid;       // the next puzzle
    uint4 nt;            // trow[npid] = {packed root state, next(npid), 0, 0}, prefetched
    uint32_t outcome;    // outcome_reward of the last step: 0, 1 (+1), 2 (-1)
    int acc_x = 0;       // counters: reward code sum, done steps, solved, autoresets
    uint32_t acc_y = 0, acc_z = 0, acc_w = 0;
    uint2 ld, alt;       // {S_t+1, S_t+2}: gathered / when no gather was needed
    bool nd = false;     // ... whether it was needed
    bool ovr = false;    // step t+1 autoresets: S_t+2 is the next puzzle's root, `rsave`
    uint32_t rsave = 0;
    uint32_t hwa = 0, hwb = 0;   // hand-over words of the two steps the pending pair belongs to

    __device__ __forceinline__ void load(const Params& p, const uint4* trow, uint32_t i) {
        const State& s = p.st;
        const uint32_t ps = s.pos[i], ax = s.aux[i];
        const uint4 r = trow[s.pid[i]];
        npid = r.y;
        nt = trow[npid];
        outcome = (ax >> 16) & 3u;
        const uint32_t st = ((r.x & kTsNode) + (ax & 0x7FFFu)) | (((ax >> 19) & 1u) << kTsTermBit) |
                            ((ps >> 24) << kTsOffShift) | (r.x & (1u << kTsSolBit));
        alt = make_uint2(st, st);   // the "pair" before step 0 (only .y is read)
        ld = alt;
    }
    __device__ __forceinline__ uint2 resolve() const {
        uint2 v = nd ? ld : alt;
        v.y = ovr ? rsave : v.y;
        return v;
    }
    // reward code of a step from its hand-over word and the state after it (1201-1223): done:
    // +100 if the path equals a solution, else -100 unless the previous done step already set
    // outcome_reward = 1 (then 0); not done: +-1 when moved on a puzzle with solutions, else 0
    __device__ __forceinline__ int emit(uint32_t hw, uint32_t st) {
        const bool done = (hw & 3u) != 0u;
        const bool on = (st & (0x3Fu << kTsOffShift)) == 0u;
        const bool match = on & ((st >> kTsTermBit) & 1u);
        const bool mv = ((hw & 0x300u) != 0u) & ((st >> kTsSolBit) & 1u);
        const int c_done = match ? 100 : (outcome != 1u ? -100 : 0);
        const int c_move = mv ? (on ? 1 : -1) : 0;
        outcome = done ? ((match | (outcome == 1u)) ? 1u : 2u) : 0u;
        const int code = done ? c_done : c_move;
        acc_x += code;
        acc_y += (uint32_t)done;
        acc_z += (uint32_t)(done & match);
        acc_w += (hw >> 6) & 1u;
        return code;
    }
    // steps t, t+1 (hand-over words h0, h1): emit the pending pair's two steps at ca / cb (if
    // non-null), then issue {S_t+1, S_t+2}
    __device__ __forceinline__ void iter(const Params& p, const uint4* trow, uint32_t h0, uint32_t h1, uint8_t* ca,
                                         uint8_t* cb) {
        const uint2 pr = resolve();
        if (ca) *ca = (uint8_t)emit(hwa, pr.x);
        if (cb) *cb = (uint8_t)emit(hwb, pr.y);
        const bool rs0 = (h0 >> 6) & 1u, rs1 = (h1 >> 6) & 1u;   // autoreset steps (never both)
        const uint32_t rnext = nt.x;
        const uint32_t stp = rs0 ? rnext : pr.y;   // S_t, or the next root if step t resets
        const uint32_t m1 = rs0 ? kClsN : move_class(h0);
        const uint32_t m2 = move_class(h1);
        npid = (rs0 | rs1) ? nt.y : npid;
        nt = trow[npid];   // unchanged unless a lane reset
        const uint32_t off = (stp >> kTsOffShift) & 0x3Fu;
        // the two moves can touch the trie only from on it, or from one above it with a pop first
        const bool need = off <= (uint32_t)(m1 == kClsB);
        const uint32_t cs = (off != 0u ? kClsN : m1) * kClasses + m2;   // off 1: the pop is in `off`
        ld = reinterpret_cast<const uint2*>(p.tab.tab2)[need ? (stp & kTsNode) * kTab2Row + cs : 0u];
        const uint32_t s1 = stp + ((((kDeltaLut >> (2u * m1)) & 3u) - 1u) << kTsOffShift);
        alt = make_uint2(s1, s1 + ((((kDeltaLut >> (2u * m2)) & 3u) - 1u) << kTsOffShift));
        nd = need;
        ovr = rs1;
        rsave = rnext;
        hwa = h0;
        hwb = h1;
    }
    // the SoA record of the last state: local node | terminal << 15, off, current puzzle
    __device__ __forceinline__ void final_state(const uint4* trow, uint32_t st, uint32_t num_puzzles, uint32_t& nn,
                                                uint32_t& off, uint32_t& pid) const {
        pid = npid == 0u ? num_puzzles - 1u : npid - 1u;
        nn = ((st & kTsNode) - (trow[pid].x & kTsNode)) | (((st >> kTsTermBit) & 1u) << 15);
        off = (st >> kTsOffShift) & 0x3Fu;
    }
};

}  // namespace sparc
