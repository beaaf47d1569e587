// sparc_mask.hpp — the trie wave of k_rollout1s on solution LEAF SETS (device code).
//
// The reward (SPaRC_Gym.py:1201-1223) asks two questions of the path: is it a prefix of some
// solution (_is_on_solution_path, 1244-1265), and does it equal one (np.array_equal, 1206).  The
// node trie answers both with one pointer chase per step: the record of node(t) is known only
// after node(t-1)'s record arrived, so every on-trie step waits for an L2 gather (~250 cycles on
// MI355X, the critical path of the trie wave).
//
// Here the trie state is the SET of trie leaves below the path's deepest on-trie node, one bit
// per leaf (<= 31 leaves per puzzle), and each step ANDs in a mask that depends only on
// (puzzle, depth, move), never on the state:
//   forward move d at depth m (m moves so far):   A' = A & M(m, d)      (empty: the path left
//                                                                       the trie, off = 1)
//   the new node is a complete solution          <=> A' & E(m + 1) != 0
//   traceback pop back to depth m - 1:            A' = S[m - 1]        (the set one level up)
//   reset (SPaRC_Gym.py:1087):                    A' = A0 (every leaf), off = (A0 == 0)
// with M(m, d) = the leaves whose move m is d, E(k) = the leaves whose depth-k ancestor is a
// complete solution.  All leaves of A share their depth-k ancestor, so E answers "terminal" for
// the node itself.  The masks of one tile's 16 steps are gathered before any of them is used
// (the addresses need only the hand-over words: depth and puzzle index follow from the moves and
// resets), so no gather latency sits on the per-step chain.  Pops read S[m - 1] from a per-lane
// LDS stack of the sets along the path, one step ahead.
//
// Table (sparc_load_puzzles, words == 1), per puzzle q a block of R = Dmax + 2 rows (32 B each),
// row i = four uint2 pairs, pair d = {M(i - 1, d), E(i)}; row 0 = {A0, E(0) | has_solutions << 31}
// in every pair.  So the mask of a step after which the path has m' moves is pair `action` of
// row min(m', R - 1): a forward move reads M and E(m'), a pop reads E(m') (the lo half is
// unused), a reset step (m' = 0) reads the new puzzle's root set.  Row R - 1 is all zero (no
// leaf that deep).  Blocks P .. P + 15 repeat blocks 0 .. 15 (mod P), so that a tile's resets
// (<= 16, each to the next puzzle) only ever add one block to the byte offset; it is reduced
// mod P once per tile.  Launch boundaries convert to the node-trie SoA record (Env<1>::store /
// load): the node is nodeof[leafbase(q) + lowest leaf of A][depth], the sets along the path are
// rebuilt from the stored moves (traceback) or read from leafset[node] (no traceback: no pops).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "sparc_env.hpp"

namespace sparc {

constexpr uint32_t kMaskLeaves = 31;   // leaf bits per puzzle (row 0 keeps has_solutions in bit 31)

// AR: next-step autoreset (the only mode with resets inside a rollout; it also makes the
// outcome_reward carry-over of 1211 unobservable: a done step always follows a non-done one)
template <bool TB, bool AR>
struct MaskTrie {
    uint32_t A = 0;        // leaf set of the deepest on-trie node (garbage while the root is invalid)
    uint32_t hs = 0;       // the puzzle has solutions (solution_count > 0; 1205, 1217)
    uint32_t below = 0;    // S[m_on - 1], the set one level up (traceback pops)
    uint32_t pre = 0;      // LDS slot m - 2, read one step ahead (the refill after a pop)
    uint32_t off = 0;      // depth of the path beyond that node (> m: the root is invalid)
    uint32_t mt = 0;       // that node is a complete solution
    uint32_t m = 0;        // moves on the path (len(self.path) - 1)
    uint32_t pb = 0;       // byte offset of the current puzzle's block
    uint32_t outcome = 0;  // 0, 1 (+1), 2 (-1); AR: derived from the last step at the end
    uint32_t done_l = 0, match_l = 0;
    int acc_x = 0;         // reward code sum
    uint32_t acc_y = 0, acc_z = 0, acc_w = 0;   // done steps, solved, autoresets (TB)
    const uint8_t* blk = nullptr;   // mask blocks [P + 16][R][4] uint2
    uint32_t R = 0, smax = 0;       // rows per block; last stack slot (R - 1)
    uint32_t RB = 0, PRB = 0;       // bytes per block, P blocks
    uint8_t* stk = nullptr;         // this lane's column of the [R + 2 slots][64] u32 stack, slot -2

    __device__ __forceinline__ uint32_t& slot(uint32_t byte_off) {
        return *reinterpret_cast<uint32_t*>(stk + byte_off);
    }
    __device__ __forceinline__ uint2 mask(uint32_t byte_off) const {
        return *reinterpret_cast<const uint2*>(blk + byte_off);
    }
    __device__ __forceinline__ uint32_t sa_of(uint32_t mm) const { return (mm < smax ? mm : smax) * 256u; }

    // SoA record -> leaf-set state (the trie wave's part of Env<1>::load)
    template <class Src>
    __device__ __forceinline__ void load(const Params& p, const Src& src, uint32_t i) {
        const State& s = p.st;
        blk = reinterpret_cast<const uint8_t*>(p.tab.mblk);
        R = p.tab.mrows;
        smax = R - 1u;
        RB = R * 32u;
        PRB = p.tab.num_puzzles * RB;
        const uint32_t ps = s.pos[i], ax = s.aux[i];
        const uint32_t pid = s.pid[i];
        pb = pid * RB;
        off = ps >> 24;
        m = ((ps >> 16) & 0xFFu) - 1u;
        outcome = (ax >> 16) & 3u;
        mt = (ax >> 19) & 1u;
        const uint2 r0 = mask(pb);
        A = r0.x;
        hs = r0.y >> 31;
        if (A) {                                  // the root is valid: m_on = m - off >= 0
            const uint32_t mon = m - off;
            if constexpr (TB) {
                // S[k + 1] = S[k] & M(k, move k), from the stored moves; slots 0..m_on-1 = S[k]
                const uint64_t lo = s.dirs[i], hi = s.dirs[p.n + i];
                uint32_t S = A;
                for (uint32_t k0 = 0; k0 < mon; k0 += 8) {
                    uint32_t mk[8];
#pragma unroll
                    for (uint32_t j = 0; j < 8; ++j) {
                        const uint32_t k = k0 + j;
                        const uint32_t d = (uint32_t)(((k < 32 ? lo : hi) >> ((k & 31u) * 2u)) & 3u);
                        const uint32_t row = k + 1u < R ? k + 1u : R - 1u;
                        mk[j] = mask(pb + row * 32u + d * 8u).x;
                    }
#pragma unroll
                    for (uint32_t j = 0; j < 8; ++j) {
                        const uint32_t k = k0 + j;
                        if (k < mon) {
                            slot((k + 2u) * 256u) = S;
                            below = S;
                            S &= mk[j];
                        }
                    }
                }
                A = S;
            } else {
                const uint32_t tb = src.get_row1(pid).y;
                A = p.tab.leafset[tb + (ax & 0x7FFFu)];
            }
        }
        if constexpr (TB) pre = slot(sa_of(m));
    }

    // one 16-step tile: th / tr point at this lane's hand-over word / reward code of the tile's
    // first step (row stride 64 lanes).  Branch-free: a reset step is a forward move into the
    // new root from a virtual parent that holds every leaf (A = ~0, on the trie).
    __device__ __forceinline__ void tile(const uint16_t* th, uint8_t* tr) {
        uint32_t hw[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) hw[j] = th[j * 64];
        // gather pass: every step's mask (depth and puzzle follow from the words alone)
        uint2 G[16];
        uint32_t sa[17];
        uint32_t ma = m;
        sa[0] = sa_of(ma);
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const uint32_t h = hw[j];
            const uint32_t v = __builtin_amdgcn_ubfe(h, 8u, 2u);   // 1 + forward - pop
            if constexpr (AR) {
                const uint32_t rsm = (uint32_t)__builtin_amdgcn_sbfe((int32_t)h, 6u, 1u);   // 0 / ~0
                pb += rsm & RB;                                    // reset: the next puzzle's block
                ma = (ma + v - 1u) & ~rsm;
            } else {
                ma = ma + v - 1u;
            }
            const uint32_t row = ma < smax ? ma : smax;
            sa[j + 1] = row * 256u;
            G[j] = mask(pb + row * 32u + __builtin_amdgcn_ubfe(h, 10u, 2u) * 8u);
        }
        // state pass
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const uint32_t h = hw[j];
            const uint2 g = G[j];
            const uint32_t v = __builtin_amdgcn_ubfe(h, 8u, 2u);
            uint32_t Ae = A, oe = off;
            bool fwd = v == 2u;
            bool rs = false;
            if constexpr (AR) {
                rs = (h & 64u) != 0u;
                Ae = rs ? ~0u : A;
                oe = rs ? 0u : off;
                fwd = fwd | rs;
                hs = rs ? g.y >> 31 : hs;
            }
            const bool on = oe == 0u;
            const uint32_t A2 = Ae & g.x;
            const bool has = A2 != 0u;
            const bool down = fwd & on & has;
            const uint32_t noff = on ? (uint32_t)(fwd & !has) : oe + v - 1u;
            uint32_t nA, nmt;
            if constexpr (TB) {
                const bool up = (v == 0u) & on;
                slot(sa[j] + 512u) = A;                     // S[m] (matters when it goes down)
                const uint32_t X = down ? A2 : below;
                nmt = (down | up) ? (uint32_t)((X & g.y) != 0u) : mt;
                nA = down ? A2 : (up ? below : Ae);
                below = down ? Ae : (up ? pre : below);
                pre = slot(sa[j + 1]);                      // S[m' - 2], for a pop at the next step
            } else {
                nmt = down ? (uint32_t)((A2 & g.y) != 0u) : mt;
                nA = down ? A2 : Ae;
            }
            A = nA;
            mt = nmt;
            off = noff;
            const bool match = (noff == 0u) & (nmt != 0u);
            const bool done = (h & 3u) != 0u;
            const bool mv = (v != 1u) & (hs != 0u);   // moved, on a puzzle with solutions
            int code;
            if constexpr (AR) {
                // done: +-100 (match); else moved: +-1 (on the trie); else 0
                const bool pos = done ? match : (noff == 0u);
                const int mag = done ? 100 : (int)mv;
                code = pos ? mag : -mag;
                done_l = (uint32_t)done;
                match_l = (uint32_t)match;
            } else {
                code = done ? (match ? 100 : (outcome != 1u ? -100 : 0)) : (mv ? (noff == 0u ? 1 : -1) : 0);
                outcome = done ? ((match | (outcome == 1u)) ? 1u : 2u) : 0u;
            }
            tr[j * 64] = (uint8_t)code;
            acc_x += code;
            acc_z += (uint32_t)(done & match);
            if constexpr (TB) {
                acc_y += (uint32_t)done;
                acc_w += (uint32_t)rs;
            }
        }
        m = ma;
        if constexpr (AR) pb = pb >= PRB ? pb % PRB : pb;
    }

    // leaf-set state -> the node-trie fields of the SoA record: packed node (index | terminal
    // << 15) and outcome
    template <class Src>
    __device__ __forceinline__ void final_state(const Params& p, const Src& src, uint32_t& nn, uint32_t& oc) const {
        uint32_t node = 0, term = 0;
        if (off <= m && A != 0u) {                // the root is valid (else off > m, node 0)
            const uint32_t leafbase = src.get_row1(pb / RB).w;
            node = p.tab.nodeof[(size_t)(leafbase + (uint32_t)__builtin_ctz(A)) * R + (m - off)];
            term = mt;
        }
        nn = node | (term << 15);
        oc = AR ? (done_l ? (match_l ? 1u : 2u) : 0u) : outcome;
    }
};

}  // namespace sparc
