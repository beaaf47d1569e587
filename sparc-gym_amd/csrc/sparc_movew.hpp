// sparc_movew.hpp — the move wave of the multi-word split rollout (k_rolloutWs), device code.
//
// The W = 1 move step (Env<1> in sparc_env.hpp) keeps a 64-bit FREE board (in the lattice,
// not a gap, unvisited) one row up in a register, so that _get_legal_actions
// (SPaRC_Gym.py:1024-1051) is one shift.  Lattices of 9x9 to 15x15 points do not fit 64 bits,
// and registers cannot be indexed per lane, so here the same board lives in LDS:
//
//   internal pitch P2 = plain pitch + 1 (a blocked padding column), point (x, y) at bit
//   (x + 1) * P2 + y (a blocked row below x = 0), B dwords per lane, laid out [dword][64 lanes]
//   so that lane l's dword k is at 256 * k + 4 * l: every lane sits in its own bank, whatever
//   dword it reads (conflict-free divergent reads).
//
// The agent is e = x * P2 + y.  The 64-bit window w = board >> e (two dwords, one ds_read2)
// holds the four neighbours at bits 0 (left, x-1), P2-1 (up, y-1), P2+1 (down, y+1) and 2 * P2
// (right, x+1); out-of-lattice neighbours read 0 (padding column, empty row below, bits above
// the last row), so there are no bounds compares.  A move toggles one bit with a non-returning
// ds_xor_b32 (the target point for a forward move, the left point for a traceback pop).  The
// path's reversed moves sit in an LDS byte stack [M moves][64 lanes], as in LdsStack.
//
// Per step the move wave writes the 16-bit hand-over word of the trie wave (hand_word16) and
// runs no trie work; TrieLane (sparc_trie.hpp) does the solution-trie walk and the reward.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "sparc_env.hpp"

namespace sparc {

// runtime layout of k_rolloutWs, computed by the host for the pool (sparc_load_puzzles)
struct SplitGeom {
    uint32_t P2;        // internal pitch (<= 16: the window's right neighbour is bit 2 * P2 <= 32)
    uint32_t B;         // board dwords per lane (board + one zero dword above the top row)
    uint32_t BS;        // B rounded up to 4: dwords per lane in LDS and per puzzle in the reset-board table
    uint32_t M;         // move-stack bytes per lane (>= the lattice's point count, multiple of 16:
                        // a step writes slot len - 1 even when it does not move, and len <= points)
    uint32_t nbr_pos;   // window bit of each direction's neighbour, one byte per direction
    uint32_t pair;      // LDS bytes per move / trie wave pair
    uint32_t off_board, off_stack;   // their offsets within a pair
};

// 16-bit hand-over word of the multi-word kernel: bits 0-7 the flag byte, bits 8-9
// fwd - pop + 1, bits 10-11 action & 3.  The trie wave widens it to TrieLane's word (flag byte
// | (fwd - pop) << 16) and the action.
__device__ __forceinline__ uint32_t hand_word16(uint32_t a, uint32_t fwd, uint32_t pop, uint32_t f) {
    return f | ((fwd + 1u - pop) << 8) | ((a & 3u) << 10);
}
__device__ __forceinline__ uint32_t widen_hand_word(uint32_t h) {
    return (h & 0xFFu) | ((__builtin_amdgcn_ubfe(h, 8u, 2u) - 1u) << 16);
}

constexpr uint32_t kBoardRegs = 4;   // 16-B pieces of the next reset board kept in registers

template <bool TB>
struct MoveLaneW {
    uint32_t e = 0, tgt = 0, len = 1, pflags = 0, bk = 0, legal = 0, rl = 0, pnr = 0, rs = 0, pending = 0, pid = 0;
    int32_t step = 0;
    uint64_t w = 0;                  // window of the board at e, valid between steps
    uint32_t* bd = nullptr;          // this lane's dword 0 (stride 64 dwords)
    uint8_t* col = nullptr;          // this lane's stack column (stride 64 bytes)
    uint32_t s_a = 0, s_fwd = 0, s_pop = 0, s_mv = 0, s_done = 0;
    // the next autoreset's move row and reset board (puzzle pid + 1), read at the previous reset
    // (or at load) into registers: the reset then writes them to the LDS board without a memory
    // round trip in the branch (BS <= kBoardRegs * 4 dwords, host-checked)
    uint4 nrow = {0u, 0u, 0u, 0u};
    uint4 nb[kBoardRegs];

    __device__ __forceinline__ uint32_t& dw(uint32_t k) const { return bd[k * 64u]; }

    // the window at e and the legal mask of the current state (1024-1051); traceback: path[-2]
    // (the reverse of the last move, rl) is legal although visited when len >= 3, or len == 2
    // and the start is open (bk bias, as Env<1>)
    __device__ __forceinline__ void read_window(const SplitGeom& g) {
        const uint32_t k = e >> 5;
        const uint64_t pr = ((uint64_t)dw(k + 1u) << 32) | dw(k);
        w = pr >> (e & 31u);
        const uint32_t lo = (uint32_t)w;
        const uint32_t ud = __builtin_amdgcn_ubfe(lo, g.P2 - 2u, 4u);
        uint32_t m = (ud & 10u) | ((lo << 2) & 4u) | ((uint32_t)(w >> (2u * g.P2)) & 1u);
        if constexpr (TB) m |= ((len + bk) >> 31) << rl;
        legal = m;
    }

    __device__ __forceinline__ void apply_row(const uint4 r) {
        e = r.x & 0xFFFFu;
        tgt = r.x >> 16;
        pflags = r.y;
        bk = 0x7FFFFFFDu + ((~pflags >> 2) & 1u);
    }

    // gymnasium next-step autoreset (reset(), SPaRC_Gym.py:1087): puzzle index + 1 mod P, its
    // reset board copied into this lane's board.  Resets are rare per lane; the row and board
    // come from the L2-resident tables.
    __device__ __forceinline__ void prefetch_next(const Params& p, const SplitGeom& g, const uint4* __restrict__ mrow,
                                                  const uint32_t* __restrict__ boards) {
        const uint32_t q = pid + 1 == p.tab.num_puzzles ? 0u : pid + 1;
        nrow = mrow[q];
        const uint4* src = reinterpret_cast<const uint4*>(boards + (size_t)q * g.BS);
#pragma unroll
        for (uint32_t k = 0; k < kBoardRegs; ++k)
            if (4u * k < g.BS) nb[k] = src[k];
    }
    __device__ __forceinline__ void reset_next(const Params& p, const SplitGeom& g, const uint4* __restrict__ mrow,
                                               const uint32_t* __restrict__ boards) {
        if (pending & (uint32_t)(p.autoreset == 1)) {
            pid = pid + 1 == p.tab.num_puzzles ? 0u : pid + 1;
            apply_row(nrow);
#pragma unroll
            for (uint32_t k = 0; k < kBoardRegs; ++k) {
                if (4u * k < g.BS) {
                    dw(4u * k) = nb[k].x;
                    dw(4u * k + 1u) = nb[k].y;
                    dw(4u * k + 2u) = nb[k].z;
                    dw(4u * k + 3u) = nb[k].w;
                }
            }
            len = 1;
            step = -1;   // this step's increment brings it to 0
            rs = 1;
            // the row's uses above happen before the reads below (memory clobber), so the reads
            // can land in the same registers: copied on from temporaries instead, the branch
            // would wait for them
            asm volatile("" ::"v"(e), "v"(tgt), "v"(bk) : "memory");
            prefetch_next(p, g, mrow, boards);   // waited for at the next reset
        }
    }

    // one step's move part (1131-1199): legality, move or traceback pop, path, terminated /
    // truncated; returns the flag byte
    __device__ __forceinline__ uint32_t phase_move(const Params& p, const SplitGeom& g, uint32_t a) {
        const uint32_t P = g.P2;
        step = __builtin_elementwise_add_sat(step, 1);                              // 1132
        const bool trunc0 = step >= p.max_steps;                                    // 1134
        const uint32_t moved = (legal >> (a < 4u ? a : 4u)) & (rs ^ 1u) & 1u;       // 1137
        const uint32_t pos = __builtin_amdgcn_ubfe(g.nbr_pos, a << 3, 8u);
        // the only legal move onto a non-free point is the traceback pop (1141-1166)
        const uint32_t pop = TB ? moved & ~(uint32_t)(w >> pos) & 1u : 0u;
        const uint32_t fwd = moved ^ pop;                                            // 1167-1188
        // free board: a forward move takes the target (bit e + pos), a pop frees the point it
        // leaves (bit e + P)
        const uint32_t tog = e + (fwd ? pos : P);
        __hip_atomic_fetch_xor(&dw(tog >> 5), moved << (tog & 31u), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
        if constexpr (TB) {
            const uint32_t ar = a ^ 2u;
            col[(len - 1u) * 64u] = (uint8_t)ar;     // the new top if fwd, above the top otherwise
            rl = fwd ? ar : (pop ? pnr : rl);
        }
        len = len + fwd - pop;
        e = (uint32_t)((int32_t)e + __mul24((int32_t)moved, (int32_t)pos - (int32_t)P));
        read_window(g);
        const uint32_t live = rs ^ 1u;                                               // 0 on a reset step
        const uint32_t term = e == tgt ? live : 0u;                                  // 1192
        const uint32_t trunc = (trunc0 | (legal == 0)) ? live ^ term : 0u;          // 1195-1199
        const uint32_t done = term | trunc;
        pending = done;
        if constexpr (TB) pnr = col[__builtin_elementwise_sub_sat(len, 3u) * 64u];  // next step's pop
        s_a = a;
        s_fwd = fwd;
        s_pop = pop;
        s_mv = moved & pflags & 1u;   // moved, and the puzzle has solutions (1205, 1217)
        s_done = done;
        const uint32_t f = (legal << 2) | (rs << 6) | term | (trunc << 1);
        rs = 0;
        return f;
    }

    // ---- SoA <-> LDS.  HBM keeps the generic plain layout (bit x * pitch + y, W words,
    // Env<W>); the board is converted row by row at the start and the end of a launch.
    template <int W>
    __device__ __forceinline__ void load(const Params& p, const SplitGeom& g, const uint4* __restrict__ mrow, uint32_t i) {
        const State& s = p.st;
        const uint32_t pitch = p.pitch;
        uint64_t fr[W];
        pid = s.pid[i];
        const uint4 inf = p.tab.info[pid];
        const uint32_t X = inf.x & 0xFFu, Y = (inf.x >> 8) & 0xFFu;
#pragma unroll
        for (int k = 0; k < W; ++k) fr[k] = p.tab.open[(size_t)pid * W + k] & ~s.vis[(size_t)k * p.n + i];
        for (uint32_t k = 0; k < g.BS; ++k) dw(k) = 0u;
        const uint64_t ymask = (1ull << Y) - 1ull;
        for (uint32_t x = 0; x < X; ++x) {
            const uint32_t sb = x * pitch, j = sb >> 6, o = sb & 63u;
            const uint64_t lo = bb_word<W>(fr, j), hi = bb_word<W>(fr, j + 1u);
            const uint64_t row = ((lo >> o) | (o ? hi << (64u - o) : 0ull)) & ymask;
            const uint32_t db = (x + 1u) * g.P2 + 0u;
            const uint64_t v = row << (db & 31u);
            dw(db >> 5) |= (uint32_t)v;
            if (v >> 32) dw((db >> 5) + 1u) |= (uint32_t)(v >> 32);
        }
        const uint32_t ps = s.pos[i];
        e = (ps & 0xFFu) * g.P2 + ((ps >> 8) & 0xFFu);
        len = (ps >> 16) & 0xFFu;
        const uint32_t ax = s.aux[i];
        pending = (ax >> 18) & 1u;
        step = (int32_t)s.step[i];
        const uint4 r = mrow[pid];
        tgt = r.x >> 16;
        pflags = r.y;
        bk = 0x7FFFFFFDu + ((~pflags >> 2) & 1u);
        if constexpr (TB) {
            const uint32_t moves = len >= 1 ? len - 1 : 0u;
#pragma unroll
            for (int j = 0; j < 2 * W; ++j) {
                const uint64_t d = s.dirs[(size_t)j * p.n + i] ^ kRev2;
                for (uint32_t k = 32u * j; k < moves && k < 32u * (j + 1); ++k)
                    col[k * 64u] = (uint8_t)((d >> ((k & 31u) * 2u)) & 3u);
            }
            rl = len >= 2 ? col[(len - 2u) * 64u] : 0u;
            pnr = col[__builtin_elementwise_sub_sat(len, 3u) * 64u];
        }
        rs = 0;
        read_window(g);
    }

    // S, outcome: the trie wave's final trie state (off << 16 | packed node) and outcome_reward
    template <int W>
    __device__ __forceinline__ void store(const Params& p, const SplitGeom& g, uint32_t i, uint32_t S,
                                          uint32_t outcome) const {
        const State& s = p.st;
        const uint32_t pitch = p.pitch;
        const uint4 inf = p.tab.info[pid];
        const uint32_t X = inf.x & 0xFFu, Y = (inf.x >> 8) & 0xFFu;
        const uint32_t sx = (inf.x >> 16) & 0xFFu, sy = inf.x >> 24;
        uint64_t vis[W];
#pragma unroll
        for (int k = 0; k < W; ++k) vis[k] = 0;
        const uint64_t ymask = (1ull << Y) - 1ull;
        for (uint32_t x = 0; x < X; ++x) {
            const uint32_t db = (x + 1u) * g.P2, k = db >> 5;
            const uint64_t pr = ((uint64_t)dw(k + 1u) << 32) | dw(k);
            const uint64_t row = ~(pr >> (db & 31u)) & ymask;   // not free
            const uint32_t sb = x * pitch, j = sb >> 6, o = sb & 63u;
#pragma unroll
            for (int q = 0; q < W; ++q) {
                vis[q] |= (j == (uint32_t)q) ? row << o : 0ull;
                vis[q] |= (o && j + 1u == (uint32_t)q) ? row >> (64u - o) : 0ull;
            }
        }
        // visited = in the puzzle and not free, plus the start (always on the path)
        const uint32_t sbit = sx * pitch + sy;
#pragma unroll
        for (int q = 0; q < W; ++q) {
            uint64_t v = vis[q] & p.tab.open[(size_t)pid * W + q];
            v |= ((sbit >> 6) == (uint32_t)q) ? 1ull << (sbit & 63u) : 0ull;
            s.vis[(size_t)q * p.n + i] = v;
        }
        if constexpr (TB) {
            const uint32_t moves = len >= 1 ? len - 1 : 0u;
#pragma unroll
            for (int j = 0; j < 2 * W; ++j) {
                uint64_t d = 0;
                for (uint32_t k = 32u * j; k < moves && k < 32u * (j + 1); ++k)
                    d |= (uint64_t)((col[k * 64u] ^ 2u) & 3u) << ((k & 31u) * 2u);
                s.dirs[(size_t)j * p.n + i] = d;
            }
        }
        const uint32_t x = e / g.P2, y = e - x * g.P2;
        s.pos[i] = x | (y << 8) | (len << 16) | ((S >> 16) << 24);
        s.aux[i] = (S & 0x7FFFu) | (outcome << 16) | (pending << 18) | (((S >> 15) & 1u) << 19);
        s.step[i] = (uint32_t)step;
        s.pid[i] = pid;
    }
};

}  // namespace sparc
