// sparc_move1.hpp — the move wave of the W = 1 split rollout (k_rollout1s), device code.
//
// The split kernel runs each env's step() (SPaRC_Gym.py:1111-1238) over two waves: this MOVE
// wave (legality, move or traceback pop, path, terminated / truncated) and the trie wave
// (TrieLane, sparc_trie.hpp: solution trie, reward).  A lone wave issues in order, so every
// instruction of the move wave's step lies on its time line; this lane keeps only what the
// step's dependency chain needs and pushes the rest to the I/O wave and the host:
//
//  * the I/O wave hands over, per env-step, the WINDOW POSITION of the action's target instead
//    of the action: pos = bit of the target point in the window w = fr >> e (right 2P, up P-1,
//    left 0, down P+1; Env<1> in sparc_env.hpp explains the padded board, one row up), and P
//    for an illegal action (>= 4): bit P of the window is the agent's own point, never free,
//    so an illegal action tests "not free" and moves nowhere (SPaRC_Gym.py:1137);
//  * a forward move is legal iff bit pos of w is set; the traceback pop (1141-1166) iff pos is
//    the window position of path[-2] (rp, kept in a register) and the traceback rule holds
//    (bias: len >= 3, or len == 2 with an open start);
//  * the stack holds the back positions (2P - pos of each move), so the pop needs no
//    direction arithmetic;
//  * the legal-action mask (1024-1051) and the flag byte are not built here: the word carries
//    the step's legal window bits lw = (w & NBM) | bias << rp, at-target and done, and the I/O
//    wave turns four words into four flag bytes (flag_bytes4, sparc_kernels.hip: the legal bits
//    via one multiply by p.lmagic, which carries the four bits right / up / left / down to bits
//    18..21 without carries);
//  * lw == 0 is the empty legal set (truncation, 1195);
//  * an autoreset step hands over at-target set and done clear, a pair no other step has (at the
//    target is done), so the reset needs no bit of its own.
//
// Hand-over word (to the trie wave and the I/O wave):
//   bits 0..18   lw (window bits of the legal actions after the step)
//   bit 24       at the target, or an autoreset step
//   bit 25       done: terminated or truncated (0 on an autoreset step)
//   bits 30..31  fwd - pop, two's complement (+1 forward, -1 pop, 0 no move)
//   other bits   0
// Valid for pitches 3..9 (host-checked): the legal-bit constant needs 2P <= 18.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "sparc_env.hpp"

namespace sparc {

constexpr uint32_t kHwLw = 0x7FFFFu, kHwTgt = 1u << 24, kHwDone = 1u << 25;
// the step of hand-over word hw was an autoreset step
__device__ __forceinline__ bool hw_reset(uint32_t hw) { return (hw & (kHwTgt | kHwDone)) == kHwTgt; }

// Row slots (k_rollout1s on pools past the LDS row budget).  The trie wave runs one tile behind
// the move wave, so the move wave, which reads both rows of the next puzzle from the L2 at the
// previous reset anyway, hands the trie row over through LDS: per env kRowSlots slots and one
// spare, [kRowSlots + 1][256 envs] uint4.  The move wave writes reset r's row to slot r %
// kRowSlots during the interval of its tile t_r; the trie wave reads it during interval t_r + 1
// (reset ordinals r = 0, 1, ... count this launch's resets of the env; both waves count the same
// events).  The write is allowed when the slot's previous occupant, reset r - kRowSlots, was read
// in an earlier interval: t_(r - kRowSlots) <= t_r - 2, i.e. r < C(t_r - 2) + kRowSlots with C(t)
// the resets in tiles <= t.  Both waves evaluate that rule from their own counts; when it fails
// the move wave writes the spare slot instead and the trie wave reads the row from the L2 itself
// (an episode of a few steps: two resets within two tiles).  Barriers separate every write from
// its read and from the next write of the slot.
constexpr uint32_t kRowSlots = 2, kRowSlotStride = 256u * 16u;

// the carry-free gather constant and the neighbour mask of the window for pitch P (host and
// device): window bits {2P, P-1, 0, P+1} -> product bits 18, 19, 20, 21 (right, up, left, down)
__host__ __device__ constexpr uint32_t legal_magic(uint32_t P) {
    return (1u << (18u - 2u * P)) + (1u << (20u - P)) + (1u << 20u);
}
__host__ __device__ constexpr uint32_t window_nbm(uint32_t P) {
    return 1u | (1u << (P - 1u)) | (1u << (P + 1u)) | (1u << (2u * P));
}
__host__ __device__ constexpr bool split1_pitch_ok(uint32_t P) { return P >= 3u && P <= 9u; }

// direction <-> window position of its neighbour (only at launch start / end)
__device__ __forceinline__ uint32_t dir_pos1(uint32_t d, uint32_t P) {
    return d == 0u ? 2u * P : d == 1u ? P - 1u : d == 2u ? 0u : P + 1u;
}
__device__ __forceinline__ uint32_t pos_dir1(uint32_t pos, uint32_t P) {
    return pos == 2u * P ? 0u : pos == P - 1u ? 1u : pos == 0u ? 2u : 3u;
}

template <bool TB>
struct MoveLane1 {
    uint64_t fr = 0;          // free board, one row up (bit e + P = point e)
    uint32_t e = 0, w = 0;    // agent bit; window (fr >> e) between steps, 0 on a reset step
    uint32_t tgt = 0, pflags = 0, len = 1;
    bool pending = false;                 // the last step was done (not an autoreset step)
    int32_t step = 0;
    // traceback: sq = the LDS byte address of stack slot len-3 (slot len-1 is sq + 128: the step
    // writes it through the instruction's offset field and reads slot len-3 with no address add),
    // the rule bias and its constant
    uint32_t sq = 0, bks = 0, bias = 0;
    uint32_t rp = 0, pnr = 0;             // traceback: back position of the last move / the one before
    uint4 rr = {0u, 0u, 0u, 0u};          // the next autoreset's move row: row word, free board, the puzzle after it
    // global rows (k_rollout1s<…, LDS_TABLE = false>, row_slots below): the next autoreset's trie
    // row, handed to the trie wave through its slot; this launch's reset count and the tile
    // bookkeeping of the slot rule
    // (4-vectors, so that each row keeps one register tuple through the loop and the next read
    // lands in it: as a struct the compiler split the move row and copied the read's result into
    // the pieces, waiting for the L2 in the reset branch)
    typedef uint32_t v4u __attribute__((ext_vector_type(4)));
    typedef __attribute__((address_space(3))) v4u lds_v4;
    v4u rg = {0u, 0u, 0u, 0u}, rt = {0u, 0u, 0u, 0u};
    uint32_t nres = 0, lim = kRowSlots, cA = 0;

    typedef __attribute__((address_space(3))) uint8_t lds_u8;
    __device__ __forceinline__ static lds_u8* lds_byte(uint32_t a) { return (lds_u8*)(uintptr_t)a; }
    __device__ __forceinline__ static uint32_t lds_addr(const uint8_t* g) { return (uint32_t)(uintptr_t)(lds_u8*)g; }

    __device__ __forceinline__ void set_bks(uint32_t col_addr) {
        // (sq + bks) >> 31 = len >= 3, or len == 2 and the start is open (pflags bit 2 clear)
        bks = 0x80000000u - col_addr + 64u * ((~pflags >> 2) & 1u);
    }
    __device__ __forceinline__ void prefetch_reset(const uint4* mrow, uint32_t q) {
        rr = mrow[q];
    }

    // gymnasium next-step autoreset (reset(), SPaRC_Gym.py:1087): the next puzzle's row and
    // board from registers (read at the previous reset); the step then moves nowhere (w = 0,
    // bias = 0), is never done and hands over at-target (step_pos); returns whether it reset.  ar:
    // p.autoreset == 1 (a compile-time true in the kernels that serve only that mode).  The row of the reset
    // after it is read inside the branch straight into the same registers, so nothing waits for
    // it until the next reset (at least two steps later: a reset step is never done).  Copied
    // on from temporaries instead, the branch waited for the LDS read on every reset (about a
    // fifth of all wave-steps take the branch)
    __device__ __forceinline__ bool reset_next(const bool ar, const uint4* mrow, uint32_t col_addr) {
        const bool rs = pending & ar;
        if (rs) {
            e = rr.x & 0xFFu;
            tgt = (rr.x >> 8) & 0xFFu;
            pflags = rr.x >> 16;
            fr = ((uint64_t)rr.z << 32) | rr.y;
            w = 0;
            if constexpr (TB) {
                sq = col_addr - 128u;   // len = 1
                set_bks(col_addr);
                bias = 0;
            } else {
                len = 1;
            }
            step = -1;   // this step's increment brings it to 0
            // keep the uses of the old row above the read (as TrieLane::step_core): without this
            // the compiler issued the read first into temporaries and waited for it in the branch
            __asm__ volatile("" ::"v"(fr), "v"(e), "v"(tgt), "v"(pflags) : "memory");
            rr = mrow[rr.w];
        }
        return rs;
    }

    // the same from global rows: the move row and the trie row of the next puzzle are read from
    // the L2-resident tables into registers at the previous reset (the wave waits for them only
    // at its next reset); the trie row goes on to the trie wave through slot nres % kRowSlots
    // (row_slots), or to this lane's spare slot when the rule forbids the write
    __device__ __forceinline__ void prefetch_reset_g(const uint4* __restrict__ mrow, const uint4* __restrict__ trow,
                                                     uint32_t q) {
        rg = ld_off(reinterpret_cast<const v4u*>(mrow), q << 4);
        rt = ld_off(reinterpret_cast<const v4u*>(trow), q << 4);
    }
    __device__ __forceinline__ bool reset_next_g(const bool ar, const uint4* __restrict__ mrow,
                                                 const uint4* __restrict__ trow, uint32_t col_addr, uint32_t slot_addr) {
        const bool rs = pending & ar;
        if (rs) {
            e = rg.x & 0xFFu;
            tgt = (rg.x >> 8) & 0xFFu;
            pflags = rg.x >> 16;
            fr = ((uint64_t)rg.z << 32) | rg.y;
            w = 0;
            if constexpr (TB) {
                sq = col_addr - 128u;
                set_bks(col_addr);
                bias = 0;
            } else {
                len = 1;
            }
            step = -1;
            const uint32_t s = nres < lim ? (nres & (kRowSlots - 1u)) : kRowSlots;
            *(lds_v4*)(uintptr_t)(slot_addr + s * kRowSlotStride) = rt;
            nres += 1u;
            __asm__ volatile("" ::"v"(fr), "v"(e), "v"(tgt), "v"(pflags) : "memory");
            const uint32_t q = rg.w << 4;
            rg = ld_off(reinterpret_cast<const v4u*>(mrow), q);
            rt = ld_off(reinterpret_cast<const v4u*>(trow), q);
        }
        return rs;
    }
    // after each tile: lim = resets through the tile before last + kRowSlots (row_slots)
    __device__ __forceinline__ void tile_end() {
        lim = cA + kRowSlots;
        cA = nres;
    }

    // one env-step's move part (1131-1199) from the target's window position; rs: the step is an
    // autoreset step (reset_next).  Returns the hand-over word
    __device__ __forceinline__ uint32_t step_pos(const Params& p, uint32_t pos, bool rs) {
        const uint32_t P = p.pitch;
        step = __builtin_elementwise_add_sat(step, 1);                              // 1132
        const bool trunc0 = step >= p.max_steps;                                    // 1134
        const uint32_t fwd = __builtin_amdgcn_ubfe(w, pos, 1u);                     // 1137, 1167
        uint32_t pop = 0;
        if constexpr (TB) pop = pos == rp ? bias : 0u;                              // 1141-1166
        const uint32_t moved = fwd | pop;
        const int32_t d = (int32_t)pos - (int32_t)P;
        // free board: a forward move takes the target (bit e + P + d), a pop frees the point it
        // leaves (bit e + P); fwd * d as one full-rate v_mad_u32_u24 (only tog & 63 is used)
        uint32_t tog;
        asm("v_mad_u32_u24 %0, %1, %2, %3" : "=v"(tog) : "v"(fwd), "v"(d), "v"(e + P));
        fr ^= (uint64_t)moved << (tog & 63u);
        const int32_t dl = (int32_t)fwd - (int32_t)pop;
        if constexpr (TB) {
            const uint32_t arp = 2u * P - pos;         // back position of this move
            *lds_byte(sq + 128u) = (uint8_t)arp;       // slot len-1: the new top if fwd
            rp = fwd ? arp : (pop ? pnr : rp);
            sq += (uint32_t)dl << 6;
            bias = (sq + bks) >> 31;
        } else {
            len += fwd;
        }
        e = (uint32_t)((int32_t)e + __mul24((int32_t)moved, d));
        w = (uint32_t)(fr >> (e & 63u));
        // legal window bits; traceback: path[-2] (window bit rp) is legal although visited
        uint32_t lw = w & p.nbm;
        if constexpr (TB) lw |= bias << rp;
        const bool at_tgt = e == tgt;                                                // 1192
        const bool done = trunc0 | (lw == 0u) | at_tgt;                             // 1195-1199
        // an autoreset step is never done (w = 0 before it: lw was 0) and reports at-target
        pending = done & !rs;
        // the move before the last (slot len-3 after the step), for the next pop
        if constexpr (TB) pnr = *lds_byte(sq);
        return ((uint32_t)dl << 30) | ((at_tgt | rs) ? kHwTgt : 0u) | (pending ? kHwDone : 0u) | lw;
    }

    // ---- SoA <-> registers / LDS stack (launch start and end; the Env<1> state format)
    __device__ __forceinline__ void load(const Params& p, uint32_t i, uint8_t* col, uint32_t col_addr) {
        const State& s = p.st;
        const uint32_t P = p.pitch;
        const uint64_t vis = s.vis[i];
        const uint32_t ps = s.pos[i], ax = s.aux[i];
        const uint32_t pid = s.pid[i];
        e = (ps & 0xFFu) * P + ((ps >> 8) & 0xFFu);
        len = (ps >> 16) & 0xFFu;
        pending = ((ax >> 18) & 1u) != 0u;
        step = (int32_t)s.step[i];
        const uint4 r = p.tab.row1[pid];
        tgt = (r.x >> 8) & 0xFFu;
        pflags = r.x >> 16;
        fr = (p.tab.open[pid] & ~vis) << P;
        w = (uint32_t)(fr >> (e & 63u));
        if constexpr (TB) {
            const uint32_t moves = len >= 1 ? len - 1 : 0u;
            const uint64_t lo = s.dirs[i], hi = s.dirs[(size_t)p.n + i];
            for (uint32_t k = 0; k < moves; ++k) {
                const uint32_t a = (uint32_t)(((k < 32 ? lo : hi) >> ((k & 31u) * 2u)) & 3u);
                col[k * 64u] = (uint8_t)dir_pos1(a ^ 2u, P);
            }
            sq = col_addr + (len - 1u) * 64u - 128u;
            set_bks(col_addr);
            bias = (sq + bks) >> 31;
            rp = len >= 2 ? col[(len - 2u) * 64u] : 0u;
            pnr = *lds_byte(sq);
        }
    }

    // S, outcome, pid: the trie wave's final trie state (off << 16 | packed node), outcome_reward
    // and puzzle index
    __device__ __forceinline__ void store(const Params& p, uint32_t i, const uint8_t* col, uint32_t col_addr,
                                          uint32_t S, uint32_t outcome, uint32_t pid) {
        const State& s = p.st;
        const uint32_t P = p.pitch;
        const uint64_t open = p.tab.open[pid];
        const uint32_t sb = p.tab.row1[pid].x & 0xFFu;
        // visited = in the puzzle and not free, plus the start (always on the path)
        const uint64_t vis = ((~fr) >> P & open) | (1ull << sb);
        s.vis[i] = vis;
        if constexpr (TB) {
            len = (sq + 128u - col_addr) / 64u + 1u;
            uint64_t lo = 0, hi = 0;
            for (uint32_t k = 0; k + 1 < len; ++k) {
                const uint64_t v = (uint64_t)(pos_dir1(col[k * 64u], P) ^ 2u) << ((k & 31u) * 2u);
                lo |= k < 32 ? v : 0ull;
                hi |= k < 32 ? 0ull : v;
            }
            s.dirs[i] = lo;
            s.dirs[(size_t)p.n + i] = hi;
        }
        const uint32_t x = e / P, y = e - x * P;
        const uint32_t pend = pending ? 1u : 0u;
        s.pos[i] = x | (y << 8) | (len << 16) | ((S >> 16) << 24);
        s.aux[i] = (S & 0x7FFFu) | (outcome << 16) | (pend << 18) | (((S >> 15) & 1u) << 19);
        s.step[i] = (uint32_t)step;
        s.pid[i] = pid;
    }
};

}  // namespace sparc
