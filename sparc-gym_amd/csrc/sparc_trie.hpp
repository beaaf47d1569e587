// sparc_trie.hpp — the trie wave of the split rollout kernels (device code).
//
// The solution-prefix test of step() (_is_on_solution_path, SPaRC_Gym.py:1244-1265, and the
// np.array_equal test of 1206) walks a per-puzzle trie of the solution paths.  It needs from
// the move wave only what the move did, so in the split kernels a TRIE wave runs it one tile
// behind the move wave of the same 64 envs, from a hand-over word per env-step and the step's
// action (which the trie wave reads from the action tile itself).  The word tells whether the
// step was an autoreset step and done, and fwd - pop (+1 forward move, -1 traceback pop, 0 no
// move); step() decodes the multi-word kernel's layout (widen_hand_word, sparc_movew.hpp: flag
// byte term | trunc << 1 | legal << 2 | autoreset << 6 at bits 0-7, fwd - pop at 16-31), step1()
// the W = 1 move wave's (sparc_move1.hpp: autoreset iff bit 24 set and bit 25 clear, done at
// bit 25, fwd - pop at 30-31).
//
// Geometry-independent: the same lane serves the W = 1 and the multi-word kernels.
//
// Trie records are 8 bytes (trie8): four 16-bit fields, field d = the child in direction d,
// as a packed node (index | terminal << 15, 0xFFFF = none).  The PARENT sits in the field of
// the direction back to it: a node reached by move d_in can never have a child in direction
// d_in ^ 2 (that point is the previous one on the path, visited), and a traceback pop from the
// node moves exactly in direction d_in ^ 2.  So forward move and pop are the same lookup,
// field[action].
//
// Mixed tables (TrieLaneT<true>, k_rollout1s<…, C = true>: pools past the LDS row budget): a
// puzzle whose trie has at most 127 nodes gets COMPACT records, 4 bytes per node, four 8-bit
// fields (index | terminal << 7, 0xFF = none), and its lanes keep S = off << 8 | packed node; the
// others keep the 8-B records.  The format is a per-lane register set at each reset (fm, from the
// trie row), the transition the same with the field width, the perm selector, the key bound and
// the depth / terminal shifts in registers, one shift more per step (the action's field offset).
// Twice the nodes share an L2 line: the trie wave's record gathers are what misses the L2 on
// pools whose records outgrow an XCD's 4 MB.
//
// Lane state: S = off << 16 | packed node (off = depth off the trie, 0 = on it), and Oneg =
// the reward code a done step gets off a solution: -100, or 0 when the previous done step ended
// with outcome_reward == 1 (1211: a post-done step then gets 0).  Everything is integer
// arithmetic and single-compare selects: no SGPR mask chains, no branch but the reset and the
// gather.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "sparc_env.hpp"
#include "sparc_move1.hpp"

namespace sparc {

// per puzzle trie row: {root children right | up << 16, root children left | down << 16,
// trie base, root S | has solutions << 14 | trie max << 17}; root S = 0 or 0x8000 ([start]
// itself a solution) when some solution starts at start, else 0x10000 (off the trie from the
// start).  Rootless: children 0xFFFF.  Mixed tables (C): the base is a BYTE offset, and a compact
// puzzle's row holds {its root's 4-B record, ~0, base, root S (0, 0x80 or 0x100) | 1 << 13 | has
// solutions << 14 | trie max << 17}.
template <bool C = false>
struct TrieLaneT {
    typedef uint2 Rec;   // one 8-B load per gather (a compact record is its low half)
    // S layout: node index below bit nb, terminal at bit nb, depth off the trie from bit os; wide
    // records nb = 15, os = 16; compact (C, fm = 1) nb = 7, os = 8
    uint32_t fm = 0, sh8 = 0;   // C: 1 compact / 0 wide, and fm << 3
    // C: the record's bit offset in (ry:rx): a gather loads the 8-B aligned word holding the
    // record, so an odd compact record sits in its high half (32); 0 otherwise
    uint32_t hb = 0;
    __device__ __forceinline__ uint32_t NB() const { return C ? 15u - sh8 : 15u; }
    __device__ __forceinline__ uint32_t OS() const { return C ? 16u - sh8 : 16u; }
    __device__ __forceinline__ uint32_t kNode() const { return C ? 0x7FFFu >> sh8 : 0x7FFFu; }
    __device__ __forceinline__ uint32_t kKey() const { return C ? 0xFFFFu >> sh8 : 0xFFFFu; }
    // the row's format (C): bit 13 of its w
    __device__ __forceinline__ void set_format(uint32_t w) {
        if constexpr (C) {
            fm = __builtin_amdgcn_ubfe(w, 13u, 1u);
            sh8 = fm << 3;
        }
    }
    __device__ __forceinline__ uint32_t root_S(uint32_t w) const { return w & (0x18000u >> (C ? sh8 : 0u)); }
    typedef uint32_t v4u __attribute__((ext_vector_type(4)));
    typedef __attribute__((address_space(3))) v4u lds_v4;
    // row q of a row table (LDS or global) as one 4-vector, so that a read lands in one register tuple
    template <class Rows>
    __device__ __forceinline__ static v4u row4(const Rows& t, uint32_t q) {
        return *reinterpret_cast<const v4u*>(&t[q]);
    }
    uint32_t S = 0;
    int32_t Oneg = -100;
    uint32_t rx = ~0u, ry = ~0u;   // record of the current node (S & kNode(); compact: rx)
    uint32_t base = 0, tmax = 0;
    int32_t hs = 0, hsn = 0;        // the puzzle has solutions (the +-1 rewards apply, 1217); -hs
    uint32_t hsb = 0;               // hs << 2 (the class byte's bit 2, CODES = false)
    uint32_t pid = 0, npid = 0;
    v4u nx;                         // trie row of npid, read at the previous reset
    int acc_x = 0;                  // sum of reward codes
    uint32_t acc_y = 0, acc_z = 0;  // done steps, done steps on a solution

    __device__ __forceinline__ static uint32_t next_pid(uint32_t q, uint32_t num_puzzles) {
        return q + 1 == num_puzzles ? 0u : q + 1;   // reset() without options, SPaRC_Gym.py:1087
    }
    __device__ __forceinline__ void set_rec(const uint2 r) {
        rx = r.x;
        ry = r.y;
    }
    // byte offset of node k's record (C: base is a byte offset, the record 4 or 8 B)
    __device__ __forceinline__ uint32_t rec_off(uint32_t k) const {
        if constexpr (C) return base + (k << (3u - fm));
        return (base + k) << 3;
    }
    // the record of node k into (ry:rx) (C: the aligned 8-B word holding it, and hb)
    __device__ __forceinline__ void fetch(const Rec* __restrict__ trie8, uint32_t k) {
        const uint32_t o = rec_off(k);
        if constexpr (C) {
            set_rec(ld_off(trie8, o & ~7u));
            hb = (o & 4u) << 3;
        } else {
            set_rec(ld_off(trie8, o));
        }
    }
    // S in the SoA state's layout (off << 16 | terminal << 15 | node), for the launch-end hand-off
    __device__ __forceinline__ uint32_t std_S() const {
        if constexpr (!C) return S;
        return ((S >> OS()) << 16) | (((S >> NB()) & 1u) << 15) | (S & kNode());
    }

    // state at the start of a launch: the SoA record (pos: off in bits 24-31; aux: node,
    // outcome << 16 (1: +1), node_term << 19), the node's record and the next puzzle's row
    template <class Rows>
    __device__ __forceinline__ void load(const uint32_t ps, const uint32_t ax, const uint32_t q, const Rows& trow,
                                         const Rec* __restrict__ trie8, uint32_t num_puzzles) {
        pid = q;
        const uint4 r = trow[q];
        base = r.z;
        tmax = r.w >> 17;
        hs = (int32_t)((r.w >> 14) & 1u);
        hsn = -hs;
        hsb = (uint32_t)hs << 2;
        set_format(r.w);
        S = ((ps >> 24) << OS()) | (ax & 0x7FFFu) | (((ax >> 19) & 1u) << NB());
        Oneg = ((ax >> 16) & 3u) == 1u ? 0 : -100;
        if ((r.w & (1u << OS())) == 0u) {   // rootless puzzles keep off >= 1: the record is never read
            const uint32_t node = ax & 0x7FFFu;
            fetch(trie8, node < tmax ? node : tmax);
        }
        npid = next_pid(q, num_puzzles);
        nx = row4(trow, npid);
    }

    // ---- row slots (k_rollout1s on pools past the LDS row budget; sparc_move1.hpp row_slots):
    // the next reset's trie row comes from the slot the move wave wrote, read at the start of
    // each tile and after each reset (LDS reads, waited for with the step's other LDS reads), or
    // from the L2 when the slot rule failed for that reset
    uint32_t nres = 0, lim = 0, cA = 0, slot_addr = 0;
    uint4 nxs = {0u, 0u, 0u, 0u};
    __device__ __forceinline__ void slot_read(uint32_t slots, uint32_t stride) {
        const v4u v = *(const lds_v4*)(uintptr_t)(slot_addr + (nres & (slots - 1u)) * stride);
        nxs = make_uint4(v.x, v.y, v.z, v.w);
    }
    // after each tile (the same bookkeeping as MoveLane1::tile_end)
    __device__ __forceinline__ void slot_tile_end(uint32_t slots) {
        lim = cA + slots;
        cA = nres;
    }
    template <bool CODES, uint32_t SLOTS, uint32_t STRIDE, class Rows>
    __device__ __forceinline__ int step1s(const uint32_t hw, const uint32_t a16, const Rows& trow,
                                          const Rec* __restrict__ trie8, uint32_t num_puzzles) {
        const bool reset = hw_reset(hw);
        if (reset) {
            const bool fb = nres >= lim;
            pid = npid;
            npid = next_pid(npid, num_puzzles);
            apply_row(nxs);
            nres += 1u;
            if (fb) apply_row(ld_off(trow, pid << 4));   // the move wave wrote its spare slot: the L2 row
        }
        if (walk1(hw, a16)) gather(trie8);
        const int code = finish<CODES>(hw >= 0x40000000u, (hw & kHwDone) != 0u);
        // the next reset's slot, in case that reset falls in this tile (at least two steps later:
        // waited for with the LDS reads of a later step)
        if (reset) slot_read(SLOTS, STRIDE);
        return code;
    }
    __device__ __forceinline__ void apply_row(const uint4 r) {
        rx = r.x;
        ry = r.y;
        hb = 0;
        base = r.z;
        set_format(r.w);
        S = root_S(r.w);
        hs = (int32_t)((r.w >> 14) & 1u);
        hsn = -hs;
        hsb = (uint32_t)hs << 2;
        tmax = r.w >> 17;
    }

    // ---- look-ahead form (k_rollout1s on small grids).  The trie wave runs a tile behind the
    // move wave, so it knows the NEXT step's action too.  After each step it gathers, from trieg
    // (entry 4k + d = the record of node k's field-d node), the record the next step moves to IF
    // it moves along the trie: one unconditional 8-B gather per step whose data is used a whole
    // step later (the plain form's gather of the new node's own record is used half a step
    // later).  It pays only on small grids (MI355X, 2,000-step launches: c2 at 4,096 envs
    // 0.350 -> 0.337 ms; c3 at 65,536 envs 0.392 -> 0.410 ms), so the host uses it for grids of at
    // most 64 workgroups.  The c3 loss is not the L2 load of 65,536 lanes gathering every step: an
    // exec-masked variant that gathers for on-trie lanes only costs the same 6-7 %
    // (profiles/r05/ab_c3_la/); it is this form's per-step row read, selects and address on a
    // SIMD the trie wave shares with the move wave, whose chain is the other half of the step.
    uint32_t nrx = ~0u, nry = ~0u;  // record of field[a] of the current node (a = this step's action)

    // the class byte of a step (CODES = false): min(S >> 15, 2) (0 on the trie, 1 on a solution,
    // 2 off it) | hs << 2.  With next-step autoreset the reward code is a function of this byte and
    // the step's hand-over word alone (a done step never follows a done step, so Oneg is -100 at
    // every done step), and the I/O wave computes it (io_codes4, k_rollout1s)
    __device__ __forceinline__ uint32_t class_byte(uint32_t x) const { return (x < 2u ? x : 2u) | hsb; }
    // Oneg after the launch's last step (CODES = false): 0 iff that step was done on a solution
    __device__ __forceinline__ void finish_oneg(uint32_t last_hw_done) {
        Oneg = (last_hw_done != 0u && (S >> NB()) == 1u) ? 0 : -100;
    }

    // after load(): the first step's look-ahead record (a016: its action << 4)
    __device__ __forceinline__ void prime(const uint32_t a016, const uint2* __restrict__ trieg) {
        const uint32_t node = S & 0x7FFFu;
        const uint2 rec = trieg[((base + (node < tmax ? node : tmax)) << 2) + __builtin_amdgcn_ubfe(a016, 4u, 2u)];
        nrx = rec.x;
        nry = rec.y;
    }

    // step1 (the W = 1 move wave's word, a16 = action << 4) with the look-ahead record; an16: the
    // next step's action << 4
    template <bool CODES = true, class Rows>
    __device__ __forceinline__ int step1la(const uint32_t hw, const uint32_t a16, const uint32_t an16, const Rows& trow,
                                           const uint2* __restrict__ trieg, uint32_t num_puzzles) {
        if (hw_reset(hw)) {
            pid = npid;
            npid = next_pid(npid, num_puzzles);
            rx = nx.x;
            ry = nx.y;
            base = nx.z;
            S = nx.w & 0x18000u;
            hs = (int32_t)((nx.w >> 14) & 1u);
            hsn = -hs;
            hsb = (uint32_t)hs << 2;
            tmax = nx.w >> 17;
        }
        nx = row4(trow, npid);
        const bool take = walk1(hw, a16);
        // the new node's record arrived with the previous step's look-ahead gather (a reset
        // step never takes: it does not move)
        rx = take ? nrx : rx;
        ry = take ? nry : ry;
        // the next step's: field[an] of the node now current (on or off the trie, the node is
        // one of this puzzle's: in bounds; used only if that step takes).  Unconditional: an
        // exec-masked gather for on-trie lanes only measured slower here (c2: 0.346 vs 0.337 ms;
        // round 5: 0.2863 vs 0.3215 ms, profiles/r05/ab_handover)
        const uint2 rec = trieg[((base + (S & 0x7FFFu)) << 2) + __builtin_amdgcn_ubfe(an16, 4u, 2u)];
        nrx = rec.x;
        nry = rec.y;
        return finish<CODES>(hw >= 0x40000000u, (hw & kHwDone) != 0u);
    }

    // one env-step from its hand-over word (layout above) and action; returns the reward code
    // (x100, 1201-1223)
    template <bool CODES = true, class Rows>
    __device__ __forceinline__ int step(const uint32_t hw, const uint32_t a, const Rows& trow,
                                        const uint2* __restrict__ trie8, uint32_t num_puzzles) {
        return step_core<CODES>((hw & 0x40u) != 0u, hw & 0xFFFF0000u, hw >= 0x10000u, (hw & 3u) != 0u, a, trow, trie8,
                         num_puzzles);
    }
    // the same from the W = 1 split move wave's word (sparc_move1.hpp: reset iff at-target set and
    // done clear, done at bit 25, fwd - pop at bits 30-31) and a16 = the action << 4 (the I/O wave
    // stores the trie wave's actions that way, k_rollout1s)
    template <bool CODES = true, class Rows>
    __device__ __forceinline__ int step1(const uint32_t hw, const uint32_t a16, const Rows& trow,
                                         const Rec* __restrict__ trie8, uint32_t num_puzzles) {
        if (hw_reset(hw)) reset_from_nx<CODES>(trow, num_puzzles);
        if (walk1(hw, a16)) gather(trie8);
        return finish<CODES>(hw >= 0x40000000u, (hw & kHwDone) != 0u);
    }

    // reset: an autoreset step; dd = (fwd - pop) << 16 (bit 16: moved); moved = dd != 0; done:
    // terminated or truncated.  CODES = false: the step returns the class byte instead of the
    // reward code and keeps no counters (the I/O wave derives both, k_rollout1s<…, IOR>)
    template <bool CODES = true, class Rows>
    __device__ __forceinline__ int step_core(const bool reset, const uint32_t dd, const bool moved, const bool done,
                                             const uint32_t a, const Rows& trow, const uint2* __restrict__ trie8,
                                             uint32_t num_puzzles) {
        if (reset) reset_from_nx<CODES>(trow, num_puzzles);
        // forward move or pop on the trie: field[action] (a child, or the parent).  key has
        // bits above 15 set when the lane is off the trie or did not move, so one compare
        // decides; off the trie (or without a child) the move counts the depth instead.
        const uint64_t xy = ((uint64_t)ry << 32) | rx;
        const uint32_t c = (uint32_t)(xy >> ((a << 4) & 0x30u));
        const uint32_t key = __builtin_amdgcn_ubfe(c, 0u, 16u) | (S & 0xFFFF0000u) | (~dd & 0x10000u);
        const bool take = key < 0xFFFFu;
        S = take ? key : S + dd;
        if (take) gather(trie8);
        return finish<CODES>(moved, done);
    }

    // the W = 1 transition (step_core's, from the hand-over word itself): not moved is bit 30 of
    // the word clear (fwd - pop = 0), which keeps key above 0xFFFF as bit 16 does there, and the
    // depth step is (fwd - pop) << 16 from one arithmetic shift: field / key / depth in 8
    // instructions against 11 (the extraction of dd and of the not-moved bit)
    //   C, compact lanes (fm = 1): the field is byte a16 / 16 of the 4-B record (the shift halved),
    //   the perm selector takes one byte of it, the key bound is 0xFF and the depth sits at bit 8
    __device__ __forceinline__ bool walk1(const uint32_t hw, const uint32_t a16) {
        const uint64_t xy = ((uint64_t)ry << 32) | rx;
        const uint32_t c = (uint32_t)(xy >> ((C ? (a16 >> fm) | hb : a16) & 63u));   // a16 & 15 == 0: field a16 / 16
        // field | S's depth half: one v_perm_b32 (the compiler's and / and / or3 took three)
        const uint32_t key = __builtin_amdgcn_perm(S, c, C ? 0x07060100u + (fm << 10) : 0x07060100u) |
                             (~hw & 0x40000000u);
        const bool take = key < kKey();
        // fwd - pop by a signed field extract, shifted and added in one v_lshl_add_u32 (written
        // plainly, the compiler rewrote (hw >> 30) << 16 into a shift, a mask and an add)
        const int32_t dl = __builtin_amdgcn_sbfe((int32_t)hw, 30u, 2u);
        uint32_t Sm;
        if constexpr (C) asm("v_lshl_add_u32 %0, %1, %2, %3" : "=v"(Sm) : "v"(dl), "v"(OS()), "v"(S));
        else asm("v_lshl_add_u32 %0, %1, 16, %2" : "=v"(Sm) : "v"(dl), "v"(S));
        S = take ? key : Sm;
        return take;
    }
    // the record changes only with the node (exec-masked gather; a random walk is off the trie on
    // most steps).  Every field of a record holds a node of the same puzzle (validated by
    // sparc_load_puzzles), so no clamp here; load() clamps the stored node.
    __device__ __forceinline__ void gather(const Rec* __restrict__ trie8) { fetch(trie8, S & kNode()); }
    // autoreset step: the next puzzle's rows and its trie root
    template <bool CODES, class Rows>
    __device__ __forceinline__ void reset_from_nx(const Rows& trow, uint32_t num_puzzles) {
        pid = npid;
        npid = next_pid(npid, num_puzzles);
        rx = nx.x;
        ry = nx.y;
        hb = 0;
        base = nx.z;
        set_format(nx.w);
        S = root_S(nx.w);
        hs = (int32_t)((nx.w >> 14) & 1u);
        hsn = -hs;
        hsb = (uint32_t)hs << 2;
        tmax = nx.w >> 17;
        // the row of the next reset, read here into the same registers, so nothing waits for it
        // until that reset (at least two steps later).  MI355X, c3: 0.4003-0.4014 -> 0.3950-0.3962
        // ms per 2,000-step launch against the read on every step (profiles/r04/ab_run2).  The
        // empty asm takes the values made from the old row as operands, so they exist before the
        // read is issued, and nx is one 4-vector: with only a memory clobber the compiler landed
        // the read in temporaries and waited for it in the branch to copy it into nx (as
        // MoveLane1::reset_next; round 5: c3 -4.3 % with the hand-over word below, c2 -6.8 %)
        if constexpr (CODES) __asm__ volatile("" ::"v"(rx), "v"(ry), "v"(base), "v"(S), "v"(hs), "v"(hsn) : "memory");
        else __asm__ volatile("" ::"v"(rx), "v"(ry), "v"(base), "v"(S), "v"(hsb) : "memory");
        nx = row4(trow, npid);
    }
    // reward code: done: +100 on a solution, else Oneg; otherwise +-1 when moved on a puzzle with
    // solutions (on / off the trie), else 0 (an autoreset step neither moves nor is done)
    template <bool CODES>
    __device__ __forceinline__ int finish(const bool moved, const bool done) {
        const uint32_t x = S >> NB();                          // 0 on, 1 on a solution, >= 2 off
        if constexpr (!CODES) return (int)class_byte(x);
        const int cd = x == 1u ? 100 : Oneg;
        const int cm = moved ? (x < 2u ? hs : hsn) : 0;
        const int code = done ? cd : cm;
        Oneg = done ? (cd < 0 ? cd : 0) : -100;
        acc_x += code;
        acc_y += (uint32_t)done;
        acc_z += (uint32_t)(code == 100);
        return code;
    }
};
using TrieLane = TrieLaneT<false>;

}  // namespace sparc
