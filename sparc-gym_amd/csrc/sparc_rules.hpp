// sparc_rules.hpp — per-lane rule audit for gfx950 (device code).
//
// Restates SPaRC_Gym._validate_rules (SPaRC_Gym.py:941-950) for one env per lane, on the
// same bitboards as the step (bit x*pitch + y, W words):
//   _compute_regions (423-454)  regions = connected components of {cell centres} ∪ {free
//                               lattice points}, free = in lattice, not a gap, not on the
//                               path.  Found by bitboard flood fill from the lowest unassigned
//                               cell (the reference's x-major scan order gives the region ids).
//   _collect_region_symbols     per-cell multiplicity (symbol layers set at the cell) and colour
//   (456-481)                   as bit-planes: counts are popcounts of region ∧ plane.
//   reached_target (487-495)    agent == target
//   path_not_crossing (497-505) always true: a move only enters an unvisited point and a pop
//                               removes the last one, so the path never repeats a point
//   no_gap_violations (507-517) visited ∧ gaps == ∅ (the path's point set is `visited`)
//   all_dots_collected (519-531) dots ∧ ¬visited == ∅
//   square_color_separation     per region: at most one non-zero square colour
//   (533-551)
//   star_pairing_exact (553-619) per region: no colourless star; for each star colour c the
//                               region holds exactly 2 symbol occurrences of colour c
//   triangles_edge_count        per triangle cell with count > 0: path points among its 4
//   (622-646)                   neighbours == count, as a bit-sliced 4-input popcount
//   poly_ylop_area (648-709)    per region holding instances: area == Σpoly − Σylop, then the
//                               exact-fit search of 736-838 (exists / not: the same answer for
//                               any complete search order, so identical ylops are placed in
//                               non-decreasing anchor order and polys by distinct shape)
// Output bit k = RULE k in the order of _run_rule_validators (899-939), bit 8 = all.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "sparc_env.hpp"

namespace sparc {

constexpr uint32_t kErrRuleTable = 8, kErrJoin = 16;   // Params::err bits (sparc_sync)
// rule-plane indices of include/sparc_gym_amd.h (SPARC_RULE_PLANES), then the planes the loader
// (sparc_load_rules) derives from the instance list for the device copy: the net instance area
// of each cell (Σ poly areas − Σ ylop areas of the instances there, 8-bit two's complement,
// bit-sliced), so a region's area check (_polyfit_check_area 700-709) is 8 popcounts instead of
// a walk over the puzzle's instance list with two dependent loads per instance.  RP_INST of the
// device copy is rewritten from the list too (cells holding an instance).
enum : uint32_t {
    RP_CELLS = 0, RP_LATTICE, RP_GAPS, RP_DOTS, RP_TRI, RP_TRI0, RP_TRI1, RP_TRI2, RP_STAR, RP_SQUARE,
    RP_COLORED, RP_COL1, RP_M0 = RP_COL1 + 8, RP_M1, RP_M2, RP_NOTFIRST, RP_NOTLAST, RP_INST, RP_ABI,
    RP_AREA0 = RP_ABI, RP_COUNT = RP_AREA0 + 8
};
constexpr int kAreaPlanes = 8;
constexpr int kFitCells = 64;     // cell grid of the exact fit (15 x 15 lattice: 7 x 7 = 49)
// The GPU's search keeps its per-region lists in registers / scratch of these sizes; a puzzle with
// more ylops or distinct poly shapes (instances sit at cell centres, one per cell, so never more
// than 64 of either) is flagged by the loader (kHostFit) and its searches run on the host
// (exact_fit<..., kHostFitMax, kHostFitMax, kHostFitPlanes>, sparc_kernels.hip host_fit)
constexpr int kFitYlops = 16;
constexpr int kFitShapes = 16;
constexpr int kFitDepth = 64;
constexpr int kHostFitMax = 64, kHostFitPlanes = 8;   // every valid puzzle: <= 64 cells, counts >= -65
constexpr uint32_t kHostFit = 0x80000000u;            // instance count flag: searches on the host
// default node cap of one exact-fit search on the GPU (sparc_set_fit_cap): a search that passes it
// stops, and the host finishes it without a cap (FitQueue below, the C ABI's fallback), so
// callers see the reference's unbounded answer
constexpr uint32_t kFitCap = 1u << 26;

// Exact-fit searches that passed the GPU's node cap, handed to the host (sparc_rules_finish runs
// exact_fit on them without a cap and patches the outputs): the output index of the audit (pos:
// env, or t * N + env in a rollout), the region's cell mask, the puzzle and the region id.
struct FitTodo {
    uint64_t pos;
    uint64_t rm;
    uint32_t q, rid;
};
struct FitQueue {
    unsigned long long* count;   // entries pushed (may pass cap: the host grows the queue and re-runs)
    FitTodo* items;
    uint64_t cap;
};
__device__ __forceinline__ void fit_queue_push(const FitQueue& fq, uint64_t pos, uint64_t rm, uint32_t q, uint32_t rid) {
    const unsigned long long k = atomicAdd(fq.count, 1ull);   // 64-bit: no wrap however many are queued
    if (k < fq.cap) fq.items[k] = FitTodo{pos, rm, q, rid};
}

// Exact-fit answers the host has finished (sparc_rules_finish: searches past the node cap, and
// every search of a kHostFit puzzle), kept on the device so that an audit looks them up instead of
// queueing the same (puzzle, region cells) search again at every later step.  Open addressing over
// (q, rm), linear probing, load factor <= 1/2 (so a probe always ends at an empty slot); entry
// {rm low, rm high, q, answer | valid << 1}.  used == 0: empty (no probe at all).
struct HostFits {
    const uint4* tab;
    uint32_t mask;   // slots - 1 (a power of two)
    uint32_t used;
};
__host__ __device__ __forceinline__ uint32_t hostfit_slot(uint32_t q, uint64_t rm, uint32_t mask) {
    uint64_t h = rm * 0x9E3779B97F4A7C15ull ^ ((uint64_t)q * 0xC2B2AE3D27D4EB4Full);
    h ^= h >> 29;
    return (uint32_t)h & mask;
}
// 1 / 0: the host's answer, -1: not finished on the host
__device__ __forceinline__ int hostfit_find(const HostFits& hf, uint32_t q, uint64_t rm) {
    if (hf.used == 0) return -1;
    for (uint32_t s = hostfit_slot(q, rm, hf.mask);; s = (s + 1u) & hf.mask) {
        const uint4 e = hf.tab[s];
        if (!(e.w & 2u)) return -1;
        if (e.x == (uint32_t)rm && e.y == (uint32_t)(rm >> 32) && e.z == q) return (int)(e.w & 1u);
    }
}

struct RulesTab {
    const uint64_t* __restrict__ planes;      // [P][RP_COUNT][W]
    const uint2* __restrict__ inst_fc;        // [P] {first, count | kHostFit} into inst
    const uint32_t* __restrict__ inst;        // bit | ylop << 10 | shape << 11
    const uint2* __restrict__ shape_range;    // [S] {first offset, count} into shape_off
    const int32_t* __restrict__ shape_area;   // [S] sum of the shape array (the area of 722-723)
    const int8_t* __restrict__ shape_off;     // [offsets][2] (dcx, dcy) in cell units
    uint32_t num_puzzles;
    uint32_t area;   // 1: the RP_AREA planes hold every cell's net area (else the list is walked)
    uint32_t fit_cap;   // search nodes of one exact fit before it is handed to the host
    // the per-region check codes (region_code) of every region cell mask of each puzzle with at
    // most kRegTabCells cells, computed once by sparc_load_rules: reg_off[q] = the puzzle's first
    // entry (a multiple of 8) or kNoRegTab; entries of 4 bits, 8 per word of reg_tab.  May be
    // null (no table).
    const uint32_t* __restrict__ reg_off;
    const uint32_t* __restrict__ reg_tab;
    FitQueue fq;   // count null: no queue (region-table builds: the host scans the table instead)
    HostFits hf;   // answers the host finished for earlier audits (looked up before a GPU search)
    // [P][rule_row_u64<W>()]: what an audit reads when its env changes puzzle, in one contiguous
    // record (puzzle_rules): the kBasePlanes planes, then reg_off | inst first << 32, then the
    // puzzle's info words x | y << 32 with y's bits 24-31 = instance count | host-fit flag << 7
    // (W = 1: 96 B; the planes alone are spread over 264 B of the plane table)
    const uint64_t* __restrict__ rows;
};
template <int W>
__host__ __device__ constexpr uint32_t rule_row_u64() { return 10u * W + 2u; }
constexpr uint32_t kNoRegTab = 0xFFFFFFFFu;
constexpr uint32_t kRegTabCells = 12;

template <int W>
struct BB {
    uint64_t w[W];
    // (host and device: the host finishes exact-fit searches that pass the GPU's node cap)
    __host__ __device__ __forceinline__ static BB zero() { BB r; for (int k = 0; k < W; ++k) r.w[k] = 0; return r; }
    __host__ __device__ __forceinline__ static BB load(const uint64_t* p) { BB r; for (int k = 0; k < W; ++k) r.w[k] = p[k]; return r; }
    __host__ __device__ __forceinline__ BB operator&(const BB& o) const { BB r; for (int k = 0; k < W; ++k) r.w[k] = w[k] & o.w[k]; return r; }
    __host__ __device__ __forceinline__ BB operator|(const BB& o) const { BB r; for (int k = 0; k < W; ++k) r.w[k] = w[k] | o.w[k]; return r; }
    __host__ __device__ __forceinline__ BB operator^(const BB& o) const { BB r; for (int k = 0; k < W; ++k) r.w[k] = w[k] ^ o.w[k]; return r; }
    __host__ __device__ __forceinline__ BB andnot(const BB& o) const { BB r; for (int k = 0; k < W; ++k) r.w[k] = w[k] & ~o.w[k]; return r; }
    __host__ __device__ __forceinline__ bool any() const { uint64_t a = 0; for (int k = 0; k < W; ++k) a |= w[k]; return a != 0; }
    __host__ __device__ __forceinline__ bool operator==(const BB& o) const {
        uint64_t a = 0; for (int k = 0; k < W; ++k) a |= w[k] ^ o.w[k]; return a == 0;
    }
    __host__ __device__ __forceinline__ int popc() const { int s = 0; for (int k = 0; k < W; ++k) s += __builtin_popcountll(w[k]); return s; }
    __host__ __device__ __forceinline__ bool test(uint32_t b) const { return (w[b >> 6] >> (b & 63)) & 1ull; }
    __host__ __device__ __forceinline__ void set(uint32_t b) { w[b >> 6] |= 1ull << (b & 63); }
    // lowest set bit index (requires any())
    __host__ __device__ __forceinline__ uint32_t lowest() const {
        for (int k = 0; k < W; ++k)
            if (w[k]) return 64u * k + (uint32_t)__builtin_ctzll(w[k]);
        return 0;
    }
    // toward higher bit indices by s (0 < s < 64)
    __host__ __device__ __forceinline__ BB shl(uint32_t s) const {
        BB r;
        for (int k = W - 1; k >= 0; --k) r.w[k] = (w[k] << s) | (k ? w[k - 1] >> (64 - s) : 0);
        return r;
    }
    __host__ __device__ __forceinline__ BB shr(uint32_t s) const {
        BB r;
        for (int k = 0; k < W; ++k) r.w[k] = (w[k] >> s) | (k + 1 < W ? w[k + 1] << (64 - s) : 0);
        return r;
    }
};

// the puzzle's instance list and shapes for the exact fit, by value (the search is a call: a
// pointer to a kernel-argument table, or a reference to a region board, would put them in
// scratch memory on every region)
struct FitIn {
    const uint32_t* inst;
    const uint2* shape_range;
    const int8_t* shape_off;
    uint32_t first, count;   // the puzzle's instance range
    uint32_t CX, CY;         // cell grid
    uint32_t cap;            // search nodes before the search is handed to the host (0: kHostFit)
};
// cf = count | kHostFit: a flagged puzzle's searches are never run on the GPU (cap 0)
__host__ __device__ __forceinline__ FitIn fit_in(const RulesTab& rt, uint32_t first, uint32_t cf, uint32_t X,
                                                 uint32_t Y) {
    return FitIn{rt.inst, rt.shape_range, rt.shape_off, first, cf & ~kHostFit, (X - 1) / 2, (Y - 1) / 2,
                 (cf & kHostFit) ? 0u : rt.fit_cap};
}

// ---------------------------------------------------------------- exact fit (736-838)
// The search runs on the cell grid (CX x CY <= 7 x 7 cells, bit cx*CY + cy of a u64: the
// reference's row-major order, so "the first negative cell" is the lowest set bit).  Cell
// counts are two's-complement bit-sliced counters (kFitPlanes planes, -32..31 >= -(1 + 16
// ylops); the host's kHostFitPlanes: -128..127); placing a shape adds or subtracts its cell mask with a ripple over the planes.  A
// shape is its cell pattern relative to its anchor (the shape's first cell in row-major order,
// _get_offsets 840-855) plus the set of anchors at which it fits the grid (_try_place_polys
// 858-871).
constexpr int kFitPlanes = 6;
template <int NP = kFitPlanes>
struct FitGrid {
    uint64_t p[NP];
    __host__ __device__ __forceinline__ void add(uint64_t m) {
#pragma unroll
        for (int i = 0; i < NP; ++i) { const uint64_t t = p[i] & m; p[i] ^= m; m = t; }
    }
    __host__ __device__ __forceinline__ void sub(uint64_t m) {
#pragma unroll
        for (int i = 0; i < NP; ++i) { const uint64_t t = ~p[i] & m; p[i] ^= m; m = t; }
    }
    __host__ __device__ __forceinline__ uint64_t neg() const { return p[NP - 1]; }
    __host__ __device__ __forceinline__ uint64_t nonzero() const {
        uint64_t a = 0;
#pragma unroll
        for (int i = 0; i < NP; ++i) a |= p[i];
        return a;
    }
};

// pattern (relative to the anchor) and fitting anchors of shape `sh` on a CX x CY cell grid
__host__ __device__ __forceinline__ void fit_shape(const FitIn& rt, uint32_t sh, uint32_t CX, uint32_t CY, uint64_t& pat,
                                          uint64_t& va) {
    const uint2 sr = rt.shape_range[sh];
    const uint32_t o0 = sr.x, n = sr.y;
    int mdx = 0, mdy0 = 0, mdy1 = 0;
    pat = 0;
    bool ok = true;
    for (uint32_t k = 0; k < n; ++k) {
        const int dx = rt.shape_off[2 * (o0 + k)], dy = rt.shape_off[2 * (o0 + k) + 1];
        mdx = dx > mdx ? dx : mdx;
        mdy0 = dy < mdy0 ? dy : mdy0;
        mdy1 = dy > mdy1 ? dy : mdy1;
        const int lin = dx * (int)CY + dy;
        if (lin < 0 || lin > 63) ok = false;
        else pat |= 1ull << lin;
    }
    va = 0;
    if (!ok) return;   // wider than the grid: it fits nowhere
    for (int ax = 0; ax + mdx < (int)CX; ++ax)
        for (int ay = -mdy0; ay + mdy1 < (int)CY; ++ay) va |= 1ull << (ax * (int)CY + ay);
}

// the region's cells on the exact fit's cell grid (bit cx * CY + cy): per cell row, the 32 board
// bits from the row's first cell centre, the cell centres (every other bit, CY <= 7) kept and
// compressed with three shift-or-mask steps
template <int W>
__device__ __forceinline__ uint32_t bits32_at(const BB<W>& b, uint32_t pos) {
    const uint32_t k = pos >> 6, r = pos & 63u;
    uint64_t lo = 0, hi = 0;
#pragma unroll
    for (int j = 0; j < W; ++j) {
        lo = (uint32_t)j == k ? b.w[j] : lo;
        hi = (uint32_t)j == k + 1 ? b.w[j] : hi;
    }
    return (uint32_t)((lo >> r) | (r ? hi << (64 - r) : 0ull));
}
template <int W>
__device__ __forceinline__ uint64_t cell_mask(const FitIn& in, const BB<W>& Rc, uint32_t pitch) {
    const uint32_t alt = 0x1555u & ((1u << (2 * in.CY - 1)) - 1u);   // cell centres of one row
    uint64_t rm = 0;
    for (uint32_t cx = 0; cx < in.CX; ++cx) {
        uint32_t v = bits32_at<W>(Rc, (2 * cx + 1) * pitch + 1) & alt;
        v = (v | (v >> 1)) & 0x3333u;
        v = (v | (v >> 2)) & 0x0F0Fu;
        v = (v | (v >> 4)) & 0x00FFu;
        rm |= (uint64_t)v << (cx * in.CY);
    }
    return rm;
}

// cell_mask of a one-word board of pitch 8 (every pool up to 7 x 7): lattice row x is byte x,
// so the cell rows (bytes 1, 3, 5) come together in one v_perm_b32 and their centres (bits 1, 3,
// 5 of each byte, CY <= 3) compress in all three bytes at once
__device__ __forceinline__ uint64_t cell_mask_p8(const FitIn& in, uint64_t rc) {
    uint32_t w = __builtin_amdgcn_perm((uint32_t)(rc >> 32), (uint32_t)rc, 0x0C050301u);
    w = (w >> 1) & 0x151515u;
    w = (w | (w >> 1)) & 0x131313u;
    w = (w | (w >> 2)) & 0x070707u;
    return (w & 7u) | (((w >> 8) & 7u) << in.CY) | (((w >> 16) & 7u) << (2 * in.CY));
}

// _polyfit_region_exact with the area check passed (so net = area > 0 and the grid starts at
// -1 on the region's cells), as a depth-first search over the same choices (existence only:
// identical ylops take non-decreasing anchors, polys are tried by distinct shape).  Returns 1 (fits),
// 0 (does not fit) or -1: the search passed `cap` nodes without an answer (on the GPU the audit
// then queues the region for the host, which runs this same function without a cap: the
// reference's search is unbounded).  rm: the region's cells (cell_mask).
//   NY, ND, PLANES: list sizes and counter planes (the GPU's; the host runs the puzzles the
// loader flagged kHostFit with kHostFitMax / kHostFitPlanes).  cap == 0: -1 at once (a flagged
// puzzle on the GPU).
template <int W, class I = uint32_t, int NY = kFitYlops, int ND = kFitShapes, int PLANES = kFitPlanes>
__host__ __device__ __noinline__ int exact_fit(const FitIn in, const BB<W> Rc, uint64_t rm, I cap) {
    if (cap == 0) return -1;
    const FitIn& rt = in;
    const uint32_t CX = in.CX, CY = in.CY;
    FitGrid<PLANES> g;
#pragma unroll
    for (int i = 0; i < PLANES; ++i) g.p[i] = rm;    // -1 on the region
    uint32_t ysh[NY], dsh[ND];
    int cnt[ND];
    int ny = 0, nd = 0, np = 0;
    for (uint32_t k = 0; k < in.count; ++k) {
        const uint32_t e = rt.inst[in.first + k];
        if (!Rc.test(e & 0x3FFu)) continue;
        const uint32_t sh = e >> 11;
        if ((e >> 10) & 1u) {                 // ylop, kept sorted by shape (insertion sort)
            int j = ny++;
            while (j > 0 && ysh[j - 1] > sh) { ysh[j] = ysh[j - 1]; --j; }
            ysh[j] = sh;
        } else {
            int j = 0;
            while (j < nd && dsh[j] != sh) ++j;
            if (j == nd) { dsh[nd] = sh; cnt[nd] = 0; ++nd; }
            ++cnt[j];
            ++np;
        }
    }
    uint64_t ypat[NY], yva[NY], dpat[ND], dva[ND];
    for (int k = 0; k < ny; ++k) fit_shape(rt, ysh[k], CX, CY, ypat[k], yva[k]);
    for (int k = 0; k < nd; ++k) fit_shape(rt, dsh[k], CX, CY, dpat[k], dva[k]);
    int cur[NY + kFitDepth + 1];
    int pat[kFitDepth + 1];
    const int LMAX = ny + np;
    int L = 0;
    cur[0] = -1;
    I iters = 0;
    while (true) {
        if (++iters > cap) return -1;
        if (L < ny) {                                            // _polyfit_place_ylops
            int a = cur[L];
            if (a >= 0) g.add(ypat[L] << a);
            a = a < 0 ? ((L > 0 && ysh[L] == ysh[L - 1]) ? cur[L - 1] : 0) : a + 1;
            const uint64_t cand = a < 64 ? yva[L] & (~0ull << a) : 0ull;
            if (!cand) {
                cur[L] = -1;
                if (L == 0) return 0;
                --L;
                continue;
            }
            a = __builtin_ctzll(cand);
            g.sub(ypat[L] << a);
            cur[L] = a;
            cur[++L] = -1;
            continue;
        }
        const int lv = L - ny;                                   // _polyfit_place_polys
        int j = cur[L];
        if (j < 0) {
            const uint64_t ng = g.neg();
            const bool pos = (g.nonzero() & ~ng) != 0;
            bool done = false, ok = false;
            if (pos) done = true;                                // any(grid > 0): False
            else if (L == LMAX) { done = true; ok = ng == 0; }    // no polys left
            else if (ng == 0) { done = true; ok = true; }        // no negative cell: True
            if (done) {
                if (ok) return 1;
                if (L == 0) return 0;
                --L;
                continue;
            }
            pat[lv] = __builtin_ctzll(ng);                       // the first negative cell
        } else {
            g.sub(dpat[j] << pat[lv]);
            ++cnt[j];
        }
        ++j;
        while (j < nd && (cnt[j] == 0 || !((dva[j] >> pat[lv]) & 1ull))) ++j;
        if (j >= nd) {
            cur[L] = -1;
            if (L == 0) return 0;
            --L;
            continue;
        }
        g.add(dpat[j] << pat[lv]);
        --cnt[j];
        cur[L] = j;
        cur[++L] = -1;
    }
}

// Per-lane memo of exact-fit answers for the audit after every step of a rollout: the answer
// depends only on the puzzle and the region's cells, and one step moves the path by one point,
// so most regions (and their fit answers) carry over from the previous steps.  K entries of
// (cell mask, answer) for one puzzle, replaced round robin; a miss runs the search.
// All-zero bytes are an empty memo (HBM copies are zeroed): a zero key matches no region.
template <int K>
struct FitMemo {
    uint64_t key[K];
    uint32_t res, pid, next, pad;
    __device__ __forceinline__ FitMemo() : res(0), pid(0), next(0), pad(0) {
#pragma unroll
        for (int k = 0; k < K; ++k) key[k] = 0;   // a region holds cells: its mask is never 0
    }
    // 1 / 0: the memoised answer, -1: not known
    __device__ __forceinline__ int find(uint32_t q, uint64_t rm) const {
        int r = -1;
#pragma unroll
        for (int k = 0; k < K; ++k) r = (q == pid && key[k] == rm) ? (int)((res >> k) & 1u) : r;
        return r;
    }
    __device__ __forceinline__ void put(uint32_t q, uint64_t rm, int fits) {
        if (q != pid) {
            pid = q;
#pragma unroll
            for (int k = 0; k < K; ++k) key[k] = 0;
            next = 0;
        }
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const bool here = next == (uint32_t)k;
            key[k] = here ? rm : key[k];
            res = here ? ((res & ~(1u << k)) | ((uint32_t)fits << k)) : res;
        }
        next = next + 1 == (uint32_t)K ? 0u : next + 1;
    }
};
struct NoMemo {};
constexpr int kMemo = 4;   // memo entries per env

// Σ over the region's instances of (poly area − ylop area), and whether it holds any
// (_polyfit_check_area 700-709 on the instances of 687-697).  Rc: the region's cell centres.
template <int W>
__device__ __forceinline__ bool region_net_area(const RulesTab& rt, const FitIn& fin, uint32_t q, const BB<W>& Rc,
                                                const BB<W>& inst_plane, int& net) {
    net = 0;
    if (!(Rc & inst_plane).any()) return false;               // regions without instances skip this
    if (rt.area) {                                             // the bit-sliced planes: 8 popcounts
        const uint64_t* ga = rt.planes + ((size_t)q * RP_COUNT + RP_AREA0) * W;
        BB<W> ap[kAreaPlanes];
#pragma unroll
        for (int k = 0; k < kAreaPlanes; ++k) ap[k] = BB<W>::load(ga + k * W);
#pragma unroll
        for (int k = 0; k < kAreaPlanes - 1; ++k) net += (Rc & ap[k]).popc() << k;
        net -= (Rc & ap[kAreaPlanes - 1]).popc() << (kAreaPlanes - 1);
        return true;
    }
    bool has = false;
    for (uint32_t k = 0; k < fin.count; ++k) {
        const uint32_t e = rt.inst[fin.first + k];
        if (!Rc.test(e & 0x3FFu)) continue;
        has = true;
        const int a = rt.shape_area[e >> 11];
        net += ((e >> 10) & 1u) ? -a : a;
    }
    return has;
}

// ---------------------------------------------------------------- per-region checks
// The per-region rules of region cells Rc (rm: its cell mask), as a 4-bit code: bit 0 squares
// ok (533-551: at most one non-zero colour), bit 1 stars ok (553-619: no colourless star, and
// for each star colour c exactly 2 symbol occurrences of colour c), bits 2-3 the poly / ylop
// check (648-838): 0 no instance in the region, 1 passed (area and exact fit), 2 failed, 3 the
// exact-fit search was exhausted.  pl: the puzzle's SPARC_RULE_PLANES planes.
enum : uint32_t { kRcSq = 1u, kRcStar = 2u, kRcPolyShift = 2u };
template <int W, class Memo>
__device__ uint32_t region_code(const RulesTab& rt, const FitIn& fin, uint32_t q, const BB<W>& Rc, uint64_t rm,
                                const BB<W>* pl, Memo* memo) {
    uint32_t code = kRcSq | kRcStar;
    const BB<W> sq = Rc & pl[RP_SQUARE];
    if (sq.any()) {
        int ncol = 0;
#pragma unroll
        for (int c = 0; c < 8; ++c) ncol += (sq & pl[RP_COL1 + c]).any();
        if (ncol > 1) code &= ~kRcSq;
    }
    const BB<W> st = Rc & pl[RP_STAR];
    if (st.any()) {
        bool ok = !st.andnot(pl[RP_COLORED]).any();
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            const BB<W> col = Rc & pl[RP_COL1 + c];
            if (!(st & col).any()) continue;
            const int tot = (col & pl[RP_M0]).popc() + 2 * (col & pl[RP_M1]).popc() + 4 * (col & pl[RP_M2]).popc();
            ok &= tot == 2;
        }
        if (!ok) code &= ~kRcStar;
    }
    int net;
    if (region_net_area<W>(rt, fin, q, Rc, pl[RP_INST], net)) {
        uint32_t poly = 2;
        if (Rc.popc() == net) {
            int r = -1;
            if constexpr (!std::is_same<Memo, NoMemo>::value) r = memo->find(q, rm);
            if (r < 0) {
                r = hostfit_find(rt.hf, q, rm);                  // finished on the host earlier
                if (r < 0) r = exact_fit<W>(fin, Rc, rm, fin.cap);
                if constexpr (!std::is_same<Memo, NoMemo>::value)
                    if (r >= 0) memo->put(q, rm, r);
            }
            poly = r < 0 ? 3u : (r ? 1u : 2u);
        }
        code |= poly << kRcPolyShift;
    }
    return code;
}

// One word of the region-code table: the codes of region cell masks 8·g .. 8·g + 7 of puzzle q
// (4 bits each; masks that are no region of any state are never looked up).
template <int W>
__device__ uint32_t region_table_word(const Params& p, const RulesTab& rt, uint32_t q, uint32_t g) {
    const uint4 inf = p.tab.info[q];
    const uint32_t X = inf.x & 0xFFu, Y = (inf.x >> 8) & 0xFFu;
    const uint2 fc = rt.inst_fc[q];
    const FitIn fin = fit_in(rt, fc.x, fc.y, X, Y);
    const uint32_t cells = fin.CX * fin.CY;
    BB<W> pl[RP_ABI];
    const uint64_t* gp = rt.planes + (size_t)q * RP_COUNT * W;
    for (int k = 0; k < (int)RP_ABI; ++k) pl[k] = BB<W>::load(gp + k * W);
    uint32_t word = 0;
    for (uint32_t j = 0; j < 8; ++j) {
        const uint32_t m = 8u * g + j;
        if (m == 0 || m >= (1u << cells)) continue;
        BB<W> Rc = BB<W>::zero();
        for (uint32_t b = 0; b < cells; ++b)
            if ((m >> b) & 1u) Rc.set((2 * (b / fin.CY) + 1) * p.pitch + 2 * (b % fin.CY) + 1);
        word |= region_code<W, NoMemo>(rt, fin, q, Rc, (uint64_t)m, pl, nullptr) << (4 * j);
    }
    return word;
}

// ---------------------------------------------------------------- the audit
template <int W>
struct RuleOut {
    uint32_t bits;
    uint64_t fit_ok;   // bit r: region r held instances and passed the area check and the fit
};

// What the audit reads of puzzle q besides the state: the planes the regions and the path rules
// need, the target, the cell grid and the region-code table offset (a rule rollout keeps it in
// registers while the env stays on its puzzle).
template <int W>
struct PuzzleRules {
    BB<W> pl[10];   // kBasePlanes order
    uint32_t q, fo, tx, ty;
    uint32_t tbit;  // the target's board bit tx * pitch + ty
    FitIn fin;
};
constexpr uint32_t kBasePlanes[10] = {RP_CELLS, RP_LATTICE, RP_GAPS, RP_DOTS, RP_TRI, RP_TRI0, RP_TRI1, RP_TRI2,
                                      RP_NOTFIRST, RP_NOTLAST};
enum : uint32_t { kB_CELLS = 0, kB_LATTICE, kB_GAPS, kB_DOTS, kB_TRI, kB_TRI0, kB_TRI1, kB_TRI2, kB_NOTFIRST, kB_NOTLAST };
template <int W>
__device__ __forceinline__ PuzzleRules<W> puzzle_rules(const Params& p, const RulesTab& rt, uint32_t q) {
    PuzzleRules<W> r;
    const uint64_t* g = rt.rows + (size_t)q * rule_row_u64<W>();
#pragma unroll
    for (int k = 0; k < 10; ++k) r.pl[k] = BB<W>::load(g + k * W);
    const uint64_t m0 = g[10 * W], m1 = g[10 * W + 1];
    const uint32_t ix = (uint32_t)m1, iy = (uint32_t)(m1 >> 32);
    const uint32_t X = ix & 0xFFu, Y = (ix >> 8) & 0xFFu;
    r.q = q;
    r.fo = (uint32_t)m0;
    r.tx = iy & 0xFFu;
    r.ty = (iy >> 8) & 0xFFu;
    r.tbit = r.tx * p.pitch + r.ty;
    const uint32_t cf = ((iy >> 24) & 0x7Fu) | ((iy >> 31) ? kHostFit : 0u);
    r.fin = fit_in(rt, (uint32_t)(m0 >> 32), cf, X, Y);
    return r;
}

// The path rules of _run_rule_validators as their output bits: reached_target (487-495, bit 0),
// path_not_crossing (497-505, bit 1: true by construction, a move only enters an unvisited point
// and a pop removes the last one), no_gap_violations (507-517, bit 2), all_dots_collected (519-531,
// bit 3) and triangles_edge_count (622-646, bit 6).  They read only the path and the puzzle's
// planes (vis: path points, reached: the agent is on the target), not the regions.
template <int W>
__device__ __forceinline__ uint32_t audit_path(uint32_t P, const PuzzleRules<W>& pr, const BB<W>& vis, bool reached) {
    // triangles: bit-sliced count of path neighbours (x±1: ±P, y±1: ±1)
    const BB<W> a = vis.shr(P), b = vis.shl(P), c = vis.shr(1), d = vis.shl(1);
    const BB<W> s1 = a ^ b, c1 = a & b, s2 = c ^ d, c2 = c & d;
    const BB<W> n0 = s1 ^ s2, k0 = s1 & s2, n1 = c1 ^ c2 ^ k0, n2 = c1 & c2;
    const BB<W> bad = pr.pl[kB_TRI] & ((n0 ^ pr.pl[kB_TRI0]) | (n1 ^ pr.pl[kB_TRI1]) | (n2 ^ pr.pl[kB_TRI2]));
    const bool tri_ok = !bad.any();
    const bool gap_ok = !(pr.pl[kB_GAPS] & vis).any();
    const bool dot_ok = !pr.pl[kB_DOTS].andnot(vis).any();
    return (uint32_t)reached | 2u | ((uint32_t)gap_ok << 2) | ((uint32_t)dot_ok << 3) | ((uint32_t)tri_ok << 6);
}

// One dilation of R (within a) on the padded one-word board: a y step off the lattice lands on a
// blocked bit, so each lattice row's runs of allowed bits end below a zero.  Toward +y the whole
// run above each bit of R fills in one add: the carry from R ripples up through the run (the
// allowed bits it clears, plus the seeds, are the fill).  -y and +-x stay one step per iteration.
// Flood iterations per 64-env wave-step (c3 pool, random walks, regions in lock step): one step
// each way 39.9, +y runs 34.4.  The -y runs by the same add on the bit-reversed board (two more
// 64-bit adds and four bit reversals per iteration) cost more than the iterations they save:
// MI355X, c3r 2,000-step launches 3.956 -> 4.11-4.14 ms (profiles/r06/ab_c3r_inc).
// (a & ~(a + r)) | r | (x & a) = (a & ~((a + r) & ~x)) | r (r lies in a): one v_bitop3 per half,
// 6 logic VALU against the compiler's 8 (two v_not, four v_or3, two v_and); with the flood loop
// two dilations per trip (audit_r) c3r 2.97 -> 2.72 ms per 2,000-step launch (bitop3 alone 2.88,
// the loop alone 2.93; profiles/r06/ab_c3r_flood)
__device__ __forceinline__ uint64_t dilate_w1(uint64_t r, uint64_t a, uint32_t P) {
    const uint64_t s = a + r, x = (r >> 1) | (r << P) | (r >> P);
    uint32_t lo, hi;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0xb0" : "=v"(lo) : "v"((uint32_t)a), "v"((uint32_t)s), "v"((uint32_t)x));
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0xb0" : "=v"(hi) : "v"((uint32_t)(a >> 32)), "v"((uint32_t)(s >> 32)), "v"((uint32_t)(x >> 32)));
    return ((((uint64_t)hi) << 32) | lo) | r;
}

// vis: path points; reached: the agent is on the target (_rule_reached_target 487-495); pr: the
// env's puzzle (puzzle_rules).  region_out (may be null): region id per bit.  memo (FitMemo, or
// NoMemo): exact-fit answers carried between calls of one lane (puzzles without a region-code
// table).  TABLE_ONLY: every region is looked up in the region-code table (the caller checked
// that the puzzle has one), so no check and no exact-fit search is compiled in.  pos: the index
// of this audit's outputs, for the FitQueue entry of a search that passes the node cap (its
// region then counts as passing and the bits carry SPARC_RULE_SEARCH_EXHAUSTED until the host has
// finished the search; the region-code table never holds such a code after sparc_load_rules).
template <int W, class Memo = NoMemo, bool TABLE_ONLY = false>
__device__ RuleOut<W> audit_r(const Params& p, const RulesTab& rt, const PuzzleRules<W>& pr, const BB<W>& vis,
                              bool reached, uint8_t* region_out, Memo* memo = nullptr, uint64_t pos = 0) {
    const uint32_t q = pr.q, fo = pr.fo;
    const FitIn& fin = pr.fin;
    // the symbol planes only for a puzzle without a region-code table
    BB<W> pl[RP_ABI];
    if (!TABLE_ONLY && fo == kNoRegTab) {
        const uint64_t* g = rt.planes + (size_t)q * RP_COUNT * W;
#pragma unroll
        for (uint32_t k = RP_STAR; k <= RP_M2; ++k) pl[k] = BB<W>::load(g + k * W);
        pl[RP_INST] = BB<W>::load(g + RP_INST * W);
    }
    const uint32_t P = p.pitch;
    const BB<W> cells = pr.pl[kB_CELLS];
    const BB<W> gaps = pr.pl[kB_GAPS];
    const BB<W> nfirst = pr.pl[kB_NOTFIRST], nlast = pr.pl[kB_NOTLAST];
    const BB<W> allowed = pr.pl[kB_LATTICE].andnot(gaps | vis) | cells;

    bool sq_ok = true, star_ok = true, poly_ok = true, exhausted = false;
    uint64_t fit_ok = 0;
    auto take = [&](uint32_t code, uint32_t r) {
        sq_ok &= (code & kRcSq) != 0;
        star_ok &= (code & kRcStar) != 0;
        const uint32_t poly = code >> kRcPolyShift;
        exhausted |= poly == 3u;
        poly_ok &= poly != 2u;   // 3: passing until the host has finished the search
        if (poly == 1u) fit_ok |= 1ull << (r & 63);
    };
    // a table lookup is consumed one region later, so its L2 latency overlaps the next flood fill
    uint32_t tw = 0, tsh = 0, trid = 0;
    bool tpend = false;
    BB<W> remaining = cells;
    uint32_t rid = 0;
    while (remaining.any()) {
        BB<W> R = BB<W>::zero();
        R.set(remaining.lowest());
        if constexpr (W == 1) {   // two dilations per trip: no register copy of R per iteration
            // (four per trip measured slower: 2.77 against 2.72 ms, profiles/r06/ab_c3r_flood)
            uint64_t r0 = R.w[0];
            const uint64_t aw = allowed.w[0];
            while (true) {
                const uint64_t r1 = dilate_w1(r0, aw, P);
                if (r1 == r0) break;
                r0 = dilate_w1(r1, aw, P);
                if (r0 == r1) break;
            }
            R.w[0] = r0;
        } else while (true) {                                    // flood fill (BFS 431-452)
            BB<W> N;
            if constexpr (W == 1)
                N.w[0] = dilate_w1(R.w[0], allowed.w[0], P);   // whole +y runs per iteration
            else
                N = R | (R.shl(1) & nfirst) | (R.shr(1) & nlast) | R.shl(P) | R.shr(P);
            N = N & allowed;
            if (N == R) break;
            R = N;
        }
        const BB<W> Rc = R & cells;
        remaining = remaining.andnot(Rc);
        if (region_out) {
            BB<W> t = Rc;
            while (t.any()) {
                const uint32_t b = t.lowest();
                region_out[b] = (uint8_t)rid;
                t.w[b >> 6] &= t.w[b >> 6] - 1;
            }
        }
        uint64_t rm;
        if constexpr (W == 1)
            rm = P == 8u ? cell_mask_p8(fin, Rc.w[0]) : cell_mask<W>(fin, Rc, P);
        else
            rm = cell_mask<W>(fin, Rc, P);
        if (tpend) take((tw >> tsh) & 15u, trid);
        tpend = false;
        if (TABLE_ONLY || fo != kNoRegTab) {                     // the precomputed code
            const uint32_t m = (uint32_t)rm;
            tw = rt.reg_tab[(fo + m) >> 3];
            tsh = (m & 7u) * 4u;
            trid = rid;
            tpend = true;
        } else if constexpr (!TABLE_ONLY) {
            const uint32_t code = region_code<W, Memo>(rt, fin, q, Rc, rm, pl, memo);
            if ((code >> kRcPolyShift) == 3u && rt.fq.count) fit_queue_push(rt.fq, pos, rm, q, rid);
            take(code, rid);
        }
        ++rid;
    }
    if (tpend) take((tw >> tsh) & 15u, trid);
    const uint32_t pb = audit_path<W>(P, pr, vis, reached);
    uint32_t bits = pb | ((uint32_t)sq_ok << 4) | ((uint32_t)star_ok << 5) | ((uint32_t)poly_ok << 7);
    bits |= (uint32_t)((bits & 0xFFu) == 0xFFu) << 8;
    bits |= (uint32_t)exhausted << 9;
    return RuleOut<W>{bits, fit_ok};
}

// ---------------------------------------------------------------- incremental regions (W = 1)
// A rule rollout audits every step of an env, and consecutive steps differ by ONE path point
// (a forward move adds it, a traceback pop removes it); the regions (_compute_regions 422-454)
// are a function of the allowed set alone, so they follow incrementally:
//  * a point p leaving the allowed set (a move onto it): only the region holding it changes.  When
//    the allowed 4-neighbours of p lie in one run of allowed points around p (its 8-ring, each
//    ring point 4-adjacent to the next: kRingSimple below), any path through p detours through
//    the ring, so the region just loses p (its cells, and so its check code, are unchanged); else
//    the region is flooded again from its cells (it may split; pieces without a cell are no
//    region);
//  * a point p joining the allowed set (a pop): the regions of its allowed 4-neighbours merge
//    with p (and with any isolated corner point next to it: every allowed edge point touches a
//    cell, so the only allowed points outside every region are corners whose four edge points are
//    blocked).  Merging two or more regions makes a new cell mask: one table lookup.
// The rule bits need the regions only as a set (squares, stars and poly / ylop are per-region
// codes, AND-ed), so the slots carry no order.  A reset, a puzzle change or any other change of
// more than one point rebuilds the set by the full flood.
constexpr int kRegions1 = 9;   // cells of a one-word board (7 x 7 lattice: 3 x 3)

// the 3 x 3 neighbourhood of p as a 9-bit index, bit 3 (dx + 1) + (dy + 1) = point (x + dx, y + dy)
// allowed (a: allowed board, bit x * P + y; needs p + P + 1 < 64 + P + 1 and the board below bit
// 63 - P - 1, host-checked)
__device__ __forceinline__ uint32_t ring_index(uint64_t a, uint32_t p, uint32_t P) {
    const uint64_t b = (a << (P + 1u)) >> p;
    return (uint32_t)(b & 7u) | ((uint32_t)((b >> P) & 7u) << 3) | ((uint32_t)((b >> (2u * P)) & 7u) << 6);
}
// 1 when the allowed 4-neighbours of the centre lie in at most one run of the ring (index as
// ring_index; the centre bit ignored)
__host__ __device__ inline uint32_t ring_simple(uint32_t idx) {
    const int order[8] = {3, 6, 7, 8, 5, 2, 1, 0};   // ring: (0,-1) (1,-1) (1,0) (1,1) (0,1) (-1,1) (-1,0) (-1,-1)
    int first_gap = -1;
    for (int k = 0; k < 8; ++k)
        if (!((idx >> order[k]) & 1u)) { first_gap = k; break; }
    if (first_gap < 0) return 1u;                     // the whole ring allowed: one run
    int runs = 0;
    bool in = false, has4 = false;
    for (int k = 1; k <= 8; ++k) {                    // walk the ring from just after a gap
        const int pos = (first_gap + k) & 7;
        const bool on = (idx >> order[pos]) & 1u;
        if (on) {
            if (!in) { in = true; has4 = false; }
            has4 |= (pos & 1) == 0;                   // even ring positions are the 4-neighbours
        } else if (in) {
            in = false;
            runs += has4 ? 1 : 0;
        }
    }
    if (in) runs += has4 ? 1 : 0;
    return runs <= 1 ? 1u : 0u;
}

// Slot k holds region k's points (bits below kRingShift = 57: every board of a rule rollout) and,
// in bits 60-63, its region code; 0: a free slot.
constexpr uint32_t kRsCodeShift = 60;
constexpr uint64_t kRsPoints = (1ull << kRsCodeShift) - 1ull;
struct RegionSet1 {
    uint64_t m[kRegions1];      // region points | code << kRsCodeShift
    uint32_t agg = 0;           // kRcSq | kRcStar | poly_ok << 2 | exhausted << 3 over the regions
    uint64_t vis = 0;           // the path board they describe
    uint32_t q = 0xFFFFFFFFu;   // and its puzzle (none yet)

    __device__ __forceinline__ static uint64_t flood(uint64_t seed, uint64_t a, uint32_t P) {
        uint64_t r = seed;
        while (true) {   // as audit_r's W = 1 flood
            const uint64_t nx = dilate_w1(r, a, P);
            if (nx == r) return r;
            r = nx;
        }
    }
    // R's points | its region code << kRsCodeShift
    __device__ __forceinline__ static uint64_t with_code(const RulesTab& rt, const PuzzleRules<1>& pr, uint64_t R,
                                                         uint32_t P) {
        const uint64_t rc = R & pr.pl[kB_CELLS].w[0];
        BB<1> Rc;
        Rc.w[0] = rc;
        const uint32_t m = (uint32_t)(P == 8u ? cell_mask_p8(pr.fin, rc) : cell_mask<1>(pr.fin, Rc, P));
        const uint32_t code = (rt.reg_tab[(pr.fo + m) >> 3] >> ((m & 7u) * 4u)) & 15u;
        return R | ((uint64_t)code << kRsCodeShift);
    }
    __device__ __forceinline__ void set_agg() {
        uint32_t sq = kRcSq, st = kRcStar, po = 1u, ex = 0u;
#pragma unroll
        for (int k = 0; k < kRegions1; ++k) {
            const bool live = m[k] != 0ull;
            const uint32_t code = (uint32_t)(m[k] >> kRsCodeShift);
            sq &= live ? code : kRcSq;
            st &= live ? code : kRcStar;
            po &= (live && (code >> kRcPolyShift) == 2u) ? 0u : 1u;
            ex |= (live && (code >> kRcPolyShift) == 3u) ? 1u : 0u;
        }
        agg = (sq & kRcSq) | (st & kRcStar) | (po << 2) | (ex << 3);
    }
    // every region from scratch (a reset, another puzzle, a change of more than one point)
    __device__ void rebuild(const RulesTab& rt, const PuzzleRules<1>& pr, uint64_t a, uint32_t P) {
        uint64_t remaining = pr.pl[kB_CELLS].w[0];
#pragma unroll
        for (int k = 0; k < kRegions1; ++k) {
            m[k] = 0ull;
            if (remaining) {
                const uint64_t R = flood(remaining & (~remaining + 1ull), a, P);
                m[k] = with_code(rt, pr, R, P);
                remaining &= ~R;
            }
        }
        set_agg();
    }
    // p left the allowed set (a = the allowed board without it)
    __device__ void remove(const RulesTab& rt, const PuzzleRules<1>& pr, uint64_t a, uint32_t p, uint32_t P,
                           const uint8_t* simple) {
        const uint64_t bit = 1ull << p;
        uint64_t hit = 0ull;
#pragma unroll
        for (int k = 0; k < kRegions1; ++k) hit |= m[k] & bit;
        if (!hit) return;                                         // an isolated corner: no region
        if (simple[ring_index(a, p, P)]) {                        // no split: the region loses p
#pragma unroll
            for (int k = 0; k < kRegions1; ++k) m[k] &= ~bit;
            return;
        }
        uint64_t R = 0ull;
#pragma unroll
        for (int k = 0; k < kRegions1; ++k) {
            const bool h = (m[k] & bit) != 0ull;
            R = h ? m[k] & kRsPoints & ~bit : R;
            m[k] = h ? 0ull : m[k];
        }
        uint64_t rest = R & pr.pl[kB_CELLS].w[0];
        while (rest) {                                            // the pieces that hold cells
            const uint64_t piece = flood(rest & (~rest + 1ull), a, P);
            const uint64_t e = with_code(rt, pr, piece, P);
            bool placed = false;
#pragma unroll
            for (int k = 0; k < kRegions1; ++k) {
                const bool here = !placed && m[k] == 0ull;
                m[k] = here ? e : m[k];
                placed |= here;
            }
            rest &= ~piece;
        }
        set_agg();
    }
    // p joined the allowed set (a = the allowed board with it)
    __device__ void add(const RulesTab& rt, const PuzzleRules<1>& pr, uint64_t a, uint32_t p, uint32_t P) {
        const uint64_t bit = 1ull << p;
        if (!(a & bit)) return;                                   // a gap left the path: no change
        const uint64_t nb = (((bit << 1) | (bit >> 1) | (bit << P) | (bit >> P)) & a);
        uint64_t all = 0ull, merged = 0ull, keep = 0ull;
        uint32_t hits = 0;
#pragma unroll
        for (int k = 0; k < kRegions1; ++k) {
            all |= m[k];
            const bool h = (m[k] & nb) != 0ull;
            keep = (h && hits == 0u) ? m[k] : keep;               // the first region hit (its code)
            merged |= h ? m[k] : 0ull;
            hits += h ? 1u : 0u;
        }
        if (hits == 0u) return;                                   // p and isolated corners: no cell
        // p, and the isolated corners beside it
        merged = (merged & kRsPoints) | bit | (nb & ~all);
        uint64_t e = merged | (keep & ~kRsPoints);
        if (hits > 1u) e = with_code(rt, pr, merged, P);          // a new cell set: its code
        bool placed = false;
#pragma unroll
        for (int k = 0; k < kRegions1; ++k) {
            const bool h = (m[k] & nb) != 0ull;
            m[k] = h ? (placed ? 0ull : e) : m[k];
            placed |= h;
        }
        if (hits > 1u) set_agg();
    }
    // the audit of the path board v (agent on the target: reached) of puzzle pr
    __device__ uint32_t audit(const Params& p, const RulesTab& rt, const PuzzleRules<1>& pr, uint64_t v, bool reached,
                              const uint8_t* simple) {
        const uint32_t P = p.pitch;
        const uint64_t cells = pr.pl[kB_CELLS].w[0];
        const uint64_t a = (pr.pl[kB_LATTICE].w[0] & ~(pr.pl[kB_GAPS].w[0] | v)) | cells;
        const uint64_t d = v ^ vis;
        if (pr.q != q || (d & (d - 1ull)) != 0ull) {
            rebuild(rt, pr, a, P);
            q = pr.q;
        } else if (d) {
            const uint32_t pt = (uint32_t)__builtin_ctzll(d);
            if (v & d) remove(rt, pr, a, pt, P, simple);
            else add(rt, pr, a, pt, P);
        }
        vis = v;
        BB<1> vb;
        vb.w[0] = v;
        uint32_t bits = audit_path<1>(P, pr, vb, reached) | ((agg & 3u) << 4) | (((agg >> 2) & 1u) << 7);
        bits |= (uint32_t)((bits & 0xFFu) == 0xFFu) << 8;
        bits |= ((agg >> 3) & 1u) << 9;
        return bits;
    }
};

// the audit with the agent at (x, y)
template <int W, class Memo = NoMemo>
__device__ __forceinline__ RuleOut<W> audit(const Params& p, const RulesTab& rt, const PuzzleRules<W>& pr,
                                            const BB<W>& vis, uint32_t x, uint32_t y, uint8_t* region_out,
                                            Memo* memo = nullptr, uint64_t pos = 0) {
    return audit_r<W, Memo, false>(p, rt, pr, vis, x == pr.tx && y == pr.ty, region_out, memo, pos);
}

}  // namespace sparc
