#!/usr/bin/env python3
"""Build timing-only variants of the kernel library for A/B runs (tools/ab_run.sh, prof_rollout
--lib): the product sources are copied to a scratch directory, one named text substitution set is
applied (each `old` must occur exactly once), and the copy is built into ab/lib_<variant>.so.  The
product sources carry no diagnostic switches; variants that cut work give WRONG answers and exist
only to locate time (never loaded by tests, smoke or bench).

    python tools/ab_variants.py [--rev REV] <variant> [<variant> ...]   (list: python tools/ab_variants.py)

--rev: the sources of git revision REV instead of the working tree (ab/lib_<variant>_<REV>.so).
Variants whose text no longer occurs in the sources are removed once their A/B is recorded
under profiles/ (the logs and a diff of the variant stay there).
"""
import os
import shutil
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "sparc-gym_amd", "csrc")

VARIANTS = {
    # the in-tree sources, built the same way (the A/B baseline)
    "head": [],
    # k_rollout1s: the I/O wave stores each lane's four target positions of a read
    # group as one word ([group][lane][4 steps] bytes, 16 byte stores per tile), the move wave
    # reads one ds_read_b32 per group and extracts byte j with v_bfe_u32, instead of four
    # ds_read_u8 and their zero-extensions
    "posword": [("sparc_kernels.hip", "                *reinterpret_cast<u32x4*>(smem + kS_Pos + o) = q;",
                 """                {
                    uint8_t* pq = smem + kS_Pos + io * kS_Pair + (k % 3) * (kTile * 64) + (r >> 2) * 256u + (r & 3u) + c * 4u;
#pragma unroll
                    for (int kk = 0; kk < 16; ++kk) pq[kk * 4] = (uint8_t)(q[kk >> 2] >> (8 * (kk & 3)));
                }"""),
                ("sparc_kernels.hip", "            const uint8_t* tp = pb + kS_Pos + (k % 3) * (kTile * 64) + lane;",
                 "            const uint8_t* tp = pb + kS_Pos + (k % 3) * (kTile * 64) + lane * 4u;"),
                ("sparc_kernels.hip", "                        pv[j] = tp[(g + j) * 64];",
                 "                        pv[j] = __builtin_amdgcn_ubfe(*reinterpret_cast<const uint32_t*>(tp + g * 64), 8u * j, 8u);")],
    # k_rollout1r audit waves: region codes not looked up (a constant code instead of reg_tab)
    "notab": [("sparc_rules.hpp", "            tw = rt.reg_tab[(fo + m) >> 3];", "            tw = 0x55555555u;")],
    # k_rollout1r audit waves: the puzzle's rule data loaded once, not on every puzzle change
    "noreload": [("sparc_kernels.hip", "                if (pid != pr.q) pr = puzzle_rules<1>(p, rt, pid);",
                  "                if (pr.q == 0xFFFFFFFFu) pr = puzzle_rules<1>(p, rt, pid);")],
    # the audit's flood fill cut to one dilation per region
    "noflood": [("sparc_rules.hpp", """            while (true) {
                const uint64_t r1 = dilate_w1(r0, aw, P);
                if (r1 == r0) break;
                r0 = dilate_w1(r1, aw, P);
                if (r0 == r1) break;
            }""", "            r0 = dilate_w1(r0, aw, P);")],
    # k_rollout1r audit waves do no audit at all (the step wave, rings and barriers only)
    "noaudit": [("sparc_kernels.hip", "            if (wg_base + ec < n) {\n                if (pid != pr.q) pr = puzzle_rules<1>(p, rt, pid);",
                 "            if (false) {\n                if (pid != pr.q) pr = puzzle_rules<1>(p, rt, pid);")],
    # the flood loop with a wave-uniform exit (no per-lane exec masks in the loop)
    "funi": [("sparc_rules.hpp", '            while (true) {\n                const uint64_t r1 = dilate_w1(r0, aw, P);\n                if (r1 == r0) break;\n                r0 = dilate_w1(r1, aw, P);\n                if (r0 == r1) break;\n            }', '            while (true) {   // a wave-uniform exit: converged lanes dilate on unchanged (idempotent)\n                const uint64_t r1 = dilate_w1(r0, aw, P);\n                const uint64_t r2 = dilate_w1(r1, aw, P);\n                const bool ch = r2 != r1;\n                r0 = r2;\n                if (!__any(ch)) break;\n            }')],
    # the move wave's pop test and back-position select without VCC (a shift and two v_bfi)
    "valusel": [("sparc_move1.hpp", '        if constexpr (TB) pop = pos == rp ? bias : 0u;                              // 1141-1166', '        if constexpr (TB) pop = bias >> (pos ^ rp);   // pos == rp ? bias : 0 (both < 32): no VCC   1141-1166'), ("sparc_move1.hpp", '            rp = fwd ? arp : (pop ? pnr : rp);', '            uint32_t r1;   // rp = fwd ? arp : (pop ? pnr : rp) by two v_bfi (fwd, pop in {0, 1})\n            asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(r1) : "v"(0u - pop), "v"(pnr), "v"(rp));\n            asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(rp) : "v"(0u - fwd), "v"(arp), "v"(r1));')],
    # W = 1 rule rows loaded in the order the audit uses them (regions first, path planes last)
    "roworder": [("sparc_rules.hpp", '#pragma unroll\n    for (int k = 0; k < 10; ++k) r.pl[k] = BB<W>::load(g + k * W);\n    const uint64_t m0 = g[10 * W], m1 = g[10 * W + 1];', '    uint64_t m0, m1;\n    if constexpr (W == 1) {\n        // what the regions need first (cells, lattice, gaps: bytes 0-23; the meta words 80-95),\n        // then the path-rule planes (24-63), so the flood waits for the first three loads only\n        const ulonglong2* g2 = reinterpret_cast<const ulonglong2*>(g);\n        const ulonglong2 a = g2[0], b = g2[1], m = g2[5];\n        __asm__ volatile("" ::: "memory");\n        const ulonglong2 c = g2[2], d = g2[3];\n        r.pl[0].w[0] = a.x; r.pl[1].w[0] = a.y; r.pl[2].w[0] = b.x; r.pl[3].w[0] = b.y;\n        r.pl[4].w[0] = c.x; r.pl[5].w[0] = c.y; r.pl[6].w[0] = d.x; r.pl[7].w[0] = d.y;\n        r.pl[8].w[0] = 0; r.pl[9].w[0] = 0;   // NOTFIRST / NOTLAST: the W > 1 flood only\n        m0 = m.x;\n        m1 = m.y;\n    } else {\n#pragma unroll\n        for (int k = 0; k < 10; ++k) r.pl[k] = BB<W>::load(g + k * W);\n        m0 = g[10 * W];\n        m1 = g[10 * W + 1];\n    }')],
    # the path rules' triangle count by v_bitop3 (audit_path)
    "tribitop": [("sparc_rules.hpp", '    // triangles: bit-sliced count of path neighbours (x±1: ±P, y±1: ±1)\n    const BB<W> a = vis.shr(P), b = vis.shl(P), c = vis.shr(1), d = vis.shl(1);\n    const BB<W> s1 = a ^ b, c1 = a & b, s2 = c ^ d, c2 = c & d;\n    const BB<W> n0 = s1 ^ s2, k0 = s1 & s2, n1 = c1 ^ c2 ^ k0, n2 = c1 & c2;\n    const BB<W> bad = pr.pl[kB_TRI] & ((n0 ^ pr.pl[kB_TRI0]) | (n1 ^ pr.pl[kB_TRI1]) | (n2 ^ pr.pl[kB_TRI2]));\n    const bool tri_ok = !bad.any();', '    // triangles: bit-sliced count of path neighbours (x±1: ±P, y±1: ±1) per 32-bit half, a full\n    // adder of a, b, c (sum s, carry M) plus d: bit 0 s ^ d, bit 1 M ^ (s & d), bit 2 M & s & d,\n    // each compared with the planes by v_bitop3 (7 per half against 13 plain logic VALU)\n    const BB<W> a = vis.shr(P), b = vis.shl(P), c = vis.shr(1), d = vis.shl(1);\n    uint32_t bad = 0;\n#pragma unroll\n    for (int h = 0; h < 2 * W; ++h) {\n        auto half = [h](const BB<W>& x) { return (uint32_t)(x.w[h >> 1] >> (32 * (h & 1))); };\n        const uint32_t ah = half(a), bh = half(b), ch = half(c), dh = half(d);\n        const uint32_t s = bitop3<0x96>(ah, bh, ch);                     // a ^ b ^ c\n        const uint32_t M = bitop3<0xE8>(ah, bh, ch);                     // majority (the carry)\n        const uint32_t e0 = bitop3<0x96>(s, dh, half(pr.pl[kB_TRI0]));   // count bit 0 ^ TRI0\n        const uint32_t n1 = bitop3<0x78>(M, s, dh);                      // M ^ (s & d)\n        const uint32_t n2 = bitop3<0x80>(M, s, dh);                      // M & s & d\n        const uint32_t f = bitop3<0xF6>(e0, n1, half(pr.pl[kB_TRI1]));   // e0 | (n1 ^ TRI1)\n        const uint32_t g = bitop3<0xF6>(f, n2, half(pr.pl[kB_TRI2]));    // f | (n2 ^ TRI2)\n        bad |= g & half(pr.pl[kB_TRI]);\n    }\n    const bool tri_ok = bad == 0u;'), ("sparc_rules.hpp", 'template <int W>\n__device__ __forceinline__ uint32_t audit_path(', '// v_bitop3_b32 d = TT[x << 2 | y << 1 | z] bitwise (gfx950)\ntemplate <uint32_t TT>\n__device__ __forceinline__ uint32_t bitop3(uint32_t x, uint32_t y, uint32_t z) {\n    uint32_t d;\n    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:%4" : "=v"(d) : "v"(x), "v"(y), "v"(z), "i"(TT));\n    return d;\n}\n\ntemplate <int W>\n__device__ __forceinline__ uint32_t audit_path(')],
    # the plane writer's piece loop unrolled twice (more stores in flight per wave)
    "obsun2": [("sparc_kernels.hip", """    const uint32_t dl = 256u / XY, dc = 256u - dl * XY;   // a 64-piece stride in envs / cells
    for (; f < total; f += 256u) {""", """    const uint32_t dl = 256u / XY, dc = 256u - dl * XY;   // a 64-piece stride in envs / cells
#pragma unroll 2
    for (; f < total; f += 256u) {""")],
    # k_rollout1s with the move rows (mrow) read from global memory although the table fits LDS
    "mrowg": [("sparc_kernels.hip", """        mrow = lm;
        trow = lt;
    }""", """        trow = lt;
    }""")],
    # k_rollout1s with the trie rows (trow) read from global memory although the table fits LDS
    "trowg": [("sparc_kernels.hip", """        mrow = lm;
        trow = lt;
    }""", """        mrow = lm;
    }""")],
    # k_rollout1s without the trie wave's priority (re-checked after IOR balanced the chains)
    # the look-ahead trie wave (step1la) on every LDS-table grid, not only on <= 64 workgroups
    "la": [("sparc_kernels.hip", "if (lds_s && blocks <= 64) launch_s1(k_rollout1s<TB, false, true, true, IOR, false, 1>, d_act);",
            "if (lds_s) launch_s(k_rollout1s<TB, false, true, true, IOR>, d_act);")],
    # "la" with the look-ahead gather issued by on-trie lanes only (off-trie lanes cannot take on
    # the next step): fewer L2 requests at 65,536 envs, one exec-masked branch per step
    "lamask": [("sparc_kernels.hip", "if (lds_s && blocks <= 64) launch_s1(k_rollout1s<TB, false, true, true, IOR, false, 1>, d_act);",
                "if (lds_s) launch_s(k_rollout1s<TB, false, true, true, IOR>, d_act);"),
               ("sparc_trie.hpp", """        const uint2 rec = trieg[((base + (S & 0x7FFFu)) << 2) + __builtin_amdgcn_ubfe(an16, 4u, 2u)];
        nrx = rec.x;
        nry = rec.y;
        return finish""", """        if (S < 0x10000u) {
            const uint2 rec = trieg[((base + (S & 0x7FFFu)) << 2) + __builtin_amdgcn_ubfe(an16, 4u, 2u)];
            nrx = rec.x;
            nry = rec.y;
        }
        return finish""")],
    # k_rollout_obsw occupancy: waves per SIMD allowed by the register budget
    "obsw6": [("sparc_kernels.hip", "__launch_bounds__(kBlockOw) __attribute__((amdgpu_waves_per_eu(4)))",
               "__launch_bounds__(kBlockOw) __attribute__((amdgpu_waves_per_eu(6)))")],
    "obsw8": [("sparc_kernels.hip", "__launch_bounds__(kBlockOw) __attribute__((amdgpu_waves_per_eu(4)))",
               "__launch_bounds__(kBlockOw) __attribute__((amdgpu_waves_per_eu(8)))")],
    # k_rollout1s: trie wave at priority 2, move wave at 1, I/O waves at 0 (the I/O waves yield)
    "prio21": [("sparc_kernels.hip", """        __builtin_amdgcn_s_setprio(1);
        static_assert(!(C && LA),""", """        __builtin_amdgcn_s_setprio(2);
        static_assert(!(C && LA),"""),
               ("sparc_kernels.hip", """    if (wv < (uint32_t)PR) {                                     // ---- move waves
        MoveLane1<TB> m;""", """    if (wv < (uint32_t)PR) {                                     // ---- move waves
        __builtin_amdgcn_s_setprio(1);
        MoveLane1<TB> m;""")],
    # the same with the move and trie waves at 1 (only the I/O waves yield)
    "prio11": [("sparc_kernels.hip", """    if (wv < (uint32_t)PR) {                                     // ---- move waves
        MoveLane1<TB> m;""", """    if (wv < (uint32_t)PR) {                                     // ---- move waves
        __builtin_amdgcn_s_setprio(1);
        MoveLane1<TB> m;""")],
    # the split tables without the 128-B line alignment of each puzzle's trie records
    "noalign": [("sparc_kernels.hip", "            nn8 = (nn8 + 15u) & ~(size_t)15u;\n", "")],
    # k_rollout1s: the move and trie waves read a whole 16-step tile's inputs at once
    "group16": [("sparc_kernels.hip", "constexpr int kGroup1s = 4;", "constexpr int kGroup1s = 16;")],
    "group8": [("sparc_kernels.hip", "constexpr int kGroup1s = 4;", "constexpr int kGroup1s = 8;")],
    # c2 (grids of at most 64 workgroups) on the plain trie wave instead of the look-ahead form
    "nola": [("sparc_kernels.hip", "if (lds_s && blocks <= 64) launch_s1(k_rollout1s<TB, false, true, true, IOR, false, 1>, d_act);",
              "if (lds_s && blocks <= 0) launch_s1(k_rollout1s<TB, false, true, true, IOR, false, 1>, d_act);")],
    "noprio": [("sparc_kernels.hip", """        __builtin_amdgcn_s_setprio(1);
        static_assert(!(C && LA),""", """        static_assert(!(C && LA),""")],
    # MoveLane1 (k_rollout1s move wave): the stack byte a pop needs (slot len-4) read one step
    # ahead, off the chain; pnr (slot len-3) then follows by selects: a forward move makes it the
    # old rp, a pop the prefetched byte, no move keeps it (the LDS read latency leaves the chain)
    "pnrahead": [("sparc_move1.hpp", "    uint32_t rp = 0, pnr = 0;             // traceback: back position of the last move / the one before",
                  "    uint32_t rp = 0, pnr = 0, pp = 0;     // traceback: back position of the last move / the one before"),
                 ("sparc_move1.hpp", "            rp = fwd ? arp : (pop ? pnr : rp);",
                  "            const uint32_t orp = rp;\n            rp = fwd ? arp : (pop ? pnr : rp);\n            pnr = fwd ? orp : (pop ? pp : pnr);"),
                 ("sparc_move1.hpp", "        if constexpr (TB) pnr = *lds_byte(sq);",
                  "        if constexpr (TB) pp = *lds_byte(sq - 64u);"),
                 ("sparc_move1.hpp", "            pnr = *lds_byte(sq);\n",
                  "            pnr = *lds_byte(sq);\n            pp = *lds_byte(sq - 64u);\n")],
    # MoveLane1: at-target / no-legal-move / done / pending and the hand-over word's bits by VALU
    # integer ops (x == 0 as (x - 1) >> 31) instead of v_cmp -> s_or / s_and -> v_cndmask chains
    "valudone": [("sparc_move1.hpp", """        const bool at_tgt = e == tgt;                                                // 1192
        const bool done = trunc0 | (lw == 0u) | at_tgt;                             // 1195-1199
        // an autoreset step is never done (w = 0 before it: lw was 0) and reports at-target
        pending = done & !rs;""", """        auto eq0 = [](uint32_t x) {   // 1 iff x == 0 (x < 2^31), VALU only
            uint32_t r;
            asm("v_add_u32 %0, -1, %1\\n\\tv_lshrrev_b32 %0, 31, %0" : "=&v"(r) : "v"(x));
            return r;
        };
        const uint32_t at = eq0(e ^ tgt);
        const uint32_t rsu = rs ? 1u : 0u;
        const uint32_t pu = (at | eq0(lw) | (trunc0 ? 1u : 0u)) & (rsu ^ 1u);
        pending = pu != 0u;"""),
                 ("sparc_move1.hpp", "        return ((uint32_t)dl << 30) | ((at_tgt | rs) ? kHwTgt : 0u) | (pending ? kHwDone : 0u) | lw;",
                  "        return ((uint32_t)dl << 30) | ((at | rsu) << 24) | (pu << 25) | lw;")],
    # MoveLaneW (k_rolloutWs move wave) with the free board in 16 VGPRs instead of LDS (VERDICT
    # r5 item 6): the window is a select of the dword pair around the agent, the toggle a
    # select-and-xor; LDS keeps the board only across load / store
    "regboard": [
        ("sparc_movew.hpp", "    uint32_t* bd = nullptr;          // this lane's dword 0 (stride 64 dwords)",
         """    uint32_t* bd = nullptr;          // this lane's dword 0 (stride 64 dwords)
    uint32_t rb[16];
    __device__ __forceinline__ uint32_t rget(uint32_t k) const {
        uint32_t v = 0u;
#pragma unroll
        for (uint32_t j = 0; j < 16u; ++j) v = k == j ? rb[j] : v;
        return v;
    }
    __device__ __forceinline__ void rxor(uint32_t k, uint32_t m) {
#pragma unroll
        for (uint32_t j = 0; j < 16u; ++j) rb[j] ^= k == j ? m : 0u;
    }"""),
        ("sparc_movew.hpp", """        const uint32_t k = e >> 5;
        const uint64_t pr = ((uint64_t)dw(k + 1u) << 32) | dw(k);
        w = pr >> (e & 31u);""", """        const uint32_t k = e >> 5;
        const uint64_t pr = ((uint64_t)rget(k + 1u) << 32) | rget(k);
        w = pr >> (e & 31u);"""),
        ("sparc_movew.hpp", "        __hip_atomic_fetch_xor(&dw(tog >> 5), moved << (tog & 31u), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);",
         "        rxor(tog >> 5, moved << (tog & 31u));"),
        ("sparc_movew.hpp", """                if (4u * k < g.BS) {
                    dw(4u * k) = nb[k].x;
                    dw(4u * k + 1u) = nb[k].y;
                    dw(4u * k + 2u) = nb[k].z;
                    dw(4u * k + 3u) = nb[k].w;
                }""", """                if (4u * k < g.BS) {
                    rb[4u * k] = nb[k].x;
                    rb[4u * k + 1u] = nb[k].y;
                    rb[4u * k + 2u] = nb[k].z;
                    rb[4u * k + 3u] = nb[k].w;
                }"""),
        ("sparc_movew.hpp", """        rs = 0;
        read_window(g);
    }""", """        rs = 0;
#pragma unroll
        for (uint32_t j = 0; j < 16u; ++j) rb[j] = j < g.BS ? dw(j) : 0u;
        read_window(g);
    }"""),
        ("sparc_movew.hpp", """        const uint32_t sx = (inf.x >> 16) & 0xFFu, sy = inf.x >> 24;
        uint64_t vis[W];""", """        const uint32_t sx = (inf.x >> 16) & 0xFFu, sy = inf.x >> 24;
#pragma unroll
        for (uint32_t j = 0; j < 16u; ++j)
            if (j < g.BS) dw(j) = rb[j];
        uint64_t vis[W];""")],
    # k_rollout1r with s_memtime stamps (timing only: the stats buffer receives, per wave, role |
    # total | barrier-wait | audit cycles at index N/2 + block * 16 + wave; tools/diag_r1r.py)
    "stamps": [
        ("sparc_kernels.hip", """        __syncthreads();                                         // B_0
        for (int32_t k = 0; k < K; ++k) {
            const int32_t cnt = tile_cnt(k);
            const uint32_t b = (uint32_t)k & 1u;
            if (tact) {""", """        uint64_t dg_bar = 0;
        const uint64_t dg_t0 = __builtin_amdgcn_s_memtime();
        __syncthreads();                                         // B_0
        for (int32_t k = 0; k < K; ++k) {
            const int32_t cnt = tile_cnt(k);
            const uint32_t b = (uint32_t)k & 1u;
            if (tact) {"""),
        ("sparc_kernels.hip", """                store_bits(k - 2);
            }
            __syncthreads();                                     // B_{k+1}""", """                store_bits(k - 2);
            }
            { const uint64_t s0_ = __builtin_amdgcn_s_memtime(); __syncthreads(); dg_bar += __builtin_amdgcn_s_memtime() - s0_; }"""),
        ("sparc_kernels.hip", """        store_bits(K - 1);
        if (!active) return;
        e.store(p, src, i);
        if (stats) {""", """        store_bits(K - 1);
        if (lane == 0 && stats) stats[p.n / 2 + blockIdx.x * 16 + wv] = make_int4(0, (int)(__builtin_amdgcn_s_memtime() - dg_t0), (int)dg_bar, 0);
        if (!active) return;
        e.store(p, src, i);
        if (false) {"""),
        ("sparc_kernels.hip", """    PuzzleRules<1> pr;
    pr.q = 0xFFFFFFFFu;
    __syncthreads();                                             // B_0
    __syncthreads();                                             // B_1 (interval 0: no tile yet)""", """    PuzzleRules<1> pr;
    pr.q = 0xFFFFFFFFu;
    uint64_t dg_bar = 0, dg_aud = 0;
    const uint64_t dg_t0 = __builtin_amdgcn_s_memtime();
    __syncthreads();                                             // B_0
    { const uint64_t s0_ = __builtin_amdgcn_s_memtime(); __syncthreads(); dg_bar += __builtin_amdgcn_s_memtime() - s0_; }"""),
        ("sparc_kernels.hip", """            uint32_t out = 0;
            if (wg_base + ec < n) {
                if (pid != pr.q) pr = puzzle_rules<1>(p, rt, pid);""", """            uint32_t out = 0;
            const uint64_t sa_ = __builtin_amdgcn_s_memtime();
            if (wg_base + ec < n) {
                if (pid != pr.q) pr = puzzle_rules<1>(p, rt, pid);"""),
        ("sparc_kernels.hip", """            tbt[at(b, j, ec)] = (uint16_t)out;
        }
        __syncthreads();                                         // B_{k+1}
    }
}""", """            tbt[at(b, j, ec)] = (uint16_t)out;
            dg_aud += __builtin_amdgcn_s_memtime() - sa_;
        }
        { const uint64_t s0_ = __builtin_amdgcn_s_memtime(); __syncthreads(); dg_bar += __builtin_amdgcn_s_memtime() - s0_; }
    }
    if (lane == 0 && stats) stats[p.n / 2 + blockIdx.x * 16 + wv] = make_int4((int)q + 1, (int)(__builtin_amdgcn_s_memtime() - dg_t0), (int)dg_bar, (int)dg_aud);
}"""),
    ],
}


def build(name, jobs_dir, rev=None):
    d = os.path.join(jobs_dir, name)
    if rev:   # the sources of a git revision (e.g. the A/B baseline of uncommitted work)
        os.makedirs(d)
        arch = subprocess.run(["git", "-C", REPO, "archive", rev, "sparc-gym_amd/csrc"], check=True,
                              capture_output=True).stdout
        subprocess.run(["tar", "-x", "-C", d, "--strip-components=2"], input=arch, check=True)
    else:
        shutil.copytree(CSRC, d)
    for fname, old, new in VARIANTS[name]:
        path = os.path.join(d, fname)
        src = open(path).read()
        if src.count(old) != 1:
            raise SystemExit(f"variant {name}: {old!r} occurs {src.count(old)} times in {fname}")
        open(path, "w").write(src.replace(old, new))
    out = os.path.join(REPO, "ab", f"lib_{name}{'_' + rev.replace('/', '_') if rev else ''}.so")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
           "-I" + os.path.join(REPO, "include"), "-I" + d, "-o", out, os.path.join(d, "sparc_kernels.hip")]
    return subprocess.Popen(cmd), out


def main():
    names = sys.argv[1:]
    rev = None
    if names[:1] == ["--rev"]:
        rev, names = names[1], names[2:]
    if not names:
        print("variants:", ", ".join(VARIANTS))
        return
    with tempfile.TemporaryDirectory() as tmp:
        procs = [build(n, tmp, rev) for n in names]
        rc = 0
        for p, out in procs:
            rc |= p.wait()
            print(out, "ok" if p.returncode == 0 else f"FAILED ({p.returncode})")
    sys.exit(rc)


if __name__ == "__main__":
    main()
