// Diagnostic build of the W = 1 split rollout: the product translation unit plus a copy of
// k_rollout1s whose waves stamp s_memtime around their work and their barrier waits, so each
// role's share of a tile interval is measured on the GPU (tools/diag_split.py runs it).
// Not product code: the product library never contains this kernel.
#include "../../sparc-gym_amd/csrc/sparc_kernels.hip"

namespace {

__device__ __forceinline__ uint64_t stamp() { return __builtin_amdgcn_s_memtime(); }

// TrieLane with the record gather replaced (G = 1: from an LDS table, valid memory but fake
// records; G = 2: no gather, the record stays): timing only, the outputs are wrong
template <int G>
struct DiagTrieLane : TrieLane {
    const uint4* lds_rows = nullptr;
    template <class Rows>
    __device__ __forceinline__ int step1d(const uint32_t hw, const uint32_t a, const Rows& trow,
                                          const uint2* __restrict__ trie8, uint32_t num_puzzles) {
        if constexpr (G == 0) return step1(hw, a, trow, trie8, num_puzzles);
        const bool reset = (hw & 0x400000u) != 0u;
        const uint32_t dd = (uint32_t)((int32_t)hw >> 14) & 0xFFFF0000u;
        const bool moved = hw >= 0x40000000u, done = (hw & 0x30000u) != 0u;
        if (reset) {
            pid = npid;
            npid = next_pid(npid, num_puzzles);
            rx = nx.x;
            ry = nx.y;
            base = nx.z;
            S = nx.w & 0x18000u;
            hs = (int32_t)((nx.w >> 14) & 1u);
            hsn = -hs;
            tmax = nx.w >> 17;
        }
        nx = trow[npid];
        const uint64_t xy = ((uint64_t)ry << 32) | rx;
        const uint32_t c = (uint32_t)(xy >> ((a << 4) & 0x30u));
        const uint32_t key = __builtin_amdgcn_ubfe(c, 0u, 16u) | (S & 0xFFFF0000u) | (~dd & 0x10000u);
        const bool take = key < 0xFFFFu;
        S = take ? key : S + dd;
        if constexpr (G == 1) {
            if (take) {
                const uint4 r = lds_rows[(S & 0x7FFFu) & 1023u];
                rx = r.x;
                ry = r.y;
            }
        }
        const uint32_t x = S >> 15;
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

// per wave: [0] cycles working (barrier release -> next barrier arrival), [1] cycles waiting at
// barriers, [2] cycles in the whole tile loop, [3] tiles
template <bool TB, int G>
__global__ void __launch_bounds__(kBlock1s) k_rollout1s_diag(Params p, int32_t T, const uint8_t* __restrict__ act,
                                                             int8_t* __restrict__ rew, uint8_t* __restrict__ flg,
                                                             int4* __restrict__ stats, uint64_t* __restrict__ times) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    const uint32_t NP = p.tab.num_puzzles;
    uint4* lm = reinterpret_cast<uint4*>(smem + kS_Base);
    uint4* lt = lm + NP;
    for (uint32_t k = threadIdx.x; k < NP; k += kBlock1s) {
        lm[k] = p.tab.mrow[k];
        lt[k] = p.tab.trow[k];
    }
    __syncthreads();
    const uint4* mrow = lm;
    const uint4* trow = lt;
    const size_t n = p.n;
    const uint32_t wg_base = blockIdx.x * 256u;
    const int32_t K = T / kTile;
    uint64_t t_work = 0, t_bar = 0, t_all = 0, tiles = 0;
    uint64_t t0 = stamp();
    const uint64_t start = t0;
    auto bar = [&]() {          // one barrier, stamped
        const uint64_t a = stamp();
        t_work += a - t0;
        __syncthreads();
        t0 = stamp();
        t_bar += t0 - a;
        ++tiles;
    };
    auto flush = [&]() {
        t_all = stamp() - start;
        if (lane == 0) {
            uint64_t* o = times + ((size_t)blockIdx.x * 12u + wv) * 4u;
            o[0] = t_work;
            o[1] = t_bar;
            o[2] = t_all;
            o[3] = tiles;
        }
    };
    if (wv >= 8) {
        const uint32_t io = wv - 8u;
        const uint32_t r = lane >> 2, c = (lane & 3u) * 16u;
        const uint32_t pppp = p.pitch * 0x01010101u;
        auto load_tile = [&](int32_t k) {
            u32x4 v = nt_load16(act + (size_t)(k * kTile + r) * n + wg_base + io * 64 + c);
            v.x = clamp_actions4(v.x);
            v.y = clamp_actions4(v.y);
            v.z = clamp_actions4(v.z);
            v.w = clamp_actions4(v.w);
            const size_t o = io * kS_Pair + (k % 3) * (kTile * 64) + r * 64 + c;
            *reinterpret_cast<u32x4*>(smem + kS_Act + o) = v;
            u32x4 q;
            q.x = __builtin_amdgcn_perm(pppp, p.nbr_pos, v.x);
            q.y = __builtin_amdgcn_perm(pppp, p.nbr_pos, v.y);
            q.z = __builtin_amdgcn_perm(pppp, p.nbr_pos, v.z);
            q.w = __builtin_amdgcn_perm(pppp, p.nbr_pos, v.w);
            *reinterpret_cast<u32x4*>(smem + kS_Pos + o) = q;
        };
        auto store_tile = [&](int32_t k) {
            const uint32_t r8 = lane >> 3, c8 = (lane & 7u) * 16u;
            const uint32_t h = io >> 1, q = io & 1u;
            const uint32_t row = (uint32_t)((k * kTile) & (kRing - 1)) + h * 8 + r8;
            const uint32_t w = 2 * q + (c8 >> 6);
            const uint8_t* base = smem + w * kS_Pair + row * 64 + (c8 & 63u);
            const size_t o = (size_t)(k * kTile + h * 8 + r8) * n + wg_base + q * 128 + c8;
            nt_store16(reinterpret_cast<uint8_t*>(rew) + o, *reinterpret_cast<const u32x4*>(base + kS_Rew));
            const u32x4* fh = reinterpret_cast<const u32x4*>(smem + w * kS_Pair + kS_FH + row * 256 + 4 * (c8 & 63u));
            u32x4 v;
            v.x = flag_bytes4(fh[0]);
            v.y = flag_bytes4(fh[1]);
            v.z = flag_bytes4(fh[2]);
            v.w = flag_bytes4(fh[3]);
            nt_store16(flg + o, v);
        };
        if (K > 0) load_tile(0);
        bar();
        for (int32_t k = 0; k <= K; ++k) {
            if (k + 1 < K) load_tile(k + 1);
            if (k >= 2) store_tile(k - 2);
            bar();
        }
        if (K >= 1) store_tile(K - 1);
        bar();
        flush();
        return;
    }
    const uint32_t pr = wv & 3u;
    const uint32_t i = wg_base + pr * 64u + lane;
    uint8_t* pb = smem + pr * kS_Pair;
    uint4* fin = reinterpret_cast<uint4*>(smem + kS_Fin) + 2u * (pr * 64u + lane);
    if (wv < 4) {
        MoveLane1<TB> m;
        uint8_t* col = pb + kS_Stk + lane;
        const uint32_t col_addr = MoveLane1<TB>::lds_addr(col);
        m.load(p, i, col, col_addr);
        const uint32_t pid0 = p.st.pid[i];
        m.prefetch_reset(mrow, pid0 + 1 == NP ? 0u : pid0 + 1);
        const uint32_t pend0 = m.pending ? 1u : 0u;
        uint32_t* th = reinterpret_cast<uint32_t*>(pb + kS_FH) + lane;
        bar();
        for (int32_t k = 0; k < K; ++k) {
            const uint8_t* tp = pb + kS_Pos + (k % 3) * (kTile * 64) + lane;
#pragma unroll 1
            for (int g = 0; g < kTile; g += 4) {
                uint32_t pv[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) pv[j] = tp[(g + j) * 64];
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const uint32_t row = (uint32_t)(k * kTile + g + j) & (kRing - 1);
                    m.reset_next(p, mrow, col_addr);
                    th[row * 64] = m.step_pos(p, pv[j]);
                }
            }
            bar();
        }
        bar();
        bar();
        const uint4 fs = fin[0];
        const uint4 fc = fin[1];
        const uint32_t pend = m.pending ? 1u : 0u;
        m.store(p, i, col, col_addr, fs.x, pend ? (fs.y == 0u ? 1u : 2u) : 0u, fc.y);
        if (stats) {
            const uint32_t resets = p.autoreset == 1 ? pend0 + fc.x - pend : 0u;
            int4 st = stats[i];
            st.x += (int)fs.z;
            st.y += (int)fc.x;
            st.z += (int)fs.w;
            st.w += (int)resets;
            stats[i] = st;
        }
        flush();
    } else {
        __builtin_amdgcn_s_setprio(1);
        DiagTrieLane<G> tl;
        tl.lds_rows = lt;
        tl.load(p.st.pos[i], p.st.aux[i], p.st.pid[i], trow, p.tab.trie8, NP);
        const uint32_t* th = reinterpret_cast<const uint32_t*>(pb + kS_FH) + lane;
        uint8_t* tr = pb + kS_Rew + lane;
        bar();
        bar();
        for (int32_t k = 1; k <= K; ++k) {
            const uint8_t* ta = pb + kS_Act + ((k - 1) % 3) * (kTile * 64) + lane;
#pragma unroll 1
            for (int g = 0; g < kTile; g += 4) {
                const uint32_t row0 = (uint32_t)((k - 1) * kTile + g) & (kRing - 1);
                uint32_t hb[4], av[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    hb[j] = th[(row0 + j) * 64];
                    av[j] = ta[(g + j) * 64];
                }
#pragma unroll
                for (int j = 0; j < 4; ++j) tr[(row0 + j) * 64] = (uint8_t)tl.step1d(hb[j], av[j], trow, p.tab.trie8, NP);
            }
            bar();
        }
        fin[0] = make_uint4(tl.S, (uint32_t)tl.Oneg, (uint32_t)tl.acc_x, tl.acc_z);
        fin[1] = make_uint4(tl.acc_y, tl.pid, 0u, 0u);
        bar();
        flush();
    }
}

}  // namespace

extern "C" int sparc_diag_rollout1s(void* ctx, int32_t T, const uint8_t* d_act, int8_t* d_rew, uint8_t* d_flags,
                                    int32_t* d_stats, uint64_t* d_times, int32_t variant) {
    Ctx* c = static_cast<Ctx*>(ctx);
    int rc = check_ctx(c, true);
    if (rc) return rc;
    if (c->W != 1 || c->n % 256 || T % kTile || !d_act || !d_rew || !d_flags || !d_times)
        return fail(c, SPARC_E_INVALID, "diag: W = 1, whole workgroups, whole tiles, all buffers");
    const Params p = make_params(c);
    const size_t shm = kS_Base + split_table_bytes(c->num_puzzles);
    if (shm > kMaxDynLds) return fail(c, SPARC_E_INVALID, "diag: table does not fit LDS");
    auto go = [&](auto kern) {
        rc = allow_big_lds(c, reinterpret_cast<const void*>(kern));
        if (rc) return;
        kern<<<dim3(c->n / 256), kBlock1s, shm, c->stream>>>(p, T, d_act, d_rew, d_flags,
                                                            reinterpret_cast<int4*>(d_stats), d_times);
    };
    // variant: the trie wave's record gather, 0 = global (the product's), 1 = LDS, 2 = none
    if (c->cfg.traceback) {
        if (variant == 1) go(k_rollout1s_diag<true, 1>);
        else if (variant == 2) go(k_rollout1s_diag<true, 2>);
        else go(k_rollout1s_diag<true, 0>);
    } else {
        if (variant == 1) go(k_rollout1s_diag<false, 1>);
        else if (variant == 2) go(k_rollout1s_diag<false, 2>);
        else go(k_rollout1s_diag<false, 0>);
    }
    if (rc) return rc;
    return launch_check(c);
}
