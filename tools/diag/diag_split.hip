// Diagnostic build of the W = 1 split rollout: the product translation unit plus a copy of
// k_rollout1s whose waves stamp s_memtime around their work and their barrier waits, so each
// role's share of a tile interval is measured on the GPU (tools/diag_split.py runs it).
// Not product code: the product library never contains this kernel.
#include "../../sparc-gym_amd/csrc/sparc_kernels.hip"

namespace {

__device__ __forceinline__ uint64_t stamp() { return __builtin_amdgcn_s_memtime(); }

// TrieLane with the record gather replaced (G = 1: from an LDS table, valid memory but fake
// records; G = 2: no gather, the record stays: timing only, the outputs are wrong; G = 3: the
// current node's record reloaded every step, no exec-masked branch: correct; G = 4: the
// product's step1 (walk1) with the gather left out: timing only)
template <int G>
struct DiagTrieLane : TrieLane {
    const uint4* lds_rows = nullptr;
    // CODES = false (IOR): the product's class byte for G == 0; the timing-only gather variants
    // (G != 0) keep their reward codes
    template <bool CODES = true, class Rows>
    __device__ __forceinline__ int step1d(const uint32_t hw, const uint32_t a, const Rows& trow,
                                          const uint2* __restrict__ trie8, uint32_t num_puzzles) {
        if constexpr (G == 0) return step1<CODES>(hw, a, trow, trie8, num_puzzles);
        if constexpr (G == 4) {   // the product's step1 without the record gather (timing only)
            if (hw_reset(hw)) reset_from_nx<CODES>(trow, num_puzzles);
            walk1(hw, a);
            return finish<CODES>(hw >= 0x40000000u, (hw & kHwDone) != 0u);
        }
        const bool reset = hw_reset(hw);
        const uint32_t dd = (uint32_t)((int32_t)hw >> 14) & 0xFFFF0000u;
        const bool moved = hw >= 0x40000000u, done = (hw & kHwDone) != 0u;
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
        nx = row4(trow, npid);
        const uint64_t xy = ((uint64_t)ry << 32) | rx;
        const uint32_t c = (uint32_t)(xy >> (a & 0x30u));   // a: action << 4 (k_rollout1s)
        const uint32_t key = __builtin_amdgcn_ubfe(c, 0u, 16u) | (S & 0xFFFF0000u) | (~dd & 0x10000u);
        const bool take = key < 0xFFFFu;
        S = take ? key : S + dd;
        if constexpr (G == 1) {
            if (take) {
                const uint4 r = lds_rows[(S & 0x7FFFu) & 1023u];
                rx = r.x;
                ry = r.y;
            }
        } else if constexpr (G == 3) {   // every step: the current node's record (unchanged unless taken)
            const uint2 rec = trie8[base + (S & 0x7FFFu)];
            rx = rec.x;
            ry = rec.y;
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


// MoveLane1 with the autoreset variants: MV 0 the product's (divergent branch), 1 none (timing
// only), 2 a wave-uniform branch around it (no exec save / restore when no lane resets), 4 the
// branch without the next-row prefetch (timing only); and the LDS-wait variants (timing only,
// wrong outputs): 5 the target positions from registers instead of the I/O wave's LDS tile
// (pos_v), 6 the stack byte of the next pop (pnr) from a register instead of an LDS read
template <bool TB, int MV>
struct DiagMoveLane1 : MoveLane1<TB> {
    using B = MoveLane1<TB>;
    // the group's target position j (MV 5: a register pattern over the four window positions)
    __device__ __forceinline__ uint32_t pos_v(const uint8_t* tp, uint32_t sj, uint32_t P) const {
        if constexpr (MV == 5) {
            const uint32_t a = (sj * 0x9E3779B1u + B::e * 7u) >> 30;
            return a == 0 ? 2u * P : a == 1 ? P - 1u : a == 2 ? 0u : P + 1u;
        }
        return tp[sj * 64];
    }
    __device__ __forceinline__ uint32_t step_pos(const Params& p, uint32_t pos, bool rs) {
        if constexpr (MV != 6) return B::step_pos(p, pos, rs);
        // the product's step_pos with pnr kept in a register (no LDS read of slot len-3)
        const uint32_t P = p.pitch;
        B::step = __builtin_elementwise_add_sat(B::step, 1);
        const bool trunc0 = B::step >= p.max_steps;
        const uint32_t fwd = __builtin_amdgcn_ubfe(B::w, pos, 1u);
        uint32_t pop = 0;
        if constexpr (TB) pop = pos == B::rp ? B::bias : 0u;
        const uint32_t moved = fwd | pop;
        const int32_t d = (int32_t)pos - (int32_t)P;
        uint32_t tog;
        asm("v_mad_u32_u24 %0, %1, %2, %3" : "=v"(tog) : "v"(fwd), "v"(d), "v"(B::e + P));
        B::fr ^= (uint64_t)moved << (tog & 63u);
        const int32_t dl = (int32_t)fwd - (int32_t)pop;
        if constexpr (TB) {
            const uint32_t arp = 2u * P - pos;
            *B::lds_byte(B::sq + 128u) = (uint8_t)arp;
            const uint32_t orp = B::rp;
            B::rp = fwd ? arp : (pop ? B::pnr : B::rp);
            B::sq += (uint32_t)dl << 6;
            B::bias = (B::sq + B::bks) >> 31;
            B::pnr = fwd ? orp : B::pnr;   // a register stand-in for slot len-3
        } else {
            B::len += fwd;
        }
        B::e = (uint32_t)((int32_t)B::e + __mul24((int32_t)moved, d));
        B::w = (uint32_t)(B::fr >> (B::e & 63u));
        uint32_t lw = B::w & p.nbm;
        if constexpr (TB) lw |= B::bias << B::rp;
        const bool at_tgt = B::e == B::tgt;
        const bool done = trunc0 | (lw == 0u) | at_tgt;
        B::pending = done & !rs;
        return ((uint32_t)dl << 30) | ((at_tgt | rs) ? kHwTgt : 0u) | (B::pending ? kHwDone : 0u) | lw;
    }
    __device__ __forceinline__ bool reset_v(const bool ar, const uint4* mrow, uint32_t col_addr) {
        if constexpr (MV == 0) {
            return B::reset_next(ar, mrow, col_addr);
        } else if constexpr (MV == 2) {
            if (__builtin_amdgcn_ballot_w64(B::pending & ar)) return B::reset_next(ar, mrow, col_addr);
            return false;
        } else if constexpr (MV == 4) {
            const bool rs = B::pending & ar;
            if (rs) {
                B::e = B::rr.x & 0xFFu;
                B::tgt = (B::rr.x >> 8) & 0xFFu;
                B::pflags = B::rr.x >> 16;
                B::fr = ((uint64_t)B::rr.z << 32) | B::rr.y;
                B::w = 0;
                if constexpr (TB) {
                    B::sq = col_addr - 128u;
                    B::set_bks(col_addr);
                    B::bias = 0;
                } else {
                    B::len = 1;
                }
                B::step = -1;
            }
            return rs;
        } else {
            return false;
        }
    }
};

// per wave: [0] cycles working (barrier release -> next barrier arrival), [1] cycles waiting at
// barriers, [2] cycles in the whole kernel after the prologue, [3] barriers
#include "diag_kernel.inc"

}  // namespace

extern "C" int sparc_diag_rollout1s(void* ctx, int32_t T, const uint8_t* d_act, int8_t* d_rew, uint8_t* d_flags,
                                    int32_t* d_stats, uint64_t* d_times, int32_t variant) {
    Ctx* c = static_cast<Ctx*>(ctx);
    int rc = check_ctx(c, true);
    if (rc) return rc;
    if (c->W != 1 || c->n % 256 || T % kTile || !d_act || !d_rew || !d_flags || !d_times)
        return fail(c, SPARC_E_INVALID, "diag: W = 1, whole workgroups, whole tiles, all buffers");
    const Params p = make_params(c);
    if (!split1_pitch_ok(p.pitch)) return fail(c, SPARC_E_INVALID, "diag: pitch outside 3..9");
    // pools past the LDS row budget: the global-row kernel (row slots), product waves only
    const bool lds = kS_Base + split_table_bytes(c->num_puzzles) <= kMaxDynLds;
    const size_t shm = kS_Base + (lds ? split_table_bytes(c->num_puzzles) : kS_SlotBytes);
    if (!lds && variant != 0) return fail(c, SPARC_E_INVALID, "diag: global-row pools run variant 0 only");
    auto go = [&](auto kern) {
        rc = allow_big_lds(c, reinterpret_cast<const void*>(kern));
        if (rc) return;
        kern<<<dim3(c->n / 256), kBlock1s, shm, c->stream>>>(p, T, d_act, 0, 0, d_rew, d_flags,
                                                            reinterpret_cast<int4*>(d_stats), d_times);
    };
    // the product's I/O-wave reward codes (IOR: next-step autoreset, the bench configs)
    if (p.autoreset != 1) return fail(c, SPARC_E_INVALID, "diag: needs next-step autoreset (IOR)");
    // variant % 10: the trie wave's record gather, 0 = global (the product's), 1 = LDS, 2 = none;
    // variant / 10: the move wave's autoreset (DiagMoveLane1)
    const int g = variant % 10, mv = variant / 10;
    auto pick = [&](auto tb) {
        constexpr bool TB = decltype(tb)::value;
        if (!lds) {
            go(k_rollout1s_diag<TB, false, false, 0, 0, false, true>);
            return;
        }
        auto pg = [&](auto mvc) {
            constexpr int MV = decltype(mvc)::value;
            if (g == 1) go(k_rollout1s_diag<TB, false, true, 1, MV, false, true>);
            else if (g == 2) go(k_rollout1s_diag<TB, false, true, 2, MV, false, true>);
            else if (g == 3) go(k_rollout1s_diag<TB, false, true, 3, MV, false, true>);
            else if (g == 4) go(k_rollout1s_diag<TB, false, true, 4, MV, false, true>);
            else go(k_rollout1s_diag<TB, false, true, 0, MV, false, true>);
        };
        if (mv == 1) pg(std::integral_constant<int, 1>{});
        else if (mv == 2) pg(std::integral_constant<int, 2>{});
        else if (mv == 4) pg(std::integral_constant<int, 4>{});
        else if (mv == 5) pg(std::integral_constant<int, 5>{});
        else if (mv == 6) pg(std::integral_constant<int, 6>{});
        else pg(std::integral_constant<int, 0>{});
    };
    if (c->cfg.traceback) pick(std::true_type{});
    else pick(std::false_type{});
    if (rc) return rc;
    return launch_check(c);
}
