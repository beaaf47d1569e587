// sparc_kernels.hip — HIP kernels (gfx950) and the C ABI of include/sparc_gym_amd.h.
//
// Kernels (one lane per env, 256-lane workgroups, SoA state in HBM):
//   k_reset    reset/_load_puzzle for masked envs                 (SPaRC_Gym.py:1057-1108)
//   k_step     one step() per env, state HBM -> VGPR -> HBM        (SPaRC_Gym.py:1111-1238)
//   k_rollout  T steps per launch with the state kept in VGPRs; actions [T][N] prefetched a
//              chunk ahead, reward/flags streamed out per step     (the episode loop of
//              Final_Product.py:26-38 / llm_host.py:182-242, batched)
//   k_obs_pack dense int32 visited / agent_location planes         (_get_obs, SPaRC_Gym.py:979)
//   k_rules    rule audit of the current state                      (_validate_rules, 941-950)
// No MFMA: this is integer / bitboard work, bound by latency and HBM.
#include <hip/hip_runtime.h>
#include <dlfcn.h>

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <type_traits>
#include <vector>

#include "sparc_env.hpp"
#include "sparc_trie.hpp"
#include "sparc_movew.hpp"
#include "sparc_move1.hpp"
#include "sparc_rules.hpp"
#include "sparc_gym_amd.h"

using namespace sparc;

namespace {

constexpr int kBlock = 256;
constexpr int kTile = 16;                             // env-steps per LDS-transposed I/O tile
constexpr int kWaves = kBlock / 64;
// per-wave LDS I/O tiles of the generic-width rollout (actions, reward codes, flags), EPW envs
// per wave
template <int W, int EPW>
__host__ __device__ constexpr size_t tiles_lds_bytes() { return (size_t)kWaves * 3 * EPW * kTile; }
// per-wave LDS tile of the rule bits of a rule rollout ([16 steps][EPW envs] uint16), then one
// flag word per wave (the audit-pair join, k_rollout)
template <int EPW>
__host__ __device__ constexpr size_t bits_lds_bytes() { return (size_t)kWaves * 2 * EPW * kTile + 4 * kWaves; }
constexpr size_t kMaxDynLds = 160 * 1024;   // one workgroup may own all 160 KiB (gfx950)

// LDS bytes of the staged puzzle rows: (W = 1) compact row + reset board, or (W > 1) info +
// root record + the open bitboard that the generic step reads every step
template <int W>
__host__ __device__ constexpr size_t table_lds_bytes(uint32_t P) {
    return W == 1 ? (size_t)P * (sizeof(uint4) + sizeof(uint64_t))
                  : (size_t)P * (2 * sizeof(uint4) + W * sizeof(uint64_t));
}
// per-wave LDS direction stack of the W = 1 traceback rollout: [64 moves][EPW lanes] bytes
template <int W, bool TB, int EPW>
__host__ __device__ constexpr size_t stack_lds_bytes() {
    return (W == 1 && TB) ? (size_t)kWaves * 64 * EPW : 0;
}

template <int W, bool TB>
__global__ void __launch_bounds__(kBlock) k_reset(Params p, const uint32_t* __restrict__ q,
                                                  const uint8_t* __restrict__ mask, uint8_t* __restrict__ flg) {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= p.n) return;
    if (mask && !mask[i]) return;
    const uint32_t pid = q[i];
    if (pid >= p.tab.num_puzzles) {
        atomicOr(p.err, (int)kErrPuzzle);
        return;
    }
    const PuzzleSrc<W> src{p.tab.info, p.tab.root, p.tab.open, p.tab.init, p.tab.row1};
    Env<W, TB> e;
    e.reset(p, src, pid);
    e.store(p, src, i);
    if (flg) flg[i] = (uint8_t)(e.legal << 2);
}

// counter-based random actions [T][N]: entry (t, i) = sparc_rand_action(seed, env_offset + i,
// t0 + t), the device form of env.action_space.sample() (Final_Product.py:29) for every env.
// Seeded by the GLOBAL env id, so the shards of a multi-GPU job draw exactly the actions one
// process over all envs would (the RAND rollouts draw the same values in registers).  Four
// envs per lane, one 4-byte store when the row is aligned.
__global__ void __launch_bounds__(kBlock) k_rand_actions(uint64_t seed, uint64_t env_offset, uint64_t t0, uint32_t n,
                                                         uint32_t T, uint8_t* __restrict__ out) {
    const uint32_t per_row = (n + 3u) / 4u;
    const uint64_t k = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (k >= (uint64_t)per_row * T) return;
    const uint32_t t = (uint32_t)(k / per_row), i0 = (uint32_t)(k - (uint64_t)t * per_row) * 4u;
    uint8_t* row = out + (size_t)t * n;
    uint32_t v = 0;
#pragma unroll
    for (uint32_t j = 0; j < 4; ++j)
        if (i0 + j < n) v |= uint_rand_action(seed, env_offset + i0 + j, t0 + t) << (8u * j);
    if (i0 + 4u <= n && ((reinterpret_cast<uintptr_t>(row + i0) & 3u) == 0)) {
        *reinterpret_cast<uint32_t*>(row + i0) = v;
    } else {
        for (uint32_t j = 0; j < 4 && i0 + j < n; ++j) row[i0 + j] = (uint8_t)(v >> (8u * j));
    }
}

template <int W, bool TB>
__global__ void __launch_bounds__(kBlock) k_step(Params p, const uint8_t* __restrict__ act,
                                                 int8_t* __restrict__ rew, uint8_t* __restrict__ flg) {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= p.n) return;
    const PuzzleSrc<W> src{p.tab.info, p.tab.root, p.tab.open, p.tab.init, p.tab.row1};
    Env<W, TB> e;
    e.load(p, src, i);
    uint32_t f;
    const int c = e.advance(p, src, act[i], f);
    e.store(p, src, i);
    rew[i] = (int8_t)c;
    flg[i] = (uint8_t)f;
}

// One env of the context in one round trip (sparc_env_step / _reset / _read: the drop-in
// SPaRC_Gym, SPaRC_Gym.py:1057-1238): op 0 reads the state, 1 steps it with action `arg`, 2 resets
// it onto puzzle `arg`; the new state goes straight into the caller's pinned record.  One lane.
template <int W, bool TB>
__global__ void __launch_bounds__(64) k_env_op(Params p, uint32_t i, int32_t op, uint32_t arg,
                                               sparc_env_record* __restrict__ rec) {
    if (threadIdx.x != 0 || i >= p.n) return;
    const PuzzleSrc<W> src{p.tab.info, p.tab.root, p.tab.open, p.tab.init, p.tab.row1};
    Env<W, TB> e;
    int code = 0;
    uint32_t f = 0;
    if (op == 2) {
        e.reset(p, src, arg);
        f = e.legal << 2;
    } else {
        e.load(p, src, i);
        if (op == 1) code = e.advance(p, src, arg, f);
        else f = e.legal << 2;
    }
    if (op != 0) e.store(p, src, i);
    const State& s = p.st;
    const uint32_t ps = s.pos[i], ax = s.aux[i], oc = (ax >> 16) & 3u;
    rec->reward_code = (int8_t)code;
    rec->flags = (uint8_t)f;
    rec->x = (uint8_t)(ps & 0xFFu);
    rec->y = (uint8_t)((ps >> 8) & 0xFFu);
    rec->path_len = (uint8_t)((ps >> 16) & 0xFFu);
    rec->outcome = (int8_t)(oc == 1u ? 1 : (oc == 2u ? -1 : 0));
    rec->pending = (uint8_t)((ax >> 18) & 1u);
    rec->audited = 0;
    rec->step = s.step[i];
    rec->puzzle = s.pid[i];
    rec->rule_bits = 0;
    rec->host_fits = 0;
    rec->fit = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) rec->visited[k] = k < W ? s.vis[(size_t)k * p.n + i] : 0ull;
}

// the rule audit of env i (k_rules' outputs for every env of the context) and the exact fits it
// queued for the host, into the same record
__global__ void __launch_bounds__(64) k_env_audit(uint32_t i, uint32_t W, const uint16_t* __restrict__ bits,
                                                  const uint8_t* __restrict__ region, const uint64_t* __restrict__ fit,
                                                  const unsigned long long* __restrict__ queued,
                                                  sparc_env_record* __restrict__ rec) {
    const uint32_t l = threadIdx.x, nb = 64u * W;
    for (uint32_t b = l; b < 256u; b += 64u) rec->region[b] = b < nb ? region[(size_t)i * nb + b] : (uint8_t)0xFF;
    if (l == 0) {
        const unsigned long long q = *queued;
        rec->rule_bits = bits[i];
        rec->fit = fit[i];
        rec->host_fits = q > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)q;
        rec->audited = 1;
    }
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// streamed-once I/O: nontemporal so that actions / outputs do not evict the trie from L2
__device__ __forceinline__ u32x4 nt_load16(const uint8_t* q) {
    return __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(q));
}
__device__ __forceinline__ void nt_store16(uint8_t* q, u32x4 v) {
    __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(q));
}

// orders one wave's LDS accesses across its lanes (a wave's DS instructions execute in order;
// this only stops the compiler from moving them)
__device__ __forceinline__ void wave_lds_fence() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

// ---------------------------------------------------------------------------------------------
// 'new' observation planes, obs['base']['visited'] and obs['base']['agent_location']
// (SPaRC_Gym.py:956-979; int32 [x][y] planes), written by one wave for its 64 envs.
//
// Layout [...][N][XD][YD] int32, the lattice padded to XD x YD (the pool's largest).  A wave's
// envs own one contiguous run of 64 * XD * YD entries per plane, so instead of each lane
// writing its own env's plane (64 scattered rows per store instruction) every lane stages its
// board and agent bit in LDS and the wave then writes the run in 16-B pieces: piece j holds
// entries 4j..4j+3, whichever env they belong to, and one store instruction covers 1 KB of
// contiguous memory.  A LUT maps plane cell x*YD + y to board bit x*pitch + y (0xFFFF when
// the cell is outside the board).
constexpr uint32_t kObsCells = 256;   // XD * YD limit
constexpr uint16_t kObsNone = 0xFFFFu;
template <int W>
struct ObsWave {
    uint32_t vis[2 * W][64];   // visited board in 32-bit halves, half-major
    uint32_t ab[64];           // agent bit index (kObsNone for lanes without an env)
};
template <int W>
__host__ __device__ constexpr size_t obs_lds_bytes() { return kWaves * sizeof(ObsWave<W>) + kObsCells * sizeof(uint16_t); }

__device__ __forceinline__ void obs_build_lut(uint16_t* lut, uint32_t XD, uint32_t YD, uint32_t pitch, uint32_t W,
                                              uint32_t tid, uint32_t nthreads) {
    for (uint32_t c = tid; c < kObsCells; c += nthreads) {
        const uint32_t x = c / YD, y = c - x * YD, b = x * pitch + y;
        lut[c] = (c < XD * YD && y < pitch && b < 64u * W) ? (uint16_t)b : kObsNone;
    }
}

// this lane's env board and agent bit into the wave's staging area (kObsNone: no env)
template <int W>
__device__ __forceinline__ void obs_stage(ObsWave<W>* ow, uint32_t lane, bool has_env, const uint64_t (&v)[W],
                                          uint32_t ab) {
#pragma unroll
    for (int k = 0; k < W; ++k) {
        ow->vis[2 * k][lane] = (uint32_t)v[k];
        ow->vis[2 * k + 1][lane] = (uint32_t)(v[k] >> 32);
    }
    ow->ab[lane] = has_env ? ab : (uint32_t)kObsNone;
}

// the staged envs [0, cnt) of ow -> planes at vout / aout (run starts); every lane of the
// writing wave calls this (wave-uniform)
template <int W>
__device__ __forceinline__ void obs_write(const ObsWave<W>* ow, const uint16_t* lut, uint32_t lane, uint32_t cnt,
                                          uint32_t XY, int32_t* __restrict__ vout, int32_t* __restrict__ aout);

// the wave's envs [0, cnt) -> planes at vout / aout (run starts, entry `base` of the whole
// array, for the alignment test); every lane of the wave must call this (wave-uniform)
template <int W>
__device__ __forceinline__ void obs_emit(ObsWave<W>* ow, const uint16_t* lut, uint32_t lane, bool has_env,
                                         const uint64_t (&v)[W], uint32_t ab, uint32_t cnt, uint32_t XY,
                                         int32_t* __restrict__ vout, int32_t* __restrict__ aout) {
    obs_stage<W>(ow, lane, has_env, v, ab);
    wave_lds_fence();
    obs_write<W>(ow, lut, lane, cnt, XY, vout, aout);
    wave_lds_fence();
}

template <int W>
__device__ __forceinline__ void obs_write(const ObsWave<W>* ow, const uint16_t* lut, uint32_t lane, uint32_t cnt,
                                          uint32_t XY, int32_t* __restrict__ vout, int32_t* __restrict__ aout) {
    const uint32_t total = cnt * XY;
    // 16-B stores need both runs 16-B aligned (true whenever N * XY % 4 == 0)
    const bool vec = (((reinterpret_cast<uintptr_t>(vout) | reinterpret_cast<uintptr_t>(aout)) & 15u) == 0);
    uint32_t f = 4u * lane;                       // first entry of this lane's piece
    uint32_t l = f / XY, c = f - l * XY;          // its env and cell
    const uint32_t dl = 256u / XY, dc = 256u - dl * XY;   // a 64-piece stride in envs / cells
    for (; f < total; f += 256u) {
        uint32_t vv[4], aa[4];
        uint32_t ll = l, cc = c;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t b = lut[cc];
            const uint32_t word = ow->vis[(b >> 5) & (2 * W - 1)][ll & 63u];
            vv[k] = b == kObsNone ? 0u : (word >> (b & 31u)) & 1u;
            aa[k] = b == ow->ab[ll & 63u] ? 1u : 0u;
            ++cc;
            if (cc == XY) {
                cc = 0;
                ++ll;
            }
        }
        if (vec && f + 4u <= total) {
            if (vout) __builtin_nontemporal_store(u32x4{vv[0], vv[1], vv[2], vv[3]}, reinterpret_cast<u32x4*>(vout + f));
            if (aout) __builtin_nontemporal_store(u32x4{aa[0], aa[1], aa[2], aa[3]}, reinterpret_cast<u32x4*>(aout + f));
        } else {
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                if (f + k < total) {
                    if (vout) vout[f + k] = (int32_t)vv[k];
                    if (aout) aout[f + k] = (int32_t)aa[k];
                }
            }
        }
        c += dc;
        l += dl;
        if (c >= XY) {
            c -= XY;
            ++l;
        }
    }
}

// Bit-stream staging (k_rollout_obsw on multi-word pools, whose board bit x * pitch + y IS plane
// cell x * YD + y: pitch == YD).  The planes of a wave's 64 envs are one run of 64 * XY entries,
// entry f = env l, cell f - l * XY; staged as two bit streams (visited, agent) in which bit f is
// entry f, every piece of 4 entries is 4 bits of one 32-bit word, whichever env they belong to:
// the writer reads one word per plane and piece (against 12 LDS reads and ~30 VALU through the
// LUT) and zeroes the words it has read for the next use of the buffer.  Each compute lane ORs its
// board, shifted to bit l * XY, into the stream (ds_or_b32: the end words are shared with the
// neighbour envs).
template <int W>
struct ObsStream {
    uint32_t vis[128 * W + 1];   // 64 envs x at most 64 W bits, + the last lane's shifted spill
    uint32_t ag[128 * W + 1];
};
// stream staging applies: the board bit of cell (x, y) is x * YD + y, and a run of 64 envs fits the
// stream (XD * YD <= 64 W bits per env; a pool padded past its largest lattice, x_dim > x_max, can
// have more cells than board bits and takes the LUT path)
template <int W>
__host__ __device__ constexpr bool obs_stream_ok(uint32_t pitch, uint32_t XD, uint32_t YD) {
    return W > 1 && pitch == YD && XD * YD <= 64u * W;
}

template <int W>
__device__ __forceinline__ void obs_stage_stream(ObsStream<W>* os, uint32_t lane, bool has_env,
                                                 const uint64_t (&v)[W], uint32_t ab, uint32_t XY) {
    if (!has_env) return;
    const uint32_t o = lane * XY, w0 = o >> 5, sh = o & 31u;
    uint32_t b[2 * W];
#pragma unroll
    for (int k = 0; k < W; ++k) {
        b[2 * k] = (uint32_t)v[k];
        b[2 * k + 1] = (uint32_t)(v[k] >> 32);
    }
    // word j of the board shifted up by sh (bits at and above XY are 0: the board has none)
#pragma unroll
    for (int j = 0; j <= 2 * W; ++j) {
        const uint64_t pair = ((uint64_t)(j < 2 * W ? b[j] : 0u) << 32) | (j > 0 ? b[j - 1] : 0u);
        atomicOr(&os->vis[w0 + j], (uint32_t)(pair >> (32u - sh)));
    }
    const uint32_t a = o + ab;
    atomicOr(&os->ag[a >> 5], 1u << (a & 31u));
}

// the staged envs [0, cnt) -> planes at vout / aout (run starts); zeroes the words it read.
// Every lane of the writing wave calls this (wave-uniform)
template <int W>
__device__ __forceinline__ void obs_write_stream(ObsStream<W>* os, uint32_t lane, uint32_t cnt, uint32_t XY,
                                                 int32_t* __restrict__ vout, int32_t* __restrict__ aout) {
    const uint32_t total = cnt * XY;
    const bool vec = (((reinterpret_cast<uintptr_t>(vout) | reinterpret_cast<uintptr_t>(aout)) & 15u) == 0);
    for (uint32_t f = 4u * lane; f < total; f += 256u) {
        const uint32_t wv = os->vis[f >> 5], wa = os->ag[f >> 5], sh = f & 31u;
        uint32_t vv[4], aa[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            vv[k] = __builtin_amdgcn_ubfe(wv, sh + k, 1u);
            aa[k] = __builtin_amdgcn_ubfe(wa, sh + k, 1u);
        }
        if (sh == 0u) {   // after the reads of all 8 lanes of this word (in order within the wave)
            os->vis[f >> 5] = 0u;
            os->ag[f >> 5] = 0u;
        }
        if (vec && f + 4u <= total) {
            if (vout) __builtin_nontemporal_store(u32x4{vv[0], vv[1], vv[2], vv[3]}, reinterpret_cast<u32x4*>(vout + f));
            if (aout) __builtin_nontemporal_store(u32x4{aa[0], aa[1], aa[2], aa[3]}, reinterpret_cast<u32x4*>(aout + f));
        } else {
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                if (f + k < total) {
                    if (vout) vout[f + k] = (int32_t)vv[k];
                    if (aout) aout[f + k] = (int32_t)aa[k];
                }
            }
        }
    }
}

// step() + the 'new' observation in one launch (SPaRCVecEnv.step): the gym one-call-per-step
// contract with the planes, the puzzle index and the agent (x | y << 8) of every env
// the gym outputs of sparc_step_gym_device (each pointer may be null) and the action width
struct GymOut {
    const void* act;      // [N] uint8 (>= 4 illegal), int32 or int64 (< 0 or >= 4 illegal)
    uint32_t abytes;      // 1, 4 or 8
    double* r64;          // reward code / 100
    uint8_t* term;
    uint8_t* trunc;
    uint8_t* legal;
    uint8_t* areset;
    int32_t* loc;         // [N][2] (x, y)
};

__device__ __forceinline__ uint32_t read_action(const GymOut& g, uint32_t i) {
    if (g.abytes == 1) return static_cast<const uint8_t*>(g.act)[i];
    const int64_t v = g.abytes == 4 ? (int64_t) static_cast<const int32_t*>(g.act)[i]
                                    : static_cast<const int64_t*>(g.act)[i];
    return (v >= 0 && v < 4) ? (uint32_t)v : 255u;
}

template <int W, bool TB>
__global__ void __launch_bounds__(kBlock) k_step_obs(Params p, GymOut g, int8_t* __restrict__ rew,
                                                     uint8_t* __restrict__ flg, int32_t* __restrict__ vout,
                                                     int32_t* __restrict__ aout, uint32_t XD, uint32_t YD,
                                                     uint32_t* __restrict__ pidx, uint32_t* __restrict__ xy) {
    __shared__ ObsWave<W> ow[kWaves];
    __shared__ uint16_t lut[kObsCells];
    obs_build_lut(lut, XD, YD, p.pitch, W, threadIdx.x, kBlock);
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x, wave_base = i - lane;
    if (wave_base >= p.n) return;                 // wave-uniform
    const bool active = i < p.n;
    const PuzzleSrc<W> src{p.tab.info, p.tab.root, p.tab.open, p.tab.init, p.tab.row1};
    Env<W, TB> e;
    uint64_t v[W];
#pragma unroll
    for (int k = 0; k < W; ++k) v[k] = 0;
    uint32_t ab = 0;
    if (active) {
        e.load(p, src, i);
        uint32_t f;
        const int c = e.advance(p, src, read_action(g, i), f);
        e.store(p, src, i);
        if (rew) rew[i] = (int8_t)c;
        if (flg) flg[i] = (uint8_t)f;
        // reward code / 100 in float64: the reference's exact values (REWARD_SCALE in vec_env)
        if (g.r64) g.r64[i] = (double)c / 100.0;
        if (g.term) g.term[i] = (uint8_t)(f & 1u);
        if (g.trunc) g.trunc[i] = (uint8_t)((f >> 1) & 1u);
        if (g.legal) g.legal[i] = (uint8_t)((f >> 2) & 15u);
        if (g.areset) g.areset[i] = (uint8_t)((f >> 6) & 1u);
        e.obs_words(p, src, v, ab);
        if (pidx) pidx[i] = e.pid;
        if (xy || g.loc) {
            const uint32_t a = e.agent_xy(p);
            if (xy) xy[i] = a;
            if (g.loc) reinterpret_cast<int2*>(g.loc)[i] = make_int2((int)(a & 0xFFu), (int)((a >> 8) & 0xFFu));
        }
    }
    const uint32_t XY = XD * YD, cnt = p.n - wave_base < 64u ? p.n - wave_base : 64u;
    const size_t run = (size_t)wave_base * XY;
    obs_emit<W>(&ow[wv], lut, lane, active, v, ab, cnt, XY, vout ? vout + run : nullptr, aout ? aout + run : nullptr);
}

// T steps per env with the state in VGPRs.  Full waves with `tiled` (16-B aligned I/O, n % 16
// == 0) move actions / reward codes / flags in [16 steps][64 envs] tiles: one dwordx4 load and
// two dwordx4 stores per lane per 16 steps, transposed through a per-wave LDS tile, the next
// action tile prefetched one tile ahead.  Other waves / the tail use per-step byte accesses.
// With LDS_TABLE the puzzle rows (info, root record, open bitboard) are staged in LDS once, so
// autoresets issue no global load; the only global reads in the loop are trie records, issued
// at on-trie transitions and first consumed at the next one.
// EPW = envs per wave: 64, or 32 when the batch gives fewer than two full waves per SIMD (a
// lone wave issues a VALU op only every ~4 cycles and cannot hide its own trie-record wait;
// two half-width waves per SIMD fill each other's gaps).
// OBS: after every step the wave also writes the 'new' observation planes of step t to
// vout / aout + t * N * XD * YD (obs_emit; [T][N][XD][YD] int32 traces, either may be NULL).
struct ObsTrace {
    int32_t* vout;
    int32_t* aout;
    uint32_t XD, YD;
};
// RULES: after every step the wave also runs the rule audit of every env's new state
// (_validate_rules, which the reference's step() runs every step, SPaRC_Gym.py:1227 / 1011) and
// writes its bits to bits + t * N ([T][N] uint16, as sparc_rules_device's bits).  A rule
// rollout runs TWO waves per EPW envs (waves 2j and 2j+1 of a workgroup): both step the same envs
// (the step is deterministic and ~1/7 of the work), wave parity q audits the steps t with
// t % 2 == q, and only wave 0 of the pair writes the rewards, flags, stats, state and memo.  The
// audit is a latency-bound chain (flood fills, table lookups; ~40 % of its cycles waiting at one
// wave per SIMD); two per SIMD interleave (MI355X, c3r at 65,536 envs: see DESIGN.md §5)
constexpr uint32_t kAuditWaves = 2;   // waves per EPW envs in a rule rollout (a divisor of kWaves and kTile)
struct RuleTrace {
    RulesTab rt;
    uint16_t* bits;
    FitMemo<kMemo>* memo;   // [N] per-env exact-fit memo, carried between launches (may be null)
};
template <int W, bool TB, bool RAND, bool LDS_TABLE, int EPW, bool OBS = false, bool RULES = false>
__global__ void __launch_bounds__(kBlock) k_rollout(Params p, int32_t T, const uint8_t* __restrict__ act,
                                                    uint64_t seed, uint64_t t0, int8_t* __restrict__ rew,
                                                    uint8_t* __restrict__ flg, int4* __restrict__ stats,
                                                    uint32_t tiled, ObsTrace ot, RuleTrace rtr) {
    static_assert(!OBS || EPW == 64, "the observation writer needs full 64-lane waves");
    constexpr int kUnrollSteps = (OBS || RULES) ? 1 : 4;   // OBS / RULES: one step body (the plane writer / audit is long)
    // LDS: [I/O tiles, 3*16*EPW B per wave][W=1 traceback: move stacks, 64*EPW B per wave][rows]
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint8_t* ta = smem + wv * (3 * EPW * kTile);
    uint8_t* tr = ta + EPW * kTile;
    uint8_t* tf = tr + EPW * kTile;
    constexpr size_t kStackOff = tiles_lds_bytes<W, EPW>();
    constexpr size_t kObsOff = kStackOff + stack_lds_bytes<W, TB, EPW>();
    constexpr size_t kBitsOff = kObsOff + (OBS ? obs_lds_bytes<W>() : 0);
    constexpr size_t kTableOff = kBitsOff + (RULES ? bits_lds_bytes<EPW>() : 0);
    uint16_t* tbits = reinterpret_cast<uint16_t*>(smem + kBitsOff) + wv * (EPW * kTile);
    // RULES: per wave pair, set by the partner wave when it is done; the lead wave stores the
    // state and memo only after that, so the partner never loads a state the lead already wrote
    uint32_t* pair_done = reinterpret_cast<uint32_t*>(smem + kBitsOff + (size_t)kWaves * 2 * EPW * kTile);
    if constexpr (RULES) {
        if (threadIdx.x < kWaves) pair_done[threadIdx.x] = 0u;
        __syncthreads();
    }
    PuzzleSrc<W> src{p.tab.info, p.tab.root, p.tab.open, p.tab.init, p.tab.row1};
    ObsWave<W>* ow = reinterpret_cast<ObsWave<W>*>(smem + kObsOff) + wv;
    const uint16_t* lut = reinterpret_cast<const uint16_t*>(smem + kObsOff + kWaves * sizeof(ObsWave<W>));
    if constexpr (OBS) {
        obs_build_lut(const_cast<uint16_t*>(lut), ot.XD, ot.YD, p.pitch, W, threadIdx.x, kBlock);
        if constexpr (!LDS_TABLE) __syncthreads();
    }
    if constexpr (LDS_TABLE) {
        const uint32_t P = p.tab.num_puzzles;
        if constexpr (W == 1) {
            uint4* lrow1 = reinterpret_cast<uint4*>(smem + kTableOff);
            uint64_t* linit = reinterpret_cast<uint64_t*>(lrow1 + P);
            for (uint32_t k = threadIdx.x; k < P; k += kBlock) {
                lrow1[k] = p.tab.row1[k];
                linit[k] = p.tab.init[k];
            }
            __syncthreads();
            src = PuzzleSrc<W>{p.tab.info, p.tab.root, p.tab.open, linit, lrow1};
        } else {
            uint4* linfo = reinterpret_cast<uint4*>(smem + kTableOff);
            uint4* lroot = linfo + P;
            uint64_t* lopen = reinterpret_cast<uint64_t*>(lroot + P);
            for (uint32_t k = threadIdx.x; k < P; k += kBlock) {
                linfo[k] = p.tab.info[k];
                lroot[k] = p.tab.root[k];
            }
            for (uint32_t k = threadIdx.x; k < P * W; k += kBlock) lopen[k] = p.tab.open[k];
            __syncthreads();
            src = PuzzleSrc<W>{linfo, lroot, lopen, p.tab.init, p.tab.row1};
        }
    }
    // RULES: wave pairs on the same envs (above); q = the steps this wave audits (t % 2 == q)
    constexpr uint32_t kPerEnv = RULES ? kAuditWaves : 1u;
    const uint32_t q = RULES ? (wv % kAuditWaves) : 0u;
    const bool lead = q == 0u;   // writes the outputs, stats, state and memo
    const uint32_t wave_base = (blockIdx.x * (kWaves / kPerEnv) + wv / kPerEnv) * EPW;
    if (wave_base >= p.n || lane >= (uint32_t)EPW) return;   // no block-level barrier after here
    const uint32_t i = wave_base + lane;
    const bool active = i < p.n;
    const bool full = tiled && wave_base + EPW <= p.n;   // wave-uniform
    const size_t n = p.n;
    const uint64_t gid = p.env_offset + i;
    constexpr uint32_t kPieces = EPW / 16;                 // 16-byte pieces per tile row
    const uint32_t r = lane / kPieces, c = (lane % kPieces) * 16;   // this lane's piece of a tile
    using Stack = typename std::conditional<(W == 1 && TB), LdsStack<EPW>, RegStack>::type;
    Env<W, TB, Stack> e;
    if constexpr (W == 1 && TB) e.stk.col = smem + kStackOff + wv * (64 * EPW) + lane;
    if (active) e.load(p, src, i);
    int4 acc = make_int4(0, 0, 0, 0);
    const uint32_t XY = ot.XD * ot.YD;
    const uint32_t ocnt = p.n - wave_base < (uint32_t)EPW ? p.n - wave_base : (uint32_t)EPW;
    auto obs = [&](int32_t t) {                      // planes after step t (wave-uniform call)
        if constexpr (OBS) {
            uint64_t v[W];
#pragma unroll
            for (int k = 0; k < W; ++k) v[k] = 0;
            uint32_t ab = 0;
            if (active) e.obs_words(p, src, v, ab);
            const size_t run = ((size_t)t * n + wave_base) * XY;
            obs_emit<W>(ow, lut, lane, active, v, ab, ocnt, XY, ot.vout ? ot.vout + run : nullptr,
                        ot.aout ? ot.aout + run : nullptr);
        }
    };
    // exact-fit answers of this lane's recent regions (the path moves one point per step),
    // carried between launches and audit calls in HBM
    FitMemo<kMemo> memo;
    PuzzleRules<W> pr;   // W = 1 rule rollouts: the env's puzzle rule data (pr.q = its puzzle)
    pr.q = 0xFFFFFFFFu;
    if constexpr (RULES)
        if (rtr.memo && i < p.n) memo = rtr.memo[i];
    auto audit_step = [&](int32_t t, uint16_t* slot) {   // rule bits of the state after step t -> slot
        if constexpr (RULES) {
            if ((uint32_t)t % kAuditWaves != q) return;   // a partner wave's step (wave-uniform)
            uint64_t v[W];
            uint32_t ab;
            e.obs_words(p, src, v, ab);
            BB<W> vb;
#pragma unroll
            for (int k = 0; k < W; ++k) vb.w[k] = v[k];
            const uint32_t xy = e.agent_xy(p);
            RuleOut<W> ro;
            const uint64_t pos = (uint64_t)t * n + i;   // this audit's rule-bits entry (FitQueue)
            if constexpr (W == 1) {   // the puzzle's rule data stays in registers until the env's puzzle changes
                if (e.pid != pr.q) pr = puzzle_rules<W>(p, rtr.rt, e.pid);
                ro = audit<W>(p, rtr.rt, pr, vb, xy & 0xFFu, (xy >> 8) & 0xFFu, nullptr, &memo, pos);
            } else {
                ro = audit<W>(p, rtr.rt, puzzle_rules<W>(p, rtr.rt, e.pid), vb, xy & 0xFFu, (xy >> 8) & 0xFFu, nullptr,
                              &memo, pos);
            }
            *slot = (uint16_t)ro.bits;
        }
    };
    u32x4 anext = {0u, 0u, 0u, 0u};
    if (!RAND && full && T >= kTile) anext = nt_load16(act + (size_t)r * n + wave_base + c);

    for (int32_t tb = 0; tb < T; tb += kTile) {
        const int32_t cnt = T - tb < kTile ? T - tb : kTile;
        if (full && cnt == kTile) {
            if constexpr (!RAND) {
                const u32x4 acur = anext;
                if (tb + 2 * kTile <= T) anext = nt_load16(act + (size_t)(tb + kTile + r) * n + wave_base + c);
                *reinterpret_cast<u32x4*>(ta + r * EPW + c) = acur;
                wave_lds_fence();
            }
            // 4 groups of 4 steps: each group reads its 4 actions first (one LDS wait), then
            // steps; a full 16-step unroll spills SGPRs
#pragma unroll 1
            for (int g = 0; g < kTile; g += 4) {
                uint32_t av[4];
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    av[j] = RAND ? uint_rand_action(seed, gid, t0 + (uint64_t)(tb + g + j)) : ta[(g + j) * EPW + lane];
#pragma unroll kUnrollSteps
                for (int j = 0; j < 4; ++j) {
                    const int k = g + j;
                    uint32_t f;
                    const int code = e.advance(p, src, av[j], f);
                    obs(tb + k);
                    audit_step(tb + k, tbits + k * EPW + lane);
                    tr[k * EPW + lane] = (uint8_t)code;
                    tf[k * EPW + lane] = (uint8_t)f;
                    if constexpr (W == 1) {   // per-step flags the W = 1 step already has
                        acc.x += code;
                        acc.y += (int)e.pending;
                        acc.z += (int)e.solved;
                        acc.w += (int)e.was_reset;
                    } else {
                        acc.x += code;
                        acc.y += (f & 3u) ? 1 : 0;
                        acc.z += ((f & 3u) && code == 100) ? 1 : 0;
                        acc.w += (f & 64u) ? 1 : 0;
                    }
                }
            }
            wave_lds_fence();
            const size_t o = (size_t)(tb + r) * n + wave_base + c;
            if (lead) {
                if (rew) nt_store16(reinterpret_cast<uint8_t*>(rew) + o, *reinterpret_cast<const u32x4*>(tr + r * EPW + c));
                if (flg) nt_store16(flg + o, *reinterpret_cast<const u32x4*>(tf + r * EPW + c));
            }
            if constexpr (RULES) {   // the tile's rule bits of this wave's steps (rows t % 2 == q; tb is even):
                                     // whole 16-B pieces of each step's EPW-env run
                constexpr uint32_t kPer = EPW / 8, kPieces = kTile / kAuditWaves * kPer;   // 16-B pieces per row / this wave's rows
#pragma unroll
                for (uint32_t pi = lane; pi < kPieces; pi += 64) {
                    const uint32_t row = kAuditWaves * (pi / kPer) + q, col = (pi % kPer) * 8;
                    nt_store16(reinterpret_cast<uint8_t*>(rtr.bits + (size_t)(tb + row) * n + wave_base + col),
                               *reinterpret_cast<const u32x4*>(tbits + row * EPW + col));
                }
            }
            wave_lds_fence();
        } else if (active || OBS) {
            for (int k = 0; k < cnt; ++k) {
                const int32_t t = tb + k;
                if (active) {
                    const uint32_t a = RAND ? uint_rand_action(seed, gid, t0 + (uint64_t)t) : act[(size_t)t * n + i];
                    uint32_t f;
                    const int code = e.advance(p, src, a, f);
                    if (rew && lead) rew[(size_t)t * n + i] = (int8_t)code;
                    if (flg && lead) flg[(size_t)t * n + i] = (uint8_t)f;
                    acc.x += code;
                    acc.y += (f & 3u) ? 1 : 0;
                    acc.z += ((f & 3u) && code == 100) ? 1 : 0;
                    acc.w += (f & 64u) ? 1 : 0;
                    audit_step(t, rtr.bits + (size_t)t * n + i);
                }
                obs(t);
            }
        }
    }
    if constexpr (RULES) {   // the join of the audit pair (see pair_done)
        const uint32_t pair = wv / kAuditWaves;
        if (!lead) {
            __hip_atomic_store(&pair_done[pair], 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        } else {
            // bounded (the partner runs the same loop and always gets here; a bound keeps a fault
            // from hanging the GPU): on timeout the context's error word reports it (sparc_sync)
            uint32_t k = 0;
            for (; k < (1u << 26) &&
                   __hip_atomic_load(&pair_done[pair], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) == 0u;
                 ++k)
                __builtin_amdgcn_s_sleep(2);
            if (k == (1u << 26) && lane == 0) atomicOr(p.err, (int)kErrJoin);
        }
    }
    if (!active || !lead) return;
    e.store(p, src, i);
    if constexpr (RULES)
        if (rtr.memo) rtr.memo[i] = memo;
    if (stats) {
        int4 s = stats[i];
        s.x += acc.x;
        s.y += acc.y;
        s.z += acc.z;
        s.w += acc.w;
        stats[i] = s;
    }
}

// ---------------------------------------------------------------------------------------------
// Rollout with the 'new' observation planes after every step (config c4: ~1 KB of plane stores per
// env-step), the planes written by a WRITER wave.  vmcnt counts loads and stores in issue order,
// so a wave that both gathers trie records and stores planes (k_rollout<..., OBS>) waits, at each
// step's record wait, for every plane store it issued in the step before: its stores drain in
// bursts (MI355X, c4: 62-78 % of 8 TB/s, 0.71 of the box's fill_ bandwidth).  Here a workgroup of
// 256 envs has 4 compute waves (Env<W>, one lane per env) and 4 writer waves: in iteration t the
// compute waves run step t and stage each env's board and agent bit in LDS buffer t % 2
// (obs_stage), while writer k streams the planes of step t - 1 of compute wave k's envs from the
// other buffer (obs_write: 16-B pieces of each 64-env run, every store instruction 1 KB of
// contiguous memory); one barrier per step hands the buffers over.  The writers issue no load and
// never wait for their stores; the compute waves' own stores are a byte of reward code and of
// flags per env-step.  One writer per workgroup was issue-bound (the plane assembly is ~40
// instructions and 12 LDS reads per 16-B piece: MI355X, c4 3.26 ms per launch against 2.54 ms
// inline)
constexpr int kBlockOw = 512;
// one staging buffer: ObsWave (LUT path) or ObsStream (bit streams), [2 steps][4 compute waves]
template <int W>
__host__ __device__ constexpr size_t obsw_buf_bytes() {
    return ((sizeof(ObsWave<W>) > sizeof(ObsStream<W>) ? sizeof(ObsWave<W>) : sizeof(ObsStream<W>)) + 15) / 16 * 16;
}
template <int W, bool TB>
__host__ __device__ constexpr size_t obsw_lds_bytes() {
    return 8 * obsw_buf_bytes<W>() + kObsCells * sizeof(uint16_t) + ((W == 1 && TB) ? 4 * 64 * 64 : 0);
}
template <int W, bool TB, bool RAND>
__global__ void __launch_bounds__(kBlockOw) __attribute__((amdgpu_waves_per_eu(4)))
    k_rollout_obsw(Params p, int32_t T, const uint8_t* __restrict__ act, uint64_t seed, uint64_t t0,
                   int8_t* __restrict__ rew, uint8_t* __restrict__ flg, int4* __restrict__ stats, ObsTrace ot) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    constexpr size_t kBuf = obsw_buf_bytes<W>();   // buffer (t & 1) * 4 + k at smem + that * kBuf
    uint16_t* lut = reinterpret_cast<uint16_t*>(smem + 8 * kBuf);
    const bool stream = obs_stream_ok<W>(p.pitch, ot.XD, ot.YD);   // block-uniform
    if (stream) {   // the bit streams start at 0 (the writers zero them after each read)
        for (uint32_t k = threadIdx.x; k < 8 * kBuf / 4; k += kBlockOw) reinterpret_cast<uint32_t*>(smem)[k] = 0u;
    } else {
        obs_build_lut(lut, ot.XD, ot.YD, p.pitch, W, threadIdx.x, kBlockOw);
    }
    __syncthreads();
    auto buf = [&](uint32_t j) { return smem + j * kBuf; };
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    const size_t n = p.n;
    const uint32_t XY = ot.XD * ot.YD;
    if (wv >= 4) {                                               // ---- the writer waves
        const uint32_t k = wv - 4u;                              // compute wave k's envs
        const size_t wb = (size_t)blockIdx.x * 256u + k * 64u;
        const uint32_t cnt = wb >= n ? 0u : (n - wb < 64u ? (uint32_t)(n - wb) : 64u);
        for (int32_t t = 0; t <= T; ++t) {
            if (t > 0 && cnt > 0) {
                const size_t run = ((size_t)(t - 1) * n + wb) * XY;
                uint8_t* bk = buf(((t - 1) & 1) * 4 + k);
                int32_t* vo = ot.vout ? ot.vout + run : nullptr;
                int32_t* ao = ot.aout ? ot.aout + run : nullptr;
                if (stream) obs_write_stream<W>(reinterpret_cast<ObsStream<W>*>(bk), lane, cnt, XY, vo, ao);
                else obs_write<W>(reinterpret_cast<const ObsWave<W>*>(bk), lut, lane, cnt, XY, vo, ao);
            }
            __syncthreads();                                     // B_t
        }
        return;
    }
    const uint32_t i = blockIdx.x * 256u + wv * 64u + lane;     // ---- compute waves
    const bool active = i < n;
    const PuzzleSrc<W> src{p.tab.info, p.tab.root, p.tab.open, p.tab.init, p.tab.row1};
    using Stack = typename std::conditional<(W == 1 && TB), LdsStack<64>, RegStack>::type;
    Env<W, TB, Stack> e;
    if constexpr (W == 1 && TB) e.stk.col = smem + 8 * kBuf + kObsCells * sizeof(uint16_t) + wv * 64 * 64 + lane;
    if (active) e.load(p, src, i);
    int4 acc = make_int4(0, 0, 0, 0);
    const uint64_t gid = p.env_offset + i;
    for (int32_t t = 0; t < T; ++t) {
        uint64_t v[W];
#pragma unroll
        for (int k = 0; k < W; ++k) v[k] = 0;
        uint32_t ab = 0;
        if (active) {
            const uint32_t a = RAND ? uint_rand_action(seed, gid, t0 + (uint64_t)t) : act[(size_t)t * n + i];
            uint32_t f;
            const int code = e.advance(p, src, a, f);
            if (rew) rew[(size_t)t * n + i] = (int8_t)code;
            if (flg) flg[(size_t)t * n + i] = (uint8_t)f;
            acc.x += code;
            acc.y += (f & 3u) ? 1 : 0;
            acc.z += ((f & 3u) && code == 100) ? 1 : 0;
            acc.w += (f & 64u) ? 1 : 0;
            e.obs_words(p, src, v, ab);
        }
        uint8_t* bk = buf((t & 1) * 4 + wv);
        if (stream) obs_stage_stream<W>(reinterpret_cast<ObsStream<W>*>(bk), lane, active, v, ab, XY);
        else obs_stage<W>(reinterpret_cast<ObsWave<W>*>(bk), lane, active, v, ab);
        __syncthreads();                                         // B_t
    }
    __syncthreads();                                             // B_T: the writer's last step
    if (!active) return;
    e.store(p, src, i);
    if (stats) {
        int4 st = stats[i];
        st.x += acc.x;
        st.y += acc.y;
        st.z += acc.z;
        st.w += acc.w;
        stats[i] = st;
    }
}

// ---------------------------------------------------------------------------------------------
// W = 1 rollout: 4 env waves + 1 I/O wave per workgroup (256 envs).
//
// The env waves only issue trie-record gathers to global memory.  Their vmcnt counter is in
// order, so every wait for a gather would also wait for any older action prefetch or output
// store; the I/O wave therefore moves all streamed data: it loads the action tile of tile k+1
// into a double buffer and writes the reward / flag tiles of tile k-2 out of four-tile LDS
// rings while the env waves step tile k, and one workgroup barrier per 16-step tile hands the
// buffers over.  Env wave iteration t runs the trie phase of step t-1 next to the move phase
// of step t (independent dependency chains; the gather issued in iteration t-1 has a whole
// iteration to arrive).  Iteration 0's trie phase replays the stored step and changes
// nothing; its outputs are subtracted from the stats.  Workgroups that are not full (or
// unaligned I/O) step every env with per-step byte accesses and no I/O wave.
constexpr int kBlock1 = 320;
constexpr int kRing = 64;                              // output ring rows (4 tiles)
constexpr size_t kW1Act = 2 * kTile * 64;              // per env wave: actions, double buffer
constexpr size_t kW1Wave = kW1Act + 2 * kRing * 64 + 64 * 64;   // + reward / flag rings + move stack
constexpr size_t kW1Base = 4 * kW1Wave;

template <bool TB, bool RAND, bool LDS_TABLE>
__global__ void __launch_bounds__(kBlock1) k_rollout1(Params p, int32_t T, const uint8_t* __restrict__ act,
                                                      uint64_t seed, uint64_t t0, int8_t* __restrict__ rew,
                                                      uint8_t* __restrict__ flg, int4* __restrict__ stats,
                                                      uint32_t tiled) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    PuzzleSrc<1> src{p.tab.info, p.tab.root, p.tab.open, p.tab.init, p.tab.row1};
    if constexpr (LDS_TABLE) {
        const uint32_t P = p.tab.num_puzzles;
        uint4* lrow1 = reinterpret_cast<uint4*>(smem + kW1Base);
        uint64_t* linit = reinterpret_cast<uint64_t*>(lrow1 + P);
        for (uint32_t k = threadIdx.x; k < P; k += kBlock1) {
            lrow1[k] = p.tab.row1[k];
            linit[k] = p.tab.init[k];
        }
        __syncthreads();
        src = PuzzleSrc<1>{p.tab.info, p.tab.root, p.tab.open, linit, lrow1};
    }
    const size_t n = p.n;
    const uint32_t wg_base = blockIdx.x * 256u;
    const bool wg_full = tiled && (size_t)wg_base + 256 <= n;   // block-uniform
    const int32_t K = wg_full ? T / kTile : 0;                   // full tiles
    const uint32_t r = lane >> 2, c = (lane & 3u) * 16u;         // this lane's piece of a tile

    if (wv == 4) {                                               // ---- the I/O wave
        if (!wg_full) return;
        auto load_tile = [&](int32_t k) {                        // actions of tile k -> buffer k & 1
            if constexpr (!RAND) {
                u32x4 v[4];
#pragma unroll
                for (int w = 0; w < 4; ++w) v[w] = nt_load16(act + (size_t)(k * kTile + r) * n + wg_base + w * 64 + c);
#pragma unroll
                for (int w = 0; w < 4; ++w)
                    *reinterpret_cast<u32x4*>(smem + w * kW1Wave + (k & 1) * (kTile * 64) + r * 64 + c) = v[w];
            }
        };
        // tile k's outputs -> HBM: each store instruction covers 8 rows x 128 B (two env waves'
        // row segments), whole 128-B lines, so no partial-line writes reach HBM
        auto store_tile = [&](int32_t k) {
            const uint32_t r8 = lane >> 3, c8 = (lane & 7u) * 16u;     // row / byte of this lane
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const uint32_t row = (uint32_t)((k * kTile) & (kRing - 1)) + h * 8 + r8;
#pragma unroll
                for (int q = 0; q < 2; ++q) {
                    const int w = 2 * q + (int)(c8 >> 6);
                    const uint8_t* base = smem + w * kW1Wave + kW1Act + row * 64 + (c8 & 63u);
                    const size_t o = (size_t)(k * kTile + h * 8 + r8) * n + wg_base + q * 128 + c8;
                    if (rew) nt_store16(reinterpret_cast<uint8_t*>(rew) + o, *reinterpret_cast<const u32x4*>(base));
                    if (flg) nt_store16(flg + o, *reinterpret_cast<const u32x4*>(base + kRing * 64));
                }
            }
        };
        if (K > 0) load_tile(0);
        __syncthreads();                                         // B_0
        for (int32_t k = 0; k < K; ++k) {
            if (k + 1 < K) load_tile(k + 1);
            if (k >= 2) store_tile(k - 2);
            __syncthreads();                                     // B_{k+1}
        }
        __syncthreads();                                         // B_end
        if (K >= 2) store_tile(K - 2);
        if (K >= 1) store_tile(K - 1);
        return;
    }

    // ---- env waves
    const uint32_t i = wg_base + wv * 64u + lane;
    const bool active = i < n;
    const uint64_t gid = p.env_offset + i;
    uint8_t* wbase = smem + wv * kW1Wave;
    uint8_t* tr = wbase + kW1Act;                                // reward ring [64][64]
    uint8_t* tf = tr + kRing * 64;                               // flag ring [64][64]
    using Stack = typename std::conditional<TB, LdsStack<64>, RegStack>::type;
    Env<1, TB, Stack> e;
    if constexpr (TB) e.stk.col = tf + kRing * 64 + lane;
    int4 acc = make_int4(0, 0, 0, 0);
    if (active) {
        e.load(p, src, i);
        int c0;
        uint32_t s0;
        e.replay_outputs(c0, s0);
        acc.x -= c0;
        acc.z -= (int)s0;
    }
    auto put_rew = [&](int32_t t, int code) {                   // reward code of step t
        if (t < K * kTile) tr[(t & (kRing - 1)) * 64 + lane] = (uint8_t)code;
        else if (rew) rew[(size_t)t * n + i] = (int8_t)code;
    };
    if (wg_full) __syncthreads();                                // B_0
    for (int32_t k = 0; k < K; ++k) {
        const uint8_t* ta = wbase + (k & 1) * (kTile * 64);
#pragma unroll 1
        for (int g = 0; g < kTile; g += 4) {
            uint32_t av[4];
#pragma unroll
            for (int j = 0; j < 4; ++j)
                av[j] = RAND ? uint_rand_action(seed, gid, t0 + (uint64_t)(k * kTile + g + j)) : ta[(g + j) * 64 + lane];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int32_t t = k * kTile + g + j;
                e.reset_next(p, src);
                const int code = e.phase_trie(p);
                tr[((t - 1) & (kRing - 1)) * 64 + lane] = (uint8_t)code;   // step t-1 (t = 0: unused row)
                const uint32_t f = e.phase_move(p, av[j]);
                tf[(t & (kRing - 1)) * 64 + lane] = (uint8_t)f;
                acc.x += code;
                acc.z += (int)e.solved;
                acc.y += (int)e.pending;
                acc.w += (int)e.s_rs;
            }
        }
        __syncthreads();                                         // B_{k+1}
    }
    if (active) {
        for (int32_t t = K * kTile; t < T; ++t) {                // tail steps / partial workgroups
            const uint32_t a = RAND ? uint_rand_action(seed, gid, t0 + (uint64_t)t) : act[(size_t)t * n + i];
            e.reset_next(p, src);
            const int code = e.phase_trie(p);
            if (t > 0) put_rew(t - 1, code);
            const uint32_t f = e.phase_move(p, a);
            if (flg) flg[(size_t)t * n + i] = (uint8_t)f;
            acc.x += code;
            acc.z += (int)e.solved;
            acc.y += (int)e.pending;
            acc.w += (int)e.s_rs;
        }
        const int code = e.phase_trie(p);                        // the last step's trie phase
        put_rew(T - 1, code);
        acc.x += code;
        acc.z += (int)e.solved;
    }
    if (wg_full) __syncthreads();                                // B_end: rings complete
    if (!active) return;
    e.store(p, src, i);
    if (stats) {
        int4 st = stats[i];
        st.x += acc.x;
        st.y += acc.y;
        st.z += acc.z;
        st.w += acc.w;
        stats[i] = st;
    }
}

// ---------------------------------------------------------------------------------------------
// W = 1 rollout with each env's step split over TWO waves (k_rollout1s).
//
// A lone wave issues one instruction every ~5 cycles while its SIMD can take one every ~2.5
// from two waves, and at 65,536 envs there is exactly one 64-env wave per SIMD.  So the step is
// cut where its data flow is one-way: a MOVE wave (MoveLane1, sparc_move1.hpp) runs the
// autoreset, legality, move, path and flags and hands each env-step over to a TRIE wave as one
// 32-bit LDS word; the trie wave (TrieLane::step1) runs the solution-trie walk, the record
// gathers, the reward code and the episode counters one 16-step tile behind.  Nothing flows
// back: the reward code never feeds the move.  I/O waves stream action tiles in (the actions
// for the trie wave, each action's target window position for the move wave) and reward / flag
// tiles out (the flag bytes from the hand-over words, flag_bytes4).  Per workgroup 256 envs = 4 move waves (0-3) + 4 trie waves (4-7, on
// the same SIMDs as the move waves of their envs) + 4 I/O waves (8-11, one per SIMD); one
// barrier per tile:
//   interval k (between barriers B_k and B_k+1): move waves step tile k; trie waves finish
//   tile k-1; the I/O waves load the actions of tile k+1 and store the outputs of tile k-2.
// Only full workgroups, T % 16 == 0, 16-B aligned I/O and pitches 3..9 (split1_pitch_ok); the
// host runs any tail (and other pools) through k_rollout1.  The state after the launch is the same SoA record (the trie wave hands its
// final trie state and counters to the move wave through LDS before the store).
constexpr int kBlock1s = 768;
// steps per LDS read group of the move and trie waves: a group's inputs (target positions;
// hand-over words and actions) are read together and waited for once
constexpr int kGroup1s = 4;
static_assert(kTile % kGroup1s == 0, "k_rollout1s read groups");
constexpr size_t kS_Act = 0;                          // actions << 4 [3 tiles][16][64] (trie wave)
constexpr size_t kS_Pos = kS_Act + 3 * kTile * 64;    // target window positions [3 tiles][16][64] (move wave)
constexpr size_t kS_Rew = kS_Pos + 3 * kTile * 64;    // reward ring [64 steps][64]
constexpr size_t kS_FH = kS_Rew + kRing * 64;         // hand-over ring [64 steps][64] u32
constexpr size_t kS_Stk = kS_FH + 4 * kRing * 64;     // move stack [64 moves][64]
constexpr size_t kS_Pair = kS_Stk + 64 * 64;          // per move / trie wave pair
constexpr size_t kS_Fin = 4 * kS_Pair;                // trie wave's final state [4][64] 2 x uint4
// IOR: the final state is one uint4 per env (S, Oneg, pid) and the second half of the region holds
// the per-env counters [3][256] int32 of the I/O waves (so that c3's 1,024 staged puzzle rows
// still fit: 128 KB of tiles + 8 KB + 32 KB = 160 KB)
constexpr size_t kS_Cnt = kS_Fin + 256 * sizeof(uint4);
constexpr size_t kS_Base = kS_Fin + 4 * 64 * 2 * sizeof(uint4);
static_assert(kS_Cnt + 3 * 256 * sizeof(int32_t) <= kS_Base, "k_rollout1s IOR counters");
// LDS bytes of the staged rows: move rows + trie rows, 16 B each per puzzle
__host__ __device__ constexpr size_t split_table_bytes(uint32_t P) { return (size_t)P * 2 * sizeof(uint4); }
// LDS_TABLE = false (pools past the row budget): the trie rows' slots at kS_Base (sparc_move1.hpp)
constexpr size_t kS_SlotBytes = (kRowSlots + 1) * kRowSlotStride;
static_assert(kRowSlotStride == 256 * sizeof(uint4) && (kRowSlots & (kRowSlots - 1)) == 0, "row slots");

// four action bytes with every byte >= 4 mapped to 4 (never legal: legal bit 4 is 0), so the
// move wave tests legality with one shift
__device__ __forceinline__ uint32_t clamp_actions4(uint32_t x) {
    const uint32_t t = x & 0xFCFCFCFCu;                                   // bits that make a byte >= 4
    const uint32_t nz = (((t & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | t) & 0x80808080u;   // 0x80: byte >= 4
    const uint32_t bm = (nz >> 7) * 0xFFu;                               // 0xFF in those bytes
    return (x & ~bm) | (bm & 0x04040404u);
}

// byte b of four words, side by side (sel = 0x0C0C0400 + b * 0x0101)
__device__ __forceinline__ uint32_t bytes4(const u32x4 w, uint32_t sel) {
    return __builtin_amdgcn_perm(w.y, w.x, sel) | (__builtin_amdgcn_perm(w.w, w.z, sel) << 16);
}
// the flag bytes (term | trunc << 1 | legal << 2 | autoreset << 6) of four hand-over words of
// the W = 1 move wave (sparc_move1.hpp), four bytes side by side; magic = legal_magic(pitch).
// The legal bits: lw * magic carries the window bits right / up / left / down to bits 18..21
// (v_mul_u32_u24 reads bits 0..23 of the word: lw alone).  Byte 3 holds at-target (bit 0) and
// done (bit 1); at-target without done marks an autoreset step
__device__ __forceinline__ uint32_t flag_bytes4(const u32x4 w, uint32_t magic) {
    u32x4 m;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        uint32_t t;
        asm("v_mul_u32_u24 %0, %1, %2" : "=v"(t) : "v"(w[j]), "s"(magic));
        m[j] = t;
    }
    const uint32_t L = bytes4(m, 0x0C0C0602u) & 0x3C3C3C3Cu;          // legal << 2
    const uint32_t B = bytes4(w, 0x0C0C0703u);                         // tgt | done << 1
    const uint32_t term = B & (B >> 1) & 0x01010101u;                  // done at the target
    const uint32_t trunc = B & ~(B << 1) & 0x02020202u;                // done elsewhere
    const uint32_t rs = (B << 6) & ~(B << 5) & 0x40404040u;            // at-target, not done
    return term | trunc | L | rs;
}

// k_rollout1s<…, IOR> (next-step autoreset): the reward codes of four env-steps from their
// hand-over words w, flag bytes F (flag_bytes4) and the trie wave's class bytes tb
// (TrieLane::class_byte: class 0 on the trie, 1 on a solution, 2 off it, | hs << 2), four
// bytes side by side (SWAR).  step() 1201-1223 with Oneg = -100 at every done step (a done step
// is always followed by its autoreset step): done -> +100 on a solution else -100; moved ->
// +hs on the trie, -hs off it; else 0.  Byte counters per env: done steps (cy), +100 steps (cz),
// +1 steps (cp), -1 steps (cm); the episode reward sum is 200 cz - 100 cy + cp - cm.
struct IoCounters {
    uint32_t cy[4] = {0u, 0u, 0u, 0u}, cz[4] = {0u, 0u, 0u, 0u}, cp[4] = {0u, 0u, 0u, 0u}, cm[4] = {0u, 0u, 0u, 0u};
};
// m1: 0x01 in the bytes of the steps that moved
__device__ __forceinline__ uint32_t io_codes4m(uint32_t m1, uint32_t F, uint32_t tb, uint32_t& cy, uint32_t& cz,
                                               uint32_t& cp, uint32_t& cm) {
    const uint32_t d1 = (F | (F >> 1)) & 0x01010101u;             // terminated | truncated
    const uint32_t c2 = (tb >> 1) & 0x01010101u;                  // off the trie
    const uint32_t c1 = tb & ~(tb >> 1) & 0x01010101u;            // on a solution
    const uint32_t mh = m1 & (tb >> 2) & ~d1;                     // moved, not done, hs
    const uint32_t pl = mh & ~c2, mi = mh & c2, dz = d1 & c1;
    cy += d1;
    cz += dz;
    cp += pl;
    cm += mi;
    // selector 0: 0, 1: +1, 2: -1, 4: -100, 5: +100
    return __builtin_amdgcn_perm(0x0000649Cu, 0x00FF0100u, pl | (mi << 1) | (d1 << 2) | dz);
}
// the W = 1 hand-over words (sparc_move1.hpp): byte 3 holds fwd - pop at bits 6-7, bit 6 set iff
// the step moved
__device__ __forceinline__ uint32_t io_codes4(const u32x4 w, uint32_t F, uint32_t tb, uint32_t& cy, uint32_t& cz,
                                              uint32_t& cp, uint32_t& cm) {
    const uint32_t mv = __builtin_amdgcn_perm(w.y, w.x, 0x0C0C0703u) | (__builtin_amdgcn_perm(w.w, w.z, 0x0C0C0703u) << 16);
    return io_codes4m((mv >> 6) & 0x01010101u, F, tb, cy, cz, cp, cm);
}
// the multi-word kernel's 16-bit words (hand_word16) of four env-steps, as two dwords lo, hi:
// byte 0 the flag byte, byte 1 bits 0-1 fwd - pop + 1 (1: no move)
__device__ __forceinline__ uint32_t io_codes4w(uint32_t lo, uint32_t hi, uint32_t F, uint32_t tb, uint32_t& cy,
                                               uint32_t& cz, uint32_t& cp, uint32_t& cm) {
    const uint32_t x = __builtin_amdgcn_perm(hi, lo, 0x07050301u) ^ 0x01010101u;   // 0 iff no move
    return io_codes4m((x | (x >> 1)) & 0x01010101u, F, tb, cy, cz, cp, cm);
}
// the I/O wave's byte counters of its 16 envs (env columns col0 .. col0 + 15) into the per-env LDS
// counters cnt[3][256] (reward sum, done steps, +100 steps)
__device__ __forceinline__ void io_flush(IoCounters& ct, int32_t* cnt, uint32_t col0) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            const uint32_t y = __builtin_amdgcn_ubfe(ct.cy[j], 8u * b, 8u), z = __builtin_amdgcn_ubfe(ct.cz[j], 8u * b, 8u);
            const int32_t pm = (int32_t)__builtin_amdgcn_ubfe(ct.cp[j], 8u * b, 8u) -
                               (int32_t)__builtin_amdgcn_ubfe(ct.cm[j], 8u * b, 8u);
            const uint32_t c = col0 + 4u * j + b;
            atomicAdd(cnt + c, 200 * (int32_t)z - 100 * (int32_t)y + pm);
            atomicAdd(cnt + 256 + c, (int32_t)y);
            atomicAdd(cnt + 512 + c, (int32_t)z);
        }
    }
    ct = IoCounters{};
}

// C: mixed trie tables, compact 4-B records for tries of at most 127 nodes (TrieLaneT<true>;
// p.tab.trie8 / trow then point at trie4 / trow4)
// PR: move / trie wave pairs per workgroup (64 envs each), with PR I/O waves: 4 (256 envs, 12 waves:
// one workgroup fills a CU, its roles share the SIMDs) or 1 (64 envs, 3 waves, each on a SIMD of
// its own: for grids that leave most CUs idle, c2's 4,096 envs)
template <bool TB, bool RAND, bool LDS_TABLE, bool LA = false, bool IOR = false, bool C = false, int PR = 4>
__global__ void __launch_bounds__(192 * PR) k_rollout1s(Params p, int32_t T, const uint8_t* __restrict__ act,
                                                        uint64_t seed, uint64_t t0, int8_t* __restrict__ rew,
                                                        uint8_t* __restrict__ flg, int4* __restrict__ stats) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    const uint32_t NP = p.tab.num_puzzles;
    const uint4* mrow = p.tab.mrow;
    const uint4* trow = p.tab.trow;
    if constexpr (LDS_TABLE) {
        uint4* lm = reinterpret_cast<uint4*>(smem + kS_Base);
        uint4* lt = lm + NP;
        for (uint32_t k = threadIdx.x; k < NP; k += 192u * PR) {
            lm[k] = p.tab.mrow[k];
            lt[k] = p.tab.trow[k];
        }
        __syncthreads();
        mrow = lm;
        trow = lt;
    }
    const size_t n = p.n;
    const uint32_t wg_base = blockIdx.x * (64u * PR);
    const int32_t K = T / kTile;

    if (wv >= 2u * PR) {                                         // ---- the I/O waves
        // one per SIMD (waves 8-11), each a quarter of the streamed traffic: I/O wave j loads
        // the action tile of pair j and stores rows 8 * (j >> 1) .. + 7 of env half j & 1 of
        // the output tiles (whole 128-B lines).  With one I/O wave for all four pairs its
        // issue load sat on one SIMD (MI355X, c3: 0.468 -> 0.466 ms per launch with four)
        const uint32_t io = wv - 2u * PR;
        const uint32_t r = lane >> 2, c = (lane & 3u) * 16u;
        const uint32_t pppp = p.pitch * 0x01010101u;
        IoCounters ct;
        auto load_tile = [&](int32_t k) {                        // actions of tile k -> buffer k % 3
            if constexpr (!RAND) {
                u32x4 v = nt_load16(act + (size_t)(k * kTile + r) * n + wg_base + io * 64 + c);
                v.x = clamp_actions4(v.x);
                v.y = clamp_actions4(v.y);
                v.z = clamp_actions4(v.z);
                v.w = clamp_actions4(v.w);
                const size_t o = io * kS_Pair + (k % 3) * (kTile * 64) + r * 64 + c;
                // the trie wave's copy as action << 4 (bytes <= 4: no carry between bytes), the
                // shift of its record field (TrieLane::walk1)
                *reinterpret_cast<u32x4*>(smem + kS_Act + o) = u32x4{v.x << 4, v.y << 4, v.z << 4, v.w << 4};
                // the move wave's input: each action's target window position (byte a of
                // nbr_pos; P, the agent's own never-free bit, for the illegal action 4)
                u32x4 q;
                q.x = __builtin_amdgcn_perm(pppp, p.nbr_pos, v.x);
                q.y = __builtin_amdgcn_perm(pppp, p.nbr_pos, v.y);
                q.z = __builtin_amdgcn_perm(pppp, p.nbr_pos, v.z);
                q.w = __builtin_amdgcn_perm(pppp, p.nbr_pos, v.w);
                *reinterpret_cast<u32x4*>(smem + kS_Pos + o) = q;
            }
        };
        auto store_tile = [&](int32_t k) {                       // whole 128-B lines, as k_rollout1
            // PR = 4: I/O wave io stores rows 8 * (io >> 1) .. + 7 of env half io & 1 (pairs 2q, 2q+1);
            // PR = 1: the one I/O wave stores all 16 rows of its pair, 64 B per row
            const uint32_t r8 = PR == 4 ? lane >> 3 : lane >> 2, c8 = PR == 4 ? (lane & 7u) * 16u : (lane & 3u) * 16u;
            const uint32_t h = PR == 4 ? io >> 1 : 0u, q = PR == 4 ? io & 1u : 0u;
            const uint32_t row = (uint32_t)((k * kTile) & (kRing - 1)) + h * 8 + r8;
            const uint32_t w = 2 * q + (c8 >> 6);
            const uint8_t* base = smem + w * kS_Pair + row * 64 + (c8 & 63u);
            const size_t o = (size_t)(k * kTile + h * 8 + r8) * n + wg_base + q * 128 + c8;
            const u32x4* fh = reinterpret_cast<const u32x4*>(smem + w * kS_Pair + kS_FH + row * 256 + 4 * (c8 & 63u));
            if constexpr (IOR) {
                // the reward codes from the class bytes and hand-over words (io_codes4)
                const u32x4 tb = *reinterpret_cast<const u32x4*>(base + kS_Rew);
                u32x4 f, v;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const u32x4 hw = fh[j];
                    f[j] = flag_bytes4(hw, p.lmagic);
                    v[j] = io_codes4(hw, f[j], tb[j], ct.cy[j], ct.cz[j], ct.cp[j], ct.cm[j]);
                }
                if (rew) nt_store16(reinterpret_cast<uint8_t*>(rew) + o, v);
                if (flg) nt_store16(flg + o, f);
            } else {
                if (rew) nt_store16(reinterpret_cast<uint8_t*>(rew) + o, *reinterpret_cast<const u32x4*>(base + kS_Rew));
                if (flg) {   // the flag bytes of 16 hand-over words
                    u32x4 v;
                    v.x = flag_bytes4(fh[0], p.lmagic);
                    v.y = flag_bytes4(fh[1], p.lmagic);
                    v.z = flag_bytes4(fh[2], p.lmagic);
                    v.w = flag_bytes4(fh[3], p.lmagic);
                    nt_store16(flg + o, v);
                }
            }
        };
        // IOR: the byte counters of this lane's 16 envs into the per-env LDS counters (reward sum,
        // done steps, +100 steps), at least every 255 tiles (a lane counts one row per tile)
        auto flush_counts = [&]() {
            io_flush(ct, reinterpret_cast<int32_t*>(smem + kS_Cnt),
                     PR == 4 ? (io & 1u) * 128u + (lane & 7u) * 16u : (lane & 3u) * 16u);
        };
        if constexpr (IOR) {
            int32_t* cnt = reinterpret_cast<int32_t*>(smem + kS_Cnt);
            for (uint32_t x = io * 64u + lane; x < 3u * 256u; x += 64u * PR) cnt[x] = 0;
        }
        if (K > 0) load_tile(0);
        __syncthreads();                                         // B_0
        for (int32_t k = 0; k <= K; ++k) {
            if (k + 1 < K) load_tile(k + 1);
            if (k >= 2) {
                store_tile(k - 2);
                if constexpr (IOR)
                    if (((k - 2) & 127) == 127) flush_counts();
            }
            __syncthreads();                                     // B_{k+1}
        }
        if (K >= 1) store_tile(K - 1);
        if constexpr (IOR) flush_counts();
        __syncthreads();                                         // B_{K+2}
        return;
    }

    const uint32_t pr = wv & (PR - 1u);                          // the pair's 64 envs
    const uint32_t i = wg_base + pr * 64u + lane;
    uint8_t* pb = smem + pr * kS_Pair;
    uint4* fin = reinterpret_cast<uint4*>(smem + kS_Fin) + (IOR ? 1u : 2u) * (pr * 64u + lane);
    // LDS_TABLE = false: this env's trie-row slots (row_slots, sparc_move1.hpp)
    const uint32_t slot_addr = MoveLane1<TB>::lds_addr(smem + kS_Base + (size_t)(pr * 64u + lane) * sizeof(uint4));
    if (wv < (uint32_t)PR) {                                     // ---- move waves
        MoveLane1<TB> m;
        uint8_t* col = pb + kS_Stk + lane;
        const uint32_t col_addr = MoveLane1<TB>::lds_addr(col);
        m.load(p, i, col, col_addr);
        const uint32_t pid0 = p.st.pid[i];
        if constexpr (LDS_TABLE) m.prefetch_reset(mrow, pid0 + 1 == NP ? 0u : pid0 + 1);
        else m.prefetch_reset_g(mrow, trow, pid0 + 1 == NP ? 0u : pid0 + 1);
        const uint32_t pend0 = m.pending ? 1u : 0u;
        const bool ar = IOR || p.autoreset == 1;   // IOR kernels serve next-step autoreset only
        const uint64_t gid = p.env_offset + i;
        uint32_t* th = reinterpret_cast<uint32_t*>(pb + kS_FH) + lane;
        __syncthreads();                                         // B_0
        for (int32_t k = 0; k < K; ++k) {
            // tile k's target positions (buffer k % 3; the trie wave reads the actions one tile
            // later)
            const uint8_t* tp = pb + kS_Pos + (k % 3) * (kTile * 64) + lane;
            uint8_t* ta = pb + kS_Act + (k % 3) * (kTile * 64) + lane;
#pragma unroll 1
            for (int g = 0; g < kTile; g += kGroup1s) {
                uint32_t pv[kGroup1s];
#pragma unroll
                for (int j = 0; j < kGroup1s; ++j) {
                    if constexpr (RAND) {
                        const uint32_t a = uint_rand_action(seed, gid, t0 + (uint64_t)(k * kTile + g + j));
                        ta[(g + j) * 64] = (uint8_t)(a << 4);   // the trie wave's action << 4
                        pv[j] = __builtin_amdgcn_ubfe(p.nbr_pos, a << 3, 8u);
                    } else {
                        pv[j] = tp[(g + j) * 64];
                    }
                }
#pragma unroll
                for (int j = 0; j < kGroup1s; ++j) {
                    const uint32_t row = (uint32_t)(k * kTile + g + j) & (kRing - 1);
                    bool rs;
                    if constexpr (LDS_TABLE) rs = m.reset_next(ar, mrow, col_addr);
                    else rs = m.reset_next_g(ar, mrow, trow, col_addr, slot_addr);
                    th[row * 64] = m.step_pos(p, pv[j], rs);
                }
            }
            if constexpr (!LDS_TABLE) m.tile_end();
            __syncthreads();                                     // B_{k+1}
        }
        __syncthreads();                                         // B_{K+1}
        __syncthreads();                                         // B_{K+2}: the trie state is in fin
        uint4 fs = fin[0], fc;
        if constexpr (IOR) {   // the counters from the I/O waves (io_codes4)
            const int32_t* cnt = reinterpret_cast<const int32_t*>(smem + kS_Cnt) + pr * 64u + lane;
            fc = make_uint4((uint32_t)cnt[256], fs.z, 0u, 0u);
            fs.z = (uint32_t)cnt[0];
            fs.w = (uint32_t)cnt[512];
        } else {
            fc = fin[1];
        }
        const uint32_t pend = m.pending ? 1u : 0u;
        m.store(p, i, col, col_addr, fs.x, pend ? (fs.y == 0u ? 1u : 2u) : 0u, fc.y);
        if (stats) {
            // autoresets: one per done step before the last, plus one for a done step carried in
            const uint32_t resets = p.autoreset == 1 ? pend0 + fc.x - pend : 0u;
            int4 st = stats[i];
            st.x += (int)fs.z;
            st.y += (int)fc.x;
            st.z += (int)fs.w;
            st.w += (int)resets;
            stats[i] = st;
        }
    } else {                                                     // ---- trie waves
        // the trie wave wins VALU arbitration against its (older) move wave partner (c3: 0.289
        // -> 0.266 ms per 1,000 steps with the earlier trie wave; with TrieLane, 2,000 steps:
        // 0.456 ms, 0.476 without priority, 0.477 with the move wave at 1 instead)
        __builtin_amdgcn_s_setprio(1);
        static_assert(!(C && LA), "compact records: the plain trie wave only");
        using TL = TrieLaneT<C>;
        using Rec = typename TL::Rec;
        const Rec* trie = reinterpret_cast<const Rec*>(p.tab.trie8);
        TL tl;
        tl.load(p.st.pos[i], p.st.aux[i], p.st.pid[i], trow, trie, NP);
        const uint32_t* th = reinterpret_cast<const uint32_t*>(pb + kS_FH) + lane;
        uint8_t* tr = pb + kS_Rew + lane;
        static_assert(!(LA && RAND), "the look-ahead trie wave reads the next tile's actions from HBM tiles");
        __syncthreads();                                         // B_0
        __syncthreads();                                         // B_1 (interval 0: no tile yet)
        if constexpr (LA)
            if (K > 0) tl.prime(pb[kS_Act + lane], p.tab.trieg);   // step 0's action (tile 0, buffer 0)
        if constexpr (!LDS_TABLE) {
            tl.slot_addr = slot_addr;
            tl.lim = kRowSlots;
        }
        for (int32_t k = 1; k <= K; ++k) {
            const uint8_t* ta = pb + kS_Act + ((k - 1) % 3) * (kTile * 64) + lane;   // tile k-1's actions
            if constexpr (!LDS_TABLE) tl.slot_read(kRowSlots, kRowSlotStride);   // written in interval k-1 or before
            // LA: tile k's first action is the look-ahead of tile k-1's last step; buffer k % 3
            // holds tile k during this interval (loaded by the I/O wave in the last one; after
            // the last tile it is stale, and that look-ahead is never used)
            const uint32_t a_next = LA ? pb[kS_Act + (k % 3) * (kTile * 64) + lane] : 0u;
#pragma unroll 1
            for (int g = 0; g < kTile; g += kGroup1s) {
                // the group's hand-over words and actions (LA: and the next one) first (one LDS
                // wait), then its steps
                const uint32_t row0 = (uint32_t)((k - 1) * kTile + g) & (kRing - 1);
                uint32_t hb[kGroup1s], av[kGroup1s + 1];
#pragma unroll
                for (int j = 0; j < kGroup1s; ++j) {
                    hb[j] = th[(row0 + j) * 64];
                    av[j] = ta[(g + j) * 64];
                }
                if constexpr (LA) av[kGroup1s] = g + kGroup1s < kTile ? (uint32_t)ta[(g + kGroup1s) * 64] : a_next;
#pragma unroll
                for (int j = 0; j < kGroup1s; ++j) {
                    int code;
                    if constexpr (LA) code = tl.template step1la<!IOR>(hb[j], av[j], av[j + 1], trow, p.tab.trieg, NP);
                    else if constexpr (LDS_TABLE) code = tl.template step1<!IOR>(hb[j], av[j], trow, trie, NP);
                    else code = tl.template step1s<!IOR, kRowSlots, kRowSlotStride>(hb[j], av[j], trow, trie, NP);
                    tr[(row0 + j) * 64] = (uint8_t)code;
                }
            }
            if constexpr (!LDS_TABLE) tl.slot_tile_end(kRowSlots);
            __syncthreads();                                     // B_{k+1}
        }
        if constexpr (IOR)   // the last step's hand-over word is still in the ring
            if (K > 0) tl.finish_oneg(th[((uint32_t)(K * kTile - 1) & (kRing - 1)) * 64u] & kHwDone);
        if constexpr (IOR) {
            fin[0] = make_uint4(tl.std_S(), (uint32_t)tl.Oneg, tl.pid, 0u);
        } else {
            fin[0] = make_uint4(tl.std_S(), (uint32_t)tl.Oneg, (uint32_t)tl.acc_x, tl.acc_z);
            fin[1] = make_uint4(tl.acc_y, tl.pid, 0u, 0u);
        }
        __syncthreads();                                         // B_{K+2}
    }
}

// ---------------------------------------------------------------------------------------------
// W = 1 rollout with the rule audit after every step (k_rollout1r: sparc_rollout_rules_device on
// pools whose every puzzle has a region-code table).  The reference audits every step()
// (_validate_rules at SPaRC_Gym.py:1227, again in _get_info 1011; info['rule_status'] 941-950).
// That audit — a flood fill per region and one table lookup per region (sparc_rules.hpp) — costs
// about ten times the step and is one latency-bound dependency chain per lane, so it runs in
// waves of its own: per 64 envs one STEP wave (Env<1>::advance: the step, the stats, the outputs)
// and A AUDIT waves.  The audit waves take the workgroup's tile of env-steps in env-major order,
// a wave's 64 lanes on consecutive steps of a few envs: their regions differ by a point or two,
// so the lanes' flood fills run nearly in lock step (MI355X, c3r: 3.97 -> 2.97 ms per 2,000-step
// launch against lanes on 64 envs at one step; profiles/r06/ab_c3r_em).  Nothing is computed
// twice and no audit wave carries step state.
//   The step wave hands every env-step over as one u64 and one u32 in LDS rings: the visited
// board (the bits below kRingShift: every W = 1 pool with x_size * pitch <= 57) | the agent's bit
// << 57, and the puzzle index after the step.  An audit lane keeps the rule row of its last
// job's puzzle in registers (a job of another puzzle reloads it from the L2).  The step wave is
// pipelined as k_rollout1's env waves (the trie phase of step t-1 next to the move phase of step
// t), and keeps the reset board of its env's puzzle for the visited plane, so its tile of steps
// stays shorter than the audit waves' (MI355X: with the fused step and the path rules moved onto
// it, it was the longer chain, 1,890 cycles per step against 840 per audit and audit wave).
//   Per workgroup 64 * G envs = G step waves (0..G-1) + G * A audit waves (group g = wave % G);
// tiles of RT steps, one barrier per tile.  In interval k the step waves step tile k and store
// the rewards / flags and the rule bits of tile k-2 (whole 16-B pieces of the workgroup's rows;
// three reward / flag buffers, as tile k-1's last reward code is written in interval k), the
// audit waves audit tile k-1.  Only the step waves read and write the env state.
// Shape <G, A, RT>: G 64-env groups per workgroup, A audit waves per group (so G * (1 + A) waves
// <= 16), RT steps per tile (a multiple of A: RT / A audits per audit lane and tile).
template <int G, int A, int RT>
struct R1Geom {
    static_assert(G * (1 + A) <= 16 && RT % A == 0, "k_rollout1r shape");
    static constexpr int kBlock = 64 * G * (1 + A);
    static constexpr uint32_t kEnvs = 64u * G;                            // envs per workgroup (a tile row)
    static constexpr size_t kRing = 0;                                      // [2][RT][kEnvs] u64
    static constexpr size_t kPid = kRing + 2 * RT * kEnvs * 8;             // [2][RT][kEnvs] u32 puzzle index
    static constexpr size_t kRew = kPid + 2 * RT * kEnvs * 4;              // [3][RT][kEnvs] reward codes
    static constexpr size_t kFlg = kRew + 3 * RT * kEnvs;                  // [3][RT][kEnvs] flags
    static constexpr size_t kBits = kFlg + 3 * RT * kEnvs;                 // [2][RT][kEnvs] u16 rule bits
    static constexpr size_t kAct = kBits + 2 * RT * kEnvs * 2;             // [G][RT][64] actions of the tile
    static constexpr size_t kStk = kAct + G * RT * 64;                     // [G][64 moves][64] move stacks
    static constexpr size_t kSimple = kStk + (size_t)G * 64 * 64;          // [512] ring_simple (INC audits)
    static constexpr size_t kBase = kSimple + 512;                         // then the W = 1 puzzle rows
};
constexpr uint32_t kRingShift = 57;

// INC: incremental audits (RegionSet1, sparc_rules.hpp): audit wave q takes the steps of the
// q-th block of RT / A consecutive steps of each tile in order, keeping the env's regions from
// one step to the next (A = 1: across tiles too, so a full flood only after a reset or a puzzle
// change; A > 1: one full flood at the start of each block).
// amdgpu_waves_per_eu(6): two 12-wave workgroups per CU (3 waves per SIMD each).  Left to itself
// the compiler takes 92 VGPRs (5 waves per SIMD, one workgroup per CU: 0.145 ms per 50-step launch
// against 0.121 ms with 80 VGPRs and 24 B of scratch touched once per tile).
template <bool TB, bool RAND, bool LDS_TABLE, int G, int A, int RT, bool INC = false, int WPE = 6>
__global__ void __launch_bounds__(64 * G * (1 + A)) __attribute__((amdgpu_waves_per_eu(WPE)))
    k_rollout1r(Params p, int32_t T, const uint8_t* __restrict__ act, uint64_t seed, uint64_t t0,
                int8_t* __restrict__ rew, uint8_t* __restrict__ flg, int4* __restrict__ stats, uint32_t tiled,
                RulesTab rt, uint16_t* __restrict__ bits) {
    using Geo = R1Geom<G, A, RT>;
    constexpr uint32_t E = Geo::kEnvs;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    const uint32_t g = wv % (uint32_t)G;                         // the wave's 64-env group
    const size_t n = p.n;
    const uint32_t wg_base = blockIdx.x * E;
    const uint32_t col = g * 64u + lane;                         // the env's column in a tile row
    const uint32_t i = wg_base + col;
    const bool active = i < n;
    const bool full = tiled && (size_t)wg_base + E <= n;         // block-uniform: 16-B row pieces
    const int32_t K = (T + RT - 1) / RT;
    uint64_t* ring = reinterpret_cast<uint64_t*>(smem + Geo::kRing);
    uint32_t* rpid = reinterpret_cast<uint32_t*>(smem + Geo::kPid);
    uint8_t* trw = smem + Geo::kRew;
    uint8_t* tfl = smem + Geo::kFlg;
    uint16_t* tbt = reinterpret_cast<uint16_t*>(smem + Geo::kBits);
    auto at = [](uint32_t b, int32_t j, uint32_t c) { return (b * (uint32_t)RT + (uint32_t)j) * E + c; };
    auto tile_cnt = [&](int32_t k) { return T - k * RT < RT ? T - k * RT : RT; };
    PuzzleSrc<1> src{p.tab.info, p.tab.root, p.tab.open, p.tab.init, p.tab.row1};
    if constexpr (INC) {   // read by the audit waves after B_1
        for (uint32_t k = threadIdx.x; k < 512u; k += Geo::kBlock) smem[Geo::kSimple + k] = (uint8_t)ring_simple(k);
    }
    if constexpr (LDS_TABLE) {
        const uint32_t P = p.tab.num_puzzles;
        uint4* lrow1 = reinterpret_cast<uint4*>(smem + Geo::kBase);
        uint64_t* linit = reinterpret_cast<uint64_t*>(lrow1 + P);
        for (uint32_t k = threadIdx.x; k < P; k += Geo::kBlock) {
            lrow1[k] = p.tab.row1[k];
            linit[k] = p.tab.init[k];
        }
        __syncthreads();
        src = PuzzleSrc<1>{p.tab.info, p.tab.root, p.tab.open, linit, lrow1};
    }

    if (wv < (uint32_t)G) {                                      // ---- step waves
        using Stack = typename std::conditional<TB, LdsStack<64>, RegStack>::type;
        Env<1, TB, Stack> e;
        if constexpr (TB) e.stk.col = smem + Geo::kStk + g * 4096u + lane;
        int4 acc = make_int4(0, 0, 0, 0);
        // the visited plane after a step is (free board at reset & ~free board now) | start: the
        // reset board and start bit of the env's puzzle, kept from its last reset
        uint64_t initc = 0;
        uint32_t sbit = 0;
        if (active) {
            e.load(p, src, i);
            // the step is pipelined as in k_rollout1: iteration t runs the trie phase of step
            // t-1 next to the move phase of step t, so the trie-record gather of one step has a
            // whole step to arrive; iteration 0's trie phase replays the stored step (its
            // outputs are subtracted from the stats)
            int c0;
            uint32_t s0;
            e.replay_outputs(c0, s0);
            acc.x -= c0;
            acc.z -= (int)s0;
            initc = src.get_init(e.pid);
            sbit = src.get_row1(e.pid).x & 0xFFu;
        }
        const uint64_t gid = p.env_offset + i;
        uint8_t* ta = smem + Geo::kAct + g * (RT * 64u);
        const uint32_t r = lane >> 2, c = (lane & 3u) * 16u;    // this lane's 16-B piece of an action tile
        const bool tact = !RAND && full;                         // actions through the tile prefetch
        u32x4 anext = {0u, 0u, 0u, 0u};
        if (tact && (int32_t)r < tile_cnt(0)) anext = nt_load16(act + (size_t)r * n + wg_base + g * 64u + c);
        // tile kt's rewards / flags, or rule bits, from LDS to HBM by the E step-wave lanes
        auto store_rf = [&](int32_t kt) {   // (reward / flag tiles: buffer kt % 3)
            const int32_t cnt = tile_cnt(kt);
            const uint32_t b = (uint32_t)kt % 3u;
            if (full) {
                constexpr uint32_t kPer = E / 16u;               // 16-B pieces per row
                for (uint32_t pi = col; pi < kPer * (uint32_t)cnt; pi += E) {
                    const uint32_t row = pi / kPer, cb = (pi % kPer) * 16u;
                    const size_t o = (size_t)(kt * RT + (int32_t)row) * n + wg_base + cb;
                    if (rew) nt_store16(reinterpret_cast<uint8_t*>(rew) + o, *reinterpret_cast<const u32x4*>(trw + at(b, (int32_t)row, cb)));
                    if (flg) nt_store16(flg + o, *reinterpret_cast<const u32x4*>(tfl + at(b, (int32_t)row, cb)));
                }
            } else if (active) {
                for (int32_t j = 0; j < cnt; ++j) {
                    const size_t o = (size_t)(kt * RT + j) * n + i;
                    if (rew) rew[o] = (int8_t)trw[at(b, j, col)];
                    if (flg) flg[o] = tfl[at(b, j, col)];
                }
            }
        };
        auto store_bits = [&](int32_t kt) {
            const int32_t cnt = tile_cnt(kt);
            const uint32_t b = (uint32_t)kt & 1u;
            if (full) {
                constexpr uint32_t kPer = E / 8u;                // 16-B pieces (8 entries) per row
                for (uint32_t pi = col; pi < kPer * (uint32_t)cnt; pi += E) {
                    const uint32_t row = pi / kPer, ce = (pi % kPer) * 8u;
                    const size_t o = (size_t)(kt * RT + (int32_t)row) * n + wg_base + ce;
                    nt_store16(reinterpret_cast<uint8_t*>(bits + o), *reinterpret_cast<const u32x4*>(tbt + at(b, (int32_t)row, ce)));
                }
            } else if (active) {
                for (int32_t j = 0; j < cnt; ++j) bits[(size_t)(kt * RT + j) * n + i] = tbt[at(b, j, col)];
            }
        };
        __syncthreads();                                         // B_0
        for (int32_t k = 0; k < K; ++k) {
            const int32_t cnt = tile_cnt(k);
            const uint32_t b = (uint32_t)k & 1u;
            if (tact) {
                const u32x4 acur = anext;
                if (k + 1 < K && (int32_t)r < tile_cnt(k + 1))
                    anext = nt_load16(act + (size_t)((k + 1) * RT + (int32_t)r) * n + wg_base + g * 64u + c);
                if ((int32_t)r < cnt) *reinterpret_cast<u32x4*>(ta + r * 64u + c) = acur;
                wave_lds_fence();
            }
#pragma unroll 1
            for (int32_t j = 0; j < cnt; ++j) {
                const int32_t t = k * RT + j;
                uint32_t a = 0;
                if constexpr (RAND) a = uint_rand_action(seed, gid, t0 + (uint64_t)t);
                else if (tact) a = ta[j * 64 + (int32_t)lane];
                else if (active) a = act[(size_t)t * n + i];
                uint32_t f = 0;
                uint64_t w = 0;
                uint32_t q_after = 0;
                if (active) {
                    e.reset_next(p, src);                        // step t's autoreset: rows and board
                    if (e.rs) {
                        initc = e.fr;
                        sbit = e.e;
                    }
                    const int code = e.phase_trie(p);            // step t-1
                    f = e.phase_move(p, a);                      // step t
                    acc.x += code;
                    acc.z += (int)e.solved;
                    acc.y += (int)e.pending;
                    acc.w += (int)e.s_rs;
                    if (t > 0) {                                 // step t-1's reward code
                        const int32_t tp = t - 1;
                        trw[((uint32_t)(tp / RT) % 3u * (uint32_t)RT + (uint32_t)(tp % RT)) * E + col] = (uint8_t)code;
                    }
                    w = (((initc & ~e.fr) >> p.pitch) | (1ull << sbit)) | ((uint64_t)e.e << kRingShift);
                    q_after = e.pid;
                }
                ring[at(b, j, col)] = w;
                rpid[at(b, j, col)] = q_after;
                tfl[((uint32_t)k % 3u * (uint32_t)RT + (uint32_t)j) * E + col] = (uint8_t)f;
            }
            // interval k stores the rewards / flags of tile k-2 (tile k-1's last reward code is
            // written in this interval) and the rule bits of tile k-2 (audited in interval k-1)
            if (k >= 2) {
                store_rf(k - 2);
                store_bits(k - 2);
            }
            __syncthreads();                                     // B_{k+1}
        }
        if (active) {                                            // the last step's trie phase
            const int code = e.phase_trie(p);
            acc.x += code;
            acc.z += (int)e.solved;
            const int32_t tp = T - 1;
            trw[((uint32_t)(tp / RT) % 3u * (uint32_t)RT + (uint32_t)(tp % RT)) * E + col] = (uint8_t)code;
        }
        if (K >= 2) {                                            // interval K: the last tile's audits run
            store_rf(K - 2);
            store_bits(K - 2);
        }
        __syncthreads();                                         // B_{K+1}
        store_rf(K - 1);
        store_bits(K - 1);
        if (!active) return;
        e.store(p, src, i);
        if (stats) {
            int4 st = stats[i];
            st.x += acc.x;
            st.y += acc.y;
            st.z += acc.z;
            st.w += acc.w;
            stats[i] = st;
        }
        return;
    }

    // ---- audit waves
    // the audit waves set the pace (the step waves alone: 1.30 ms per 2,000-step launch), so they
    // win VALU arbitration against their step wave (MI355X, c3r: 2.72 -> 2.58 ms per launch,
    // profiles/r06/ab_c3r_flood)
    __builtin_amdgcn_s_setprio(1);
    const uint32_t q = wv / (uint32_t)G - 1u;                    // audits the steps t % A == q (INC: block q)
    PuzzleRules<1> pr;
    pr.q = 0xFFFFFFFFu;
    __syncthreads();                                             // B_0
    __syncthreads();                                             // B_1 (interval 0: no tile yet)
    if constexpr (INC) {
        constexpr int32_t BL = RT / A;                           // steps per block
        const uint8_t* simple = smem + Geo::kSimple;
        RegionSet1 rs;
        for (int32_t k = 1; k <= K; ++k) {
            const int32_t kt = k - 1, cnt = tile_cnt(kt);
            const uint32_t b = (uint32_t)kt & 1u;
            const int32_t j0 = (int32_t)q * BL, j1 = j0 + BL < cnt ? j0 + BL : cnt;
            if (A > 1) rs.q = 0xFFFFFFFFu;                       // the block's first step: a full flood
#pragma unroll 1
            for (int32_t j = j0; j < j1; ++j) {
                const uint64_t w = ring[at(b, j, col)];
                const uint32_t pid = rpid[at(b, j, col)];
                uint32_t out = 0;
                if (active) {
                    if (pr.q != pid) pr = puzzle_rules<1>(p, rt, pid);
                    const uint32_t ab = (uint32_t)(w >> kRingShift) & 63u;
                    out = rs.audit(p, rt, pr, w & ((1ull << kRingShift) - 1ull), ab == pr.tbit, simple);
                }
                tbt[at(b, j, col)] = (uint16_t)out;
            }
            __syncthreads();                                     // B_{k+1}
        }
        return;
    }
    // The tile's RT * E audits in env-major order (job J: env column J / RT, step J % RT), the 64
    // lanes of a wave on 64 consecutive jobs: the consecutive steps of a few envs, whose regions
    // differ by a point or two, so the lanes' flood fills and region counts run nearly in lock
    // step (tools/audit_lockstep_sim.py, random walks on 7 x 7 lattices: 15.7 lock-step flood
    // iterations per wave-audit against 22.8 with a wave's lanes on 64 envs at one step)
    constexpr uint32_t kSlots = (uint32_t)(A * G) * 64u;         // audit lanes per workgroup
    const uint32_t s0 = (wv - (uint32_t)G) * 64u + lane;         // this lane's first job
    (void)q;
    for (int32_t k = 1; k <= K; ++k) {
        const int32_t kt = k - 1, cnt = tile_cnt(kt);
        const uint32_t b = (uint32_t)kt & 1u;
#pragma unroll 1
        for (uint32_t J = s0; J < (uint32_t)RT * E; J += kSlots) {   // RT / A jobs per lane
            const uint32_t ec = J / (uint32_t)RT, jj = J - ec * (uint32_t)RT;
            const int32_t j = (int32_t)jj;
            if (j >= cnt) continue;                               // a partial last tile
            const uint64_t w = ring[at(b, j, ec)];
            const uint32_t pid = rpid[at(b, j, ec)];
            uint32_t out = 0;
            if (wg_base + ec < n) {
                if (pid != pr.q) pr = puzzle_rules<1>(p, rt, pid);
                BB<1> vb;
                vb.w[0] = w & ((1ull << kRingShift) - 1ull);
                const uint32_t ab = (uint32_t)(w >> kRingShift) & 63u;
                out = audit_r<1, NoMemo, true>(p, rt, pr, vb, ab == pr.tbit, nullptr, nullptr).bits;
            }
            tbt[at(b, j, ec)] = (uint16_t)out;
        }
        __syncthreads();                                         // B_{k+1}
    }
}

// ---------------------------------------------------------------------------------------------
// Multi-word split rollout (k_rolloutWs, W = 2 / 4: lattices of 9x9 to 15x15 points).  The same
// wave roles and tile schedule as k_rollout1s: per workgroup 256 envs = 4 move waves
// (MoveLaneW, sparc_movew.hpp: the free board in LDS) + 4 trie waves (TrieLane, the same as
// W = 1) + 4 I/O waves; 16-bit hand-over words.  LDS per pair (SplitGeom, runtime):
//   actions [2][16][64] B | reward ring [64][64] B | hand-over ring [64][64] u16 |
//   boards [BS][64] u32 | move stacks [M][64] B
// then the trie waves' final state [4][64] 2 x uint4 and, when it fits, the trie rows.
constexpr size_t kW_Act = 0, kW_Rew = 2 * kTile * 64, kW_Hand = kW_Rew + kRing * 64, kW_Board = kW_Hand + 2 * kRing * 64;
__host__ __device__ constexpr size_t splitw_fin_bytes() { return 4 * 64 * 2 * sizeof(uint4); }

template <int W, bool TB, bool RAND, bool LDS_TABLE, bool IOR = false>
__global__ void __launch_bounds__(kBlock1s) k_rolloutWs(Params p, SplitGeom g, const uint4* __restrict__ mrow,
                                                        const uint32_t* __restrict__ boards, int32_t T,
                                                        const uint8_t* __restrict__ act, uint64_t seed, uint64_t t0,
                                                        int8_t* __restrict__ rew, uint8_t* __restrict__ flg,
                                                        int4* __restrict__ stats) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    const uint32_t NP = p.tab.num_puzzles;
    const size_t fin_off = 4 * (size_t)g.pair;
    const uint4* trow = p.tab.trow;
    if constexpr (LDS_TABLE) {
        uint4* lt = reinterpret_cast<uint4*>(smem + fin_off + splitw_fin_bytes());
        for (uint32_t k = threadIdx.x; k < NP; k += kBlock1s) lt[k] = p.tab.trow[k];
        __syncthreads();
        trow = lt;
    }
    const size_t n = p.n;
    const uint32_t wg_base = blockIdx.x * 256u;
    const int32_t K = T / kTile;

    // IOR (as k_rollout1s): the final state one uint4 per env, the counters in the second half
    int32_t* const cnt = reinterpret_cast<int32_t*>(smem + fin_off + 256 * sizeof(uint4));
    if (wv >= 8) {                                               // ---- the I/O waves (as k_rollout1s)
        const uint32_t io = wv - 8u;
        const uint32_t r = lane >> 2, c = (lane & 3u) * 16u;
        IoCounters ct;
        auto load_tile = [&](int32_t k) {
            if constexpr (!RAND) {
                const u32x4 v = nt_load16(act + (size_t)(k * kTile + r) * n + wg_base + io * 64 + c);
                *reinterpret_cast<u32x4*>(smem + io * g.pair + kW_Act + (k & 1) * (kTile * 64) + r * 64 + c) = v;
            }
        };
        auto store_tile = [&](int32_t k) {
            const uint32_t r8 = lane >> 3, c8 = (lane & 7u) * 16u;
            const uint32_t h = io >> 1, q = io & 1u;
            const uint32_t row = (uint32_t)((k * kTile) & (kRing - 1)) + h * 8 + r8;
            const uint32_t w = 2 * q + (c8 >> 6);
            const uint8_t* base = smem + w * g.pair + row * 64 + (c8 & 63u);
            const size_t o = (size_t)(k * kTile + h * 8 + r8) * n + wg_base + q * 128 + c8;
            const u32x4* fh = reinterpret_cast<const u32x4*>(smem + w * g.pair + kW_Hand + row * 128 + 2 * (c8 & 63u));
            if constexpr (IOR) {
                const u32x4 a = fh[0], b = fh[1];
                const u32x4 tb = *reinterpret_cast<const u32x4*>(base + kW_Rew);
                u32x4 f, v;
                f.x = __builtin_amdgcn_perm(a.y, a.x, 0x06040200u);
                f.y = __builtin_amdgcn_perm(a.w, a.z, 0x06040200u);
                f.z = __builtin_amdgcn_perm(b.y, b.x, 0x06040200u);
                f.w = __builtin_amdgcn_perm(b.w, b.z, 0x06040200u);
                v.x = io_codes4w(a.x, a.y, f.x, tb.x, ct.cy[0], ct.cz[0], ct.cp[0], ct.cm[0]);
                v.y = io_codes4w(a.z, a.w, f.y, tb.y, ct.cy[1], ct.cz[1], ct.cp[1], ct.cm[1]);
                v.z = io_codes4w(b.x, b.y, f.z, tb.z, ct.cy[2], ct.cz[2], ct.cp[2], ct.cm[2]);
                v.w = io_codes4w(b.z, b.w, f.w, tb.w, ct.cy[3], ct.cz[3], ct.cp[3], ct.cm[3]);
                if (rew) nt_store16(reinterpret_cast<uint8_t*>(rew) + o, v);
                if (flg) nt_store16(flg + o, f);
            } else {
                if (rew) nt_store16(reinterpret_cast<uint8_t*>(rew) + o, *reinterpret_cast<const u32x4*>(base + kW_Rew));
                if (flg) {   // byte 0 of 16 u16 hand-over words
                    const u32x4 a = fh[0], b = fh[1];
                    u32x4 v;
                    v.x = __builtin_amdgcn_perm(a.y, a.x, 0x06040200u);
                    v.y = __builtin_amdgcn_perm(a.w, a.z, 0x06040200u);
                    v.z = __builtin_amdgcn_perm(b.y, b.x, 0x06040200u);
                    v.w = __builtin_amdgcn_perm(b.w, b.z, 0x06040200u);
                    nt_store16(flg + o, v);
                }
            }
        };
        if constexpr (IOR)
            for (uint32_t x = io * 64u + lane; x < 3u * 256u; x += 256u) cnt[x] = 0;
        if (K > 0) load_tile(0);
        __syncthreads();                                         // B_0
        for (int32_t k = 0; k <= K; ++k) {
            if (k + 1 < K) load_tile(k + 1);
            if (k >= 2) {
                store_tile(k - 2);
                if constexpr (IOR)
                    if (((k - 2) & 127) == 127) io_flush(ct, cnt, (io & 1u) * 128u + (lane & 7u) * 16u);
            }
            __syncthreads();                                     // B_{k+1}
        }
        if (K >= 1) store_tile(K - 1);
        if constexpr (IOR) io_flush(ct, cnt, (io & 1u) * 128u + (lane & 7u) * 16u);
        __syncthreads();                                         // B_{K+2}
        return;
    }

    const uint32_t pr = wv & 3u;
    const uint32_t i = wg_base + pr * 64u + lane;
    uint8_t* pb = smem + pr * g.pair;
    uint4* fin = reinterpret_cast<uint4*>(smem + fin_off) + (IOR ? 1u : 2u) * (pr * 64u + lane);
    if (wv < 4) {                                                // ---- move waves
        MoveLaneW<TB> m;
        m.bd = reinterpret_cast<uint32_t*>(pb + g.off_board) + lane;
        m.col = pb + g.off_stack + lane;
        m.template load<W>(p, g, mrow, i);
        m.prefetch_next(p, g, mrow, boards);
        const uint32_t pend0 = m.pending;
        const uint64_t gid = p.env_offset + i;
        uint16_t* th = reinterpret_cast<uint16_t*>(pb + kW_Hand) + lane;
        __syncthreads();                                         // B_0
        for (int32_t k = 0; k < K; ++k) {
            const uint8_t* ta = pb + kW_Act + (k & 1) * (kTile * 64) + lane;
#pragma unroll 1
            for (int gq = 0; gq < kTile; gq += 4) {
                uint32_t av[4];
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    av[j] = RAND ? uint_rand_action(seed, gid, t0 + (uint64_t)(k * kTile + gq + j)) : ta[(gq + j) * 64];
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const uint32_t row = (uint32_t)(k * kTile + gq + j) & (kRing - 1);
                    m.reset_next(p, g, mrow, boards);
                    const uint32_t f = m.phase_move(p, g, av[j]);
                    th[row * 64] = (uint16_t)hand_word16(m.s_a, m.s_fwd, m.s_pop, f);
                }
            }
            __syncthreads();                                     // B_{k+1}
        }
        __syncthreads();                                         // B_{K+1}
        __syncthreads();                                         // B_{K+2}: the trie state is in fin
        uint4 fs = fin[0], fc;
        if constexpr (IOR) {   // the counters from the I/O waves (io_codes4w)
            const uint32_t col = pr * 64u + lane;
            fc = make_uint4((uint32_t)cnt[256 + col], 0u, 0u, 0u);
            fs.z = (uint32_t)cnt[col];
            fs.w = (uint32_t)cnt[512 + col];
        } else {
            fc = fin[1];
        }
        m.template store<W>(p, g, i, fs.x, m.pending ? (fs.y == 0u ? 1u : 2u) : 0u);
        if (stats) {
            const uint32_t resets = p.autoreset == 1 ? pend0 + fc.x - m.pending : 0u;
            int4 st = stats[i];
            st.x += (int)fs.z;
            st.y += (int)fc.x;
            st.z += (int)fs.w;
            st.w += (int)resets;
            stats[i] = st;
        }
    } else {                                                     // ---- trie waves
        // no priority here: with the board in LDS the move wave's chain is the longer one
        // (MI355X, c3g7: 0.613 ms per 2,000-step launch with the trie wave at s_setprio 1,
        // 0.558 without, 0.561 with the move wave at 1)
        TrieLane tl;
        tl.load(p.st.pos[i], p.st.aux[i], p.st.pid[i], trow, p.tab.trie8, NP);
        const uint16_t* th = reinterpret_cast<const uint16_t*>(pb + kW_Hand) + lane;
        uint8_t* tr = pb + kW_Rew + lane;
        __syncthreads();                                         // B_0
        __syncthreads();                                         // B_1
        for (int32_t k = 1; k <= K; ++k) {
#pragma unroll 1
            for (int gq = 0; gq < kTile; gq += 4) {
                const uint32_t row0 = (uint32_t)((k - 1) * kTile + gq) & (kRing - 1);
                uint32_t hb[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) hb[j] = th[(row0 + j) * 64];
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    tr[(row0 + j) * 64] = (uint8_t)tl.step<!IOR>(widen_hand_word(hb[j]), __builtin_amdgcn_ubfe(hb[j], 10u, 2u),
                                                                 trow, p.tab.trie8, NP);
            }
            __syncthreads();                                     // B_{k+1}
        }
        if constexpr (IOR) {   // the last step's hand-over word is still in the ring
            if (K > 0) tl.finish_oneg(th[((uint32_t)(K * kTile - 1) & (kRing - 1)) * 64u] & 3u);
            fin[0] = make_uint4(tl.S, (uint32_t)tl.Oneg, 0u, 0u);
        } else {
            fin[0] = make_uint4(tl.S, (uint32_t)tl.Oneg, (uint32_t)tl.acc_x, tl.acc_z);
            fin[1] = make_uint4(tl.acc_y, 0u, 0u, 0u);
        }
        __syncthreads();                                         // B_{K+2}
    }
}

template <int W>
__global__ void __launch_bounds__(kBlock) k_obs_pack(Params p, int32_t* __restrict__ vis_out,
                                                     int32_t* __restrict__ agent_out, uint32_t xd, uint32_t yd) {
    const size_t o = (size_t)blockIdx.x * kBlock + threadIdx.x;
    const size_t per = (size_t)xd * yd;
    if (o >= per * p.n) return;
    const uint32_t i = (uint32_t)(o / per);
    const uint32_t c = (uint32_t)(o - (size_t)i * per);
    const uint32_t x = c / yd, y = c - x * yd;
    const uint32_t ps = p.st.pos[i];
    int32_t v = 0;
    if (y < p.pitch) {
        const uint32_t b = x * p.pitch + y;
        if (b < 64u * W) v = (int32_t)((p.st.vis[(size_t)(b >> 6) * p.n + i] >> (b & 63)) & 1ull);
    }
    if (vis_out) vis_out[o] = v;
    if (agent_out) agent_out[o] = (x == (ps & 0xFFu) && y == ((ps >> 8) & 0xFFu)) ? 1 : 0;
}

template <int W>
__global__ void __launch_bounds__(kBlock) k_rules(Params p, RulesTab rt, uint16_t* __restrict__ bits,
                                                  uint8_t* __restrict__ region, uint64_t* __restrict__ fit,
                                                  FitMemo<kMemo>* __restrict__ memos) {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= p.n) return;
    const uint32_t q = p.st.pid[i];
    if (q >= rt.num_puzzles) {
        atomicOr(p.err, (int)kErrRuleTable);
        return;
    }
    BB<W> vis;
    for (int k = 0; k < W; ++k) vis.w[k] = p.st.vis[(size_t)k * p.n + i];
    const uint32_t ps = p.st.pos[i];
    uint8_t* ro = region ? region + (size_t)i * 64 * W : nullptr;
    if (ro)
        for (int k = 0; k < 64 * W; ++k) ro[k] = 0xFF;
    // the env's exact-fit memo: the reference audits every step() (SPaRC_Gym.py:1227), and
    // consecutive states share most regions
    FitMemo<kMemo> memo = memos[i];
    const RuleOut<W> r = audit<W>(p, rt, puzzle_rules<W>(p, rt, q), vis, ps & 0xFFu, (ps >> 8) & 0xFFu, ro, &memo, i);
    memos[i] = memo;
    if (bits) bits[i] = (uint16_t)r.bits;
    if (fit) fit[i] = r.fit_ok;
}

// the region-code table (sparc_rules.hpp region_table_word): one word per (puzzle, mask group)
// (exhausted: the number of codes whose exact-fit search passed the node cap, which the host then
// finishes, sparc_load_rules)
template <int W>
__global__ void __launch_bounds__(kBlock) k_region_table(Params p, RulesTab rt, const uint2* __restrict__ items,
                                                         uint32_t count, uint32_t* __restrict__ tab,
                                                         unsigned long long* __restrict__ exhausted) {
    const uint32_t k = blockIdx.x * kBlock + threadIdx.x;
    if (k >= count) return;
    const uint2 it = items[k];
    const uint32_t w = region_table_word<W>(p, rt, it.x, it.y);
    tab[rt.reg_off[it.x] / 8u + it.y] = w;
    uint32_t ex = 0;
    for (uint32_t j = 0; j < 8; ++j) ex += ((w >> (4u * j + kRcPolyShift)) & 3u) == 3u ? 1u : 0u;
    if (ex) atomicAdd(exhausted, (unsigned long long)ex);
}

// sparc_rules_finish's corrections of one output entry: rule bits &= ~clear, fit |= fit_or (the
// host ran the queued exact-fit searches; every entry appears once)
struct RulePatch {
    uint64_t pos, fit_or;
    uint32_t clear, pad;
};
__global__ void __launch_bounds__(kBlock) k_rule_patch(const RulePatch* __restrict__ pt, uint32_t count,
                                                       uint16_t* __restrict__ bits, uint64_t* __restrict__ fit) {
    const uint32_t k = blockIdx.x * kBlock + threadIdx.x;
    if (k >= count) return;
    const RulePatch r = pt[k];
    bits[r.pos] = (uint16_t)(bits[r.pos] & ~r.clear);
    if (fit && r.fit_or) fit[r.pos] |= r.fit_or;
}

// ------------------------------------------------------------------------------ host side
// The last audit call that may queue exact-fit searches (sparc_rules_finish): its outputs and
// extent (entries: N, or T * N), and for a generic rule rollout its launch, so that a call whose
// queue overflowed runs again on a larger queue from the state it started from (Ctx::snap).
struct AuditCall {
    int kind = 0;   // 0 none, 1 sparc_rules_device, 2 rule rollout
    bool snap = false;   // kind 2: the generic rule kernel ran it from a snapshot (re-runnable)
    uint64_t extent = 0;
    uint16_t* bits = nullptr;
    uint8_t* region = nullptr;
    uint64_t* fit = nullptr;
    int32_t T = 0;
    const uint8_t* act = nullptr;
    uint64_t seed = 0, t0 = 0;
    int8_t* rew = nullptr;
    uint8_t* flags = nullptr;
    int32_t* stats = nullptr;
};

struct Ctx {
    sparc_config cfg{};
    int device = 0;
    hipStream_t own = nullptr, stream = nullptr;
    uint32_t n = 0;
    int W = 1;
    bool loaded = false, has_state = false;
    uint32_t num_puzzles = 0, num_nodes = 0;
    std::vector<uint32_t> h_info;      // host copy of the loaded table's info rows [P][4]
    // device buffers
    uint64_t *vis = nullptr, *dirs = nullptr;
    uint32_t *pos = nullptr, *aux = nullptr, *step = nullptr, *pid = nullptr;
    uint64_t* t_open = nullptr;
    uint4 *t_info = nullptr, *t_root = nullptr, *t_trie = nullptr;
    uint64_t* t_init = nullptr;
    uint4* t_row1 = nullptr;
    uint2* t_trie8 = nullptr;          // split-kernel tables (null: a puzzle's trie exceeds 15-bit nodes)
    uint2* t_trieg = nullptr;          // [nodes][4]: the record of each node's field-d node (k_rollout1s)
    // mixed split tables (sparc_trie.hpp TrieLaneT<true>): 4-B records for tries of at most 127
    // nodes, 8-B ones for the rest, byte-addressed, and their trie rows; taken by k_rollout1s on
    // pools past the LDS row budget
    uint8_t* t_trie4 = nullptr;
    uint4* t_trow4 = nullptr;
    bool mixed_pays = false;   // the 8-B records outgrow an XCD's L2 (sparc_load_puzzles, sparc_reset_host)
    std::vector<uint32_t> nodes8;   // W = 1: trie nodes (8-B records) per puzzle, for the XCD hot set
    int mixed_trie = 0;        // SPARC_VARIANT_MIXED_TRIE: 0 when it pays, 1 always, 2 never
    uint4 *t_trow = nullptr, *t_mrow = nullptr;
    // multi-word split kernel (k_rolloutWs): move rows and reset boards; split_w false when the
    // pool does not fit its layout (pitch > 15, LDS, or no trie8)
    uint4* t_mroww = nullptr;
    uint32_t* t_boardw = nullptr;
    SplitGeom sgeom{};
    bool split_w = false;
    int32_t* err = nullptr;
    uint8_t *s_act = nullptr, *s_flags = nullptr, *s_mask = nullptr;
    int8_t* s_rew = nullptr;
    uint32_t* s_pidx = nullptr;
    // rule table (sparc_load_rules)
    bool rules = false;
    uint64_t* r_planes = nullptr;   // [P][RP_COUNT][W] (sparc_rules.hpp: the ABI planes + derived ones)
    bool r_area = false;
    uint2* r_inst_fc = nullptr;     // [P] {first, count | kHostFit} (sparc_rules.hpp RulesTab)
    uint32_t* r_inst = nullptr;
    uint2* r_shape_range = nullptr;  // [S] {first offset, count}
    int32_t* r_shape_area = nullptr;
    int8_t* r_shape_off = nullptr;
    FitMemo<kMemo>* r_memo = nullptr;   // [N] per-env exact-fit memo of the audit (zeroed at sparc_load_rules)
    uint32_t *r_reg_off = nullptr, *r_reg_tab = nullptr;   // region-code table (sparc_rules.hpp)
    uint64_t* r_rows = nullptr;   // the audit's per-puzzle rows (RulesTab::rows)
    bool r_tab_all = false;   // every puzzle has a region-code table (k_rollout1r's audit)
    bool ring_ok = false;     // W = 1 and every board fits below kRingShift (k_rollout1r's ring word)
    // kernel variants with identical results, set only by sparc_set_variant (A/B runs, tests)
    bool rules_generic = false;   // rule rollouts on k_rollout<..., RULES>
    bool io_codes_off = false;    // k_rollout1s / k_rolloutWs keep the reward codes on the trie wave
    int r1r_shape = 0;            // k_rollout1r's <G, A, RT> (0: <2, 5, 15>; 1-5: A/B, tests)
    bool obs_inline = false;      // 'new'-plane rollouts on k_rollout<..., OBS> instead of k_rollout_obsw
    // exact-fit searches past the GPU's node cap (sparc_set_fit_cap) are finished on the host
    // from these copies of the rule table (sparc_rules.hpp exact_fit, the same code)
    uint32_t fit_cap = kFitCap;
    size_t reg_entries = (size_t)1 << 28;   // region-code table budget (entries of 4 bits)
    std::vector<uint32_t> h_inst;
    std::vector<uint2> h_inst_fc, h_shape_range;
    size_t host_fit_puzzles = 0;    // puzzles flagged kHostFit by the last sparc_load_rules
    std::vector<int8_t> h_shape_off;
    unsigned long long* fq_count = nullptr;   // FitQueue of the audits (sparc_rules_finish)
    FitTodo* fq_items = nullptr;
    uint64_t fq_cap = 0;            // its capacity (grown by sparc_rules_finish on overflow)
    uint64_t fq_last = 0, fq_reruns = 0;   // searches the last finish ran; calls run again
    uint64_t* h_count = nullptr;    // pinned host word the queue count is read into
    // answers of the host's exact fits (sparc_rules.hpp HostFits), so that later audits look them
    // up instead of queueing the same search again: host mirror + device copy
    std::vector<uint4> h_hf;
    uint4* d_hf = nullptr;
    uint32_t hf_used = 0;
    bool hostfits_off = false;    // SPARC_VARIANT_HOST_FITS = 1: answers not kept (tests: the queue path)
    // the one-env record of sparc_env_step / _reset / _read (pinned, written by the kernels)
    sparc_env_record* h_rec = nullptr;
    sparc_env_record* d_rec = nullptr;
    AuditCall last_audit;           // the last queueing audit call (sparc_rules_finish)
    // the state a generic rule rollout started from (re-run on a queue overflow)
    void* snap = nullptr;
    size_t snap_bytes = 0;
    uint16_t* s_bits = nullptr;
    uint8_t* s_region = nullptr;
    uint64_t* s_fit = nullptr;
    std::string msg;
};

thread_local std::string g_err;

int fail(Ctx* c, int code, const std::string& m) {
    if (c) c->msg = m;
    g_err = m;
    return code;
}

#define HIPCHK(c, expr)                                                              \
    do {                                                                             \
        hipError_t _e = (expr);                                                      \
        if (_e != hipSuccess)                                                        \
            return fail((c), SPARC_E_HIP, std::string(#expr ": ") + hipGetErrorString(_e)); \
    } while (0)

// Every ABI entry point leaves the caller's current device as it found it: check_ctx (and
// create / destroy / sync) switch to the context's device for the call, and this guard, declared
// first in the entry point, switches back on return.
struct DevGuard {
    int dev = -1;
    DevGuard() {
        if (hipGetDevice(&dev) != hipSuccess) dev = -1;
    }
    ~DevGuard() {
        int cur = -1;
        if (dev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != dev) (void)hipSetDevice(dev);
    }
    DevGuard(const DevGuard&) = delete;
    DevGuard& operator=(const DevGuard&) = delete;
};

Params make_params(const Ctx* c) {
    Params p{};
    p.tab.open = c->t_open;
    p.tab.info = c->t_info;
    p.tab.root = c->t_root;
    p.tab.trie = c->t_trie;
    p.tab.init = c->t_init;
    p.tab.row1 = c->t_row1;
    p.tab.trie8 = c->t_trie8;
    p.tab.trieg = c->t_trieg;
    p.tab.trow = c->t_trow;
    p.tab.mrow = c->t_mrow;
    p.tab.num_puzzles = c->num_puzzles;
    p.st.vis = c->vis;
    p.st.dirs = c->dirs;
    p.st.pos = c->pos;
    p.st.aux = c->aux;
    p.st.step = c->step;
    p.st.pid = c->pid;
    p.n = c->n;
    p.pitch = (uint32_t)c->cfg.pitch;
    p.max_steps = c->cfg.max_steps;
    p.autoreset = c->cfg.autoreset;
    p.env_offset = (uint64_t)c->cfg.env_offset;
    p.err = c->err;
    const uint32_t P = p.pitch;
    p.nbr_pos = (2u * P) | ((P - 1u) << 8) | (0u << 16) | ((P + 1u) << 24);
    if (c->W == 1 && split1_pitch_ok(P)) {
        p.nbm = window_nbm(P);
        p.lmagic = legal_magic(P);
    }
    return p;
}

inline dim3 grid_for(size_t n) { return dim3((unsigned)((n + kBlock - 1) / kBlock)); }

// lift a kernel's dynamic-LDS limit to kMaxDynLds once per (device, kernel) (the call is not
// free, and a rollout call should cost one launch: it sits inside the bench's timed region)
int allow_big_lds(Ctx* c, const void* kern) {
    static std::mutex mu;
    static std::vector<std::pair<int, const void*>> done;
    std::lock_guard<std::mutex> lock(mu);
    for (const auto& k : done)
        if (k.first == c->device && k.second == kern) return SPARC_OK;
    HIPCHK(c, hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kMaxDynLds));
    done.emplace_back(c->device, kern);
    return SPARC_OK;
}

// call f(integral_constant<W>, bool_constant<TB>) for the runtime (W, TB)
template <class F>
void dispatch_w_tb(int w, bool tb, F&& f) {
    using T1 = std::integral_constant<int, 1>;
    using T2 = std::integral_constant<int, 2>;
    using T4 = std::integral_constant<int, 4>;
    if (w == 1) tb ? f(T1{}, std::true_type{}) : f(T1{}, std::false_type{});
    else if (w == 2) tb ? f(T2{}, std::true_type{}) : f(T2{}, std::false_type{});
    else tb ? f(T4{}, std::true_type{}) : f(T4{}, std::false_type{});
}

int check_ctx(Ctx* c, bool need_state) {
    if (!c) return fail(nullptr, SPARC_E_INVALID, "null context");
    if (!c->loaded) return fail(c, SPARC_E_STATE, "sparc_load_puzzles has not been called");
    if (need_state && !c->has_state) return fail(c, SPARC_E_STATE, "sparc_reset has not been called");
    HIPCHK(c, hipSetDevice(c->device));
    return SPARC_OK;
}

int launch_check(Ctx* c) {
    HIPCHK(c, hipGetLastError());
    return SPARC_OK;
}

template <int G_, int A_, int RT_, bool INC_ = false, int WPE_ = 6>
struct R1Shape {
    static constexpr int G = G_, A = A_, RT = RT_, WPE = WPE_;
    static constexpr bool INC = INC_;
};

constexpr uint64_t kFitQueueCap = 1u << 16;   // exact fits past the node cap per audit call (grown)
constexpr size_t kMixedTrieBytes = (size_t)4 << 20;   // an XCD's L2: past it the mixed trie tables pay
// puzzles an env plays per 2,000-step launch under random actions (episodes of ~300 steps, next
// puzzle on each autoreset): the window of its start puzzle that xcd_hot_bytes counts
constexpr uint32_t kHotWalk = 8;
constexpr uint64_t kFitQueueMax = (uint64_t)1 << 28;   // 6 GB of FitTodo

// the loaded rule table as the kernels take it; queue: push searches past the node cap to the
// FitQueue (audits), or not (the region-code table build: the host scans the table instead)
RulesTab rules_tab(const Ctx* c, bool queue) {
    RulesTab rt{};
    rt.planes = c->r_planes;
    rt.inst_fc = c->r_inst_fc;
    rt.inst = c->r_inst;
    rt.shape_range = c->r_shape_range;
    rt.shape_area = c->r_shape_area;
    rt.shape_off = c->r_shape_off;
    rt.num_puzzles = c->num_puzzles;
    rt.area = c->r_area ? 1u : 0u;
    rt.fit_cap = c->fit_cap;
    rt.reg_off = c->r_reg_off;
    rt.reg_tab = c->r_reg_tab;
    rt.fq = FitQueue{queue ? c->fq_count : nullptr, c->fq_items, c->fq_cap};
    rt.hf = c->hostfits_off ? HostFits{nullptr, 0u, 0u}
                            : HostFits{c->d_hf, c->h_hf.empty() ? 0u : (uint32_t)c->h_hf.size() - 1u, c->d_hf ? c->hf_used : 0u};
    rt.rows = c->r_rows;
    return rt;
}

// _polyfit_region_exact (SPaRC_Gym.py:738-853) of puzzle q's region with cell mask rm on the
// HOST, without a node cap (the reference's search is unbounded): exact_fit of sparc_rules.hpp,
// the code the GPU runs, over the host copies of the rule table.  1 fits, 0 does not.
template <int W>
int host_fit_w(const Ctx* c, uint32_t q, uint64_t rm) {
    const uint32_t w0 = c->h_info[4 * (size_t)q], X = w0 & 0xFFu, Y = (w0 >> 8) & 0xFFu;
    RulesTab rt{};
    rt.inst = c->h_inst.data();
    rt.shape_range = c->h_shape_range.data();
    rt.shape_off = c->h_shape_off.data();
    const uint2 fc = c->h_inst_fc[q];
    const FitIn fin = fit_in(rt, fc.x, fc.y & ~kHostFit, X, Y);
    const uint32_t P = (uint32_t)c->cfg.pitch;
    BB<W> Rc = BB<W>::zero();
    for (uint32_t b = 0; b < fin.CX * fin.CY; ++b)
        if ((rm >> b) & 1ull) Rc.set((2 * (b / fin.CY) + 1) * P + 2 * (b % fin.CY) + 1);
    // a kHostFit puzzle: the same search with lists and counters sized for any puzzle
    if (fc.y & kHostFit) return exact_fit<W, uint64_t, kHostFitMax, kHostFitMax, kHostFitPlanes>(fin, Rc, rm, ~0ull);
    return exact_fit<W, uint64_t>(fin, Rc, rm, ~0ull);
}
int host_fit(const Ctx* c, uint32_t q, uint64_t rm) {
    return c->W == 1 ? host_fit_w<1>(c, q, rm) : c->W == 2 ? host_fit_w<2>(c, q, rm) : host_fit_w<4>(c, q, rm);
}

// fn(k) for k in [0, n) on up to 16 host threads (the host's exact-fit searches)
template <class F>
void parallel_for(size_t n, F&& fn) {
    std::atomic<size_t> next{0};
    auto work = [&]() {
        for (size_t k; (k = next.fetch_add(1)) < n;) fn(k);
    };
    const size_t nt = std::min<size_t>({n, 16, (size_t)std::max(1u, std::thread::hardware_concurrency())});
    std::vector<std::thread> pool;
    for (size_t k = 1; k < nt; ++k) pool.emplace_back(work);
    work();
    for (auto& th : pool) th.join();
}

}  // namespace

extern "C" {

int sparc_abi_version(void) { return SPARC_ABI_VERSION; }

const char* sparc_last_error(const void* ctx) {
    return ctx ? static_cast<const Ctx*>(ctx)->msg.c_str() : g_err.c_str();
}

int sparc_create(int device, const sparc_config* cfg, void** ctx_out) {
    DevGuard dg;
    if (!cfg || !ctx_out) return fail(nullptr, SPARC_E_INVALID, "null argument");
    *ctx_out = nullptr;
    if (cfg->num_envs < 1) return fail(nullptr, SPARC_E_INVALID, "num_envs must be >= 1");
    if (cfg->words != 1 && cfg->words != 2 && cfg->words != 4)
        return fail(nullptr, SPARC_E_INVALID, "words must be 1, 2 or 4");
    if (cfg->pitch < 1 || cfg->pitch > 255) return fail(nullptr, SPARC_E_INVALID, "pitch must be in 1..255");
    if (cfg->traceback != 0 && cfg->traceback != 1) return fail(nullptr, SPARC_E_INVALID, "traceback must be 0/1");
    if (cfg->autoreset != SPARC_AUTORESET_NONE && cfg->autoreset != SPARC_AUTORESET_NEXT_STEP)
        return fail(nullptr, SPARC_E_INVALID, "unknown autoreset mode");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
        return fail(nullptr, SPARC_E_HIP, "no HIP device available");
    if (device < 0 || device >= ndev) return fail(nullptr, SPARC_E_INVALID, "bad device ordinal");
    Ctx* c = new Ctx();
    c->cfg = *cfg;
    c->device = device;
    c->n = (uint32_t)cfg->num_envs;
    c->W = cfg->words;
    const size_t n = c->n;
    auto cleanup = [&](int code) {
        sparc_destroy(c);
        return code;
    };
    if (hipSetDevice(device) != hipSuccess) return cleanup(fail(nullptr, SPARC_E_HIP, "hipSetDevice failed"));
    if (hipStreamCreateWithFlags(&c->own, hipStreamNonBlocking) != hipSuccess)
        return cleanup(fail(nullptr, SPARC_E_HIP, "hipStreamCreate failed"));
    c->stream = c->own;
    bool ok = hipMalloc(&c->vis, sizeof(uint64_t) * n * c->W) == hipSuccess &&
              hipMalloc(&c->pos, sizeof(uint32_t) * n) == hipSuccess &&
              hipMalloc(&c->aux, sizeof(uint32_t) * n) == hipSuccess &&
              hipMalloc(&c->step, sizeof(uint32_t) * n) == hipSuccess &&
              hipMalloc(&c->pid, sizeof(uint32_t) * n) == hipSuccess &&
              hipMalloc(&c->err, sizeof(int32_t)) == hipSuccess &&
              hipMalloc(&c->s_act, n) == hipSuccess && hipMalloc(&c->s_flags, n) == hipSuccess &&
              hipMalloc(&c->s_mask, n) == hipSuccess && hipMalloc(&c->s_rew, n) == hipSuccess &&
              hipMalloc(&c->s_pidx, sizeof(uint32_t) * n) == hipSuccess;
    if (ok && cfg->traceback) ok = hipMalloc(&c->dirs, sizeof(uint64_t) * n * 2 * c->W) == hipSuccess;
    if (!ok) return cleanup(fail(nullptr, SPARC_E_NOMEM, "hipMalloc failed for the env state"));
    if (hipMemset(c->err, 0, sizeof(int32_t)) != hipSuccess)
        return cleanup(fail(nullptr, SPARC_E_HIP, "hipMemset failed"));
    *ctx_out = c;
    return SPARC_OK;
}

int sparc_destroy(void* ctx) {
    DevGuard dg;
    Ctx* c = static_cast<Ctx*>(ctx);
    if (!c) return SPARC_OK;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    void* bufs[] = {c->vis, c->dirs, c->pos, c->aux, c->step, c->pid, c->t_open, c->t_info, c->t_root, c->t_trie, c->t_init, c->t_row1,
                    c->t_trie8, c->t_trow, c->t_mrow, c->t_mroww, c->t_boardw, c->err, c->s_act, c->s_flags, c->s_mask, c->s_rew, c->s_pidx, c->r_planes, c->r_inst_fc,
                    c->r_inst, c->r_shape_range, c->r_shape_area, c->r_shape_off, c->r_memo, c->s_bits, c->s_region, c->s_fit, c->r_reg_off, c->r_reg_tab, c->fq_count, c->fq_items, c->r_rows,
                    c->t_trieg, c->d_hf, c->t_trie4, c->t_trow4};
    for (void* b : bufs)
        if (b) (void)hipFree(b);
    if (c->snap) (void)hipFree(c->snap);
    if (c->h_count) (void)hipHostFree(c->h_count);
    if (c->h_rec) (void)hipHostFree(c->h_rec);
    if (c->own) (void)hipStreamDestroy(c->own);
    delete c;
    return SPARC_OK;
}

int sparc_set_stream(void* ctx, void* stream) {
    DevGuard dg;
    Ctx* c = static_cast<Ctx*>(ctx);
    if (!c) return fail(nullptr, SPARC_E_INVALID, "null context");
    c->stream = static_cast<hipStream_t>(stream);   // NULL is the HIP null stream, used as such
    return SPARC_OK;
}

int sparc_use_own_stream(void* ctx) {
    DevGuard dg;
    Ctx* c = static_cast<Ctx*>(ctx);
    if (!c) return fail(nullptr, SPARC_E_INVALID, "null context");
    c->stream = c->own;
    return SPARC_OK;
}

int sparc_sync(void* ctx) {
    DevGuard dg;
    Ctx* c = static_cast<Ctx*>(ctx);
    if (!c) return fail(nullptr, SPARC_E_INVALID, "null context");
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    int32_t e = 0;
    HIPCHK(c, hipMemcpy(&e, c->err, sizeof(e), hipMemcpyDeviceToHost));
    if (e) {
        HIPCHK(c, hipMemset(c->err, 0, sizeof(int32_t)));
        if (e & 2) return fail(c, SPARC_E_STATE, "device-side trie node out of range (state corrupted)");
        if (e & 8) return fail(c, SPARC_E_STATE, "rule audit: env puzzle index outside the rule table");
        if (e & kErrJoin) return fail(c, SPARC_E_STATE, "rule rollout: an audit wave pair did not join (outputs unreliable)");
        return fail(c, SPARC_E_INVALID, "device-side puzzle index out of range in a reset");
    }
    return SPARC_OK;
}

int sparc_load_puzzles(void* ctx, const sparc_puzzle_table* t) {
    DevGuard dg;
    Ctx* c = static_cast<Ctx*>(ctx);
    if (!c || !t || !t->open || !t->info) return fail(c, SPARC_E_INVALID, "null argument");
    if (t->num_puzzles < 1) return fail(c, SPARC_E_INVALID, "empty puzzle table");
    if (t->num_nodes < 0 || (t->num_nodes > 0 && !t->trie)) return fail(c, SPARC_E_INVALID, "bad trie");
    const int W = c->W;
    const uint32_t pitch = (uint32_t)c->cfg.pitch;
    // validate every index the kernels will follow, so no launch can read out of bounds
    for (int q = 0; q < t->num_puzzles; ++q) {
        const uint32_t* inf = t->info + 4 * (size_t)q;
        const uint32_t X = inf[0] & 0xFF, Y = (inf[0] >> 8) & 0xFF;
        const uint32_t sx = (inf[0] >> 16) & 0xFF, sy = inf[0] >> 24;
        const uint32_t tx = inf[1] & 0xFF, ty = (inf[1] >> 8) & 0xFF, fl = inf[1] >> 16;
        const uint32_t base = inf[2], cnt = inf[3];
        char m[160];
        const bool fits = W == 1 ? (Y < pitch && pitch <= 15 && (X + 1) * pitch <= 64u)
                                 : (Y <= pitch && (X - 1) * pitch + Y <= 64u * W);
        if (X < 1 || Y < 1 || !fits) {
            snprintf(m, sizeof m, "puzzle %d: lattice %ux%u does not fit pitch %u / %d words%s", q, X, Y, pitch, W,
                     W == 1 ? " (words=1 needs the padded layout)" : "");
            return fail(c, SPARC_E_INVALID, m);
        }
        if (sx >= X || sy >= Y || tx >= X || ty >= Y) {
            snprintf(m, sizeof m, "puzzle %d: start/target outside the lattice", q);
            return fail(c, SPARC_E_INVALID, m);
        }
        if ((fl & 2u) && (cnt == 0 || (uint64_t)base + cnt > (uint64_t)t->num_nodes || cnt > (W == 1 ? 0x7FFFu : 0xFFFFu))) {
            snprintf(m, sizeof m, "puzzle %d: trie range out of bounds", q);
            return fail(c, SPARC_E_INVALID, m);
        }
        if (fl & 2u) {
            for (uint32_t k = 0; k < cnt; ++k) {
                const uint32_t* r = t->trie + 4 * ((size_t)base + k);
                const uint32_t ch[4] = {r[0] & 0xFFFF, r[0] >> 16, r[1] & 0xFFFF, r[1] >> 16};
                for (uint32_t v : ch)
                    if (v != kNone && v >= cnt) return fail(c, SPARC_E_INVALID, "trie child out of range");
                const uint32_t par = r[2] & 0xFFFF;
                if (k > 0 && par >= cnt) return fail(c, SPARC_E_INVALID, "trie parent out of range");
            }
        }
    }
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (c->t_open) HIPCHK(c, hipFree(c->t_open));
    if (c->t_info) HIPCHK(c, hipFree(c->t_info));
    if (c->t_trie) HIPCHK(c, hipFree(c->t_trie));
    if (c->t_root) HIPCHK(c, hipFree(c->t_root));
    if (c->t_init) HIPCHK(c, hipFree(c->t_init));
    if (c->t_row1) HIPCHK(c, hipFree(c->t_row1));
    if (c->t_trie8) HIPCHK(c, hipFree(c->t_trie8));
    if (c->t_trieg) HIPCHK(c, hipFree(c->t_trieg));
    if (c->t_trie4) HIPCHK(c, hipFree(c->t_trie4));
    if (c->t_trow4) HIPCHK(c, hipFree(c->t_trow4));
    c->t_trie4 = nullptr;
    c->t_trow4 = nullptr;
    c->mixed_pays = false;
    c->nodes8.clear();
    if (c->t_trow) HIPCHK(c, hipFree(c->t_trow));
    if (c->t_mrow) HIPCHK(c, hipFree(c->t_mrow));
    if (c->t_mroww) HIPCHK(c, hipFree(c->t_mroww));
    if (c->t_boardw) HIPCHK(c, hipFree(c->t_boardw));
    c->t_mroww = nullptr;
    c->t_boardw = nullptr;
    c->split_w = false;
    c->t_trie8 = nullptr;
    c->t_trieg = nullptr;
    c->t_trow = nullptr;
    c->t_mrow = nullptr;
    c->t_init = nullptr;
    c->t_row1 = nullptr;
    c->t_open = nullptr;
    c->t_info = nullptr;
    c->t_root = nullptr;
    c->t_trie = nullptr;
    const size_t P = (size_t)t->num_puzzles, nn = (size_t)(t->num_nodes > 0 ? t->num_nodes : 1);
    HIPCHK(c, hipMalloc(&c->t_open, sizeof(uint64_t) * P * W));
    HIPCHK(c, hipMalloc(&c->t_info, sizeof(uint4) * P));
    HIPCHK(c, hipMalloc(&c->t_trie, sizeof(uint4) * nn));
    HIPCHK(c, hipMalloc(&c->t_root, sizeof(uint4) * P));
    // each puzzle's root record, so that a reset needs no dependent trie load
    std::vector<uint4> roots(P, make_uint4(0xFFFFFFFFu, 0xFFFFFFFFu, kNone, 0u));
    for (size_t q = 0; q < P; ++q) {
        const uint32_t* inf = t->info + 4 * q;
        if ((inf[1] >> 16) & 2u) {
            const uint32_t* r = t->trie + 4 * (size_t)inf[2];
            roots[q] = make_uint4(r[0], r[1], r[2], r[3]);
        }
    }
    HIPCHK(c, hipMemcpy(c->t_root, roots.data(), sizeof(uint4) * P, hipMemcpyHostToDevice));
    HIPCHK(c, hipMemcpy(c->t_open, t->open, sizeof(uint64_t) * P * W, hipMemcpyHostToDevice));
    // device copy of info: w3 = trie node count | legal mask of the reset state << 16, and for
    // the padded W = 1 layout the compact rows and the free board at reset
    std::vector<uint4> dinfo(P);
    std::vector<uint64_t> init(P, 0);
    std::vector<uint4> row1(P, make_uint4(0u, 0u, 0u, 0u));
    for (size_t q = 0; q < P; ++q) {
        const uint32_t* inf = t->info + 4 * q;
        const uint32_t X = inf[0] & 0xFF, Y = (inf[0] >> 8) & 0xFF;
        const uint32_t sx = (inf[0] >> 16) & 0xFF, sy = inf[0] >> 24;
        auto open_at = [&](uint32_t x, uint32_t y) {
            const uint32_t b = x * pitch + y;
            return (t->open[q * W + (b >> 6)] >> (b & 63)) & 1ull;
        };
        uint32_t legal0 = 0;
        const int dx[4] = {1, 0, -1, 0}, dy[4] = {0, -1, 0, 1};
        for (int d = 0; d < 4; ++d) {
            const int nx = (int)sx + dx[d], ny = (int)sy + dy[d];
            if (nx >= 0 && ny >= 0 && nx < (int)X && ny < (int)Y && open_at(nx, ny)) legal0 |= 1u << d;
        }
        const uint32_t root_term = ((inf[1] >> 16) & 2u) ? ((roots[q].z >> 16) & 1u) : 0u;
        dinfo[q] = make_uint4(inf[0], (inf[1] & 0x0007FFFFu) | (root_term << 19), inf[2],
                              (inf[3] & 0xFFFFu) | (legal0 << 16));
        if (W == 1) {
            const uint32_t tx = inf[1] & 0xFF, ty = (inf[1] >> 8) & 0xFF;
            // free board at reset, one row up (Env<1>): open points except the start
            init[q] = (t->open[q] & ~(1ull << (sx * pitch + sy))) << pitch;
            const uint32_t cnt = inf[3] & 0xFFFFu;
            row1[q] = make_uint4((sx * pitch + sy) | ((tx * pitch + ty) << 8) | (dinfo[q].y & 0xFFFF0000u),
                                 inf[2], (cnt ? cnt - 1u : 0u) | (legal0 << 16), 0u);
        }
    }
    HIPCHK(c, hipMalloc(&c->t_row1, sizeof(uint4) * P));
    HIPCHK(c, hipMemcpy(c->t_row1, row1.data(), sizeof(uint4) * P, hipMemcpyHostToDevice));
    HIPCHK(c, hipMalloc(&c->t_init, sizeof(uint64_t) * P));
    HIPCHK(c, hipMemcpy(c->t_info, dinfo.data(), sizeof(uint4) * P, hipMemcpyHostToDevice));
    HIPCHK(c, hipMemcpy(c->t_init, init.data(), sizeof(uint64_t) * P, hipMemcpyHostToDevice));
    HIPCHK(c, hipMemset(c->t_trie, 0xFF, sizeof(uint4) * nn));
    if (t->num_nodes > 0)
        HIPCHK(c, hipMemcpy(c->t_trie, t->trie, sizeof(uint4) * (size_t)t->num_nodes, hipMemcpyHostToDevice));
    // split-kernel tables (sparc_trie.hpp): 8-B records, field d = the child in direction d,
    // and the parent in the field of the direction back to it (the reverse of the move that
    // reached the node: no reachable child lives there, as that point is on the path); per
    // puzzle the trie row (root children, base, max node, flags) and, for W = 1, the move row
    bool small = true;
    for (size_t q = 0; q < P; ++q)
        if (((t->info[4 * q + 1] >> 16) & 2u) && (t->info[4 * q + 3] & 0xFFFFu) > 0x7FFFu) small = false;
    if (small) {
        // each puzzle's records start on a 128-B line (16 records; rootless puzzles: base 0): in
        // breadth-first order the root and the nodes near it, which most walks never leave,
        // share ONE line per puzzle instead of straddling two, so pools whose tries outgrow an
        // XCD's L2 refill fewer lines (the relative node indices, and so the env state, are
        // unchanged; only the split tables move)
        std::vector<size_t> b8(P, 0);
        size_t nn8 = 0;
        for (size_t q = 0; q < P; ++q) {
            const uint32_t* inf = t->info + 4 * q;
            if (!((inf[1] >> 16) & 2u)) continue;
            nn8 = (nn8 + 15u) & ~(size_t)15u;
            b8[q] = nn8;
            nn8 += inf[3] & 0xFFFFu;
        }
        nn8 = std::max<size_t>(nn8, 1);
        if (W == 1) {   // Env<1> (k_step, k_rollout1) reads trie8 at row1.y too
            for (size_t q = 0; q < P; ++q) row1[q].y = (uint32_t)b8[q];
            HIPCHK(c, hipMemcpy(c->t_row1, row1.data(), sizeof(uint4) * P, hipMemcpyHostToDevice));
        }
        std::vector<uint2> t8(nn8, make_uint2(0xFFFFFFFFu, 0xFFFFFFFFu));
        auto packed = [&](size_t base, uint32_t k) {   // node k of a puzzle as index | terminal << 15
            return k | (((t->trie[4 * (base + k) + 2] >> 16) & 1u) << 15);
        };
        for (size_t q = 0; q < P; ++q) {
            const uint32_t* inf = t->info + 4 * q;
            if (!((inf[1] >> 16) & 2u)) continue;
            const size_t base = inf[2], bq = b8[q];
            const uint32_t cnt = inf[3] & 0xFFFFu;
            for (uint32_t k = 0; k < cnt; ++k) {
                const uint32_t* r = t->trie + 4 * (base + k);
                const uint32_t ch[4] = {r[0] & 0xFFFFu, r[0] >> 16, r[1] & 0xFFFFu, r[1] >> 16};
                uint32_t f[4];
                for (int d = 0; d < 4; ++d) f[d] = ch[d] == kNone ? 0xFFFFu : packed(base, ch[d]);
                t8[bq + k] = make_uint2(f[0] | (f[1] << 16), f[2] | (f[3] << 16));
            }
            for (uint32_t k = 0; k < cnt; ++k) {           // parents, after every child field
                const uint32_t* r = t->trie + 4 * (base + k);
                const uint32_t ch[4] = {r[0] & 0xFFFFu, r[0] >> 16, r[1] & 0xFFFFu, r[1] >> 16};
                for (uint32_t d = 0; d < 4; ++d) {
                    if (ch[d] == kNone) continue;
                    uint2& cr = t8[bq + ch[d]];
                    const uint32_t back = d ^ 2u, sh = (back & 1u) * 16u;
                    uint32_t& w = back < 2 ? cr.x : cr.y;
                    w = (w & ~(0xFFFFu << sh)) | (packed(base, k) << sh);
                }
            }
        }
        std::vector<uint4> trow(P), mrow(P, make_uint4(0u, 0u, 0u, 0u));
        for (size_t q = 0; q < P; ++q) {
            const uint32_t* inf = t->info + 4 * q;
            const uint32_t fl = (dinfo[q].y >> 16) & 0xFFFFu;
            const uint32_t cnt = inf[3] & 0xFFFFu;
            const uint2 rr = (fl & 2u) ? t8[b8[q]] : make_uint2(0xFFFFFFFFu, 0xFFFFFFFFu);
            // flags as row1: bit0 solutions, bit1 root valid, bit3 root terminal
            const uint32_t tf = (fl & 3u) | (((dinfo[q].y >> 19) & 1u) << 3);
            const uint32_t rootS = (tf & 2u) ? ((tf >> 3) & 1u) << 15 : 0x10000u;
            trow[q] = make_uint4(rr.x, rr.y, (uint32_t)b8[q], rootS | ((tf & 1u) << 14) | ((cnt ? cnt - 1u : 0u) << 17));
            // W = 1 move row: row word, reset board, and the puzzle the autoreset after it loads
            if (W == 1) mrow[q] = make_uint4(row1[q].x, (uint32_t)init[q], (uint32_t)(init[q] >> 32),
                                             q + 1 == P ? 0u : (uint32_t)q + 1u);
        }
        HIPCHK(c, hipMalloc(&c->t_trie8, sizeof(uint2) * nn8));
        HIPCHK(c, hipMemcpy(c->t_trie8, t8.data(), sizeof(uint2) * nn8, hipMemcpyHostToDevice));
        // look-ahead records (TrieLane::step1la): entry 4k + d = the record of node k's field-d
        // node (child, or the parent in the back direction), all ones where the field is empty;
        // at least 4 entries, so that a rootless puzzle's lane (base 0, node 0) reads in bounds
        std::vector<uint2> tg(4 * nn8, make_uint2(0xFFFFFFFFu, 0xFFFFFFFFu));
        for (size_t q = 0; q < P; ++q) {
            const uint32_t* inf = t->info + 4 * q;
            if (!((inf[1] >> 16) & 2u)) continue;
            const size_t base = b8[q];
            const uint32_t cnt = inf[3] & 0xFFFFu;
            for (uint32_t k = 0; k < cnt; ++k) {
                const uint2 r = t8[base + k];
                const uint32_t f[4] = {r.x & 0xFFFFu, r.x >> 16, r.y & 0xFFFFu, r.y >> 16};
                for (int d = 0; d < 4; ++d)
                    if (f[d] != 0xFFFFu) tg[4 * (base + k) + d] = t8[base + (f[d] & 0x7FFFu)];
            }
        }
        HIPCHK(c, hipMalloc(&c->t_trieg, sizeof(uint2) * tg.size()));
        HIPCHK(c, hipMemcpy(c->t_trieg, tg.data(), sizeof(uint2) * tg.size(), hipMemcpyHostToDevice));
        HIPCHK(c, hipMalloc(&c->t_trow, sizeof(uint4) * P));
        HIPCHK(c, hipMemcpy(c->t_trow, trow.data(), sizeof(uint4) * P, hipMemcpyHostToDevice));
        // mixed tables (TrieLaneT<true>): a trie of at most 127 nodes as 4-B records (each 16-bit
        // field of trie8 as an 8-bit one, index | terminal << 7, 0xFF none), a larger one as its
        // 8-B records; each puzzle's records start on a 128-B line, the base is a byte offset, and
        // bit 13 of the row's w marks a compact puzzle (root S then 0x80 / 0x100).  Used when the
        // 8-B records outgrow an XCD's 4 MB L2: below that the per-lane format costs the trie chain
        // more than the misses it saves (MI355X, c3: 4,096 puzzles, 2 MB of records, +5 %; 16,384
        // puzzles, 8.4 MB, -7.4 %; profiles/r06/ab_bigpool); SPARC_VARIANT_MIXED_TRIE overrides
        c->mixed_pays = nn8 * sizeof(uint2) > kMixedTrieBytes;
        if (W == 1 && c->mixed_pays) {   // sparc_reset_host refines the choice per XCD (xcd_hot_bytes)
            c->nodes8.resize(P);
            for (size_t q = 0; q < P; ++q) c->nodes8[q] = t->info[4 * q + 3] & 0xFFFFu;
        }
        if (W == 1) {
            std::vector<size_t> bo(P, 0);
            size_t nb = 0;
            auto tiny = [&](size_t q) { return (t->info[4 * q + 3] & 0xFFFFu) <= 127u; };
            for (size_t q = 0; q < P; ++q) {
                if (!((t->info[4 * q + 1] >> 16) & 2u)) continue;
                nb = (nb + 127u) & ~(size_t)127u;
                bo[q] = nb;
                nb += (size_t)(t->info[4 * q + 3] & 0xFFFFu) * (tiny(q) ? 4u : 8u);
            }
            nb += 8;   // an 8-B gather of the last 4-B record stays in bounds
            auto f8 = [](uint32_t f16) { return f16 == 0xFFFFu ? 0xFFu : (f16 & 0x7Fu) | ((f16 >> 15) << 7); };
            auto rec4 = [&](uint2 r) {
                return f8(r.x & 0xFFFFu) | (f8(r.x >> 16) << 8) | (f8(r.y & 0xFFFFu) << 16) | (f8(r.y >> 16) << 24);
            };
            std::vector<uint8_t> tb(nb, 0xFF);
            std::vector<uint4> trow4(P);
            for (size_t q = 0; q < P; ++q) {
                const uint32_t cnt = t->info[4 * q + 3] & 0xFFFFu;
                const bool rooted = (t->info[4 * q + 1] >> 16) & 2u, small4 = rooted && tiny(q);
                const uint32_t w = trow[q].w;
                uint2 root = make_uint2(trow[q].x, trow[q].y);
                if (rooted) {
                    for (uint32_t k = 0; k < cnt; ++k) {
                        const uint2 r8 = t8[b8[q] + k];
                        if (small4) {
                            const uint32_t v = rec4(r8);
                            memcpy(&tb[bo[q] + 4 * (size_t)k], &v, 4);
                        } else {
                            memcpy(&tb[bo[q] + 8 * (size_t)k], &r8, 8);
                        }
                    }
                    if (small4) root = make_uint2(rec4(root), 0xFFFFFFFFu);
                }
                // root S 0x80 (terminal) / 0x100 (off the trie) in the compact layout
                const uint32_t rs = small4 ? ((w & 0x10000u) ? 0x100u : ((w >> 15) & 1u) << 7) : (w & 0x18000u);
                trow4[q] = make_uint4(root.x, root.y, (uint32_t)bo[q],
                                      rs | (small4 ? 1u << 13 : 0u) | (w & 0x4000u) | (w & ~0x1FFFFu));
            }
            HIPCHK(c, hipMalloc(&c->t_trie4, nb));
            HIPCHK(c, hipMemcpy(c->t_trie4, tb.data(), nb, hipMemcpyHostToDevice));
            HIPCHK(c, hipMalloc(&c->t_trow4, sizeof(uint4) * P));
            HIPCHK(c, hipMemcpy(c->t_trow4, trow4.data(), sizeof(uint4) * P, hipMemcpyHostToDevice));
        }
        HIPCHK(c, hipMalloc(&c->t_mrow, sizeof(uint4) * P));
        HIPCHK(c, hipMemcpy(c->t_mrow, mrow.data(), sizeof(uint4) * P, hipMemcpyHostToDevice));
        // multi-word split geometry (sparc_movew.hpp): internal pitch + 1, the board plus a
        // zero row above and one spare dword, the longest possible path in the move stack
        if (W > 1 && pitch <= 15u) {
            SplitGeom g{};
            g.P2 = pitch + 1u;
            uint32_t xmax = 1, pts = 1;
            for (size_t q = 0; q < P; ++q) {
                const uint32_t X = t->info[4 * q] & 0xFFu, Y = (t->info[4 * q] >> 8) & 0xFFu;
                xmax = std::max(xmax, X);
                pts = std::max(pts, X * Y);
            }
            g.B = ((xmax + 2u) * g.P2 + 31u) / 32u + 1u;
            g.BS = (g.B + 3u) & ~3u;
            // the move wave writes slot len - 1 on every step, moved or not, and len reaches pts
            // on a path through every point: pts slots, not pts - 1
            g.M = c->cfg.traceback ? ((pts + 15u) & ~15u) : 0u;
            g.nbr_pos = (2u * g.P2) | ((g.P2 - 1u) << 8) | (0u << 16) | ((g.P2 + 1u) << 24);
            g.off_board = (uint32_t)kW_Board;
            g.off_stack = g.off_board + g.BS * 256u;
            g.pair = (g.off_stack + g.M * 64u + 15u) & ~15u;
            // the move wave keeps the next reset board in kBoardRegs 16-B registers
            if (4 * (size_t)g.pair + splitw_fin_bytes() <= kMaxDynLds && g.BS <= 4u * kBoardRegs) {
                std::vector<uint4> mw(P);
                std::vector<uint32_t> bw(P * g.BS, 0u);
                for (size_t q = 0; q < P; ++q) {
                    const uint32_t* inf = t->info + 4 * q;
                    const uint32_t X = inf[0] & 0xFF, Y = (inf[0] >> 8) & 0xFF;
                    const uint32_t sx = (inf[0] >> 16) & 0xFF, sy = inf[0] >> 24;
                    const uint32_t tx = inf[1] & 0xFF, ty = (inf[1] >> 8) & 0xFF;
                    mw[q] = make_uint4((sx * g.P2 + sy) | ((tx * g.P2 + ty) << 16), (inf[1] >> 16) & 7u, 0u, 0u);
                    for (uint32_t x = 0; x < X; ++x)
                        for (uint32_t y = 0; y < Y; ++y) {
                            const uint32_t b = x * pitch + y;
                            if (!((t->open[q * W + (b >> 6)] >> (b & 63)) & 1ull) || (x == sx && y == sy)) continue;
                            const uint32_t d = (x + 1u) * g.P2 + y;
                            bw[q * g.BS + (d >> 5)] |= 1u << (d & 31u);
                        }
                }
                HIPCHK(c, hipMalloc(&c->t_mroww, sizeof(uint4) * P));
                HIPCHK(c, hipMemcpy(c->t_mroww, mw.data(), sizeof(uint4) * P, hipMemcpyHostToDevice));
                HIPCHK(c, hipMalloc(&c->t_boardw, sizeof(uint32_t) * bw.size()));
                HIPCHK(c, hipMemcpy(c->t_boardw, bw.data(), sizeof(uint32_t) * bw.size(), hipMemcpyHostToDevice));
                c->sgeom = g;
                c->split_w = true;
            }
        }
    }
    c->ring_ok = W == 1;
    for (size_t q = 0; q < P; ++q)
        if ((t->info[4 * q] & 0xFFu) * pitch > kRingShift) c->ring_ok = false;
    c->num_puzzles = (uint32_t)t->num_puzzles;
    c->num_nodes = (uint32_t)t->num_nodes;
    c->h_info.assign(t->info, t->info + 4 * P);
    c->loaded = true;
    c->rules = false;       // the rule table indexes the old puzzles
    c->has_state = false;   // old state may point at puzzles that no longer exist
    return SPARC_OK;
}

int sparc_reset_device(void* ctx, const uint32_t* d_q, const uint8_t* d_mask, uint8_t* d_flags) {
    DevGuard dg;
    Ctx* c = static_cast<Ctx*>(ctx);
    int rc = check_ctx(c, false);
    if (rc) return rc;
    if (!d_q) return fail(c, SPARC_E_INVALID, "null puzzle_index");
    if (d_mask && !c->has_state) return fail(c, SPARC_E_STATE, "first reset must cover every env (mask NULL)");
    const Params p = make_params(c);
    dispatch_w_tb(c->W, c->cfg.traceback, [&](auto w, auto tb) {
        k_reset<decltype(w)::value, decltype(tb)::value><<<grid_for(c->n), kBlock, 0, c->stream>>>(p, d_q, d_mask, d_flags);
    });
    rc = launch_check(c);
    if (rc) return rc;
    c->has_state = true;
    return SPARC_OK;
}

// The 8-B trie records one XCD's L2 must hold for the envs of a full reset: k_rollout1s runs 256
// envs per workgroup and workgroups b, b + 8, ... share an XCD (round-robin dispatch,
// MI355X_MICROARCH.md), so XCD group g holds envs i with (i / 256) % 8 == g, and each env plays
// its start puzzle and the next kHotWalk - 1.  Returns the largest group's bytes.  A pool whose
// envs are placed XCD-locally (bench.initial_puzzles 'xcd') keeps the 8-B records past 4 MB of
// them (MI355X, c3 at 16,384 puzzles: 0.362 ms with 8-B records against 0.379 ms mixed; the
// hash placement 0.405 ms, mixed 0.394; profiles/r06/ab_xcd_place).
static size_t xcd_hot_bytes(const Ctx* c, const uint32_t* q) {
    const uint32_t P = c->num_puzzles;
    std::vector<uint8_t> seen(P, 0);   // bit g: counted for group g
    size_t bytes[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (uint32_t i = 0; i < c->n; ++i) {
        const uint32_t g = (i / 256u) & 7u;
        uint32_t u = q[i];
        for (uint32_t k = 0; k < kHotWalk; ++k, u = u + 1 == P ? 0u : u + 1) {
            if (seen[u] & (1u << g)) continue;
            seen[u] |= (uint8_t)(1u << g);
            bytes[g] += (size_t)c->nodes8[u] * sizeof(uint2);
        }
    }
    return *std::max_element(bytes, bytes + 8);
}

int sparc_reset_host(void* ctx, const uint32_t* q, const uint8_t* mask, uint8_t* flags) {
    DevGuard dg;
    Ctx* c = static_cast<Ctx*>(ctx);
    int rc = check_ctx(c, false);
    if (rc) return rc;
    if (!q) return fail(c, SPARC_E_INVALID, "null puzzle_index");
    for (uint32_t i = 0; i < c->n; ++i)
        if ((!mask || mask[i]) && q[i] >= c->num_puzzles) return fail(c, SPARC_E_INVALID, "puzzle index out of range");
    if (!mask && c->nodes8.size() == c->num_puzzles) c->mixed_pays = xcd_hot_bytes(c, q) > kMixedTrieBytes;
    HIPCHK(c, hipMemcpyAsync(c->s_pidx, q, sizeof(uint32_t) * c->n, hipMemcpyHostToDevice, c->stream));
    if (mask) HIPCHK(c, hipMemcpyAsync(c->s_mask, mask, c->n, hipMemcpyHostToDevice, c->stream));
    rc = sparc_reset_device(c, c->s_pidx, mask ? c->s_mask : nullptr, flags ? c->s_flags : nullptr);
    if (rc) return rc;
    if (flags) HIPCHK(c, hipMemcpyAsync(flags, c->s_flags, c->n, hipMemcpyDeviceToHost, c->stream));
    return sparc_sync(c);
}

int sparc_step_device(void* ctx, const uint8_t* d_act, int8_t* d_rew, uint8_t* d_flags) {
    DevGuard dg;
    Ctx* c = static_cast<Ctx*>(ctx);
    int rc = check_ctx(c, true);
    if (rc) return rc;
    if (!d_act || !d_rew || !d_flags) return fail(c, SPARC_E_INVALID, "null argument");
    const Params p = make_params(c);
    dispatch_w_tb(c->W, c->cfg.traceback, [&](auto w, auto tb) {
        k_step<decltype(w)::value, decltype(tb)::value><<<grid_for(c->n), kBlock, 0, c->stream>>>(p, d_act, d_rew,
                                                                                                  d_flags);
    });
    return launch_check(c);
}

int sparc_step_host(void* ctx, const uint8_t* act, int8_t* rew, uint8_t* flags) {
    DevGuard dg;
    Ctx* c = static_cast<Ctx*>(ctx);
    int rc = check_ctx(c, true);
    if (rc) return rc;
    if (!act || !rew || !flags) return fail(c, SPARC_E_INVALID, "null argument");
    HIPCHK(c, hipMemcpyAsync(c->s_act, act, c->n, hipMemcpyHostToDevice, c->stream));
    rc = sparc_step_device(c, c->s_act, c->s_rew, c->s_flags);
    if (rc) return rc;
    HIPCHK(c, hipMemcpyAsync(rew, c->s_rew, c->n, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(flags, c->s_flags, c->n, hipMemcpyDeviceToHost, c->stream));
    return sparc_sync(c);
}

int sparc_random_actions_device(void* ctx, int32_t T, uint64_t seed, uint64_t t0, uint8_t* d_actions) {
    DevGuard dg;
    Ctx* c = static_cast<Ctx*>(ctx);
    if (!c) return fail(nullptr, SPARC_E_INVALID, "null context");
    if (!d_actions) return fail(c, SPARC_E_INVALID, "null actions");
    if (T < 0) return fail(c, SPARC_E_INVALID, "T must be >= 0");
    if (T == 0) return SPARC_OK;
    HIPCHK(c, hipSetDevice(c->device));
    const uint64_t lanes = (uint64_t)((c->n + 3u) / 4u) * (uint64_t)T;
    if (lanes > (uint64_t)kBlock * 0x7FFFFFFFull) return fail(c, SPARC_E_INVALID, "T*N too large");
    k_rand_actions<<<dim3((unsigned)((lanes + kBlock - 1) / kBlock)), kBlock, 0, c->stream>>>(
        seed, (uint64_t)c->cfg.env_offset, t0, c->n, (uint32_t)T, d_actions);
    return launch_check(c);
}

}  // extern "C"

namespace {
// rule rollouts that run k_rollout1r (W = 1 pools whose every puzzle has a region-code table and
// whose boards fit the ring word); the rest run the generic k_rollout<..., RULES>
bool r1r_rollout(const Ctx* c) { return c->W == 1 && c->r_tab_all && c->ring_ok && !c->rules_generic; }

// sparc_rollout_device / sparc_rollout_obs_device; `ot` non-null: observation traces
int rollout_impl(Ctx* c, int32_t T, const uint8_t* d_act, uint64_t seed, uint64_t t0, int8_t* d_rew,
                 uint8_t* d_flags, int32_t* d_stats, const ObsTrace* ot, const RuleTrace* rtr = nullptr) {
    int rc = check_ctx(c, true);
    if (rc) return rc;
    if (T < 0) return fail(c, SPARC_E_INVALID, "T must be >= 0");
    if (T == 0) return SPARC_OK;
    if ((uint64_t)T * c->n > (1ull << 40)) return fail(c, SPARC_E_INVALID, "T*N too large");
    const Params p = make_params(c);
    const ObsTrace no_obs{nullptr, nullptr, 1u, 1u};
    const RuleTrace no_rules{RulesTab{}, nullptr, nullptr};
    int lds_rc = SPARC_OK;   // allow_big_lds failure inside a launch lambda (then no launch)
    int4* st = reinterpret_cast<int4*>(d_stats);
    auto aligned = [](const void* q) { return q == nullptr || (reinterpret_cast<uintptr_t>(q) & 15u) == 0; };
    const uint32_t tiled = (c->n % 16 == 0) && aligned(d_act) && aligned(d_rew) && aligned(d_flags) &&
                           (!rtr || aligned(rtr->bits));
    // the puzzle rows are staged in LDS when they fit next to the I/O tiles without costing
    // occupancy: budget = LDS per CU / resident workgroups per CU (256 CUs)
    // envs per wave: 64.  (Measured on MI355X at 65,536 envs: 32-wide waves, two per SIMD, are
    // 1.3x slower than one full wave per SIMD — a half-empty wave costs the full issue time.)
    const bool half = false;
    if (c->W == 1 && !ot && !rtr) {
        const size_t blocks = (c->n + 255) / 256;
        const size_t per_cu = (blocks + 255) / 256;
        const size_t budget = std::min(kMaxDynLds, (size_t)160 * 1024 / (per_cu ? per_cu : 1));
        const size_t tbytes = table_lds_bytes<1>(c->num_puzzles);
        // the full tiles of full workgroups go through the split move / trie kernel (MI355X, c3
        // at 65,536 envs: 0.266 vs 0.312 ms per 1,000 steps); a tail of T % 16 steps or a batch
        // that is not a multiple of 256 envs goes through k_rollout1 below
        if (tiled && c->n % 256 == 0 && T >= kTile && c->t_trie8 && split1_pitch_ok((uint32_t)c->cfg.pitch)) {
            const int32_t T16 = T / kTile * kTile;
            const size_t sbytes = split_table_bytes(c->num_puzzles);
            const bool lds_s = kS_Base + sbytes <= budget;
            // past the row budget: rows from the L2, the trie rows handed over through slots
            const size_t shm_s = kS_Base + (lds_s ? sbytes : kS_SlotBytes);
            // past the row budget the mixed tables (tries of at most 127 nodes in 4-B records:
            // twice the nodes per L2 line; sparc_trie.hpp TrieLaneT<true>)
            const bool compact = !lds_s && c->t_trie4 && (c->mixed_trie == 1 || (c->mixed_trie == 0 && c->mixed_pays));
            Params ps = p;
            if (compact) {
                ps.tab.trie8 = reinterpret_cast<const uint2*>(c->t_trie4);
                ps.tab.trow = c->t_trow4;
            }
            auto launch_s = [&](auto kern, const uint8_t* a) {
                if (shm_s > 64 * 1024 && (lds_rc = allow_big_lds(c, reinterpret_cast<const void*>(kern)))) return;
                kern<<<dim3((unsigned)blocks), kBlock1s, shm_s, c->stream>>>(ps, T16, a, seed, t0, d_rew, d_flags, st);
            };
            // one wave pair (and its I/O wave) per workgroup (k_rollout1s<..., PR = 1>): 4x the
            // workgroups, each role on a SIMD of its own, for grids of at most 64 256-env
            // workgroups (MI355X, c2 at 4,096 envs: 0.2811-0.2817 -> 0.2744-0.2750 ms per 2,000-step
            // launch, profiles/r06/ab_c2_pr1)
            auto launch_s1 = [&](auto kern, const uint8_t* a) {
                if (shm_s > 64 * 1024 && (lds_rc = allow_big_lds(c, reinterpret_cast<const void*>(kern)))) return;
                kern<<<dim3((unsigned)(4 * blocks)), kBlock1s / 4, shm_s, c->stream>>>(ps, T16, a, seed, t0, d_rew, d_flags,
                                                                                     st);
            };
            // IOR (next-step autoreset): the I/O waves derive the reward codes and counters from
            // the trie wave's class bytes (io_codes4), which takes them off the trie wave's chain
            auto go_s = [&](auto tb, auto ior) {
                constexpr bool TB = decltype(tb)::value, IOR = decltype(ior)::value;
                if (d_act) {
                    // look-ahead trie gathers on grids of at most 64 workgroups (sparc_trie.hpp)
                    if (lds_s && blocks <= 64) launch_s1(k_rollout1s<TB, false, true, true, IOR, false, 1>, d_act);
                    else if (lds_s) launch_s(k_rollout1s<TB, false, true, false, IOR>, d_act);
                    else if (compact) launch_s(k_rollout1s<TB, false, false, false, IOR, true>, d_act);
                    else launch_s(k_rollout1s<TB, false, false, false, IOR>, d_act);
                } else {
                    if (lds_s) launch_s(k_rollout1s<TB, true, true, false, IOR>, nullptr);
                    else if (compact) launch_s(k_rollout1s<TB, true, false, false, IOR, true>, nullptr);
                    else launch_s(k_rollout1s<TB, true, false, false, IOR>, nullptr);
                }
            };
            const bool ior = p.autoreset == 1 && !c->io_codes_off;
            if (c->cfg.traceback) {
                if (ior) go_s(std::true_type{}, std::true_type{});
                else go_s(std::true_type{}, std::false_type{});
            } else {
                if (ior) go_s(std::false_type{}, std::true_type{});
                else go_s(std::false_type{}, std::false_type{});
            }
            if (lds_rc) return lds_rc;
            rc = launch_check(c);
            if (rc || T16 == T) return rc;
            const size_t adv = (size_t)T16 * c->n;
            if (d_act) d_act += adv;
            if (d_rew) d_rew += adv;
            if (d_flags) d_flags += adv;
            t0 += (uint64_t)T16;
            T -= T16;
        }
        const bool lds_table = kW1Base + tbytes <= budget;
        const size_t shm = kW1Base + (lds_table ? tbytes : 0);
        auto launch = [&](auto kern, const uint8_t* a) {
            if (shm > 64 * 1024 && (lds_rc = allow_big_lds(c, reinterpret_cast<const void*>(kern)))) return;
            kern<<<dim3((unsigned)blocks), kBlock1, shm, c->stream>>>(p, T, a, seed, t0, d_rew, d_flags, st, tiled);
        };
        auto go1 = [&](auto tb) {
            constexpr bool TB = decltype(tb)::value;
            if (d_act) {
                if (lds_table) launch(k_rollout1<TB, false, true>, d_act);
                else launch(k_rollout1<TB, false, false>, d_act);
            } else {
                if (lds_table) launch(k_rollout1<TB, true, true>, nullptr);
                else launch(k_rollout1<TB, true, false>, nullptr);
            }
        };
        if (c->cfg.traceback) go1(std::true_type{});
        else go1(std::false_type{});
        if (lds_rc) return lds_rc;
        return launch_check(c);
    }
    if (rtr && r1r_rollout(c)) {
        // rule rollouts of W = 1 pools with every puzzle in the region-code table: step waves +
        // audit waves (k_rollout1r; shape <G, A, RT> = c->r1r_shape)
        auto go_shape = [&](auto geo_c) {
            using Geo = decltype(geo_c);
            constexpr int G = Geo::G, A = Geo::A, RT = Geo::RT, WPE = Geo::WPE;
            constexpr bool INC = Geo::INC;
            using GG = R1Geom<G, A, RT>;
            const size_t blocks = (c->n + GG::kEnvs - 1) / GG::kEnvs;
            const size_t tbytes = table_lds_bytes<1>(c->num_puzzles);
            // the puzzle rows go to LDS only while a 12-wave workgroup still leaves room for a
            // second one on the CU (80 KB each); past that the step waves read them from the L2
            // (their resets have slack: the audit waves set the pace)
            const bool lds_table = GG::kBase + tbytes <= (GG::kBlock <= 768 ? (size_t)80 * 1024 : kMaxDynLds);
            const size_t shm = GG::kBase + (lds_table ? tbytes : 0);
            auto launch = [&](auto kern, const uint8_t* a) {
                if (shm > 64 * 1024 && (lds_rc = allow_big_lds(c, reinterpret_cast<const void*>(kern)))) return;
                kern<<<dim3((unsigned)blocks), GG::kBlock, shm, c->stream>>>(p, T, a, seed, t0, d_rew, d_flags, st, tiled,
                                                                            rtr->rt, rtr->bits);
            };
            auto go = [&](auto tb) {
                constexpr bool TB = decltype(tb)::value;
                if (d_act) {
                    if (lds_table) launch(k_rollout1r<TB, false, true, G, A, RT, INC, WPE>, d_act);
                    else launch(k_rollout1r<TB, false, false, G, A, RT, INC, WPE>, d_act);
                } else {
                    if (lds_table) launch(k_rollout1r<TB, true, true, G, A, RT, INC, WPE>, nullptr);
                    else launch(k_rollout1r<TB, true, false, G, A, RT, INC, WPE>, nullptr);
                }
            };
            if (c->cfg.traceback) go(std::true_type{});
            else go(std::false_type{});
        };
        // <2, 5, 15>: 128 envs, 2 step + 10 audit waves per workgroup, two workgroups per CU (six
        // waves per SIMD at 66-80 VGPRs), three jobs per audit lane and 15-step tile (the waves'
        // skew at the tile barrier averages over more jobs), the puzzle rows from the L2 (76 KB of
        // rings per workgroup); MI355X, c3r 2,000-step launches: 2.51 ms against 2.60 for
        // <2, 5, 10> (profiles/r06/ab_c3r_flood).  Round 4, 50-step launches: <2, 5, 10> 0.1245 ms
        // against 0.1338 for <4, 3, 12> (one 16-wave workgroup per CU, its LDS) and 0.1275 for
        // <2, 4, 12> (profiles/r04/ab_run2)
        switch (c->r1r_shape) {
            case 1: go_shape(R1Shape<4, 3, 12>{}); break;
            case 2: go_shape(R1Shape<2, 4, 12>{}); break;
            // incremental audits (INC, RegionSet1): slower in lock step, kept for A/B and tests —
            // c3r 2,000-step launches 7.6 ms (<4, 1, 4>) and 6.1-6.3 ms (<2, 3, 15>) against 3.92-3.99
            // (<2, 1, 8> 9.2, <2, 2, 16> 7.8; profiles/r06/ab_c3r_inc)
            case 3: go_shape(R1Shape<4, 1, 4, true, 4>{}); break;
            case 4: go_shape(R1Shape<2, 3, 15, true, 4>{}); break;
            case 5: go_shape(R1Shape<2, 5, 10>{}); break;
            default: go_shape(R1Shape<2, 5, 15>{}); break;
        }
        if (lds_rc) return lds_rc;
        return launch_check(c);
    }
    if (c->W > 1 && !ot && !rtr && c->split_w && tiled && c->n % 256 == 0 && T >= kTile) {
        // the full tiles of whole 256-env workgroups go through the multi-word split kernel; a
        // tail of T % 16 steps through k_rollout below (the state round-trips HBM exactly)
        const int32_t T16 = T / kTile * kTile;
        const SplitGeom& g = c->sgeom;
        const size_t blocks = c->n / 256;
        const size_t base = 4 * (size_t)g.pair + splitw_fin_bytes();
        const bool lds_t = base + sizeof(uint4) * c->num_puzzles <= kMaxDynLds;
        const size_t shm = base + (lds_t ? sizeof(uint4) * c->num_puzzles : 0);
        dispatch_w_tb(c->W, c->cfg.traceback, [&](auto w, auto tb) {
            constexpr int W = decltype(w)::value;
            constexpr bool TB = decltype(tb)::value;
            if constexpr (W > 1) {
                auto launch = [&](auto kern, const uint8_t* a) {
                    if (shm > 64 * 1024 && (lds_rc = allow_big_lds(c, reinterpret_cast<const void*>(kern)))) return;
                    kern<<<dim3((unsigned)blocks), kBlock1s, shm, c->stream>>>(p, g, c->t_mroww, c->t_boardw, T16, a, seed,
                                                                              t0, d_rew, d_flags, st);
                };
                auto go = [&](auto ior) {
                    constexpr bool IOR = decltype(ior)::value;
                    if (d_act) {
                        if (lds_t) launch(k_rolloutWs<W, TB, false, true, IOR>, d_act);
                        else launch(k_rolloutWs<W, TB, false, false, IOR>, d_act);
                    } else {
                        if (lds_t) launch(k_rolloutWs<W, TB, true, true, IOR>, nullptr);
                        else launch(k_rolloutWs<W, TB, true, false, IOR>, nullptr);
                    }
                };
                // IOR (next-step autoreset): reward codes and counters on the I/O waves (k_rollout1s)
                if (p.autoreset == 1 && !c->io_codes_off) go(std::true_type{});
                else go(std::false_type{});
            }
        });
        if (lds_rc) return lds_rc;
        rc = launch_check(c);
        if (rc || T16 == T) return rc;
        const size_t adv = (size_t)T16 * c->n;
        if (d_act) d_act += adv;
        if (d_rew) d_rew += adv;
        if (d_flags) d_flags += adv;
        t0 += (uint64_t)T16;
        T -= T16;
    }
    if (ot && !c->obs_inline) {
        // the 'new' planes by writer waves (k_rollout_obsw): 256-env workgroups, one barrier per step
        dispatch_w_tb(c->W, c->cfg.traceback, [&](auto w, auto tb) {
            constexpr int W = decltype(w)::value;
            constexpr bool TB = decltype(tb)::value;
            const size_t shm = obsw_lds_bytes<W, TB>();
            const dim3 g((unsigned)((c->n + 255) / 256));
            auto launch = [&](auto kern, const uint8_t* a) {
                if (shm > 64 * 1024 && (lds_rc = allow_big_lds(c, reinterpret_cast<const void*>(kern)))) return;
                kern<<<g, kBlockOw, shm, c->stream>>>(p, T, a, seed, t0, d_rew, d_flags, st, *ot);
            };
            if (d_act) launch(k_rollout_obsw<W, TB, false>, d_act);
            else launch(k_rollout_obsw<W, TB, true>, nullptr);
        });
        if (lds_rc) return lds_rc;
        return launch_check(c);
    }
    dispatch_w_tb(c->W, c->cfg.traceback, [&](auto w, auto tb) {
        constexpr int W = decltype(w)::value;
        constexpr bool TB = decltype(tb)::value;
        auto go = [&](auto epw_c, auto obs_c, auto rules_c) {
            constexpr int EPW = decltype(epw_c)::value;
            constexpr bool OBS = decltype(obs_c)::value;
            constexpr bool RULES = decltype(rules_c)::value;
            if constexpr (W == 1 && !OBS && !RULES) return;   // k_rollout1 above
            constexpr size_t kEnvsPerBlock = (size_t)kWaves * EPW / (RULES ? kAuditWaves : 1);   // RULES: wave groups
            const size_t blocks = (c->n + kEnvsPerBlock - 1) / kEnvsPerBlock;
            const size_t per_cu = (blocks + 255) / 256;
            const size_t budget = std::min(kMaxDynLds, (size_t)160 * 1024 / (per_cu ? per_cu : 1));
            const size_t base = tiles_lds_bytes<W, EPW>() + stack_lds_bytes<W, TB, EPW>() + (OBS ? obs_lds_bytes<W>() : 0) +
                                (RULES ? bits_lds_bytes<EPW>() : 0);
            const size_t tbytes = table_lds_bytes<W>(c->num_puzzles);
            const bool lds_table = base + tbytes <= budget;
            const size_t shm = base + (lds_table ? tbytes : 0);
            const dim3 g((unsigned)blocks);
            auto launch = [&](auto kern, const uint8_t* a) {
                if (shm > 64 * 1024 && (lds_rc = allow_big_lds(c, reinterpret_cast<const void*>(kern)))) return;
                kern<<<g, kBlock, shm, c->stream>>>(p, T, a, seed, t0, d_rew, d_flags, st, tiled, ot ? *ot : no_obs,
                                                    rtr ? *rtr : no_rules);
            };
            if (d_act) {
                if (lds_table) launch(k_rollout<W, TB, false, true, EPW, OBS, RULES>, d_act);
                else launch(k_rollout<W, TB, false, false, EPW, OBS, RULES>, d_act);
            } else {
                if (lds_table) launch(k_rollout<W, TB, true, true, EPW, OBS, RULES>, nullptr);
                else launch(k_rollout<W, TB, true, false, EPW, OBS, RULES>, nullptr);
            }
        };
        using E64 = std::integral_constant<int, 64>;
        if (ot) go(E64{}, std::true_type{}, std::false_type{});
        else if (rtr) go(E64{}, std::false_type{}, std::true_type{});
        else if (half) go(std::integral_constant<int, 32>{}, std::false_type{}, std::false_type{});
        else go(E64{}, std::false_type{}, std::false_type{});
    });
    if (lds_rc) return lds_rc;
    return launch_check(c);
}

// The state, exact-fit memo and stats a generic rule rollout starts from, saved to / restored from
// Ctx::snap on the context's stream (sparc_rules_finish re-runs a call whose queue overflowed)
int snapshot(Ctx* c, int32_t* d_stats, bool save) {
    const size_t n = c->n, W = (size_t)c->W;
    const std::pair<void*, size_t> parts[] = {
        {c->vis, 8 * W * n}, {c->dirs, c->cfg.traceback ? 16 * W * n : 0}, {c->pos, 4 * n}, {c->aux, 4 * n},
        {c->step, 4 * n}, {c->pid, 4 * n}, {c->r_memo, sizeof(FitMemo<kMemo>) * n}, {d_stats, d_stats ? 16 * n : 0}};
    size_t total = 0;
    for (const auto& pt : parts) total += (pt.first ? pt.second : 0);
    if (save && total > c->snap_bytes) {
        if (c->snap) HIPCHK(c, hipFree(c->snap));
        c->snap = nullptr;
        c->snap_bytes = 0;
        HIPCHK(c, hipMalloc(&c->snap, total));
        c->snap_bytes = total;
    }
    size_t off = 0;
    for (const auto& pt : parts) {
        if (!pt.first || !pt.second) continue;
        uint8_t* sp = static_cast<uint8_t*>(c->snap) + off;
        if (save) HIPCHK(c, hipMemcpyAsync(sp, pt.first, pt.second, hipMemcpyDeviceToDevice, c->stream));
        else HIPCHK(c, hipMemcpyAsync(pt.first, sp, pt.second, hipMemcpyDeviceToDevice, c->stream));
        off += pt.second;
    }
    return SPARC_OK;
}

// launch the recorded audit call (sparc_rules_device / sparc_rollout_rules_device)
int launch_rules(Ctx* c, const AuditCall& a) {
    if (a.kind == 2) {
        const RuleTrace rtr{rules_tab(c, true), a.bits, c->r_memo};
        const bool generic = c->rules_generic;
        if (a.snap) c->rules_generic = true;   // the kernel the call was recorded with
        const int rc = rollout_impl(c, a.T, a.act, a.seed, a.t0, a.rew, a.flags, a.stats, nullptr, &rtr);
        c->rules_generic = generic;
        return rc;
    }
    const Params p = make_params(c);
    const RulesTab rt = rules_tab(c, true);
    const dim3 g = grid_for(c->n);
    if (c->W == 1) k_rules<1><<<g, kBlock, 0, c->stream>>>(p, rt, a.bits, a.region, a.fit, c->r_memo);
    else if (c->W == 2) k_rules<2><<<g, kBlock, 0, c->stream>>>(p, rt, a.bits, a.region, a.fit, c->r_memo);
    else k_rules<4><<<g, kBlock, 0, c->stream>>>(p, rt, a.bits, a.region, a.fit, c->r_memo);
    return launch_check(c);
}

int check_obs_dims(Ctx* c, int32_t xd, int32_t yd) {
    if (xd < 1 || yd < 1 || (uint32_t)xd * (uint32_t)yd > kObsCells)
        return fail(c, SPARC_E_INVALID, "observation planes need x_dim, y_dim >= 1 and x_dim * y_dim <= 256");
    return SPARC_OK;
}
}  // namespace

extern "C" {

int sparc_rollout_device(void* ctx, int32_t T, const uint8_t* d_act, uint64_t seed, uint64_t t0, int8_t* d_rew,
                         uint8_t* d_flags, int32_t* d_stats) {
    return rollout_impl(static_cast<Ctx*>(ctx), T, d_act, seed, t0, d_rew, d_flags, d_stats, nullptr);
}

int sparc_rollout_obs_device(void* ctx, int32_t T, const uint8_t* d_act, uint64_t seed, uint64_t t0,
                             int8_t* d_rew, uint8_t* d_flags, int32_t* d_stats, int32_t* d_visited,
                             int32_t* d_agent, int32_t x_dim, int32_t y_dim) {
    DevGuard dg;
    Ctx* c = static_cast<Ctx*>(ctx);
    if (!c) return fail(nullptr, SPARC_E_INVALID, "null context");
    int rc = check_obs_dims(c, x_dim, y_dim);
    if (rc) return rc;
    if (!d_visited && !d_agent) return rollout_impl(c, T, d_act, seed, t0, d_rew, d_flags, d_stats, nullptr);
    const ObsTrace ot{d_visited, d_agent, (uint32_t)x_dim, (uint32_t)y_dim};
    return rollout_impl(c, T, d_act, seed, t0, d_rew, d_flags, d_stats, &ot);
}

int sparc_rollout_rules_device(void* ctx, int32_t T, const uint8_t* d_act, uint64_t seed, uint64_t t0,
                               int8_t* d_rew, uint8_t* d_flags, int32_t* d_stats, uint16_t* d_rule_bits) {
    DevGuard dg;
    Ctx* c = static_cast<Ctx*>(ctx);
    int rc = check_ctx(c, true);
    if (rc) return rc;
    if (!c->rules) return fail(c, SPARC_E_STATE, "sparc_load_rules has not been called");
    if (!d_rule_bits) return fail(c, SPARC_E_INVALID, "null rule_bits");
    if (T < 0) return fail(c, SPARC_E_INVALID, "T must be >= 0");
    HIPCHK(c, hipMemsetAsync(c->fq_count, 0, sizeof(*c->fq_count), c->stream));
    AuditCall a;
    a.kind = 2;
    a.extent = (uint64_t)T * c->n;
    a.bits = d_rule_bits;
    a.T = T;
    a.act = d_act;
    a.seed = seed;
    a.t0 = t0;
    a.rew = d_rew;
    a.flags = d_flags;
    a.stats = d_stats;
    // the generic rule kernel queues searches past the node cap: keep the state it starts from, so
    // that sparc_rules_finish can run the call again on a larger queue (k_rollout1r never queues).
    // The call records which it was: finish re-runs exactly this kernel, whatever
    // sparc_set_variant has selected since
    a.snap = !r1r_rollout(c);
    c->last_audit = a;
    if (a.snap) {
        rc = snapshot(c, d_stats, true);
        if (rc) return rc;
    }
    return launch_rules(c, a);
}

int sparc_step_obs_device(void* ctx, const uint8_t* d_act, int8_t* d_rew, uint8_t* d_flags, int32_t* d_visited,
                          int32_t* d_agent, int32_t x_dim, int32_t y_dim, uint32_t* d_puzzle, uint32_t* d_xy) {
    DevGuard dg;
    Ctx* c = static_cast<Ctx*>(ctx);
    int rc = check_ctx(c, true);
    if (rc) return rc;
    if (!d_act || !d_rew || !d_flags) return fail(c, SPARC_E_INVALID, "null argument");
    rc = check_obs_dims(c, x_dim, y_dim);
    if (rc) return rc;
    const Params p = make_params(c);
    const GymOut g{d_act, 1u, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
    dispatch_w_tb(c->W, c->cfg.traceback, [&](auto w, auto tb) {
        k_step_obs<decltype(w)::value, decltype(tb)::value><<<grid_for(c->n), kBlock, 0, c->stream>>>(
            p, g, d_rew, d_flags, d_visited, d_agent, (uint32_t)x_dim, (uint32_t)y_dim, d_puzzle, d_xy);
    });
    return launch_check(c);
}

int sparc_step_gym_device(void* ctx, const void* d_act, int32_t action_bytes, double* d_reward, uint8_t* d_term,
                          uint8_t* d_trunc, uint8_t* d_legal, uint8_t* d_areset, int8_t* d_rew_code,
                          uint8_t* d_flags, int32_t* d_visited, int32_t* d_agent, int32_t x_dim, int32_t y_dim,
                          uint32_t* d_puzzle, int32_t* d_loc) {
    DevGuard dg;
    Ctx* c = static_cast<Ctx*>(ctx);
    int rc = check_ctx(c, true);
    if (rc) return rc;
    if (!d_act) return fail(c, SPARC_E_INVALID, "null actions");
    if (action_bytes != 1 && action_bytes != 4 && action_bytes != 8)
        return fail(c, SPARC_E_INVALID, "action_bytes must be 1, 4 or 8");
    if (d_visited || d_agent) {
        rc = check_obs_dims(c, x_dim, y_dim);
        if (rc) return rc;
    } else {
        x_dim = y_dim = 1;
    }
    const Params p = make_params(c);
    const GymOut g{d_act, (uint32_t)action_bytes, d_reward, d_term, d_trunc, d_legal, d_areset, d_loc};
    dispatch_w_tb(c->W, c->cfg.traceback, [&](auto w, auto tb) {
        k_step_obs<decltype(w)::value, decltype(tb)::value><<<grid_for(c->n), kBlock, 0, c->stream>>>(
            p, g, d_rew_code, d_flags, d_visited, d_agent, (uint32_t)x_dim, (uint32_t)y_dim, d_puzzle, nullptr);
    });
    return launch_check(c);
}

int sparc_obs_pack_device(void* ctx, int32_t* d_vis, int32_t* d_agent, int32_t xd, int32_t yd) {
    DevGuard dg;
    Ctx* c = static_cast<Ctx*>(ctx);
    int rc = check_ctx(c, true);
    if (rc) return rc;
    if (xd < 1 || yd < 1 || xd > 255 || yd > 255) return fail(c, SPARC_E_INVALID, "bad plane dims");
    const Params p = make_params(c);
    const size_t total = (size_t)c->n * xd * yd;
    const dim3 g = grid_for(total);
    if (c->W == 1) k_obs_pack<1><<<g, kBlock, 0, c->stream>>>(p, d_vis, d_agent, xd, yd);
    else if (c->W == 2) k_obs_pack<2><<<g, kBlock, 0, c->stream>>>(p, d_vis, d_agent, xd, yd);
    else k_obs_pack<4><<<g, kBlock, 0, c->stream>>>(p, d_vis, d_agent, xd, yd);
    return launch_check(c);
}

int sparc_load_rules(void* ctx, const sparc_rules_table* t) {
    DevGuard dg;
    Ctx* c = static_cast<Ctx*>(ctx);
    int rc = check_ctx(c, false);
    if (rc) return rc;
    if (!t || !t->planes || !t->inst_first || !t->shape_first) return fail(c, SPARC_E_INVALID, "null argument");
    if ((uint32_t)t->num_puzzles != c->num_puzzles)
        return fail(c, SPARC_E_INVALID, "rule table puzzle count differs from the loaded puzzle table");
    if (t->num_inst < 0 || t->num_shapes < 0 || t->num_offsets < 0 || t->num_shapes >= (1 << 21) ||
        (t->num_inst && !t->inst) || (t->num_shapes && !t->shape_area) || (t->num_offsets && !t->shape_off))
        return fail(c, SPARC_E_INVALID, "bad rule table sizes");
    const int W = c->W;
    const size_t P = (size_t)t->num_puzzles, S = (size_t)t->num_shapes;
    std::vector<uint4> info(P);
    HIPCHK(c, hipMemcpy(info.data(), c->t_info, sizeof(uint4) * P, hipMemcpyDeviceToHost));
    // the device's ranges: {first, count} per shape and {first, count | kHostFit} per puzzle
    std::vector<uint2> srange(std::max<size_t>(1, S), make_uint2(0u, 0u)), ifc(P);
    if (t->shape_first[0] != 0) return fail(c, SPARC_E_INVALID, "shape offsets must start at 0");
    for (size_t sh = 0; sh < S; ++sh) {
        const uint32_t o0 = t->shape_first[sh], o1 = t->shape_first[sh + 1];
        if (o1 < o0 || o1 > (uint32_t)t->num_offsets) return fail(c, SPARC_E_INVALID, "shape offsets out of range");
        srange[sh] = make_uint2(o0, o1 - o0);
    }
    if (t->inst_first[0] != 0) return fail(c, SPARC_E_INVALID, "instance offsets must start at 0");
    size_t host_fit_puzzles = 0;
    for (size_t q = 0; q < P; ++q) {
        const uint32_t X = info[q].x & 0xFFu, Y = (info[q].x >> 8) & 0xFFu;
        const uint32_t f = t->inst_first[q], f1 = t->inst_first[q + 1];
        char m[160];
        if (X > 15 || Y > 15) {
            snprintf(m, sizeof m, "puzzle %zu: the rule audit supports lattices up to 15x15", q);
            return fail(c, SPARC_E_INVALID, m);
        }
        if (f1 < f || f1 > (uint32_t)t->num_inst) return fail(c, SPARC_E_INVALID, "instance range out of bounds");
        const uint32_t n = f1 - f;
        const uint32_t cells = ((X - 1) / 2) * ((Y - 1) / 2);
        if (n > cells) {   // _extract_poly_instances: one instance per cell centre
            snprintf(m, sizeof m, "puzzle %zu: %u instances on %u cells", q, n, cells);
            return fail(c, SPARC_E_INVALID, m);
        }
        int ny = 0, nd = 0;
        uint32_t ds[kHostFitMax];
        for (uint32_t k = 0; k < n; ++k) {
            const uint32_t e = t->inst[f + k], b = e & 0x3FFu, sh = e >> 11;
            if (b >= 64u * W || sh >= (uint32_t)S) return fail(c, SPARC_E_INVALID, "bad instance");
            if ((e >> 10) & 1u) { ++ny; continue; }
            int j = 0;
            while (j < nd && ds[j] != sh) ++j;
            if (j == nd) ds[nd++] = sh;
        }
        // past the GPU search's list sizes: the puzzle's searches run on the host (kHostFit)
        const bool hf = ny > kFitYlops || nd > kFitShapes;
        host_fit_puzzles += hf;
        ifc[q] = make_uint2(f, n | (hf ? kHostFit : 0u));
    }
    void* old[] = {c->r_planes, c->r_inst_fc, c->r_inst, c->r_shape_range, c->r_shape_area, c->r_shape_off,
                   c->r_reg_off, c->r_reg_tab, c->r_rows};
    for (void* b : old)
        if (b) HIPCHK(c, hipFree(b));
    c->r_planes = nullptr; c->r_inst_fc = nullptr; c->r_inst = nullptr;
    c->r_shape_range = nullptr; c->r_shape_area = nullptr; c->r_shape_off = nullptr;
    c->r_reg_off = nullptr; c->r_reg_tab = nullptr; c->r_rows = nullptr;
    c->rules = false;
    c->r_tab_all = false;
    c->host_fit_puzzles = host_fit_puzzles;
    // the device copy: the caller's SPARC_RULE_PLANES planes per puzzle, RP_INST rewritten from the
    // instance list, then the bit-sliced net area of each cell (kAreaPlanes planes, sparc_rules.hpp)
    static_assert(RP_ABI == SPARC_RULE_PLANES, "rule plane layout");
    const size_t np_ = P * RP_COUNT * W;
    std::vector<uint64_t> dev_planes(np_, 0ull);
    bool area_ok = true;
    for (size_t q = 0; q < P; ++q) {
        uint64_t* d = dev_planes.data() + q * RP_COUNT * W;
        std::copy(t->planes + q * RP_ABI * W, t->planes + (q + 1) * RP_ABI * W, d);
        for (int k = 0; k < W; ++k) d[RP_INST * W + k] = 0;
        int32_t net[256] = {0};
        const uint32_t f = ifc[q].x, n = ifc[q].y & ~kHostFit;
        for (uint32_t k = 0; k < n; ++k) {
            const uint32_t e = t->inst[f + k], b = e & 0x3FFu;
            const int64_t a = t->shape_area[e >> 11];
            net[b] = (int32_t)std::max<int64_t>(-(1 << 20), std::min<int64_t>(1 << 20, net[b] + (((e >> 10) & 1u) ? -a : a)));
            d[RP_INST * W + (b >> 6)] |= 1ull << (b & 63);
        }
        for (uint32_t b = 0; b < 64u * W; ++b) {
            if (net[b] < -(1 << (kAreaPlanes - 1)) || net[b] >= (1 << (kAreaPlanes - 1))) area_ok = false;
            for (int k = 0; k < kAreaPlanes; ++k)
                if (((uint32_t)net[b] >> k) & 1u) d[(RP_AREA0 + k) * W + (b >> 6)] |= 1ull << (b & 63);
        }
    }
    const size_t ni = std::max<size_t>(1, t->num_inst), ns = std::max<size_t>(1, t->num_shapes),
                 no = std::max<size_t>(1, t->num_offsets);
    HIPCHK(c, hipMalloc(&c->r_planes, sizeof(uint64_t) * np_));
    HIPCHK(c, hipMalloc(&c->r_inst_fc, sizeof(uint2) * P));
    HIPCHK(c, hipMalloc(&c->r_inst, sizeof(uint32_t) * ni));
    HIPCHK(c, hipMalloc(&c->r_shape_range, sizeof(uint2) * ns));
    HIPCHK(c, hipMalloc(&c->r_shape_area, sizeof(int32_t) * ns));
    HIPCHK(c, hipMalloc(&c->r_shape_off, 2 * no));
    HIPCHK(c, hipMemcpy(c->r_planes, dev_planes.data(), sizeof(uint64_t) * np_, hipMemcpyHostToDevice));
    c->r_area = area_ok;   // a cell's net area outside -128..127: the audit walks the list instead
    HIPCHK(c, hipMemcpy(c->r_inst_fc, ifc.data(), sizeof(uint2) * P, hipMemcpyHostToDevice));
    if (t->num_inst) HIPCHK(c, hipMemcpy(c->r_inst, t->inst, sizeof(uint32_t) * t->num_inst, hipMemcpyHostToDevice));
    HIPCHK(c, hipMemcpy(c->r_shape_range, srange.data(), sizeof(uint2) * ns, hipMemcpyHostToDevice));
    if (S) HIPCHK(c, hipMemcpy(c->r_shape_area, t->shape_area, sizeof(int32_t) * S, hipMemcpyHostToDevice));
    if (t->num_offsets) HIPCHK(c, hipMemcpy(c->r_shape_off, t->shape_off, 2 * (size_t)t->num_offsets, hipMemcpyHostToDevice));
    // host copies for the exact fits the host finishes (searches past the node cap, kHostFit puzzles)
    c->h_inst.assign(t->inst, t->inst + t->num_inst);
    c->h_inst.resize(ni, 0u);
    c->h_inst_fc = ifc;
    c->h_shape_range = srange;
    c->h_shape_off.assign(t->shape_off, t->shape_off + 2 * (size_t)t->num_offsets);
    c->h_shape_off.resize(2 * no, 0);
    if (!c->fq_count) {
        HIPCHK(c, hipMalloc(&c->fq_count, sizeof(*c->fq_count)));
        HIPCHK(c, hipMalloc(&c->fq_items, sizeof(FitTodo) * kFitQueueCap));
        c->fq_cap = kFitQueueCap;
    }
    HIPCHK(c, hipMemset(c->fq_count, 0, sizeof(*c->fq_count)));
    c->last_audit = AuditCall{};
    // the host's answers name puzzles of the old table
    c->hf_used = 0;
    std::fill(c->h_hf.begin(), c->h_hf.end(), make_uint4(0u, 0u, 0u, 0u));
    // the memo's entries name puzzles of the old table: start empty (a zero key matches no region)
    if (!c->r_memo) HIPCHK(c, hipMalloc(&c->r_memo, sizeof(FitMemo<kMemo>) * (size_t)c->n));
    HIPCHK(c, hipMemset(c->r_memo, 0, sizeof(FitMemo<kMemo>) * (size_t)c->n));
    // the per-region check code (squares, stars, poly/ylop area + exact fit) of every region cell
    // mask of each puzzle with at most kRegTabCells cells, computed once here by the audit's own
    // region_code (k_region_table): the audit then looks codes up per region instead of running
    // the checks (the memo serves the larger puzzles, and the puzzles past the table budget:
    // 2^28 entries, 128 MB, unless sparc_set_rule_limits sets another).  An exact fit that passes
    // the node cap here is finished on the host, so the table holds only final answers.
    std::vector<uint32_t> reg_off(P, kNoRegTab);
    std::vector<uint2> items;
    size_t entries = 0;
    const size_t kMaxRegEntries = c->reg_entries;
    for (size_t q = 0; q < P; ++q) {
        const uint32_t X = info[q].x & 0xFFu, Y = (info[q].x >> 8) & 0xFFu;
        const uint32_t cells = ((X - 1) / 2) * ((Y - 1) / 2);
        if (cells > kRegTabCells) continue;
        const uint32_t words = cells <= 3 ? 1u : 1u << (cells - 3);
        if (entries + 8u * words > kMaxRegEntries) break;
        reg_off[q] = (uint32_t)entries;
        for (uint32_t g = 0; g < words; ++g) items.push_back(make_uint2((uint32_t)q, g));
        entries += 8u * words;
    }
    c->r_tab_all = std::none_of(reg_off.begin(), reg_off.end(), [](uint32_t o) { return o == kNoRegTab; });
    if (!items.empty()) {
        const size_t words = entries / 8;
        uint2* d_items = nullptr;
        HIPCHK(c, hipMalloc(&c->r_reg_off, sizeof(uint32_t) * P));
        HIPCHK(c, hipMalloc(&c->r_reg_tab, sizeof(uint32_t) * words));
        HIPCHK(c, hipMalloc(&d_items, sizeof(uint2) * items.size()));
        HIPCHK(c, hipMemcpy(c->r_reg_off, reg_off.data(), sizeof(uint32_t) * P, hipMemcpyHostToDevice));
        HIPCHK(c, hipMemcpy(d_items, items.data(), sizeof(uint2) * items.size(), hipMemcpyHostToDevice));
        const Params p = make_params(c);
        RulesTab rt = rules_tab(c, false);
        rt.reg_tab = nullptr;
        const dim3 g((unsigned)((items.size() + kBlock - 1) / kBlock));
        const uint32_t n_items = (uint32_t)items.size();
        if (W == 1) k_region_table<1><<<g, kBlock, 0, c->stream>>>(p, rt, d_items, n_items, c->r_reg_tab, c->fq_count);
        else if (W == 2) k_region_table<2><<<g, kBlock, 0, c->stream>>>(p, rt, d_items, n_items, c->r_reg_tab, c->fq_count);
        else k_region_table<4><<<g, kBlock, 0, c->stream>>>(p, rt, d_items, n_items, c->r_reg_tab, c->fq_count);
        rc = launch_check(c);
        HIPCHK(c, hipStreamSynchronize(c->stream));
        HIPCHK(c, hipFree(d_items));
        if (rc) return rc;
        unsigned long long exhausted = 0;
        HIPCHK(c, hipMemcpy(&exhausted, c->fq_count, sizeof(exhausted), hipMemcpyDeviceToHost));
        if (exhausted) {   // finish those searches on the host and rewrite their codes
            HIPCHK(c, hipMemset(c->fq_count, 0, sizeof(*c->fq_count)));
            std::vector<uint32_t> tab(words);
            HIPCHK(c, hipMemcpy(tab.data(), c->r_reg_tab, sizeof(uint32_t) * words, hipMemcpyDeviceToHost));
            parallel_for(items.size(), [&](size_t k) {   // each word belongs to one item
                const uint2 it = items[k];
                uint32_t& w = tab[reg_off[it.x] / 8u + it.y];
                for (uint32_t j = 0; j < 8; ++j) {
                    const uint32_t sh = 4u * j + kRcPolyShift;
                    if (((w >> sh) & 3u) != 3u) continue;
                    const uint32_t poly = host_fit(c, it.x, 8ull * it.y + j) ? 1u : 2u;
                    w = (w & ~(3u << sh)) | (poly << sh);
                }
            });
            HIPCHK(c, hipMemcpy(c->r_reg_tab, tab.data(), sizeof(uint32_t) * words, hipMemcpyHostToDevice));
        }
    }
    // the audit's per-puzzle rows (RulesTab::rows): base planes, table offset, instance range, info
    {
        const size_t RW = W == 1 ? rule_row_u64<1>() : W == 2 ? rule_row_u64<2>() : rule_row_u64<4>();
        std::vector<uint64_t> rows(P * RW, 0ull);
        for (size_t q = 0; q < P; ++q) {
            uint64_t* r = rows.data() + q * RW;
            for (int k = 0; k < 10; ++k)
                for (int w = 0; w < W; ++w) r[k * W + w] = dev_planes[(q * RP_COUNT + kBasePlanes[k]) * W + w];
            // info.y bits 24-31 (free: flags use 16-18) carry the instance count | kHostFit << 7
            const uint32_t cf = (ifc[q].y & 0x7Fu) | ((ifc[q].y & kHostFit) ? 0x80u : 0u);
            r[10 * W] = (uint64_t)reg_off[q] | ((uint64_t)ifc[q].x << 32);
            r[10 * W + 1] = (uint64_t)info[q].x | ((uint64_t)((info[q].y & 0x00FFFFFFu) | (cf << 24)) << 32);
        }
        HIPCHK(c, hipMalloc(&c->r_rows, sizeof(uint64_t) * rows.size()));
        HIPCHK(c, hipMemcpy(c->r_rows, rows.data(), sizeof(uint64_t) * rows.size(), hipMemcpyHostToDevice));
    }
    c->rules = true;
    return SPARC_OK;
}

}  // extern "C"

namespace {
// per-env audit outputs of the host-pointer / one-env calls (device scratch)
int audit_scratch(Ctx* c) {
    if (c->s_bits) return SPARC_OK;
    const size_t n = c->n;
    HIPCHK(c, hipMalloc(&c->s_bits, 2 * n));
    HIPCHK(c, hipMalloc(&c->s_region, n * 64 * c->W));
    HIPCHK(c, hipMalloc(&c->s_fit, 8 * n));
    return SPARC_OK;
}

// the FitQueue count of the last audit call (one stream sync)
int read_queue_count(Ctx* c, uint64_t& n) {
    if (!c->h_count) HIPCHK(c, hipHostMalloc(reinterpret_cast<void**>(&c->h_count), sizeof(uint64_t), hipHostMallocDefault));
    HIPCHK(c, hipMemcpyAsync(c->h_count, c->fq_count, sizeof(uint64_t), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    n = *c->h_count;
    return SPARC_OK;
}

// one answer into the host mirror of HostFits (false: already there)
bool hostfits_insert(std::vector<uint4>& t, uint32_t q, uint64_t rm, uint32_t fits) {
    const uint32_t mask = (uint32_t)t.size() - 1u;
    for (uint32_t s = hostfit_slot(q, rm, mask);; s = (s + 1u) & mask) {
        uint4& e = t[s];
        if (!(e.w & 2u)) {
            e = make_uint4((uint32_t)rm, (uint32_t)(rm >> 32), q, fits | 2u);
            return true;
        }
        if (e.x == (uint32_t)rm && e.y == (uint32_t)(rm >> 32) && e.z == q) return false;
    }
}

// Keep the answers of one finish for later audits (sparc_rules.hpp HostFits): the table grows to
// keep its load factor <= 1/2, up to kHostFitsMax slots (64 MB); past that new answers are not
// kept (audits then queue those searches again; the results are the same).
constexpr size_t kHostFitsMin = (size_t)1 << 12, kHostFitsMax = (size_t)1 << 22;
int hostfits_add(Ctx* c, const std::vector<std::pair<uint32_t, uint64_t>>& keys, const std::vector<int8_t>& res) {
    if (c->hostfits_off) return SPARC_OK;
    const size_t need = (size_t)c->hf_used + keys.size();
    size_t cap = c->h_hf.size();
    if (2 * need > cap && cap < kHostFitsMax) {
        size_t ncap = std::max(cap, kHostFitsMin);
        while (2 * need > ncap && ncap < kHostFitsMax) ncap *= 2;
        std::vector<uint4> t(ncap, make_uint4(0u, 0u, 0u, 0u));
        for (const uint4& e : c->h_hf)
            if (e.w & 2u) hostfits_insert(t, e.z, (uint64_t)e.x | ((uint64_t)e.y << 32), e.w & 1u);
        c->h_hf.swap(t);
        if (c->d_hf) HIPCHK(c, hipFree(c->d_hf));
        c->d_hf = nullptr;
        HIPCHK(c, hipMalloc(&c->d_hf, sizeof(uint4) * ncap));
    }
    bool added = false;
    for (size_t k = 0; k < keys.size() && 2 * ((size_t)c->hf_used + 1) <= c->h_hf.size(); ++k)
        if (hostfits_insert(c->h_hf, keys[k].first, keys[k].second, res[k] == 1 ? 1u : 0u)) {
            ++c->hf_used;
            added = true;
        }
    if (added) HIPCHK(c, hipMemcpyAsync(c->d_hf, c->h_hf.data(), sizeof(uint4) * c->h_hf.size(), hipMemcpyHostToDevice, c->stream));
    return SPARC_OK;
}

// sparc_rules_finish once the queue count of the last audit call is known (cnt entries pushed)
int finish_queue(Ctx* c, uint64_t cnt, uint16_t* d_bits, uint64_t* d_fit) {
    int rc = SPARC_OK;
    c->fq_last = cnt;
    if (cnt == 0) return SPARC_OK;
    const AuditCall a = c->last_audit;
    if (a.kind == 0) return fail(c, SPARC_E_STATE, "queued exact-fit searches without a recorded audit call");
    if (!d_bits || d_bits != a.bits) return fail(c, SPARC_E_STATE, "sparc_rules_finish: not the last audit call's bits");
    if (cnt > c->fq_cap) {
        // the queue overflowed: a larger queue, and the call again from where it started (an
        // audit is deterministic: the same searches are queued, and the memo holds final answers)
        if (a.kind == 2 && !a.snap) return fail(c, SPARC_E_STATE, "queue overflow of a rule rollout without a snapshot");
        uint64_t cap = c->fq_cap;
        while (cap < cnt) cap *= 2;
        if (cap > kFitQueueMax) return fail(c, SPARC_E_NOMEM, "exact-fit queue past 2^28 entries in one audit call");
        HIPCHK(c, hipFree(c->fq_items));
        c->fq_items = nullptr;
        c->fq_cap = 0;
        HIPCHK(c, hipMalloc(&c->fq_items, sizeof(FitTodo) * cap));
        c->fq_cap = cap;
        if (a.kind == 2 && (rc = snapshot(c, a.stats, false))) return rc;
        HIPCHK(c, hipMemsetAsync(c->fq_count, 0, sizeof(*c->fq_count), c->stream));
        if ((rc = launch_rules(c, a))) return rc;
        ++c->fq_reruns;
        if ((rc = read_queue_count(c, cnt))) return rc;
        if (cnt > c->fq_cap) return fail(c, SPARC_E_STATE, "exact-fit queue overflow on the re-run");
    }
    std::vector<FitTodo> todo(cnt);
    HIPCHK(c, hipMemcpy(todo.data(), c->fq_items, sizeof(FitTodo) * cnt, hipMemcpyDeviceToHost));
    c->fq_last = cnt;
    for (const FitTodo& it : todo)
        if (it.pos >= a.extent || it.q >= c->num_puzzles)
            return fail(c, SPARC_E_STATE, "exact-fit queue entry outside the last audit call");
    // each distinct (puzzle, region cells) search once, on up to 16 host threads
    std::vector<std::pair<uint32_t, uint64_t>> keys(cnt);
    for (uint64_t k = 0; k < cnt; ++k) keys[k] = {todo[k].q, todo[k].rm};
    std::sort(keys.begin(), keys.end());
    keys.erase(std::unique(keys.begin(), keys.end()), keys.end());
    std::vector<int8_t> res(keys.size(), 0);
    parallel_for(keys.size(), [&](size_t k) { res[k] = (int8_t)host_fit(c, keys[k].first, keys[k].second); });
    auto fits = [&](uint32_t q, uint64_t rm) {
        const auto it = std::lower_bound(keys.begin(), keys.end(), std::make_pair(q, rm));
        return res[(size_t)(it - keys.begin())] == 1;
    };
    // per output entry: every queued region's answer (all must fit for poly_ylop_area), and the
    // fit mask of the regions that do
    std::sort(todo.begin(), todo.end(), [](const FitTodo& x, const FitTodo& y) { return x.pos < y.pos; });
    std::vector<RulePatch> patch;
    for (size_t k = 0; k < todo.size();) {
        RulePatch r{todo[k].pos, 0ull, SPARC_RULE_SEARCH_EXHAUSTED, 0u};
        bool ok = true;
        for (; k < todo.size() && todo[k].pos == r.pos; ++k) {
            const bool f = fits(todo[k].q, todo[k].rm);
            ok &= f;
            if (f) r.fit_or |= 1ull << (todo[k].rid & 63u);
        }
        if (!ok) r.clear |= SPARC_RULE_POLY_YLOP | SPARC_RULE_ALL;
        patch.push_back(r);
    }
    RulePatch* d_patch = nullptr;
    HIPCHK(c, hipMalloc(&d_patch, sizeof(RulePatch) * patch.size()));
    HIPCHK(c, hipMemcpyAsync(d_patch, patch.data(), sizeof(RulePatch) * patch.size(), hipMemcpyHostToDevice, c->stream));
    k_rule_patch<<<grid_for(patch.size()), kBlock, 0, c->stream>>>(d_patch, (uint32_t)patch.size(), d_bits, d_fit);
    rc = launch_check(c);
    HIPCHK(c, hipMemsetAsync(c->fq_count, 0, sizeof(*c->fq_count), c->stream));
    if (!rc) rc = hostfits_add(c, keys, res);
    HIPCHK(c, hipStreamSynchronize(c->stream));
    HIPCHK(c, hipFree(d_patch));
    return rc;
}
}  // namespace

extern "C" {

int sparc_rules_device(void* ctx, uint16_t* d_bits, uint8_t* d_region, uint64_t* d_fit) {
    DevGuard dg;
    Ctx* c = static_cast<Ctx*>(ctx);
    int rc = check_ctx(c, true);
    if (rc) return rc;
    if (!c->rules) return fail(c, SPARC_E_STATE, "sparc_load_rules has not been called");
    // a fresh queue for this call (a caller that skipped sparc_rules_finish leaves no entries that
    // name another call's outputs), and the call recorded for sparc_rules_finish
    HIPCHK(c, hipMemsetAsync(c->fq_count, 0, sizeof(*c->fq_count), c->stream));
    AuditCall a;
    a.kind = 1;
    a.extent = c->n;
    a.bits = d_bits;
    a.region = d_region;
    a.fit = d_fit;
    c->last_audit = a;
    return launch_rules(c, a);
}

int sparc_rules_queue_stats(void* ctx, uint64_t* out) {
    Ctx* c = static_cast<Ctx*>(ctx);
    if (!c || !out) return fail(c, SPARC_E_INVALID, "null argument");
    out[0] = c->fq_cap;
    out[1] = c->fq_last;
    out[2] = c->fq_reruns;
    return SPARC_OK;
}

int sparc_set_variant(void* ctx, int32_t which, int32_t value) {
    Ctx* c = static_cast<Ctx*>(ctx);
    if (!c) return fail(nullptr, SPARC_E_INVALID, "null context");
    switch (which) {
        case SPARC_VARIANT_IO_CODES_OFF:
            if (value != 0 && value != 1) break;
            c->io_codes_off = value == 1;
            return SPARC_OK;
        case SPARC_VARIANT_RULE_ROLLOUT_GENERIC:
            if (value != 0 && value != 1) break;
            c->rules_generic = value == 1;
            return SPARC_OK;
        case SPARC_VARIANT_R1R_SHAPE:
            if (value < 0 || value > 5) break;
            c->r1r_shape = value;
            return SPARC_OK;
        case SPARC_VARIANT_OBS_INLINE:
            if (value != 0 && value != 1) break;
            c->obs_inline = value == 1;
            return SPARC_OK;
        case SPARC_VARIANT_MIXED_TRIE:
            if (value < 0 || value > 2) break;
            c->mixed_trie = value;
            return SPARC_OK;
        case SPARC_VARIANT_HOST_FITS:
            if (value != 0 && value != 1) break;
            c->hostfits_off = value == 1;
            return SPARC_OK;
        default:
            return fail(c, SPARC_E_INVALID, "unknown variant");
    }
    return fail(c, SPARC_E_INVALID, "bad variant value");
}

int sparc_set_rule_limits(void* ctx, uint32_t fit_cap_nodes, uint64_t table_entries) {
    DevGuard dg;
    Ctx* c = static_cast<Ctx*>(ctx);
    if (!c) return fail(nullptr, SPARC_E_INVALID, "null context");
    c->fit_cap = fit_cap_nodes ? fit_cap_nodes : kFitCap;
    c->reg_entries = table_entries ? (size_t)std::min<uint64_t>(table_entries, (uint64_t)1 << 28) : (size_t)1 << 28;
    return SPARC_OK;
}

int sparc_rules_finish(void* ctx, uint16_t* d_bits, uint64_t* d_fit) {
    DevGuard dg;
    Ctx* c = static_cast<Ctx*>(ctx);
    int rc = check_ctx(c, false);
    if (rc) return rc;
    if (!c->rules) return fail(c, SPARC_E_STATE, "sparc_load_rules has not been called");
    uint64_t cnt = 0;
    if ((rc = read_queue_count(c, cnt))) return rc;
    return finish_queue(c, cnt, d_bits, d_fit);
}

int sparc_rules_host(void* ctx, uint16_t* bits, uint8_t* region, uint64_t* fit) {
    DevGuard dg;
    Ctx* c = static_cast<Ctx*>(ctx);
    int rc = check_ctx(c, true);
    if (rc) return rc;
    const size_t n = c->n, rb = n * 64 * c->W;
    if ((rc = audit_scratch(c))) return rc;
    rc = sparc_rules_device(c, c->s_bits, region ? c->s_region : nullptr, fit ? c->s_fit : nullptr);
    if (rc) return rc;
    // the queue count travels with the outputs: one synchronisation when nothing was queued (an
    // exact fit past the GPU's node cap is rare), else the host finishes the searches and the
    // patched bits / fit are read again
    if (!c->h_count) HIPCHK(c, hipHostMalloc(reinterpret_cast<void**>(&c->h_count), sizeof(uint64_t), hipHostMallocDefault));
    HIPCHK(c, hipMemcpyAsync(c->h_count, c->fq_count, sizeof(uint64_t), hipMemcpyDeviceToHost, c->stream));
    if (bits) HIPCHK(c, hipMemcpyAsync(bits, c->s_bits, 2 * n, hipMemcpyDeviceToHost, c->stream));
    if (region) HIPCHK(c, hipMemcpyAsync(region, c->s_region, rb, hipMemcpyDeviceToHost, c->stream));
    if (fit) HIPCHK(c, hipMemcpyAsync(fit, c->s_fit, 8 * n, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    const uint64_t cnt = *c->h_count;
    if ((rc = finish_queue(c, cnt, c->s_bits, fit ? c->s_fit : nullptr)) || cnt == 0) return rc;
    if (bits) HIPCHK(c, hipMemcpyAsync(bits, c->s_bits, 2 * n, hipMemcpyDeviceToHost, c->stream));
    if (fit) HIPCHK(c, hipMemcpyAsync(fit, c->s_fit, 8 * n, hipMemcpyDeviceToHost, c->stream));
    return sparc_sync(c);
}

}  // extern "C"

namespace {
// one env, one round trip (sparc_env_step / _reset / _read)
int env_call(Ctx* c, int32_t env, int32_t op, uint32_t arg, int32_t audit, sparc_env_record* out) {
    int rc = check_ctx(c, op != 2);
    if (rc) return rc;
    if (!out) return fail(c, SPARC_E_INVALID, "null record");
    if (env < 0 || (uint32_t)env >= c->n) return fail(c, SPARC_E_INVALID, "env index out of range");
    if (op == 2 && !c->has_state && c->n != 1)
        return fail(c, SPARC_E_STATE, "first reset must cover every env (sparc_reset_*)");
    if (op == 2 && arg >= c->num_puzzles) return fail(c, SPARC_E_INVALID, "puzzle index out of range");
    if (audit && !c->rules) return fail(c, SPARC_E_STATE, "sparc_load_rules has not been called");
    if (!c->h_rec) {
        HIPCHK(c, hipHostMalloc(reinterpret_cast<void**>(&c->h_rec), sizeof(sparc_env_record), hipHostMallocMapped));
        HIPCHK(c, hipHostGetDevicePointer(reinterpret_cast<void**>(&c->d_rec), c->h_rec, 0));
    }
    const Params p = make_params(c);
    dispatch_w_tb(c->W, c->cfg.traceback, [&](auto w, auto tb) {
        k_env_op<decltype(w)::value, decltype(tb)::value><<<1, 64, 0, c->stream>>>(p, (uint32_t)env, op, arg, c->d_rec);
    });
    if ((rc = launch_check(c))) return rc;
    if (op == 2) c->has_state = true;
    if (audit) {
        if ((rc = audit_scratch(c))) return rc;
        if ((rc = sparc_rules_device(c, c->s_bits, c->s_region, c->s_fit))) return rc;
        k_env_audit<<<1, 64, 0, c->stream>>>((uint32_t)env, (uint32_t)c->W, c->s_bits, c->s_region, c->s_fit,
                                             c->fq_count, c->d_rec);
        if ((rc = launch_check(c))) return rc;
    }
    HIPCHK(c, hipStreamSynchronize(c->stream));
    *out = *c->h_rec;
    if (audit) c->fq_last = 0;
    if (audit && out->host_fits) {   // exact fits past the GPU's node cap: finished on the host
        uint64_t cnt = 0;
        if ((rc = read_queue_count(c, cnt))) return rc;
        if ((rc = finish_queue(c, cnt, c->s_bits, c->s_fit))) return rc;
        HIPCHK(c, hipMemcpyAsync(&out->rule_bits, c->s_bits + env, 2, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipMemcpyAsync(&out->fit, c->s_fit + env, 8, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
    }
    return SPARC_OK;
}
}  // namespace

extern "C" {

int sparc_env_step(void* ctx, int32_t env, int32_t action, int32_t audit, sparc_env_record* out) {
    DevGuard dg;
    // outside 0..3 nothing is legal (`action in legal_actions` fails, SPaRC_Gym.py:1137)
    const uint32_t a = (action >= 0 && action < 4) ? (uint32_t)action : 255u;
    return env_call(static_cast<Ctx*>(ctx), env, 1, a, audit, out);
}

int sparc_env_reset(void* ctx, int32_t env, uint32_t puzzle_index, int32_t audit, sparc_env_record* out) {
    DevGuard dg;
    return env_call(static_cast<Ctx*>(ctx), env, 2, puzzle_index, audit, out);
}

int sparc_env_read(void* ctx, int32_t env, int32_t audit, sparc_env_record* out) {
    DevGuard dg;
    return env_call(static_cast<Ctx*>(ctx), env, 0, 0u, audit, out);
}

int sparc_read_state(void* ctx, const sparc_state_host* o) {
    DevGuard dg;
    Ctx* c = static_cast<Ctx*>(ctx);
    int rc = check_ctx(c, true);
    if (rc) return rc;
    if (!o) return fail(c, SPARC_E_INVALID, "null argument");
    const size_t n = c->n;
    std::vector<uint32_t> pos(n), aux(n);
    HIPCHK(c, hipMemcpyAsync(pos.data(), c->pos, 4 * n, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(aux.data(), c->aux, 4 * n, hipMemcpyDeviceToHost, c->stream));
    if (o->step) HIPCHK(c, hipMemcpyAsync(o->step, c->step, 4 * n, hipMemcpyDeviceToHost, c->stream));
    if (o->puzzle) HIPCHK(c, hipMemcpyAsync(o->puzzle, c->pid, 4 * n, hipMemcpyDeviceToHost, c->stream));
    if (o->visited)
        HIPCHK(c, hipMemcpyAsync(o->visited, c->vis, 8 * n * c->W, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    for (size_t i = 0; i < n; ++i) {
        if (o->x) o->x[i] = (uint8_t)(pos[i] & 0xFF);
        if (o->y) o->y[i] = (uint8_t)((pos[i] >> 8) & 0xFF);
        if (o->path_len) o->path_len[i] = (uint16_t)((pos[i] >> 16) & 0xFF);
        const uint32_t oc = (aux[i] >> 16) & 3u;
        if (o->outcome) o->outcome[i] = (int8_t)(oc == 1 ? 1 : (oc == 2 ? -1 : 0));
        if (o->pending) o->pending[i] = (uint8_t)((aux[i] >> 18) & 1u);
    }
    return SPARC_OK;
}

int sparc_set_visited_host(void* ctx, const uint64_t* visited) {
    DevGuard dg;
    Ctx* c = static_cast<Ctx*>(ctx);
    int rc = check_ctx(c, true);
    if (rc) return rc;
    if (!visited) return fail(c, SPARC_E_INVALID, "null visited");
    // every env's board must hold its start point (visited[start] = 1 at every load,
    // SPaRC_Gym.py:185; no pop can clear it) and nothing outside its puzzle's lattice
    const size_t n = c->n;
    std::vector<uint32_t> pid(n);
    HIPCHK(c, hipMemcpyAsync(pid.data(), c->pid, 4 * n, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    const uint32_t pitch = (uint32_t)c->cfg.pitch;
    const size_t W = (size_t)c->W;
    std::vector<uint64_t> lat(c->num_puzzles * W, 0ull);   // each puzzle's lattice points
    for (size_t q = 0; q < c->num_puzzles; ++q) {
        const uint32_t w0 = c->h_info[4 * q], X = w0 & 0xFFu, Y = (w0 >> 8) & 0xFFu;
        for (uint32_t x = 0; x < X; ++x)
            for (uint32_t y = 0; y < Y; ++y) {
                const uint32_t b = x * pitch + y;
                lat[q * W + (b >> 6)] |= 1ull << (b & 63u);
            }
    }
    for (size_t i = 0; i < n; ++i) {
        const uint32_t q = pid[i];
        if (q >= c->num_puzzles) return fail(c, SPARC_E_STATE, "env puzzle index out of range");
        const uint32_t w0 = c->h_info[4 * (size_t)q];
        const uint32_t X = w0 & 0xFFu, Y = (w0 >> 8) & 0xFFu, sb = ((w0 >> 16) & 0xFFu) * pitch + (w0 >> 24);
        for (size_t k = 0; k < W; ++k) {
            const uint64_t v = visited[k * n + i];
            char m[128];
            if (v & ~lat[q * W + k]) {
                snprintf(m, sizeof m, "env %zu: visited bits outside its puzzle's %ux%u lattice", i, X, Y);
                return fail(c, SPARC_E_INVALID, m);
            }
            if ((sb >> 6) == k && !((v >> (sb & 63u)) & 1ull)) {
                snprintf(m, sizeof m, "env %zu: the start point is not set in visited", i);
                return fail(c, SPARC_E_INVALID, m);
            }
        }
    }
    HIPCHK(c, hipMemcpyAsync(c->vis, visited, sizeof(uint64_t) * c->W * c->n, hipMemcpyHostToDevice, c->stream));
    return sparc_sync(c);
}

int sparc_state_ptr(void* ctx, int32_t which, void** d_ptr) {
    DevGuard dg;
    Ctx* c = static_cast<Ctx*>(ctx);
    if (!c || !d_ptr) return fail(c, SPARC_E_INVALID, "null argument");
    switch (which) {
        case 0: *d_ptr = c->vis; break;
        case 1: *d_ptr = c->pos; break;
        case 2: *d_ptr = c->aux; break;
        case 3: *d_ptr = c->step; break;
        case 4: *d_ptr = c->pid; break;
        case 5: *d_ptr = c->dirs; break;
        default: return fail(c, SPARC_E_INVALID, "unknown state field");
    }
    return SPARC_OK;
}

int sparc_copy_state_device(void* ctx, int32_t which, void* d_out) {
    DevGuard dg;
    Ctx* c = static_cast<Ctx*>(ctx);
    int rc = check_ctx(c, true);
    if (rc) return rc;
    if (!d_out) return fail(c, SPARC_E_INVALID, "null argument");
    void* src = nullptr;
    rc = sparc_state_ptr(c, which, &src);
    if (rc) return rc;
    if (!src) return fail(c, SPARC_E_INVALID, "state field not allocated (traceback off)");
    const size_t n = c->n;
    const size_t bytes = which == 0 ? 8 * n * c->W : which == 5 ? 16 * n * c->W : 4 * n;
    HIPCHK(c, hipMemcpyAsync(d_out, src, bytes, hipMemcpyDeviceToDevice, c->stream));
    return SPARC_OK;
}

}  // extern "C"

// ---------------------------------------------------------------------------------------------
// End-of-batch collective over RCCL (xGMI between the GPUs of a node): one communicator per
// process / GPU, one ncclAllGather of the per-env stats per rollout batch on the context's
// stream (SURVEY §8b sparc_rccl_gather; the reference is single-process, llm_host.py:257-264).
// librccl is opened on first use, so the library loads (and the step path runs) without it.
namespace {
// The few RCCL declarations the gather uses, as rccl.h (RCCL 2.x ABI) declares them: librccl is
// dlopen'ed, so neither the library nor its headers are needed to build or load this library.
typedef struct ncclComm* ncclComm_t;
typedef struct {
    char internal[128];
} ncclUniqueId;
typedef int ncclResult_t;                           // ncclSuccess = 0, errors > 0
constexpr ncclResult_t ncclSuccess = 0;
typedef int ncclDataType_t;
constexpr ncclDataType_t ncclInt32 = 2;             // rccl.h: ncclInt32 = 2
static_assert(sizeof(ncclUniqueId) == SPARC_COMM_ID_BYTES, "SPARC_COMM_ID_BYTES is NCCL_UNIQUE_ID_BYTES");

struct Rccl {
    bool tried = false, ok = false;
    std::string why;
    ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
    ncclResult_t (*comm_init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
    ncclResult_t (*all_gather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
    const char* (*error_string)(ncclResult_t) = nullptr;
};

Rccl& rccl() {
    static Rccl r;
    static std::mutex mu;
    std::lock_guard<std::mutex> lock(mu);
    if (r.tried) return r;
    r.tried = true;
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_GLOBAL);
    if (!h) {
        const char* e = dlerror();
        r.why = std::string("cannot open librccl: ") + (e ? e : "?");
        return r;
    }
    r.get_unique_id = reinterpret_cast<decltype(r.get_unique_id)>(dlsym(h, "ncclGetUniqueId"));
    r.comm_init_rank = reinterpret_cast<decltype(r.comm_init_rank)>(dlsym(h, "ncclCommInitRank"));
    r.comm_destroy = reinterpret_cast<decltype(r.comm_destroy)>(dlsym(h, "ncclCommDestroy"));
    r.all_gather = reinterpret_cast<decltype(r.all_gather)>(dlsym(h, "ncclAllGather"));
    r.error_string = reinterpret_cast<decltype(r.error_string)>(dlsym(h, "ncclGetErrorString"));
    r.ok = r.get_unique_id && r.comm_init_rank && r.comm_destroy && r.all_gather && r.error_string;
    if (!r.ok) r.why = "librccl lacks an entry point (ncclGetUniqueId / CommInitRank / CommDestroy / AllGather)";
    return r;
}

struct Comm {
    ncclComm_t nc = nullptr;
    int nranks = 0, rank = 0, device = -1;
};

#define RCCLCHK(c, expr)                                                                         \
    do {                                                                                         \
        ncclResult_t _r = (expr);                                                                \
        if (_r != ncclSuccess)                                                                   \
            return fail((c), SPARC_E_COMM, std::string(#expr ": ") + rccl().error_string(_r)); \
    } while (0)
}  // namespace

extern "C" {

int sparc_comm_unique_id(uint8_t* id_out) {
    if (!id_out) return fail(nullptr, SPARC_E_INVALID, "null id_out");
    Rccl& r = rccl();
    if (!r.ok) return fail(nullptr, SPARC_E_COMM, r.why);
    ncclUniqueId id;
    RCCLCHK(nullptr, r.get_unique_id(&id));
    memcpy(id_out, id.internal, SPARC_COMM_ID_BYTES);
    return SPARC_OK;
}

int sparc_comm_init(void* ctx, int32_t nranks, int32_t rank, const uint8_t* id, void** comm_out) {
    DevGuard dg;
    Ctx* c = static_cast<Ctx*>(ctx);
    if (!c || !id || !comm_out) return fail(c, SPARC_E_INVALID, "null argument");
    *comm_out = nullptr;
    if (nranks < 1 || rank < 0 || rank >= nranks) return fail(c, SPARC_E_INVALID, "need 0 <= rank < nranks");
    Rccl& r = rccl();
    if (!r.ok) return fail(c, SPARC_E_COMM, r.why);
    HIPCHK(c, hipSetDevice(c->device));
    ncclUniqueId uid;
    memcpy(uid.internal, id, SPARC_COMM_ID_BYTES);
    Comm* m = new Comm();
    m->nranks = nranks;
    m->rank = rank;
    m->device = c->device;
    const ncclResult_t rc = r.comm_init_rank(&m->nc, nranks, uid, rank);
    if (rc != ncclSuccess) {
        delete m;
        return fail(c, SPARC_E_COMM, std::string("ncclCommInitRank: ") + r.error_string(rc));
    }
    *comm_out = m;
    return SPARC_OK;
}

int sparc_comm_destroy(void* comm) {
    DevGuard dg;
    Comm* m = static_cast<Comm*>(comm);
    if (!m) return SPARC_OK;
    if (m->device >= 0) (void)hipSetDevice(m->device);
    if (m->nc) (void)rccl().comm_destroy(m->nc);
    delete m;
    return SPARC_OK;
}

int sparc_gather_stats(void* ctx, void* comm, const int32_t* d_stats, int32_t* d_out) {
    DevGuard dg;
    Ctx* c = static_cast<Ctx*>(ctx);
    Comm* m = static_cast<Comm*>(comm);
    if (!c || !m || !d_stats || !d_out) return fail(c, SPARC_E_INVALID, "null argument");
    if (m->device != c->device) return fail(c, SPARC_E_INVALID, "communicator and context are on different GPUs");
    HIPCHK(c, hipSetDevice(c->device));
    RCCLCHK(c, rccl().all_gather(d_stats, d_out, (size_t)4 * c->n, ncclInt32, m->nc, c->stream));
    return SPARC_OK;
}

}  // extern "C"
