// Issue-cost microbenchmarks for the instruction mix of the W = 1 step (one wave per SIMD):
// cycles per instruction for chains of 64 independent / dependent instructions, timed with
// s_memtime around an unrolled loop.  Output: one line per pattern.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define REP8(x) x x x x x x x x
#define REP64(x) REP8(REP8(x))

template <int K>
__global__ void __launch_bounds__(256) kern(uint64_t* out, uint32_t seed) {
    uint32_t a = threadIdx.x ^ seed, b = a * 3u + 1u, c = a * 7u + 5u, d = a ^ 0x55u;
    uint64_t x = ((uint64_t)a << 32) | b, y = ((uint64_t)c << 32) | d;
    __shared__ uint8_t lds[4096];
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < 64; ++it) {
        if constexpr (K == 0) {       // independent VALU u32 (4 chains)
            REP64(asm volatile("v_add_u32 %0, %0, %4\n v_add_u32 %1, %1, %4\n v_add_u32 %2, %2, %4\n v_add_u32 %3, %3, %4" : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(seed));)
        } else if constexpr (K == 1) {  // dependent VALU u32 chain
            REP64(asm volatile("v_add_u32 %0, %0, %1\n v_add_u32 %0, %0, %1\n v_add_u32 %0, %0, %1\n v_add_u32 %0, %0, %1" : "+v"(a) : "v"(seed));)
        } else if constexpr (K == 2) {  // independent 64-bit shifts
            REP64(asm volatile("v_lshrrev_b64 %0, %2, %0\n v_lshrrev_b64 %1, %2, %1\n v_lshlrev_b64 %0, %2, %0\n v_lshlrev_b64 %1, %2, %1" : "+v"(x), "+v"(y) : "v"(seed & 7u));)
        } else if constexpr (K == 3) {  // v_cmp -> sgpr mask -> v_cndmask (dependent pairs)
            uint64_t m0, m1;
            REP64(asm volatile("v_cmp_eq_u32 %1, %3, %4\n v_cndmask_b32 %0, %0, %4, %1\n v_cmp_eq_u32 %2, %3, %0\n v_cndmask_b32 %0, %0, %3, %2" : "+v"(a), "=s"(m0), "=s"(m1) : "v"(b), "v"(c));)
        } else if constexpr (K == 4) {  // v_cmp -> s_and -> v_cndmask chain
            uint64_t m0, m1;
            REP64(asm volatile("v_cmp_eq_u32 %2, %1, %4\n s_and_b64 %3, %2, exec\n v_cndmask_b32 %0, %0, %4, %3\n v_add_u32 %1, %1, %0" : "+v"(a), "+v"(b), "=s"(m0), "=s"(m1) : "v"(c) : "scc");)
        } else if constexpr (K == 5) {  // independent SALU
            uint32_t s0 = seed, s1 = seed + 1, s2 = seed + 2, s3 = seed + 3;
            REP64(asm volatile("s_add_u32 %0, %0, 1\n s_add_u32 %1, %1, 1\n s_add_u32 %2, %2, 1\n s_add_u32 %3, %3, 1" : "+s"(s0), "+s"(s1), "+s"(s2), "+s"(s3) :: "scc");)
            d += s0 + s1 + s2 + s3;
        } else if constexpr (K == 6) {  // ds_write_b8, 4 lanes per dword (the ring layout)
            REP64(asm volatile("ds_write_b8 %0, %1\n ds_write_b8 %0, %1 offset:64\n ds_write_b8 %0, %1 offset:128\n ds_write_b8 %0, %1 offset:192" :: "v"((uint32_t)threadIdx.x & 63u), "v"(a));)
            asm volatile("s_waitcnt lgkmcnt(0)");
        } else if constexpr (K == 7) {  // v_bfe / v_bitop3 / v_lshl_or mix (independent)
            REP64(asm volatile("v_bfe_u32 %0, %0, %4, 3\n v_bfe_u32 %1, %1, %4, 3\n v_lshl_or_b32 %2, %2, 1, %4\n v_lshl_or_b32 %3, %3, 1, %4" : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(seed & 15u));)
        } else if constexpr (K == 8) {  // v_lshl_add_u64 (address arithmetic)
            REP64(asm volatile("v_lshl_add_u64 %0, %0, 1, %2\n v_lshl_add_u64 %1, %1, 1, %2\n v_lshl_add_u64 %0, %0, 1, %2\n v_lshl_add_u64 %1, %1, 1, %2" : "+v"(x), "+v"(y) : "v"(x));)
        } else if constexpr (K == 9) {  // 64-bit and/or/xor as pairs of u32 ops
            REP64(asm volatile("v_xor_b32 %0, %0, %2\n v_xor_b32 %1, %1, %3\n v_or_b32 %0, %0, %3\n v_and_b32 %1, %1, %2" : "+v"(a), "+v"(b) : "v"(c), "v"(d));)
        } else if constexpr (K == 10) { // v_add_i32 clamp / v_sub_u32 clamp
            REP64(asm volatile("v_add_i32 %0, %0, %2 clamp\n v_add_i32 %1, %1, %2 clamp\n v_sub_u32 %0, %0, %2 clamp\n v_sub_u32 %1, %1, %2 clamp" : "+v"(a), "+v"(b) : "v"(c));)
        } else if constexpr (K == 12) { // ds_write_b8, one lane per dword (no bank conflict)
            REP64(asm volatile("ds_write_b8 %0, %1\n ds_write_b8 %0, %1 offset:256\n ds_write_b8 %0, %1 offset:512\n ds_write_b8 %0, %1 offset:768" :: "v"(((uint32_t)threadIdx.x & 63u) * 4u), "v"(a));)
            asm volatile("s_waitcnt lgkmcnt(0)");
        } else if constexpr (K == 13) { // ds_write_b32, one lane per dword
            REP64(asm volatile("ds_write_b32 %0, %1\n ds_write_b32 %0, %1 offset:256\n ds_write_b32 %0, %1 offset:512\n ds_write_b32 %0, %1 offset:768" :: "v"(((uint32_t)threadIdx.x & 63u) * 4u), "v"(a));)
            asm volatile("s_waitcnt lgkmcnt(0)");
        } else if constexpr (K == 14) { // v_cmp -> s_or -> s_or -> s_or (one VALU->SALU edge per 4)
            uint64_t m0, m1;
            REP64(asm volatile("v_cmp_eq_u32 %1, %3, %4\n s_or_b64 %2, %1, exec\n s_or_b64 %2, %2, %1\n s_or_b64 %2, %2, %1" : "+v"(a), "=s"(m0), "=s"(m1) : "v"(b), "v"(c) : "scc");)
        } else if constexpr (K == 15) { // VALU-only boolean: v_cmp -> v_cndmask 0/1 -> v_and -> v_cmp
            uint64_t m0;
            REP64(asm volatile("v_cmp_eq_u32 %1, %2, %3\n v_cndmask_b32 %0, 0, 1, %1\n v_and_b32 %0, %0, %2\n v_cmp_ne_u32 %1, 0, %0" : "+v"(a), "=s"(m0) : "v"(b), "v"(c));)
        } else if constexpr (K == 16) { // v_cmp -> s_and (independent of the next v_cmp)
            uint64_t m0, m1, m2, m3;
            REP64(asm volatile("v_cmp_eq_u32 %0, %4, %5\n v_cmp_eq_u32 %1, %5, %4\n s_and_b64 %2, %0, exec\n s_and_b64 %3, %1, exec" : "=s"(m0), "=s"(m1), "=s"(m2), "=s"(m3) : "v"(b), "v"(c) : "scc");)
        } else if constexpr (K == 11) { // ds_read_u8 then use (dependent LDS latency)
            a &= 63u;
            REP8(asm volatile("ds_read_u8 %0, %0\n s_waitcnt lgkmcnt(0)\n v_and_b32 %0, 63, %0" : "+v"(a));)
        }
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) out[blockIdx.x] = t1 - t0;
    if (a == 0x12345678u && b == 1u && c == 2u && x == 3u && y == 4u) out[blockIdx.x + 8192] = a + b + c + d;
}

template <int K>
double run(uint64_t* d, int blocks, int instr_per_iter) {
    kern<K><<<blocks, 256>>>(d, 12345u);
    (void)hipDeviceSynchronize();
    std::vector<uint64_t> h(blocks);
    (void)hipMemcpy(h.data(), d, 8 * blocks, hipMemcpyDeviceToHost);
    double s = 0;
    for (auto v : h) s += (double)v;
    return s / blocks / (64.0 * instr_per_iter);   // s_memtime ticks per instruction (per wave)
}

int main() {
    uint64_t* d;
    (void)hipMalloc(&d, 8 * 16384);
    const int blocks = 256;   // 1 workgroup of 4 waves per CU: one wave per SIMD
    const char* names2[] = {"ds_write_b8 1/dword", "ds_write_b32", "v_cmp->s_or->s_or->s_or", "valu-only bool", "v_cmp,v_cmp,s_and,s_and"};
    const char* names[] = {"valu u32 indep", "valu u32 dep chain", "v_lsh*_b64 indep", "v_cmp->v_cndmask dep",
                           "v_cmp->s_and->v_cndmask", "salu indep", "ds_write_b8 x4/dword", "bfe/lshl_or indep",
                           "v_lshl_add_u64", "64-bit logic as u32 pairs", "add/sub clamp", "ds_read_u8 dep latency"};
    double r[12];
    for (int pass = 0; pass < 2; ++pass) {   // first pass warms clocks
        r[0] = run<0>(d, blocks, 256); r[1] = run<1>(d, blocks, 256); r[2] = run<2>(d, blocks, 256);
        r[3] = run<3>(d, blocks, 256); r[4] = run<4>(d, blocks, 256); r[5] = run<5>(d, blocks, 256);
        r[6] = run<6>(d, blocks, 256); r[7] = run<7>(d, blocks, 256); r[8] = run<8>(d, blocks, 256);
        r[9] = run<9>(d, blocks, 256); r[10] = run<10>(d, blocks, 256); r[11] = run<11>(d, blocks, 24);
    }
    for (int k = 0; k < 12; ++k) printf("%-28s %8.3f ticks/instr\n", names[k], r[k]);
    double r2[5];
    for (int pass = 0; pass < 2; ++pass) {
        r2[0] = run<12>(d, blocks, 256); r2[1] = run<13>(d, blocks, 256); r2[2] = run<14>(d, blocks, 256);
        r2[3] = run<15>(d, blocks, 256); r2[4] = run<16>(d, blocks, 256);
    }
    for (int k = 0; k < 5; ++k) printf("%-28s %8.3f ticks/instr\n", names2[k], r2[k]);
    // two waves per SIMD (two workgroups per CU): per-wave ticks per instruction
    double r3[4];
    for (int pass = 0; pass < 2; ++pass) {
        r3[0] = run<0>(d, 2 * blocks, 256); r3[1] = run<1>(d, 2 * blocks, 256);
        r3[2] = run<2>(d, 2 * blocks, 256); r3[3] = run<6>(d, 2 * blocks, 256);
    }
    printf("2 waves/SIMD: valu indep %.3f, valu dep %.3f, b64 shifts %.3f, ds_write_b8 %.3f ticks/instr/wave\n",
           r3[0], r3[1], r3[2], r3[3]);
    return 0;
}
