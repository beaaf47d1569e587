// Calibration of the rocprofv3 memory-side counters on gfx950 against KNOWN byte counts, in the
// access patterns the rollout kernels use (c2's raw FETCH_SIZE exceeded its
// algorithmic reads, so the blanket 2 x FETCH_SIZE correction was unaudited for that launch
// shape).  Every kernel below moves a known number of bytes between HBM and the GPU, once per
// launch, on buffers no earlier kernel touched (so nothing is served from the L2 / Infinity
// Cache by accident); each pattern runs at the c2 launch shape (16 workgroups) and at a
// full-chip shape (4,096 workgroups).  The program prints one JSON line per dispatch (kernel
// name, grid, expected read / write bytes); tools/pmc_calib/analyze.py joins them with the
// counter passes:
//   rocprofv3 --kernel-trace --pmc FETCH_SIZE ...                                   (fetch)
//   rocprofv3 --kernel-trace --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum
//             TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum ...                        (rdreq)
//   rocprofv3 --kernel-trace --pmc WRITE_SIZE ...                                   (write)
//   hipcc -O3 --offload-arch=gfx950 -o /tmp/pmc_calib tools/pmc_calib/pmc_calib.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

#define CHECK(x)                                                                              \
    do {                                                                                      \
        hipError_t e_ = (x);                                                                  \
        if (e_ != hipSuccess) {                                                               \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                          \
        }                                                                                     \
    } while (0)

constexpr int kBlock = 256;

// ---- reads (each workgroup xor-reduces what it read into one dword of `sink`)
__device__ __forceinline__ void sink_write(unsigned* sink, unsigned acc) {
    __shared__ unsigned red[kBlock];
    red[threadIdx.x] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int k = 1; k < kBlock; ++k) acc ^= red[k];
        sink[blockIdx.x] = acc;
    }
}
// 16 B per lane, nontemporal: the I/O waves' action tiles
__global__ void __launch_bounds__(kBlock) r16nt(const u32x4* __restrict__ src, size_t n, unsigned* sink) {
    unsigned acc = 0;
    for (size_t i = blockIdx.x * (size_t)kBlock + threadIdx.x; i < n; i += (size_t)gridDim.x * kBlock) {
        const u32x4 v = __builtin_nontemporal_load(src + i);
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    sink_write(sink, acc);
}
// 16 B per lane, default policy: the stats records (int4) and the table rows staged in LDS
__global__ void __launch_bounds__(kBlock) r16(const u32x4* __restrict__ src, size_t n, unsigned* sink) {
    unsigned acc = 0;
    for (size_t i = blockIdx.x * (size_t)kBlock + threadIdx.x; i < n; i += (size_t)gridDim.x * kBlock) {
        const u32x4 v = src[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    sink_write(sink, acc);
}
// 8 B per lane: the visited / direction-stack words of the SoA state
__global__ void __launch_bounds__(kBlock) r8(const unsigned long long* __restrict__ src, size_t n, unsigned* sink) {
    unsigned acc = 0;
    for (size_t i = blockIdx.x * (size_t)kBlock + threadIdx.x; i < n; i += (size_t)gridDim.x * kBlock) {
        const unsigned long long v = src[i];
        acc ^= (unsigned)v ^ (unsigned)(v >> 32);
    }
    sink_write(sink, acc);
}
// 4 B per lane: pos / aux / step / pid of the SoA state
__global__ void __launch_bounds__(kBlock) r4(const unsigned* __restrict__ src, size_t n, unsigned* sink) {
    unsigned acc = 0;
    for (size_t i = blockIdx.x * (size_t)kBlock + threadIdx.x; i < n; i += (size_t)gridDim.x * kBlock) acc ^= src[i];
    sink_write(sink, acc);
}
// random 8-B gathers from a table: the trie records.  Every workgroup gathers `per` records at
// pseudo-random indices; a table far smaller than the gathers is read whole by every XCD whose
// L2 serves a workgroup (expected bytes: table bytes x XCDs used, printed by the host)
__global__ void __launch_bounds__(kBlock) rgather8(const unsigned long long* __restrict__ tab, unsigned entries,
                                                   unsigned per, unsigned* sink) {
    unsigned acc = 0, x = blockIdx.x * 0x9E3779B9u + threadIdx.x * 0x85EBCA6Bu + 1u;
    for (unsigned k = threadIdx.x; k < per; k += kBlock) {
        x ^= x << 13;
        x ^= x >> 17;
        x ^= x << 5;
        const unsigned long long v = tab[x % entries];
        acc ^= (unsigned)v;
    }
    sink_write(sink, acc);
}

// ---- writes
// 16 B per lane, nontemporal, whole lines: the I/O waves' reward / flag tiles, the plane writer
__global__ void __launch_bounds__(kBlock) w16nt(u32x4* __restrict__ dst, size_t n) {
    const u32x4 v = {1u, 2u, 3u, blockIdx.x};
    for (size_t i = blockIdx.x * (size_t)kBlock + threadIdx.x; i < n; i += (size_t)gridDim.x * kBlock)
        __builtin_nontemporal_store(v, dst + i);
}
// 16 B per lane, nontemporal, each wave writing 64-B row segments (4 lanes per row) of rows
// `pitch` bytes apart, the other half of every 128-B line written by the NEXT wave: the generic
// k_rollout's per-wave [16 steps][64 envs] tiles
__global__ void __launch_bounds__(kBlock) w16half(unsigned char* __restrict__ dst, size_t rows, size_t pitch) {
    const u32x4 v = {1u, 2u, 3u, blockIdx.x};
    const unsigned lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    const size_t col = ((size_t)blockIdx.x * (kBlock / 64) + wave) * 64;   // this wave's 64-B column
    if (col + 64 > pitch) return;
    for (size_t r = lane >> 2; r < rows; r += 16) __builtin_nontemporal_store(v, (u32x4*)(dst + r * pitch + col + (lane & 3u) * 16));
}
// 8 B per lane and 4 B per lane coalesced stores: the SoA state stores
__global__ void __launch_bounds__(kBlock) w8(unsigned long long* __restrict__ dst, size_t n) {
    for (size_t i = blockIdx.x * (size_t)kBlock + threadIdx.x; i < n; i += (size_t)gridDim.x * kBlock) dst[i] = i;
}
__global__ void __launch_bounds__(kBlock) w4(unsigned* __restrict__ dst, size_t n) {
    for (size_t i = blockIdx.x * (size_t)kBlock + threadIdx.x; i < n; i += (size_t)gridDim.x * kBlock) dst[i] = (unsigned)i;
}
// a 48-B record per lane stored as three 16-B stores (lanes 48 B apart): the exact-fit memo
__global__ void __launch_bounds__(kBlock) w48(u32x4* __restrict__ dst, size_t recs) {
    const u32x4 v = {1u, 2u, 3u, blockIdx.x};
    for (size_t i = blockIdx.x * (size_t)kBlock + threadIdx.x; i < recs; i += (size_t)gridDim.x * kBlock) {
        dst[3 * i] = v;
        dst[3 * i + 1] = v;
        dst[3 * i + 2] = v;
    }
}

int main() {
    const size_t bytes = 64ull << 20;   // per pattern: past one XCD's 4 MB L2, a fresh buffer each time
    std::vector<void*> bufs;
    auto fresh = [&](size_t b) {
        void* p = nullptr;
        CHECK(hipMalloc(&p, b));
        bufs.push_back(p);
        return p;
    };
    unsigned* sink = (unsigned*)fresh(1 << 20);
    auto report = [&](const char* kern, int grid, double rd, double wr, const char* note) {
        CHECK(hipDeviceSynchronize());
        printf("{\"kernel\": \"%s\", \"grid\": %d, \"read_bytes\": %.0f, \"write_bytes\": %.0f, \"note\": \"%s\"}\n", kern,
               grid, rd, wr, note);
        fflush(stdout);
    };
    const double sinkw = 4.0;   // one dword per workgroup (added to the write bytes)
    for (int grid : {16, 4096}) {
        // source buffers are initialised by a memset BEFORE the timed kernel (the memset's writes
        // are its own dispatch); then dropped from the caches by streaming 512 MB elsewhere
        void* a = fresh(bytes);
        void* b = fresh(bytes);
        void* c = fresh(bytes);
        void* d = fresh(bytes);
        void* flush = fresh(512ull << 20);
        CHECK(hipMemset(a, 1, bytes));
        CHECK(hipMemset(b, 2, bytes));
        CHECK(hipMemset(c, 3, bytes));
        CHECK(hipMemset(d, 4, bytes));
        CHECK(hipMemset(flush, 5, 512ull << 20));
        CHECK(hipDeviceSynchronize());
        r16nt<<<grid, kBlock>>>((const u32x4*)a, bytes / 16, sink);
        report("r16nt", grid, bytes, sinkw * grid, "16 B / lane nontemporal loads (action tiles)");
        r16<<<grid, kBlock>>>((const u32x4*)b, bytes / 16, sink);
        report("r16", grid, bytes, sinkw * grid, "16 B / lane loads (stats, table rows)");
        r8<<<grid, kBlock>>>((const unsigned long long*)c, bytes / 8, sink);
        report("r8", grid, bytes, sinkw * grid, "8 B / lane loads (visited, direction stack)");
        r4<<<grid, kBlock>>>((const unsigned*)d, bytes / 4, sink);
        report("r4", grid, bytes, sinkw * grid, "4 B / lane loads (pos, aux, step, pid)");
        // 2 MB table, 64 gathers per table line per workgroup: every line is read by every
        // workgroup, so each XCD in use fetches the whole table once into its L2
        void* tab = fresh(2ull << 20);
        CHECK(hipMemset(tab, 6, 2ull << 20));
        CHECK(hipMemset(flush, 7, 512ull << 20));
        CHECK(hipDeviceSynchronize());
        const unsigned entries = (2u << 20) / 8u, per = entries * 4u;
        const int xcds = grid < 8 ? grid : 8;
        rgather8<<<grid, kBlock>>>((const unsigned long long*)tab, entries, per, sink);
        report("rgather8", grid, (double)(2u << 20) * xcds, sinkw * grid,
               "random 8 B gathers from a 2 MB table (trie records); expected = table x XCDs in use");
        void* o1 = fresh(bytes);
        void* o2 = fresh(bytes);
        void* o3 = fresh(bytes);
        void* o4 = fresh(bytes);
        void* o5 = fresh(3 * (bytes / 4));
        w16nt<<<grid, kBlock>>>((u32x4*)o1, bytes / 16);
        report("w16nt", grid, 0, bytes, "16 B / lane nontemporal stores, whole lines (reward / flag tiles, planes)");
        // rows of `pitch` bytes, every 64-B column written by one wave: grid * 4 waves * 64 B per row
        const size_t pitch = (size_t)grid * 4 * 64, rows = bytes / pitch;
        w16half<<<grid, kBlock>>>((unsigned char*)o2, rows, pitch);
        report("w16half", grid, 0, (double)rows * pitch, "64-B row segments per wave, half lines (generic k_rollout tiles)");
        w8<<<grid, kBlock>>>((unsigned long long*)o3, bytes / 8);
        report("w8", grid, 0, bytes, "8 B / lane stores (state)");
        w4<<<grid, kBlock>>>((unsigned*)o4, bytes / 4);
        report("w4", grid, 0, bytes, "4 B / lane stores (state)");
        w48<<<grid, kBlock>>>((u32x4*)o5, bytes / 64);
        report("w48", grid, 0, 48.0 * (bytes / 64), "48-B records as 3 x 16 B per lane (exact-fit memo)");
        for (void* p : bufs)
            if (p != sink) CHECK(hipFree(p));
        bufs.assign(1, sink);
    }
    CHECK(hipFree(sink));
    return 0;
}
