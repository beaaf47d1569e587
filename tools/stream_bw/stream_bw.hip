// Achievable HBM bandwidth on this box ("measure achievable bandwidth
// with a stream-copy kernel"), the ceiling the c4 plane writer is compared with:
//   store  : 16-B nontemporal stores per lane, grid-stride over a 4 GiB buffer
//   copy   : 16-B nontemporal load + store (bytes = read + written)
//   store4 : 4 x 16-B default-policy stores per lane per iteration
//   read   : 16-B loads, xor-reduced, one word per workgroup written
// The same access width and policy as the rollout kernels' streamed tiles and planes.
// Timed with HIP events over R launches after 2 warm-ups; prints one line per pattern in GB/s
// (1e9 B/s).  Build and run on the GPU box:
//   hipcc -O3 --offload-arch=gfx950 -o /tmp/stream_bw tools/stream_bw/stream_bw.hip && /tmp/stream_bw
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

#define CHECK(x)                                                                         \
    do {                                                                                 \
        hipError_t e_ = (x);                                                             \
        if (e_ != hipSuccess) {                                                          \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                     \
        }                                                                                \
    } while (0)

__global__ void __launch_bounds__(256) k_store(u32x4* __restrict__ dst, size_t n, unsigned seed) {
    const u32x4 v = {seed, seed ^ 1u, seed ^ 2u, seed ^ 3u};
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        __builtin_nontemporal_store(v, dst + i);
}

// default cache policy, 4 x 16 B per lane per iteration (64 B per lane, a wave covers 4 KB)
__global__ void __launch_bounds__(256) k_store4(u32x4* __restrict__ dst, size_t n, unsigned seed) {
    const u32x4 v = {seed, seed ^ 1u, seed ^ 2u, seed ^ 3u};
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i + 3 * stride < n; i += 4 * stride) {
        dst[i] = v;
        dst[i + stride] = v;
        dst[i + 2 * stride] = v;
        dst[i + 3 * stride] = v;
    }
}

__global__ void __launch_bounds__(256) k_copy(u32x4* __restrict__ dst, const u32x4* __restrict__ src, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        __builtin_nontemporal_store(__builtin_nontemporal_load(src + i), dst + i);
}

__global__ void __launch_bounds__(256) k_read(unsigned* __restrict__ out, const u32x4* __restrict__ src, size_t n) {
    unsigned acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const u32x4 v = __builtin_nontemporal_load(src + i);
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    __shared__ unsigned red[256];
    red[threadIdx.x] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int k = 1; k < 256; ++k) acc ^= red[k];
        out[blockIdx.x] = acc;
    }
}

int main() {
    const size_t bytes = 4ull << 30, n = bytes / 16;
    const int R = 10;
    u32x4 *a, *b;
    unsigned* out;
    CHECK(hipMalloc(&a, bytes));
    CHECK(hipMalloc(&b, bytes));
    CHECK(hipMalloc(&out, 1 << 20));
    CHECK(hipMemset(a, 1, bytes));
    CHECK(hipMemset(b, 2, bytes));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    int cus = 0;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    for (int pat = 0; pat < 4; ++pat) {
        for (int gmul : {8, 32}) {
            const int grid = cus * gmul;
            auto launch = [&](int r) {
                if (pat == 0) k_store<<<grid, 256>>>(a, n, (unsigned)r);
                else if (pat == 1) k_copy<<<grid, 256>>>(b, a, n);
                else if (pat == 2) k_read<<<grid, 256>>>(out, a, n);
                else k_store4<<<grid, 256>>>(a, n, (unsigned)r);
            };
            launch(0);
            launch(1);
            CHECK(hipDeviceSynchronize());
            CHECK(hipEventRecord(e0));
            for (int r = 0; r < R; ++r) launch(r);
            CHECK(hipEventRecord(e1));
            CHECK(hipEventSynchronize(e1));
            CHECK(hipGetLastError());
            float ms = 0;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            const double moved = (pat == 1 ? 2.0 : 1.0) * bytes * R;
            printf("%-6s grid %5d x 256: %7.1f GB/s (%.3f ms per launch, %.2f GiB moved per launch)\n",
                   pat == 0 ? "store" : pat == 1 ? "copy" : pat == 2 ? "read" : "store4", grid, moved / (ms * 1e-3) / 1e9, ms / R,
                   moved / R / (1 << 30));
        }
    }
    CHECK(hipFree(a));
    CHECK(hipFree(b));
    CHECK(hipFree(out));
    return 0;
}
