// Microbenchmark (diagnostic tool, not the product): random-gather rate from
// tables of different sizes on gfx950, to price the per-event LUT gather.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

__device__ __forceinline__ uint32_t hash32(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    return x;
}

// each lane: ITERS x 16 independent gathers; index from a hash (no index stream)
template <typename T, int ILP>
__global__ __launch_bounds__(256) void k_gather(const T *__restrict__ tab, uint32_t mask, int iters,
                                                uint32_t *__restrict__ out) {
    uint32_t acc = 0;
    uint32_t seed = blockIdx.x * 256u + threadIdx.x;
    for (int it = 0; it < iters; ++it) {
        T v[ILP];
#pragma unroll
        for (int u = 0; u < ILP; ++u) v[u] = tab[hash32(seed + (uint32_t)(it * ILP + u) * 0x9e3779b9u) & mask];
#pragma unroll
        for (int u = 0; u < ILP; ++u) acc += (uint32_t)v[u];
    }
    out[blockIdx.x * 256 + threadIdx.x] = acc;
}

// streaming read for comparison (int4)
__global__ __launch_bounds__(256) void k_stream(const int4 *__restrict__ src, long long n4,
                                                uint32_t *__restrict__ out) {
    uint32_t acc = 0;
    for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n4; i += (long long)gridDim.x * 256) {
        int4 v = src[i];
        acc += v.x ^ v.y ^ v.z ^ v.w;
    }
    out[blockIdx.x * 256 + threadIdx.x] = acc;
}

int main() {
    const int blocks = 256 * 8;
    uint32_t *out;
    hipMalloc(&out, blocks * 256 * 4);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (size_t bytes : {32u << 10, 512u << 10, 1u << 20, 2u << 20, 4u << 20, 16u << 20, 64u << 20, 512u << 20}) {
        uint16_t *t16;
        hipMalloc(&t16, bytes);
        hipMemset(t16, 1, bytes);
        const uint32_t n = (uint32_t)(bytes / 2);
        const uint32_t mask = n - 1;
        const int iters = 64;
        for (int rep = 0; rep < 2; ++rep) {
            hipEventRecord(a);
            hipLaunchKernelGGL((k_gather<uint16_t, 16>), dim3(blocks), dim3(256), 0, 0, t16, mask, iters, out);
            hipEventRecord(b);
            hipEventSynchronize(b);
        }
        float ms;
        hipEventElapsedTime(&ms, a, b);
        const double g = (double)blocks * 256 * iters * 16;
        printf("{\"table_bytes\": %zu, \"elem\": 2, \"gathers_per_s\": %.4g, \"per_clk_per_cu_at_2.1GHz\": %.3f}\n",
               bytes, g / (ms * 1e-3), g / (ms * 1e-3) / 256 / 2.1e9);
        hipFree(t16);
    }
    {
        const long long n = 1LL << 28;  // 1 GiB of int
        int *src;
        hipMalloc(&src, n * 4);
        hipMemset(src, 0, n * 4);
        float ms = 0;
        for (int rep = 0; rep < 3; ++rep) {
            hipEventRecord(a);
            hipLaunchKernelGGL(k_stream, dim3(blocks), dim3(256), 0, 0, (const int4 *)src, n / 4, out);
            hipEventRecord(b);
            hipEventSynchronize(b);
            hipEventElapsedTime(&ms, a, b);
        }
        printf("{\"stream_read_GBs\": %.1f}\n", n * 4.0 / (ms * 1e-3) / 1e9);
        hipFree(src);
    }
    return 0;
}
