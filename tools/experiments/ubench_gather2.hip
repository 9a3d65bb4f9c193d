// Microbenchmark (diagnostic tool, not the product): cost of a random-gather
// wave instruction vs the number of active lanes, on gfx950.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__device__ __forceinline__ uint32_t hash32(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    return x;
}

// ACTIVE of every 64 lanes gather; the others skip (predicated off)
template <int ILP>
__global__ __launch_bounds__(256) void k_gather(const uint32_t *__restrict__ tab, uint32_t mask,
                                                int iters, int active, uint32_t *__restrict__ out) {
    uint32_t acc = 0;
    const uint32_t seed = blockIdx.x * 256u + threadIdx.x;
    const bool on = (int)(threadIdx.x & 63) < active;
    for (int it = 0; it < iters; ++it) {
        uint32_t v[ILP];
#pragma unroll
        for (int u = 0; u < ILP; ++u) {
            const uint32_t i = hash32(seed + (uint32_t)(it * ILP + u) * 0x9e3779b9u) & mask;
            v[u] = on ? tab[i] : i;
        }
#pragma unroll
        for (int u = 0; u < ILP; ++u) acc += v[u];
    }
    out[blockIdx.x * 256 + threadIdx.x] = acc;
}

int main() {
    const int blocks = 256 * 8;
    uint32_t *out, *tab;
    (void)hipMalloc(&out, blocks * 256 * 4);
    const size_t n = (2u << 20) / 4;  // 2 MB table
    (void)hipMalloc(&tab, n * 4);
    (void)hipMemset(tab, 1, n * 4);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    for (int active : {64, 32, 16, 8, 4, 1, 0}) {
        float ms = 0;
        for (int rep = 0; rep < 2; ++rep) {
            (void)hipEventRecord(a);
            hipLaunchKernelGGL((k_gather<16>), dim3(blocks), dim3(256), 0, 0, tab, (uint32_t)(n - 1), 64, active, out);
            (void)hipEventRecord(b);
            (void)hipEventSynchronize(b);
            (void)hipEventElapsedTime(&ms, a, b);
        }
        const double instr = (double)blocks * 4 * 64 * 16;  // wave instructions
        printf("{\"active_lanes\": %d, \"ms\": %.4f, \"wave_gathers_per_s\": %.4g, \"lane_gathers_per_s\": %.4g}\n",
               active, ms, instr / (ms * 1e-3), instr * active / (ms * 1e-3));
    }
    return 0;
}
