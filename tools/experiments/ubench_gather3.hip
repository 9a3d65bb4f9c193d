// Microbenchmark (diagnostic tool, not the product): random-gather rate from an
// L2-resident table for each load flavour (plain / nt / sc0 / sc1 / sc0 sc1),
// to find whether the L1 fill of a whole line per lane is what bounds the
// per-event LUT gather on gfx950.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>

__device__ __forceinline__ uint32_t hash32(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    return x;
}

typedef __attribute__((address_space(1))) const uint16_t g_u16;
typedef __attribute__((address_space(1))) const uint32_t g_u32;

template <int AUX>
__device__ __forceinline__ uint32_t ld16(__amdgpu_buffer_rsrc_t r, uint32_t idx) {
    return __builtin_amdgcn_raw_buffer_load_b16(r, idx * 2u, 0, AUX);
}

template <int MODE, int ILP>
__global__ __launch_bounds__(256) void k_gather(const uint16_t *__restrict__ tab, uint32_t mask,
                                                int iters, uint32_t *__restrict__ out) {
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void *)tab, 0, (int)((mask + 1) * 2), 0x00020000);
    uint32_t acc = 0;
    const uint32_t seed = blockIdx.x * 256u + threadIdx.x;
    for (int it = 0; it < iters; ++it) {
        uint32_t v[ILP];
#pragma unroll
        for (int u = 0; u < ILP; ++u)
            v[u] = ld16<MODE>(r, hash32(seed + (uint32_t)(it * ILP + u) * 0x9e3779b9u) & mask);
#pragma unroll
        for (int u = 0; u < ILP; ++u) acc += v[u];
    }
    out[blockIdx.x * 256 + threadIdx.x] = acc;
}

// LDS random gather for comparison (64 KB table of u16)
template <int ILP>
__global__ __launch_bounds__(256) void k_lds(const uint16_t *__restrict__ tab, int iters, uint32_t *__restrict__ out) {
    __shared__ uint16_t s[32768];
    for (int i = threadIdx.x; i < 32768; i += 256) s[i] = tab[i];
    __syncthreads();
    uint32_t acc = 0;
    const uint32_t seed = blockIdx.x * 256u + threadIdx.x;
    for (int it = 0; it < iters; ++it) {
        uint32_t v[ILP];
#pragma unroll
        for (int u = 0; u < ILP; ++u) v[u] = s[hash32(seed + (uint32_t)(it * ILP + u) * 0x9e3779b9u) & 32767u];
#pragma unroll
        for (int u = 0; u < ILP; ++u) acc += v[u];
    }
    out[blockIdx.x * 256 + threadIdx.x] = acc;
}

template <int MODE>
static void run(const char *name, const uint16_t *tab, size_t bytes, uint32_t *out, hipEvent_t a, hipEvent_t b) {
    const int blocks = 256 * 8, iters = 64;
    float ms = 0;
    for (int rep = 0; rep < 3; ++rep) {
        (void)hipEventRecord(a);
        hipLaunchKernelGGL((k_gather<MODE, 16>), dim3(blocks), dim3(256), 0, 0, tab, (uint32_t)(bytes / 2 - 1), iters, out);
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        (void)hipEventElapsedTime(&ms, a, b);
    }
    const double g = (double)blocks * 256 * iters * 16;
    if (hipGetLastError() != hipSuccess) { printf("launch error\n"); exit(1); }
    printf("{\"mode\": \"%s\", \"table_bytes\": %zu, \"gathers_per_s\": %.4g}\n", name, bytes, g / (ms * 1e-3));
}

int main() {
    uint32_t *out;
    (void)hipMalloc(&out, 256 * 8 * 256 * 4);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    uint16_t *tab;
    (void)hipMalloc(&tab, 4u << 20);
    (void)hipMemset(tab, 1, 4u << 20);
    for (size_t bytes : {(size_t)16 << 10, (size_t)1 << 20, (size_t)4 << 20}) {
        run<0>("aux0", tab, bytes, out, a, b);
        run<1>("aux1", tab, bytes, out, a, b);
        run<2>("aux2", tab, bytes, out, a, b);
        run<3>("aux3", tab, bytes, out, a, b);
        run<16>("aux16", tab, bytes, out, a, b);
        run<17>("aux17", tab, bytes, out, a, b);
    }
    float ms = 0;
    for (int rep = 0; rep < 3; ++rep) {
        (void)hipEventRecord(a);
        hipLaunchKernelGGL((k_lds<16>), dim3(256 * 8), dim3(256), 0, 0, tab, 64, out);
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        (void)hipEventElapsedTime(&ms, a, b);
    }
    printf("{\"mode\": \"lds\", \"table_bytes\": 65536, \"gathers_per_s\": %.4g}\n", 256.0 * 8 * 256 * 64 * 16 / (ms * 1e-3));
    return 0;
}
