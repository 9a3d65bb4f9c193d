// ubench_sgather.hip -- can table-miss gathers leave the vector memory path?
//
// The sieve's table misses (~11 % of DREAM events) gather a 4-byte LUT word
// each; measured, they cost ~0.06 ms whatever their issue distance, at the
// chip's random-gather rate, serialized with the event stream in the vector
// memory pipeline (DESIGN.md "Where k_sieve's time goes").  This probe streams
// 1.12 GB of {pid, toa} like the sieve (256 blocks x 1024 threads, 8 events
// per thread per chunk, next chunk loaded while this one is worked) and:
//   mode 0  stream only
//   mode 1  + a vector gather per event (misses ~11 %, hits load out of range)
//   mode 2  + the misses gathered by scalar loads (readlane -> s_load ->
//           select), so they travel the scalar cache's path to L2 instead
//   mode 3  + the misses compacted per wave through LDS and gathered by
//           ceil(misses / 64) full instructions (is the cost per lane or per
//           instruction?)
//   mode 4  mode 1 with the non-temporal cache policy on the gathers
//   mode 5  mode 1 into a 16 KB table (L1-resident)
//   mode 6  mode 0 with the sieve's pipeline: two chunks in flight, the
//           chunk pointers read from an LDS table and taken with readlane
// argv[2]: dynamic LDS bytes per block (160 KB: one block per CU, as the sieve)
// Build: hipcc --offload-arch=gfx950 -O3 tools/ubench_sgather.hip -o /tmp/ubench_sgather
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef int v4i __attribute__((ext_vector_type(4)));
typedef const __attribute__((address_space(4))) uint32_t cu32;

constexpr int kThreads = 1024, kEPT = 8, kChunk = kThreads * kEPT;

__device__ __forceinline__ uint32_t mix(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    return x;
}

__global__ void k_fill(int *pid, int *toa, long long n) {
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
        pid[i] = (int)mix((uint32_t)i);
        toa[i] = (int)mix((uint32_t)i ^ 0x9e3779b9u);
    }
}

__global__ void k_fill_lut(uint32_t *lut, uint32_t L) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < L; i += gridDim.x * blockDim.x) lut[i] = mix(i * 7u + 1u);
}

template <int MODE>
__global__ __launch_bounds__(kThreads) void k_probe(const int *__restrict__ pid, const int *__restrict__ toa,
                                                    long long n_chunks, const uint32_t *__restrict__ lut,
                                                    uint32_t L, uint32_t miss_per_mille, uint32_t *out,
                                                    unsigned long long *trace) {
    const int tid = threadIdx.x, lane = tid & 63;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    const long long cb = (long long)blockIdx.x * n_chunks / gridDim.x;
    const long long ce = ((long long)blockIdx.x + 1) * n_chunks / gridDim.x;
    const __amdgpu_buffer_rsrc_t rl = __builtin_amdgcn_make_buffer_rsrc((void *)lut, (short)0, (int)(L * 4u), 0x00020000);
    cu32 *cl = (cu32 *)lut;
    __shared__ uint32_t s_q[kThreads / 64][kEPT * 64];
    __shared__ unsigned long long s_ptr[2 * 512];
    extern __shared__ uint32_t s_dyn[];
    if (MODE == 6) {
        for (long long c = cb + tid; c <= ce + 2; c += kThreads) {
            s_ptr[2 * (c - cb)] = (unsigned long long)(pid + (c < ce ? c : cb) * kChunk);
            s_ptr[2 * (c - cb) + 1] = (unsigned long long)(toa + (c < ce ? c : cb) * kChunk);
        }
        __syncthreads();
    }
    uint32_t *sq = s_q[tid >> 6];
    const uint32_t Lg = MODE == 5 ? 4096u : L;
    uint32_t acc = 0;
    v4i p[2], t[2], pn[2], tn[2];
    auto load = [&](long long c, v4i (&pp)[2], v4i (&tt)[2]) {
        const long long base = c * kChunk;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const long long off = base + (long long)(j * kThreads + tid) * 4;
            pp[j] = __builtin_nontemporal_load((const v4i *)(pid + off));
            tt[j] = __builtin_nontemporal_load((const v4i *)(toa + off));
        }
    };
    if (MODE == 6) {
        // two chunks in flight; pointers from LDS via readlane (the sieve's fetch/ptrs)
        auto fetch = [&](long long c) -> uint32_t {
            const uint32_t *w = reinterpret_cast<const uint32_t *>(s_ptr);
            return w[(uint32_t)(c - cb) * 4u + (uint32_t)(lane & 3)];
        };
        auto ld2 = [&](uint32_t dv, v4i (&pp)[2], v4i (&tt)[2]) {
            const uint32_t w0 = __builtin_amdgcn_readlane((int)dv, 0), w1 = __builtin_amdgcn_readlane((int)dv, 1);
            const uint32_t w2 = __builtin_amdgcn_readlane((int)dv, 2), w3 = __builtin_amdgcn_readlane((int)dv, 3);
            const int *pp0 = reinterpret_cast<const int *>(((unsigned long long)w1 << 32) | w0);
            const int *tq0 = reinterpret_cast<const int *>(((unsigned long long)w3 << 32) | w2);
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int off = (j * kThreads + tid) * 4;
                pp[j] = __builtin_nontemporal_load((const v4i *)(pp0 + off));
                tt[j] = __builtin_nontemporal_load((const v4i *)(tq0 + off));
            }
        };
        v4i pB[2], tB[2];
        uint32_t dA = fetch(cb), dB = fetch(cb + 1);
        if (cb < ce) {
            ld2(dA, p, t);
            ld2(dB, pB, tB);
            dA = fetch(cb + 2);
            dB = fetch(cb + 3);
        }
        for (long long c = cb; c < ce; c += 2) {
#pragma unroll
            for (int e = 0; e < kEPT; ++e) acc += (uint32_t)t[e >> 2][e & 3] ^ (uint32_t)p[e >> 2][e & 3];
            ld2(dA, p, t);
            dA = fetch(c + 4 < ce + 2 ? c + 4 : ce + 2);
            if (c + 1 >= ce) break;
#pragma unroll
            for (int e = 0; e < kEPT; ++e) acc += (uint32_t)tB[e >> 2][e & 3] ^ (uint32_t)pB[e >> 2][e & 3];
            ld2(dB, pB, tB);
            dB = fetch(c + 5 < ce + 2 ? c + 5 : ce + 2);
        }
        if (tid == 0) s_dyn[0] = acc;
    }
    if (cb < ce && MODE != 6) load(cb, p, t);
    for (long long c = cb; MODE != 6 && c < ce; ++c) {
        if (c + 1 < ce) load(c + 1, pn, tn);
        uint32_t q[kEPT], g[kEPT];
        bool miss[kEPT];
#pragma unroll
        for (int e = 0; e < kEPT; ++e) {
            const uint32_t x = (uint32_t)p[e >> 2][e & 3];
            q[e] = (x >> 8) % Lg;
            miss[e] = (x & 1023u) < miss_per_mille;
            g[e] = 0;
        }
        if (MODE == 1 || MODE == 5) {
#pragma unroll
            for (int e = 0; e < kEPT; ++e)
                g[e] = __builtin_amdgcn_raw_buffer_load_b32(rl, (int)(miss[e] ? q[e] * 4u : 0x80000000u), 0, 0);
        } else if (MODE == 4) {
#pragma unroll
            for (int e = 0; e < kEPT; ++e)
                g[e] = __builtin_amdgcn_raw_buffer_load_b32(rl, (int)(miss[e] ? q[e] * 4u : 0x80000000u), 0, 2);
        } else if (MODE == 3) {
            // compact (e, lane) misses: positions from the ballots
            uint32_t pos[kEPT], cnt = 0;
#pragma unroll
            for (int e = 0; e < kEPT; ++e) {
                const unsigned long long m = __builtin_amdgcn_ballot_w64(miss[e]);
                pos[e] = cnt + (uint32_t)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
                if (miss[e]) sq[pos[e]] = q[e];
                cnt += (uint32_t)__popcll(m);
            }
            __builtin_amdgcn_wave_barrier();
            for (uint32_t i = 0; i < cnt; i += 64) {
                const uint32_t k = i + (uint32_t)lane;
                const uint32_t qq = sq[k];
                const uint32_t v = __builtin_amdgcn_raw_buffer_load_b32(rl, (int)(k < cnt ? qq * 4u : 0x80000000u), 0, 0);
                __builtin_amdgcn_wave_barrier();
                if (k < cnt) sq[k] = v;
            }
            __builtin_amdgcn_wave_barrier();
#pragma unroll
            for (int e = 0; e < kEPT; ++e) g[e] = miss[e] ? sq[pos[e]] : 0u;
            __builtin_amdgcn_wave_barrier();
        } else if (MODE == 2) {
#pragma unroll
            for (int e = 0; e < kEPT; ++e) {
                unsigned long long m = __builtin_amdgcn_ballot_w64(miss[e]);
                while (m) {
                    uint32_t v[8];
                    int ln[8];
#pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        ln[j] = -1;
                        if (m) {
                            ln[j] = __builtin_ctzll(m);
                            m &= m - 1;
                            v[j] = cl[__builtin_amdgcn_readlane((int)q[e], ln[j])];
                        }
                    }
#pragma unroll
                    for (int j = 0; j < 8; ++j)
                        if (ln[j] >= 0) g[e] = lane == ln[j] ? v[j] : g[e];
                }
            }
        }
#pragma unroll
        for (int e = 0; e < kEPT; ++e) acc += (uint32_t)t[e >> 2][e & 3] ^ g[e] ^ (uint32_t)p[e >> 2][e & 3];
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            p[j] = pn[j];
            t[j] = tn[j];
        }
    }
    out[(size_t)blockIdx.x * kThreads + tid] = acc;
    if (tid == 0) {
        trace[2 * blockIdx.x] = t0;
        trace[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime();
    }
}

int main(int argc, char **argv) {
    const long long n = 140000000LL / kChunk * kChunk;
    const uint32_t L = 491521;
    const uint32_t miss = argc > 1 ? (uint32_t)atoi(argv[1]) : 116;  // per 1024 (~11.3 %)
    const size_t dyn = argc > 2 ? (size_t)atoi(argv[2]) : 0;
    int *pid, *toa;
    uint32_t *lut, *out;
    // argv[3]: toa placed this many MiB after pid in one allocation (0: its own)
    const long long toa_mib = argc > 3 ? atoll(argv[3]) : 0;
    if (toa_mib > 0) {
        hipMalloc(&pid, (size_t)toa_mib * 1048576 + n * 4);
        toa = pid + (size_t)toa_mib * 1048576 / 4;
    } else {
        hipMalloc(&pid, n * 4);
        hipMalloc(&toa, n * 4);
    }
    printf("pid %p toa %p (toa - pid = %lld B)\n", (void *)pid, (void *)toa, (long long)((char *)toa - (char *)pid));
    hipMalloc(&lut, L * 4);
    hipMalloc(&out, 256 * kThreads * 4);
    unsigned long long *tr;
    hipMallocManaged(&tr, 512 * 8);
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, pid, toa, n);
    hipLaunchKernelGGL(k_fill_lut, dim3(1024), dim3(256), 0, 0, lut, L);
    hipDeviceSynchronize();
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    if (dyn)
        for (const void *f : {(const void *)k_probe<0>, (const void *)k_probe<1>, (const void *)k_probe<2>,
                              (const void *)k_probe<3>, (const void *)k_probe<4>, (const void *)k_probe<5>,
                              (const void *)k_probe<6>})
            hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)dyn);
    const long long nc = n / kChunk;
    for (int rep = 0; rep < 1; ++rep)
        for (int mode = 0; mode < 7; ++mode) {
            float best = 1e9f;
            for (int it = 0; it < 5; ++it) {
                hipEventRecord(a);
                if (mode == 0) hipLaunchKernelGGL(k_probe<0>, dim3(256), dim3(kThreads), dyn, 0, pid, toa, nc, lut, L, miss, out, tr);
                if (mode == 1) hipLaunchKernelGGL(k_probe<1>, dim3(256), dim3(kThreads), dyn, 0, pid, toa, nc, lut, L, miss, out, tr);
                if (mode == 2) hipLaunchKernelGGL(k_probe<2>, dim3(256), dim3(kThreads), dyn, 0, pid, toa, nc, lut, L, miss, out, tr);
                if (mode == 3) hipLaunchKernelGGL(k_probe<3>, dim3(256), dim3(kThreads), dyn, 0, pid, toa, nc, lut, L, miss, out, tr);
                if (mode == 4) hipLaunchKernelGGL(k_probe<4>, dim3(256), dim3(kThreads), dyn, 0, pid, toa, nc, lut, L, miss, out, tr);
                if (mode == 5) hipLaunchKernelGGL(k_probe<5>, dim3(256), dim3(kThreads), dyn, 0, pid, toa, nc, lut, L, miss, out, tr);
                if (mode == 6) hipLaunchKernelGGL(k_probe<6>, dim3(256), dim3(kThreads), dyn, 0, pid, toa, nc, lut, L, miss, out, tr);
                hipEventRecord(b);
                hipEventSynchronize(b);
                float ms;
                hipEventElapsedTime(&ms, a, b);
                if (ms < best) best = ms;
            }
            unsigned long long s0 = ~0ull, s1 = 0, e0 = ~0ull, e1 = 0;
            double span = 0;
            for (int b = 0; b < 256; ++b) {
                s0 = tr[2 * b] < s0 ? tr[2 * b] : s0; s1 = tr[2 * b] > s1 ? tr[2 * b] : s1;
                e0 = tr[2 * b + 1] < e0 ? tr[2 * b + 1] : e0; e1 = tr[2 * b + 1] > e1 ? tr[2 * b + 1] : e1;
                span += (double)(tr[2 * b + 1] - tr[2 * b]) / 256 / 100.0;
            }
            printf("mode %d miss %u/1024: %.4f ms  %.2f TB/s  (last run: start spread %.2f us, end spread %.2f us, "
                   "mean block span %.2f us, first start -> last end %.2f us)\n", mode, miss, best, n * 8.0 / best / 1e9,
                   (s1 - s0) / 100.0, (e1 - e0) / 100.0, span, (e1 - s0) / 100.0);
        }
    hipError_t e = hipGetLastError();
    printf("%s\n", hipGetErrorString(e));
    return 0;
}
