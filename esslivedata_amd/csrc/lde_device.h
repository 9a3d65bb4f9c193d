// lde_device.h -- device helpers shared by the binning kernels (TOA lookup,
// LUT decode, event key, wave/block scans, chunk loads).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "lde_internal.h"

namespace lde {

typedef int v4i __attribute__((ext_vector_type(4)));

// Event arrays arrive as generic pointers inside segment descriptors; loads
// through them would compile to flat_load, which the waitcnt logic cannot
// order (every use waits for vmcnt(0) and lgkmcnt(0), which serializes the
// chunk prefetch).  These casts make them global_load.
typedef __attribute__((address_space(1))) const v4i g_v4i;
typedef __attribute__((address_space(1))) const int g_int;
__device__ __forceinline__ v4i ld_stream4(const int *p) {
    return __builtin_nontemporal_load((const g_v4i *)p);
}
__device__ __forceinline__ int ld_global(const int *p) { return *(const g_int *)p; }
__device__ __forceinline__ uint32_t ld_global_u32(const uint32_t *p) {
    return *(const __attribute__((address_space(1))) uint32_t *)p;
}

// ---------------------------------------------------------------------------
// Kernel prologues: tables from global memory into LDS.  dst[i] = val(i) for
// i < n, with the R loads of a thread issued before any of its stores.  A
// plain `dst[i] = src[i]` loop waits for each load in turn (the compiler
// cannot rule out that the LDS stores alias a generic source), which made
// the sieve's 49 KB prologue four serial global round trips (~6 us).
// val(i) must read global memory through address_space(1) (g_ld).
// ---------------------------------------------------------------------------
template <typename T>
__device__ __forceinline__ T g_ld(const T *p) {
    return *(const __attribute__((address_space(1))) T *)p;
}
__device__ __forceinline__ uint4 g_ld(const uint4 *p) {  // (HIP's uint4 is a class)
    typedef unsigned int v4u_t __attribute__((ext_vector_type(4)));
    const v4u_t v = *(const __attribute__((address_space(1))) v4u_t *)p;
    return make_uint4(v[0], v[1], v[2], v[3]);
}
// (the form with `at`: element i goes to *at(i), for two tables in one round)
template <int R, typename T, typename F, typename A>
__device__ __forceinline__ void lds_fill(T *, int n, F val, A at) {
    const int nt = (int)blockDim.x, tid = (int)threadIdx.x;
    for (int b = 0; b < n; b += R * nt) {
        T v[R];
#pragma unroll
        for (int k = 0; k < R; ++k) {
            const int i = b + k * nt + tid;
            v[k] = val(i < n ? i : n - 1);
        }
#pragma unroll
        for (int k = 0; k < R; ++k) {
            const int i = b + k * nt + tid;
            if (i < n) *at(i) = v[k];
        }
    }
}
template <int R, typename T, typename F>
__device__ __forceinline__ void lds_fill(T *dst, int n, F val) {
    const int nt = (int)blockDim.x, tid = (int)threadIdx.x;
    for (int b = 0; b < n; b += R * nt) {
        T v[R];
#pragma unroll
        for (int k = 0; k < R; ++k) {
            const int i = b + k * nt + tid;
            v[k] = val(i < n ? i : n - 1);
        }
#pragma unroll
        for (int k = 0; k < R; ++k) {
            const int i = b + k * nt + tid;
            if (i < n) dst[i] = v[k];
        }
    }
}

// ---------------------------------------------------------------------------
// TOA lookup
// ---------------------------------------------------------------------------
__device__ __forceinline__ void load_toa_tables(unsigned char *s_tab,
                                                const unsigned char *__restrict__ g_tab,
                                                const ToaParams &tp) {
    const uint4 *src = reinterpret_cast<const uint4 *>(g_tab);
    lds_fill<4>(reinterpret_cast<uint4 *>(s_tab), (int)(toa_lds_bytes(tp) / 16),
                [&](int i) { return g_ld(src + i); });
}

template <bool FAST>
__device__ __forceinline__ int toa_bin(int t, const unsigned char *s_tab, const ToaParams &tp) {
    if (FAST) {
        const unsigned d = (unsigned)t - (unsigned)tp.lo;
        if (d >= tp.span) return -1;
        const uint32_t *rthr = reinterpret_cast<const uint32_t *>(s_tab);
        const uint16_t *bst =
            reinterpret_cast<const uint16_t *>(s_tab + align16((size_t)(tp.T + 1) * 4));
        const int b = bst[d >> tp.shift];
        return b + (d >= rthr[b + 1] ? 1 : 0);
    } else {
        const long long tt = t;
        if (tt < tp.lo || tt >= tp.hi) return -1;
        const long long *thr = reinterpret_cast<const long long *>(s_tab);
        const uint32_t *bp =
            reinterpret_cast<const uint32_t *>(s_tab + align16((size_t)(tp.T + 1) * 8));
        const uint32_t pr = bp[(unsigned)((unsigned long long)(tt - tp.lo) >> tp.shift)];
        int b = (int)(pr & 0xFFFFu);
        int e = (int)(pr >> 16);
        while (b < e) {
            const int m = (b + e + 1) >> 1;
            if (tt >= thr[m]) b = m; else e = m - 1;
        }
        return b;
    }
}

// TOA bin without a branch (fast layout): out-of-range times look up a
// clamped bucket and are dropped by the final select, so the two LDS reads of
// every event can be in flight together
__device__ __forceinline__ int toa_bin_nb(int t, const unsigned char *s_tab, const ToaParams &tp) {
    const unsigned d = (unsigned)t - (unsigned)tp.lo;
    const unsigned dc = d < tp.span ? d : tp.span - 1u;
    const uint32_t *rthr = reinterpret_cast<const uint32_t *>(s_tab);
    const uint16_t *bst = reinterpret_cast<const uint16_t *>(s_tab + align16((size_t)(tp.T + 1) * 4));
    const int b = bst[dc >> tp.shift];
    const int r = b + (dc >= rthr[b + 1] ? 1 : 0);
    return d < tp.span ? r : -1;
}
// LUT entry -> flat histogram base (screen * T) or -1
__device__ __forceinline__ int lut_base(const uint16_t *__restrict__ lut, unsigned p, int T) {
    const unsigned v = lut[p];
    return v == 0xFFFFu ? -1 : (int)(v * (unsigned)T);
}
__device__ __forceinline__ int lut_base(const int *__restrict__ lut, unsigned p, int) {
    return lut[p];
}

template <typename LT, bool FAST>
__device__ __forceinline__ int event_key(int pid, int t, const LT *__restrict__ lut, int pid_off,
                                        unsigned L, const unsigned char *s_tab,
                                        const ToaParams &tp) {
    const unsigned p = (unsigned)pid - (unsigned)pid_off;
    if (p >= L) return -1;
    const int base = lut_base(lut, p, tp.T);
    if (base < 0) return -1;
    const int b = toa_bin<FAST>(t, s_tab, tp);
    return b < 0 ? -1 : base + b;
}

// ---------------------------------------------------------------------------
// wave / block helpers
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t lanes_below(unsigned long long m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                     __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// Global u32 += 1 for every active lane with k >= 0, equal keys of the wave
// merged first (CDNA has no match_any): each of up to ROUNDS rounds takes the
// lowest remaining lane's key and adds the number of lanes holding it with
// one atomic; lanes still left add alone.  Zipf-hot bins then cost one
// memory-side atomic per wave instead of one per event.  Safe under
// divergence (ballots see active lanes only).
template <int ROUNDS>
__device__ __forceinline__ void wave_add_aggregated(uint32_t *hist, int k) {
    const int lane = threadIdx.x & 63;
    unsigned long long act = __builtin_amdgcn_ballot_w64(k >= 0);
#pragma unroll
    for (int r = 0; r < ROUNDS; ++r) {
        if (!act) return;
        const int lead = __builtin_ctzll(act);
        const int kl = __builtin_amdgcn_readlane(k, lead);
        const unsigned long long m = __builtin_amdgcn_ballot_w64(k == kl) & act;
        if (lane == lead) atomicAdd(hist + kl, (uint32_t)__popcll(m));
        act &= ~m;
    }
    if ((act >> lane) & 1ull) atomicAdd(hist + k, 1u);
}

__device__ __forceinline__ uint32_t wave_inclusive_scan(uint32_t x) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(x, d, 64);
        if (lane >= d) x += y;
    }
    return x;
}

// exclusive prefix of v across the block; *total = block sum.  s_w >= 17
// uint32; contains two __syncthreads().
__device__ __forceinline__ uint32_t block_exclusive_scan(uint32_t v, uint32_t *s_w,
                                                         uint32_t *total) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int nw = blockDim.x >> 6;
    const uint32_t inc = wave_inclusive_scan(v);
    if (lane == 63) s_w[wid] = inc;
    __syncthreads();
    if (wid == 0) {
        const uint32_t w = lane < nw ? s_w[lane] : 0u;
        const uint32_t wi = wave_inclusive_scan(w);
        if (lane < nw) s_w[lane] = wi - w;
        if (lane == nw - 1) s_w[16] = wi;
    }
    __syncthreads();
    *total = s_w[16];
    return inc - v + s_w[wid];
}


// ---------------------------------------------------------------------------
// chunk loads for the partition kernels
// ---------------------------------------------------------------------------
struct ChunkRegs {
    int p[kPartEventsPerThread];
    int t[kPartEventsPerThread];
};

__device__ __forceinline__ void load_chunk(const SegDesc *s_seg, int n_segs, long long c,
                                           int pid_off, ChunkRegs &r) {
    int s = 0;
    while (s + 1 < n_segs && s_seg[s + 1].chunk0 <= c) ++s;
    const SegDesc sd = s_seg[s];
    const long long base = (c - sd.chunk0) * kChunk;
    const bool vec = (((uintptr_t)sd.pid | (uintptr_t)sd.toa) & 15u) == 0;
    const int tid = threadIdx.x;
#pragma unroll
    for (int j = 0; j < kPartEventsPerThread / 4; ++j) {
        const long long e0 = base + ((long long)j * kPartThreads + tid) * 4;
        if (vec && e0 + 3 < sd.n) {
            const v4i p = ld_stream4(sd.pid + e0);
            const v4i t = ld_stream4(sd.toa + e0);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                r.p[j * 4 + q] = p[q];
                r.t[j * 4 + q] = t[q];
            }
        } else {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const bool ok = e0 + q < sd.n;
                r.p[j * 4 + q] = ok ? ld_global(sd.pid + e0 + q) : pid_off - 1;  // outside the LUT: dropped
                r.t[j * 4 + q] = ok ? ld_global(sd.toa + e0 + q) : 0;
            }
        }
    }
}

}  // namespace lde
