// lde_hotset.hip -- hot-set selection of the SPLIT strategy (SIEVE pass).
//
// Detector event streams are skewed (DREAM: Zipf pixel intensities; the top
// 1 % of pixels carry more than half of the events).
// The screens that receive most events get a full TOA row of u32 counters in
// every sieve block's LDS (lde_sieve.hip), and the most-sampled pixels a slot
// in its LDS pixel table; both are chosen from a sample of the batch:
//
//   k_sample_screens : per-screen and per-pixel event counts of a few sampled
//                      chunks (LDS, aggregated per block)
//   k_screen_sum     : column sums of the samples
//   k_select_hot     : top-H screens -> row numbers (single block)
//
// The hot set is a performance hint only: every event lands in the same bin
// whether its row is hot or cold, so the counts stay bit-exact whatever the
// sample picked.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "lde_device.h"
#include "lde_internal.h"

namespace lde {

namespace {

// Loads one chunk's pixel ids.  The vector/element choice is block-uniform (a
// scalar branch), so no divergent control flow sits between these loads and
// their uses.
template <int THREADS, int EPT>
__device__ __forceinline__ void load_chunk_pids(const SegDesc *__restrict__ segs, int n_segs,
                                                long long c, int fill, int (&p)[EPT]) {
    int lo = 0, hi = n_segs - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (segs[mid].chunk0 <= c) lo = mid; else hi = mid - 1;
    }
    const SegDesc sd = segs[lo];
    const long long base = (c - sd.chunk0) * kChunk;
    if (((uintptr_t)sd.pid & 15u) == 0 && base + kChunk <= sd.n) {
#pragma unroll
        for (int j = 0; j < EPT / 4; ++j) {
            const long long e0 = base + ((long long)j * THREADS + threadIdx.x) * 4;
            const v4i pv = ld_stream4(sd.pid + e0);
#pragma unroll
            for (int q = 0; q < 4; ++q) p[j * 4 + q] = pv[q];
        }
    } else {
        // tail chunk or misaligned segment: element loads of a clamped index
#pragma unroll
        for (int j = 0; j < EPT / 4; ++j) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const long long e = base + ((long long)j * THREADS + threadIdx.x) * 4 + q;
                const bool ok = e < sd.n;
                const int pv = ld_global(sd.pid + (ok ? e : 0));
                p[j * 4 + q] = ok ? pv : fill;
            }
        }
    }
}

__device__ __forceinline__ int screen_of(const uint16_t *__restrict__ lut, unsigned p, int) {
    const unsigned v = lut[p];
    return v == 0xFFFFu ? -1 : (int)v;
}
__device__ __forceinline__ int screen_of(const int *__restrict__ lut, unsigned p, int T) {
    const int v = lut[p];
    return v < 0 ? -1 : v / T;
}

}  // namespace

// ---------------------------------------------------------------------------
// hot-set selection
// ---------------------------------------------------------------------------
// Per-pixel sample counts are aggregated in an LDS open-addressing table
// (keys | counts, 2^hbits slots after the S screen counters) and flushed with
// one global atomic per distinct pixel per block: a Zipf-hot pixel then takes
// at most one memory-side atomic per sampled block instead of one per event
// (round 1: 1.14 ms for DREAM, every hot-pixel event serialized on one
// address).  A pixel that finds no slot within kSampleMaxProbe probes falls
// back to its own global atomic, so the counts stay exact.
constexpr int kSampleMaxProbe = 8;
constexpr uint32_t kSampleEmpty = 0xFFFFFFFFu;
template <typename LT>
__global__ __launch_bounds__(kSplitThreads) void k_sample_screens(
    const SegDesc *__restrict__ segs, int n_segs, long long n_chunks, const LT *__restrict__ lut,
    int pid_off, unsigned L, int T, int S, uint32_t *__restrict__ part,
    uint32_t *__restrict__ pix_cnt, int hbits) {
    extern __shared__ __attribute__((aligned(16))) uint32_t s_cnt[];
    const uint32_t H = (pix_cnt && hbits > 0) ? (1u << hbits) : 0u;
    uint32_t *s_key = s_cnt + align4(S);
    uint32_t *s_val = s_key + H;
    for (int i = threadIdx.x; i < S; i += kSplitThreads) s_cnt[i] = 0;
    for (uint32_t i = threadIdx.x; i < H; i += kSplitThreads) {
        s_key[i] = kSampleEmpty;
        s_val[i] = 0;
    }
    __syncthreads();
    const long long c = (long long)blockIdx.x * n_chunks / gridDim.x;
    int p[kSplitEPT];
    load_chunk_pids<kSplitThreads, kSplitEPT>(segs, n_segs, c, pid_off - 1, p);
#pragma unroll
    for (int e = 0; e < kSplitEPT; ++e) {
        const unsigned q = (unsigned)p[e] - (unsigned)pid_off;
        const int s = q < L ? screen_of(lut, q, T) : -1;
        if (s >= 0) atomicAdd(&s_cnt[s], 1u);
        // pixel counts of every id inside the LUT, dropped pixels included: the
        // SIEVE table then holds frequent dropped pixels too, so their events
        // need no gather (a view that drops most of the detector, e.g.
        // mantle_front_layer, would otherwise gather nearly every event)
        if (q < L && pix_cnt) {
            {
                bool done = false;
                if (H) {
                    uint32_t h = (q * 2654435761u) >> (32 - hbits);
                    for (int k = 0; k < kSampleMaxProbe && !done; ++k) {
                        const uint32_t old = atomicCAS(&s_key[h], kSampleEmpty, q);
                        if (old == kSampleEmpty || old == q) {
                            atomicAdd(&s_val[h], 1u);
                            done = true;
                        }
                        h = (h + 1u) & (H - 1u);
                    }
                }
                if (!done) atomicAdd(pix_cnt + q, 1u);
            }
        }
    }
    __syncthreads();
    uint32_t *dst = part + (size_t)blockIdx.x * S;
    for (int i = threadIdx.x; i < S; i += kSplitThreads) dst[i] = s_cnt[i];
    for (uint32_t i = threadIdx.x; i < H; i += kSplitThreads) {
        const uint32_t k = s_key[i];
        if (k != kSampleEmpty) atomicAdd(pix_cnt + k, s_val[i]);
    }
}

__global__ __launch_bounds__(256) void k_screen_sum(const uint32_t *__restrict__ part, int rows,
                                                    int S, uint32_t *__restrict__ cnt) {
    const int s = blockIdx.x * 256 + threadIdx.x;
    if (s >= S) return;
    uint32_t v = 0;
    for (int r = 0; r < rows; ++r) v += part[(size_t)r * S + s];
    cnt[s] = v;
}

// Top-H screens by sampled count.  Counts fall into log2 classes; every class
// above the one that overflows H is taken whole, the overflowing class is
// taken in screen order.  stats = {sampled events, events in hot rows, rows}.
__global__ __launch_bounds__(1024) void k_select_hot(const uint32_t *__restrict__ cnt, int S,
                                                     int H, uint16_t *__restrict__ screen_row,
                                                     uint32_t *__restrict__ row_screen,
                                                     uint32_t *__restrict__ stats) {
    __shared__ uint32_t s_cls[33];
    __shared__ uint32_t s_w[32];
    __shared__ uint32_t s_sel[4];
    const int tid = threadIdx.x;
    if (H >= S) {  // a row for every screen, sampled or not: no event is cold
        uint32_t tot = 0;
        for (int s = tid; s < S; s += 1024) {
            tot += cnt[s];
            screen_row[s] = (uint16_t)(s + 1);
            row_screen[s] = (uint32_t)s;
        }
        uint32_t tt;
        (void)block_exclusive_scan(tot, s_w, &tt);
        if (tid == 0) {
            stats[0] = stats[1] = tt;
            stats[2] = (uint32_t)S;
            stats[3] = 0;
        }
        return;
    }
    if (tid < 33) s_cls[tid] = 0;
    __syncthreads();
    const int per = (S + 1023) / 1024;
    const int s0 = min(S, tid * per), s1 = min(S, s0 + per);
    uint32_t tot = 0;
    for (int s = s0; s < s1; ++s) {
        const uint32_t c = cnt[s];
        tot += c;
        if (c) atomicAdd(&s_cls[32 - __clz(c)], 1u);
    }
    __syncthreads();
    if (tid == 0) {
        uint32_t acc = 0;
        int k = 32;
        for (; k >= 1; --k) {
            if (acc + s_cls[k] > (uint32_t)H) break;
            acc += s_cls[k];
        }
        s_sel[0] = (uint32_t)(k < 1 ? 0 : k);  // class taken partially (0: none)
        s_sel[1] = acc;                        // screens taken in full
    }
    __syncthreads();
    const uint32_t kpart = s_sel[0], full = s_sel[1];
    auto cls = [](uint32_t c) { return c ? (uint32_t)(32 - __clz(c)) : 0u; };
    uint32_t n1 = 0, n2 = 0;
    for (int s = s0; s < s1; ++s) {
        const uint32_t k = cls(cnt[s]);
        n1 += (k > kpart && k > 0) ? 1u : 0u;
        n2 += (kpart > 0 && k == kpart) ? 1u : 0u;
    }
    uint32_t t1, t2;
    uint32_t o1 = block_exclusive_scan(n1, s_w, &t1);
    __syncthreads();
    uint32_t o2 = block_exclusive_scan(n2, s_w, &t2);
    const uint32_t room = (uint32_t)H - full;
    uint32_t hot = 0;
    for (int s = s0; s < s1; ++s) {
        const uint32_t c = cnt[s];
        const uint32_t k = cls(c);
        uint32_t row = 0xFFFFFFFFu;
        if (k > kpart && k > 0) {
            row = o1++;
        } else if (kpart > 0 && k == kpart) {
            if (o2 < room) row = full + o2;
            ++o2;
        }
        if (row != 0xFFFFFFFFu) {
            screen_row[s] = (uint16_t)(row + 1);
            row_screen[row] = (uint32_t)s;
            hot += c;
        } else {
            screen_row[s] = 0;
        }
    }
    __syncthreads();
    uint32_t ht;
    (void)block_exclusive_scan(hot, s_w, &ht);
    __syncthreads();
    uint32_t tt;
    (void)block_exclusive_scan(tot, s_w, &tt);
    if (tid == 0) {
        stats[0] = tt;
        stats[1] = ht;
        stats[2] = min(t1 + min(t2, room), (uint32_t)H);
        stats[3] = 0;  // k_sieve_table: sampled events of the table's pixels
    }
}

// ---------------------------------------------------------------------------
// launch wrappers
// ---------------------------------------------------------------------------
// Hot-set selection in two steps: launch_hot_sample (per-screen and per-pixel
// counts of the sampled chunks), then launch_hot_pick (top a.rows screens).
hipError_t launch_hot_sample(const SplitArgs &a, int replica, hipStream_t st) {
    if (a.cache_bits > 0) {
        const hipError_t e = hipMemsetAsync(a.pix_cnt, 0, (size_t)a.L * 4, st);
        if (e != hipSuccess) return e;
    }
    // LDS: S screen counters + the pixel table (keys | counts), up to 2^13 slots
    int hbits = 0;
    if (a.cache_bits > 0) {
        hbits = 13;
        while (hbits > 6 && ((size_t)align4(a.S) + (2u << hbits)) * 4 > kSplitSmemMax) --hbits;
        if (((size_t)align4(a.S) + (2u << hbits)) * 4 > kSplitSmemMax) hbits = 0;
    }
    const size_t sm = ((size_t)align4(a.S) + (hbits ? (2u << hbits) : 0u)) * 4;
    // no room for the table (hbits 0): plain global atomics
    uint32_t *pix_cnt = a.cache_bits > 0 ? a.pix_cnt : nullptr;
    const void *lut_r = a.lut16 ? (const void *)((const uint16_t *)a.lut + (size_t)replica * a.L)
                                : (const void *)((const int *)a.lut + (size_t)replica * a.L);
    if (a.lut16) {
        (void)hipFuncSetAttribute((const void *)k_sample_screens<uint16_t>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)sm);
        hipLaunchKernelGGL(k_sample_screens<uint16_t>, dim3(a.sample_blocks), dim3(kSplitThreads), sm,
                           st, a.segs, a.n_segs, a.n_chunks, (const uint16_t *)lut_r, a.pid_off,
                           (unsigned)a.L, a.tp.T, a.S, a.sample_part, pix_cnt, hbits);
    } else {
        (void)hipFuncSetAttribute((const void *)k_sample_screens<int>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)sm);
        hipLaunchKernelGGL(k_sample_screens<int>, dim3(a.sample_blocks), dim3(kSplitThreads), sm, st,
                           a.segs, a.n_segs, a.n_chunks, (const int *)lut_r, a.pid_off,
                           (unsigned)a.L, a.tp.T, a.S, a.sample_part, pix_cnt, hbits);
    }
    hipLaunchKernelGGL(k_screen_sum, dim3((a.S + 255) / 256), dim3(256), 0, st, a.sample_part,
                       a.sample_blocks, a.S, a.screen_cnt);
    return hipGetLastError();
}

hipError_t launch_hot_pick(const SplitArgs &a, hipStream_t st) {
    hipLaunchKernelGGL(k_select_hot, dim3(1), dim3(1024), 0, st, a.screen_cnt, a.S, a.rows,
                       a.screen_row, a.row_screen, a.stats);
    return hipGetLastError();
}

}  // namespace lde
