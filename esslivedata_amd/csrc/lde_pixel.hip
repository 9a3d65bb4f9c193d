// lde_pixel.hip -- PIXEL strategy: partition by pixel range, no LUT gather.
//
// PAGED (lde_paged.hip) partitions events by tile of the (S, T) histogram, so
// pass A gathers every event's LUT entry (one random L2 request per event:
// LOKI's 1.6 MB u16 LUT, bound by the L2 request rate).  When the screen
// footprint of a range of consecutive pixel ids fits in LDS (xy_plane and
// cylinder projections of ordered pixels: a 4,096-pixel range of LOKI bank 0
// lands in at most 288 screens), events can be partitioned by pixel range
// instead, with no gather at all, and the LUT lookup moves to pass B, where
// the range's slice of the LUT sits in LDS:
//
//   k_pix_count      events per (block, range), pid stream only
//   k_pix_scan       range-major exclusive offsets, range starts, work items
//   k_pix_scatter    per 8,192-event chunk: rank by range (LDS atomics), scan,
//                    range-sorted LDS staging, coalesced runs to each range's
//                    (block) slot; payload = local pixel | bin << rb (24 bits;
//                    0xFFFFFF = TOA outside the edges)
//   k_pix_accumulate one item = part of one range: the range's LUT slice
//                    (footprint-local screen index, u16) and its footprint
//                    counters (F x T u32) in LDS; flush with coalesced atomics
//
// Unknown ids (pid outside the LUT) are dropped in the count and the
// scatter alike; pixels the view drops map to 0xFFFF in the slice.  Counts
// are bit-identical to every other strategy.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "lde_device.h"
#include "lde_internal.h"

namespace lde {

namespace {

constexpr int kPixThreads = kPartThreads;          // 512
constexpr int kPixEPT = kPartEventsPerThread;      // 16 events per thread and chunk
constexpr uint32_t kPixDropped = 0xFFFFFFu;

// chunk c of the staged batch: pid (and toa) of every event this thread owns;
// events past a message's end read as pid_off - 1 (outside the LUT)
template <bool TOA>
__device__ __forceinline__ void pix_load(const SegDesc *__restrict__ segs, int n_segs, long long c,
                                         int pid_off, int (&p)[kPixEPT], int (&t)[kPixEPT]) {
    int lo = 0, hi = n_segs - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (segs[mid].chunk0 <= c) lo = mid; else hi = mid - 1;
    }
    const SegDesc sd = segs[lo];
    const long long base = (c - sd.chunk0) * kChunk;
    const uintptr_t al = TOA ? ((uintptr_t)sd.pid | (uintptr_t)sd.toa) : (uintptr_t)sd.pid;
    const bool vec = (al & 15u) == 0;
    const int tid = threadIdx.x;
#pragma unroll
    for (int j = 0; j < kPixEPT / 4; ++j) {
        const long long e0 = base + ((long long)j * kPixThreads + tid) * 4;
        if (vec && e0 + 3 < sd.n) {
            const v4i pv = ld_stream4(sd.pid + e0);
#pragma unroll
            for (int q = 0; q < 4; ++q) p[j * 4 + q] = pv[q];
            if (TOA) {
                const v4i tv = ld_stream4(sd.toa + e0);
#pragma unroll
                for (int q = 0; q < 4; ++q) t[j * 4 + q] = tv[q];
            }
        } else {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const bool ok = e0 + q < sd.n;
                p[j * 4 + q] = ok ? ld_global(sd.pid + e0 + q) : pid_off - 1;
                if (TOA) t[j * 4 + q] = ok ? ld_global(sd.toa + e0 + q) : 0;
            }
        }
    }
}

__device__ __forceinline__ void block_chunks(long long n, long long &cb, long long &ce) {
    cb = (long long)blockIdx.x * n / gridDim.x;
    ce = ((long long)blockIdx.x + 1) * n / gridDim.x;
}

}  // namespace

// ---------------------------------------------------------------------------
// Every chunk's run of a range is padded to a multiple of 4 payloads (the
// pads are dropped payloads), so the scatter writes whole 16-byte groups;
// the count sums those padded run lengths per (block, range).
__global__ __launch_bounds__(kPixThreads) void k_pix_count(PixArgs a) {
    __shared__ uint32_t s_cnt[kPixMaxRanges], s_tot[kPixMaxRanges];
    for (int r = threadIdx.x; r < a.nr; r += kPixThreads) s_cnt[r] = s_tot[r] = 0;
    __syncthreads();
    long long cb, ce;
    block_chunks(a.n_chunks, cb, ce);
    int p[kPixEPT], t[kPixEPT];
    for (long long c = cb; c < ce; ++c) {
        pix_load<false>(a.segs, a.n_segs, c, a.pid_off, p, t);
#pragma unroll
        for (int e = 0; e < kPixEPT; ++e) {
            const uint32_t q = (uint32_t)p[e] - (uint32_t)a.pid_off;
            if (q < a.L) atomicAdd(&s_cnt[q >> a.rb], 1u);
        }
        __syncthreads();
        for (int r = threadIdx.x; r < a.nr; r += kPixThreads) {
            s_tot[r] += (s_cnt[r] + 3u) & ~3u;
            s_cnt[r] = 0;
        }
        __syncthreads();
    }
    for (int r = threadIdx.x; r < a.nr; r += kPixThreads) a.counts[(size_t)blockIdx.x * a.nr + r] = s_tot[r];
}

// One block per range r: its total over the blocks and the exclusive prefix
// over blocks (counts[b][r] becomes the offset of (block b, range r) inside
// range r).
__global__ __launch_bounds__(1024) void k_pix_scan_blocks(PixArgs a, int grid,
                                                          uint32_t *__restrict__ rtot) {
    __shared__ uint32_t s_w[32];
    const int r = blockIdx.x;
    uint32_t carry = 0;
    for (int b0 = 0; b0 < grid; b0 += 1024) {
        const int b = b0 + (int)threadIdx.x;
        const size_t i = (size_t)b * a.nr + r;
        const uint32_t v = b < grid ? a.counts[i] : 0u;
        uint32_t tot;
        const uint32_t x = block_exclusive_scan(v, s_w, &tot);
        if (b < grid) a.counts[i] = carry + x;
        carry += tot;
        __syncthreads();
    }
    if (threadIdx.x == 0) rtot[r] = carry;
}

// One block of 1024 threads, thread r = range r: range starts (rstart) and
// work items, every range split into pieces of at most item_events.
__global__ __launch_bounds__(1024) void k_pix_scan(PixArgs a, const uint32_t *__restrict__ rtot,
                                                   uint32_t item_events, uint4 *__restrict__ items,
                                                   uint32_t *__restrict__ item_count, int max_items) {
    __shared__ uint32_t s_w[32];
    const int r = threadIdx.x;
    const uint32_t tot = r < a.nr ? rtot[r] : 0u;
    uint32_t all;
    const uint32_t start = block_exclusive_scan(tot, s_w, &all);
    const uint32_t k = tot > 0 ? (tot + item_events - 1) / item_events : 0u;
    uint32_t n_items;
    const uint32_t ifirst = block_exclusive_scan(k, s_w, &n_items);
    if (r < a.nr) {
        a.rstart[r] = start;
        for (uint32_t j = 0; j < k && ifirst + j < (uint32_t)max_items; ++j) {
            const uint32_t b0 = start + j * item_events;
            const uint32_t b1 = b0 + item_events < start + tot ? b0 + item_events : start + tot;
            items[ifirst + j] = make_uint4((uint32_t)r, b0, b1, 0u);
        }
    }
    if (threadIdx.x == 0) {
        a.rstart[a.nr] = all;
        *item_count = n_items < (uint32_t)max_items ? n_items : (uint32_t)max_items;
    }
}

// LDS: staging (kChunk u32) | counts, chunk offsets, cursors (nr each) |
// scan scratch (32) | TOA image
size_t pix_scatter_smem(const ToaParams &tp) {
    return 4 * ((size_t)kChunk + 4 * (size_t)kPixMaxRanges + 3 * (size_t)kPixMaxRanges + 32) +
           toa_lds_bytes(tp);
}

template <bool FAST>
__global__ __launch_bounds__(kPixThreads) void k_pix_scatter(PixArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    uint32_t *s_stg = reinterpret_cast<uint32_t *>(smem);
    uint32_t *s_cnt = s_stg + kChunk + 4 * kPixMaxRanges;  // staging holds the pads too
    uint32_t *s_off = s_cnt + kPixMaxRanges;
    uint32_t *s_cur = s_off + kPixMaxRanges;
    uint32_t *s_w = s_cur + kPixMaxRanges;
    unsigned char *s_tab = reinterpret_cast<unsigned char *>(s_w + 32);
    load_toa_tables(s_tab, a.tab, a.tp);
    const int tid = threadIdx.x;
    for (int r = tid; r < a.nr; r += kPixThreads) {
        s_cnt[r] = 0;
        s_cur[r] = a.rstart[r] + a.counts[(size_t)blockIdx.x * a.nr + r];  // this block's slot of range r
    }
    __syncthreads();
    const uint32_t mask = (1u << a.rb) - 1u;
    long long cb, ce;
    block_chunks(a.n_chunks, cb, ce);
    int p[kPixEPT], t[kPixEPT];
    if (cb < ce) pix_load<true>(a.segs, a.n_segs, cb, a.pid_off, p, t);
    for (long long c = cb; c < ce; ++c) {
        uint32_t word[kPixEPT], rank[kPixEPT];
#pragma unroll
        for (int e = 0; e < kPixEPT; ++e) {
            const uint32_t q = (uint32_t)p[e] - (uint32_t)a.pid_off;
            const int b = toa_bin<FAST>(t[e], s_tab, a.tp);
            const uint32_t r = q >> a.rb;
            word[e] = q < a.L ? ((r << 24) | (b < 0 ? kPixDropped : ((q & mask) | ((uint32_t)b << a.rb))))
                              : 0xFFFFFFFFu;
            rank[e] = q < a.L ? atomicAdd(&s_cnt[r], 1u) : 0xFFFFFFFFu;  // unknown id: no slot
        }
        // the next chunk's events load while this one is partitioned
        if (c + 1 < ce) pix_load<true>(a.segs, a.n_segs, c + 1, a.pid_off, p, t);
        __syncthreads();
        // runs padded to 4: staging offsets, slot cursors and the pads are
        // 16-byte aligned groups
        uint32_t v = 0, total;
        if (tid < a.nr) v = (s_cnt[tid] + 3u) & ~3u;  // nr <= kPixMaxRanges <= kPixThreads
        const uint32_t off = block_exclusive_scan(v, s_w, &total);
        if (tid < a.nr) {
            s_off[tid] = off;
            for (uint32_t j = s_cnt[tid]; j < v; ++j) s_stg[off + j] = ((uint32_t)tid << 24) | kPixDropped;
        }
        __syncthreads();
#pragma unroll
        for (int e = 0; e < kPixEPT; ++e)
            if (rank[e] != 0xFFFFFFFFu) s_stg[s_off[word[e] >> 24] + rank[e]] = word[e];
        __syncthreads();
        // a 4-group never straddles two runs; its slot position is 4-aligned
        for (uint32_t g = (uint32_t)tid * 4u; g < total; g += kPixThreads * 4u) {
            const uint4 w = *reinterpret_cast<const uint4 *>(s_stg + g);
            const uint32_t r = w.x >> 24;
            *reinterpret_cast<uint4 *>(a.payload + s_cur[r] + (g - s_off[r])) =
                make_uint4(w.x & 0xFFFFFFu, w.y & 0xFFFFFFu, w.z & 0xFFFFFFu, w.w & 0xFFFFFFu);
        }
        __syncthreads();
        for (int r = tid; r < a.nr; r += kPixThreads) {
            s_cur[r] += (s_cnt[r] + 3u) & ~3u;
            s_cnt[r] = 0;
        }
        __syncthreads();
    }
}

// LDS: LUT slice (2^rb u16) | footprint counters (F x T u32)
size_t pix_acc_smem(int rb, int fmax, int T) {
    return align16(((size_t)2 << rb)) + 4 * (size_t)fmax * (size_t)T;
}

__global__ __launch_bounds__(1024) void k_pix_accumulate(PixArgs a, const uint16_t *__restrict__ loc,
                                                         const uint32_t *__restrict__ fp_off,
                                                         const uint32_t *__restrict__ fp_scr,
                                                         const uint4 *__restrict__ items,
                                                         const uint32_t *__restrict__ item_count,
                                                         int T, uint32_t *__restrict__ hist) {
    if (blockIdx.x >= *item_count) return;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const uint4 it = items[blockIdx.x];
    const uint32_t r = it.x;
    const uint32_t f0 = fp_off[r], nf = fp_off[r + 1] - f0;
    const uint32_t nbin = nf * (uint32_t)T;
    const uint32_t span = 1u << a.rb;
    uint16_t *s_loc = reinterpret_cast<uint16_t *>(smem);
    uint32_t *s_cnt = reinterpret_cast<uint32_t *>(smem + align16((size_t)2 << a.rb));
    const size_t q0 = (size_t)r << a.rb;
    for (uint32_t j = threadIdx.x; j < span; j += blockDim.x)
        s_loc[j] = q0 + j < a.L ? loc[q0 + j] : (uint16_t)0xFFFFu;
    for (uint32_t j = threadIdx.x; j < nbin; j += blockDim.x) s_cnt[j] = 0;
    __syncthreads();
    const uint32_t mask = span - 1u;
    const uint32_t e0 = it.y, e1 = it.z;
    auto add = [&](uint32_t w) __attribute__((always_inline)) {
        if (w == kPixDropped) return;
        const uint32_t f = s_loc[w & mask];
        if (f != 0xFFFFu) atomicAdd(&s_cnt[f * (uint32_t)T + (w >> a.rb)], 1u);
    };
    // head to a 16-byte boundary, then four payloads per lane
    const uint32_t h = e0 + ((4u - (e0 & 3u)) & 3u) < e1 ? e0 + ((4u - (e0 & 3u)) & 3u) : e1;
    if (threadIdx.x < h - e0) add(a.payload[e0 + threadIdx.x]);
    const uint32_t n4 = (e1 - h) >> 2;
    // U groups of 4 per lane and iteration, the next iteration's loads issued
    // before this one's LDS work (the loop is otherwise load-latency bound)
    constexpr int U = 4;
    const int *pl = reinterpret_cast<const int *>(a.payload) + h;
    const uint32_t step = blockDim.x * U;
    v4i cur[U], nxt[U];
    uint32_t i0 = threadIdx.x;
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const uint32_t i = i0 + u * blockDim.x;
        cur[u] = i < n4 ? ld_stream4(pl + 4 * i) : v4i{-1, -1, -1, -1};
    }
    for (; i0 < n4; i0 += step) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t i = i0 + step + u * blockDim.x;
            nxt[u] = i < n4 ? ld_stream4(pl + 4 * i) : v4i{-1, -1, -1, -1};
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int q = 0; q < 4; ++q) add((uint32_t)cur[u][q] & 0xFFFFFFu);
#pragma unroll
        for (int u = 0; u < U; ++u) cur[u] = nxt[u];
    }
    const uint32_t tail = h + 4 * n4;
    if (tail + threadIdx.x < e1) add(a.payload[tail + threadIdx.x]);
    __syncthreads();
    // flush: consecutive counters of one screen row are consecutive bins
    for (uint32_t j = threadIdx.x; j < nbin; j += blockDim.x) {
        const uint32_t n = s_cnt[j];
        if (n) {
            const uint32_t f = j / (uint32_t)T;
            atomicAdd(&hist[(size_t)fp_scr[f0 + f] * T + (j - f * (uint32_t)T)], n);
        }
    }
}

hipError_t launch_pixel(const PixArgs &a, const PixSetup &s, int replica, uint32_t item_events,
                        int max_items, uint4 *items, uint32_t *item_count, uint32_t *hist,
                        hipStream_t st, int phase) {
    if (a.nr > kPixMaxRanges || a.nr > 1024) return hipErrorInvalidValue;
    if (phase == 0) {
        hipLaunchKernelGGL(k_pix_count, dim3(a.grid), dim3(kPixThreads), 0, st, a);
        hipLaunchKernelGGL(k_pix_scan_blocks, dim3(a.nr), dim3(1024), 0, st, a, a.grid, a.rstart + a.nr + 1);
        hipLaunchKernelGGL(k_pix_scan, dim3(1), dim3(1024), 0, st, a, a.rstart + a.nr + 1, item_events,
                           items, item_count, max_items);
        const size_t sm = pix_scatter_smem(a.tp);
        if (a.tp.fast) {
            (void)hipFuncSetAttribute((const void *)k_pix_scatter<true>,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)sm);
            hipLaunchKernelGGL(k_pix_scatter<true>, dim3(a.grid), dim3(kPixThreads), sm, st, a);
        } else {
            (void)hipFuncSetAttribute((const void *)k_pix_scatter<false>,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)sm);
            hipLaunchKernelGGL(k_pix_scatter<false>, dim3(a.grid), dim3(kPixThreads), sm, st, a);
        }
    } else {
        const size_t sm = pix_acc_smem(s.rb, s.fmax, a.tp.T);
        (void)hipFuncSetAttribute((const void *)k_pix_accumulate,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)sm);
        hipLaunchKernelGGL(k_pix_accumulate, dim3((unsigned)max_items), dim3(1024), sm, st, a,
                           s.loc + (size_t)replica * a.L, s.fp_off, s.fp_scr, items, item_count,
                           a.tp.T, hist);
    }
    return hipGetLastError();
}

}  // namespace lde
