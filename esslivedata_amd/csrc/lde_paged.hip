// lde_paged.hip -- PAGED partition strategy (default for large batches).
//
// Same per-event work as PARTITION (lde_binning.hip) but pass A appends each
// tile's tile-sorted run to a per-(block, tile) chain of 2 KB pages taken from
// a block-private page pool (LDS counter, no global atomics).  A tile's open
// page line stays L2-resident between chunks, so the short runs of cold tiles
// are merged in L2 before they reach HBM, and pass B streams whole pages
// (1024 u16 entries = one wave, two 16-byte loads per lane) instead of walking
// thousands of short chunk-runs.
//
//   k_paged_partition : keys, LDS rank/scan/sort, page allocation, write-out
//   k_page_count      : per (block, tile) page and event counts
//   k_page_scan       : per tile exclusive scan over blocks
//   k_page_plan       : tile page-list bases + balanced work items
//   k_page_scatter    : per-tile page lists
//   k_page_accumulate : LDS sub-histogram per item, coalesced atomic flush
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "lde_device.h"
#include "lde_internal.h"

namespace lde {

__device__ __forceinline__ void load_chunk_global(const SegDesc *__restrict__ segs, int n_segs,
                                                  long long c, int pid_off, ChunkRegs &r) {
    // segment of chunk c: binary search over chunk0 (uniform per block)
    int lo = 0, hi = n_segs - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (segs[mid].chunk0 <= c) lo = mid; else hi = mid - 1;
    }
    const SegDesc sd = segs[lo];
    const long long base = (c - sd.chunk0) * kChunk;
    const bool vec = (((uintptr_t)sd.pid | (uintptr_t)sd.toa) & 15u) == 0;
    const int tid = threadIdx.x;
#pragma unroll
    for (int j = 0; j < kPartEventsPerThread / 4; ++j) {
        const long long e0 = base + ((long long)j * kPartThreads + tid) * 4;
        if (vec && e0 + 3 < sd.n) {
            const v4i p = __builtin_nontemporal_load(reinterpret_cast<const v4i *>(sd.pid + e0));
            const v4i t = __builtin_nontemporal_load(reinterpret_cast<const v4i *>(sd.toa + e0));
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                r.p[j * 4 + q] = p[q];
                r.t[j * 4 + q] = t[q];
            }
        } else {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const bool ok = e0 + q < sd.n;
                r.p[j * 4 + q] = ok ? sd.pid[e0 + q] : pid_off - 1;  // outside the LUT: dropped
                r.t[j * 4 + q] = ok ? sd.toa[e0 + q] : 0;
            }
        }
    }
}

// staging holds every tile run padded to a multiple of 8 entries (sentinel
// 0xFFFF offsets), so runs start 16-byte aligned in LDS and in their pages
size_t paged_smem(int n_tiles, int subc, const ToaParams &tp) {
    return 4 * ((size_t)kChunk + 8 * (size_t)n_tiles) +
           4 * ((size_t)align4(n_tiles * subc + 1) + 4 * (size_t)align4(n_tiles) + 36) +
           toa_lds_bytes(tp);
}

template <int TILE_BITS, typename LT, bool FAST, int SUBC>
__global__ __launch_bounds__(kPartThreads, kPartMinWavesPerEU) void k_paged_partition(
    const SegDesc *__restrict__ segs, int n_segs, long long n_chunks, const LT *__restrict__ lut,
    int pid_off, unsigned L, const unsigned char *__restrict__ g_tab, ToaParams tp, int n_tiles,
    uint16_t *__restrict__ pages, uint32_t *__restrict__ page_tile, uint32_t *__restrict__ page_cnt,
    uint32_t *__restrict__ pool_used, int cap, uint32_t *__restrict__ overflow) {
    constexpr int EPT = kPartEventsPerThread;
    constexpr int TPT = kMaxTiles / kPartThreads;
    constexpr uint32_t MASK = (1u << TILE_BITS) - 1u;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    // LDS carve: staging (tile<<16 | offset) | sub-counters/starts | fill | cur | new | scan | pool | TOA
    uint32_t *s_stg = reinterpret_cast<uint32_t *>(smem);
    uint32_t *s_cnt = s_stg + kChunk + 8 * n_tiles;
    uint32_t *s_fill = s_cnt + align4(n_tiles * SUBC + 1);
    uint32_t *s_cur = s_fill + align4(n_tiles);
    uint32_t *s_new = s_cur + align4(n_tiles);
    uint32_t *s_loc = s_new + align4(n_tiles);
    uint32_t *s_w = s_loc + align4(n_tiles);
    uint32_t *s_pool = s_w + 32;
    unsigned char *s_tab = reinterpret_cast<unsigned char *>(s_pool + 4);
    const uint32_t pool_base = (uint32_t)blockIdx.x * (uint32_t)cap;
    load_toa_tables(s_tab, g_tab, tp);
    for (int i = threadIdx.x; i < n_tiles * SUBC; i += blockDim.x) s_cnt[i] = 0;
    for (int t = threadIdx.x; t < n_tiles; t += blockDim.x) {
        s_fill[t] = 0;
        s_cur[t] = pool_base + t;  // first page of every tile, pre-assigned
        s_new[t] = 0;
        page_tile[pool_base + t] = (uint32_t)t;
    }
    if (threadIdx.x == 0) s_pool[0] = (uint32_t)n_tiles;
    __syncthreads();

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int sub = lane & (SUBC - 1);
    ChunkRegs nxt;
    if ((long long)blockIdx.x < n_chunks) load_chunk_global(segs, n_segs, blockIdx.x, pid_off, nxt);
    for (long long c = blockIdx.x; c < n_chunks; c += gridDim.x) {
        int key[EPT];
        uint32_t rank[EPT];
#pragma unroll
        for (int e = 0; e < EPT; ++e)
            key[e] = event_key<LT, FAST>(nxt.p[e], nxt.t[e], lut, pid_off, L, s_tab, tp);
        // the next chunk's events load while this chunk runs its LDS phases
        if (c + gridDim.x < n_chunks) load_chunk_global(segs, n_segs, c + gridDim.x, pid_off, nxt);
        // ---- rank inside (tile, sub-counter): SUBC counters per tile spread a hot
        // tile's same-address LDS atomics over SUBC banks
#pragma unroll
        for (int e = 0; e < EPT; ++e) {
            rank[e] = 0;
            if (key[e] >= 0) rank[e] = atomicAdd(&s_cnt[(key[e] >> TILE_BITS) * SUBC + sub], 1u);
        }
        __syncthreads();
        // ---- scan of padded tile totals, sub-run starts, padding, page allocation
        // (thread tid owns tiles [tid*TPT, tid*TPT + TPT))
        uint32_t sum = 0;
        const int t0 = tid * TPT;
        for (int t = t0; t < t0 + TPT && t < n_tiles; ++t) {
            uint32_t n = 0;
#pragma unroll
            for (int s2 = 0; s2 < SUBC; ++s2) n += s_cnt[t * SUBC + s2];
            s_loc[t] = n;
            sum += (n + 7u) & ~7u;
        }
        uint32_t total;
        uint32_t run = block_exclusive_scan(sum, s_w, &total);
        for (int t = t0; t < t0 + TPT && t < n_tiles; ++t) {
            const uint32_t n_t = s_loc[t];
            const uint32_t padded = (n_t + 7u) & ~7u;
            if (n_t > 0) {
                uint32_t st = run;
#pragma unroll
                for (int s2 = 0; s2 < SUBC; ++s2) {
                    const uint32_t n = s_cnt[t * SUBC + s2];
                    s_cnt[t * SUBC + s2] = st;
                    st += n;
                }
                for (uint32_t k = run + n_t; k < run + padded; ++k)
                    s_stg[k] = ((uint32_t)t << 16) | 0xFFFFu;  // sentinel padding
                const uint32_t fill = s_fill[t];
                const uint32_t room = (uint32_t)kPage - fill;
                if (padded > room) {
                    const uint32_t n_new = (padded - room + kPage - 1) >> kPageBits;
                    const uint32_t off = atomicAdd(s_pool, n_new);
                    if (off + n_new > (uint32_t)cap) {  // cannot happen by construction
                        atomicOr(overflow, 1u);
                        s_new[t] = s_cur[t];
                    } else {
                        const uint32_t first = pool_base + off;
                        s_new[t] = first;
                        page_cnt[s_cur[t]] = kPage;  // the open page is now full
                        for (uint32_t k = 0; k < n_new; ++k) {
                            page_tile[first + k] = (uint32_t)t;
                            page_cnt[first + k] = kPage;
                        }
                    }
                }
            }
            run += padded;
        }
        __syncthreads();
        // ---- scatter into LDS staging (tile-sorted), tile id beside the offset
#pragma unroll
        for (int e = 0; e < EPT; ++e) {
            if (key[e] >= 0) {
                const uint32_t t = (uint32_t)key[e] >> TILE_BITS;
                s_stg[s_cnt[t * SUBC + sub] + rank[e]] = (t << 16) | ((uint32_t)key[e] & MASK);
            }
        }
        __syncthreads();
        // ---- write-out: one 16-byte store per 8-entry group (runs are 8-aligned)
        for (uint32_t g = (uint32_t)tid * 8u; g < total; g += kPartThreads * 8u) {
            const uint4 v0 = *reinterpret_cast<const uint4 *>(s_stg + g);
            const uint4 v1 = *reinterpret_cast<const uint4 *>(s_stg + g + 4);
            const uint32_t t = v0.x >> 16;
            const uint32_t pos = s_fill[t] + (g - s_cnt[t * SUBC]);
            const uint32_t k = pos >> kPageBits;
            const uint32_t page = k == 0 ? s_cur[t] : s_new[t] + k - 1;
            uint4 w;
            w.x = (v0.x & 0xFFFFu) | (v0.y << 16);
            w.y = (v0.z & 0xFFFFu) | (v0.w << 16);
            w.z = (v1.x & 0xFFFFu) | (v1.y << 16);
            w.w = (v1.z & 0xFFFFu) | (v1.w << 16);
            if (page - pool_base < (uint32_t)cap)  // always true unless the pool overflowed
                *reinterpret_cast<uint4 *>(pages + (size_t)page * kPage + (pos & (kPage - 1))) = w;
        }
        __syncthreads();
        // ---- advance the open page of the owned tiles, reset the counters
        for (int t = t0; t < t0 + TPT && t < n_tiles; ++t) {
            const uint32_t n_t = s_loc[t];
            if (n_t > 0) {
                const uint32_t end = s_fill[t] + ((n_t + 7u) & ~7u);
                const uint32_t k_end = (end - 1) >> kPageBits;
                if (k_end > 0) s_cur[t] = s_new[t] + k_end - 1;
                s_fill[t] = end - (k_end << kPageBits);
            }
#pragma unroll
            for (int s2 = 0; s2 < SUBC; ++s2) s_cnt[t * SUBC + s2] = 0;
        }
        __syncthreads();
    }
    for (int t = threadIdx.x; t < n_tiles; t += blockDim.x) page_cnt[s_cur[t]] = s_fill[t];
    if (threadIdx.x == 0) pool_used[blockIdx.x] = min(s_pool[0], (uint32_t)cap);
}

// per (block, tile): number of non-empty pages and events
__global__ __launch_bounds__(256) void k_page_count(const uint32_t *__restrict__ page_tile,
                                                    const uint32_t *__restrict__ page_cnt,
                                                    const uint32_t *__restrict__ pool_used, int cap,
                                                    int n_tiles, uint32_t *__restrict__ cntp,
                                                    uint32_t *__restrict__ evp) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    uint32_t *s_np = reinterpret_cast<uint32_t *>(smem);
    uint32_t *s_ev = s_np + n_tiles;
    for (int t = threadIdx.x; t < n_tiles; t += blockDim.x) s_np[t] = s_ev[t] = 0;
    __syncthreads();
    const uint32_t base = blockIdx.x * (uint32_t)cap;
    const uint32_t used = min(pool_used[blockIdx.x], (uint32_t)cap);
    for (uint32_t p = threadIdx.x; p < used; p += blockDim.x) {
        const uint32_t c = page_cnt[base + p];
        if (c) {
            const uint32_t t = page_tile[base + p];
            atomicAdd(&s_np[t], 1u);
            atomicAdd(&s_ev[t], c);
        }
    }
    __syncthreads();
    for (int t = threadIdx.x; t < n_tiles; t += blockDim.x) {
        cntp[(size_t)blockIdx.x * n_tiles + t] = s_np[t];
        evp[(size_t)blockIdx.x * n_tiles + t] = s_ev[t];
    }
}

// per tile: exclusive scan of page counts over blocks (in place), totals
__global__ __launch_bounds__(256) void k_page_scan(uint32_t *__restrict__ cntp,
                                                   const uint32_t *__restrict__ evp, int rows,
                                                   int n_tiles, uint32_t *__restrict__ tile_pages,
                                                   uint32_t *__restrict__ tile_events) {
    __shared__ uint32_t s_w[32];
    const int t = blockIdx.x;
    uint32_t carry = 0, ev = 0;
    for (int r0 = 0; r0 < rows; r0 += blockDim.x) {
        const int r = r0 + threadIdx.x;
        const uint32_t v = r < rows ? cntp[(size_t)r * n_tiles + t] : 0u;
        ev += r < rows ? evp[(size_t)r * n_tiles + t] : 0u;
        uint32_t tot;
        const uint32_t ex = block_exclusive_scan(v, s_w, &tot);
        if (r < rows) cntp[(size_t)r * n_tiles + t] = carry + ex;
        carry += tot;
        __syncthreads();
    }
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) ev += __shfl_xor(ev, d, 64);
    if ((threadIdx.x & 63) == 0) s_w[20 + (threadIdx.x >> 6)] = ev;
    __syncthreads();
    if (threadIdx.x == 0) {
        tile_pages[t] = carry;
        tile_events[t] = s_w[20] + s_w[21] + s_w[22] + s_w[23];
    }
}

// tile list bases + work items (t, first list index, last list index)
__global__ __launch_bounds__(1024) void k_page_plan(const uint32_t *__restrict__ tile_pages,
                                                    const uint32_t *__restrict__ tile_events,
                                                    int n_tiles, uint32_t item_events,
                                                    uint32_t *__restrict__ tile_base,
                                                    uint4 *__restrict__ items,
                                                    uint32_t *__restrict__ item_count,
                                                    uint32_t max_items) {
    __shared__ uint32_t s_w[32];
    constexpr int TPT = kMaxTiles / 1024;
    const int tid = threadIdx.x;
    const int t0 = tid * TPT;
    uint32_t np[TPT], ni[TPT];
    uint32_t psum = 0, isum = 0;
#pragma unroll
    for (int q = 0; q < TPT; ++q) {
        const int t = t0 + q;
        np[q] = t < n_tiles ? tile_pages[t] : 0u;
        const uint32_t ev = t < n_tiles ? tile_events[t] : 0u;
        uint32_t n = ev == 0 ? 0u : (ev + item_events - 1) / item_events;
        if (n > np[q]) n = np[q];
        ni[q] = n;
        psum += np[q];
        isum += ni[q];
    }
    uint32_t ptot, itot;
    uint32_t pbase = block_exclusive_scan(psum, s_w, &ptot);
    __syncthreads();
    uint32_t ibase = block_exclusive_scan(isum, s_w, &itot);
#pragma unroll
    for (int q = 0; q < TPT; ++q) {
        const int t = t0 + q;
        if (t < n_tiles) {
            tile_base[t] = pbase;
            for (uint32_t j = 0; j < ni[q] && ibase + j < max_items; ++j) {
                const uint32_t lo = pbase + (uint32_t)((unsigned long long)j * np[q] / ni[q]);
                const uint32_t hi = pbase + (uint32_t)((unsigned long long)(j + 1) * np[q] / ni[q]);
                items[ibase + j] = make_uint4((uint32_t)t, lo, hi, 0u);
            }
        }
        pbase += np[q];
        ibase += ni[q];
    }
    if (tid == 0) *item_count = itot < max_items ? itot : max_items;
}

// per-tile page lists
__global__ __launch_bounds__(256) void k_page_scatter(const uint32_t *__restrict__ page_tile,
                                                      const uint32_t *__restrict__ page_cnt,
                                                      const uint32_t *__restrict__ pool_used,
                                                      int cap, int n_tiles,
                                                      const uint32_t *__restrict__ cntp,
                                                      const uint32_t *__restrict__ tile_base,
                                                      uint32_t *__restrict__ list) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    uint32_t *s_rank = reinterpret_cast<uint32_t *>(smem);
    for (int t = threadIdx.x; t < n_tiles; t += blockDim.x) s_rank[t] = 0;
    __syncthreads();
    const uint32_t base = blockIdx.x * (uint32_t)cap;
    const uint32_t used = min(pool_used[blockIdx.x], (uint32_t)cap);
    const uint32_t *off = cntp + (size_t)blockIdx.x * n_tiles;
    for (uint32_t p = threadIdx.x; p < used; p += blockDim.x) {
        if (page_cnt[base + p]) {
            const uint32_t t = page_tile[base + p];
            const uint32_t r = atomicAdd(&s_rank[t], 1u);
            list[tile_base[t] + off[t] + r] = base + p;
        }
    }
}

// pass B over pages
template <int TILE_BITS>
__global__ __launch_bounds__(kTileThreads) void k_page_accumulate(
    const uint16_t *__restrict__ pages, const uint32_t *__restrict__ page_cnt,
    const uint32_t *__restrict__ list, const uint4 *__restrict__ items,
    const uint32_t *__restrict__ item_count, uint32_t *__restrict__ hist, long long n_bins) {
    constexpr int TB = 1 << TILE_BITS;
    constexpr int NW = kTileThreads / 64;
    __shared__ __attribute__((aligned(16))) uint32_t s_tile[TB];
    if (blockIdx.x >= *item_count) return;
    const uint4 it = items[blockIdx.x];
    for (int i = threadIdx.x * 4; i < TB; i += kTileThreads * 4)
        *reinterpret_cast<uint4 *>(s_tile + i) = make_uint4(0, 0, 0, 0);
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const uint32_t wid = (uint32_t)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t e0 = (uint32_t)lane * 16u;
    uint32_t idx = it.y + wid;
    uint32_t page = 0, cnt = 0;
    uint4 a = make_uint4(0, 0, 0, 0), b = make_uint4(0, 0, 0, 0);
    if (idx < it.z) {
        page = list[idx];
        cnt = page_cnt[page];
        const uint4 *src = reinterpret_cast<const uint4 *>(pages + (size_t)page * kPage + e0);
        if (e0 < cnt) a = src[0];
        if (e0 + 8u < cnt) b = src[1];
    }
    while (idx < it.z) {
        // prefetch the wave's next page while adding this one
        const uint32_t nidx = idx + NW;
        uint32_t npage = 0, ncnt = 0;
        uint4 na = make_uint4(0, 0, 0, 0), nb = make_uint4(0, 0, 0, 0);
        if (nidx < it.z) {
            npage = list[nidx];
            ncnt = page_cnt[npage];
            const uint4 *src = reinterpret_cast<const uint4 *>(pages + (size_t)npage * kPage + e0);
            if (e0 < ncnt) na = src[0];
            if (e0 + 8u < ncnt) nb = src[1];
        }
        const uint32_t w[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            const uint32_t v = (w[q >> 1] >> ((q & 1) * 16)) & 0xFFFFu;
            if (e0 + (uint32_t)q < cnt && v != 0xFFFFu) atomicAdd(&s_tile[v], 1u);
        }
        idx = nidx;
        page = npage;
        cnt = ncnt;
        a = na;
        b = nb;
    }
    __syncthreads();
    const long long base = (long long)it.x << TILE_BITS;
    for (int i = threadIdx.x; i < TB; i += kTileThreads) {
        const uint32_t v = s_tile[i];
        if (v != 0u && base + i < n_bins) atomicAdd(hist + base + i, v);
    }
}

// ---------------------------------------------------------------------------
// launch wrappers
// ---------------------------------------------------------------------------
template <int TB, typename LT, bool FAST, int SUBC>
static hipError_t launch_paged_t(const PagedArgs &a, const LT *lut, hipStream_t st) {
    const size_t sm = paged_smem(a.n_tiles, SUBC, a.tp);
    (void)hipFuncSetAttribute((const void *)k_paged_partition<TB, LT, FAST, SUBC>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)sm);
    hipLaunchKernelGGL((k_paged_partition<TB, LT, FAST, SUBC>), dim3(a.grid), dim3(kPartThreads),
                       sm, st, a.segs, a.n_segs, a.n_chunks, lut, a.pid_off, a.L, a.tab, a.tp,
                       a.n_tiles, a.pages, a.page_tile, a.page_cnt, a.pool_used, a.cap, a.overflow);
    return hipGetLastError();
}

template <int TB, typename LT>
static hipError_t launch_paged_tl(const PagedArgs &a, const LT *lut, hipStream_t st) {
    if (a.tp.fast)
        return a.subc == 4 ? launch_paged_t<TB, LT, true, 4>(a, lut, st)
                           : launch_paged_t<TB, LT, true, 1>(a, lut, st);
    return a.subc == 4 ? launch_paged_t<TB, LT, false, 4>(a, lut, st)
                       : launch_paged_t<TB, LT, false, 1>(a, lut, st);
}

template <int TB>
static hipError_t launch_paged_tb(const PagedArgs &a, hipStream_t st) {
    return a.lut16 ? launch_paged_tl<TB>(a, (const uint16_t *)a.lut, st)
                   : launch_paged_tl<TB>(a, (const int *)a.lut, st);
}

hipError_t launch_paged_partition(const PagedArgs &a, hipStream_t st) {
    switch (a.tile_bits) {
    case 13: return launch_paged_tb<13>(a, st);
    case 14: return launch_paged_tb<14>(a, st);
    case 15: return launch_paged_tb<15>(a, st);
    default: return hipErrorInvalidValue;
    }
}

hipError_t launch_page_plan(const PagedArgs &a, uint32_t item_events, uint32_t *cntp,
                            uint32_t *evp, uint32_t *tile_pages, uint32_t *tile_events,
                            uint32_t *tile_base, uint4 *items, uint32_t *item_count,
                            uint32_t max_items, uint32_t *list, hipStream_t st) {
    const size_t sm2 = (size_t)a.n_tiles * 8;
    hipLaunchKernelGGL(k_page_count, dim3(a.grid), dim3(256), sm2, st, a.page_tile, a.page_cnt,
                       a.pool_used, a.cap, a.n_tiles, cntp, evp);
    hipLaunchKernelGGL(k_page_scan, dim3(a.n_tiles), dim3(256), 0, st, cntp, evp, a.grid,
                       a.n_tiles, tile_pages, tile_events);
    hipLaunchKernelGGL(k_page_plan, dim3(1), dim3(1024), 0, st, tile_pages, tile_events,
                       a.n_tiles, item_events, tile_base, items, item_count, max_items);
    hipLaunchKernelGGL(k_page_scatter, dim3(a.grid), dim3(256), (size_t)a.n_tiles * 4, st,
                       a.page_tile, a.page_cnt, a.pool_used, a.cap, a.n_tiles, cntp, tile_base,
                       list);
    return hipGetLastError();
}

hipError_t launch_page_accumulate(int tile_bits, const PagedArgs &a, const uint32_t *list,
                                  const uint4 *items, const uint32_t *item_count, uint32_t *hist,
                                  long long n_bins, int grid, hipStream_t st) {
    switch (tile_bits) {
    case 13:
        hipLaunchKernelGGL(k_page_accumulate<13>, dim3(grid), dim3(kTileThreads), 0, st, a.pages,
                           a.page_cnt, list, items, item_count, hist, n_bins);
        break;
    case 14:
        hipLaunchKernelGGL(k_page_accumulate<14>, dim3(grid), dim3(kTileThreads), 0, st, a.pages,
                           a.page_cnt, list, items, item_count, hist, n_bins);
        break;
    case 15:
        hipLaunchKernelGGL(k_page_accumulate<15>, dim3(grid), dim3(kTileThreads), 0, st, a.pages,
                           a.page_cnt, list, items, item_count, hist, n_bins);
        break;
    default:
        return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace lde
