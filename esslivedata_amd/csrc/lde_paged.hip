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

template <bool KEYS>
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
    const uintptr_t al = KEYS ? (uintptr_t)sd.pid : ((uintptr_t)sd.pid | (uintptr_t)sd.toa);
    const bool vec = (al & 15u) == 0;
    // key mode: sd.pid holds u32 keys; padding entries are -1 (dropped)
    const int fill = KEYS ? -1 : pid_off - 1;  // pid_off - 1 is outside the LUT: dropped
    const int tid = threadIdx.x;
#pragma unroll
    for (int j = 0; j < kPartEventsPerThread / 4; ++j) {
        const long long e0 = base + ((long long)j * kPartThreads + tid) * 4;
        if (vec && e0 + 3 < sd.n) {
            const v4i p = ld_stream4(sd.pid + e0);
#pragma unroll
            for (int q = 0; q < 4; ++q) r.p[j * 4 + q] = p[q];
            if (!KEYS) {
                const v4i t = ld_stream4(sd.toa + e0);
#pragma unroll
                for (int q = 0; q < 4; ++q) r.t[j * 4 + q] = t[q];
            }
        } else {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const bool ok = e0 + q < sd.n;
                r.p[j * 4 + q] = ok ? ld_global(sd.pid + e0 + q) : fill;
                if (!KEYS) r.t[j * 4 + q] = ok ? ld_global(sd.toa + e0 + q) : 0;
            }
        }
    }
}

// LDS carve of k_paged_partition (u32 words):
//   staging   kChunk + 16 * NT   tile runs, each [carry | new entries] rounded up to 8
//   counters  2 x align4(NT * SUBC + 1)   rank sub-counters, double-buffered by chunk parity
//   tile info 7 x align4(NT)    run, end, write fill, write page, new page, fill, page
//   carry     4 x NT            <= 7 pending u16 offsets per tile (one 16-byte group)
//   scan + pool 36, then the TOA lookup image
size_t paged_smem(int n_tiles, int subc, const ToaParams &tp) {
    const size_t nt4 = (size_t)align4(n_tiles);
    return 4 * ((size_t)kChunk + 16 * (size_t)n_tiles + 2 * (size_t)align4(n_tiles * subc + 1) +
                7 * nt4 + 4 * nt4 + 36) +
           toa_lds_bytes(tp);
}

// raw LUT entry of one event (the gather); p >= L reads nothing
__device__ __forceinline__ int lut_raw(const uint16_t *__restrict__ lut, unsigned p, unsigned L) {
    return p < L ? (int)lut[p] : 0xFFFF;
}
__device__ __forceinline__ int lut_raw(const int *__restrict__ lut, unsigned p, unsigned L) {
    return p < L ? lut[p] : -1;
}
__device__ __forceinline__ int raw_base(const uint16_t *, int v, int T) {
    return v == 0xFFFF ? -1 : v * T;
}
__device__ __forceinline__ int raw_base(const int *, int v, int) { return v; }

// Pass A.  Per 8192-event chunk:
//   R  rank every event inside its (tile, sub-counter)                 | sync
//   S  owner threads (tile t -> thread t mod 512): run sizes incl. the  |
//      tile's carried tail, block scan, sub-run starts, carry copied    |
//      to the head of the run, page allocation for the full 8-groups    | sync
//   P  scatter (tile << 16 | offset) into staging; then the NEXT chunk's |
//      LUT gathers + TOA bins are issued and its successor's events     |
//      are requested                                                    | sync
//   W  16-byte page stores of every full 8-group; owners keep the tail  |
//      (< 8 entries) in LDS for the next chunk and reset the counters   |
// so only whole 16-byte groups reach the pages; the tails are flushed once
// per launch, padded with 0xFFFF sentinels.
//
// KEYS: the segments hold ready (screen * T + bin) keys (the cold events of the
// SPLIT strategy) and the chunk count is read from n_chunks_dev.
template <int TILE_BITS, typename LT, bool FAST, int SUBC, bool KEYS>
__global__ __launch_bounds__(kPartThreads, kPartMinWavesPerEU) void k_paged_partition(
    const SegDesc *__restrict__ segs, int n_segs, long long n_chunks,
    const long long *__restrict__ n_chunks_dev, const LT *__restrict__ lut,
    int pid_off, unsigned L, const unsigned char *__restrict__ g_tab, ToaParams tp, int n_tiles,
    uint16_t *__restrict__ pages, uint32_t *__restrict__ page_tile, uint32_t *__restrict__ page_cnt,
    uint32_t *__restrict__ pool_used, int cap, uint32_t *__restrict__ overflow, int tail_release) {
    constexpr int EPT = kPartEventsPerThread;
    constexpr uint32_t MASK = (1u << TILE_BITS) - 1u;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int nt4 = align4(n_tiles);
    const int ncnt = align4(n_tiles * SUBC + 1);
    uint32_t *s_stg = reinterpret_cast<uint32_t *>(smem);
    uint32_t *s_cnt0 = s_stg + kChunk + 16 * n_tiles;
    uint32_t *s_run = s_cnt0 + 2 * ncnt;
    uint32_t *s_end = s_run + nt4;
    uint32_t *s_wfill = s_end + nt4;
    uint32_t *s_wcur = s_wfill + nt4;
    uint32_t *s_new = s_wcur + nt4;
    uint32_t *s_fill = s_new + nt4;
    uint32_t *s_cur = s_fill + nt4;
    uint32_t *s_carry = s_cur + nt4;  // 4 words per tile; word 3 bits 16..31 hold the count
    uint32_t *s_w = s_carry + 4 * nt4;
    uint32_t *s_pool = s_w + 32;
    unsigned char *s_tab = reinterpret_cast<unsigned char *>(s_pool + 4);
    const uint32_t pool_base = (uint32_t)blockIdx.x * (uint32_t)cap;
    if (KEYS) n_chunks = *n_chunks_dev;
    else load_toa_tables(s_tab, g_tab, tp);
    for (int i = threadIdx.x; i < 2 * ncnt; i += blockDim.x) s_cnt0[i] = 0;
    for (int t = threadIdx.x; t < n_tiles; t += blockDim.x) {
        s_fill[t] = 0;
        s_cur[t] = pool_base + t;  // first page of every tile, pre-assigned
        s_carry[4 * t + 3] = 0;
        page_tile[pool_base + t] = (uint32_t)t;
    }
    if (threadIdx.x == 0) s_pool[0] = (uint32_t)n_tiles;
    __syncthreads();

    const int tid = threadIdx.x;
    const int sub = tid & (SUBC - 1);
    int key[EPT];
    uint32_t rank[EPT];
    ChunkRegs nxt;
    // prologue: keys of the first chunk, events of the second in flight
    if ((long long)blockIdx.x < n_chunks) {
        load_chunk_global<KEYS>(segs, n_segs, blockIdx.x, pid_off, nxt);
#pragma unroll
        for (int e = 0; e < EPT; ++e) {
            if (KEYS) {
                key[e] = nxt.p[e];
                rank[e] = 0;
            } else {
                key[e] = lut_raw(lut, (unsigned)nxt.p[e] - (unsigned)pid_off, L);
                rank[e] = (uint32_t)toa_bin<FAST>(nxt.t[e], s_tab, tp);
            }
        }
        if ((long long)blockIdx.x + gridDim.x < n_chunks)
            load_chunk_global<KEYS>(segs, n_segs, blockIdx.x + gridDim.x, pid_off, nxt);
    }
    int parity = 0;
    for (long long c = blockIdx.x; c < n_chunks; c += gridDim.x, parity ^= 1) {
        uint32_t *s_cnt = s_cnt0 + parity * ncnt;
        // ---- R: finish the keys (the gathers were issued one phase earlier), rank
#pragma unroll
        for (int e = 0; e < EPT; ++e) {
            if (!KEYS) {
                const int base = raw_base(lut, key[e], tp.T);
                const int b = (int)rank[e];
                key[e] = (base < 0 || b < 0) ? -1 : base + b;
            }
            rank[e] = 0;
            if (key[e] >= 0) rank[e] = atomicAdd(&s_cnt[(key[e] >> TILE_BITS) * SUBC + sub], 1u);
        }
        __syncthreads();
        // ---- S: owner threads
        uint32_t sum = 0;
        for (int t = tid; t < n_tiles; t += kPartThreads) {
            uint32_t n = s_carry[4 * t + 3] >> 16;
#pragma unroll
            for (int s2 = 0; s2 < SUBC; ++s2) n += s_cnt[t * SUBC + s2];
            s_end[t] = n;  // run length for now; the run end after the scan
            sum += (n + 7u) & ~7u;
        }
        uint32_t total;
        uint32_t run = block_exclusive_scan(sum, s_w, &total);
        for (int t = tid; t < n_tiles; t += kPartThreads) {
            const uint32_t mt = s_end[t];
            if (mt > 0) {
                const uint4 cw = *reinterpret_cast<const uint4 *>(s_carry + 4 * t);
                const uint32_t cn = cw.w >> 16;
                uint32_t st = run + cn;
#pragma unroll
                for (int s2 = 0; s2 < SUBC; ++s2) {
                    const uint32_t n = s_cnt[t * SUBC + s2];
                    s_cnt[t * SUBC + s2] = st;
                    st += n;
                }
                const uint32_t hi = (uint32_t)t << 16;
                const uint32_t cv[7] = {cw.x & 0xFFFFu, cw.x >> 16, cw.y & 0xFFFFu, cw.y >> 16,
                                        cw.z & 0xFFFFu, cw.z >> 16, cw.w & 0xFFFFu};
#pragma unroll
                for (int j = 0; j < 7; ++j)
                    if ((uint32_t)j < cn) s_stg[run + j] = hi | cv[j];
                const uint32_t full = mt & ~7u;
                const uint32_t fill = s_fill[t];
                const uint32_t cur = s_cur[t];
                s_run[t] = run;
                s_end[t] = run + mt;
                s_wfill[t] = fill;
                s_wcur[t] = cur;
                if (full > 0) {
                    const uint32_t room = (uint32_t)kPage - fill;
                    uint32_t first = cur;
                    if (full > room) {
                        const uint32_t n_new = (full - room + kPage - 1) >> kPageBits;
                        const uint32_t off = atomicAdd(s_pool, n_new);
                        if (off + n_new > (uint32_t)cap) {  // cannot happen by construction
                            atomicOr(overflow, 1u);
                        } else {
                            first = pool_base + off;
                            page_cnt[cur] = kPage;  // the open page is now full
                            for (uint32_t q = 0; q < n_new; ++q) {
                                page_tile[first + q] = (uint32_t)t;
                                page_cnt[first + q] = kPage;
                            }
                        }
                    }
                    s_new[t] = first;
                    const uint32_t end = fill + full;
                    const uint32_t k_end = (end - 1) >> kPageBits;
                    if (k_end > 0) s_cur[t] = first + k_end - 1;
                    s_fill[t] = end - (k_end << kPageBits);
                }
                run += (mt + 7u) & ~7u;
            } else {
                s_run[t] = 0;  // s_end[t] == 0: empty run
            }
        }
        __syncthreads();
        // ---- P: scatter, then start the next chunk's keys
#pragma unroll
        for (int e = 0; e < EPT; ++e) {
            if (key[e] >= 0) {
                const uint32_t t = (uint32_t)key[e] >> TILE_BITS;
                s_stg[s_cnt[t * SUBC + sub] + rank[e]] = (t << 16) | ((uint32_t)key[e] & MASK);
            }
        }
        if (c + gridDim.x < n_chunks) {
#pragma unroll
            for (int e = 0; e < EPT; ++e) {
                if (KEYS) {
                    key[e] = nxt.p[e];
                } else {
                    key[e] = lut_raw(lut, (unsigned)nxt.p[e] - (unsigned)pid_off, L);
                    rank[e] = (uint32_t)toa_bin<FAST>(nxt.t[e], s_tab, tp);
                }
            }
            if (c + 2LL * gridDim.x < n_chunks)
                load_chunk_global<KEYS>(segs, n_segs, c + 2LL * gridDim.x, pid_off, nxt);
        }
        __syncthreads();
        // ---- W: full 8-groups to the pages (runs start 8-aligned in staging)
        for (uint32_t g = (uint32_t)tid * 8u; g < total; g += kPartThreads * 8u) {
            const uint4 v0 = *reinterpret_cast<const uint4 *>(s_stg + g);
            const uint32_t t = v0.x >> 16;
            if (g + 8u <= s_end[t]) {
                const uint4 v1 = *reinterpret_cast<const uint4 *>(s_stg + g + 4);
                const uint32_t pos = s_wfill[t] + (g - s_run[t]);
                const uint32_t k = pos >> kPageBits;
                const uint32_t page = k == 0 ? s_wcur[t] : s_new[t] + k - 1;
                uint4 w;
                w.x = (v0.x & 0xFFFFu) | (v0.y << 16);
                w.y = (v0.z & 0xFFFFu) | (v0.w << 16);
                w.z = (v1.x & 0xFFFFu) | (v1.y << 16);
                w.w = (v1.z & 0xFFFFu) | (v1.w << 16);
                if (page - pool_base < (uint32_t)cap)  // always true unless the pool overflowed
                    *reinterpret_cast<uint4 *>(pages + (size_t)page * kPage + (pos & (kPage - 1))) = w;
            }
        }
        // owners: keep the tail, reset this parity's counters
        for (int t = tid; t < n_tiles; t += kPartThreads) {
            {
                const uint32_t mt = s_end[t] - s_run[t];
                if (mt > 0) {
                    const uint32_t cn = mt & 7u;
                    const uint32_t b = s_run[t] + (mt & ~7u);
                    uint32_t v[7];
#pragma unroll
                    for (int j = 0; j < 7; ++j) v[j] = (uint32_t)j < cn ? (s_stg[b + j] & 0xFFFFu) : 0u;
                    *reinterpret_cast<uint4 *>(s_carry + 4 * t) =
                        make_uint4(v[0] | (v[1] << 16), v[2] | (v[3] << 16), v[4] | (v[5] << 16),
                                   v[6] | (cn << 16));
                }
#pragma unroll
                for (int s2 = 0; s2 < SUBC; ++s2) s_cnt[t * SUBC + s2] = 0;
            }
        }
    }
    __syncthreads();
    // flush: every tile's tail as one sentinel-padded group
    for (int t = threadIdx.x; t < n_tiles; t += blockDim.x) {
        const uint4 cw = *reinterpret_cast<const uint4 *>(s_carry + 4 * t);
        const uint32_t cn = cw.w >> 16;
        uint32_t fill = s_fill[t], cur = s_cur[t];
        if (cn > 0) {
            bool ok = true;
            if (fill == (uint32_t)kPage) {
                const uint32_t off = atomicAdd(s_pool, 1u);
                if (off + 1 > (uint32_t)cap) {
                    atomicOr(overflow, 1u);
                    ok = false;
                } else {
                    page_cnt[cur] = kPage;
                    cur = pool_base + off;
                    page_tile[cur] = (uint32_t)t;
                    fill = 0;
                }
            }
            if (ok) {
                uint32_t v[8];
                const uint32_t cv[7] = {cw.x & 0xFFFFu, cw.x >> 16, cw.y & 0xFFFFu, cw.y >> 16,
                                        cw.z & 0xFFFFu, cw.z >> 16, cw.w & 0xFFFFu};
#pragma unroll
                for (int j = 0; j < 8; ++j) v[j] = (j < 7 && (uint32_t)j < cn) ? cv[j] : 0xFFFFu;
                *reinterpret_cast<uint4 *>(pages + (size_t)cur * kPage + fill) =
                    make_uint4(v[0] | (v[1] << 16), v[2] | (v[3] << 16), v[4] | (v[5] << 16),
                               v[6] | (v[7] << 16));
                fill += 8;
            }
        }
        page_cnt[cur] = fill;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        pool_used[blockIdx.x] = min(s_pool[0], (uint32_t)cap);
        // this XCD's dirty page lines written back while other blocks still
        // run, not all in the end-of-kernel release (LDE_TAIL_RELEASE & 8)
        if (tail_release) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    }
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

// tile list bases + work items (t, first list index, last list index).  Tile
// prefixes go to LDS, then every thread emits items independently (binary
// search of its item's tile), so a hot tile's items are not written serially.
__device__ __forceinline__ uint32_t split_point(uint32_t j, uint32_t np, uint32_t ni) {
    const unsigned long long x = (unsigned long long)j * np;
    return x <= 0xffffffffULL ? (uint32_t)x / ni : (uint32_t)(x / ni);
}

__global__ __launch_bounds__(1024) void k_page_plan(const uint32_t *__restrict__ tile_pages,
                                                    const uint32_t *__restrict__ tile_events,
                                                    int n_tiles, uint32_t item_events,
                                                    uint32_t *__restrict__ tile_base,
                                                    uint4 *__restrict__ items,
                                                    uint32_t *__restrict__ item_count,
                                                    uint32_t max_items) {
    __shared__ uint32_t s_w[32];
    __shared__ uint32_t s_ib[kMaxTiles + 1];  // item prefix per tile
    __shared__ uint32_t s_pb[kMaxTiles];      // page-list prefix per tile
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
            s_pb[t] = pbase;
            s_ib[t] = ibase;
        }
        pbase += np[q];
        ibase += ni[q];
    }
    if (tid == 0) s_ib[n_tiles] = itot;
    __syncthreads();
    const uint32_t n_items = itot < max_items ? itot : max_items;
    for (uint32_t i = (uint32_t)tid; i < n_items; i += 1024u) {
        int lo = 0, hi = n_tiles - 1;  // last tile with s_ib[t] <= i
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (s_ib[mid] <= i) lo = mid; else hi = mid - 1;
        }
        const uint32_t nt_items = s_ib[lo + 1] - s_ib[lo];
        const uint32_t j = i - s_ib[lo];
        const uint32_t pages_t = (lo + 1 < n_tiles ? s_pb[lo + 1] : ptot) - s_pb[lo];
        items[i] = make_uint4((uint32_t)lo, s_pb[lo] + split_point(j, pages_t, nt_items),
                              s_pb[lo] + split_point(j + 1, pages_t, nt_items), 0u);
    }
    if (tid == 0) *item_count = n_items;
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
template <int TB, typename LT, bool FAST, int SUBC, bool KEYS = false>
static hipError_t launch_paged_t(const PagedArgs &a, const LT *lut, hipStream_t st,
                                 const long long *n_chunks_dev = nullptr) {
    const size_t sm = paged_smem(a.n_tiles, SUBC, a.tp);
    (void)hipFuncSetAttribute((const void *)k_paged_partition<TB, LT, FAST, SUBC, KEYS>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)sm);
    hipLaunchKernelGGL((k_paged_partition<TB, LT, FAST, SUBC, KEYS>), dim3(a.grid),
                       dim3(kPartThreads), sm, st, a.segs, a.n_segs, a.n_chunks, n_chunks_dev, lut,
                       a.pid_off, a.L, a.tab, a.tp, a.n_tiles, a.pages, a.page_tile, a.page_cnt,
                       a.pool_used, a.cap, a.overflow, a.tail_release);
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
