// lde_binning.hip -- CDNA4 (gfx950) event-binning kernels.
//
// Hot path, per event:
//   pid -> LUT[replica][pid - pid_offset]   screen index or invalid; folds
//          group_event_data membership + pixel index + projection
//          (group_by_pixel.py:46-54, projectors.py:118-152 / 243-270)
//   toa -> TOA bin under scipp's half-open float64-edge rule (providers.py:205-210)
//   count[screen*T + bin] += 1
//
// Exact integer TOA binning: for int32 t and float64 edge e, t >= e <=> t >= ceil(e).
// The host turns the f64 edges into integer thresholds and builds the LDS
// image of a lookup table; two layouts:
//   FAST    : u32 thresholds relative to lo + u16 bucket table whose buckets are
//             narrower than every bin, so bin = bst[d >> shift] + (d >= rthr[b+1])
//             (one LDS gather, one compare, no branch).
//   general : int64 thresholds + (first, last) candidate pairs per bucket with a
//             binary search inside the bucket (any sorted edges).
//
// Strategies (bit-identical integer counts):
//   ATOMIC    : one pass, agent-scope u32 atomics, equal keys of a wave merged
//               first (wave_add_aggregated).
//   PARTITION : pass A partitions events into LDS-sized tiles of the (S, T)
//               histogram (chunk-major tile-sorted runs, no global atomics);
//               k_plan splits tiles into balanced work items; pass B
//               accumulates each item in an LDS sub-histogram and flushes the
//               non-zero bins with coalesced atomics.
//   monitors  : conflict-free per-lane-column LDS histogram.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "lde_device.h"
#include "lde_internal.h"

namespace lde {

// ---------------------------------------------------------------------------
// ATOMIC strategy: one pass, global u32 atomics (agent scope)
// ---------------------------------------------------------------------------
// events i0, i0 + stride, ... of one message, wave-aggregated atomics
template <typename LT, bool FAST>
__device__ __forceinline__ void atomic_stream(const SegDesc &seg, long long i0, long long stride,
                                              const LT *__restrict__ lut, int pid_off, unsigned L,
                                              const unsigned char *smem, const ToaParams &tp,
                                              uint32_t *__restrict__ hist) {
    const long long n = seg.n;
    long long tail = 0;
    if ((((uintptr_t)seg.pid | (uintptr_t)seg.toa) & 15u) == 0) {
        const long long n4 = n >> 2;
        for (long long i = i0; i < n4; i += stride) {
            const v4i p = ld_stream4(seg.pid + 4 * i);
            const v4i t = ld_stream4(seg.toa + 4 * i);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                wave_add_aggregated<4>(hist, event_key<LT, FAST>(p[q], t[q], lut, pid_off, L, smem, tp));
            }
        }
        tail = n4 << 2;
    }
    for (long long i = tail + i0; i < n; i += stride) {
        wave_add_aggregated<4>(hist, event_key<LT, FAST>(ld_global(seg.pid + i), ld_global(seg.toa + i),
                                                         lut, pid_off, L, smem, tp));
    }
}

template <typename LT, bool FAST>
__global__ __launch_bounds__(256) void k_bin_atomic(const SegKargAtomic segs, int n_segs,
                                                    const LT *__restrict__ lut, int pid_off,
                                                    unsigned L,
                                                    const unsigned char *__restrict__ g_tab,
                                                    ToaParams tp, uint32_t *__restrict__ hist) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    load_toa_tables(smem, g_tab, tp);
    __syncthreads();
    // up to kKargSegsAtomic messages per launch (small batches: BIFROST's 45
    // bank messages of 1,000 events take one launch instead of 45).  The host
    // gives every message a contiguous range of blocks (SegDesc::chunk0 = its
    // first block; at least one each): a block finds its message with a
    // binary search and streams it at the range's stride.  (Before, every
    // block walked the messages in order to find its own, a chain of
    // dependent descriptor loads that grew the launch by ~0.4 us per message.)
    int lo = 0, hi = n_segs - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (segs.s[mid].chunk0 <= (long long)blockIdx.x) lo = mid; else hi = mid - 1;
    }
    const SegDesc seg = segs.s[lo];
    const long long b0 = seg.chunk0;
    const long long b1 = lo + 1 < n_segs ? segs.s[lo + 1].chunk0 : (long long)gridDim.x;
    atomic_stream<LT, FAST>(seg, ((long long)blockIdx.x - b0) * blockDim.x + threadIdx.x,
                            (b1 - b0) * blockDim.x, lut, pid_off, L, smem, tp, hist);
}

// More messages than fit the kernel arguments (BIFROST at the reference
// cadence: a batch of 14 pulses x 45 bank messages is one push): one
// descriptor per block in device memory, chunk0 = (the block's index inside
// its message's block range) << 32 | (that range's length), so a block reads
// its message with one descriptor load, no search.
template <typename LT, bool FAST>
__global__ __launch_bounds__(256) void k_bin_atomic_blocks(const SegDesc *__restrict__ blocks,
                                                           const LT *__restrict__ lut, int pid_off,
                                                           unsigned L,
                                                           const unsigned char *__restrict__ g_tab,
                                                           ToaParams tp, uint32_t *__restrict__ hist) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    load_toa_tables(smem, g_tab, tp);
    __syncthreads();
    const SegDesc seg = blocks[blockIdx.x];
    const long long j = (long long)((unsigned long long)seg.chunk0 >> 32);
    const long long nb = seg.chunk0 & 0xffffffffLL;
    atomic_stream<LT, FAST>(seg, j * blockDim.x + threadIdx.x, nb * blockDim.x, lut, pid_off, L, smem,
                            tp, hist);
}

// ---------------------------------------------------------------------------
// PARTITION strategy, pass A: chunk-major tile partition
//   One launch covers up to kMaxSegs staged segments (ev44 messages); global
//   chunk c maps to the segment with segs[s].chunk0 <= c < segs[s+1].chunk0.
//   The valid events of chunk c are written tile-sorted to payload[c*CH ...]
//   as u16 offsets inside their tile, with per-tile run starts
//   starts[c*(NT+1) + t].  The next chunk's events are prefetched into
//   registers while the current chunk runs its LDS phases.
// ---------------------------------------------------------------------------
template <int TILE_BITS, typename LT, bool FAST>
__global__ __launch_bounds__(kPartThreads, kPartMinWavesPerEU) void k_partition(
    const SegDesc *__restrict__ segs, int n_segs, long long c_begin, long long n_chunks,
    const LT *__restrict__ lut, int pid_off, unsigned L, const unsigned char *__restrict__ g_tab,
    ToaParams tp, int n_tiles, uint16_t *__restrict__ payload, uint32_t *__restrict__ starts,
    uint32_t *__restrict__ part) {
    constexpr int EPT = kPartEventsPerThread;
    constexpr int CH = kChunk;
    constexpr int TPT = kMaxTiles / kPartThreads;  // tiles per thread in the scan
    constexpr uint32_t MASK = (1u << TILE_BITS) - 1u;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    // LDS carve: staging | counts | totals | scan | segments | TOA tables
    uint16_t *s_stg = reinterpret_cast<uint16_t *>(smem);
    uint32_t *s_cnt = reinterpret_cast<uint32_t *>(smem + CH * 2);
    uint32_t *s_tot = s_cnt + align4(n_tiles + 1);
    uint32_t *s_w = s_tot + align4(n_tiles);
    SegDesc *s_seg = reinterpret_cast<SegDesc *>(s_w + 32);
    unsigned char *s_tab = reinterpret_cast<unsigned char *>(s_seg + kMaxSegs);
    load_toa_tables(s_tab, g_tab, tp);
    for (int i = threadIdx.x; i < n_segs; i += blockDim.x) s_seg[i] = segs[i];
    for (int i = threadIdx.x; i <= n_tiles; i += blockDim.x) s_cnt[i] = 0;
    for (int i = threadIdx.x; i < n_tiles; i += blockDim.x) s_tot[i] = 0;
    __syncthreads();

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    ChunkRegs nxt;
    if (c_begin + blockIdx.x < n_chunks)
        load_chunk(s_seg, n_segs, c_begin + blockIdx.x, pid_off, nxt);
    for (long long c = c_begin + blockIdx.x; c < n_chunks; c += gridDim.x) {
        int key[EPT];
        uint32_t rank[EPT];
        if (LDE_DIAG(tp.pad) == 0) {
#pragma unroll
            for (int e = 0; e < EPT; ++e)
                key[e] = event_key<LT, FAST>(nxt.p[e], nxt.t[e], lut, pid_off, L, s_tab, tp);
        } else {  // LDE_ABLATE diagnostics: timing only, results are wrong by design
#pragma unroll
            for (int e = 0; e < EPT; ++e) {
                const unsigned p = (unsigned)nxt.p[e] - (unsigned)pid_off;
                const int base = (LDE_DIAG(tp.pad) & 1) ? (int)((p & 16383u) * (unsigned)tp.T)
                                              : (p < L ? lut_base(lut, p, tp.T) : -1);
                const int b = (LDE_DIAG(tp.pad) & 2) ? (int)((unsigned)nxt.t[e] & 63u) : toa_bin<FAST>(nxt.t[e], s_tab, tp);
                key[e] = (p >= L || base < 0 || b < 0) ? -1 : base + b;
            }
        }
        // the next chunk's events load while this chunk runs its LDS phases
        if (c + gridDim.x < n_chunks) load_chunk(s_seg, n_segs, c + gridDim.x, pid_off, nxt);
        // ---- rank inside tile: LDS returning atomics
#pragma unroll
        for (int e = 0; e < EPT; ++e) {
            const int tile = key[e] >= 0 ? (key[e] >> TILE_BITS) : -1;
            rank[e] = 0;
            if (LDE_DIAG(tp.pad) & 4) {
                rank[e] = (uint32_t)(e * 64 + lane) & 255u;
            } else if (tile >= 0) {
                rank[e] = atomicAdd(&s_cnt[tile], 1u);
            }
        }
        __syncthreads();
        // ---- exclusive scan of the tile counts
        uint32_t loc[TPT];
        uint32_t sum = 0;
        const int t0 = tid * TPT;
#pragma unroll
        for (int q = 0; q < TPT; ++q) {
            const int t = t0 + q;
            loc[q] = t < n_tiles ? s_cnt[t] : 0u;
            sum += loc[q];
        }
        uint32_t total;
        uint32_t run = block_exclusive_scan(sum, s_w, &total);
        uint32_t *g_starts = starts + c * (long long)(n_tiles + 1);
#pragma unroll
        for (int q = 0; q < TPT; ++q) {
            const int t = t0 + q;
            if (t < n_tiles) {
                s_cnt[t] = run;  // becomes the run start
                g_starts[t] = run;
                s_tot[t] += loc[q];
            }
            run += loc[q];
        }
        if (tid == 0) g_starts[n_tiles] = total;
        __syncthreads();
        // ---- scatter into LDS staging (tile-sorted)
        if (!(LDE_DIAG(tp.pad) & 8)) {
#pragma unroll
            for (int e = 0; e < EPT; ++e)
                if (key[e] >= 0) s_stg[s_cnt[key[e] >> TILE_BITS] + rank[e]] = (uint16_t)(key[e] & MASK);
        } else {
            int acc = 0;
#pragma unroll
            for (int e = 0; e < EPT; ++e) acc += key[e];
            if (acc == 0x7fffffff) s_stg[tid] = 1;
        }
        __syncthreads();
        // ---- coalesced write-out of the valid prefix (16 B per lane)
        uint16_t *g_out = payload + c * (long long)CH;
        if (!(LDE_DIAG(tp.pad) & 8))
            for (int i = tid * 8; i < (int)total; i += kPartThreads * 8)
                *reinterpret_cast<uint4 *>(g_out + i) = *reinterpret_cast<const uint4 *>(s_stg + i);
        for (int i = tid; i <= n_tiles; i += blockDim.x) s_cnt[i] = 0;
        __syncthreads();
    }
    // per-block tile totals (row blockIdx.x is owned by this block; accumulates
    // across the launches of one accumulate, which run in stream order)
    uint32_t *g_part = part + (long long)blockIdx.x * n_tiles;
    for (int t = threadIdx.x; t < n_tiles; t += blockDim.x) g_part[t] += s_tot[t];
}

// ---------------------------------------------------------------------------
// PARTITION strategy, plan: per-tile totals -> balanced work items
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_tile_totals(const uint32_t *__restrict__ part,
                                                     int part_rows, int n_tiles,
                                                     uint32_t *__restrict__ totals) {
    __shared__ uint32_t s_r[4];
    const int t = blockIdx.x;
    uint32_t v = 0;
    for (int r = threadIdx.x; r < part_rows; r += blockDim.x) v += part[(long long)r * n_tiles + t];
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) v += __shfl_xor(v, d, 64);
    if ((threadIdx.x & 63) == 0) s_r[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0) totals[t] = s_r[0] + s_r[1] + s_r[2] + s_r[3];
}

__global__ __launch_bounds__(1024) void k_plan(const uint32_t *__restrict__ totals, int n_tiles,
                                               long long n_chunks, uint32_t item_events,
                                               uint32_t *__restrict__ tile_items,
                                               uint2 *__restrict__ items,
                                               uint32_t *__restrict__ item_count,
                                               uint32_t max_items) {
    __shared__ uint32_t s_w[32];
    constexpr int TPT = kMaxTiles / 1024;
    const int tid = threadIdx.x;
    uint32_t ni[TPT];
    uint32_t lane_mode[TPT];
    uint32_t sum = 0;
    const int t0 = tid * TPT;
#pragma unroll
    for (int q = 0; q < TPT; ++q) {
        const int t = t0 + q;
        const uint32_t tot = t < n_tiles ? totals[t] : 0u;
        ni[q] = tot == 0 ? 0u : (tot + item_events - 1) / item_events;
        // short average runs per chunk: one lane per chunk in pass B
        lane_mode[q] = (long long)tot < (long long)kLaneModeRun * n_chunks ? 0x80000000u : 0u;
        sum += ni[q];
    }
    uint32_t total;
    uint32_t run = block_exclusive_scan(sum, s_w, &total);
#pragma unroll
    for (int q = 0; q < TPT; ++q) {
        const int t = t0 + q;
        if (t < n_tiles) {
            tile_items[t] = ni[q];
            for (uint32_t j = 0; j < ni[q] && run + j < max_items; ++j)
                items[run + j] = make_uint2((uint32_t)t, j | lane_mode[q]);
        }
        run += ni[q];
    }
    if (tid == 0) *item_count = total < max_items ? total : max_items;
}

// ---------------------------------------------------------------------------
// PARTITION strategy, pass B: LDS sub-histogram per work item
//   item = (tile t, slice j of n_t of the chunk range).  Tiles whose runs are
//   short on average (cold tiles) walk chunks one LANE per chunk so a wave
//   covers 64 chunks per step; hot tiles walk one WAVE per chunk run with
//   16-byte loads (8 events per lane).
// ---------------------------------------------------------------------------
template <int TILE_BITS>
__global__ __launch_bounds__(kTileThreads) void k_tile_accumulate(
    const uint16_t *__restrict__ payload, const uint32_t *__restrict__ starts, int n_tiles,
    long long n_chunks, const uint2 *__restrict__ items, const uint32_t *__restrict__ item_count,
    const uint32_t *__restrict__ tile_items, uint32_t *__restrict__ hist, long long n_bins) {
    constexpr int TB = 1 << TILE_BITS;
    __shared__ __attribute__((aligned(16))) uint32_t s_tile[TB];
    if (blockIdx.x >= *item_count) return;
    const uint2 it = items[blockIdx.x];
    const int t = (int)it.x;
    const bool lane_mode = (it.y & 0x80000000u) != 0;
    const long long j = it.y & 0x7fffffffu;
    const long long nt = tile_items[t];
    const long long c0 = j * n_chunks / nt;
    const long long c1 = (j + 1) * n_chunks / nt;
    for (int i = threadIdx.x * 4; i < TB; i += kTileThreads * 4)
        *reinterpret_cast<uint4 *>(s_tile + i) = make_uint4(0, 0, 0, 0);
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    constexpr int NW = kTileThreads / 64;
    const long long stride = (long long)(n_tiles + 1);
    if (lane_mode) {
        // one lane per chunk run; each lane reads its run with aligned 16-byte
        // loads (8 entries), masking entries outside [s, e)
        long long g = c0 + (long long)wid * 64;
        uint32_t ns = 0, ne = 0;
        if (g + lane < c1) {
            ns = starts[(g + lane) * stride + t];
            ne = starts[(g + lane) * stride + t + 1];
        }
        for (; g < c1; g += (long long)NW * 64) {
            const long long c = g + lane;
            const uint32_t s = ns, e = ne;
            const long long gn = g + (long long)NW * 64;  // prefetch the next group's run bounds
            ns = ne = 0;
            if (gn + lane < c1) {
                ns = starts[(gn + lane) * stride + t];
                ne = starts[(gn + lane) * stride + t + 1];
            }
            const uint16_t *p = payload + c * kChunk;
            for (uint32_t i = s & ~7u;; i += 16u) {
                if (!__any(i < e)) break;
                uint4 v0 = make_uint4(0, 0, 0, 0), v1 = make_uint4(0, 0, 0, 0);
                if (i < e) v0 = *reinterpret_cast<const uint4 *>(p + i);
                if (i + 8u < e) v1 = *reinterpret_cast<const uint4 *>(p + i + 8u);
                const uint32_t w[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
#pragma unroll
                for (int q = 0; q < 16; ++q) {
                    const uint32_t k = i + (uint32_t)q;
                    if (k >= s && k < e) atomicAdd(&s_tile[(w[q >> 1] >> ((q & 1) * 16)) & 0xFFFFu], 1u);
                }
            }
        }
    } else {
        for (long long c = c0 + wid; c < c1; c += NW) {
            const uint32_t s = starts[c * stride + t];
            const uint32_t e = starts[c * stride + t + 1];
            const uint16_t *p = payload + c * kChunk;
            const uint32_t a0 = (s + 7u) & ~7u;  // 16-byte aligned body [a0, a1)
            const uint32_t a1 = e & ~7u;
            if (a0 >= a1) {
                for (uint32_t i = s + lane; i < e; i += 64) atomicAdd(&s_tile[p[i]], 1u);
                continue;
            }
            if (s + lane < a0) atomicAdd(&s_tile[p[s + lane]], 1u);
            if (a1 + lane < e) atomicAdd(&s_tile[p[a1 + lane]], 1u);
            for (uint32_t i = a0 + lane * 8u; i < a1; i += 512u) {
                const uint4 v = *reinterpret_cast<const uint4 *>(p + i);
                atomicAdd(&s_tile[v.x & 0xFFFFu], 1u);
                atomicAdd(&s_tile[v.x >> 16], 1u);
                atomicAdd(&s_tile[v.y & 0xFFFFu], 1u);
                atomicAdd(&s_tile[v.y >> 16], 1u);
                atomicAdd(&s_tile[v.z & 0xFFFFu], 1u);
                atomicAdd(&s_tile[v.z >> 16], 1u);
                atomicAdd(&s_tile[v.w & 0xFFFFu], 1u);
                atomicAdd(&s_tile[v.w >> 16], 1u);
            }
        }
    }
    __syncthreads();
    const long long base = (long long)t << TILE_BITS;
    for (int i = threadIdx.x; i < TB; i += kTileThreads) {
        const uint32_t v = s_tile[i];
        if (v != 0u && base + i < n_bins) atomicAdd(hist + base + i, v);
    }
}

// ---------------------------------------------------------------------------
// Monitor: 1-D TOA histogram, LDS layout [bin][32 columns] so the 32 lanes of
// each half-wave always hit 32 distinct banks (conflict-free for any skew).
// ---------------------------------------------------------------------------
// PF: the next iteration's U groups are loaded before this one's are binned
// (twice the bytes in flight per lane)
template <bool FAST, bool COLUMNS>
__global__ __launch_bounds__(256) void k_monitor(const SegKarg segs, int n_segs,
                                                 const unsigned char *__restrict__ g_tab,
                                                 ToaParams tp, uint32_t *__restrict__ hist) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    uint32_t *s_h = reinterpret_cast<uint32_t *>(smem);
    const int HB = COLUMNS ? tp.T * 32 : tp.T;
    unsigned char *s_tab = smem + align16((size_t)(HB + 64) * 4);
    load_toa_tables(s_tab, g_tab, tp);
    for (int i = threadIdx.x; i < HB + 64; i += blockDim.x) s_h[i] = 0;
    __syncthreads();
    const int col = threadIdx.x & 31;
    const uint32_t dummy = (uint32_t)HB + (threadIdx.x & 63u);  // dropped events count here
    // branch-free: every event adds 1 to its bin's counter or to the lane's
    // dummy word, so no lane waits inside a branch around its LDS atomic
    auto add = [&](int t, bool valid) __attribute__((always_inline)) {
        const int b = FAST ? toa_bin_nb(t, s_tab, tp) : toa_bin<false>(t, s_tab, tp);
        const uint32_t k = (valid && b >= 0) ? (COLUMNS ? (uint32_t)b * 32u + (uint32_t)col : (uint32_t)b) : dummy;
        atomicAdd(&s_h[k], 1u);
    };
    // up to kKargSegs messages per launch, their descriptors passed as kernel
    // arguments (no descriptor upload in front); per lane U groups of four
    // events in flight (indices clamped, so the loads are unconditional).
    // Block ranges (host: every message at least a block; chunk0 = its first
    // block): each block streams one message with that message's own stride,
    // so no lane sweeps a message's partial last stride and moves on.
    // U = 8 (32 events per lane in flight): 102.6 -> 100.4 us on the monitor
    // bench against U = 4; U = 16 (109-128 VGPRs) 111 us
    constexpr int U = 8;
    int si = 0;
    for (int j = 1; j < n_segs; ++j)
        if ((long long)blockIdx.x >= segs.s[j].chunk0) si = j;
    const long long b0 = segs.s[si].chunk0;
    const long long b1 = si + 1 < n_segs ? segs.s[si + 1].chunk0 : (long long)gridDim.x;
    const SegDesc seg = segs.s[si];
    const long long n = seg.n;
    const long long stride = (b1 - b0) * blockDim.x;
    const long long i0 = ((long long)blockIdx.x - b0) * blockDim.x + threadIdx.x;
    long long tail = 0;
    if (((uintptr_t)seg.toa & 15u) == 0 && n >= 4) {
        const long long n4 = n >> 2;
        for (long long i = i0; i < n4; i += stride * U) {
            v4i t[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const long long k = i + u * stride;
                t[u] = ld_stream4(seg.toa + 4 * (k < n4 ? k : n4 - 1));
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const bool ok = i + u * stride < n4;
#pragma unroll
                for (int q = 0; q < 4; ++q) add(t[u][q], ok);
            }
        }
        tail = n4 << 2;
    }
    for (long long i = tail + i0; i < n; i += stride) add(ld_global(seg.toa + i), true);
    __syncthreads();
    for (int b = threadIdx.x; b < tp.T; b += blockDim.x) {
        uint32_t v = 0;
        if (COLUMNS) {
            for (int c = 0; c < 32; ++c) v += s_h[b * 32 + ((c + b) & 31)];
        } else {
            v = s_h[b];
        }
        if (v) atomicAdd(hist + b, v);
    }
}

// ---------------------------------------------------------------------------
// launch wrappers
// ---------------------------------------------------------------------------
size_t partition_smem(int n_tiles, const ToaParams &tp) {
    return (size_t)kChunk * 2 + 4 * ((size_t)align4(n_tiles + 1) + align4(n_tiles) + 32) +
           sizeof(SegDesc) * kMaxSegs + toa_lds_bytes(tp);
}

template <typename LT>
static hipError_t launch_bin_atomic_t(const SegKargAtomic &seg, int n_segs, const LT *lut, int pid_off,
                                      unsigned L, const unsigned char *tab, const ToaParams &tp,
                                      uint32_t *hist, int grid, hipStream_t st, hipEvent_t start,
                                      hipEvent_t stop) {
    const size_t sm = toa_lds_bytes(tp);
    if (tp.fast) {
        (void)hipFuncSetAttribute((const void *)k_bin_atomic<LT, true>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)sm);
        hipExtLaunchKernelGGL((k_bin_atomic<LT, true>), dim3(grid), dim3(256), sm, st, start, stop, 0,
                              seg, n_segs, lut, pid_off, L, tab, tp, hist);
    } else {
        (void)hipFuncSetAttribute((const void *)k_bin_atomic<LT, false>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)sm);
        hipExtLaunchKernelGGL((k_bin_atomic<LT, false>), dim3(grid), dim3(256), sm, st, start, stop, 0,
                              seg, n_segs, lut, pid_off, L, tab, tp, hist);
    }
    return hipGetLastError();
}

template <typename LT>
static hipError_t launch_bin_atomic_blocks_t(const SegDesc *blocks, int grid, const LT *lut, int pid_off,
                                             unsigned L, const unsigned char *tab, const ToaParams &tp,
                                             uint32_t *hist, hipStream_t st, hipEvent_t start,
                                             hipEvent_t stop) {
    const size_t sm = toa_lds_bytes(tp);
    if (tp.fast) {
        (void)hipFuncSetAttribute((const void *)k_bin_atomic_blocks<LT, true>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)sm);
        hipExtLaunchKernelGGL((k_bin_atomic_blocks<LT, true>), dim3(grid), dim3(256), sm, st, start, stop, 0,
                              blocks, lut, pid_off, L, tab, tp, hist);
    } else {
        (void)hipFuncSetAttribute((const void *)k_bin_atomic_blocks<LT, false>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)sm);
        hipExtLaunchKernelGGL((k_bin_atomic_blocks<LT, false>), dim3(grid), dim3(256), sm, st, start, stop, 0,
                              blocks, lut, pid_off, L, tab, tp, hist);
    }
    return hipGetLastError();
}

hipError_t launch_bin_atomic_blocks(const SegDesc *blocks, int grid, const void *lut, bool lut16, int pid_off,
                                    unsigned L, const unsigned char *tab, const ToaParams &tp, uint32_t *hist,
                                    hipStream_t st, hipEvent_t start, hipEvent_t stop) {
    if (grid < 1) return hipErrorInvalidValue;
    return lut16 ? launch_bin_atomic_blocks_t(blocks, grid, (const uint16_t *)lut, pid_off, L, tab, tp, hist,
                                              st, start, stop)
                 : launch_bin_atomic_blocks_t(blocks, grid, (const int *)lut, pid_off, L, tab, tp, hist, st,
                                              start, stop);
}

hipError_t launch_bin_atomic(const SegKargAtomic &seg, int n_segs, const void *lut, bool lut16, int pid_off,
                             unsigned L, const unsigned char *tab, const ToaParams &tp,
                             uint32_t *hist, int grid, hipStream_t st, hipEvent_t start,
                             hipEvent_t stop) {
    if (n_segs < 1 || n_segs > kKargSegsAtomic) return hipErrorInvalidValue;
    return lut16 ? launch_bin_atomic_t(seg, n_segs, (const uint16_t *)lut, pid_off, L, tab, tp, hist, grid, st,
                                       start, stop)
                 : launch_bin_atomic_t(seg, n_segs, (const int *)lut, pid_off, L, tab, tp, hist, grid, st,
                                       start, stop);
}

template <int TB, typename LT, bool FAST>
static hipError_t launch_partition_t(const PartitionArgs &a, const LT *lut, hipStream_t st) {
    const size_t sm = partition_smem(a.n_tiles, a.tp);
    (void)hipFuncSetAttribute((const void *)k_partition<TB, LT, FAST>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)sm);
    hipLaunchKernelGGL((k_partition<TB, LT, FAST>), dim3(a.grid), dim3(kPartThreads), sm,
                       st, a.segs, a.n_segs, a.c_begin, a.n_chunks, lut, a.pid_off, a.L, a.tab,
                       a.tp, a.n_tiles, a.payload, a.starts, a.part);
    return hipGetLastError();
}

template <int TB, typename LT>
static hipError_t launch_partition_tl(const PartitionArgs &a, const LT *lut, hipStream_t st) {
    return a.tp.fast ? launch_partition_t<TB, LT, true>(a, lut, st)
                     : launch_partition_t<TB, LT, false>(a, lut, st);
}

template <int TB>
static hipError_t launch_partition_tb(const PartitionArgs &a, hipStream_t st) {
    return a.lut16 ? launch_partition_tl<TB>(a, (const uint16_t *)a.lut, st)
                   : launch_partition_tl<TB>(a, (const int *)a.lut, st);
}

hipError_t launch_partition(const PartitionArgs &a, hipStream_t st) {
    switch (a.tile_bits) {
    case 14: return launch_partition_tb<14>(a, st);
    case 15: return launch_partition_tb<15>(a, st);
    default: return hipErrorInvalidValue;
    }
}

hipError_t launch_plan(const uint32_t *part, int part_rows, int n_tiles, long long n_chunks,
                       uint32_t item_events, uint32_t *totals, uint32_t *tile_items, uint2 *items,
                       uint32_t *item_count, uint32_t max_items, hipStream_t st) {
    hipLaunchKernelGGL(k_tile_totals, dim3(n_tiles), dim3(256), 0, st, part, part_rows, n_tiles,
                       totals);
    hipLaunchKernelGGL(k_plan, dim3(1), dim3(1024), 0, st, totals, n_tiles, n_chunks, item_events,
                       tile_items, items, item_count, max_items);
    return hipGetLastError();
}

hipError_t launch_tile_accumulate(int tile_bits, const uint16_t *payload, const uint32_t *starts,
                                  int n_tiles, long long n_chunks, const uint2 *items,
                                  const uint32_t *item_count, const uint32_t *tile_items,
                                  uint32_t *hist, long long n_bins, int grid, hipStream_t st) {
    switch (tile_bits) {
    case 14:
        hipLaunchKernelGGL(k_tile_accumulate<14>, dim3(grid), dim3(kTileThreads), 0, st, payload,
                           starts, n_tiles, n_chunks, items, item_count, tile_items, hist, n_bins);
        break;
    case 15:
        hipLaunchKernelGGL(k_tile_accumulate<15>, dim3(grid), dim3(kTileThreads), 0, st, payload,
                           starts, n_tiles, n_chunks, items, item_count, tile_items, hist, n_bins);
        break;
    default:
        return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_monitor(const SegKarg &segs, int n_segs, const unsigned char *tab,
                          const ToaParams &tp, uint32_t *hist, int grid, hipStream_t st,
                          hipEvent_t start, hipEvent_t stop) {
    if (n_segs < 1 || n_segs > kKargSegs) return hipErrorInvalidValue;
    const bool columns = tp.T <= kMonitorColumnsMaxT;
    const size_t hb = align16((size_t)((columns ? tp.T * 32 : tp.T) + 64) * 4);
    const size_t sm = hb + toa_lds_bytes(tp);
#define LDE_MON(F, C)                                                                              \
    do {                                                                                           \
        (void)hipFuncSetAttribute((const void *)k_monitor<F, C>,                                   \
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)sm);            \
        hipExtLaunchKernelGGL((k_monitor<F, C>), dim3(grid), dim3(256), sm, st, start, stop, 0, segs, \
                              n_segs, tab, tp, hist);                                              \
    } while (0)
    if (tp.fast && columns) LDE_MON(true, true);
    else if (tp.fast) LDE_MON(true, false);
    else if (columns) LDE_MON(false, true);
    else LDE_MON(false, false);
#undef LDE_MON
    return hipGetLastError();
}

}  // namespace lde
