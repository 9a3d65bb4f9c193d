// lde_kernels.hip -- CDNA4 (gfx950) kernels of the event-binning engine.
//
// Hot path: per event
//   pid -> LUT[replica][pid - pid_offset] (screen*T or -1; folds group_event_data
//          membership, pixel index and projection, group_by_pixel.py:46-54,
//          projectors.py:118-152 / 243-270)
//   toa -> TOA bin under scipp's half-open f64-edge rule (providers.py:205-210)
//   count[screen*T + bin] += 1
//
// Two strategies produce bit-identical integer counts:
//   * ATOMIC    : one pass, one agent-scope u32 atomic per event (small batches).
//   * PARTITION : pass A partitions events into LDS-sized tiles of the (S,T)
//                 histogram (chunk-major, tile-sorted runs, no global atomics),
//                 a 1-block plan kernel splits tiles into balanced work items,
//                 pass B accumulates each item in an LDS sub-histogram and
//                 flushes non-zero bins with coalesced atomics.
// Monitors (S = 1) use a conflict-free per-lane-column LDS histogram.
//
// TOA binning is exact integer arithmetic: for int32 t and f64 edge e,
// t >= e  <=>  t >= ceil(e), so the f64 edges become int64 thresholds on the
// host and a bucket table (uniform buckets of 2^shift ns over the edge span,
// each storing the first/last candidate bin) narrows the search to 0-1 steps
// for the reference's linear and geometric edges.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "lde_internal.h"

namespace lde {

// ---------------------------------------------------------------------------
// TOA lookup helpers
// ---------------------------------------------------------------------------
__device__ __forceinline__ int toa_bin(int t, const long long *__restrict__ s_thr,
                                       const uint32_t *__restrict__ s_bp, const ToaParams &tp) {
    const long long tt = t;
    if (tt < tp.lo || tt >= tp.hi) return -1;
    const unsigned g = (unsigned)((unsigned long long)(tt - tp.lo) >> tp.shift);
    const uint32_t bp = s_bp[g];
    int b = (int)(bp & 0xFFFFu);
    int e = (int)(bp >> 16);
    while (b < e) {  // binary search inside the bucket's candidate range
        const int m = (b + e + 1) >> 1;
        if (tt >= s_thr[m]) b = m; else e = m - 1;
    }
    return b;
}

__device__ __forceinline__ void load_toa_tables(long long *s_thr, uint32_t *s_bp,
                                                const long long *__restrict__ g_thr,
                                                const uint32_t *__restrict__ g_bp,
                                                const ToaParams &tp) {
    for (int i = threadIdx.x; i <= tp.T; i += blockDim.x) s_thr[i] = g_thr[i];
    for (int i = threadIdx.x; i < tp.G; i += blockDim.x) s_bp[i] = g_bp[i];
}

// flat output index (screen*T + bin) of one event, or -1
__device__ __forceinline__ int event_key(int pid, int t, const int *__restrict__ lut,
                                        int pid_off, unsigned L, const long long *s_thr,
                                        const uint32_t *s_bp, const ToaParams &tp) {
    const unsigned p = (unsigned)(pid - pid_off);
    if (p >= L) return -1;
    const int base = lut[p];
    if (base < 0) return -1;
    const int b = toa_bin(t, s_thr, s_bp, tp);
    return b < 0 ? -1 : base + b;
}

// ---------------------------------------------------------------------------
// Block-wide exclusive scan (blockDim multiple of 64, <= 1024)
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t wave_inclusive_scan(uint32_t x) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(x, d, 64);
        if (lane >= d) x += y;
    }
    return x;
}

// returns exclusive prefix of v across the block; *total = block sum.
// s_w must hold >= 17 uint32.  Contains two __syncthreads().
__device__ __forceinline__ uint32_t block_exclusive_scan(uint32_t v, uint32_t *s_w,
                                                         uint32_t *total) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int nw = blockDim.x >> 6;
    const uint32_t inc = wave_inclusive_scan(v);
    if (lane == 63) s_w[wid] = inc;
    __syncthreads();
    if (wid == 0) {
        uint32_t w = lane < nw ? s_w[lane] : 0u;
        const uint32_t wi = wave_inclusive_scan(w);
        if (lane < nw) s_w[lane] = wi - w;
        if (lane == nw - 1) s_w[16] = wi;
    }
    __syncthreads();
    *total = s_w[16];
    return inc - v + s_w[wid];
}

// ---------------------------------------------------------------------------
// ATOMIC strategy: one pass, global u32 atomics (agent scope)
// ---------------------------------------------------------------------------
template <bool VEC>
__global__ __launch_bounds__(256) void k_bin_atomic(const int *__restrict__ pid,
                                                    const int *__restrict__ toa, long long n,
                                                    const int *__restrict__ lut, int pid_off,
                                                    unsigned L, const long long *__restrict__ g_thr,
                                                    const uint32_t *__restrict__ g_bp, ToaParams tp,
                                                    uint32_t *__restrict__ hist) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    long long *s_thr = reinterpret_cast<long long *>(smem);
    uint32_t *s_bp = reinterpret_cast<uint32_t *>(smem + thr_bytes(tp.T));
    load_toa_tables(s_thr, s_bp, g_thr, g_bp, tp);
    __syncthreads();
    const long long stride = (long long)gridDim.x * blockDim.x;
    if (VEC) {
        const long long n4 = n >> 2;
        const int4 *p4 = reinterpret_cast<const int4 *>(pid);
        const int4 *t4 = reinterpret_cast<const int4 *>(toa);
        for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
            const int4 p = p4[i];
            const int4 t = t4[i];
            int k;
            k = event_key(p.x, t.x, lut, pid_off, L, s_thr, s_bp, tp); if (k >= 0) atomicAdd(hist + k, 1u);
            k = event_key(p.y, t.y, lut, pid_off, L, s_thr, s_bp, tp); if (k >= 0) atomicAdd(hist + k, 1u);
            k = event_key(p.z, t.z, lut, pid_off, L, s_thr, s_bp, tp); if (k >= 0) atomicAdd(hist + k, 1u);
            k = event_key(p.w, t.w, lut, pid_off, L, s_thr, s_bp, tp); if (k >= 0) atomicAdd(hist + k, 1u);
        }
        for (long long i = (n4 << 2) + (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
             i += stride) {
            const int k = event_key(pid[i], toa[i], lut, pid_off, L, s_thr, s_bp, tp);
            if (k >= 0) atomicAdd(hist + k, 1u);
        }
    } else {
        for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
            const int k = event_key(pid[i], toa[i], lut, pid_off, L, s_thr, s_bp, tp);
            if (k >= 0) atomicAdd(hist + k, 1u);
        }
    }
}

// ---------------------------------------------------------------------------
// PARTITION strategy, pass A: chunk-major tile partition
//   chunk c covers events [c*CH, (c+1)*CH) of the segment; its valid events are
//   written tile-sorted to payload[(chunk0+c)*CH ...] as u16 offsets inside the
//   tile, with per-tile run starts starts[(chunk0+c)*(NT+1) + t].
// ---------------------------------------------------------------------------
template <int TILE_BITS, bool VEC>
__global__ __launch_bounds__(kPartThreads) void k_partition(
    const int *__restrict__ pid, const int *__restrict__ toa, long long n,
    const int *__restrict__ lut, int pid_off, unsigned L, const long long *__restrict__ g_thr,
    const uint32_t *__restrict__ g_bp, ToaParams tp, int n_tiles, long long chunk0,
    long long n_chunks, uint16_t *__restrict__ payload, uint32_t *__restrict__ starts,
    uint32_t *__restrict__ part) {
    constexpr int EPT = kPartEventsPerThread;  // 16 events per thread
    constexpr int CH = kChunk;                 // 16384 events per chunk
    constexpr uint32_t MASK = (1u << TILE_BITS) - 1u;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    // LDS carve: staging | counts | totals | scan | thresholds | buckets
    uint16_t *s_stg = reinterpret_cast<uint16_t *>(smem);
    uint32_t *s_cnt = reinterpret_cast<uint32_t *>(smem + CH * 2);
    uint32_t *s_tot = s_cnt + align4(n_tiles + 1);
    uint32_t *s_w = s_tot + align4(n_tiles);
    long long *s_thr = reinterpret_cast<long long *>(s_w + 32);
    uint32_t *s_bp = reinterpret_cast<uint32_t *>(reinterpret_cast<unsigned char *>(s_thr) +
                                                  thr_bytes(tp.T));
    load_toa_tables(s_thr, s_bp, g_thr, g_bp, tp);
    for (int i = threadIdx.x; i <= n_tiles; i += blockDim.x) s_cnt[i] = 0;
    for (int i = threadIdx.x; i < n_tiles; i += blockDim.x) s_tot[i] = 0;
    __syncthreads();

    const int tid = threadIdx.x;
    for (long long c = blockIdx.x; c < n_chunks; c += gridDim.x) {
        const long long base = c * CH;
        int key[EPT];
        uint32_t rank[EPT];
        // ---- load 16 events per thread: 4 x (int4 pid, int4 toa), coalesced
#pragma unroll
        for (int j = 0; j < EPT / 4; ++j) {
            const long long e0 = base + ((long long)j * kPartThreads + tid) * 4;
            int pv[4], tv[4];
            if (VEC && e0 + 3 < n) {
                const int4 p = *reinterpret_cast<const int4 *>(pid + e0);
                const int4 t = *reinterpret_cast<const int4 *>(toa + e0);
                pv[0] = p.x; pv[1] = p.y; pv[2] = p.z; pv[3] = p.w;
                tv[0] = t.x; tv[1] = t.y; tv[2] = t.z; tv[3] = t.w;
            } else {
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const bool ok = e0 + q < n;
                    pv[q] = ok ? pid[e0 + q] : pid_off - 1;  // out-of-LUT id -> dropped
                    tv[q] = ok ? toa[e0 + q] : 0;
                }
            }
#pragma unroll
            for (int q = 0; q < 4; ++q)
                key[j * 4 + q] = event_key(pv[q], tv[q], lut, pid_off, L, s_thr, s_bp, tp);
        }
        // ---- rank inside tile (LDS returning atomics)
#pragma unroll
        for (int e = 0; e < EPT; ++e) {
            rank[e] = 0;
            if (key[e] >= 0) rank[e] = atomicAdd(&s_cnt[key[e] >> TILE_BITS], 1u);
        }
        __syncthreads();
        // ---- exclusive scan of tile counts (<= 4 tiles per thread)
        uint32_t loc[kMaxTilesPerThread];
        uint32_t sum = 0;
        const int t0 = tid * kMaxTilesPerThread;
#pragma unroll
        for (int q = 0; q < kMaxTilesPerThread; ++q) {
            const int t = t0 + q;
            loc[q] = t < n_tiles ? s_cnt[t] : 0u;
            sum += loc[q];
        }
        uint32_t total;
        uint32_t run = block_exclusive_scan(sum, s_w, &total);
        uint32_t *g_starts = starts + (chunk0 + c) * (long long)(n_tiles + 1);
#pragma unroll
        for (int q = 0; q < kMaxTilesPerThread; ++q) {
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
#pragma unroll
        for (int e = 0; e < EPT; ++e)
            if (key[e] >= 0) s_stg[s_cnt[key[e] >> TILE_BITS] + rank[e]] = (uint16_t)(key[e] & MASK);
        __syncthreads();
        // ---- coalesced write-out of the valid prefix (16 B per lane)
        uint16_t *g_out = payload + (chunk0 + c) * (long long)CH;
        for (int i = tid * 8; i < (int)total; i += kPartThreads * 8)
            *reinterpret_cast<uint4 *>(g_out + i) = *reinterpret_cast<const uint4 *>(s_stg + i);
        for (int i = tid; i <= n_tiles; i += blockDim.x) s_cnt[i] = 0;
        __syncthreads();
    }
    // per-block tile totals (row blockIdx.x owned by this block; accumulates
    // across segment launches on the same stream)
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
                                               uint32_t item_events,
                                               uint32_t *__restrict__ tile_items,
                                               uint2 *__restrict__ items,
                                               uint32_t *__restrict__ item_count,
                                               uint32_t max_items) {
    __shared__ uint32_t s_w[32];
    const int tid = threadIdx.x;
    uint32_t ni[kMaxTilesPerThread];
    uint32_t sum = 0;
    const int t0 = tid * kMaxTilesPerThread;
#pragma unroll
    for (int q = 0; q < kMaxTilesPerThread; ++q) {
        const int t = t0 + q;
        const uint32_t tot = t < n_tiles ? totals[t] : 0u;
        ni[q] = tot == 0 ? 0u : (tot + item_events - 1) / item_events;
        sum += ni[q];
    }
    uint32_t total;
    uint32_t run = block_exclusive_scan(sum, s_w, &total);
#pragma unroll
    for (int q = 0; q < kMaxTilesPerThread; ++q) {
        const int t = t0 + q;
        if (t < n_tiles) {
            tile_items[t] = ni[q];
            for (uint32_t j = 0; j < ni[q] && run + j < max_items; ++j)
                items[run + j] = make_uint2((uint32_t)t, j);
        }
        run += ni[q];
    }
    if (tid == 0) *item_count = total < max_items ? total : max_items;
}

// ---------------------------------------------------------------------------
// PARTITION strategy, pass B: LDS sub-histogram per work item
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
    const long long j = it.y;
    const long long nt = tile_items[t];
    const long long c0 = j * n_chunks / nt;
    const long long c1 = (j + 1) * n_chunks / nt;
    for (int i = threadIdx.x * 4; i < TB; i += kTileThreads * 4)
        *reinterpret_cast<uint4 *>(s_tile + i) = make_uint4(0, 0, 0, 0);
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    constexpr int NW = kTileThreads / 64;
    constexpr int U = 4;  // chunks in flight per wave
    const long long stride = (long long)(n_tiles + 1);
    for (long long c = c0 + wid; c < c1; c += (long long)NW * U) {
        uint32_t s[U], e[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long long cc = c + (long long)u * NW;
            if (cc < c1) {
                s[u] = starts[cc * stride + t];
                e[u] = starts[cc * stride + t + 1];
            } else {
                s[u] = e[u] = 0;
            }
        }
        uint16_t v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long long cc = c + (long long)u * NW;
            const uint32_t i = s[u] + lane;
            v[u] = i < e[u] ? payload[cc * kChunk + i] : (uint16_t)0;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (s[u] + lane < e[u]) atomicAdd(&s_tile[v[u]], 1u);
        }
        // long runs (> 64 events): finish them
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long long cc = c + (long long)u * NW;
            for (uint32_t i = s[u] + 64 + lane; i < e[u]; i += 64)
                atomicAdd(&s_tile[payload[cc * kChunk + i]], 1u);
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
template <bool VEC, bool COLUMNS>
__global__ __launch_bounds__(256) void k_monitor(const int *__restrict__ toa, long long n,
                                                 const long long *__restrict__ g_thr,
                                                 const uint32_t *__restrict__ g_bp, ToaParams tp,
                                                 uint32_t *__restrict__ hist) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    uint32_t *s_h = reinterpret_cast<uint32_t *>(smem);
    const int HB = COLUMNS ? tp.T * 32 : tp.T;
    long long *s_thr = reinterpret_cast<long long *>(smem + align16((size_t)HB * 4));
    uint32_t *s_bp = reinterpret_cast<uint32_t *>(reinterpret_cast<unsigned char *>(s_thr) +
                                                  thr_bytes(tp.T));
    load_toa_tables(s_thr, s_bp, g_thr, g_bp, tp);
    for (int i = threadIdx.x; i < HB; i += blockDim.x) s_h[i] = 0;
    __syncthreads();
    const int col = threadIdx.x & 31;
    const long long stride = (long long)gridDim.x * blockDim.x;
    auto add = [&](int t) {
        const int b = toa_bin(t, s_thr, s_bp, tp);
        if (b >= 0) atomicAdd(&s_h[COLUMNS ? b * 32 + col : b], 1u);
    };
    if (VEC) {
        const long long n4 = n >> 2;
        const int4 *t4 = reinterpret_cast<const int4 *>(toa);
        for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
            const int4 t = t4[i];
            add(t.x); add(t.y); add(t.z); add(t.w);
        }
        for (long long i = (n4 << 2) + (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
             i += stride)
            add(toa[i]);
    } else {
        for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
            add(toa[i]);
    }
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
// Window / cumulative maintenance
// ---------------------------------------------------------------------------
// win64 += win32; win32 = 0   (u32 overflow guard, only for huge windows)
__global__ void k_fold_window(uint32_t *__restrict__ win32, unsigned long long *__restrict__ win64,
                              long long n) {
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (long long)gridDim.x * blockDim.x) {
        win64[i] += win32[i];
        win32[i] = 0;
    }
}

// f32 mode (BIFROST): per accumulate, mirror the reference's per-push f32 adds:
// window_f32 += f32(batch), cumulative_f32 += f32(batch); then fold the batch
// into the integer window.
__global__ void k_merge_f32(uint32_t *__restrict__ batch, unsigned long long *__restrict__ win64,
                            float *__restrict__ winf, float *__restrict__ cumf, long long n,
                            int first_win, int first_cum) {
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (long long)gridDim.x * blockDim.x) {
        const uint32_t b = batch[i];
        const float fb = (float)b;
        winf[i] = first_win ? fb : winf[i] + fb;
        cumf[i] = first_cum ? fb : cumf[i] + fb;
        win64[i] += b;
        batch[i] = 0;
    }
}

// snapshot: out = a (+ b) (+ c) as u64, for reads that must not finalize
__global__ void k_sum3(const unsigned long long *__restrict__ a, const unsigned long long *__restrict__ b,
                       const uint32_t *__restrict__ c, unsigned long long *__restrict__ out,
                       long long n) {
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (long long)gridDim.x * blockDim.x) {
        unsigned long long v = c[i];
        if (a) v += a[i];
        if (b) v += b[i];
        out[i] = v;
    }
}

// Finalize (f64/integer mode): w = win64 + win32; cum += w; row sums over the
// TOA range; totals.  One wave per screen row.
template <typename OUT>
__global__ __launch_bounds__(256) void k_finalize(uint32_t *__restrict__ win32,
                                                  unsigned long long *__restrict__ win64,
                                                  unsigned long long *__restrict__ cum,
                                                  unsigned long long *__restrict__ snap,
                                                  long long S, int T, int lo, int hi,
                                                  OUT *__restrict__ cur_img,
                                                  OUT *__restrict__ cum_img,
                                                  unsigned long long *__restrict__ totals) {
    __shared__ unsigned long long s_tot[4][4];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    unsigned long long acc[4] = {0, 0, 0, 0};
    for (long long s = (long long)blockIdx.x * 4 + wid; s < S; s += (long long)gridDim.x * 4) {
        unsigned long long rw = 0, rc = 0, tw = 0, tc = 0;
        for (int i = lane; i < T; i += 64) {
            const long long k = s * T + i;
            unsigned long long w = win32[k];
            if (win64) {
                w += win64[k];
                win64[k] = 0;
            }
            const unsigned long long c = cum[k] + w;
            cum[k] = c;
            if (snap) snap[k] = w;
            win32[k] = 0;
            tw += w;
            tc += c;
            if (i >= lo && i < hi) {
                rw += w;
                rc += c;
            }
        }
#pragma unroll
        for (int d = 32; d > 0; d >>= 1) {
            rw += __shfl_xor(rw, d, 64);
            rc += __shfl_xor(rc, d, 64);
            tw += __shfl_xor(tw, d, 64);
            tc += __shfl_xor(tc, d, 64);
        }
        if (lane == 0) {
            if (cur_img) cur_img[s] = (OUT)rw;
            if (cum_img) cum_img[s] = (OUT)rc;
            acc[0] += tw;
            acc[1] += rw;
            acc[2] += tc;
            acc[3] += rc;
        }
    }
    if (lane == 0)
        for (int q = 0; q < 4; ++q) s_tot[wid][q] = acc[q];
    __syncthreads();
    if (threadIdx.x < 4) {
        const unsigned long long v = s_tot[0][threadIdx.x] + s_tot[1][threadIdx.x] +
                                     s_tot[2][threadIdx.x] + s_tot[3][threadIdx.x];
        if (v) atomicAdd(totals + threadIdx.x, v);
    }
}

// f32-mode image rows: sum of f32 values over the TOA range in f64, rounded once
__global__ __launch_bounds__(256) void k_rows_f32(const float *__restrict__ h, long long S, int T,
                                                  int lo, int hi, float *__restrict__ img) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    for (long long s = (long long)blockIdx.x * 4 + wid; s < S; s += (long long)gridDim.x * 4) {
        double r = 0.0;
        for (int i = lane + lo; i < hi; i += 64) r += (double)h[s * T + i];
#pragma unroll
        for (int d = 32; d > 0; d >>= 1) r += __shfl_xor(r, d, 64);
        if (lane == 0) img[s] = (float)r;
    }
}

// ---------------------------------------------------------------------------
// host-side launch wrappers
// ---------------------------------------------------------------------------
size_t partition_smem(int n_tiles, const ToaParams &tp) {
    return (size_t)kChunk * 2 + 4 * ((size_t)align4(n_tiles + 1) + align4(n_tiles) + 32) +
           thr_bytes(tp.T) + (size_t)tp.G * 4;
}

hipError_t launch_bin_atomic(const int *pid, const int *toa, long long n, const int *lut,
                             int pid_off, unsigned L, const long long *thr, const uint32_t *bp,
                             const ToaParams &tp, uint32_t *hist, bool vec, int grid,
                             hipStream_t st) {
    const size_t sm = thr_bytes(tp.T) + (size_t)tp.G * 4;
    if (vec)
        hipLaunchKernelGGL(k_bin_atomic<true>, dim3(grid), dim3(256), sm, st, pid, toa, n, lut,
                           pid_off, L, thr, bp, tp, hist);
    else
        hipLaunchKernelGGL(k_bin_atomic<false>, dim3(grid), dim3(256), sm, st, pid, toa, n, lut,
                           pid_off, L, thr, bp, tp, hist);
    return hipGetLastError();
}

template <int TB>
static hipError_t launch_partition_t(const int *pid, const int *toa, long long n, const int *lut,
                                     int pid_off, unsigned L, const long long *thr,
                                     const uint32_t *bp, const ToaParams &tp, int n_tiles,
                                     long long chunk0, long long n_chunks, uint16_t *payload,
                                     uint32_t *starts, uint32_t *part, bool vec, int grid,
                                     hipStream_t st) {
    const size_t sm = partition_smem(n_tiles, tp);
    if (vec) {
        (void)hipFuncSetAttribute((const void *)k_partition<TB, true>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)sm);
        hipLaunchKernelGGL((k_partition<TB, true>), dim3(grid), dim3(kPartThreads), sm, st, pid,
                           toa, n, lut, pid_off, L, thr, bp, tp, n_tiles, chunk0, n_chunks,
                           payload, starts, part);
    } else {
        (void)hipFuncSetAttribute((const void *)k_partition<TB, false>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)sm);
        hipLaunchKernelGGL((k_partition<TB, false>), dim3(grid), dim3(kPartThreads), sm, st, pid,
                           toa, n, lut, pid_off, L, thr, bp, tp, n_tiles, chunk0, n_chunks,
                           payload, starts, part);
    }
    return hipGetLastError();
}

hipError_t launch_partition(int tile_bits, const int *pid, const int *toa, long long n,
                            const int *lut, int pid_off, unsigned L, const long long *thr,
                            const uint32_t *bp, const ToaParams &tp, int n_tiles, long long chunk0,
                            long long n_chunks, uint16_t *payload, uint32_t *starts,
                            uint32_t *part, bool vec, int grid, hipStream_t st) {
    switch (tile_bits) {
    case 13:
        return launch_partition_t<13>(pid, toa, n, lut, pid_off, L, thr, bp, tp, n_tiles, chunk0,
                                      n_chunks, payload, starts, part, vec, grid, st);
    case 14:
        return launch_partition_t<14>(pid, toa, n, lut, pid_off, L, thr, bp, tp, n_tiles, chunk0,
                                      n_chunks, payload, starts, part, vec, grid, st);
    case 15:
        return launch_partition_t<15>(pid, toa, n, lut, pid_off, L, thr, bp, tp, n_tiles, chunk0,
                                      n_chunks, payload, starts, part, vec, grid, st);
    default:
        return hipErrorInvalidValue;
    }
}

hipError_t launch_plan(const uint32_t *part, int part_rows, int n_tiles, uint32_t item_events,
                       uint32_t *totals, uint32_t *tile_items, uint2 *items,
                       uint32_t *item_count, uint32_t max_items, hipStream_t st) {
    hipLaunchKernelGGL(k_tile_totals, dim3(n_tiles), dim3(256), 0, st, part, part_rows, n_tiles,
                       totals);
    hipLaunchKernelGGL(k_plan, dim3(1), dim3(1024), 0, st, totals, n_tiles, item_events,
                       tile_items, items, item_count, max_items);
    return hipGetLastError();
}

hipError_t launch_tile_accumulate(int tile_bits, const uint16_t *payload, const uint32_t *starts,
                                  int n_tiles, long long n_chunks, const uint2 *items,
                                  const uint32_t *item_count, const uint32_t *tile_items,
                                  uint32_t *hist, long long n_bins, int grid, hipStream_t st) {
    switch (tile_bits) {
    case 13:
        hipLaunchKernelGGL(k_tile_accumulate<13>, dim3(grid), dim3(kTileThreads), 0, st, payload,
                           starts, n_tiles, n_chunks, items, item_count, tile_items, hist, n_bins);
        break;
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

hipError_t launch_monitor(const int *toa, long long n, const long long *thr, const uint32_t *bp,
                          const ToaParams &tp, uint32_t *hist, bool vec, int grid,
                          hipStream_t st) {
    const bool columns = tp.T <= kMonitorColumnsMaxT;
    const size_t hb = align16((size_t)(columns ? tp.T * 32 : tp.T) * 4);
    const size_t sm = hb + thr_bytes(tp.T) + (size_t)tp.G * 4;
#define LDE_MON(V, C)                                                                         \
    do {                                                                                      \
        (void)hipFuncSetAttribute((const void *)k_monitor<V, C>,                                    \
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)sm);             \
        hipLaunchKernelGGL((k_monitor<V, C>), dim3(grid), dim3(256), sm, st, toa, n, thr, bp, \
                           tp, hist);                                                         \
    } while (0)
    if (vec && columns) LDE_MON(true, true);
    else if (vec) LDE_MON(true, false);
    else if (columns) LDE_MON(false, true);
    else LDE_MON(false, false);
#undef LDE_MON
    return hipGetLastError();
}

hipError_t launch_fold_window(uint32_t *win32, unsigned long long *win64, long long n,
                              hipStream_t st) {
    hipLaunchKernelGGL(k_fold_window, dim3(grid_for(n)), dim3(256), 0, st, win32, win64, n);
    return hipGetLastError();
}

hipError_t launch_merge_f32(uint32_t *batch, unsigned long long *win64, float *winf, float *cumf,
                            long long n, int first_win, int first_cum, hipStream_t st) {
    hipLaunchKernelGGL(k_merge_f32, dim3(grid_for(n)), dim3(256), 0, st, batch, win64, winf, cumf,
                       n, first_win, first_cum);
    return hipGetLastError();
}

hipError_t launch_sum3(const unsigned long long *a, const unsigned long long *b, const uint32_t *c,
                       unsigned long long *out, long long n, hipStream_t st) {
    hipLaunchKernelGGL(k_sum3, dim3(grid_for(n)), dim3(256), 0, st, a, b, c, out, n);
    return hipGetLastError();
}

hipError_t launch_finalize(bool f32_images, uint32_t *win32, unsigned long long *win64,
                           unsigned long long *cum, unsigned long long *snap, long long S, int T,
                           int lo, int hi, void *cur_img, void *cum_img,
                           unsigned long long *totals, hipStream_t st) {
    long long blocks = (S + 3) / 4;
    if (blocks > 2048) blocks = 2048;
    if (blocks < 1) blocks = 1;
    if (f32_images)
        hipLaunchKernelGGL(k_finalize<float>, dim3((unsigned)blocks), dim3(256), 0, st, win32,
                           win64, cum, snap, S, T, lo, hi, (float *)cur_img, (float *)cum_img,
                           totals);
    else
        hipLaunchKernelGGL(k_finalize<double>, dim3((unsigned)blocks), dim3(256), 0, st, win32,
                           win64, cum, snap, S, T, lo, hi, (double *)cur_img, (double *)cum_img,
                           totals);
    return hipGetLastError();
}

hipError_t launch_rows_f32(const float *h, long long S, int T, int lo, int hi, float *img,
                           hipStream_t st) {
    long long blocks = (S + 3) / 4;
    if (blocks > 2048) blocks = 2048;
    if (blocks < 1) blocks = 1;
    hipLaunchKernelGGL(k_rows_f32, dim3((unsigned)blocks), dim3(256), 0, st, h, S, T, lo, hi, img);
    return hipGetLastError();
}

}  // namespace lde
