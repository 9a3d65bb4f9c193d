// lde_coord.hip -- wavelength-mode event coordinate.
//
// In wavelength mode the detector view histograms a per-event coordinate
// computed from the pixel's flight path and the event's time of arrival
// through a lookup table (SRC/workflows/detector_view/factory.py:134-169:
// 'wavelength' mode, GenericUnwrapWorkflow's table; providers.py:77-95), then
// bins it against float64 edges with scipp's half-open rule.
//
// Restated interpolation (bilinear on a regular (distance, time) grid, the
// RegularGridInterpolator 'linear' form; NaN or outside the grid -> dropped):
//   x = (d - d0) * inv_dd,  i = min(floor(x), nd - 2),  fx = x - i   (dropped unless 0 <= x <= nd - 1)
//   y = (t - t0) * inv_dt,  j = min(floor(y), nt - 2),  fy = y - j   (dropped unless 0 <= y <= nt - 1)
//   a = v[i][j] + fy * (v[i][j+1] - v[i][j]);  b = v[i+1][j] + fy * (v[i+1][j+1] - v[i+1][j])
//   c = a + fx * (b - a)
// evaluated in float64 without contraction (no FMA), so the CPU oracle's
// numpy restatement gives the same bits.  The kernel writes the coordinate's
// bin index (or -1) as an int32 "time" per event; the engine then bins
// (pid, bin) with its usual strategies against the integer edges 0..T, so every
// strategy and skew path is reused bit for bit.
//
// Per event: the pid and TOA streams, one 8-byte gather of the pixel's
// distance (the only random access), the table in LDS when it fits (4 LDS
// reads), and the bin from a bucket table over the edges (a start candidate,
// then a few compares with the edges in LDS: exact for any sorted edges,
// however the bucket arithmetic rounds).
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "lde_device.h"
#include "lde_internal.h"

#pragma clang fp contract(off)

namespace lde {

// largest b with e[b] <= v < e[b + 1] (half-open, last bin too; NaN dropped)
// FIXED: the host checked that every bucket's candidate lies within [-1, +2]
// of the true bin for any value whose bucket index rounds to it (buckets at
// most half the narrowest bin wide), so one step down and two up, without
// branches, give the loop's answer and the events of a lane interleave
template <bool FIXED = false>
__device__ __forceinline__ int coord_bin(double v, const double *e, const uint16_t *bk, int T,
                                         double e0, double inv_w, int G) {
    if (!(v >= e[0]) || !(v < e[T])) return -1;
    int g = (int)((v - e0) * inv_w);
    g = g < 0 ? 0 : (g >= G ? G - 1 : g);
    int b = bk[g];
    if (FIXED) {
        // true bin in [b - 1, b + 2]: below b iff v < e[b] (b > 0; at b = 0
        // v >= e[0] holds), else b plus the edges e[b + 1], e[b + 2] <= v;
        // the three reads are independent (e[T + 1] = +inf pads the table)
        const double lo = e[b], h1 = e[b + 1], h2 = e[b + 2];
        return b - ((v < lo) ? 1 : 0) + ((v >= h1) ? 1 : 0) + ((v >= h2) ? 1 : 0);
    }
    while (b > 0 && v < e[b]) --b;
    while (v >= e[b + 1]) ++b;
    return b;
}

// coord_bin<true> with the outer edges held in registers (e_first = e[0],
// e_last = e[T]): two LDS reads fewer per event
__device__ __forceinline__ int coord_bin_fast(double v, const double *e, const uint16_t *bk, double e_first,
                                              double e_last, double e0, double inv_w, int G) {
    if (!(v >= e_first) || !(v < e_last)) return -1;
    int g = (int)((v - e0) * inv_w);
    g = g < 0 ? 0 : (g >= G ? G - 1 : g);
    const int b = bk[g];
    const double lo = e[b], h1 = e[b + 1], h2 = e[b + 2];
    return b - ((v < lo) ? 1 : 0) + ((v >= h1) ? 1 : 0) + ((v >= h2) ? 1 : 0);
}

typedef unsigned int v4u __attribute__((ext_vector_type(4)));
typedef unsigned int v3u __attribute__((ext_vector_type(3)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t coord_rsrc(const void *p, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), (short)0, (int)bytes,
                                             (int)0x00020000);  // raw buffer, 32-bit format
}

template <bool TLDS, bool ELDS>
__global__ __launch_bounds__(256) void k_event_coord(CoordArgs a, const int *__restrict__ pid,
                                                     const int *__restrict__ toa, long long n,
                                                     int *__restrict__ out) {
    extern __shared__ double sm[];
    // LDS: edges (T + 1, when they fit) | table (TLDS) | bucket table (u16)
    double *s_e = sm;
    const int ne = ELDS ? a.T + 1 : 0;
    double *s_t = s_e + ((ne + 1) & ~1);
    const int ntab = TLDS ? a.nd * a.nt : 0;
    uint16_t *s_b = reinterpret_cast<uint16_t *>(s_t + ntab);
    if (ne) lds_fill<2>(s_e, ne, [&](int i) { return g_ld(a.edges + i); });
    if (ntab) lds_fill<4>(s_t, ntab, [&](int i) { return g_ld(a.table + i); });
    if (a.G) lds_fill<4>(s_b, a.G, [&](int i) { return g_ld(a.buckets + i); });
    __syncthreads();
    // compile-time LDS or global: a runtime choice makes every edge read a
    // flat load (counted by both vmcnt and lgkmcnt)
    const double *e = ELDS ? s_e : a.edges;
    const double *tab = TLDS ? s_t : a.table;
    const double xmax = (double)(a.nd - 1), ymax = (double)(a.nt - 1);
    // one event: its pixel's distance d (NaN: none) and time t -> bin or -1
    auto coord = [&](double d, int t) __attribute__((always_inline)) {
        const double x = (d - a.d0) * a.inv_dd;
        const double y = ((double)t - a.t0) * a.inv_dt;
        int bin = -1;
        if (x >= 0.0 && x <= xmax && y >= 0.0 && y <= ymax) {
            int i = (int)floor(x);
            if (i > a.nd - 2) i = a.nd - 2;
            int j = (int)floor(y);
            if (j > a.nt - 2) j = a.nt - 2;
            const double fx = x - (double)i;
            const double fy = y - (double)j;
            const double *r0 = tab + (size_t)i * a.nt + j;
            const double *r1 = r0 + a.nt;
            const double v00 = r0[0], v01 = r0[1], v10 = r1[0], v11 = r1[1];
            const double ra = v00 + fy * (v01 - v00);
            const double rb = v10 + fy * (v11 - v10);
            bin = coord_bin(ra + fx * (rb - ra), e, s_b, a.T, a.e0, a.inv_w, a.G);
        }
        return bin;
    };
    auto dist = [&](int p) __attribute__((always_inline)) {
        // monitors carry no pixel ids: every event is at the one distance
        const unsigned q = pid ? (unsigned)p - (unsigned)a.pid_off : 0u;
        return q < a.L ? a.pix_d[q] : __builtin_nan("");
    };
    constexpr int V = 8;  // events per thread and iteration: every load issued first
    const bool vec = ((((uintptr_t)pid | (uintptr_t)toa | (uintptr_t)out) & 15u) == 0) && pid;
    const long long stride = (long long)gridDim.x * blockDim.x * V;
    long long k0 = ((long long)blockIdx.x * blockDim.x + threadIdx.x) * V;
    if (vec) {
        // the next group's events are requested before this group's gathers
        // and arithmetic (one group of loads always in flight)
        int p[V], t[V];
        auto load = [&](long long k, int (&pp)[V], int (&tt)[V]) __attribute__((always_inline)) {
#pragma unroll
            for (int h = 0; h < V / 4; ++h) {
                const v4i pv = ld_stream4(pid + k + 4 * h);
                const v4i tv = ld_stream4(toa + k + 4 * h);
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    pp[4 * h + q] = pv[q];
                    tt[4 * h + q] = tv[q];
                }
            }
        };
        if (k0 + V <= n) load(k0, p, t);
        for (; k0 + V <= n; k0 += stride) {
            int np[V], nt[V];
            const bool more = k0 + stride + V <= n;
            if (more) load(k0 + stride, np, nt);
            double d[V];
#pragma unroll
            for (int q = 0; q < V; ++q) d[q] = dist(p[q]);
            int b[V];
#pragma unroll
            for (int q = 0; q < V; ++q) b[q] = coord(d[q], t[q]);
#pragma unroll
            for (int h = 0; h < V / 4; ++h)
                *reinterpret_cast<int4 *>(out + k0 + 4 * h) =
                    make_int4(b[4 * h], b[4 * h + 1], b[4 * h + 2], b[4 * h + 3]);
            if (more) {
#pragma unroll
                for (int q = 0; q < V; ++q) {
                    p[q] = np[q];
                    t[q] = nt[q];
                }
            }
        }
    }
    // the vectorized loop's last, partial group; or every group of a segment
    // that is not 16-byte aligned (and monitors)
    for (long long k = k0; k < n; k += stride) {
        for (long long kk = k; kk < n && kk < k + V; ++kk)
            out[kk] = coord(dist(pid ? ld_global(pid + kk) : 0), ld_global(toa + kk));
        if (vec) break;
    }
}

// ---------------------------------------------------------------------------
// keyed pass: coordinate bin + pixel word -> the sieve's final word per event
// ---------------------------------------------------------------------------
// per slot the pixel's grid coordinate x = (d - d0) * inv_dd, the event
// pass's first two operations (same operations, no contraction: same bits).
// pre (KeyArgs::pre): the distance row instead, i = min(floor(x), nd - 2) into
// tab_i (0xFF: x outside [0, nd - 1] or NaN) and fx = x - i into tab_d, the
// event pass's next five operations
__device__ __forceinline__ void key_row(double x, int nd, double &fx, uint32_t &i) {
    const double xmax = (double)(nd - 1);
    int r = (int)floor(x);
    if (r > nd - 2) r = nd - 2;
    fx = x - (double)r;
    i = (x >= 0.0 && x <= xmax) ? (uint32_t)r : 0xFFu;
}

__global__ __launch_bounds__(256) void k_key_dist(const uint32_t *__restrict__ tab, int cbits,
                                                  const double *__restrict__ pix_d, unsigned L, double d0,
                                                  double inv_dd, int pre_nd, double *__restrict__ tab_d,
                                                  uint8_t *__restrict__ tab_i) {
    const unsigned j = blockIdx.x * 256u + threadIdx.x;
    if (j >= (1u << cbits)) return;
    const uint32_t w = tab[j];
    double d = __builtin_nan("");
    if (w & kSieveValid) {
        const unsigned q = (((w >> kSieveTagShift) & 0xFFu) << cbits) | j;
        if (q < L) d = pix_d[q];
    }
    const double x = (d - d0) * inv_dd;
    if (pre_nd) {
        double fx;
        uint32_t i;
        key_row(x, pre_nd, fx, i);
        tab_d[j] = fx;
        tab_i[j] = (uint8_t)i;
    } else {
        tab_d[j] = x;
    }
}

// LDS: pixel table (C words) | slot distances (C doubles) | edges | table | buckets
size_t key_smem(const KeyArgs &a, bool table_lds) {
    const size_t C = (size_t)1 << a.cbits;
    const int ne = a.c.edges_lds ? a.c.T + 2 : 0;
    return 12 * C + 8 * (size_t)((ne + 1) & ~1) + (table_lds ? 8 * (size_t)a.c.nd * a.c.nt : 0) +
           2 * (size_t)((a.c.G + 7) & ~7) + 16 * (size_t)kKeyLdsChunks + (a.pre ? C : 0);
}

// One block per CU walks a contiguous range of the batch's global chunks;
// thread t handles events (j * 1024 + t) * 4 + q (j < 2, q < 4) of a chunk,
// the sieve's layout.  Per event: the pixel's table slot in LDS (a hit gives
// its word and distance), else two gathers (word, distance; none for ids
// outside the LUT); the coordinate bin as in k_event_coord; the word
// (tag bits cleared) plus the bin, or 0 when the pixel or the bin is invalid.
template <bool TLDS, bool ELDS, bool FAST>
__global__ __launch_bounds__(1024) void k_event_key(KeyArgs k) {
    extern __shared__ double sm[];
    const CoordArgs &a = k.c;
    // the messages: kernel-argument descriptors (<= kKargSegs, no upload in
    // front of the pass) or the device table
    const SegDesc *segs = k.karg ? k.sk.s : k.segs;
    const uint32_t C = 1u << k.cbits;
    uint32_t *s_w = reinterpret_cast<uint32_t *>(sm);
    double *s_d = sm + C / 2;
    double *s_e = s_d + C;
    const int ne = ELDS ? a.T + 2 : 0;  // + e[T + 1] = +inf (FAST bin correction)
    double *s_t = s_e + ((ne + 1) & ~1);
    const int ntab = TLDS ? a.nd * a.nt : 0;
    uint16_t *s_b = reinterpret_cast<uint16_t *>(s_t + ntab);
    // FAST: per slot the distance row (u8, after the chunk pointers) and fx
    uint8_t *s_i = reinterpret_cast<uint8_t *>(s_b + ((a.G + 7) & ~7)) + 16 * kKeyLdsChunks;
    lds_fill<8>(s_w, (int)C, [&](int i) { return g_ld(k.pix_tab + i); });
    lds_fill<8>(s_d, (int)C, [&](int i) { return g_ld(k.tab_d + i); });
    if (FAST) lds_fill<8>(s_i, (int)C, [&](int i) { return g_ld(k.tab_i + i); });
    if (ne)
        lds_fill<2>(s_e, ne, [&](int i) {
            const double v = g_ld(a.edges + (i <= a.T ? i : a.T));
            return i <= a.T ? v : __builtin_inf();
        });
    if (ntab) lds_fill<4>(s_t, ntab, [&](int i) { return g_ld(a.table + i); });
    if (a.G) lds_fill<4>(s_b, a.G, [&](int i) { return g_ld(a.buckets + i); });
    __syncthreads();
    const double *e = ELDS ? s_e : a.edges;
    const double *tab = TLDS ? s_t : a.table;
    const double e_first = FAST ? e[0] : 0.0, e_last = FAST ? e[a.T] : 0.0;
    const double xmax = (double)(a.nd - 1), ymax = (double)(a.nt - 1);
    const __amdgpu_buffer_rsrc_t rrs = coord_rsrc(k.rec, (a.L + 1u) * 12u);
    const uint32_t cmask = C - 1u;
    const uint32_t pid_off = (uint32_t)a.pid_off;
    const uint32_t Lc = a.L;
    // x: the pixel's grid coordinate (k_key_dist / k_key_records); FAST: x is
    // fx and ir its distance row (0xFF: x outside the grid), both precomputed
    auto coord = [&](double x, uint32_t ir, int t) __attribute__((always_inline)) {
        const double y = ((double)t - a.t0) * a.inv_dt;
        int bin = -1;
        const bool xin = FAST ? ir != 0xFFu : (x >= 0.0 && x <= xmax);
        if (xin && y >= 0.0 && y <= ymax) {
            // x, y >= 0 here: truncation is the floor (one conversion, no v_floor)
            int i = FAST ? (int)ir : (int)x;
            if (!FAST && i > a.nd - 2) i = a.nd - 2;
            int j = (int)y;
            if (j > a.nt - 2) j = a.nt - 2;
            const double fx = FAST ? x : x - (double)i;
            const double fy = y - (double)j;
            const double *r0 = tab + (size_t)i * a.nt + j;
            const double *r1 = r0 + a.nt;
            const double v00 = r0[0], v01 = r0[1], v10 = r1[0], v11 = r1[1];
            const double ra = v00 + fy * (v01 - v00);
            const double rb = v10 + fy * (v11 - v10);
            const double v = ra + fx * (rb - ra);
            bin = FAST ? coord_bin_fast(v, e, s_b, e_first, e_last, a.e0, a.inv_w, a.G)
                       : coord_bin<false>(v, e, s_b, a.T, a.e0, a.inv_w, a.G);
        }
        return bin;
    };
    const long long n = k.n_chunks;
    const long long cb = (long long)blockIdx.x * n / gridDim.x;
    const long long ce = ((long long)blockIdx.x + 1) * n / gridDim.x;
    const int tid = threadIdx.x;
    // The block's chunks in windows of kKeyLdsChunks: each window's {pid, toa}
    // pointers go to LDS first (one segment search per chunk, by its own
    // thread), with chunks that are not full and 16-byte aligned mapped to the
    // all-invalid dummy chunk and redone element-wise after the window.  The
    // main loop then has one load path and reads its pointers from LDS, so
    // the in-order vmcnt waits for exactly the gathers it needs while the
    // next chunk's loads stay in flight.
    const int **s_cp = reinterpret_cast<const int **>(s_b + ((a.G + 7) & ~7));  // [window][2]
    auto chunk_ptrs = [&](long long c, const int *&pp, const int *&tp) -> bool {
        int lo = 0, hi = k.n_segs - 1;  // last segment with chunk0 <= c
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (segs[mid].chunk0 <= c) lo = mid; else hi = mid - 1;
        }
        const SegDesc sd = segs[lo];
        const long long base = (c - sd.chunk0) * kChunk;
        pp = sd.pid + base;
        tp = sd.toa + base;
        return ((((uintptr_t)pp | (uintptr_t)tp) & 15u) == 0) && base + kChunk <= sd.n;
    };
    auto fetch = [&](long long w0, long long c, int (&p)[8], int (&t)[8]) __attribute__((always_inline)) {
        const int *pp = s_cp[2 * (c - w0)], *tp = s_cp[2 * (c - w0) + 1];
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int e0 = (j * 1024 + tid) * 4;
            const v4i pv = ld_stream4(pp + e0);
            const v4i tv = ld_stream4(tp + e0);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                p[j * 4 + q] = pv[q];
                t[j * 4 + q] = tv[q];
            }
        }
    };
    // one chunk's words: table probe, the misses' gathers, then `next` (the
    // next chunk's loads, issued after the gathers), then the arithmetic
    auto words = [&](const int (&p)[8], const int (&t)[8], int (&out)[8], auto &&next)
        __attribute__((always_inline)) {
        uint32_t w[8], g[8], slot[8];
        double d[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const uint32_t pq = (uint32_t)p[q] - pid_off;
            slot[q] = pq & cmask;
            const uint32_t tw = s_w[slot[q]];
            const bool hit = ((tw >> kSieveTagShift) & 0xFFu) == (pq >> k.cbits);
            // hits and ids outside the LUT load out of range (no request, 0);
            // the word of an id outside the LUT is 0 (dropped)
            const bool skip = hit || pq >= Lc || (LDE_DIAG(k.ablate) & 1);
            const v3u r = __builtin_amdgcn_raw_buffer_load_b96(rrs, skip ? (int)0x80000000 : (int)(pq * 12u),
                                                                0, 0);
            g[q] = r[0];
            d[q] = __builtin_bit_cast(double, ((unsigned long long)r[2] << 32) | r[1]);
            w[q] = hit ? (tw & (kSieveValid | kSieveHot | kSieveValueMask)) : 0u;
            slot[q] = hit ? slot[q] : 0xFFFFFFFFu;
        }
        int tc[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) tc[q] = t[q];
        // issue order fixed: every gather, then the next chunk's loads
        __builtin_amdgcn_sched_barrier(0);
        next();
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const bool h = slot[q] != 0xFFFFFFFFu;
            const double dq = h ? s_d[slot[q]] : d[q];
            // FAST: a record's distance row rides in its word's (zero) tag bits
            const uint32_t ir = FAST ? (h ? (uint32_t)s_i[slot[q]] : (g[q] >> kSieveTagShift) & 0xFFu) : 0u;
            const uint32_t word = w[q] | (FAST ? g[q] & ~(0xFFu << kSieveTagShift) : g[q]);
            const int b = (LDE_DIAG(k.ablate) & 2) ? (int)(((uint32_t)tc[q] ^ (uint32_t)dq) & 63u)
                          : (word & kSieveValid) ? coord(dq, ir, tc[q]) : -1;
            out[q] = b >= 0 ? (int)(word + (uint32_t)b) : 0;
        }
    };
    auto store = [&](long long c, const int (&out)[8]) __attribute__((always_inline)) {
        if (LDE_DIAG(k.ablate) & 4) {  // diagnostics: one word per lane kept live, not stored
            int x = 0;
#pragma unroll
            for (int q = 0; q < 8; ++q) x ^= out[q];
            if (x == 0x7FFFFFFF) k.keys[tid] = x;
            return;
        }
#pragma unroll
        for (int j = 0; j < 2; ++j)
            *reinterpret_cast<int4 *>(k.keys + c * kChunk + ((long long)j * 1024 + tid) * 4) =
                make_int4(out[j * 4], out[j * 4 + 1], out[j * 4 + 2], out[j * 4 + 3]);
    };
    for (long long w0 = cb; w0 < ce; w0 += kKeyLdsChunks) {
        const long long w1 = w0 + kKeyLdsChunks < ce ? w0 + kKeyLdsChunks : ce;
        __syncthreads();  // the previous window's pointers are dead
        for (long long c = w0 + tid; c < w1; c += blockDim.x) {
            const int *pp, *tp;
            const bool full = chunk_ptrs(c, pp, tp);
            s_cp[2 * (c - w0)] = full ? pp : k.dummy;
            s_cp[2 * (c - w0) + 1] = full ? tp : k.dummy;
        }
        __syncthreads();
        int p[8], t[8];
        fetch(w0, w0, p, t);
        for (long long c = w0; c < w1; ++c) {
            int out[8];
            // the window's last chunk reloads itself: the loads stay
            // unconditional (a branch around them makes the compiler wait for
            // every outstanding load after it, the next chunk's included)
            const long long cn = c + 1 < w1 ? c + 1 : c;
            words(p, t, out, [&]() __attribute__((always_inline)) { fetch(w0, cn, p, t); });
            store(c, out);
        }
        // the window's chunks that are not full and aligned: element loads
        for (long long c = w0; c < w1; ++c) {
            if (s_cp[2 * (c - w0)] != k.dummy) continue;  // block-uniform
            const int *pp, *tp;
            (void)chunk_ptrs(c, pp, tp);
            long long left;
            {
                int lo = 0, hi = k.n_segs - 1;
                while (lo < hi) {
                    const int mid = (lo + hi + 1) >> 1;
                    if (segs[mid].chunk0 <= c) lo = mid; else hi = mid - 1;
                }
                left = segs[lo].n - (c - segs[lo].chunk0) * kChunk;
            }
            int pe[8], te[8], out[8];
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const long long e = ((long long)j * 1024 + tid) * 4 + q;
                    const bool ok = e < left;
                    pe[j * 4 + q] = ok ? ld_global(pp + e) : a.pid_off - 1;  // dropped
                    te[j * 4 + q] = ok ? ld_global(tp + e) : 0;
                }
            words(pe, te, out, []() {});
            store(c, out);
        }
    }
}

// per pixel {word, distance}: a table miss gathers one 12-byte record
// instead of a word and a distance from two tables (entry L: word 0).  12
// bytes, not 16: the record array (5.9 MB for DREAM) is then mostly
// L2/MALL-resident for the Zipf tail's random misses
__global__ __launch_bounds__(256) void k_key_records(const uint32_t *__restrict__ glut,
                                                     const double *__restrict__ pix_d, unsigned L,
                                                     double d0, double inv_dd, int pre_nd,
                                                     uint32_t *__restrict__ rec) {
    const unsigned q = blockIdx.x * 256u + threadIdx.x;
    if (q > L) return;
    double d = ((q < L ? pix_d[q] : __builtin_nan("")) - d0) * inv_dd;  // x, as k_key_dist
    uint32_t ir = 0;
    if (pre_nd) key_row(d, pre_nd, d, ir);  // fx; the row in the word's tag bits
    const unsigned long long b = __builtin_bit_cast(unsigned long long, d);
    rec[3 * (size_t)q] = q < L ? (glut[q] | (pre_nd ? ir << kSieveTagShift : 0u)) : 0u;
    rec[3 * (size_t)q + 1] = (uint32_t)b;
    rec[3 * (size_t)q + 2] = (uint32_t)(b >> 32);
}

hipError_t launch_key_records(const uint32_t *glut, const double *pix_d, unsigned L, double d0,
                              double inv_dd, int pre_nd, uint32_t *rec, hipStream_t st) {
    hipLaunchKernelGGL(k_key_records, dim3((L + 1u + 255u) / 256u), dim3(256), 0, st, glut, pix_d, L, d0,
                       inv_dd, pre_nd, rec);
    return hipGetLastError();
}

hipError_t launch_key_dist(const uint32_t *pix_tab, int cbits, const double *pix_d, unsigned L,
                           double d0, double inv_dd, int pre_nd, double *tab_d, uint8_t *tab_i,
                           hipStream_t st, hipEvent_t start) {
    hipExtLaunchKernelGGL(k_key_dist, dim3(((1u << cbits) + 255) / 256), dim3(256), 0, st, start, nullptr, 0,
                          pix_tab, cbits, pix_d, L, d0, inv_dd, pre_nd, tab_d, tab_i);
    return hipGetLastError();
}

template <bool TLDS, bool ELDS, bool FIXED>
static void launch_key_t(const KeyArgs &a, size_t sm, int grid, hipStream_t st, hipEvent_t start,
                         hipEvent_t stop) {
    (void)hipFuncSetAttribute((const void *)k_event_key<TLDS, ELDS, FIXED>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)sm);
    hipExtLaunchKernelGGL((k_event_key<TLDS, ELDS, FIXED>), dim3((unsigned)grid), dim3(1024), sm, st, start,
                          stop, 0, a);
}

hipError_t launch_event_key(const KeyArgs &a, int grid, hipStream_t st, hipEvent_t start, hipEvent_t stop) {
    if (a.n_chunks <= 0) {
        if (start) (void)hipEventRecord(start, st);
        return stop ? hipEventRecord(stop, st) : hipSuccess;
    }
    const bool tl = key_smem(a, true) <= kCoordSmemMax;
    const size_t sm = key_smem(a, tl);
    if (sm > kCoordSmemMax) return hipErrorInvalidValue;
    if (grid > a.n_chunks) grid = (int)a.n_chunks;
    // FAST (branch-free bin correction, precomputed distance rows) only with
    // the edges in LDS (the common case)
    const bool fx = a.pre && a.c.fixed_bin && a.c.edges_lds;
    if (a.pre && !fx) return hipErrorInvalidValue;  // the caller pairs pre with FAST
    if (tl) {
        if (fx) launch_key_t<true, true, true>(a, sm, grid, st, start, stop);
        else if (a.c.edges_lds) launch_key_t<true, true, false>(a, sm, grid, st, start, stop);
        else launch_key_t<true, false, false>(a, sm, grid, st, start, stop);
    } else {
        if (fx) launch_key_t<false, true, true>(a, sm, grid, st, start, stop);
        else if (a.c.edges_lds) launch_key_t<false, true, false>(a, sm, grid, st, start, stop);
        else launch_key_t<false, false, false>(a, sm, grid, st, start, stop);
    }
    return hipGetLastError();
}

size_t coord_smem(const CoordArgs &a, bool table_lds) {
    const int ne = a.edges_lds ? a.T + 1 : 0;
    return 8 * (size_t)((ne + 1) & ~1) + (table_lds ? 8 * (size_t)a.nd * a.nt : 0) + 2 * (size_t)a.G;
}

template <bool TLDS, bool ELDS>
static void launch_coord_t(const CoordArgs &a, const int *pid, const int *toa, long long n, int *out,
                           size_t sm, long long g, hipStream_t st) {
    (void)hipFuncSetAttribute((const void *)k_event_coord<TLDS, ELDS>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)sm);
    hipLaunchKernelGGL((k_event_coord<TLDS, ELDS>), dim3((unsigned)g), dim3(256), sm, st, a, pid, toa, n,
                       out);
}

hipError_t launch_event_coord(const CoordArgs &a, const int *pid, const int *toa, long long n,
                              int *out, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    // 256-thread blocks, several per CU; the table in LDS when it fits
    const bool tl = coord_smem(a, true) <= kCoordSmemMax;
    const size_t sm = coord_smem(a, tl);
    if (sm > kCoordSmemMax) return hipErrorInvalidValue;
    long long g = (n + 256LL * 8 - 1) / (256LL * 8);
    if (g > 4096) g = 4096;
    if (tl) {
        if (a.edges_lds) launch_coord_t<true, true>(a, pid, toa, n, out, sm, g, st);
        else launch_coord_t<true, false>(a, pid, toa, n, out, sm, g, st);
    } else {
        if (a.edges_lds) launch_coord_t<false, true>(a, pid, toa, n, out, sm, g, st);
        else launch_coord_t<false, false>(a, pid, toa, n, out, sm, g, st);
    }
    return hipGetLastError();
}

}  // namespace lde
