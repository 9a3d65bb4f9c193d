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
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "lde_device.h"
#include "lde_internal.h"

#pragma clang fp contract(off)

namespace lde {

// largest b with e[b] <= v < e[b + 1] (half-open, last bin too; NaN dropped)
__device__ __forceinline__ int coord_bin(double v, const double *e, const uint16_t *bk, int T,
                                         double e0, double inv_w, int G) {
    if (!(v >= e[0]) || !(v < e[T])) return -1;
    int g = (int)((v - e0) * inv_w);
    g = g < 0 ? 0 : (g >= G ? G - 1 : g);
    int b = bk[g];
    while (b > 0 && v < e[b]) --b;
    while (v >= e[b + 1]) ++b;
    return b;
}

template <bool TLDS>
__global__ __launch_bounds__(256) void k_event_coord(CoordArgs a, const int *__restrict__ pid,
                                                     const int *__restrict__ toa, long long n,
                                                     int *__restrict__ out) {
    extern __shared__ double sm[];
    // LDS: edges (T + 1, when they fit) | table (TLDS) | bucket table (u16)
    const int ne = a.edges_lds ? a.T + 1 : 0;
    double *s_e = sm;
    double *s_t = sm + ((ne + 1) & ~1);
    const int ntab = TLDS ? a.nd * a.nt : 0;
    uint16_t *s_b = reinterpret_cast<uint16_t *>(s_t + ntab);
    for (int i = threadIdx.x; i < ne; i += blockDim.x) s_e[i] = a.edges[i];
    for (int i = threadIdx.x; i < ntab; i += blockDim.x) s_t[i] = a.table[i];
    for (int i = threadIdx.x; i < a.G; i += blockDim.x) s_b[i] = a.buckets[i];
    __syncthreads();
    const double *e = a.edges_lds ? s_e : a.edges;
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
        for (; k0 + V <= n; k0 += stride) {
            int p[V], t[V];
#pragma unroll
            for (int h = 0; h < V / 4; ++h) {
                const v4i pv = ld_stream4(pid + k0 + 4 * h);
                const v4i tv = ld_stream4(toa + k0 + 4 * h);
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    p[4 * h + q] = pv[q];
                    t[4 * h + q] = tv[q];
                }
            }
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

size_t coord_smem(const CoordArgs &a, bool table_lds) {
    const int ne = a.edges_lds ? a.T + 1 : 0;
    return 8 * (size_t)((ne + 1) & ~1) + (table_lds ? 8 * (size_t)a.nd * a.nt : 0) +
           2 * (size_t)a.G;
}

hipError_t launch_event_coord(const CoordArgs &a, const int *pid, const int *toa, long long n,
                              int *out, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    long long g = (n + 256 * 8 - 1) / (256 * 8);
    if (g > 4096) g = 4096;
    const bool tl = coord_smem(a, true) <= kCoordSmemMax;
    const size_t sm = coord_smem(a, tl);
    if (sm > kCoordSmemMax) return hipErrorInvalidValue;
    if (tl) {
        (void)hipFuncSetAttribute((const void *)k_event_coord<true>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)sm);
        hipLaunchKernelGGL(k_event_coord<true>, dim3((unsigned)g), dim3(256), sm, st, a, pid, toa,
                           n, out);
    } else {
        (void)hipFuncSetAttribute((const void *)k_event_coord<false>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)sm);
        hipLaunchKernelGGL(k_event_coord<false>, dim3((unsigned)g), dim3(256), sm, st, a, pid, toa,
                           n, out);
    }
    return hipGetLastError();
}

}  // namespace lde
