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
//   per pixel (host, setup time):  x = (d - d0) * inv_dd,  i = min(floor(x), nd - 2),
//                                  fx = x - i               (pi = -1 when invalid)
//   per event (here):              y = (t - t0) * inv_dt,  j = min(floor(y), nt - 2),
//                                  fy = y - j               (dropped unless 0 <= y <= nt - 1)
//   a = v[i][j] + fy * (v[i][j+1] - v[i][j]);  b = v[i+1][j] + fy * (v[i+1][j+1] - v[i+1][j])
//   c = a + fx * (b - a)
// evaluated in float64 without contraction (no FMA), so the CPU oracle's
// numpy restatement gives the same bits.  The kernel writes the coordinate's
// bin index (or -1) as an int32 "time" per event; the engine then bins
// (pid, bin) with its usual strategies against the integer edges 0..T, so every
// strategy and skew path is reused bit for bit.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "lde_device.h"
#include "lde_internal.h"

#pragma clang fp contract(off)

namespace lde {

// largest b with edges[b] <= v, or -1 (half-open, last bin too; NaN dropped)
__device__ __forceinline__ int coord_bin(double v, const double *s_e, int T) {
    if (!(v >= s_e[0]) || !(v < s_e[T])) return -1;
    int lo = 0, hi = T;  // s_e[lo] <= v < s_e[hi]
    while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (s_e[mid] <= v) lo = mid; else hi = mid;
    }
    return lo;
}

__global__ __launch_bounds__(256) void k_event_coord(CoordArgs a, const int *__restrict__ pid,
                                                     const int *__restrict__ toa, long long n,
                                                     int *__restrict__ out) {
    extern __shared__ double s_e[];
    for (int i = threadIdx.x; i <= a.T; i += blockDim.x) s_e[i] = a.edges[i];
    __syncthreads();
    const double ymax = (double)(a.nt - 1);
    for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < n;
         e += (long long)gridDim.x * blockDim.x) {
        // monitors carry no pixel ids: every event is at the one distance
        const unsigned q = pid ? (unsigned)ld_global(pid + e) - (unsigned)a.pid_off : 0u;
        int bin = -1;
        if (q < a.L) {
            const int pi = a.pix_i[q];
            if (pi >= 0) {
                const double y = ((double)ld_global(toa + e) - a.t0) * a.inv_dt;
                if (y >= 0.0 && y <= ymax) {
                    int j = (int)floor(y);
                    if (j > a.nt - 2) j = a.nt - 2;
                    const double fy = y - (double)j;
                    const double fx = a.pix_f[q];
                    const double *r0 = a.table + (size_t)pi * a.nt + j;
                    const double *r1 = r0 + a.nt;
                    const double v00 = r0[0], v01 = r0[1], v10 = r1[0], v11 = r1[1];
                    const double ra = v00 + fy * (v01 - v00);
                    const double rb = v10 + fy * (v11 - v10);
                    bin = coord_bin(ra + fx * (rb - ra), s_e, a.T);
                }
            }
        }
        out[e] = bin;
    }
}

hipError_t launch_event_coord(const CoordArgs &a, const int *pid, const int *toa, long long n,
                              int *out, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    long long g = (n + 255) / 256;
    if (g > 4096) g = 4096;
    hipLaunchKernelGGL(k_event_coord, dim3((unsigned)g), dim3(256), (size_t)(a.T + 1) * 8, st, a,
                       pid, toa, n, out);
    return hipGetLastError();
}

}  // namespace lde
