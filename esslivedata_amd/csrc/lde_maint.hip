// lde_maint.hip -- window/cumulative maintenance kernels of the binning engine:
// u32->u64 window fold, BIFROST f32 per-push merge, snapshots and the
// finalize kernel (cumulative += window, images, totals), mirroring
// NoCopyAccumulator / the window accumulator (SRC/preprocessors/accumulators.py:86-195)
// and detector_image / counts_total / counts_in_range
// (SRC/workflows/detector_view/providers.py:236-357).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "lde_internal.h"

namespace lde {

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
// launch wrappers
// ---------------------------------------------------------------------------
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
