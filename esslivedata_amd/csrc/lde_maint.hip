// lde_maint.hip -- window/cumulative maintenance kernels of the binning engine:
// u32->u64 window fold, BIFROST f32 per-push merge, snapshots and the
// finalize kernel (cumulative += window, images, totals), mirroring
// NoCopyAccumulator / the window accumulator (SRC/preprocessors/accumulators.py:86-195)
// and detector_image / counts_total / counts_in_range
// (SRC/workflows/detector_view/providers.py:236-357).
#include <hip/hip_ext.h>
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

// one push of exact counts (the RCCL sum of every rank's push, u64) into a
// float32 view's accumulators in the reference order: f32 += float32(count)
// (accumulators.py:129-135, the cast of bifrost/specs.py:295), exact u64
// window += count; the source is left as it is
__global__ void k_merge_f32_u64(const unsigned long long *__restrict__ src,
                                unsigned long long *__restrict__ win64, float *__restrict__ winf,
                                float *__restrict__ cumf, long long n, int first_win, int first_cum) {
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (long long)gridDim.x * blockDim.x) {
        const unsigned long long b = src[i];
        const float fb = (float)b;  // one rounding, as float32(float64(count))
        winf[i] = first_win ? fb : winf[i] + fb;
        cumf[i] = first_cum ? fb : cumf[i] + fb;
        win64[i] += b;
    }
}

// a push's batch counts out as u64 (the push buffer of a sharded float32
// view), the batch emptied for the next push
__global__ void k_push_export(uint32_t *__restrict__ batch, unsigned long long *__restrict__ out,
                              long long n) {
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (long long)gridDim.x * blockDim.x) {
        out[i] = batch[i];
        batch[i] = 0;
    }
}

// snapshot: out = a (+ b) (+ c) as u64, for reads that must not finalize
// A cumulative in split form (cum32 = its bin count, wide-row views): u32 low
// words [cum32] then u32 high words [cum32], so the finalize moves 4 bytes per
// bin instead of 8 and carries into the high word only on a wrap.
__device__ __forceinline__ unsigned long long cum_at(const unsigned long long *cum, long long cum32, size_t i) {
    if (!cum32) return cum[i];
    const uint32_t *lo = reinterpret_cast<const uint32_t *>(cum);
    return (unsigned long long)lo[i] | ((unsigned long long)lo[cum32 + i] << 32);
}

__global__ void k_sum3(const unsigned long long *__restrict__ a, const unsigned long long *__restrict__ b,
                       const uint32_t *__restrict__ c, unsigned long long *__restrict__ out,
                       long long n, long long a32) {
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (long long)gridDim.x * blockDim.x) {
        unsigned long long v = c ? c[i] : 0ull;
        if (a) v += cum_at(a, a32, (size_t)i);
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
                                                  unsigned long long *__restrict__ totals,
                                                  const uint32_t *__restrict__ ovf_src,
                                                  uint32_t *__restrict__ ovf_dst) {
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
    // per-block partials (summed by k_sum_totals, or by the host from the
    // finalize pack): thousands of same-word atomics would serialize at the
    // memory side
    if (ovf_dst && blockIdx.x == 0 && threadIdx.x == 4) *ovf_dst = ovf_src ? *ovf_src : 0u;
    if (threadIdx.x < 4)
        totals[4 + (size_t)blockIdx.x * 4 + threadIdx.x] =
            s_tot[0][threadIdx.x] + s_tot[1][threadIdx.x] + s_tot[2][threadIdx.x] + s_tot[3][threadIdx.x];
}

// Same as k_finalize for T % 4 == 0 and T <= 128: a 32-lane group per screen
// row (two rows per wave), 4 bins per lane with 16-byte loads and stores, and
// 5-step group reductions instead of 6-step wave reductions per row.
template <typename OUT>
__global__ __launch_bounds__(256) void k_finalize_v4(uint32_t *__restrict__ win32,
                                                     unsigned long long *__restrict__ win64,
                                                     unsigned long long *__restrict__ cum,
                                                     unsigned long long *__restrict__ snap,
                                                     long long S, int T, int lo, int hi,
                                                     OUT *__restrict__ cur_img,
                                                     OUT *__restrict__ cum_img,
                                                     unsigned long long *__restrict__ totals,
                                                  const uint32_t *__restrict__ ovf_src,
                                                  uint32_t *__restrict__ ovf_dst) {
    typedef unsigned long long u64;
    __shared__ u64 s_tot[8][4];
    __shared__ OUT s_img[2][8];
    const int gl = threadIdx.x & 31, grp = threadIdx.x >> 5;  // 8 row groups per block
    u64 acc[4] = {0, 0, 0, 0};
    const int i0 = gl * 4;
    const bool act = i0 < T;
    // uniform loop over the block's 8-row slices: the slice's image values
    // leave through LDS as two contiguous 8-element runs (one store
    // instruction each), which matters when the images are host-mapped
    for (long long base = (long long)blockIdx.x * 8; base < S; base += (long long)gridDim.x * 8) {
        const long long s = base + grp;
        u64 rw = 0, rc = 0, tw = 0, tc = 0;
        if (act && s < S) {
            const long long k = s * T + i0;
            const uint4 w4 = *reinterpret_cast<const uint4 *>(win32 + k);
            u64 w[4] = {w4.x, w4.y, w4.z, w4.w};
            if (win64) {
                const ulonglong2 a = *reinterpret_cast<const ulonglong2 *>(win64 + k);
                const ulonglong2 b = *reinterpret_cast<const ulonglong2 *>(win64 + k + 2);
                w[0] += a.x; w[1] += a.y; w[2] += b.x; w[3] += b.y;
                *reinterpret_cast<ulonglong2 *>(win64 + k) = make_ulonglong2(0, 0);
                *reinterpret_cast<ulonglong2 *>(win64 + k + 2) = make_ulonglong2(0, 0);
            }
            const ulonglong2 c01 = *reinterpret_cast<const ulonglong2 *>(cum + k);
            const ulonglong2 c23 = *reinterpret_cast<const ulonglong2 *>(cum + k + 2);
            const u64 c[4] = {c01.x + w[0], c01.y + w[1], c23.x + w[2], c23.y + w[3]};
            *reinterpret_cast<ulonglong2 *>(cum + k) = make_ulonglong2(c[0], c[1]);
            *reinterpret_cast<ulonglong2 *>(cum + k + 2) = make_ulonglong2(c[2], c[3]);
            if (snap) {
                *reinterpret_cast<ulonglong2 *>(snap + k) = make_ulonglong2(w[0], w[1]);
                *reinterpret_cast<ulonglong2 *>(snap + k + 2) = make_ulonglong2(w[2], w[3]);
            }
            *reinterpret_cast<uint4 *>(win32 + k) = make_uint4(0, 0, 0, 0);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                tw += w[q];
                tc += c[q];
                if (i0 + q >= lo && i0 + q < hi) {
                    rw += w[q];
                    rc += c[q];
                }
            }
        }
#pragma unroll
        for (int d = 16; d > 0; d >>= 1) {
            rw += __shfl_xor(rw, d, 32);
            rc += __shfl_xor(rc, d, 32);
            tw += __shfl_xor(tw, d, 32);
            tc += __shfl_xor(tc, d, 32);
        }
        if (gl == 0) {
            s_img[0][grp] = (OUT)rw;
            s_img[1][grp] = (OUT)rc;
            acc[0] += tw;
            acc[1] += rw;
            acc[2] += tc;
            acc[3] += rc;
        }
        __syncthreads();
        if (threadIdx.x < 16) {
            const int r = threadIdx.x & 7;
            OUT *img = threadIdx.x < 8 ? cur_img : cum_img;
            if (img && base + r < S) img[base + r] = s_img[threadIdx.x >> 3][r];
        }
        __syncthreads();
    }
    if (gl == 0)
        for (int q = 0; q < 4; ++q) s_tot[grp][q] = acc[q];
    __syncthreads();
    if (ovf_dst && blockIdx.x == 0 && threadIdx.x == 4) *ovf_dst = ovf_src ? *ovf_src : 0u;
    if (threadIdx.x < 4) {
        u64 v = 0;
        for (int g = 0; g < 8; ++g) v += s_tot[g][threadIdx.x];
        totals[4 + (size_t)blockIdx.x * 4 + threadIdx.x] = v;
    }
}

// Same as k_finalize for T % 4 == 0 and larger T (the WIDE views: 164 ..
// 10,000 bins): one wave per screen row, 4 bins per lane with 16-byte window
// loads and 2 x 16-byte cumulative loads and stores, two row slices in flight
// per lane (k_finalize's scalar loop held one 4-byte load per lane in flight:
// 3.7 TB/s on DREAM at 1,000 bins).
template <typename OUT, bool CUM32, bool INC>
__global__ __launch_bounds__(256) void k_finalize_w4(uint32_t *__restrict__ win32,
                                                     unsigned long long *__restrict__ win64,
                                                     unsigned long long *__restrict__ cum,
                                                     unsigned long long *__restrict__ snap,
                                                     long long S, int T, int lo, int hi,
                                                     OUT *__restrict__ cur_img,
                                                     OUT *__restrict__ cum_img,
                                                     unsigned long long *__restrict__ totals,
                                                     const uint32_t *__restrict__ ovf_src,
                                                     uint32_t *__restrict__ ovf_dst,
                                                     unsigned long long *__restrict__ cumrow, long long cum32) {
    typedef unsigned long long u64;
    constexpr bool inc = INC;
    __shared__ u64 s_tot[4][4];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    u64 acc[4] = {0, 0, 0, 0};
    for (long long s = (long long)blockIdx.x * 4 + wid; s < S; s += (long long)gridDim.x * 4) {
        u64 rw = 0, rc = 0, tw = 0, tc = 0;
#pragma unroll 2
        for (int i0 = lane * 4; i0 < T; i0 += 256) {
            const long long k = s * T + i0;
            const uint4 w4 = *reinterpret_cast<const uint4 *>(win32 + k);
            u64 w[4] = {w4.x, w4.y, w4.z, w4.w};
            if (win64) {
                const ulonglong2 a = *reinterpret_cast<const ulonglong2 *>(win64 + k);
                const ulonglong2 b = *reinterpret_cast<const ulonglong2 *>(win64 + k + 2);
                w[0] += a.x; w[1] += a.y; w[2] += b.x; w[3] += b.y;
                *reinterpret_cast<ulonglong2 *>(win64 + k) = make_ulonglong2(0, 0);
                *reinterpret_cast<ulonglong2 *>(win64 + k + 2) = make_ulonglong2(0, 0);
            }
            // with the per-screen cumulative sums kept (inc), a group the
            // window left empty neither reads nor writes the cumulative
            const bool nz = (w[0] | w[1] | w[2] | w[3]) != 0;
            u64 c[4] = {0, 0, 0, 0};
            if (CUM32 && (!inc || nz)) {
                // split form: low words read and written, a wrap carries into
                // the high word (read only to recompute the sums)
                uint32_t *lo32 = reinterpret_cast<uint32_t *>(cum);
                uint32_t *hi32 = lo32 + cum32;
                const uint4 l4 = *reinterpret_cast<const uint4 *>(lo32 + k);
                const uint32_t l[4] = {l4.x, l4.y, l4.z, l4.w};
                uint32_t nl[4], cy[4];
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    nl[q] = l[q] + (uint32_t)w[q];
                    cy[q] = (uint32_t)(w[q] >> 32) + (nl[q] < l[q] ? 1u : 0u);
                }
                if (!inc) {
                    const uint4 h4 = *reinterpret_cast<const uint4 *>(hi32 + k);
                    const uint32_t h[4] = {h4.x, h4.y, h4.z, h4.w};
#pragma unroll
                    for (int q = 0; q < 4; ++q) c[q] = (((u64)h[q] << 32) | l[q]) + w[q];
                }
                if (nz) {
                    *reinterpret_cast<uint4 *>(lo32 + k) = make_uint4(nl[0], nl[1], nl[2], nl[3]);
#pragma unroll
                    for (int q = 0; q < 4; ++q)
                        if (cy[q]) hi32[k + q] += cy[q];  // (this thread owns the bin)
                }
            } else if (!CUM32 && (!inc || nz)) {
                const ulonglong2 c01 = *reinterpret_cast<const ulonglong2 *>(cum + k);
                const ulonglong2 c23 = *reinterpret_cast<const ulonglong2 *>(cum + k + 2);
                c[0] = c01.x + w[0];
                c[1] = c01.y + w[1];
                c[2] = c23.x + w[2];
                c[3] = c23.y + w[3];
                if (nz) {
                    *reinterpret_cast<ulonglong2 *>(cum + k) = make_ulonglong2(c[0], c[1]);
                    *reinterpret_cast<ulonglong2 *>(cum + k + 2) = make_ulonglong2(c[2], c[3]);
                }
            }
            if (snap) {
                *reinterpret_cast<ulonglong2 *>(snap + k) = make_ulonglong2(w[0], w[1]);
                *reinterpret_cast<ulonglong2 *>(snap + k + 2) = make_ulonglong2(w[2], w[3]);
            }
            if (w4.x | w4.y | w4.z | w4.w) *reinterpret_cast<uint4 *>(win32 + k) = make_uint4(0, 0, 0, 0);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                tw += w[q];
                tc += c[q];
                if (i0 + q >= lo && i0 + q < hi) {
                    rw += w[q];
                    rc += c[q];
                }
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
            if (cumrow) {
                // the screen's cumulative sums (in range, all bins): kept
                // across finalizes, recomputed from the bins when !inc
                if (inc) {
                    rc = cumrow[s] + rw;
                    tc = cumrow[S + s] + tw;
                }
                cumrow[s] = rc;
                cumrow[S + s] = tc;
            }
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
    if (ovf_dst && blockIdx.x == 0 && threadIdx.x == 4) *ovf_dst = ovf_src ? *ovf_src : 0u;
    if (threadIdx.x < 4)
        totals[4 + (size_t)blockIdx.x * 4 + threadIdx.x] =
            s_tot[0][threadIdx.x] + s_tot[1][threadIdx.x] + s_tot[2][threadIdx.x] + s_tot[3][threadIdx.x];
}

// totals[q] = sum over blocks of the partials at totals[4 + 4 * block + q].
// Thread i sums the partials i, i + 1024, ... (all of quantity i & 3) with
// independent loads, then the 256 threads of each quantity reduce in LDS.
// The four sums also go to `copy` (the finalize pack / a partials buffer) and
// the page-pool overflow flag is carried along to `ovf_dst`, so finalize needs
// no separate device-to-device copies (each a ~5 us blit).
__global__ __launch_bounds__(1024) void k_sum_totals(unsigned long long *__restrict__ totals,
                                                     int blocks, unsigned long long *__restrict__ copy,
                                                     const uint32_t *__restrict__ ovf_src,
                                                     uint32_t *__restrict__ ovf_dst) {
    __shared__ unsigned long long s[1024];
    const int n = 4 * blocks;
    unsigned long long v = 0;
    for (int j = threadIdx.x; j < n; j += 1024) v += totals[4 + j];
    s[threadIdx.x] = v;
    __syncthreads();
    for (int d = 512; d >= 4; d >>= 1) {
        if ((int)threadIdx.x < d) s[threadIdx.x] += s[threadIdx.x + d];
        __syncthreads();
    }
    if (threadIdx.x < 4) {
        totals[threadIdx.x] = s[threadIdx.x];
        if (copy) copy[threadIdx.x] = s[threadIdx.x];
    }
    if (ovf_dst && threadIdx.x == 4) *ovf_dst = ovf_src ? *ovf_src : 0u;
}

// Finalize of a float32 view (BIFROST) in one pass, with the window's last
// push still in the u32 batch (the reference cadence is one push per
// finalize, SRC/core/job.py:413-433): per bin that push's f32 adds in the
// reference order (window += f32(b), cumulative += f32(b); the adds k_merge_f32
// would have made), the images as k_rows_f32 sums them (f32 values over the
// TOA range in f64, rounded once), the exact integer totals and cumulative
// (cum += win64 + b), and the window reset (f32, u64 and the batch).  batch =
// nullptr: no pending push.  snap (optional): the f32 window before its reset.
// One wave per screen row; per-block total partials at totals[4 + 4 b].
__global__ __launch_bounds__(256) void k_finalize_f32(
    uint32_t *__restrict__ batch, unsigned long long *__restrict__ win64,
    unsigned long long *__restrict__ cum, float *__restrict__ winf, float *__restrict__ cumf,
    float *__restrict__ snap, long long S, int T, int lo, int hi, int first_win, int first_cum,
    float *__restrict__ cur_img, float *__restrict__ cum_img, unsigned long long *__restrict__ totals,
    const uint32_t *__restrict__ ovf_src, uint32_t *__restrict__ ovf_dst) {
    typedef unsigned long long u64;
    __shared__ u64 s_tot[4][4];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    u64 acc[4] = {0, 0, 0, 0};
    for (long long s = (long long)blockIdx.x * 4 + wid; s < S; s += (long long)gridDim.x * 4) {
        double rwf = 0.0, rcf = 0.0;
        u64 rw = 0, rc = 0, tw = 0, tc = 0;
        for (int i = lane; i < T; i += 64) {
            const long long k = s * T + i;
            const uint32_t b = batch ? batch[k] : 0u;
            float wf = winf[k], cf = cumf[k];
            if (batch) {
                const float fb = (float)b;
                wf = first_win ? fb : wf + fb;
                cf = first_cum ? fb : cf + fb;
                batch[k] = 0;
            }
            cumf[k] = cf;
            winf[k] = 0.f;
            if (snap) snap[k] = wf;
            const u64 w = win64[k] + b;
            const u64 c = cum[k] + w;
            win64[k] = 0;
            cum[k] = c;
            tw += w;
            tc += c;
            if (i >= lo && i < hi) {
                rw += w;
                rc += c;
                rwf += (double)wf;
                rcf += (double)cf;
            }
        }
#pragma unroll
        for (int d = 32; d > 0; d >>= 1) {
            rwf += __shfl_xor(rwf, d, 64);
            rcf += __shfl_xor(rcf, d, 64);
            rw += __shfl_xor(rw, d, 64);
            rc += __shfl_xor(rc, d, 64);
            tw += __shfl_xor(tw, d, 64);
            tc += __shfl_xor(tc, d, 64);
        }
        if (lane == 0) {
            if (cur_img) cur_img[s] = (float)rwf;
            if (cum_img) cum_img[s] = (float)rcf;
            acc[0] += tw;
            acc[1] += rw;
            acc[2] += tc;
            acc[3] += rc;
        }
    }
    if (lane == 0)
        for (int q = 0; q < 4; ++q) s_tot[wid][q] = acc[q];
    __syncthreads();
    if (ovf_dst && blockIdx.x == 0 && threadIdx.x == 4) *ovf_dst = ovf_src ? *ovf_src : 0u;
    if (threadIdx.x < 4)
        totals[4 + (size_t)blockIdx.x * 4 + threadIdx.x] =
            s_tot[0][threadIdx.x] + s_tot[1][threadIdx.x] + s_tot[2][threadIdx.x] + s_tot[3][threadIdx.x];
}


// ---------------------------------------------------------------------------
// Screen-group spectra: ROI spectra (SRC/workflows/detector_view/roi.py:188-266)
// and spectrum views (SRC/workflows/detector_view/providers.py:300-325).
// out[g][t] = sum over the screens s of group g of H[s][t], H = the window
// (mode 0: win32 + win64), the cumulative as finalize would publish it
// (mode 1: cum + win32 + win64) or an integer-valued f32 accumulator (mode 2).
// One block per work item (<= GROUP_ITEM screens of one group); a thread owns
// TOA bins t, t + blockDim, ... and reads the item's rows coalesced along t.
// Groups may overlap (ROIs do), so items of one group add with u64 atomics into
// the zeroed output; integer sums make the result order independent.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(128) void k_group_spectra(
    int mode, const int4 *__restrict__ items, const int *__restrict__ screens, int T,
    const uint32_t *__restrict__ win32, const unsigned long long *__restrict__ win64,
    const unsigned long long *__restrict__ cum, const float *__restrict__ fsrc,
    unsigned long long *__restrict__ out, long long cum32) {
    const int4 it = items[blockIdx.x];  // {group, begin, end, single}
    for (int t = threadIdx.x; t < T; t += blockDim.x) {
        unsigned long long acc = 0;
        int k = it.y;
        for (; k + 4 <= it.z; k += 4) {
            size_t i0 = (size_t)screens[k] * T + t, i1 = (size_t)screens[k + 1] * T + t;
            size_t i2 = (size_t)screens[k + 2] * T + t, i3 = (size_t)screens[k + 3] * T + t;
            if (mode == 2) {
                acc += (unsigned long long)fsrc[i0] + (unsigned long long)fsrc[i1] +
                       (unsigned long long)fsrc[i2] + (unsigned long long)fsrc[i3];
            } else {
                acc += (unsigned long long)win32[i0] + win32[i1] + win32[i2] + win32[i3];
                if (win64) acc += win64[i0] + win64[i1] + win64[i2] + win64[i3];
                if (mode == 1)
                    acc += cum_at(cum, cum32, i0) + cum_at(cum, cum32, i1) + cum_at(cum, cum32, i2) +
                           cum_at(cum, cum32, i3);
            }
        }
        for (; k < it.z; ++k) {
            const size_t i = (size_t)screens[k] * T + t;
            if (mode == 2) {
                acc += (unsigned long long)fsrc[i];
            } else {
                acc += win32[i];
                if (win64) acc += win64[i];
                if (mode == 1) acc += cum_at(cum, cum32, i);
            }
        }
        unsigned long long *o = out + (size_t)it.x * T + t;
        if (it.w)
            *o = acc;  // the group's only item: plain store
        else
            atomicAdd(o, acc);
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

hipError_t launch_merge_f32_u64(const unsigned long long *src, unsigned long long *win64, float *winf,
                                float *cumf, long long n, int first_win, int first_cum,
                                hipStream_t st) {
    hipLaunchKernelGGL(k_merge_f32_u64, dim3(grid_for(n)), dim3(256), 0, st, src, win64, winf, cumf,
                       n, first_win, first_cum);
    return hipGetLastError();
}

hipError_t launch_push_export(uint32_t *batch, unsigned long long *out, long long n, hipStream_t st) {
    hipLaunchKernelGGL(k_push_export, dim3(grid_for(n)), dim3(256), 0, st, batch, out, n);
    return hipGetLastError();
}

hipError_t launch_sum3(const unsigned long long *a, const unsigned long long *b, const uint32_t *c,
                       unsigned long long *out, long long n, hipStream_t st, long long a32) {
    hipLaunchKernelGGL(k_sum3, dim3(grid_for(n)), dim3(256), 0, st, a, b, c, out, n, a32);
    return hipGetLastError();
}

// host_parts (non-null): the per-block partials go there (inside the finalize
// pack) for the host to sum, block 0 copies the overflow flag, and no
// k_sum_totals launch follows; *n_parts = the number of partial blocks.
template <typename OUT>
static void launch_finalize_t(uint32_t *win32, unsigned long long *win64, unsigned long long *cum,
                              unsigned long long *snap, long long S, int T, int lo, int hi,
                              void *cur_img, void *cum_img, unsigned long long *totals,
                              unsigned long long *tot_copy, const uint32_t *ovf_src,
                              uint32_t *ovf_dst, unsigned long long *host_parts, int *n_parts,
                              hipStream_t st, unsigned long long *cumrow, int *cumrow_ok, long long cum32) {
    const bool v4 = T % 4 == 0 && T <= 128;
    const long long rows_per_block = v4 ? 8 : 4;
    long long blocks = (S + rows_per_block - 1) / rows_per_block;
    const long long cap = host_parts ? kHostPartials : (v4 ? 8192 : 2048);
    if (blocks > cap) blocks = cap;
    if (blocks < 1) blocks = 1;
    unsigned long long *dst = host_parts ? host_parts - 4 : totals;  // partial b at dst[4 + 4 b]
    const uint32_t *ks = host_parts ? ovf_src : nullptr;
    uint32_t *kd = host_parts ? ovf_dst : nullptr;
    if (v4)
        hipLaunchKernelGGL(k_finalize_v4<OUT>, dim3((unsigned)blocks), dim3(256), 0, st, win32, win64,
                           cum, snap, S, T, lo, hi, (OUT *)cur_img, (OUT *)cum_img, dst, ks, kd);
    else if (T % 4 == 0) {
        // (the per-screen sums current: empty groups skip the cumulative)
        const bool inc = cumrow && cumrow_ok && *cumrow_ok;
#define LDE_FW4(C, I)                                                                                        \
    hipLaunchKernelGGL((k_finalize_w4<OUT, C, I>), dim3((unsigned)blocks), dim3(256), 0, st, win32, win64, cum, \
                       snap, S, T, lo, hi, (OUT *)cur_img, (OUT *)cum_img, dst, ks, kd, cumrow, C ? cum32 : 0LL)
        if (cum32 && inc) LDE_FW4(true, true);
        else if (cum32) LDE_FW4(true, false);
        else if (inc) LDE_FW4(false, true);
        else LDE_FW4(false, false);
#undef LDE_FW4
    }
    else
        hipLaunchKernelGGL(k_finalize<OUT>, dim3((unsigned)blocks), dim3(256), 0, st, win32, win64,
                           cum, snap, S, T, lo, hi, (OUT *)cur_img, (OUT *)cum_img, dst, ks, kd);
    // the per-screen cumulative sums are current after a wide-row finalize only
    if (cumrow_ok) *cumrow_ok = cumrow && !v4 && T % 4 == 0 ? 1 : 0;
    if (n_parts) *n_parts = (int)blocks;
    if (!host_parts)
        hipLaunchKernelGGL(k_sum_totals, dim3(1), dim3(1024), 0, st, totals, (int)blocks, tot_copy,
                           ovf_src, ovf_dst);
}

// image element type: 0 f64, 2 u64 (exact partial sums for multi-GPU); float32
// views finalize with k_finalize_f32
hipError_t launch_finalize(int img_kind, uint32_t *win32, unsigned long long *win64,
                           unsigned long long *cum, unsigned long long *snap, long long S, int T,
                           int lo, int hi, void *cur_img, void *cum_img,
                           unsigned long long *totals, unsigned long long *tot_copy,
                           const uint32_t *ovf_src, uint32_t *ovf_dst, hipStream_t st,
                           unsigned long long *host_parts, int *n_parts, unsigned long long *cumrow,
                           int *cumrow_ok, long long cum32) {
    if (img_kind == 1) return hipErrorInvalidValue;
    // the split cumulative exists for wide rows only (k_finalize_w4)
    if (cum32 && !(T % 4 == 0 && T > 128)) return hipErrorInvalidValue;
    if (img_kind == 2)
        launch_finalize_t<unsigned long long>(win32, win64, cum, snap, S, T, lo, hi, cur_img,
                                              cum_img, totals, tot_copy, ovf_src, ovf_dst,
                                              host_parts, n_parts, st, cumrow, cumrow_ok, cum32);
    else
        launch_finalize_t<double>(win32, win64, cum, snap, S, T, lo, hi, cur_img, cum_img, totals,
                                  tot_copy, ovf_src, ovf_dst, host_parts, n_parts, st, cumrow, cumrow_ok, cum32);
    return hipGetLastError();
}

hipError_t launch_finalize_f32(uint32_t *batch, unsigned long long *win64, unsigned long long *cum,
                               float *winf, float *cumf, float *snap, long long S, int T, int lo, int hi,
                               int first_win, int first_cum, float *cur_img, float *cum_img,
                               unsigned long long *host_parts, const uint32_t *ovf_src, uint32_t *ovf_dst,
                               int *n_parts, hipStream_t st, hipEvent_t start, hipEvent_t stop) {
    long long blocks = (S + 3) / 4;
    if (blocks > kHostPartials) blocks = kHostPartials;
    if (blocks < 1) blocks = 1;
    hipExtLaunchKernelGGL(k_finalize_f32, dim3((unsigned)blocks), dim3(256), 0, st, start, stop, 0, batch,
                          win64, cum, winf, cumf, snap, S, T, lo, hi, first_win, first_cum, cur_img, cum_img,
                          host_parts - 4, ovf_src, ovf_dst);
    *n_parts = (int)blocks;
    return hipGetLastError();
}

hipError_t launch_group_spectra(int mode, const int4 *items, int n_items, const int *screens,
                                int T, const uint32_t *win32, const unsigned long long *win64,
                                const unsigned long long *cum, const float *fsrc,
                                unsigned long long *out, hipStream_t st, long long cum32) {
    if (n_items <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_group_spectra, dim3((unsigned)n_items), dim3(128), 0, st, mode, items,
                       screens, T, win32, win64, cum, fsrc, out, cum32);
    return hipGetLastError();
}

// Histogram-mode monitors: rebin a float64 histogram onto the view's edges
// and add it into the window and the cumulative accumulator in one pass
// (monitor_workflow.py:101-108 `rebin`, then the accumulator pushes of
// accumulators.py:129-160).  One thread per output bin; source bins in
// ascending order, each adding value * overlap / width (uniform density
// inside a source bin, as scipp's rebin).
__global__ void k_rebin_f64(const double *__restrict__ se, const double *__restrict__ sv, long long ns,
                            const double *__restrict__ de, long long nd, double *__restrict__ out_a,
                            double *__restrict__ out_b) {
    const long long j = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= nd) return;
    const double lo = de[j], hi = de[j + 1];
    // first source bin whose upper edge is above lo
    long long a = 0, b = ns;
    while (a < b) {
        const long long m = (a + b) >> 1;
        if (se[m + 1] <= lo) a = m + 1; else b = m;
    }
    double acc = 0.0;
    for (long long i = a; i < ns && se[i] < hi; ++i) {
        const double xl = se[i], xh = se[i + 1];
        const double ov = fmin(xh, hi) - fmax(xl, lo);
        if (ov > 0.0) acc += sv[i] * ov / (xh - xl);
    }
    if (out_a) out_a[j] += acc;
    if (out_b) out_b[j] += acc;
}

hipError_t launch_rebin_f64(const double *se, const double *sv, long long ns, const double *de,
                            long long nd, double *out_a, double *out_b, hipStream_t st) {
    hipLaunchKernelGGL(k_rebin_f64, dim3((unsigned)((nd + 255) / 256)), dim3(256), 0, st, se, sv, ns,
                       de, nd, out_a, out_b);
    return hipGetLastError();
}

}  // namespace lde
