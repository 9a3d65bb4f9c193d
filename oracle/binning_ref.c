/*
 * binning_ref.c -- CPU oracle / CPU baseline (TEST INFRASTRUCTURE ONLY).
 *
 * Plain-C restatement of the reference's per-batch detector-view pipeline, the
 * work scipp 26.3.1 does in C++/TBB on the reference's hot path
 * (reference = scipp/esslivedata, SRC = src/ess/livedata):
 *
 *   group_event_data   SRC/preprocessors/group_by_pixel.py:46-54
 *       event_id -> pixel index through the detector_number table; unknown ids
 *       dropped.
 *   project_events     SRC/workflows/detector_view/projectors.py:105-152
 *       pixel -> screen index of the batch's replica (precomputed per pixel
 *       from the replica coordinates at setup, as the projector does once per
 *       job).
 *   hist               SRC/workflows/detector_view/providers.py:205-210
 *       int32 TOA compared against float64 edges, half-open [e_i, e_{i+1})
 *       including the last bin, by binary search (std::upper_bound rule).
 *   cumulative +=      SRC/preprocessors/accumulators.py:129-160
 *
 * Counts go to per-thread private histograms (OpenMP) that are summed at the
 * end, like scipp's threaded hist.  Only tests/, smoke() and bench.py's
 * cpu_baseline leg use it; the product path never links or calls it.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* largest b with edges[b] <= x, or -1; x >= edges[T] -> -1 (half-open) */
static inline int64_t toa_bin(double x, const double *edges, int64_t T) {
    if (!(x >= edges[0]) || !(x < edges[T])) return -1; /* also drops NaN */
    int64_t lo = 0, hi = T; /* invariant: edges[lo] <= x < edges[hi] */
    while (hi - lo > 1) {
        const int64_t mid = (lo + hi) >> 1;
        if (edges[mid] <= x) lo = mid; else hi = mid;
    }
    return lo;
}

/*
 * hist[S*T] (uint64) += counts of events (pid, toa) for one batch.
 *   pid_table[pid - pid_offset] = pixel index or -1 (length L)
 *   pixel_screen[pixel]         = screen index of this batch's replica or -1
 * Returns the number of threads used.
 */
int ref_bin_batch(const int32_t *pid, const int32_t *toa, int64_t n, const int64_t *pid_table,
                  int32_t pid_offset, int64_t L, const int64_t *pixel_screen, int64_t S,
                  const double *edges, int64_t T, uint64_t *hist, int threads) {
    const int64_t nb = S * T;
    int used = 1;
#ifdef _OPENMP
    if (threads <= 0) threads = omp_get_max_threads();
    omp_set_num_threads(threads);
#pragma omp parallel
    {
#pragma omp single
        used = omp_get_num_threads();
        uint32_t *priv = (uint32_t *)calloc((size_t)nb, sizeof(uint32_t));
#pragma omp for schedule(static)
        for (int64_t i = 0; i < n; ++i) {
            const int64_t p = (int64_t)pid[i] - pid_offset;
            if (p < 0 || p >= L) continue;
            const int64_t px = pid_table[p];
            if (px < 0) continue;
            const int64_t s = pixel_screen[px];
            if (s < 0) continue;
            const int64_t b = toa_bin((double)toa[i], edges, T);
            if (b < 0) continue;
            priv[s * T + b] += 1u;
        }
#pragma omp critical
        for (int64_t k = 0; k < nb; ++k) hist[k] += priv[k];
        free(priv);
    }
#else
    (void)threads;
    for (int64_t i = 0; i < n; ++i) {
        const int64_t p = (int64_t)pid[i] - pid_offset;
        if (p < 0 || p >= L) continue;
        const int64_t px = pid_table[p];
        if (px < 0) continue;
        const int64_t s = pixel_screen[px];
        if (s < 0) continue;
        const int64_t b = toa_bin((double)toa[i], edges, T);
        if (b < 0) continue;
        hist[s * T + b] += 1u;
    }
#endif
    return used;
}
