// lde_engine.cpp -- host side of the C ABI declared in include/lde.h.
//
// Owns the device state of one detector view / monitor job:
//   LUT  [R][L] int32  screen*T or -1          (setup-time, projectors.py:306-352)
//   TOA thresholds [T+1] int64 + bucket table  (setup-time, providers.py:205-207)
//   window u32 [S*T] (+ u64 fold buffer)       (window accumulator, accumulators.py:138-163)
//   cumulative u64 [S*T]                       (NoCopyAccumulator, accumulators.py:86-135)
//   f32 window/cumulative for LDE_F32 views    (BIFROST, bifrost/specs.py:295)
//   staging: pinned host ring -> device event buffers (ToNXevent_data.add, to_nxevent_data.py:140-153)
//   partition workspace (payload, run starts, plan tables)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <new>
#include <atomic>
#include <chrono>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include <unistd.h>

#include "../../include/lde.h"
#include "lde_internal.h"

namespace {

thread_local std::string g_create_error;

struct Segment {
    const int *pid;
    const int *toa;
    long long n;
};

struct TimedLaunch {
    int kid;
    hipEvent_t a, b;
};

}  // namespace

struct lde_handle {
    int device = 0;
    hipStream_t stream = nullptr;
    bool own_stream = false;
    int cus = 256;

    int pid_off = 0;
    int R = 1;
    long long L = 0;
    bool monitor = false;
    long long S = 1;
    int T = 1;
    long long nbins = 1;
    int out_dtype = LDE_F64;
    int strategy = LDE_STRATEGY_AUTO;
    int range_lo = 0, range_hi = 1;
    lde::ToaParams tp{};

    void *d_lut = nullptr;
    bool lut16 = false;
    unsigned char *d_tab = nullptr;
    int subc = 4;

    uint32_t *d_win32 = nullptr;
    unsigned long long *d_win64 = nullptr;
    unsigned long long *d_cum = nullptr;
    // per screen: cumulative sum in the TOA range | over all bins (2 x S),
    // current when cumrow_ok (kept by the wide-row finalize, launch_finalize)
    unsigned long long *d_cumrow = nullptr;
    int cumrow_ok = 0;
    // > 0: d_cum holds the cumulative in split form (u32 low words, then u32
    // high words, cum32 bins each): integer views with wide rows, whose
    // finalize (k_finalize_w4) then moves 4 bytes of cumulative per bin
    long long cum32 = 0;
    // a finalize enqueued by lde_finalize_begin, read by lde_finalize_end:
    // images to copy out of the pack (not mapped), their element size, and
    // the number of per-block total partials
    bool fin_pending = false;
    void *fin_images[2] = {nullptr, nullptr};
    size_t fin_isz = 8;
    int fin_parts = 0;
    float *d_winf = nullptr;
    float *d_cumf = nullptr;

    // staging
    int *d_spid = nullptr, *d_stoa = nullptr;
    long long stage_cap = 0, staged_host = 0;
    int *h_ppid = nullptr, *h_ptoa = nullptr;
    long long pin_cap = 0;
    hipEvent_t pin_done = nullptr;
    bool pin_pending = false;
    std::vector<Segment> dev_segments;

    // partition workspace
    int tile_bits = 14, n_tiles = 0;
    uint16_t *d_payload = nullptr;
    uint32_t *d_starts = nullptr;
    long long chunk_cap = 0;
    uint32_t *d_part = nullptr;
    int part_rows = 0;
    int part_grid = 0;
    uint32_t *d_ttot = nullptr, *d_tile_items = nullptr, *d_item_count = nullptr;
    uint2 *d_items = nullptr;
    long long items_cap = 0;
    // PAGED workspace
    uint16_t *d_pages = nullptr;
    size_t pages_cap = 0;  // entries
    uint32_t *d_page_tile = nullptr, *d_page_cnt = nullptr, *d_list = nullptr;
    size_t page_meta_cap = 0;  // pages
    uint32_t *d_pool_used = nullptr, *d_cntp = nullptr, *d_evp = nullptr;
    uint32_t *d_tile_pages = nullptr, *d_tile_events = nullptr, *d_tile_base = nullptr;
    uint32_t *d_overflow = nullptr;
    uint4 *d_items4 = nullptr;
    long long items4_cap = 0;
    lde::SegDesc *d_segs = nullptr, *h_segs = nullptr;
    long long segs_cap = 0;
    hipEvent_t segs_done = nullptr;
    bool segs_pending = false;
    long long item_events_override = 0;  // diagnostics: pass-B item size
    // SPLIT (SIEVE event pass, lde_sieve.hip): hot rows in LDS, cold keys
    // through an exact counting sort and a tile pass
    bool split_ok = false;
    int hot_rows = 0;
    int split_grid = 0;
    int cache_bits = 0;
    int hot_refresh = 256;      // re-select a replica's hot set after this many batches
    double split_min_cov = 0.3; // sampled hot fraction below which AUTO stays PAGED
    uint32_t *d_pix_cnt = nullptr;     // [L] sampled events per pixel
    uint32_t *d_row_screen = nullptr;  // [R][kHotMaxRows]
    uint32_t *d_sel_stats = nullptr;   // [R][4]
    uint32_t *d_sample_part = nullptr, *d_screen_cnt = nullptr;
    uint16_t *d_screen_row = nullptr;
    uint32_t *h_sel_stats = nullptr;   // pinned
    std::vector<int> hot_uses;         // per replica: -1 = not selected yet
    std::vector<double> hot_cov;
    std::vector<char> all_hot;         // per replica: every screen has a hot row
    uint32_t *d_hot_part = nullptr;
    size_t hot_part_cap = 0;
    uint32_t *d_cold = nullptr;
    size_t cold_total_cap = 0;
    uint32_t *d_cold_cnt = nullptr;
    uint32_t *d_hot_fmt = nullptr;  // per sieve block: hot rows flushed as u16 (1) or u32 (0)
    unsigned long long *d_trace = nullptr;  // LDE_SIEVE_TRACE: per-block sieve timeline
    std::vector<double> trace_stats;        // per launch: start spread, end spread, mean span (us)
    uint32_t *d_glut = nullptr;       // [R][L + 1] pixel words
    uint32_t *d_sieve_tab = nullptr;  // [R][1 << cache_bits] LDS table images
    std::vector<uint32_t> ttab;       // TOA bucket words (host copy)
    uint32_t *d_ttab = nullptr;
    uint32_t ttab_cap = 0;
    int ttab_shift = 0;
    lde::ChunkPtrs *d_chunk_tab = nullptr;
    size_t chunk_tab_cap = 0;
    int *d_sieve_dummy = nullptr;     // kChunk x (pid_off - 1): the all-invalid chunk
    // SIEVE cold keys: per (block, tile) counts and offsets, tile-major u16 keys, items
    uint32_t *d_cold_tcnt = nullptr, *d_cold_boff = nullptr;
    size_t cold_tcnt_cap = 0, cold_boff_cap = 0;
    uint16_t *d_cold_keys = nullptr;
    size_t cold_keys_cap = 0;
    uint4 *d_cold_items = nullptr;
    size_t cold_items_cap = 0;
    uint32_t *d_cold_ttot = nullptr;  // [n_tiles]
    int sieve_ablate = 0;             // LDE_SIEVE_ABLATE (diagnostics build)
    int cold_sort_ablate = 0;         // LDE_COLD_SORT_ABLATE (diagnostics build)
    // wavelength mode (lde_set_coord_lut): per-pixel distances, the lookup
    // table, the coordinate edges, per-event bin scratch
    bool coord = false;
    lde::CoordArgs cargs{};
    uint16_t *d_cbuck = nullptr;  // coordinate bucket table
    double *d_cpd = nullptr, *d_ctable = nullptr, *d_cedges = nullptr;
    int *d_cbin = nullptr;
    size_t cbin_cap = 0;
    // keyed wavelength pass (SIEVE path): one k_event_key launch emits the
    // sieve's finished words
    double *d_key_dist = nullptr;  // [R][1 << cache_bits] grid coordinate x (or fx) of each slot
    std::vector<char> key_ok;  // per replica: its key tables are current (1: x layout, 2: FAST layout)
    uint8_t *d_key_tabi = nullptr;  // [R][1 << cache_bits] distance row of each slot (FAST pass)
    uint32_t *d_key_rec = nullptr;  // [R][L + 1] x 12 B {word, x} per pixel
    // PIXEL strategy (lde_pixel.hip): pixel-range footprints built from the LUT
    bool pixel_ok = false;
    lde::PixSetup pix{};
    uint16_t *d_ploc = nullptr;
    uint32_t *d_pfp_off = nullptr, *d_pfp_scr = nullptr;
    uint32_t *d_pcounts = nullptr, *d_prstart = nullptr, *d_ppayload = nullptr;
    size_t ppayload_cap = 0;
    uint4 *d_pitems = nullptr;
    size_t pitems_cap = 0;
    lde::PixChunk *d_pctab = nullptr;
    size_t pctab_cap = 0;
    uint32_t *d_pitem_count = nullptr;
    int pix_grid = 0, pix_unit = 2;
    // predicted slots: the last scatter's run totals (d_pprev) size this
    // batch's slots, no count pass
    uint32_t *d_pprev = nullptr, *d_povf = nullptr;
    uint4 *d_povf_grp = nullptr;
    size_t povf_cap = 0;
    long long pix_prev_n = 0, pix_prev_units = 0;
    bool pix_last_pred = false;  // the last PIXEL batch used predicted slots
    int pix_prev_grid = 0;
    std::vector<double> edges;  // the create-time edges (event unit)
    // WIDE strategy (lde_wide.hip): any TOA edges, any S * T < 2^32 bins
    bool wide_ok = false;
    lde::WideToa wtoa{};
    uint32_t *d_wtree = nullptr;
    int wide_levels = 0, wide_pbits = 0, wide_parts = 0, wide_tpb_bits = 0, wide_tiles = 0, wide_cbits = 0;
    std::vector<int> wide_uses;  // per replica: batches since its pixel table was built (-1: none)
    uint32_t *d_wtab = nullptr, *d_wpixcnt = nullptr, *d_wcounters = nullptr;
    lde::PixChunk *d_wctab = nullptr;
    size_t wctab_cap = 0;
    unsigned char *d_wpages1 = nullptr;
    size_t wpages1_cap = 0;  // bytes
    uint16_t *d_wpages2 = nullptr;
    size_t wpages2_cap = 0;  // entries
    uint32_t *d_wpage_cnt = nullptr, *d_wpage_part = nullptr, *d_wlist = nullptr;
    size_t wmeta_cap = 0;  // pages (each of the three arrays)
    uint32_t *d_wrows1 = nullptr, *d_wrows2 = nullptr;
    size_t wrows1_cap = 0, wrows2_cap = 0;  // words
    uint4 *d_witems1 = nullptr, *d_witems2 = nullptr;
    size_t witems1_cap = 0, witems2_cap = 0;
    uint2 *d_wband = nullptr;

    // finalize scratch
    unsigned long long *d_tot4 = nullptr;
    // finalize outputs: [current image S x 8 B][cumulative image S x 8 B]
    // [totals 32 B][overflow flag 16 B][per-block total partials], in coherent
    // host memory the finalize kernel writes directly (hd_pack = its device
    // address): no copy command after the kernel
    unsigned char *h_pack = nullptr, *hd_pack = nullptr;
    hipEvent_t fin_event = nullptr;  // system-scope release after the kernel
    hipEvent_t block_event = nullptr;  // blocking-sync event: waits past the spin budget
    double wait_pred_us = 0.0;         // predicted stream wait of a finalize (EMA)
    long long waits_blocked = 0, waits_total = 0;
    size_t pack_bytes = 0;
    unsigned long long *d_snap = nullptr;

    // screen groupings (ROI spectra, spectrum views), lde_set_groups
    struct GroupSet {
        long long n_groups = 0;
        int n_items = 0;
        bool all_single = true;
        int4 *d_items = nullptr;
        int *d_screens = nullptr;
        unsigned long long *d_out = nullptr;  // [n_groups * T]
    } groups[LDE_MAX_GROUP_SETS];

    // state
    bool window_has_data = false;
    bool cum_has_data = false;
    // float32 views: the last push's counts wait in the u32 batch (d_win32)
    // until the next accumulate merges them or the finalize fuses their f32
    // adds (k_finalize_f32); the first-push flags are those of that push
    bool f32_pending = false;
    int pend_first_win = 0, pend_first_cum = 0;
    bool win64_dirty = false;
    unsigned long long win_events = 0;
    long long events_binned = 0;
    int last_strategy = 0;

    // timing
    hipEvent_t bin_stop_ext = nullptr;  // BINNING stop event for the last kernel to stamp
    bool bin_stop_used = false;
    bool timing = false;
    uint32_t timing_mask = 0xffffffffu;  // LDE_K_* ids recorded while timing
    std::vector<TimedLaunch> launches;
    std::vector<hipEvent_t> event_pool;
    double kms[LDE_K_COUNT] = {};
    long long kcount[LDE_K_COUNT] = {};

    std::string err;
    // LDE_HOST_PROBE: host time from lde_accumulate entry to the sieve launch
    bool probe = false;
    std::chrono::steady_clock::time_point t_acc0;
    double probe_us = 0.0, probe_min = 0.0;
    long long probe_n = 0;
    double probe_fin_post_us = 0.0;  // finalize: from the stream wait's return to the return
    long long probe_fin_n = 0;
};

namespace {

int fail(lde_handle *h, int code, const char *fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    if (h) h->err = buf;
    else g_create_error = buf;
    return code;
}

#define HIPCALL(h, expr)                                                                  \
    do {                                                                                  \
        hipError_t e_ = (expr);                                                           \
        if (e_ != hipSuccess)                                                             \
            return fail((h), LDE_EHIP, "%s failed: %s", #expr, hipGetErrorString(e_));   \
    } while (0)

struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) (void)hipSetDevice(dev);
    }
    ~DeviceGuard() {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
};

// Runtime settings.  The product library reads only the documented
// deployment settings below; every tuning knob of the engine (strategy
// internals, kernel variants, probes) is fixed at its measured default and
// selectable only in the diagnostics build (-DLDE_DIAGNOSTICS,
// libesslivedata_amd_diag.so), which the parity tests load to run every
// exact variant (tests/test_gpu_parity.py VARIANTS).
//   LDE_VERBOSE        setup and strategy lines on stderr
//   LDE_STAGE_THREADS  host threads copying ev44 payloads into the pinned ring
bool runtime_setting(const char *name) {
#ifdef LDE_DIAGNOSTICS
    (void)name;
    return true;
#else
    return std::strcmp(name, "LDE_VERBOSE") == 0 || std::strcmp(name, "LDE_STAGE_THREADS") == 0;
#endif
}

long long env_ll(const char *name, long long dflt) {
    if (!runtime_setting(name)) return dflt;
    const char *v = std::getenv(name);
    if (!v || !*v) return dflt;
    return std::atoll(v);
}

// Diagnostic ablations produce wrong counts by design; the product library
// has none compiled in and refuses the variables that would select them.
// Any other LDE_* variable only changes how the engine computes (every knob
// is exact); they are named once on stderr so a stray one is visible.
int check_knobs() {
#ifndef LDE_DIAGNOSTICS
    static const char *const diag[] = {"LDE_ABLATE", "LDE_SIEVE_ABLATE", "LDE_COLD_SORT_ABLATE",
                                       "LDE_PIX_ABLATE", "LDE_KEY_ABLATE", "LDE_WIDE_ABLATE"};
    for (const char *n : diag)
        if (const char *v = std::getenv(n); v && std::atoll(v) != 0)
            return fail(nullptr, LDE_EINVAL,
                        "%s selects a diagnostic ablation (wrong results by design), which only "
                        "the LDE_DIAGNOSTICS build has",
                        n);
#endif
    static std::once_flag once;
    std::call_once(once, [] {
        std::string used, ignored;
        for (char **e = environ; e && *e; ++e)
            if (std::strncmp(*e, "LDE_", 4) == 0) {
                std::string n(*e, std::strcspn(*e, "="));
                // host-side (Python) settings are not the engine's
                if (n == "LDE_LIBRARY" || n == "LDE_BENCH_BACKEND" || n == "LDE_BENCH_UNTIMED" ||
                    n == "LDE_OFFLOAD_ARCH")
                    continue;
                (runtime_setting(n.c_str()) ? used : ignored) += ' ' + n;
            }
#ifdef LDE_DIAGNOSTICS
        if (!used.empty()) used += " [diagnostics build]";
#endif
        if (!used.empty()) fprintf(stderr, "lde: engine settings from the environment:%s\n", used.c_str());
        if (!ignored.empty())
            fprintf(stderr, "lde: ignored (tuning knobs exist only in the diagnostics build):%s\n",
                    ignored.c_str());
    });
    return LDE_OK;
}

// Wait for the handle's stream.  Finalize returns results the caller waits
// for, so the wake-up latency is GPU idle time before the next batch, but a
// thread spinning through the whole wait burns a host core per job (the
// reference service runs job_threads=5 jobs, service_factory.py:65).  So:
//   * sleep through the predicted part of the wait (EMA of this handle's past
//     waits) minus a wake-up margin, then
//   * spin on hipStreamQuery for the last stretch, at most kSpinCapUs, then
//   * block on an interrupt-driven (hipEventBlockingSync) event.
// A steady stream of batches spins ~kWakeUs per finalize; a wait with no
// history, or longer than predicted, spins kSpinCapUs and then sleeps.
// ev (optional): wait for that event instead of the whole stream (created
// with hipEventBlockingSync, so the blocking fallback sleeps on it)
hipError_t wait_stream(lde_handle *h, hipEvent_t ev = nullptr) {
    using clk = std::chrono::steady_clock;
    constexpr double kWakeUs = 100.0;    // wake this long before the predicted end
    constexpr double kSpinCapUs = 150.0; // spin budget before the blocking wait
    auto query = [&]() { return ev ? hipEventQuery(ev) : hipStreamQuery(h->stream); };
    hipError_t e = query();
    if (e != hipErrorNotReady) return e;
    ++h->waits_total;
    const auto t0 = clk::now();
    auto since = [](clk::time_point t) {
        return std::chrono::duration<double, std::micro>(clk::now() - t).count();
    };
    const double pred = h->wait_pred_us;
    if (pred > 2.0 * kWakeUs) {
        std::this_thread::sleep_for(std::chrono::microseconds((long long)(pred - kWakeUs)));
        e = query();
        if (e != hipErrorNotReady) {
            // done before the wake-up: the end is unknown, so the prediction
            // drops to half the time slept at once (a load drop, e.g. a 5 ms
            // wait becoming 0.5 ms, must not oversleep finalize after finalize;
            // the spin phase re-learns the true wait from the next one)
            h->wait_pred_us = 0.5 * since(t0);
            return e;
        }
    }
    const auto ts = clk::now();
    bool blocked = false;
    while ((e = query()) == hipErrorNotReady) {
        if (since(ts) > kSpinCapUs) {
            blocked = true;
            ++h->waits_blocked;
            if (ev) {
                e = hipEventSynchronize(ev);
                break;
            }
            if (!h->block_event) {
                e = hipEventCreateWithFlags(&h->block_event,
                                            hipEventBlockingSync | hipEventDisableTiming);
                if (e != hipSuccess) {
                    h->block_event = nullptr;
                    return hipStreamSynchronize(h->stream);
                }
            }
            e = hipEventRecord(h->block_event, h->stream);
            if (e == hipSuccess) e = hipEventSynchronize(h->block_event);
            break;
        }
    }
    const double took = since(t0);
    // a blocked wait ends late by the wake-up latency: learn from it too
    h->wait_pred_us = pred <= 0.0 ? took : 0.7 * pred + 0.3 * (blocked ? 0.9 * took : took);
    return e;
}


template <typename T>
int dev_alloc(lde_handle *h, T **p, size_t count) {
    *p = nullptr;
    if (count == 0) count = 1;
    hipError_t e = hipMalloc((void **)p, count * sizeof(T));
    if (e != hipSuccess) {
        *p = nullptr;
        return fail(h, LDE_ENOMEM, "hipMalloc(%zu bytes) failed: %s", count * sizeof(T),
                    hipGetErrorString(e));
    }
    return LDE_OK;
}

template <typename T>
void dev_free(T *&p) {
    if (p) (void)hipFree((void *)p);
    p = nullptr;
}

// ---- TOA edge preprocessing (exact f64 -> int thresholds) -----------------
long long ceil_clamped(double e) {
    // t (int32) >= e  <=>  t >= ceil(e); clamp into [INT32_MIN, INT32_MAX + 1]
    const double lo = -2147483648.0, hi = 2147483648.0;
    if (e <= lo) return (long long)lo;
    if (e >= hi) return (long long)hi;
    return (long long)std::ceil(e);
}

// bin(x) = largest b in [0, T-1] with thr[b] <= x (x in [lo, hi))
static int bin_of(const std::vector<long long> &thr, int T, long long x) {
    int b = (int)(std::upper_bound(thr.begin(), thr.begin() + T, x) - thr.begin()) - 1;
    return std::max(0, std::min(b, T - 1));
}

// Builds the LDS image of the TOA lookup (layouts documented in lde_binning.hip).
int build_toa_tables(lde_handle *h, const double *edges, int T, std::vector<unsigned char> &img,
                     lde::ToaParams &tp) {
    if (!edges) return fail(h, LDE_EINVAL, "toa_edges is NULL");
    if (T < 1 || T > 65535) return fail(h, LDE_EINVAL, "n_toa_bins=%d out of range [1, 65535]", T);
    for (int i = 0; i <= T; ++i) {
        if (!std::isfinite(edges[i]))
            return fail(h, LDE_EINVAL, "toa edge %d is not finite", i);
        if (i > 0 && edges[i] < edges[i - 1])
            return fail(h, LDE_EINVAL, "toa edges must be sorted (edge %d < edge %d)", i, i - 1);
    }
    std::vector<long long> thr(T + 1);
    for (int i = 0; i <= T; ++i) thr[i] = ceil_clamped(edges[i]);
    std::memset(&tp, 0, sizeof tp);
    tp.T = T;
    tp.lo = thr[0];
    tp.hi = thr[T];
    const long long span = tp.hi - tp.lo;  // 0 .. 2^32
    // fast layout: u32 relative thresholds, buckets narrower than every bin
    if (span >= 1 && span <= 0xffffffffLL && tp.lo <= 0x7fffffffLL &&
        !(runtime_setting("LDE_TOA_GENERAL") && std::getenv("LDE_TOA_GENERAL") != nullptr)) {
        long long min_width = span;
        for (int i = 0; i < T; ++i)
            if (thr[i + 1] > thr[i]) min_width = std::min(min_width, thr[i + 1] - thr[i]);
        int shift = 0;
        while ((2LL << shift) <= min_width) ++shift;  // 2^shift <= min non-empty bin width
        while (((span - 1) >> shift) >= lde::kMaxFastBuckets) ++shift;
        const int G = (int)(((span - 1) >> shift) + 1);
        std::vector<uint16_t> bst(G);
        bool one_step = true;
        for (int g = 0; g < G && one_step; ++g) {
            const long long x0 = tp.lo + ((long long)g << shift);
            long long x1 = std::min(tp.lo + (((long long)g + 1) << shift) - 1, tp.hi - 1);
            const int b0 = bin_of(thr, T, x0), b1 = bin_of(thr, T, x1);
            if (b1 - b0 > 1) one_step = false;
            bst[g] = (uint16_t)b0;
        }
        if (one_step) {
            tp.fast = 1;
            tp.span = (unsigned)span;
            tp.shift = shift;
            tp.G = G;
            img.assign(lde::toa_lds_bytes(tp), 0);
            uint32_t *rthr = reinterpret_cast<uint32_t *>(img.data());
            for (int i = 0; i <= T; ++i) rthr[i] = (uint32_t)(thr[i] - tp.lo);
            std::memcpy(img.data() + lde::align16((size_t)(T + 1) * 4), bst.data(), (size_t)G * 2);
            return LDE_OK;
        }
    }
    // general layout: int64 thresholds + (first, last) candidate bins per bucket
    int shift = 0;
    while (span > 0 && ((span - 1) >> shift) >= lde::kMaxBuckets) ++shift;
    tp.fast = 0;
    tp.shift = shift;
    tp.G = span > 0 ? (int)(((span - 1) >> shift) + 1) : 1;
    img.assign(lde::toa_lds_bytes(tp), 0);
    std::memcpy(img.data(), thr.data(), (size_t)(T + 1) * 8);
    uint32_t *bp = reinterpret_cast<uint32_t *>(img.data() + lde::align16((size_t)(T + 1) * 8));
    for (int g = 0; g < tp.G; ++g) {
        const long long x0 = tp.lo + ((long long)g << shift);
        long long x1 = tp.lo + (((long long)g + 1) << shift) - 1;
        if (x1 > tp.hi - 1) x1 = tp.hi - 1;
        const int b0 = span > 0 ? bin_of(thr, T, x0) : 0;
        const int b1 = span > 0 ? bin_of(thr, T, std::max(x0, x1)) : 0;
        bp[g] = (uint32_t)b0 | ((uint32_t)b1 << 16);
    }
    return LDE_OK;
}

// SIEVE TOA image: one u32 per bucket, (offset of the next threshold inside
// the bucket, capped at the bucket width) << 8 | bin of the bucket start.
// Buckets (2^shift2 wide, the fast layout's) hold at most one threshold, so
// bin = (w & 0xFF) + (offset of d in its bucket >= (w >> 8)); d >= span (and
// TOAs before the first edge, which wrap) clamp to `cap` and land on a word
// whose bin comes out as T (dropped).  (Log-linear buckets, 2^M per octave,
// were measured +-0 in round 3 and removed in round 5.)
bool build_sieve_toa(const lde::ToaParams &tp, const std::vector<unsigned char> &img,
                     std::vector<uint32_t> &words, int &shift2, uint32_t &cap) {
    if (!tp.fast || tp.T > lde::kSieveMaxT || tp.span == 0) return false;
    const uint32_t *rthr = reinterpret_cast<const uint32_t *>(img.data());
    const int T = tp.T;
    shift2 = std::min(tp.shift, 23);
    const unsigned long long span = tp.span;
    const unsigned long long G = ((span - 1) >> shift2) + 1;
    if (G > (unsigned long long)lde::kMaxFastBuckets) return false;
    const unsigned long long W = 1ULL << shift2;
    words.assign((size_t)lde::align4((int)G + 1), 0u);
    int b = 0;
    for (unsigned long long g = 0; g < G; ++g) {
        const unsigned long long start = g << shift2;
        while (b + 1 < T && rthr[b + 1] <= start) ++b;
        // the fast layout guarantees one threshold per bucket at most
        const unsigned long long nxt = rthr[b + 1] > start ? rthr[b + 1] - start : 0;
        words[(size_t)g] = (uint32_t)(std::min<unsigned long long>(nxt, W) << 8) | (uint32_t)b;
    }
    words[(size_t)G] = 0xFFu;
    cap = (G << shift2) > 0xffffffffULL ? 0xffffffffu : (uint32_t)(G << shift2);
    return true;
}

// WIDE TOA tree (lde_internal.h WideToa) over the integer thresholds thr[0..T]
// of the edges.  A bucket [x, x + 2^sh) is a leaf when at most one threshold
// lies strictly inside it; its word holds the bin at x (the largest b < T with
// thr[b] - lo <= x) and that threshold's offset from the start of its ROOT
// bucket, so the kernel needs no per-level width.  A bucket with two or more
// (equal thresholds count separately) becomes 2^fb children of width
// 2^max(0, sh - fb); a width-1 bucket never holds one inside, so the descent
// ends.  (sh0, fb) are chosen for the fewest words (LDS first), then the
// shallowest tree.
struct WideTreeBuilder {
    const std::vector<long long> &r;  // thresholds relative to lo, r[0] = 0
    int T, sh0, fb;
    std::vector<uint32_t> words;
    int depth = 0;
    bool ok = true;
    WideTreeBuilder(const std::vector<long long> &r_, int T_, int sh0_, int fb_) : r(r_), T(T_), sh0(sh0_), fb(fb_) {}
    // bin at x: largest b in [0, T - 1] with r[b] <= x
    int bin_at(long long x) const {
        const int b = (int)(std::upper_bound(r.begin(), r.begin() + T, x) - r.begin()) - 1;
        return std::max(0, std::min(b, T - 1));
    }
    // thresholds r[1..T-1] strictly inside [x, x + w): indices [a, e)
    void inside(long long x, long long w, int &a, int &e) const {
        a = (int)(std::upper_bound(r.begin() + 1, r.begin() + T, x) - r.begin());
        e = (int)(std::upper_bound(r.begin() + 1, r.begin() + T, x + w - 1) - r.begin());
    }
    // word of bucket [x, x + 2^sh) at level lv; root_x: its root bucket's start
    uint32_t node(long long x, int sh, int lv, long long root_x) {
        int a, e;
        inside(x, 1LL << sh, a, e);
        const uint32_t b0 = (uint32_t)bin_at(x);
        if (e - a == 0) {
            depth = std::max(depth, lv);
            return b0 | (0xFFFFu << 16);
        }
        if (e - a == 1) {
            depth = std::max(depth, lv);
            return b0 | ((uint32_t)(r[(size_t)a] - root_x) << 16);
        }
        const int F = 1 << fb;
        const size_t base = words.size();
        if (base + (size_t)F > 0xFFFFu || lv >= 32) {
            ok = false;
            return 0;
        }
        words.resize(base + (size_t)F);
        const int csh = std::max(0, sh - fb);
        for (int k = 0; k < F && ok; ++k) {
            // nodes narrower than the fan-out: child k is position (x & ~(F - 1)) + k
            // (the kernel indexes width-1 children by the low fb bits of d)
            const long long cx = sh >= fb ? x + ((long long)k << csh) : (x & ~(long long)(F - 1)) + k;
            words[base + (size_t)k] = node(cx, csh, lv + 1, root_x);
        }
        return 0xFFFFu | ((uint32_t)base << 16);
    }
    // reads of words at index >= from per event, for TOAs spread evenly over
    // the span (from = kWideTreeLds: the reads past the kernel's LDS copy of a
    // tree too large for LDS; 0: all reads)
    double reads(long long span, size_t from) const {
        const long long nroot = (span + (1LL << sh0) - 1) >> sh0;
        const int F = 1 << fb;
        double c = 0;
        struct Walk {
            const std::vector<uint32_t> &w;
            int F;
            size_t from;
            double cost(uint32_t word, double wt) const {
                if ((word & 0xFFFFu) != 0xFFFFu) return 0;  // a leaf
                const uint32_t base = word >> 16;
                double c = 0;
                for (int k = 0; k < F; ++k) {
                    const size_t i = (size_t)base + (size_t)k;
                    c += (i >= from ? wt / F : 0) + cost(w[i], wt / F);
                }
                return c;
            }
        } walk{words, F, from};
        for (long long g = 0; g < nroot; ++g) {
            const double wt = (double)std::min<long long>(1LL << sh0, span - (g << sh0)) / (double)span;
            c += ((size_t)g >= from ? wt : 0) + walk.cost(words[(size_t)g], wt);
        }
        return c;
    }
    bool build(long long span) {
        const long long nroot = (span + (1LL << sh0) - 1) >> sh0;
        if (nroot > 0xFFFF) return false;
        words.assign((size_t)nroot, 0u);
        for (long long g = 0; g < nroot && ok; ++g) {
            const uint32_t w = node(g << sh0, sh0, 0, g << sh0);
            words[(size_t)g] = w;
        }
        return ok;
    }
};

bool build_wide_tree(const std::vector<double> &edges, int T, std::vector<uint32_t> &tree, lde::WideToa &wt) {
    std::vector<long long> thr((size_t)T + 1);
    for (int i = 0; i <= T; ++i) thr[(size_t)i] = ceil_clamped(edges[(size_t)i]);
    const long long lo = thr[0], span = thr[(size_t)T] - thr[0];
    std::memset(&wt, 0, sizeof wt);
    wt.lo = (uint32_t)lo;
    wt.fb = 2;
    if (span <= 0) {  // no event can be in range
        wt.empty = 1;
        tree.assign(4, 0u);
        wt.words = 1;
        return true;
    }
    if (span > (1LL << 31)) return false;  // root buckets <= 2^15 wide, at most 65535 of them
    wt.last = (uint32_t)(span - 1);
    std::vector<long long> r((size_t)T + 1);
    for (int i = 0; i <= T; ++i) r[(size_t)i] = thr[(size_t)i] - lo;
    size_t best = ~(size_t)0;
    int bsh = -1, bfb = 0, bdepth = 0;
    double bl2 = 0;
    const bool shallow = env_ll("LDE_WIDE_TREE_SHALLOW", 1) != 0;  // (diagnostics: 0 = fewest words)
    // (diagnostics: 0 = a tree past LDS takes the fewest words)
    const bool hybrid = env_ll("LDE_WIDE_TREE_L2PICK", 1) != 0;
    for (int sh0 = 15; sh0 >= 0; --sh0) {
        if (((span + (1LL << sh0) - 1) >> sh0) > 0xFFFF) break;
        for (int fb = 2; fb <= 4; ++fb) {
            WideTreeBuilder b(r, T, sh0, fb);
            if (!b.build(span)) continue;
            const size_t n = b.words.size();
            // LDS-sized trees first; among those the shallowest (every level
            // below the root is one more dependent LDS read for the waves
            // whose events reach it: DREAM's 1000 log bins, 20 % of the
            // events in three narrow hot bins, took a second level in every
            // wave), then the fewest words; trees too large for LDS: the
            // fewest reads past the LDS copy of their first kWideTreeLds words
            // (for TOAs spread evenly), then the fewest words
            const bool fits = n <= (size_t)lde::kWideTreeLds, bfits = best <= (size_t)lde::kWideTreeLds;
            const double l2 = fits ? 0.0 : (hybrid ? b.reads(span, (size_t)lde::kWideTreeLds) : 0.0);
            const bool better = fits && shallow ? (b.depth < bdepth || (b.depth == bdepth && n < best))
                                : !fits && hybrid ? (l2 < bl2 - 1e-6 || (l2 <= bl2 + 1e-6 && n < best))
                                                  : n < best;
            if (bsh < 0 || (fits && !bfits) || (fits == bfits && better)) {
                best = n;
                bsh = sh0;
                bfb = fb;
                bdepth = b.depth;
                bl2 = l2;
                tree = std::move(b.words);
            }
        }
    }
    if (bsh < 0) return false;
    wt.sh0 = bsh;
    wt.fb = bfb;
    wt.depth = bdepth;
    wt.words = (int)tree.size();
    tree.resize((size_t)lde::align4(wt.words), 0u);
    return true;
}

// ---- timing ----------------------------------------------------------------
hipEvent_t pool_event(lde_handle *h) {
    if (!h->event_pool.empty()) {
        hipEvent_t e = h->event_pool.back();
        h->event_pool.pop_back();
        return e;
    }
    hipEvent_t e = nullptr;
    // timing-only events: no system-scope fence (cache write-back and
    // invalidate) at every stamped dispatch (LDE_EVENT_FLAGS overrides)
    static const unsigned flags = (unsigned)env_ll("LDE_EVENT_FLAGS", hipEventDisableSystemFence);
    if (hipEventCreateWithFlags(&e, flags) != hipSuccess) return nullptr;
    return e;
}

struct Timed {
    lde_handle *h;
    int kid;
    hipEvent_t a = nullptr;
    Timed(lde_handle *h_, int kid_) : h(h_), kid(kid_) {
        if (h->timing && ((h->timing_mask >> kid) & 1u)) {
            a = pool_event(h);
            if (a) (void)hipEventRecord(a, h->stream);
        }
    }
    ~Timed() {
        if (a) {
            hipEvent_t b = pool_event(h);
            if (b) {
                (void)hipEventRecord(b, h->stream);
                h->launches.push_back({kid, a, b});
            } else {
                h->event_pool.push_back(a);
            }
        }
    }
};

// Timing of a span of launches by the dispatches themselves: `a` is stamped
// by the span's first dispatch, `b` by its last (hipExtLaunchKernelGGL), so no
// marker packets sit between kernels (unlike Timed).  The launcher must stamp
// both (or record them) when the span is non-empty.
struct Stamp {
    lde_handle *h;
    int kid;
    hipEvent_t a = nullptr, b = nullptr;
    Stamp(lde_handle *h_, int kid_) : h(h_), kid(kid_) {
        if (h->timing && ((h->timing_mask >> kid) & 1u)) {
            a = pool_event(h);
            b = a ? pool_event(h) : nullptr;
            if (a && !b) {
                h->event_pool.push_back(a);
                a = nullptr;
            }
        }
    }
    // set once the stamped launch succeeded: a launch that failed recorded
    // neither event, so they go back to the pool instead of being resolved
    bool done = false;
    ~Stamp() {
        if (!a) return;
        if (done) {
            h->launches.push_back({kid, a, b});
        } else {
            h->event_pool.push_back(a);
            h->event_pool.push_back(b);
        }
    }
};

void resolve_timing(lde_handle *h) {
    for (auto &l : h->launches) {
        float ms = 0.f;
        if (hipEventSynchronize(l.b) == hipSuccess && hipEventElapsedTime(&ms, l.a, l.b) == hipSuccess) {
            h->kms[l.kid] += ms;
            h->kcount[l.kid] += 1;
        }
        h->event_pool.push_back(l.a);
        h->event_pool.push_back(l.b);
    }
    h->launches.clear();
}

// ---- staging ---------------------------------------------------------------
int ensure_stage_capacity(lde_handle *h, long long need) {
    if (need <= h->stage_cap && need <= h->pin_cap) return LDE_OK;
    long long cap = std::max<long long>(need, std::max<long long>(2 * h->stage_cap, 1 << 20));
    HIPCALL(h, hipStreamSynchronize(h->stream));
    int *np = nullptr, *nt = nullptr;
    if (!h->monitor) {
        if (int rc = dev_alloc(h, &np, cap)) return rc;
    }
    if (int rc = dev_alloc(h, &nt, cap)) {
        dev_free(np);
        return rc;
    }
    if (h->staged_host > 0) {
        if (!h->monitor)
            HIPCALL(h, hipMemcpy(np, h->d_spid, h->staged_host * 4, hipMemcpyDeviceToDevice));
        HIPCALL(h, hipMemcpy(nt, h->d_stoa, h->staged_host * 4, hipMemcpyDeviceToDevice));
    }
    dev_free(h->d_spid);
    dev_free(h->d_stoa);
    h->d_spid = np;
    h->d_stoa = nt;
    h->stage_cap = cap;
    // pinned host ring (previous content already copied to the device)
    if (h->h_ppid) (void)hipHostFree(h->h_ppid);
    if (h->h_ptoa) (void)hipHostFree(h->h_ptoa);
    h->h_ppid = h->h_ptoa = nullptr;
    h->pin_cap = 0;
    if (!h->monitor) HIPCALL(h, hipHostMalloc((void **)&h->h_ppid, cap * 4, hipHostMallocDefault));
    HIPCALL(h, hipHostMalloc((void **)&h->h_ptoa, cap * 4, hipHostMallocDefault));
    h->pin_cap = cap;
    h->pin_pending = false;
    return LDE_OK;
}

int ensure_partition_capacity(lde_handle *h, long long chunks, long long max_items) {
    if (chunks > h->chunk_cap) {
        long long cap = std::max(chunks, 2 * h->chunk_cap);
        HIPCALL(h, hipStreamSynchronize(h->stream));
        dev_free(h->d_payload);
        dev_free(h->d_starts);
        if (int rc = dev_alloc(h, &h->d_payload, (size_t)cap * lde::kChunk)) return rc;
        if (int rc = dev_alloc(h, &h->d_starts, (size_t)cap * (h->n_tiles + 1))) return rc;
        h->chunk_cap = cap;
    }
    if (max_items > h->items_cap) {
        long long cap = std::max(max_items, 2 * h->items_cap);
        HIPCALL(h, hipStreamSynchronize(h->stream));
        dev_free(h->d_items);
        if (int rc = dev_alloc(h, &h->d_items, (size_t)cap)) return rc;
        h->items_cap = cap;
    }
    return LDE_OK;
}

bool aligned16(const void *p) { return ((uintptr_t)p & 15u) == 0; }

// ---- binning ---------------------------------------------------------------
int ensure_segs_cap(lde_handle *h, long long n) {
    if (n <= h->segs_cap && h->d_segs) return LDE_OK;
    if (h->segs_pending) {
        HIPCALL(h, hipEventSynchronize(h->segs_done));
        h->segs_pending = false;
    }
    {
        HIPCALL(h, hipStreamSynchronize(h->stream));
        dev_free(h->d_segs);
        if (h->h_segs) (void)hipHostFree(h->h_segs);
        h->h_segs = nullptr;
        h->segs_cap = 0;
        const long long cap = std::max<long long>(n, 256);
        if (int rc = dev_alloc(h, &h->d_segs, (size_t)cap)) return rc;
        HIPCALL(h, hipHostMalloc((void **)&h->h_segs, cap * sizeof(lde::SegDesc), hipHostMallocDefault));
        h->segs_cap = cap;
    }
    return LDE_OK;
}

int upload_segments(lde_handle *h, const std::vector<lde::SegDesc> &sd) {
    if (h->segs_pending) {
        HIPCALL(h, hipEventSynchronize(h->segs_done));
        h->segs_pending = false;
    }
    if (int rc = ensure_segs_cap(h, (long long)sd.size())) return rc;
    std::memcpy(h->h_segs, sd.data(), sd.size() * sizeof(lde::SegDesc));
    HIPCALL(h, hipMemcpyAsync(h->d_segs, h->h_segs, sd.size() * sizeof(lde::SegDesc),
                              hipMemcpyHostToDevice, h->stream));
    HIPCALL(h, hipEventRecord(h->segs_done, h->stream));
    h->segs_pending = true;
    return LDE_OK;
}

template <typename T>
int grow(lde_handle *h, T **p, size_t &cap, size_t need) {
    if (need <= cap && *p) return LDE_OK;
    HIPCALL(h, hipStreamSynchronize(h->stream));
    dev_free(*p);
    const size_t n = std::max(need, cap * 2);
    if (int rc = dev_alloc(h, p, n)) return rc;
    cap = n;
    return LDE_OK;
}

// PAGED pass A + plan + pass B over `segs` (device table).
int paged_core(lde_handle *h, const lde::SegDesc *segs, int n_segs, long long chunks,
               long long total, const void *lut) {
    const int grid = (int)std::min<long long>(chunks, (long long)h->part_grid);
    const long long per_block = (chunks + grid - 1) / grid;
    const int cap = (int)((per_block * lde::kChunk + lde::kPage - 1) / lde::kPage) + 2 * h->n_tiles + 2;
    const size_t pages = (size_t)grid * (size_t)cap;
    if (pages > 0xffffffffULL) return fail(h, LDE_EINVAL, "batch too large for the page pool");
    // pass-B work items: as many as fit resident at once (as for the SIEVE
    // cold keys), every item pays a flush of its whole tile
    const long long resident =
        (long long)h->cus * std::max<long long>(1, (160LL * 1024) / (4LL << h->tile_bits));
    const long long per_items = std::max<long long>(h->cus, resident - h->n_tiles);
    long long item_events = h->item_events_override > 0
                                ? h->item_events_override
                                : std::max<long long>(32768, (total + per_items - 1) / per_items);
    if (item_events > 0x7fffffffLL) item_events = 0x7fffffffLL;
    const long long max_items = (total + item_events - 1) / item_events + h->n_tiles;
    if (int rc = grow(h, &h->d_pages, h->pages_cap, pages * lde::kPage)) return rc;
    if (pages > h->page_meta_cap || !h->d_page_tile) {
        HIPCALL(h, hipStreamSynchronize(h->stream));
        const size_t n = std::max(pages, h->page_meta_cap * 2);
        dev_free(h->d_page_tile);
        dev_free(h->d_page_cnt);
        dev_free(h->d_list);
        h->page_meta_cap = 0;
        if (int rc = dev_alloc(h, &h->d_page_tile, n)) return rc;
        if (int rc = dev_alloc(h, &h->d_page_cnt, n)) return rc;
        if (int rc = dev_alloc(h, &h->d_list, n)) return rc;
        h->page_meta_cap = n;
    }
    if (!h->d_pool_used) {
        const size_t rows = (size_t)h->part_rows;
        if (int rc = dev_alloc(h, &h->d_pool_used, rows)) return rc;
        if (int rc = dev_alloc(h, &h->d_cntp, rows * h->n_tiles)) return rc;
        if (int rc = dev_alloc(h, &h->d_evp, rows * h->n_tiles)) return rc;
        if (int rc = dev_alloc(h, &h->d_tile_pages, (size_t)h->n_tiles)) return rc;
        if (int rc = dev_alloc(h, &h->d_tile_events, (size_t)h->n_tiles)) return rc;
        if (int rc = dev_alloc(h, &h->d_tile_base, (size_t)h->n_tiles)) return rc;
        if (int rc = dev_alloc(h, &h->d_overflow, 1)) return rc;
        HIPCALL(h, hipMemsetAsync(h->d_overflow, 0, 4, h->stream));
    }
    size_t icap = (size_t)h->items4_cap;
    if (int rc = grow(h, &h->d_items4, icap, (size_t)max_items)) return rc;
    h->items4_cap = (long long)icap;
    lde::PagedArgs a;
    a.tile_bits = h->tile_bits;
    a.lut16 = h->lut16;
    a.subc = h->subc;
    a.segs = segs;
    a.n_segs = n_segs;
    a.n_chunks = chunks;
    a.lut = lut;
    a.pid_off = h->pid_off;
    a.L = (unsigned)h->L;
    a.tab = h->d_tab;
    a.tp = h->tp;
    a.n_tiles = h->n_tiles;
    a.pages = h->d_pages;
    a.page_tile = h->d_page_tile;
    a.page_cnt = h->d_page_cnt;
    a.pool_used = h->d_pool_used;
    a.cap = cap;
    a.overflow = h->d_overflow;
    a.grid = grid;
    {
        Timed tm(h, LDE_K_PAGED);
        HIPCALL(h, lde::launch_paged_partition(a, h->stream));
    }
    {
        Timed tm(h, LDE_K_PAGE_PLAN);
        HIPCALL(h, lde::launch_page_plan(a, (uint32_t)item_events, h->d_cntp, h->d_evp,
                                         h->d_tile_pages, h->d_tile_events, h->d_tile_base,
                                         h->d_items4, h->d_item_count, (uint32_t)max_items,
                                         h->d_list, h->stream));
    }
    {
        Timed tm(h, LDE_K_PAGE_ACC);
        HIPCALL(h, lde::launch_page_accumulate(h->tile_bits, a, h->d_list, h->d_items4,
                                               h->d_item_count, h->d_win32, h->nbins,
                                               (int)max_items, h->stream));
    }
    return LDE_OK;
}

int bin_paged(lde_handle *h, const std::vector<lde::SegDesc> &sd, long long chunks,
              long long total, const void *lut) {
    if (int rc = upload_segments(h, sd)) return rc;
    return paged_core(h, h->d_segs, (int)sd.size(), chunks, total, lut);
}

// Wavelength mode, bin stream: every event's coordinate bin (k_event_coord)
// replaces its time, contiguously in d_cbin, for the non-keyed strategies.
int coord_prepass(lde_handle *h, std::vector<Segment> &segs) {
    long long total = 0;
    for (const Segment &s : segs) total += s.n;
    if (total == 0) return LDE_OK;
    if (int rc = grow(h, &h->d_cbin, h->cbin_cap, (size_t)total)) return rc;
    long long off = 0;
    Timed tm(h, LDE_K_COORD);
    for (Segment &s : segs) {
        HIPCALL(h, lde::launch_event_coord(h->cargs, s.pid, s.toa, s.n, h->d_cbin + off, h->stream));
        s.toa = h->d_cbin + off;
        off += s.n;
    }
    return LDE_OK;
}

int coord_prepass(lde_handle *h, std::vector<lde::SegDesc> &sd) {
    std::vector<Segment> segs;
    for (const lde::SegDesc &d : sd) segs.push_back({d.pid, d.toa, d.n});
    if (int rc = coord_prepass(h, segs)) return rc;
    for (size_t i = 0; i < sd.size(); ++i) sd[i].toa = segs[i].toa;
    return LDE_OK;
}

// AUTO: the partitioned family (SPLIT, PIXEL, WIDE, PAGED; LDE_STRATEGY_PAGED
// stands for it here) from 2^20 events on -- WIDE's cost does not grow with the
// histogram, so a batch smaller than the histogram is no reason for ATOMIC's
// memory-side atomics (DREAM at 10,000 bins: 1.4e8 events, 2.6e8 bins) --
// else ATOMIC.  Without WIDE, PAGED needs half as many events as bins.
int auto_strategy(const lde_handle *h, long long total) {
    if (h->strategy != LDE_STRATEGY_AUTO) return h->strategy;
    if (h->wide_ok) return total >= (1 << 20) ? LDE_STRATEGY_PAGED : LDE_STRATEGY_ATOMIC;
    const long long thr = std::max<long long>(1 << 20, h->nbins / 2);
    return (h->n_tiles > 0 && total >= thr) ? LDE_STRATEGY_PAGED : LDE_STRATEGY_ATOMIC;
}

// Wavelength mode: the coordinate pass can be deferred into the SIEVE path
// (keyed pass) when the batch may take it; bin_segments runs the plain
// pass for whatever does not.
bool coord_keyed_candidate(const lde_handle *h, long long total) {
    if (!h->coord || h->monitor || !h->split_ok || h->n_tiles == 0) return false;
    const int strat = auto_strategy(h, total);
    return strat == LDE_STRATEGY_SPLIT ||
           (h->strategy == LDE_STRATEGY_AUTO && strat == LDE_STRATEGY_PAGED);
}

// SPLIT: the SIEVE pass bins this replica's hot rows in LDS and emits cold
// keys, sorted into tiles and accumulated by the cold pipeline.  Returns 1
// (nothing launched) when AUTO should take another strategy.  coord_deferred
// (wavelength mode): `sd` still holds times; the keyed pass (k_event_key)
// turns them into the sieve's finished words.
int bin_split(lde_handle *h, std::vector<lde::SegDesc> &sd, long long chunks,
              long long total, int replica, bool forced, bool coord_deferred) {
    // the descriptor table is uploaded lazily: the SIEVE pass of a batch of
    // at most kKargSegs messages passes it as kernel arguments instead
    if (int rc = ensure_segs_cap(h, (long long)sd.size())) return rc;  // d_segs fixed from here
    bool uploaded = false;
    auto upload = [&]() -> int {
        if (uploaded) return LDE_OK;
        uploaded = true;
        return upload_segments(h, sd);
    };
    lde::SplitArgs a;
    a.segs = h->d_segs;
    a.n_segs = (int)sd.size();
    a.n_chunks = chunks;
    a.lut = h->d_lut;
    a.lut16 = h->lut16;
    a.L = h->L;
    a.pid_off = h->pid_off;
    a.S = (int)h->S;
    a.tp = h->tp;
    a.rows = h->hot_rows;
    a.sample_blocks = (int)std::min<long long>(lde::kSampleBlocks, chunks);
    a.sample_part = h->d_sample_part;
    a.screen_cnt = h->d_screen_cnt;
    a.screen_row = h->d_screen_row;
    a.cache_bits = h->cache_bits;
    a.pix_cnt = h->d_pix_cnt;
    const int grid = (int)std::min<long long>(chunks, (long long)h->split_grid);
    const uint32_t *row_screen = h->d_row_screen + (size_t)lde::kHotMaxRows * replica;
    // Hot-set selection samples this batch.  The first time any replica is
    // needed, every replica is selected from the same batch (one host sync in
    // all, instead of one per replica on its first batch); afterwards each
    // replica is re-selected after hot_refresh of its own batches.  The SIEVE
    // tables are built right after each selection, while d_screen_row holds
    // that replica's rows.
    int &uses = h->hot_uses[replica];
    if (uses < 0 || uses >= h->hot_refresh) {
        if (int rc = upload()) return rc;
        std::vector<int> todo;
        for (int r = 0; r < h->R; ++r)
            if (r == replica || h->hot_uses[(size_t)r] < 0) todo.push_back(r);
        for (int r : todo) {
            lde::SplitArgs b = a;
            b.stats = h->d_sel_stats + 4 * r;
            b.row_screen = h->d_row_screen + (size_t)lde::kHotMaxRows * r;
            Timed tm(h, LDE_K_SPLIT_AUX);
            HIPCALL(h, lde::launch_hot_sample(b, r, h->stream));
            HIPCALL(h, lde::launch_hot_pick(b, h->stream));
            if ((size_t)r < h->key_ok.size()) h->key_ok[(size_t)r] = 0;  // new glut / table image
            HIPCALL(h, lde::launch_sieve_tables(
                           (const unsigned char *)h->d_lut + (size_t)r * h->L * (h->lut16 ? 2 : 4), h->lut16,
                           h->L, h->T, h->T, h->d_screen_row, h->d_pix_cnt, h->cache_bits,
                           h->d_glut + (size_t)(h->L + 1) * r, h->d_sieve_tab + ((size_t)r << h->cache_bits),
                           b.stats, h->stream));
        }
        HIPCALL(h, hipMemcpyAsync(h->h_sel_stats, h->d_sel_stats, (size_t)h->R * 16,
                                  hipMemcpyDeviceToHost, h->stream));
        HIPCALL(h, hipStreamSynchronize(h->stream));
        for (int r : todo) {
            const uint32_t *st = h->h_sel_stats + 4 * r;
            const double sampled = (double)st[0];
            h->hot_cov[(size_t)r] = sampled > 0 ? (double)st[1] / sampled : 0.0;
            h->all_hot[(size_t)r] = st[2] == (uint32_t)h->S ? 1 : 0;
            h->hot_uses[(size_t)r] = 0;
            if (env_ll("LDE_VERBOSE", 0))
                fprintf(stderr, "lde split: replica %d sampled %u, hot rows %u cover %.3f, pixel table covers %.3f\n",
                        r, st[0], st[2], h->hot_cov[(size_t)r], sampled > 0 ? (double)st[3] / sampled : 0.0);
        }
    }
    ++uses;
    if (!forced && h->hot_cov[replica] < h->split_min_cov) {
        if (env_ll("LDE_VERBOSE", 0))
            fprintf(stderr, "lde split: replica %d hot cover %.3f < %.3f -> paged\n", replica,
                    h->hot_cov[replica], h->split_min_cov);
        return 1;
    }
    const long long per_block = (chunks + grid - 1) / grid;
    // cold slots are reserved in multiples of 4 per wave and half chunk
    const long long cold_cap = per_block * (lde::kChunk + 4 * 2 * (lde::kSplitThreads / 64));
    // the rare batch too large for the regions' 32-bit offsets takes PAGED (exact)
    if ((unsigned long long)cold_cap * 4ULL >= 0x80000000ULL) return 1;
    const int hr = h->hot_rows;
    const int ht4 = (hr * h->T + 7) & ~7;  // multiple of 8: the u16 hot-row flush
    if (int rc = grow(h, &h->d_hot_part, h->hot_part_cap, (size_t)grid * ht4)) return rc;
    // regions of 24-bit keys (as u32 units: 3 / 4 of that would do)
    if (int rc = grow(h, &h->d_cold, h->cold_total_cap,
                      (size_t)grid * (size_t)(cold_cap + lde::kSplitThreads / 64)))
        return rc;
    if (int rc = grow(h, &h->d_chunk_tab, h->chunk_tab_cap, (size_t)chunks + 1)) return rc;
    const size_t nt = (size_t)h->n_tiles;
    if (int rc = grow(h, &h->d_cold_tcnt, h->cold_tcnt_cap, (size_t)grid * lde::kColdGroups * nt)) return rc;
    if (int rc = grow(h, &h->d_cold_boff, h->cold_boff_cap, (size_t)grid * lde::kColdGroups * nt)) return rc;
    // tile-major u16 keys: at most every staged slot, + the 8-key padding of
    // every (row, tile) range, + slack for pass B's 16-byte loads
    if (int rc = grow(h, &h->d_cold_keys, h->cold_keys_cap,
                      (size_t)grid * (size_t)cold_cap + (size_t)grid * lde::kColdGroups * nt * 8 + 64))
        return rc;
    const double cold_est = std::min(1.0, std::max(0.05, 1.0 - h->hot_cov[replica])) * (double)total;
    // pass B items: as many as fit resident at once (LDS: one 2^tile_bits
    // u32 tile per block), so no second round of blocks; a tile with n keys
    // gets ceil(n / item_keys) <= n / item_keys + 1 items, hence the
    // n_tiles subtracted (DREAM: 2 x 256 slots, 157 tiles -> ~96K keys per
    // item, 3 items per tile; one item per tile measured 12 us slower)
    const long long resident =
        (long long)h->cus * std::max<long long>(1, (160LL * 1024) / (4LL << h->tile_bits));
    const long long slots = resident - h->n_tiles;
    const long long item_keys =
        h->item_events_override > 0
            ? h->item_events_override
            : std::max<long long>(32768, (long long)(cold_est / (double)(slots >= h->cus / 2
                                                                          ? slots
                                                                          : std::max(1, h->cus / 2))));
    const long long max_items = ((long long)grid * cold_cap) / item_keys + h->n_tiles + 1;
    if (int rc = grow(h, &h->d_cold_items, h->cold_items_cap, (size_t)max_items)) return rc;
    // wavelength mode: the keyed pass turns (pid, toa) into the sieve's
    // finished words, one chunk-aligned stream (ssd) the sieve reads
    std::vector<lde::SegDesc> ksd;
    if (coord_deferred) {
        // k_event_key takes the messages as kernel arguments when they fit
        // (no H2D copy in front of it), else from d_segs
        const bool kkarg = (long long)sd.size() <= lde::kKargSegs;
        if (!kkarg)
            if (int rc = upload()) return rc;
        if (int rc = grow(h, &h->d_cbin, h->cbin_cap, (size_t)chunks * lde::kChunk)) return rc;
        // per replica: each table slot's distance row / fx (or x) and each
        // pixel's 12-byte record, built once after the replica's hot-set
        // selection (or a new coordinate LUT) and reused by its batches
        const size_t C = (size_t)1 << h->cache_bits;
        if (!h->d_key_dist)
            if (int rc = dev_alloc(h, &h->d_key_dist, C * (size_t)h->R)) return rc;
        const uint32_t *tab_r = h->d_sieve_tab + ((size_t)replica << h->cache_bits);
        // FAST event pass: fixed bin correction + each pixel's distance row
        // and fx precomputed (rows fit the record word's 8 tag bits)
        const bool pre = h->cargs.fixed_bin && h->cargs.edges_lds && h->cargs.nd <= 256;
        const int pre_nd = pre ? h->cargs.nd : 0;
        if (pre && !h->d_key_tabi)
            if (int rc = dev_alloc(h, &h->d_key_tabi, C * (size_t)h->R)) return rc;
        if (!h->d_key_rec)
            if (int rc = dev_alloc(h, &h->d_key_rec, 3 * ((size_t)h->L + 1) * (size_t)h->R)) return rc;
        if (h->key_ok.size() != (size_t)h->R) h->key_ok.assign((size_t)h->R, 0);
        double *kd_r = h->d_key_dist + C * (size_t)replica;
        uint8_t *ki_r = pre ? h->d_key_tabi + C * (size_t)replica : nullptr;
        uint32_t *kr_r = h->d_key_rec + 3 * ((size_t)h->L + 1) * (size_t)replica;
        const char want = pre ? 2 : 1;  // the layout the replica's tables hold
        if (h->key_ok[(size_t)replica] != want) {
            HIPCALL(h, lde::launch_key_dist(tab_r, h->cache_bits, h->d_cpd, (unsigned)h->L, h->cargs.d0,
                                            h->cargs.inv_dd, pre_nd, kd_r, ki_r, h->stream));
            HIPCALL(h, lde::launch_key_records(h->d_glut + (size_t)(h->L + 1) * replica, h->d_cpd,
                                               (unsigned)h->L, h->cargs.d0, h->cargs.inv_dd, pre_nd, kr_r,
                                               h->stream));
            h->key_ok[(size_t)replica] = want;
        }
        lde::KeyArgs ka;
        ka.c = h->cargs;
        ka.segs = h->d_segs;
        ka.karg = kkarg ? 1 : 0;
        if (kkarg)
            for (size_t i = 0; i < sd.size(); ++i) ka.sk.s[i] = sd[i];
        ka.n_segs = (int)sd.size();
        ka.n_chunks = chunks;
        ka.glut = h->d_glut + (size_t)(h->L + 1) * replica;
        ka.pix_tab = tab_r;
        ka.tab_d = kd_r;
        ka.tab_i = ki_r;
        ka.pre = pre ? 1 : 0;
        ka.rec = kr_r;
        ka.cbits = h->cache_bits;
        ka.keys = h->d_cbin;
        ka.dummy = h->d_sieve_dummy;
        ka.ablate = (int)env_ll("LDE_KEY_ABLATE", 0);
        Stamp sp(h, LDE_K_COORD);  // k_event_key, stamped by its own dispatch
        HIPCALL(h, lde::launch_event_key(ka, h->cus, h->stream, sp.a, sp.b));
        sp.done = true;
        ksd.push_back({h->d_cbin, h->d_cbin, chunks * lde::kChunk, 0});
    }
    const std::vector<lde::SegDesc> &ssd = coord_deferred ? ksd : sd;
    lde::SieveArgs sa;
    sa.keyed = coord_deferred ? 1 : 0;
    sa.segs = h->d_segs;
    sa.n_segs = (int)ssd.size();
    sa.n_chunks = chunks;
    sa.chunk_tab = h->d_chunk_tab;
    sa.glut = h->d_glut + (size_t)(h->L + 1) * replica;
    sa.L = (uint32_t)h->L;
    sa.pid_off = h->pid_off;
    sa.ttab = h->d_ttab;
    sa.toa_lo = (uint32_t)h->tp.lo;
    sa.toa_cap = h->ttab_cap;
    sa.toa_shift = h->ttab_shift;
    sa.toa_words4 = (int)h->ttab.size();
    sa.T = h->T;
    sa.pix_tab = h->d_sieve_tab + ((size_t)replica << h->cache_bits);
    sa.cbits = h->cache_bits;
    sa.hot_words = ht4;
    sa.hot_part = h->d_hot_part;
    sa.cold = h->d_cold;
    sa.cold_cap = cold_cap;
    sa.cold_cnt = h->d_cold_cnt;
    sa.tile_bits = h->tile_bits;
    sa.n_tiles = h->n_tiles;
    sa.cold_tcnt = h->d_cold_tcnt;
    sa.ablate = h->sieve_ablate;
    sa.hot_fmt = h->d_hot_fmt;
    sa.trace = h->d_trace;
    {
        // k_sieve is timed by its own dispatch (start/stop events stamped
        // by hipExtLaunchKernelGGL): no marker packets around it
        Stamp sp(h, LDE_K_SPLIT);
        // the sieve builds its chunk table in LDS (no launch in front of
        // it) when the block's chunk range fits, from descriptors passed
        // as kernel arguments when they fit too, else from d_segs
        sa.lds_ctab = per_block + 1 <= lde::kSieveLdsChunks;
        sa.karg = (long long)ssd.size() <= lde::kKargSegs;
        sa.dummy = h->d_sieve_dummy;
        if (sa.lds_ctab && sa.karg) {
            for (size_t i = 0; i < ssd.size(); ++i) sa.sk.s[i] = ssd[i];
        } else if (sa.lds_ctab) {
            if (int rc = upload()) return rc;
        } else if ((!uploaded || coord_deferred) && (long long)ssd.size() <= lde::kKargSegs) {
            // (keyed: also rewrites d_segs to the key stream's descriptor,
            // which the sieve's deferred-chunk pass reads)
            HIPCALL(h, lde::launch_chunk_tab_karg(ssd.data(), sa.n_segs, chunks, h->d_sieve_dummy,
                                                  h->d_chunk_tab, h->d_segs, h->stream));
        } else {
            if (int rc = upload()) return rc;
            HIPCALL(h, lde::launch_chunk_tab(h->d_segs, sa.n_segs, chunks, h->d_sieve_dummy,
                                             h->d_chunk_tab, h->stream));
        }
        HIPCALL(h, lde::launch_sieve(sa, grid, h->stream, sp.a, sp.b));
        sp.done = true;
        if (h->d_trace) {  // diagnostic only: a host sync per batch
            std::vector<unsigned long long> tr((size_t)grid * 4);
            HIPCALL(h, hipMemcpyAsync(tr.data(), h->d_trace, tr.size() * 8, hipMemcpyDeviceToHost,
                                      h->stream));
            HIPCALL(h, hipStreamSynchronize(h->stream));
            unsigned long long s0 = ~0ull, s1 = 0, m0 = ~0ull, m1 = 0, e0 = ~0ull, e1 = 0;
            double span = 0, init = 0;  // mean block init -> stream end, start -> init
            for (int b = 0; b < grid; ++b) {
                span += (double)(tr[4 * b + 1] - tr[4 * b + 3]) / grid;
                init += (double)(tr[4 * b + 3] - tr[4 * b]) / grid;
                s0 = std::min(s0, tr[4 * b]); s1 = std::max(s1, tr[4 * b]);
                m0 = std::min(m0, tr[4 * b + 1]); m1 = std::max(m1, tr[4 * b + 1]);
                e0 = std::min(e0, tr[4 * b + 2]); e1 = std::max(e1, tr[4 * b + 2]);
            }
            const double us = 1e6 / 100e6;  // s_memrealtime: 100 MHz
            h->trace_stats.push_back((s1 - s0) * us);
            h->trace_stats.push_back((m1 - m0) * us);
            h->trace_stats.push_back((e1 - e0) * us);
            h->trace_stats.push_back((e1 - s0) * us);
            h->trace_stats.push_back(span * us);
            h->trace_stats.push_back(init * us);
            if (env_ll("LDE_SIEVE_TRACE", 0) > 1) {  // per block: stream end after the first start
                fprintf(stderr, "lde sieve trace blocks:");
                for (int b = 0; b < grid; ++b) fprintf(stderr, " %.1f", (tr[4 * b + 1] - s0) * us);
                fprintf(stderr, "\n");
            }
        }
        if (h->probe) {
            const double us = std::chrono::duration<double, std::micro>(
                                  std::chrono::steady_clock::now() - h->t_acc0).count();
            h->probe_us += us;
            h->probe_min = h->probe_n ? std::min(h->probe_min, us) : us;
            ++h->probe_n;
        }
    }
    lde::ColdArgs c;
    c.hot_part = h->d_hot_part;
    c.row_screen = row_screen;
    c.ht = hr * h->T;
    c.ht4 = ht4;
    c.T = h->T;
    c.tile_bits = h->tile_bits;
    c.n_tiles = h->n_tiles;
    c.rows = grid;
    c.cold = h->d_cold;
    c.stride = cold_cap + lde::kSplitThreads / 64;
    c.cap = cold_cap;
    c.cold_cnt = h->d_cold_cnt;
    c.tcnt = h->d_cold_tcnt;
    c.boff = h->d_cold_boff;
    c.tile_total = h->d_cold_ttot;
    c.item_keys = (uint32_t)std::min<long long>(item_keys, 0x7fffffffLL);
    c.max_items = (uint32_t)max_items;
    c.items = h->d_cold_items;
    c.item_count = h->d_item_count;
    c.keys = h->d_cold_keys;
    c.hist = h->d_win32;
    c.n_bins = h->nbins;
    c.hot_fmt = h->d_hot_fmt;
    c.ablate = h->cold_sort_ablate;
    c.all_hot = h->all_hot[replica];
    Timed tm(h, LDE_K_PAGED);
    HIPCALL(h, lde::launch_cold_pipeline(c, h->stream, h->bin_stop_ext));
    if (h->bin_stop_ext) h->bin_stop_used = true;
    return LDE_OK;
}

int bin_pixel(lde_handle *h, const std::vector<lde::SegDesc> &sd, long long chunks, long long total,
              int replica) {
    if (int rc = upload_segments(h, sd)) return rc;
    // runs padded to 4 payloads: at most 3 pads per (unit, range); 24-bit
    // payloads take 3 bytes each
    const long long units = (chunks + h->pix_unit - 1) / h->pix_unit;
    const int grid = (int)std::min<long long>(units, (long long)h->pix_grid);
    size_t n_pay = (size_t)total + 3 * (size_t)units * (size_t)h->pix.nr + 4;
    // predicted slots: the previous batch had the same blocks and a similar
    // size, and slots average >= 256 events (margins <= 22 %).  Slot sum
    // bound: caps <= 1.25 x pred + 20 per slot, run totals <= events + pads
    const long long slots = (long long)grid * h->pix.nr;
    const double ratio = h->pix_prev_n > 0 ? (double)total / (double)h->pix_prev_n : 0.0;
    const double pred_pay = 1.25 * ratio * (double)(h->pix_prev_n + 3 * h->pix_prev_units * h->pix.nr) +
                            20.0 * (double)slots + 4.0;
    const bool pred = h->pix_prev_grid == grid && ratio >= 0.5 && ratio <= 2.0 &&
                      total >= 256 * slots && pred_pay < 0x7FFFFFF0;
    // overflow list: 1/32 of the batch's groups (a Poisson stream overflows
    // ~0.4 % of them at 2 sigma margins) -- groups past it are added by pass A
    // itself with global atomics, so any stream stays exact
    const long long cap_knob = env_ll("LDE_PIX_OVF_CAP", 0);  // diagnostics: force the fallback
    const size_t ovf_groups = cap_knob > 0 ? (size_t)cap_knob : std::max<size_t>(65536, n_pay / 4 / 32 + 1);
    if (pred) {
        n_pay = std::max(n_pay, (size_t)pred_pay);
        if (int rc = grow(h, &h->d_povf_grp, h->povf_cap, ovf_groups)) return rc;
    }
    if (int rc = grow(h, &h->d_ppayload, h->ppayload_cap, (n_pay * 3 + 3) / 4 + 4)) return rc;
    // pass-B items: each flushes its range's whole footprint (F x T
    // atomics), so as few as keep the CUs busy: one per range up to twice the
    // mean range total, larger ranges (skewed streams) split (LOKI: 196
    // items, pass B 0.157 -> 0.120 ms against ~600 items of total / 2 CUs)
    const long long per = (std::max<long long>(65536, (2 * total + h->pix.nr - 1) / h->pix.nr) + 3) & ~3LL;
    const long long max_items = (long long)(n_pay / (size_t)per) + h->pix.nr + 1;
    if (int rc = grow(h, &h->d_pitems, h->pitems_cap, (size_t)max_items)) return rc;
    if (int rc = grow(h, &h->d_pctab, h->pctab_cap, (size_t)chunks)) return rc;
    lde::PixArgs a;
    a.ctab = h->d_pctab;
    a.ept = h->pix_unit == 2 ? 16 : 8;
    a.segs = h->d_segs;
    a.n_segs = (int)sd.size();
    a.n_chunks = chunks;
    a.pid_off = h->pid_off;
    a.L = (unsigned)h->L;
    a.rb = h->pix.rb;
    a.ablate = (int)env_ll("LDE_PIX_ABLATE", 0);
    a.nr = h->pix.nr;
    a.rs = h->pix.rs;
    a.tab = h->d_tab;
    a.tp = h->tp;
    a.counts = h->d_pcounts;
    a.rstart = h->d_prstart;
    a.payload = h->d_ppayload;
    a.unit = h->pix_unit;
    a.grid = grid;
    a.prev = h->d_pprev;
    a.ovf = h->d_povf;
    if (pred) {
        a.pred = (float)ratio;
        a.ovf_grp = h->d_povf_grp;
        a.ovf_cap = (uint32_t)ovf_groups;
        a.ovf_loc = h->pix.loc + (size_t)replica * h->L;
        a.ovf_fp_off = h->pix.fp_off;
        a.ovf_fp_scr = h->pix.fp_scr;
        a.ovf_hist = h->d_win32;
    }
    h->pix_last_pred = pred;
    h->pix_prev_n = total;  // the scatter records this batch's run totals
    h->pix_prev_units = units;
    h->pix_prev_grid = grid;
    {
        Stamp sp(h, LDE_K_PIXEL);
        HIPCALL(h, lde::launch_pixel(a, h->pix, replica, (uint32_t)per, (int)max_items, h->d_pitems,
                                     h->d_pitem_count, h->d_win32, h->stream, 0, sp.a, sp.b));
        sp.done = true;
    }
    {
        Stamp sp(h, LDE_K_PAGE_ACC);
        HIPCALL(h, lde::launch_pixel(a, h->pix, replica, (uint32_t)per, (int)max_items, h->d_pitems,
                                     h->d_pitem_count, h->d_win32, h->stream, 1, sp.a, sp.b));
        sp.done = true;
    }
    return LDE_OK;
}

// WIDE setup (lde_create; lde_set_coord_lut rebuilds the tree for integer
// bins): the TOA tree, the partition form and the pixel table size.  Leaves
// wide_ok false (nothing allocated) where the strategy does not apply.
int wide_tree(lde_handle *h, const std::vector<double> &edges) {
    std::vector<uint32_t> tree;
    lde::WideToa wt;
    if (!build_wide_tree(edges, h->T, tree, wt)) {
        h->wide_ok = false;
        return LDE_OK;
    }
    uint32_t *d = nullptr;
    if (int rc = dev_alloc(h, &d, tree.size())) return rc;
    const hipError_t e = hipMemcpy(d, tree.data(), tree.size() * 4, hipMemcpyHostToDevice);
    if (e != hipSuccess) {
        dev_free(d);
        return fail(h, LDE_EHIP, "tree upload failed: %s", hipGetErrorString(e));
    }
    dev_free(h->d_wtree);
    h->d_wtree = d;
    wt.tree = d;
    wt.lds = wt.words <= lde::kWideTreeLds ? 1 : 0;
    h->wtoa = wt;
    return LDE_OK;
}

int setup_wide(lde_handle *h) {
    h->wide_ok = false;
    if (h->monitor || env_ll("LDE_WIDE", 1) == 0) return LDE_OK;  // (diagnostics: off)
    const unsigned long long nb = (unsigned long long)h->S * (unsigned long long)h->T;
    if (nb == 0 || nb >= 0xFFFFFFFFULL || h->S >= (long long)0x3FFFFF || h->L < 1 || h->L >= 0x7FFFFFFFLL)
        return LDE_OK;
    if (int rc = wide_tree(h, h->edges)) return rc;
    if (!h->d_wtree) return LDE_OK;
    const long long tiles = (long long)((nb + (1ULL << lde::kWideTileBits) - 1) >> lde::kWideTileBits);
    if (tiles <= lde::kWideMaxParts && env_ll("LDE_WIDE_LEVELS", 1) < 2) {
        h->wide_levels = 1;
        h->wide_pbits = lde::kWideTileBits;
        h->wide_parts = (int)tiles;
        h->wide_tpb_bits = 0;
    } else {  // bands of tpb tiles (at most kWideMaxBands of them), then tiles
        // (LDE_WIDE_LEVELS=2, diagnostics: the two-level form at any size).
        // Partitions per pass balanced (the larger of the bands and the tiles
        // per band as small as it goes): a pass into few partitions ranks with
        // LDS atomics that many lanes of a wave aim at one counter.
        int tb = 1;
        while (((tiles + (1LL << tb) - 1) >> tb) > lde::kWideMaxBands) ++tb;
        long long best = -1;
        for (int b = tb; b <= 8; ++b) {
            const long long m = std::max<long long>((tiles + (1LL << b) - 1) >> b, 1LL << b);
            if (best < 0 || m < best) {
                best = m;
                tb = b;
            }
        }
        const long long force = env_ll("LDE_WIDE_TPB_BITS", 0);  // (diagnostics)
        if (force > 0 && force <= 8 && ((tiles + (1LL << force) - 1) >> force) <= lde::kWideMaxBands) tb = (int)force;
        h->wide_levels = 2;
        h->wide_tpb_bits = tb;
        h->wide_pbits = lde::kWideTileBits + tb;
        h->wide_parts = (int)((nb + (1ULL << h->wide_pbits) - 1) >> h->wide_pbits);
    }
    h->wide_tiles = (int)tiles;
    // pixel table: 2^13 slots (the whole LUT when it fits in half of that),
    // tags of 9 bits; smaller when the first pass's LDS needs the room
    auto bits = [](long long n) { int b = 0; while ((1LL << b) < n) ++b; return b; };
    int cb = (int)std::max<long long>(0, std::min<long long>(lde::kWideMaxCacheBits,
                                                             env_ll("LDE_WIDE_CACHE_BITS", lde::kWideMaxCacheBits)));
    // (at least 4 slots: the table is copied into LDS in 16-byte units)
    if (cb > 0 && (1LL << cb) >= 2 * h->L) cb = std::max(2, bits(h->L));
    if (cb > 0 && ((h->L - 1) >> cb) > 511) cb = 0;  // tags of 9 bits: beyond 2^22 pixels, no table
    lde::WideArgs a{};
    a.n_parts = h->wide_parts;
    a.toa = h->wtoa;
    auto fits = [&](int c) {
        a.cbits = c;
        return lde::wide_scatter_smem(a) <= 160 * 1024;
    };
    while (cb > 8 && !fits(cb)) --cb;
    if (!fits(cb)) {  // the tree from global memory instead
        h->wtoa.lds = 0;
        a.toa = h->wtoa;
    }
    if (!fits(cb)) cb = 0;
    if (!fits(cb)) return LDE_OK;
    h->wide_cbits = cb;
    if (cb > 0) {
        if (int rc = dev_alloc(h, &h->d_wtab, (size_t)h->R << cb)) return rc;
        if (int rc = dev_alloc(h, &h->d_wpixcnt, (size_t)h->L)) return rc;
    }
    if (int rc = dev_alloc(h, &h->d_wcounters, 8)) return rc;
    if (!h->d_overflow) {
        if (int rc = dev_alloc(h, &h->d_overflow, 1)) return rc;
        HIPCALL(h, hipMemset(h->d_overflow, 0, 4));
    }
    if (int rc = dev_alloc(h, &h->d_wband, (size_t)lde::kWideMaxParts)) return rc;
    h->wide_uses.assign((size_t)h->R, -1);
    h->wide_ok = true;
    if (env_ll("LDE_VERBOSE", 0))
        fprintf(stderr, "lde wide: %lld tiles, %d level(s), %d partitions of 2^%d bins, TOA tree %d words "
                        "(root 2^%d, fan-out %d, depth %d, %s), pixel table 2^%d, %zu B LDS\n",
                tiles, h->wide_levels, h->wide_parts, h->wide_pbits, h->wtoa.words, h->wtoa.sh0, 1 << h->wtoa.fb,
                h->wtoa.depth, h->wtoa.lds ? "LDS" : "global", cb, lde::wide_scatter_smem(a));
    return LDE_OK;
}

// WIDE: key, partition into pages, (second level), tile pass B
int bin_wide(lde_handle *h, const std::vector<lde::SegDesc> &sd, long long chunks, long long total, int replica) {
    // up to kKargSegs messages reach the chunk-table kernel as kernel
    // arguments (no descriptor upload in front of it)
    const bool karg = (long long)sd.size() <= lde::kKargSegs;
    if (karg) {
        if (int rc = ensure_segs_cap(h, (long long)sd.size())) return rc;
    } else if (int rc = upload_segments(h, sd)) {
        return rc;
    }
    const int P = h->wide_parts;
    const long long units = (chunks + 1) / 2;
    const int grid1 = (int)std::min<long long>(units, std::min<long long>(h->cus, lde::kWideMaxRows));
    const long long upb = (units + grid1 - 1) / grid1;
    // a block's pool: its events plus the runs' pads (< 4 per partition and
    // unit) in whole pages, plus one partly filled page per partition
    const uint32_t cap1 =
        (uint32_t)((upb * ((long long)lde::kWideUnit + 3LL * P) + lde::kWidePage - 1) / lde::kWidePage + P + 1);
    const size_t pages1 = (size_t)grid1 * cap1;
    const size_t esz1 = h->wide_levels == 1 ? 2 : 4;
    // work items: pass B about one per tile (a tile past item_max entries,
    // a hot one, is split over several, added with atomics); the second pass
    // ~2 per CU
    // pass B: items of at most 1/(2 x CUs) of the batch (half as large as
    // one per CU: the hot tiles' items finish with the rest; DREAM 1,000 bins
    // −20 µs, 10,000 bins −0.12 ms).  (diagnostics: LDE_WIDE_ITEM_DIV)
    // The second level's tile items at 1/(3 x CUs) (10,000 bins: pass B
    // 0.39 -> 0.33 ms; one level at 1/3: +7 us).  (diagnostics: _DIV2)
    const long long idiv = std::max<long long>(1, std::min<long long>(16, env_ll("LDE_WIDE_ITEM_DIV", 2)));
    const long long idiv2 = std::max<long long>(1, std::min<long long>(16, env_ll("LDE_WIDE_ITEM_DIV2", 3)));
    const long long item_max1 = h->wide_levels == 1
                                    ? std::max<long long>(65536, (total + idiv * h->cus - 1) / (idiv * h->cus))
                                    : std::max<long long>(65536, (total + 2LL * h->cus - 1) / (2LL * h->cus));
    const long long item_max2 = std::max<long long>(65536, (total + idiv2 * h->cus - 1) / (idiv2 * h->cus));
    const long long max_items1 = P + total / item_max1 + 2;
    const long long max_items2 = h->wide_levels == 2 ? h->wide_tiles + total / item_max2 + 2 : 0;
    const int tpb = 1 << h->wide_tpb_bits;
    // second-pass pool: every item's allocation (k_wide_split) summed: the
    // first pass's entries with their pads, this pass's pads (<= 3 per tile
    // and 16-page unit, + 2 units per item), one partly filled page per tile
    const long long in1 = (long long)grid1 * upb * ((long long)lde::kWideUnit + 3LL * P);
    const long long pages_in = in1 / lde::kWidePage + (long long)grid1 * P;  // (+ partly filled pages)
    const long long units2 = pages_in / 16 + pages_in / 1024 + 2 * max_items1 + 1;
    const size_t pool2 = h->wide_levels == 2
                             ? (size_t)((in1 + 3LL * tpb * units2) / lde::kWidePage) + (size_t)max_items1 * (tpb + 3) + 1
                             : 0;
    if (pages1 + pool2 >= 0xFFFFFFF0ULL || total >= 0xFFFFFFFFLL)
        return fail(h, LDE_EINVAL, "batch too large for the WIDE page pools");
    if (int rc = grow(h, &h->d_wctab, h->wctab_cap, (size_t)chunks)) return rc;
    if (int rc = grow(h, &h->d_wpages1, h->wpages1_cap, pages1 * lde::kWidePage * esz1)) return rc;
    if (pool2)
        if (int rc = grow(h, &h->d_wpages2, h->wpages2_cap, pool2 * lde::kWidePage)) return rc;
    size_t mc = h->wmeta_cap;
    if (pages1 + pool2 > mc || !h->d_wpage_cnt) {
        HIPCALL(h, hipStreamSynchronize(h->stream));
        const size_t n = std::max(pages1 + pool2, mc * 2);
        dev_free(h->d_wpage_cnt);
        dev_free(h->d_wpage_part);
        dev_free(h->d_wlist);
        h->wmeta_cap = 0;
        if (int rc = dev_alloc(h, &h->d_wpage_cnt, n)) return rc;
        if (int rc = dev_alloc(h, &h->d_wpage_part, n)) return rc;
        if (int rc = dev_alloc(h, &h->d_wlist, n)) return rc;
        h->wmeta_cap = n;
    }
    if (int rc = grow(h, &h->d_wrows1, h->wrows1_cap, (size_t)grid1 * ((size_t)3 * P + 1))) return rc;
    if (int rc = grow(h, &h->d_witems1, h->witems1_cap, (size_t)max_items1)) return rc;
    if (h->wide_levels == 2) {
        if (int rc = grow(h, &h->d_wrows2, h->wrows2_cap, (size_t)max_items1 * ((size_t)3 * tpb + 1))) return rc;
        if (int rc = grow(h, &h->d_witems2, h->witems2_cap, (size_t)max_items2)) return rc;
    }
    lde::WideArgs a{};
    a.ctab = h->d_wctab;
    a.segs = h->d_segs;
    a.n_segs = (int)sd.size();
    a.n_chunks = chunks;
    a.pid_off = h->pid_off;
    a.L = (unsigned)h->L;
    a.lut = (const unsigned char *)h->d_lut + (size_t)replica * h->L * (h->lut16 ? 2 : 4);
    a.lut16 = h->lut16 ? 1 : 0;
    a.T = h->T;
    a.cbits = h->wide_cbits;
    a.pix_tab = h->wide_cbits ? h->d_wtab + ((size_t)replica << h->wide_cbits) : nullptr;
    a.toa = h->wtoa;
    a.levels = h->wide_levels;
    a.pbits = h->wide_pbits;
    a.n_parts = P;
    a.tpb_bits = h->wide_tpb_bits;
    a.n_tiles = h->wide_tiles;
    a.pages1 = h->d_wpages1;
    a.pages2 = h->d_wpages2;
    a.page_cnt = h->d_wpage_cnt;
    a.page_part = h->d_wpage_part;
    a.list = h->d_wlist;
    a.cap1 = cap1;
    a.rows1 = {h->d_wrows1, h->d_wrows1 + (size_t)grid1 * P, h->d_wrows1 + (size_t)2 * grid1 * P,
               h->d_wrows1 + (size_t)3 * grid1 * P, P};
    if (h->wide_levels == 2)
        a.rows2 = {h->d_wrows2, h->d_wrows2 + (size_t)max_items1 * tpb, h->d_wrows2 + (size_t)2 * max_items1 * tpb,
                   h->d_wrows2 + (size_t)3 * max_items1 * tpb, tpb};
    a.pool2_next = h->d_wcounters + 2;
    a.pool2_cap = (uint32_t)pool2;
    a.page0_2 = (uint32_t)pages1;
    a.items1 = h->d_witems1;
    a.items2 = h->d_witems2;
    a.counters = h->d_wcounters;
    a.overflow = h->d_overflow;
    a.max_items1 = (uint32_t)max_items1;
    a.max_items2 = (uint32_t)max_items2;
    a.band_items = h->d_wband;
    a.item_max1 = (uint32_t)std::min<long long>(item_max1, 0x7FFFFFFF);
    a.item_max2 = (uint32_t)std::min<long long>(item_max2, 0x7FFFFFFF);
    a.hist = h->d_win32;
    a.n_bins = h->nbins;
    a.grid1 = grid1;
#ifdef LDE_DIAGNOSTICS
    a.ablate = (int)env_ll("LDE_WIDE_ABLATE", 0);
    a.acc_depth = (int)env_ll("LDE_WIDE_ACC_DEPTH", 4);
    a.tree_hybrid = (int)env_ll("LDE_WIDE_TREE_HYBRID", 1);
#endif
    // an integer view's u32 window is all zero until its first batch after
    // a finalize / clear (both zero it; win_events counts what this window's
    // earlier pieces added): pass B then stores its tiles without reading them
    a.wzero = (h->out_dtype != LDE_F32 && !h->window_has_data && h->win_events == 0 && !h->f32_pending &&
               env_ll("LDE_WIDE_WZERO", 1) != 0)
                  ? 1
                  : 0;
    HIPCALL(h, lde::launch_wide_chunks(a, karg ? sd.data() : nullptr, h->stream));
    int &uses = h->wide_uses[(size_t)replica];
    if (h->wide_cbits && (uses < 0 || uses >= h->hot_refresh)) {
        Timed tm(h, LDE_K_SPLIT_AUX);
        HIPCALL(h, lde::launch_wide_table(a, a.lut, h->d_wpixcnt, const_cast<uint32_t *>(a.pix_tab), h->stream));
        uses = 0;
    }
    ++uses;
    Stamp sa(h, LDE_K_WIDE);
    Stamp sb(h, LDE_K_WIDE_ACC);
    HIPCALL(h, lde::launch_wide(a, h->stream, sa.a, sa.b, sb.a, sb.b));
    sa.done = sb.done = true;
    return LDE_OK;
}

int bin_segments(lde_handle *h, std::vector<Segment> segs, long long total, int replica,
                 bool coord_deferred) {
    const size_t lut_es = h->lut16 ? 2 : 4;
    const void *lut = h->monitor ? nullptr
                                 : (const void *)((const unsigned char *)h->d_lut +
                                                  (size_t)replica * h->L * lut_es);
    if (h->monitor) {
        // one launch per kKargSegs messages (a batch of 14 pulses: one)
        h->last_strategy = LDE_STRATEGY_AUTO;
        lde::SegKarg ka{};
        int k = 0;
        long long n = 0;
        auto flush = [&]() -> int {
            if (k == 0) return LDE_OK;
            long long g = (n / 32 + 255) / 256;  // 32 events per lane and iteration
            // four blocks per CU (2, 3, 6, 8 measured slower: 149, 114, 111, 122
            // vs 102 us on the monitor bench)
            g = std::max<long long>(1, std::min<long long>(g, (long long)h->cus * 4));
            // blocks in ranges proportional to the message sizes, at least one
            // per message (each block streams one message at its own stride)
            g = std::max<long long>(g, k);
            long long acc = 0;
            for (int i = 0; i < k; ++i) {
                // first block of message i: i + its share of the other g - k blocks
                ka.s[i].chunk0 = i + (long long)((double)(g - k) * (double)acc / (double)n);
                acc += ka.s[i].n;
            }
            Stamp sp(h, LDE_K_MONITOR);
            HIPCALL(h, lde::launch_monitor(ka, k, h->d_tab, h->tp, h->d_win32, (int)g, h->stream, sp.a, sp.b));
            sp.done = true;
            k = 0;
            n = 0;
            return LDE_OK;
        };
        for (const Segment &s : segs) {
            if (s.n == 0) continue;
            ka.s[k++] = {nullptr, s.toa, s.n, 0};
            n += s.n;
            if (k == lde::kKargSegs)
                if (int rc = flush()) return rc;
        }
        return flush();
    }
    int strat = auto_strategy(h, total);
    const bool auto_split = h->strategy == LDE_STRATEGY_AUTO && strat == LDE_STRATEGY_PAGED && h->split_ok;
    // AUTO without SPLIT or PIXEL: WIDE (any edges, any histogram size)
    // before PAGED; a forced strategy that cannot run takes WIDE too
    const bool auto_wide = h->strategy == LDE_STRATEGY_AUTO && strat == LDE_STRATEGY_PAGED && h->wide_ok;
    if (strat == LDE_STRATEGY_WIDE && !h->wide_ok) strat = LDE_STRATEGY_PAGED;
    if (strat == LDE_STRATEGY_SPLIT && !h->split_ok) strat = h->wide_ok ? LDE_STRATEGY_WIDE : LDE_STRATEGY_PAGED;
    // PIXEL's payload offsets are u32: batches whose payload (events + pads)
    // could reach 2^31 take PAGED
    const long long max_chunks = total / lde::kChunk + (long long)segs.size() + 1;
    const bool pixel_ok = h->pixel_ok && total + 3LL * (max_chunks / h->pix_unit + 1) * h->pix.nr < 0x7FFFFFF0LL;
    if (strat == LDE_STRATEGY_PIXEL && !pixel_ok) strat = h->wide_ok ? LDE_STRATEGY_WIDE : LDE_STRATEGY_PAGED;
    // AUTO without skew: PIXEL (no LUT gather) where the footprints fit
    const bool auto_pixel = h->strategy == LDE_STRATEGY_AUTO && strat == LDE_STRATEGY_PAGED && pixel_ok;
    if (auto_pixel && !auto_split) strat = LDE_STRATEGY_PIXEL;
    else if (auto_wide && !auto_split) strat = LDE_STRATEGY_WIDE;
    if ((strat == LDE_STRATEGY_PARTITION || strat == LDE_STRATEGY_PAGED) && h->n_tiles == 0)
        strat = h->wide_ok ? LDE_STRATEGY_WIDE : LDE_STRATEGY_ATOMIC;
    if (coord_deferred && !coord_keyed_candidate(h, total)) {
        // this piece does not take the keyed path: the plain coordinate pass
        if (int rc = coord_prepass(h, segs)) return rc;
        coord_deferred = false;
    }
    h->last_strategy = strat;
    if (strat == LDE_STRATEGY_ATOMIC) {
        // up to kKargSegsAtomic messages: one launch, descriptors as kernel
        // arguments; more: one launch with per-block descriptors in HBM
        lde::SegKargAtomic ka{};
        long long n_msgs = 0;
        for (const Segment &s : segs) n_msgs += s.n > 0 ? 1 : 0;
        if (n_msgs > lde::kKargSegsAtomic) {
            // more messages than fit the kernel arguments (BIFROST's 630 bank
            // messages of a 14-pulse batch, one push): one launch with a
            // descriptor per block in device memory -- per message
            // ceil(n / 1024) blocks, or (beyond 8 blocks per CU in all) a share
            // proportional to its size, at least one
            const long long cap = std::max<long long>((long long)h->cus * 8, n_msgs);
            long long g = 0;
            for (const Segment &s : segs)
                if (s.n > 0) g += std::max<long long>(1, (s.n + 1023) / 1024);
            const bool prop = g > cap;
            std::vector<lde::SegDesc> bd;
            bd.reserve((size_t)std::min(g, cap + n_msgs));
            for (const Segment &s : segs) {
                if (s.n == 0) continue;
                const long long nb = prop ? std::max<long long>(1, (long long)((double)cap * (double)s.n /
                                                                                (double)total))
                                          : std::max<long long>(1, (s.n + 1023) / 1024);
                for (long long j = 0; j < nb; ++j)
                    bd.push_back({s.pid, s.toa, s.n, (long long)(((unsigned long long)j << 32) | (unsigned long long)nb)});
            }
            if (int rc = upload_segments(h, bd)) return rc;
            Stamp sp(h, LDE_K_ATOMIC);
            HIPCALL(h, lde::launch_bin_atomic_blocks(h->d_segs, (int)bd.size(), lut, h->lut16, h->pid_off,
                                                     (unsigned)h->L, h->d_tab, h->tp, h->d_win32, h->stream,
                                                     sp.a, sp.b));
            sp.done = true;
            return LDE_OK;
        }
        int k = 0;
        long long n = 0;
        auto flush = [&]() -> int {
            if (k == 0) return LDE_OK;
            // block ranges per message (k_bin_atomic): a group of 4 events per
            // lane when the grid allows, else ranges proportional to the sizes,
            // at least one block per message
            const long long cap = std::max<long long>((long long)h->cus * 8, k);
            long long g = 0;
            for (int i = 0; i < k; ++i) g += std::max<long long>(1, (ka.s[i].n + 1023) / 1024);
            if (g <= cap) {
                long long b = 0;
                for (int i = 0; i < k; ++i) {
                    ka.s[i].chunk0 = b;
                    b += std::max<long long>(1, (ka.s[i].n + 1023) / 1024);
                }
            } else {
                g = cap;
                long long acc = 0;
                for (int i = 0; i < k; ++i) {
                    ka.s[i].chunk0 = i + (long long)((double)(g - k) * (double)acc / (double)n);
                    acc += ka.s[i].n;
                }
            }
            Stamp sp(h, LDE_K_ATOMIC);
            HIPCALL(h, lde::launch_bin_atomic(ka, k, lut, h->lut16, h->pid_off, (unsigned)h->L, h->d_tab,
                                              h->tp, h->d_win32, (int)g, h->stream, sp.a, sp.b));
            sp.done = true;
            k = 0;
            n = 0;
            return LDE_OK;
        };
        for (const Segment &s : segs) {
            if (s.n == 0) continue;
            ka.s[k++] = {s.pid, s.toa, s.n, 0};
            n += s.n;
        }
        return flush();
    }
    // PARTITION / PAGED
    long long chunks = 0;
    std::vector<lde::SegDesc> sd;
    for (const Segment &s : segs) {
        if (s.n == 0) continue;
        sd.push_back({s.pid, s.toa, s.n, chunks});
        chunks += (s.n + lde::kChunk - 1) / lde::kChunk;
    }
    if (chunks == 0) return LDE_OK;
    if (strat == LDE_STRATEGY_SPLIT || auto_split) {
        const int rc = bin_split(h, sd, chunks, total, replica, strat == LDE_STRATEGY_SPLIT,
                                 coord_deferred);
        if (rc != 1) {
            if (rc == LDE_OK) h->last_strategy = LDE_STRATEGY_SPLIT;
            return rc;
        }
        // AUTO falls back (or a forced SPLIT batch is too large for its
        // regions): in wavelength mode the plain coordinate pass first
        if (coord_deferred)
            if (int rc2 = coord_prepass(h, sd)) return rc2;
        if (auto_pixel) {
            h->last_strategy = LDE_STRATEGY_PIXEL;
            return bin_pixel(h, sd, chunks, total, replica);
        }
        if (h->wide_ok) {
            h->last_strategy = LDE_STRATEGY_WIDE;
            return bin_wide(h, sd, chunks, total, replica);
        }
        // (bin_split uploads the descriptors lazily: this batch's may not be)
        h->last_strategy = LDE_STRATEGY_PAGED;
        return bin_paged(h, sd, chunks, total, lut);
    }
    if (strat == LDE_STRATEGY_PIXEL) return bin_pixel(h, sd, chunks, total, replica);
    if (strat == LDE_STRATEGY_WIDE) return bin_wide(h, sd, chunks, total, replica);
    if (strat == LDE_STRATEGY_PAGED) return bin_paged(h, sd, chunks, total, lut);
    long long item_events = h->item_events_override > 0
                                ? h->item_events_override
                                : std::max<long long>(32768, (total + 2LL * h->cus - 1) / (2LL * h->cus));
    if (item_events > 0x7fffffffLL) item_events = 0x7fffffffLL;
    const long long max_items = (total + item_events - 1) / item_events + h->n_tiles;
    if (int rc = ensure_partition_capacity(h, chunks, max_items)) return rc;
    if (int rc = upload_segments(h, sd)) return rc;
    const int grid_a = (int)std::min<long long>(chunks, (long long)h->part_grid);
    HIPCALL(h, hipMemsetAsync(h->d_part, 0, (size_t)grid_a * h->n_tiles * 4, h->stream));
    for (size_t s0 = 0; s0 < sd.size(); s0 += lde::kMaxSegs) {
        const int ns = (int)std::min<size_t>(lde::kMaxSegs, sd.size() - s0);
        // chunk ids are global: launch the whole range, segments outside this
        // group are skipped by clamping the chunk window
        const long long c_lo = sd[s0].chunk0;
        const long long c_hi = (s0 + ns < sd.size()) ? sd[s0 + ns].chunk0 : chunks;
        lde::PartitionArgs pa;
        pa.tile_bits = h->tile_bits;
        pa.lut16 = h->lut16;
        pa.segs = h->d_segs + s0;
        pa.n_segs = ns;
        pa.c_begin = c_lo;
        pa.n_chunks = c_hi;
        pa.lut = lut;
        pa.pid_off = h->pid_off;
        pa.L = (unsigned)h->L;
        pa.tab = h->d_tab;
        pa.tp = h->tp;
#ifdef LDE_DIAGNOSTICS
        pa.tp.pad = (int)env_ll("LDE_ABLATE", 0);
#else
        pa.tp.pad = 0;
#endif
        pa.n_tiles = h->n_tiles;
        pa.payload = h->d_payload;
        pa.starts = h->d_starts;
        pa.part = h->d_part;
        pa.grid = (int)std::min<long long>(grid_a, c_hi - c_lo);
        Timed tm(h, LDE_K_PARTITION);
        HIPCALL(h, lde::launch_partition(pa, h->stream));
    }
    {
        Timed tm(h, LDE_K_PLAN);
        HIPCALL(h, lde::launch_plan(h->d_part, grid_a, h->n_tiles, chunks, (uint32_t)item_events,
                                    h->d_ttot, h->d_tile_items, h->d_items, h->d_item_count,
                                    (uint32_t)max_items, h->stream));
    }
    {
        Timed tm(h, LDE_K_TILE);
        HIPCALL(h, lde::launch_tile_accumulate(h->tile_bits, h->d_payload, h->d_starts,
                                               h->n_tiles, chunks, h->d_items, h->d_item_count,
                                               h->d_tile_items, h->d_win32, h->nbins,
                                               (int)max_items, h->stream));
    }
    return LDE_OK;
}

// validate the host LUT and copy it into the device format (allocated once)
// the device form of a host LUT (u16 screen or i32 screen * T), validated
int convert_lut(lde_handle *h, const int32_t *out_lut, std::vector<uint16_t> &l16,
                std::vector<int> &l32) {
    const long long n = (long long)h->R * h->L;
    if (h->lut16) l16.resize((size_t)n); else l32.resize((size_t)n);
    for (long long i = 0; i < n; ++i) {
        const int v = out_lut[i];
        if (v < -1 || v >= h->S)
            return fail(h, LDE_EINVAL, "out_lut[%lld] = %d outside [-1, %lld)", i, v, h->S);
        if (h->lut16) l16[(size_t)i] = v < 0 ? (uint16_t)0xFFFF : (uint16_t)v;
        else l32[(size_t)i] = v < 0 ? -1 : (int)((long long)v * h->T);
    }
    return LDE_OK;
}

int upload_lut(lde_handle *h, const int32_t *out_lut) {
    const long long n = (long long)h->R * h->L;
    std::vector<uint16_t> l16;
    std::vector<int> l32;
    if (int rc = convert_lut(h, out_lut, l16, l32)) return rc;
    const size_t bytes = (size_t)n * (h->lut16 ? 2 : 4);
    if (!h->d_lut) {
        if (h->lut16) {
            if (int rc = dev_alloc(h, (uint16_t **)&h->d_lut, (size_t)n)) return rc;
        } else {
            if (int rc = dev_alloc(h, (int **)&h->d_lut, (size_t)n)) return rc;
        }
    }
    // the previous batch's kernels may still read the old table
    HIPCALL(h, hipStreamSynchronize(h->stream));
    HIPCALL(h, hipMemcpy(h->d_lut, h->lut16 ? (const void *)l16.data() : (const void *)l32.data(),
                         bytes, hipMemcpyHostToDevice));
    // every replica's hot set / SIEVE tables derive from the LUT: rebuild lazily
    for (auto &u : h->hot_uses) u = -1;
    return LDE_OK;
}

// PIXEL setup: ranges of 2^rb consecutive pixels, each range's screen
// footprint over every replica (sorted screen list) and every pixel's index
// in its range's footprint.  Available when the ranges fit kPixMaxRanges and
// the largest footprint's counters fit LDS (pix_acc_smem).
// PIXEL tables of a LUT, built into fresh device buffers without touching the
// handle's current ones (lde_set_lut commits them only once everything it
// needs has been built, so a failure leaves the old placement in place)
struct PixStaged {
    bool ok = false;  // PIXEL available for this LUT
    lde::PixSetup pix{};
    uint16_t *ploc = nullptr;
    uint32_t *fp_off = nullptr, *fp_scr = nullptr;
    PixStaged() = default;
    PixStaged(const PixStaged &) = delete;
    PixStaged &operator=(const PixStaged &) = delete;
    ~PixStaged() {
        dev_free(ploc);
        dev_free(fp_off);
        dev_free(fp_scr);
    }
};

int stage_pixel(lde_handle *h, const int32_t *lut, PixStaged &st) {
    st.ok = false;
    if (h->monitor || h->n_tiles == 0 || env_ll("LDE_PIXEL", 1) == 0) return LDE_OK;  // (diagnostics: off)
    const long long L = h->L, R = h->R, S = h->S;
    const int T = h->T;
    // ranges of 2^rb pixels: the smallest rb with at most 256 ranges (LOKI
    // bank 0: 196 ranges of 4096 pixels; 392 of 2048 keep the same 288-screen
    // widest footprint, so pass B gains nothing and pass A's runs get shorter;
    // 256 ranges of 3,136 pixels, one per CU by multiply-high, measured pass B
    // -3.7 us and pass A +19 us)
    const long long max_nr = 256;
    int rb = 8;
    while (rb < 20 && ((L + (1LL << rb) - 1) >> rb) > max_nr) ++rb;
    int tbits = 0;
    while ((1 << tbits) < T) ++tbits;
    const int nr = (int)((L + (1LL << rb) - 1) >> rb);
    // scatter staging word: range (rbits, the all-ones range never used) above
    // an rs-bit payload whose all-ones value is the dropped marker; stored
    // payloads are 24-bit (0xFFFFFF dropped), so local pixel | bin << rb
    // must stay below both
    int rbits = 0;
    while ((1 << rbits) < nr + 1) ++rbits;
    const int rs = 32 - rbits;
    if (rb + tbits > std::min(23, rs - 1)) return LDE_OK;
    std::vector<int> stamp((size_t)S, -1), pos((size_t)S, 0);
    std::vector<uint32_t> fp_off((size_t)nr + 1, 0), fp;
    std::vector<uint16_t> loc((size_t)(R * L), 0xFFFF);
    int fmax = 0;
    for (int r = 0; r < nr; ++r) {
        const long long q0 = (long long)r << rb, q1 = std::min(L, q0 + (1LL << rb));
        const size_t first = fp.size();
        for (long long rep = 0; rep < R; ++rep)
            for (long long q = q0; q < q1; ++q) {
                const int sc = lut[rep * L + q];
                if (sc >= 0 && stamp[(size_t)sc] != r) {
                    stamp[(size_t)sc] = r;
                    fp.push_back((uint32_t)sc);
                }
            }
        std::sort(fp.begin() + (long)first, fp.end());
        const int nf = (int)(fp.size() - first);
        if (nf > 0xFFFE) return LDE_OK;
        fmax = std::max(fmax, nf);
        if (lde::pix_acc_smem(rb, fmax, T) > 150 * 1024) return LDE_OK;  // footprint too wide
        for (int i = 0; i < nf; ++i) pos[fp[first + (size_t)i]] = i;
        for (long long rep = 0; rep < R; ++rep)
            for (long long q = q0; q < q1; ++q) {
                const int sc = lut[rep * L + q];
                if (sc >= 0) loc[(size_t)(rep * L + q)] = (uint16_t)pos[(size_t)sc];
            }
        fp_off[(size_t)r + 1] = (uint32_t)fp.size();
    }
    if (int rc = dev_alloc(h, &st.ploc, loc.size())) return rc;
    if (int rc = dev_alloc(h, &st.fp_off, fp_off.size())) return rc;
    if (int rc = dev_alloc(h, &st.fp_scr, std::max<size_t>(1, fp.size()))) return rc;
    HIPCALL(h, hipMemcpy(st.ploc, loc.data(), loc.size() * 2, hipMemcpyHostToDevice));
    HIPCALL(h, hipMemcpy(st.fp_off, fp_off.data(), fp_off.size() * 4, hipMemcpyHostToDevice));
    if (!fp.empty()) HIPCALL(h, hipMemcpy(st.fp_scr, fp.data(), fp.size() * 4, hipMemcpyHostToDevice));
    // per-batch workspace (allocated once; harmless if the LUT is not committed)
    if (!h->d_pcounts) {
        if (int rc = dev_alloc(h, &h->d_pcounts, (size_t)h->cus * 4 * lde::kPixMaxRanges)) return rc;
        if (int rc = dev_alloc(h, &h->d_pprev, (size_t)h->cus * 4 * lde::kPixMaxRanges)) return rc;
        if (int rc = dev_alloc(h, &h->d_povf, 1)) return rc;
        if (int rc = dev_alloc(h, &h->d_prstart, 2 * (size_t)lde::kPixMaxRanges + 1)) return rc;
        if (int rc = dev_alloc(h, &h->d_pitem_count, 1)) return rc;
    }
    st.pix.rb = rb;
    st.pix.nr = nr;
    st.pix.rs = rs;
    st.pix.fmax = fmax;
    st.ok = true;
    return LDE_OK;
}

// Swap the staged PIXEL tables in (no failure path: the handle state and the
// staged buffers only exchange owners).  The caller has synchronized the
// stream, so no kernel still reads the old tables.
void commit_pixel(lde_handle *h, PixStaged &st) {
    std::swap(h->d_ploc, st.ploc);
    std::swap(h->d_pfp_off, st.fp_off);
    std::swap(h->d_pfp_scr, st.fp_scr);
    h->pixel_ok = st.ok;
    if (!st.ok) return;
    // partition blocks of 1024 threads, one per CU (half the slots of two,
    // so relatively smaller prediction margins: LOKI step 0.529 -> 0.520 ms);
    // units of two chunks (16 events per thread), or one (8) when the TOA
    // table leaves no room for a two-chunk staging area
    h->pix_unit = 2;
    // fewer partition blocks (diagnostics: the tests' way to fill the slots
    // of small batches, so predicted slots are exercised)
    h->pix_grid = (int)std::max<long long>(1, env_ll("LDE_PIX_GRID", h->cus));
    while (h->pix_unit > 1 && lde::pix_scatter_smem(h->tp, h->pix_unit) > 150 * 1024) --h->pix_unit;
    if (lde::pix_scatter_smem(h->tp, h->pix_unit) > 160 * 1024) {
        h->pixel_ok = false;
        return;
    }
    h->pix_prev_n = 0;  // ranges may have changed: the next batch counts
    h->pix = st.pix;
    h->pix.loc = h->d_ploc;
    h->pix.fp_off = h->d_pfp_off;
    h->pix.fp_scr = h->d_pfp_scr;
    if (env_ll("LDE_VERBOSE", 0))
        fprintf(stderr, "lde pixel: %d ranges of 2^%d pixels, widest footprint %d screens (%zu B LDS); "
                        "pass A unit %d, %zu B LDS\n",
                h->pix.nr, h->pix.rb, h->pix.fmax, lde::pix_acc_smem(h->pix.rb, h->pix.fmax, h->T), h->pix_unit,
                lde::pix_scatter_smem(h->tp, h->pix_unit));
}

int build_pixel(lde_handle *h, const int32_t *lut) {
    PixStaged st;
    if (int rc = stage_pixel(h, lut, st)) return rc;
    HIPCALL(h, hipStreamSynchronize(h->stream));
    commit_pixel(h, st);
    return LDE_OK;
}

int ensure_win64(lde_handle *h) {
    if (h->d_win64) return LDE_OK;
    if (int rc = dev_alloc(h, &h->d_win64, (size_t)h->nbins)) return rc;
    HIPCALL(h, hipMemsetAsync(h->d_win64, 0, (size_t)h->nbins * 8, h->stream));
    return LDE_OK;
}

int zero_state(lde_handle *h) {
    const size_t nb = (size_t)h->nbins;
    HIPCALL(h, hipMemsetAsync(h->d_win32, 0, nb * 4, h->stream));
    HIPCALL(h, hipMemsetAsync(h->d_cum, 0, nb * 8, h->stream));
    if (h->d_cumrow) HIPCALL(h, hipMemsetAsync(h->d_cumrow, 0, (size_t)h->S * 16, h->stream));
    h->cumrow_ok = h->d_cumrow ? 1 : 0;
    if (h->d_win64) HIPCALL(h, hipMemsetAsync(h->d_win64, 0, nb * 8, h->stream));
    if (h->d_winf) HIPCALL(h, hipMemsetAsync(h->d_winf, 0, nb * 4, h->stream));
    if (h->d_cumf) HIPCALL(h, hipMemsetAsync(h->d_cumf, 0, nb * 4, h->stream));
    h->window_has_data = false;
    h->cum_has_data = false;
    h->win64_dirty = false;
    h->win_events = 0;
    h->f32_pending = false;
    return LDE_OK;
}

// float32 views: the pending push's f32 adds (k_merge_f32), before anything
// else reads or writes the f32 accumulators or the batch
int flush_f32(lde_handle *h) {
    if (!h->f32_pending) return LDE_OK;
    Timed tm(h, LDE_K_FINALIZE);
    HIPCALL(h, lde::launch_merge_f32(h->d_win32, h->d_win64, h->d_winf, h->d_cumf, h->nbins,
                                     h->pend_first_win, h->pend_first_cum, h->stream));
    h->f32_pending = false;
    return LDE_OK;
}

void convert_u64(const unsigned long long *src, void *dst, long long n, int dtype) {
    if (dtype == LDE_F32) {
        float *d = (float *)dst;
        for (long long i = 0; i < n; ++i) d[i] = (float)src[i];
    } else {
        double *d = (double *)dst;
        for (long long i = 0; i < n; ++i) d[i] = (double)src[i];
    }
}

void release(lde_handle *h) {
    if (!h) return;
    if (h->stream) (void)hipStreamSynchronize(h->stream);
    for (auto &l : h->launches) {
        (void)hipEventDestroy(l.a);
        (void)hipEventDestroy(l.b);
    }
    for (auto e : h->event_pool) (void)hipEventDestroy(e);
    for (void *p : {(void *)h->d_lut, (void *)h->d_tab, (void *)h->d_cbuck, (void *)h->d_cpd,
                    (void *)h->d_ctable, (void *)h->d_cedges, (void *)h->d_cbin, (void *)h->d_key_dist,
                    (void *)h->d_key_rec, (void *)h->d_key_tabi, (void *)h->d_ploc, (void *)h->d_pfp_off,
                    (void *)h->d_pfp_scr, (void *)h->d_pcounts, (void *)h->d_prstart, (void *)h->d_ppayload,
                    (void *)h->d_pctab, (void *)h->d_pitems, (void *)h->d_pitem_count, (void *)h->d_pprev,
                    (void *)h->d_povf, (void *)h->d_povf_grp, (void *)h->d_win32, (void *)h->d_win64,
                    (void *)h->d_cum, (void *)h->d_cumrow, (void *)h->d_winf, (void *)h->d_cumf, (void *)h->d_spid,
                    (void *)h->d_stoa, (void *)h->d_payload, (void *)h->d_starts, (void *)h->d_part,
                    (void *)h->d_ttot, (void *)h->d_tile_items, (void *)h->d_item_count, (void *)h->d_items,
                    (void *)h->d_segs, (void *)h->d_pages, (void *)h->d_page_tile, (void *)h->d_page_cnt,
                    (void *)h->d_list, (void *)h->d_pool_used, (void *)h->d_cntp, (void *)h->d_evp,
                    (void *)h->d_tile_pages, (void *)h->d_tile_events, (void *)h->d_tile_base,
                    (void *)h->d_overflow, (void *)h->d_items4, (void *)h->d_pix_cnt, (void *)h->d_glut,
                    (void *)h->d_sieve_tab, (void *)h->d_ttab, (void *)h->d_chunk_tab, (void *)h->d_sieve_dummy,
                    (void *)h->d_cold_tcnt, (void *)h->d_cold_boff, (void *)h->d_cold_keys,
                    (void *)h->d_cold_items, (void *)h->d_cold_ttot, (void *)h->d_row_screen,
                    (void *)h->d_sel_stats, (void *)h->d_sample_part, (void *)h->d_screen_cnt,
                    (void *)h->d_screen_row, (void *)h->d_hot_part, (void *)h->d_cold, (void *)h->d_cold_cnt,
                    (void *)h->d_hot_fmt, (void *)h->d_tot4, (void *)h->d_snap, (void *)h->d_wtree,
                    (void *)h->d_wtab, (void *)h->d_wpixcnt, (void *)h->d_wcounters, (void *)h->d_wctab,
                    (void *)h->d_wpages1, (void *)h->d_wpages2, (void *)h->d_wpage_cnt, (void *)h->d_wpage_part,
                    (void *)h->d_wlist, (void *)h->d_wrows1, (void *)h->d_wrows2, (void *)h->d_witems1,
                    (void *)h->d_witems2, (void *)h->d_wband})
        if (p) (void)hipFree(p);
    for (void *p : {(void *)h->h_ppid, (void *)h->h_ptoa, (void *)h->h_segs, (void *)h->h_sel_stats,
                    (void *)h->h_pack})
        if (p) (void)hipHostFree(p);
    for (hipEvent_t e : {h->pin_done, h->segs_done, h->fin_event, h->block_event})
        if (e) (void)hipEventDestroy(e);
    if (h->d_trace && !h->trace_stats.empty()) {
        const size_t n = h->trace_stats.size() / 6;
        double a[6] = {0, 0, 0, 0, 0, 0};
        for (size_t i = 0; i < n; ++i)
            for (int q = 0; q < 6; ++q) a[q] += h->trace_stats[6 * i + q];
        fprintf(stderr,
                "lde sieve trace (%zu launches, us): block start spread %.2f, stream-end spread %.2f, "
                "end spread %.2f, first start -> last end %.2f, mean block init -> stream end %.2f, "
                "mean block start -> init %.2f\n",
                n, a[0] / n, a[1] / n, a[2] / n, a[3] / n, a[4] / n, a[5] / n);
    }
    dev_free(h->d_trace);
    for (auto &g : h->groups) {
        dev_free(g.d_items);
        dev_free(g.d_screens);
        dev_free(g.d_out);
    }
    if (h->own_stream && h->stream) (void)hipStreamDestroy(h->stream);
    delete h;
}

}  // namespace

// ===========================================================================
// C ABI
// ===========================================================================
extern "C" {

int lde_abi_version(void) { return LDE_ABI_VERSION; }

// lde_host_alloc blocks: host base -> (bytes, device address)
namespace {
struct HostBlock {
    size_t bytes;
    unsigned char *dev;
};
std::mutex g_host_mu;
std::map<uintptr_t, HostBlock> g_host_blocks;

// device address of host pointer p inside an lde_host_alloc block with n
// bytes from p on, else nullptr
void *mapped_device_ptr(const void *p, size_t n) {
    if (!p) return nullptr;
    const uintptr_t a = (uintptr_t)p;
    std::lock_guard<std::mutex> lk(g_host_mu);
    if (g_host_blocks.empty()) return nullptr;
    auto it = g_host_blocks.upper_bound(a);
    if (it == g_host_blocks.begin()) return nullptr;
    --it;
    if (a + n > it->first + it->second.bytes) return nullptr;
    return it->second.dev + (a - it->first);
}
}  // namespace

int lde_host_alloc(int64_t bytes, void **out) {
    if (!out) return fail(nullptr, LDE_EINVAL, "out is NULL");
    *out = nullptr;
    if (bytes <= 0) return fail(nullptr, LDE_EINVAL, "bytes must be positive");
    void *p = nullptr;
    hipError_t e = hipHostMalloc(&p, (size_t)bytes, hipHostMallocCoherent | hipHostMallocPortable);
    if (e != hipSuccess)
        return fail(nullptr, LDE_ENOMEM, "hipHostMalloc(%lld bytes) failed: %s", (long long)bytes,
                    hipGetErrorString(e));
    void *d = nullptr;
    e = hipHostGetDevicePointer(&d, p, 0);
    if (e != hipSuccess) {
        (void)hipHostFree(p);
        return fail(nullptr, LDE_EHIP, "hipHostGetDevicePointer failed: %s", hipGetErrorString(e));
    }
    {
        std::lock_guard<std::mutex> lk(g_host_mu);
        g_host_blocks[(uintptr_t)p] = HostBlock{(size_t)bytes, (unsigned char *)d};
    }
    *out = p;
    return LDE_OK;
}

int lde_host_free(void *p) {
    if (!p) return LDE_OK;
    {
        std::lock_guard<std::mutex> lk(g_host_mu);
        auto it = g_host_blocks.find((uintptr_t)p);
        if (it == g_host_blocks.end())
            return fail(nullptr, LDE_EINVAL, "pointer was not returned by lde_host_alloc");
        g_host_blocks.erase(it);
    }
    hipError_t e = hipHostFree(p);
    if (e != hipSuccess) return fail(nullptr, LDE_EHIP, "hipHostFree failed: %s", hipGetErrorString(e));
    return LDE_OK;
}

const char *lde_last_error(const lde_handle *h) {
    return h ? h->err.c_str() : g_create_error.c_str();
}

int lde_create(const lde_config *cfg, lde_handle **out) {
    if (!out) return fail(nullptr, LDE_EINVAL, "out is NULL");
    *out = nullptr;
    if (!cfg) return fail(nullptr, LDE_EINVAL, "config is NULL");
    if (cfg->abi_version != LDE_ABI_VERSION)
        return fail(nullptr, LDE_EINVAL, "abi_version %d != %d", cfg->abi_version, LDE_ABI_VERSION);
    if (int rc = check_knobs()) return rc;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
        return fail(nullptr, LDE_EHIP, "no HIP device available");
    if (cfg->device_id < 0 || cfg->device_id >= ndev)
        return fail(nullptr, LDE_EINVAL, "device_id %d out of range (%d devices)", cfg->device_id, ndev);
    if (cfg->n_screen < 1) return fail(nullptr, LDE_EINVAL, "n_screen must be >= 1");
    if (cfg->n_replicas < 1) return fail(nullptr, LDE_EINVAL, "n_replicas must be >= 1");
    if (cfg->out_dtype != LDE_F64 && cfg->out_dtype != LDE_F32)
        return fail(nullptr, LDE_EINVAL, "out_dtype must be LDE_F64 or LDE_F32");
    const bool monitor = cfg->out_lut == nullptr;
    if (monitor && (cfg->n_screen != 1 || cfg->n_replicas != 1))
        return fail(nullptr, LDE_EINVAL, "a NULL out_lut (monitor) requires n_screen = n_replicas = 1");
    if (!monitor && (cfg->lut_len < 1 || cfg->lut_len > 0x7fffffffLL))
        return fail(nullptr, LDE_EINVAL, "lut_len must be in [1, 2^31)");
    const long long nbins = cfg->n_screen * (long long)cfg->n_toa_bins;
    if (cfg->n_toa_bins < 1 || nbins > 0x7fffffffLL)
        return fail(nullptr, LDE_EINVAL, "n_screen * n_toa_bins must be in [1, 2^31)");

    lde_handle *h = new (std::nothrow) lde_handle();
    if (!h) return fail(nullptr, LDE_ENOMEM, "out of host memory");
    h->device = cfg->device_id;
    DeviceGuard guard(h->device);
    std::vector<unsigned char> tab;
    int rc = build_toa_tables(h, cfg->toa_edges, cfg->n_toa_bins, tab, h->tp);
    if (!rc) h->edges.assign(cfg->toa_edges, cfg->toa_edges + cfg->n_toa_bins + 1);
    if (rc) {
        g_create_error = h->err;
        release(h);
        return rc;
    }
#define CREATE_CHECK(expr)                          \
    do {                                            \
        int rc_ = (expr);                           \
        if (rc_) {                                  \
            g_create_error = h->err;                \
            release(h);                             \
            return rc_;                             \
        }                                           \
    } while (0)
#define CREATE_HIP(expr) CREATE_CHECK(((expr) == hipSuccess) ? 0 : fail(h, LDE_EHIP, "%s failed", #expr))

    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, h->device) == hipSuccess && prop.multiProcessorCount > 0)
        h->cus = prop.multiProcessorCount;
    if (cfg->stream) {
        h->stream = (hipStream_t)cfg->stream;
    } else {
        CREATE_HIP(hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking));
        h->own_stream = true;
    }
    h->pid_off = cfg->pid_offset;
    h->R = cfg->n_replicas;
    h->L = monitor ? 0 : cfg->lut_len;
    h->monitor = monitor;
    h->S = cfg->n_screen;
    h->T = cfg->n_toa_bins;
    h->nbins = nbins;
    h->out_dtype = cfg->out_dtype;
    h->strategy = cfg->strategy;
    if (cfg->range_lo < 0 && cfg->range_hi < 0) {
        h->range_lo = 0;
        h->range_hi = h->T;
    } else {
        if (cfg->range_lo < 0 || cfg->range_hi > h->T || cfg->range_lo > cfg->range_hi) {
            int r = fail(h, LDE_EINVAL, "range [%d, %d) invalid for %d bins", cfg->range_lo,
                         cfg->range_hi, h->T);
            g_create_error = h->err;
            release(h);
            return r;
        }
        h->range_lo = cfg->range_lo;
        h->range_hi = cfg->range_hi;
    }

    // LUT: u16 screen index (0xFFFF = dropped) when S < 65535, else int32
    // screen*T premultiplied (-1 = dropped); validated here
    if (!monitor) {
        h->lut16 = h->S < 0xFFFF && env_ll("LDE_LUT32", 0) == 0;
        CREATE_CHECK(upload_lut(h, cfg->out_lut));
        if (cfg->strategy < LDE_STRATEGY_AUTO || cfg->strategy > LDE_STRATEGY_WIDE)
            CREATE_CHECK(fail(h, LDE_EINVAL, "unknown strategy %d", cfg->strategy));
    }
    CREATE_CHECK(dev_alloc(h, &h->d_tab, tab.size()));
    CREATE_HIP(hipMemcpy(h->d_tab, tab.data(), tab.size(), hipMemcpyHostToDevice));

    // histograms
    CREATE_CHECK(dev_alloc(h, &h->d_win32, (size_t)nbins));
    CREATE_CHECK(dev_alloc(h, &h->d_cum, (size_t)nbins));
    CREATE_CHECK(dev_alloc(h, &h->d_cumrow, (size_t)h->S * 2));
    h->cum32 = (h->out_dtype != LDE_F32 && h->T % 4 == 0 && h->T > 128 && env_ll("LDE_CUM32", 1) != 0) ? nbins : 0;
    if (h->out_dtype == LDE_F32) {
        CREATE_CHECK(dev_alloc(h, &h->d_winf, (size_t)nbins));
        CREATE_CHECK(dev_alloc(h, &h->d_cumf, (size_t)nbins));
        CREATE_CHECK(ensure_win64(h));
    }
    CREATE_CHECK(dev_alloc(h, &h->d_tot4, 4 + 4 * 8192));  // totals + per-block partials
    // the finalize pack in coherent host memory the finalize kernel writes:
    // [current image S x 8][cumulative image S x 8][totals 32][overflow 16]
    // [per-block total partials, kHostPartials x 32] (summed on the host)
    h->pack_bytes = (size_t)h->S * 16 + 48 + 32 * (size_t)lde::kHostPartials;
    CREATE_HIP(hipHostMalloc((void **)&h->h_pack, h->pack_bytes, hipHostMallocCoherent));
    CREATE_HIP(hipHostGetDevicePointer((void **)&h->hd_pack, h->h_pack, 0));
    CREATE_HIP(hipEventCreateWithFlags(&h->fin_event, hipEventDisableTiming));
    CREATE_CHECK(zero_state(h));

    // partition workspace: tiles of 2^14 bins, or 2^15 when that keeps the
    // tiles <= kMaxTiles and the PAGED pass-A carve within its LDS
    if (!monitor) {
        int tb = (int)std::max<long long>(14, std::min<long long>(15, env_ll("LDE_TILE_BITS", 14)));
        auto tiles = [&](int b) { return (nbins + (1LL << b) - 1) >> b; };
        while (tb < 15 && (tiles(tb) > lde::kMaxTiles ||
                           lde::paged_smem((int)std::min<long long>(tiles(tb), lde::kMaxTiles), 1,
                                           h->tp) > lde::kPagedSmemMax))
            ++tb;
        const long long nt = tiles(tb);
        const bool smem_ok = nt <= lde::kMaxTiles &&
                             lde::partition_smem((int)nt, h->tp) <= 64 * 1024 &&
                             lde::paged_smem((int)nt, 1, h->tp) <= lde::kPagedSmemMax;
        h->subc = (smem_ok && lde::paged_smem((int)nt, 4, h->tp) <= lde::kPagedSmemMax) ? 4 : 1;
        if (nt <= lde::kMaxTiles && smem_ok) {
            h->tile_bits = tb;
            h->n_tiles = (int)nt;
            h->part_rows = 2 * h->cus;
            h->part_grid = (int)std::min<long long>(
                h->part_rows, std::max<long long>(1, env_ll("LDE_PART_GRID", 2LL * h->cus)));
            CREATE_CHECK(dev_alloc(h, &h->d_part, (size_t)h->part_rows * h->n_tiles));
            CREATE_CHECK(dev_alloc(h, &h->d_ttot, (size_t)h->n_tiles));
            CREATE_CHECK(dev_alloc(h, &h->d_tile_items, (size_t)h->n_tiles));
            CREATE_CHECK(dev_alloc(h, &h->d_item_count, 1));
        } else {
            h->n_tiles = 0;  // partition unavailable -> atomic strategy
        }
        // SPLIT (the SIEVE pass): needs the LDS pixel table, the fast TOA
        // layout with T <= 254, keys below 2^22, table tags below 255 and a
        // tile-sorted cold pipeline of <= kSortThreads tiles; its LDS carve
        // bounds the hot rows
        auto bits = [](long long n) { int b = 0; while ((1LL << b) < n) ++b; return b; };
        int cbits = (int)std::max<long long>(0, std::min<long long>(16, env_ll("LDE_PIXEL_CACHE_BITS", 13)));
        // whole LUT fits; at least 4 slots, as the sieve copies the table and
        // the TOA words in 16-byte units from offset C (a 2-pixel
        // view had C = 2, so no table word was copied and the TOA words
        // landed at the table's offset)
        if ((1LL << cbits) >= 2 * h->L) cbits = std::max(2, bits(h->L));
        std::vector<uint32_t> tt;
        int tsh = 0;
        uint32_t tcap = 0;
        const size_t budget = lde::kSplitSmemMax;
        if (h->n_tiles > 0 && h->n_tiles <= lde::kSortThreadsHost && h->S * 4 <= 160 * 1024 && cbits > 0 &&
            env_ll("LDE_SPLIT", 1) != 0 && build_sieve_toa(h->tp, tab, tt, tsh, tcap) &&
            (unsigned long long)h->S * h->T <= (unsigned long long)lde::kSieveValueMask + 1ULL &&
            ((h->L - 1) >> cbits) < 255 && h->L < 0x3fffffffLL) {
            // room for the integer-edge table of wavelength mode (edges 0..T:
            // T + 1 bucket words), so lde_set_coord_lut keeps the sieve
            if (tt.size() < (size_t)lde::align4(h->T + 2)) tt.resize((size_t)lde::align4(h->T + 2), 0u);
            auto rows_for = [&](int cb) {
                const size_t fixed = lde::sieve_smem(0, cb, (int)tt.size(), h->n_tiles);
                int H = 0;
                if (fixed < budget)
                    H = (int)std::min<long long>(lde::kHotMaxRows, (long long)((budget - fixed) / (4 * (size_t)h->T)));
                while (H > 0 && lde::sieve_smem((H * h->T + 7) & ~7, cb, (int)tt.size(), h->n_tiles) > budget) --H;
                return (int)std::min<long long>(H, h->S);
            };
            // the pixel table never takes the room of the last 64 hot rows
            while (cbits > 8 && rows_for(cbits) < std::min<long long>(64, h->S)) --cbits;
            // views with few screens (DREAM strip_view: 256): a smaller pixel
            // table (down to 2^10 slots) when it makes room for a hot row per
            // screen, so that no event is cold and the cold-key pipeline never
            // runs (a table miss costs a gather; a cold key a sort and a pass)
            if (h->S <= lde::kHotMaxRows && rows_for(cbits) < h->S)
                for (int cb = cbits - 1; cb >= 10; --cb)
                    if (rows_for(cb) >= h->S) {
                        cbits = cb;
                        break;
                    }
            int H = rows_for(cbits);
            const long long hmax = env_ll("LDE_HOT_ROWS", 0);  // diagnostics: a row budget
            if (hmax > 0) H = (int)std::min<long long>(H, hmax);
            if (H >= 8 && (unsigned long long)H * h->T <= (unsigned long long)lde::kSieveValueMask + 1ULL &&
                ((h->L - 1) >> cbits) < 255) {
                h->split_ok = true;
                h->hot_rows = H;
                h->cache_bits = cbits;
                h->ttab = std::move(tt);
                h->ttab_shift = tsh;
                h->ttab_cap = tcap;
            }
        }
        if (h->split_ok) {
            h->split_grid = (int)std::max<long long>(1, env_ll("LDE_SPLIT_GRID", (long long)h->cus));
            h->hot_refresh = (int)std::max<long long>(1, env_ll("LDE_HOT_REFRESH", 256));
            h->split_min_cov = (double)env_ll("LDE_SPLIT_MIN_COV_PCT", 30) / 100.0;
            h->hot_uses.assign((size_t)h->R, -1);
            h->hot_cov.assign((size_t)h->R, 0.0);
            h->all_hot.assign((size_t)h->R, 0);
            const int cbits2 = h->cache_bits;
            CREATE_CHECK(dev_alloc(h, &h->d_pix_cnt, (size_t)h->L));
            CREATE_CHECK(dev_alloc(h, &h->d_glut, (size_t)h->R * (size_t)(h->L + 1)));
            CREATE_CHECK(dev_alloc(h, &h->d_sieve_tab, (size_t)h->R << cbits2));
            CREATE_CHECK(dev_alloc(h, &h->d_ttab, h->ttab.size()));
            CREATE_HIP(hipMemcpy(h->d_ttab, h->ttab.data(), h->ttab.size() * 4, hipMemcpyHostToDevice));
            std::vector<int> dum((size_t)lde::kChunk, (int)((unsigned)h->pid_off - 1u));
            CREATE_CHECK(dev_alloc(h, &h->d_sieve_dummy, dum.size()));
            CREATE_HIP(hipMemcpy(h->d_sieve_dummy, dum.data(), dum.size() * 4, hipMemcpyHostToDevice));
            CREATE_CHECK(dev_alloc(h, &h->d_cold_ttot, (size_t)h->n_tiles));
            CREATE_CHECK(dev_alloc(h, &h->d_row_screen, (size_t)h->R * lde::kHotMaxRows));
            CREATE_CHECK(dev_alloc(h, &h->d_sel_stats, (size_t)h->R * 4));
            CREATE_CHECK(dev_alloc(h, &h->d_sample_part, (size_t)lde::kSampleBlocks * h->S));
            CREATE_CHECK(dev_alloc(h, &h->d_screen_cnt, (size_t)h->S));
            CREATE_CHECK(dev_alloc(h, &h->d_screen_row, (size_t)h->S));
            CREATE_CHECK(dev_alloc(h, &h->d_cold_cnt, (size_t)h->split_grid * (lde::kSplitThreads / 64)));
            CREATE_CHECK(dev_alloc(h, &h->d_hot_fmt, (size_t)h->split_grid));
            if (env_ll("LDE_SIEVE_TRACE", 0) != 0)
                CREATE_CHECK(dev_alloc(h, &h->d_trace, (size_t)h->split_grid * 4));
            CREATE_HIP(hipHostMalloc((void **)&h->h_sel_stats, (size_t)h->R * 16, hipHostMallocDefault));
        }
#ifdef LDE_DIAGNOSTICS
        h->sieve_ablate = (int)env_ll("LDE_SIEVE_ABLATE", 0);
        h->cold_sort_ablate = (int)env_ll("LDE_COLD_SORT_ABLATE", 0);
#endif
        h->probe = env_ll("LDE_HOST_PROBE", 0) != 0;
        h->item_events_override = env_ll("LDE_ITEM_EVENTS", 0);
    }
    if (!monitor) CREATE_CHECK(build_pixel(h, cfg->out_lut));
    if (!monitor) CREATE_CHECK(setup_wide(h));
    CREATE_HIP(hipEventCreateWithFlags(&h->pin_done, hipEventDisableTiming));
    CREATE_HIP(hipEventCreateWithFlags(&h->segs_done, hipEventDisableTiming));
    CREATE_HIP(hipStreamSynchronize(h->stream));
#undef CREATE_CHECK
#undef CREATE_HIP
    *out = h;
    return LDE_OK;
}

void lde_destroy(lde_handle *h) {
    if (!h) return;
    if (h->probe && h->probe_n)
        fprintf(stderr, "lde probe: accumulate entry -> sieve launched %.2f us mean, %.2f us min (%lld)\n",
                h->probe_us / h->probe_n, h->probe_min, h->probe_n);
    if (h->probe && h->probe_fin_n)
        fprintf(stderr, "lde probe: finalize after the stream wait (copies, totals) %.2f us mean (%lld)\n",
                h->probe_fin_post_us / h->probe_fin_n, h->probe_fin_n);
    DeviceGuard guard(h->device);
    release(h);
}

int lde_stage(lde_handle *h, const int32_t *pid, const int32_t *toa, int64_t n) {
    if (!h) return fail(nullptr, LDE_EINVAL, "handle is NULL");
    if (n < 0) return fail(h, LDE_EINVAL, "negative event count");
    if (n == 0) return LDE_OK;
    if (!toa || (!h->monitor && !pid))
        return fail(h, LDE_EINVAL, "event arrays must not be NULL");
    DeviceGuard guard(h->device);
    // the pinned ring is reused batch to batch: wait for the previous batch's copies
    if (h->staged_host == 0 && h->pin_pending) {
        HIPCALL(h, hipEventSynchronize(h->pin_done));
        h->pin_pending = false;
    }
    if (int rc = ensure_stage_capacity(h, h->staged_host + n)) return rc;
    const long long off = h->staged_host;
    // Large messages: split into chunks; worker threads each memcpy a chunk
    // into the pinned ring and queue its H2D right away, so the host copies
    // run in parallel and overlap the PCIe transfers of earlier chunks.  The
    // single-thread memcpy, not PCIe, bounded the end-to-end rate.
    const long long chunk = 1 << 20;
    const int arrays = h->monitor ? 1 : 2;
    const long long n_chunks = (n + chunk - 1) / chunk;
    const int workers = (int)std::min<long long>(
        std::max<long long>(1, env_ll("LDE_STAGE_THREADS", 8)), n_chunks * arrays);
    auto copy_chunk = [&](long long item) -> hipError_t {
        const int a = (int)(item % arrays);
        const long long c0 = (item / arrays) * chunk;
        const long long cn = std::min(chunk, n - c0);
        int *hp = (a == 0 ? h->h_ptoa : h->h_ppid) + off + c0;
        int *dp = (a == 0 ? h->d_stoa : h->d_spid) + off + c0;
        const int32_t *src = (a == 0 ? toa : pid) + c0;
        std::memcpy(hp, src, (size_t)cn * 4);
        return hipMemcpyAsync(dp, hp, (size_t)cn * 4, hipMemcpyHostToDevice, h->stream);
    };
    if (workers <= 1) {
        for (long long it = 0; it < n_chunks * arrays; ++it) HIPCALL(h, copy_chunk(it));
    } else {
        std::atomic<long long> next{0};
        std::atomic<int> err{(int)hipSuccess};
        auto work = [&]() {
            (void)hipSetDevice(h->device);
            for (long long it; (it = next.fetch_add(1)) < n_chunks * arrays;) {
                const hipError_t e = copy_chunk(it);
                if (e != hipSuccess) err.store((int)e);
            }
        };
        std::vector<std::thread> pool;
        pool.reserve(workers - 1);
        for (int w = 1; w < workers; ++w) pool.emplace_back(work);
        work();
        for (auto &t : pool) t.join();
        HIPCALL(h, (hipError_t)err.load());
    }
    HIPCALL(h, hipEventRecord(h->pin_done, h->stream));
    h->pin_pending = true;
    h->staged_host += n;
    return LDE_OK;
}

int lde_rebin_f64(const double *d_src_edges, const double *d_src_values, int64_t n_src,
                  const double *d_dst_edges, int64_t n_dst, double *d_out_a, double *d_out_b,
                  void *stream) {
    if (n_src < 1 || n_dst < 1) return fail(nullptr, LDE_EINVAL, "rebin needs at least one bin");
    if (!d_src_edges || !d_src_values || !d_dst_edges)
        return fail(nullptr, LDE_EINVAL, "rebin arrays must not be NULL");
    if (!d_out_a && !d_out_b) return LDE_OK;
    const hipError_t e = lde::launch_rebin_f64(d_src_edges, d_src_values, n_src, d_dst_edges, n_dst,
                                               d_out_a, d_out_b, (hipStream_t)stream);
    if (e != hipSuccess) return fail(nullptr, LDE_EHIP, "k_rebin_f64: %s", hipGetErrorString(e));
    return LDE_OK;
}

int lde_ev44_decode(const uint8_t *buf, int64_t len, lde_ev44_view *out) {
    std::string err;
    const int rc = lde::ev44_parse(buf, len, out, &err);
    if (rc) return fail(nullptr, rc, "%s", err.c_str());
    return LDE_OK;
}

int lde_stage_ev44(lde_handle *h, const uint8_t *buf, int64_t len, int64_t kafka_timestamp_ms,
                   int32_t flags, int64_t *timestamp_ns) {
    if (!h) return fail(nullptr, LDE_EINVAL, "handle is NULL");
    if (flags & ~(LDE_EV44_SINGLE_PULSE | LDE_EV44_MONITOR))
        return fail(h, LDE_EINVAL, "unknown ev44 flags 0x%x", (unsigned)flags);
    if ((flags & LDE_EV44_MONITOR) && !h->monitor)
        return fail(h, LDE_EINVAL, "LDE_EV44_MONITOR on a detector handle");
    if (h->monitor) flags |= LDE_EV44_MONITOR;
    lde_ev44_view v;
    std::string err;
    int rc = lde::ev44_parse(buf, len, &v, &err);
    if (!rc) rc = lde::ev44_events(&v, kafka_timestamp_ms, flags, timestamp_ns, &err);
    if (rc) return fail(h, rc, "%s", err.c_str());
    // the vectors may be unaligned inside the payload: lde_stage only memcpy's them
    return lde_stage(h, h->monitor ? nullptr : (const int32_t *)v.pixel_id,
                     (const int32_t *)v.time_of_flight, v.n_time_of_flight);
}

int lde_stage_device(lde_handle *h, const void *d_pid, const void *d_toa, int64_t n) {
    if (!h) return fail(nullptr, LDE_EINVAL, "handle is NULL");
    if (n < 0) return fail(h, LDE_EINVAL, "negative event count");
    if (n == 0) return LDE_OK;
    if (!d_toa || (!h->monitor && !d_pid))
        return fail(h, LDE_EINVAL, "event arrays must not be NULL");
    h->dev_segments.push_back({(const int *)d_pid, (const int *)d_toa, (long long)n});
    return LDE_OK;
}

int lde_stage_device_batch(lde_handle *h, int64_t count, const void *const *d_pids,
                           const void *const *d_toas, const int64_t *ns) {
    if (!h) return fail(nullptr, LDE_EINVAL, "handle is NULL");
    if (count < 0) return fail(h, LDE_EINVAL, "negative message count");
    if (count > 0 && (!d_toas || !ns || (!h->monitor && !d_pids)))
        return fail(h, LDE_EINVAL, "message arrays must not be NULL");
    for (int64_t i = 0; i < count; ++i) {
        if (ns[i] < 0) return fail(h, LDE_EINVAL, "negative event count in message %lld", (long long)i);
        if (ns[i] > 0 && (!d_toas[i] || (!h->monitor && !d_pids[i])))
            return fail(h, LDE_EINVAL, "event arrays of message %lld must not be NULL", (long long)i);
    }
    for (int64_t i = 0; i < count; ++i)
        if (ns[i] > 0)
            h->dev_segments.push_back({h->monitor ? nullptr : (const int *)d_pids[i],
                                       (const int *)d_toas[i], (long long)ns[i]});
    return LDE_OK;
}

namespace {
int accumulate_impl(lde_handle *h, int32_t replica, unsigned long long *d_push);
}

int lde_accumulate(lde_handle *h, int32_t replica) { return accumulate_impl(h, replica, nullptr); }

int lde_accumulate_push(lde_handle *h, int32_t replica, void *d_counts) {
    if (!h) return fail(nullptr, LDE_EINVAL, "handle is NULL");
    if (!d_counts) return fail(h, LDE_EINVAL, "push buffer is NULL");
    if (h->out_dtype != LDE_F32)
        return fail(h, LDE_EINVAL, "push export is for float32 views (integer views merge exactly "
                                   "at finalize)");
    return accumulate_impl(h, replica, (unsigned long long *)d_counts);
}

int lde_push_u64(lde_handle *h, const void *d_counts) {
    if (!h) return fail(nullptr, LDE_EINVAL, "handle is NULL");
    if (!d_counts) return fail(h, LDE_EINVAL, "push buffer is NULL");
    if (h->out_dtype != LDE_F32) return fail(h, LDE_EINVAL, "lde_push_u64 is for float32 views");
    DeviceGuard guard(h->device);
    if (int rc = ensure_win64(h)) return rc;
    if (int rc = flush_f32(h)) return rc;
    {
        Timed tm(h, LDE_K_FINALIZE);
        HIPCALL(h, lde::launch_merge_f32_u64((const unsigned long long *)d_counts, h->d_win64,
                                             h->d_winf, h->d_cumf, h->nbins,
                                             h->window_has_data ? 0 : 1, h->cum_has_data ? 0 : 1,
                                             h->stream));
    }
    h->win64_dirty = true;
    h->window_has_data = true;
    h->cum_has_data = true;
    return LDE_OK;
}

namespace {
int accumulate_impl(lde_handle *h, int32_t replica, unsigned long long *d_push) {
    if (!h) return fail(nullptr, LDE_EINVAL, "handle is NULL");
    if (replica < 0 || replica >= h->R)
        return fail(h, LDE_EINVAL, "replica %d out of range [0, %d)", replica, h->R);
    DeviceGuard guard(h->device);
    if (h->probe) h->t_acc0 = std::chrono::steady_clock::now();
    // the batch buffer is about to be binned into: the last push merges first
    if (int rc = flush_f32(h)) return rc;
    std::vector<Segment> segs;
    if (h->staged_host > 0) segs.push_back({h->d_spid, h->d_stoa, h->staged_host});
    for (const Segment &s : h->dev_segments) segs.push_back(s);
    long long total = 0;
    for (const Segment &s : segs) total += s.n;
    // wavelength mode: every event's coordinate bin replaces its time as the
    // value binned against the integer edges 0..T -- computed here, or inside
    // the SIEVE path by the keyed pass (coord_deferred)
    const bool coord_deferred = h->coord && total > 0 && coord_keyed_candidate(h, total);
    if (h->coord && total > 0 && !coord_deferred)
        if (int rc = coord_prepass(h, segs)) return rc;

    // split into pieces that cannot overflow a u32 window bin
    const long long piece_max = 1LL << 31;
    std::vector<std::vector<Segment>> pieces;
    {
        std::vector<Segment> cur;
        long long in_cur = 0;
        for (Segment s : segs) {
            while (s.n > 0) {
                const long long take = std::min(s.n, piece_max - in_cur);
                cur.push_back({s.pid ? s.pid : nullptr, s.toa, take});
                in_cur += take;
                s.pid = s.pid ? s.pid + take : nullptr;
                s.toa += take;
                s.n -= take;
                if (in_cur == piece_max) {
                    pieces.push_back(cur);
                    cur.clear();
                    in_cur = 0;
                }
            }
        }
        if (!cur.empty()) pieces.push_back(cur);
    }
    const bool f32 = h->out_dtype == LDE_F32;
    {
        // BINNING range: a start marker (the GPU waits for the host here
        // anyway) and, on the sieve path, a stop stamped by the last kernel's
        // own dispatch instead of a marker in front of the finalize kernels
        hipEvent_t bin_a = nullptr, bin_b = nullptr;
        if (h->timing && ((h->timing_mask >> LDE_K_BINNING) & 1u)) {
            bin_a = pool_event(h);
            bin_b = bin_a ? pool_event(h) : nullptr;
            if (bin_a && !bin_b) {
                h->event_pool.push_back(bin_a);
                bin_a = nullptr;
            }
            if (bin_a) (void)hipEventRecord(bin_a, h->stream);
        }
        struct BinRange {
            lde_handle *h;
            hipEvent_t a, b;
            ~BinRange() {
                h->bin_stop_ext = nullptr;
                if (!a) return;
                if (!h->bin_stop_used) (void)hipEventRecord(b, h->stream);
                h->launches.push_back({LDE_K_BINNING, a, b});
            }
        } bin_range{h, bin_a, bin_b};
        h->bin_stop_used = false;
        for (size_t pi = 0; pi < pieces.size(); ++pi) {
            auto &p = pieces[pi];
            h->bin_stop_ext = pi + 1 == pieces.size() ? bin_b : nullptr;
            long long n = 0;
            for (auto &s : p) n += s.n;
            if (!f32 && h->win_events + (unsigned long long)n > 0xffffffffULL) {
                if (int rc = ensure_win64(h)) return rc;
                HIPCALL(h, lde::launch_fold_window(h->d_win32, h->d_win64, h->nbins, h->stream));
                h->win64_dirty = true;
                h->win_events = 0;
            }
            if (int rc = bin_segments(h, p, n, replica, coord_deferred)) return rc;
            h->win_events += (unsigned long long)n;
        }
    }
    if (d_push) {
        // the push's exact counts leave for the merge (lde_push_u64 on the
        // root); this handle's accumulators are untouched
        HIPCALL(h, lde::launch_push_export(h->d_win32, d_push, h->nbins, h->stream));
        h->win_events = 0;
        h->events_binned += total;
        h->staged_host = 0;
        h->dev_segments.clear();
        return LDE_OK;
    }
    if (f32) {
        // this push's f32 adds wait for the next accumulate or the finalize
        h->f32_pending = true;
        h->pend_first_win = h->window_has_data ? 0 : 1;
        h->pend_first_cum = h->cum_has_data ? 0 : 1;
        h->win64_dirty = true;
        h->win_events = 0;
    }
    h->events_binned += total;
    h->window_has_data = true;
    h->cum_has_data = true;
    h->staged_host = 0;
    h->dev_segments.clear();
    return LDE_OK;
}
}  // namespace

int lde_finalize_begin(lde_handle *h, lde_outputs *out) {
    if (!h) return fail(nullptr, LDE_EINVAL, "handle is NULL");
    if (h->fin_pending) return fail(h, LDE_ESTATE, "a finalize is pending (lde_finalize_end)");
    if (!h->window_has_data) return fail(h, LDE_ENODATA, "No data has been added");
    DeviceGuard guard(h->device);
    const bool f32 = h->out_dtype == LDE_F32;
    const size_t nb = (size_t)h->nbins;
    lde_outputs dummy;
    std::memset(&dummy, 0, sizeof dummy);
    if (!out) out = &dummy;
    const bool want_cur_hist = out->current_hist != nullptr;
    const bool want_cum_hist = out->cumulative_hist != nullptr;
    if (want_cur_hist && !f32 && !h->d_snap)
        if (int rc = dev_alloc(h, &h->d_snap, nb)) return rc;
    // outputs go straight into the host-mapped pack, images into the caller's
    // lde_host_alloc memory in place when they live there
    unsigned char *pk = h->hd_pack;
    void *img_cur = pk, *img_cum = pk + (size_t)h->S * 8;
    const size_t img_bytes = (size_t)h->S * (f32 ? 4 : 8);
    void *const map_cur = mapped_device_ptr(out->current_image, img_bytes);
    void *const map_cum = mapped_device_ptr(out->cumulative_image, img_bytes);
    if (map_cur) img_cur = map_cur;
    if (map_cum) img_cum = map_cum;
    int n_parts = 0;
    // the per-block total partials and the overflow flag land in the pack
    // (summed here on the host: no k_sum_totals launch and gap)
    unsigned char *d_tail = pk + (size_t)h->S * 16;
    if (f32) {
        // one pass: the pending push's f32 adds, images, exact totals and
        // cumulative, window reset (k_finalize_f32)
        float *snap = nullptr;
        if (want_cur_hist) {
            if (!h->d_snap)
                if (int rc = dev_alloc(h, &h->d_snap, nb)) return rc;
            snap = reinterpret_cast<float *>(h->d_snap);
        }
        {
            Stamp sp(h, LDE_K_FINALIZE);
            HIPCALL(h, lde::launch_finalize_f32(
                           h->f32_pending ? h->d_win32 : nullptr, h->d_win64, h->d_cum, h->d_winf, h->d_cumf, snap,
                           h->S, h->T, h->range_lo, h->range_hi, h->pend_first_win, h->pend_first_cum,
                           out->current_image ? (float *)img_cur : nullptr,
                           out->cumulative_image ? (float *)img_cum : nullptr, (unsigned long long *)(d_tail + 48),
                           h->d_overflow, (uint32_t *)(d_tail + 32), &n_parts, h->stream, sp.a, sp.b));
            sp.done = true;
        }
        h->cumrow_ok = 0;  // (the f32 finalize does not keep the per-screen sums)
        h->f32_pending = false;
        if (want_cur_hist)
            HIPCALL(h, hipMemcpyAsync(out->current_hist, snap, nb * 4, hipMemcpyDeviceToHost, h->stream));
        if (want_cum_hist)
            HIPCALL(h, hipMemcpyAsync(out->cumulative_hist, h->d_cumf, nb * 4, hipMemcpyDeviceToHost,
                                      h->stream));
    } else {
        Timed tm(h, LDE_K_FINALIZE);
        HIPCALL(h, lde::launch_finalize(
                       0, h->d_win32, h->win64_dirty ? h->d_win64 : nullptr, h->d_cum,
                       want_cur_hist ? h->d_snap : nullptr, h->S, h->T, h->range_lo,
                       h->range_hi, out->current_image ? img_cur : nullptr,
                       out->cumulative_image ? img_cum : nullptr, h->d_tot4,
                       (unsigned long long *)d_tail, h->d_overflow, (uint32_t *)(d_tail + 32),
                       h->stream, (unsigned long long *)(d_tail + 48), &n_parts, h->d_cumrow, &h->cumrow_ok,
                       h->cum32));
    }
    const size_t isz = f32 ? 4 : 8;
    // a system-scope release after the kernel: its host writes are visible
    // once the stream has passed this point
    HIPCALL(h, hipEventRecord(h->fin_event, h->stream));
    std::vector<unsigned long long> tmp;
    if (!f32 && (want_cur_hist || want_cum_hist)) tmp.resize(nb);
    if (!f32 && want_cur_hist) {
        HIPCALL(h, hipMemcpyAsync(tmp.data(), h->d_snap, nb * 8, hipMemcpyDeviceToHost, h->stream));
        HIPCALL(h, hipStreamSynchronize(h->stream));
        convert_u64(tmp.data(), out->current_hist, (long long)nb, LDE_F64);
    }
    if (!f32 && want_cum_hist) {
        const unsigned long long *src = h->d_cum;
        if (h->cum32) {  // the split words joined (d_snap is free again: copied above)
            if (!h->d_snap)
                if (int rc = dev_alloc(h, &h->d_snap, nb)) return rc;
            HIPCALL(h, lde::launch_sum3(h->d_cum, nullptr, nullptr, h->d_snap, (long long)nb, h->stream, h->cum32));
            src = h->d_snap;
        }
        HIPCALL(h, hipMemcpyAsync(tmp.data(), src, nb * 8, hipMemcpyDeviceToHost, h->stream));
        HIPCALL(h, hipStreamSynchronize(h->stream));
        convert_u64(tmp.data(), out->cumulative_hist, (long long)nb, LDE_F64);
    }
    // the outputs are complete once fin_event has passed (lde_finalize_end);
    // the window restarts now, so the next accumulate may be enqueued first
    h->fin_pending = true;
    h->fin_images[0] = out->current_image && !map_cur ? out->current_image : nullptr;
    h->fin_images[1] = out->cumulative_image && !map_cum ? out->cumulative_image : nullptr;
    h->fin_isz = isz;
    h->fin_parts = n_parts;
    h->window_has_data = false;
    h->win64_dirty = false;
    h->win_events = 0;
    return LDE_OK;
}

int lde_finalize_end(lde_handle *h, lde_outputs *out) {
    if (!h) return fail(nullptr, LDE_EINVAL, "handle is NULL");
    if (!h->fin_pending) return fail(h, LDE_ESTATE, "no finalize is pending (lde_finalize_begin)");
    DeviceGuard guard(h->device);
    h->fin_pending = false;
    HIPCALL(h, wait_stream(h, h->fin_event));
    const auto t_waited = h->probe ? std::chrono::steady_clock::now() : std::chrono::steady_clock::time_point();
    struct PostProbe {
        lde_handle *h;
        std::chrono::steady_clock::time_point t0;
        ~PostProbe() {
            if (!h->probe) return;
            h->probe_fin_post_us += std::chrono::duration<double, std::micro>(
                                        std::chrono::steady_clock::now() - t0).count();
            ++h->probe_fin_n;
        }
    } post_probe{h, t_waited};
    const unsigned char *h_tail = h->h_pack + (size_t)h->S * 16;
    uint32_t ovf = 0;
    std::memcpy(&ovf, h_tail + 32, 4);
    if (ovf) return fail(h, LDE_ESTATE, "page pool overflow (internal error)");
    if (h->fin_images[0]) std::memcpy(h->fin_images[0], h->h_pack, (size_t)h->S * h->fin_isz);
    if (h->fin_images[1]) std::memcpy(h->fin_images[1], h->h_pack + (size_t)h->S * 8, (size_t)h->S * h->fin_isz);
    unsigned long long tot[4] = {0, 0, 0, 0};
    const unsigned long long *parts = reinterpret_cast<const unsigned long long *>(h_tail + 48);
    for (int b = 0; b < h->fin_parts; ++b)
        for (int q = 0; q < 4; ++q) tot[q] += parts[4 * b + q];
    if (out)
        for (int q = 0; q < 4; ++q) out->totals[q] = tot[q];
    return LDE_OK;
}

int lde_finalize(lde_handle *h, lde_outputs *out) {
    if (int rc = lde_finalize_begin(h, out)) return rc;
    return lde_finalize_end(h, out);
}

int lde_finalize_partials(lde_handle *h, void *d_out) {
    if (!h) return fail(nullptr, LDE_EINVAL, "handle is NULL");
    if (!d_out) return fail(h, LDE_EINVAL, "output buffer is NULL");
    DeviceGuard guard(h->device);
    if (int rc = flush_f32(h)) return rc;  // the pending push's f32 adds before the window restarts
    unsigned long long *o = (unsigned long long *)d_out;
    {
        // float32 views keep exact integer window (win64) and cumulative
        // counts beside their f32 accumulators: the partials come from those
        Timed tm(h, LDE_K_FINALIZE);
        HIPCALL(h, lde::launch_finalize(2, h->d_win32, h->win64_dirty ? h->d_win64 : nullptr,
                                        h->d_cum, nullptr, h->S, h->T, h->range_lo, h->range_hi,
                                        o, o + h->S, h->d_tot4, o + 2 * h->S, nullptr, nullptr,
                                        h->stream, nullptr, nullptr, h->d_cumrow, &h->cumrow_ok, h->cum32));
    }
    if (h->out_dtype == LDE_F32)  // the window's f32 accumulator restarts too
        HIPCALL(h, hipMemsetAsync(h->d_winf, 0, (size_t)h->nbins * 4, h->stream));
    h->window_has_data = false;
    h->win64_dirty = false;
    h->win_events = 0;
    return LDE_OK;
}

int lde_read_histogram(lde_handle *h, int32_t which, void *host_out) {
    if (!h) return fail(nullptr, LDE_EINVAL, "handle is NULL");
    if (!host_out) return fail(h, LDE_EINVAL, "host_out is NULL");
    if (which != LDE_CURRENT && which != LDE_CUMULATIVE)
        return fail(h, LDE_EINVAL, "which must be LDE_CURRENT or LDE_CUMULATIVE");
    if (which == LDE_CURRENT && !h->window_has_data)
        return fail(h, LDE_ENODATA, "No data has been added");
    if (which == LDE_CUMULATIVE && !h->cum_has_data)
        return fail(h, LDE_ENODATA, "No data has been added");
    DeviceGuard guard(h->device);
    const size_t nb = (size_t)h->nbins;
    if (h->out_dtype == LDE_F32) {
        if (int rc = flush_f32(h)) return rc;
        HIPCALL(h, hipMemcpyAsync(host_out, which == LDE_CURRENT ? h->d_winf : h->d_cumf, nb * 4,
                                  hipMemcpyDeviceToHost, h->stream));
        HIPCALL(h, hipStreamSynchronize(h->stream));
        return LDE_OK;
    }
    if (!h->d_snap)
        if (int rc = dev_alloc(h, &h->d_snap, nb)) return rc;
    const unsigned long long *w64 = h->win64_dirty ? h->d_win64 : nullptr;
    if (which == LDE_CURRENT)
        HIPCALL(h, lde::launch_sum3(w64, nullptr, h->d_win32, h->d_snap, h->nbins, h->stream));
    else
        HIPCALL(h, lde::launch_sum3(h->d_cum, w64, h->d_win32, h->d_snap, h->nbins, h->stream, h->cum32));
    std::vector<unsigned long long> tmp(nb);
    HIPCALL(h, hipMemcpyAsync(tmp.data(), h->d_snap, nb * 8, hipMemcpyDeviceToHost, h->stream));
    HIPCALL(h, hipStreamSynchronize(h->stream));
    convert_u64(tmp.data(), host_out, (long long)nb, LDE_F64);
    return LDE_OK;
}

int lde_set_groups(lde_handle *h, int32_t slot, int64_t n_groups, const int64_t *offsets,
                   const int32_t *screens) {
    if (!h) return fail(nullptr, LDE_EINVAL, "handle is NULL");
    if (slot < 0 || slot >= LDE_MAX_GROUP_SETS)
        return fail(h, LDE_EINVAL, "group slot %d out of range [0, %d)", slot, LDE_MAX_GROUP_SETS);
    if (n_groups < 0 || n_groups > (1LL << 24))
        return fail(h, LDE_EINVAL, "n_groups %lld out of range", (long long)n_groups);
    if (n_groups > 0 && !offsets) return fail(h, LDE_EINVAL, "offsets is NULL");
    const long long n_ref = n_groups > 0 ? (long long)offsets[n_groups] : 0;
    if (n_ref > 0 && !screens) return fail(h, LDE_EINVAL, "screens is NULL");
    if (n_groups > 0 && offsets[0] != 0) return fail(h, LDE_EINVAL, "offsets[0] must be 0");
    if (n_ref > (1LL << 30)) return fail(h, LDE_EINVAL, "too many group members");
    for (long long g = 0; g < n_groups; ++g)
        if (offsets[g + 1] < offsets[g]) return fail(h, LDE_EINVAL, "offsets must be non-decreasing");
    for (long long k = 0; k < n_ref; ++k)
        if (screens[k] < 0 || screens[k] >= h->S)
            return fail(h, LDE_EINVAL, "screen index %d out of range [0, %lld)", screens[k],
                        (long long)h->S);
    // work items of at most GROUP_ITEM screens; empty groups get no item (zeros)
    std::vector<int4> items;
    bool all_single = true;
    for (long long g = 0; g < n_groups; ++g) {
        const long long b = offsets[g], e = offsets[g + 1];
        if (e == b) {
            all_single = false;
            continue;
        }
        const bool single = e - b <= lde::GROUP_ITEM;
        if (!single) all_single = false;
        for (long long k = b; k < e; k += lde::GROUP_ITEM)
            items.push_back(make_int4((int)g, (int)k, (int)std::min(e, k + lde::GROUP_ITEM), single ? 1 : 0));
    }
    if (items.size() > 0x7fffffffULL) return fail(h, LDE_EINVAL, "too many group items");
    DeviceGuard guard(h->device);
    HIPCALL(h, hipStreamSynchronize(h->stream));
    auto &gs = h->groups[slot];
    dev_free(gs.d_items);
    dev_free(gs.d_screens);
    dev_free(gs.d_out);
    gs = lde_handle::GroupSet{};
    if (n_groups == 0) return LDE_OK;
    if (int rc = dev_alloc(h, &gs.d_items, items.size())) return rc;
    if (int rc = dev_alloc(h, &gs.d_screens, (size_t)n_ref)) return rc;
    if (int rc = dev_alloc(h, &gs.d_out, (size_t)n_groups * h->T)) return rc;
    if (!items.empty())
        HIPCALL(h, hipMemcpy(gs.d_items, items.data(), items.size() * sizeof(int4),
                             hipMemcpyHostToDevice));
    if (n_ref > 0)
        HIPCALL(h, hipMemcpy(gs.d_screens, screens, (size_t)n_ref * 4, hipMemcpyHostToDevice));
    gs.n_groups = n_groups;
    gs.n_items = (int)items.size();
    gs.all_single = all_single;
    return LDE_OK;
}

int lde_group_spectra(lde_handle *h, int32_t slot, int32_t which, void *host_out) {
    if (!h) return fail(nullptr, LDE_EINVAL, "handle is NULL");
    if (slot < 0 || slot >= LDE_MAX_GROUP_SETS)
        return fail(h, LDE_EINVAL, "group slot %d out of range [0, %d)", slot, LDE_MAX_GROUP_SETS);
    if (which != LDE_CURRENT && which != LDE_CUMULATIVE)
        return fail(h, LDE_EINVAL, "which must be LDE_CURRENT or LDE_CUMULATIVE");
    if (which == LDE_CURRENT && !h->window_has_data)
        return fail(h, LDE_ENODATA, "No data has been added");
    if (which == LDE_CUMULATIVE && !h->cum_has_data)
        return fail(h, LDE_ENODATA, "No data has been added");
    auto &gs = h->groups[slot];
    if (gs.n_groups == 0) return LDE_OK;
    if (!host_out) return fail(h, LDE_EINVAL, "host_out is NULL");
    DeviceGuard guard(h->device);
    const size_t n = (size_t)gs.n_groups * h->T;
    const bool f32 = h->out_dtype == LDE_F32;
    if (f32)
        if (int rc = flush_f32(h)) return rc;
    if (!gs.all_single) HIPCALL(h, hipMemsetAsync(gs.d_out, 0, n * 8, h->stream));
    {
        Timed tm(h, LDE_K_FINALIZE);
        HIPCALL(h, lde::launch_group_spectra(
                       f32 ? 2 : (which == LDE_CUMULATIVE ? 1 : 0), gs.d_items, gs.n_items,
                       gs.d_screens, h->T, h->d_win32, h->win64_dirty ? h->d_win64 : nullptr,
                       h->d_cum, f32 ? (which == LDE_CUMULATIVE ? h->d_cumf : h->d_winf) : nullptr,
                       gs.d_out, h->stream, h->cum32));
    }
    std::vector<unsigned long long> tmp(n);
    HIPCALL(h, hipMemcpyAsync(tmp.data(), gs.d_out, n * 8, hipMemcpyDeviceToHost, h->stream));
    HIPCALL(h, hipStreamSynchronize(h->stream));
    convert_u64(tmp.data(), host_out, (long long)n, h->out_dtype);
    return LDE_OK;
}

int lde_clear(lde_handle *h) {
    if (!h) return fail(nullptr, LDE_EINVAL, "handle is NULL");
    DeviceGuard guard(h->device);
    h->staged_host = 0;
    h->dev_segments.clear();
    return zero_state(h);
}

int lde_reset_cumulative(lde_handle *h) {
    if (!h) return fail(nullptr, LDE_EINVAL, "handle is NULL");
    DeviceGuard guard(h->device);
    return zero_state(h);
}

int lde_export_window(lde_handle *h, void *d_dst) {
    if (!h) return fail(nullptr, LDE_EINVAL, "handle is NULL");
    if (!d_dst) return fail(h, LDE_EINVAL, "destination is NULL");
    if (h->out_dtype == LDE_F32 || h->win64_dirty)
        return fail(h, LDE_ESTATE, "window is not in uint32 form (f32 view or folded window)");
    DeviceGuard guard(h->device);
    HIPCALL(h, hipMemcpyAsync(d_dst, h->d_win32, (size_t)h->nbins * 4, hipMemcpyDeviceToDevice,
                              h->stream));
    return LDE_OK;
}

int lde_import_window(lde_handle *h, const void *d_src) {
    if (!h) return fail(nullptr, LDE_EINVAL, "handle is NULL");
    if (!d_src) return fail(h, LDE_EINVAL, "source is NULL");
    if (h->out_dtype == LDE_F32 || h->win64_dirty)
        return fail(h, LDE_ESTATE, "window is not in uint32 form (f32 view or folded window)");
    DeviceGuard guard(h->device);
    HIPCALL(h, hipMemcpyAsync(h->d_win32, d_src, (size_t)h->nbins * 4, hipMemcpyDeviceToDevice,
                              h->stream));
    h->window_has_data = true;
    h->cum_has_data = true;
    return LDE_OK;
}

int lde_export_window_u64(lde_handle *h, void *d_dst) {
    if (!h) return fail(nullptr, LDE_EINVAL, "handle is NULL");
    if (!d_dst) return fail(h, LDE_EINVAL, "destination is NULL");
    if (h->out_dtype == LDE_F32)
        return fail(h, LDE_EINVAL, "u64 window export needs an integer-exact (float64) view");
    DeviceGuard guard(h->device);
    HIPCALL(h, lde::launch_sum3(h->win64_dirty ? h->d_win64 : nullptr, nullptr, h->d_win32,
                                (unsigned long long *)d_dst, h->nbins, h->stream));
    return LDE_OK;
}

int lde_import_window_u64(lde_handle *h, const void *d_src) {
    if (!h) return fail(nullptr, LDE_EINVAL, "handle is NULL");
    if (!d_src) return fail(h, LDE_EINVAL, "source is NULL");
    if (h->out_dtype == LDE_F32)
        return fail(h, LDE_EINVAL, "u64 window import needs an integer-exact (float64) view");
    DeviceGuard guard(h->device);
    if (int rc = ensure_win64(h)) return rc;
    const size_t nb = (size_t)h->nbins;
    HIPCALL(h, hipMemcpyAsync(h->d_win64, d_src, nb * 8, hipMemcpyDeviceToDevice, h->stream));
    HIPCALL(h, hipMemsetAsync(h->d_win32, 0, nb * 4, h->stream));
    // the merged counts live in the u64 part; the u32 part is empty again
    h->win64_dirty = true;
    h->win_events = 0;
    h->window_has_data = true;
    h->cum_has_data = true;
    return LDE_OK;
}

int lde_set_coord_lut(lde_handle *h, const lde_coord_lut *lut) {
    if (!h) return fail(nullptr, LDE_EINVAL, "handle is NULL");
    if (!lut) return fail(h, LDE_EINVAL, "lut is NULL");
    // a monitor handle has one flight path (n_pixels = 1) for all its events
    const long long n_pix = h->monitor ? 1 : h->L;
    // entering wavelength mode re-bins against integer edges, so it needs an
    // empty engine; once in it, a new table or new pixel distances (a detector
    // move) only change the per-event coordinate and keep the accumulated data
    const bool rebind = h->coord;
    if (!rebind && (h->window_has_data || h->cum_has_data || h->staged_host > 0 ||
                    !h->dev_segments.empty()))
        return fail(h, LDE_ESTATE, "set the coordinate table before the first accumulate (or after clear)");
    if (lut->n_pixels != n_pix)
        return fail(h, LDE_EINVAL, "n_pixels %lld != %lld (%s)", (long long)lut->n_pixels, n_pix,
                    h->monitor ? "one distance for a monitor" : "lut_len");
    if (lut->n_dist < 2 || lut->n_time < 2) return fail(h, LDE_EINVAL, "the grid needs n_dist, n_time >= 2");
    if (!lut->table || !lut->pixel_distance) return fail(h, LDE_EINVAL, "NULL table");
    if (!(lut->dist_step > 0) || !(lut->time_step > 0) || !std::isfinite(lut->dist0) ||
        !std::isfinite(lut->time0))
        return fail(h, LDE_EINVAL, "grid origin must be finite and steps > 0");
    if ((long long)lut->n_dist * lut->n_time > (1LL << 28)) return fail(h, LDE_EINVAL, "table too large");
    if (h->out_dtype == LDE_F32) return fail(h, LDE_EINVAL, "wavelength mode: float64 views only");
    DeviceGuard guard(h->device);
    const int T = h->T;
    HIPCALL(h, hipStreamSynchronize(h->stream));  // in-flight launches may read the old table
    // Everything new is built and uploaded into temporaries first; the handle
    // is changed only once every allocation and copy succeeded, so a failure
    // leaves it binning exactly as before (no half-switched tables, no freed
    // buffers still referenced by cargs).
    struct Staged {
        unsigned char *tab = nullptr;
        uint32_t *ttab = nullptr;
        uint32_t *wtree = nullptr;
        double *cpd = nullptr, *ctable = nullptr, *cedges = nullptr;
        uint16_t *cbuck = nullptr;
        ~Staged() {  // whatever was not committed
            dev_free(tab);
            dev_free(ttab);
            dev_free(wtree);
            dev_free(cpd);
            dev_free(ctable);
            dev_free(cedges);
            dev_free(cbuck);
        }
    } st;
    lde::ToaParams tp = h->tp;
    std::vector<uint32_t> tt;
    int tsh = 0;
    uint32_t tcap = 0;
    bool sieve_fits = h->split_ok;
    lde::WideToa wt = h->wtoa;
    bool wide_fits = h->wide_ok;
    if (!rebind) {
        // the binning stage now sees integer bins: edges 0..T
        std::vector<double> idx((size_t)T + 1);
        for (int i = 0; i <= T; ++i) idx[(size_t)i] = (double)i;
        std::vector<unsigned char> tab;
        if (int rc = build_toa_tables(h, idx.data(), T, tab, tp)) return rc;
        if (h->wide_ok) {  // WIDE's TOA tree over the integer edges
            std::vector<uint32_t> tree;
            wide_fits = build_wide_tree(idx, T, tree, wt);
            if (wide_fits) {
                if (int rc = dev_alloc(h, &st.wtree, tree.size())) return rc;
                HIPCALL(h, hipMemcpy(st.wtree, tree.data(), tree.size() * 4, hipMemcpyHostToDevice));
                wt.tree = st.wtree;
                // (integer edges: a flat tree, never larger than the create-time one)
                wt.lds = h->wtoa.lds && wt.words <= h->wtoa.words ? 1 : 0;
            }
        }
        if (int rc = dev_alloc(h, &st.tab, tab.size())) return rc;
        HIPCALL(h, hipMemcpy(st.tab, tab.data(), tab.size(), hipMemcpyHostToDevice));
        if (h->split_ok) {
            sieve_fits = build_sieve_toa(tp, tab, tt, tsh, tcap) && tt.size() <= h->ttab.size();
            if (sieve_fits) {
                if (int rc = dev_alloc(h, &st.ttab, h->ttab.size())) return rc;
                HIPCALL(h, hipMemcpy(st.ttab, tt.data(), tt.size() * 4, hipMemcpyHostToDevice));
            } else if (env_ll("LDE_VERBOSE", 0)) {
                fprintf(stderr, "lde coord: integer bin table does not fit the sieve (%zu > %zu words)\n",
                        tt.size(), h->ttab.size());
            }
        }
    }
    // bucket table over the edge range: a start candidate per bucket (the
    // kernel corrects it against the edges, so rounding never matters)
    const std::vector<double> &ed = h->edges;
    const double span = ed[(size_t)T] - ed[0];
    double min_w = span;
    for (int b = 0; b < T; ++b)
        if (ed[(size_t)b + 1] > ed[(size_t)b]) min_w = std::min(min_w, ed[(size_t)b + 1] - ed[(size_t)b]);
    int G = 1;
    if (span > 0 && std::isfinite(span) && min_w > 0)
        G = (int)std::max(1.0, std::min(4096.0, std::ceil(2.0 * span / min_w)));
    std::vector<uint16_t> buck((size_t)G, 0);
    const double w = span > 0 ? span / G : 1.0;
    for (int g = 0; g < G; ++g) {
        const double x = ed[0] + g * w;
        int b = (int)(std::upper_bound(ed.begin(), ed.end(), x) - ed.begin()) - 1;
        buck[(size_t)g] = (uint16_t)std::min(std::max(b, 0), std::min(T - 1, 65535));
    }
    // branch-free correction (coord_bin<true>): one step down, two up cover
    // every value whose bucket index rounds to g, even one bucket off either
    // way, when bin(e0 + (g - 1) w) >= buck[g] - 1 and bin(e0 + (g + 2) w) <=
    // buck[g] + 2 for every g (bins of the clamped, sorted edges)
    auto bin_of = [&](double x) {
        if (!(x >= ed[0])) return 0;
        if (!(x < ed[(size_t)T])) return T - 1;
        return std::max(0, (int)(std::upper_bound(ed.begin(), ed.end(), x) - ed.begin()) - 1);
    };
    // LDE_COORD_FIXED_BIN=0 (diagnostics): the general bin search, for tests
    bool fixed_bin = span > 0 && std::isfinite(span) && env_ll("LDE_COORD_FIXED_BIN", 1) != 0;
    for (int g = 0; g < G && fixed_bin; ++g) {
        const int lo_b = bin_of(ed[0] + (g - 1) * w), hi_b = bin_of(ed[0] + (g + 2) * w);
        if (lo_b < (int)buck[(size_t)g] - 1 || hi_b > (int)buck[(size_t)g] + 2) fixed_bin = false;
    }
    const size_t nt = (size_t)lut->n_dist * (size_t)lut->n_time;
    if (int rc = dev_alloc(h, &st.cpd, (size_t)n_pix)) return rc;
    if (int rc = dev_alloc(h, &st.ctable, nt)) return rc;
    if (int rc = dev_alloc(h, &st.cedges, (size_t)T + 1)) return rc;
    if (int rc = dev_alloc(h, &st.cbuck, (size_t)G)) return rc;
    HIPCALL(h, hipMemcpy(st.cpd, lut->pixel_distance, (size_t)n_pix * 8, hipMemcpyHostToDevice));
    HIPCALL(h, hipMemcpy(st.ctable, lut->table, nt * 8, hipMemcpyHostToDevice));
    HIPCALL(h, hipMemcpy(st.cedges, ed.data(), ((size_t)T + 1) * 8, hipMemcpyHostToDevice));
    HIPCALL(h, hipMemcpy(st.cbuck, buck.data(), (size_t)G * 2, hipMemcpyHostToDevice));
    // ---- commit (no failure past this point)
    if (!rebind) {
        std::swap(h->d_tab, st.tab);
        h->tp = tp;
        if (h->wide_ok && wide_fits) {
            std::swap(h->d_wtree, st.wtree);
            h->wtoa = wt;
        } else {
            h->wide_ok = false;
        }
        if (h->split_ok && sieve_fits) {
            std::swap(h->d_ttab, st.ttab);
            h->ttab = std::move(tt);
            h->ttab_shift = tsh;
            h->ttab_cap = tcap;
        } else {
            h->split_ok = false;
        }
    }
    std::swap(h->d_cpd, st.cpd);
    std::swap(h->d_ctable, st.ctable);
    std::swap(h->d_cedges, st.cedges);
    std::swap(h->d_cbuck, st.cbuck);
    lde::CoordArgs &c = h->cargs;
    c.pid_off = h->monitor ? 0 : h->pid_off;
    c.L = (unsigned)n_pix;
    c.pix_d = h->d_cpd;
    c.d0 = lut->dist0;
    c.inv_dd = 1.0 / lut->dist_step;
    c.nd = lut->n_dist;
    c.nt = lut->n_time;
    c.table = h->d_ctable;
    c.t0 = lut->time0;
    c.inv_dt = 1.0 / lut->time_step;
    c.edges = h->d_cedges;
    c.T = T;
    c.buckets = h->d_cbuck;
    c.G = G;
    c.e0 = ed[0];
    c.inv_w = 1.0 / w;
    c.fixed_bin = fixed_bin ? 1 : 0;
    c.edges_lds = 1;
    if (lde::coord_smem(c, false) > lde::kCoordSmemMax) c.edges_lds = 0;  // huge T: edges from HBM
    h->coord = true;
    h->key_ok.assign(h->key_ok.size(), 0);  // new distances, grid or edges
    if (!rebind)
        for (auto &u : h->hot_uses) u = -1;  // hot sets re-select on the new value
    return LDE_OK;
}

int lde_set_lut(lde_handle *h, const int32_t *out_lut) {
    if (!h) return fail(nullptr, LDE_EINVAL, "handle is NULL");
    if (h->monitor) return fail(h, LDE_EINVAL, "a monitor handle has no LUT");
    if (!out_lut) return fail(h, LDE_EINVAL, "out_lut is NULL");
    DeviceGuard guard(h->device);
    // transactional: validate and build everything first (new LUT image, new
    // PIXEL tables in fresh buffers); a failure up to here leaves the engine
    // binning with the old placement (workflows.py _move relies on it)
    std::vector<uint16_t> l16;
    std::vector<int> l32;
    if (int rc = convert_lut(h, out_lut, l16, l32)) return rc;
    PixStaged st;
    if (int rc = stage_pixel(h, out_lut, st)) return rc;
    // commit: the previous batch's kernels may still read the old tables
    HIPCALL(h, hipStreamSynchronize(h->stream));
    const size_t bytes = (size_t)h->R * h->L * (h->lut16 ? 2 : 4);
    const hipError_t e = hipMemcpy(h->d_lut, h->lut16 ? (const void *)l16.data() : (const void *)l32.data(),
                                   bytes, hipMemcpyHostToDevice);
    if (e != hipSuccess) {  // the device is failing: nothing consistent to keep
        h->pixel_ok = false;
        return fail(h, LDE_EHIP, "LUT upload failed: %s", hipGetErrorString(e));
    }
    // every replica's hot set / SIEVE tables derive from the LUT: rebuild lazily
    for (auto &u : h->hot_uses) u = -1;
    for (auto &u : h->wide_uses) u = -1;  // and the WIDE pixel tables
    commit_pixel(h, st);
    return LDE_OK;
}

int lde_get_stream(lde_handle *h, void **stream) {
    if (!h) return fail(nullptr, LDE_EINVAL, "handle is NULL");
    if (!stream) return fail(h, LDE_EINVAL, "stream is NULL");
    *stream = (void *)h->stream;
    return LDE_OK;
}

int lde_synchronize(lde_handle *h) {
    if (!h) return fail(nullptr, LDE_EINVAL, "handle is NULL");
    DeviceGuard guard(h->device);
    HIPCALL(h, hipStreamSynchronize(h->stream));
    return LDE_OK;
}

int lde_timing_select(lde_handle *h, uint32_t mask) {
    if (!h) return fail(nullptr, LDE_EINVAL, "handle is NULL");
    h->timing_mask = mask;
    return LDE_OK;
}

int lde_timing_enable(lde_handle *h, int32_t enable) {
    if (!h) return fail(nullptr, LDE_EINVAL, "handle is NULL");
    DeviceGuard guard(h->device);
    (void)hipStreamSynchronize(h->stream);
    resolve_timing(h);
    for (int k = 0; k < LDE_K_COUNT; ++k) {
        h->kms[k] = 0.0;
        h->kcount[k] = 0;
    }
    h->timing = enable != 0;
    return LDE_OK;
}

int lde_kernel_stats(lde_handle *h, int32_t kernel_id, double *ms, int64_t *launches) {
    if (!h) return fail(nullptr, LDE_EINVAL, "handle is NULL");
    if (kernel_id < 0 || kernel_id >= LDE_K_COUNT)
        return fail(h, LDE_EINVAL, "kernel id %d out of range", kernel_id);
    DeviceGuard guard(h->device);
    resolve_timing(h);
    if (ms) *ms = h->kms[kernel_id];
    if (launches) *launches = h->kcount[kernel_id];
    return LDE_OK;
}

int lde_counter(lde_handle *h, int32_t id, int64_t *value) {
    if (!h) return fail(nullptr, LDE_EINVAL, "handle is NULL");
    if (!value) return fail(h, LDE_EINVAL, "value is NULL");
    DeviceGuard guard(h->device);
    switch (id) {
    case LDE_C_PIX_OVERFLOW: {
        *value = 0;
        if (!h->d_povf || !h->pix_last_pred) return LDE_OK;
        uint32_t n = 0;
        HIPCALL(h, hipStreamSynchronize(h->stream));
        HIPCALL(h, hipMemcpy(&n, h->d_povf, 4, hipMemcpyDeviceToHost));
        *value = n;
        return LDE_OK;
    }
    case LDE_C_PIX_OVERFLOW_CAP:
        *value = (int64_t)h->povf_cap;
        return LDE_OK;
    case LDE_C_PIX_PREDICTED:
        *value = h->pix_last_pred ? 1 : 0;
        return LDE_OK;
    case LDE_C_WAITS:
        *value = h->waits_total;
        return LDE_OK;
    case LDE_C_WAITS_BLOCKED:
        *value = h->waits_blocked;
        return LDE_OK;
    case LDE_C_WAIT_PRED_US:
        *value = (int64_t)h->wait_pred_us;
        return LDE_OK;
    case 6:  // reserved (removed sieve pair counters)
    case 7:
        *value = 0;
        return LDE_OK;
    case LDE_C_WIDE_LEVELS:
        *value = h->wide_ok ? h->wide_levels : 0;
        return LDE_OK;
    case LDE_C_WIDE_PARTS:
        *value = h->wide_ok ? h->wide_parts : 0;
        return LDE_OK;
    case LDE_C_WIDE_TREE_WORDS:
        *value = h->wide_ok ? h->wtoa.words : 0;
        return LDE_OK;
    case LDE_C_WIDE_TREE_LDS:
        *value = h->wide_ok ? h->wtoa.lds : 0;
        return LDE_OK;
    case LDE_C_WIDE_ITEMS: {
        *value = 0;
        if (!h->d_wcounters) return LDE_OK;
        uint32_t c[5] = {0, 0, 0, 0, 0};  // items of several / single items per pass
        HIPCALL(h, hipStreamSynchronize(h->stream));
        HIPCALL(h, hipMemcpy(c, h->d_wcounters, sizeof c, hipMemcpyDeviceToHost));
        *value = h->wide_levels == 2 ? c[1] + c[4] : c[0] + c[3];
        return LDE_OK;
    }
    default:
        return fail(h, LDE_EINVAL, "unknown counter id %d", id);
    }
}

int lde_info(lde_handle *h, int64_t *n_screen, int32_t *n_toa_bins, int64_t *staged,
             int32_t *tile_bits, int32_t *n_tiles, int64_t *events_binned,
             int32_t *last_strategy) {
    if (!h) return fail(nullptr, LDE_EINVAL, "handle is NULL");
    long long st = h->staged_host;
    for (const Segment &s : h->dev_segments) st += s.n;
    if (n_screen) *n_screen = h->S;
    if (n_toa_bins) *n_toa_bins = h->T;
    if (staged) *staged = st;
    if (tile_bits) *tile_bits = h->tile_bits;
    if (n_tiles) *n_tiles = h->n_tiles;
    if (events_binned) *events_binned = h->events_binned;
    if (last_strategy) *last_strategy = h->last_strategy;
    return LDE_OK;
}

}  // extern "C"
