/*
 * lde.h -- C ABI of the MI355X live-data event-binning engine ("lde").
 *
 * The engine replaces the per-event work the reference runs inside scipp on
 * the detector-view and monitor-histogram path (reference = scipp/esslivedata,
 * SRC = src/ess/livedata):
 *
 *   ToNXevent_data.add/get          SRC/preprocessors/to_nxevent_data.py:127-208
 *   GroupByPixel.get (group_event_data)   SRC/preprocessors/group_by_pixel.py:43-54
 *   GeometricProjector.project_events     SRC/workflows/detector_view/projectors.py:80-152
 *   LogicalProjector.project_events       SRC/workflows/detector_view/projectors.py:243-270
 *   compute_detector_histogram (hist)     SRC/workflows/detector_view/providers.py:169-214
 *   _histogram_monitor (event mode)       SRC/workflows/monitor_workflow.py:65-112
 *   NoCopyAccumulator / window pair       SRC/preprocessors/accumulators.py:86-195
 *   detector_image/counts_total/counts_in_range  providers.py:236-357
 *
 * Plain C types only: host pointers, device pointers as void*, sizes as
 * int64_t.  No C++ exceptions cross this boundary.  Every entry point returns
 * LDE_OK (0) or a negative error code; lde_last_error() gives the message.
 * The Python host maps LDE_EINVAL to ValueError and everything else to
 * RuntimeError, matching the reference's error conventions.
 *
 * Threading: a handle is single-thread-affine (one job per worker thread in
 * the reference, SRC/core/job_manager.py:698-701); distinct handles are
 * independent and may be driven from different threads concurrently.  Each
 * handle owns its HIP stream unless the caller passes one.
 */
#ifndef LDE_H
#define LDE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LDE_ABI_VERSION 1

/* error codes */
#define LDE_OK 0
#define LDE_EINVAL (-1)   /* invalid argument  -> ValueError   */
#define LDE_ESTATE (-2)   /* invalid call order -> RuntimeError */
#define LDE_ENOMEM (-3)   /* allocation failed  -> RuntimeError */
#define LDE_EHIP (-4)     /* HIP runtime error  -> RuntimeError */
#define LDE_ENODATA (-5)  /* nothing accumulated -> ValueError ("No data has been added") */

/* output element types */
#define LDE_F64 0 /* float64 counts (reference default, unit 'counts') */
#define LDE_F32 1 /* float32 counts (BIFROST logical view, bifrost/specs.py:295) */

/* binning strategies (LDE_AUTO lets the engine choose per batch) */
#define LDE_STRATEGY_AUTO 0
#define LDE_STRATEGY_ATOMIC 1      /* one pass, global atomics             */
#define LDE_STRATEGY_PARTITION 2   /* tile partition (chunk-major runs) + LDS sub-histograms */
#define LDE_STRATEGY_PAGED 3       /* tile partition into per-block page chains + LDS sub-histograms */
#define LDE_STRATEGY_SPLIT 4       /* hot screen rows in LDS + cold keys sorted into tiles (skewed streams) */
#define LDE_STRATEGY_PIXEL 5       /* partition by pixel range (no LUT gather) + the range's LUT slice and
                                      screen footprint in LDS; needs footprints that fit (else WIDE) */
#define LDE_STRATEGY_WIDE 6        /* any TOA edges and histogram size: pixel-table front end, keys into page
                                      chains by tile (one level, or bands then tiles), LDS tiles (lde_wide.hip) */

/* histogram selectors for lde_read_histogram */
#define LDE_CURRENT 0    /* window since the last finalize  (accumulators.py:138-163) */
#define LDE_CUMULATIVE 1 /* since job start / last reset     (accumulators.py:86-135)  */

typedef struct lde_handle lde_handle;

/*
 * Engine configuration.  The pid -> output LUT folds the reference's
 * group_event_data membership test (unknown ids dropped), the pixel index and
 * the per-replica geometric/logical projection into one table:
 *
 *   out_lut[r * lut_len + (pid - pid_offset)] = flat screen index, or -1.
 *
 * A monitor is the special case n_screen = 1, n_replicas = 1 with a NULL
 * out_lut: every event maps to screen 0 and pixel ids are ignored.
 */
typedef struct lde_config {
    int32_t abi_version;      /* must be LDE_ABI_VERSION */
    int32_t device_id;        /* HIP device ordinal */
    void *stream;             /* hipStream_t to run on, or NULL = engine-owned */
    int32_t pid_offset;       /* smallest pixel id the LUT covers */
    int32_t n_replicas;       /* R >= 1 (noise replicas, projectors.py:105-113) */
    int64_t lut_len;          /* L: pixel ids pid_offset .. pid_offset+L-1 */
    const int32_t *out_lut;   /* host [R*L] screen index or -1; NULL for monitors */
    int64_t n_screen;         /* S >= 1 */
    int32_t n_toa_bins;       /* T >= 1 */
    const double *toa_edges;  /* host [T+1] float64 edges in the event unit (ns) */
    int32_t out_dtype;        /* LDE_F64 or LDE_F32 */
    int32_t strategy;         /* LDE_STRATEGY_* */
    int32_t range_lo;         /* TOA-range bin slice [range_lo, range_hi) used for */
    int32_t range_hi;         /*  detector_image / counts_in_range (-1,-1 = all)   */
} lde_config;

/* Finalize outputs.  Every pointer is an optional host buffer (NULL = skip).
 * Image element type = out_dtype; totals are exact integer counts. */
typedef struct lde_outputs {
    void *current_image;       /* [S]   sum over TOA range of the window     */
    void *cumulative_image;    /* [S]   sum over TOA range of the cumulative */
    void *current_hist;        /* [S*T] full window histogram                */
    void *cumulative_hist;     /* [S*T] full cumulative histogram            */
    uint64_t totals[4];        /* current total, current in-range,
                                  cumulative total, cumulative in-range      */
} lde_outputs;

/* Create / destroy.  On failure *out is NULL and lde_last_error(NULL) holds
 * the message (thread-local). */
int lde_create(const lde_config *cfg, lde_handle **out);
void lde_destroy(lde_handle *h);
const char *lde_last_error(const lde_handle *h);
int lde_abi_version(void);

/* Stage one ev44 message worth of events (replaces ToNXevent_data.add).
 * Host pointers; copied H2D asynchronously on the handle's stream before the
 * call returns (the caller may reuse its buffers).  pid may be NULL for a
 * monitor.  n == 0 is accepted (empty message). */
int lde_stage(lde_handle *h, const int32_t *pid, const int32_t *toa, int64_t n);

/* ev44 messages (ess-streaming-data-types ev44 flatbuffer, file identifier
 * "ev44").  lde_ev44_decode decodes one payload in place, replacing
 * eventdata_ev44.deserialise_ev44 / Event44Message.GetRootAs as called by
 *   KafkaToEv44Adapter.adapt           SRC/kafka/message_adapter.py:192-204
 *   KafkaToMonitorEventsAdapter.adapt  SRC/kafka/message_adapter.py:380-409
 * Every offset and extent is checked against len: garbage, empty, truncated
 * or wrong-schema payloads return LDE_EINVAL (message in
 * lde_last_error(NULL), thread-local) where the reference raises and drops
 * the message.  Vector pointers point into buf (zero copy, possibly
 * unaligned); `present` flags which fields the payload carries. */
#define LDE_EV44_HAS_SOURCE_NAME (1u << 0)
#define LDE_EV44_HAS_MESSAGE_ID (1u << 1)
#define LDE_EV44_HAS_REFERENCE_TIME (1u << 2)
#define LDE_EV44_HAS_REFERENCE_TIME_INDEX (1u << 3)
#define LDE_EV44_HAS_TIME_OF_FLIGHT (1u << 4)
#define LDE_EV44_HAS_PIXEL_ID (1u << 5)
typedef struct lde_ev44_view {
    const char *source_name;           /* UTF-8, not NUL-terminated */
    int64_t source_name_len;
    int64_t message_id;
    const void *reference_time;        /* int64 [n_reference_time], ns since epoch */
    int64_t n_reference_time;
    const void *reference_time_index;  /* int32 [n_reference_time_index] */
    int64_t n_reference_time_index;
    const void *time_of_flight;        /* int32 [n_time_of_flight], ns */
    int64_t n_time_of_flight;
    const void *pixel_id;              /* int32 [n_pixel_id] */
    int64_t n_pixel_id;
    uint32_t present;                  /* LDE_EV44_HAS_* bits */
} lde_ev44_view;
int lde_ev44_decode(const uint8_t *buf, int64_t len, lde_ev44_view *out);

/* Decode one ev44 payload and stage its events (lde_stage semantics) in one
 * call: the adapter chain KafkaToEv44Adapter -> Ev44ToDetectorEventsAdapter ->
 * DetectorEvents.from_ev44 (message_adapter.py:192-204, 412-437;
 * to_nxevent_data.py:16-19, 57-69) for detector handles, and
 * KafkaToMonitorEventsAdapter (time_of_flight only, pixel_id ignored) for
 * monitor handles.  flags: LDE_EV44_SINGLE_PULSE applies
 * _require_single_pulse (-> LDE_ENOTSUP, NotImplementedError in Python);
 * LDE_EV44_MONITOR (the monitor rules) is implied by a monitor handle and
 * invalid on a detector handle.  *timestamp_ns (optional) receives
 * reference_time[-1], or kafka_timestamp_ms * 1e6 when that vector is empty.
 * A rejected payload stages nothing. */
#define LDE_ENOTSUP (-6) /* unsupported message -> NotImplementedError */
#define LDE_EV44_SINGLE_PULSE 1
#define LDE_EV44_MONITOR 2
int lde_stage_ev44(lde_handle *h, const uint8_t *buf, int64_t len, int64_t kafka_timestamp_ms,
                   int32_t flags, int64_t *timestamp_ns);

/* Stage events already resident in HBM.  No copy.  The engine orders nothing
 * against other streams: the caller makes the handle's stream (lde_get_stream)
 * wait for the work that produces the buffers, and keeps them allocated until
 * the kernels the next lde_accumulate enqueues on that stream have completed
 * (e.g. an event recorded on it after lde_accumulate).  The Python host does
 * both (event wait + allocator stream recording) when the producer's stream
 * is not the handle's. */
int lde_stage_device(lde_handle *h, const void *d_pid, const void *d_toa, int64_t n);

/* The hipStream_t the handle runs on (cfg->stream, or the one it created). */
int lde_get_stream(lde_handle *h, void **stream);

/* Stage a whole batch of device-resident messages in one call (the batch
 * ToNXevent_data.get hands over, to_nxevent_data.py:155-200): message i is
 * d_pids[i] / d_toas[i] with ns[i] events, same rules as lde_stage_device.
 * Nothing is staged unless every message is valid. */
int lde_stage_device_batch(lde_handle *h, int64_t count, const void *const *d_pids,
                           const void *const *d_toas, const int64_t *ns);

/* Bin everything staged since the last call into the current window using
 * noise replica `replica` (0 <= replica < R).  Replaces
 * GroupByPixel.get + project_events + hist + accumulator push. */
int lde_accumulate(lde_handle *h, int32_t replica);

/* Finalize: cumulative += window, fill the requested outputs, clear the
 * window (window accumulator on_finalize).  Returns LDE_ENODATA when nothing
 * was accumulated since the last finalize (the reference's empty window
 * accumulator raises ValueError). */
int lde_finalize(lde_handle *h, lde_outputs *out);

/* lde_finalize in two halves, so that a service can enqueue its next
 * lde_accumulate before it waits for this window's outputs: the device bins
 * the next batch while the host serializes and publishes the outputs of this
 * one (the reference runs Job.get, job.py:435-467, and the next batch's
 * Job.add one after the other on the host; the outputs are the same).  _begin enqueues the
 * finalize and restarts the window (histogram outputs, when requested, are
 * complete on return); _end waits for the finalize alone -- not for work
 * enqueued after it -- and fills out->totals and the images (same `out`).
 * One finalize may be pending per handle: _begin returns LDE_ESTATE until
 * _end has run.  lde_finalize == _begin + _end. */
int lde_finalize_begin(lde_handle *h, lde_outputs *out);
int lde_finalize_end(lde_handle *h, lde_outputs *out);

/* Page-locked, device-mapped host memory for finalize outputs.  An image
 * pointer of lde_outputs that lies inside such a block is written by the
 * finalize kernel directly (no staging buffer, no host copy after the wait):
 * the caller's numpy arrays can be views of these blocks.  Blocks are not tied
 * to a handle; free them with lde_host_free once nothing reads them.  (Host
 * side of the reference's finalize -> da00 hand-off, job.py:435-467: the
 * outputs are read once, serialized, and dropped.) */
int lde_host_alloc(int64_t bytes, void **out);
int lde_host_free(void *p);

/* Read a full histogram (LDE_CURRENT or LDE_CUMULATIVE) without finalizing. */
int lde_read_histogram(lde_handle *h, int32_t which, void *host_out);

/* Replace the pid -> screen LUT (same R, lut_len and n_screen as at create),
 * e.g. rebuilt from moved pixel positions after a detector-transform change
 * (geometry_signal.py:27-51; the projector is rebuilt with the geometry).
 * out_lut as in lde_config.  Counts already binned are kept; the workflow
 * resets them (lde_reset_cumulative) as the reference's accumulators do. */
int lde_set_lut(lde_handle *h, const int32_t *out_lut);

/* Wavelength mode (detector_view/factory.py:134-169 'wavelength',
 * providers.py:77-95): the histogrammed event coordinate is looked up per event
 * from its pixel's flight path and its time of arrival, then binned against
 * the view's float64 edges (cfg->toa_edges, in the coordinate's unit) with
 * the same half-open rule as TOA.  Bilinear interpolation on the regular grid
 *   distance dist0 + i * dist_step (i < n_dist), time time0 + j * time_step ns
 * of table[i * n_time + j]; NaN values, NaN distances and points outside the
 * grid are dropped.  Arithmetic (restated in oracle/ and lde_coord.hip):
 *   x = (d - dist0) * (1 / dist_step), i = min(floor x, n_dist - 2), fx = x - i
 *   y = (t - time0) * (1 / time_step), j = min(floor y, n_time - 2), fy = y - j
 *   c = a + fx * (b - a), a = v[i][j] + fy * (v[i][j+1] - v[i][j]),
 *                         b = v[i+1][j] + fy * (v[i+1][j+1] - v[i+1][j])
 * in float64 without fused multiply-adds.  Monitor handles take one distance
 * (n_pixels = 1) for all their events (monitor_workflow.py:126-132).  The first
 * call comes before the first lde_accumulate (or after lde_clear), later calls
 * (new pixel distances after a detector move, a new table) may come at any time
 * and keep the counts already binned.  n_dist, n_time >= 2. */
typedef struct lde_coord_lut {
    const double *pixel_distance; /* [n_pixels] per pixel id (pid_offset + k) */
    int64_t n_pixels;             /* lut_len (detector) or 1 (monitor) */
    const double *table;          /* [n_dist * n_time] */
    int32_t n_dist, n_time;
    double dist0, dist_step;
    double time0, time_step;      /* event unit (ns) */
} lde_coord_lut;
int lde_set_coord_lut(lde_handle *h, const lde_coord_lut *lut);

/* Reset semantics: clear both (workflow.clear / Job.reset) or drop the
 * cumulative and window because the geometry coord changed
 * (NoCopyAccumulator._reset_if_geometry_changed, accumulators.py:116-131). */
int lde_clear(lde_handle *h);
int lde_reset_cumulative(lde_handle *h);

/* Multi-GPU merge support (no reference counterpart): export the window
 * counts (uint32 [S*T]) into a caller device buffer, and import merged
 * counts back (e.g. after an RCCL reduce over xGMI). */
int lde_export_window(lde_handle *h, void *d_dst);
/* Multi-GPU finalize without moving the histogram: cumulative += window,
 * window cleared (as lde_finalize), and this rank's exact partial outputs
 * written to caller device memory, uint64 [S] current image | [S] cumulative
 * image | [4] totals (lde_outputs.totals order), asynchronously on the
 * handle's stream.  Summed over ranks (RCCL reduce) they equal the outputs of
 * one handle that binned every rank's events.  An empty window is allowed
 * (zeros for the current outputs).  float32 views (BIFROST) export their exact
 * integer counts too (kept beside the f32 accumulators); their merge is NOT
 * the reference's float32 result beyond 2^24 counts per bin (the reference
 * rounds once per push), so sharded float32 views merge per push instead
 * (lde_accumulate_push / lde_push_u64 below). */
int lde_finalize_partials(lde_handle *h, void *d_out);
int lde_import_window(lde_handle *h, const void *d_src);
/* Exact window merge in any window state (also after the uint32 window has
 * folded into its uint64 part): export writes uint64 [S*T] window counts to
 * caller device memory; import replaces the window with uint64 [S*T] counts
 * (e.g. the RCCL sum of every rank's export).  Integer (float64) views only:
 * LDE_EINVAL for f32 views. */
int lde_export_window_u64(lde_handle *h, void *d_dst);
int lde_import_window_u64(lde_handle *h, const void *d_src);

/* Exact sharded float32 views (BIFROST), one collective per push.  The
 * reference adds every push to its float32 window and cumulative
 * (accumulators.py:129-135; the cast is bifrost/specs.py:295), so a sharded
 * view must merge the ranks' counts of a push BEFORE that push's f32 add:
 *   lde_accumulate_push: bins the staged events like lde_accumulate but
 *     writes the push's exact counts, uint64 [S*T], to caller device memory
 *     instead of adding them (this handle's accumulators are untouched);
 *   lde_push_u64: adds one push of exact counts (e.g. the RCCL sum of every
 *     rank's lde_accumulate_push) in the reference order: window and
 *     cumulative f32 += float32(count), the exact integer window += count.
 * Float32 views only (LDE_EINVAL otherwise: integer views merge exactly at
 * finalize, lde_finalize_partials / lde_export_window_u64). */
int lde_accumulate_push(lde_handle *h, int32_t replica, void *d_counts);
int lde_push_u64(lde_handle *h, const void *d_counts);

/* Screen groupings: per-group TOA spectra summed on the device, replacing the
 * host-side reductions of the finalize outputs
 *   roi_spectra (rectangle slices / polygon masks)  SRC/workflows/detector_view/roi.py:188-266
 *   spectrum_view (per-instrument regrouping)       SRC/workflows/detector_view/providers.py:300-325
 *                                                   (BIFROST: config/instruments/bifrost/specs.py:311-329)
 * Group g holds the flat screen indices screens[offsets[g] .. offsets[g+1]);
 * groups may overlap and may be empty.  n_groups == 0 clears the slot.
 * lde_group_spectra writes out[g * T + t] (out_dtype) for LDE_CURRENT (the
 * window since the last finalize) or LDE_CUMULATIVE (the cumulative as the
 * next finalize publishes it, i.e. including the window).  Call it before
 * lde_finalize to get the current-window spectra of that finalize.  Sums are
 * exact integers on the device; an empty slot writes nothing. */
#define LDE_MAX_GROUP_SETS 4
int lde_set_groups(lde_handle *h, int32_t slot, int64_t n_groups, const int64_t *offsets,
                   const int32_t *screens);
int lde_group_spectra(lde_handle *h, int32_t slot, int32_t which, void *host_out);

/* Histogram-mode monitors (monitor_workflow.py:101-108): rebin a float64
 * histogram (n_src bins, n_src + 1 ascending edges, already in the target
 * unit) onto n_dst bins and ADD the result into d_out_a and d_out_b (either
 * may be NULL), i.e. the window and cumulative pushes of one message.  All
 * arrays are device memory; runs on `stream` (hipStream_t, NULL = default).
 * Errors: LDE_EINVAL, message in lde_last_error(NULL). */
int lde_rebin_f64(const double *d_src_edges, const double *d_src_values, int64_t n_src,
                  const double *d_dst_edges, int64_t n_dst, double *d_out_a, double *d_out_b,
                  void *stream);

/* Wait for all work queued on the handle's stream. */
int lde_synchronize(lde_handle *h);

/* Kernel timing, measured with HIP events recorded on the handle's stream
 * around each launch of the engine's kernels (ids LDE_K_*).  Recording is off
 * until lde_timing_enable(h, 1); enabling again resets the statistics.
 * lde_kernel_stats synchronizes the stream and returns the summed kernel
 * milliseconds and the launch count for one kernel id. */
#define LDE_K_ATOMIC 0    /* k_bin_atomic: one-pass global-atomic binning   */
#define LDE_K_PARTITION 1 /* k_partition: pass A, tile partition            */
#define LDE_K_PLAN 2      /* k_tile_totals + k_plan                          */
#define LDE_K_TILE 3      /* k_tile_accumulate: pass B, LDS sub-histograms   */
#define LDE_K_MONITOR 4   /* k_monitor: 1-D TOA histogram                    */
#define LDE_K_FINALIZE 5  /* k_finalize / merge kernels                      */
#define LDE_K_BINNING 6   /* whole binning sequence of one accumulate        */
#define LDE_K_PAGED 7     /* PAGED pass A (k_paged_partition); SPLIT: the cold-key path (k_hot_reduce_scan + k_cold_sort + k_cold_accumulate) */
#define LDE_K_PAGE_PLAN 8 /* k_page_count/scan/plan/scatter                   */
#define LDE_K_PAGE_ACC 9  /* pass B: k_page_accumulate (PAGED), k_pix_accumulate (PIXEL) */
#define LDE_K_SPLIT 10    /* k_sieve: SPLIT event pass (hot rows in LDS, cold keys out) */
#define LDE_K_SPLIT_AUX 11 /* hot-set selection, hot-row reduce, cold segment table */
#define LDE_K_COORD 12    /* k_event_coord / k_event_key: wavelength-mode coordinate pass */
#define LDE_K_PIXEL 13    /* k_pix_scatter: PIXEL pass A (stamped by its own dispatch) */
#define LDE_K_WIDE 14     /* k_wide_scatter: WIDE first pass (stamped by its own dispatch) */
#define LDE_K_WIDE_ACC 15 /* k_wide_accumulate: WIDE pass B (stamped by its own dispatch) */
#define LDE_K_COUNT 16
int lde_timing_enable(lde_handle *h, int32_t enable);
/* Record only the kernels whose bit (1 << LDE_K_*) is set in mask (default:
 * all).  Fewer recorded events = less host work per batch. */
int lde_timing_select(lde_handle *h, uint32_t mask);
int lde_kernel_stats(lde_handle *h, int32_t kernel_id, double *ms, int64_t *launches);

/* Counters for tests and reports (lde_counter):
 *   LDE_C_PIX_OVERFLOW      groups of four events the last PIXEL batch could not
 *                           place in their predicted slots (synchronizes the stream)
 *   LDE_C_PIX_OVERFLOW_CAP  the overflow list's capacity in groups (groups past it
 *                           are added by pass A itself, exactly)
 *   LDE_C_PIX_PREDICTED     1 if the last PIXEL batch used predicted slots
 *   LDE_C_WAITS             finalize waits that found the GPU still busy
 *   LDE_C_WAITS_BLOCKED     ... of which ended in a blocking (interrupt) wait
 *   LDE_C_WAIT_PRED_US      the predicted finalize wait (us), slept through */
#define LDE_C_PIX_OVERFLOW 0
#define LDE_C_PIX_OVERFLOW_CAP 1
#define LDE_C_PIX_PREDICTED 2
#define LDE_C_WAITS 3
#define LDE_C_WAITS_BLOCKED 4
#define LDE_C_WAIT_PRED_US 5
/* 6, 7: reserved (sieve pair counters of round 4, removed; read as 0) */
#define LDE_C_WIDE_LEVELS 8      /* WIDE partition levels (1 or 2; 0: WIDE unavailable for this view) */
#define LDE_C_WIDE_PARTS 9       /* WIDE first-level partitions (tiles or bands) */
#define LDE_C_WIDE_TREE_WORDS 10 /* words of the WIDE TOA lookup tree */
#define LDE_C_WIDE_TREE_LDS 11   /* 1 if the whole tree is kept in LDS (else its first 6,144 words, the rest read through L2) */
#define LDE_C_WIDE_ITEMS 12      /* pass-B work items of the last WIDE batch (synchronizes) */
int lde_counter(lde_handle *h, int32_t id, int64_t *value);

/* Introspection for tests and reports. */
int lde_info(lde_handle *h, int64_t *n_screen, int32_t *n_toa_bins, int64_t *staged,
             int32_t *tile_bits, int32_t *n_tiles, int64_t *events_binned,
             int32_t *last_strategy);

#ifdef __cplusplus
}
#endif

#endif /* LDE_H */
