// lde_internal.h -- shared constants and launch prototypes (not part of the ABI)
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include <string>

struct lde_ev44_view;  // include/lde.h

// Diagnostic ablations (timing probes whose results are wrong by design:
// LDE_ABLATE, LDE_SIEVE_ABLATE, LDE_COLD_SORT_ABLATE) exist only in a
// -DLDE_DIAGNOSTICS build (python -m esslivedata_amd.build --diagnostics);
// in the product library LDE_DIAG(x) is the constant 0, so their branches and
// kernel variants are not compiled, and lde_create refuses those variables.
#ifdef LDE_DIAGNOSTICS
#define LDE_DIAG(x) (x)
#else
#define LDE_DIAG(x) 0
#endif

namespace lde {

constexpr int kPartThreads = 512;                  // pass A block
constexpr int kPartMinWavesPerEU = 4;              // 2 pass-A blocks per CU
constexpr int kPartEventsPerThread = 16;           // 4 x int4 per array
constexpr int kChunk = kPartThreads * kPartEventsPerThread;  // 8192 events
constexpr int kMaxTiles = 4096;                    // tiles of the (S,T) histogram
constexpr int kTileThreads = 512;                  // pass B block
constexpr int kMonitorColumnsMaxT = 512;           // conflict-free monitor layout
constexpr int kMaxBuckets = 4096;                  // TOA bucket table (general layout)
constexpr int kMaxFastBuckets = 16384;             // TOA bucket table (fast layout)
constexpr int kMaxSegs = 64;                       // segments per pass-A launch
constexpr int kLaneModeRun = 48;                   // pass B: lane-per-chunk below this avg run
constexpr int kPageBits = 10;                      // PAGED strategy: 1024-entry (2 KB) pages
constexpr int kPage = 1 << kPageBits;
constexpr size_t kPagedSmemMax = 80 * 1024;        // two pass-A blocks per CU (160 KB LDS)
constexpr int kSplitThreads = 1024;                // SPLIT event pass block (one per CU)
constexpr int kSplitEPT = kChunk / kSplitThreads;  // 8 events per thread per chunk
constexpr size_t kSplitSmemMax = 160 * 1024;       // hot rows + TOA image, one block per CU
constexpr int kHotMaxRows = 1022;
constexpr int kSampleBlocks = 64;                  // sampled chunks per hot-set selection

struct SegDesc {  // one staged ev44 message (device pointers)
    const int *pid;
    const int *toa;
    long long n;
    long long chunk0;  // first global chunk of this segment
};

// Batches of up to kKargSegs messages: the descriptors travel as kernel
// arguments (no pinned staging + H2D copy before the event pass): the sieve's
// chunk-table path, the monitor and the atomic strategy.
constexpr int kKargSegs = 24;
struct SegKarg {
    SegDesc s[kKargSegs];
};
// the ATOMIC strategy's launches take up to 64 (BIFROST: a pulse's 45 bank
// messages in one launch instead of two; 2 KB of kernel arguments)
constexpr int kKargSegsAtomic = 64;
struct SegKargAtomic {
    SegDesc s[kKargSegsAtomic];
};

struct ToaParams {
    long long lo;   // ceil(edge[0])  (clamped to [INT32_MIN, INT32_MAX + 1])
    long long hi;   // ceil(edge[T])
    unsigned span;  // hi - lo (fast layout only)
    int shift;      // bucket width = 2^shift
    int G;          // number of buckets
    int T;          // number of TOA bins
    int fast;       // 1: u32 relative thresholds + one-step u16 buckets
    int pad;
};

__host__ __device__ constexpr inline int align4(int x) { return (x + 3) & ~3; }
__host__ __device__ constexpr inline size_t align16(size_t x) { return (x + 15) & ~size_t(15); }
// bytes of the TOA lookup image copied verbatim into LDS
__host__ __device__ inline size_t toa_lds_bytes(const ToaParams &tp) {
    return tp.fast ? align16((size_t)(tp.T + 1) * 4) + align16((size_t)tp.G * 2)
                   : align16((size_t)(tp.T + 1) * 8) + align16((size_t)tp.G * 4);
}

struct PartitionArgs {
    int tile_bits;
    bool lut16;
    const SegDesc *segs;
    int n_segs;
    long long c_begin, n_chunks;
    const void *lut;
    int pid_off;
    unsigned L;
    const unsigned char *tab;
    ToaParams tp;
    int n_tiles;
    uint16_t *payload;
    uint32_t *starts;
    uint32_t *part;
    int grid;
};

inline unsigned grid_for(long long n) {
    long long g = (n + 255) / 256;
    if (g > 4096) g = 4096;
    if (g < 1) g = 1;
    return (unsigned)g;
}

size_t partition_smem(int n_tiles, const ToaParams &tp);

hipError_t launch_bin_atomic(const SegKargAtomic &seg, int n_segs, const void *lut, bool lut16, int pid_off,
                             unsigned L, const unsigned char *tab, const ToaParams &tp,
                             uint32_t *hist, int grid, hipStream_t st, hipEvent_t start = nullptr,
                             hipEvent_t stop = nullptr);
// one descriptor per block (chunk0 = block index in its message << 32 | the
// message's block count), any number of messages
hipError_t launch_bin_atomic_blocks(const SegDesc *blocks, int grid, const void *lut, bool lut16, int pid_off,
                                    unsigned L, const unsigned char *tab, const ToaParams &tp, uint32_t *hist,
                                    hipStream_t st, hipEvent_t start = nullptr, hipEvent_t stop = nullptr);
hipError_t launch_partition(const PartitionArgs &a, hipStream_t st);
struct PagedArgs {
    int tile_bits;
    bool lut16;
    int subc;  // LDS rank sub-counters per tile (1 or 4)
    const SegDesc *segs;  // device segment table (all staged segments)
    int n_segs;
    long long n_chunks;
    const void *lut;
    int pid_off;
    unsigned L;
    const unsigned char *tab;
    ToaParams tp;
    int n_tiles;
    uint16_t *pages;
    uint32_t *page_tile;
    uint32_t *page_cnt;
    uint32_t *pool_used;
    int cap;  // pages per block pool
    uint32_t *overflow;
    int grid;
    int tail_release = 0;  // pass-A blocks end with an agent-scope release
};

size_t paged_smem(int n_tiles, int subc, const ToaParams &tp);
hipError_t launch_paged_partition(const PagedArgs &a, hipStream_t st);

// hot-set selection of the SPLIT strategy (lde_hotset.hip)
struct SplitArgs {
    const SegDesc *segs;  // staged event segments
    int n_segs;
    long long n_chunks;
    const void *lut;  // d_lut (all replicas)
    bool lut16;
    long long L;
    int pid_off;
    int S;
    ToaParams tp;
    int rows;  // hot rows H
    int sample_blocks;
    uint32_t *sample_part, *screen_cnt, *stats;
    uint16_t *screen_row;
    uint32_t *row_screen;  // this replica's row -> screen
    int cache_bits;        // LDS pixel table bits (0: off)
    uint32_t *pix_cnt;     // [L] sampled events per pixel (zeroed before each selection)
};
// SIEVE: the lean SPLIT event pass (lde_sieve.hip).  Pixel word, in the LDS
// table and in the HBM LUT: valid | hot | tag (table only) | value, where
// value = row * T (hot) or screen * T (cold).
constexpr uint32_t kSieveValid = 0x80000000u;
constexpr uint32_t kSieveHot = 0x40000000u;
constexpr int kSieveTagShift = 22;
constexpr uint32_t kSieveValueMask = (1u << kSieveTagShift) - 1u;
constexpr uint32_t kSieveEmpty = 0xFFu << kSieveTagShift;  // tag 255, not valid
constexpr int kSieveMaxT = 254;
// finalize: per-block total partials summed on the host (at most this many blocks)
constexpr int kHostPartials = 1024;
constexpr int kColdGroups = 8;  // SIEVE cold keys: wave groups per block, one sort block each

// SIEVE: chunk tables of up to this many entries per block live in LDS,
// built by the sieve itself from kernel-argument descriptors
constexpr int kSieveLdsChunks = 128;

struct ChunkPtrs {  // one 8192-event chunk of the staged batch (or the dummy chunk)
    const int *pid;
    const int *toa;
};

struct SieveArgs {
    const SegDesc *segs;
    int n_segs;
    long long n_chunks;
    const ChunkPtrs *chunk_tab;  // [n_chunks + 1]; deferred chunks and entry n_chunks: dummy
    int lds_ctab;                // 1: build the block's chunk table in LDS (no chunk_tab)
    int karg;                    // lds_ctab: descriptors from sk (else from segs)
    SegKarg sk;                  // lds_ctab: the message descriptors (n_segs <= kKargSegs)
    const int *dummy;            // the all-invalid chunk
    const uint32_t *glut;  // this replica's pixel words, L + 1 entries (entry L = 0)
    uint32_t L;
    int pid_off;
    const uint32_t *ttab;  // TOA bucket words (+ sentinel), padded to toa_words4
    uint32_t toa_lo, toa_cap;
    int toa_shift, toa_words4;
    int T;
    const uint32_t *pix_tab;  // this replica's LDS table image (1 << cbits words)
    int cbits;
    int hot_words;  // align8(rows * T): the hot rows' LDS words
    uint32_t *hot_part;
    uint32_t *cold;
    long long cold_cap;  // 24-bit keys per block region (region stride cold_cap + 16)
    uint32_t *cold_cnt;
    int tile_bits, n_tiles;  // cold keys are counted per tile of 2^tile_bits bins
    uint32_t *cold_tcnt;     // [n_tiles][grid][kColdGroups]
    int ablate;  // diagnostics build: timing ablation (0 = the real pass)
    uint32_t *hot_fmt = nullptr;  // [grid] 1: the block's hot rows left as u16, 0: as u32
    unsigned long long *trace = nullptr;  // diagnostic [grid][4]: start, stream end, end, init done (realtime)
    int keyed = 0;  // the 'toa' stream holds finished pixel words (k_event_key): no probe/gather/TOA
};
size_t sieve_smem(int hot_words, int cbits, int toa_words4, int n_tiles);
// cold keys of SIEVE: per-tile scan, plan, exact counting sort into a
// tile-major u16 array, pass B
struct ColdArgs {
    int tile_bits, n_tiles;
    int rows;    // sieve blocks (one sort block per wave group)
    // hot rows of the sieve blocks, reduced into hist in the same launch as
    // the per-tile scan (hot_part == nullptr: none)
    const uint32_t *hot_part = nullptr;
    const uint32_t *row_screen = nullptr;
    int ht = 0, ht4 = 0, T = 1;  // hot words (rows * T) and their row stride
    const uint32_t *cold;
    long long stride, cap;  // region stride and capacity (keys)
    const uint32_t *cold_cnt, *tcnt;
    uint32_t *boff, *tile_total;
    uint32_t item_keys, max_items;
    uint4 *items;
    uint32_t *item_count;
    uint16_t *keys;  // tile-major, 16-byte aligned, >= total + 8 entries
    uint32_t *hist;
    long long n_bins;
    const uint32_t *hot_fmt = nullptr;  // per sieve block: hot rows as u16 (1) or u32 (0)
    int ablate = 0;     // cold-sort diagnostics (wrong results): 1 no writes, 2 no scatter,
                        // 16 prologue only
    int all_hot = 0;    // every screen has a hot row (no cold keys): hot-row reduce only
};
constexpr int kSortThreadsHost = 256;          // cold-sort block (thread t owns tile t)
constexpr size_t kColdSortSmem = 52 * 1024;    // cold-sort LDS: three blocks per CU
// start/stop: optional HIP events stamped by the kernel dispatch itself
// (hipExtLaunchKernelGGL), so timing adds no marker packets between kernels
hipError_t launch_cold_pipeline(const ColdArgs &c, hipStream_t st, hipEvent_t stop = nullptr);
hipError_t launch_sieve_tables(const void *lut, bool lut16, long long L, int T, int W,
                               const uint16_t *screen_row, const uint32_t *pix_cnt, int cbits,
                               uint32_t *glut, uint32_t *tab, uint32_t *stats, hipStream_t st);
// dummy: kChunk x (pid_off - 1), the all-invalid chunk
hipError_t launch_chunk_tab(const SegDesc *segs, int n_segs, long long n_chunks, const int *dummy,
                            ChunkPtrs *tab, hipStream_t st,
                            hipEvent_t start = nullptr);
hipError_t launch_chunk_tab_karg(const SegDesc *host_segs, int n_segs, long long n_chunks,
                                 const int *dummy, ChunkPtrs *tab, SegDesc *segs_out,
                                 hipStream_t st);
hipError_t launch_sieve(const SieveArgs &a, int grid, hipStream_t st, hipEvent_t start = nullptr,
                        hipEvent_t stop = nullptr);
hipError_t launch_hot_sample(const SplitArgs &a, int replica, hipStream_t st);
hipError_t launch_hot_pick(const SplitArgs &a, hipStream_t st);
hipError_t launch_page_plan(const PagedArgs &a, uint32_t item_events, uint32_t *cntp,
                            uint32_t *evp, uint32_t *tile_pages, uint32_t *tile_events,
                            uint32_t *tile_base, uint4 *items, uint32_t *item_count,
                            uint32_t max_items, uint32_t *list, hipStream_t st);
hipError_t launch_page_accumulate(int tile_bits, const PagedArgs &a, const uint32_t *list,
                                  const uint4 *items, const uint32_t *item_count, uint32_t *hist,
                                  long long n_bins, int grid, hipStream_t st);
hipError_t launch_plan(const uint32_t *part, int part_rows, int n_tiles, long long n_chunks,
                       uint32_t item_events, uint32_t *totals, uint32_t *tile_items, uint2 *items,
                       uint32_t *item_count, uint32_t max_items, hipStream_t st);
hipError_t launch_tile_accumulate(int tile_bits, const uint16_t *payload, const uint32_t *starts,
                                  int n_tiles, long long n_chunks, const uint2 *items,
                                  const uint32_t *item_count, const uint32_t *tile_items,
                                  uint32_t *hist, long long n_bins, int grid, hipStream_t st);
// start/stop (optional): HIP events stamped by the dispatch itself
// messages in block ranges: SegDesc::chunk0 = the message's first block
hipError_t launch_monitor(const SegKarg &segs, int n_segs, const unsigned char *tab,
                          const ToaParams &tp, uint32_t *hist, int grid, hipStream_t st,
                          hipEvent_t start = nullptr, hipEvent_t stop = nullptr);
hipError_t launch_fold_window(uint32_t *win32, unsigned long long *win64, long long n,
                              hipStream_t st);
hipError_t launch_merge_f32(uint32_t *batch, unsigned long long *win64, float *winf, float *cumf,
                            long long n, int first_win, int first_cum, hipStream_t st);
hipError_t launch_merge_f32_u64(const unsigned long long *src, unsigned long long *win64, float *winf,
                                float *cumf, long long n, int first_win, int first_cum,
                                hipStream_t st);
hipError_t launch_push_export(uint32_t *batch, unsigned long long *out, long long n, hipStream_t st);
// a32: a is a split cumulative of a32 bins (u32 low words, then high words)
hipError_t launch_sum3(const unsigned long long *a, const unsigned long long *b, const uint32_t *c,
                       unsigned long long *out, long long n, hipStream_t st, long long a32 = 0);
hipError_t launch_finalize(int img_kind, uint32_t *win32, unsigned long long *win64,
                           unsigned long long *cum, unsigned long long *snap, long long S, int T,
                           int lo, int hi, void *cur_img, void *cum_img,
                           unsigned long long *totals, unsigned long long *tot_copy,
                           const uint32_t *ovf_src, uint32_t *ovf_dst, hipStream_t st,
                           unsigned long long *host_parts = nullptr, int *n_parts = nullptr,
                           unsigned long long *cumrow = nullptr, int *cumrow_ok = nullptr, long long cum32 = 0);
// cumrow: 2 x S u64, each screen's cumulative sum in the TOA range and over
// all bins.  *cumrow_ok in: they are current (the wide-row finalize then skips
// the cumulative of groups the window left empty); out: current afterwards.
// float32 finalize in one pass with the window's pending push (batch, may be
// null): f32 adds, images, exact totals and cumulative, window reset
hipError_t launch_finalize_f32(uint32_t *batch, unsigned long long *win64, unsigned long long *cum,
                               float *winf, float *cumf, float *snap, long long S, int T, int lo, int hi,
                               int first_win, int first_cum, float *cur_img, float *cum_img,
                               unsigned long long *host_parts, const uint32_t *ovf_src, uint32_t *ovf_dst,
                               int *n_parts, hipStream_t st, hipEvent_t start = nullptr,
                               hipEvent_t stop = nullptr);
// items: {group, begin, end, group has a single item}; out zeroed unless every
// group is a single item
constexpr int GROUP_ITEM = 64;  // screens per work item of k_group_spectra
hipError_t launch_group_spectra(int mode, const int4 *items, int n_items, const int *screens,
                                int T, const uint32_t *win32, const unsigned long long *win64,
                                const unsigned long long *cum, const float *fsrc,
                                unsigned long long *out, hipStream_t st, long long cum32 = 0);

// wavelength mode (lde_coord.hip): per-event coordinate bin via a (distance,
// time) lookup table, written as the int32 "time" of a second binning pass
struct CoordArgs {
    int pid_off;
    unsigned L;             // pixels with a distance (1 for a monitor)
    const double *pix_d;    // [L] flight path per pixel id, NaN = no coordinate
    double d0, inv_dd;      // distance grid: d0 + i / inv_dd
    int nd, nt;
    const double *table;    // [nd * nt] row-major (distance, time)
    double t0, inv_dt;      // time grid: t0 + j / inv_dt (event unit, ns)
    const double *edges;    // [T + 1] coordinate edges
    int T;
    int edges_lds;          // 1: the edges are copied into LDS
    const uint16_t *buckets;  // [G] first candidate bin per bucket of the edge range
    int G;
    double e0, inv_w;       // bucket g = (v - e0) * inv_w
    int fixed_bin = 0;      // 1: every bucket's candidate is within [-1, +2] of the
                            // true bin (checked on the host): branch-free correction
};
constexpr size_t kCoordSmemMax = 160 * 1024;
size_t coord_smem(const CoordArgs &a, bool table_lds);
hipError_t launch_event_coord(const CoordArgs &a, const int *pid, const int *toa, long long n,
                              int *out, hipStream_t st);

// Wavelength mode on the SIEVE path: one pass over the batch that computes
// each event's coordinate bin AND looks up its pixel word, emitting the
// sieve's final word (valid | hot | row*T + bin or screen*T + bin; 0 =
// dropped) per event, chunk-aligned (entry c * kChunk + i of global chunk c,
// unused tail entries 0).  The keyed sieve (launch_sieve with keyed = 1) then
// reads 4 bytes per event and does no table probe, gather or TOA lookup.
struct KeyArgs {
    CoordArgs c;              // coordinate arithmetic (its cache fields unused)
    const SegDesc *segs;      // the batch's messages (device table)
    SegKarg sk;               // karg: the messages as kernel arguments (n_segs <= kKargSegs)
    int karg = 0;
    int n_segs;
    long long n_chunks;
    const uint32_t *glut;     // this replica's pixel words, L + 1 entries (entry L = 0)
    const uint32_t *pix_tab;  // this replica's LDS pixel-table image (1 << cbits words)
    const double *tab_d;      // grid coordinate x of each table slot's pixel (1 << cbits)
    const uint32_t *rec;      // per pixel 12 bytes {word, x lo, hi}, L + 1 entries (k_key_records)
    int cbits;
    int *keys;                // [n_chunks * kChunk]
    const int *dummy;         // kChunk x (pid_off - 1): the all-invalid chunk
    const uint8_t *tab_i = nullptr;  // pre: distance row of each slot's pixel (0xFF: outside)
    int pre = 0;              // 1: tab_d / rec hold fx and the row (k_key_dist / k_key_records
                              // with pre_nd = nd), the FAST event pass
    int ablate = 0;           // diagnostics build (LDE_KEY_ABLATE): 1 no gathers, 2 no
                              // coordinate arithmetic, 4 no stores (results invalid)
};
constexpr int kKeyLdsChunks = 128;  // k_event_key: chunk pointers per LDS window
size_t key_smem(const KeyArgs &a, bool table_lds);
hipError_t launch_event_key(const KeyArgs &a, int grid, hipStream_t st, hipEvent_t start = nullptr,
                            hipEvent_t stop = nullptr);
// distance of every pixel-table slot's pixel (NaN for empty slots)
// x = (d - d0) * inv_dd of every pixel-table slot's pixel (NaN for empty slots)
// (pre_nd > 0: fx and the distance row instead, see k_key_dist)
hipError_t launch_key_dist(const uint32_t *pix_tab, int cbits, const double *pix_d, unsigned L,
                           double d0, double inv_dd, int pre_nd, double *tab_d, uint8_t *tab_i,
                           hipStream_t st, hipEvent_t start = nullptr);
hipError_t launch_key_records(const uint32_t *glut, const double *pix_d, unsigned L, double d0,
                              double inv_dd, int pre_nd, uint32_t *rec, hipStream_t st);

// PIXEL strategy (lde_pixel.hip): events partitioned by pixel range, the
// LUT lookup done in pass B from the range's LDS slice
constexpr int kPixMaxRanges = 512;
struct PixChunk {                // one chunk of the batch (k_pix_chunks)
    const int *pid;
    const int *toa;
    int n;                       // valid events; kChunk: full and aligned, -kChunk: full, misaligned
    int pad;
};
struct PixArgs {
    const PixChunk *ctab;        // [n_chunks]
    const SegDesc *segs;
    int n_segs;
    long long n_chunks;
    int pid_off;
    unsigned L;
    int rb;                      // range of pixel q: q >> rb
    int nr;                      // ranges (<= kPixMaxRanges)
    int rs;                      // scatter staging word: range << rs | payload (rs bits)
    const unsigned char *tab;    // TOA lookup image
    ToaParams tp;
    uint32_t *counts;            // [grid][nr] events, then payload offsets
    uint32_t *rstart;            // [nr + 1] range starts, then [nr] range totals (scratch)
    uint32_t *payload;           // local pixel | bin << rb per event, range-major
                                 // (24-bit payloads packed 4 per 12 bytes)
    int grid;
    int unit = 1;                // chunks per partition step (runs padded per unit)
    int ept = 8;                 // events per thread and load: unit * kChunk / ept threads
    // predicted slots (no count pass): every (block, range) slot is sized
    // from the previous batch's run totals (prev) scaled by pred; a run past
    // its slot goes to the overflow groups, added at the end of pass B.  pred = 0:
    // exact slots from k_pix_count.  The scatter always records prev.
    float pred = 0.f;
    uint32_t *prev = nullptr;    // [grid][nr] padded run totals of the last scatter
    uint32_t *ovf = nullptr;     // [1] overflow groups written (reset by k_pix_chunks)
    uint4 *ovf_grp = nullptr;    // [ovf_cap] staging words (range << rs | payload) x 4
    uint32_t ovf_cap = 0;        // sized from the prediction margin; groups past it are
                                 // added by pass A itself (global atomics, exact):
    const uint16_t *ovf_loc = nullptr;     // the replica's footprint-local screens [L]
    const uint32_t *ovf_fp_off = nullptr;  // [nr + 1]
    const uint32_t *ovf_fp_scr = nullptr;
    uint32_t *ovf_hist = nullptr;          // the window
    int ablate = 0;              // LDE_PIX_ABLATE (diagnostics build): 1 no payload stores
};
struct PixSetup {                // setup-time tables (lde_create / lde_set_lut)
    int rb = 0, nr = 0, fmax = 0, rs = 24;
    const uint16_t *loc = nullptr;     // [R][L] footprint-local screen of every pixel (0xFFFF: dropped)
    const uint32_t *fp_off = nullptr;  // [nr + 1] footprint list offsets
    const uint32_t *fp_scr = nullptr;  // footprint screens, range after range
};
size_t pix_scatter_smem(const ToaParams &tp, int unit);
size_t pix_acc_smem(int rb, int fmax, int T);
// phase 0: count (exact slots) + scan + scatter; phase 1: accumulate (+ the
// overflow groups with predicted slots)
// phase 0 (pass A) takes optional start/stop events, stamped by its first and
// last dispatch
hipError_t launch_pixel(const PixArgs &a, const PixSetup &s, int replica, uint32_t item_events,
                        int max_items, uint4 *items, uint32_t *item_count, uint32_t *hist,
                        hipStream_t st, int phase, hipEvent_t start = nullptr, hipEvent_t stop = nullptr);

// WIDE strategy (lde_wide.hip): any TOA edges, any S * T up to 2^32 bins.
// Events are keyed (screen * T + bin) by a front end with an LDS table of
// the most frequent pixels (misses gather the LUT) and an LDS bucket tree
// over the TOA range, then partitioned into page chains by tile of 2^15 bins
// (one level, <= kWideMaxParts tiles) or by band of tiles first (two levels),
// and every tile is histogrammed in LDS.  Each partitioning pass writes, per
// row (its block or work item) and partition, the pages / events / offset of
// the partition's pages in the row's sorted page list; a plan pass turns those
// into work items (partition, row range) for the next pass.
constexpr int kWideThreads = 1024;        // partition passes: one block per CU
constexpr int kWideEPT = 16;              // entries per thread per unit
constexpr int kWideUnit = kWideThreads * kWideEPT;  // 16,384 entries (two chunks)
constexpr int kWidePageBits = 10;
constexpr int kWidePage = 1 << kWidePageBits;       // entries per page
constexpr int kWideTileBits = 15;         // pass-B tile: 2^15 u32 counters (128 KB LDS)
constexpr int kWideMaxParts = 1024;       // partitions of one pass (one owner thread each)
constexpr int kWideMaxBands = 512;        // first-level bands of the two-level form
constexpr int kWideMaxRows = 1024;        // rows per work item
constexpr int kWideTreeLds = 6144;        // TOA tree words kept in LDS (larger trees: global)
constexpr int kWideMaxCacheBits = 13;     // pixel table slots (2^13 words of LDS)
constexpr int kWideLdsChunks = 128;
constexpr int kWideSample = 64;           // chunks sampled per pixel-table selection

// TOA lookup tree over d = t - lo in [0, last]: root buckets of 2^sh0, each
// word either a leaf (bits 0..15 bin at the bucket start, bits 16..31 offset
// of the only threshold inside it, 0xFFFF none; leaf width <= 2^15) or an
// internal node (bits 0..15 = 0xFFFF, bits 16..31 first word of its 2^fb
// children of width / 2^fb).  Exact for any sorted edges: a bucket holding two
// or more thresholds (or equal thresholds) is split until it holds at most one.
struct WideToa {
    uint32_t lo;     // ceil(edge[0]) as u32 (d = (u32)t - lo)
    uint32_t last;   // span - 1; valid d <= last
    int empty;       // span == 0: no event is in range
    int sh0, fb;     // root bucket width 2^sh0, fan-out 2^fb
    int words;       // tree words
    int lds;         // 1: the tree fits kWideTreeLds words (copied into LDS)
    int depth;       // deepest leaf below the root
    const uint32_t *tree;  // device copy
};

struct WideRows {  // per-row output of a partitioning pass
    uint32_t *cnt;   // [row][ncols] pages of each partition
    uint32_t *ev;    // [row][ncols] entries
    uint32_t *off;   // [row][ncols] first index of the partition in the row's page list
    uint32_t *pool;  // [row] first page of the row's pool
    int ncols;
};

struct WideArgs {
    // batch
    const PixChunk *ctab;        // [n_chunks] (k_wide_chunks)
    const SegDesc *segs;
    int n_segs;
    long long n_chunks;
    int pid_off;
    unsigned L;
    const void *lut;             // this replica's LUT (u16 screen or i32 screen * T)
    int lut16;
    int T;
    const uint32_t *pix_tab;     // this replica's pixel table image (1 << cbits words)
    int cbits;
    WideToa toa;
    // first pass
    int levels;                  // 1: parts are tiles; 2: parts are bands of tpb tiles
    int pbits;                   // part = key >> pbits (15, or the band bits)
    int n_parts;
    int tpb_bits;                // two levels: tiles per band = 1 << tpb_bits
    int n_tiles;
    void *pages1;                // first-pass pages (u16 tile-local, or u32 band-local entries)
    void *pages2;                // second-pass pages (u16 tile-local)
    uint32_t *page_cnt, *page_part;  // per page (both passes share the numbering)
    uint32_t *list;              // sorted page lists, at each row's pool
    uint32_t cap1;               // pages per first-pass block pool
    WideRows rows1, rows2;
    uint32_t *pool2_next;        // second-pass page allocator
    uint32_t pool2_cap;
    uint32_t page0_2;            // first second-pass page (= grid1 * cap1; pages2 holds pages from here)
    uint4 *items1, *items2;      // plans: {part, row begin, row end, flags}
    uint32_t *counters;          // items of several [0] items1, [1] items2; single [3], [4]
                                 // (zeroed by k_wide_chunks; [2] is pool2_next)
    uint32_t *overflow;          // pool / plan overflow flag (internal error, reported by finalize)
    uint32_t max_items1, max_items2;
    uint2 *band_items;           // [band] the second pass's rows of the band
    uint32_t item_max1, item_max2;
    uint32_t *hist;              // the window
    long long n_bins;
    int grid1;                   // first-pass blocks
    int ablate = 0;              // LDE_WIDE_ABLATE (diagnostics build): first-pass timing ablations
    int wzero = 0;               // 1: the window is all zero before this batch (pass B stores, reads nothing)
    int acc_depth = 4;           // pass-B pages in flight per wave (diagnostics: 8)
    int tree_hybrid = 1;         // a tree past the LDS slot: its first words from LDS (diagnostics: 0)
};

// the batch's chunk table; call before launch_wide_table / launch_wide.
// host_segs (the batch's descriptors on the host): passed as kernel
// arguments when they fit kKargSegs, else a.segs (device) is read
hipError_t launch_wide_chunks(const WideArgs &a, const SegDesc *host_segs, hipStream_t st);
// pixel-table selection for one replica: sample the batch, pick the most
// frequent pixel of every slot (pix_cnt zeroed here)
hipError_t launch_wide_table(const WideArgs &a, const void *lut_rep, uint32_t *pix_cnt, uint32_t *tab,
                             hipStream_t st);
// first pass + plan (+ second pass + plan) + pass B; start/stop stamp the
// first pass, bstop the end of pass B (optional)
hipError_t launch_wide(const WideArgs &a, hipStream_t st, hipEvent_t start = nullptr,
                       hipEvent_t stop = nullptr, hipEvent_t bstart = nullptr, hipEvent_t bstop = nullptr);
size_t wide_scatter_smem(const WideArgs &a);

hipError_t launch_rebin_f64(const double *se, const double *sv, long long ns, const double *de,
                            long long nd, double *out_a, double *out_b, hipStream_t st);

// ev44 flatbuffer decode (lde_ev44.cpp): in-place parse with bounds checks,
// then the adapter rules (timestamp fallback, single pulse, lengths).
int ev44_parse(const uint8_t *buf, int64_t len, ::lde_ev44_view *v, std::string *err);
int ev44_events(const ::lde_ev44_view *v, int64_t kafka_timestamp_ms, int32_t flags,
                int64_t *timestamp_ns, std::string *err);

}  // namespace lde
