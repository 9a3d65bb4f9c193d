// lde_wide.hip -- WIDE strategy: large and arbitrary TOA binnings.
//
// The reference's EdgesModel allows 1..10,000 TOA bins, linear or log, from
// any start (SRC/parameter_models.py:82-105, 290-295; the detector view's
// edges, SRC/workflows/detector_view_specs.py:73-124), so a DREAM-sized view
// (25,600 screens) reaches 2.56e8 (screen, bin) counters.  SIEVE and PIXEL
// keep rows or footprints of the histogram in LDS and stop scaling at a few
// hundred bins; WIDE instead keys every event and sorts the keys into tiles
// of 2^15 bins through page chains, so its cost per event does not depend on
// T or on the edges:
//
//   k_wide_chunks     the batch's chunk table; zeroes the pass counters
//   k_wide_scatter    first pass, one 1024-thread block per CU.  Per unit of
//                     16,384 events: pixel word from an LDS table of the
//                     sampled most frequent pixels (misses gather the LUT
//                     with a raw buffer load; hits load out of range, which
//                     issues no request), TOA bin from an LDS bucket tree
//                     (WideToa), key = screen * T + bin; rank by partition
//                     (LDS atomics), block scan, page allocation from the
//                     block's pool (owner thread per partition), key-sorted
//                     LDS staging (runs padded to 4), and each run appended
//                     to its partition's open page in groups of four entries
//                     (8- or 16-byte buffer stores).  At its end the block
//                     sorts its pages by partition into its page list and
//                     writes, per partition, pages / entries / list offset
//                     (WideRows).
//   k_wide_plan       a wave per partition: work items (partition, range of
//                     rows) of at most ~item_max entries, one reservation per
//                     block; items of multi-item (hot) partitions first
//   k_wide_split      two-level form only (more than kWideMaxParts tiles):
//                     per item of a band, its u32 band-local keys partitioned
//                     by tile as the first pass does, with a rank counter per
//                     8-lane group (few partitions per band)
//   k_wide_accumulate per item of a tile: its pages histogrammed in a 128 KB
//                     LDS tile, then added to the window (store-only on a
//                     fresh window, a 16-byte read-modify-write when the tile
//                     has one item, global atomics when hot tiles are split)
//
// Counts are integers and every event is added exactly once whatever the
// table holds or how the work is split, so the histogram is bit-identical to
// the other strategies and to the oracle.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "lde_device.h"
#include "lde_internal.h"

namespace lde {

namespace {

constexpr int NT = kWideThreads;
constexpr int EPT = kWideEPT;
constexpr int UNIT = kWideUnit;
constexpr int PAGE = kWidePage;
constexpr int PB = kWidePageBits;
constexpr int CT = kChunk / EPT;  // threads per chunk of a unit (512)
constexpr uint32_t kNone = 0xFFFFFFFFu;
constexpr uint32_t kOOB = 0x80000000u;         // buffer offset past every num_records
constexpr uint32_t kRsrcWord3 = 0x00020000u;   // gfx9 raw buffer, 32-bit data format
constexpr uint32_t kTabValid = 0x80000000u;    // pixel table word: valid | tag << 22 | screen
constexpr int kTagShift = 22;
constexpr uint32_t kTabValue = (1u << kTagShift) - 1u;  // (the value kTabValue: a dropped pixel)
constexpr uint32_t kTagMask = 0x1FFu;
constexpr uint32_t kLeafNone = 0xFFFFu;        // leaf: no threshold inside / internal-node marker

typedef unsigned int v4u __attribute__((ext_vector_type(4)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void *p, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), (short)0, (int)bytes, (int)kRsrcWord3);
}

// TM: where the TOA tree is read -- 1: all of it from LDS; 2: its first
// kWideTreeLds words (the builder puts the root level first, then each root
// bucket's subtree in TOA order) from LDS and the rest through a buffer load
// that has no request for an LDS-resident index; 0: all through L2
// (diagnostics)
template <int TM>
__device__ __forceinline__ uint32_t tree_word(const uint32_t *tree, __amdgpu_buffer_rsrc_t gt, uint32_t i) {
    if (TM == 1) return tree[i];  // LDS
    if (TM == 0) return __builtin_amdgcn_raw_buffer_load_b32(gt, (int)(i << 2), 0, 0);
    const bool in_lds = i < (uint32_t)kWideTreeLds;
    const uint32_t l = tree[in_lds ? i : 0u];
    const uint32_t g = __builtin_amdgcn_raw_buffer_load_b32(gt, (int)(in_lds ? kOOB : i << 2), 0, 0);
    return in_lds ? l : g;
}

// TOA bins of N events t[o..o+N) (kNone: outside the edges).  All root
// words are read first; the descent is one wave-uniform round per tree level
// that still holds an internal node in some lane (none for most edge sets).
template <int TM, int N, int O>
__device__ __forceinline__ void toa_bins(const WideToa &tp, const uint32_t *tree, __amdgpu_buffer_rsrc_t gt,
                                         const int (&t)[EPT], uint32_t (&bin)[N]) {
    uint32_t dc[N], w[N];
    const uint32_t rmask = (1u << tp.sh0) - 1u;
#pragma unroll
    for (int e = 0; e < N; ++e) {
        const uint32_t d = (uint32_t)t[O + e] - tp.lo;
        const bool ok = d <= tp.last && !tp.empty;
        dc[e] = ok ? d : 0u;
        bin[e] = ok ? 0u : kNone;
        w[e] = tree_word<TM>(tree, gt, dc[e] >> tp.sh0);
    }
    const uint32_t fmask = (1u << tp.fb) - 1u;
    for (int lv = 1; lv <= tp.depth; ++lv) {
        bool any = false;
#pragma unroll
        for (int e = 0; e < N; ++e) any |= (w[e] & 0xFFFFu) == kLeafNone;
        if (!__builtin_amdgcn_ballot_w64(any)) break;
        const int sh = max(0, tp.sh0 - lv * tp.fb);  // (nodes narrower than the fan-out: width-1 children)
        // (branch-free: leaves read word 0 and keep their word)
#pragma unroll
        for (int e = 0; e < N; ++e) {
            const bool in = (w[e] & 0xFFFFu) == kLeafNone;
            const uint32_t nw = tree_word<TM>(tree, gt, in ? (w[e] >> 16) + ((dc[e] >> sh) & fmask) : 0u);
            w[e] = in ? nw : w[e];
        }
    }
    // leaf: bin at its start + (the offset inside the ROOT bucket reached the
    // one threshold inside the leaf)
#pragma unroll
    for (int e = 0; e < N; ++e)
        bin[e] = bin[e] == kNone ? kNone : (w[e] & 0xFFFFu) + ((dc[e] & rmask) >= (w[e] >> 16) ? 1u : 0u);
}

// events of unit u: chunks 2u, 2u + 1; thread tid takes chunk 2u + tid / CT
// (wave-uniform) as thread tid % CT of it.  Chunk pointers from the block's
// LDS copy of the chunk table (s_ct, chunks from c0 on) or the global table.
// (u >= ue, past the block's units: dropped events, no loads -- p and t are
// always assigned, so the caller needs no branch and the registers no
// liveness across the unit)
__device__ __forceinline__ void unit_load(const WideArgs &a, const PixChunk *s_ct, long long c0, long long u,
                                          long long ue, int (&p)[EPT], int (&t)[EPT]) {
    const int tid = threadIdx.x;
    const long long c = u * 2 + __builtin_amdgcn_readfirstlane(tid / CT);
    const int tl = tid % CT;
    if (c >= a.n_chunks || u >= ue) {
#pragma unroll
        for (int e = 0; e < EPT; ++e) {
            p[e] = a.pid_off - 1;  // outside the LUT: dropped
            t[e] = 0;
        }
        return;
    }
    const PixChunk ch = s_ct ? s_ct[c - c0] : a.ctab[c];
    if (ch.n == kChunk) {  // full and 16-byte aligned
#pragma unroll
        for (int j = 0; j < EPT / 4; ++j) {
            const int off = (j * CT + tl) * 4;
            const v4i pv = ld_stream4(ch.pid + off);
            const v4i tv = ld_stream4(ch.toa + off);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                p[j * 4 + q] = pv[q];
                t[j * 4 + q] = tv[q];
            }
        }
        return;
    }
    const int rem = ch.n < 0 ? -ch.n : ch.n;  // < 0: full but misaligned
#pragma unroll
    for (int j = 0; j < EPT / 4; ++j) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int off = (j * CT + tl) * 4 + q;
            const bool ok = off < rem;
            p[j * 4 + q] = ok ? ld_global(ch.pid + off) : a.pid_off - 1;
            t[j * 4 + q] = ok ? ld_global(ch.toa + off) : 0;
        }
    }
}

// ---------------------------------------------------------------------------
// The partitioning step shared by both passes.  LDS (words): staging
// [UNIT + 3 P4] (runs padded to 4) | counts x 2 (unit parity) [P4 + 64 lane
// dummies] | staging offset and write fill per partition [P4] (offset | fill
// << 16) | page of the run's first entries [P4] | first new page [P4] | scan
// scratch [32] | pool [4].  Thread p < P owns partition p: its open page and
// fill, and the row's page and entry counts, live in that thread's registers.
// Every run is padded to a multiple of 4 entries (pads: kNone in staging,
// kPad16 / kNone in the pages, skipped by the readers), so fills stay 4-aligned
// and the write-out moves groups of four entries (one 16-byte LDS read, one 8-
// or 16-byte store) that never straddle a run or a page.
// ---------------------------------------------------------------------------
constexpr uint32_t kPad16 = 0xFFFFu;

struct PartLds {
    uint32_t *stg, *cnt0, *cnt1, *w, *pool;
    uint32_t *offw;  // per partition: staging offset | write fill << 16 (read per event: one word, banks spread)
    uint2 *pg;       // per partition: {page of the run's first entries, first new page}
};

// sub: rank counters per partition (lane groups of 64 / sub lanes each own
// one), so lanes of one wave that hit the same partition spread over sub
// counters; the counts become per-group staging offsets after the scan
__host__ __device__ constexpr size_t part_words(int P, int sub = 1) {
    return (size_t)UNIT + 3 * (size_t)align4(P) + 2 * ((size_t)align4(P) * sub + 64) + 3 * (size_t)align4(P) + 32 + 4;
}
constexpr int kWideMaxTpb = 256;  // tiles per band (second pass partitions)
// first pass: partition layout | pixel table | TOA tree | chunk table
constexpr size_t kWideScatterWords = part_words(kWideMaxParts) + ((size_t)1 << kWideMaxCacheBits) + kWideTreeLds +
                                     sizeof(PixChunk) / 4 * kWideLdsChunks;
static_assert(kWideScatterWords * 4 <= 160 * 1024, "first pass LDS");
// second pass: partition layout | item row prefix | staged page ids, counts
constexpr int kWideSplitSub = 8;  // the second pass: few partitions (<= 256 tiles of a band)
constexpr size_t kWideSplitWords = part_words(kWideMaxTpb, kWideSplitSub) + kWideMaxRows + 1 + 2 * 1024;

__device__ __forceinline__ PartLds part_lds(uint32_t *sm, int P, int sub = 1) {
    const uint32_t P4 = (uint32_t)align4(P);
    PartLds s;
    s.stg = sm;
    s.cnt0 = s.stg + UNIT + 3 * P4;
    s.cnt1 = s.cnt0 + P4 * (uint32_t)sub + 64;
    s.offw = s.cnt1 + P4 * (uint32_t)sub + 64;
    s.pg = reinterpret_cast<uint2 *>(s.offw + P4);  // (8-byte aligned: P4 a multiple of 4)
    s.w = s.offw + 3 * P4;
    s.pool = s.w + 32;
    return s;
}

struct Owner {  // registers of the owner thread of one partition
    uint32_t cur = kNone, fill = (uint32_t)PAGE, np = 0, ev = 0;
};

// One unit: keys (kNone = no entry) are ranked per partition (part = key >>
// pbits) with returning LDS atomics, staged sorted by partition and appended
// to the partitions' pages (entries: key & emask, as u16 or u32).  next()
// runs right after the rank atomics (the next unit's loads), mid() between
// the staging and the write-out (the next unit's front end, whose gathers
// then fly behind the write-out).
template <bool E16, int ABL = 0, int SUB = 1, typename NEXT, typename MID>
__device__ __forceinline__ void part_unit(const PartLds &s, int P, int pbits, uint32_t emask, int parity,
                                          const uint32_t (&key)[EPT], Owner &own, uint32_t pool_base,
                                          uint32_t cap, __amdgpu_buffer_rsrc_t pool, uint32_t *__restrict__ page_cnt,
                                          uint32_t *__restrict__ page_part, uint32_t *overflow, NEXT next, MID mid) {
    const int tid = threadIdx.x;
    const uint32_t P4 = (uint32_t)align4(P);
    uint32_t *cnt = parity ? s.cnt1 : s.cnt0;
    uint32_t *cnt_next = parity ? s.cnt0 : s.cnt1;
    const uint32_t dummy = P4 * SUB + (uint32_t)(tid & 63);
    // this lane's counter of a partition (SUB > 1: its lane group's)
    const uint32_t grp = SUB > 1 ? (uint32_t)(tid & 63) / (64u / SUB) : 0u;
    uint32_t rank[EPT];
#pragma unroll
    for (int e = 0; e < EPT; ++e)
        rank[e] = __hip_atomic_fetch_add(cnt + (key[e] != kNone ? (key[e] >> pbits) * SUB + grp : dummy), 1u,
                                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    next();
    __syncthreads();
    uint32_t n = 0, v = 0;
    uint32_t sc[SUB];
    if (tid < P) {
#pragma unroll
        for (int c = 0; c < SUB; ++c) {
            sc[c] = cnt[tid * SUB + c];
            n += sc[c];
            cnt_next[tid * SUB + c] = 0;
        }
        v = (n + 3u) & ~3u;
    }
    // exclusive scan of the padded runs with one barrier: every wave adds
    // the totals of the waves before it itself (16 broadcast LDS reads)
    const uint32_t inc = wave_inclusive_scan(v);
    const int wid = tid >> 6;
    if ((tid & 63) == 63) s.w[wid] = inc;
    __syncthreads();
    // lanes 0..15 hold the wave totals; their inclusive scan gives this
    // wave's base (lane wid - 1) and the unit total (lane 15)
    const int lane = tid & 63;
    uint32_t x = lane < NT / 64 ? s.w[lane] : 0u;
#pragma unroll
    for (int d = 1; d < NT / 64; d <<= 1) {
        const uint32_t y = __shfl_up(x, d, 64);
        if (lane >= d) x += y;
    }
    const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)x, NT / 64 - 1);
    const uint32_t wbase = wid ? (uint32_t)__builtin_amdgcn_readlane((int)x, wid - 1) : 0u;
    const uint32_t off = wbase + inc - v;
    if (SUB > 1 && tid < P) {
        // the lane groups' staging offsets, over their counts
        uint32_t o = off;
#pragma unroll
        for (int c = 0; c < SUB; ++c) {
            cnt[tid * SUB + c] = o;
            o += sc[c];
        }
    }
    if (tid < P && n > 0) {
        for (uint32_t j = n; j < v; ++j) s.stg[off + j] = kNone;  // the run's pads
        // the run occupies positions [fill, fill + v) of the partition's
        // chain: < PAGE in the open page, the rest in n_new new pages
        const uint32_t room = (uint32_t)PAGE - own.fill;
        uint32_t first = kNone;
        bool lost = false;
        if (v > room) {
            const uint32_t n_new = (v - room + PAGE - 1) >> PB;
            const uint32_t o = __hip_atomic_fetch_add(s.pool, n_new, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (o + n_new <= cap) {
                first = pool_base + o;
                if (own.cur != kNone) page_cnt[own.cur] = PAGE;
                for (uint32_t k = 0; k < n_new; ++k) {
                    page_part[first + k] = (uint32_t)tid;
                    page_cnt[first + k] = PAGE;
                }
                own.np += n_new;
            } else {
                // pool exhausted (cannot happen with the host's pool size):
                // the reserved pages inside the pool are marked unused, the
                // run's entries past its open page are dropped, and the flag
                // makes finalize fail
                *overflow = 1u;
                for (uint32_t k = o; k < cap && k < o + n_new; ++k) page_part[pool_base + k] = kNone;
                lost = true;
            }
        }
        s.offw[tid] = off | (own.fill << 16);
        s.pg[tid] = make_uint2(own.cur, first);
        const uint32_t end = own.fill + v;
        if (lost) {  // the open page is full now: the next run allocates again
            if (own.cur != kNone) page_cnt[own.cur] = PAGE;
            own.cur = kNone;
            own.fill = PAGE;
        } else if (end > (uint32_t)PAGE) {
            const uint32_t k_last = (end - 1) >> PB;  // the last entry's page, counted from the open one
            own.cur = first + k_last - 1;
            own.fill = end - (k_last << PB);
        } else {
            own.fill = end;
        }
        own.ev += v;
    }
    __syncthreads();
    if (ABL & 4) {  // (ablation: counts and pages only)
        mid();
        return;
    }
    // (branch-free: entries without a key store into the lane's dummy word
    // of the other count array, which is never read)
#pragma unroll
    for (int e = 0; e < EPT; ++e) {
        const bool ok = key[e] != kNone;
        const uint32_t o = SUB > 1 ? cnt[ok ? (key[e] >> pbits) * SUB + grp : 0u]
                                   : s.offw[ok ? key[e] >> pbits : 0u] & 0xFFFFu;
        uint32_t *dst = ok ? s.stg + o + rank[e] : cnt_next + dummy;
        *dst = key[e];
    }
    __syncthreads();
    mid();
#pragma unroll 1
    for (uint32_t g = (uint32_t)tid * 4u; g < total; g += NT * 4u) {
        const uint4 k4 = *reinterpret_cast<const uint4 *>(s.stg + g);
        const uint32_t part = k4.x >> pbits;  // a group's first entry is never a pad
        const uint32_t ow = s.offw[part];
        const uint2 pp = s.pg[part];  // (one 8-byte read for both pages)
        const uint32_t x = (ow >> 16) + g - (ow & 0xFFFFu);
        const uint32_t np = pp.y, wc = pp.x;
        const uint32_t page = x < (uint32_t)PAGE ? wc : np + (x >> PB) - 1u;
        const bool lost = x < (uint32_t)PAGE ? wc == kNone : np == kNone;  // pool overflow (flagged)
        // byte offset inside the row's pool (a store out of range is dropped)
        const uint32_t at = ((page - pool_base) << PB) + (x & (PAGE - 1));
        const int boff = (lost || (ABL & 2)) ? (int)kOOB : (int)(at << (E16 ? 1 : 2));
        // (diagnostics, ABL & 64: the page stores with the non-temporal hint)
        constexpr int kAux = (ABL & 64) ? 2 : 0;
        if (E16) {
            auto e16 = [&](uint32_t k) { return k == kNone ? kPad16 : (k & emask); };
            typedef unsigned int v2u __attribute__((ext_vector_type(2)));
            __builtin_amdgcn_raw_buffer_store_b64(v2u{e16(k4.x) | (e16(k4.y) << 16), e16(k4.z) | (e16(k4.w) << 16)},
                                                  pool, boff, 0, kAux);
        } else {
            auto e32 = [&](uint32_t k) { return k == kNone ? kNone : (k & emask); };
            __builtin_amdgcn_raw_buffer_store_b128(v4u{e32(k4.x), e32(k4.y), e32(k4.z), e32(k4.w)}, pool, boff,
                                                   0, kAux);
        }
    }
}

// End of a partitioning block: the open pages' counts, the row's counts and
// its page list sorted by partition (rows.*[row][p], list[pool_base ..]).
__device__ __forceinline__ void part_finish(const PartLds &s, int P, const Owner &own, uint32_t pool_base,
                                            uint32_t cap, uint32_t *__restrict__ page_cnt,
                                            const uint32_t *__restrict__ page_part, uint32_t *__restrict__ list,
                                            const WideRows &rows, uint32_t row) {
    const int tid = threadIdx.x;
    __syncthreads();  // the last unit's write-out read offw / cnt0
    if (tid < P) {
        if (own.cur != kNone) page_cnt[own.cur] = own.fill;
        rows.cnt[(size_t)row * rows.ncols + tid] = own.np;
        rows.ev[(size_t)row * rows.ncols + tid] = own.ev;
    }
    uint32_t tot;
    const uint32_t lo = block_exclusive_scan(tid < P ? own.np : 0u, s.w, &tot);
    if (tid < P) {
        rows.off[(size_t)row * rows.ncols + tid] = lo;
        s.cnt0[tid] = lo;  // list cursors
    }
    if (tid == 0) rows.pool[row] = pool_base;
    __syncthreads();
    const uint32_t used = min(s.pool[0], cap);
    for (uint32_t i = (uint32_t)tid; i < used; i += NT) {
        const uint32_t part = page_part[pool_base + i];
        if (part >= (uint32_t)P) continue;  // (a page of a failed allocation: overflow, flagged)
        const uint32_t slot = __hip_atomic_fetch_add(s.cnt0 + part, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        list[pool_base + slot] = pool_base + i;
    }
}

}  // namespace

// ---------------------------------------------------------------------------
// chunk table (+ the counters of this batch's passes)
// ---------------------------------------------------------------------------
// KARG: the messages come as kernel arguments (at most kKargSegs: a batch of
// 14 pulses), so no descriptor upload precedes the launch
template <bool KARG>
__global__ __launch_bounds__(256) void k_wide_chunks(WideArgs a, SegKarg sk, PixChunk *__restrict__ ctab) {
    const long long c = (long long)blockIdx.x * 256 + threadIdx.x;
    if (c == 0) {
        a.counters[0] = a.counters[1] = a.counters[3] = a.counters[4] = 0u;
        *a.pool2_next = 0u;
    }
    if (c >= a.n_chunks) return;
    SegDesc sd;
    if (KARG) {  // last message with chunk0 <= c (static indices: scalar kernarg loads)
        sd = sk.s[0];
#pragma unroll
        for (int i = 1; i < kKargSegs; ++i)
            if (i < a.n_segs && sk.s[i].chunk0 <= c) sd = sk.s[i];
    } else {
        int lo = 0, hi = a.n_segs - 1;
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (a.segs[mid].chunk0 <= c) lo = mid; else hi = mid - 1;
        }
        sd = a.segs[lo];
    }
    const long long base = (c - sd.chunk0) * kChunk;
    const long long left = sd.n - base;
    PixChunk ch;
    ch.pid = sd.pid + base;
    ch.toa = sd.toa + base;
    ch.n = (int)(left < kChunk ? left : kChunk);
    if (ch.n == kChunk && (((uintptr_t)ch.pid | (uintptr_t)ch.toa) & 15u) != 0) ch.n = -kChunk;
    ch.pad = 0;
    ctab[c] = ch;
}

// ---------------------------------------------------------------------------
// pixel table: sampled pixel counts, then per slot the most frequent pixel
// ---------------------------------------------------------------------------
// sampled chunks: per block, counts aggregated in an LDS table of 2048
// tagged slots first (a Zipf-hot pixel holds a large share of a DREAM sample:
// one global address would serialize at the memory side), then one global
// atomic per slot; pixels whose slot is taken count with global atomics
__global__ __launch_bounds__(256) void k_wide_sample(WideArgs a, uint32_t *__restrict__ cnt) {
    constexpr int NS = 2048;
    __shared__ uint32_t s_key[NS], s_cnt[NS];
    for (int i = threadIdx.x; i < NS; i += 256) {
        s_key[i] = kNone;
        s_cnt[i] = 0;
    }
    __syncthreads();
    const long long n = a.n_chunks;
    const long long c = (long long)blockIdx.x * n / gridDim.x;
    if (c < n) {
        const PixChunk ch = a.ctab[c];
        const int m = ch.n < 0 ? -ch.n : ch.n;
        for (int i = threadIdx.x; i < m; i += 256) {
            const uint32_t q = (uint32_t)ld_global(ch.pid + i) - (uint32_t)a.pid_off;
            if (q >= a.L) continue;
            const uint32_t slot = (q * 2654435761u) >> 21;
            const uint32_t old = atomicCAS(s_key + slot, kNone, q);
            if (old == kNone || old == q) atomicAdd(s_cnt + slot, 1u);
            else atomicAdd(cnt + q, 1u);
        }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < NS; i += 256)
        if (s_key[i] != kNone) atomicAdd(cnt + s_key[i], s_cnt[i]);
}

template <bool L16>
__global__ __launch_bounds__(256) void k_wide_table(WideArgs a, const void *__restrict__ lut_rep,
                                                    const uint32_t *__restrict__ cnt, uint32_t *__restrict__ tab) {
    const uint32_t C = 1u << a.cbits;
    const uint32_t j = blockIdx.x * 256u + threadIdx.x;
    if (j >= C) return;
    uint32_t best = 0, bq = kNone;
    for (uint32_t q = j; q < a.L; q += C) {
        const uint32_t v = cnt[q];
        if (v > best || bq == kNone) {
            best = v;
            bq = q;
        }
    }
    uint32_t w = 0;  // empty slot: never a hit
    if (bq != kNone) {
        uint32_t val;
        if (L16) {
            const uint32_t v = reinterpret_cast<const uint16_t *>(lut_rep)[bq];
            val = v == 0xFFFFu ? kTabValue : v;
        } else {
            const int v = reinterpret_cast<const int *>(lut_rep)[bq];
            val = v < 0 ? kTabValue : (uint32_t)v / (uint32_t)a.T;
        }
        w = kTabValid | ((bq >> a.cbits) << kTagShift) | val;
    }
    tab[j] = w;
}

// ---------------------------------------------------------------------------
// first pass
// ---------------------------------------------------------------------------
// ABL (diagnostics build only, wrong results by design): timing ablations of
// the first pass -- 1 no gathers, 2 no page stores, 4 no staging or
// write-out, 16 no front end (keys from a hash of the raw words)
template <bool L16, int TM, bool E16, int ABL = 0>
__global__ __launch_bounds__(NT) void k_wide_scatter(WideArgs a) {
    // static layout for the largest partition count and table, so every LDS
    // address is a constant (fewer live scalar registers in the loop)
    __shared__ __attribute__((aligned(16))) uint32_t sm[kWideScatterWords];
    const int P = a.n_parts;
    const PartLds s = part_lds(sm, kWideMaxParts);
    const uint32_t C = a.cbits ? 1u << a.cbits : 0u;
    uint32_t *s_tab = sm + part_words(kWideMaxParts);
    uint32_t *s_tree = s_tab + (1u << kWideMaxCacheBits);
    const uint32_t tw = TM == 1 ? (uint32_t)align4(a.toa.words) : TM == 2 ? (uint32_t)kWideTreeLds : 0u;
    const __amdgpu_buffer_rsrc_t gtree = make_rsrc(a.toa.tree, (uint32_t)a.toa.words * 4u);
    PixChunk *s_ctab = reinterpret_cast<PixChunk *>(s_tree + kWideTreeLds);
    const int tid = threadIdx.x;
    {  // pixel table and TOA tree, each into its own slot: every load of a
       // thread issued before its stores
        const uint4 *pt = reinterpret_cast<const uint4 *>(a.pix_tab);
        const uint4 *tt = reinterpret_cast<const uint4 *>(a.toa.tree);
        const int c4 = (int)(C / 4u), t4 = (int)(tw / 4u);
        lds_fill<4>(reinterpret_cast<uint4 *>(s_tab), c4 + t4, [&](int i) {
            return g_ld(i < c4 ? pt + i : tt + (i - c4));
        }, [&](int i) { return reinterpret_cast<uint4 *>(i < c4 ? s_tab + 4 * i : s_tree + 4 * (i - c4)); });
    }
    for (int i = tid; i < 2 * (kWideMaxParts + 64); i += NT) s.cnt0[i] = 0;
    if (tid == 0) s.pool[0] = 0;
    const long long n_units = (a.n_chunks + 1) / 2;
    const long long cb = (long long)blockIdx.x * n_units / gridDim.x;
    const long long ce = ((long long)blockIdx.x + 1) * n_units / gridDim.x;
    const long long c0 = cb * 2, c1 = ce * 2 < a.n_chunks ? ce * 2 : a.n_chunks;
    const bool fit = c1 - c0 <= kWideLdsChunks;
    if (fit)
        for (long long i = tid; i < c1 - c0; i += NT) s_ctab[i] = a.ctab[c0 + i];
    __syncthreads();
    const PixChunk *s_ct = fit ? s_ctab : nullptr;
    const uint32_t pool_base = blockIdx.x * a.cap1;
    // the block's pool (its pages only), as a buffer: 32-bit store offsets
    const __amdgpu_buffer_rsrc_t pool = make_rsrc(
        reinterpret_cast<unsigned char *>(a.pages1) + (size_t)pool_base * PAGE * (E16 ? 2 : 4),
        a.cap1 * (uint32_t)PAGE * (E16 ? 2u : 4u));
    const uint32_t cmask = C ? C - 1u : 0u;
    const uint32_t lut_bytes = a.L * (L16 ? 2u : 4u);
    const __amdgpu_buffer_rsrc_t lut = make_rsrc(a.lut, lut_bytes);
    const uint32_t T = (uint32_t)a.T;
    const uint32_t emask = (1u << a.pbits) - 1u;
    Owner own;
    int p[EPT], t[EPT];
    // Front end of a unit, in two steps so its latency hides behind the
    // previous unit's write-out: issue() bins the TOA (t dies), probes the
    // pixel table and issues the gathers of the misses (hits and unknown ids
    // load out of range: no request); finish() turns the words into keys.
    uint32_t q[EPT], w[EPT], g[EPT], bin[EPT];
    auto issue = [&]() __attribute__((always_inline)) {
        if (ABL & 16) return;
        toa_bins<TM, EPT, 0>(a.toa, s_tree, gtree, t, bin);
#pragma unroll
        for (int e = 0; e < EPT; ++e) {
            q[e] = (uint32_t)p[e] - (uint32_t)a.pid_off;
            w[e] = C ? s_tab[q[e] & cmask] : 0u;
        }
#pragma unroll
        for (int e = 0; e < EPT; ++e) {
            const bool hit = (w[e] & kTabValid) && ((w[e] >> kTagShift) & kTagMask) == (q[e] >> a.cbits);
            const bool miss = q[e] < a.L && !hit;
            const uint32_t off = miss ? q[e] * (L16 ? 2u : 4u) : kOOB;
            if (ABL & 1)
                g[e] = q[e] & 0xFFu;
            else
                g[e] = L16 ? (uint32_t)__builtin_amdgcn_raw_buffer_load_b16(lut, (int)off, 0, 0)
                           : __builtin_amdgcn_raw_buffer_load_b32(lut, (int)off, 0, 0);
            // a hit keeps its word with the valid bit cleared, so no word --
            // not a dropped pixel's under tag 511 either -- reads as kNone
            w[e] = hit ? (w[e] & ~kTabValid) : kNone;
        }
    };
    auto finish = [&](uint32_t (&key)[EPT]) __attribute__((always_inline)) {
        if (ABL & 16) {  // (ablation: no front end; issue() did nothing)
#pragma unroll
            for (int e = 0; e < EPT; ++e)
                key[e] = ((uint32_t)p[e] * 2654435761u ^ (uint32_t)t[e]) & ((1u << (a.pbits + 9)) - 1u);
            return;
        }
#pragma unroll
        for (int e = 0; e < EPT; ++e) {
            uint32_t base;
            bool ok;
            if (w[e] != kNone) {
                const uint32_t v = w[e] & kTabValue;
                ok = v != kTabValue;
                base = v * T;
            } else if (L16) {
                ok = q[e] < a.L && g[e] != 0xFFFFu;
                base = g[e] * T;
            } else {
                ok = q[e] < a.L && (int)g[e] >= 0;
                base = g[e];
            }
            key[e] = ok && bin[e] != kNone ? base + bin[e] : kNone;
        }
    };
    unit_load(a, s_ct, c0, cb, ce, p, t);
    issue();
    for (long long u = cb; u < ce; ++u) {
        uint32_t key[EPT];
        finish(key);
        part_unit<E16, ABL>(s, P, a.pbits, emask, (int)(u & 1), key, own, pool_base, a.cap1, pool, a.page_cnt,
                       a.page_part, a.overflow,
                       // (unconditional: past the last unit, dropped events)
                       [&]() __attribute__((always_inline)) { unit_load(a, s_ct, c0, u + 1, ce, p, t); },
                       [&]() __attribute__((always_inline)) { issue(); });
    }
    part_finish(s, P, own, pool_base, a.cap1, a.page_cnt, a.page_part, a.list, a.rows1, blockIdx.x);
}

// ---------------------------------------------------------------------------
// plan: per partition p, items of consecutive rows (rows [0, nrows) of the
// first pass, or the second pass's rows of p's band); band_out: the items of
// each partition (the second pass's rows of that band).  Items of partitions
// that need several (the hot ones: Zipf pixels, peaked TOA) are numbered from
// the front (count[0]), single items from the back (count[1] of them, at
// max_items - 1 down), so the consuming pass -- which takes item_at(block) --
// runs the long items first and the short ones fill the tail.
// ---------------------------------------------------------------------------
constexpr int kPlanWaves = 16;  // partitions per plan block (a wave each)
__global__ __launch_bounds__(64 * kPlanWaves) void k_wide_plan(WideRows rows, int nrows,
                                                              const uint2 *__restrict__ band_rows, int tpb_bits,
                                                              uint32_t item_max, uint4 *__restrict__ items,
                                                              uint32_t *__restrict__ count,
                                                              uint32_t *__restrict__ count1, uint32_t max_items,
                                                              uint2 *__restrict__ band_out,
                                                              uint32_t *__restrict__ overflow, int n_parts) {
    __shared__ uint32_t s_n[kPlanWaves], s_base[kPlanWaves];
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int p = blockIdx.x * kPlanWaves + wv;
    uint32_t r0 = 0, nr = (uint32_t)nrows, col = (uint32_t)p, n = 0;
    if (p < n_parts) {
        if (band_rows) {
            const uint2 br = band_rows[p >> tpb_bits];
            r0 = br.x;
            nr = br.y;
            col = (uint32_t)p & ((1u << tpb_bits) - 1u);
        }
        unsigned long long sum = 0;
        for (uint32_t r = lane; r < nr; r += 64) sum += rows.ev[(size_t)(r0 + r) * rows.ncols + col];
#pragma unroll
        for (int d = 32; d > 0; d >>= 1) sum += __shfl_xor(sum, d, 64);
        if (sum > 0) {
            const unsigned long long k = (sum + item_max - 1) / item_max;
            n = (uint32_t)(k < nr ? k : nr);
            if (n > (uint32_t)kWideMaxRows) n = kWideMaxRows;
            n = n < 1 ? 1 : n;
        }
    }
    if (lane == 0) s_n[wv] = n;
    __syncthreads();
    if (threadIdx.x == 0) {
        // one reservation per block and end (a single counter that every
        // partition hit serialised the plan of 8k tiles)
        uint32_t multi = 0, singles = 0;
        for (int i = 0; i < kPlanWaves; ++i) {
            multi += s_n[i] > 1 ? s_n[i] : 0u;
            singles += s_n[i] == 1 ? 1u : 0u;
        }
        uint32_t bm = multi ? atomicAdd(count, multi) : 0u;
        uint32_t bs = singles ? atomicAdd(count1, singles) : 0u;
        // (the two ends cannot meet with the host's bound: max_items counts
        // every partition once more than the item sizes need)
        const bool meet = multi && bm + multi + *count1 > max_items;
        for (int i = 0; i < kPlanWaves; ++i) {
            uint32_t ni = s_n[i], base = 0;
            if (ni > 1) {
                base = bm;
                bm += ni;
            } else if (ni == 1) {
                const uint32_t k = bs++;
                base = k < max_items ? max_items - 1u - k : max_items;
            }
            if (ni && (base + ni > max_items || meet)) {
                *overflow = 1u;  // cannot happen with the host's bound
                ni = 0;
            }
            s_n[i] = ni;
            s_base[i] = base;
            const int pi = blockIdx.x * kPlanWaves + i;
            if (band_out && pi < n_parts) band_out[pi] = make_uint2(base, ni);
        }
    }
    __syncthreads();
    n = s_n[wv];
    const uint32_t base = s_base[wv];
    for (uint32_t j = lane; j < n; j += 64)
        items[base + j] = make_uint4((uint32_t)p, r0 + (uint32_t)((unsigned long long)j * nr / n),
                                     r0 + (uint32_t)((unsigned long long)(j + 1) * nr / n), n == 1 ? 1u : 0u);
}

// item of block b: the multi-item partitions' items first, then the singles
__device__ __forceinline__ uint32_t item_at(uint32_t b, const uint32_t *count, const uint32_t *count1,
                                            uint32_t max_items) {
    const uint32_t nm = *count, ns = *count1;
    if (b < nm) return b;
    return b - nm < ns ? max_items - 1u - (b - nm) : kNone;
}

namespace {

// The pages of one item (partition col of rows [r0, r0 + nr)): prefix of the
// rows' page counts in LDS (s_pref[nr] = the item's pages).  Ends with a barrier.
__device__ __forceinline__ uint32_t item_prefix(const WideRows &rows, uint32_t r0, uint32_t nr, uint32_t col,
                                                uint32_t *s_pref, uint32_t *s_w) {
    const int tid = threadIdx.x;
    const uint32_t v = (uint32_t)tid < nr ? rows.cnt[(size_t)(r0 + tid) * rows.ncols + col] : 0u;
    uint32_t tot;
    const uint32_t x = block_exclusive_scan(v, s_w, &tot);
    if ((uint32_t)tid <= nr) s_pref[tid] = (uint32_t)tid < nr ? x : tot;
    __syncthreads();
    return tot;
}

// page k of the item: its row (last r with s_pref[r] <= k), then the list entry
__device__ __forceinline__ uint32_t item_page(const WideRows &rows, const uint32_t *__restrict__ list,
                                              uint32_t r0, uint32_t nr, uint32_t col, const uint32_t *s_pref,
                                              uint32_t k) {
    uint32_t lo = 0, hi = nr - 1;
    while (lo < hi) {
        const uint32_t mid = (lo + hi + 1) >> 1;
        if (s_pref[mid] <= k) lo = mid; else hi = mid - 1;
    }
    const size_t r = r0 + lo;
    return list[rows.pool[r] + rows.off[r * rows.ncols + col] + (k - s_pref[lo])];
}

}  // namespace

// The pages of an item, staged in LDS in chunks of kWidePagesLds: page id and
// entry count of pages [base, base + m) (independent loads, one round trip).
constexpr int kWidePagesLds = 1024;
__device__ __forceinline__ void stage_pages(const WideRows &rows, const uint32_t *__restrict__ list,
                                            const uint32_t *__restrict__ page_cnt, uint32_t r0, uint32_t nr,
                                            uint32_t col, const uint32_t *s_pref, uint32_t base, uint32_t m,
                                            uint32_t *s_pg, uint32_t *s_pc) {
    for (uint32_t k = threadIdx.x; k < m; k += blockDim.x) {
        const uint32_t page = item_page(rows, list, r0, nr, col, s_pref, base + k);
        s_pg[k] = page;
        s_pc[k] = page_cnt[page];
    }
}

// ---------------------------------------------------------------------------
// second pass (two-level form): one item of a band -> tile pages
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(NT) void k_wide_split(WideArgs a) {
    __shared__ __attribute__((aligned(16))) uint32_t sm[kWideSplitWords];
    const uint32_t item = item_at(blockIdx.x, a.counters, a.counters + 3, a.max_items1);
    if (item == kNone) return;
    const uint4 it = a.items1[item];
    const int P = 1 << a.tpb_bits;
    const PartLds s = part_lds(sm, kWideMaxTpb, kWideSplitSub);
    uint32_t *s_pref = sm + part_words(kWideMaxTpb, kWideSplitSub);
    uint32_t *s_pg = s_pref + kWideMaxRows + 1;
    uint32_t *s_pc = s_pg + kWidePagesLds;
    __shared__ unsigned long long s_ev[16];
    const int tid = threadIdx.x;
    const uint32_t band = it.x, r0 = it.y, nr = it.z - it.y;
    for (int i = tid; i < 2 * (kWideMaxTpb * kWideSplitSub + 64); i += NT) s.cnt0[i] = 0;
    // the item's entries size its pool (one allocation per item)
    unsigned long long ev = (uint32_t)tid < nr ? a.rows1.ev[(size_t)(r0 + tid) * a.rows1.ncols + band] : 0u;
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) ev += __shfl_xor(ev, d, 64);
    if ((tid & 63) == 0) s_ev[tid >> 6] = ev;
    const uint32_t n_pages = item_prefix(a.rows1, r0, nr, band, s_pref, s.w);
    if (tid == 0) {
        unsigned long long e = 0;
        for (int i = 0; i < NT / 64; ++i) e += s_ev[i];
        // entries in (first-pass pads included) + this pass's pads (<= 3 per
        // partition and unit; a unit per 16 pages, one more per LDS chunk)
        const unsigned long long units = (n_pages + NT / 64 - 1) / (NT / 64) + (n_pages + kWidePagesLds - 1) / kWidePagesLds;
        const unsigned long long need = (e + 3ull * P * units + PAGE - 1) / PAGE + (unsigned long long)P + 1;
        const uint32_t base = atomicAdd(a.pool2_next, (uint32_t)(need < 0x7FFFFFFFull ? need : 0x7FFFFFFFull));
        uint32_t cap = (uint32_t)need;
        if ((unsigned long long)base + need > a.pool2_cap) {
            *a.overflow = 1u;  // cannot happen with the host's bound
            cap = 0;
        }
        s.pool[0] = 0;
        s.pool[1] = a.page0_2 + base;  // second-pass pages follow the first pass's
        s.pool[2] = cap;
    }
    __syncthreads();
    const uint32_t pool_base = s.pool[1], cap = s.pool[2];
    const __amdgpu_buffer_rsrc_t pool = make_rsrc(
        reinterpret_cast<unsigned char *>(a.pages2) + (size_t)(pool_base - a.page0_2) * PAGE * 2, cap * (uint32_t)PAGE * 2u);
    const int lane = tid & 63;
    const uint32_t wv = (uint32_t)__builtin_amdgcn_readfirstlane(tid >> 6);
    const uint32_t *pages1 = reinterpret_cast<const uint32_t *>(a.pages1);
    Owner own;
    uint32_t key[EPT], nxt[EPT];
    uint32_t u = 0;  // units so far (parity)
    for (uint32_t pb = 0; pb < n_pages; pb += kWidePagesLds) {
        const uint32_t m = min((uint32_t)kWidePagesLds, n_pages - pb);
        __syncthreads();  // the previous chunk's readers are done with s_pg / s_pc
        stage_pages(a.rows1, a.list, a.page_cnt, r0, nr, band, s_pref, pb, m, s_pg, s_pc);
        __syncthreads();
        // unit: pages 16v .. 16v + 15 of the chunk, wave wv takes one, each
        // lane 16 consecutive entries (4 x 16 bytes)
        auto load = [&](uint32_t v, uint32_t (&k)[EPT]) __attribute__((always_inline)) {
            const uint32_t j = v * (NT / 64) + wv;
            const uint32_t cnt = j < m ? s_pc[j] : 0u;
            const uint32_t e0 = (uint32_t)lane * EPT;
            const uint4 *src = reinterpret_cast<const uint4 *>(pages1 + (size_t)(j < m ? s_pg[j] : 0u) * PAGE + e0);
#pragma unroll
            for (int q = 0; q < EPT / 4; ++q) {
                const uint4 x = e0 + 4u * q < cnt ? src[q] : make_uint4(kNone, kNone, kNone, kNone);
                k[4 * q] = x.x;
                k[4 * q + 1] = x.y;
                k[4 * q + 2] = x.z;
                k[4 * q + 3] = x.w;
            }
#pragma unroll
            for (int e = 0; e < EPT; ++e)
                if (e0 + (uint32_t)e >= cnt) k[e] = kNone;  // (pads are kNone already)
        };
        const uint32_t n_units = (m + NT / 64 - 1) / (NT / 64);
        load(0, nxt);
        for (uint32_t v = 0; v < n_units; ++v, ++u) {
#pragma unroll
            for (int e = 0; e < EPT; ++e) key[e] = nxt[e];
            part_unit<true, 0, kWideSplitSub>(s, P, kWideTileBits, (1u << kWideTileBits) - 1u, (int)(u & 1), key, own,
                                              pool_base, cap,
                            pool, a.page_cnt, a.page_part, a.overflow,
                            [&]() __attribute__((always_inline)) { load(v + 1, nxt); },
                            []() {});
        }
    }
    part_finish(s, P, own, pool_base, cap, a.page_cnt, a.page_part, a.list, a.rows2, item);
}

// ---------------------------------------------------------------------------
// pass B: one item of a tile histogrammed in LDS
// ---------------------------------------------------------------------------
constexpr int kWideAccThreads = 1024;
constexpr int kWideAccDepth = 4;  // pages in flight per wave
template <int D>
__global__ __launch_bounds__(kWideAccThreads) void k_wide_accumulate(const uint4 *__restrict__ items,
                                                                     const uint32_t *__restrict__ item_count,
                                                                     const uint32_t *__restrict__ item_count1,
                                                                     uint32_t max_items,
                                                                     WideRows rows, const uint32_t *__restrict__ list,
                                                                     const uint32_t *__restrict__ page_cnt,
                                                                     const uint16_t *__restrict__ pages,
                                                                     uint32_t page0, uint32_t colmask,
                                                                     uint32_t *__restrict__ hist, long long n_bins,
                                                                     int wzero) {
    constexpr int NB = 1 << kWideTileBits;
    constexpr int NW = kWideAccThreads / 64;
    __shared__ __attribute__((aligned(16))) uint32_t s_tile[NB + 64];
    __shared__ uint32_t s_pref[kWideMaxRows + 1];
    __shared__ uint32_t s_pg[kWidePagesLds], s_pc[kWidePagesLds];
    __shared__ uint32_t s_w[32];
    const uint32_t item = item_at(blockIdx.x, item_count, item_count1, max_items);
    if (item == kNone) return;
    const uint4 it = items[item];
    const int tid = threadIdx.x;
    for (int i = tid * 4; i < NB + 64; i += kWideAccThreads * 4)
        *reinterpret_cast<uint4 *>(s_tile + i) = make_uint4(0, 0, 0, 0);
    const uint32_t tile = it.x, r0 = it.y, nr = it.z - it.y, col = tile & colmask;
    const uint32_t n_pages = item_prefix(rows, r0, nr, col, s_pref, s_w);  // (+ the barrier for s_tile)
    const int lane = tid & 63;
    const uint32_t wv = (uint32_t)__builtin_amdgcn_readfirstlane(tid >> 6);
    const uint32_t e0 = (uint32_t)lane * 16u;
    const uint32_t dummy = NB + (uint32_t)lane;
    for (uint32_t pb = 0; pb < n_pages; pb += kWidePagesLds) {
        const uint32_t m = min((uint32_t)kWidePagesLds, n_pages - pb);
        if (pb) __syncthreads();
        stage_pages(rows, list, page_cnt, r0, nr, col, s_pref, pb, m, s_pg, s_pc);
        __syncthreads();
        // each wave D pages at a time: 2 x 16 bytes per lane and page
        for (uint32_t k0 = wv; k0 < m; k0 += NW * D) {
            uint4 x[D], y[D];
            uint32_t c[D];
#pragma unroll
            for (int d = 0; d < D; ++d) {
                const uint32_t k = k0 + (uint32_t)d * NW;
                c[d] = k < m ? s_pc[k] : 0u;
                const uint4 *src =
                    reinterpret_cast<const uint4 *>(pages + (size_t)((k < m ? s_pg[k] : page0) - page0) * PAGE + e0);
                x[d] = c[d] > e0 ? src[0] : make_uint4(0, 0, 0, 0);
                y[d] = c[d] > e0 + 8u ? src[1] : make_uint4(0, 0, 0, 0);
            }
#pragma unroll
            for (int d = 0; d < D; ++d) {
                const uint32_t wd[8] = {x[d].x, x[d].y, x[d].z, x[d].w, y[d].x, y[d].y, y[d].z, y[d].w};
#pragma unroll
                for (int q = 0; q < 16; ++q) {
                    const uint32_t v = (wd[q >> 1] >> ((q & 1) * 16)) & 0xFFFFu;
                    __hip_atomic_fetch_add(s_tile + (e0 + (uint32_t)q < c[d] && v != kPad16 ? v : dummy), 1u,
                                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                }
            }
        }
    }
    __syncthreads();
    const long long base = (long long)tile << kWideTileBits;
    if ((it.w & 1u) && base + NB <= n_bins && wzero) {
        // the tile's only item owns its bins, and the window held nothing
        // before this batch: its non-zero groups are stored, nothing is read
        constexpr int V = NB / 4 / kWideAccThreads;
        uint4 *h4 = reinterpret_cast<uint4 *>(hist + base);
        const uint4 *s4 = reinterpret_cast<const uint4 *>(s_tile);
#pragma unroll
        for (int u = 0; u < V; ++u) {
            const uint4 v = s4[u * kWideAccThreads + tid];
            if (v.x | v.y | v.z | v.w) h4[u * kWideAccThreads + tid] = v;
        }
    } else if ((it.w & 1u) && base + NB <= n_bins) {
        // the tile's only item owns its bins: 16-byte read-modify-write
        constexpr int V = NB / 4 / kWideAccThreads;
        uint4 *h4 = reinterpret_cast<uint4 *>(hist + base);
        const uint4 *s4 = reinterpret_cast<const uint4 *>(s_tile);
        uint4 hv[V];
#pragma unroll
        for (int u = 0; u < V; ++u) hv[u] = h4[u * kWideAccThreads + tid];
#pragma unroll
        for (int u = 0; u < V; ++u) {
            const uint4 v = s4[u * kWideAccThreads + tid];
            if (v.x | v.y | v.z | v.w)
                h4[u * kWideAccThreads + tid] = make_uint4(hv[u].x + v.x, hv[u].y + v.y, hv[u].z + v.z, hv[u].w + v.w);
        }
    } else {
        for (int i = tid; i < NB; i += kWideAccThreads) {
            const uint32_t v = s_tile[i];
            if (v != 0u && base + i < n_bins) atomicAdd(hist + base + i, v);
        }
    }
}

// ---------------------------------------------------------------------------
// launch wrappers
// ---------------------------------------------------------------------------
size_t wide_scatter_smem(const WideArgs &a) {
    // (static layout: fits when the table and the tree fit their slots)
    if (a.cbits > kWideMaxCacheBits || a.n_parts > kWideMaxParts || (a.toa.lds && a.toa.words > kWideTreeLds))
        return 1u << 30;
    return kWideScatterWords * 4;
}

hipError_t launch_wide_chunks(const WideArgs &a, const SegDesc *host_segs, hipStream_t st) {
    const unsigned g = (unsigned)((a.n_chunks + 255) / 256);
    SegKarg sk{};
    if (host_segs && a.n_segs <= kKargSegs) {
        for (int i = 0; i < a.n_segs; ++i) sk.s[i] = host_segs[i];
        hipLaunchKernelGGL(k_wide_chunks<true>, dim3(g > 0 ? g : 1), dim3(256), 0, st, a, sk,
                           const_cast<PixChunk *>(a.ctab));
    } else {
        hipLaunchKernelGGL(k_wide_chunks<false>, dim3(g > 0 ? g : 1), dim3(256), 0, st, a, sk,
                           const_cast<PixChunk *>(a.ctab));
    }
    return hipGetLastError();
}

hipError_t launch_wide_table(const WideArgs &a, const void *lut_rep, uint32_t *pix_cnt, uint32_t *tab,
                             hipStream_t st) {
    if (a.cbits == 0) return hipSuccess;
    hipError_t e = hipMemsetAsync(pix_cnt, 0, (size_t)a.L * 4, st);
    if (e != hipSuccess) return e;
    const int g = (int)(a.n_chunks < kWideSample ? a.n_chunks : kWideSample);
    if (g > 0) hipLaunchKernelGGL(k_wide_sample, dim3(g), dim3(256), 0, st, a, pix_cnt);
    const unsigned gt = (unsigned)(((1u << a.cbits) + 255) / 256);
    if (a.lut16)
        hipLaunchKernelGGL(k_wide_table<true>, dim3(gt), dim3(256), 0, st, a, lut_rep, pix_cnt, tab);
    else
        hipLaunchKernelGGL(k_wide_table<false>, dim3(gt), dim3(256), 0, st, a, lut_rep, pix_cnt, tab);
    return hipGetLastError();
}

template <bool L16, int TM, bool E16>
static hipError_t launch_scatter_t(const WideArgs &a, hipStream_t st, hipEvent_t start, hipEvent_t stop) {
    if (wide_scatter_smem(a) > 160 * 1024) return hipErrorInvalidValue;
#ifdef LDE_DIAGNOSTICS
    if (a.ablate && L16 && TM == 1 && E16) {
        switch (a.ablate) {
#define LDE_WABL(m)                                                                                         \
    case m:                                                                                                 \
        hipExtLaunchKernelGGL((k_wide_scatter<true, 1, true, m>), dim3(a.grid1), dim3(NT), 0, st, start, stop, \
                              0, a);                                                                        \
        return hipGetLastError();
            LDE_WABL(1) LDE_WABL(2) LDE_WABL(3) LDE_WABL(4) LDE_WABL(5) LDE_WABL(16) LDE_WABL(18) LDE_WABL(20)
            LDE_WABL(64)
#undef LDE_WABL
        default: return hipErrorInvalidValue;
        }
    }
#endif
    hipExtLaunchKernelGGL((k_wide_scatter<L16, TM, E16>), dim3(a.grid1), dim3(NT), 0, st, start, stop, 0, a);
    return hipGetLastError();
}

template <bool L16, int TM>
static hipError_t launch_scatter_tl(const WideArgs &a, hipStream_t st, hipEvent_t start, hipEvent_t stop) {
    return a.levels == 1 ? launch_scatter_t<L16, TM, true>(a, st, start, stop)
                         : launch_scatter_t<L16, TM, false>(a, st, start, stop);
}

// the tree in LDS when it fits, else its first kWideTreeLds words in LDS and
// the rest through L2 (diagnostics: tree_hybrid = 0, all through L2)
template <bool L16>
static hipError_t launch_scatter_l(const WideArgs &a, hipStream_t st, hipEvent_t start, hipEvent_t stop) {
    if (a.toa.lds) return launch_scatter_tl<L16, 1>(a, st, start, stop);
    if (a.tree_hybrid) return launch_scatter_tl<L16, 2>(a, st, start, stop);
    return launch_scatter_tl<L16, 0>(a, st, start, stop);
}

static unsigned plan_grid(int parts) { return (unsigned)((parts + kPlanWaves - 1) / kPlanWaves); }

hipError_t launch_wide(const WideArgs &a, hipStream_t st, hipEvent_t start, hipEvent_t stop, hipEvent_t bstart,
                       hipEvent_t bstop) {
    if (a.n_parts < 1 || a.n_parts > kWideMaxParts || a.grid1 < 1 || a.grid1 > kWideMaxRows ||
        (a.levels == 2 && a.n_parts > kWideMaxBands))
        return hipErrorInvalidValue;
    hipError_t e = a.lut16 ? launch_scatter_l<true>(a, st, start, stop) : launch_scatter_l<false>(a, st, start, stop);
    if (e != hipSuccess) return e;
    WideRows rows = a.rows1;
    const uint4 *items = a.items1;
    const uint32_t *count = a.counters, *count1 = a.counters + 3;
    const uint16_t *pages = reinterpret_cast<const uint16_t *>(a.pages1);
    uint32_t colmask = 0xFFFFFFFFu;
    uint32_t max_items = a.max_items1;
    uint32_t page0 = 0;
    if (a.levels == 1) {
        hipLaunchKernelGGL(k_wide_plan, dim3(plan_grid(a.n_parts)), dim3(64 * kPlanWaves), 0, st, a.rows1,
                           a.grid1, (const uint2 *)nullptr, 0, a.item_max1, a.items1, a.counters, a.counters + 3,
                           a.max_items1, (uint2 *)nullptr, a.overflow, a.n_parts);
    } else {
        hipLaunchKernelGGL(k_wide_plan, dim3(plan_grid(a.n_parts)), dim3(64 * kPlanWaves), 0, st, a.rows1,
                           a.grid1, (const uint2 *)nullptr, 0, a.item_max1, a.items1, a.counters, a.counters + 3,
                           a.max_items1, a.band_items, a.overflow, a.n_parts);
        if (a.tpb_bits > 8) return hipErrorInvalidValue;
        hipLaunchKernelGGL(k_wide_split, dim3(a.max_items1), dim3(NT), 0, st, a);
        hipLaunchKernelGGL(k_wide_plan, dim3(plan_grid(a.n_tiles)), dim3(64 * kPlanWaves), 0, st, a.rows2, 0,
                           (const uint2 *)a.band_items, a.tpb_bits, a.item_max2, a.items2, a.counters + 1,
                           a.counters + 4, a.max_items2, (uint2 *)nullptr, a.overflow, a.n_tiles);
        rows = a.rows2;
        items = a.items2;
        count = a.counters + 1;
        count1 = a.counters + 4;
        pages = reinterpret_cast<const uint16_t *>(a.pages2);
        colmask = (1u << a.tpb_bits) - 1u;
        max_items = a.max_items2;
        page0 = a.page0_2;
    }
#ifdef LDE_DIAGNOSTICS
    if (a.acc_depth == 8) {  // (diagnostics: eight pages in flight per wave)
        hipExtLaunchKernelGGL(k_wide_accumulate<8>, dim3(max_items), dim3(kWideAccThreads), 0, st, bstart, bstop, 0,
                              items, count, count1, max_items, rows, a.list, a.page_cnt, pages, page0, colmask, a.hist,
                              a.n_bins, a.wzero);
        return hipGetLastError();
    }
#endif
    hipExtLaunchKernelGGL(k_wide_accumulate<kWideAccDepth>, dim3(max_items), dim3(kWideAccThreads), 0, st, bstart,
                          bstop, 0, items, count, count1, max_items, rows, a.list, a.page_cnt, pages, page0, colmask,
                          a.hist, a.n_bins, a.wzero);
    return hipGetLastError();
}

}  // namespace lde
