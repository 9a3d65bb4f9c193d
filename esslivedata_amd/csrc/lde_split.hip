// lde_split.hip -- SPLIT strategy: hot screen rows privatized in LDS, cold
// remainder through the paged partition in key mode.
//
// Detector event streams are skewed (DREAM: Zipf pixel intensities; the top
// 1 % of pixels carry more than half of the events).
// The screen pixels that receive most events get a full TOA row (T u32
// counters) in every block's LDS, so their events cost one LDS atomic and
// nothing else.  Everything else ("cold") is appended as a 4-byte
// (screen*T + bin) key to a block-private region and binned by the PAGED pass
// A in key mode + the usual page plan and pass B.
//
//   k_sample_screens : per-screen event counts of a few sampled chunks (LDS)
//   k_screen_sum     : column sums of the samples
//   k_select_hot     : top-H screens -> row numbers (single block)
//   k_build_hot_lut  : u32 LUT of one replica: (hot row + 1) << 22 | screen
//   k_split          : the event pass (one read of pid + toa per event)
//   k_hot_reduce     : per-block hot rows summed into the window
//   k_cold_segs      : segment table of the cold regions for pass A (keys)
//
// The hot set is a performance hint only: every event lands in the same bin
// whether its row is hot or cold, so the counts stay bit-exact whatever the
// sample picked.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "lde_device.h"
#include "lde_internal.h"

namespace lde {

namespace {

// Loads one chunk's events.  The vector/element choice is block-uniform (a
// scalar branch), so no divergent control flow sits between these loads and
// their uses.
template <int THREADS, int EPT, bool WITH_TOA>
__device__ __forceinline__ void load_chunk_t(const SegDesc *__restrict__ segs, int n_segs,
                                             long long c, int fill, int (&p)[EPT], int (&t)[EPT]) {
    int lo = 0, hi = n_segs - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (segs[mid].chunk0 <= c) lo = mid; else hi = mid - 1;
    }
    const SegDesc sd = segs[lo];
    const long long base = (c - sd.chunk0) * kChunk;
    const uintptr_t align = WITH_TOA ? ((uintptr_t)sd.pid | (uintptr_t)sd.toa) : (uintptr_t)sd.pid;
    if ((align & 15u) == 0 && base + kChunk <= sd.n) {
#pragma unroll
        for (int j = 0; j < EPT / 4; ++j) {
            const long long e0 = base + ((long long)j * THREADS + threadIdx.x) * 4;
            const v4i pv = ld_stream4(sd.pid + e0);
#pragma unroll
            for (int q = 0; q < 4; ++q) p[j * 4 + q] = pv[q];
            if (WITH_TOA) {
                const v4i tv = ld_stream4(sd.toa + e0);
#pragma unroll
                for (int q = 0; q < 4; ++q) t[j * 4 + q] = tv[q];
            }
        }
    } else {
        // tail chunk or misaligned segment: element loads of a clamped index
#pragma unroll
        for (int j = 0; j < EPT / 4; ++j) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const long long e = base + ((long long)j * THREADS + threadIdx.x) * 4 + q;
                const bool ok = e < sd.n;
                const long long ec = ok ? e : 0;
                const int pv = ld_global(sd.pid + ec);
                p[j * 4 + q] = ok ? pv : fill;
                if (WITH_TOA) {
                    const int tv = ld_global(sd.toa + ec);
                    t[j * 4 + q] = ok ? tv : 0;
                }
            }
        }
    }
}

// branch-free TOA bin (no early return, so no divergent flow around loads)
template <bool FAST>
__device__ __forceinline__ int toa_bin_nb(int t, const unsigned char *s_tab, const ToaParams &tp) {
    if (FAST) {
        const unsigned d = (unsigned)t - (unsigned)tp.lo;
        const bool in = d < tp.span;
        const unsigned dc = in ? d : 0u;
        const uint32_t *rthr = reinterpret_cast<const uint32_t *>(s_tab);
        const uint16_t *bst =
            reinterpret_cast<const uint16_t *>(s_tab + align16((size_t)(tp.T + 1) * 4));
        const int b = bst[dc >> tp.shift];
        const int r = b + (dc >= rthr[b + 1] ? 1 : 0);
        return in ? r : -1;
    }
    return toa_bin<false>(t, s_tab, tp);
}

__device__ __forceinline__ int screen_of(const uint16_t *__restrict__ lut, unsigned p, int) {
    const unsigned v = lut[p];
    return v == 0xFFFFu ? -1 : (int)v;
}
__device__ __forceinline__ int screen_of(const int *__restrict__ lut, unsigned p, int T) {
    const int v = lut[p];
    return v < 0 ? -1 : v / T;
}

}  // namespace

// ---------------------------------------------------------------------------
// hot-set selection
// ---------------------------------------------------------------------------
// Per-pixel sample counts are aggregated in an LDS open-addressing table
// (keys | counts, 2^hbits slots after the S screen counters) and flushed with
// one global atomic per distinct pixel per block: a Zipf-hot pixel then takes
// at most one memory-side atomic per sampled block instead of one per event
// (round 1: 1.14 ms for DREAM, every hot-pixel event serialized on one
// address).  A pixel that finds no slot within kSampleMaxProbe probes falls
// back to its own global atomic, so the counts stay exact.
constexpr int kSampleMaxProbe = 8;
constexpr uint32_t kSampleEmpty = 0xFFFFFFFFu;
template <typename LT>
__global__ __launch_bounds__(kSplitThreads) void k_sample_screens(
    const SegDesc *__restrict__ segs, int n_segs, long long n_chunks, const LT *__restrict__ lut,
    int pid_off, unsigned L, int T, int S, uint32_t *__restrict__ part,
    uint32_t *__restrict__ pix_cnt, int hbits) {
    extern __shared__ __attribute__((aligned(16))) uint32_t s_cnt[];
    const uint32_t H = (pix_cnt && hbits > 0) ? (1u << hbits) : 0u;
    uint32_t *s_key = s_cnt + align4(S);
    uint32_t *s_val = s_key + H;
    for (int i = threadIdx.x; i < S; i += kSplitThreads) s_cnt[i] = 0;
    for (uint32_t i = threadIdx.x; i < H; i += kSplitThreads) {
        s_key[i] = kSampleEmpty;
        s_val[i] = 0;
    }
    __syncthreads();
    const long long c = (long long)blockIdx.x * n_chunks / gridDim.x;
    int p[kSplitEPT], t[kSplitEPT];
    load_chunk_t<kSplitThreads, kSplitEPT, false>(segs, n_segs, c, pid_off - 1, p, t);
#pragma unroll
    for (int e = 0; e < kSplitEPT; ++e) {
        const unsigned q = (unsigned)p[e] - (unsigned)pid_off;
        const int s = q < L ? screen_of(lut, q, T) : -1;
        if (s >= 0) atomicAdd(&s_cnt[s], 1u);
        // pixel counts of every id inside the LUT, dropped pixels included: the
        // SIEVE table then holds frequent dropped pixels too, so their events
        // need no gather (a view that drops most of the detector, e.g.
        // mantle_front_layer, would otherwise gather nearly every event)
        if (q < L && pix_cnt) {
            {
                bool done = false;
                if (H) {
                    uint32_t h = (q * 2654435761u) >> (32 - hbits);
                    for (int k = 0; k < kSampleMaxProbe && !done; ++k) {
                        const uint32_t old = atomicCAS(&s_key[h], kSampleEmpty, q);
                        if (old == kSampleEmpty || old == q) {
                            atomicAdd(&s_val[h], 1u);
                            done = true;
                        }
                        h = (h + 1u) & (H - 1u);
                    }
                }
                if (!done) atomicAdd(pix_cnt + q, 1u);
            }
        }
    }
    __syncthreads();
    uint32_t *dst = part + (size_t)blockIdx.x * S;
    for (int i = threadIdx.x; i < S; i += kSplitThreads) dst[i] = s_cnt[i];
    for (uint32_t i = threadIdx.x; i < H; i += kSplitThreads) {
        const uint32_t k = s_key[i];
        if (k != kSampleEmpty) atomicAdd(pix_cnt + k, s_val[i]);
    }
}

// TOA-bin histogram of the sampled chunks (those of k_sample_screens), for
// the SIEVE hot rows' TOA window: global u32 [T], zeroed before
template <bool FAST>
__global__ __launch_bounds__(kSplitThreads) void k_sample_toa(const SegDesc *__restrict__ segs, int n_segs,
                                                              long long n_chunks, int pid_off,
                                                              const unsigned char *__restrict__ g_tab,
                                                              ToaParams tp, uint32_t *__restrict__ hist) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    uint32_t *s_h = reinterpret_cast<uint32_t *>(smem);
    unsigned char *s_tab = smem + align16((size_t)tp.T * 4);
    for (int i = threadIdx.x; i < tp.T; i += kSplitThreads) s_h[i] = 0;
    load_toa_tables(s_tab, g_tab, tp);
    __syncthreads();
    const long long c = (long long)blockIdx.x * n_chunks / gridDim.x;
    int p[kSplitEPT], t[kSplitEPT];
    load_chunk_t<kSplitThreads, kSplitEPT, true>(segs, n_segs, c, pid_off - 1, p, t);
#pragma unroll
    for (int e = 0; e < kSplitEPT; ++e) {
        const int b = toa_bin_nb<FAST>(t[e], s_tab, tp);
        if (b >= 0 && p[e] != pid_off - 1) atomicAdd(&s_h[b], 1u);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < tp.T; i += kSplitThreads)
        if (s_h[i]) atomicAdd(hist + i, s_h[i]);
}

__global__ __launch_bounds__(256) void k_screen_sum(const uint32_t *__restrict__ part, int rows,
                                                    int S, uint32_t *__restrict__ cnt) {
    const int s = blockIdx.x * 256 + threadIdx.x;
    if (s >= S) return;
    uint32_t v = 0;
    for (int r = 0; r < rows; ++r) v += part[(size_t)r * S + s];
    cnt[s] = v;
}

// Top-H screens by sampled count.  Counts fall into log2 classes; every class
// above the one that overflows H is taken whole, the overflowing class is
// taken in screen order.  stats = {sampled events, events in hot rows, rows}.
__global__ __launch_bounds__(1024) void k_select_hot(const uint32_t *__restrict__ cnt, int S,
                                                     int H, uint16_t *__restrict__ screen_row,
                                                     uint32_t *__restrict__ row_screen,
                                                     uint32_t *__restrict__ stats) {
    __shared__ uint32_t s_cls[33];
    __shared__ uint32_t s_w[32];
    __shared__ uint32_t s_sel[4];
    const int tid = threadIdx.x;
    if (H >= S) {  // a row for every screen, sampled or not: no event is cold
        uint32_t tot = 0;
        for (int s = tid; s < S; s += 1024) {
            tot += cnt[s];
            screen_row[s] = (uint16_t)(s + 1);
            row_screen[s] = (uint32_t)s;
        }
        uint32_t tt;
        (void)block_exclusive_scan(tot, s_w, &tt);
        if (tid == 0) {
            stats[0] = stats[1] = tt;
            stats[2] = (uint32_t)S;
            stats[3] = 0;
        }
        return;
    }
    if (tid < 33) s_cls[tid] = 0;
    __syncthreads();
    const int per = (S + 1023) / 1024;
    const int s0 = min(S, tid * per), s1 = min(S, s0 + per);
    uint32_t tot = 0;
    for (int s = s0; s < s1; ++s) {
        const uint32_t c = cnt[s];
        tot += c;
        if (c) atomicAdd(&s_cls[32 - __clz(c)], 1u);
    }
    __syncthreads();
    if (tid == 0) {
        uint32_t acc = 0;
        int k = 32;
        for (; k >= 1; --k) {
            if (acc + s_cls[k] > (uint32_t)H) break;
            acc += s_cls[k];
        }
        s_sel[0] = (uint32_t)(k < 1 ? 0 : k);  // class taken partially (0: none)
        s_sel[1] = acc;                        // screens taken in full
    }
    __syncthreads();
    const uint32_t kpart = s_sel[0], full = s_sel[1];
    auto cls = [](uint32_t c) { return c ? (uint32_t)(32 - __clz(c)) : 0u; };
    uint32_t n1 = 0, n2 = 0;
    for (int s = s0; s < s1; ++s) {
        const uint32_t k = cls(cnt[s]);
        n1 += (k > kpart && k > 0) ? 1u : 0u;
        n2 += (kpart > 0 && k == kpart) ? 1u : 0u;
    }
    uint32_t t1, t2;
    uint32_t o1 = block_exclusive_scan(n1, s_w, &t1);
    __syncthreads();
    uint32_t o2 = block_exclusive_scan(n2, s_w, &t2);
    const uint32_t room = (uint32_t)H - full;
    uint32_t hot = 0;
    for (int s = s0; s < s1; ++s) {
        const uint32_t c = cnt[s];
        const uint32_t k = cls(c);
        uint32_t row = 0xFFFFFFFFu;
        if (k > kpart && k > 0) {
            row = o1++;
        } else if (kpart > 0 && k == kpart) {
            if (o2 < room) row = full + o2;
            ++o2;
        }
        if (row != 0xFFFFFFFFu) {
            screen_row[s] = (uint16_t)(row + 1);
            row_screen[row] = (uint32_t)s;
            hot += c;
        } else {
            screen_row[s] = 0;
        }
    }
    __syncthreads();
    uint32_t ht;
    (void)block_exclusive_scan(hot, s_w, &ht);
    __syncthreads();
    uint32_t tt;
    (void)block_exclusive_scan(tot, s_w, &tt);
    if (tid == 0) {
        stats[0] = tt;
        stats[1] = ht;
        stats[2] = min(t1 + min(t2, room), (uint32_t)H);
        stats[3] = 0;  // k_build_pix_table: sampled events of the table's pixels
    }
}

template <typename LT>
__global__ __launch_bounds__(256) void k_build_hot_lut(const LT *__restrict__ lut, long long L,
                                                       int T, const uint16_t *__restrict__ screen_row,
                                                       uint32_t *__restrict__ hlut) {
    const long long p = (long long)blockIdx.x * 256 + threadIdx.x;
    if (p >= L) return;
    const int s = screen_of(lut, (unsigned)p, T);
    hlut[p] = s < 0 ? kHotDrop : (((uint32_t)screen_row[s] << kHotRowShift) | (uint32_t)s);
}

// Pixel table image of one replica: slot j holds the most-sampled pixel q with
// q mod C == j (C = 1 << cbits), as
//   tag (q >> cbits) << tag_shift | (row + 1) << screen_bits | screen
// or 0xFFFFFFFF when no sampled pixel maps there.
__global__ __launch_bounds__(256) void k_build_pix_table(const uint32_t *__restrict__ cnt,
                                                         const uint32_t *__restrict__ hlut,
                                                         long long L, int cbits, int screen_bits,
                                                         int tag_shift, uint32_t *__restrict__ tab,
                                                         uint32_t *__restrict__ stats) {
    const long long C = 1LL << cbits;
    const long long j = (long long)blockIdx.x * 256 + threadIdx.x;
    if (j >= C) return;
    uint32_t best = 0;
    long long bq = -1;
    for (long long q = j; q < L; q += C) {
        const uint32_t c = cnt[q];
        if (c > best && hlut[q] != kHotDrop) {
            best = c;
            bq = q;
        }
    }
    uint32_t w = 0xFFFFFFFFu;
    if (bq >= 0) {
        atomicAdd(stats + 3, best);
        const uint32_t v = hlut[bq];
        w = ((uint32_t)(bq >> cbits) << tag_shift) | ((v >> kHotRowShift) << screen_bits) |
            (v & kHotBaseMask);
    }
    tab[j] = w;
}

// ---------------------------------------------------------------------------
// the event pass
// ---------------------------------------------------------------------------
// Pixel table: a direct-mapped LDS table of hot-LUT entries for the pixels
// the hot-set sample saw most (k_build_pix_table), copied into every block's
// LDS at start.  Slot = q mod C, one u32 word:
//   tag (q / C) << (row_bits + screen_bits) | (row + 1) << screen_bits | screen
// (0xFFFFFFFF = empty; a valid word keeps bit 31 clear).  A hit costs one LDS
// read; a miss reads the global hot LUT, so on a skewed stream the L2 gather
// rate (one random request per event, ~2.7e11/s chip-wide) stops bounding the
// pass.
struct PixelCache {
    int cbits;        // log2 C (0: no cache)
    int screen_bits;
    int tag_shift;    // row_bits + screen_bits
};

// The main loop keeps the number of vector-memory instructions per
// iteration fixed (every chunk slot loads, every lookup gathers, every bin
// stores), so the compiler's in-order vmcnt accounting can wait for exactly
// the operation a value comes from instead of draining the queue:
//   * a chunk that is not a full 16-byte-aligned chunk of its segment (or is
//     past the end) loads a 16-byte dummy and is binned afterwards by a plain
//     per-element pass ("deferred");
//   * cache hits and out-of-range pixels gather entry 0 of the hot LUT (one
//     shared line) and discard it;
//   * lanes without a cold key store to a per-wave scratch word.
template <bool FAST, bool CACHE>
__global__ __launch_bounds__(kSplitThreads) void k_split(
    const SegDesc *__restrict__ segs, int n_segs, long long n_chunks,
    const uint32_t *__restrict__ hlut, int pid_off, unsigned L,
    const unsigned char *__restrict__ g_tab, ToaParams tp, int ht4, PixelCache pc,
    uint32_t *__restrict__ hot_part, uint32_t *__restrict__ cold, long long cold_cap,
    uint32_t *__restrict__ cold_cnt, const uint32_t *__restrict__ pix_tab,
    const int *__restrict__ dummy) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    uint32_t *s_hot = reinterpret_cast<uint32_t *>(smem);
    uint32_t *s_pc = s_hot + ht4;
    const int n_pc = CACHE ? (1 << pc.cbits) : 0;
    uint32_t *s_cur = s_pc + n_pc;
    unsigned char *s_tab = reinterpret_cast<unsigned char *>(s_cur + 4);
    const int tid = threadIdx.x;
    for (int i = tid * 4; i < ht4; i += kSplitThreads * 4)
        *reinterpret_cast<uint4 *>(s_hot + i) = make_uint4(0, 0, 0, 0);
    if (CACHE)
        for (int i = tid * 4; i < n_pc; i += kSplitThreads * 4)
            *reinterpret_cast<uint4 *>(s_pc + i) = *reinterpret_cast<const uint4 *>(pix_tab + i);
    if (tid == 0) s_cur[0] = 0;
    load_toa_tables(s_tab, g_tab, tp);
    __syncthreads();
    // cold region of this block: cold_cap keys, then one scratch word per wave
    uint32_t *my_cold = cold + (size_t)blockIdx.x * (size_t)(cold_cap + kSplitThreads / 64);
    uint32_t *my_dump = my_cold + cold_cap + (tid >> 6);
    const int T = tp.T;
    const uint32_t cmask = (uint32_t)n_pc - 1u;
    const uint32_t smask = (1u << pc.screen_bits) - 1u;
    const uint32_t rmask = (1u << (pc.tag_shift - pc.screen_bits)) - 1u;

    // chunk c -> base pointers of its events (block-uniform); !clean -> dummy
    auto locate = [&](long long c, const int *&pp, const int *&tq) __attribute__((always_inline)) {
        bool clean = false;
        pp = dummy;
        tq = dummy;
        if (c < n_chunks) {
            int lo = 0, hi = n_segs - 1;
            while (lo < hi) {
                const int mid = (lo + hi + 1) >> 1;
                if (segs[mid].chunk0 <= c) lo = mid; else hi = mid - 1;
            }
            const SegDesc sd = segs[lo];
            const long long base = (c - sd.chunk0) * kChunk;
            clean = ((((uintptr_t)sd.pid | (uintptr_t)sd.toa) & 15u) == 0) && base + kChunk <= sd.n;
            if (clean) {
                pp = sd.pid + base;
                tq = sd.toa + base;
            }
        }
        return clean;
    };
    auto load = [&](const int *pp, const int *tq, bool clean, int (&p)[kSplitEPT],
                    int (&t)[kSplitEPT]) __attribute__((always_inline)) {
#pragma unroll
        for (int j = 0; j < kSplitEPT / 4; ++j) {
            const int off = clean ? (j * kSplitThreads + tid) * 4 : 0;
            const v4i pv = ld_stream4(pp + off);
            const v4i tv = ld_stream4(tq + off);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                p[j * 4 + q] = pv[q];
                t[j * 4 + q] = tv[q];
            }
        }
    };

    uint32_t v[kSplitEPT], qq[kSplitEPT];
    int b[kSplitEPT];
    // stage 2: TOA bins and table probes (LDS), then one gather per event (a
    // miss reads its pixel, everything else entry 0)
    auto lookup = [&](const int (&p)[kSplitEPT], const int (&t)[kSplitEPT])
                      __attribute__((always_inline)) {
        uint32_t w[kSplitEPT];
#pragma unroll
        for (int e = 0; e < kSplitEPT; ++e) {
            const unsigned q = (unsigned)p[e] - (unsigned)pid_off;
            qq[e] = q;
            b[e] = toa_bin_nb<FAST>(t[e], s_tab, tp);
            if (CACHE) w[e] = s_pc[q & cmask];
        }
#pragma unroll
        for (int e = 0; e < kSplitEPT; ++e) {
            const unsigned q = qq[e];
            const bool inr = q < L;
            bool hit = false;
            uint32_t dec = kHotDrop;
            if (CACHE) {
                hit = inr && w[e] != 0xFFFFFFFFu && (w[e] >> pc.tag_shift) == (q >> pc.cbits);
                dec = (((w[e] >> pc.screen_bits) & rmask) << kHotRowShift) | (w[e] & smask);
            }
            const bool need = inr && !hit;
            const uint32_t g = hlut[need ? q : 0u];
            v[e] = need ? g : (hit ? dec : kHotDrop);
        }
    };
    // stage 3: bin the looked-up chunk (hot rows in LDS, cold keys out); a
    // chunk that is not live bins nothing but issues the same stores
    auto bin = [&](bool live) __attribute__((always_inline)) {
        uint32_t key[kSplitEPT];
        unsigned long long bal[kSplitEPT];
        uint32_t pre[kSplitEPT];
        bool cold_e[kSplitEPT];
        uint32_t tot = 0;
#pragma unroll
        for (int e = 0; e < kSplitEPT; ++e) {
            const bool ok = live && v[e] != kHotDrop && b[e] >= 0;
            const uint32_t row = v[e] >> kHotRowShift;
            key[e] = (v[e] & kHotBaseMask) * (uint32_t)T + (uint32_t)b[e];
            if (ok && row != 0u) atomicAdd(&s_hot[(row - 1u) * (uint32_t)T + (uint32_t)b[e]], 1u);
            cold_e[e] = ok && row == 0u;
            bal[e] = __ballot(cold_e[e]);
            pre[e] = tot;
            tot += (uint32_t)__popcll(bal[e]);
        }
        uint32_t wbase = 0;
        if ((tid & 63) == 0) wbase = atomicAdd(s_cur, tot);
        wbase = (uint32_t)__builtin_amdgcn_readfirstlane(wbase);
#pragma unroll
        for (int e = 0; e < kSplitEPT; ++e) {
            uint32_t *dst = cold_e[e] ? my_cold + (wbase + pre[e] + lanes_below(bal[e])) : my_dump;
            *dst = key[e];
        }
    };

    // Pipeline over this block's chunks c0, c0 + G, ...: chunk i is binned
    // while chunk i+1 is looked up and chunks i+2, i+3 stream in (register
    // sets A and B alternate).
    int pA[kSplitEPT], tA[kSplitEPT], pB[kSplitEPT], tB[kSplitEPT];
    const long long G = gridDim.x;
    const long long c0 = blockIdx.x;
    const int *ppA, *tqA, *ppB, *tqB;
    bool clA, clB, clV;
    if (c0 < n_chunks) {
        clA = locate(c0, ppA, tqA);
        load(ppA, tqA, clA, pA, tA);
        clB = locate(c0 + G, ppB, tqB);
        load(ppB, tqB, clB, pB, tB);
        lookup(pA, tA);
        clV = clA;
        clA = locate(c0 + 2 * G, ppA, tqA);
        load(ppA, tqA, clA, pA, tA);
        for (long long c = c0; c < n_chunks; c += 2 * G) {
            bin(clV);  // chunk c
            lookup(pB, tB);
            clV = clB;
            clB = locate(c + 3 * G, ppB, tqB);
            load(ppB, tqB, clB, pB, tB);
            if (c + G >= n_chunks) break;
            bin(clV);  // chunk c + G
            lookup(pA, tA);
            clV = clA;
            clA = locate(c + 4 * G, ppA, tqA);
            load(ppA, tqA, clA, pA, tA);
        }
    }
    // deferred chunks (tails, misaligned segments): plain per-element pass
    for (long long c = c0; c < n_chunks; c += G) {
        const int *pp, *tq;
        if (locate(c, pp, tq)) continue;
        int p[kSplitEPT], t[kSplitEPT];
        load_chunk_t<kSplitThreads, kSplitEPT, true>(segs, n_segs, c, pid_off - 1, p, t);
        lookup(p, t);
        bin(true);
    }
    __syncthreads();
    uint32_t *dst = hot_part + (size_t)blockIdx.x * ht4;
    for (int i = tid * 4; i < ht4; i += kSplitThreads * 4)
        *reinterpret_cast<uint4 *>(dst + i) = *reinterpret_cast<const uint4 *>(s_hot + i);
    if (tid == 0) cold_cnt[blockIdx.x] = s_cur[0];
}

// window[row_screen[row] * T + b] += sum over blocks of hot_part[.][row * T + b]
__global__ __launch_bounds__(256) void k_hot_reduce(const uint32_t *__restrict__ hot_part,
                                                    int rows, int ht, int ht4, int T,
                                                    int rows_per_slice,
                                                    const uint32_t *__restrict__ row_screen,
                                                    uint32_t *__restrict__ win) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= ht) return;
    const int j0 = blockIdx.y * rows_per_slice;
    const int j1 = min(rows, j0 + rows_per_slice);
    uint32_t sum = 0;
    for (int j = j0; j < j1; ++j) sum += hot_part[(size_t)j * ht4 + i];
    if (sum) {
        const int row = i / T;
        atomicAdd(win + (size_t)row_screen[row] * T + (i - row * T), sum);
    }
}

// segment table of the cold regions (one per split block) for pass A in key mode
__global__ __launch_bounds__(1024) void k_cold_segs(const uint32_t *__restrict__ cold_cnt, int rows,
                                                    const uint32_t *__restrict__ cold,
                                                    long long cold_cap, SegDesc *__restrict__ segs,
                                                    long long *__restrict__ n_chunks) {
    __shared__ uint32_t s_w[32];
    uint32_t carry = 0;
    for (int r0 = 0; r0 < rows; r0 += 1024) {
        const int r = r0 + threadIdx.x;
        const uint32_t n = r < rows ? cold_cnt[r] : 0u;
        const uint32_t ch = (n + kChunk - 1) / kChunk;
        uint32_t tot;
        const uint32_t ex = block_exclusive_scan(ch, s_w, &tot);
        if (r < rows) {
            SegDesc d;
            d.pid = reinterpret_cast<const int *>(cold + (size_t)r * (size_t)(cold_cap + kSplitThreads / 64));
            d.toa = nullptr;
            d.n = n;
            d.chunk0 = carry + ex;
            segs[r] = d;
        }
        carry += tot;
        __syncthreads();
    }
    if (threadIdx.x == 0) *n_chunks = carry;
}

// ---------------------------------------------------------------------------
// launch wrappers
// ---------------------------------------------------------------------------
size_t split_smem(int ht4, int cache_words, const ToaParams &tp) {
    return (size_t)ht4 * 4 + (size_t)cache_words * 4 + 16 + toa_lds_bytes(tp);
}

// Hot-set selection in two steps, so the host can size the rows from the
// sample in between: launch_hot_sample (per-screen and per-pixel counts of the
// sampled chunks; with toa_hist, also their TOA-bin histogram), then
// launch_hot_pick (top a.rows screens, hot LUT, pixel table).
hipError_t launch_hot_sample(const SplitArgs &a, int replica, uint32_t *toa_hist, hipStream_t st) {
    if (a.cache_bits > 0) {
        const hipError_t e = hipMemsetAsync(a.pix_cnt, 0, (size_t)a.L * 4, st);
        if (e != hipSuccess) return e;
    }
    // LDS: S screen counters + the pixel table (keys | counts), up to 2^13 slots
    int hbits = 0;
    if (a.cache_bits > 0) {
        hbits = 13;
        while (hbits > 6 && ((size_t)align4(a.S) + (2u << hbits)) * 4 > kSplitSmemMax) --hbits;
        if (((size_t)align4(a.S) + (2u << hbits)) * 4 > kSplitSmemMax) hbits = 0;
    }
    const size_t sm = ((size_t)align4(a.S) + (hbits ? (2u << hbits) : 0u)) * 4;
    // no room for the table (hbits 0): plain global atomics
    uint32_t *pix_cnt = a.cache_bits > 0 ? a.pix_cnt : nullptr;
    const void *lut_r = a.lut16 ? (const void *)((const uint16_t *)a.lut + (size_t)replica * a.L)
                                : (const void *)((const int *)a.lut + (size_t)replica * a.L);
    if (a.lut16) {
        (void)hipFuncSetAttribute((const void *)k_sample_screens<uint16_t>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)sm);
        hipLaunchKernelGGL(k_sample_screens<uint16_t>, dim3(a.sample_blocks), dim3(kSplitThreads), sm,
                           st, a.segs, a.n_segs, a.n_chunks, (const uint16_t *)lut_r, a.pid_off,
                           (unsigned)a.L, a.tp.T, a.S, a.sample_part, pix_cnt, hbits);
    } else {
        (void)hipFuncSetAttribute((const void *)k_sample_screens<int>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)sm);
        hipLaunchKernelGGL(k_sample_screens<int>, dim3(a.sample_blocks), dim3(kSplitThreads), sm, st,
                           a.segs, a.n_segs, a.n_chunks, (const int *)lut_r, a.pid_off,
                           (unsigned)a.L, a.tp.T, a.S, a.sample_part, pix_cnt, hbits);
    }
    hipLaunchKernelGGL(k_screen_sum, dim3((a.S + 255) / 256), dim3(256), 0, st, a.sample_part,
                       a.sample_blocks, a.S, a.screen_cnt);
    if (toa_hist) {
        hipError_t e = hipMemsetAsync(toa_hist, 0, (size_t)a.tp.T * 4, st);
        if (e != hipSuccess) return e;
        const size_t smt = align16((size_t)a.tp.T * 4) + toa_lds_bytes(a.tp);
        if (a.tp.fast) {
            (void)hipFuncSetAttribute((const void *)k_sample_toa<true>,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)smt);
            hipLaunchKernelGGL(k_sample_toa<true>, dim3(a.sample_blocks), dim3(kSplitThreads), smt, st,
                               a.segs, a.n_segs, a.n_chunks, a.pid_off, a.tab, a.tp, toa_hist);
        } else {
            (void)hipFuncSetAttribute((const void *)k_sample_toa<false>,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)smt);
            hipLaunchKernelGGL(k_sample_toa<false>, dim3(a.sample_blocks), dim3(kSplitThreads), smt, st,
                               a.segs, a.n_segs, a.n_chunks, a.pid_off, a.tab, a.tp, toa_hist);
        }
    }
    return hipGetLastError();
}

hipError_t launch_hot_pick(const SplitArgs &a, int replica, hipStream_t st) {
    const void *lut_r = a.lut16 ? (const void *)((const uint16_t *)a.lut + (size_t)replica * a.L)
                                : (const void *)((const int *)a.lut + (size_t)replica * a.L);
    hipLaunchKernelGGL(k_select_hot, dim3(1), dim3(1024), 0, st, a.screen_cnt, a.S, a.rows,
                       a.screen_row, a.row_screen, a.stats);
    const unsigned g = (unsigned)((a.L + 255) / 256);
    if (a.lut16)
        hipLaunchKernelGGL(k_build_hot_lut<uint16_t>, dim3(g), dim3(256), 0, st,
                           (const uint16_t *)lut_r, a.L, a.tp.T, a.screen_row, a.hlut);
    else
        hipLaunchKernelGGL(k_build_hot_lut<int>, dim3(g), dim3(256), 0, st, (const int *)lut_r, a.L,
                           a.tp.T, a.screen_row, a.hlut);
    if (a.cache_bits > 0)
        hipLaunchKernelGGL(k_build_pix_table, dim3((unsigned)(((1LL << a.cache_bits) + 255) / 256)),
                           dim3(256), 0, st, a.pix_cnt, a.hlut, a.L, a.cache_bits, a.screen_bits,
                           a.screen_bits + a.row_bits, a.pix_tab, a.stats);
    return hipGetLastError();
}

template <bool FAST, bool CACHE>
static hipError_t launch_split_t(const SplitArgs &a, hipStream_t st) {
    const int ht4 = align4(a.rows * a.tp.T);
    PixelCache pc;
    pc.cbits = a.cache_bits;
    pc.screen_bits = a.screen_bits;
    pc.tag_shift = a.screen_bits + a.row_bits;
    const size_t sm = split_smem(ht4, CACHE ? (1 << a.cache_bits) : 0, a.tp);
    (void)hipFuncSetAttribute((const void *)k_split<FAST, CACHE>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)sm);
    hipLaunchKernelGGL((k_split<FAST, CACHE>), dim3(a.grid), dim3(kSplitThreads), sm, st, a.segs,
                       a.n_segs, a.n_chunks, a.hlut, a.pid_off, (unsigned)a.L, a.tab, a.tp, ht4, pc,
                       a.hot_part, a.cold, a.cold_cap, a.cold_cnt, a.pix_tab, a.dummy);
    return hipGetLastError();
}

hipError_t launch_split(const SplitArgs &a, hipStream_t st) {
    if (a.tp.fast)
        return a.cache_bits > 0 ? launch_split_t<true, true>(a, st) : launch_split_t<true, false>(a, st);
    return a.cache_bits > 0 ? launch_split_t<false, true>(a, st) : launch_split_t<false, false>(a, st);
}

hipError_t launch_hot_reduce(const SplitArgs &a, uint32_t *win, hipStream_t st) {
    const int ht = a.rows * a.tp.T;
    const int ht4 = align4(ht);
    const int slices = 8;
    const int per = (a.grid + slices - 1) / slices;
    hipLaunchKernelGGL(k_hot_reduce, dim3((ht + 255) / 256, slices), dim3(256), 0, st, a.hot_part,
                       a.grid, ht, ht4, a.tp.T, per, a.row_screen, win);
    return hipGetLastError();
}

hipError_t launch_split_tail(const SplitArgs &a, uint32_t *win, SegDesc *cold_segs,
                             long long *n_cold_chunks, hipStream_t st) {
    const int ht = a.rows * a.tp.T;
    const int ht4 = align4(ht);
    const int slices = 8;
    const int per = (a.grid + slices - 1) / slices;
    hipLaunchKernelGGL(k_hot_reduce, dim3((ht + 255) / 256, slices), dim3(256), 0, st, a.hot_part,
                       a.grid, ht, ht4, a.tp.T, per, a.row_screen, win);
    hipLaunchKernelGGL(k_cold_segs, dim3(1), dim3(1024), 0, st, a.cold_cnt, a.grid, a.cold,
                       a.cold_cap, cold_segs, n_cold_chunks);
    return hipGetLastError();
}

}  // namespace lde
