// lde_sieve.hip -- the event pass of the SPLIT strategy ("sieve") and its
// cold-key path.
//
// Every event of the batch is binned either into a hot screen row
// privatized in LDS or emitted as a cold (screen * T + bin) key, so the
// counts are bit-exact whatever the hot set is (lde_hotset.hip picks it from
// a sample).  The per-event instruction stream is kept short and branch-free:
//
//   * one 32-bit word per pixel, in LDS (direct-mapped table of the sampled
//     hottest pixels) and in HBM (the replica's LUT), with the same payload:
//         bit 31 valid | bit 30 hot | bits 22..29 tag (table only) | bits 0..21 value
//     value = row * T for a hot screen, screen * T for a cold one;
//   * table misses gather the HBM word with a raw buffer load; hits (and
//     out-of-range pixels, clamped to the zero sentinel at index L) load at an
//     out-of-range offset, which returns 0 without a memory request, so
//     word = table_hit_word | gathered_word needs no per-event branch;
//   * one LDS read bins the TOA: bucket word = offset-of-next-edge << 8 | bin,
//     bin = word & 0xFF + (low bits >= word >> 8); a sentinel bucket past the
//     last edge gives bin 256 (dropped);
//   * hot lanes add 1 to their LDS row, the others to a lane-private dummy
//     word; cold keys are compacted per wave in LDS and leave as one 12-byte
//     store (four 24-bit keys) per lane per half chunk (lanes past the count store out of range,
//     which is discarded) -- so every iteration issues the same memory
//     operations and the compiler's in-order vmcnt / lgkmcnt accounting can
//     wait for exactly the operation a value comes from;
//   * each block walks a contiguous chunk range; the {pid, toa} pointers of
//     every chunk come from a small descriptor table (k_chunk_tab) read with a
//     vector load, so the loop has no segment search and no scalar loads.
//
// Deferred chunks (partial tails, segments that are not 16-byte aligned) are
// replaced by an all-invalid dummy chunk in the pipeline and binned afterwards
// by a plain element-wise pass.
//
// Cold path (three launches): k_hot_reduce_scan adds the blocks' hot rows to
// the window and scans the sieve's exact per-(block, wave group, tile) cold
// counts into range offsets; k_cold_sort moves every group's keys into its
// ranges of a tile-major u16 array (one LDS atomic + one u16 store per key);
// k_cold_accumulate histograms each tile's keys in LDS.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "lde_device.h"
#include "lde_internal.h"

namespace lde {

namespace {

constexpr uint32_t kOOB = 0x80000000u;        // buffer offset past every num_records
constexpr uint32_t kOOBi = 0xFFFFFFF0u;       // same, as an inline constant (-16): loads only
constexpr uint32_t kRsrcWord3 = 0x00020000u;  // gfx9 raw buffer: 32-bit data format
constexpr int kEPT = kSplitEPT;               // 8 events per thread per chunk
constexpr uint32_t kSieveStage = 256;         // cold staging words per wave (half a chunk)
constexpr int kSieveKeyed = 262144;           // mode bit: the stream holds finished words
typedef unsigned int v4u __attribute__((ext_vector_type(4)));
typedef unsigned int v3u __attribute__((ext_vector_type(3)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void *p, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), (short)0, (int)bytes,
                                             (int)kRsrcWord3);
}

__device__ __forceinline__ int screen_of_lut(const uint16_t *__restrict__ lut, long long q, int) {
    const unsigned v = lut[q];
    return v == 0xFFFFu ? -1 : (int)v;
}
__device__ __forceinline__ int screen_of_lut(const int *__restrict__ lut, long long q, int T) {
    const int v = lut[q];
    return v < 0 ? -1 : v / T;
}

// v_cndmask on a wave mask: m's lane bit ? t : f.  Written as asm so the
// compiler cannot turn a select between LDS addresses into a branch.
__device__ __forceinline__ uint32_t vsel(unsigned long long m, uint32_t t, uint32_t f) {
    uint32_t r;
    asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(f), "v"(t), "s"(m));
    return r;
}

// LDS word at a byte offset (the sieve keeps its LDS indices pre-scaled)
__device__ __forceinline__ uint32_t &lds_at(uint32_t *sm, uint32_t byte_off) {
    return *reinterpret_cast<uint32_t *>(reinterpret_cast<unsigned char *>(sm) + byte_off);
}

// Four cold keys (scaled by 4; pads all ones) as 24-bit keys in 12 bytes (the
// sieve's S * T <= 2^22): 25 % fewer bytes written by the sieve and read by
// the sort than 32-bit keys.  The pad is 0xFFFFFF.
__device__ __forceinline__ v3u pack_keys24(v4u k4) {
    const uint32_t k0 = (k4[0] >> 2) & 0xFFFFFFu, k1 = (k4[1] >> 2) & 0xFFFFFFu;
    const uint32_t k2 = (k4[2] >> 2) & 0xFFFFFFu, k3 = (k4[3] >> 2) & 0xFFFFFFu;
    return v3u{k0 | (k1 << 24), (k1 >> 8) | (k2 << 16), (k2 >> 16) | (k3 << 8)};
}
// back to scaled keys, the pad to 0xFFFFFFFF
__device__ __forceinline__ void unpack_keys24(v3u w, uint32_t *k) {
    const uint32_t r[4] = {w[0] & 0xFFFFFFu, (w[0] >> 24) | ((w[1] & 0xFFFFu) << 8),
                           (w[1] >> 16) | ((w[2] & 0xFFu) << 16), w[2] >> 8};
#pragma unroll
    for (int q = 0; q < 4; ++q) k[q] = r[q] == 0xFFFFFFu ? 0xFFFFFFFFu : r[q] << 2;
}

}  // namespace

// ---------------------------------------------------------------------------
// tables (rebuilt with the hot set, i.e. every hot_refresh batches)
// ---------------------------------------------------------------------------
template <typename LT>
__global__ __launch_bounds__(256) void k_sieve_glut(const LT *__restrict__ lut, long long L, int T, int W,
                                                    const uint16_t *__restrict__ screen_row,
                                                    uint32_t *__restrict__ glut) {
    const long long q = (long long)blockIdx.x * 256 + threadIdx.x;
    if (q > L) return;
    uint32_t w = 0;  // q == L: the zero sentinel of clamped out-of-range pixels
    if (q < L) {
        const int s = screen_of_lut(lut, q, T);
        if (s >= 0) {
            const uint32_t r1 = screen_row[s];
            w = r1 ? (kSieveValid | kSieveHot | ((r1 - 1u) * (uint32_t)W))
                   : (kSieveValid | ((uint32_t)s * (uint32_t)T));
        }
    }
    glut[q] = w;
}

// slot j of the LDS pixel table: the most-sampled pixel q = j (mod C), with
// the pixel's word (0 for a dropped pixel: valid bit clear) and its tag
__global__ __launch_bounds__(256) void k_sieve_table(const uint32_t *__restrict__ cnt,
                                                     const uint32_t *__restrict__ glut, long long L,
                                                     int cbits, uint32_t *__restrict__ tab,
                                                     uint32_t *__restrict__ stats) {
    const long long C = 1LL << cbits;
    const long long j = (long long)blockIdx.x * 256 + threadIdx.x;
    if (j >= C) return;
    uint32_t best = 0;
    long long bq = -1;
    for (long long q = j; q < L; q += C) {
        const uint32_t c = cnt[q];
        if (c > best) {  // dropped pixels too: their word is 0 (a hit drops the event)
            best = c;
            bq = q;
        }
    }
    tab[j] = bq < 0 ? kSieveEmpty
                    : (glut[bq] | ((uint32_t)(bq >> cbits) << kSieveTagShift));
    if (best) atomicAdd(stats + 3, best);  // sampled events the table catches
}

// chunk c -> its event pointers, or the dummy chunk (deferred / past the end)
__global__ __launch_bounds__(256) void k_chunk_tab(const SegDesc *__restrict__ segs, int n_segs,
                                                   long long n_chunks, const int *dummy,
                                                   ChunkPtrs *__restrict__ tab) {
    const long long c = (long long)blockIdx.x * 256 + threadIdx.x;
    if (c > n_chunks) return;
    ChunkPtrs r{dummy, dummy};
    if (c < n_chunks) {
        int lo = 0, hi = n_segs - 1;
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (segs[mid].chunk0 <= c) lo = mid; else hi = mid - 1;
        }
        const SegDesc sd = segs[lo];
        const long long base = (c - sd.chunk0) * kChunk;
        if (((((uintptr_t)sd.pid | (uintptr_t)sd.toa) & 15u) == 0) && base + kChunk <= sd.n) {
            r.pid = sd.pid + base;
            r.toa = sd.toa + base;
        }
    }
    tab[c] = r;
}

// k_chunk_tab with the descriptors in kernel arguments: every index into the
// argument array is static (unrolled), so the reads stay scalar kernarg loads
__global__ __launch_bounds__(256) void k_chunk_tab_karg(SegKarg sk, int n_segs, long long n_chunks,
                                                        const int *dummy,
                                                        ChunkPtrs *__restrict__ tab,
                                                        SegDesc *__restrict__ segs_out) {
    if (blockIdx.x == 0) {
#pragma unroll
        for (int i = 0; i < kKargSegs; ++i)
            if ((int)threadIdx.x == i && i < n_segs) segs_out[i] = sk.s[i];
    }
    const long long c = (long long)blockIdx.x * 256 + threadIdx.x;
    if (c > n_chunks) return;
    ChunkPtrs r{dummy, dummy};
    if (c < n_chunks) {
        // last segment whose first chunk is <= c (chunk0 ascending)
        SegDesc sd = sk.s[0];
#pragma unroll
        for (int i = 1; i < kKargSegs; ++i)
            if (i < n_segs && sk.s[i].chunk0 <= c) sd = sk.s[i];
        const long long base = (c - sd.chunk0) * kChunk;
        if (((((uintptr_t)sd.pid | (uintptr_t)sd.toa) & 15u) == 0) && base + kChunk <= sd.n) {
            r.pid = sd.pid + base;
            r.toa = sd.toa + base;
        }
    }
    tab[c] = r;
}

// ---------------------------------------------------------------------------
// the event pass
// ---------------------------------------------------------------------------
// ABL: kSieveKeyed (the stream holds finished words, wavelength mode) or, in
// the diagnostics build only, a timing ablation (results wrong by design): 1
// no hot LDS atomics, 2 no gathers, 4 no cold stores, 4096 loads only (the
// stream skeleton), 16384 loads + probes with the binning folded into a
// register (+ the gathers with 32768), 131072 gathers confined to 64 KB.
// GCT: the chunk table comes from global memory (k_chunk_tab), for blocks
// whose chunk range exceeds kSieveLdsChunks.  Otherwise each block builds its
// own in LDS, and GCT is a template switch rather than a runtime branch so
// that the loop has one fetch path: with both, the compiler's wait-count
// insertion merged the paths into a vmcnt(0) at the loop head.
template <int ABL, int GCT>
__global__ __launch_bounds__(kSplitThreads) void k_sieve(SieveArgs a) {
    // static, so LDS addresses need no runtime base (one block per CU anyway)
    __shared__ __attribute__((aligned(16))) uint32_t sm[kSplitSmemMax / 4];
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const uint32_t C = 1u << a.cbits;
    const unsigned long long t_start = a.trace ? __builtin_amdgcn_s_memrealtime() : 0ull;
    // LDS carve (words): hot rows | pixel table | TOA buckets | 64 dummies |
    // cursor (4) | cold staging (256 per wave) | cold keys per tile
    const uint32_t o_pc = (uint32_t)a.hot_words;
    const uint32_t o_tt = o_pc + C;
    const uint32_t o_dum = o_tt + (uint32_t)a.toa_words4;
    const uint32_t o_cur = o_dum + 64u;
    const uint32_t o_stg = o_cur + 4u;
    const uint32_t o_tcnt = o_stg + kSieveStage * (kSplitThreads / 64);
    // block-local chunk table (kSieveLdsChunks entries of {pid, toa}) and the
    // message descriptors it is built from (lds_ctab mode)
    const uint32_t o_ctab = o_tcnt + (uint32_t)(kColdGroups * align4(a.n_tiles));
    const uint32_t o_seg = o_ctab + 4u * kSieveLdsChunks;
    SegDesc *s_seg = reinterpret_cast<SegDesc *>(sm + o_seg);
    for (uint32_t i = (uint32_t)tid * 4u; i < (uint32_t)a.hot_words; i += kSplitThreads * 4u)
        *reinterpret_cast<uint4 *>(sm + i) = make_uint4(0, 0, 0, 0);
    {  // pixel table and TOA buckets (contiguous in LDS): one round of loads
        const uint4 *pt = reinterpret_cast<const uint4 *>(a.pix_tab);
        const uint4 *tt = reinterpret_cast<const uint4 *>(a.ttab);
        const int c4 = (int)(C / 4u);
        lds_fill<4>(reinterpret_cast<uint4 *>(sm + o_pc), c4 + a.toa_words4 / 4,
                    [&](int i) { return g_ld(i < c4 ? pt + i : tt + (i - c4)); });
    }
    if (tid < 64) sm[o_dum + tid] = 0;
    // cursor, hot-count overflow vote
    if (tid == 0) sm[o_cur] = sm[o_cur + 1] = sm[o_cur + 2] = sm[o_cur + 3] = 0;
    for (uint32_t i = (uint32_t)tid; i < kSieveStage * (kSplitThreads / 64); i += kSplitThreads)
        sm[o_stg + i] = 0xFFFFFFFFu;
    for (int i = tid; i < kColdGroups * align4(a.n_tiles); i += kSplitThreads) sm[o_tcnt + i] = 0;
    if (!GCT && a.karg) {  // descriptors from the kernel arguments (static indices)
#pragma unroll
        for (int i = 0; i < kKargSegs; ++i)
            if (tid == i && i < a.n_segs) s_seg[i] = a.sk.s[i];
    }
    __syncthreads();

    const __amdgpu_buffer_rsrc_t glut = make_rsrc(a.glut, (a.L + 1u) * 4u);
    // this block's cold region: cold_cap 24-bit keys (3 bytes each)
    unsigned char *my_cold = reinterpret_cast<unsigned char *>(a.cold) +
                             (size_t)blockIdx.x * (size_t)(a.cold_cap + kSplitThreads / 64) * 3u;
    const __amdgpu_buffer_rsrc_t cold = make_rsrc(my_cold, (uint32_t)a.cold_cap * 3u);
    // one lane's four keys (scaled by 4) as 12 bytes at key index off / 4
    // (kOOB: discarded)
    auto store_keys = [&](v4u kv, uint32_t off) __attribute__((always_inline)) {
        __builtin_amdgcn_raw_buffer_store_b96(pack_keys24(kv), cold,
                                              (int)(off == kOOB ? kOOB : (off >> 2) * 3u), 0, 0);
    };
    const uint32_t cmask = C - 1u;
    const uint32_t pid_off = (uint32_t)a.pid_off;
    const uint32_t Lc = a.L;
    const uint32_t toa_lo = a.toa_lo, toa_cap = a.toa_cap;
    const uint32_t wmask = (1u << a.toa_shift) - 1u;
    const uint32_t T = (uint32_t)a.T;
    const uint32_t dum_idx = o_dum + (uint32_t)lane;
    const uint32_t dum4 = dum_idx * 4u;
    const uint32_t o_stg_w = o_stg + kSieveStage * (uint32_t)(tid >> 6);
    // cold keys are counted per tile for each of the kColdGroups wave groups
    // (one sort block per group)
    const uint32_t grp = (uint32_t)(tid >> 6) / (uint32_t)((kSplitThreads / 64) / kColdGroups);
    const uint32_t o_pc4 = o_pc * 4u, o_tt4 = o_tt * 4u;
    const uint32_t o_tcnt4 = (o_tcnt + grp * (uint32_t)align4(a.n_tiles)) * 4u;
    const int tsh = a.tile_bits + 2;
    // this wave's sub-region of the block's cold region (keys), 16-B aligned
    const uint32_t capw = (uint32_t)(a.cold_cap / (kSplitThreads / 64));
    const uint32_t wave_base = capw * (uint32_t)(tid >> 6);

    // ---- contiguous chunk range of this block
    const long long n = a.n_chunks;
    const long long cb = (long long)blockIdx.x * n / gridDim.x;
    const long long ce = ((long long)blockIdx.x + 1) * n / gridDim.x;
    // chunk descriptor {pid, toa} pointers, fetched by four lanes with a
    // vector load (in-order vmcnt) and read back with readlane; chunks outside
    // [cb, ce) and deferred chunks map to the all-invalid dummy chunk
    const uint32_t *ctab = reinterpret_cast<const uint32_t *>(a.chunk_tab);
    if (!GCT) {
        // entry j = chunk cb + j of this block (entry ce - cb: the dummy chunk);
        // replaces the k_chunk_tab launch in front of the sieve
        const SegDesc *sg = a.karg ? s_seg : a.segs;
        for (long long j = tid; j <= ce - cb; j += kSplitThreads) {
            const long long c = cb + j;
            ChunkPtrs r{a.dummy, a.dummy};
            if (c < ce) {
                int lo = 0, hi = a.n_segs - 1;  // last segment with chunk0 <= c
                while (lo < hi) {
                    const int mid = (lo + hi + 1) >> 1;
                    if (sg[mid].chunk0 <= c) lo = mid; else hi = mid - 1;
                }
                const SegDesc sd = sg[lo];
                const long long base = (c - sd.chunk0) * kChunk;
                if (((((uintptr_t)sd.pid | (uintptr_t)sd.toa) & 15u) == 0) && base + kChunk <= sd.n) {
                    r.pid = sd.pid + base;
                    r.toa = sd.toa + base;
                }
            }
            *reinterpret_cast<ChunkPtrs *>(sm + o_ctab + 4u * (uint32_t)j) = r;
        }
        __syncthreads();
    }
    const unsigned long long t_init = a.trace ? __builtin_amdgcn_s_memrealtime() : 0ull;
    const uint32_t o_ctab4 = o_ctab * 4u;
    auto fetch = [&](long long c) __attribute__((always_inline)) {
        if (!GCT) {
            const uint32_t j = (uint32_t)((c < ce ? c : ce) - cb);
            return lds_at(sm, o_ctab4 + ((j * 4u + (uint32_t)(lane & 3)) << 2));
        }
        const long long ci = c < ce ? c : n;
        return ld_global_u32(ctab + (size_t)ci * 4 + (lane & 3));
    };
    auto ptrs = [&](uint32_t dv, const int *&pp, const int *&tq) __attribute__((always_inline)) {
        const uint32_t w0 = (uint32_t)__builtin_amdgcn_readlane((int)dv, 0);
        const uint32_t w1 = (uint32_t)__builtin_amdgcn_readlane((int)dv, 1);
        const uint32_t w2 = (uint32_t)__builtin_amdgcn_readlane((int)dv, 2);
        const uint32_t w3 = (uint32_t)__builtin_amdgcn_readlane((int)dv, 3);
        pp = reinterpret_cast<const int *>(((unsigned long long)w1 << 32) | w0);
        tq = reinterpret_cast<const int *>(((unsigned long long)w3 << 32) | w2);
    };
    auto load = [&](uint32_t dv, int (&p)[kEPT], int (&t)[kEPT]) __attribute__((always_inline)) {
        const int *pp, *tq;
        ptrs(dv, pp, tq);
#pragma unroll
        for (int j = 0; j < kEPT / 4; ++j) {
            const int off = (j * kSplitThreads + tid) * 4;
            if (ABL & kSieveKeyed) {  // finished words only (k_event_key)
                const v4i tv = ld_stream4(tq + off);
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    p[j * 4 + q] = 0;
                    t[j * 4 + q] = tv[q];
                }
                continue;
            }
            const v4i pv = ld_stream4(pp + off);
            const v4i tv = ld_stream4(tq + off);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                p[j * 4 + q] = pv[q];
                t[j * 4 + q] = tv[q];
            }
        }
    };
    // stage 2a: table probe + TOA bucket, LDS reads only (issued before the
    // previous chunk's LDS atomics, so their latency hides behind its binning)
    auto probe = [&](const int (&p)[kEPT], const int (&t)[kEPT], uint32_t (&w)[kEPT],
                     uint32_t (&qs)[kEPT], uint32_t (&dc)[kEPT], uint32_t (&tw)[kEPT])
                     __attribute__((always_inline)) {
#pragma unroll
        for (int e = 0; e < kEPT; ++e) {
            if (ABL & kSieveKeyed) {  // the word is the event: nothing to look up
                qs[e] = (uint32_t)t[e];
                w[e] = dc[e] = tw[e] = 0u;
                continue;
            }
            const uint32_t q = (uint32_t)p[e] - pid_off;
            qs[e] = q;
            const uint32_t d = min((uint32_t)t[e] - toa_lo, toa_cap);
            dc[e] = d;
            w[e] = lds_at(sm, o_pc4 + ((q & cmask) << 2));
            tw[e] = lds_at(sm, o_tt4 + ((d >> a.toa_shift) << 2));
        }
    };
    // stage 2b: tag check, one gather per event (a table hit or an
    // out-of-range pixel loads out of range: no request, returns 0); w -> the
    // table word of hits (0 otherwise), qs -> the gathered word
    auto finish = [&](uint32_t (&w)[kEPT], uint32_t (&qs)[kEPT]) __attribute__((always_inline)) {
        if (ABL & kSieveKeyed) return;
#pragma unroll
        for (int e = 0; e < kEPT; ++e) {
            const unsigned long long hit =
                __builtin_amdgcn_ballot_w64(((w[e] >> kSieveTagShift) & 0xFFu) == (qs[e] >> a.cbits));
            uint32_t off = vsel(hit, kOOBi, min(qs[e], Lc) << 2);
            if (LDE_DIAG(ABL & 131072)) off = (off & 0x80000000u) | (off & 0xFFFCu);  // gathers in 64 KB
            w[e] = vsel(hit, w[e], 0u);
            qs[e] = LDE_DIAG(ABL & 2) ? (off & 0x3u) : __builtin_amdgcn_raw_buffer_load_b32(glut, (int)off, 0, 0);
        }
    };
    // stage 3: bin, in two halves of four events per lane.  Hot lanes add 1
    // to their LDS row (the others to a lane-private dummy); cold keys are
    // compacted into the wave's 256-word LDS staging area (the others write a
    // dummy) and leave as one 12-byte store per lane into the wave's own
    // sub-region of the block's cold region, at an SGPR cursor (no atomics).
    // The staged words are read back right away but stored one half later,
    // so that read's LDS latency is not waited for.  Staging words are reset
    // to -1, so the <= 3 pad keys of round4(count) are dropped by the sort.
    v4u pend_kv = {0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
    uint32_t pend_off = kOOB;
    uint32_t wcur = 0;  // this wave's cold keys so far (wave-uniform)
    uint32_t junk = 0;  // diagnostic probes: folded words
    auto bin = [&](const uint32_t (&ws)[kEPT], const uint32_t (&g)[kEPT], const uint32_t (&dc)[kEPT],
                   const uint32_t (&tw)[kEPT]) __attribute__((always_inline)) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            uint32_t tot = 0;
#pragma unroll
            for (int e = h * kEPT / 2; e < (h + 1) * kEPT / 2; ++e) {
                const uint32_t v = ws[e] | g[e];
                const uint32_t b = (ABL & kSieveKeyed) ? 0u
                                                        : (tw[e] & 0xFFu) + (((dc[e] & wmask) >= (tw[e] >> 8)) ? 1u : 0u);
                const uint32_t fl = v >> 30;
                // hot rows start at LDS byte 0, so the scaled key is the hot
                // counter's address; cold keys leave scaled by 4 as well
                const uint32_t k4 = ((v & kSieveValueMask) + b) << 2;
                // lane masks straight from the compares (no bool round trip)
                const unsigned long long inb = __builtin_amdgcn_ballot_w64(b < T);
                const unsigned long long bal = inb & __builtin_amdgcn_ballot_w64(fl == 2u);
                const unsigned long long hm = inb & __builtin_amdgcn_ballot_w64(fl == 3u);
                const uint32_t pos4 = (lanes_below(bal) + o_stg_w + tot) << 2;
                tot += (uint32_t)__popcll(bal);
                lds_at(sm, vsel(bal, pos4, dum4)) = k4;
                // hot and cold lanes are disjoint: one LDS atomic adds 1 to the
                // hot counter (hot lanes), the tile's cold-key count (cold
                // lanes) or the lane's dummy word (the rest)
                const uint32_t tidx4 = vsel(bal, ((k4 >> tsh) << 2) + o_tcnt4, dum4);
                const uint32_t aidx4 = LDE_DIAG(ABL & 1) ? tidx4 : vsel(hm, k4, tidx4);
                __hip_atomic_fetch_add(&lds_at(sm, aidx4), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
            const uint32_t res = (tot + 3u) & ~3u;
            // the previous half's keys leave now (their LDS read is long done)
            if (!LDE_DIAG(ABL & 4)) store_keys(pend_kv, pend_off);
            else sm[o_dum + lane] += pend_kv[0] ^ pend_off;
            __builtin_amdgcn_wave_barrier();
            uint4 *slot = reinterpret_cast<uint4 *>(sm + o_stg_w + 4u * (uint32_t)lane);
            const uint4 kv = *slot;
            *slot = make_uint4(0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu);
            __builtin_amdgcn_wave_barrier();
            pend_off = 4u * (uint32_t)lane < res ? (wave_base + wcur + 4u * (uint32_t)lane) << 2 : kOOB;
            pend_kv = v4u{kv.x, kv.y, kv.z, kv.w};
            wcur += res;
        }
    };

    // ---- pipeline (register sets A/B and X/Y alternate): chunk i is binned
    // while chunk i+1 is probed (before) and gathered (after), chunks i+2..3
    // are in flight and chunk i+4..5's descriptors are fetched
    int pA[kEPT], tA[kEPT], pB[kEPT], tB[kEPT];
    uint32_t wsX[kEPT], gX[kEPT], dX[kEPT], twX[kEPT];
    uint32_t wsY[kEPT], gY[kEPT], dY[kEPT], twY[kEPT];
    if (LDE_DIAG(ABL & 16384) && cb < ce) {
        // decomposition probe: the main loop with bin() replaced by folding
        // the chunk's words into junk (+ finish() when ABL & 32768)
        auto eat = [&](const uint32_t (&ws)[kEPT], const uint32_t (&g)[kEPT], const uint32_t (&dc)[kEPT],
                       const uint32_t (&tw)[kEPT]) __attribute__((always_inline)) {
#pragma unroll
            for (int e = 0; e < kEPT; ++e) junk ^= ws[e] ^ g[e] ^ dc[e] ^ tw[e];
        };
        uint32_t dA = fetch(cb), dB = fetch(cb + 1);
        load(dA, pA, tA);
        load(dB, pB, tB);
        dA = fetch(cb + 2);
        dB = fetch(cb + 3);
        probe(pA, tA, wsX, gX, dX, twX);
        if (ABL & 32768) finish(wsX, gX);
        load(dA, pA, tA);
        dA = fetch(cb + 4);
        for (long long c = cb; c < ce; c += 2) {
            probe(pB, tB, wsY, gY, dY, twY);
            eat(wsX, gX, dX, twX);
            if (ABL & 32768) finish(wsY, gY);
            load(dB, pB, tB);
            dB = fetch(c + 5);
            if (c + 1 >= ce) break;
            probe(pA, tA, wsX, gX, dX, twX);
            eat(wsY, gY, dY, twY);
            if (ABL & 32768) finish(wsX, gX);
            load(dA, pA, tA);
            dA = fetch(c + 6);
        }
    } else if (LDE_DIAG(ABL & 4096) && cb < ce) {  // stream skeleton: loads only
        uint32_t dA = fetch(cb), dB = fetch(cb + 1);
        load(dA, pA, tA);
        load(dB, pB, tB);
        dA = fetch(cb + 2);
        dB = fetch(cb + 3);
        for (long long c = cb; c < ce; c += 2) {
#pragma unroll
            for (int e = 0; e < kEPT; ++e) junk ^= (uint32_t)(pA[e] ^ tA[e]);
            load(dA, pA, tA);
            dA = fetch(c + 4);
#pragma unroll
            for (int e = 0; e < kEPT; ++e) junk ^= (uint32_t)(pB[e] ^ tB[e]);
            load(dB, pB, tB);
            dB = fetch(c + 5);
        }
    } else if (cb < ce) {
        uint32_t dA = fetch(cb), dB = fetch(cb + 1);
        load(dA, pA, tA);
        load(dB, pB, tB);
        dA = fetch(cb + 2);
        dB = fetch(cb + 3);
        probe(pA, tA, wsX, gX, dX, twX);
        finish(wsX, gX);
        load(dA, pA, tA);
        dA = fetch(cb + 4);
        for (long long c = cb; c < ce; c += 2) {
            probe(pB, tB, wsY, gY, dY, twY);  // chunk c + 1
            bin(wsX, gX, dX, twX);             // chunk c
            finish(wsY, gY);
            load(dB, pB, tB);  // chunk c + 3
            dB = fetch(c + 5);
            if (c + 1 >= ce) break;
            probe(pA, tA, wsX, gX, dX, twX);  // chunk c + 2
            bin(wsY, gY, dY, twY);             // chunk c + 1
            finish(wsX, gX);
            load(dA, pA, tA);  // chunk c + 4
            dA = fetch(c + 6);
        }
    }

    // ---- deferred chunks: element-wise loads of a clamped index
    if (cb < ce) {
        const SegDesc *segs = (!GCT && a.karg) ? s_seg : a.segs;
        int si = 0;
        {
            int lo = 0, hi = a.n_segs - 1;
            while (lo < hi) {
                const int mid = (lo + hi + 1) >> 1;
                if (segs[mid].chunk0 <= cb) lo = mid; else hi = mid - 1;
            }
            si = lo;
        }
        for (long long c = cb; c < ce; ++c) {
            while (si + 1 < a.n_segs && segs[si + 1].chunk0 <= c) ++si;
            const SegDesc sd = segs[si];
            const long long base = (c - sd.chunk0) * kChunk;
            if (((((uintptr_t)sd.pid | (uintptr_t)sd.toa) & 15u) == 0) && base + kChunk <= sd.n)
                continue;
            int p[kEPT], t[kEPT];
#pragma unroll
            for (int j = 0; j < kEPT / 4; ++j) {
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const long long ei = base + ((long long)j * kSplitThreads + tid) * 4 + q;
                    const bool ok = ei < sd.n;
                    const long long ec = ok ? ei : 0;
                    const int pv = ld_global(sd.pid + ec);
                    const int tv = ld_global(sd.toa + ec);
                    p[j * 4 + q] = ok ? pv : a.pid_off - 1;  // outside the LUT: dropped
                    t[j * 4 + q] = tv;
                }
            }
            probe(p, t, wsX, gX, dX, twX);
            finish(wsX, gX);
            bin(wsX, gX, dX, twX);
        }
    }
    // the last half's keys
    if (!LDE_DIAG(ABL & 4)) store_keys(pend_kv, pend_off);
    if (LDE_DIAG(ABL & (4096 | 16384))) sm[o_dum + lane] = junk;
    if (lane == 0) a.cold_cnt[(size_t)blockIdx.x * (kSplitThreads / 64) + (tid >> 6)] = wcur;
    __syncthreads();
    const unsigned long long t_stream = a.trace ? __builtin_amdgcn_s_memrealtime() : 0ull;
    // hot rows leave as u16 counts (half the bytes written here and read by
    // k_hot_reduce_scan) unless a count of this block exceeds 0xFFFF
    uint32_t *dst = a.hot_part + (size_t)blockIdx.x * a.hot_words;
    uint32_t big = 0;
    for (int i = tid * 4; i < a.hot_words; i += kSplitThreads * 4) {
        const uint4 v = *reinterpret_cast<const uint4 *>(sm + i);
        big |= (v.x | v.y | v.z | v.w) >> 16;
    }
    if (big) sm[o_cur + 1] = 1u;  // benign race: every writer stores 1
    __syncthreads();
    const bool packed = sm[o_cur + 1] == 0u;
    if (packed) {
        uint4 *d16 = reinterpret_cast<uint4 *>(dst);  // 8 counts per 16 bytes
        for (int i = tid * 8; i < a.hot_words; i += kSplitThreads * 8) {
            const uint4 v0 = *reinterpret_cast<const uint4 *>(sm + i);
            const uint4 v1 = *reinterpret_cast<const uint4 *>(sm + i + 4);
            d16[i >> 3] = make_uint4(v0.x | (v0.y << 16), v0.z | (v0.w << 16), v1.x | (v1.y << 16),
                                     v1.z | (v1.w << 16));
        }
    } else {
        for (int i = tid * 4; i < a.hot_words; i += kSplitThreads * 4)
            *reinterpret_cast<uint4 *>(dst + i) = *reinterpret_cast<const uint4 *>(sm + i);
    }
    if (tid == 0) a.hot_fmt[blockIdx.x] = packed ? 1u : 0u;
    if (a.trace) {  // diagnostic: per-block timeline (LDE_SIEVE_TRACE)
        __syncthreads();
        if (tid < 4)
            a.trace[(size_t)blockIdx.x * 4 + tid] =
                tid == 0 ? t_start : tid == 1 ? t_stream : tid == 2 ? __builtin_amdgcn_s_memrealtime() : t_init;
    }
    // tile-major [tile][block][group]: each tile's counts contiguous for
    // k_hot_reduce_scan (a block's eight groups are one 32-byte piece)
    for (int i = tid; i < kColdGroups * a.n_tiles; i += kSplitThreads) {
        const int t = i / kColdGroups, g = i % kColdGroups;
        a.cold_tcnt[((size_t)t * gridDim.x + blockIdx.x) * kColdGroups + g] = sm[o_tcnt + g * align4(a.n_tiles) + t];
    }
    // write this XCD's dirty lines back while other blocks still stream,
    // instead of all at the end-of-kernel release (round 2: -10 to -15 us)
    __syncthreads();
    if (tid == 0) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
}

// ---------------------------------------------------------------------------
// cold keys: exact counting sort into a tile-major u16 array, then pass B
// ---------------------------------------------------------------------------
// One launch, two block roles (saves a dependent launch between the sieve
// and the sort): blocks [0, hot_blocks) add the sieve blocks' private hot rows
// into the window (8 row slices per column of 256 hot bins); the other
// n_tiles blocks scan, per tile, the sieve blocks' cold-key counts into the
// blocks' offsets inside the tile (boff) and the tile totals.
__global__ __launch_bounds__(256) void k_hot_reduce_scan(ColdArgs c, int hot_blocks) {
    __shared__ uint32_t s_w[32];
    if ((int)blockIdx.x < hot_blocks) {
        constexpr int kSlices = 8;
        const int col = blockIdx.x / kSlices, slice = blockIdx.x % kSlices;
        const int i = col * 256 + threadIdx.x;
        if (i >= c.ht) return;
        const int per = (c.rows + kSlices - 1) / kSlices;
        const int j0 = slice * per, j1 = min(c.rows, j0 + per);
        uint32_t sum = 0;
        bool all16 = c.hot_fmt != nullptr;  // block-uniform: every row of the slice packed
        if (all16)
            for (int j = j0; j < j1; ++j) all16 &= c.hot_fmt[j] != 0u;
        if (all16) {
            // the common case: independent u16 loads, eight rows in flight
            const uint16_t *col = reinterpret_cast<const uint16_t *>(c.hot_part) + i;
            const size_t rs = (size_t)c.ht4 * 2;  // row stride in u16
            int j = j0;
            for (; j + 8 <= j1; j += 8) {
                uint32_t v[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) v[u] = col[(size_t)(j + u) * rs];
#pragma unroll
                for (int u = 0; u < 8; ++u) sum += v[u];
            }
            for (; j < j1; ++j) sum += col[(size_t)j * rs];
        } else {
            for (int j = j0; j < j1; ++j) {
                const uint32_t *row = c.hot_part + (size_t)j * c.ht4;
                sum += (c.hot_fmt && c.hot_fmt[j]) ? (uint32_t)reinterpret_cast<const uint16_t *>(row)[i]
                                                   : row[i];
            }
        }
        if (sum) {
            const int row = i / c.T;
            atomicAdd(c.hist + (size_t)c.row_screen[row] * c.T + (i - row * c.T), sum);
        }
        return;
    }
    const int t = blockIdx.x - hot_blocks;
    const int rows = c.rows * kColdGroups;
    // eight rows per thread per round (one sieve block's groups: two 16-byte
    // loads of the tile-major counts), all loads issued before the scan
    constexpr int R = kColdGroups;
    static_assert(R == 8, "one sieve block per thread");
    const uint32_t *col = c.tcnt + (size_t)t * rows;
    uint32_t *ocol = c.boff + (size_t)t * rows;
    uint32_t carry = 0;
    for (int r0 = 0; r0 < rows; r0 += 256 * R) {
        const int rb = r0 + (int)threadIdx.x * R;
        uint32_t v[R], sum = 0;
        if (rb < rows) {
            const uint4 a = *reinterpret_cast<const uint4 *>(col + rb);
            const uint4 b = *reinterpret_cast<const uint4 *>(col + rb + 4);
            v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
            v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
        } else {
#pragma unroll
            for (int u = 0; u < R; ++u) v[u] = 0u;
        }
#pragma unroll
        for (int u = 0; u < R; ++u) {
            v[u] = (v[u] + 7u) & ~7u;  // k_cold_sort: 16-byte aligned (row, tile) ranges
            sum += v[u];
        }
        uint32_t tot;
        uint32_t ex = carry + block_exclusive_scan(sum, s_w, &tot);
#pragma unroll
        for (int u = 0; u < R; ++u) {
            const uint32_t x = ex;
            ex += v[u];
            v[u] = x;
        }
        if (rb < rows) {
            *reinterpret_cast<uint4 *>(ocol + rb) = make_uint4(v[0], v[1], v[2], v[3]);
            *reinterpret_cast<uint4 *>(ocol + rb + 4) = make_uint4(v[4], v[5], v[6], v[7]);
        }
        carry += tot;
        __syncthreads();
    }
    if (threadIdx.x == 0) c.tile_total[t] = carry;
}

constexpr int kSortThreads = kSortThreadsHost;
constexpr int kSortWaves = kSortThreads / 64;
constexpr int kGroupWaves = (kSplitThreads / 64) / kColdGroups;  // sieve waves per group
constexpr int kSortSPW = kSortWaves / kGroupWaves;               // sort waves per sieve wave
static_assert(kSortSPW >= 1 && kSortWaves % kGroupWaves == 0, "sort waves per sieve wave");
constexpr int kSortKPT = 48;    // keys per lane per piece (piece path)
constexpr int kColdDepth = 1;   // direct path: steps of 16 keys per lane per load round
                                // (two rounds in flight; 3: +1.4 us on DREAM)

// Balanced pass-B items (tile, first key, end key, tile has one item) of the
// tile-major key array: a tile with n keys gets ceil(n / item_keys) items.
// Run by sort block 0 (kSortThreads threads) before its pieces; s_ib / s_kb are
// kMaxTiles + 1 words of scratch LDS each.
__device__ void plan_items(const uint32_t *__restrict__ tile_total, int n_tiles,
                           uint32_t item_keys, uint4 *__restrict__ items,
                           uint32_t *__restrict__ item_count, uint32_t max_items, uint32_t *s_w,
                           uint32_t *s_ib, uint32_t *s_kb) {
    constexpr int TPT = kMaxTiles / kSortThreads;
    const int tid = threadIdx.x;
    uint32_t nk[TPT], ni[TPT], ksum = 0, isum = 0;
#pragma unroll
    for (int q = 0; q < TPT; ++q) {
        const int t = tid * TPT + q;
        nk[q] = t < n_tiles ? tile_total[t] : 0u;
        ni[q] = (nk[q] + item_keys - 1) / item_keys;
        ksum += nk[q];
        isum += ni[q];
    }
    uint32_t ktot, itot;
    uint32_t kb = block_exclusive_scan(ksum, s_w, &ktot);
    __syncthreads();
    uint32_t ib = block_exclusive_scan(isum, s_w, &itot);
#pragma unroll
    for (int q = 0; q < TPT; ++q) {
        const int t = tid * TPT + q;
        if (t < n_tiles) {
            s_kb[t] = kb;
            s_ib[t] = ib;
        }
        kb += nk[q];
        ib += ni[q];
    }
    if (tid == 0) {
        s_ib[n_tiles] = itot;
        s_kb[n_tiles] = ktot;
    }
    __syncthreads();
    const uint32_t n_items = itot < max_items ? itot : max_items;
    for (uint32_t i = (uint32_t)tid; i < n_items; i += (uint32_t)kSortThreads) {
        int lo = 0, hi = n_tiles - 1;  // last tile with s_ib[t] <= i
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (s_ib[mid] <= i) lo = mid; else hi = mid - 1;
        }
        const uint32_t j = i - s_ib[lo], nt = s_ib[lo + 1] - s_ib[lo];
        const uint32_t k0 = s_kb[lo], kn = s_kb[lo + 1] - k0;
        const uint32_t b0 = k0 + (uint32_t)((unsigned long long)j * kn / nt);
        const uint32_t b1 = k0 + (uint32_t)((unsigned long long)(j + 1) * kn / nt);
        items[i] = make_uint4((uint32_t)lo, b0, b1, nt == 1u ? 1u : 0u);
    }
    if (tid == 0) *item_count = n_items;
    __syncthreads();
}

// The keys one sort wave reads: part (wv % kSortSPW) of the region of sieve
// wave (grp * kGroupWaves + wv / kSortSPW), split at multiples of 4 keys (one
// 12-byte group)
struct WaveKeys {
    __amdgpu_buffer_rsrc_t rs;
    uint32_t n;
};
__device__ __forceinline__ WaveKeys wave_keys(const ColdArgs &c, int b, int grp, int wv) {
    constexpr int NW = kSplitThreads / 64;
    const int sw = grp * kGroupWaves + wv / kSortSPW, part = wv % kSortSPW;
    const uint32_t n_w = c.cold_cnt[(size_t)b * NW + sw];
    const uint32_t q = (n_w + 4u * kSortSPW - 1u) / (4u * kSortSPW) * 4u;
    const uint32_t lo = min(n_w, (uint32_t)part * q), hi = min(n_w, lo + q);
    const uint32_t capw = (uint32_t)(c.cap / NW);
    const unsigned char *base = reinterpret_cast<const unsigned char *>(c.cold) +
                                ((size_t)b * (size_t)c.stride + (size_t)sw * capw + lo) * 3u;
    return WaveKeys{make_rsrc(base, (hi - lo) * 3u), hi - lo};
}

// The wave's keys in rounds of D steps of 64 x 16 keys (lane: 4 x 4 keys of
// each step as 12-byte groups; past the region: zeros, masked at use)
constexpr uint32_t kSortStep = 64u * 16u;
template <int D>
using SortRound = v3u[D][4];
template <int D>
__device__ __forceinline__ void sort_fetch(const WaveKeys &wk, SortRound<D> &buf, uint32_t r0, int lane) {
#pragma unroll
    for (int d = 0; d < D; ++d)
#pragma unroll
        for (int j = 0; j < 4; ++j)
            buf[d][j] = __builtin_amdgcn_raw_buffer_load_b96(
                wk.rs, (int)((r0 + (uint32_t)d * kSortStep + (uint32_t)j * 256u + (uint32_t)lane * 4u) * 3u), 0,
                0);
}

// Cold-key sort of one (sieve block, wave group) row into its tile ranges of
// the tile-major u16 key array.  The sieve counted the row's keys per tile
// exactly, so its ranges are known before any key is read (range (row, t) at
// tile base + boff, length rounded up to 8 keys, 16-byte aligned).
//
// Direct path (the row's keys fit the LDS image, cap keys): each key takes
// the next slot of its tile's segment with one LDS atomic and lands there as
// u16 (two random LDS operations per key, no count pass, no pieces); the
// image then leaves as whole 16-byte groups, pads (0xFFFF, skipped by pass B)
// pre-filled.  Piece path (a row larger than the image, rare): pieces of
// kSortThreads * kSortKPT keys are counted, scanned and scattered with
// per-wave cursors, carrying partial 8-key groups between pieces.
template <int TB, int D>
__device__ void cold_sort_direct(const ColdArgs &c, uint32_t *sm, int row, uint32_t cap, uint32_t cnt,
                                 uint32_t B, uint32_t tot8, uint32_t gpos, const WaveKeys &wk,
                                 SortRound<D> &bA) {
    constexpr uint32_t MASK = (1u << TB) - 1u;
    constexpr int SH = TB + 2;  // keys are scaled by 4
    const int n_tiles = c.n_tiles;
    const int nt4 = align4(n_tiles);
    const int tid = threadIdx.x, lane = tid & 63;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    // LDS: cursors [tile] + 64 lane dummies | segment base [tile] | global
    // position [tile] | 8-key groups [tile] | image (cap + 64 lane dummies) |
    // group -> tile (u16)
    uint32_t *s_cur = sm;
    uint32_t *s_B = s_cur + nt4 + 64;
    uint32_t *s_pos = s_B + nt4;
    uint32_t *s_ng = s_pos + nt4;
    uint16_t *img = reinterpret_cast<uint16_t *>(s_ng + nt4);
    uint16_t *s_gt = img + cap + 64;
    const bool own = tid < n_tiles;
    if (own) {
        s_cur[tid] = B;
        s_B[tid] = B;
        s_pos[tid] = gpos;
        const uint32_t n8 = (cnt + 7u) & ~7u;
        s_ng[tid] = n8 >> 3;
        for (uint32_t i = B + cnt; i < B + n8; ++i) img[i] = 0xFFFFu;  // the range's pads
    }
    if (tid < 64) s_cur[nt4 + tid] = cap + (uint32_t)tid;  // lane dummies never move far
    __syncthreads();
    if (LDE_DIAG(c.ablate) & 16) return;  // diagnostics: the prologue only
    const uint32_t dcur = (uint32_t)(nt4 + lane);
    // two rounds in flight (D = 3, most of a wave's keys requested at once,
    // measured no better: the sort is bound by its read + write traffic, not
    // latency); the first round was requested before the prologue's scans
    constexpr uint32_t STEP = kSortStep, ROUND = STEP * (uint32_t)D;
    typedef SortRound<D> Round;
    auto fetch = [&](Round &buf, uint32_t r0) __attribute__((always_inline)) { sort_fetch<D>(wk, buf, r0, lane); };
    auto scatter = [&](const Round &buf, uint32_t r0) __attribute__((always_inline)) {
#pragma unroll
        for (int d = 0; d < D; ++d) {
            const uint32_t p0 = r0 + (uint32_t)d * STEP;
            if (p0 >= wk.n) break;  // wave-uniform
            uint32_t key[16];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                uint32_t kk[4];
                unpack_keys24(buf[d][j], kk);
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const uint32_t e = p0 + (uint32_t)j * 256u + (uint32_t)lane * 4u + (uint32_t)q;
                    key[j * 4 + q] = e < wk.n ? kk[q] : 0xFFFFFFFFu;
                }
            }
            if (LDE_DIAG(c.ablate) & 2) {  // diagnostics: loads only, keys folded into one word
                uint32_t x = 0;
#pragma unroll
                for (int e = 0; e < 16; ++e) x ^= key[e];
                if (x == 0x12345678u) img[lane] = (uint16_t)x;
                continue;
            }
            uint32_t slot[16];
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                const bool ok = key[e] != 0xFFFFFFFFu;
                slot[e] = __hip_atomic_fetch_add(s_cur + (ok ? (key[e] >> SH) : dcur), 1u, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_WORKGROUP);
            }
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                const bool ok = key[e] != 0xFFFFFFFFu;
                img[ok ? slot[e] : cap + (uint32_t)lane] = (uint16_t)((key[e] >> 2) & MASK);
            }
        }
    };
    Round bB;
    for (uint32_t r0 = 0; r0 < wk.n; r0 += 2 * ROUND) {
        if (r0 + ROUND < wk.n) fetch(bB, r0 + ROUND);
        scatter(bA, r0);
        if (r0 + ROUND >= wk.n) break;
        if (r0 + 2 * ROUND < wk.n) fetch(bA, r0 + 2 * ROUND);
        scatter(bB, r0 + ROUND);
    }
    // every group's tile, a wave per tile (its lanes over the tile's groups)
    for (int t = wv; t < n_tiles; t += kSortWaves) {
        const uint32_t g0 = s_B[t] >> 3, ng = s_ng[t];
        for (uint32_t j = (uint32_t)lane; j < ng; j += 64u) s_gt[g0 + j] = (uint16_t)t;
    }
    __syncthreads();
    const uint4 *img4 = reinterpret_cast<const uint4 *>(img);
    for (uint32_t gi = (uint32_t)tid; gi < (tot8 >> 3); gi += kSortThreads) {
        const int t = s_gt[gi];
        const uint32_t k = gi - (s_B[t] >> 3);
        if (!(LDE_DIAG(c.ablate) & 1))
            *reinterpret_cast<uint4 *>(c.keys + s_pos[t] + 8u * k) = img4[gi];
    }
}

template <int TB>
__device__ void cold_sort_pieces(const ColdArgs &c, uint32_t *sm, int row, uint32_t gpos, const WaveKeys &wk) {
    constexpr int KPT = kSortKPT;
    constexpr int PIECE = kSortThreads * KPT;
    const int n_tiles = c.n_tiles;
    uint16_t *__restrict__ out = c.keys;
    constexpr uint32_t MASK = (1u << TB) - 1u;
    constexpr int SH = TB + 2;  // keys are scaled by 4
    const int nt4 = align4(n_tiles);
    const int img_words = align4((PIECE + 16 * nt4) / 2);
    uint16_t *img = reinterpret_cast<uint16_t *>(sm);   // tile segments, 16-byte aligned
    uint32_t *s_cnt = sm + img_words;                    // [wave][tile]
    uint32_t *s_pos = s_cnt + kSortWaves * nt4;          // [tile] next global position (8-aligned)
    uint32_t *s_B = s_pos + nt4;                         // [tile] segment base in the image (u16)
    uint32_t *s_full = s_B + nt4;                        // [tile] full groups of this piece
    uint32_t *s_ng = s_full + nt4;                       // [tile] 8-key groups of its segment
    uint4 *s_carry = reinterpret_cast<uint4 *>(s_ng + nt4);  // [tile] 8 carried u16
    uint32_t *s_w = reinterpret_cast<uint32_t *>(s_carry + nt4);
    uint16_t *s_gt = reinterpret_cast<uint16_t *>(s_w + 32);  // [group] its tile
    const int tid = threadIdx.x;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
    const bool own = tid < n_tiles;  // thread tid owns tile tid
    if (own) s_pos[tid] = gpos;
    if (lane == 0) s_w[20 + wv] = (wk.n + 64 * KPT - 1) / (64 * KPT);
    __syncthreads();
    uint32_t npieces = 0;
#pragma unroll
    for (int q = 0; q < kSortWaves; ++q) npieces = max(npieces, s_w[20 + q]);
    __syncthreads();  // s_w is the scan's scratch below
    uint32_t *my_cnt = s_cnt + wv * nt4;
    uint32_t cn = 0;  // own tile: carried keys
    for (uint32_t p = 0; p < npieces; ++p) {
        for (int i = lane; i < nt4; i += 64) my_cnt[i] = 0;
        uint32_t key[KPT];
#pragma unroll
        for (int j = 0; j < KPT / 4; ++j) {
            const uint32_t e0 = p * (uint32_t)(64 * KPT) + (uint32_t)j * 256u + (uint32_t)lane * 4u;
            uint32_t kk[4];
            unpack_keys24(__builtin_amdgcn_raw_buffer_load_b96(wk.rs, (int)(e0 * 3u), 0, 0), kk);
#pragma unroll
            for (int q = 0; q < 4; ++q) key[j * 4 + q] = e0 + (uint32_t)q < wk.n ? kk[q] : 0xFFFFFFFFu;
        }
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int e = 0; e < KPT; ++e)
            if (key[e] != 0xFFFFFFFFu)
                __hip_atomic_fetch_add(my_cnt + (key[e] >> SH), 1u, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_WORKGROUP);
        __syncthreads();
        // own tile: wave counts -> wave offsets inside the run (serial over
        // the waves), run length, segment [carry | run] rounded up to 8
        uint32_t n = 0;
        if (own) {
#pragma unroll
            for (int w = 0; w < kSortWaves; ++w) {
                const uint32_t v = s_cnt[w * nt4 + tid];
                s_cnt[w * nt4 + tid] = n + cn;  // offset inside the segment
                n += v;
            }
            n += cn;
        }
        uint32_t gtotal;
        const uint32_t B = block_exclusive_scan((n + 7u) & ~7u, s_w, &gtotal);
        if (own) {
            s_B[tid] = B;
            s_full[tid] = n >> 3;
            s_ng[tid] = (n + 7u) >> 3;
            if (cn) {  // the carried keys head the segment
                const uint4 cv = s_carry[tid];
                const uint32_t cw[4] = {cv.x, cv.y, cv.z, cv.w};
#pragma unroll
                for (uint32_t i = 0; i < 7; ++i)
                    if (i < cn) img[B + i] = (uint16_t)(cw[i >> 1] >> ((i & 1) * 16));
            }
        }
        __syncthreads();
        // scatter: each key takes the next slot of its wave's part of the run
        // (the order inside a run is irrelevant: pass B only counts)
#pragma unroll
        for (int e = 0; e < KPT; ++e) {
            uint32_t k = key[e];
            asm volatile("" : "+v"(k));  // keeps the count pass's addresses dead
            if (k != 0xFFFFFFFFu) {
                const uint32_t t = k >> SH;
                img[s_B[t] + __hip_atomic_fetch_add(my_cnt + t, 1u, __ATOMIC_RELAXED,
                                                    __HIP_MEMORY_SCOPE_WORKGROUP)] =
                    (uint16_t)((k >> 2) & MASK);
            }
        }
        for (int t = wv; t < n_tiles; t += kSortWaves) {
            const uint32_t g0 = s_B[t] >> 3, ng = s_ng[t];
            for (uint32_t j = (uint32_t)lane; j < ng; j += 64u) s_gt[g0 + j] = (uint16_t)t;
        }
        __syncthreads();
        // one thread per 8-key group: full groups leave as 16-byte stores,
        // a segment's partial last group becomes the tile's new carry
        const uint32_t G = gtotal >> 3;
        for (uint32_t gi = (uint32_t)tid; gi < G; gi += kSortThreads) {
            const uint32_t pos = gi * 8u;
            const int lo = s_gt[gi];
            const uint32_t k = (pos - s_B[lo]) >> 3;
            const uint4 v = *reinterpret_cast<const uint4 *>(img + pos);
            if (k < s_full[lo]) {
                if (!(LDE_DIAG(c.ablate) & 1))
                    *reinterpret_cast<uint4 *>(out + s_pos[lo] + 8u * k) = v;
            } else {
                s_carry[lo] = v;
            }
        }
        __syncthreads();
        if (own) {
            s_pos[tid] += 8u * (n >> 3);
            cn = n & 7u;
        }
        // (the next piece's first barrier orders these before their readers)
    }
    // the last carry of the own tile, padded with 0xFFFF
    if (own && cn) {
        const uint4 cv = s_carry[tid];
        uint32_t cw[4] = {cv.x, cv.y, cv.z, cv.w};
#pragma unroll
        for (uint32_t i = 0; i < 8; ++i)
            if (i >= cn) cw[i >> 1] |= 0xFFFFu << ((i & 1) * 16);
        if (!(LDE_DIAG(c.ablate) & 1))
            *reinterpret_cast<uint4 *>(out + s_pos[tid]) = make_uint4(cw[0], cw[1], cw[2], cw[3]);
    }
}

size_t cold_sort_pieces_smem(int n_tiles) {
    const size_t nt4 = (size_t)align4(n_tiles);
    const size_t img_words = (size_t)align4((int)(((size_t)kSortThreads * kSortKPT + 16 * nt4) / 2));
    const size_t gt_words = ((size_t)kSortThreads * kSortKPT / 8 + nt4 + 1) / 2;
    return 4 * (img_words + (size_t)kSortWaves * nt4 + 5 * nt4 + 4 * nt4 + 32 + gt_words);
}

// keys of the direct path's image in smem bytes of LDS
uint32_t cold_sort_cap(int n_tiles, size_t smem) {
    const long long nt4 = align4(n_tiles);
    const long long words = (long long)(smem / 4) - (4 * nt4 + 64) - 32;  // headers, image dummies
    if (words <= 0) return 0;
    // cap / 2 image words + cap / 16 group-tile words
    return (uint32_t)((words * 16 / 9) & ~63LL);
}

// One block per (sieve block, wave group) row; block 0 also plans pass B's
// items.  cap: the direct path's image size in keys (from the launch's LDS).
template <int TB, int D>
__global__ __launch_bounds__(kSortThreads) void k_cold_sort(ColdArgs c, uint32_t cap) {
    extern __shared__ __attribute__((aligned(16))) uint32_t sm[];
    __shared__ uint32_t s_w[32];
    const int n_tiles = c.n_tiles;
    const int tid = threadIdx.x;
    int row = blockIdx.x;
    if ((c.rows & 7) == 0) {
        // the rows of sieve block b on XCD b % 8, where that block ran and
        // wrote its keys (workgroups go round-robin over the eight XCDs):
        // DREAM -1.5 us
        const int x = blockIdx.x & 7, k = blockIdx.x >> 3;
        row = ((k / kColdGroups) * 8 + x) * kColdGroups + k % kColdGroups;
    }
    if (blockIdx.x == 0)
        plan_items(c.tile_total, n_tiles, c.item_keys, c.items, c.item_count, c.max_items, s_w, sm,
                   sm + kMaxTiles + 1);
    const bool own = tid < n_tiles;
    // the wave's key region and its first round of keys, requested before
    // the scans below (they only feed the direct path's loop: a row taking
    // the piece path reads its keys again)
    const WaveKeys wk = wave_keys(c, row / kColdGroups, row % kColdGroups,
                                  __builtin_amdgcn_readfirstlane(tid >> 6));
    SortRound<D> bA;
    if (wk.n) sort_fetch<D>(wk, bA, 0, tid & 63);
    // own tile: global position of this row's range, the row's exact count
    const uint32_t tt = own ? c.tile_total[tid] : 0u;
    const size_t rows_all = (size_t)c.rows * kColdGroups;
    const uint32_t cnt = own ? c.tcnt[(size_t)tid * rows_all + row] : 0u;
    uint32_t total;
    const uint32_t base = block_exclusive_scan(tt, s_w, &total);
    const uint32_t gpos = own ? base + c.boff[(size_t)tid * rows_all + row] : 0u;
    __syncthreads();
    uint32_t tot8;
    const uint32_t B = block_exclusive_scan((cnt + 7u) & ~7u, s_w, &tot8);
    __syncthreads();
    if (tot8 <= cap)
        cold_sort_direct<TB, D>(c, sm, row, cap, cnt, B, tot8, gpos, wk, bA);
    else
        cold_sort_pieces<TB>(c, sm, row, gpos, wk);
}

// pass B: one item = a contiguous key range of one tile
template <int TB>
__global__ __launch_bounds__(kTileThreads) void k_cold_accumulate(
    const uint16_t *__restrict__ keys, const uint4 *__restrict__ items,
    const uint32_t *__restrict__ item_count, uint32_t *__restrict__ hist, long long n_bins) {
    constexpr int NB = 1 << TB;
    // + 64 lane-private dummy counters: pads and keys outside the item count
    // there, so no lane branches around its LDS atomic
    __shared__ __attribute__((aligned(16))) uint32_t s_tile[NB + 64];
    // the item and the count together (items holds the grid's max_items
    // entries), one round trip before the first key load instead of two
    const uint32_t n_items = *item_count;
    const uint4 it = items[blockIdx.x];
    if (blockIdx.x >= n_items) return;
    for (int i = threadIdx.x * 4; i < NB + 64; i += kTileThreads * 4)
        *reinterpret_cast<uint4 *>(s_tile + i) = make_uint4(0, 0, 0, 0);
    __syncthreads();
    const uint32_t dummy = NB + (threadIdx.x & 63u);
    // 16-byte groups of 8 keys; four per thread per iteration, the next
    // iteration's four issued before this one's atomics (indices clamped so
    // every load is unconditional; keys outside [it.y, it.z) count into the
    // dummy)
    constexpr uint32_t STEP = kTileThreads * 32u;
    const uint32_t k0 = it.y & ~7u;
    const uint32_t last = (it.z - 1u) & ~7u;  // the item's last group (it.z > it.y)
    auto ld = [&](uint32_t i) __attribute__((always_inline)) {
        return *reinterpret_cast<const uint4 *>(keys + (i <= last ? i : last));
    };
    uint4 cur[4], nxt[4];
    uint32_t i0 = k0 + (uint32_t)threadIdx.x * 8u;
#pragma unroll
    for (int u = 0; u < 4; ++u) cur[u] = ld(i0 + (uint32_t)u * kTileThreads * 8u);
    for (; i0 < it.z; i0 += STEP) {
#pragma unroll
        for (int u = 0; u < 4; ++u) nxt[u] = ld(i0 + STEP + (uint32_t)u * kTileThreads * 8u);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const uint32_t i = i0 + (uint32_t)u * kTileThreads * 8u;
            const uint32_t w[4] = {cur[u].x, cur[u].y, cur[u].z, cur[u].w};
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                const uint32_t idx = i + (uint32_t)q;
                const uint32_t key = (w[q >> 1] >> ((q & 1) * 16)) & 0xFFFFu;
                // 0xFFFF: pad of an aligned range (never a key: tile_bits <= 15)
                const bool ok = idx >= it.y && idx < it.z && key != 0xFFFFu;
                __hip_atomic_fetch_add(s_tile + (ok ? key : dummy), 1u, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_WORKGROUP);
            }
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) cur[u] = nxt[u];
    }
    __syncthreads();
    // a tile's only item owns its bins (hot rows are other screens, added by
    // k_hot_reduce before this launch): plain adds; split tiles add atomically
    const long long base = (long long)it.x << TB;
    if (it.w && base + NB <= n_bins) {
        // 16-byte read-modify-write, every load of the thread issued first
        constexpr int V = NB / 4 / kTileThreads;
        uint4 *h4 = reinterpret_cast<uint4 *>(hist + base);
        const uint4 *s4 = reinterpret_cast<const uint4 *>(s_tile);
        uint4 hv[V];
#pragma unroll
        for (int u = 0; u < V; ++u) hv[u] = h4[u * kTileThreads + threadIdx.x];
#pragma unroll
        for (int u = 0; u < V; ++u) {
            const uint4 a = s4[u * kTileThreads + threadIdx.x];
            if (a.x | a.y | a.z | a.w)
                h4[u * kTileThreads + threadIdx.x] =
                    make_uint4(hv[u].x + a.x, hv[u].y + a.y, hv[u].z + a.z, hv[u].w + a.w);
        }
    } else {
        for (int i = threadIdx.x; i < NB; i += kTileThreads) {
            const uint32_t v = s_tile[i];
            if (v != 0u && base + i < n_bins) atomicAdd(hist + base + i, v);
        }
    }
}

// ---------------------------------------------------------------------------
// launch wrappers
// ---------------------------------------------------------------------------
size_t sieve_smem(int hot_words, int cbits, int toa_words4, int n_tiles) {
    return 4 * ((size_t)hot_words + ((size_t)1 << cbits) + (size_t)toa_words4 + 64 + 4 +
                (size_t)kSieveStage * (kSplitThreads / 64) + (size_t)kColdGroups * align4(n_tiles) +
                4 * (size_t)kSieveLdsChunks + sizeof(SegDesc) / 4 * (size_t)kKargSegs);
}

hipError_t launch_sieve_tables(const void *lut, bool lut16, long long L, int T, int W,
                               const uint16_t *screen_row, const uint32_t *pix_cnt, int cbits,
                               uint32_t *glut, uint32_t *tab, uint32_t *stats, hipStream_t st) {
    const unsigned g = (unsigned)((L + 1 + 255) / 256);
    if (lut16)
        hipLaunchKernelGGL(k_sieve_glut<uint16_t>, dim3(g), dim3(256), 0, st,
                           (const uint16_t *)lut, L, T, W, screen_row, glut);
    else
        hipLaunchKernelGGL(k_sieve_glut<int>, dim3(g), dim3(256), 0, st, (const int *)lut, L, T, W,
                           screen_row, glut);
    hipLaunchKernelGGL(k_sieve_table, dim3((unsigned)(((1LL << cbits) + 255) / 256)), dim3(256), 0,
                       st, pix_cnt, glut, L, cbits, tab, stats);
    return hipGetLastError();
}

hipError_t launch_chunk_tab(const SegDesc *segs, int n_segs, long long n_chunks, const int *dummy,
                            ChunkPtrs *tab, hipStream_t st,
                            hipEvent_t start) {
    hipExtLaunchKernelGGL(k_chunk_tab, dim3((unsigned)((n_chunks + 1 + 255) / 256)), dim3(256), 0, st,
                          start, nullptr, 0,
                       segs, n_segs, n_chunks, dummy, tab);
    return hipGetLastError();
}

hipError_t launch_chunk_tab_karg(const SegDesc *host_segs, int n_segs, long long n_chunks,
                                 const int *dummy, ChunkPtrs *tab, SegDesc *segs_out,
                                 hipStream_t st) {
    if (n_segs < 1 || n_segs > kKargSegs) return hipErrorInvalidValue;
    SegKarg sk{};
    for (int i = 0; i < n_segs; ++i) sk.s[i] = host_segs[i];
    hipLaunchKernelGGL(k_chunk_tab_karg, dim3((unsigned)((n_chunks + 1 + 255) / 256)), dim3(256), 0,
                       st, sk, n_segs, n_chunks, dummy, tab, segs_out);
    return hipGetLastError();
}

hipError_t launch_cold_pipeline(const ColdArgs &c, hipStream_t st, hipEvent_t stop) {
    const int hot_blocks = c.hot_part ? ((c.ht + 255) / 256) * 8 : 0;
    if (c.all_hot && hot_blocks > 0) {
        // every screen has a hot row: the sieve wrote no cold key, only the
        // hot rows go into the window
        hipLaunchKernelGGL(k_hot_reduce_scan, dim3(hot_blocks), dim3(256), 0, st, c, hot_blocks);
        if (stop) (void)hipEventRecord(stop, st);
        return hipGetLastError();
    }
    hipLaunchKernelGGL(k_hot_reduce_scan, dim3(hot_blocks + c.n_tiles), dim3(256), 0, st, c,
                       hot_blocks);
    const size_t sma = kColdSortSmem;
    const uint32_t cap = cold_sort_cap(c.n_tiles, sma);
    if (cold_sort_pieces_smem(c.n_tiles) > sma || 4 * (size_t)(2 * (kMaxTiles + 1)) > sma)
        return hipErrorInvalidValue;
    switch (c.tile_bits) {
#define LDE_COLD(TB)                                                                              \
    case TB:                                                                                      \
        (void)hipFuncSetAttribute((const void *)k_cold_sort<TB, kColdDepth>,                      \
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)sma);          \
        hipLaunchKernelGGL((k_cold_sort<TB, kColdDepth>), dim3(c.rows * kColdGroups),             \
                           dim3(kSortThreads), sma, st, c, cap);                                  \
        if (!LDE_DIAG(c.ablate)) /* diagnostics: the keys are not valid */                       \
            hipExtLaunchKernelGGL(k_cold_accumulate<TB>, dim3(c.max_items), dim3(kTileThreads), 0, \
                                  st, nullptr, stop, 0, c.keys, c.items, c.item_count, c.hist,   \
                                  c.n_bins);                                                     \
        else if (stop) /* the binning's end marker is still recorded */                          \
            (void)hipEventRecord(stop, st);                                                      \
        break;
        LDE_COLD(14)
        LDE_COLD(15)
#undef LDE_COLD
    default:
        return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

template <int ABL>
static hipError_t launch_sieve_t(const SieveArgs &a, int grid, hipStream_t st, hipEvent_t start,
                                 hipEvent_t stop) {
    if (sieve_smem(a.hot_words, a.cbits, a.toa_words4, a.n_tiles) > kSplitSmemMax || !a.hot_fmt)
        return hipErrorInvalidValue;
    if (a.lds_ctab)
        hipExtLaunchKernelGGL(k_sieve<ABL, 0>, dim3(grid), dim3(kSplitThreads), 0, st, start, stop, 0,
                              a);  // static LDS
    else
        hipExtLaunchKernelGGL(k_sieve<ABL, 1>, dim3(grid), dim3(kSplitThreads), 0, st, start, stop, 0,
                              a);
    return hipGetLastError();
}

hipError_t launch_sieve(const SieveArgs &a, int grid, hipStream_t st, hipEvent_t start,
                        hipEvent_t stop) {
    const int mode = a.keyed ? kSieveKeyed : LDE_DIAG(a.ablate);
    switch (mode) {
#define LDE_SIEVE_MODE(m) \
    case m: return launch_sieve_t<m>(a, grid, st, start, stop);
    LDE_SIEVE_MODE(0) LDE_SIEVE_MODE(kSieveKeyed)
#ifdef LDE_DIAGNOSTICS
    // timing probes (wrong results), diagnostics build only
    LDE_SIEVE_MODE(1) LDE_SIEVE_MODE(2) LDE_SIEVE_MODE(4) LDE_SIEVE_MODE(6) LDE_SIEVE_MODE(4096)
    LDE_SIEVE_MODE(16384) LDE_SIEVE_MODE(49152) LDE_SIEVE_MODE(131072)
#endif
#undef LDE_SIEVE_MODE
    default: return hipErrorInvalidValue;
    }
}

}  // namespace lde
