// lde_sieve.hip -- lean event pass of the SPLIT strategy ("sieve").
//
// Same contract as k_split (lde_split.hip): every event of the batch is
// binned either into a hot screen row privatized in LDS or emitted as a cold
// (screen * T + bin) key for the paged pass, so the counts are bit-exact
// whatever the hot set is.  What changes is the per-event instruction stream,
// which in k_split was ~66 VALU operations per event with a vmcnt(0) drain per
// chunk (rocprofv3 SQ_INSTS_VALU, round 1):
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
//     word; cold keys are compacted per wave in LDS and leave as one 16-byte
//     store per lane per half chunk (lanes past the count store out of range,
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
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "lde_device.h"
#include "lde_internal.h"

namespace lde {

namespace {

constexpr uint32_t kOOB = 0x80000000u;        // buffer offset past every num_records
constexpr uint32_t kOOBi = 0xFFFFFFF0u;       // same, as an inline constant (-16): loads only
constexpr uint32_t kRsrcWord3 = 0x00020000u;  // gfx9 raw buffer: 32-bit data format
constexpr int kEPT = kSplitEPT;               // 8 events per thread per chunk
constexpr uint32_t kSieveStage = 256;         // cold staging words per wave (half a chunk)
typedef unsigned int v4u __attribute__((ext_vector_type(4)));

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

}  // namespace

// ---------------------------------------------------------------------------
// tables (rebuilt with the hot set, i.e. every hot_refresh batches)
// ---------------------------------------------------------------------------
template <typename LT>
__global__ __launch_bounds__(256) void k_sieve_glut(const LT *__restrict__ lut, long long L, int T,
                                                    const uint16_t *__restrict__ screen_row,
                                                    uint32_t *__restrict__ glut) {
    const long long q = (long long)blockIdx.x * 256 + threadIdx.x;
    if (q > L) return;
    uint32_t w = 0;  // q == L: the zero sentinel of clamped out-of-range pixels
    if (q < L) {
        const int s = screen_of_lut(lut, q, T);
        if (s >= 0) {
            const uint32_t r1 = screen_row[s];
            w = r1 ? (kSieveValid | kSieveHot | ((r1 - 1u) * (uint32_t)T))
                   : (kSieveValid | ((uint32_t)s * (uint32_t)T));
        }
    }
    glut[q] = w;
}

// slot j of the LDS pixel table: the most-sampled valid pixel q = j (mod C)
__global__ __launch_bounds__(256) void k_sieve_table(const uint32_t *__restrict__ cnt,
                                                     const uint32_t *__restrict__ glut, long long L,
                                                     int cbits, uint32_t *__restrict__ tab) {
    const long long C = 1LL << cbits;
    const long long j = (long long)blockIdx.x * 256 + threadIdx.x;
    if (j >= C) return;
    uint32_t best = 0;
    long long bq = -1;
    for (long long q = j; q < L; q += C) {
        const uint32_t c = cnt[q];
        if (c > best && glut[q] != 0u) {
            best = c;
            bq = q;
        }
    }
    tab[j] = bq < 0 ? kSieveEmpty
                    : (glut[bq] | ((uint32_t)(bq >> cbits) << kSieveTagShift));
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
// ABL (benchmark ablations only, results are wrong when nonzero): 1 no hot
// LDS atomics, 2 no gathers, 4 no cold stores, 8 no LDS probes, 16 every
// gather lane out of range, 32 every gather lane on the first two words
template <int ABL>
__global__ __launch_bounds__(kSplitThreads) void k_sieve(SieveArgs a) {
    // static, so LDS addresses need no runtime base (one block per CU anyway)
    __shared__ __attribute__((aligned(16))) uint32_t sm[kSplitSmemMax / 4];
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const uint32_t C = 1u << a.cbits;
    // LDS carve (words): hot rows | pixel table | TOA buckets | 64 dummies |
    // cursor (4) | cold staging (256 per wave) | cold keys per tile
    const uint32_t o_pc = (uint32_t)a.hot_words;
    const uint32_t o_tt = o_pc + C;
    const uint32_t o_dum = o_tt + (uint32_t)a.toa_words4;
    const uint32_t o_cur = o_dum + 64u;
    const uint32_t o_stg = o_cur + 4u;
    const uint32_t o_tcnt = o_stg + kSieveStage * (kSplitThreads / 64);
    for (uint32_t i = (uint32_t)tid * 4u; i < (uint32_t)a.hot_words; i += kSplitThreads * 4u)
        *reinterpret_cast<uint4 *>(sm + i) = make_uint4(0, 0, 0, 0);
    for (uint32_t i = (uint32_t)tid * 4u; i < C; i += kSplitThreads * 4u)
        *reinterpret_cast<uint4 *>(sm + o_pc + i) = *reinterpret_cast<const uint4 *>(a.pix_tab + i);
    for (uint32_t i = (uint32_t)tid * 4u; i < (uint32_t)a.toa_words4; i += kSplitThreads * 4u)
        *reinterpret_cast<uint4 *>(sm + o_tt + i) = *reinterpret_cast<const uint4 *>(a.ttab + i);
    if (tid < 64) sm[o_dum + tid] = 0;
    if (tid == 0) sm[o_cur] = 0;
    for (uint32_t i = (uint32_t)tid; i < kSieveStage * (kSplitThreads / 64); i += kSplitThreads)
        sm[o_stg + i] = 0xFFFFFFFFu;
    for (int i = tid; i < a.n_tiles * a.tgroups; i += kSplitThreads) sm[o_tcnt + i] = 0;
    __syncthreads();

    const __amdgpu_buffer_rsrc_t glut = make_rsrc(a.glut, (a.L + 1u) * 4u);
    uint32_t *my_cold = a.cold + (size_t)blockIdx.x * (size_t)(a.cold_cap + kSplitThreads / 64);
    const __amdgpu_buffer_rsrc_t cold = make_rsrc(my_cold, (uint32_t)a.cold_cap * 4u);  // 16-B aligned
    const uint32_t cmask = C - 1u;
    const uint32_t pid_off = (uint32_t)a.pid_off;
    const uint32_t Lc = a.L;
    const uint32_t toa_lo = a.toa_lo, toa_cap = a.toa_cap;
    const uint32_t wmask = (1u << a.toa_shift) - 1u;
    const uint32_t T = (uint32_t)a.T;
    const uint32_t dum_idx = o_dum + (uint32_t)lane;
    const uint32_t dum4 = dum_idx * 4u;
    const uint32_t o_stg_w = o_stg + kSieveStage * (uint32_t)(tid >> 6);
    // cold keys are counted per tile for each group of 16 / tgroups waves
    const uint32_t grp = (uint32_t)(tid >> 6) / (uint32_t)((kSplitThreads / 64) / a.tgroups);
    const uint32_t o_pc4 = o_pc * 4u, o_tt4 = o_tt * 4u;
    const uint32_t o_tcnt4 = (o_tcnt + grp * (uint32_t)a.n_tiles) * 4u;
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
    auto fetch = [&](long long c) __attribute__((always_inline)) {
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
            const uint32_t q = (uint32_t)p[e] - pid_off;
            qs[e] = q;
            const uint32_t d = min((uint32_t)t[e] - toa_lo, toa_cap);
            dc[e] = d;
            if (ABL & 8) {
                w[e] = q ^ d;
                tw[e] = d & 0xFFFu;
            } else {
                w[e] = lds_at(sm, o_pc4 + ((q & cmask) << 2));
                tw[e] = lds_at(sm, o_tt4 + ((d >> a.toa_shift) << 2));
            }
        }
    };
    // stage 2b: tag check, one gather per event (a table hit or an
    // out-of-range pixel loads out of range: no request, returns 0); w -> the
    // table word of hits (0 otherwise), qs -> the gathered word
    auto finish = [&](uint32_t (&w)[kEPT], uint32_t (&qs)[kEPT]) __attribute__((always_inline)) {
#pragma unroll
        for (int e = 0; e < kEPT; ++e) {
            const unsigned long long hit =
                __builtin_amdgcn_ballot_w64(((w[e] >> kSieveTagShift) & 0xFFu) == (qs[e] >> a.cbits));
            uint32_t off = vsel(hit, kOOBi, min(qs[e], Lc) << 2);
            if (ABL & 16) off = kOOB | (off & 4u);
            if (ABL & 32) off = off & 4u;
            w[e] = vsel(hit, w[e], 0u);
            qs[e] = (ABL & 2) ? (off & 0x3u) : __builtin_amdgcn_raw_buffer_load_b32(glut, (int)off, 0, 0);
        }
    };
    // stage 3: bin, in two halves of four events per lane.  Hot lanes add 1
    // to their LDS row (the others to a lane-private dummy); cold keys are
    // compacted into the wave's 256-word LDS staging area (the others write a
    // dummy) and leave as one 16-byte store per lane into the wave's own
    // sub-region of the block's cold region, at an SGPR cursor (no atomics).
    // The staged words are read back right away but stored one half later,
    // so that read's LDS latency is not waited for.  Staging words are reset
    // to -1, so the <= 3 pad keys of round4(count) are dropped by the sort.
    v4u pend_kv = {0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
    uint32_t pend_off = kOOB;
    uint32_t wcur = 0;  // this wave's cold keys so far (wave-uniform)
    auto bin = [&](const uint32_t (&ws)[kEPT], const uint32_t (&g)[kEPT], const uint32_t (&dc)[kEPT],
                   const uint32_t (&tw)[kEPT]) __attribute__((always_inline)) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            uint32_t tot = 0;
#pragma unroll
            for (int e = h * kEPT / 2; e < (h + 1) * kEPT / 2; ++e) {
                const uint32_t v = ws[e] | g[e];
                const uint32_t b = (tw[e] & 0xFFu) + (((dc[e] & wmask) >= (tw[e] >> 8)) ? 1u : 0u);
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
                const uint32_t hidx4 = vsel(hm, k4, dum4);
                if (!(ABL & 1))
                    __hip_atomic_fetch_add(&lds_at(sm, hidx4), 1u, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_WORKGROUP);
                else
                    tot += hidx4 & 1u;
                lds_at(sm, vsel(bal, pos4, dum4)) = k4;
                const uint32_t tidx4 = vsel(bal, ((k4 >> tsh) << 2) + o_tcnt4, dum4);
                __hip_atomic_fetch_add(&lds_at(sm, tidx4), 1u, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_WORKGROUP);
            }
            const uint32_t res = (tot + 3u) & ~3u;
            // the previous half's keys leave now (their LDS read is long done)
            if (!(ABL & 4)) __builtin_amdgcn_raw_buffer_store_b128(pend_kv, cold, (int)pend_off, 0, 0);
            else sm[o_dum + lane] += pend_kv[0] ^ pend_off;
            __builtin_amdgcn_wave_barrier();
            uint4 *slot = reinterpret_cast<uint4 *>(sm + o_stg_w + 4u * (uint32_t)lane);
            const uint4 kv = *slot;
            *slot = make_uint4(0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu);
            __builtin_amdgcn_wave_barrier();
            pend_kv = v4u{kv.x, kv.y, kv.z, kv.w};
            pend_off = 4u * (uint32_t)lane < res ? (wave_base + wcur + 4u * (uint32_t)lane) << 2 : kOOB;
            wcur += res;
        }
    };

    // ---- pipeline: chunk i is binned while chunk i+1 is probed (before) and
    // gathered (after), chunks i+2, i+3 stream in and the descriptor of i+4 is
    // fetched (register sets A/B and X/Y alternate)
    int pA[kEPT], tA[kEPT], pB[kEPT], tB[kEPT];
    uint32_t wsX[kEPT], gX[kEPT], dX[kEPT], twX[kEPT];
    uint32_t wsY[kEPT], gY[kEPT], dY[kEPT], twY[kEPT];
    if (cb < ce) {
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
        int si = 0;
        {
            int lo = 0, hi = a.n_segs - 1;
            while (lo < hi) {
                const int mid = (lo + hi + 1) >> 1;
                if (a.segs[mid].chunk0 <= cb) lo = mid; else hi = mid - 1;
            }
            si = lo;
        }
        for (long long c = cb; c < ce; ++c) {
            while (si + 1 < a.n_segs && a.segs[si + 1].chunk0 <= c) ++si;
            const SegDesc sd = a.segs[si];
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
    if (!(ABL & 4)) __builtin_amdgcn_raw_buffer_store_b128(pend_kv, cold, (int)pend_off, 0, 0);
    if (lane == 0) a.cold_cnt[(size_t)blockIdx.x * (kSplitThreads / 64) + (tid >> 6)] = wcur;
    __syncthreads();
    uint32_t *dst = a.hot_part + (size_t)blockIdx.x * a.hot_words;
    for (int i = tid * 4; i < a.hot_words; i += kSplitThreads * 4)
        *reinterpret_cast<uint4 *>(dst + i) = *reinterpret_cast<const uint4 *>(sm + i);
    for (int i = tid; i < a.n_tiles * a.tgroups; i += kSplitThreads)
        a.cold_tcnt[(size_t)blockIdx.x * a.tgroups * a.n_tiles + i] = sm[o_tcnt + i];
}

// ---------------------------------------------------------------------------
// cold keys: exact counting sort into a tile-major u16 array, then pass B
// ---------------------------------------------------------------------------
// per tile: exclusive scan over sieve blocks of their key counts
__global__ __launch_bounds__(256) void k_cold_scan(const uint32_t *__restrict__ tcnt, int rows,
                                                   int n_tiles, uint32_t *__restrict__ boff,
                                                   uint32_t *__restrict__ tile_total) {
    __shared__ uint32_t s_w[32];
    const int t = blockIdx.x;
    uint32_t carry = 0;
    for (int r0 = 0; r0 < rows; r0 += 256) {
        const int r = r0 + threadIdx.x;
        const uint32_t v = r < rows ? tcnt[(size_t)r * n_tiles + t] : 0u;
        uint32_t tot;
        const uint32_t ex = block_exclusive_scan(v, s_w, &tot);
        if (r < rows) boff[(size_t)r * n_tiles + t] = carry + ex;
        carry += tot;
        __syncthreads();
    }
    if (threadIdx.x == 0) tile_total[t] = carry;
}

// tile bases of the tile-major key array + balanced pass-B items
// (tile, first key, end key); a tile with n keys gets ceil(n / item_keys) items
__global__ __launch_bounds__(1024) void k_cold_plan(const uint32_t *__restrict__ tile_total,
                                                    int n_tiles, uint32_t item_keys,
                                                    uint32_t *__restrict__ tile_base,
                                                    uint4 *__restrict__ items,
                                                    uint32_t *__restrict__ item_count,
                                                    uint32_t max_items) {
    __shared__ uint32_t s_w[32];
    __shared__ uint32_t s_ib[kMaxTiles + 1];
    __shared__ uint32_t s_kb[kMaxTiles + 1];
    constexpr int TPT = kMaxTiles / 1024;
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
            tile_base[t] = kb;
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
    for (uint32_t i = (uint32_t)tid; i < n_items; i += 1024u) {
        int lo = 0, hi = n_tiles - 1;  // last tile with s_ib[t] <= i
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (s_ib[mid] <= i) lo = mid; else hi = mid - 1;
        }
        const uint32_t j = i - s_ib[lo], nt = s_ib[lo + 1] - s_ib[lo];
        const uint32_t k0 = s_kb[lo], kn = s_kb[lo + 1] - k0;
        const uint32_t b0 = k0 + (uint32_t)((unsigned long long)j * kn / nt);
        const uint32_t b1 = k0 + (uint32_t)((unsigned long long)(j + 1) * kn / nt);
        items[i] = make_uint4((uint32_t)lo, b0, b1, 0u);
    }
    if (tid == 0) *item_count = n_items;
}

// One block per sieve block: its cold region (keys scaled by 4, -1 pads; 16
// wave sub-regions) is sorted by tile in 16K-key
// pieces in LDS (rank by LDS atomics, scan over tiles, scatter), and each
// piece's tile runs are written as u16 tile-local keys at the block's exact
// offsets of the tile-major array.  Pad keys (-1) are skipped.
constexpr int kSortThreads = 1024;
constexpr int kSortPiece = 16384;
size_t cold_sort_smem(int n_tiles) {
    return 4 * ((size_t)kSortPiece + 3 * (size_t)align4(n_tiles) + 32);
}

// halves == 2: two blocks share a region (two blocks per CU), the first
// half's pieces fill each tile's slots upward from the region's tile offset,
// the second half's downward from its end (offset + the region's tile count),
// so the halves need no count of each other's keys.
template <int TB>
__global__ __launch_bounds__(kSortThreads) void k_cold_sort(
    const uint32_t *__restrict__ cold, long long stride, long long cap,
    const uint32_t *__restrict__ cold_cnt, const uint32_t *__restrict__ boff,
    const uint32_t *__restrict__ tcnt, const uint32_t *__restrict__ tile_base, int n_tiles,
    int groups, int halves, uint16_t *__restrict__ out) {
    constexpr int KPT = kSortPiece / kSortThreads;  // 16 keys per thread
    constexpr uint32_t MASK = (1u << TB) - 1u;
    extern __shared__ __attribute__((aligned(16))) uint32_t sm[];
    const int nt4 = align4(n_tiles);
    uint32_t *s_sorted = sm;
    uint32_t *s_cnt = sm + kSortPiece;
    uint32_t *s_start = s_cnt + nt4;
    uint32_t *s_cur = s_start + nt4;
    uint32_t *s_w = s_cur + nt4;
    const int tid = threadIdx.x;
    // block = (sieve block b, wave group g): waves [g * WPG, (g + 1) * WPG) of
    // the sieve block's cold region, which is 16 wave sub-regions of cap / 16
    // keys, each filled to a multiple of 4; logical key i lives in the
    // sub-region of the last wave whose prefix is <= i
    constexpr int NW = kSplitThreads / 64;
    const int row = blockIdx.x / halves, half = blockIdx.x % halves;
    const int b = row / groups, g = row % groups;
    const int WPG = NW / groups;
    if (tid == 0) {
        uint32_t acc = 0;
        for (int w = 0; w < NW; ++w) {
            s_w[w] = acc;
            if (w >= g * WPG && w < (g + 1) * WPG) acc += cold_cnt[(size_t)b * NW + w];
        }
        s_w[NW] = acc;
    }
    __syncthreads();
    uint32_t pre[NW + 1];
#pragma unroll
    for (int w = 0; w <= NW; ++w) pre[w] = s_w[w];
    __syncthreads();
    const uint32_t n = pre[NW];
    const uint32_t npieces = (n + kSortPiece - 1) / kSortPiece;
    const uint32_t mid = halves > 1 ? min(n, ((npieces + 1) / 2) * (uint32_t)kSortPiece) : n;
    const uint32_t pb = half ? mid : 0u, pe = half ? n : mid;  // this block's logical keys
    const uint32_t capw = (uint32_t)(cap / NW);
    auto phys = [&](uint32_t i) __attribute__((always_inline)) {
        uint32_t w = 0;
#pragma unroll
        for (int q = 1; q < NW; ++q) w = i >= pre[q] ? (uint32_t)q : w;
        return i < n ? (w * capw + (i - pre[w])) * 4u : 0x80000000u;
    };
    const uint32_t *src = cold + (size_t)b * (size_t)stride;
    const __amdgpu_buffer_rsrc_t rs = make_rsrc(src, (uint32_t)(cap * 4));
    for (int t = tid; t < n_tiles; t += kSortThreads)
        s_cur[t] = tile_base[t] + boff[(size_t)row * n_tiles + t] +
                   (half ? tcnt[(size_t)row * n_tiles + t] : 0u);
    constexpr int TPT = kMaxTiles / kSortThreads;
    // the next piece's keys are requested before the current piece is sorted
    v4u nk[KPT / 4];
    auto fetch = [&](uint32_t p0) __attribute__((always_inline)) {
#pragma unroll
        for (int j = 0; j < KPT / 4; ++j) {
            const uint32_t e0 = p0 + ((uint32_t)j * kSortThreads + (uint32_t)tid) * 4u;
            nk[j] = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)phys(e0), 0, 0);
        }
    };
    if (pb < pe) fetch(pb);
    for (uint32_t p0 = pb; p0 < pe; p0 += kSortPiece) {
        for (int t = tid; t < n_tiles; t += kSortThreads) s_cnt[t] = 0;
        uint32_t key[KPT], rank[KPT];
#pragma unroll
        for (int j = 0; j < KPT / 4; ++j) {
            const uint32_t e0 = p0 + ((uint32_t)j * kSortThreads + (uint32_t)tid) * 4u;
#pragma unroll
            for (int q = 0; q < 4; ++q) key[j * 4 + q] = e0 + (uint32_t)q < pe ? nk[j][q] : 0xFFFFFFFFu;
        }
        if (p0 + kSortPiece < pe) fetch(p0 + kSortPiece);
        __syncthreads();
#pragma unroll
        for (int e = 0; e < KPT; ++e) {
            rank[e] = 0;
            if (key[e] != 0xFFFFFFFFu)
                rank[e] = __hip_atomic_fetch_add(s_cnt + (key[e] >> (TB + 2)), 1u, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        __syncthreads();
        uint32_t c[TPT], sum = 0;
#pragma unroll
        for (int q = 0; q < TPT; ++q) {
            const int t = tid * TPT + q;
            c[q] = t < n_tiles ? s_cnt[t] : 0u;
            sum += c[q];
        }
        uint32_t total;
        uint32_t run = block_exclusive_scan(sum, s_w, &total);
#pragma unroll
        for (int q = 0; q < TPT; ++q) {
            const int t = tid * TPT + q;
            if (t < n_tiles) s_start[t] = run;
            run += c[q];
        }
        __syncthreads();
#pragma unroll
        for (int e = 0; e < KPT; ++e)
            if (key[e] != 0xFFFFFFFFu) s_sorted[s_start[key[e] >> (TB + 2)] + rank[e]] = key[e];
        __syncthreads();
        if (half == 0) {
            for (uint32_t i = (uint32_t)tid; i < total; i += kSortThreads) {
                const uint32_t k = s_sorted[i];
                const uint32_t t = k >> (TB + 2);
                out[s_cur[t] + (i - s_start[t])] = (uint16_t)((k >> 2) & MASK);
            }
        } else {
            for (uint32_t i = (uint32_t)tid; i < total; i += kSortThreads) {
                const uint32_t k = s_sorted[i];
                const uint32_t t = k >> (TB + 2);
                out[s_cur[t] - 1u - (i - s_start[t])] = (uint16_t)((k >> 2) & MASK);
            }
        }
        __syncthreads();
        if (half == 0)
            for (int t = tid; t < n_tiles; t += kSortThreads) s_cur[t] += s_cnt[t];
        else
            for (int t = tid; t < n_tiles; t += kSortThreads) s_cur[t] -= s_cnt[t];
    }
}

// pass B: one item = a contiguous key range of one tile
template <int TB>
__global__ __launch_bounds__(kTileThreads) void k_cold_accumulate(
    const uint16_t *__restrict__ keys, const uint4 *__restrict__ items,
    const uint32_t *__restrict__ item_count, uint32_t *__restrict__ hist, long long n_bins) {
    constexpr int NB = 1 << TB;
    __shared__ __attribute__((aligned(16))) uint32_t s_tile[NB];
    if (blockIdx.x >= *item_count) return;
    const uint4 it = items[blockIdx.x];
    for (int i = threadIdx.x * 4; i < NB; i += kTileThreads * 4)
        *reinterpret_cast<uint4 *>(s_tile + i) = make_uint4(0, 0, 0, 0);
    __syncthreads();
    // four 16-byte loads (32 keys) per thread in flight per iteration
    const uint32_t k0 = it.y & ~7u;
    for (uint32_t i0 = k0 + (uint32_t)threadIdx.x * 8u; i0 < it.z; i0 += kTileThreads * 32u) {
        uint4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const uint32_t i = i0 + (uint32_t)u * kTileThreads * 8u;
            v[u] = i < it.z ? *reinterpret_cast<const uint4 *>(keys + i) : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const uint32_t i = i0 + (uint32_t)u * kTileThreads * 8u;
            const uint32_t w[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                const uint32_t idx = i + (uint32_t)q;
                if (idx >= it.y && idx < it.z)
                    __hip_atomic_fetch_add(s_tile + ((w[q >> 1] >> ((q & 1) * 16)) & 0xFFFFu), 1u,
                                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
        }
    }
    __syncthreads();
    const long long base = (long long)it.x << TB;
    for (int i = threadIdx.x; i < NB; i += kTileThreads) {
        const uint32_t v = s_tile[i];
        if (v != 0u && base + i < n_bins) atomicAdd(hist + base + i, v);
    }
}

// ---------------------------------------------------------------------------
// launch wrappers
// ---------------------------------------------------------------------------
size_t sieve_smem(int hot_words, int cbits, int toa_words4, int n_tiles, int tgroups) {
    return 4 * ((size_t)hot_words + ((size_t)1 << cbits) + (size_t)toa_words4 + 64 + 4 +
                (size_t)kSieveStage * (kSplitThreads / 64) + (size_t)align4(n_tiles * tgroups));
}

hipError_t launch_sieve_tables(const void *lut, bool lut16, long long L, int T,
                               const uint16_t *screen_row, const uint32_t *pix_cnt, int cbits,
                               uint32_t *glut, uint32_t *tab, hipStream_t st) {
    const unsigned g = (unsigned)((L + 1 + 255) / 256);
    if (lut16)
        hipLaunchKernelGGL(k_sieve_glut<uint16_t>, dim3(g), dim3(256), 0, st,
                           (const uint16_t *)lut, L, T, screen_row, glut);
    else
        hipLaunchKernelGGL(k_sieve_glut<int>, dim3(g), dim3(256), 0, st, (const int *)lut, L, T,
                           screen_row, glut);
    hipLaunchKernelGGL(k_sieve_table, dim3((unsigned)(((1LL << cbits) + 255) / 256)), dim3(256), 0,
                       st, pix_cnt, glut, L, cbits, tab);
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
    hipLaunchKernelGGL(k_cold_scan, dim3(c.n_tiles), dim3(256), 0, st, c.tcnt, c.rows * c.groups,
                       c.n_tiles, c.boff, c.tile_total);
    hipLaunchKernelGGL(k_cold_plan, dim3(1), dim3(1024), 0, st, c.tile_total, c.n_tiles, c.item_keys,
                       c.tile_base, c.items, c.item_count, c.max_items);
    const size_t sm = cold_sort_smem(c.n_tiles);
    hipError_t e = hipSuccess;
    switch (c.tile_bits) {
#define LDE_COLD(TB)                                                                              \
    case TB:                                                                                      \
        (void)hipFuncSetAttribute((const void *)k_cold_sort<TB>,                                  \
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)sm);           \
        hipLaunchKernelGGL(k_cold_sort<TB>, dim3(c.rows * c.groups * c.halves), dim3(kSortThreads), \
                           sm, st, c.cold, c.stride, c.cap, c.cold_cnt, c.boff, c.tcnt,           \
                           c.tile_base, c.n_tiles, c.groups, c.halves, c.keys);                   \
        hipExtLaunchKernelGGL(k_cold_accumulate<TB>, dim3(c.max_items), dim3(kTileThreads), 0, st,\
                              nullptr, stop, 0, c.keys, c.items, c.item_count, c.hist, c.n_bins); \
        break;
        LDE_COLD(13)
        LDE_COLD(14)
        LDE_COLD(15)
#undef LDE_COLD
    default:
        e = hipErrorInvalidValue;
    }
    if (e != hipSuccess) return e;
    return hipGetLastError();
}

template <int ABL>
static hipError_t launch_sieve_t(const SieveArgs &a, int grid, hipStream_t st, hipEvent_t start,
                                 hipEvent_t stop) {
    if (sieve_smem(a.hot_words, a.cbits, a.toa_words4, a.n_tiles, a.tgroups) > kSplitSmemMax)
        return hipErrorInvalidValue;
    hipExtLaunchKernelGGL(k_sieve<ABL>, dim3(grid), dim3(kSplitThreads), 0, st, start, stop, 0,
                          a);  // static LDS
    return hipGetLastError();
}

hipError_t launch_sieve(const SieveArgs &a, int grid, hipStream_t st, hipEvent_t start,
                        hipEvent_t stop) {
    switch (a.ablate) {
    case 1: return launch_sieve_t<1>(a, grid, st, start, stop);
    case 2: return launch_sieve_t<2>(a, grid, st, start, stop);
    case 4: return launch_sieve_t<4>(a, grid, st, start, stop);
    case 7: return launch_sieve_t<7>(a, grid, st, start, stop);
    case 15: return launch_sieve_t<15>(a, grid, st, start, stop);
    case 16: return launch_sieve_t<16>(a, grid, st, start, stop);
    case 32: return launch_sieve_t<32>(a, grid, st, start, stop);
    default: return launch_sieve_t<0>(a, grid, st, start, stop);
    }
}

}  // namespace lde
