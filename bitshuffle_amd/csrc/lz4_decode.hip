// lz4_decode.hip -- K6: block index rebuild; K4+K2 fused: LZ4 block decode +
// inverse bit transpose, one 64-lane wavefront per block.
//
// Reference path: bshuf_decompress_lz4 -> bshuf_blocked_wrap_fun ->
// bshuf_decompress_lz4_block (src/bitshuffle.c:83-119): read BE32 length,
// LZ4_decompress_safe into a block-sized buffer (lz4/lz4.c:2451), require
// exactly bs*E bytes (-91), bshuf_untrans_bit_elem.  The reference finds block
// k's header by walking the chain serially (iochain, src/iochain.c:42-64).
//
// Index rebuild (no serial walk):  the framed region [0, Cb) is cut into
// chunks of CH bytes (CH >= the largest possible record).  The chain enters
// chunk s at its first header e_s >= s*CH, which must lie in
// [s*CH, s*CH + maxfoot).  Phase 1 (k_idx_exits): one wave per chunk tries
// EVERY position of that window whose BE32 is a plausible block length,
// follows each such chain to the first position >= the chunk end (or exactly
// Cb), and drops chains that hit an implausible header.  The true chain is
// among the survivors, so if all survivors agree on the exit, that exit IS
// e_{s+1}, independent of everything before the chunk.  Chunks whose
// survivors disagree are resolved in phase 2 by chasing forward from the
// nearest agreed exit.  Phase 2 (k_idx_walk, count) walks each chunk from its
// entry, phase 3 scans the counts, phase 4 (k_idx_walk, write) stores the
// header offsets.  A stream whose chain does not end exactly at Cb with the
// expected number of blocks is rejected.
#include <hipcub/hipcub.hpp>

#include <cstdlib>

#include "launch.h"
#include "lds_copy.h"
#include "lz4_scan.h"

namespace bshuf {

namespace {

constexpr int64_t kAmbiguous = -2;
constexpr int64_t kDead = -1;
constexpr int kIdxWinMax = 32768;  // LDS window for candidate screening
constexpr int kIdxCandCap = 512;   // LDS list of screened candidates (u32 window offsets)

// Diagnostic build only (-DBSHUF_DIAG, tools/diag_decode.py): k_lz4_decode's
// per-phase s_memtime cycle sums and event counts (slots 0..7 cycles, 8..15
// counts; 64 copies picked by workgroup).  The product build's DDiag is empty.
#ifdef BSHUF_DIAG
constexpr int kDDiagCopies = 64;
__device__ unsigned long long g_ddiag[kDDiagCopies * 16];
struct DDiag {
    uint64_t t, acc[8];
    uint32_t cnt[8];
    __device__ DDiag() : t(__builtin_amdgcn_s_memtime()) {
        for (int i = 0; i < 8; i++) acc[i] = 0, cnt[i] = 0;
    }
    __device__ __forceinline__ void stamp(int i) {
        const uint64_t n = __builtin_amdgcn_s_memtime();
        acc[i] += n - t;
        t = n;
    }
    __device__ __forceinline__ void count(int i, uint32_t v) { cnt[i] += v; }
    __device__ void flush(int lane) {
        if (lane == 0)
            for (int i = 0; i < 8; i++) {
                atomicAdd(&g_ddiag[(blockIdx.x % kDDiagCopies) * 16 + i], (unsigned long long)acc[i]);
                atomicAdd(&g_ddiag[(blockIdx.x % kDDiagCopies) * 16 + 8 + i], (unsigned long long)cnt[i]);
            }
    }
};
#else
struct DDiag {
    __device__ __forceinline__ void stamp(int) {}
    __device__ __forceinline__ void count(int, uint32_t) {}
    __device__ __forceinline__ void flush(int) {}
};
#endif

// global, not generic, byte loads: a flat load also counts on lgkmcnt (an LDS
// wait then waits for it too) and reads as divergent to the compiler
__device__ __forceinline__ uint32_t be32_global(const uint8_t* p) {
    const gbl8c* q = (const gbl8c*)p;
    return ((uint32_t)q[0] << 24) | ((uint32_t)q[1] << 16) | ((uint32_t)q[2] << 8) | q[3];
}

// Follow the chain from p until it reaches/passes `stop` or Cb; returns the
// position reached (>= stop, or == Cb), or kDead on an implausible header.
__device__ int64_t chase(const uint8_t* in, int64_t p, int64_t stop, int64_t Cb,
                         uint32_t maxlen) {
    while (p < stop && p != Cb) {
        if (p + 4 > Cb) return kDead;
        const uint32_t len = be32_global(in + p);
        if (len == 0 || len > maxlen || p + 4 + (int64_t)len > Cb) return kDead;
        p += 4 + len;
    }
    return p;
}

// Chunk c of the index rebuild: its stream (the single one, or stream
// chunk_seg[c] of a batch), its chunk number inside that stream and where that
// stream's blocks and error word live.
struct IdxArgs {
    const uint8_t* in;   // single stream
    int64_t Cb;          // single stream: framed region bytes
    int64_t nblocks;
    int64_t* err;
    const Seg* segs;     // batch (nullptr: single stream)
    const uint32_t* chunk_seg;
    int64_t* errs;       // batch: one word per stream
    int64_t CH;          // chunk bytes
    int64_t W;           // candidate window (largest record)
    uint32_t maxlen;
    int64_t win_lds;     // k_idx_exits' LDS window bytes
    int64_t wsub;        // candidates per k_idx_exits workgroup (gridDim.y of them per chunk)
    // single stream with its length in device memory (bshuf_decompress_lz4_dev_dlen):
    // Cb is then resolved on the device from *dlen, the capacity and the raw tail
    const int64_t* dlen;
    int64_t cap;
    int64_t tail;
};

// Readable stream bytes of a device-held length word: a negative word (an
// upstream error, e.g. the compress result) reads nothing; never past cap.
__device__ __forceinline__ int64_t readable_bytes(int64_t d, int64_t cap) {
    return d < 0 ? 0 : (d < cap ? d : cap);
}

// Resolves a device-held stream length once per kernel (single stream).
__device__ __forceinline__ void resolve_len(IdxArgs& x) {
    if (x.dlen) {
        x.Cb = max(readable_bytes(*x.dlen, x.cap) - x.tail, (int64_t)0);
        x.dlen = nullptr;
    }
}

struct ChunkLoc {
    const uint8_t* in;
    int64_t Cb;
    int64_t s;      // chunk index inside the stream
    int64_t c0;     // global index of the stream's first chunk
    int64_t first;  // global index of the stream's first block
    int64_t nb;     // blocks of the stream
    int64_t* err;
};

__device__ __forceinline__ ChunkLoc chunk_loc(const IdxArgs& x, int64_t c) {
    ChunkLoc l;
    if (!x.segs) {
        l.in = x.in;
        l.Cb = x.Cb;
        l.s = c;
        l.c0 = 0;
        l.first = 0;
        l.nb = x.nblocks;
        l.err = x.err;
    } else {
        const uint32_t g = x.chunk_seg[c];
        const Seg& sg = x.segs[g];
        l.in = sg.in;
        l.Cb = max(sg.in_nbytes - sg.tail, (int64_t)0);
        l.s = c - sg.chunk0;
        l.c0 = sg.chunk0;
        l.first = sg.first;
        l.nb = sg.nfull + (sg.last ? 1 : 0);
        l.err = x.errs + g;
    }
    return l;
}

__global__ __launch_bounds__(64) void k_idx_exits(IdxArgs x, int64_t* __restrict__ exits,
                                                  int64_t* __restrict__ his) {
    // the candidate window (largest record + 4, +64 slack), sized at launch:
    // the chases below are latency-bound, so a small window buys residency
    extern __shared__ __attribute__((aligned(16))) uint8_t win[];
    int win_off = 0;
    const int lane = threadIdx.x;
    resolve_len(x);
    const ChunkLoc L = chunk_loc(x, blockIdx.x);
    const uint8_t* in = L.in;
    const int64_t Cb = L.Cb, CH = x.CH, W = x.W;
    const uint32_t maxlen = x.maxlen;
    const int64_t s = L.s;
    const int64_t cs = s * CH;
    if (s > 0 && cs >= Cb) {
        // past the stream's end (chunks sized by a capacity, device-held
        // length): no entry, and nothing ever chases from here
        if (gridDim.y == 1 && lane == 0) exits[blockIdx.x] = kDead;
        return;
    }
    const int64_t ce = min(cs + CH, Cb);
    // candidate window [cs, cs + W), split over gridDim.y workgroups of wsub
    // candidates each (large blocks: a window of the largest record does not
    // fit the LDS, and one wave per chunk would leave most CUs idle)
    const int64_t cwin = (s == 0) ? cs + 1 : min(cs + W, Cb);
    const int64_t cb0 = min(cs + (int64_t)blockIdx.y * x.wsub, cwin);
    const int64_t cend = min(cb0 + x.wsub, cwin);
    const int64_t wbytes = max(min(cend + 3, Cb) - cb0, (int64_t)0);
    // 16-byte loads of the candidate window, aligned on the ABSOLUTE address:
    // an aligned granule never crosses a page, so the bytes it reads outside
    // [cb0, cb0+wbytes) cannot fault and are never used
    const uintptr_t start = (uintptr_t)(in + cb0);
    const int sh = (int)(start & 15);
    const int64_t nch = (sh + wbytes + 15) >> 4;
    const bool use_lds = nch * 16 <= x.win_lds;
    if (use_lds) {
        const gbl128c* g4 = g128_aligned_down(in + cb0);
        lds128* w4 = (lds128*)to_lds(win);
        for (int c = lane; c < (int)nch; c += kWave) w4[c] = g4[c];
        __syncthreads();
        win_off = sh;
    }
    int64_t lo = INT64_MAX, hi = -1;
    auto try_cand = [&](int64_t c, uint32_t len) {
        if (c >= cend || c + 4 > Cb) return;
        if (len == 0 || len > maxlen || c + 4 + (int64_t)len > Cb) return;
        const int64_t xx = chase(in, c + 4 + len, ce, Cb, maxlen);
        if (xx == kDead) return;
        lo = min(lo, xx);
        hi = max(hi, xx);
    };
    if (use_lds) {
        // Screen, then chase: 4 consecutive candidates per lane (two dword
        // reads cover the 7 bytes of their four big-endian length words); the
        // plausible ones go to an LDS list (wave prefix sum of per-lane
        // counts), and the list is chased 64 candidates at a time -- one
        // chase loop per 64 plausible positions instead of one per screening
        // step that holds any (large blocks: 1,027 steps per chunk window).
        const lds8* wq = (const lds8*)to_lds(win) + win_off;
        lds32* list = (lds32*)(to_lds(win) + x.win_lds);
        int nl = 0;  // wave-uniform list length
        auto plausible = [&](int64_t c, uint32_t len) {
            return c < cend && c + 4 <= Cb && len != 0 && len <= maxlen && c + 4 + (int64_t)len <= Cb;
        };
        auto chase_list = [&]() {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            for (int i = lane; i < nl; i += kWave) {
                const int r = (int)list[i];
                const uint32_t len = __builtin_bswap32(lds_rd32(wq, r));
                const int64_t xx = chase(in, cb0 + r + 4 + len, ce, Cb, maxlen);
                if (xx != kDead) {
                    lo = min(lo, xx);
                    hi = max(hi, xx);
                }
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            nl = 0;
        };
        for (int64_t c0 = cb0 + 4 * lane; __builtin_amdgcn_readfirstlane((int)(c0 - 4 * lane < cend)); c0 += 4 * kWave) {
            const int r = (int)(c0 - cb0);
            const uint32_t a = lds_rd32(wq, r), b = lds_rd32(wq, r + 4);
            uint32_t pm = 0;
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const uint32_t le = __builtin_amdgcn_alignbyte(b, a, (uint32_t)k);
                pm |= plausible(c0 + k, __builtin_bswap32(le)) ? 1u << k : 0u;
            }
            const int cnt = __builtin_popcount(pm);
            const int incl = wave_incl_sum(cnt, lane);
            const int total = __builtin_amdgcn_readlane(incl, kWave - 1);
            if (total == 0) continue;
            if (nl + total > kIdxCandCap) chase_list();
            int at = nl + incl - cnt;
#pragma unroll
            for (int k = 0; k < 4; k++)
                if (pm & (1u << k)) list[at++] = (uint32_t)(r + k);
            nl += total;
        }
        chase_list();
    } else {
        // window larger than the LDS budget (large blocks): the same 4
        // candidates per lane from three absolute-aligned global dwords (an
        // aligned dword never crosses a page; bytes past Cb are never used),
        // several iterations' loads in flight at once
#pragma unroll 8
        for (int64_t c0 = cb0 + 4 * lane; c0 < cend; c0 += 4 * kWave) {
            const uintptr_t ap = (uintptr_t)(in + c0), al = ap & ~(uintptr_t)3;
            const uint32_t sh = (uint32_t)(ap & 3);
            const uint32_t w0 = *(const gbl32c*)al, w1 = *(const gbl32c*)(al + 4),
                           w2 = *(const gbl32c*)(al + 8);
            const uint32_t a = __builtin_amdgcn_alignbyte(w1, w0, sh), b = __builtin_amdgcn_alignbyte(w2, w1, sh);
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const uint32_t le = __builtin_amdgcn_alignbyte(b, a, (uint32_t)k);
                try_cand(c0 + k, __builtin_bswap32(le));
            }
        }
    }
    for (int o = 32; o >= 1; o >>= 1) {
        lo = min(lo, (int64_t)__shfl_xor(lo, o));
        hi = max(hi, (int64_t)__shfl_xor(hi, o));
    }
    if (gridDim.y == 1) {
        if (lane == 0) exits[blockIdx.x] = (hi < 0) ? kDead : (lo == hi ? lo : kAmbiguous);
    } else if (lane == 0) {
        // split window: min / max of the surviving exits over the chunk's
        // workgroups (exits[] pre-filled with INT64_MAX, his[] with -1), made
        // an exit by k_idx_exits_join
        if (hi >= 0) {
            atomicMin((long long*)&exits[blockIdx.x], (long long)lo);
            atomicMax((long long*)&his[blockIdx.x], (long long)hi);
        }
    }
}

// Split windows: one exit per chunk from the min / max the workgroups left.
__global__ void k_idx_exits_join(int64_t* __restrict__ exits, const int64_t* __restrict__ his,
                                 int64_t nch) {
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= nch) return;
    const int64_t lo = exits[c], hi = his[c];
    exits[c] = (hi < 0) ? kDead : (lo == hi ? lo : kAmbiguous);
}

// Entry e_s of chunk s (of the stream whose chunk 0 is exits[0]): the agreed
// exit of chunk s-1, else chase forward from the nearest chunk with an agreed
// exit (or from offset 0).
__device__ int64_t chunk_entry(const uint8_t* in, const int64_t* exits, int64_t s, int64_t CH,
                               int64_t Cb, uint32_t maxlen) {
    if (s == 0) return 0;
    int64_t t = s - 1;
    while (t >= 0 && exits[t] < 0) t--;
    int64_t p = (t < 0) ? 0 : exits[t];
    for (int64_t u = t + 1; u < s && p != kDead; u++) p = chase(in, p, min((u + 1) * CH, Cb), Cb, maxlen);
    return p;
}

// Walk chunk c from its entry.  mode 0: count headers into cnt[c];
// mode 1: write the offsets of the stream's blocks (base = exclusive scan of
// the counts over all chunks of all streams).  A broken link sets the
// stream's error word.
__global__ __launch_bounds__(64) void k_idx_walk(IdxArgs x, int64_t nchunks_total,
                                                 const int64_t* __restrict__ exits,
                                                 uint64_t* __restrict__ cnt,
                                                 const uint64_t* __restrict__ base,
                                                 uint64_t* __restrict__ offs, int mode) {
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= nchunks_total) return;
    resolve_len(x);
    const ChunkLoc L = chunk_loc(x, c);
    const int64_t CH = x.CH, Cb = L.Cb;
    const uint32_t maxlen = x.maxlen;
    if (L.s > 0 && L.s * CH >= Cb) {  // past the stream's end: no headers
        if (!mode) cnt[c] = 0;
        return;
    }
    const int64_t ce = min((L.s + 1) * CH, Cb);
    int64_t p = chunk_entry(L.in, exits + L.c0, L.s, CH, Cb, maxlen);
    if (p == kDead) {
        atomicMax((unsigned long long*)L.err, 1ull);
        return;
    }
    uint64_t k = mode ? base[c] - base[L.c0] : 0;  // block index inside the stream
    uint64_t n = 0;
    while (p < ce) {
        if (p + 4 > Cb) {
            atomicMax((unsigned long long*)L.err, 1ull);
            return;
        }
        const uint32_t len = be32_global(L.in + p);
        if (len == 0 || len > maxlen || p + 4 + (int64_t)len > Cb) {
            atomicMax((unsigned long long*)L.err, 1ull);
            return;
        }
        if (mode) {
            if ((int64_t)k < L.nb) offs[L.first + k] = (uint64_t)p;
            k++;
        }
        n++;
        p += 4 + len;
    }
    if (!mode) cnt[c] = n;
}

// Every stream must have produced exactly its number of headers.
__global__ void k_idx_check(IdxArgs x, const uint64_t* base, int64_t nchunks) {
    if (!x.segs) {
        if (threadIdx.x == 0 && (int64_t)base[nchunks] != x.nblocks)
            atomicMax((unsigned long long*)x.err, 2ull);
        return;
    }
    const Seg& g = x.segs[blockIdx.x];
    const int64_t nb = g.nfull + (g.last ? 1 : 0);
    if (threadIdx.x == 0 && (int64_t)(base[g.chunk0 + g.nchunks] - base[g.chunk0]) != nb)
        atomicMax((unsigned long long*)(x.errs + blockIdx.x), 2ull);
}

// ---------------------------------------------------------------------------
// Per-block LZ4 decode
// ---------------------------------------------------------------------------

// ---------------------------------------------------------------------------
// Two-phase decode (default).  Phase 1 (k_seq_scan, one LANE per block) walks
// each record's token chain straight from HBM, applies every check of
// LZ4_decompress_safe with the same error positions, and stores the payload
// position of each sequence's token.  Phase 2 (lz4_exec_block, one wave per
// block) then has no serial walk left: 64 lanes decode 64 sequences at once,
// a DPP prefix sum places them, every literal run is copied in parallel, and
// the matches run in batches of consecutive sequences that cannot depend on
// each other (their sources end before the batch's first output byte).
// ---------------------------------------------------------------------------

// x mod d for 0 <= x < 2^24, d > 0, via the f32 reciprocal (one correction
// step either way covers its rounding).
__device__ __forceinline__ int small_mod(int x, int d, float rinv) {
    const int q = (int)((float)x * rinv);
    int r = x - q * d;
    if (r < 0) r += d;
    if (r >= d) r -= d;
    return r;
}

// Self-overlapping matches with a period dividing 4 and at most kDecPer bytes
// run per lane in the batch's short-copy step (0: every self-overlapping
// match by the wave; A/B builds with -DBSHUF_DEC_PER=N).
#ifndef BSHUF_DEC_PER
#define BSHUF_DEC_PER 16
#endif
// BSHUF_DEC_FILL1 (A/B builds only, off by default): wave fills of period 1 /
// 2 / 4 from one read and masked dword writes (1: every dword masked, 2: only
// the edge dwords) instead of the byte reads and byte edges below.  Bit-exact,
// but measured slower (round 6, profiles/r06/dec_ab: k_lz4_decode 2 GiB G1
// 0.779 -> 0.875 ms, G2 1.451 -> 1.782, E = 3 1.650 -> 1.951 with form 2).
#ifndef BSHUF_DEC_FILL1
#define BSHUF_DEC_FILL1 0
#endif
constexpr int kDecPer = BSHUF_DEC_PER;
static_assert(kDecPer % 16 == 0 && kDecPer <= 64, "periodic per-lane fills: whole 16-byte pieces, <= 64");

// The whole wave runs one match D[mop, mop+ml) = LZ4 copy from mop-off.
// Non-overlapping (off >= ml): a plain forward copy.  Overlapping (off < ml):
// the output is periodic with period off, byte i = D[mop-off + i mod off], so
// every byte reads the (final) bytes before the match and the interior goes
// out as aligned dwords with no dependency on this match's own stores.
// Offset 0 (accepted by LZ4_decompress_safe, never emitted by a compressor)
// writes zeros, as LZ4's LZ4_write32(op, 0) seed makes it (lz4/lz4.c:501, 2407).
__device__ __forceinline__ void wave_match(lds8* D, int mop, int off, int ml, int lane) {
    if (off >= ml) {
        wave_copy(D, mop - off, D, mop, ml, lane);
        return;
    }
    if (off == 0) {
        for (int i = lane; i < ml; i += kWave) D[mop + i] = 0;
        return;
    }
    const int s = mop - off;
#if BSHUF_DEC_FILL1
    if (off == 1 || off == 2 || off == 4) {
        // a period dividing 4: ONE uniform read of the period's bytes, the
        // pattern dword by v_perm (byte j = D[s + j mod off]), the same value
        // rotated into every aligned dword of the fill, and one masked write
        // per dword -- the edges included, so there are no byte writes and
        // only the one LDS round trip
        const uint32_t w = lds_rd32(D, s);
        const uint32_t v = __builtin_amdgcn_perm(w, w, off == 1 ? 0x00000000u : off == 2 ? 0x01000100u
                                                                                      : 0x03020100u);
        const int a0 = mop & ~3, end = mop + ml;
        // every aligned dword A holds pattern bytes from (A - s) mod off on
        const uint32_t pv = __builtin_amdgcn_alignbit(v, v, 8u * ((uint32_t)(a0 - s) & 3u));
        const int ndw = ((end + 3) >> 2) - (a0 >> 2);
        const uint32_t base = (uint32_t)(uintptr_t)(D + a0);
        for (int c = lane; c < ndw; c += kWave) {
            const int A = a0 + 4 * c;
            const uint32_t m = low_bytes_mask(end - A) & ~low_bytes_mask(mop - A);
            if (BSHUF_DEC_FILL1 == 1 || m != 0xFFFFFFFFu)
                lds_write_masked(base + 4u * (uint32_t)c, m, pv & m);
            else
                *(lds32*)(D + A) = pv;
        }
        return;
    }
#endif
    // v_rcp_f32 (1 ulp): small_mod's one correction step either way and the
    // [2^16/off, 2^16/off + 2) window below both absorb its error (x < 2^17)
    const float rinv = __builtin_amdgcn_rcpf((float)off);
    if (ml <= kWave) {
        // i mod off for i < 64, off < 64: q = (i * inv) >> 16 with inv in
        // [2^16 / off, 2^16 / off + 2) is exact (its error i * 2 / 2^16 < 1/512
        // stays below the gap 1/off to the next integer), on full-rate 24-bit
        // multiplies
        const uint32_t inv = (uint32_t)(65536.0f * rinv) + 1u;
        if (lane < ml) {
            const uint32_t q = __umul24((uint32_t)lane, inv) >> 16;
            D[mop + lane] = D[s + lane - (int)__umul24(q, (uint32_t)off)];
        }
        return;
    }
    const int q0 = (mop + 3) & ~3, q1 = (mop + ml) & ~3;
    if (q1 <= q0) {
        for (int i = lane; i < ml; i += kWave) D[mop + i] = D[s + small_mod(i, off, rinv)];
        return;
    }
    if (off == 1 || off == 2 || off == 4) {
        // period dividing 4 (offset 2 is 40 % of the matches of bit-shuffled
        // int16 data): every aligned dword of the fill is the same rotated
        // pattern dword
        const uint32_t b0 = D[s], b1 = D[s + (off > 1 ? 1 : 0)], b2 = D[s + (off > 2 ? 2 : 0)],
                       b3 = D[s + (off > 2 ? 3 : off - 1)];
        const uint32_t v = off == 1 ? b0 * 0x01010101u
                         : off == 2 ? (b0 | (b1 << 8)) * 0x00010001u
                                    : (b0 | (b1 << 8) | (b2 << 16) | (b3 << 24));
        const int head = q0 - mop, tailn = mop + ml - q1;
        const uint32_t rot = 8u * (uint32_t)(head & (off - 1));
        const uint32_t w = rot ? (v >> rot) | (v << (32u - rot)) : v;
        const int e = lane + (lane < 4 ? 0 : ml - tailn - 4);
        if ((lane < head) | ((lane >= 4) & (lane < 4 + tailn)))
            D[mop + e] = (uint8_t)(v >> (8 * (e & (off - 1))));
        const int nw = (q1 - q0) >> 2;
        lds32* W = (lds32*)(D + q0);
        for (int c = lane; c < nw; c += kWave) W[c] = w;
        return;
    }
    // <= 3 head and <= 3 tail bytes, then the aligned interior dwords
    const int head = q0 - mop, tailn = mop + ml - q1;
    const int e = lane + (lane < 4 ? 0 : ml - tailn - 4);
    if ((lane < head) | ((lane >= 4) & (lane < 4 + tailn)))
        D[mop + e] = D[s + small_mod(e, off, rinv)];
    const int nw = (q1 - q0) >> 2;
    const int step = small_mod(4 * kWave, off, rinv);
    int r = small_mod(head + 4 * lane, off, rinv);
    lds32* W = (lds32*)(D + q0);
    for (int c = lane; c < nw; c += kWave) {
        int r1 = r + 1;
        r1 = r1 >= off ? r1 - off : r1;
        int r2 = r1 + 1;
        r2 = r2 >= off ? r2 - off : r2;
        int r3 = r2 + 1;
        r3 = r3 >= off ? r3 - off : r3;
        W[c] = (uint32_t)D[s + r] | ((uint32_t)D[s + r1] << 8) | ((uint32_t)D[s + r2] << 16) |
               ((uint32_t)D[s + r3] << 24);
        r += step;
        r = r >= off ? r - off : r;
    }
}

// Where phase 2 reads a record from.  LdsRec: the record staged in LDS (byte
// p at C[p]).  GblRec (VAR & 16): straight from the stream in HBM / L2, byte p
// at base + p, so the LDS holds only the decoded block (twice the resident
// waves).  Reads are absolute-aligned dwords clamped to the last dword holding
// a payload byte, so an over-read never leaves the record's pages; the bytes
// past the payload it returns are never used (the scan validated every field).
struct LdsRec {
    const lds8* C;
    __device__ __forceinline__ uint64_t rd64(int p) const { return lds_rd64(C, p); }
    __device__ __forceinline__ void copy16(int sp, lds8* D, int dp, int n) const {
        lane_copy16(C, sp, D, dp, n);
    }
    __device__ __forceinline__ void copyw(int sp, lds8* D, int dp, int n, int lane) const {
        wave_copy(C, sp, D, dp, n, lane);
    }
};


struct GblRec {
    uintptr_t base;   // absolute address of payload byte 0
    uintptr_t lastw;  // the last aligned dword holding a payload byte
    __device__ __forceinline__ uint32_t w(uintptr_t a) const {
        return *(gbl32c*)(a < lastw ? a : lastw);
    }
    __device__ __forceinline__ uint64_t rd64(int p) const {
        const uintptr_t a = base + (uintptr_t)p, al = a & ~(uintptr_t)3;
        const uint32_t s = (uint32_t)(a & 3);
        const uint32_t w0 = w(al), w1 = w(al + 4), w2 = w(al + 8);
        return (uint64_t)__builtin_amdgcn_alignbyte(w1, w0, s) |
               ((uint64_t)__builtin_amdgcn_alignbyte(w2, w1, s) << 32);
    }
    __device__ __forceinline__ void copy16(int sp, lds8* D, int dp, int n) const {
        const uintptr_t a = base + (uintptr_t)sp, al = a & ~(uintptr_t)3;
        lane_put16(w(al), w(al + 4), w(al + 8), w(al + 12), w(al + 16), (uint32_t)(a & 3), D, dp, n);
    }
    __device__ __forceinline__ void copyw(int sp, lds8* D, int dp, int n, int lane) const {
        const gbl8c* S = (const gbl8c*)(base + (uintptr_t)sp);
        if (n <= kWave) {
            if (lane < n) D[dp + lane] = S[lane];
            return;
        }
        const int q0 = (dp + 3) & ~3, q1 = (dp + n) & ~3;
        const int head = q0 - dp, tailn = dp + n - q1;
        const int e = lane + (lane < 4 ? 0 : n - tailn - 4);
        if ((lane < head) | ((lane >= 4) & (lane < 4 + tailn))) D[dp + e] = S[e];
        const int nw = (q1 - q0) >> 2;
        const uintptr_t a0 = base + (uintptr_t)(sp + head);
        const uint32_t sh = (uint32_t)(a0 & 3);
        const uintptr_t al0 = a0 & ~(uintptr_t)3;
        for (int c = lane; c < nw; c += kWave) {
            const uintptr_t al = al0 + 4 * (uintptr_t)c;
            ((lds32*)(D + q0))[c] = __builtin_amdgcn_alignbyte(w(al + 4), w(al), sh);
        }
    }
};

// LZ4 length continuation starting at record byte q, whose next `av` bytes
// (av <= 8) are already in w: returns the added length, advances q.
template <class Src>
__device__ __forceinline__ int read_ext(const Src& Cb, int& q, uint64_t w, int av) {
    int v = 0;
    for (;;) {
        uint64_t inv = ~w;
        if (av < 8) inv &= (1ull << (8 * av)) - 1ull;
        if (inv) {
            const int k = (__ffsll((unsigned long long)inv) - 1) >> 3;
            q += k + 1;
            return v + 255 * k + (int)((w >> (8 * k)) & 255u);
        }
        v += 255 * av;
        q += av;
        w = Cb.rd64(q);
        av = 8;
    }
}

// Phase 2 for one block.  The record payload starts at byte cp of the
// 4-aligned LDS buffer Cb; pos[0..nseq) are its token positions (payload-
// relative, validated by the scan); pos0 is this lane's prefetched pos[lane].
// dg: the diagnostic build's phase clock (fields, literals, matches).
template <bool kInPlace = false, int ABL = 0, class Src>
__device__ __forceinline__ void lz4_exec_block(const Src& Cb, const int cp, lds8* D,
                               const uint32_t* __restrict__ pos, const int nseq, uint32_t pos0,
                               const int lane, DDiag& dg) {
    dg.count(0, (uint32_t)nseq);
    int opb = 0;
    uint32_t pnext = pos0;
    for (int c0 = 0; c0 < nseq; c0 += kWave) {
        const int j = c0 + lane;
        const bool act = j < nseq;
        const int tp = act ? (int)pnext : 0;
        if (c0 + kWave < nseq && c0 + kWave + lane < nseq) pnext = pos[c0 + kWave + lane];
        // ---- sequence fields, lane = sequence: the token and the 7 bytes
        // behind it in one read (a zero-literal sequence's offset and first
        // length bytes are among them), else one more read at the offset
        const int p = cp + tp;
        const uint64_t x = Cb.rd64(p);
        const int tok = (int)(x & 255u);
        int lit = act ? tok >> 4 : 0;
        int q = p + 1;
        if (lit == 15) lit += read_ext(Cb, q, x >> 8, 7);
        const int lsrc = q;
        q += lit;
        int off = 0, ml = 0;
        if (act && j + 1 < nseq) {  // the last sequence has no match
            const int d = q - p;    // bytes of x already behind q
            const uint64_t y = d <= 6 ? x >> (8 * d) : Cb.rd64(q);
            const int yav = d <= 6 ? 8 - d : 8;
            off = (int)(y & 0xFFFFu);
            q += 2;
            ml = tok & 15;
            if (ml == 15) ml += read_ext(Cb, q, y >> 16, yav - 2);
            ml += kMinMatch;
        }
        const int len = lit + ml;
        const int incl = wave_incl_sum(len, lane);
        const int op = opb + incl - len;
        opb += __builtin_amdgcn_readlane(incl, kWave - 1);
        dg.stamp(0);
        // ---- literals: short runs per lane, long runs by the whole wave
        // (ABL: diagnostic-build timing ablations -- 1 no literal copies, 2
        // no match copies; wrong output)
        if constexpr ((ABL & 1) != 0) {
        } else if constexpr (!kInPlace) {
            if (lit > 0 && lit <= 16) Cb.copy16(lsrc, D, op, lit);
            for (uint64_t lm = ballot(lit > 16); lm; lm &= lm - 1) {
                const int l = ffs64(lm);
                Cb.copyw(__builtin_amdgcn_readlane(lsrc, l), D, __builtin_amdgcn_readlane(op, l),
                         __builtin_amdgcn_readlane(lit, l), lane);
            }
        } else {
            // the record sits in the output buffer: copies run in SEQUENCE
            // order -- the short runs between two long ones as one parallel
            // step (all of its reads precede its writes), each long run by the
            // wave -- so no sequence's writes come before an earlier
            // sequence's reads; the scan's margin test keeps every write below
            // every later sequence's record bytes
            uint64_t lm = ballot(lit > 16), done = 0;
            const uint64_t sm = ballot(lit > 0) & ~lm;
            for (;;) {
                const int l = lm ? ffs64(lm) : kWave;
                const uint64_t below = l >= kWave ? ~0ull : ((1ull << l) - 1ull);
                if (sm & below & ~done) {
                    if (__builtin_amdgcn_inverse_ballot_w64(sm & below & ~done)) Cb.copy16(lsrc, D, op, lit);
                }
                if (l >= kWave) break;
                done = below | (1ull << l);
                Cb.copyw(__builtin_amdgcn_readlane(lsrc, l), D, __builtin_amdgcn_readlane(op, l),
                         __builtin_amdgcn_readlane(lit, l), lane);
                lm &= lm - 1;
            }
        }
        dg.stamp(1);
        // ---- matches, in batches of mutually independent sequences
        // A later sequence joins the batch when the bytes its match reads
        // from before its own output ([mop - off, rend), rend = mop - off +
        // min(ml, off): a self-overlapping match makes the rest itself) were
        // all final before the batch started; self-overlapping and long
        // matches run one after another by the wave (coop), short ones per
        // lane.  Every per-lane test is made once per 64 sequences; a batch
        // costs one readlane and one compare, the rest is scalar mask work
        // (inverse ballots turn the masks back into lane predicates).
        const int mop = op + lit;
        const int rend = mop - off + min(ml, off);
        const uint64_t mm = (ABL & 2) ? 0ull : ballot(ml > 0);
        // self-overlapping matches whose period divides 4 (offsets 1, 2, 4;
        // offset 2 is 40 % of the matches of bit-shuffled int16 data) up to
        // kDecPer bytes are periodic fills run by their own lane, 16 bytes
        // per step from one pattern dword, beside the batch's short copies
        const bool per = kDecPer > 0 && off < ml && ml <= kDecPer && (off == 1 || off == 2 || off == 4);
        const uint64_t pm = ballot(per);
        // the wave runs the long and the other self-overlapping matches
        const uint64_t cmask = mm & (ballot(ml > 16) | ballot(off < ml)) & ~pm;
        uint64_t todo = mm;
        while (todo) {
            const int f = ffs64(todo);
            const int opf = __builtin_amdgcn_readlane(mop, f);
            const uint64_t above = ~((2ull << f) - 1ull);  // lanes > f (none for f = 63)
            const uint64_t sm = ballot(rend > opf) & mm & above;
            const uint64_t batch = todo & (sm ? (1ull << ffs64(sm)) - 1ull : ~0ull);
            if constexpr (kDecPer > 0) {
                if (__builtin_amdgcn_inverse_ballot_w64(batch & ~cmask)) {
                    // one set of source reads serves both kinds: a copy's 16
                    // bytes at mop - off, or a fill's period (its first bytes)
                    const int sp = mop - off;
                    const lds32* w = (const lds32*)(D + (sp & ~3));
                    uint32_t x0 = w[0], x1 = w[1], x2 = w[2], x3 = w[3], x4 = w[4];
                    uint32_t sh = (uint32_t)(sp & 3);
                    if (per) {
                        const uint32_t b = __builtin_amdgcn_alignbyte(x1, x0, sh);
                        const uint32_t v = off == 4 ? b : off == 2 ? (b & 0xFFFFu) * 0x00010001u
                                                                   : (b & 0xFFu) * 0x01010101u;
                        x0 = x1 = x2 = x3 = x4 = v;
                        sh = 0;
                    }
                    lane_put16(x0, x1, x2, x3, x4, sh, D, mop, min(ml, 16));
#pragma unroll
                    for (int k = 16; k < kDecPer; k += 16) {
                        // 16 | the period: every later piece is the same pattern
                        if (__builtin_amdgcn_inverse_ballot_w64(batch & pm & ballot(ml > k)))
                            lane_put16(x0, x0, x0, x0, x0, 0u, D, mop + k, min(ml - k, 16));
                    }
                }
            } else {
                if (__builtin_amdgcn_inverse_ballot_w64(batch & ~cmask)) lane_copy16(D, mop - off, D, mop, ml);
            }
            dg.count(1, 1);
            dg.count(2, (uint32_t)__builtin_popcountll(batch & cmask));
            for (uint64_t cm = batch & cmask; cm; cm &= cm - 1) {
                const int l = ffs64(cm);
                wave_match(D, __builtin_amdgcn_readlane(mop, l), __builtin_amdgcn_readlane(off, l),
                           __builtin_amdgcn_readlane(ml, l), lane);
            }
            todo &= ~batch;
        }
        dg.stamp(2);
    }
}

struct DecArgs {
    const uint8_t* in;
    int64_t in_nbytes;
    const uint64_t* offs;
    uint8_t* out;
    int64_t* status;
    long long* bad;  // highest failing block index (init -1)
    Layout L;
    uint32_t maxlen;
    int32_t cap;     // LDS bytes reserved for the decoded block
    uint32_t* seq;   // token positions (k_seq_scan -> lz4_exec_block)
    const Seg* segs; // batch: per-stream table (nullptr: the single stream above)
    const uint32_t* blk_seg;
    int32_t stage_off;  // EK == 0: LDS offset of the output staging block (0: none,
                        // -1: through registers into the block's own LDS)
    int32_t ip_end;     // VAR & 512: the in-place record region ends at this LDS offset
    int64_t blk0, blk1; // k_seq_scan / k_lz4_decode: this launch's blocks [blk0, blk1)
    const int64_t* dlen;  // single stream: length in device memory (in_nbytes = capacity)
};

// The single stream's readable bytes from its device-held length, once per kernel.
__device__ __forceinline__ void resolve_len(DecArgs& a) {
    if (a.dlen) {
        a.in_nbytes = readable_bytes(*a.dlen, a.in_nbytes);
        a.dlen = nullptr;
    }
}

// Where block k lives: its stream's framed bytes, output, token-position area
// and failure word, its element count and whether it is its stream's last.
struct BlockLoc {
    const uint8_t* in;
    int64_t in_nbytes;
    uint8_t* out;       // the block's decoded bytes
    uint32_t* seq;
    long long* bad;
    int m;
    bool last;
};

__device__ __forceinline__ BlockLoc block_loc(const DecArgs& a, int64_t k, int64_t nb, uint32_t s) {
    BlockLoc b;
    if (!a.segs) {
        b.in = a.in;
        b.in_nbytes = a.in_nbytes;
        b.out = a.out + k * (int64_t)a.L.bs * a.L.E;
        b.seq = a.seq;
        b.bad = a.bad;
        b.m = k < a.L.nfull ? a.L.bs : a.L.last;
        b.last = k + 1 >= nb;
    } else {
        const Seg& g = a.segs[s];
        const int64_t local = k - g.first;
        b.in = g.in;
        b.in_nbytes = g.in_nbytes;
        b.out = g.out + local * (int64_t)a.L.bs * a.L.E;
        b.seq = a.seq + g.seq0;
        b.bad = a.bad + s;
        b.m = local < g.nfull ? a.L.bs : g.last;
        b.last = local + 1 >= g.nfull + (g.last ? 1 : 0);
    }
    return b;
}

// Record span [o0, o1) clamped into the stream: an offset the index could not
// resolve (launch_index leaves it at the all-ones sentinel) or a corrupt one
// becomes an empty span at the stream end, which the header check rejects
// (-1001) without reading anything; a span never exceeds the largest record.
__device__ __forceinline__ void clamp_span(int64_t& o0, int64_t& o1, int64_t in_nbytes,
                                           uint32_t maxlen) {
    if (o0 < 0 || o0 > in_nbytes) o0 = in_nbytes;
    if (o1 < 0 || o1 > in_nbytes) o1 = in_nbytes;
    if (o0 > o1) o0 = o1;
    if (o1 > o0 + 4 + (int64_t)maxlen) o1 = o0 + 4 + (int64_t)maxlen;
}

// Byte range [o0, o1) of block k's record ([BE32 c][c bytes]) in the stream.
// Consecutive records are contiguous, so the next offset ends this record;
// the last record is bounded by its worst-case size.
struct Span {
    int64_t o0, o1;
    int64_t scan;  // k_seq_scan's result: sequence count, or the block's error code
    BlockLoc loc;
};

// 16-byte chunks covering a record of an 8 KiB block: (8244 + 30) / 16 / 64 -> 9.
constexpr int kPayIters = 9;

// The in-place decoder prefetches only the first kPayItersIP granule rows
// (5 KiB: every G1/G2 record of typical size) to stay within 96 VGPRs (5
// waves per SIMD); a longer record's remainder is copied when it lands.
constexpr int kPayItersIP = 5;

template <int IT = kPayIters>
struct PayRegsT {
    u32x4 v[IT];
    uint32_t pos;  // token position of sequence `lane` (two-phase path)
};
using PayRegs = PayRegsT<>;

// Record bytes [o0, o1) are read as whole 16-byte granules aligned on the
// absolute address (a granule never crosses a page: the extra bytes at either
// end cannot fault and are never used); they land in LDS at Cbuf + (addr & 15).
__device__ __forceinline__ const gbl128c* span_base(const DecArgs& a, const Span& sp) {
    return g128_aligned_down(sp.loc.in + sp.o0);
}
__device__ __forceinline__ int span_shift(const DecArgs& a, const Span& sp) {
    return (int)((uintptr_t)(sp.loc.in + sp.o0) & 15);
}
__device__ __forceinline__ int span_chunks(const DecArgs& a, const Span& sp) {
    return (span_shift(a, sp) + (int)(sp.o1 - sp.o0) + 15) >> 4;
}

__device__ __forceinline__ bool span_fits(const DecArgs& a, const Span& sp) {
    return span_chunks(a, sp) <= kPayIters * kWave;
}

template <int IT>
__device__ __forceinline__ void issue_pay(PayRegsT<IT>& R, const DecArgs& a, const Span& sp, int lane) {
    const gbl128c* g4 = span_base(a, sp);
    const int nch = span_chunks(a, sp);
#pragma unroll
    for (int it = 0; it < IT; it++) {
        const int c = it * kWave + lane;
        if (c < nch) R.v[it] = g4[c];
    }
    R.pos = sp.loc.seq[sp.o0 / 3 + lane];
}

// Lands the prefetched rows; rows beyond IT (a record longer than the
// prefetch) come straight from global memory.
template <int IT>
__device__ __forceinline__ void land_pay(const PayRegsT<IT>& R, const DecArgs& a, const Span& sp,
                                         lds8* C, int lane) {
    const int nch = span_chunks(a, sp);
#pragma unroll
    for (int it = 0; it < IT; it++) {
        const int c = it * kWave + lane;
        if (c < nch) ((lds128*)C)[c] = R.v[it];
    }
    if (IT * kWave < nch) {
        const gbl128c* g4 = span_base(a, sp);
        for (int c = IT * kWave + lane; c < nch; c += kWave) ((lds128*)C)[c] = g4[c];
    }
}

// Raw offsets of a record, loaded one block before they are turned into a
// Span, so the load's latency is covered by a parse.  Lanes 0 and 1 load
// offs[k] and offs[k+1]: a lane-varying value stays in VGPRs until
// span_from's readlanes (a uniform load would be moved to SGPRs, and waited
// for, right away).
struct OffRegs {
    uint64_t v;
    int64_t k;  // block index
};

__device__ __forceinline__ OffRegs issue_offs(const DecArgs& a, int64_t k, int64_t nb, int lane) {
    OffRegs r;
    r.v = 0;
    r.k = k;
    if (lane < 2) {
        if (k + lane < nb) r.v = a.offs[k + lane];
    } else if (lane == 2) {
        r.v = (uint64_t)a.status[k];  // the scan's verdict
    } else if (lane == 3 && a.segs) {
        r.v = a.blk_seg[k];  // the block's stream (batch)
    }
    return r;
}

__device__ __forceinline__ Span span_from(const DecArgs& a, const OffRegs& r, int64_t nb) {
    auto rl = [&](int l) {
        return (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(r.v >> 32), l) << 32) |
                         (uint32_t)__builtin_amdgcn_readlane((int)r.v, l));
    };
    Span sp;
    sp.loc = block_loc(a, r.k, nb, (uint32_t)__builtin_amdgcn_readlane((int)r.v, 3));
    sp.o0 = rl(0);
    sp.o1 = sp.loc.last ? sp.o0 + 4 + (int64_t)a.maxlen : rl(1);
    sp.scan = rl(2);
    clamp_span(sp.o0, sp.o1, sp.loc.in_nbytes, a.maxlen);
    return sp;
}

// Phase 1: one lane per block.  A 32-byte window of the lane's record lives
// in registers as two absolute-aligned granules (a granule never crosses a
// page; the second is loaded only when it holds payload bytes).
struct GWin {
    int w0;  // payload position of window byte 0
    u32x4 a, b;
};

__device__ __forceinline__ uint32_t gw_byte(GWin& g, const uint8_t* P, int clen, int p) {
    if ((unsigned)(p - g.w0) >= 32u) {
        const uint8_t* ap = P + p;
        g.w0 = p - (int)((uintptr_t)ap & 15);
        const gbl128c* q = g128_aligned_down(ap);
        g.a = q[0];
        if (g.w0 + 16 < clen) g.b = q[1];
    }
    const int t = p - g.w0;
    const u32x4 v = t < 16 ? g.a : g.b;
    const int d = (t >> 2) & 3;
    const uint32_t x = d == 0 ? v.x : (d == 1 ? v.y : (d == 2 ? v.z : v.w));
    return (x >> (8 * (t & 3))) & 255u;
}

// Record header checks shared by both paths: -1001 when the record does not
// fit the stream, -91 for an impossible length.  A length above the LZ4 bound
// is -91 from the header alone, whatever follows it (the host walk stages
// only such a header, and must get the device API's code for the same bytes).
__device__ __forceinline__ int header_status(int64_t clen, int64_t avail, bool last, uint32_t maxlen) {
    if (avail < 4 || clen == 0) return -1000 - 1;  // clen 0: LZ4's srcSize == 0 -> -1
    if (clen < 0 || clen > (int64_t)maxlen) return -91;
    if (clen + 4 > avail) return -1000 - 1;
    if (!last && clen + 4 != avail) return -91;
    return 0;
}

// Byte reader of the scan: the lane's register window.
struct GReader {
    GWin g;
    const uint8_t* P;
    int clen;
    __device__ __forceinline__ uint32_t operator()(int p) { return gw_byte(g, P, clen, p); }
};

// Token positions of one lane's block, four per 16-byte store: entry i sits
// in dword slot (ph + i) & 3 of its absolute 16-byte chunk, and a chunk is
// stored whole once its slot 3 is filled -- unless it begins before the
// block's first entry (that part belongs to the previous block's range), in
// which case its entries go dword by dword, as do the last chunk's at flush.
// A quarter of the scattered position stores (each costs a whole write
// transaction, and on gfx9's in-order vmcnt every store issued before a
// window load is waited for with it).
constexpr int kMxBias = 1 << 14;
// Bytes behind the decoded block reserved for the in-place record (keeps one
// buffer within 7 LDS granules = 8,960 bytes: 18 waves per CU)
constexpr int kInPlaceMargin = 704;
struct SeqOut {
    typedef __attribute__((address_space(1))) uint32_t g32;
    uint32_t* base;
    int ph;  // dword phase of base within its 16-byte chunk
    u32x4 buf;
    int mx = -(1 << 20);  // max over sequences of (output start - token position)
    __device__ __forceinline__ static uint32_t sel(const u32x4 b, int s) {
        return s == 0 ? b.x : (s == 1 ? b.y : (s == 2 ? b.z : b.w));
    }
    __device__ __forceinline__ void put(int i, uint32_t v, int op) {
        mx = max(mx, op - (int)v);
        const int s = (ph + i) & 3;
        buf.x = s == 0 ? v : buf.x;
        buf.y = s == 1 ? v : buf.y;
        buf.z = s == 2 ? v : buf.z;
        buf.w = s == 3 ? v : buf.w;
        if (s == 3) {
            if (i >= 3) {
                *(gbl128*)(base + i - 3) = buf;
            } else {
                for (int j = ph; j < 4; j++) ((g32*)base)[j - ph] = sel(buf, j);
            }
        }
    }
    // entries [0, cnt) put; store those of the unfinished last chunk
    __device__ __forceinline__ void flush(int cnt) {
        const int s_end = (ph + cnt) & 3;  // slots [lo, s_end) of the last chunk pending
        if (cnt <= 0 || s_end == 0) return;
        const int lo = cnt < s_end ? ph : 0;
        const int i0 = cnt - (s_end - lo);
        for (int j = lo; j < s_end; j++) ((g32*)base)[i0 + j - lo] = sel(buf, j);
    }
};

// status[k] = number of sequences, or the block's final error code (r - 1000
// for an LZ4 failure, -91 when the block does not decode to exactly n bytes).
// seq[offs[k]/3 + i] = payload position of sequence i's token (a sequence
// takes >= 3 record bytes, so the per-block ranges are disjoint).
__global__ __launch_bounds__(256) void k_seq_scan(DecArgs a, int64_t nb) {
    const int64_t k = a.blk0 + (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (k >= a.blk1) return;
    resolve_len(a);
    const BlockLoc loc = block_loc(a, k, nb, a.segs ? a.blk_seg[k] : 0u);
    const int n = loc.m * a.L.E;
    int64_t o0 = (int64_t)a.offs[k];
    int64_t o1 = !loc.last ? (int64_t)a.offs[k + 1] : o0 + 4 + (int64_t)a.maxlen;
    clamp_span(o0, o1, loc.in_nbytes, a.maxlen);
    const int64_t avail = o1 - o0;
    const int64_t clen = avail >= 4 ? (int64_t)(int32_t)be32_global(loc.in + o0) : 0;
    int64_t st = header_status(clen, avail, loc.last, a.maxlen);
    if (st == 0) {
        int cnt = 0;
        GReader rd;
        rd.g.w0 = -(1 << 30);
        rd.P = loc.in + o0 + 4;
        rd.clen = (int)clen;
        SeqOut out;
        out.base = loc.seq + o0 / 3;
        out.ph = (int)(((uintptr_t)out.base >> 2) & 3);
        out.buf = u32x4{0u, 0u, 0u, 0u};
        const int r = scan_block(rd, (int)clen, n, out, cnt);
        out.flush(cnt);  // a rejected block's positions are never read
        st = r < 0 ? (int64_t)r - 1000 : (r == n ? (int64_t)cnt : -91);
        // valid: bits 32..47 carry max(output start - token position) + 2^14,
        // the in-place decoder's safety margin test (kInPlace below)
        if (st >= 0) st |= (int64_t)min(max(out.mx + kMxBias, 0), 0xFFFF) << 32;
    }
    a.status[k] = st;
}

// Blocks above max_lds_decode_bytes: one WAVE per block runs the same scan
// (a lane-per-block walk of a ~100 KiB record pays a global round trip every
// 32 bytes).  All 64 lanes step the state machine in lockstep on the same
// bytes -- so the control flow stays uniform -- and the record streams
// through an LDS window, refilled 8 KiB at a time by the whole wave with
// coalesced 16-byte loads; only lane 0 stores the token positions.
constexpr int kScanWin = 8192;
struct WaveReader {
    const uint8_t* P;
    int clen;
    int w0;  // record position of window byte 0
    lds8* W;
    int lane;
    __device__ __forceinline__ uint32_t operator()(int p) {
        if ((unsigned)(p - w0) >= (unsigned)kScanWin) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            const uintptr_t ap = (uintptr_t)(P + p);
            w0 = p - (int)(ap & 15);
            const gbl128c* q = g128_aligned_down(P + p);
            for (int c = lane; c < kScanWin / 16; c += kWave)
                if (w0 + 16 * c < clen) ((lds128*)W)[c] = q[c];
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
        }
        return W[p - w0];
    }
};
struct SeqOutLane0 {
    SeqOut o;
    int lane;
    __device__ __forceinline__ void put(int i, uint32_t v, int op) {
        if (lane == 0) o.put(i, v, op);
    }
};

// BSHUF_SCAN_BIG_LDS=0 (default): the window lives in registers instead --
// 1 KiB of the record in four VGPRs (lane l, dword d: bytes 4l + 256d) plus the
// next 1 KiB already in flight -- and a byte is one v_readlane of a uniform
// lane, so the whole walk runs on the scalar unit without an LDS round trip per
// byte, and with no LDS the wave count per CU is not capped by the window.
#ifndef BSHUF_SCAN_BIG_LDS
#define BSHUF_SCAN_BIG_LDS 1
#endif
#ifndef BSHUF_SCAN_BIG_PF  // 1: the next 1 KiB loaded ahead into four more VGPRs
#define BSHUF_SCAN_BIG_PF 0
#endif
struct RegWin {
    uint32_t d0, d1, d2, d3;
};
struct WaveRegReader {
    const uint8_t* P;
    int clen;
    int w0;  // record position of window byte 0 (P + w0 is 4-byte aligned)
    int lane;
    RegWin cur, nxt;
    // dwords wholly past the record read as 0; one that holds a record byte
    // never crosses a page (aligned), and bytes before P are the header's
    __device__ __forceinline__ RegWin load(int base) const {
        RegWin r{0u, 0u, 0u, 0u};
        const int b = base + 4 * lane;
        const gbl32c* q = (const gbl32c*)(P + b);
        if (b < clen) r.d0 = q[0];
        if (b + 256 < clen) r.d1 = q[64];
        if (b + 512 < clen) r.d2 = q[128];
        if (b + 768 < clen) r.d3 = q[192];
        return r;
    }
    __device__ __forceinline__ uint32_t operator()(int p) {
        int rel = p - w0;
        if ((unsigned)rel >= 1024u) {
#if BSHUF_SCAN_BIG_PF
            if ((unsigned)(rel - 1024) < 1024u) {
                cur = nxt;
                w0 += 1024;
            } else {
                w0 = p - (int)((uintptr_t)(P + p) & 3);
                cur = load(w0);
            }
            nxt = load(w0 + 1024);
#else
            w0 = p - (int)((uintptr_t)(P + p) & 3);
            cur = load(w0);
#endif
            // wait for the window here, once: redefined by the asm, its
            // registers are no longer pending loads at the reads below (which
            // would otherwise each wait for every load and store in flight)
            asm volatile("" : "+v"(cur.d0), "+v"(cur.d1), "+v"(cur.d2), "+v"(cur.d3));
            rel = p - w0;
        }
        const int d = rel >> 8;
        // scalar selects of four readlanes: a vector select of the fields
        // would become a variable index into the reader (kept in memory then)
        const int li = (rel >> 2) & 63;
        const uint32_t x0 = (uint32_t)__builtin_amdgcn_readlane((int)cur.d0, li);
        const uint32_t x1 = (uint32_t)__builtin_amdgcn_readlane((int)cur.d1, li);
        const uint32_t x2 = (uint32_t)__builtin_amdgcn_readlane((int)cur.d2, li);
        const uint32_t x3 = (uint32_t)__builtin_amdgcn_readlane((int)cur.d3, li);
        const uint32_t x = d == 0 ? x0 : (d == 1 ? x1 : (d == 2 ? x2 : x3));
        return (x >> (8 * (rel & 3))) & 255u;
    }
};

__global__ __launch_bounds__(64) void k_seq_scan_big(DecArgs a, int64_t nb) {
#if BSHUF_SCAN_BIG_LDS
    __shared__ __attribute__((aligned(16))) uint8_t win[kScanWin];
#endif
    const int lane = threadIdx.x;
    const int64_t k = blockIdx.x;
    resolve_len(a);
    const BlockLoc loc = block_loc(a, k, nb, a.segs ? a.blk_seg[k] : 0u);
    const int n = loc.m * a.L.E;
    int64_t o0 = (int64_t)a.offs[k];
    int64_t o1 = !loc.last ? (int64_t)a.offs[k + 1] : o0 + 4 + (int64_t)a.maxlen;
    clamp_span(o0, o1, loc.in_nbytes, a.maxlen);
    const int64_t avail = o1 - o0;
    // the same for every lane (a divergent clen would take the whole walk onto
    // the vector unit with exec masks)
    const int64_t clen =
        avail >= 4 ? (int64_t)__builtin_amdgcn_readfirstlane((int)be32_global(loc.in + o0)) : 0;
    int64_t st = header_status(clen, avail, loc.last, a.maxlen);
    if (st == 0) {
        int cnt = 0;
#if BSHUF_SCAN_BIG_LDS
        WaveReader rd{loc.in + o0 + 4, (int)clen, -(1 << 30), to_lds(win), lane};
#else
        WaveRegReader rd;
        rd.P = loc.in + o0 + 4;
        rd.clen = (int)clen;
        rd.w0 = -(1 << 30);
        rd.lane = lane;
        rd.cur = rd.nxt = RegWin{0u, 0u, 0u, 0u};
#endif
        SeqOutLane0 out;
        out.lane = lane;
        out.o.base = loc.seq + o0 / 3;
        out.o.ph = (int)(((uintptr_t)out.o.base >> 2) & 3);
        out.o.buf = u32x4{0u, 0u, 0u, 0u};
        const int r = scan_block(rd, (int)clen, n, out, cnt);
        if (lane == 0) out.o.flush(cnt);
        st = r < 0 ? (int64_t)r - 1000 : (r == n ? (int64_t)cnt : -91);
    }
    if (lane == 0) a.status[k] = st;
}

// VAR & 32: one dword of every 128-byte line of a record, loaded two blocks
// ahead so that phase 2's reads of it hit L2; the values are never used.
struct Touch {
    uint32_t v0, v1;
};
__device__ __forceinline__ Touch touch_record(const Span& sp, int lane) {
    Touch t{0u, 0u};
    const int64_t len = sp.o1 - sp.o0;
    const uintptr_t b = (uintptr_t)(sp.loc.in + sp.o0) & ~(uintptr_t)127;
    const uintptr_t e = (uintptr_t)(sp.loc.in + sp.o1);
    const uintptr_t a0 = b + 128 * (uintptr_t)lane, a1 = a0 + 128 * kWave;
    if (len > 0 && a0 < e) t.v0 = *(gbl32c*)a0;
    if (len > 0 && a1 < e) t.v1 = *(gbl32c*)a1;
    return t;
}
__device__ __forceinline__ void touch_done(const Touch& t) {
    asm volatile("" : : "v"(t.v0), "v"(t.v1));
}

// Returns this lane's token position of the record (two-phase path).
template <int IT>
__device__ __forceinline__ uint32_t land_record(const PayRegsT<IT>& R, bool in_regs, const DecArgs& a,
                                                const Span& sp, lds8* Cbuf, int lane) {
    if (in_regs) {
        land_pay(R, a, sp, Cbuf, lane);
        return R.pos;
    }
    const gbl128c* g4 = span_base(a, sp);
    const int nch = span_chunks(a, sp);
    for (int c = lane; c < nch; c += kWave) ((lds128*)Cbuf)[c] = g4[c];
    return sp.loc.seq[sp.o0 / 3 + lane];
}

// Persistent: workgroup w decodes blocks w, w+G, ...  Software pipeline, per
// iteration: parse block i; land record i+1 (its loads were issued one whole
// parse earlier); issue the offsets of i+3 and the record of i+2; store block
// i.  Every wait on HBM therefore follows a parse, so neither load latency nor
// the completion of the previous block's stores (gfx9 counts loads and stores
// on one in-order vmcnt) stalls the wave.
template <int EK, int VAR>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu((VAR & 512) ? (EK == 0 ? 4 : 5) : 1)))
void k_lz4_decode(DecArgs a, int64_t nb) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int lane = threadIdx.x;
    const int E = EK ? EK : a.L.E;
    lds8* D = to_lds(smem);             // decoded (bit-shuffled) block
    lds8* Cbuf = to_lds(smem) + a.cap + 16;  // record bytes, 16-aligned base
    // VAR & 16: phase 2 reads the record from global memory (no LDS copy)
    constexpr bool kG = (VAR & 16) != 0;
    // VAR & 512 (default): the record lands IN PLACE, at the end of the
    // decoded block's own LDS buffer (LZ4 in-place decompression).  Sequence j
    // writes output [op_j, ...) below its own token position, which the scan
    // proved per block (bits 32..47 of its verdict: max(op_j - tp_j)); a
    // block that fails the test reads its record from global memory instead.
    // One ~8.9 KiB buffer per wave: every record read is an LDS read and the
    // occupancy of the global-read decoder stays.
    constexpr bool kIP = (VAR & 512) != 0;
    auto cbuf_of = [&](const Span& sp) -> lds8* {
        return kIP ? to_lds(smem) + a.ip_end - 16 * span_chunks(a, sp) : Cbuf;
    };
    const int64_t stride = gridDim.x;
    int64_t blk = a.blk0 + blockIdx.x;
    const int64_t end = a.blk1;  // this launch's blocks [blk0, end); nb: the whole stream(s)
    if (blk >= end) return;
    resolve_len(a);

    PayRegsT<kIP ? kPayItersIP : kPayIters> R;
    // in place: every record is prefetched (partly, when long) into R
    auto fits = [&](const Span& sp) { return kIP || span_fits(a, sp); };
    Span cur = span_from(a, issue_offs(a, blk, nb, lane), nb);
    uint32_t cur_pos;
    if constexpr (kG) {
        cur_pos = cur.loc.seq[cur.o0 / 3 + lane];
    } else {
        const bool in_regs = fits(cur);
        if (in_regs) issue_pay(R, a, cur, lane);
        cur_pos = land_record(R, in_regs, a, cur, cbuf_of(cur), lane);
    }
    int64_t next = blk + stride;
    Span nxt = {};
    bool nxt_in_regs = false;
    uint32_t pref_pos = 0;  // kG: token position of block `next`, loaded a parse early
    constexpr bool kTouch = (VAR & 32) != 0;
    Touch t_cur{0u, 0u}, t_nxt{0u, 0u}, t_nxt2{0u, 0u};
    if (next < end) {
        nxt = span_from(a, issue_offs(a, next, nb, lane), nb);
        if constexpr (kG) {
            pref_pos = nxt.loc.seq[nxt.o0 / 3 + lane];
            if constexpr (kTouch) t_nxt = touch_record(nxt, lane);
        } else {
            nxt_in_regs = fits(nxt);
            if (nxt_in_regs) issue_pay(R, a, nxt, lane);
        }
    }
    OffRegs O{0, 0};
    if (next + stride < end) O = issue_offs(a, next + stride, nb, lane);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    // diagnostic build: 0 fields, 1 literals, 2 matches, 3 inverse transpose
    // + stores, 4 next record landing + loads ahead, 5 the rest
    DDiag dg;

    for (;;) {
        dg.stamp(5);
        const int P = cur.loc.m / 8;
        const int cp = span_shift(a, cur);
        lds8* const CB = cbuf_of(cur);
        const lds8* C = CB + cp;
        // the scan's verdict: sequence count, or the block's error code
        int status = 0, clen = 0;
        if (cur.scan < 0) {
            status = (int)cur.scan;
        } else if constexpr (kG) {
            if constexpr (kTouch) touch_done(t_cur);  // this block's (issued two blocks ago)
            const uint8_t* rec = cur.loc.in + cur.o0;
            clen = (int)be32_global(rec);
            const uintptr_t b0 = (uintptr_t)(rec + 4);
            const GblRec src{b0, (b0 + (uintptr_t)clen - 1) & ~(uintptr_t)3};
            if (!(VAR & 64))
                lz4_exec_block(src, 0, D, cur.loc.seq + cur.o0 / 3, (int)cur.scan, cur_pos, lane, dg);
        } else {
            clen = (int)(((uint32_t)C[0] << 24) | ((uint32_t)C[1] << 16) | ((uint32_t)C[2] << 8) | C[3]);
            const int mx = (int)((cur.scan >> 32) & 0xFFFF) - kMxBias;
            if (!kIP || mx <= (int)(CB - D) + cp + 4) {
                if (!(VAR & 64))
                    lz4_exec_block<kIP, (VAR >> 10) & 3>(LdsRec{CB}, cp + 4, D, cur.loc.seq + cur.o0 / 3,
                                        (int)cur.scan, cur_pos, lane, dg);
            } else {
                // too little room to decode in place: the record from L2
                const uintptr_t b0 = (uintptr_t)(cur.loc.in + cur.o0 + 4);
                const GblRec src{b0, (b0 + (uintptr_t)clen - 1) & ~(uintptr_t)3};
                if (!(VAR & 64))
                    lz4_exec_block(src, 0, D, cur.loc.seq + cur.o0 / 3, (int)cur.scan, cur_pos, lane, dg);
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        // the next record replaces this one in LDS; then the loads two ahead
        const int64_t nn = next + stride;
        Span nxt2 = {};
        bool nxt2_in_regs = false;
        uint32_t nxt_pos = 0;
        if (next < end) {
            if constexpr (kG) {
                nxt_pos = pref_pos;
                if (nn < end) {
                    nxt2 = span_from(a, O, nb);
                    if (nn + stride < end) O = issue_offs(a, nn + stride, nb, lane);
                    pref_pos = nxt2.loc.seq[nxt2.o0 / 3 + lane];
                    if constexpr (kTouch) t_nxt2 = touch_record(nxt2, lane);
                }
            } else if constexpr (!kIP) {
                nxt_pos = land_record(R, nxt_in_regs, a, nxt, Cbuf, lane);
                if (nn < end) {
                    nxt2 = span_from(a, O, nb);
                    if (nn + stride < end) O = issue_offs(a, nn + stride, nb, lane);
                    nxt2_in_regs = fits(nxt2);
                    if (nxt2_in_regs) issue_pay(R, a, nxt2, lane);
                }
            }
        }
        if (status != 0) {
            if (lane == 0) atomicMax(cur.loc.bad, (long long)blk);
        } else if (!(VAR & 8)) {
            uint8_t* dst = cur.loc.out;
            if constexpr (EK != 0) {
                // four groups per lane (EK <= 4; 8-byte elements would hold
                // 192 registers): one LDS dword per plane, the bit-sliced
                // transpose of untranspose4, 32*EK contiguous bytes out.
                // (Reordering the groups through LDS for fully coalesced
                // stores sped the store path up -- 0.94 -> 0.60 ms without
                // sequence execution, 2 GiB G1 -- but slowed the whole kernel
                // 2-8 %: the decode is issue-bound, not store-bound.)
                const int P4 = (EK <= 4 && (P & 3) == 0) ? P >> 2 : 0;
                const lds32* D32 = (const lds32*)D;
                for (int q = lane; q < P4; q += kWave) {
                    uint32_t x[8 * EK];
#pragma unroll
                    for (int r = 0; r < 8 * EK; r++) x[r] = D32[r * P4 + q];
                    untranspose4_rows<EK>(x);
                    // global (not flat) stores: a flat store also counts in
                    // lgkmcnt, so the next LDS wait would wait for it too
                    gbl128* o4 = (gbl128*)(dst + (int64_t)q * 32 * EK);
#pragma unroll
                    for (int v = 0; v < 2 * EK; v++)
                        o4[v] = u32x4{untranspose4_word<EK>(x, 4 * v), untranspose4_word<EK>(x, 4 * v + 1),
                                      untranspose4_word<EK>(x, 4 * v + 2), untranspose4_word<EK>(x, 4 * v + 3)};
                }
                for (int g = (P4 ? P : lane); g < P; g += kWave) {
                    uint32_t w[2 * EK];
#pragma unroll
                    for (int i = 0; i < 2 * EK; i++) w[i] = 0;
#pragma unroll
                    for (int b = 0; b < EK; b++) {
                        uint64_t v = 0;
#pragma unroll
                        for (int j = 0; j < 8; j++) v |= (uint64_t)D[(8 * b + j) * P + g] << (8 * j);
                        scatter_byte_plane<EK>(w, b, tr8x8(v));
                    }
                    store_group<EK>(dst + (int64_t)g * 8 * EK, w);
                }
            } else if (a.stage_off < 0) {
                // any element size, blocks of <= 8 KiB (every default block
                // size): the inverse transpose of all the block's (group,
                // byte) items into registers (16 per lane), then their bytes
                // back over the block's own LDS in raw element order, then
                // coalesced 8-byte stores.  No staging buffer: the decoder
                // keeps 18 resident waves per CU (a staged 8 KiB block needs
                // 14 LDS granules instead of 7: 9 waves).
                constexpr int kRegItems = 8192 / 8 / kWave;
                const uint32_t magic = (uint32_t)((0x100000000ull + (uint64_t)E - 1) / (uint64_t)E);
                const int items = P * E;  // 8-byte words of the block, <= 1024
                uint64_t v[kRegItems];
#pragma unroll
                for (int r = 0; r < kRegItems; r++) {
                    const int i = lane + kWave * r;
                    v[r] = 0;
                    if (i < items) {
                        const int g = (int)__umulhi((uint32_t)i, magic), b = i - g * E;
                        uint64_t x = 0;
#pragma unroll
                        for (int j = 0; j < 8; j++) x |= (uint64_t)D[(8 * b + j) * P + g] << (8 * j);
                        v[r] = tr8x8(x);
                    }
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
#pragma unroll
                for (int r = 0; r < kRegItems; r++) {
                    const int i = lane + kWave * r;
                    if (i < items) {
                        const int g = (int)__umulhi((uint32_t)i, magic), b = i - g * E;
                        lds8* y = D + 8 * g * E + b;
#pragma unroll
                        for (int k = 0; k < 8; k++) y[k * E] = (uint8_t)(v[r] >> (8 * k));
                    }
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                for (int i = lane; i < items; i += kWave) ((gbl64*)dst)[i] = ((const lds64v*)D)[i];
            } else if (a.stage_off) {
                // any element size: inverse transpose into an LDS staging
                // block, then coalesced 8-byte stores (outputs 8-aligned)
                lds8* S = to_lds(smem) + a.stage_off;
                const uint32_t magic = (uint32_t)((0x100000000ull + (uint64_t)E - 1) / (uint64_t)E);
                for (int i = lane; i < P * E; i += kWave) {
                    const int g = (int)__umulhi((uint32_t)i, magic), b = i - g * E;
                    uint64_t v = 0;
#pragma unroll
                    for (int j = 0; j < 8; j++) v |= (uint64_t)D[(8 * b + j) * P + g] << (8 * j);
                    v = tr8x8(v);
                    lds8* y = S + 8 * g * E + b;
#pragma unroll
                    for (int k = 0; k < 8; k++) y[k * E] = (uint8_t)(v >> (8 * k));
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                const int nw = P * E;  // 8-byte words of the block
                for (int i = lane; i < nw; i += kWave) {
                    ((gbl64*)dst)[i] = ((const lds64v*)S)[i];
                }
            } else {
                for (int i = lane; i < P * E; i += kWave) {
                    const int g = i / E, b = i - g * E;
                    uint64_t v = 0;
#pragma unroll
                    for (int j = 0; j < 8; j++) v |= (uint64_t)D[(8 * b + j) * P + g] << (8 * j);
                    v = tr8x8(v);
#pragma unroll
                    for (int k = 0; k < 8; k++)
                        ((gbl8*)dst)[(int64_t)(8 * g + k) * E + b] = (uint8_t)(v >> (8 * k));
                }
            }
        }
        dg.stamp(3);
        if (lane == 0) a.status[blk] = status == 0 ? (int64_t)clen + 4 : (int64_t)status;
        if constexpr (kIP) {
            // the decoded block has left LDS: the next record lands in place,
            // then the loads two ahead
            if (next < end) {
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                nxt_pos = land_record(R, nxt_in_regs, a, nxt, cbuf_of(nxt), lane);
                if (nn < end) {
                    nxt2 = span_from(a, O, nb);
                    if (nn + stride < end) O = issue_offs(a, nn + stride, nb, lane);
                    nxt2_in_regs = fits(nxt2);
                    if (nxt2_in_regs) issue_pay(R, a, nxt2, lane);
                }
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        dg.stamp(4);
        dg.count(3, 1);
        if (next >= end) break;
        blk = next;
        cur = nxt;
        cur_pos = nxt_pos;
        next = nn;
        nxt = nxt2;
        nxt_in_regs = nxt2_in_regs;
        if constexpr (kTouch) {
            t_cur = t_nxt;
            t_nxt = t_nxt2;
        }
    }
    dg.flush(lane);
}

// Result: bytes consumed, or the error of the LAST failing block (the
// sequential reference keeps overwriting err, src/bitshuffle_core.c:1905).
// Also copies the raw tail (whose position is only known from the index).
// A device-held stream length (dlen) that is negative is an upstream error
// (the compress result word of a chained call): it becomes the result as is.
__global__ __launch_bounds__(256) void k_decode_finish(const int64_t* __restrict__ status,
                                                       const uint64_t* __restrict__ offs,
                                                       int64_t nblocks, const long long* bad,
                                                       const int64_t* idx_err, const uint8_t* in,
                                                       int64_t in_nbytes, uint8_t* tail_dst,
                                                       int64_t tail, int64_t* result,
                                                       const int64_t* dlen) {
    if (dlen) {
        const int64_t d = *dlen;
        if (d < 0) {
            if (threadIdx.x == 0) *result = d;
            return;
        }
        in_nbytes = readable_bytes(d, in_nbytes);
    }
    const long long last_bad = *bad;
    const int64_t end = nblocks ? (int64_t)offs[nblocks - 1] + status[nblocks - 1] : 0;
    const bool idx_bad = idx_err && *idx_err != 0;
    const bool ok = last_bad < 0 && !idx_bad && end + tail <= in_nbytes;
    if (ok)
        for (int64_t i = threadIdx.x; i < tail; i += blockDim.x) tail_dst[i] = in[end + i];
    if (threadIdx.x == 0) {
        if (last_bad >= 0)
            *result = status[last_bad];
        else if (!ok)
            *result = -91;
        else
            *result = end + tail;
    }
}

// Blocks above max_lds_decode_bytes: one wave per block executes the
// sequences k_seq_scan validated (token positions in seq, verdict in status)
// into the block's slice of the global scratch, the same way lz4_exec_block
// does in LDS: 64 sequences decoded at once, a prefix sum places them, all
// literal runs copied in parallel, the matches in batches of sequences that
// cannot depend on each other.  The output is global memory, so a
// workgroup-scope fence (the stores complete; the CU's L1 is write-through)
// separates every batch from the next one that may read it.
__device__ __forceinline__ void gbl_fence() { __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup"); }

// the whole wave runs one match D[mop, mop+ml) from mop-off (LZ4 semantics;
// offset 0 writes zeros, lz4/lz4.c:501, 2407)
__device__ __forceinline__ void gbl_match(gbl8* D, int mop, int off, int ml, int lane) {
    if (off == 0) {
        for (int i = lane; i < ml; i += kWave) D[mop + i] = 0;
    } else if (off >= ml) {
        for (int i = lane; i < ml; i += kWave) D[mop + i] = D[mop - off + i];
    } else {
        const float rinv = 1.0f / (float)off;
        for (int i = lane; i < ml; i += kWave) D[mop + i] = D[mop - off + small_mod(i, off, rinv)];
    }
}

__global__ __launch_bounds__(64) void k_lz4_exec_big(const uint8_t* __restrict__ in,
                                                      const uint64_t* __restrict__ offs,
                                                      int64_t* __restrict__ status,
                                                      const uint32_t* __restrict__ seq, Layout L,
                                                      uint8_t* __restrict__ shuf, long long* bad) {
    const int lane = threadIdx.x;
    const int64_t k = blockIdx.x;
    const int64_t st = status[k];
    if (st < 0) {
        if (lane == 0) atomicMax(bad, (long long)k);
        return;
    }
    const int64_t o0 = (int64_t)offs[k];
    const uint8_t* rec = in + o0;
    const int clen = (int)be32_global(rec);
    const uintptr_t b0 = (uintptr_t)(rec + 4);
    const GblRec Cb{b0, (b0 + (uintptr_t)clen - 1) & ~(uintptr_t)3};
    const gbl8c* P = (const gbl8c*)b0;
    gbl8* D = (gbl8*)(shuf + k * (int64_t)L.bs * L.E);
    const uint32_t* pos = seq + o0 / 3;
    const int nseq = (int)st;
    int opb = 0;
    for (int c0 = 0; c0 < nseq; c0 += kWave) {
        const int j = c0 + lane;
        const bool act = j < nseq;
        const int p = act ? (int)pos[j] : 0;
        // ---- sequence fields, lane = sequence (as lz4_exec_block)
        const uint64_t x = Cb.rd64(p);
        const int tok = (int)(x & 255u);
        int lit = act ? tok >> 4 : 0;
        int q = p + 1;
        if (lit == 15) lit += read_ext(Cb, q, x >> 8, 7);
        const int lsrc = q;
        q += lit;
        int off = 0, ml = 0;
        if (act && j + 1 < nseq) {
            const int d = q - p;
            const uint64_t y = d <= 6 ? x >> (8 * d) : Cb.rd64(q);
            const int yav = d <= 6 ? 8 - d : 8;
            off = (int)(y & 0xFFFFu);
            q += 2;
            ml = tok & 15;
            if (ml == 15) ml += read_ext(Cb, q, y >> 16, yav - 2);
            ml += kMinMatch;
        }
        const int len = lit + ml;
        const int incl = wave_incl_sum(len, lane);
        const int op = opb + incl - len;
        opb += __builtin_amdgcn_readlane(incl, kWave - 1);
        // ---- literals (record -> disjoint output ranges): short runs per
        // lane, long runs by the whole wave
        if (lit > 0 && lit <= 16)
            for (int i = 0; i < lit; i++) D[op + i] = P[lsrc + i];
        for (uint64_t lm = ballot(lit > 16); lm; lm &= lm - 1) {
            const int l = ffs64(lm);
            const int o = __builtin_amdgcn_readlane(op, l), sp = __builtin_amdgcn_readlane(lsrc, l);
            const int nl = __builtin_amdgcn_readlane(lit, l);
            for (int i = lane; i < nl; i += kWave) D[o + i] = P[sp + i];
        }
        gbl_fence();
        // ---- matches, in batches of mutually independent sequences
        const int mop = op + lit;
        uint64_t todo = ballot(ml > 0);
        while (todo) {
            const int f = ffs64(todo);
            const int opf = __builtin_amdgcn_readlane(mop, f);
            const bool stop = lane > f && ml > 0 && (off < ml || mop - off + ml > opf);
            const uint64_t sm = ballot(stop);
            const int g = sm ? ffs64(sm) : kWave;
            const bool inb = lane >= f && lane < g && ml > 0;
            const bool coop = inb && (ml > 16 || off < ml);
            if (inb && !coop)
                for (int i = 0; i < ml; i++) D[mop + i] = D[mop - off + i];
            for (uint64_t cm = ballot(coop); cm; cm &= cm - 1) {
                const int l = ffs64(cm);
                gbl_match(D, __builtin_amdgcn_readlane(mop, l), __builtin_amdgcn_readlane(off, l),
                          __builtin_amdgcn_readlane(ml, l), lane);
            }
            gbl_fence();
            todo &= g >= kWave ? 0ull : (~0ull << g);
        }
    }
    if (lane == 0) status[k] = (int64_t)clen + 4;
}

}  // namespace

hipError_t launch_exec_big(const uint8_t* in, const Layout& L, const DecodeBufs& b, uint8_t* shuf,
                           hipStream_t s) {
    const int64_t nb = L.nblocks();
    if (nb == 0) return hipSuccess;
    ProfScope prof("k_lz4_exec_big", s);
    hipLaunchKernelGGL(k_lz4_exec_big, dim3((unsigned)nb), dim3(kWave), 0, s, in, b.offs, b.status, b.seq,
                       L, shuf, b.bad);
    return hipGetLastError();
}

int64_t index_chunk_bytes(const Layout& L) {
    const int64_t foot = 4 + lz4_bound(L.bs * L.E);
    int64_t ch = 128 * 1024;
    while (ch < 2 * foot) ch *= 2;
    return ch;
}

size_t decode_scan_tmp_bytes(int64_t nchunks) {
    size_t bytes = 0;
    (void)hipcub::DeviceScan::ExclusiveSum(nullptr, bytes, (const uint64_t*)nullptr, (uint64_t*)nullptr,
                                     (int)(nchunks + 1));
    return bytes;
}

namespace {

// LDS of k_idx_exits: the candidate window of the largest record (+ 3 bytes
// of the last header, + 16-byte alignment slack), capped at kIdxWinMax (a
// larger window reads its candidates from global memory instead).
int64_t idx_win_lds(uint32_t maxlen) {
    const int64_t w = ((4 + (int64_t)maxlen + 3 + 16 + 64) + 15) & ~(int64_t)15;
    return w < kIdxWinMax ? w : kIdxWinMax;
}
// Candidates per k_idx_exits workgroup: the whole window when it fits the LDS
// budget, else slices that do (staged in LDS like a small window).
int64_t idx_wsub(uint32_t maxlen) {
    const int64_t W = 4 + (int64_t)maxlen;
    return idx_win_lds(maxlen) < kIdxWinMax ? W : kIdxWinMax - 128;
}

// Index rebuild over nch chunks (of one stream, or of every stream of a batch).
hipError_t index_impl(const IdxArgs& x, int64_t nb, int64_t nch, int nsegs, const DecodeBufs& b,
                      hipStream_t s) {
    hipError_t e = dev_fill(b.idx_err, 0, sizeof(int64_t) * (size_t)nsegs, s);
    if (e != hipSuccess || nb == 0) return e;
    // offsets a broken chain never reaches stay at the all-ones sentinel
    // (clamp_span turns them into -1001 without reading the stream)
    e = dev_fill(b.offs, 0xFF, (size_t)nb * sizeof(uint64_t), s);
    if (e != hipSuccess || nch == 0) return e;
    {
        ProfScope prof("k_idx_exits", s);
        const size_t lds = (size_t)x.win_lds + sizeof(uint32_t) * kIdxCandCap;
        if (lds > 65536) {
            e = hipFuncSetAttribute(reinterpret_cast<const void*>(k_idx_exits),
                                    hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
            if (e != hipSuccess) return e;
        }
        const int64_t ny = (x.W + x.wsub - 1) / x.wsub;
        if (ny > 1) {
            // b.cnt (the walk's counts, written later) holds the maxima meanwhile
            e = dev_fill(b.exits, 0x7F, (size_t)nch * sizeof(int64_t), s);
            if (e == hipSuccess) e = dev_fill(b.cnt, 0xFF, (size_t)nch * sizeof(int64_t), s);
            if (e != hipSuccess) return e;
        }
        hipLaunchKernelGGL(k_idx_exits, dim3((unsigned)nch, (unsigned)ny), dim3(kWave), lds, s, x, b.exits,
                           (int64_t*)b.cnt);
        if (ny > 1)
            hipLaunchKernelGGL(k_idx_exits_join, dim3((unsigned)((nch + 255) / 256)), dim3(256), 0, s, b.exits,
                               (const int64_t*)b.cnt, nch);
    }
    const unsigned wg = (unsigned)((nch + 63) / 64);
    {
        ProfScope prof("k_idx_walk_count", s);
        hipLaunchKernelGGL(k_idx_walk, dim3(wg), dim3(64), 0, s, x, nch, b.exits, b.cnt,
                           (const uint64_t*)nullptr, (uint64_t*)nullptr, 0);
    }
    e = dev_fill(b.cnt + nch, 0, sizeof(uint64_t), s);
    if (e != hipSuccess) return e;
    size_t tmp = b.scan_tmp_bytes;
    {
        ProfScope prof("scan_chunk_counts", s);
        e = hipcub::DeviceScan::ExclusiveSum(b.scan_tmp, tmp, b.cnt, b.base, (int)(nch + 1), s);
    }
    if (e != hipSuccess) return e;
    {
        ProfScope prof("k_idx_walk_write", s);
        hipLaunchKernelGGL(k_idx_walk, dim3(wg), dim3(64), 0, s, x, nch, b.exits, b.cnt, b.base,
                           b.offs, 1);
    }
    hipLaunchKernelGGL(k_idx_check, dim3((unsigned)(x.segs ? nsegs : 1)), dim3(64), 0, s, x, b.base,
                       nch);
    return hipGetLastError();
}

}  // namespace

hipError_t launch_index(const uint8_t* in, int64_t Cb, const Layout& L, const DecodeBufs& b,
                        hipStream_t s, const int64_t* dlen, int64_t cap, int64_t tail) {
    const uint32_t maxlen = (uint32_t)lz4_bound(L.bs * L.E);
    IdxArgs x{in, Cb, L.nblocks(), b.idx_err, nullptr, nullptr, nullptr, b.chunk,
              4 + (int64_t)maxlen, maxlen, idx_win_lds(maxlen), idx_wsub(maxlen), dlen, cap, tail};
    return index_impl(x, L.nblocks(), b.nchunks, 1, b, s);
}

hipError_t launch_index_batch(const Seg* segs, int nsegs, const uint32_t* chunk_seg, const Layout& L,
                              int64_t nchunks, const DecodeBufs& b, hipStream_t s) {
    const uint32_t maxlen = (uint32_t)lz4_bound(L.bs * L.E);
    IdxArgs x{nullptr, 0, L.nfull, nullptr, segs, chunk_seg, b.idx_err, b.chunk,
              4 + (int64_t)maxlen, maxlen, idx_win_lds(maxlen), idx_wsub(maxlen), nullptr, 0, 0};
    return index_impl(x, L.nfull, nchunks, nsegs, b, s);
}

namespace {

hipError_t scan_big_impl(DecArgs& a, int64_t nb, hipStream_t s) {
    ProfScope prof("k_seq_scan_big", s);
    hipLaunchKernelGGL(k_seq_scan_big, dim3((unsigned)nb), dim3(kWave), 0, s, a, nb);
    return hipGetLastError();
}

// token scan of blocks [a.blk0, a.blk1) (nb: all blocks of the stream(s))
hipError_t scan_impl(const DecArgs& a, int64_t nb, hipStream_t s) {
    ProfScope prof("k_seq_scan", s);
    hipLaunchKernelGGL(k_seq_scan, dim3((unsigned)((a.blk1 - a.blk0 + 255) / 256)), dim3(256), 0, s, a, nb);
    return hipGetLastError();
}

// Scan + decode kernels over nb blocks (one stream, or all streams of a batch).
hipError_t decode_impl(DecArgs& a, int64_t nb, bool aligned, hipStream_t s) {
    const Layout& L = a.L;
    // decoded block + record (header, payload, 16-byte alignment slack)
    const size_t rec = (((size_t)a.maxlen + 4 + 32 + 15) & ~(size_t)15);
    // phase 2 reads each record straight from global memory, so the LDS holds
    // only the decoded block: 18 resident waves per CU instead of 9 (A/B
    // variant 16: the record staged in LDS, as before)
    const bool grec = tuning_variant() == 16 || tuning_variant() == 32;
    // ... and touches each record's lines two blocks ahead (variant 32: not)
    const bool touch = tuning_variant() == 16;
    // default: the record in place at the end of the block's own buffer
    const bool inplace = !grec && tuning_variant() != 64;
    a.ip_end = (int32_t)(((size_t)a.cap + kInPlaceMargin + 15) & ~(size_t)15);
    size_t lds = inplace ? (size_t)a.ip_end + 32 : (size_t)a.cap + 16 + (grec ? 0 : rec);
    const int ek = aligned && (L.E == 1 || L.E == 2 || L.E == 4 || L.E == 8) ? L.E : 0;
    // any other element size: stage the inverse transpose when every output
    // is 8-aligned (a.stage_off was set to 1 by the caller as "may") -- through
    // registers for blocks of <= 8 KiB (stage_off -1), else in an LDS block of
    // its own
    if (ek == 0 && a.stage_off && (int64_t)L.bs * L.E <= 8192) {
        a.stage_off = -1;
    } else if (ek == 0 && a.stage_off) {
        a.stage_off = (int32_t)lds;
        lds += (size_t)a.cap;
    } else {
        a.stage_off = 0;
    }
    const void* fn = nullptr;
#define BSHUF_DEC(ekv, v) reinterpret_cast<const void*>(k_lz4_decode<ekv, v>)
    switch (ek) {
        case 1: fn = inplace ? BSHUF_DEC(1, 512) : touch ? BSHUF_DEC(1, 48) : (grec ? BSHUF_DEC(1, 16) : BSHUF_DEC(1, 0)); break;
        case 2:
            fn = inplace ? BSHUF_DEC(2, 512) : touch ? BSHUF_DEC(2, 48) : (grec ? BSHUF_DEC(2, 16) : BSHUF_DEC(2, 0));
#ifdef BSHUF_DIAG
            // diagnostic build only -- ABLATIONS for timing, wrong output:
            // 8 no output stores, 64 no sequence execution
            if (diag_variant() == 8) fn = BSHUF_DEC(2, 520);
            if (diag_variant() == 64) fn = BSHUF_DEC(2, 576);
            if (diag_variant() == 72) fn = BSHUF_DEC(2, 584);
            if (diag_variant() == 1024) fn = BSHUF_DEC(2, 1536);
            if (diag_variant() == 2048) fn = BSHUF_DEC(2, 2560);
#endif
            break;
        case 4:
            fn = inplace ? BSHUF_DEC(4, 512) : touch ? BSHUF_DEC(4, 48) : (grec ? BSHUF_DEC(4, 16) : BSHUF_DEC(4, 0));
#ifdef BSHUF_DIAG
            if (diag_variant() == 8) fn = BSHUF_DEC(4, 520);
            if (diag_variant() == 64) fn = BSHUF_DEC(4, 576);
            if (diag_variant() == 72) fn = BSHUF_DEC(4, 584);
#endif
            break;
        case 8: fn = inplace ? BSHUF_DEC(8, 512) : touch ? BSHUF_DEC(8, 48) : (grec ? BSHUF_DEC(8, 16) : BSHUF_DEC(8, 0)); break;
        default: fn = inplace ? BSHUF_DEC(0, 512) : touch ? BSHUF_DEC(0, 48) : (grec ? BSHUF_DEC(0, 16) : BSHUF_DEC(0, 0)); break;
    }
#undef BSHUF_DEC
    hipError_t e = hipSuccess;
#if defined(BSHUF_DIAG) || defined(BSHUF_OCC)
    // occupancy experiment: BSHUF_DIAG_DEC_WAVES=w pads the LDS request so
    // that at most w waves fit a CU
    if (const char* w = getenv("BSHUF_DIAG_DEC_WAVES")) {
        const size_t want = (size_t)(160 * 1024 / atoi(w)) & ~(size_t)1023;
        if (want > lds) lds = want;
    }
#endif
    if (lds > 65536) {
        e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
    }
    // blocks [f0, f1) on stream st (DecArgs carries the range)
    auto dec = [&](int64_t f0, int64_t f1, hipStream_t st) -> hipError_t {
        DecArgs aa = a;
        aa.blk0 = f0;
        aa.blk1 = f1;
        const dim3 grid((unsigned)persistent_grid(fn, kWave, lds, f1 - f0));
        ProfScope prof("k_lz4_decode", st);
        void* args[] = {&aa, const_cast<int64_t*>(&nb)};
        hipError_t r = hipLaunchKernel(fn, grid, dim3(kWave), args, lds, st);
        return r != hipSuccess ? r : hipGetLastError();
    };
    // (the scan stays ahead of the whole decode: run beside it in segments on a
    // side stream, it slowed the issue-bound decoder more than it hid,
    // 4.20 -> 4.24 ms G1 / 8.00 -> 8.21 ms G2 per 4 GiB, profiles/r04/pipe)
    a.blk0 = 0;
    a.blk1 = nb;
    e = scan_impl(a, nb, s);
    return e != hipSuccess ? e : dec(0, nb, s);
}

// Batch streams with device-held lengths: each Seg's in_nbytes (its capacity,
// uploaded from the host) becomes the readable bytes of its length word.
__global__ void k_seg_dlen(Seg* __restrict__ segs, const int64_t* __restrict__ dlens, int nsegs) {
    const int i = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (i < nsegs) segs[i].in_nbytes = readable_bytes(dlens[i], segs[i].in_nbytes);
}

// Batch result per stream: bytes consumed, or the error of its LAST failing
// block (one workgroup per stream; same rules as k_decode_finish).
__global__ __launch_bounds__(64) void k_decode_finish_batch(const int64_t* __restrict__ status,
                                                            const uint64_t* __restrict__ offs,
                                                            const long long* bad,
                                                            const int64_t* idx_err, const Seg* segs,
                                                            int32_t bs, int32_t E, const int64_t* dlens) {
    const Seg& g = segs[blockIdx.x];
    if (dlens && dlens[blockIdx.x] < 0) {  // upstream error (see k_decode_finish)
        if (threadIdx.x == 0) *g.result = dlens[blockIdx.x];
        return;
    }
    const int64_t nb = g.nfull + (g.last ? 1 : 0);
    const long long last_bad = bad[blockIdx.x];
    const int64_t end = nb ? (int64_t)offs[g.first + nb - 1] + status[g.first + nb - 1] : 0;
    const bool ok = last_bad < 0 && idx_err[blockIdx.x] == 0 && end + g.tail <= g.in_nbytes;
    uint8_t* tail_dst = g.out + (g.nfull * (int64_t)bs + g.last) * E;
    if (ok)
        for (int64_t i = threadIdx.x; i < g.tail; i += blockDim.x) tail_dst[i] = g.in[end + i];
    if (threadIdx.x == 0) *g.result = last_bad >= 0 ? status[last_bad] : (!ok ? -91 : end + g.tail);
}

}  // namespace

hipError_t launch_decode(const uint8_t* in, int64_t in_nbytes, uint8_t* out, const Layout& L,
                         int64_t tail_bytes, const DecodeBufs& b, int64_t* d_result,
                         hipStream_t s, const int64_t* dlen) {
    const int64_t nb = L.nblocks();
    hipError_t e = dev_fill(b.bad, 0xFF, sizeof(long long), s);  // -1
    if (e != hipSuccess) return e;
    if (nb > 0) {
        const int64_t nmax = (int64_t)L.bs * L.E;
        DecArgs a{in, in_nbytes, b.offs, out, b.status, b.bad, L, (uint32_t)lz4_bound((int)nmax),
                  (int32_t)((nmax + 15) & ~15), b.seq, nullptr, nullptr,
                  ((uintptr_t)out & 7) == 0 ? 1 : 0, 0, 0, nb, dlen};
        if (nmax > max_lds_decode_bytes()) {
            // large blocks: validated by the same scan (a wave per block),
            // executed in global memory
            e = tuning_variant() == 1024 ? scan_impl(a, nb, s) : scan_big_impl(a, nb, s);
            if (e == hipSuccess) e = launch_decode_large(in, in_nbytes, out, L, b, b.shuf, s);
        } else {
            e = decode_impl(a, nb, ((uintptr_t)out & 15) == 0, s);
        }
        if (e != hipSuccess) return e;
    }
    uint8_t* tail_dst = out + (L.nfull * (int64_t)L.bs + L.last) * L.E;
    ProfScope prof("k_decode_finish", s);
    hipLaunchKernelGGL(k_decode_finish, dim3(1), dim3(64), 0, s, b.status, b.offs, nb,
                       (const long long*)b.bad, (const int64_t*)b.idx_err, in, in_nbytes,
                       tail_dst, tail_bytes, d_result, dlen);
    return hipGetLastError();
}

hipError_t launch_seg_dlen(Seg* segs, const int64_t* dlens, int nsegs, hipStream_t s) {
    hipLaunchKernelGGL(k_seg_dlen, dim3((unsigned)((nsegs + 255) / 256)), dim3(256), 0, s, segs, dlens, nsegs);
    return hipGetLastError();
}

hipError_t launch_decode_batch(const Seg* segs, const Seg* hsegs, int nsegs, const uint32_t* blk_seg,
                               const Layout& L, const DecodeBufs& b, hipStream_t s, const int64_t* dlens) {
    const int64_t nb = L.nfull;
    hipError_t e = dev_fill(b.bad, 0xFF, sizeof(long long) * (size_t)nsegs, s);
    if (e != hipSuccess) return e;
    if (nb > 0) {
        const int64_t nmax = (int64_t)L.bs * L.E;
        bool aligned = true, al8 = true;
        for (int i = 0; i < nsegs; i++) {
            aligned = aligned && ((uintptr_t)hsegs[i].out & 15) == 0;
            al8 = al8 && ((uintptr_t)hsegs[i].out & 7) == 0;
        }
        DecArgs a{nullptr, 0, b.offs, nullptr, b.status, b.bad, L, (uint32_t)lz4_bound((int)nmax),
                  (int32_t)((nmax + 15) & ~15), b.seq, segs, blk_seg, al8 ? 1 : 0, 0, 0, nb, nullptr};
        e = decode_impl(a, nb, aligned, s);
        if (e != hipSuccess) return e;
    }
    ProfScope prof("k_decode_finish", s);
    hipLaunchKernelGGL(k_decode_finish_batch, dim3((unsigned)nsegs), dim3(64), 0, s, b.status, b.offs,
                       (const long long*)b.bad, (const int64_t*)b.idx_err, segs, L.bs, L.E, dlens);
    return hipGetLastError();
}

}  // namespace bshuf

#ifdef BSHUF_DIAG
// Diagnostic build only: read (and reset) k_lz4_decode's phase counters
// (out[0..7] cycles, out[8..15] counts).
extern "C" int bshuf_diag_read_dec(unsigned long long* out) {
    static unsigned long long all[bshuf::kDDiagCopies * 16];
    if (hipMemcpyFromSymbol(all, HIP_SYMBOL(bshuf::g_ddiag), sizeof all) != hipSuccess) return -1;
    for (int i = 0; i < 16; i++) {
        out[i] = 0;
        for (int c = 0; c < bshuf::kDDiagCopies; c++) out[i] += all[c * 16 + i];
    }
    static const unsigned long long z[bshuf::kDDiagCopies * 16] = {0};
    return hipMemcpyToSymbol(HIP_SYMBOL(bshuf::g_ddiag), z, sizeof z) == hipSuccess ? 0 : -1;
}
#endif
