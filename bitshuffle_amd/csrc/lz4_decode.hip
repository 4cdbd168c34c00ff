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

#include "launch.h"

namespace bshuf {

namespace {

constexpr int64_t kAmbiguous = -2;
constexpr int64_t kDead = -1;
constexpr int kIdxWinMax = 32768;  // LDS window for candidate screening

__device__ __forceinline__ uint32_t be32_global(const uint8_t* p) {
    return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
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

__global__ __launch_bounds__(64) void k_idx_exits(const uint8_t* __restrict__ in, int64_t Cb,
                                                  int64_t CH, int64_t W, uint32_t maxlen,
                                                  int64_t* __restrict__ exits) {
    __shared__ __attribute__((aligned(16))) uint8_t win[kIdxWinMax + 64];
    int win_off = 0;
    const int lane = threadIdx.x;
    const int64_t s = blockIdx.x;
    const int64_t cs = s * CH;
    const int64_t ce = min(cs + CH, Cb);
    const int64_t cend = (s == 0) ? cs + 1 : min(cs + W, Cb);  // candidate window
    const int64_t wbytes = min(cend + 3, Cb) - cs;
    const bool use_lds = wbytes <= kIdxWinMax;
    if (use_lds) {
        // 16-byte loads of the candidate window, aligned on the ABSOLUTE
        // address: an aligned granule never crosses a page, so the bytes it
        // reads outside [cs, cs+wbytes) cannot fault and are never used
        const uintptr_t start = (uintptr_t)(in + cs);
        const gbl128c* g4 = g128_aligned_down(in + cs);
        const int sh = (int)(start & 15);
        const int nch = (sh + (int)wbytes + 15) >> 4;
        lds128* w4 = (lds128*)to_lds(win);
        for (int c = lane; c < nch; c += kWave) w4[c] = g4[c];
        __syncthreads();
        win_off = sh;
    }
    int64_t lo = INT64_MAX, hi = -1;
    auto try_cand = [&](int64_t c, uint32_t len) {
        if (c >= cend || c + 4 > Cb) return;
        if (len == 0 || len > maxlen || c + 4 + (int64_t)len > Cb) return;
        const int64_t x = chase(in, c + 4 + len, ce, Cb, maxlen);
        if (x == kDead) return;
        lo = min(lo, x);
        hi = max(hi, x);
    };
    if (use_lds) {
        // 4 consecutive candidates per lane: two dword reads cover the 7
        // bytes of their four big-endian length words
        const lds8* wq = (const lds8*)to_lds(win) + win_off;
        for (int64_t c0 = cs + 4 * lane; c0 < cend; c0 += 4 * kWave) {
            const int r = (int)(c0 - cs);
            const uint32_t a = lds_rd32(wq, r), b = lds_rd32(wq, r + 4);
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const uint32_t le = __builtin_amdgcn_alignbyte(b, a, (uint32_t)k);
                try_cand(c0 + k, __builtin_bswap32(le));
            }
        }
    } else {
        for (int64_t c = cs + lane; c < cend; c += kWave)
            if (c + 4 <= Cb) try_cand(c, be32_global(in + c));
    }
    for (int o = 32; o >= 1; o >>= 1) {
        lo = min(lo, (int64_t)__shfl_xor(lo, o));
        hi = max(hi, (int64_t)__shfl_xor(hi, o));
    }
    if (lane == 0) exits[s] = (hi < 0) ? kDead : (lo == hi ? lo : kAmbiguous);
}

// Entry e_s of chunk s: the agreed exit of chunk s-1, else chase forward from
// the nearest chunk with an agreed exit (or from offset 0).
__device__ int64_t chunk_entry(const uint8_t* in, const int64_t* exits, int64_t s, int64_t CH,
                               int64_t Cb, uint32_t maxlen) {
    if (s == 0) return 0;
    int64_t t = s - 1;
    while (t >= 0 && exits[t] < 0) t--;
    int64_t p = (t < 0) ? 0 : exits[t];
    for (int64_t u = t + 1; u < s && p != kDead; u++) p = chase(in, p, min((u + 1) * CH, Cb), Cb, maxlen);
    return p;
}

// Walk chunk s from its entry.  mode 0: count headers into cnt[s];
// mode 1: write offs[base[s] + i].  Any broken link sets *err.
__global__ __launch_bounds__(64) void k_idx_walk(const uint8_t* __restrict__ in, int64_t Cb,
                                                 int64_t CH, uint32_t maxlen,
                                                 const int64_t* __restrict__ exits,
                                                 uint64_t* __restrict__ cnt,
                                                 const uint64_t* __restrict__ base,
                                                 uint64_t* __restrict__ offs, int64_t nblocks,
                                                 int64_t* __restrict__ err, int mode) {
    const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t nchunks = (Cb + CH - 1) / CH;
    if (s >= nchunks) return;
    const int64_t ce = min((s + 1) * CH, Cb);
    int64_t p = chunk_entry(in, exits, s, CH, Cb, maxlen);
    if (p == kDead) {
        atomicMax((unsigned long long*)err, 1ull);
        return;
    }
    uint64_t k = mode ? base[s] : 0;
    uint64_t c = 0;
    while (p < ce) {
        if (p + 4 > Cb) {
            atomicMax((unsigned long long*)err, 1ull);
            return;
        }
        const uint32_t len = be32_global(in + p);
        if (len == 0 || len > maxlen || p + 4 + (int64_t)len > Cb) {
            atomicMax((unsigned long long*)err, 1ull);
            return;
        }
        if (mode) {
            if ((int64_t)k < nblocks) offs[k] = (uint64_t)p;
            k++;
        }
        c++;
        p += 4 + len;
    }
    if (!mode) cnt[s] = c;
}

__global__ void k_idx_check(const uint64_t* base, int64_t nchunks, int64_t nblocks,
                            int64_t* err) {
    if (threadIdx.x == 0 && (int64_t)base[nchunks] != nblocks) atomicMax((unsigned long long*)err, 2ull);
}

// ---------------------------------------------------------------------------
// Per-block LZ4 decode
// ---------------------------------------------------------------------------

// 64-byte window over the compressed block in LDS: lane l holds C[base + l].
struct Win {
    int base;
    uint32_t v;
};

__device__ __forceinline__ void win_at(Win& w, const lds8* C, int clen, int pos, int lane) {
    if (pos < w.base || pos >= w.base + kWave) {
        w.base = pos;
        const int p = pos + lane;
        w.v = p < clen ? C[p] : 0u;
    }
}

__device__ __forceinline__ int win_byte(Win& w, const lds8* C, int clen, int pos, int lane) {
    win_at(w, C, clen, pos, lane);
    return __builtin_amdgcn_readlane((int)w.v, pos - w.base);
}

// LZ4 length continuation starting at pos: adds bytes while they are 255,
// the first non-255 byte ends it.  Returns -1 if it runs past clen.
__device__ __forceinline__ int win_len(Win& w, const lds8* C, int clen, int& pos, int lane) {
    int add = 0;
    for (;;) {
        if (pos >= clen) return -1;
        win_at(w, C, clen, pos, lane);
        const int o = pos - w.base;
        const bool in = lane >= o && w.base + lane < clen;
        const uint64_t nm = ballot(in && w.v != 255u) | ballot(!(w.base + lane < clen) && lane >= o);
        if (nm == 0) {
            add += 255 * (kWave - o);
            pos = w.base + kWave;
            continue;
        }
        const int f = ffs64(nm);
        if (w.base + f >= clen) return -1;
        add += 255 * (f - o) + __builtin_amdgcn_readlane((int)w.v, f);
        pos = w.base + f + 1;
        return add;
    }
}

// Decode C[0..clen) into D[0..n).  Returns 0, or an LZ4-style error
// -(position)-1, or -91 - the only codes bshuf_decompress_lz4_block maps.
template <int ABL = 0>
__device__ int lz4_decode_block(const lds8* C, const int clen, lds8* D, const int n,
                                const int lane) {
    int ip = 0, op = 0;
    Win w{-1000000, 0};
    for (;;) {
        if (ip >= clen) return -ip - 1;
        const int tok = win_byte(w, C, clen, ip, lane);
        int q = ip + 1;
        int lit = tok >> 4;
        if (lit == 15) {
            const int add = win_len(w, C, clen, q, lane);
            if (add < 0) return -q - 1;
            lit += add;
        }
        if (q + lit > clen || op + lit > n) return -q - 1;
        if (!(ABL & 16))
            for (int i = lane; i < lit; i += kWave) D[op + i] = C[q + i];
        op += lit;
        q += lit;
        if (q == clen) break;  // last sequence carries literals only
        if (q + 2 > clen) return -q - 1;
        const int off = win_byte(w, C, clen, q, lane) | (win_byte(w, C, clen, q + 1, lane) << 8);
        q += 2;
        if (off == 0 || off > op) return -q - 1;
        int ml = tok & 15;
        if (ml == 15) {
            const int add = win_len(w, C, clen, q, lane);
            if (add < 0) return -q - 1;
            ml += add;
        }
        ml += kMinMatch;
        if (op + ml > n) return -q - 1;
        if (ABL & 32) {
        } else if (off >= kWave || off >= ml) {
            // sources of chunk c were all written before chunk c starts
            for (int i = lane; i < ml; i += kWave) D[op + i] = D[op - off + i];
        } else {
            // short period: output is periodic with period off
            int r = lane % off;
            const int step = kWave % off;
            for (int i = lane; i < ml; i += kWave) {
                D[op + i] = D[op - off + r];
                r += step;
                if (r >= off) r -= off;
            }
        }
        op += ml;
        ip = q;
    }
    return op == n ? 0 : -91;
}

// ---------------------------------------------------------------------------
// Decoder v2: 256-byte token window (lane l holds C[base+4l .. base+4l+3]; a
// byte is one v_readlane + shift), dword-granular LDS copies, a fill path for
// offset-1 matches (byte runs: the commonest match in bit planes) and whole
// 256-byte chunks for offsets >= 256 (plane-stride matches).
// ---------------------------------------------------------------------------
struct Win4 {
    int base;
    uint32_t v;
};

__device__ __forceinline__ void w4_load(Win4& w, const lds8* C, int ccap, int pos, int lane) {
    w.base = pos;
    w.v = lds_rd32(C, min(pos + 4 * lane, ccap));
}

__device__ __forceinline__ uint32_t w4_byte(const Win4& w, int pos) {
    const int t = pos - w.base;
    const uint32_t d = (uint32_t)__builtin_amdgcn_readlane((int)w.v, t >> 2);
    return (d >> ((t & 3) * 8)) & 0xFFu;
}

__device__ __forceinline__ uint32_t w4_get(Win4& w, const lds8* C, int ccap, int pos, int lane) {
    if (pos < w.base || pos >= w.base + 4 * kWave) w4_load(w, C, ccap, pos, lane);
    return w4_byte(w, pos);
}

// LZ4 length continuation at q (bytes added while they are 255); -1 on overrun.
__device__ __forceinline__ int w4_len(Win4& w, const lds8* C, int clen, int ccap, int& q,
                                      int lane) {
    int add = 0;
    for (;;) {
        if (q >= clen) return -1;
        const uint32_t b = w4_get(w, C, ccap, q, lane);
        q++;
        add += (int)b;
        if (b != 255u) return add;
    }
}

// Write dwords covering D[op, op+len) with per-lane values from `gen(db)`
// (db = first byte of the dword); the head dword keeps the bytes below op.
// Bytes past op+len in the last dword are scratch: they are overwritten by the
// next sequence before anything reads them (sources are always < op).
template <class Gen>
__device__ __forceinline__ void put_dwords(lds8* D, int op, int len, int lane, Gen gen) {
    const int d0 = op >> 2, d1 = (op + len + 3) >> 2;
    lds32* D32 = (lds32*)D;
    for (int d = d0 + lane; d < d1; d += kWave) {
        const int db = 4 * d;
        uint32_t v = gen(db);
        if (db < op) {
            const uint32_t keep = (1u << (8 * (op - db))) - 1u;
            v = (D32[d] & keep) | (v & ~keep);
        }
        D32[d] = v;
    }
}

__device__ __forceinline__ uint32_t rd32_lo(const lds8* B, int p) {
    // read32 at p where p may be up to 3 below 0: missing bytes are zero
    const int pc = max(p, 0);
    return lds_rd32(B, pc) << (8 * (pc - p));
}

__device__ __forceinline__ void copy_match(lds8* D, int op, int off, int ml, int lane) {
    if (off == 1) {
        const uint32_t fill = (uint32_t)D[op - 1] * 0x01010101u;
        put_dwords(D, op, ml, lane, [&](int) { return fill; });
        return;
    }
    if (off >= ml) {  // all sources are below op
        put_dwords(D, op, ml, lane, [&](int db) { return rd32_lo(D, db - off); });
        return;
    }
    if (off >= 4 * kWave) {  // 256-byte chunks: each chunk's sources precede it
        for (int c = 0; c < ml; c += 4 * kWave) {
            const int o = op + c;
            put_dwords(D, o, min(4 * kWave, ml - c), lane,
                       [&](int db) { return rd32_lo(D, db - off); });
        }
        return;
    }
    // short period: D[op+i] = D[op-off + i%off], all sources pre-existing
    int r = (int)((float)lane * __builtin_amdgcn_rcpf((float)off) + 0.5f / (float)off);
    r = lane - r * off;
    if (r >= off) r -= off;
    if (r < 0) r += off;
    const int step = kWave % off;
    for (int i = lane; i < ml; i += kWave) {
        D[op + i] = D[op - off + r];
        r += step;
        if (r >= off) r -= off;
    }
}

__device__ int lz4_decode_block_v2(const lds8* C, const int clen, const int ccap, lds8* D,
                                   const int n, const int lane) {
    int ip = 0, op = 0;
    Win4 w;
    w4_load(w, C, ccap, 0, lane);
    for (;;) {
        if (ip >= clen) return -ip - 1;
        const uint32_t tok = w4_get(w, C, ccap, ip, lane);
        int q = ip + 1;
        int lit = (int)(tok >> 4);
        if (lit == 15) {
            const int add = w4_len(w, C, clen, ccap, q, lane);
            if (add < 0) return -q - 1;
            lit += add;
        }
        if (q + lit > clen || op + lit > n) return -q - 1;
        if (lit) {
            const int src = q - op;
            put_dwords(D, op, lit, lane, [&](int db) { return rd32_lo(C, db + src); });
        }
        op += lit;
        q += lit;
        if (q == clen) break;  // last sequence carries literals only
        if (q + 2 > clen) return -q - 1;
        const int off = (int)(w4_get(w, C, ccap, q, lane) | (w4_get(w, C, ccap, q + 1, lane) << 8));
        q += 2;
        if (off == 0 || off > op) return -q - 1;
        int ml = (int)(tok & 15u);
        if (ml == 15) {
            const int add = w4_len(w, C, clen, ccap, q, lane);
            if (add < 0) return -q - 1;
            ml += add;
        }
        ml += kMinMatch;
        if (op + ml > n) return -q - 1;
        copy_match(D, op, off, ml, lane);
        op += ml;
        ip = q;
    }
    return op == n ? 0 : -91;
}

// Inverse transpose D (LDS) -> dst (HBM), 4 groups per lane: one dword of
// every plane per lane instead of single bytes.  Needs P % 4 == 0.
template <int EK>
__device__ __forceinline__ void untranspose_x4(const lds8* D, uint8_t* dst, int P, int lane) {
    const lds32* D32 = (const lds32*)D;
    const int P4 = P >> 2;
    for (int q = lane; q < P4; q += kWave) {
        uint32_t pl[8 * EK];
#pragma unroll
        for (int r = 0; r < 8 * EK; r++) pl[r] = D32[r * P4 + q];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            uint32_t w[2 * EK];
#pragma unroll
            for (int i = 0; i < 2 * EK; i++) w[i] = 0;
#pragma unroll
            for (int b = 0; b < EK; b++) {
                uint64_t v = 0;
#pragma unroll
                for (int j = 0; j < 8; j++) v |= (uint64_t)((pl[8 * b + j] >> (8 * k)) & 0xFFu) << (8 * j);
                scatter_byte_plane<EK>(w, b, tr8x8(v));
            }
            store_group<EK>(dst + (int64_t)(4 * q + k) * 8 * EK, w);
        }
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
    int32_t ccap;    // readable LDS bytes of the record buffer
};

// Byte range [o0, o1) of block k's record ([BE32 c][c bytes]) in the stream.
// Consecutive records are contiguous, so the next offset ends this record;
// the last record is bounded by its worst-case size.
struct Span {
    int64_t o0, o1;
};

__device__ __forceinline__ Span span_of(const DecArgs& a, int64_t k, int64_t nb) {
    Span sp;
    sp.o0 = (int64_t)a.offs[k];
    sp.o1 = (k + 1 < nb) ? (int64_t)a.offs[k + 1] : sp.o0 + 4 + (int64_t)a.maxlen;
    if (sp.o1 > a.in_nbytes) sp.o1 = a.in_nbytes;
    if (sp.o0 > sp.o1) sp.o0 = sp.o1;
    return sp;
}

// 16-byte chunks covering a record of an 8 KiB block: (8244 + 30) / 16 / 64 -> 9.
constexpr int kPayIters = 9;

struct PayRegs {
    u32x4 v[kPayIters];
};

// Record bytes [o0, o1) are read as whole 16-byte granules aligned on the
// absolute address (a granule never crosses a page: the extra bytes at either
// end cannot fault and are never used); they land in LDS at Cbuf + (addr & 15).
__device__ __forceinline__ const gbl128c* span_base(const DecArgs& a, const Span& sp) {
    return g128_aligned_down(a.in + sp.o0);
}
__device__ __forceinline__ int span_shift(const DecArgs& a, const Span& sp) {
    return (int)((uintptr_t)(a.in + sp.o0) & 15);
}
__device__ __forceinline__ int span_chunks(const DecArgs& a, const Span& sp) {
    return (span_shift(a, sp) + (int)(sp.o1 - sp.o0) + 15) >> 4;
}

__device__ __forceinline__ bool span_fits(const DecArgs& a, const Span& sp) {
    return span_chunks(a, sp) <= kPayIters * kWave;
}

__device__ __forceinline__ void issue_pay(PayRegs& R, const DecArgs& a, const Span& sp, int lane) {
    const gbl128c* g4 = span_base(a, sp);
    const int nch = span_chunks(a, sp);
#pragma unroll
    for (int it = 0; it < kPayIters; it++) {
        const int c = it * kWave + lane;
        if (c < nch) R.v[it] = g4[c];
    }
}

__device__ __forceinline__ void land_pay(const PayRegs& R, const DecArgs& a, const Span& sp,
                                         lds8* C, int lane) {
    const int nch = span_chunks(a, sp);
#pragma unroll
    for (int it = 0; it < kPayIters; it++) {
        const int c = it * kWave + lane;
        if (c < nch) ((lds128*)C)[c] = R.v[it];
    }
}

// Persistent: workgroup w decodes blocks w, w+G, ...  Offsets are fetched two
// blocks ahead and the next record's bytes one block ahead, into registers,
// so HBM latency overlaps the LDS-bound LZ4 parse of the current block.
template <int EK, int VAR>
__global__ __launch_bounds__(64) void k_lz4_decode(DecArgs a, int64_t nb) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int lane = threadIdx.x;
    const int E = EK ? EK : a.L.E;
    lds8* D = to_lds(smem);             // decoded (bit-shuffled) block
    lds8* Cbuf = to_lds(smem) + a.cap + 16;  // record bytes, 16-aligned base
    const int64_t stride = gridDim.x;
    int64_t blk = blockIdx.x;
    if (blk >= nb) return;

    Span cur = span_of(a, blk, nb);
    Span nxt = {0, 0};
    if (blk + stride < nb) nxt = span_of(a, blk + stride, nb);
    PayRegs R;
    bool cur_in_regs = span_fits(a, cur);
    if (cur_in_regs) issue_pay(R, a, cur, lane);

    for (;;) {
        const int m = blk < a.L.nfull ? a.L.bs : a.L.last;
        const int n = m * E;
        const int P = m / 8;
        // land this record in LDS
        if (cur_in_regs) {
            land_pay(R, a, cur, Cbuf, lane);
        } else {
            const gbl128c* g4 = span_base(a, cur);
            const int nch = span_chunks(a, cur);
            for (int c = lane; c < nch; c += kWave) ((lds128*)Cbuf)[c] = g4[c];
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        // prefetch: next record into registers, the one after into `nxt2`
        const int64_t next = blk + stride;
        const bool next_in_regs = next < nb && span_fits(a, nxt);
        if (next_in_regs) issue_pay(R, a, nxt, lane);
        Span nxt2 = {0, 0};
        if (next + stride < nb) nxt2 = span_of(a, next + stride, nb);

        const lds8* C = Cbuf + span_shift(a, cur);
        const int avail = (int)(cur.o1 - cur.o0);
        int status = 0, clen = 0;
        if (avail < 4) {
            status = -1000 - 1;
        } else {
            clen = (int)(((uint32_t)C[0] << 24) | ((uint32_t)C[1] << 16) | ((uint32_t)C[2] << 8) | C[3]);
            const bool last = blk + 1 == nb;
            if (clen <= 0 || (uint32_t)clen > a.maxlen || clen + 4 > avail ||
                (!last && clen + 4 != avail))
                status = (clen + 4 > avail) ? -1000 - 1 : -91;
        }
        if (status == 0) {
            const int r = (VAR & 64) ? 0
                          : (VAR & 2) ? lz4_decode_block_v2(C + 4, clen, a.ccap - 4, D, n, lane)
                                      : lz4_decode_block<VAR>(C + 4, clen, D, n, lane);
            status = (r == -91) ? -91 : (r < 0 ? r - 1000 : 0);
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        if (status == 0 && !(VAR & 8)) {
            uint8_t* dst = a.out + blk * (int64_t)a.L.bs * E;
            if constexpr (EK != 0) {
              if ((VAR & 4) && (P & 3) == 0) {
                untranspose_x4<EK>(D, dst, P, lane);
              } else {
                for (int g = lane; g < P; g += kWave) {
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
                        dst[(int64_t)(8 * g + k) * E + b] = (uint8_t)(v >> (8 * k));
                }
            }
        } else if (lane == 0) {
            atomicMax(a.bad, (long long)blk);
        }
        if (lane == 0) a.status[blk] = status == 0 ? (int64_t)clen + 4 : (int64_t)status;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        if (next >= nb) break;
        blk = next;
        cur = nxt;
        nxt = nxt2;
        cur_in_regs = next_in_regs;
    }
}

// Result: bytes consumed, or the error of the LAST failing block (the
// sequential reference keeps overwriting err, src/bitshuffle_core.c:1905).
// Also copies the raw tail (whose position is only known from the index).
__global__ __launch_bounds__(256) void k_decode_finish(const int64_t* __restrict__ status,
                                                       const uint64_t* __restrict__ offs,
                                                       int64_t nblocks, const long long* bad,
                                                       const int64_t* idx_err, const uint8_t* in,
                                                       int64_t in_nbytes, uint8_t* tail_dst,
                                                       int64_t tail, int64_t* result) {
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

}  // namespace

int64_t index_chunk_bytes(const Layout& L) {
    const int64_t foot = 4 + lz4_bound(L.bs * L.E);
    int64_t ch = 64 * 1024;
    while (ch < 2 * foot) ch *= 2;
    return ch;
}

size_t decode_scan_tmp_bytes(int64_t nchunks) {
    size_t bytes = 0;
    (void)hipcub::DeviceScan::ExclusiveSum(nullptr, bytes, (const uint64_t*)nullptr, (uint64_t*)nullptr,
                                     (int)(nchunks + 1));
    return bytes;
}

hipError_t launch_index(const uint8_t* in, int64_t Cb, const Layout& L, const DecodeBufs& b,
                        hipStream_t s) {
    const int64_t nb = L.nblocks();
    hipError_t e = hipMemsetAsync(b.idx_err, 0, sizeof(int64_t), s);
    if (e != hipSuccess || nb == 0) return e;
    const uint32_t maxlen = (uint32_t)lz4_bound(L.bs * L.E);
    const int64_t W = 4 + (int64_t)maxlen;
    const int64_t nch = b.nchunks;
    {
        ProfScope prof("k_idx_exits", s);
        hipLaunchKernelGGL(k_idx_exits, dim3((unsigned)nch), dim3(kWave), 0, s, in, Cb, b.chunk, W,
                           maxlen, b.exits);
    }
    const unsigned wg = (unsigned)((nch + 63) / 64);
    {
        ProfScope prof("k_idx_walk_count", s);
        hipLaunchKernelGGL(k_idx_walk, dim3(wg), dim3(64), 0, s, in, Cb, b.chunk, maxlen, b.exits,
                           b.cnt, (const uint64_t*)nullptr, (uint64_t*)nullptr, nb, b.idx_err, 0);
    }
    e = hipMemsetAsync(b.cnt + nch, 0, sizeof(uint64_t), s);
    if (e != hipSuccess) return e;
    size_t tmp = b.scan_tmp_bytes;
    {
        ProfScope prof("scan_chunk_counts", s);
        e = hipcub::DeviceScan::ExclusiveSum(b.scan_tmp, tmp, b.cnt, b.base, (int)(nch + 1), s);
    }
    if (e != hipSuccess) return e;
    {
        ProfScope prof("k_idx_walk_write", s);
        hipLaunchKernelGGL(k_idx_walk, dim3(wg), dim3(64), 0, s, in, Cb, b.chunk, maxlen, b.exits,
                           b.cnt, b.base, b.offs, nb, b.idx_err, 1);
    }
    hipLaunchKernelGGL(k_idx_check, dim3(1), dim3(64), 0, s, b.base, nch, nb, b.idx_err);
    return hipGetLastError();
}

hipError_t launch_decode(const uint8_t* in, int64_t in_nbytes, uint8_t* out, const Layout& L,
                         int64_t tail_bytes, const DecodeBufs& b, int64_t* d_result,
                         hipStream_t s) {
    const int64_t nb = L.nblocks();
    hipError_t e = hipMemsetAsync(b.bad, 0xFF, sizeof(long long), s);  // -1
    if (e != hipSuccess) return e;
    if (nb > 0) {
        const int64_t nmax = (int64_t)L.bs * L.E;
        DecArgs a{in, in_nbytes, b.offs, out, b.status, b.bad, L, (uint32_t)lz4_bound((int)nmax),
                  (int32_t)((nmax + 15) & ~15), 0};
        // decoded block + record (header, payload, 16-byte alignment slack)
        const size_t rec = (((size_t)a.maxlen + 4 + 32 + 15) & ~(size_t)15);
        const size_t lds = (size_t)a.cap + 16 + rec;
        a.ccap = (int32_t)(rec - 16 - 8);  // record reads stay inside the buffer
        const bool aligned = ((uintptr_t)out & 15) == 0;
        const int ek = aligned && (L.E == 1 || L.E == 2 || L.E == 4 || L.E == 8) ? L.E : 0;
        // tuning_variant(): bit1 the 256-byte-window block decoder (v2), bit2
        // the 4-groups-per-lane inverse transpose -- both measured slower than
        // the defaults on MI355X and kept for A/B; bits 3-6 are ABLATIONS for
        // timing only (wrong output): 8 no output stores, 16 no literal copy,
        // 32 no match copy, 64 no LZ4.
        const int var = tuning_variant();
        const void* fn = nullptr;
        switch (ek) {
            case 1: fn = reinterpret_cast<const void*>(k_lz4_decode<1, 0>); break;
            case 2:
                switch (var) {
#define BSHUF_DEC_VAR(v) case v: fn = reinterpret_cast<const void*>(k_lz4_decode<2, v>); break;
                    BSHUF_DEC_VAR(2) BSHUF_DEC_VAR(4) BSHUF_DEC_VAR(6) BSHUF_DEC_VAR(8)
                    BSHUF_DEC_VAR(16) BSHUF_DEC_VAR(32) BSHUF_DEC_VAR(48) BSHUF_DEC_VAR(64)
                    BSHUF_DEC_VAR(72)
#undef BSHUF_DEC_VAR
                    default: fn = reinterpret_cast<const void*>(k_lz4_decode<2, 0>); break;
                }
                break;
            case 4: fn = reinterpret_cast<const void*>(k_lz4_decode<4, 0>); break;
            case 8: fn = reinterpret_cast<const void*>(k_lz4_decode<8, 0>); break;
            default: fn = reinterpret_cast<const void*>(k_lz4_decode<0, 0>); break;
        }
        if (lds > 65536) {
            e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
            if (e != hipSuccess) return e;
        }
        const dim3 grid((unsigned)persistent_grid(fn, kWave, lds, nb));
        ProfScope prof("k_lz4_decode", s);
        void* args[] = {&a, const_cast<int64_t*>(&nb)};
        e = hipLaunchKernel(fn, grid, dim3(kWave), args, lds, s);
        if (e != hipSuccess) return e;
        e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    uint8_t* tail_dst = out + (L.nfull * (int64_t)L.bs + L.last) * L.E;
    ProfScope prof("k_decode_finish", s);
    hipLaunchKernelGGL(k_decode_finish, dim3(1), dim3(64), 0, s, b.status, b.offs, nb,
                       (const long long*)b.bad, (const int64_t*)b.idx_err, in, in_nbytes,
                       tail_dst, tail_bytes, d_result);
    return hipGetLastError();
}

}  // namespace bshuf
