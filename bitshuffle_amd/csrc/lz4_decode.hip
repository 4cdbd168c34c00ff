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
    __shared__ __attribute__((aligned(16))) uint8_t win[kIdxWinMax + 16];
    const int lane = threadIdx.x;
    const int64_t s = blockIdx.x;
    const int64_t cs = s * CH;
    const int64_t ce = min(cs + CH, Cb);
    const int64_t cend = (s == 0) ? cs + 1 : min(cs + W, Cb);  // candidate window
    const int64_t wbytes = min(cend + 3, Cb) - cs;
    const bool use_lds = wbytes <= kIdxWinMax;
    if (use_lds) {
        for (int64_t i = lane; i < wbytes; i += kWave) win[i] = in[cs + i];
        __syncthreads();
    }
    int64_t lo = INT64_MAX, hi = -1;
    for (int64_t c = cs + lane; c < cend; c += kWave) {
        if (c + 4 > Cb) continue;
        uint32_t len;
        if (use_lds) {
            const uint8_t* q = win + (c - cs);
            len = ((uint32_t)q[0] << 24) | ((uint32_t)q[1] << 16) | ((uint32_t)q[2] << 8) | q[3];
        } else {
            len = be32_global(in + c);
        }
        if (len == 0 || len > maxlen || c + 4 + (int64_t)len > Cb) continue;
        const int64_t x = chase(in, c + 4 + len, ce, Cb, maxlen);
        if (x == kDead) continue;
        lo = min(lo, x);
        hi = max(hi, x);
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

__device__ __forceinline__ void win_at(Win& w, const uint8_t* C, int clen, int pos, int lane) {
    if (pos < w.base || pos >= w.base + kWave) {
        w.base = pos;
        const int p = pos + lane;
        w.v = p < clen ? C[p] : 0u;
    }
}

__device__ __forceinline__ int win_byte(Win& w, const uint8_t* C, int clen, int pos, int lane) {
    win_at(w, C, clen, pos, lane);
    return __builtin_amdgcn_readlane((int)w.v, pos - w.base);
}

// LZ4 length continuation starting at pos: adds bytes while they are 255,
// the first non-255 byte ends it.  Returns -1 if it runs past clen.
__device__ __forceinline__ int win_len(Win& w, const uint8_t* C, int clen, int& pos, int lane) {
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
__device__ int lz4_decode_block(const uint8_t* C, const int clen, uint8_t* D, const int n,
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
        if (off >= kWave || off >= ml) {
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

struct DecArgs {
    const uint8_t* in;
    int64_t in_nbytes;
    const uint64_t* offs;
    uint8_t* out;
    int64_t* status;
    Layout L;
    uint32_t maxlen;
    int32_t cap;  // bytes reserved for the compressed block in LDS
};

template <int EK>
__global__ __launch_bounds__(64) void k_lz4_decode(DecArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int lane = threadIdx.x;
    const int64_t blk = blockIdx.x;
    const int E = EK ? EK : a.L.E;
    const int m = blk < a.L.nfull ? a.L.bs : a.L.last;
    const int n = m * E;
    const int P = m / 8;
    uint8_t* D = smem;                 // decoded (shuffled) block
    uint8_t* Cl = smem + a.cap + 16;   // compressed block (16-aligned), +shift
    const int64_t h = (int64_t)a.offs[blk];
    int status = 0;
    int clen = 0;
    if (h + 4 > a.in_nbytes) {
        status = -1000 - 1;
    } else {
        clen = (int)be32_global(a.in + h);
        if (clen <= 0 || (uint32_t)clen > a.maxlen || h + 4 + clen > a.in_nbytes) status = -1000 - 1;
    }
    if (status == 0) {
        // stage the compressed block in LDS with aligned dword loads
        const int64_t start = h + 4;
        const int64_t a0 = start & ~(int64_t)3;
        const int shift = (int)(start - a0);
        const int64_t end = start + clen;
        const int nw = (int)((end - a0 + 3) >> 2);
        const uint32_t* g32 = reinterpret_cast<const uint32_t*>(a.in + a0);
        uint32_t* l32 = reinterpret_cast<uint32_t*>(Cl);
        for (int i = lane; i < nw; i += kWave) {
            const int64_t gb = a0 + 4 * (int64_t)i;
            uint32_t v;
            if (gb + 4 <= a.in_nbytes) {
                v = g32[i];
            } else {
                v = 0;
                for (int j = 0; j < 4; j++)
                    if (gb + j < a.in_nbytes) v |= (uint32_t)a.in[gb + j] << (8 * j);
            }
            l32[i] = v;
        }
        __syncthreads();
        const int r = lz4_decode_block(reinterpret_cast<const uint8_t*>(l32) + shift, clen, D, n, lane);
        if (r == -91)
            status = -91;
        else if (r < 0)
            status = r - 1000;
    }
    if (status == 0) {
        __syncthreads();
        uint8_t* dst = a.out + blk * (int64_t)a.L.bs * E;
        if constexpr (EK != 0) {
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
        } else {
            for (int i = lane; i < P * E; i += kWave) {
                const int g = i / E, b = i - g * E;
                uint64_t v = 0;
#pragma unroll
                for (int j = 0; j < 8; j++) v |= (uint64_t)D[(8 * b + j) * P + g] << (8 * j);
                v = tr8x8(v);
#pragma unroll
                for (int k = 0; k < 8; k++) dst[(int64_t)(8 * g + k) * E + b] = (uint8_t)(v >> (8 * k));
            }
        }
    }
    if (lane == 0) a.status[blk] = status == 0 ? (int64_t)clen + 4 : (int64_t)status;
}

// Result: bytes consumed, or the error of the LAST failing block (the
// sequential reference keeps overwriting err, src/bitshuffle_core.c:1905).
// Also copies the raw tail (whose position is only known from the index).
__global__ __launch_bounds__(256) void k_decode_finish(const int64_t* __restrict__ status,
                                                       const uint64_t* __restrict__ offs,
                                                       int64_t nblocks, const int64_t* idx_err,
                                                       const uint8_t* in, int64_t in_nbytes,
                                                       uint8_t* tail_dst, int64_t tail,
                                                       int64_t* result) {
    __shared__ long long last_bad;
    if (threadIdx.x == 0) last_bad = -1;
    __syncthreads();
    for (int64_t k = threadIdx.x; k < nblocks; k += blockDim.x)
        if (status[k] < 0) atomicMax(&last_bad, (long long)k);
    __syncthreads();
    const int64_t end = nblocks ? (int64_t)offs[nblocks - 1] + status[nblocks - 1] : 0;
    const bool idx_bad = idx_err && *idx_err != 0;
    if (last_bad < 0 && !idx_bad && end + tail <= in_nbytes)
        for (int64_t i = threadIdx.x; i < tail; i += blockDim.x) tail_dst[i] = in[end + i];
    if (threadIdx.x == 0) {
        if (last_bad >= 0)
            *result = status[last_bad];
        else if (idx_bad || end + tail > in_nbytes)
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
    hipLaunchKernelGGL(k_idx_exits, dim3((unsigned)nch), dim3(kWave), 0, s, in, Cb, b.chunk, W,
                       maxlen, b.exits);
    const unsigned wg = (unsigned)((nch + 63) / 64);
    hipLaunchKernelGGL(k_idx_walk, dim3(wg), dim3(64), 0, s, in, Cb, b.chunk, maxlen, b.exits,
                       b.cnt, (const uint64_t*)nullptr, (uint64_t*)nullptr, nb, b.idx_err, 0);
    e = hipMemsetAsync(b.cnt + nch, 0, sizeof(uint64_t), s);
    if (e != hipSuccess) return e;
    size_t tmp = b.scan_tmp_bytes;
    e = hipcub::DeviceScan::ExclusiveSum(b.scan_tmp, tmp, b.cnt, b.base, (int)(nch + 1), s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_idx_walk, dim3(wg), dim3(64), 0, s, in, Cb, b.chunk, maxlen, b.exits,
                       b.cnt, b.base, b.offs, nb, b.idx_err, 1);
    hipLaunchKernelGGL(k_idx_check, dim3(1), dim3(64), 0, s, b.base, nch, nb, b.idx_err);
    return hipGetLastError();
}

hipError_t launch_decode(const uint8_t* in, int64_t in_nbytes, uint8_t* out, const Layout& L,
                         int64_t tail_bytes, const DecodeBufs& b, int64_t* d_result,
                         hipStream_t s) {
    const int64_t nb = L.nblocks();
    if (nb > 0) {
        const int64_t nmax = (int64_t)L.bs * L.E;
        DecArgs a{in, in_nbytes, b.offs, out, b.status, L, (uint32_t)lz4_bound((int)nmax),
                  (int32_t)((nmax + 15) & ~15)};
        const size_t lds = (size_t)a.cap + 16 + ((a.maxlen + 8 + 15) & ~15u) + 16;
        const bool aligned = ((uintptr_t)out & 15) == 0;
        const int ek = aligned && (L.E == 1 || L.E == 2 || L.E == 4 || L.E == 8) ? L.E : 0;
        const void* fn = nullptr;
        switch (ek) {
            case 1: fn = reinterpret_cast<const void*>(k_lz4_decode<1>); break;
            case 2: fn = reinterpret_cast<const void*>(k_lz4_decode<2>); break;
            case 4: fn = reinterpret_cast<const void*>(k_lz4_decode<4>); break;
            case 8: fn = reinterpret_cast<const void*>(k_lz4_decode<8>); break;
            default: fn = reinterpret_cast<const void*>(k_lz4_decode<0>); break;
        }
        if (lds > 65536) {
            hipError_t e =
                hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
            if (e != hipSuccess) return e;
        }
        switch (ek) {
            case 1: hipLaunchKernelGGL(k_lz4_decode<1>, dim3((unsigned)nb), dim3(kWave), lds, s, a); break;
            case 2: hipLaunchKernelGGL(k_lz4_decode<2>, dim3((unsigned)nb), dim3(kWave), lds, s, a); break;
            case 4: hipLaunchKernelGGL(k_lz4_decode<4>, dim3((unsigned)nb), dim3(kWave), lds, s, a); break;
            case 8: hipLaunchKernelGGL(k_lz4_decode<8>, dim3((unsigned)nb), dim3(kWave), lds, s, a); break;
            default: hipLaunchKernelGGL(k_lz4_decode<0>, dim3((unsigned)nb), dim3(kWave), lds, s, a); break;
        }
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    uint8_t* tail_dst = out + (L.nfull * (int64_t)L.bs + L.last) * L.E;
    hipLaunchKernelGGL(k_decode_finish, dim3(1), dim3(256), 0, s, b.status, b.offs, nb,
                       (const int64_t*)b.idx_err, in, in_nbytes, tail_dst, tail_bytes, d_result);
    return hipGetLastError();
}

}  // namespace bshuf
