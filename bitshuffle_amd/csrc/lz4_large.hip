// lz4_large.hip -- blocks too large for the LDS-resident kernels.
//
// The reference accepts any block size that is a multiple of 8
// (src/bitshuffle_core.c:1894-1897) and runs LZ4_compress_default on the
// whole block (src/bitshuffle.c:36-79; byU32 table + hash5 from 65547 bytes,
// lz4/lz4.c:1388-1393).  The wave-per-block kernels keep the block (and the
// encoder's 16 KiB table, the decoder's record) in LDS, which caps them at
// max_lds_encode_bytes() / max_lds_decode_bytes().  Larger blocks take the
// global-memory path:
//   encode: bit transpose of every block into a global scratch (the
//           k_bitshuffle kernels) -> k_lz4_encode_big (lz4_encode.hip): one
//           wave per block runs the wave-parallel parse with the table in LDS
//           and the block read from the scratch -> the usual offset scan +
//           compaction;
//   decode: the block index and k_seq_scan_big (one wave per block walks and
//           validates every record with LZ4_decompress_safe's exact checks)
//           -> k_lz4_exec_big (lz4_decode.hip): one wave per block executes
//           the sequences wave-parallel into a global scratch -> inverse bit
//           transpose into the output.
// This file holds the launchers of that path and, as A/B variant 1024 only
// (bshuf_set_variant), the round-2 kernels that parse and copy on lane 0 of
// one workgroup per block with the table in global memory.
#include "launch.h"

namespace bshuf {

namespace {

// Unaligned little-endian loads from global memory: two aligned dwords and
// v_alignbyte (the scratch is padded, so the over-read stays inside it).
__device__ __forceinline__ uint32_t g_rd32(const uint8_t* p) {
    const uint32_t* w = reinterpret_cast<const uint32_t*>((uintptr_t)p & ~(uintptr_t)3);
    return __builtin_amdgcn_alignbyte(w[1], w[0], (uint32_t)((uintptr_t)p & 3));
}

__device__ __forceinline__ uint64_t g_rd64(const uint8_t* p) {
    return (uint64_t)g_rd32(p) | ((uint64_t)g_rd32(p + 4) << 32);
}

__device__ __forceinline__ uint32_t g_hash(const uint8_t* p, bool wide) {
    return wide ? hash5(g_rd64(p)) : hash4(g_rd32(p));
}

__device__ __forceinline__ uint8_t* put_len(uint8_t* op, int len) {
    for (; len >= 255; len -= 255) *op++ = 255;
    *op++ = (uint8_t)len;
    return op;
}

__device__ __forceinline__ void copy_bytes(uint8_t* d, const uint8_t* s, int n) {
    for (int i = 0; i < n; i++) d[i] = s[i];
}

// LZ4_compress_default of src[0, n) (lz4/lz4.c:1002-1331 for noDict,
// acceleration 1, notLimited output; byU16/hash4 below 65547 bytes, else
// byU32/hash5 with the 65535 distance check) with a zeroed table `tab` in
// global memory.  Returns the compressed size.
__device__ int lz4_compress_seq(const uint8_t* src, const int n, uint8_t* dst, uint32_t* tab) {
    uint8_t* op = dst;
    int anchor = 0;
    const bool wide = n >= kU16TableLimit;
    if (n >= kLz4MinLength) {
        const int limit = n - kMfLimit + 1;  // mflimitPlusOne
        const int matchlimit = n - kLastLiterals;
        tab[g_hash(src, wide)] = 0;
        int ip = 1;
        for (;;) {
            int match;
            {
                int fwd = ip, step = 1, nbm = 64;  // skip acceleration (lz4/lz4.c:1042-1101)
                for (;;) {
                    const int cur = fwd;
                    const uint32_t h = g_hash(src + cur, wide);
                    const uint32_t cand = tab[h];
                    ip = fwd;
                    fwd += step;
                    step = nbm++ >> 6;
                    if (fwd > limit) goto last_literals;
                    tab[h] = (uint32_t)cur;
                    if (wide && cand + kMaxDistance < (uint32_t)cur) continue;
                    if (g_rd32(src + cand) == g_rd32(src + ip)) {
                        match = (int)cand;
                        break;
                    }
                }
            }
            // catch up (lz4/lz4.c:1105-1109)
            while (ip > anchor && match > 0 && src[ip - 1] == src[match - 1]) {
                ip--;
                match--;
            }
            uint8_t* token = op++;
            {
                const int lit = ip - anchor;
                if (lit >= 15) {
                    *token = 15 << 4;
                    op = put_len(op, lit - 15);
                } else {
                    *token = (uint8_t)(lit << 4);
                }
                copy_bytes(op, src + anchor, lit);
                op += lit;
            }
            for (;;) {
                const int off = ip - match;  // (lz4/lz4.c:1133-1226)
                *op++ = (uint8_t)off;
                *op++ = (uint8_t)(off >> 8);
                int a = ip + kMinMatch, b = match + kMinMatch;
                while (a + 4 <= matchlimit && g_rd32(src + a) == g_rd32(src + b)) a += 4, b += 4;
                while (a < matchlimit && src[a] == src[b]) a++, b++;
                const int mc = a - (ip + kMinMatch);
                ip += mc + kMinMatch;
                if (mc >= 15) {
                    *token += 15;
                    op = put_len(op, mc - 15);
                } else {
                    *token += (uint8_t)mc;
                }
                anchor = ip;
                if (ip >= limit) goto last_literals;
                tab[g_hash(src + ip - 2, wide)] = (uint32_t)(ip - 2);
                // immediate re-test at ip, no catch-up (lz4/lz4.c:1255-1293)
                const uint32_t h = g_hash(src + ip, wide);
                const uint32_t cand = tab[h];
                tab[h] = (uint32_t)ip;
                if ((!wide || cand + kMaxDistance >= (uint32_t)ip) &&
                    g_rd32(src + cand) == g_rd32(src + ip)) {
                    token = op++;
                    *token = 0;
                    match = (int)cand;
                    continue;
                }
                break;
            }
            ip++;
        }
    }
last_literals: {
    const int run = n - anchor;
    if (run >= 15) {
        *op++ = 15 << 4;
        op = put_len(op, run - 15);
    } else {
        *op++ = (uint8_t)(run << 4);
    }
    copy_bytes(op, src + anchor, run);
    op += run;
}
    return (int)(op - dst);
}

// One workgroup per block: record [BE32 c][c bytes] into the block's slot.
__global__ __launch_bounds__(64) void k_lz4_encode_seq(const uint8_t* __restrict__ shuf, Layout L,
                                                        uint8_t* __restrict__ scratch, int64_t slot,
                                                        uint64_t* __restrict__ foot,
                                                        uint32_t* __restrict__ tables) {
    const int64_t k = blockIdx.x;
    if (threadIdx.x != 0) return;
    const int m = k < L.nfull ? L.bs : L.last;
    const int n = m * L.E;
    uint8_t* out = scratch + k * slot;
    const int c = lz4_compress_seq(shuf + k * (int64_t)L.bs * L.E, n, out + 4,
                                   tables + k * (int64_t)kLargeTableWords);
    out[0] = (uint8_t)((uint32_t)c >> 24);
    out[1] = (uint8_t)((uint32_t)c >> 16);
    out[2] = (uint8_t)((uint32_t)c >> 8);
    out[3] = (uint8_t)c;
    foot[k] = 4 + (uint64_t)c;
}

// One workgroup per block: runs the sequences k_seq_scan validated (its
// token positions in seq, its verdict in status) into the block's slice of
// the scratch; the record format is LZ4's (lz4/lz4.c:2083-2435), the checks
// already passed, so this is the plain copy loop.  Offset 0 writes zeros
// (the LZ4_write32(op, 0) seed of lz4/lz4.c:501, 2407).
__global__ __launch_bounds__(64) void k_lz4_exec_seq(const uint8_t* __restrict__ in,
                                                      int64_t in_nbytes,
                                                      const uint64_t* __restrict__ offs,
                                                      int64_t* __restrict__ status,
                                                      const uint32_t* __restrict__ seq, Layout L,
                                                      uint8_t* __restrict__ shuf, long long* bad) {
    const int64_t k = blockIdx.x;
    if (threadIdx.x != 0) return;
    const int64_t st = status[k];
    if (st < 0) {
        atomicMax(bad, (long long)k);
        return;
    }
    const int64_t o0 = (int64_t)offs[k];
    const uint8_t* rec = in + o0;
    const int clen = (int)be32_load(rec);
    const uint8_t* P = rec + 4;
    const uint32_t* pos = seq + o0 / 3;
    uint8_t* D = shuf + k * (int64_t)L.bs * L.E;
    int op = 0;
    const int ns = (int)st;
    for (int i = 0; i < ns; i++) {
        int q = (int)pos[i];
        const int tok = P[q++];
        int lit = tok >> 4;
        if (lit == 15) {
            int b;
            do {
                b = P[q++];
                lit += b;
            } while (b == 255);
        }
        copy_bytes(D + op, P + q, lit);
        q += lit;
        op += lit;
        if (i + 1 == ns) break;  // the last sequence has no match
        const int off = P[q] | (P[q + 1] << 8);
        q += 2;
        int ml = tok & 15;
        if (ml == 15) {
            int b;
            do {
                b = P[q++];
                ml += b;
            } while (b == 255);
        }
        ml += kMinMatch;
        if (off == 0) {
            for (int j = 0; j < ml; j++) D[op + j] = 0;
        } else {
            for (int j = 0; j < ml; j++) D[op + j] = D[op - off + j];
        }
        op += ml;
    }
    (void)in_nbytes;
    status[k] = (int64_t)clen + 4;
}

}  // namespace

int64_t max_lds_encode_bytes() { return max_device_block_bytes(); }

int64_t max_lds_decode_bytes() {
    // decoded block + 16 + record (bound + header + 32 slack, 16-aligned) in 160 KiB
    int64_t n = 160 * 1024;
    while (n > 0) {
        const int64_t rec = (lz4_bound((int)n) + 4 + 32 + 15) & ~(int64_t)15;
        if (((n + 15) & ~(int64_t)15) + 16 + rec <= 160 * 1024) break;
        n -= 8;
    }
    return n;
}

hipError_t launch_encode_large(const uint8_t* in, const Layout& L, const EncodeBufs& b,
                               uint8_t* shuf, uint32_t* tables, hipStream_t s) {
    const int64_t nb = L.nblocks();
    if (nb == 0) return hipSuccess;
    hipError_t e = launch_transpose(in, shuf, L, true, s);
    if (e != hipSuccess) return e;
    if (tuning_variant() != 1024) return launch_encode_big(shuf, L, b, s);
    // A/B variant 1024: the lane-0 parse with the table in global memory
    e = dev_fill(tables, 0, (size_t)nb * kLargeTableWords * 4, s);
    if (e != hipSuccess) return e;
    ProfScope prof("k_lz4_encode_seq", s);
    hipLaunchKernelGGL(k_lz4_encode_seq, dim3((unsigned)nb), dim3(64), 0, s, shuf, L, b.scratch, b.slot,
                       b.foot, tables);
    return hipGetLastError();
}

hipError_t launch_decode_large(const uint8_t* in, int64_t in_nbytes, uint8_t* out, const Layout& L,
                               const DecodeBufs& b, uint8_t* shuf, hipStream_t s) {
    const int64_t nb = L.nblocks();
    if (nb == 0) return hipSuccess;
    hipError_t e = hipSuccess;
    if (tuning_variant() != 1024) {
        e = launch_exec_big(in, L, b, shuf, s);
    } else {  // A/B variant 1024: the lane-0 copy loop
        ProfScope prof("k_lz4_exec_seq", s);
        hipLaunchKernelGGL(k_lz4_exec_seq, dim3((unsigned)nb), dim3(64), 0, s, in, in_nbytes, b.offs,
                           b.status, b.seq, L, shuf, b.bad);
        e = hipGetLastError();
    }
    if (e != hipSuccess) return e;
    return launch_transpose(shuf, out, L, false, s);
}

}  // namespace bshuf
