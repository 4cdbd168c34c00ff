// lz4_encode.hip -- K1+K3 fused: bit transpose + LZ4 block compression, one
// 64-lane wavefront per bitshuffle block; K5: ordered placement of the blocks.
//
// Reference path: bshuf_compress_lz4 -> bshuf_blocked_wrap_fun ->
// bshuf_compress_lz4_block (src/bitshuffle.c:36-79) -> bshuf_trans_bit_elem +
// LZ4_compress_default (lz4/lz4.c:1472 -> 930-1338).  The LZ4 parse here is
// the SAME greedy parse (bit-exact output), restructured for a wavefront:
//
//  * search: the probe positions of one search are fixed in advance by the
//    skip schedule (probe_offset), so 64 lanes probe 64 consecutive candidate
//    positions at once.  The sequential semantics "read table, then insert
//    this position" are kept by (1) reading all 64 old entries, (2) inserting
//    all 64 tentatively and reading back -- a lane that does not read its own
//    position shares its hash with another lane of the window, (3) resolving
//    such groups so each lane's candidate is the latest EARLIER lane with the
//    same hash, (4) taking the first matching lane by ballot, and (5) undoing
//    the inserts of lanes after that match.
//  * catch-up, match length (LZ4_count) and the 255-run length bytes are
//    ballots over 64 byte/dword lanes.
//  * the block (8 KiB by default) and the 16 KiB hash table live in LDS;
//    compressed bytes stream straight to a per-block scratch slot in HBM.
//
// Placement (the iochain hand-off of src/iochain.c:67-89): every block writes
// [BE32 c][c bytes] into its fixed scratch slot and 4+c into foot[]; an
// exclusive scan gives the output offsets; k_compact moves each record to its
// final, packed position.
#include <hipcub/hipcub.hpp>

#include "launch.h"

namespace bshuf {

namespace {

constexpr int kTableBytes = 16384;  // byU16: 8192 x u16, byU32: 4096 x u32
constexpr int kDataPad = 16;

struct EncArgs {
    const uint8_t* in;
    uint8_t* scratch;
    uint64_t* foot;
    int64_t slot;
    Layout L;
};

// The hash table, addressed explicitly in the LDS address space: a plain
// volatile generic pointer compiles to flat_load/flat_store sc0 sc1, whose
// vmcnt(0) waits would drain every outstanding global load and store.
// volatile keeps the tentative insert -> read-back order of the search.
typedef __attribute__((address_space(3))) volatile uint16_t lds_vu16;
typedef __attribute__((address_space(3))) volatile uint32_t lds_vu32;

template <bool WIDE>
struct Table {
    uint8_t* base;
    __device__ __forceinline__ uint32_t get(uint32_t h) const {
        if constexpr (WIDE)
            return ((lds_vu32*)base)[h];
        else
            return ((lds_vu16*)base)[h];
    }
    __device__ __forceinline__ void put(uint32_t h, uint32_t v) const {
        if constexpr (WIDE)
            ((lds_vu32*)base)[h] = v;
        else
            ((lds_vu16*)base)[h] = (uint16_t)v;
    }
};

template <bool WIDE>
__device__ __forceinline__ uint32_t hash_at(const uint8_t* D, int p) {
    if constexpr (WIDE)
        return hash5(lds_rd64(D, p));
    else
        return hash4(lds_rd32(D, p));
}

// Writes v as the LZ4 255-run continuation: v/255 bytes of 255, then v%255.
__device__ __forceinline__ int put_len(uint8_t* out, int op, int v, int lane) {
    const int nb = v / 255 + 1;
    const uint8_t last = (uint8_t)(v - 255 * (nb - 1));
    for (int i = lane; i < nb; i += kWave) out[op + i] = (i < nb - 1) ? (uint8_t)255 : last;
    return op + nb;
}

__device__ __forceinline__ void copy_bytes(uint8_t* out, int op, const uint8_t* D, int from,
                                           int len, int lane) {
    for (int i = lane; i < len; i += kWave) out[op + i] = D[from + i];
}

// LZ4_count(ip, match, limit): common prefix length of D[a..] and D[b..],
// bounded so that a + len <= lim.  64 lanes compare 4 bytes each.
__device__ __forceinline__ int match_count(const uint8_t* D, int n, int a, int b, int lim,
                                           int lane) {
    int total = 0;
    for (;;) {
        const int pa = a + total + 4 * lane;
        const int pb = b + total + 4 * lane;
        const uint32_t x = lds_rd32(D, min(pa, n)) ^ lds_rd32(D, min(pb, n));
        int eq = x ? (__ffs(x) - 1) >> 3 : 4;
        eq = min(eq, max(lim - pa, 0));
        const uint64_t full = ballot(eq == 4);
        if (full == ~0ull) {
            total += 4 * kWave;
            continue;
        }
        const int f = ffs64(~full);
        return total + 4 * f + __builtin_amdgcn_readlane(eq, f);
    }
}

// Greedy LZ4 parse of D[0..n) with table T (zeroed), output to `out`.
// Returns the compressed size.  Mirrors lz4/lz4.c:1002-1331 for noDict,
// acceleration 1, notLimited output.
template <bool WIDE>
__device__ int lz4_encode_block(const uint8_t* D, const int n, const Table<WIDE> T, uint8_t* out,
                                const int lane) {
    int op = 0, anchor = 0;
    if (n >= kLz4MinLength) {
        const int limit = n - kMfLimit + 1;  // mflimitPlusOne
        const int mlimit = n - kLastLiterals;
        int ip = 1;  // position 0 is pre-inserted: a zeroed table already says 0
        for (;;) {
            // ------------------------------------------------ search
            int mpos = -1, mref = 0;
            {
                const int p0 = ip;
                for (int k0 = 0;; k0 += kWave) {
                    const int pos = p0 + probe_offset(k0 + lane);
                    const bool valid = p0 + probe_offset(k0 + lane + 1) <= limit;
                    const uint64_t vmask = ballot(valid);
                    if (vmask == 0) break;
                    uint32_t seq = 0, h = 0, cold = 0;
                    if (valid) {
                        seq = lds_rd32(D, pos);
                        if constexpr (WIDE)
                            h = hash5(lds_rd64(D, pos));
                        else
                            h = hash4(seq);
                        cold = T.get(h);
                    }
                    if (valid) T.put(h, (uint32_t)pos);
                    const uint32_t rb = valid ? T.get(h) : (uint32_t)pos;
                    const bool loser = valid && rb != (uint32_t)pos;
                    uint32_t cand = cold;
                    bool grouped = false, first = true;
                    int next_member = kWave;
                    uint64_t lmask = ballot(loser);
                    while (lmask) {
                        const int l = ffs64(lmask);
                        const uint32_t hl = (uint32_t)__builtin_amdgcn_readlane((int)h, l);
                        const bool in_g = valid && h == hl;
                        const uint64_t g = ballot(in_g);
                        if (in_g) {
                            grouped = true;
                            const uint64_t below = g & ((1ull << lane) - 1ull);
                            if (below) {
                                cand = (uint32_t)(p0 + probe_offset(k0 + fls64(below)));
                                first = false;
                            }
                            const uint64_t above = lane == 63 ? 0ull : (g & (~0ull << (lane + 1)));
                            next_member = above ? ffs64(above) : kWave;
                        }
                        lmask &= ~g;
                    }
                    bool ok = false;
                    if (valid) {
                        const bool near = !WIDE || cand + kMaxDistance >= (uint32_t)pos;
                        ok = near && lds_rd32(D, (int)cand) == seq;
                    }
                    const uint64_t mm = ballot(ok);
                    if (mm) {
                        const int js = ffs64(mm);
                        if (valid) {
                            if (!grouped) {
                                if (lane > js) T.put(h, cold);
                            } else if (lane <= js && next_member > js) {
                                T.put(h, (uint32_t)pos);
                            } else if (first && lane > js) {
                                T.put(h, cold);
                            }
                        }
                        mpos = p0 + probe_offset(k0 + js);
                        mref = __builtin_amdgcn_readlane((int)cand, js);
                        break;
                    }
                    if (vmask != ~0ull) break;  // ran past mflimit: last literals
                    if (grouped && next_member == kWave) T.put(h, (uint32_t)pos);
                }
            }
            if (mpos < 0) break;
            ip = mpos;
            int ref = mref;
            // ------------------------------------------------ catch up
            for (;;) {
                const int a = ip - 1 - lane, b = ref - 1 - lane;
                const bool c = a >= anchor && b >= 0 && D[max(a, 0)] == D[max(b, 0)];
                const uint64_t cm = ballot(c);
                const int run = (~cm) ? ffs64(~cm) : kWave;
                ip -= run;
                ref -= run;
                if (run < kWave) break;
            }
            // ------------------------------------------------ literals
            int tokpos = op++;
            int tok;
            {
                const int lit = ip - anchor;
                tok = (lit >= 15 ? 15 : lit) << 4;
                if (lit >= 15) op = put_len(out, op, lit - 15, lane);
                copy_bytes(out, op, D, anchor, lit, lane);
                op += lit;
            }
            // ------------------------------------------------ matches
            for (;;) {
                const int off = ip - ref;
                if (lane == 0) {
                    out[op] = (uint8_t)off;
                    out[op + 1] = (uint8_t)(off >> 8);
                }
                op += 2;
                const int mc = match_count(D, n, ip + kMinMatch, ref + kMinMatch, mlimit, lane);
                ip += mc + kMinMatch;
                tok |= mc >= 15 ? 15 : mc;
                if (lane == 0) out[tokpos] = (uint8_t)tok;
                if (mc >= 15) op = put_len(out, op, mc - 15, lane);
                anchor = ip;
                if (ip >= limit) break;
                // fill table at ip-2, then test ip (lz4/lz4.c:1230-1293)
                const uint32_t h2 = hash_at<WIDE>(D, ip - 2);
                const uint32_t h0 = hash_at<WIDE>(D, ip);
                if (lane == 0) T.put(h2, (uint32_t)(ip - 2));
                const uint32_t c2 = uni(T.get(h0));
                if (lane == 0) T.put(h0, (uint32_t)ip);
                const bool near = !WIDE || c2 + kMaxDistance >= (uint32_t)ip;
                if (near && lds_rd32(D, (int)c2) == lds_rd32(D, ip)) {
                    tokpos = op++;
                    tok = 0;
                    ref = (int)c2;
                    continue;
                }
                break;
            }
            if (anchor >= limit) break;
            ip = anchor + 1;
        }
    }
    // ---------------------------------------------------- last literals
    {
        const int run = n - anchor;
        if (lane == 0) out[op] = (uint8_t)((run >= 15 ? 15 : run) << 4);
        op++;
        if (run >= 15) op = put_len(out, op, run - 15, lane);
        copy_bytes(out, op, D, anchor, run, lane);
        op += run;
    }
    return op;
}

// Registers holding one 8 KiB block for EK-byte elements: 8192 / 64 lanes.
template <int EK>
struct BlockRegs {
    static constexpr int kIters = EK ? 8192 / (kWave * 8 * EK) : 1;  // 64-group iterations
    uint32_t w[kIters][2 * (EK ? EK : 1)];
};

template <int EK>
__device__ __forceinline__ void issue_block_loads(BlockRegs<EK>& R, const uint8_t* src, int P,
                                                  int lane) {
#pragma unroll
    for (int it = 0; it < BlockRegs<EK>::kIters; it++) {
        const int g = it * kWave + lane;
        if (g < P) load_group<EK>(src + (int64_t)g * 8 * EK, R.w[it]);
    }
}

template <int EK>
__device__ __forceinline__ void transpose_regs_to_lds(const BlockRegs<EK>& R, uint8_t* D, int P,
                                                      int g0, int lane) {
#pragma unroll
    for (int it = 0; it < BlockRegs<EK>::kIters; it++) {
        const int g = g0 + it * kWave + lane;
        if (g < P) {
#pragma unroll
            for (int b = 0; b < EK; b++) {
                const uint64_t v = tr8x8(gather_byte_plane<EK>(R.w[it], b));
#pragma unroll
                for (int j = 0; j < 8; j++) D[(8 * b + j) * P + g] = (uint8_t)(v >> (8 * j));
            }
        }
    }
}

// Persistent: workgroup w handles blocks w, w+G, w+2G, ...  While block k is
// parsed out of LDS, the 8 KiB of block k+G are already in flight into
// registers, so HBM latency hides under the (LDS-latency-bound) parse.
// One wave per workgroup: LDS hand-offs need no s_barrier, and avoiding
// __syncthreads() keeps its release fence from draining the prefetch.
template <int EK, bool WIDE>
__global__ __launch_bounds__(64) void k_lz4_encode(EncArgs a, int64_t nb) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int lane = threadIdx.x;
    const int E = EK ? EK : a.L.E;
    uint8_t* D = smem + kTableBytes;
    const int64_t stride = gridDim.x;
    int64_t blk = blockIdx.x;
    if (blk >= nb) return;
    auto blk_m = [&](int64_t k) { return k < a.L.nfull ? a.L.bs : a.L.last; };
    auto blk_src = [&](int64_t k) { return a.in + k * (int64_t)a.L.bs * E; };

    BlockRegs<EK> R;
    constexpr int kRegGroups = BlockRegs<EK>::kIters * kWave;
    // a block fits the prefetch registers when its groups fit
    auto fits = [&](int m) { return EK != 0 && m / 8 <= kRegGroups; };
    if constexpr (EK != 0)
        if (fits(blk_m(blk))) issue_block_loads<EK>(R, blk_src(blk), blk_m(blk) / 8, lane);

    for (;;) {
        const int m = blk_m(blk);
        const int n = m * E;
        const int P = m / 8;
        const uint8_t* src = blk_src(blk);
        // zero the hash table (LZ4_initStream) and the read pad behind the block
        for (int i = lane; i < kTableBytes / 16; i += kWave)
            reinterpret_cast<uint4*>(smem)[i] = make_uint4(0, 0, 0, 0);
        if (lane < kDataPad / 4) reinterpret_cast<uint32_t*>(D + ((n + 3) & ~3))[lane] = 0;
        // bit transpose into LDS (bshuf_trans_bit_elem)
        if constexpr (EK != 0) {
            if (fits(m)) {
                transpose_regs_to_lds<EK>(R, D, P, 0, lane);
            } else {
                for (int g0 = 0; g0 < P; g0 += kRegGroups) {
                    BlockRegs<EK> T;
#pragma unroll
                    for (int it = 0; it < BlockRegs<EK>::kIters; it++) {
                        const int g = g0 + it * kWave + lane;
                        if (g < P) load_group<EK>(src + (int64_t)g * 8 * EK, T.w[it]);
                    }
                    transpose_regs_to_lds<EK>(T, D, P, g0, lane);
                }
            }
        } else {
            for (int i = lane; i < P * E; i += kWave) {
                const int g = i / E, b = i - g * E;
                uint64_t v = 0;
#pragma unroll
                for (int k = 0; k < 8; k++)
                    v |= (uint64_t)src[(int64_t)(8 * g + k) * E + b] << (8 * k);
                v = tr8x8(v);
#pragma unroll
                for (int j = 0; j < 8; j++) D[(8 * b + j) * P + g] = (uint8_t)(v >> (8 * j));
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        // prefetch the next block while this one is parsed
        const int64_t next = blk + stride;
        if constexpr (EK != 0)
            if (next < nb && fits(blk_m(next)))
                issue_block_loads<EK>(R, blk_src(next), blk_m(next) / 8, lane);

        uint8_t* out = a.scratch + blk * a.slot;
        const Table<WIDE> T{smem};
        const int c = lz4_encode_block<WIDE>(D, n, T, out + 4, lane);
        if (lane < 4) out[lane] = (uint8_t)((uint32_t)c >> (24 - 8 * lane));
        if (lane == 0) a.foot[blk] = 4 + (uint64_t)c;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        if (next >= nb) break;
        blk = next;
    }
}

// Move each [BE32 c][c bytes] record from its scratch slot to out + offs[k].
// Destination 16-byte chunks fully inside the record are composed from five
// source dwords with v_alignbyte and stored whole; the <= 2 edge chunks per
// record use byte stores (they share dwords with the neighbouring records).
__global__ __launch_bounds__(256) void k_compact(const uint8_t* __restrict__ scratch, int64_t slot,
                                                 const uint64_t* __restrict__ offs,
                                                 uint8_t* __restrict__ out) {
    const int64_t blk = blockIdx.x;
    const uint64_t dst0 = offs[blk];
    const int64_t len = (int64_t)(offs[blk + 1] - dst0);
    const uint8_t* rec = scratch + blk * slot;
    const uint32_t* rec32 = reinterpret_cast<const uint32_t*>(rec);
    const int64_t q0 = (int64_t)(dst0 >> 4);
    const int64_t q1 = (int64_t)((dst0 + len + 15) >> 4);
    for (int64_t q = q0 + threadIdx.x; q < q1; q += 256) {
        const int64_t d = q * 16;
        const int64_t s = d - (int64_t)dst0;  // record offset of this chunk's first byte
        if (s >= 0 && s + 16 <= len) {
            const int64_t w0 = s >> 2;
            const uint32_t sh = (uint32_t)(s & 3);
            uint32_t x[5];
#pragma unroll
            for (int i = 0; i < 5; i++) x[i] = rec32[w0 + i];
            uint4 v;
            v.x = __builtin_amdgcn_alignbyte(x[1], x[0], sh);
            v.y = __builtin_amdgcn_alignbyte(x[2], x[1], sh);
            v.z = __builtin_amdgcn_alignbyte(x[3], x[2], sh);
            v.w = __builtin_amdgcn_alignbyte(x[4], x[3], sh);
            *reinterpret_cast<uint4*>(out + d) = v;
        } else {
            for (int i = 0; i < 16; i++) {
                const int64_t r = s + i;
                if (r >= 0 && r < len) out[d + i] = rec[r];
            }
        }
    }
}

// The n%8 leftover elements are copied verbatim behind the last block
// (src/bitshuffle_core.c:1919-1926); their offset is only known on the device.
__global__ void k_encode_finish(const uint64_t* offs, int64_t nblocks, const uint8_t* tail_src,
                                int64_t tail, uint8_t* out, int64_t* result) {
    const uint64_t end = offs[nblocks];
    for (int i = threadIdx.x; i < tail; i += blockDim.x) out[end + i] = tail_src[i];
    if (threadIdx.x == 0) *result = (int64_t)end + tail;
}

template <int EK, bool WIDE>
hipError_t launch_enc_t(const EncArgs& a, int64_t nb, size_t lds, hipStream_t s) {
    auto fn = k_lz4_encode<EK, WIDE>;
    if (lds > 65536) {
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(fn),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
    }
    const int64_t grid = persistent_grid(reinterpret_cast<const void*>(fn), kWave, lds, nb);
    ProfScope prof("k_lz4_encode", s);
    hipLaunchKernelGGL(fn, dim3((unsigned)grid), dim3(kWave), lds, s, a, nb);
    return hipGetLastError();
}

}  // namespace

int64_t max_device_block_bytes() { return 160 * 1024 - kTableBytes - 64; }

int64_t encode_slot_bytes(const Layout& L) {
    const int64_t n = (int64_t)L.bs * L.E;
    // header + bound + 16 for the 5-dword over-read in k_compact, 16-aligned
    return ((4 + (int64_t)lz4_bound((int)n) + 16) + 15) & ~(int64_t)15;
}

size_t encode_scan_tmp_bytes(int64_t nblocks) {
    size_t bytes = 0;
    (void)hipcub::DeviceScan::ExclusiveSum(nullptr, bytes, (const uint64_t*)nullptr, (uint64_t*)nullptr,
                                     (int)(nblocks + 1));
    return bytes;
}

hipError_t launch_encode(const uint8_t* in, uint8_t* out, const Layout& L, int64_t tail_bytes,
                         const EncodeBufs& b, int64_t* d_result, hipStream_t s) {
    const int64_t nb = L.nblocks();
    hipError_t e;
    if (nb > 0) {
        EncArgs a{in, b.scratch, b.foot, b.slot, L};
        const int64_t nmax = (int64_t)L.bs * L.E;
        const size_t lds = kTableBytes + ((nmax + 15) & ~15) + kDataPad;
        const bool wide = nmax >= kU16TableLimit;
        // the partial block decides its own table type, so a stream whose full
        // blocks need byU32 but partial block byU16 launches twice
        const bool wide_last = L.last && (int64_t)L.last * L.E >= kU16TableLimit;
        const bool aligned = ((uintptr_t)in & 15) == 0;
        const int ek = aligned && (L.E == 1 || L.E == 2 || L.E == 4 || L.E == 8) ? L.E : 0;
        auto go = [&](Layout LL, bool w, int64_t count, int64_t first) -> hipError_t {
            EncArgs aa = a;
            aa.L = LL;
            // shift the base so blockIdx 0 is block `first`
            aa.in = a.in + first * (int64_t)L.bs * L.E;
            aa.scratch = a.scratch + first * b.slot;
            aa.foot = a.foot + first;
            aa.L.nfull = LL.nfull - first;
#define BSHUF_E(EKV)                                                         \
    case EKV:                                                                \
        return w ? launch_enc_t<EKV, true>(aa, count, lds, s)                \
                 : launch_enc_t<EKV, false>(aa, count, lds, s);
            switch (ek) {
                BSHUF_E(0)
                BSHUF_E(1)
                BSHUF_E(2)
                BSHUF_E(4)
                BSHUF_E(8)
            }
#undef BSHUF_E
            return hipErrorInvalidValue;
        };
        if (wide == wide_last || !L.last) {
            e = go(L, wide, nb, 0);
        } else {
            Layout Lf = L;
            Lf.last = 0;
            e = go(Lf, wide, L.nfull, 0);
            if (e == hipSuccess) e = go(L, wide_last, 1, L.nfull);
        }
        if (e != hipSuccess) return e;
    }
    e = hipMemsetAsync(b.foot + nb, 0, sizeof(uint64_t), s);
    if (e != hipSuccess) return e;
    size_t tmp = b.scan_tmp_bytes;
    {
        ProfScope prof("scan_block_offsets", s);
        e = hipcub::DeviceScan::ExclusiveSum(b.scan_tmp, tmp, b.foot, b.offs, (int)(nb + 1), s);
    }
    if (e != hipSuccess) return e;
    if (nb > 0) {
        ProfScope prof("k_compact", s);
        hipLaunchKernelGGL(k_compact, dim3((unsigned)nb), dim3(256), 0, s, b.scratch, b.slot,
                           b.offs, out);
        e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    const uint8_t* tail_src = in + (L.nfull * (int64_t)L.bs + L.last) * L.E;
    ProfScope prof("k_encode_finish", s);
    hipLaunchKernelGGL(k_encode_finish, dim3(1), dim3(64), 0, s, b.offs, nb, tail_src, tail_bytes,
                       out, d_result);
    return hipGetLastError();
}

}  // namespace bshuf
