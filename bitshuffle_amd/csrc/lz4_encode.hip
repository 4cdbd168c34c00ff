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
//    this position" come from ONE returning LDS atomic per window
//    (ds_mskor_rtn_b32 on the u16 table, ds_wrxchg_rtn_b32 on the u32 one):
//    the LDS serialises same-entry lanes in lane order, so each lane gets the
//    latest EARLIER lane's position or the table's.  The first matching lane
//    wins by ballot, and the inserts of later lanes are undone.  The lane-order
//    property is checked on the device before first use; a device without it
//    gets the insert/read-back/group-resolution window instead (VAR bit 128).
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

#include <atomic>
#include <type_traits>
#include <cstdlib>
#include <mutex>

#include "launch.h"
#include "lds_copy.h"

namespace bshuf {

namespace {

constexpr int kTableBytes = 16384;  // byU16: 8192 x u16, byU32: 4096 x u32

// Diagnostic build only (-DBSHUF_DIAG, tools/diag_encode.py): per-phase
// s_memtime cycle sums and event counters.  The product build compiles these
// macros to nothing.
#ifdef BSHUF_DIAG
// 64 copies of the 32 counters, picked by workgroup, so the flush atomics of
// 1,536 resident waves do not serialise on 32 addresses.
constexpr int kDiagCopies = 64;
__device__ unsigned long long g_diag[kDiagCopies * 32];
#define DIAG_DECL                                   \
    uint64_t _dt = __builtin_amdgcn_s_memtime();    \
    uint64_t _acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};    \
    uint32_t _cnt[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#define STAMP(i)                                       \
    do {                                               \
        const uint64_t _n = __builtin_amdgcn_s_memtime(); \
        _acc[i] += _n - _dt;                           \
        _dt = _n;                                      \
    } while (0)
#define COUNT(i, v) (_cnt[i] += (v))
#define DIAG_FLUSH                                                          \
    do {                                                                    \
        if (lane == 0)                                                      \
            for (int _i = 0; _i < 8; _i++) {                                \
                atomicAdd(&g_diag[(blockIdx.x % kDiagCopies) * 32 + _i],   \
                          (unsigned long long)_acc[_i]);                    \
                atomicAdd(&g_diag[(blockIdx.x % kDiagCopies) * 32 + 8 + _i], \
                          (unsigned long long)_cnt[_i]);                    \
            }                                                               \
    } while (0)
// kernel-level phases of k_lz4_encode (slots 16..19): zero + transpose,
// parse, emission + copy-out, everything else
#define KDIAG_DECL                                   \
    uint64_t _kt = __builtin_amdgcn_s_memtime();     \
    uint64_t _kacc[4] = {0, 0, 0, 0};
#define KSTAMP(i)                                       \
    do {                                                \
        const uint64_t _n = __builtin_amdgcn_s_memtime(); \
        _kacc[i] += _n - _kt;                           \
        _kt = _n;                                       \
    } while (0)
#define KDIAG_FLUSH                                                                     \
    do {                                                                                \
        if (lane == 0)                                                                  \
            for (int _i = 0; _i < 4; _i++)                                              \
                atomicAdd(&g_diag[(blockIdx.x % kDiagCopies) * 32 + 16 + _i], _kacc[_i]); \
    } while (0)
#else
#define KDIAG_DECL
#define KSTAMP(i) ((void)0)
#define KDIAG_FLUSH ((void)0)
#define DIAG_DECL
#define STAMP(i) ((void)0)
#define COUNT(i, v) ((void)0)
#define DIAG_FLUSH ((void)0)
#endif
constexpr int kDataPad = 16;

struct EncArgs {
    const uint8_t* in;
    uint8_t* scratch;
    uint64_t* foot;
    int64_t slot;
    Layout L;
    int32_t desc_ok;   // LDS holds kDescBytes of sequence descriptors at D + desc_off
    int32_t desc_off;
    const Seg* segs;   // batch: per-stream table (nullptr: the single stream in/L)
    const uint32_t* blk_seg;
    int32_t raw8;      // EK == 0: every block source is 8-aligned (LDS-staged transpose)
    int64_t blk0;      // batch: global index of this launch's block 0 (pipelined segments)
};

// Returning LDS atomics as inline asm (no builtin exists for ds_mskor); the
// asm waits for its own result, so the compiler never reads it early.
__device__ __forceinline__ uint32_t lds_addr(lds8* p) { return (uint32_t)(uintptr_t)p; }
__device__ __forceinline__ uint32_t lds_addr(void* p) { return (uint32_t)(uintptr_t)(lds8*)p; }

// k_lz4_encode has no static LDS, so its dynamic LDS starts at address 0
// (checked on the host before the launch, lds_layout_ok).  Addressing it from
// the constant 0 instead of the extern array's relocated address lets the
// compiler fold constant offsets into the DS instructions' immediates.
__device__ __forceinline__ lds8* lds_origin() { return (lds8*)(uintptr_t)0; }
__device__ __forceinline__ uint32_t lds_mskor_rtn(uint32_t addr, uint32_t mask, uint32_t data) {
    uint32_t r;
    asm volatile("ds_mskor_rtn_b32 %0, %1, %2, %3\n\ts_waitcnt lgkmcnt(0)"
                 : "=v"(r) : "v"(addr), "v"(mask), "v"(data) : "memory");
    return r;
}
__device__ __forceinline__ uint32_t lds_xchg_rtn(uint32_t addr, uint32_t data) {
    uint32_t r;
    asm volatile("ds_wrxchg_rtn_b32 %0, %1, %2\n\ts_waitcnt lgkmcnt(0)"
                 : "=v"(r) : "v"(addr), "v"(data) : "memory");
    return r;
}

// The hash table, addressed explicitly in the LDS address space: a plain
// volatile generic pointer compiles to flat_load/flat_store sc0 sc1, whose
// vmcnt(0) waits would drain every outstanding global load and store.
// volatile keeps the tentative insert -> read-back order of the fallback search.
typedef __attribute__((address_space(3))) volatile uint16_t lds_vu16;
typedef __attribute__((address_space(3))) volatile uint32_t lds_vu32;

template <bool WIDE>
struct Table {
    lds8* base;
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
    // Stores v at entry h and returns the entry as this lane found it.  The
    // LDS unit serialises same-address lanes of one returning atomic in lane
    // order (checked on the device before first use: lds_atomics_lane_ordered),
    // so lane j gets the value of the highest LOWER active lane with the same
    // entry, else the table's -- exactly the sequential insert-then-lookup.
    // exchange() when `doit`, else a read of entry h that changes nothing (a
    // mask-0 ds_mskor): every lane can issue it, no exec-mask switch (byU16)
    __device__ __forceinline__ uint32_t exchange_if(uint32_t h, uint32_t v, bool doit) const {
        static_assert(!WIDE, "byU16 table only");
        const uint32_t sh = 16u * (h & 1u);
        const uint32_t old = lds_mskor_rtn(lds_addr(base + 4 * (h >> 1)), doit ? 0xFFFFu << sh : 0u,
                                           doit ? v << sh : 0u);
        return (old >> sh) & 0xFFFFu;
    }
    __device__ __forceinline__ uint32_t exchange(uint32_t h, uint32_t v) const {
        if constexpr (WIDE) {
            return lds_xchg_rtn(lds_addr(base + 4 * h), v);
        } else {
            const uint32_t sh = 16u * (h & 1u);
            const uint32_t old = lds_mskor_rtn(lds_addr(base + 4 * (h >> 1)), 0xFFFFu << sh, v << sh);
            return (old >> sh) & 0xFFFFu;
        }
    }
};

// A block in GLOBAL memory (blocks too large for the LDS, k_lz4_encode_big):
// the same reads as the LDS block's, from aligned dwords of the transposed
// scratch (which is padded, so reads up to 12 bytes past a block stay inside
// it; those bytes never decide anything, as with the LDS block's pad).
struct GblBlk {
    const uint8_t* p;
    __device__ __forceinline__ uint32_t operator[](int i) const { return ((const gbl8c*)p)[i]; }
    __device__ __forceinline__ uint32_t w32(int a) const { return *(const gbl32c*)(p + a); }
};
// (the LDS overloads live in bshuf_dev.h, outside this unnamed namespace)
using bshuf::lds_rd32;
using bshuf::lds_rd64;
__device__ __forceinline__ uint32_t lds_rd32(const GblBlk& D, int p) {
    const int a = p & ~3;
    return __builtin_amdgcn_alignbyte(D.w32(a + 4), D.w32(a), (uint32_t)(p & 3));
}
__device__ __forceinline__ uint64_t lds_rd64(const GblBlk& D, int p) {
    const int a = p & ~3;
    const uint32_t s = (uint32_t)(p & 3), w0 = D.w32(a), w1 = D.w32(a + 4), w2 = D.w32(a + 8);
    return (uint64_t)__builtin_amdgcn_alignbyte(w1, w0, s) |
           ((uint64_t)__builtin_amdgcn_alignbyte(w2, w1, s) << 32);
}
__device__ __forceinline__ uint32_t blk_w32(const lds8* D, int a) { return *(const lds32*)(D + a); }
__device__ __forceinline__ uint32_t blk_w32(const GblBlk& D, int a) { return D.w32(a); }

// A count / re-test window read at p (p < n + 260).  An LDS block is followed
// by >= 2 KiB of readable LDS (pad + descriptors), whose bytes never decide
// anything (every count is capped at mlimit), so it needs no clamp; the
// global-memory block's scratch is padded by only 12 bytes.
__device__ __forceinline__ uint32_t rdw(const lds8* D, int p, int n) {
    (void)n;
    return lds_rd32(D, p);
}
__device__ __forceinline__ uint32_t rdw(const GblBlk& D, int p, int n) { return lds_rd32(D, min(p, n)); }

template <bool WIDE, class Blk>
__device__ __forceinline__ uint32_t hash_at(const Blk& D, int p) {
    if constexpr (WIDE)
        return hash5(lds_rd64(D, p));
    else
        return hash4(lds_rd32(D, p));
}

constexpr int kWinBytes = 4 * kWave;  // bytes one dword-per-lane wave access covers

// ---------------------------------------------------------------------------
// Emission policies of the parse.  The parse reports each sequence once its
// match is final (seq) and the trailing literal run (last).
//
//  * EmitDesc (default): an 8-byte descriptor per sequence in LDS; the LZ4
//    bytes (and the record size) come afterwards from emit_sequences,
//    wave-parallel, so literal copies, length runs and size bookkeeping are
//    off the serial parse entirely.
//  * EmitBytes: writes the bytes straight to global memory from inside the
//    parse, `op` being the running compressed size (blocks whose record does
//    not fit the LDS staging area, the rare block with more sequences than
//    descriptor slots, and the A/B variant 2).
// ---------------------------------------------------------------------------

constexpr int kLaneRun = 128;              // emission: longest literal run copied per lane
constexpr int kLaneRunMin = 4;             // ... when the batch has at least this many long runs
constexpr int kDescMax = 256;              // descriptor slots per block
constexpr int kDescBytes = 8 * kDescMax;   // LDS behind the block

// Sequence s's descriptor: two dwords in LDS (ip | off << 16, lit | ml << 16,
// ml = mc + kMinMatch: the match length itself, which the asm re-test loop has
// at hand without the subtraction),
// stored by every lane (same address, same value: no exec-mask switch on the
// parse's chain).  The record size is not tracked during the parse:
// emit_sequences' prefix sum gives it.
struct EmitDesc {
    lds32* desc;
    int lane;
    int ns = 0;   // sequences recorded
    int la = 0;   // anchor of the last literal run
    // Never fails inside the parse (no early exit on its chains): past the
    // last slot it keeps overwriting that slot, and the caller re-parses the
    // block with the inline emitter when ns ends above kDescMax.
    __device__ __forceinline__ bool seq(int& op, int anchor, int ip, int off, int mc) {
        ((lds64v*)desc)[min(ns, kDescMax - 1)] = u32x2{(uint32_t)ip | ((uint32_t)off << 16),
                                                      (uint32_t)(ip - anchor) | ((uint32_t)(mc + kMinMatch) << 16)};
        ns++;
        (void)op;
        return true;
    }
    __device__ __forceinline__ void last(int& op, int anchor, int n) {
        (void)op;
        (void)n;
        la = anchor;
    }
};

template <class Blk = const lds8*>
struct EmitBytes {
    uint8_t* out;
    Blk D_;  // the block (literal source)
    int lane;
    __device__ __forceinline__ void byte(int& op, uint32_t b) {
        if (lane == 0) ((gbl8*)out)[op] = (uint8_t)b;
        op++;
    }
    __device__ __forceinline__ void len(int& op, int v) {
        const int nb = v / 255 + 1;
        const uint8_t last = (uint8_t)(v - 255 * (nb - 1));
        for (int i = lane; i < nb; i += kWave) ((gbl8*)out)[op + i] = (i < nb - 1) ? (uint8_t)255 : last;
        op += nb;
    }
    __device__ __forceinline__ void copy(int& op, const Blk& D, int from, int n) {
        if (n <= kWave) {
            if (lane < n) ((gbl8*)out)[op + lane] = (uint8_t)D[from + lane];
        } else {
            // long runs (the last literals above all): 16-byte stores to the
            // ABSOLUTE 16-byte chunks inside the run, composed from five LDS
            // dwords; the <= 15 bytes at each edge go byte-wise
            const uintptr_t a0 = (uintptr_t)(out + op), a1 = a0 + (uintptr_t)n;
            const uintptr_t q0 = (a0 + 15) & ~(uintptr_t)15, q1 = a1 & ~(uintptr_t)15;
            const int head = (int)(q0 - a0), tailn = (int)(a1 - q1);
            const int e = lane < 16 ? lane : n - tailn + (lane - 16);
            if (lane < 16 ? lane < head : lane - 16 < tailn) ((gbl8*)out)[op + e] = (uint8_t)D[from + e];
            const int nch = (int)((q1 - q0) >> 4);
            for (int c = lane; c < nch; c += kWave) {
                const int s = from + head + 16 * c;
                const int a = s & ~3;
                const uint32_t sh = (uint32_t)(s & 3);
                const uint32_t x0 = blk_w32(D, a), x1 = blk_w32(D, a + 4), x2 = blk_w32(D, a + 8),
                               x3 = blk_w32(D, a + 12), x4 = blk_w32(D, a + 16);
                *(gbl128*)(q0 + 16 * (uintptr_t)c) =
                    u32x4{__builtin_amdgcn_alignbyte(x1, x0, sh), __builtin_amdgcn_alignbyte(x2, x1, sh),
                          __builtin_amdgcn_alignbyte(x3, x2, sh), __builtin_amdgcn_alignbyte(x4, x3, sh)};
            }
        }
        op += n;
    }
    __device__ __forceinline__ bool seq(int& op, int anchor, int ip, int off, int mc) {
        const int lit = ip - anchor;
        byte(op, (uint32_t)(((lit >= 15 ? 15 : lit) << 4) | (mc >= 15 ? 15 : mc)));
        if (lit >= 15) len(op, lit - 15);
        copy(op, D_, anchor, lit);
        byte(op, (uint32_t)(off & 0xFF));
        byte(op, (uint32_t)(off >> 8));
        if (mc >= 15) len(op, mc - 15);
        return true;
    }
    __device__ __forceinline__ void last(int& op, int anchor, int n) {
        const int run = n - anchor;
        byte(op, (uint32_t)((run >= 15 ? 15 : run) << 4));
        if (run >= 15) len(op, run - 15);
        copy(op, D_, anchor, run);
    }
};

// Each lane with `mine` copies its literal run of n bytes (1..kLaneRun) from
// D[sp] to S[dp] (LDS, disjoint; the block D has readable bytes past its end):
// destination dword t is v_alignbyte of source dwords t and t+1 at one shift
// for the whole run, so only the head and tail dwords (shared with the
// token / length / offset bytes around the run) take masked writes -- the
// whole dwords between go out as plain writes, four per step, with no
// per-piece mask arithmetic (lane_copy16 recomputes five masks per 16 bytes).
#ifndef BSHUF_RUNS_PIPE
#define BSHUF_RUNS_PIPE 1
#endif
__device__ __forceinline__ void lane_runs(const lds8* D, int sp, lds8* S, int dp, int n, bool mine) {
    const int k = dp & 3;
    const int b = sp - k;  // source byte of destination dword 0's byte 0 (may be < 0: masked off)
    const uint32_t r = (uint32_t)(b & 3);
    const lds32* W = (const lds32*)(D + (b & ~3));
    lds32* O = (lds32*)(S + (dp & ~3));
    const int nd = ((dp + n + 3) >> 2) - (dp >> 2);  // destination dwords touched
    if (mine) {
        const int e = dp + n - 4 * ((dp + n - 1) >> 2);  // bytes of the run in its last dword, 1..4
        const uint32_t mt = e >= 4 ? ~0u : ((1u << (8 * e)) - 1u);
        uint32_t mh = ~0u << (8 * k);
        if (nd == 1) mh &= mt;
        const uint32_t vh = __builtin_amdgcn_alignbyte(W[1], W[0], r);
        lds_write_masked(lds_addr((lds8*)O), mh, vh & mh);
        if (nd > 1) {
            const uint32_t vt = __builtin_amdgcn_alignbyte(W[nd], W[nd - 1], r);
            lds_write_masked(lds_addr((lds8*)(O + nd - 1)), mt, vt & mt);
        }
    }
    const int last = mine ? nd - 2 : 0;  // interior dwords 1 .. last
#if BSHUF_RUNS_PIPE
    // software-pipelined: the next step's four source dwords are read before
    // this step's four writes (block and record are disjoint LDS), so a step
    // waits for reads issued one step earlier instead of its own
    if (ballot(1 <= last) == 0) return;
    uint32_t a0 = 0, a1 = 0, a2 = 0, a3 = 0, a4 = 0;
    if (1 <= last) {
        a0 = W[1];
        a1 = W[2];
        a2 = W[3];
        a3 = W[4];
        a4 = W[5];
    }
    for (int t = 1;; t += 4) {
        const bool more = t + 4 <= last;
        uint32_t b1 = 0, b2 = 0, b3 = 0, b4 = 0;
        if (more) {
            b1 = W[t + 5];
            b2 = W[t + 6];
            b3 = W[t + 7];
            b4 = W[t + 8];
        }
        if (t <= last) {
            O[t] = __builtin_amdgcn_alignbyte(a1, a0, r);
            if (t + 1 <= last) O[t + 1] = __builtin_amdgcn_alignbyte(a2, a1, r);
            if (t + 2 <= last) O[t + 2] = __builtin_amdgcn_alignbyte(a3, a2, r);
            if (t + 3 <= last) O[t + 3] = __builtin_amdgcn_alignbyte(a4, a3, r);
        }
        if (ballot(more) == 0) break;
        a0 = a4;
        a1 = b1;
        a2 = b2;
        a3 = b3;
        a4 = b4;
    }
#else
    for (int t = 1; ballot(t <= last) != 0; t += 4) {
        if (t <= last) {
            const uint32_t w0 = W[t], w1 = W[t + 1], w2 = W[t + 2], w3 = W[t + 3], w4 = W[t + 4];
            O[t] = __builtin_amdgcn_alignbyte(w1, w0, r);
            if (t + 1 <= last) O[t + 1] = __builtin_amdgcn_alignbyte(w2, w1, r);
            if (t + 2 <= last) O[t + 2] = __builtin_amdgcn_alignbyte(w3, w2, r);
            if (t + 3 <= last) O[t + 3] = __builtin_amdgcn_alignbyte(w4, w3, r);
        }
    }
#endif
}

// Builds the LZ4 bytes of a parsed block from its descriptors, wave-parallel
// (lane = sequence; a prefix sum places every sequence): record payload at
// S[4..), literals from the block D.  The last literal run is sequence ns.
// Returns the payload size.  kRuns: literal runs by lane_runs (A/B bit
// 2097152), else lane_copy16 pieces.
template <bool kRuns, class Em>
__device__ __forceinline__ int emit_sequences(const lds8* D, const Em& em, const int n, lds8* S,
                                              const int lane) {
    const int ns = em.ns, la = em.la;
    int opb = 4;
    for (int b0 = 0; b0 <= ns; b0 += kWave) {
        const int s = b0 + lane;
        const bool m = s < ns;
        const bool act = s <= ns;
        int ip = n, off = 0, lit = act ? n - la : 0, mc = 0;
        if (m) {
            const u32x2 d = ((const lds64v*)em.desc)[s];
            const uint32_t x = d.x, y = d.y;
            ip = (int)(x & 0xFFFFu);
            off = (int)(x >> 16);
            lit = (int)(y & 0xFFFFu);
            mc = (int)(y >> 16) - kMinMatch;
        }
        const int le = lz4_ext_bytes(lit), me = m ? lz4_ext_bytes(mc) : 0;
        const int len = act ? 1 + le + lit + (m ? 2 + me : 0) : 0;
        const int incl = wave_incl_sum(len, lane);
        const int op = opb + incl - len;
        opb += __builtin_amdgcn_readlane(incl, kWave - 1);
        if (act) S[op] = (uint8_t)((min(lit, 15) << 4) | (m ? min(mc, 15) : 0));
        lane_len_run(S, op + 1, le, (uint32_t)(lit - 15) % 255u);
        const int lp = op + 1 + le, lsrc = ip - lit;
        // With several long runs in the batch (literal-heavy data): runs of up
        // to kLaneRun bytes are copied by their own lanes in 16-byte pieces,
        // all at once (pieces of neighbouring runs that share a dword land by
        // masked writes); otherwise, and for longer runs, run by run by the wave
        const int lane_max =
            __builtin_popcountll(ballot(lit > 16)) >= kLaneRunMin ? kLaneRun : 16;
        if constexpr (kRuns) {
            lane_runs(D, lsrc, S, lp, lit, lit > 0 && lit <= lane_max);
        } else {
            const bool mine = lit > 0 && lit <= lane_max;
            for (int d0 = 0; ballot(mine && d0 < lit) != 0; d0 += 16)
                if (mine && d0 < lit) lane_copy16(D, lsrc + d0, S, lp + d0, min(16, lit - d0));
        }
        for (uint64_t lm = ballot(lit > lane_max); lm; lm &= lm - 1) {
            const int l = ffs64(lm);
            wave_copy(D, __builtin_amdgcn_readlane(lsrc, l), S, __builtin_amdgcn_readlane(lp, l),
                      __builtin_amdgcn_readlane(lit, l), lane);
        }
        if (m) {
            S[lp + lit] = (uint8_t)(off & 0xFF);
            S[lp + lit + 1] = (uint8_t)(off >> 8);
        }
        lane_len_run(S, lp + lit + 2, me, (uint32_t)(mc - 15) % 255u);
    }
    return opb - 4;
}

// Catch-up (lz4/lz4.c:1105-1109) and LZ4_count (lz4/lz4.c:680-703) in one
// LDS round trip: the match bytes [ip, ip+4) are equal, so counting from
// ip+4 does not depend on how far the catch-up goes back, and the caught-up
// match length is back + count(ip+4).  `tail` returns the a-side dword of
// every lane for the LAST counted 256-byte window starting at `tail_base`.
struct CountOut {
    int back;
    int cnt;
    int tail_base;
    uint32_t tail;
};

// Equal bytes from the start of one 256-byte count window (va / vb: the a-
// and b-side dword of every lane), capped at lim, the bytes the window may
// count (mlimit - window start; <= 0: none).  256 means "all equal and the
// limit lies beyond": count on.  The first differing lane comes straight
// from the compare's ballot and its first differing byte from one readlane
// (no per-lane byte counts, no second ballot).
__device__ __forceinline__ int window_equal(uint32_t va, uint32_t vb, int lim) {
    const uint64_t ne = ballot(va != vb);
    int c = kWinBytes;
    if (ne) {
        const int f = ffs64(ne);
        const uint32_t x = (uint32_t)__builtin_amdgcn_readlane((int)(va ^ vb), f);
        c = 4 * f + (__builtin_ctz(x) >> 3);
    }
    return min(c, max(lim, 0));
}

// The re-test's match test and LZ4_count in one LDS round trip: counts the
// equal bytes from ip itself (the first window's lane 0 is the 4-byte
// test).  cnt = match length beyond kMinMatch, or -1 when there is no match.
template <class Blk>
__device__ __forceinline__ CountOut test_and_count(const Blk& D, int n, int ip, int ref,
                                                   int mlimit, int lane, uint32_t va0) {
    CountOut r;
    r.back = 0;
    uint32_t va = va0, vb = rdw(D, ref + 4 * lane, n);  // va0: the a-side, read ahead
    if (__builtin_amdgcn_readfirstlane(va ^ vb) != 0) {
        r.cnt = -1;
        return r;
    }
    for (int total = 0;; total += kWinBytes) {
        const int c = window_equal(va, vb, mlimit - (ip + total));
        if (c < kWinBytes) {
            r.cnt = total + c - kMinMatch;
            r.tail_base = ip + total;
            r.tail = va;
            return r;
        }
        va = rdw(D, ip + total + kWinBytes + 4 * lane, n);
        vb = rdw(D, ref + total + kWinBytes + 4 * lane, n);
    }
}

template <class Blk>
__device__ __forceinline__ CountOut catch_and_count(const Blk& D, int n, int ip, int ref,
                                                    int anchor, int mlimit, int lane) {
    CountOut r;
    // first forward window and backward bytes together
    const int a = ip + kMinMatch, b = ref + kMinMatch;
    uint32_t va = rdw(D, a + 4 * lane, n), vb = rdw(D, b + 4 * lane, n);
    const int ba = ip - 1 - lane, bb = ref - 1 - lane;
    const uint32_t ca = (uint32_t)D[max(ba, 0)], cb = (uint32_t)D[max(bb, 0)];
    // backward
    {
        uint64_t cm = ballot(ba >= anchor && bb >= 0 && ca == cb);
        int back = (~cm) ? ffs64(~cm) : kWave;
        if (back == kWave) {
            for (int base = kWave;; base += kWave) {
                const int xa = ip - 1 - base - lane, xb = ref - 1 - base - lane;
                cm = ballot(xa >= anchor && xb >= 0 && (uint32_t)D[max(xa, 0)] == (uint32_t)D[max(xb, 0)]);
                const int run = (~cm) ? ffs64(~cm) : kWave;
                back = base + run;
                if (run < kWave) break;
            }
        }
        r.back = back;
    }
    // forward
    for (int total = 0;; total += kWinBytes) {
        const int c = window_equal(va, vb, mlimit - (a + total));
        if (c < kWinBytes) {
            r.cnt = total + c;
            r.tail_base = a + total;
            r.tail = va;
            return r;
        }
        va = rdw(D, a + total + kWinBytes + 4 * lane, n);
        vb = rdw(D, b + total + kWinBytes + 4 * lane, n);
    }
}

// One lane's probe of the search skip schedule, advanced one window (64
// probes) at a time: with t = 62 + k, q = t >> 6 grows by one per window while
// t & 63 stays, so the closed form of probe_offset (exact for k >= 1; it gives
// 1 for k = 0) moves by 64 q + (t & 63) + 1, and that step by 64.
struct ProbeLane {
    int off, step;
    __device__ __forceinline__ void advance() {
        off += step;
        step += kWave;
    }
};
__device__ __forceinline__ ProbeLane probe_lane(int k) {
    const int t = 62 + k, q = t >> 6, r = t & 63;
    return ProbeLane{1 + 32 * q * (q - 1) + q * (r + 1), 64 * q + r + 1};
}

// read32 at position p from the a-side window registers (p - base in
// [0, 252]), without an LDS round trip.
__device__ __forceinline__ uint32_t win_rd32(uint32_t v, int base, int p) {
    const int t = p - base;
    const int l = t >> 2;
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)v, l);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)v, min(l + 1, kWave - 1));
    return __builtin_amdgcn_alignbyte(hi, lo, (uint32_t)(t & 3));
}

// ---------------------------------------------------------------------------
// Descriptors buffered in VGPRs (the hand-scheduled re-test below): sequence
// s's two descriptor dwords go into lane s % 64 of dlo / dhi by v_writelane
// (no LDS access on the parse's chain), and every 64 sequences the wave stores
// the batch with one coalesced ds_write2 into the same LDS slots EmitDesc
// uses.  Past kDescMax the batches are dropped (the caller re-parses with the
// inline emitter, as with EmitDesc).
// ---------------------------------------------------------------------------
struct EmitDescV {
    lds32* desc;
    int lane;
    int ns = 0;
    int la = 0;
    uint32_t dlo = 0, dhi = 0;
    __device__ __forceinline__ void store_batch(int first, int count) const {
        if (first < kDescMax && lane < count) ((lds64v*)desc)[first + lane] = u32x2{dlo, dhi};
    }
    __device__ __forceinline__ bool seq(int& op, int anchor, int ip, int off, int mc) {
        (void)op;
        const int slot = ns & (kWave - 1);
        if (lane == slot) {
            dlo = (uint32_t)ip | ((uint32_t)off << 16);
            dhi = (uint32_t)(ip - anchor) | ((uint32_t)(mc + kMinMatch) << 16);
        }
        ns++;
        if ((ns & (kWave - 1)) == 0) store_batch(ns - kWave, kWave);
        return true;
    }
    __device__ __forceinline__ void last(int& op, int anchor, int n) {
        (void)op;
        (void)n;
        la = anchor;
        store_batch(ns & ~(kWave - 1), ns & (kWave - 1));
    }
};

// The full search windows of the parse (every probe of the window and its
// successor inside mflimit, lz4/lz4.c:1042-1075) as one hand-scheduled loop:
// per window one hash per lane, ONE lane-ordered ds_mskor_rtn exchange, the
// candidates' bytes, one ballot; the next window's bytes are read beside the
// exchange.  State: vpos / vseq the current window's probe positions and
// their bytes, vnxt / vstep the next window's positions and the step after,
// qs / qstep the next window's lane-0 position (the current last lane's
// successor) on the scalar unit.  Exits:
//  kSrPartial  the next window is not full: the caller runs it (nwin full
//              windows were done);
//  kSrMatch    lane js of the current window matched; vcand holds every
//              lane's exchanged-out entry (candidate in its low 16 bits).
enum { kSrPartial = 0, kSrMatch = 1 };

__device__ __forceinline__ int search_chain(uint32_t& vpos, uint32_t& vnxt, uint32_t& vstep, uint32_t& vseq,
                                            int& qs, int& qstep, int& nwin, uint32_t& vcand, int& js,
                                            const int limit, const int n) {
    int code;
    uint32_t vh, va, vsh, vad, vm, vd, vold, vlo, vhi, vx1;
    asm volatile(
        "L_stop%=:\n\t"
        "s_cmp_gt_i32 %[qs], %[limit]\n\t"
        "s_cbranch_scc1 L_spart%=\n\t"
        "v_mul_lo_u32 %[vh], %[vseq], %[kmul]\n\t"
        "v_min_i32 %[va], %[n], %[vnxt]\n\t"
        "s_add_u32 %[qs], %[qs], %[qstep]\n\t"
        "s_add_u32 %[qstep], %[qstep], 64\n\t"
        "v_lshrrev_b32 %[vsh], 15, %[vh]\n\t"
        "v_lshrrev_b32 %[vad], 18, %[vh]\n\t"
        "v_and_b32 %[vsh], 16, %[vsh]\n\t"
        "v_and_b32 %[vad], 0x3ffc, %[vad]\n\t"
        "v_lshlrev_b32 %[vm], %[vsh], %[ffff]\n\t"
        "v_lshlrev_b32 %[vd], %[vsh], %[vpos]\n\t"
        "v_and_b32 %[vh], -4, %[va]\n\t"
        "ds_mskor_rtn_b32 %[vold], %[vad], %[vm], %[vd]\n\t"
        "ds_read_b32 %[vlo], %[vh] offset:16384\n\t"
        "ds_read_b32 %[vhi], %[vh] offset:16388\n\t"
        "v_and_b32 %[va], 3, %[va]\n\t"
        "s_waitcnt lgkmcnt(2)\n\t"
        "v_lshrrev_b32 %[vcand], %[vsh], %[vold]\n\t"
        "v_bfe_u32 %[vm], %[vold], %[vsh], 2\n\t"
        "v_and_b32 %[vd], 0xfffc, %[vcand]\n\t"
        "ds_read_b32 %[vold], %[vd] offset:16384\n\t"
        "ds_read_b32 %[vx1], %[vd] offset:16388\n\t"
        "s_waitcnt lgkmcnt(0)\n\t"
        "v_alignbyte_b32 %[vold], %[vx1], %[vold], %[vm]\n\t"
        "v_cmp_eq_u32 vcc, %[vold], %[vseq]\n\t"
        "s_cbranch_vccnz L_smatch%=\n\t"
        "v_alignbyte_b32 %[vseq], %[vhi], %[vlo], %[va]\n\t"
        "v_mov_b32 %[vpos], %[vnxt]\n\t"
        "v_add_u32 %[vnxt], %[vnxt], %[vstep]\n\t"
        "v_add_u32 %[vstep], 64, %[vstep]\n\t"
        "s_add_u32 %[nwin], %[nwin], 1\n\t"
        "s_branch L_stop%=\n\t"
        "L_smatch%=:\n\t"
        "s_ff1_i32_b64 %[js], vcc\n\t"
        "s_mov_b32 %[code], 1\n\t"
        "s_branch L_send%=\n\t"
        "L_spart%=:\n\t"
        "s_mov_b32 %[code], 0\n\t"
        "L_send%=:"
        : [code] "=&s"(code), [js] "=&s"(js), [qs] "+s"(qs), [qstep] "+s"(qstep), [nwin] "+s"(nwin),
          [vpos] "+v"(vpos), [vnxt] "+v"(vnxt), [vstep] "+v"(vstep), [vseq] "+v"(vseq),
          [vcand] "=&v"(vcand), [vh] "=&v"(vh), [va] "=&v"(va), [vsh] "=&v"(vsh), [vad] "=&v"(vad),
          [vm] "=&v"(vm), [vd] "=&v"(vd), [vold] "=&v"(vold), [vlo] "=&v"(vlo), [vhi] "=&v"(vhi),
          [vx1] "=&v"(vx1)
        : [limit] "s"(limit), [n] "s"(n), [kmul] "s"(2654435761u), [ffff] "s"(0xFFFFu)
        : "vcc", "scc", "memory");
    return code;
}

// The re-test chain of lz4/lz4.c:1230-1293 -- emit the sequence, step past
// the match, insert ip-2, look up and insert ip, test 4 bytes, count the
// match -- as ONE hand-scheduled loop: a straight line with one taken branch
// per zero-literal sequence.
//  * The bytes at ip-2 and ip come from the previous count window's a-side
//    registers (`tail`, window start `tb`): a DPP wave shift gives every lane
//    its neighbour's dword, two v_alignbyte + two v_readlane pick them out;
//    the hashes run on the scalar unit.
//  * The table put / get / put are plain LDS ops by every lane (same address,
//    same value); the count's a-side window is in flight beside them.
//  * Test and count come from one ballot: lane 0's bit is the 4-byte test,
//    the first set bit the first differing dword.
//  * Descriptors go to lane ns % 64 of dlo / dhi (EmitDescV), M0 the lane.
// Entry: the sequence (ip, ref, mc, lit = ip - anchor) is found and counted.
// Exits (ip is past the last emitted sequence = the new anchor):
//  kRtLimit  ip >= mflimitPlusOne: last literals;
//  kRtMiss   the 4 bytes at ip differ from the table's candidate (table
//            updated): search from ip + 1;
//  kRtSlow   ip - 2 or ip + 3 lies outside the register window: the caller
//            does this re-test (hashes, table, test, count) itself;
//  kRtLong   table updated, candidate c2, and the first 256 bytes at ip all
//            equal: the caller counts on.
// Wait states: every VALU result read by v_readlane / DPP / v_readfirstlane
// has at least two instructions in between; SALU reads of VALU-written
// SGPRs / VCC are interlocked.  All LDS reads are waited for inside.
enum { kRtLimit = 0, kRtMiss = 1, kRtSlow = 2, kRtLong = 3 };

#define BSHUF_RETEST_ASM(P2_BRANCH, P2_BLOCK) \
    asm volatile( \
        "s_mov_b32 %[keep], m0\n\t" \
        "L_top%=:\n\t" \
        /* ---- sequence descriptor -> lane ns % 64 of dlo / dhi */ \
        "s_sub_u32 %[t0], %[ip], %[ref]\n\t" \
        "s_pack_ll_b32_b16 %[t0], %[ip], %[t0]\n\t" \
        "s_add_u32 %[t1], %[mc], 4\n\t" \
        "s_pack_ll_b32_b16 %[t1], %[lit], %[t1]\n\t" \
        "s_and_b32 m0, %[ns], 63\n\t" \
        "s_add_u32 %[ns], %[ns], 1\n\t" \
        "s_add_u32 %[ip], %[ip], %[mc]\n\t" \
        "v_writelane_b32 %[dlo], %[t0], m0\n\t" \
        "v_writelane_b32 %[dhi], %[t1], m0\n\t" \
        "s_and_b32 %[t2], %[ns], 63\n\t" \
        "s_cbranch_scc0 L_flush%=\n\t" \
        "L_flushed%=:\n\t" \
        /* ---- step past the match; mflimit */ \
        "s_add_u32 %[ip], %[ip], 4\n\t" \
        "s_mov_b32 %[lit], 0\n\t" \
        "s_cmp_ge_i32 %[ip], %[limit]\n\t" \
        "s_cbranch_scc1 L_lim%=\n\t" \
        /* ---- ip - 2 .. ip + 3 inside the register window? */ \
        "s_sub_u32 %[t0], %[ip], %[tb]\n\t" \
        "s_sub_u32 %[t1], %[t0], 2\n\t" \
        "s_cmp_gt_u32 %[t1], 249\n\t" \
        "s_cbranch_scc1 L_slow%=\n\t" \
        "v_mov_b32_dpp %[vn], %[tail] wave_shl:1 bound_ctrl:0\n\t" \
        "s_and_b32 %[t2], %[t0], 3\n\t" \
        "s_and_b32 %[t3], %[t1], 3\n\t" \
        "s_lshr_b32 %[t0], %[t0], 2\n\t" \
        "v_alignbyte_b32 %[vy], %[vn], %[tail], %[t2]\n\t" \
        "v_alignbyte_b32 %[vz], %[vn], %[tail], %[t3]\n\t" \
        "s_lshr_b32 %[t1], %[t1], 2\n\t" \
        "s_sub_u32 %[t2], %[ip], 2\n\t" \
        "v_readlane_b32 %[t0], %[vy], %[t0]\n\t" \
        "v_readlane_b32 %[t1], %[vz], %[t1]\n\t" \
        P2_BRANCH \
        /* ---- hash4 (lz4/lz4.c:762-768) -> entry byte addresses */ \
        "s_mul_i32 %[t0], %[t0], 0x9e3779b1\n\t" \
        "s_mul_i32 %[t1], %[t1], 0x9e3779b1\n\t" \
        "s_lshr_b32 %[t0], %[t0], 18\n\t" \
        "s_lshr_b32 %[t1], %[t1], 18\n\t" \
        "s_and_b32 %[t0], %[t0], 0x3ffe\n\t" \
        "s_and_b32 %[t1], %[t1], 0x3ffe\n\t" \
        "s_and_b32 %[t3], %[ip], -4\n\t" \
        "v_add_u32 %[vcb], %[t3], %[lane4d]\n\t" \
        "v_mov_b32 %[vn], %[t1]\n\t" \
        "v_mov_b32 %[vy], %[t2]\n\t" \
        "v_mov_b32 %[vz], %[t0]\n\t" \
        "v_mov_b32 %[vd0], %[ip]\n\t" \
        /* a-side count window at ip, then put(ip-2), get(ip), put(ip) */ \
        "ds_read_b32 %[val], %[vcb]\n\t" \
        "ds_read_b32 %[vah], %[vcb] offset:4\n\t" \
        "ds_write_b16 %[vn], %[vy]\n\t" \
        "ds_read_u16 %[vc2], %[vz]\n\t" \
        "ds_write_b16 %[vz], %[vd0]\n\t" \
        "s_and_b32 %[t3], %[ip], 3\n\t" \
        "s_sub_u32 %[t1], %[mlimit], %[ip]\n\t" \
        "s_waitcnt lgkmcnt(1)\n\t" \
        "v_and_b32 %[vcb], -4, %[vc2]\n\t" \
        "v_add_u32 %[vcb], %[vcb], %[lane4d]\n\t" \
        "ds_read_b32 %[vbl], %[vcb]\n\t" \
        "ds_read_b32 %[vbh], %[vcb] offset:4\n\t" \
        "v_readfirstlane_b32 %[c2], %[vc2]\n\t" \
        "v_alignbyte_b32 %[tail], %[vah], %[val], %[t3]\n\t" \
        "s_and_b32 %[t2], %[c2], 3\n\t" \
        "s_waitcnt lgkmcnt(0)\n\t" \
        "v_alignbyte_b32 %[vbl], %[vbh], %[vbl], %[t2]\n\t" \
        "L_cmp%=:\n\t" \
        "v_cmp_ne_u32 vcc, %[tail], %[vbl]\n\t" \
        "v_xor_b32 %[vbh], %[tail], %[vbl]\n\t" \
        "s_bitcmp1_b32 vcc_lo, 0\n\t" \
        "s_cbranch_scc1 L_miss%=\n\t" \
        "s_cmp_eq_u64 vcc, 0\n\t" \
        "s_cbranch_scc1 L_long%=\n\t" \
        /* ---- count: first differing byte of the window */ \
        "s_ff1_i32_b64 %[t0], vcc\n\t" \
        "s_mov_b32 %[ref], %[c2]\n\t" \
        "v_readlane_b32 %[t2], %[vbh], %[t0]\n\t" \
        "s_lshl_b32 %[t0], %[t0], 2\n\t" \
        "s_mov_b32 %[tb], %[ip]\n\t" \
        "s_ff1_i32_b32 %[t2], %[t2]\n\t" \
        "s_lshr_b32 %[t2], %[t2], 3\n\t" \
        "s_add_u32 %[t0], %[t0], %[t2]\n\t" \
        "s_min_i32 %[t0], %[t0], %[t1]\n\t" \
        "s_sub_u32 %[mc], %[t0], 4\n\t" \
        "s_branch L_top%=\n\t" \
        /* ---- a batch of 64 descriptors to LDS (dropped past kDescMax) */ \
        "L_flush%=:\n\t" \
        "s_sub_u32 %[t2], %[ns], 64\n\t" \
        "s_cmp_ge_u32 %[t2], 256\n\t" /* kDescMax */ \
        "s_cbranch_scc1 L_flushed%=\n\t" \
        "s_lshl_b32 %[t2], %[t2], 3\n\t" \
        "s_add_u32 %[t2], %[t2], %[desc]\n\t" \
        "v_add_u32 %[vcb], %[t2], %[lane8]\n\t" \
        "ds_write2_b32 %[vcb], %[dlo], %[dhi] offset1:1\n\t" \
        "s_branch L_flushed%=\n\t" \
        P2_BLOCK \
        "L_lim%=:\n\t" \
        "s_mov_b32 %[code], 0\n\t" \
        "s_branch L_end%=\n\t" \
        "L_miss%=:\n\t" \
        "s_mov_b32 %[code], 1\n\t" \
        "s_branch L_end%=\n\t" \
        "L_slow%=:\n\t" \
        "s_mov_b32 %[code], 2\n\t" \
        "s_branch L_end%=\n\t" \
        "L_long%=:\n\t" \
        "s_mov_b32 %[code], 3\n\t" \
        "L_end%=:\n\t" \
        "s_mov_b32 m0, %[keep]" \
        : [code] "=&s"(code), [c2] "=&s"(c2), [ip] "+s"(ip), [ref] "+s"(ref), [mc] "+s"(mc), \
          [lit] "+s"(lit), [ns] "+s"(ns), [tb] "+s"(tb), [t0] "=&s"(t0), [t1] "=&s"(t1), \
          [t2] "=&s"(t2), [t3] "=&s"(t3), [keep] "=&s"(keep), [tail] "+v"(tail), [dlo] "+v"(dlo), \
          [dhi] "+v"(dhi), [vn] "=&v"(vn), [vy] "=&v"(vy), [vz] "=&v"(vz), [vd0] "=&v"(vd0), \
          [vc2] "=&v"(vc2), [vcb] "=&v"(vcb), [val] "=&v"(val), [vah] "=&v"(vah), \
          [vbl] "=&v"(vbl), [vbh] "=&v"(vbh) \
        : [limit] "s"(limit), [mlimit] "s"(mlimit), [desc] "s"(desc), [lane4d] "v"(lane4d), \
          [lane8] "v"(lane8) \
        : "vcc", "scc", "memory")
// x0 == x2 (bytes ip-2 .. ip+3 repeat with period 2): the table entry of ip
// is the one ip-2 was just put into, so the candidate is ip-2 and the 4-byte
// test passes -- a hit with offset 2, known without the table round trip; the
// b-side window is the a-side window shifted by 2 bytes (a DPP lane shift)
#define BSHUF_P2_BRANCH \
        "s_cmp_eq_u32 %[t0], %[t1]\n\t" \
        "s_cbranch_scc1 L_p2%=\n\t"
#define BSHUF_P2_BLOCK \
        "L_p2%=:\n\t" \
        "s_and_b32 %[t3], %[ip], -4\n\t" \
        "v_add_u32 %[vcb], %[t3], %[lane4d]\n\t" \
        "s_mul_i32 %[t0], %[t0], 0x9e3779b1\n\t" \
        "ds_read_b32 %[val], %[vcb]\n\t" \
        "ds_read_b32 %[vah], %[vcb] offset:4\n\t" \
        "s_lshr_b32 %[t0], %[t0], 18\n\t" \
        "s_and_b32 %[t0], %[t0], 0x3ffe\n\t" \
        "v_mov_b32 %[vd0], %[ip]\n\t" \
        "v_mov_b32 %[vz], %[t0]\n\t" \
        "ds_write_b16 %[vz], %[vd0]\n\t" \
        "s_and_b32 %[t3], %[ip], 3\n\t" \
        "s_sub_u32 %[c2], %[ip], 2\n\t" \
        "s_waitcnt lgkmcnt(1)\n\t" \
        "v_alignbyte_b32 %[tail], %[vah], %[val], %[t3]\n\t" \
        "s_nop 1\n\t" \
        "v_mov_b32_dpp %[vbh], %[tail] wave_shr:1 bound_ctrl:0\n\t" \
        "v_alignbyte_b32 %[vbl], %[tail], %[vbh], 2\n\t" \
        "v_writelane_b32 %[vbl], %[t1], 0\n\t" \
        "s_sub_u32 %[t1], %[mlimit], %[ip]\n\t" \
        "s_branch L_cmp%=\n\t"
template <bool kP2>
__device__ __forceinline__ int retest_chain(int& ip, int& ref, int& mc, int& lit, int& ns, int& tb,
                                            uint32_t& tail, uint32_t& dlo, uint32_t& dhi, int& c2,
                                            const int limit, const int mlimit, const uint32_t desc,
                                            const uint32_t lane4d, const uint32_t lane8) {
    int code;
    int t0, t1, t2, t3, keep;
    uint32_t vn, vy, vz, vd0, vc2, vcb, val, vah, vbl, vbh;
    static_assert(kDescMax == 256, "the flush below hard-codes kDescMax");
    if constexpr (kP2)
        BSHUF_RETEST_ASM(BSHUF_P2_BRANCH, BSHUF_P2_BLOCK);
    else
        BSHUF_RETEST_ASM(, );
    return code;
}

// The hand-off from a search match to the re-test chain (OPT & 131072): the
// catch-up's first 64 bytes back (lz4/lz4.c:1105-1109) and the first count
// window (lz4/lz4.c:1111-1118 with LZ4_count, :680-703) in ONE LDS round trip
// and one straight line -- the compiled catch_and_count spends ~100
// instructions and several exec-mask regions on the same work.  Counting
// starts at mpos itself: its 4 bytes are equal (the search just compared
// them), so lane 0 of the window never differs and the match length beyond
// kMinMatch is c0 - 4 whatever the catch-up finds.  Outputs:
//   back  bytes the match extends backwards, 0..63; -1: all 64 tested bytes
//         are equal (the caller continues the catch-up);
//   c0    equal bytes from mpos in the first 256-byte window, capped at
//         mlimit - mpos; 256: all equal and the limit lies beyond (count on);
//   tail  the a-side dword of every lane of that window (window base mpos).
// Wait states: v_readlane reads v_xor's result three instructions later; its
// lane select comes from s_ff1 (SALU); SALU reads of VOP3-compare SGPRs are
// interlocked.
__device__ __forceinline__ void search_entry(const int mpos, const int mref, const int anchor,
                                             const int mlimit, const uint32_t dbase,
                                             const uint32_t lane4d, const uint32_t lanev, int& back,
                                             int& c0, uint32_t& tail) {
    int t0, t1, t2, t3, t4;
    uint32_t val, vah, vbl, vbh, vba, vbb, vca, vcb, vx;
    uint64_t ne, bm, sy, sz;
    asm volatile(
        "s_and_b32 %[t0], %[mpos], -4\n\t"
        "s_and_b32 %[t1], %[mref], -4\n\t"
        "v_add_u32 %[vx], %[t0], %[lane4d]\n\t"
        "v_add_u32 %[vbh], %[t1], %[lane4d]\n\t"
        "s_add_u32 %[t2], %[mpos], -1\n\t"
        "s_add_u32 %[t3], %[mref], -1\n\t"
        "ds_read_b32 %[val], %[vx]\n\t"
        "ds_read_b32 %[vah], %[vx] offset:4\n\t"
        "ds_read_b32 %[vbl], %[vbh]\n\t"
        "ds_read_b32 %[vbh], %[vbh] offset:4\n\t"
        /* backward bytes: lane k tests mpos-1-k against mref-1-k */
        "v_sub_u32 %[vba], %[t2], %[lanev]\n\t"
        "v_sub_u32 %[vbb], %[t3], %[lanev]\n\t"
        "v_max_i32 %[vca], 0, %[vba]\n\t"
        "v_max_i32 %[vcb], 0, %[vbb]\n\t"
        "v_add_u32 %[vca], %[dbase], %[vca]\n\t"
        "v_add_u32 %[vcb], %[dbase], %[vcb]\n\t"
        "ds_read_u8 %[vca], %[vca]\n\t"
        "ds_read_u8 %[vcb], %[vcb]\n\t"
        "s_and_b32 %[t0], %[mpos], 3\n\t"
        "s_and_b32 %[t1], %[mref], 3\n\t"
        "s_sub_u32 %[t2], %[mlimit], %[mpos]\n\t"
        "s_max_i32 %[t2], %[t2], 0\n\t"
        "s_waitcnt lgkmcnt(2)\n\t"
        "v_alignbyte_b32 %[tail], %[vah], %[val], %[t0]\n\t"
        "v_alignbyte_b32 %[vbl], %[vbh], %[vbl], %[t1]\n\t"
        "v_xor_b32 %[vx], %[tail], %[vbl]\n\t"
        "v_cmp_ne_u32 %[ne], %[tail], %[vbl]\n\t"
        "v_cmp_le_i32 %[sy], %[anchor], %[vba]\n\t"
        "v_cmp_le_i32 %[sz], 0, %[vbb]\n\t"
        "s_ff1_i32_b64 %[t3], %[ne]\n\t"
        "s_waitcnt lgkmcnt(0)\n\t"
        "v_readlane_b32 %[t4], %[vx], %[t3]\n\t"
        "v_cmp_eq_u32 %[bm], %[vca], %[vcb]\n\t"
        "s_lshl_b32 %[t3], %[t3], 2\n\t"
        "s_ff1_i32_b32 %[t4], %[t4]\n\t"
        "s_lshr_b32 %[t4], %[t4], 3\n\t"
        "s_add_u32 %[t3], %[t3], %[t4]\n\t"
        "s_cmp_eq_u64 %[ne], 0\n\t"
        "s_cselect_b32 %[t3], 256, %[t3]\n\t"
        "s_min_i32 %[c0], %[t3], %[t2]\n\t"
        "s_and_b64 %[bm], %[bm], %[sy]\n\t"
        "s_and_b64 %[bm], %[bm], %[sz]\n\t"
        "s_not_b64 %[bm], %[bm]\n\t"
        "s_ff1_i32_b64 %[back], %[bm]"
        : [back] "=&s"(back), [c0] "=&s"(c0), [tail] "=&v"(tail), [t0] "=&s"(t0), [t1] "=&s"(t1),
          [t2] "=&s"(t2), [t3] "=&s"(t3), [t4] "=&s"(t4), [val] "=&v"(val), [vah] "=&v"(vah),
          [vbl] "=&v"(vbl), [vbh] "=&v"(vbh), [vba] "=&v"(vba), [vbb] "=&v"(vbb), [vca] "=&v"(vca),
          [vcb] "=&v"(vcb), [vx] "=&v"(vx), [ne] "=&s"(ne), [bm] "=&s"(bm), [sy] "=&s"(sy),
          [sz] "=&s"(sz)
        : [mpos] "s"(mpos), [mref] "s"(mref), [anchor] "s"(anchor), [mlimit] "s"(mlimit),
          [dbase] "s"(dbase), [lane4d] "v"(lane4d), [lanev] "v"(lanev)
        : "scc", "memory");
}

// The whole parse loop of a byU16 LDS block as ONE hand-scheduled asm block
// (OPT & 524288): the search windows (search_chain), the undo of a matching
// window's later inserts, the catch-up and first count window (search_entry)
// and the re-test chain (retest_chain, with its offset-2 shortcut) jump
// straight into one another; the compiled code between them (the exits'
// dispatch, a new search's setup after every re-test miss) cost ~60
// instructions per search.  Entry 0: search from ip (anchor set); entry 1: the
// sequence (ip, ref, mc, lit) is found and counted, tail = the a-side window
// at tb.  The rare cases go back to the caller:
//   kPcLimit    ip >= mflimitPlusOne after a sequence: last literals (anchor = ip);
//   kPcPartial  the search from ip reached a window that is not full (window
//               nwin; vpos / vseq: its probe positions and their bytes);
//   kPcSlow     re-test with ip - 2 or ip + 3 outside the register window
//               (anchor = ip; table not touched);
//   kPcLong     re-test: table updated, candidate c2, the first 256 bytes at
//               ip all equal (anchor = ip): count on;
//   kPcEntry    a search match (mpos, mref; later inserts undone) whose
//               catch-up reaches 64 bytes back or whose count reaches 256.
// Wait states as in the three blocks it is made of.
enum { kPcLimit = 0, kPcPartial = 1, kPcSlow = 2, kPcLong = 3, kPcEntry = 4 };
// lz4_encode_block OPT bit (not a bshuf_set_variant value): parse_chain's
// count-first compare (the element size decides, see BSHUF_CMP_COUNT_FIRST)
constexpr int kOptCountFirst = 1 << 23;

// The re-test's compare of the 4 bytes at ip and the count window, in two
// forms (round 6, profiles/r06/enc_ab r6r/r6s): miss-first tests lane 0 by
// itself (2 instructions) before the count's per-lane work, so a re-test miss
// costs what it did; count-first computes the per-lane count beside the one
// unsigned compare that tells miss and "all equal" apart, 2 instructions fewer
// per hit and 7 more per miss.  1 GiB per launch, miss-first / count-first
// against the form before: G2 0.766 -> 0.759 / 0.747, E = 3 1.027 -> 1.019 /
// 1.032, E = 12 0.986 -> 0.977 / 0.984, G1 0.294 -> 0.294 / 0.293: G2 float32
// (142 hits, 25 misses per block) takes count-first, every other element size
// miss-first.
#define BSHUF_PARSE_ASM(CMP_BLOCK, RARE_BLOCK) \
    asm volatile( \
        "s_mov_b32 %[keep], m0\n\t" \
        /* m0 = the descriptor lane (ns % 64), ns = the batch base (ns - m0); \
           ns = base + m0 again at the exit */ \
        "s_and_b32 m0, %[ns], 63\n\t" \
        "s_andn2_b32 %[ns], %[ns], 63\n\t" \
        "s_cmp_eq_u32 %[entry], 1\n\t" \
        "s_cbranch_scc1 L_cent%=\n\t" \
        /* ======== a search from p0 = ip: the first window's bytes */ \
        "L_nsrch%=:\n\t" \
        "v_add_u32 %[vh], %[ip], %[lanev]\n\t" \
        "v_min_i32 %[vh], %[n], %[vh]\n\t" \
        "v_and_b32 %[va], -4, %[vh]\n\t" \
        "ds_read_b32 %[vlo], %[va] offset:16384\n\t" \
        "ds_read_b32 %[vhi], %[va] offset:16388\n\t" \
        "v_and_b32 %[vh], 3, %[vh]\n\t" \
        "v_add_u32 %[vpos], %[ip], %[pq_off]\n\t" \
        "v_add_u32 %[vnxt], %[ip], %[pq_nxt]\n\t" \
        "v_mov_b32 %[vstep], %[pq_stp]\n\t" \
        "s_add_u32 %[qs], %[ip], 64\n\t" \
        "s_movk_i32 %[qstep], 0x7f\n\t" \
        "s_mov_b32 %[nwin], 0\n\t" \
        "s_waitcnt lgkmcnt(0)\n\t" \
        "v_alignbyte_b32 %[vseq], %[vhi], %[vlo], %[vh]\n\t" \
        /* ======== full search windows (search_chain) */ \
        "L_stop%=:\n\t" \
        "s_cmp_gt_i32 %[qs], %[limit]\n\t" \
        "s_cbranch_scc1 L_spart%=\n\t" \
        "v_mul_lo_u32 %[vh], %[vseq], %[kmul]\n\t" \
        "v_min_i32 %[va], %[n], %[vnxt]\n\t" \
        "s_add_u32 %[qs], %[qs], %[qstep]\n\t" \
        "s_add_u32 %[qstep], %[qstep], 64\n\t" \
        "v_lshrrev_b32 %[vsh], 15, %[vh]\n\t" \
        "v_lshrrev_b32 %[vad], 18, %[vh]\n\t" \
        "v_and_b32 %[vsh], 16, %[vsh]\n\t" \
        "v_and_b32 %[vad], 0x3ffc, %[vad]\n\t" \
        "v_lshlrev_b32 %[vm], %[vsh], %[ffff]\n\t" \
        "v_lshlrev_b32 %[vd], %[vsh], %[vpos]\n\t" \
        "v_and_b32 %[vh], -4, %[va]\n\t" \
        "ds_mskor_rtn_b32 %[vold], %[vad], %[vm], %[vd]\n\t" \
        "ds_read_b32 %[vlo], %[vh] offset:16384\n\t" \
        "ds_read_b32 %[vhi], %[vh] offset:16388\n\t" \
        "v_and_b32 %[va], 3, %[va]\n\t" \
        "s_waitcnt lgkmcnt(2)\n\t" \
        "v_lshrrev_b32 %[vcand], %[vsh], %[vold]\n\t" \
        "v_bfe_u32 %[vm], %[vold], %[vsh], 2\n\t" \
        "v_and_b32 %[vd], 0xfffc, %[vcand]\n\t" \
        "ds_read_b32 %[vold], %[vd] offset:16384\n\t" \
        "ds_read_b32 %[vx1], %[vd] offset:16388\n\t" \
        "s_waitcnt lgkmcnt(0)\n\t" \
        "v_alignbyte_b32 %[vold], %[vx1], %[vold], %[vm]\n\t" \
        "v_cmp_eq_u32 vcc, %[vold], %[vseq]\n\t" \
        "s_cbranch_vccnz L_smatch%=\n\t" \
        "v_alignbyte_b32 %[vseq], %[vhi], %[vlo], %[va]\n\t" \
        "v_mov_b32 %[vpos], %[vnxt]\n\t" \
        "v_add_u32 %[vnxt], %[vnxt], %[vstep]\n\t" \
        "v_add_u32 %[vstep], 64, %[vstep]\n\t" \
        "s_add_u32 %[nwin], %[nwin], 1\n\t" \
        "s_branch L_stop%=\n\t" \
        /* ======== a match at lane js: later lanes whose found entry is \
           <= mpos put it back (positions after the match were never inserted) */ \
        "L_smatch%=:\n\t" \
        "s_ff1_i32_b64 %[t0], vcc\n\t" \
        "v_and_b32 %[vd], 0xffff, %[vcand]\n\t" \
        "v_lshlrev_b32 %[vm], %[vsh], %[ffff]\n\t" \
        "v_lshlrev_b32 %[vx1], %[vsh], %[vd]\n\t" \
        "v_readlane_b32 %[mpos], %[vpos], %[t0]\n\t" \
        "v_readlane_b32 %[mref], %[vd], %[t0]\n\t" \
        "s_lshl_b64 %[sy], -2, %[t0]\n\t" \
        "v_cmp_ge_u32 %[sz], %[mpos], %[vd]\n\t" \
        "s_and_b64 %[sy], %[sy], %[sz]\n\t" \
        "s_and_saveexec_b64 %[sz], %[sy]\n\t" \
        "ds_mskor_b32 %[vad], %[vm], %[vx1]\n\t" \
        "s_mov_b64 exec, %[sz]\n\t" \
        /* ======== catch-up (64 bytes back) and the first count window from \
           mpos, one LDS round trip (search_entry) */ \
        "s_and_b32 %[t0], %[mpos], -4\n\t" \
        "s_and_b32 %[t1], %[mref], -4\n\t" \
        "v_add_u32 %[vx1], %[t0], %[lane4d]\n\t" \
        "v_add_u32 %[vbh], %[t1], %[lane4d]\n\t" \
        "s_add_u32 %[t2], %[mpos], -1\n\t" \
        "s_add_u32 %[t3], %[mref], -1\n\t" \
        "ds_read_b32 %[val], %[vx1]\n\t" \
        "ds_read_b32 %[vah], %[vx1] offset:4\n\t" \
        "ds_read_b32 %[vbl], %[vbh]\n\t" \
        "ds_read_b32 %[vbh], %[vbh] offset:4\n\t" \
        "v_sub_u32 %[vy], %[t2], %[lanev]\n\t" \
        "v_sub_u32 %[vz], %[t3], %[lanev]\n\t" \
        "v_max_i32 %[vn], 0, %[vy]\n\t" \
        "v_max_i32 %[vd0], 0, %[vz]\n\t" \
        "ds_read_u8 %[vn], %[vn] offset:16384\n\t" \
        "ds_read_u8 %[vd0], %[vd0] offset:16384\n\t" \
        "s_and_b32 %[t0], %[mpos], 3\n\t" \
        "s_and_b32 %[t1], %[mref], 3\n\t" \
        "s_sub_u32 %[t2], %[mlimit], %[mpos]\n\t" \
        "s_max_i32 %[t2], %[t2], 0\n\t" \
        "s_waitcnt lgkmcnt(2)\n\t" \
        "v_alignbyte_b32 %[tail], %[vah], %[val], %[t0]\n\t" \
        "v_alignbyte_b32 %[vbl], %[vbh], %[vbl], %[t1]\n\t" \
        "v_xor_b32 %[vx1], %[tail], %[vbl]\n\t" \
        "v_cmp_ne_u32 %[ne], %[tail], %[vbl]\n\t" \
        "v_cmp_le_i32 %[sy], %[anchor], %[vy]\n\t" \
        "v_cmp_le_i32 %[sz], 0, %[vz]\n\t" \
        "s_ff1_i32_b64 %[t3], %[ne]\n\t" \
        "s_waitcnt lgkmcnt(0)\n\t" \
        "v_readlane_b32 %[t4], %[vx1], %[t3]\n\t" \
        "v_cmp_eq_u32 %[bm], %[vn], %[vd0]\n\t" \
        "s_lshl_b32 %[t3], %[t3], 2\n\t" \
        "s_ff1_i32_b32 %[t4], %[t4]\n\t" \
        "s_lshr_b32 %[t4], %[t4], 3\n\t" \
        "s_add_u32 %[t3], %[t3], %[t4]\n\t" \
        "s_cmp_eq_u64 %[ne], 0\n\t" \
        "s_cselect_b32 %[t3], 256, %[t3]\n\t" \
        "s_min_i32 %[t3], %[t3], %[t2]\n\t" \
        "s_and_b64 %[bm], %[bm], %[sy]\n\t" \
        "s_and_b64 %[bm], %[bm], %[sz]\n\t" \
        "s_not_b64 %[bm], %[bm]\n\t" \
        "s_ff1_i32_b64 %[t4], %[bm]\n\t" \
        "s_cmp_lt_i32 %[t4], 0\n\t" \
        "s_cbranch_scc1 L_eslow%=\n\t" \
        "s_cmpk_eq_u32 %[t3], 0x100\n\t" \
        "s_cbranch_scc1 L_eslow%=\n\t" \
        "s_sub_u32 %[ip], %[mpos], %[t4]\n\t" \
        "s_sub_u32 %[c2], %[mref], %[t4]\n\t" \
        "s_add_u32 %[mc], %[t3], %[t4]\n\t" \
        "s_sub_u32 %[lit], %[ip], %[anchor]\n\t" \
        "s_mov_b32 %[tb], %[mpos]\n\t" \
        /* ======== the re-test chain (retest_chain).  Round 6: in here mc \
           holds the match length ml = mc + 4 (the descriptor's field), the \
           candidate stays in c2, and a loop iteration has no literals and \
           starts from the previous count window based at the previous ip, \
           so ip - tb = ml: no ref / tb / lit bookkeeping per sequence. \
           L_tope: a sequence with literals, count window based at tb (the \
           search's hand-off above falls into it; L_cent, the entry from C++ \
           with mc beyond kMinMatch and the candidate in ref, jumps to it); \
           the loop's own head is the tail of the count below. */ \
        "L_tope%=:\n\t" \
        "s_sub_u32 %[t0], %[ip], %[c2]\n\t" \
        "s_pack_ll_b32_b16 %[t0], %[ip], %[t0]\n\t" \
        "s_pack_ll_b32_b16 %[t1], %[lit], %[mc]\n\t" \
        "s_add_u32 %[ip], %[ip], %[mc]\n\t" \
        "s_sub_u32 %[mc], %[ip], %[tb]\n\t" \
        /* descriptor -> lane ns % 64 of dlo / dhi; mc = ip - tb from here */ \
        "L_desc%=:\n\t" \
        "v_writelane_b32 %[dlo], %[t0], m0\n\t" \
        "v_writelane_b32 %[dhi], %[t1], m0\n\t" \
        "s_add_u32 m0, m0, 1\n\t" \
        "s_cmp_eq_u32 m0, 64\n\t" \
        "s_cbranch_scc1 L_flush%=\n\t" \
        "L_flushed%=:\n\t" \
        "s_cmp_ge_i32 %[ip], %[limit]\n\t" \
        "s_cbranch_scc1 L_lim%=\n\t" \
        "s_sub_u32 %[t1], %[mc], 2\n\t" \
        "s_cmp_gt_u32 %[t1], 249\n\t" \
        "s_cbranch_scc1 L_slow%=\n\t" \
        "v_mov_b32_dpp %[vn], %[tail] wave_shl:1 bound_ctrl:0\n\t" \
        "s_and_b32 %[t2], %[mc], 3\n\t" \
        "s_and_b32 %[t3], %[t1], 3\n\t" \
        "s_lshr_b32 %[t0], %[mc], 2\n\t" \
        "v_alignbyte_b32 %[vy], %[vn], %[tail], %[t2]\n\t" \
        "v_alignbyte_b32 %[vz], %[vn], %[tail], %[t3]\n\t" \
        "s_lshr_b32 %[t1], %[t1], 2\n\t" \
        "s_sub_u32 %[t2], %[ip], 2\n\t" \
        "v_readlane_b32 %[t0], %[vy], %[t0]\n\t" \
        "v_readlane_b32 %[t1], %[vz], %[t1]\n\t" \
        "s_cmp_eq_u32 %[t0], %[t1]\n\t" \
        "s_cbranch_scc1 L_p2%=\n\t" \
        "s_mul_i32 %[t0], %[t0], 0x9e3779b1\n\t" \
        "s_mul_i32 %[t1], %[t1], 0x9e3779b1\n\t" \
        "s_lshr_b32 %[t0], %[t0], 18\n\t" \
        "s_lshr_b32 %[t1], %[t1], 18\n\t" \
        "s_and_b32 %[t0], %[t0], 0x3ffe\n\t" \
        "s_and_b32 %[t1], %[t1], 0x3ffe\n\t" \
        "s_and_b32 %[t3], %[ip], -4\n\t" \
        "v_add_u32 %[vcb], %[t3], %[lane4d]\n\t" \
        "v_mov_b32 %[vn], %[t1]\n\t" \
        "v_mov_b32 %[vy], %[t2]\n\t" \
        "v_mov_b32 %[vz], %[t0]\n\t" \
        "v_mov_b32 %[vd0], %[ip]\n\t" \
        "ds_read_b32 %[val], %[vcb]\n\t" \
        "ds_read_b32 %[vah], %[vcb] offset:4\n\t" \
        "ds_write_b16 %[vn], %[vy]\n\t" \
        "ds_read_u16 %[vc2], %[vz]\n\t" \
        "ds_write_b16 %[vz], %[vd0]\n\t" \
        "s_and_b32 %[t3], %[ip], 3\n\t" \
        "s_waitcnt lgkmcnt(1)\n\t" \
        "v_and_b32 %[vcb], -4, %[vc2]\n\t" \
        "v_add_u32 %[vcb], %[vcb], %[lane4d]\n\t" \
        "ds_read_b32 %[vbl], %[vcb]\n\t" \
        "ds_read_b32 %[vbh], %[vcb] offset:4\n\t" \
        "v_readfirstlane_b32 %[c2], %[vc2]\n\t" \
        "v_alignbyte_b32 %[tail], %[vah], %[val], %[t3]\n\t" \
        "s_and_b32 %[t2], %[c2], 3\n\t" \
        "s_waitcnt lgkmcnt(0)\n\t" \
        "v_alignbyte_b32 %[vbl], %[vbh], %[vbl], %[t2]\n\t" \
        CMP_BLOCK \
        /* count: ml = the first differing byte of the window from ip (its \
           first 4 bytes are the tested ones), capped at mlimit - ip */ \
        "s_sub_u32 %[t1], %[mlimit], %[ip]\n\t" \
        "v_readlane_b32 %[t2], %[vbh], %[t0]\n\t" \
        "s_min_i32 %[mc], %[t2], %[t1]\n\t" \
        /* the next sequence's descriptor fields (no literals) and ip */ \
        "s_sub_u32 %[t0], %[ip], %[c2]\n\t" \
        "s_pack_ll_b32_b16 %[t0], %[ip], %[t0]\n\t" \
        "s_lshl_b32 %[t1], %[mc], 16\n\t" \
        "s_add_u32 %[ip], %[ip], %[mc]\n\t" \
        "s_branch L_desc%=\n\t" \
        /* a batch of 64 descriptors to LDS (dropped past kDescMax) */ \
        "L_flush%=:\n\t" \
        "s_mov_b32 m0, 0\n\t" \
        "s_cmp_ge_u32 %[ns], 256\n\t" /* kDescMax */ \
        "s_cbranch_scc1 L_fldone%=\n\t" \
        "s_lshl_b32 %[t2], %[ns], 3\n\t" \
        "s_add_u32 %[t2], %[t2], %[desc]\n\t" \
        "v_add_u32 %[vcb], %[t2], %[lane8]\n\t" \
        "ds_write2_b32 %[vcb], %[dlo], %[dhi] offset1:1\n\t" \
        "L_fldone%=:\n\t" \
        "s_add_u32 %[ns], %[ns], 64\n\t" \
        "s_branch L_flushed%=\n\t" \
        /* offset-2 shortcut (retest_chain) */ \
        "L_p2%=:\n\t" \
        "s_and_b32 %[t3], %[ip], -4\n\t" \
        "v_add_u32 %[vcb], %[t3], %[lane4d]\n\t" \
        "s_mul_i32 %[t0], %[t0], 0x9e3779b1\n\t" \
        "ds_read_b32 %[val], %[vcb]\n\t" \
        "ds_read_b32 %[vah], %[vcb] offset:4\n\t" \
        "s_lshr_b32 %[t0], %[t0], 18\n\t" \
        "s_and_b32 %[t0], %[t0], 0x3ffe\n\t" \
        "v_mov_b32 %[vd0], %[ip]\n\t" \
        "v_mov_b32 %[vz], %[t0]\n\t" \
        "ds_write_b16 %[vz], %[vd0]\n\t" \
        "s_and_b32 %[t3], %[ip], 3\n\t" \
        "s_sub_u32 %[c2], %[ip], 2\n\t" \
        "s_waitcnt lgkmcnt(1)\n\t" \
        "v_alignbyte_b32 %[tail], %[vah], %[val], %[t3]\n\t" \
        "s_nop 1\n\t" \
        "v_mov_b32_dpp %[vbh], %[tail] wave_shr:1 bound_ctrl:0\n\t" \
        "v_alignbyte_b32 %[vbl], %[tail], %[vbh], 2\n\t" \
        "v_writelane_b32 %[vbl], %[t1], 0\n\t" \
        "s_branch L_cmp%=\n\t" \
        /* ======== a re-test miss: search from anchor + 1 */ \
        RARE_BLOCK \
        "L_miss%=:\n\t" \
        "s_mov_b32 %[anchor], %[ip]\n\t" \
        "s_add_u32 %[ip], %[ip], 1\n\t" \
        "s_branch L_nsrch%=\n\t" \
        "L_lim%=:\n\t" \
        "s_mov_b32 %[code], 0\n\t" \
        "s_mov_b32 %[anchor], %[ip]\n\t" \
        "s_branch L_end%=\n\t" \
        "L_spart%=:\n\t" \
        "s_mov_b32 %[code], 1\n\t" \
        "s_branch L_end%=\n\t" \
        "L_slow%=:\n\t" \
        "s_mov_b32 %[code], 2\n\t" \
        "s_mov_b32 %[anchor], %[ip]\n\t" \
        "s_branch L_end%=\n\t" \
        "L_long%=:\n\t" \
        "s_mov_b32 %[code], 3\n\t" \
        "s_mov_b32 %[anchor], %[ip]\n\t" \
        "s_branch L_end%=\n\t" \
        "L_cent%=:\n\t" \
        "s_add_u32 %[mc], %[mc], 4\n\t" \
        "s_mov_b32 %[c2], %[ref]\n\t" \
        "s_branch L_tope%=\n\t" \
        "L_eslow%=:\n\t" \
        "s_mov_b32 %[code], 4\n\t" \
        "L_end%=:\n\t" \
        "s_add_u32 %[ns], %[ns], m0\n\t" \
        "s_mov_b32 m0, %[keep]" \
        : [code] "=&s"(code), [ip] "+s"(ip), [anchor] "+s"(anchor), [ref] "+s"(ref), [mc] "+s"(mc), \
          [lit] "+s"(lit), [ns] "+s"(ns), [tb] "+s"(tb), [nwin] "+s"(nwin), [mpos] "+s"(mpos), \
          [mref] "+s"(mref), [c2] "+s"(c2), [t0] "=&s"(t0), [t1] "=&s"(t1), [t2] "=&s"(t2), \
          [t3] "=&s"(t3), [t4] "=&s"(t4), [keep] "=&s"(keep), [qs] "=&s"(qs), [qstep] "=&s"(qstep), \
          [ne] "=&s"(ne), [bm] "=&s"(bm), [sy] "=&s"(sy), [sz] "=&s"(sz), [tail] "+v"(tail), \
          [dlo] "+v"(dlo), [dhi] "+v"(dhi), [vseq] "+v"(vseq), [vpos] "+v"(vpos), [vh] "=&v"(vh), \
          [va] "=&v"(va), [vsh] "=&v"(vsh), [vad] "=&v"(vad), [vm] "=&v"(vm), [vd] "=&v"(vd), \
          [vold] "=&v"(vold), [vlo] "=&v"(vlo), [vhi] "=&v"(vhi), [vx1] "=&v"(vx1), [vnxt] "=&v"(vnxt), \
          [vstep] "=&v"(vstep), [vcand] "=&v"(vcand), [vn] "=&v"(vn), [vy] "=&v"(vy), [vz] "=&v"(vz), \
          [vd0] "=&v"(vd0), [vc2] "=&v"(vc2), [vcb] "=&v"(vcb), [val] "=&v"(val), [vah] "=&v"(vah), \
          [vbl] "=&v"(vbl), [vbh] "=&v"(vbh) \
        : [entry] "s"(entry), [limit] "s"(limit), [mlimit] "s"(mlimit), [n] "s"(n), [desc] "s"(desc), \
          [kmul] "s"(2654435761u), [ffff] "s"(0xFFFFu), [lane4d] "v"(lane4d), [lane8] "v"(lane8), \
          [lanev] "v"(lanev), [pq_off] "v"(pq_off), [pq_nxt] "v"(pq_nxt), [pq_stp] "v"(pq_stp) \
        : "vcc", "scc", "memory")

#define BSHUF_CMP_MISS_FIRST \
        "L_cmp%=:\n\t" \
        "v_cmp_ne_u32 vcc, %[tail], %[vbl]\n\t" \
        "v_xor_b32 %[vbh], %[tail], %[vbl]\n\t" \
        "s_bitcmp1_b32 vcc_lo, 0\n\t" \
        "s_cbranch_scc1 L_miss%=\n\t" \
        /* every lane: the window byte of its first difference (4 lane + \
           first differing bit / 8; garbage in equal lanes, never read), \
           beside the scalar tests */ \
        "v_ffbl_b32 %[vbh], %[vbh]\n\t" \
        "v_lshrrev_b32 %[vbh], 3, %[vbh]\n\t" \
        "v_lshl_add_u32 %[vbh], %[lanev], 2, %[vbh]\n\t" \
        "s_ff1_i32_b64 %[t0], vcc\n\t" \
        "s_cmp_lt_i32 %[t0], 0\n\t" \
        "s_cbranch_scc1 L_long%=\n\t"
#define BSHUF_CMP_COUNT_FIRST \
        "L_cmp%=:\n\t" \
        /* every lane: the window byte of its first difference (4 lane + \
           first differing bit / 8; garbage in equal lanes, never read) */ \
        "v_cmp_ne_u32 vcc, %[tail], %[vbl]\n\t" \
        "v_xor_b32 %[vbh], %[tail], %[vbl]\n\t" \
        "v_ffbl_b32 %[vbh], %[vbh]\n\t" \
        "v_lshrrev_b32 %[vbh], 3, %[vbh]\n\t" \
        "v_lshl_add_u32 %[vbh], %[lanev], 2, %[vbh]\n\t" \
        /* the first differing lane: 0 = the 4-byte test failed (miss), none \
           = all 256 bytes equal (long), both by one unsigned compare */ \
        "s_ff1_i32_b64 %[t0], vcc\n\t" \
        "s_sub_u32 %[t3], %[t0], 1\n\t" \
        "s_cmp_gt_u32 %[t3], 62\n\t" \
        "s_cbranch_scc1 L_rare%=\n\t"
#define BSHUF_RARE_COUNT_FIRST \
        "L_rare%=:\n\t" \
        "s_cmp_lg_u32 %[t0], 0\n\t" \
        "s_cbranch_scc1 L_long%=\n\t"

template <bool kMissFirst>
__device__ __forceinline__ int parse_chain(const int entry, int& ip, int& anchor, int& ref, int& mc, int& lit,
                                           int& ns, int& tb, int& nwin, int& mpos, int& mref, int& c2,
                                           uint32_t& tail, uint32_t& dlo, uint32_t& dhi, uint32_t& vseq,
                                           uint32_t& vpos, const int limit, const int mlimit, const int n,
                                           const uint32_t desc, const uint32_t lane4d, const uint32_t lane8,
                                           const uint32_t lanev, const uint32_t pq_off, const uint32_t pq_nxt,
                                           const uint32_t pq_stp) {
    int code, t0, t1, t2, t3, t4, keep, qs, qstep;
    uint64_t ne, bm, sy, sz;
    uint32_t vh, va, vsh, vad, vm, vd, vold, vlo, vhi, vx1, vnxt, vstep, vcand;
    uint32_t vn, vy, vz, vd0, vc2, vcb, val, vah, vbl, vbh;
    if constexpr (kMissFirst)
        BSHUF_PARSE_ASM(BSHUF_CMP_MISS_FIRST, );
    else
        BSHUF_PARSE_ASM(BSHUF_CMP_COUNT_FIRST, BSHUF_RARE_COUNT_FIRST);
    return code;
}

// Greedy LZ4 parse of D[0..n) with table T (zeroed).  Every sequence goes to
// em.seq() once its match is final, the trailing literal run to em.last().
// Returns the compressed size, or -1 when the emitter ran out of descriptor
// slots.  Mirrors lz4/lz4.c:1002-1331 for noDict, acceleration 1, notLimited
// output.
template <bool WIDE, bool READBACK, int OPT, class Emit, class Blk>
__device__ int lz4_encode_block(const Blk D, const int n, const Table<WIDE> T, Emit& em,
                                const int lane) {
    DIAG_DECL
    // the hand-scheduled re-test chain: LDS block (table at LDS 0, block at
    // kTableBytes) with VGPR-buffered descriptors
    constexpr bool kAsmRetest = !WIDE && !READBACK && std::is_same<Emit, EmitDescV>::value &&
                                !std::is_same<Blk, GblBlk>::value;
    // the hand-scheduled full search windows (OPT & 16384): LDS block too
    constexpr bool kAsmSearch = !WIDE && !READBACK && (OPT & 16384) != 0 && (OPT & 512) == 0 &&
                                !std::is_same<Blk, GblBlk>::value;
    // the search-match -> re-test hand-off in one asm block (OPT & 131072)
    constexpr bool kAsmEntry = kAsmRetest && (OPT & 131072) != 0;
    // the whole loop in one asm block (OPT & 524288, parse_chain)
    constexpr bool kFused = kAsmRetest && (OPT & 524288) != 0;
    int op = 0, anchor = 0;
    if constexpr (kFused) {
        if (n >= kLz4MinLength) {
            const int limit = n - kMfLimit + 1;  // mflimitPlusOne
            const int mlimit = n - kLastLiterals;
            const uint32_t lane4d = (uint32_t)(uintptr_t)D + 4u * (uint32_t)lane;
            const uint32_t lane8 = 8u * (uint32_t)lane;
            const uint32_t desc_addr = (uint32_t)(uintptr_t)em.desc;
            // this lane's probe offsets in a search's first window (probe_lane)
            const ProbeLane q = probe_lane(lane);
            const uint32_t pq_off = (uint32_t)(q.off - (lane == 0 ? 1 : 0));
            const uint32_t pq_nxt = (uint32_t)(q.off + q.step), pq_stp = (uint32_t)(q.step + kWave);
            int ip = 1, entry = 0, ref = 0, mc = 0, lit = 0, tb = 0, nwin = 0, mpos = 0, mref = 0, c2 = 0;
            uint32_t tail = 0, vseq = 0, vpos = 0;
            for (;;) {
                // every scalar the asm keeps in SGPRs, provably uniform here
                entry = uni(entry), ip = uni(ip), anchor = uni(anchor), ref = uni(ref), mc = uni(mc);
                lit = uni(lit), em.ns = uni(em.ns), tb = uni(tb), nwin = uni(nwin), mpos = uni(mpos);
                mref = uni(mref), c2 = uni(c2);
                const int code = parse_chain<(OPT & kOptCountFirst) == 0>(entry, ip, anchor, ref, mc, lit, em.ns, tb, nwin, mpos, mref, c2,
                                             tail, em.dlo, em.dhi, vseq, vpos, limit, mlimit, n, desc_addr,
                                             lane4d, lane8, (uint32_t)lane, pq_off, pq_nxt, pq_stp);
                if (code == kPcLimit) break;
                CountOut co;
                if (code == kPcPartial) {
                    // the search from p0 = ip reached a window that is not
                    // full: its valid probes by the general window
                    const int p0 = ip, k0 = kWave * nwin;
                    const ProbeLane q1 = probe_lane(k0 + lane + 1);
                    const bool valid = p0 + q1.off <= limit;
                    const uint64_t vmask = ballot(valid);
                    if (vmask == 0) break;
                    const uint32_t h = hash4(vseq);
                    const uint32_t cand = T.exchange_if(h, vpos, valid);
                    const uint32_t dcand = lds_rd32(D, (int)cand);
                    const uint64_t mm = vmask & ballot(dcand == vseq);
                    if (!mm) break;
                    const int js = ffs64(mm);
                    mpos = __builtin_amdgcn_readlane((int)vpos, js);
                    if (valid && lane > js && cand <= (uint32_t)mpos) T.put(h, cand);
                    mref = __builtin_amdgcn_readlane((int)cand, js);
                    co = catch_and_count(D, n, mpos, mref, anchor, mlimit, lane);
                } else if (code == kPcEntry) {
                    co = catch_and_count(D, n, mpos, mref, anchor, mlimit, lane);
                } else {
                    // re-test outside the register window (kPcSlow: table ops
                    // here) or longer than 256 bytes (kPcLong): from the window at ip
                    if (code == kPcSlow) {
                        const uint32_t h2 = hash4(lds_rd32(D, ip - 2)), h0 = hash4(lds_rd32(D, ip));
                        T.put(h2, (uint32_t)(ip - 2));
                        c2 = uni((int)T.get(h0));
                        T.put(h0, (uint32_t)ip);
                    }
                    uint32_t va = rdw(D, ip + 4 * lane, n), vb = rdw(D, c2 + 4 * lane, n);
                    uint64_t ne = ballot(va != vb);
                    if (ne & 1ull) {
                        entry = 0;  // a miss: search from anchor + 1
                        ip = anchor + 1;
                        continue;
                    }
                    int total = 0, c;
                    for (;;) {
                        c = kWinBytes;
                        if (ne) {
                            const int f = ffs64(ne);
                            const uint32_t x = (uint32_t)__builtin_amdgcn_readlane((int)(va ^ vb), f);
                            c = 4 * f + (__builtin_ctz(x) >> 3);
                        }
                        c = min(c, max(mlimit - (ip + total), 0));
                        if (c < kWinBytes) break;
                        total += kWinBytes;
                        va = rdw(D, ip + total + 4 * lane, n);
                        vb = rdw(D, c2 + total + 4 * lane, n);
                        ne = ballot(va != vb);
                    }
                    tail = va;
                    tb = ip + total;
                    ref = c2;
                    mc = total + c - kMinMatch;
                    lit = 0;
                    entry = 1;
                    continue;
                }
                // a search match (mpos, mref), caught up and counted here
                ip = mpos - co.back;
                ref = mref - co.back;
                mc = co.back + co.cnt;
                lit = ip - anchor;
                tb = co.tail_base;
                tail = co.tail;
                entry = 1;
            }
        }
        em.last(op, anchor, n);
        return op;
    }
    if (n >= kLz4MinLength) {
        const int limit = n - kMfLimit + 1;  // mflimitPlusOne
        const int mlimit = n - kLastLiterals;
        int ip = 1;  // position 0 is pre-inserted: a zeroed table already says 0
        // sequence of the first probe window, issued ahead of need
        uint32_t pre = lds_rd32(D, min(ip + lane, n));
        for (;;) {
            // ------------------------------------------------ search
            int mpos = -1, mref = 0;
            {
                const int p0 = ip;
                COUNT(6, 1);
                uint32_t seq_cur = pre;  // valid for k0 == 0 (positions p0 + lane)
                // probe offsets by addition: this lane's probe k and probe k+1
                // (the closed form's value, which is 1 for k = 0: `bias`)
                ProbeLane q0 = probe_lane(lane), q1 = probe_lane(lane + 1);
                int bias = lane == 0 ? 1 : 0;
                if constexpr (!READBACK && !WIDE && (OPT & 512) == 0) {
                    // full windows (every probe and its successor inside
                    // mflimit) are told by the last lane's successor offset,
                    // kept on the scalar unit: no validity ballot, no masks;
                    // the one partial window at the end takes the general
                    // path below.  A/B variant 512: every window general.
                    ProbeLane qs = probe_lane(kWave);
                    int k0 = 0;
                    if constexpr (kAsmSearch) {
                        // the full windows by search_chain
                        uint32_t vpos = (uint32_t)(p0 + q0.off - bias);
                        uint32_t vnxt = (uint32_t)(p0 + q0.off + q0.step);
                        uint32_t vstep = (uint32_t)(q0.step + kWave);
                        uint32_t vseq = seq_cur, vcand = 0;
                        int sqs = p0 + qs.off, sqstep = qs.step, nwin = 0, js = 0;
                        const int code = search_chain(vpos, vnxt, vstep, vseq, sqs, sqstep, nwin, vcand, js,
                                                      limit, n);
                        if (code == kSrMatch) {
                            const uint32_t cand = vcand & 0xFFFFu;
                            mpos = __builtin_amdgcn_readlane((int)vpos, js);
                            if (lane > js && cand <= (uint32_t)mpos) T.put(hash4(vseq), cand);
                            mref = __builtin_amdgcn_readlane((int)cand, js);
                            goto have_match;
                        }
                        // the partial window below: window nwin
                        k0 = kWave * nwin;
                        seq_cur = vseq;
                        q0 = probe_lane(k0 + lane);
                        bias = (k0 == 0 && lane == 0) ? 1 : 0;
                    }
                    for (; !kAsmSearch && p0 + qs.off <= limit; k0 += kWave) {
                        COUNT(1, 1);
                        const int pos = p0 + q0.off - bias;
                        const int pos_n = p0 + q0.off + q0.step;
                        q0.advance();
                        qs.advance();
                        bias = 0;
                        const uint32_t seq_nxt = lds_rd32(D, min(pos_n, n));
                        const uint32_t h = hash4(seq_cur);
                        const uint32_t cand = T.exchange(h, (uint32_t)pos);
                        const uint32_t dcand = lds_rd32(D, (int)cand);
                        const uint64_t mm = ballot(dcand == seq_cur);
                        if (mm) {
                            const int js = ffs64(mm);
                            mpos = __builtin_amdgcn_readlane(pos, js);
                            if (lane > js && cand <= (uint32_t)mpos) T.put(h, cand);
                            mref = __builtin_amdgcn_readlane((int)cand, js);
                            goto have_match;  // every exit goes straight to its code
                        }
                        seq_cur = seq_nxt;
                    }
                    {
                        // the partial window (if any probe of it is valid)
                        q1 = probe_lane(k0 + lane + 1);
                        const int pos = p0 + q0.off - bias;
                        const bool valid = p0 + q1.off <= limit;
                        const uint64_t vmask = ballot(valid);
                        if (vmask != 0) {
                            COUNT(1, 1);
                            const uint32_t h = hash4(seq_cur);
                            const uint32_t cand = T.exchange_if(h, (uint32_t)pos, valid);
                            const uint32_t dcand = lds_rd32(D, (int)cand);
                            const uint64_t mm = vmask & ballot(dcand == seq_cur);
                            if (mm) {
                                const int js = ffs64(mm);
                                mpos = __builtin_amdgcn_readlane(pos, js);
                                if (valid && lane > js && cand <= (uint32_t)mpos) T.put(h, cand);
                                mref = __builtin_amdgcn_readlane((int)cand, js);
                                goto have_match;
                            }
                        }
                        goto last_literals;
                    }
                }
                for (int k0 = 0; READBACK || WIDE || (OPT & 512) != 0; k0 += kWave) {
                    COUNT(1, 1);
                    const int pos = p0 + q0.off - bias;
                    const bool valid = p0 + q1.off <= limit;
                    const uint64_t vmask = ballot(valid);
                    if (vmask == 0) break;
                    // next window's sequences, in flight while this one resolves
                    const int pos_n = p0 + q0.off + q0.step;
                    q0.advance();
                    q1.advance();
                    bias = 0;
                    const uint32_t seq_nxt = lds_rd32(D, min(pos_n, n));
                    const uint32_t seq = seq_cur;
                    if constexpr (!READBACK) {
                        // one lane-ordered exchange = every lane's sequential
                        // insert-then-lookup; candidate bytes come from the
                        // (immutable) block in LDS
                        uint32_t h = 0, cand = 0;
                        if (valid) {
                            if constexpr (WIDE)
                                h = hash5(lds_rd64(D, pos));
                            else
                                h = hash4(seq);
                            cand = T.exchange(h, (uint32_t)pos);
                        }
                        const uint32_t dcand = lds_rd32(D, (int)cand);
                        // the compare's own mask, and-ed with the valid lanes on the
                        // scalar unit (a ballot of a combined bool is materialised)
                        const bool near = !WIDE || cand + kMaxDistance >= (uint32_t)pos;
                        const uint64_t mm = vmask & ballot(WIDE ? (near & (dcand == seq)) : dcand == seq);
                        if (mm) {
                            const int js = ffs64(mm);
                            mpos = __builtin_amdgcn_readlane(pos, js);
                            // positions after the match were never inserted: the
                            // first later lane of each entry puts back what it found
                            // (found <= mpos: no lane between wrote that entry)
                            if (valid && lane > js && cand <= (uint32_t)mpos) T.put(h, cand);
                            mref = __builtin_amdgcn_readlane((int)cand, js);
                            break;
                        }
                    } else {
                        uint32_t h = 0, cold = 0;
                        if (valid) {
                            if constexpr (WIDE)
                                h = hash5(lds_rd64(D, pos));
                            else
                                h = hash4(seq);
                            cold = T.get(h);
                        }
                        if (valid) T.put(h, (uint32_t)pos);
                        const uint32_t rb = valid ? T.get(h) : (uint32_t)pos;
                        const uint32_t dcold = lds_rd32(D, (int)cold);
                        const bool loser = valid && rb != (uint32_t)pos;
                        uint32_t cand = cold;
                        int pred = -1;
                        bool grouped = false, first = true;
                        int next_member = kWave;
                        uint64_t lmask = ballot(loser);
                        COUNT(2, lmask ? 1 : 0);
                        while (lmask) {
                            const int l = ffs64(lmask);
                            const uint32_t hl = (uint32_t)__builtin_amdgcn_readlane((int)h, l);
                            const bool in_g = valid && h == hl;
                            const uint64_t g = ballot(in_g);
                            if (in_g) {
                                grouped = true;
                                const uint64_t below = g & ((1ull << lane) - 1ull);
                                if (below) {
                                    pred = fls64(below);
                                    cand = (uint32_t)(p0 + probe_offset(k0 + pred));
                                    first = false;
                                }
                                const uint64_t above = lane == 63 ? 0ull : (g & (~0ull << (lane + 1)));
                                next_member = above ? ffs64(above) : kWave;
                            }
                            lmask &= ~g;
                        }
                        // candidate bytes: the table's position, or the in-window predecessor's
                        const uint32_t dpred = (uint32_t)__shfl((int)seq, pred < 0 ? lane : pred);
                        const uint32_t dcand = pred < 0 ? dcold : dpred;
                        // the compare's own mask, and-ed with the valid lanes on the
                        // scalar unit (a ballot of a combined bool is materialised)
                        const bool near = !WIDE || cand + kMaxDistance >= (uint32_t)pos;
                        const uint64_t mm = vmask & ballot(WIDE ? (near & (dcand == seq)) : dcand == seq);
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
                        if (vmask == ~0ull && grouped && next_member == kWave)
                            T.put(h, (uint32_t)pos);
                    }
                    if (vmask != ~0ull) break;  // ran past mflimit: last literals
                    seq_cur = seq_nxt;
                }
            }
            STAMP(0);
            if (mpos < 0) break;
        have_match:
            STAMP(0);  // (the search's match exits jump here)
            COUNT(0, 1);
            // ------------------------------------------------ catch up + count
            CountOut co;
            if constexpr (kAsmEntry) {
                // one round trip (search_entry); the long cases continue here
                int back, c0;
                search_entry(mpos, mref, anchor, mlimit, (uint32_t)(uintptr_t)D,
                             (uint32_t)(uintptr_t)D + 4u * (uint32_t)lane, (uint32_t)lane, back, c0,
                             co.tail);
                if (back < 0) {
                    // all 64 bytes back are equal: on 64 at a time
                    for (int base = kWave;; base += kWave) {
                        const int xa = mpos - 1 - base - lane, xb = mref - 1 - base - lane;
                        const uint64_t cm = ballot(xa >= anchor && xb >= 0 &&
                                                   (uint32_t)D[max(xa, 0)] == (uint32_t)D[max(xb, 0)]);
                        const int run = (~cm) ? ffs64(~cm) : kWave;
                        back = base + run;
                        if (run < kWave) break;
                    }
                }
                int total = 0;
                while (c0 == kWinBytes) {
                    // the first 256 bytes from mpos are equal: count on
                    total += kWinBytes;
                    const uint32_t va = rdw(D, mpos + total + 4 * lane, n);
                    const uint32_t vb = rdw(D, mref + total + 4 * lane, n);
                    c0 = window_equal(va, vb, mlimit - (mpos + total));
                    co.tail = va;
                }
                co.back = back;
                co.cnt = total + c0 - kMinMatch;  // beyond the 4 bytes at mpos
                co.tail_base = mpos + total;
            } else {
                co = catch_and_count(D, n, mpos, mref, anchor, mlimit, lane);
            }
            ip = mpos - co.back;
            int ref = mref - co.back;
            int mc = co.back + co.cnt;
            STAMP(1);
            if constexpr (kAsmRetest) {
                // the hand-scheduled re-test chain (retest_chain); the rare
                // cases it hands back are finished here
                int lit = ip - anchor, tb = co.tail_base;
                uint32_t tail = co.tail;
                const uint32_t lane4d = (uint32_t)(uintptr_t)D + 4u * (uint32_t)lane;
                const uint32_t lane8 = 8u * (uint32_t)lane;
                const uint32_t desc_addr = (uint32_t)(uintptr_t)em.desc;
                for (;;) {
                    int c2 = 0;
                    const int code = retest_chain<(OPT & 32768) != 0>(ip, ref, mc, lit, em.ns, tb, tail, em.dlo, em.dhi, c2,
                                                  limit, mlimit, desc_addr, lane4d, lane8);
                    anchor = ip;
                    if (code == kRtLimit) {
                        STAMP(4);
                        goto last_literals;
                    }
                    if (code == kRtMiss) break;
                    if (code == kRtSlow) {
                        // ip - 2 or ip + 3 outside the register window: from LDS
                        const uint32_t h2 = hash4(lds_rd32(D, ip - 2)), h0 = hash4(lds_rd32(D, ip));
                        T.put(h2, (uint32_t)(ip - 2));
                        c2 = uni((int)T.get(h0));
                        T.put(h0, (uint32_t)ip);
                    }
                    // kRtSlow: test and count; kRtLong: count on past the
                    // first (all-equal) window -- from the window at ip
                    uint32_t va = rdw(D, ip + 4 * lane, n), vb = rdw(D, c2 + 4 * lane, n);
                    uint64_t ne = ballot(va != vb);
                    if (ne & 1ull) break;
                    int total = 0, c;
                    for (;;) {
                        c = kWinBytes;
                        if (ne) {
                            const int f = ffs64(ne);
                            const uint32_t x = (uint32_t)__builtin_amdgcn_readlane((int)(va ^ vb), f);
                            c = 4 * f + (__builtin_ctz(x) >> 3);
                        }
                        c = min(c, max(mlimit - (ip + total), 0));
                        if (c < kWinBytes) break;
                        total += kWinBytes;
                        va = rdw(D, ip + total + 4 * lane, n);
                        vb = rdw(D, c2 + total + 4 * lane, n);
                        ne = ballot(va != vb);
                    }
                    tail = va;
                    tb = ip + total;
                    ref = c2;
                    mc = total + c - kMinMatch;
                    lit = 0;
                }
                STAMP(4);
                // a miss: search from anchor + 1 (its first window's bytes;
                // read beside every re-test's table ops instead, variant
                // 172032 in round 4: no change on G1 / G2 / E = 3 / E = 12)
                pre = rdw(D, ip + 1 + lane, n);
                ip = anchor + 1;
                continue;
            }
            for (;;) {
                // ------------------------------------------------ emit sequence
                if (!em.seq(op, anchor, ip, ip - ref, mc)) return -1;
                COUNT(5, ip - anchor);
                ip += mc + kMinMatch;
                anchor = ip;
                STAMP(3);
                if (ip >= limit) goto last_literals;  // straight out: the miss exit below stays the only break
                // fill table at ip-2, then test ip (lz4/lz4.c:1230-1293)
                const int t = ip - co.tail_base;
                uint32_t x2, x0, h2, h0;
                if (!WIDE && t >= 2 && t <= 4 * kWave - 8) {
                    x2 = win_rd32(co.tail, co.tail_base, ip - 2);
                    x0 = win_rd32(co.tail, co.tail_base, ip);
                    h2 = hash4(x2);
                    h0 = hash4(x0);
                } else {
                    x0 = lds_rd32(D, ip);
                    h2 = hash_at<WIDE>(D, ip - 2);
                    h0 = hash_at<WIDE>(D, ip);
                }
                // the next search window's bytes and the test's a-side window,
                // in flight during the table exchange
                pre = rdw(D, ip + 1 + lane, n);
                const uint32_t va0 = rdw(D, ip + 4 * lane, n);
                uint32_t c2 = 0;
                if constexpr ((OPT & 8) == 0) {
                    // plain ops by every lane (same address, same value; the
                    // read is a broadcast), in order: the read sees the ip-2
                    // insert when both hashes agree.  No exec-mask switch, and
                    // c2 stays in a VGPR (no readfirstlane on the chain).
                    T.put(h2, (uint32_t)(ip - 2));
                    c2 = T.get(h0);
                    T.put(h0, (uint32_t)ip);
                } else {
                    // A/B variant 8: lane 0 alone, one returning exchange
                    if (lane == 0) {
                        T.put(h2, (uint32_t)(ip - 2));
                        c2 = T.exchange(h0, (uint32_t)ip);
                    }
                    c2 = uni(c2);
                }
                if constexpr (!WIDE && (OPT & 2048) == 0) {
                    // the 4-byte test is lane 0's bit of the count's first
                    // ballot (no separate readfirstlane compare); A/B variant
                    // 2048: test_and_count
                    uint32_t va = va0, vb = rdw(D, (int)c2 + 4 * lane, n);
                    uint64_t ne = ballot(va != vb);
                    if (ne & 1ull) {
                        STAMP(4);
                        break;
                    }
                    int total = 0, c;
                    for (;;) {
                        c = kWinBytes;
                        if (ne) {
                            const int f = ffs64(ne);
                            const uint32_t x = (uint32_t)__builtin_amdgcn_readlane((int)(va ^ vb), f);
                            c = 4 * f + (__builtin_ctz(x) >> 3);
                        }
                        c = min(c, max(mlimit - (ip + total), 0));
                        if (c < kWinBytes) break;
                        total += kWinBytes;
                        va = rdw(D, ip + total + 4 * lane, n);
                        vb = rdw(D, (int)c2 + total + 4 * lane, n);
                        ne = ballot(va != vb);
                    }
                    co.tail = va;
                    co.tail_base = ip + total;
                    ref = (int)c2;
                    mc = total + c - kMinMatch;
                    COUNT(3, 1);
                    STAMP(4);
                    continue;
                }
                const bool near = !WIDE || c2 + kMaxDistance >= (uint32_t)ip;
                if (near) {
                    co = test_and_count(D, n, ip, (int)c2, mlimit, lane, va0);
                    if (co.cnt >= 0) {
                        // zero-literal sequence, no catch-up on this path
                        ref = (int)c2;
                        mc = co.cnt;
                        COUNT(3, 1);
                        STAMP(4);
                        continue;
                    }
                }
                STAMP(4);
                break;
            }
            // a miss: anchor < limit (the re-test ran), search from anchor + 1
            ip = anchor + 1;
        }
    }
    // ---------------------------------------------------- last literals
last_literals:
    em.last(op, anchor, n);
    STAMP(5);
    COUNT(4, 1);
    DIAG_FLUSH;
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
__device__ __forceinline__ void transpose_regs_to_lds(const BlockRegs<EK>& R, lds8* D, int P,
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

// 4-groups-per-lane variant (P % 4 == 0): lane q owns groups 4q..4q+3, i.e.
// 32*EK contiguous input bytes, and writes ONE dword per plane to LDS.
template <int EK>
struct BlockRegs4 {
    static constexpr int kIters = (EK ? 8192 / (kWave * 32 * EK) : 1) > 0
                                      ? (EK ? 8192 / (kWave * 32 * EK) : 1) : 1;
    uint32_t w[kIters][4][2 * (EK ? EK : 1)];
};

template <int EK>
__device__ __forceinline__ void issue_block_loads4(BlockRegs4<EK>& R, const uint8_t* src, int P,
                                                   int lane) {
    const int P4 = P >> 2;
#pragma unroll
    for (int it = 0; it < BlockRegs4<EK>::kIters; it++) {
        const int q = it * kWave + lane;
        if (q < P4) {
#pragma unroll
            for (int k = 0; k < 4; k++) load_group<EK>(src + ((int64_t)q * 4 + k) * 8 * EK, R.w[it][k]);
        }
    }
}

template <int EK>
__device__ __forceinline__ void transpose4_regs_to_lds(const BlockRegs4<EK>& R, lds8* D, int P,
                                                       int lane) {
    const int P4 = P >> 2;
    lds32* D32 = (lds32*)D;
#pragma unroll
    for (int it = 0; it < BlockRegs4<EK>::kIters; it++) {
        const int q = it * kWave + lane;
        if (q < P4) {
            uint32_t pl[8 * EK];
#pragma unroll
            for (int r = 0; r < 8 * EK; r++) pl[r] = 0;
#pragma unroll
            for (int k = 0; k < 4; k++) {
#pragma unroll
                for (int b = 0; b < EK; b++) {
                    const uint64_t v = tr8x8(gather_byte_plane<EK>(R.w[it][k], b));
#pragma unroll
                    for (int j = 0; j < 8; j++)
                        pl[8 * b + j] |= (uint32_t)((v >> (8 * j)) & 0xFFu) << (8 * k);
                }
            }
#pragma unroll
            for (int r = 0; r < 8 * EK; r++) D32[r * P4 + q] = pl[r];
        }
    }
}

// The same, bit-sliced over the lane's four groups at once (A/B variant bit
// 262144): x[8b + i] gathers byte b of element i of all four groups (byte k =
// group k, three v_perm_b32), one 8x8 bit transpose per byte lane across those
// eight registers (untranspose4_rows: the transpose is its own inverse) leaves
// x[8b + j] = plane 8b + j of the four groups -- ONE dword per plane as above.
#ifndef BSHUF_TR_SOFF
#define BSHUF_TR_SOFF 1
#endif
template <int EK>
__device__ __forceinline__ void transpose4s_regs_to_lds(const BlockRegs4<EK>& R, lds8* D, int P,
                                                        int lane) {
    const int P4 = P >> 2;
    lds32* D32 = (lds32*)D;
#pragma unroll
    for (int it = 0; it < BlockRegs4<EK>::kIters; it++) {
        const int q = it * kWave + lane;
        if (q < P4) {
            uint32_t x[8 * EK];
#pragma unroll
            for (int b = 0; b < EK; b++) {
#pragma unroll
                for (int i = 0; i < 8; i++) {
                    const int o = i * EK + b, d = o >> 2;
                    const uint32_t sel = (uint32_t)(o & 3) | ((uint32_t)(4 + (o & 3)) << 8) | 0x0C0C0000u;
                    const uint32_t lo = __builtin_amdgcn_perm(R.w[it][1][d], R.w[it][0][d], sel);
                    const uint32_t hi = __builtin_amdgcn_perm(R.w[it][3][d], R.w[it][2][d], sel);
                    x[8 * b + i] = __builtin_amdgcn_perm(hi, lo, 0x05040100u);
                }
            }
            untranspose4_rows<EK>(x);
            // plane r's dword of this lane at Dq + r * rs: the row offsets are
            // wave-uniform (scalar multiplies), not per-lane 64-bit mads
            lds8* const Dq = D + 4 * q;
            const int rs = 4 * P4;
            int ro = 0;
#pragma unroll
            for (int r = 0; r < 8 * EK; r++) {
                *(lds32*)(Dq + ro) = x[r];
                ro += rs;
                // E >= 4: an opaque scalar (one v_add per row instead of a
                // 64-bit v_mad per row; 1 GiB G2 -2.2 %, E = 2 measured flat or
                // worse beside the pipelined lane_runs, profiles/r06/enc_ab)
                if constexpr (BSHUF_TR_SOFF && EK >= 4) asm volatile("" : "+s"(ro));
            }
        }
    }
}

// Any element size (EK == 0): the block's raw bytes (<= kRawBytes) travel
// from HBM as coalesced 8-byte loads into registers (prefetched like the
// EK-specialised paths), land in the still-unused hash-table LDS, and the
// bit transpose gathers each 8-element group's byte b from there -- the
// strided byte gathers hit LDS instead of HBM.
constexpr int kRawBytes = 8192;
#ifndef BSHUF_EK0_DEFER
#define BSHUF_EK0_DEFER 1
#endif
constexpr int kRawIters = kRawBytes / (8 * kWave);
struct RawRegs {
    uint2 w[kRawIters];
};
__device__ __forceinline__ void issue_raw_loads(RawRegs& R, const uint8_t* src, int nbytes, int lane) {
#pragma unroll
    for (int it = 0; it < kRawIters; it++) {
        const int i = it * kWave + lane;
        if (8 * i < nbytes) R.w[it] = reinterpret_cast<const uint2*>(src)[i];
    }
}
__device__ __forceinline__ void raw_to_lds(const RawRegs& R, lds8* S, int nbytes, int lane) {
#pragma unroll
    for (int it = 0; it < kRawIters; it++) {
        const int i = it * kWave + lane;
        if (8 * i < nbytes) ((lds64v*)S)[i] = u32x2{R.w[it].x, R.w[it].y};
    }
}

#ifndef BSHUF_FLUSH4
#define BSHUF_FLUSH4 1  // A/B builds: 0 = round 5's copy-out and zeroing loops
#endif
// Persistent: workgroup w handles blocks w, w+G, w+2G, ...  While block k is
// parsed out of LDS, the 8 KiB of block k+G are already in flight into
// registers, so HBM latency hides under the (LDS-latency-bound) parse.
// One wave per workgroup: LDS hand-offs need no s_barrier, and avoiding
// __syncthreads() keeps its release fence from draining the prefetch.
template <int EK, bool WIDE, int VAR>
__global__ __launch_bounds__(64) void k_lz4_encode(EncArgs a, int64_t nb) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    // issue priority over a concurrent compaction's waves (pipelined encode)
    __builtin_amdgcn_s_setprio(2);
    const int lane = threadIdx.x;
    const int E = EK ? EK : a.L.E;
    (void)smem;
    lds8* const L0 = lds_origin();
    lds8* D = L0 + kTableBytes;
    const int64_t stride = gridDim.x;
    int64_t blk = blockIdx.x;
    if (blk >= nb) return;
    // block k -> (elements, source): one stream, or a batch of streams
    constexpr bool kBatch = (VAR & 256) != 0;
    auto blk_m = [&](int64_t k) {
        if (!kBatch) return k < a.L.nfull ? a.L.bs : a.L.last;
        const Seg& g = a.segs[a.blk_seg[k + a.blk0]];
        return k + a.blk0 - g.first < g.nfull ? a.L.bs : g.last;
    };
    auto blk_src = [&](int64_t k) {
        if (!kBatch) return a.in + k * (int64_t)a.L.bs * E;
        const Seg& g = a.segs[a.blk_seg[k + a.blk0]];
        return g.in + (k + a.blk0 - g.first) * (int64_t)a.L.bs * E;
    };

    BlockRegs<EK> R;
    BlockRegs4<EK> R4;
    RawRegs RW;
    auto raw_fits = [&](int m) { return EK == 0 && a.raw8 && m * E <= kRawBytes; };
    constexpr bool kX4 = (VAR & 4) == 0;  // 4-groups-per-lane transpose (default)
    // insert/readback search window: the fallback when the device's LDS
    // atomics do not serialise in lane order
    constexpr bool kReadback = (VAR & 128) != 0;
    constexpr int kRegGroups = BlockRegs<EK>::kIters * kWave;
    constexpr int kRegGroups4 = BlockRegs4<EK>::kIters * kWave * 4;
    // a block fits the prefetch registers when its groups fit
    auto fits = [&](int m) { return EK != 0 && m / 8 <= kRegGroups; };
    auto fits4 = [&](int m) { return kX4 && EK != 0 && (m / 8) % 4 == 0 && m / 8 <= kRegGroups4; };
    if constexpr (EK != 0) {
        const int m0 = blk_m(blk);
        if (fits4(m0))
            issue_block_loads4<EK>(R4, blk_src(blk), m0 / 8, lane);
        else if (fits(m0))
            issue_block_loads<EK>(R, blk_src(blk), m0 / 8, lane);
    } else {
        const int m0 = blk_m(blk);
        if (raw_fits(m0)) issue_raw_loads(RW, blk_src(blk), m0 * E, lane);
    }

    // Deferred copy-out (A/B variant 4096 turns it off): a block's record
    // stays in the table's LDS until the next block is transposed.
    constexpr bool kDefer = (EK != 0 || BSHUF_EK0_DEFER) && (VAR & 4096) == 0;
    constexpr bool kFlush4 = BSHUF_FLUSH4 && EK != 4;
    int64_t pend_blk = -1;
    int pend_c = 0;
    auto flush_pending = [&]() {
        if (pend_blk < 0) return;
        uint8_t* po = a.scratch + pend_blk * a.slot;
        const int nch = (4 + pend_c + 15) >> 4;
        // up to four 16-byte chunks per lane read before any is stored: one
        // LDS round trip per 4 KiB of record instead of one per KiB (with the
        // unrolled table zeroing below: 1 GiB G1 0.299 -> 0.297 ms, E = 3
        // 1.055 -> 1.040; E = 4 0.788 -> 0.809, so not there; each change
        // alone measured worse, profiles/r06/enc_ab)
        if constexpr (kFlush4) {
        for (int i0 = 0; i0 < nch; i0 += 4 * kWave) {
            // (reads past the record stay inside the table's 16 KiB: a staged
            // record has nch <= 1024 chunks, so i0 <= 768 and i < 1024)
            u32x4 v[4];
#pragma unroll
            for (int u = 0; u < 4; u++) v[u] = ((const lds128*)L0)[i0 + u * kWave + lane];
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const int i = i0 + u * kWave + lane;
                if (i < nch) ((gbl128*)po)[i] = v[u];
            }
        }
        } else {
            for (int i = lane; i < nch; i += kWave) ((gbl128*)po)[i] = ((const lds128*)L0)[i];
        }
        if (lane == 0) a.foot[pend_blk] = 4 + (uint64_t)pend_c;
        pend_blk = -1;
    };
    KDIAG_DECL
    for (;;) {
        KSTAMP(3);
        const int m = blk_m(blk);
        const int n = m * E;
        const int P = m / 8;
        const uint8_t* src = blk_src(blk);
        // any element size, staged: raw bytes into the table's LDS, bit
        // transpose from there (before the table is zeroed)
        bool staged = false;
        if constexpr (EK == 0) {
            if (raw_fits(m)) {
                staged = true;
                // deferred copy-out: the raw bytes go to the END of the table,
                // behind the previous block's record (flushed first when the
                // two would overlap -- an incompressible record)
                int rawoff = 0;
                if constexpr (kDefer) {
                    rawoff = (kTableBytes - ((n + 7) & ~7)) & ~15;
                    if (pend_blk >= 0 && 16 * ((4 + pend_c + 15) >> 4) > rawoff) {
                        flush_pending();
                        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                        __builtin_amdgcn_wave_barrier();
                    }
                }
                lds8* const RS = L0 + rawoff;
                raw_to_lds(RW, RS, n, lane);
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                // lane = (group g, byte b) with b fastest: the 8 gathers of
                // neighbouring lanes hit neighbouring bytes (no bank conflicts)
                const uint32_t magic = (uint32_t)((0x100000000ull + (uint64_t)E - 1) / (uint64_t)E);
                for (int i = lane; i < P * E; i += kWave) {
                    const int g = (int)__umulhi((uint32_t)i, magic), b = i - g * E;
                    const lds8* x = RS + 8 * g * E + b;
                    uint64_t v = 0;
#pragma unroll
                    for (int k = 0; k < 8; k++) v |= (uint64_t)x[k * E] << (8 * k);
                    v = tr8x8(v);
#pragma unroll
                    for (int j = 0; j < 8; j++) D[(8 * b + j) * P + g] = (uint8_t)(v >> (8 * j));
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
            }
        }
        // zero the hash table (LZ4_initStream) and the read pad behind the block
        // (deferred copy-out: after the transpose, once the previous record
        // has left the table's LDS)
        if constexpr (!kDefer) {
            for (int i = lane; i < kTableBytes / 16; i += kWave)
                ((lds128*)L0)[i] = u32x4{0u, 0u, 0u, 0u};
        }
        if (lane < kDataPad / 4) ((lds32*)(D + ((n + 3) & ~3)))[lane] = 0;
        // bit transpose into LDS (bshuf_trans_bit_elem)
        if (staged) {
        } else if constexpr (EK != 0) {
            if (fits4(m)) {
                if constexpr ((VAR & 262144) != 0)
                    transpose4s_regs_to_lds<EK>(R4, D, P, lane);
                else
                    transpose4_regs_to_lds<EK>(R4, D, P, lane);
            } else if (fits(m)) {
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
        if constexpr (kDefer) {
            // the previous block's record leaves now, behind this block's
            // transpose: its stores are older than the prefetch below, so the
            // next iteration's wait for that prefetch finds them long done
            // (issued at the end of a parse, they would hold it up instead)
            flush_pending();
            if constexpr (kFlush4) {
#pragma unroll
                for (int k = 0; k < kTableBytes / 16 / kWave; k++)
                    ((lds128*)L0)[k * kWave + lane] = u32x4{0u, 0u, 0u, 0u};
            } else {
                for (int i = lane; i < kTableBytes / 16; i += kWave)
                    ((lds128*)L0)[i] = u32x4{0u, 0u, 0u, 0u};
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
        }
        // prefetch the next block while this one is parsed
        const int64_t next = blk + stride;
        if constexpr (EK != 0) {
            if (next < nb) {
                const int mn = blk_m(next);
                if (fits4(mn))
                    issue_block_loads4<EK>(R4, blk_src(next), mn / 8, lane);
                else if (fits(mn))
                    issue_block_loads<EK>(R, blk_src(next), mn / 8, lane);
            }
        } else {
            if (next < nb) {
                const int mn = blk_m(next);
                if (raw_fits(mn)) issue_raw_loads(RW, blk_src(next), mn * E, lane);
            }
        }

        KSTAMP(0);
        uint8_t* out = a.scratch + blk * a.slot;
        const Table<WIDE> T{L0};
        int c = -1;
        // default: descriptors during the parse, bytes afterwards (the record
        // is staged in the table's LDS, dead once the parse is over)
        constexpr bool kDesc = !WIDE && (VAR & 2) == 0;
        if constexpr (kDesc) {
            if (a.desc_ok && 4 + lz4_bound(n) + 15 <= kTableBytes) {
                // VAR & 8192: the hand-scheduled re-test chain, whose
                // descriptors are buffered in VGPRs
                using Em = typename std::conditional<(VAR & 8192) != 0, EmitDescV, EmitDesc>::type;
                Em em{(lds32*)(D + a.desc_off), lane};
                c = lz4_encode_block<WIDE, kReadback, (VAR & (8 | 512 | 2048 | 16384 | 32768 | 131072 | 524288)) |
                                                          (EK == 4 ? kOptCountFirst : 0)>(D, n, T, em, lane);
                KSTAMP(1);
                if (em.ns > kDescMax) c = -1;  // more sequences than descriptor slots
                if (c >= 0) {
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                    __builtin_amdgcn_wave_barrier();
                    lds8* S = L0;
                    c = emit_sequences<(VAR & 2097152) != 0>(D, em, n, S, lane);
                    if (lane < 4) S[lane] = (uint8_t)((uint32_t)c >> (24 - 8 * lane));
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                    __builtin_amdgcn_wave_barrier();
                    if constexpr (kDefer) {
                        pend_blk = blk;
                        pend_c = c;
                    } else {
                        const int nch = (4 + c + 15) >> 4;
                        for (int i = lane; i < nch; i += kWave)
                            ((gbl128*)out)[i] = ((const lds128*)S)[i];
                    }
                } else {
                    // more sequences than descriptor slots: parse again with
                    // the inline emitter (fresh table)
                    for (int i = lane; i < kTableBytes / 16; i += kWave)
                        ((lds128*)L0)[i] = u32x4{0u, 0u, 0u, 0u};
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                    __builtin_amdgcn_wave_barrier();
                }
            }
        }
        if (c < 0) {
            EmitBytes<> em{out + 4, D, lane};
            c = lz4_encode_block<WIDE, kReadback, (VAR & (8 | 512 | 2048))>(D, n, T, em, lane);
            if (lane < 4) out[lane] = (uint8_t)((uint32_t)c >> (24 - 8 * lane));
        }
        if (lane == 0 && pend_blk != blk) a.foot[blk] = 4 + (uint64_t)c;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        KSTAMP(2);
        if (next >= nb) break;
        blk = next;
    }
    if constexpr (kDefer) flush_pending();
    KDIAG_FLUSH;
}

// Move each [BE32 c][c bytes] record from its scratch slot to out + offs[k].
// Every lane owns 16-byte chunks of the ABSOLUTE destination address space:
// it reads the two 16-aligned source granules under its chunk (the shift
// between source and destination is the same for every chunk of a record, so
// the dword select is wave-uniform), composes the chunk with v_alignbyte and
// stores it whole -- or, for the <= 2 edge chunks a record shares with its
// neighbours, byte by byte from the same registers.  Up to kCompactUnroll
// chunks per lane are loaded before any is stored.  One WAVE per record, four
// records per 256-thread workgroup; records first .. nb-1 (a pipelined
// segment, or all).
constexpr int kCompactPerWg = 4;
constexpr int kCompactUnroll = 4;

// 16 bytes at byte offset t (0..15, wave-uniform) of the 32-byte pair a|b.
__device__ __forceinline__ u32x4 pair_bytes(const u32x4 a, const u32x4 b, int t) {
    const uint32_t w[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    const uint32_t sh = (uint32_t)(t & 3);
    u32x4 v;
    switch (t >> 2) {
#define BSHUF_PAIR(D)                                                                          \
    case D:                                                                                     \
        v = u32x4{__builtin_amdgcn_alignbyte(w[D + 1], w[D], sh),                               \
                  __builtin_amdgcn_alignbyte(w[D + 2], w[D + 1], sh),                           \
                  __builtin_amdgcn_alignbyte(w[D + 3], w[D + 2], sh),                           \
                  __builtin_amdgcn_alignbyte(w[D + 4], w[D + 3], sh)};                          \
        break;
        BSHUF_PAIR(0)
        BSHUF_PAIR(1)
        BSHUF_PAIR(2)
        default: BSHUF_PAIR(3)
#undef BSHUF_PAIR
    }
    return v;
}

__global__ __launch_bounds__(256) void k_compact(const uint8_t* __restrict__ scratch, int64_t slot,
                                                 const uint64_t* __restrict__ offs,
                                                 uint8_t* __restrict__ out, const Seg* segs,
                                                 const uint32_t* __restrict__ blk_seg,
                                                 uint64_t* __restrict__ block_offsets, int64_t first,
                                                 int64_t nb) {
    const int64_t blk = first + (int64_t)blockIdx.x * kCompactPerWg + (threadIdx.x >> 6);
    const int tid = threadIdx.x & 63;
    if (blk >= nb) return;
    uint64_t rel0 = offs[blk];
    const int64_t len = (int64_t)(offs[blk + 1] - rel0);
    if (segs) {  // batch: offsets are relative to the block's own stream
        const Seg& g = segs[blk_seg[blk]];
        rel0 -= offs[g.first];
        out = g.out;
    }
    if (block_offsets && tid == 0) block_offsets[blk] = rel0;
    // the slot is 16-aligned and 16 bytes longer than any record
    const gbl128c* rec16 = (const gbl128c*)(scratch + blk * slot);
    const uintptr_t dst0 = (uintptr_t)(out + rel0);
    const int64_t nq = (int64_t)(((dst0 + (uintptr_t)len + 15) >> 4) - (dst0 >> 4));
    // chunk j starts at record byte s = 16 j - m: granules j - (m != 0) and
    // the next one, byte offset t in the pair
    const int m = (int)(dst0 & 15);
    const int gshift = m ? 1 : 0, t = m ? 16 - m : 0;
    gbl8* const d0 = (gbl8*)(dst0 & ~(uintptr_t)15);
    for (int64_t jb = 0; jb < nq; jb += kWave * kCompactUnroll) {
        u32x4 A[kCompactUnroll], Bv[kCompactUnroll];
#pragma unroll
        for (int u = 0; u < kCompactUnroll; u++) {
            const int64_t j = jb + u * kWave + tid;
            const int64_t g = j - gshift;
            A[u] = u32x4{0u, 0u, 0u, 0u};
            Bv[u] = u32x4{0u, 0u, 0u, 0u};
            if (j < nq) {
                if (g >= 0) A[u] = rec16[g];
                if (m) Bv[u] = rec16[g + 1];
            }
        }
#pragma unroll
        for (int u = 0; u < kCompactUnroll; u++) {
            const int64_t j = jb + u * kWave + tid;
            if (j >= nq) continue;
            const int64_t s = 16 * j - m;
            const u32x4 v = pair_bytes(A[u], Bv[u], t);
            gbl8* d = d0 + 16 * j;
            if (s >= 0 && s + 16 <= len) {
                *(gbl128*)d = v;
            } else {
                const uint32_t vw[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
                for (int i = 0; i < 16; i++)
                    if (s + i >= 0 && s + i < len) d[i] = (uint8_t)(vw[i >> 2] >> (8 * (i & 3)));
            }
        }
    }
}

// Blocks too large for the LDS (above max_lds_encode_bytes): one wave per
// block runs the same wave-parallel parse (lz4_encode_block) with only the
// 16 KiB hash table in LDS -- byU32/hash5 from 65547 bytes, as
// LZ4_compress_default picks (lz4/lz4.c:1388-1393) -- and the bit-transposed
// block read from the global scratch (GblBlk); the LZ4 bytes go straight to
// the block's scratch slot (EmitBytes).  16 KiB of LDS per wave: up to 10
// blocks resident per CU.
template <bool READBACK>
__global__ __launch_bounds__(64) void k_lz4_encode_big(const uint8_t* __restrict__ shuf, Layout L,
                                                       uint8_t* __restrict__ scratch, int64_t slot,
                                                       uint64_t* __restrict__ foot) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int lane = threadIdx.x;
    const int64_t k = blockIdx.x;
    const int m = k < L.nfull ? L.bs : L.last;
    const int n = m * L.E;
    lds8* const tb = to_lds(smem);
    for (int i = lane; i < kTableBytes / 16; i += kWave) ((lds128*)tb)[i] = u32x4{0u, 0u, 0u, 0u};
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    uint8_t* out = scratch + k * slot;
    const GblBlk D{shuf + k * (int64_t)L.bs * L.E};
    EmitBytes<GblBlk> em{out + 4, D, lane};
    // a short last block below 65547 bytes takes the byU16 table, as LZ4 does
    const int c = n >= kU16TableLimit ? lz4_encode_block<true, READBACK, 0>(D, n, Table<true>{tb}, em, lane)
                                      : lz4_encode_block<false, READBACK, 0>(D, n, Table<false>{tb}, em, lane);
    if (lane < 4) ((gbl8*)out)[lane] = (uint8_t)((uint32_t)c >> (24 - 8 * lane));
    if (lane == 0) foot[k] = 4 + (uint64_t)c;
}

// The n%8 leftover elements are copied verbatim behind the last block
// (src/bitshuffle_core.c:1919-1926); their offset is only known on the device.
__global__ void k_encode_finish(const uint64_t* offs, int64_t nblocks, const uint8_t* tail_src,
                                int64_t tail, uint8_t* out, int64_t* result) {
    const uint64_t end = offs[nblocks];
    for (int i = threadIdx.x; i < tail; i += blockDim.x) out[end + i] = tail_src[i];
    if (threadIdx.x == 0) *result = (int64_t)end + tail;
}

// Batch: one workgroup per stream.
__global__ void k_encode_finish_batch(const uint64_t* offs, const Seg* segs, int32_t bs, int32_t E) {
    const Seg& g = segs[blockIdx.x];
    const int64_t nb = g.nfull + (g.last ? 1 : 0);
    const uint64_t end = offs[g.first + nb] - offs[g.first];
    const uint8_t* tail_src = g.in + (g.nfull * (int64_t)bs + g.last) * E;
    for (int i = threadIdx.x; i < g.tail; i += blockDim.x) g.out[end + i] = tail_src[i];
    if (threadIdx.x == 0) *g.result = (int64_t)end + g.tail;
}

// Device check of the property Table::exchange relies on: same-address lanes
// of ONE returning LDS atomic (ds_mskor_rtn_b32, ds_wrxchg_rtn_b32) are
// processed in lane order.  512 patterns of active lanes / entries / halves;
// each lane compares its returned value with the lane-order prediction.
__global__ __launch_bounds__(64) void k_lds_order_check(int* fails) {
    __shared__ uint32_t S[16];
    const int lane = threadIdx.x;
    int bad = 0;
    for (int p = 0; p < 512; p++) {
        if (lane < 16) S[lane] = 0;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        const int kind = p & 3;
        const uint32_t ndw = kind == 0 ? 1u : (kind == 1 ? 2u : (kind == 2 ? 4u : 16u));
        const bool xchg = (p >> 2) & 1;
        auto pick = [&](int q) {
            uint32_t x = (uint32_t)(p * 64 + q + 1) * 0x9E3779B1u;
            x ^= x >> 15;
            x *= 0x85EBCA77u;
            return x ^ (x >> 13);
        };
        const uint32_t x = pick(lane);
        const bool active = kind == 0 || x % 3u != 0u;
        const uint32_t dw = (x >> 4) % ndw, sh = 16u * ((x >> 9) & 1u);
        if (active) {
            const uint32_t ad = lds_addr(S + dw), val = (uint32_t)(lane + 1) << sh;
            const uint32_t r = xchg ? lds_xchg_rtn(ad, val) : lds_mskor_rtn(ad, 0xFFFFu << sh, val);
            uint32_t e = 0;
            for (int q = 0; q < lane; q++) {
                const uint32_t y = pick(q);
                if (!(kind == 0 || y % 3u != 0u) || (y >> 4) % ndw != dw) continue;
                const uint32_t shq = 16u * ((y >> 9) & 1u), vq = (uint32_t)(q + 1) << shq;
                e = xchg ? vq : ((e & ~(0xFFFFu << shq)) | vq);
            }
            bad += r != e;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
    }
    if (bad) atomicAdd(fails, bad);
}

// Once per device (cached): does k_lds_order_check pass?  The check runs on a
// private stream with a private (kept) allocation, so the caller's stream is
// neither synchronised nor captured; its one hipStreamSynchronize happens on
// the first encode per device.  Inside a caller's stream capture nothing of
// this touches the captured stream.
bool lds_atomics_lane_ordered() {
    static std::atomic<int> state[64];
    static std::mutex mu;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return false;
    int st = state[dev].load(std::memory_order_acquire);
    if (st) return st == 1;
    std::lock_guard<std::mutex> g(mu);
    st = state[dev].load(std::memory_order_acquire);
    if (st) return st == 1;
    hipStream_t ps = nullptr;
    int* d = nullptr;
    int h = -1;
    bool ok = hipStreamCreateWithFlags(&ps, hipStreamNonBlocking) == hipSuccess &&
              hipMalloc(&d, sizeof(int)) == hipSuccess &&
              hipMemsetAsync(d, 0, sizeof(int), ps) == hipSuccess;
    if (ok) {
        hipLaunchKernelGGL(k_lds_order_check, dim3(1), dim3(kWave), 0, ps, d);
        ok = hipGetLastError() == hipSuccess &&
             hipMemcpyAsync(&h, d, sizeof(int), hipMemcpyDeviceToHost, ps) == hipSuccess &&
             hipStreamSynchronize(ps) == hipSuccess;
    }
    // d and ps are kept: freeing them could synchronise the device
    const bool ordered = ok && h == 0;
    state[dev].store(ok ? (ordered ? 1 : 2) : 2, std::memory_order_release);
    return ordered;
}

// The encoder addresses its dynamic LDS from address 0 (lds_origin): true
// when the kernel has no static LDS in front of it.
bool lds_layout_ok(const void* fn) {
    hipFuncAttributes at{};
    return hipFuncGetAttributes(&at, fn) == hipSuccess && at.sharedSizeBytes == 0;
}

template <bool READBACK>
hipError_t launch_big_t(const uint8_t* shuf, const Layout& L, const EncodeBufs& b, hipStream_t s) {
    const int64_t nb = L.nblocks();
    auto fn = k_lz4_encode_big<READBACK>;
    ProfScope prof("k_lz4_encode_big", s);
#ifndef BSHUF_BIG_LDS_PAD
#define BSHUF_BIG_LDS_PAD 0  // A/B builds only: fewer resident large blocks per CU
#endif
    hipLaunchKernelGGL(fn, dim3((unsigned)nb), dim3(kWave), kTableBytes + BSHUF_BIG_LDS_PAD, s, shuf, L, b.scratch,
                       b.slot, b.foot);
    return hipGetLastError();
}

template <int EK, bool WIDE, int VAR = 0>
hipError_t launch_enc_t(const EncArgs& a, int64_t nb, size_t lds, hipStream_t s) {
    if constexpr (EK == 2 && !WIDE && VAR == 0) {
        // byte-identical A/B variants (bshuf_set_variant, tools/ab.py): 2 inline
        // emitter, 4 one-group-per-lane transpose, 128 insert/readback search
        const int v = tuning_variant();
        if (v == 2) return launch_enc_t<2, false, 2>(a, nb, lds, s);
        if (v == 4) return launch_enc_t<2, false, 4>(a, nb, lds, s);
        if (v == 128) return launch_enc_t<2, false, 128>(a, nb, lds, s);
        if (v == 8) return launch_enc_t<2, false, 8>(a, nb, lds, s);
        if (v == 4096) return launch_enc_t<2, false, 4096>(a, nb, lds, s);
        if (v == 2048) return launch_enc_t<2, false, 2048>(a, nb, lds, s);
        if (v == 512) return launch_enc_t<2, false, 512>(a, nb, lds, s);
    }
    if constexpr (!WIDE && (VAR & ~256) == 0) {
        // default (byU16, every element size, single stream and batch): the
        // hand-scheduled re-test chain with its offset-2 shortcut (8192 |
        // 32768), and for E = 1, 2, 4, 8 the hand-scheduled search windows
        // (| 16384) and the bit-sliced forward transpose (| 262144).  A/B variants: 65536 the compiled re-test (round 3's
        // default), 8192 the chain without the shortcut, 16384 / 24576 /
        // 57344 the hand-scheduled search windows (alone / with the chain /
        // with the chain and its shortcut).
        const int v = tuning_variant();
        if (v == 65536) return launch_enc_t<EK, WIDE, VAR | 65536>(a, nb, lds, s);
        if (v == 8192) return launch_enc_t<EK, WIDE, VAR | 8192>(a, nb, lds, s);
        if (v == 16384) return launch_enc_t<EK, WIDE, VAR | 16384>(a, nb, lds, s);
        if (v == 24576) return launch_enc_t<EK, WIDE, VAR | 24576>(a, nb, lds, s);
        // the hand-scheduled search windows as well for the element sizes of
        // the BASELINE configs (2 GiB G1 int16 0.716 -> 0.693 ms, 1 GiB G2
        // float32 0.933 -> 0.914 ms per launch; odd element sizes without
        // them: E = 3 / 12 +0.2 % / +0.8 % with them, profiles/r04/asm_search),
        // and their bit-sliced forward transpose (0.694 -> 0.676 / 0.912 ->
        // 0.905 ms, profiles/r04/etr_sliced)
        // ... and the search-match -> re-test hand-off in asm (search_entry,
        // | 131072): k_lz4_encode 2 GiB G1 0.677 -> 0.631 ms, 1 GiB G2 0.911
        // -> 0.846, 1 GiB as E = 3 1.347 -> 1.218, E = 12 1.229 -> 1.133 per
        // launch (profiles/r05/r5b)
        // ... and the whole parse loop as one asm block (parse_chain, |
        // 524288) with the emission's literal runs by lane_runs (| 2097152):
        // 2 GiB G1 0.621 -> 0.592 ms, 1 GiB G2 0.832 -> 0.781, E = 3 1.213 ->
        // 1.036, E = 12 1.129 -> 1.001 per launch (profiles/r05/r5d; lane_runs
        // alone -0.3..-0.6 % of that); 450560 / 172032, 319488 / 40960 stay as
        // A/B variants
        if (v == 0) return launch_enc_t<EK, WIDE, VAR | (EK == 0 ? 2793472 : 3072000)>(a, nb, lds, s);
        if (v == 3072000 && EK != 0) return launch_enc_t<EK, WIDE, VAR | 3072000>(a, nb, lds, s);
        if (v == 3072000 || v == 2793472) return launch_enc_t<EK, WIDE, VAR | 2793472>(a, nb, lds, s);
        if (v == 40960) return launch_enc_t<EK, WIDE, VAR | 40960>(a, nb, lds, s);
        if (v == 57344) return launch_enc_t<EK, WIDE, VAR | 57344>(a, nb, lds, s);
        // the search-match -> re-test hand-off in asm (search_entry), compiled glue
        if (v == 172032) return launch_enc_t<EK, WIDE, VAR | 172032>(a, nb, lds, s);
        if (v == 450560 && EK != 0) return launch_enc_t<EK, WIDE, VAR | 450560>(a, nb, lds, s);
        if (v == 450560) return launch_enc_t<EK, WIDE, VAR | 172032>(a, nb, lds, s);
        if (v == 319488 && EK != 0) return launch_enc_t<EK, WIDE, VAR | 319488>(a, nb, lds, s);
        if (v == 319488) return launch_enc_t<EK, WIDE, VAR | 40960>(a, nb, lds, s);
    }
    if constexpr ((VAR & 128) == 0) {
        if (!lds_atomics_lane_ordered()) return launch_enc_t<EK, WIDE, VAR | 128>(a, nb, lds, s);
    }
    auto fn = k_lz4_encode<EK, WIDE, VAR>;
    if (!lds_layout_ok(reinterpret_cast<const void*>(fn))) return hipErrorInvalidDeviceFunction;
    if (lds > 65536) {
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(fn),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
    }
#if defined(BSHUF_DIAG) || defined(BSHUF_OCC)
    // occupancy experiment: BSHUF_DIAG_WAVES=w pads the LDS request so that at
    // most w waves fit a CU
    if (const char* w = getenv("BSHUF_DIAG_WAVES")) {
        const size_t want = (size_t)(160 * 1024 / atoi(w)) & ~(size_t)1023;
        if (want > lds) {
            lds = want;
            (void)hipFuncSetAttribute(reinterpret_cast<const void*>(fn),
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        }
    }
#endif
    const int64_t grid = persistent_grid(reinterpret_cast<const void*>(fn), kWave, lds, nb);
    ProfScope prof("k_lz4_encode", s);
    hipLaunchKernelGGL(fn, dim3((unsigned)grid), dim3(kWave), lds, s, a, nb);
    return hipGetLastError();
}

}  // namespace

int64_t max_device_block_bytes() { return 160 * 1024 - kTableBytes - 64; }

namespace {

// Pipelined encode (launch.h): parse segment i on s (enc(f_i, f_i+1)), then on
// the side stream, as soon as it is parsed, the offset scan over blocks
// [0, f_i+1) and the compaction of [f_i, f_i+1) -- overlapping the parse of
// later segments (whose waves raise their issue priority, s_setprio, so the
// compaction takes the issue slots the parse's dependency chain leaves idle).
// The scan (hipcub) needs LDS, which a running parse holds on every CU, so it
// starts as a parse segment drains, and the compaction behind it fills the
// drain: measured on one box (profiles/r04/pipe), 4 GiB G1 compress 11.47 ->
// 11.12 ms with 8 segments, 11.14 with 4; an LDS-free one-wave scan that let
// the compaction run beside the parse body instead gained only 11.47 -> 11.25 /
// 11.38 ms.  The scan of segment i reads foot[f_i+1], which segment i+1 may be
// writing; that element feeds no output of the scan.  foot[nb] = 0 before the
// fork.  The side stream joins s before `finish` runs on s.
template <class Enc, class Fin>
hipError_t encode_pipelined(int64_t nb, hipStream_t s, PipeCtx* pc, const EncodeBufs& b, Enc enc,
                            uint8_t* out, const Seg* segs, const uint32_t* blk_seg,
                            uint64_t* block_offsets, Fin finish) {
    hipError_t e = dev_fill(b.foot + nb, 0, sizeof(uint64_t), s);
    if (e == hipSuccess) e = stream_after(pc->side, s, pc->ev[0]);
    for (int i = 0; i < kPipeSegs && e == hipSuccess; i++) {
        const int64_t f0 = nb * i / kPipeSegs, f1 = nb * (i + 1) / kPipeSegs;
        if (f1 == f0) continue;
        e = enc(f0, f1);
        if (e == hipSuccess) e = stream_after(pc->side, s, pc->ev[1 + i]);
        if (e != hipSuccess) break;
        {
            size_t tmp = b.scan_tmp_bytes;
            // "_side": beside the parse (bench.py keeps these apart from the
            // step's serial kernels)
            ProfScope prof("scan_block_offsets_side", pc->side);
            e = hipcub::DeviceScan::ExclusiveSum(b.scan_tmp, tmp, b.foot, b.offs, (int)(f1 + 1), pc->side);
        }
        if (e != hipSuccess) break;
        ProfScope prof("k_compact_side", pc->side);
        hipLaunchKernelGGL(k_compact, dim3((unsigned)((f1 - f0 + kCompactPerWg - 1) / kCompactPerWg)),
                           dim3(256), 0, pc->side, b.scratch, b.slot, b.offs, out, segs, blk_seg,
                           block_offsets, f0, f1);
        e = hipGetLastError();
    }
    // join even after an error, so nothing of this call is left on the side stream unordered
    const hipError_t j = stream_after(s, pc->side, pc->ev[kPipeEvents - 1]);
    if (e != hipSuccess) return e;
    if (j != hipSuccess) return j;
    return finish(s);
}

}  // namespace

hipError_t launch_encode_big(const uint8_t* shuf, const Layout& L, const EncodeBufs& b, hipStream_t s) {
    if (L.nblocks() == 0) return hipSuccess;
    return lds_atomics_lane_ordered() ? launch_big_t<false>(shuf, L, b, s) : launch_big_t<true>(shuf, L, b, s);
}

int64_t encode_slot_bytes(const Layout& L) {
    const int64_t n = (int64_t)L.bs * L.E;
    // header + bound rounded up to the 256-byte output window (the encoder
    // flushes whole windows) + 16 for k_compact's 5-dword over-read, 16-aligned
    const int64_t payload = ((int64_t)lz4_bound((int)n) + 255) & ~(int64_t)255;
    return (4 + payload + 16 + 15) & ~(int64_t)15;
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
    if (nb > 0 && (int64_t)L.bs * L.E > max_lds_encode_bytes()) {
        e = launch_encode_large(in, L, b, b.shuf, b.tables, s);
        if (e != hipSuccess) return e;
    } else if (nb > 0) {
        const int64_t nmax = (int64_t)L.bs * L.E;
        const bool wide = nmax >= kU16TableLimit;
        // sequence descriptors behind the block when the record fits the
        // table's LDS as staging (every block of up to ~16 KiB)
        const bool desc = !wide && 4 + lz4_bound((int)nmax) + 15 <= kTableBytes;
        const int32_t desc_off = (int32_t)(((nmax + 15) & ~15) + kDataPad);
        EncArgs a{in, b.scratch, b.foot, b.slot, L, desc ? 1 : 0, desc_off, nullptr, nullptr,
                  ((uintptr_t)in & 7) == 0 ? 1 : 0};
        const size_t lds = kTableBytes + (size_t)desc_off + (desc ? kDescBytes : 0);
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
        PipeCtx* pc = (wide == wide_last || !L.last) && nb >= kPipeMinBlocks ? pipe_ctx(s) : nullptr;
        if (pc) return encode_pipelined(nb, s, pc, b, [&](int64_t f0, int64_t f1) {
            return go(L, wide, f1 - f0, f0);
        }, out, nullptr, nullptr, nullptr, [&](hipStream_t st) {
            const uint8_t* tail_src = in + (L.nfull * (int64_t)L.bs + L.last) * L.E;
            ProfScope prof("k_encode_finish", st);
            hipLaunchKernelGGL(k_encode_finish, dim3(1), dim3(64), 0, st, b.offs, nb, tail_src, tail_bytes,
                               out, d_result);
            return hipGetLastError();
        });
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
    e = dev_fill(b.foot + nb, 0, sizeof(uint64_t), s);
    if (e != hipSuccess) return e;
    size_t tmp = b.scan_tmp_bytes;
    {
        ProfScope prof("scan_block_offsets", s);
        e = hipcub::DeviceScan::ExclusiveSum(b.scan_tmp, tmp, b.foot, b.offs, (int)(nb + 1), s);
    }
    if (e != hipSuccess) return e;
    if (nb > 0) {
        ProfScope prof("k_compact", s);
        hipLaunchKernelGGL(k_compact, dim3((unsigned)((nb + kCompactPerWg - 1) / kCompactPerWg)),
                           dim3(256), 0, s, b.scratch, b.slot, b.offs, out, (const Seg*)nullptr,
                           (const uint32_t*)nullptr, (uint64_t*)nullptr, (int64_t)0, nb);
        e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    const uint8_t* tail_src = in + (L.nfull * (int64_t)L.bs + L.last) * L.E;
    ProfScope prof("k_encode_finish", s);
    hipLaunchKernelGGL(k_encode_finish, dim3(1), dim3(64), 0, s, b.offs, nb, tail_src, tail_bytes,
                       out, d_result);
    return hipGetLastError();
}

hipError_t launch_encode_batch(const Seg* segs, const Seg* hsegs, int nsegs, const uint32_t* blk_seg,
                               const Layout& L, const EncodeBufs& b, uint64_t* block_offsets,
                               hipStream_t s) {
    const int64_t nb = L.nfull;  // total blocks of the batch
    hipError_t e;
    if (nb > 0) {
        const int64_t nmax = (int64_t)L.bs * L.E;
        const bool wide = nmax >= kU16TableLimit;
        for (int i = 0; i < nsegs; i++)
            if (hsegs[i].last && ((int64_t)hsegs[i].last * L.E >= kU16TableLimit) != wide)
                return hipErrorInvalidValue;  // mixed table types: the caller splits the batch
        const bool desc = !wide && 4 + lz4_bound((int)nmax) + 15 <= kTableBytes;
        const int32_t desc_off = (int32_t)(((nmax + 15) & ~15) + kDataPad);
        bool raw8 = true;
        for (int i = 0; i < nsegs; i++) raw8 = raw8 && ((uintptr_t)hsegs[i].in & 7) == 0;
        EncArgs a{nullptr, b.scratch, b.foot, b.slot, L, desc ? 1 : 0, desc_off, segs, blk_seg,
                  raw8 ? 1 : 0};
        const size_t lds = kTableBytes + (size_t)desc_off + (desc ? kDescBytes : 0);
        bool aligned = true;
        for (int i = 0; i < nsegs; i++) aligned = aligned && ((uintptr_t)hsegs[i].in & 15) == 0;
        const int ek = aligned && (L.E == 1 || L.E == 2 || L.E == 4 || L.E == 8) ? L.E : 0;
        // blocks [f0, f1) of the batch: the segment table is indexed globally
        // (blk0), scratch slots and sizes relative to f0
        auto go = [&](int64_t f0, int64_t f1) -> hipError_t {
            EncArgs aa = a;
            aa.blk0 = f0;
            aa.scratch = a.scratch + f0 * b.slot;
            aa.foot = a.foot + f0;
            const int64_t cnt = f1 - f0;
#define BSHUF_E(EKV)                                                                  \
    case EKV:                                                                         \
        return wide ? launch_enc_t<EKV, true, 256>(aa, cnt, lds, s)                   \
                    : launch_enc_t<EKV, false, 256>(aa, cnt, lds, s);
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
        PipeCtx* pc = nb >= kPipeMinBlocks ? pipe_ctx(s) : nullptr;
        if (pc) return encode_pipelined(nb, s, pc, b, go, nullptr, segs, blk_seg, block_offsets,
                                        [&](hipStream_t st) {
            ProfScope prof("k_encode_finish", st);
            hipLaunchKernelGGL(k_encode_finish_batch, dim3((unsigned)nsegs), dim3(64), 0, st, b.offs, segs,
                               L.bs, L.E);
            return hipGetLastError();
        });
        e = go(0, nb);
        if (e != hipSuccess) return e;
    }
    e = dev_fill(b.foot + nb, 0, sizeof(uint64_t), s);
    if (e != hipSuccess) return e;
    size_t tmp = b.scan_tmp_bytes;
    {
        ProfScope prof("scan_block_offsets", s);
        e = hipcub::DeviceScan::ExclusiveSum(b.scan_tmp, tmp, b.foot, b.offs, (int)(nb + 1), s);
    }
    if (e != hipSuccess) return e;
    if (nb > 0) {
        ProfScope prof("k_compact", s);
        hipLaunchKernelGGL(k_compact, dim3((unsigned)((nb + kCompactPerWg - 1) / kCompactPerWg)),
                           dim3(256), 0, s, b.scratch, b.slot, b.offs, (uint8_t*)nullptr, segs,
                           blk_seg, block_offsets, (int64_t)0, nb);
        e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    ProfScope prof("k_encode_finish", s);
    hipLaunchKernelGGL(k_encode_finish_batch, dim3((unsigned)nsegs), dim3(64), 0, s, b.offs, segs,
                       L.bs, L.E);
    return hipGetLastError();
}

// map[first .. first + count) = s, one workgroup per segment (blocks or
// index-rebuild chunks).
__global__ void k_seg_map(const Seg* segs, uint32_t* map, int chunks) {
    const Seg& g = segs[blockIdx.x];
    const int64_t first = chunks ? g.chunk0 : g.first;
    const int64_t count = chunks ? g.nchunks : g.nfull + (g.last ? 1 : 0);
    for (int64_t i = threadIdx.x; i < count; i += blockDim.x) map[first + i] = blockIdx.x;
}

hipError_t launch_seg_map(const Seg* segs, int nsegs, uint32_t* map, bool chunks, hipStream_t s) {
    if (nsegs <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_seg_map, dim3((unsigned)nsegs), dim3(256), 0, s, segs, map, chunks ? 1 : 0);
    return hipGetLastError();
}

}  // namespace bshuf

#ifdef BSHUF_DIAG
// Diagnostic build only: read (and reset) the encoder's phase counters.
extern "C" int bshuf_diag_read(unsigned long long* out) {
    static unsigned long long all[bshuf::kDiagCopies * 32];
    if (hipMemcpyFromSymbol(all, HIP_SYMBOL(bshuf::g_diag), sizeof all) != hipSuccess) return -1;
    for (int i = 0; i < 32; i++) {
        out[i] = 0;
        for (int c = 0; c < bshuf::kDiagCopies; c++) out[i] += all[c * 32 + i];
    }
    static const unsigned long long z[bshuf::kDiagCopies * 32] = {0};
    return hipMemcpyToSymbol(HIP_SYMBOL(bshuf::g_diag), z, sizeof z) == hipSuccess ? 0 : -1;
}
#endif
