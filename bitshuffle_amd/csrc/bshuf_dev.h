// bshuf_dev.h -- device-side building blocks shared by the gfx950 kernels.
//
// Written for CDNA4 wave64: every "per block" routine below is executed by one
// 64-lane wavefront; wave-uniform state lives in SGPRs (readfirstlane), lane
// parallelism comes from ballots over 64 probe positions / 64 byte lanes.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace bshuf {

constexpr int kWave = 64;

// Reference constants (src/bitshuffle_internals.h:33-35, lz4/lz4.c:242-249, 710).
constexpr int kBlockedMult = 8;
constexpr int kMinMatch = 4;
constexpr int kMfLimit = 12;
constexpr int kLastLiterals = 5;
constexpr int kLz4MinLength = kMfLimit + 1;
constexpr int kU16TableLimit = 65536 + kMfLimit - 1;  // LZ4_64Klimit
constexpr uint32_t kMaxDistance = 65535;

__host__ __device__ inline int lz4_bound(int n) { return n + n / 255 + 16; }

// Layout of one framed stream: nfull blocks of bs elements, then one partial
// block of `last` elements (multiple of 8, may be 0), then `tail` raw bytes.
struct Layout {
    int64_t nfull;   // full blocks
    int32_t bs;      // elements per full block
    int32_t last;    // elements in the partial block (0 = none)
    int32_t E;       // bytes per element
    int64_t nblocks() const { return nfull + (last ? 1 : 0); }
};

__device__ __forceinline__ int wave_lane() { return __lane_id(); }

__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ uint32_t uni(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_readfirstlane((int)v);
}

// the wave64 ballot of a condition straight from its compare (no 0/1
// materialisation and re-compare, as __ballot(int) compiles to)
__device__ __forceinline__ uint64_t ballot(bool p) { return __builtin_amdgcn_ballot_w64(p); }
__device__ __forceinline__ int ffs64(uint64_t m) { return __ffsll((unsigned long long)m) - 1; }
__device__ __forceinline__ int fls64(uint64_t m) { return 63 - __clzll((long long)m); }

// 8x8 bit-matrix transpose of a 64-bit word: out byte j bit k = in byte k bit j.
// Three delta swaps (7, 14, 28); the first two never cross the 32-bit halves.
__host__ __device__ __forceinline__ uint64_t tr8x8(uint64_t x) {
    uint64_t t;
    t = (x ^ (x >> 7)) & 0x00AA00AA00AA00AAull;
    x ^= t ^ (t << 7);
    t = (x ^ (x >> 14)) & 0x0000CCCC0000CCCCull;
    x ^= t ^ (t << 14);
    t = (x ^ (x >> 28)) & 0x00000000F0F0F0F0ull;
    x ^= t ^ (t << 28);
    return x;
}

// Offset of probe k from the start of a search: the skip acceleration of
// lz4/lz4.c:1042-1053 (step 1 for the first 65 probes, then (63+k)>>6) in
// closed form, so all 64 lanes of a window know their probe position at once.
__host__ __device__ __forceinline__ int probe_offset(int k) {
    if (k == 0) return 0;
    const int t = 62 + k;
    const int q = t >> 6, r = t & 63;
    return 1 + 32 * q * (q - 1) + q * (r + 1);
}

// LZ4_hash4 for the byU16 table (hash log 13) on a little-endian read32.
__device__ __forceinline__ uint32_t hash4(uint32_t seq) { return (seq * 2654435761u) >> 19; }

// LZ4_hash5 for the byU32 table (hash log 12) on a little-endian read64.
__device__ __forceinline__ uint32_t hash5(uint64_t seq) {
    return (uint32_t)(((seq << 24) * 889523592379ull) >> 52);
}

// LDS-typed pointers (address space 3): 32-bit offsets, constant parts folded
// into the DS instruction's immediate offset.  Generic pointers to __shared__
// data compile to 64-bit address math plus a conversion per access.
typedef __attribute__((address_space(3))) uint8_t lds8;
typedef __attribute__((address_space(3))) uint16_t lds16;
typedef __attribute__((address_space(3))) uint32_t lds32;
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) u32x4 lds128;
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) u32x2 lds64v;
__device__ __forceinline__ u32x4 vec4(const uint4& v) { return u32x4{v.x, v.y, v.z, v.w}; }

__device__ __forceinline__ lds8* to_lds(void* p) { return (lds8*)(p); }

// Global (address space 1) pointers for loads/stores whose address went
// through integer arithmetic: without the cast they compile to flat_* ops,
// which also count on lgkmcnt and so make every LDS wait drain them.
typedef __attribute__((address_space(1))) const u32x4 gbl128c;
typedef __attribute__((address_space(1))) u32x4 gbl128;
typedef __attribute__((address_space(1))) uint8_t gbl8;
typedef __attribute__((address_space(1))) const u32x2 gbl64c;
typedef __attribute__((address_space(1))) u32x2 gbl64;
typedef __attribute__((address_space(1))) const uint8_t gbl8c;
typedef __attribute__((address_space(1))) const uint32_t gbl32c;
__device__ __forceinline__ const gbl128c* g128_aligned_down(const void* p) {
    return (const gbl128c*)((uintptr_t)p & ~(uintptr_t)15);
}

__device__ __forceinline__ uint32_t lds_rd32(const lds8* D, int p) {
    const lds32* w = (const lds32*)(D + (p & ~3));
    return __builtin_amdgcn_alignbyte(w[1], w[0], (uint32_t)(p & 3));
}

__device__ __forceinline__ uint64_t lds_rd64(const lds8* D, int p) {
    const lds32* w = (const lds32*)(D + (p & ~3));
    const uint32_t s = (uint32_t)(p & 3);
    const uint32_t lo = __builtin_amdgcn_alignbyte(w[1], w[0], s);
    const uint32_t hi = __builtin_amdgcn_alignbyte(w[2], w[1], s);
    return (uint64_t)lo | ((uint64_t)hi << 32);
}

// Unaligned little-endian loads from LDS: two aligned dwords + v_alignbyte.
__device__ __forceinline__ uint32_t lds_rd32(const uint8_t* D, int p) {
    const uint32_t* w = reinterpret_cast<const uint32_t*>(D + (p & ~3));
    return __builtin_amdgcn_alignbyte(w[1], w[0], (uint32_t)(p & 3));
}

__device__ __forceinline__ uint64_t lds_rd64(const uint8_t* D, int p) {
    const uint32_t* w = reinterpret_cast<const uint32_t*>(D + (p & ~3));
    const uint32_t s = (uint32_t)(p & 3);
    const uint32_t lo = __builtin_amdgcn_alignbyte(w[1], w[0], s);
    const uint32_t hi = __builtin_amdgcn_alignbyte(w[2], w[1], s);
    return (uint64_t)lo | ((uint64_t)hi << 32);
}

__device__ __forceinline__ uint32_t be32_load(const uint8_t* p) {
    return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}

// ---------------------------------------------------------------------------
// Bit transpose of one 8-element group, compile-time element size EK.
// Input: the group's 8*EK contiguous bytes as 2*EK dwords (little endian).
// Byte b of element k sits at byte (k*EK + b).
// ---------------------------------------------------------------------------
template <int EK>
__device__ __forceinline__ uint64_t gather_byte_plane(const uint32_t (&w)[2 * EK], int b) {
    uint64_t v = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) {
        const int i = k * EK + b;
        v |= (uint64_t)((w[i >> 2] >> ((i & 3) * 8)) & 0xFFu) << (8 * k);
    }
    return v;
}

template <int EK>
__device__ __forceinline__ void scatter_byte_plane(uint32_t (&w)[2 * EK], int b, uint64_t v) {
#pragma unroll
    for (int k = 0; k < 8; k++) {
        const int i = k * EK + b;
        w[i >> 2] |= (uint32_t)((v >> (8 * k)) & 0xFFu) << ((i & 3) * 8);
    }
}

// Bit-sliced inverse transpose of FOUR consecutive groups (4q .. 4q+3) of a
// block, in place: x[r] holds byte (4q + k) of plane r in its byte k (one LDS
// dword per plane).  The 8x8 bit transposes of all four groups run at once, as
// three swap stages between plane registers (bits of one byte never leave it):
// after them x[8b + i] byte k = byte b of element 8(4q + k) + i, and
// untranspose4_word(x, w) composes output dword w of the 32 * EK contiguous
// bytes of the four groups -- word by word, so a caller can store each 16 bytes
// as they are made and keep only x live (EK = 4: 32 registers, not 96).
template <int EK>
__device__ __forceinline__ void untranspose4_rows(uint32_t (&x)[8 * EK]) {
#pragma unroll
    for (int b = 0; b < EK; b++) {
        uint32_t* y = x + 8 * b;
#pragma unroll
        for (int j = 0; j < 8; j += 2) {  // swap bit 1<->0 blocks of rows j, j+1
            const uint32_t t = ((y[j] >> 1) ^ y[j + 1]) & 0x55555555u;
            y[j + 1] ^= t;
            y[j] ^= t << 1;
        }
#pragma unroll
        for (int j = 0; j < 8; j++) {  // rows j, j+2
            if (j & 2) continue;
            const uint32_t t = ((y[j] >> 2) ^ y[j + 2]) & 0x33333333u;
            y[j + 2] ^= t;
            y[j] ^= t << 2;
        }
#pragma unroll
        for (int j = 0; j < 4; j++) {  // rows j, j+4
            const uint32_t t = ((y[j] >> 4) ^ y[j + 4]) & 0x0F0F0F0Fu;
            y[j + 4] ^= t;
            y[j] ^= t << 4;
        }
    }
}

// output byte o = (8k + i) * EK + b  <-  x[8b + i] byte k: three v_perm_b32
// per word (two gather two bytes each, one joins them); w is a compile-time
// constant in every caller, so the selectors fold
template <int EK>
__device__ __forceinline__ uint32_t untranspose4_word(const uint32_t (&x)[8 * EK], const int w) {
    int r[4], k[4];
#pragma unroll
    for (int t = 0; t < 4; t++) {
        const int o = 4 * w + t;
        const int b = o % EK, e = o / EK;
        k[t] = e >> 3;
        r[t] = 8 * b + (e & 7);
    }
    // perm(S0, S1, sel): selector byte 0-3 takes S1's byte, 4-7 S0's, 12 a zero
    const uint32_t lo = __builtin_amdgcn_perm(x[r[1]], x[r[0]],
                                              (uint32_t)k[0] | ((uint32_t)(4 + k[1]) << 8) | 0x0C0C0000u);
    const uint32_t hi = __builtin_amdgcn_perm(x[r[3]], x[r[2]],
                                              (uint32_t)k[2] | ((uint32_t)(4 + k[3]) << 8) | 0x0C0C0000u);
    return __builtin_amdgcn_perm(hi, lo, 0x05040100u);
}

template <int EK>
__device__ __forceinline__ void load_group(const uint8_t* p, uint32_t (&w)[2 * EK]) {
    if constexpr (EK == 1) {
        const u32x2 v = *(const gbl64c*)p;
        w[0] = v.x;
        w[1] = v.y;
    } else {
#pragma unroll
        for (int i = 0; i < EK / 2; i++) {
            const u32x4 v = *(const gbl128c*)(p + 16 * i);
            w[4 * i + 0] = v.x;
            w[4 * i + 1] = v.y;
            w[4 * i + 2] = v.z;
            w[4 * i + 3] = v.w;
        }
    }
}

// The 8*EK bytes of one group, from 2*EK words.
template <int EK>
__device__ __forceinline__ void store_group(uint8_t* p, const uint32_t (&w)[2 * EK]) {
    if constexpr (EK == 1) {
        *(gbl64*)p = u32x2{w[0], w[1]};
    } else {
#pragma unroll
        for (int i = 0; i < EK / 2; i++)
            *(gbl128*)(p + 16 * i) = u32x4{w[4 * i + 0], w[4 * i + 1], w[4 * i + 2], w[4 * i + 3]};
    }
}

}  // namespace bshuf
