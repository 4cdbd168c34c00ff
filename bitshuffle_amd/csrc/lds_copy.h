// lds_copy.h -- wave-level LDS byte-movement helpers shared by the LZ4 encoder
// (sequence emission into the record staging buffer) and decoder (literal and
// match execution).  All buffers are LDS (address space 3), 4-aligned bases.
#pragma once

#include "bshuf_dev.h"

namespace bshuf {

// mem[addr] = (mem[addr] & ~mask) | data: a masked dword write in one DS
// instruction (non-returning ds_mskor_b32; data must be zero outside mask).
// Same-address lanes of one instruction are applied one after another, so
// neighbours sharing a dword both land.
__device__ __forceinline__ void lds_write_masked(uint32_t addr, uint32_t mask, uint32_t data) {
    asm volatile("ds_mskor_b32 %0, %1, %2" : : "v"(addr), "v"(mask), "v"(data) : "memory");
}

// The low r bytes of a dword set (r clamped to [0, 4]).
__device__ __forceinline__ uint32_t low_bytes_mask(int r) {
    r = min(r, 4);
    return r <= 0 ? 0u : 0xFFFFFFFFu >> (32 - 8 * r);
}

// The destination half of lane_copy16: x0..x4 are the five source dwords
// around the first source byte, sh its offset in x0.
__device__ __forceinline__ void lane_put16(uint32_t x0, uint32_t x1, uint32_t x2, uint32_t x3,
                                           uint32_t x4, uint32_t sh, lds8* Dd, int dp, int n) {
    const uint32_t u[6] = {0u,
                           __builtin_amdgcn_alignbyte(x1, x0, sh),
                           __builtin_amdgcn_alignbyte(x2, x1, sh),
                           __builtin_amdgcn_alignbyte(x3, x2, sh),
                           __builtin_amdgcn_alignbyte(x4, x3, sh),
                           0u};
    // destination dword j holds source bytes 4j - k .. 4j - k + 3
    const int k = dp & 3, e = k + n;
    const uint32_t sel = 0x03020100u + (uint32_t)(4 - k) * 0x01010101u;
    const uint32_t base = (uint32_t)(uintptr_t)(Dd + (dp & ~3));
#pragma unroll
    for (int j = 0; j < 5; j++) {
        uint32_t m = low_bytes_mask(e - 4 * j);
        if (j == 0) m &= ~low_bytes_mask(k);
        const uint32_t d = __builtin_amdgcn_perm(u[j + 1], u[j], sel) & m;
        lds_write_masked(base + 4u * (uint32_t)j, m, d);
    }
}

// One lane copies n <= 16 bytes (from a buffer with >= 16 readable bytes past
// sp, or whose over-read stays inside LDS and is discarded).  The source's 16
// bytes come from five dword reads and v_alignbyte; the <= 5 destination
// dwords they touch are each written by one masked write (v_perm shifts the
// bytes into place), so there are no per-byte branches.  Every read is issued
// before any write, so a lane may copy from bytes other lanes overwrite.
__device__ __forceinline__ void lane_copy16(const lds8* S, int sp, lds8* Dd, int dp, int n) {
    const lds32* w = (const lds32*)(S + (sp & ~3));
    lane_put16(w[0], w[1], w[2], w[3], w[4], (uint32_t)(sp & 3), Dd, dp, n);
}

// The whole wave copies n bytes whose source ends at or before the
// destination starts, lies in another buffer, or lies AFTER the destination
// (sp > dp: a forward in-place copy, as the in-place decoder's literals).
// Long runs go as aligned destination dwords built from two source dwords,
// edges byte-wise.  The edge bytes are read before the dword loop and written
// after it, and every 64-dword step reads before it writes, so no byte is
// read after something else overwrote it.
__device__ __forceinline__ void wave_copy(const lds8* S, int sp, lds8* Dd, int dp, int n, int lane) {
    if (n <= kWave) {
        if (lane < n) Dd[dp + lane] = S[sp + lane];
        return;
    }
    const int q0 = (dp + 3) & ~3, q1 = (dp + n) & ~3;
    const int head = q0 - dp, tailn = dp + n - q1;
    const int e = lane + (lane < 4 ? 0 : n - tailn - 4);
    const bool edge = (lane < head) | ((lane >= 4) & (lane < 4 + tailn));
    const uint32_t eb = edge ? (uint32_t)S[sp + e] : 0u;
    const int nw = (q1 - q0) >> 2;
    for (int c = lane; c < nw; c += kWave) {
        const int s2 = sp + head + 4 * c;
        const lds32* w = (const lds32*)(S + (s2 & ~3));
        ((lds32*)(Dd + q0))[c] = __builtin_amdgcn_alignbyte(w[1], w[0], (uint32_t)(s2 & 3));
    }
    if (edge) Dd[dp + e] = (uint8_t)eb;
}

// Inclusive prefix sum over the 64 lanes with DPP moves (no LDS round trip):
// row_shr 1/2/4/8 scan each row of 16, row_bcast:15 carries row 0 into row 1
// and row 2 into row 3, row_bcast:31 carries lanes 0-31 into rows 2-3.  Lanes
// whose DPP source is outside the row read the `old` operand, 0.  All lanes
// must be active.
__device__ __forceinline__ int wave_incl_sum(int v, int lane) {
    (void)lane;
    v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xF, 0xF, false);  // row_shr:1
    v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xF, 0xF, false);  // row_shr:2
    v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xF, 0xF, false);  // row_shr:4
    v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xF, 0xF, false);  // row_shr:8
    v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xA, 0xF, false);  // row_bcast:15
    v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xC, 0xF, false);  // row_bcast:31
    return v;
}

// LZ4 length continuation (lz4/lz4.c:1121-1130, 1205-1221): a length field
// value v >= 15 is followed by (v-15)/255 bytes of 255 and one byte (v-15)%255.
__host__ __device__ __forceinline__ int lz4_ext_bytes(int v) { return v >= 15 ? (v - 15) / 255 + 1 : 0; }

// Every lane writes its own continuation run of `cnt` bytes at p (cnt may be
// 0): cnt-1 bytes of 255, then `last`.
__device__ __forceinline__ void lane_len_run(lds8* S, int p, int cnt, uint32_t last) {
    for (int i = 0; __builtin_amdgcn_ballot_w64(i < cnt) != 0; i++)
        if (i < cnt) S[p + i] = (uint8_t)(i + 1 < cnt ? 255u : last);
}

}  // namespace bshuf
