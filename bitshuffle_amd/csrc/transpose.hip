// transpose.hip -- K1/K2: blocked bit transpose (bshuf_bitshuffle /
// bshuf_bitunshuffle, reference src/bitshuffle_core.c:1835-1870, 2049-2062).
//
// Output layout of one block of m elements x E bytes (m % 8 == 0):
//   out[r*(m/8) + g] bit k = bit (r%8) of byte (r/8) of element 8g+k,  r < 8E.
// A plane row only depends on its own 8-element groups, so a block is cut
// into tiles of 256 groups: one 256-thread workgroup per tile, one group per
// thread.  Fast path (E in {1,2,4,8}): each lane loads its group's 8E bytes
// with one/two 16-byte loads (fully coalesced across the wave), does E 8x8
// bit transposes in registers and drops the 8E result bytes into an LDS tile
// [8E planes][256]; the tile then leaves as 16-byte row stores.  The inverse
// runs the same tile backwards.  Any other E takes a byte-granular path.
#include "launch.h"

namespace bshuf {

namespace {

struct TileMap {
    int64_t blk;  // block index
    int m;        // elements in this block
    int g0;       // first group of the tile
    int ng;       // groups in the tile
};

__device__ __forceinline__ TileMap map_tile(const Layout& L, int tiles_per_full) {
    TileMap t;
    const int64_t id = blockIdx.x;
    const int64_t nfull_tiles = L.nfull * tiles_per_full;
    int tt;
    if (id < nfull_tiles) {
        t.blk = id / tiles_per_full;
        tt = (int)(id - t.blk * tiles_per_full);
        t.m = L.bs;
    } else {
        t.blk = L.nfull;
        tt = (int)(id - nfull_tiles);
        t.m = L.last;
    }
    t.g0 = tt * kTileGroups;
    const int P = t.m / 8;
    t.ng = min(kTileGroups, P - t.g0);
    return t;
}

template <int EK>
__global__ __launch_bounds__(256) void k_bitshuffle_fast(const uint8_t* __restrict__ in,
                                                         uint8_t* __restrict__ out, Layout L,
                                                         int tiles_per_full) {
    __shared__ __attribute__((aligned(16))) uint8_t tile[8 * EK * kTileGroups];
    const TileMap tm = map_tile(L, tiles_per_full);
    const int t = threadIdx.x;
    const int P = tm.m / 8;
    const int64_t boff = tm.blk * (int64_t)L.bs * EK;
    const uint8_t* src = in + boff;
    uint8_t* dst = out + boff;
    if (t < tm.ng) {
        uint32_t w[2 * EK];
        load_group<EK>(src + (int64_t)(tm.g0 + t) * 8 * EK, w);
#pragma unroll
        for (int b = 0; b < EK; b++) {
            const uint64_t v = tr8x8(gather_byte_plane<EK>(w, b));
#pragma unroll
            for (int j = 0; j < 8; j++)
                tile[(8 * b + j) * kTileGroups + t] = (uint8_t)(v >> (8 * j));
        }
    }
    __syncthreads();
    const int rows = 8 * EK;
    if ((P & 15) == 0 && (tm.ng & 15) == 0) {
        const int chunks = tm.ng >> 4;
        for (int i = t; i < rows * chunks; i += 256) {
            const int r = i / chunks, c = i - r * chunks;
            *reinterpret_cast<uint4*>(dst + (int64_t)r * P + tm.g0 + 16 * c) =
                *reinterpret_cast<const uint4*>(tile + r * kTileGroups + 16 * c);
        }
    } else {
        for (int i = t; i < rows * tm.ng; i += 256) {
            const int r = i / tm.ng, c = i - r * tm.ng;
            dst[(int64_t)r * P + tm.g0 + c] = tile[r * kTileGroups + c];
        }
    }
}

template <int EK>
__global__ __launch_bounds__(256) void k_bitunshuffle_fast(const uint8_t* __restrict__ in,
                                                           uint8_t* __restrict__ out, Layout L,
                                                           int tiles_per_full) {
    __shared__ __attribute__((aligned(16))) uint8_t tile[8 * EK * kTileGroups];
    const TileMap tm = map_tile(L, tiles_per_full);
    const int t = threadIdx.x;
    const int P = tm.m / 8;
    const int64_t boff = tm.blk * (int64_t)L.bs * EK;
    const uint8_t* src = in + boff;
    uint8_t* dst = out + boff;
    const int rows = 8 * EK;
    if ((P & 15) == 0 && (tm.ng & 15) == 0) {
        const int chunks = tm.ng >> 4;
        for (int i = t; i < rows * chunks; i += 256) {
            const int r = i / chunks, c = i - r * chunks;
            *reinterpret_cast<uint4*>(tile + r * kTileGroups + 16 * c) =
                *reinterpret_cast<const uint4*>(src + (int64_t)r * P + tm.g0 + 16 * c);
        }
    } else {
        for (int i = t; i < rows * tm.ng; i += 256) {
            const int r = i / tm.ng, c = i - r * tm.ng;
            tile[r * kTileGroups + c] = src[(int64_t)r * P + tm.g0 + c];
        }
    }
    __syncthreads();
    if (t < tm.ng) {
        uint32_t w[2 * EK];
#pragma unroll
        for (int i = 0; i < 2 * EK; i++) w[i] = 0;
#pragma unroll
        for (int b = 0; b < EK; b++) {
            uint64_t v = 0;
#pragma unroll
            for (int j = 0; j < 8; j++)
                v |= (uint64_t)tile[(8 * b + j) * kTileGroups + t] << (8 * j);
            scatter_byte_plane<EK>(w, b, tr8x8(v));
        }
        store_group<EK>(dst + (int64_t)(tm.g0 + t) * 8 * EK, w);
    }
}

// Byte-granular path for any element size: one (group, byte) word per item.
__global__ __launch_bounds__(256) void k_transpose_generic(const uint8_t* __restrict__ in,
                                                           uint8_t* __restrict__ out, Layout L,
                                                           int tiles_per_full, int forward) {
    const TileMap tm = map_tile(L, tiles_per_full);
    const int E = L.E;
    const int P = tm.m / 8;
    const int64_t boff = tm.blk * (int64_t)L.bs * E;
    const uint8_t* src = in + boff;
    uint8_t* dst = out + boff;
    for (int i = threadIdx.x; i < tm.ng * E; i += 256) {
        const int g = tm.g0 + i / E, b = i % E;
        uint64_t v = 0;
        if (forward) {
#pragma unroll
            for (int k = 0; k < 8; k++) v |= (uint64_t)src[(int64_t)(8 * g + k) * E + b] << (8 * k);
            v = tr8x8(v);
#pragma unroll
            for (int j = 0; j < 8; j++) dst[(int64_t)(8 * b + j) * P + g] = (uint8_t)(v >> (8 * j));
        } else {
#pragma unroll
            for (int j = 0; j < 8; j++) v |= (uint64_t)src[(int64_t)(8 * b + j) * P + g] << (8 * j);
            v = tr8x8(v);
#pragma unroll
            for (int k = 0; k < 8; k++) dst[(int64_t)(8 * g + k) * E + b] = (uint8_t)(v >> (8 * k));
        }
    }
}

}  // namespace

hipError_t launch_transpose(const uint8_t* in, uint8_t* out, const Layout& L, bool forward,
                            hipStream_t s) {
    const int tpf = (L.bs / 8 + kTileGroups - 1) / kTileGroups;
    const int tpl = (L.last / 8 + kTileGroups - 1) / kTileGroups;
    const int64_t tiles = L.nfull * tpf + tpl;
    if (tiles == 0) return hipSuccess;
    const dim3 grid((unsigned)tiles), block(256);
    ProfScope prof(forward ? "k_bitshuffle" : "k_bitunshuffle", s);
    const bool aligned = (((uintptr_t)in | (uintptr_t)out) & 15) == 0;
    if (aligned && (L.E == 1 || L.E == 2 || L.E == 4 || L.E == 8)) {
#define BSHUF_T(EK)                                                                        \
    case EK:                                                                               \
        if (forward)                                                                       \
            hipLaunchKernelGGL(k_bitshuffle_fast<EK>, grid, block, 0, s, in, out, L, tpf); \
        else                                                                               \
            hipLaunchKernelGGL(k_bitunshuffle_fast<EK>, grid, block, 0, s, in, out, L, tpf); \
        break;
        switch (L.E) {
            BSHUF_T(1)
            BSHUF_T(2)
            BSHUF_T(4)
            BSHUF_T(8)
        }
#undef BSHUF_T
    } else {
        hipLaunchKernelGGL(k_transpose_generic, grid, block, 0, s, in, out, L, tpf,
                           forward ? 1 : 0);
    }
    return hipGetLastError();
}

}  // namespace bshuf
