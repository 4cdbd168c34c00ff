// internals.hip -- device kernels behind the reference's internal transpose
// steps that its Cython module links (bitshuffle/ext.pyx:56-86; definitions
// src/bitshuffle_core.c:151-387): the generic element transpose
// (bshuf_trans_elem, :247-260) that covers the byte-of-element transpose
// (:163-198), the bit-row transpose (:264-272) and the byte/bit-row transpose
// (:301-324), and the 8-element bit shuffle (:328-365).  The bit transposes
// themselves (trans_bit_byte, trans_bit_elem, untrans_bit_elem) are one-block
// calls of the codec's transpose kernels (host.hip).  These are test and
// profiling hooks of the reference, not the hot path: one thread per output
// byte is plenty.
#include "launch.h"

namespace bshuf {

namespace {

// out[(j * lda + i) * es + t] = in[(i * ldb + j) * es + t]
__global__ __launch_bounds__(256) void k_trans_elem(const uint8_t* __restrict__ in,
                                                    uint8_t* __restrict__ out, int64_t lda,
                                                    int64_t ldb, int64_t es) {
    const int64_t n = lda * ldb * es;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t o = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; o < n; o += stride) {
        const int64_t t = o % es, r = o / es;
        const int64_t i = r % lda, j = r / lda;
        out[o] = in[(i * ldb + j) * es + t];
    }
}

// Per 8-element group g (8E bytes) and byte pair-row b < E: the 8 bytes at
// 8b are bit-transposed (TRANS_BIT_8X8) and byte k lands at b + k E.
__global__ __launch_bounds__(256) void k_shuffle_bit_eightelem(const uint8_t* __restrict__ in,
                                                               uint8_t* __restrict__ out,
                                                               int64_t groups, int64_t E) {
    const int64_t n = groups * E;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t w = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; w < n; w += stride) {
        const int64_t g = w / E, b = w % E;
        const uint8_t* src = in + g * 8 * E + 8 * b;
        uint64_t x = 0;
#pragma unroll
        for (int k = 0; k < 8; k++) x |= (uint64_t)src[k] << (8 * k);
        x = tr8x8(x);
        uint8_t* dst = out + g * 8 * E + b;
#pragma unroll
        for (int k = 0; k < 8; k++) dst[k * E] = (uint8_t)(x >> (8 * k));
    }
}

unsigned grid_for(int64_t n) { return (unsigned)std::max<int64_t>(1, std::min<int64_t>(4096, (n + 255) / 256)); }

}  // namespace

hipError_t launch_trans_elem(const uint8_t* in, uint8_t* out, int64_t lda, int64_t ldb, int64_t es,
                             hipStream_t s) {
    const int64_t n = lda * ldb * es;
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_trans_elem, dim3(grid_for(n)), dim3(256), 0, s, in, out, lda, ldb, es);
    return hipGetLastError();
}

hipError_t launch_shuffle_bit_eightelem(const uint8_t* in, uint8_t* out, int64_t size, int64_t E,
                                        hipStream_t s) {
    const int64_t groups = size / 8;
    if (groups <= 0 || E <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_shuffle_bit_eightelem, dim3(grid_for(groups * E)), dim3(256), 0, s, in, out,
                       groups, E);
    return hipGetLastError();
}

}  // namespace bshuf
