/*
 * bitshuffle_internals.h -- the reference's internal transpose entry points
 * that its Cython module links (bitshuffle/ext.pyx:56-86), so the unchanged
 * `bitshuffle.ext` builds and loads against this library.
 *
 * Definitions replaced (reference src/bitshuffle_core.c):
 *   bshuf_copy                          :151-159
 *   bshuf_trans_byte_elem_scal          :194-198   (remainder :163-190)
 *   bshuf_trans_bit_byte_scal           :239-243   (remainder :202-236)
 *   bshuf_trans_bitrow_eight            :264-272   (bshuf_trans_elem :247-260)
 *   bshuf_trans_bit_elem_scal           :276-296
 *   bshuf_trans_byte_bitrow_scal        :301-324
 *   bshuf_shuffle_bit_eightelem_scal    :328-365
 *   bshuf_untrans_bit_elem_scal         :369-387
 *   bshuf_trans_bit_elem / _untrans_    :1835-1870 (ISA dispatch)
 *   *_SSE  stubs :1367-1421 (-11), *_AVX stubs :1643-1674 (-12),
 *   *_NEON stubs :868-921 (-13), *_AVX512 stubs :1807-1831 (-14)
 * Declared in the reference by src/bitshuffle_internals.h:56-66 and ext.pyx.
 *
 * Host pointers, sizes in ELEMENTS, return size*elem_size or a negative code
 * (-80: a size that must be a multiple of 8 is not; -70: no HIP device).
 * Limit (a deviation: the reference's scalar functions have none): the
 * one-block bit transposes -- bshuf_trans_bit_byte_scal, bshuf_trans_bit_elem
 * (_scal), bshuf_untrans_bit_elem(_scal) -- run the whole array as ONE
 * bitshuffle block, so size*elem_size must stay below 2^30 bytes and
 * elem_size at most 65536; larger calls return -71 before touching the
 * device.
 * The scalar and ISA-dispatched variants run on the GPU (no CPU compute path):
 * the bit transposes are one-block calls of the codec's transpose kernels, the
 * byte-level steps small permutation kernels.  The CPU SIMD variants report
 * their ISA as missing, exactly as a reference build without that ISA does.
 */
#ifndef BITSHUFFLE_INTERNALS_H
#define BITSHUFFLE_INTERNALS_H

#include "bitshuffle_core.h"

#ifdef __cplusplus
extern "C" {
#endif

int64_t bshuf_copy(const void* in, void* out, const size_t size, const size_t elem_size);
int64_t bshuf_trans_byte_elem_scal(const void* in, void* out, const size_t size, const size_t elem_size);
int64_t bshuf_trans_bit_byte_scal(const void* in, void* out, const size_t size, const size_t elem_size);
int64_t bshuf_trans_bitrow_eight(const void* in, void* out, const size_t size, const size_t elem_size);
int64_t bshuf_trans_bit_elem_scal(const void* in, void* out, const size_t size, const size_t elem_size);
int64_t bshuf_trans_byte_bitrow_scal(const void* in, void* out, const size_t size, const size_t elem_size);
int64_t bshuf_shuffle_bit_eightelem_scal(const void* in, void* out, const size_t size,
                                         const size_t elem_size);
int64_t bshuf_untrans_bit_elem_scal(const void* in, void* out, const size_t size, const size_t elem_size);
int64_t bshuf_trans_bit_elem(const void* in, void* out, const size_t size, const size_t elem_size);
int64_t bshuf_untrans_bit_elem(const void* in, void* out, const size_t size, const size_t elem_size);

/* CPU SIMD variants: always "ISA missing" here. */
int64_t bshuf_trans_byte_elem_SSE(const void* in, void* out, const size_t size, const size_t elem_size);
int64_t bshuf_trans_bit_byte_SSE(const void* in, void* out, const size_t size, const size_t elem_size);
int64_t bshuf_trans_bit_elem_SSE(const void* in, void* out, const size_t size, const size_t elem_size);
int64_t bshuf_trans_byte_bitrow_SSE(const void* in, void* out, const size_t size, const size_t elem_size);
int64_t bshuf_shuffle_bit_eightelem_SSE(const void* in, void* out, const size_t size, const size_t elem_size);
int64_t bshuf_untrans_bit_elem_SSE(const void* in, void* out, const size_t size, const size_t elem_size);
int64_t bshuf_trans_bit_byte_AVX(const void* in, void* out, const size_t size, const size_t elem_size);
int64_t bshuf_trans_bit_elem_AVX(const void* in, void* out, const size_t size, const size_t elem_size);
int64_t bshuf_trans_byte_bitrow_AVX(const void* in, void* out, const size_t size, const size_t elem_size);
int64_t bshuf_shuffle_bit_eightelem_AVX(const void* in, void* out, const size_t size, const size_t elem_size);
int64_t bshuf_untrans_bit_elem_AVX(const void* in, void* out, const size_t size, const size_t elem_size);
int64_t bshuf_trans_bit_byte_AVX512(const void* in, void* out, const size_t size, const size_t elem_size);
int64_t bshuf_trans_bit_elem_AVX512(const void* in, void* out, const size_t size, const size_t elem_size);
int64_t bshuf_shuffle_bit_eightelem_AVX512(const void* in, void* out, const size_t size,
                                           const size_t elem_size);
int64_t bshuf_untrans_bit_elem_AVX512(const void* in, void* out, const size_t size, const size_t elem_size);
int64_t bshuf_trans_byte_elem_NEON(const void* in, void* out, const size_t size, const size_t elem_size);
int64_t bshuf_trans_bit_byte_NEON(const void* in, void* out, const size_t size, const size_t elem_size);
int64_t bshuf_trans_bit_elem_NEON(const void* in, void* out, const size_t size, const size_t elem_size);
int64_t bshuf_trans_byte_bitrow_NEON(const void* in, void* out, const size_t size, const size_t elem_size);
int64_t bshuf_shuffle_bit_eightelem_NEON(const void* in, void* out, const size_t size,
                                         const size_t elem_size);
int64_t bshuf_untrans_bit_elem_NEON(const void* in, void* out, const size_t size, const size_t elem_size);

#ifdef __cplusplus
}
#endif

#endif /* BITSHUFFLE_INTERNALS_H */
