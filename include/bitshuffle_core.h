/*
 * bitshuffle_core.h -- drop-in C-ABI for the bit-transpose half of the hot path,
 * served by hand-written HIP kernels on MI355X (gfx950).
 *
 * Every symbol below replaces the reference symbol of the same name:
 *   bshuf_using_SSE2/NEON/AVX2/AVX512  src/bitshuffle_core.h:62-92
 *   bshuf_default_block_size           src/bitshuffle_core.h:95-108  (impl src/bitshuffle_core.c:2038-2046)
 *   bshuf_bitshuffle                   src/bitshuffle_core.h:111-134 (impl src/bitshuffle_core.c:2049-2054)
 *   bshuf_bitunshuffle                 src/bitshuffle_core.h:137-162 (impl src/bitshuffle_core.c:2057-2062)
 * Same signatures, same argument meaning (sizes in ELEMENTS, block_size 0 =
 * auto, multiple of 8), same return convention (bytes processed, or a negative
 * error code).  Pointers are HOST pointers; the library stages through device
 * memory internally.  The *_dev variants at the bottom are additive
 * extensions taking DEVICE pointers and a hipStream_t (passed as void*).
 *
 * Error codes (reference src/bitshuffle_core.h:17-26, plus -7x for the device):
 *      -1    : Failed to allocate memory.
 *      -11/-12/-13/-14 : (reference only: missing CPU ISA; never returned here)
 *      -80   : Input size not a multiple of 8.
 *      -81   : block_size not multiple of 8.
 *      -91   : Decompression error, wrong number of bytes processed.
 *      -1YYY : Error internal to the LZ4 stage with error code -YYY.
 *      -70   : No usable HIP device / HIP runtime error (this library never
 *              falls back to a CPU path).
 *      -71   : Argument the device path does not support (e.g. misaligned
 *              device pointer for a *_dev call).
 */
#ifndef BITSHUFFLE_CORE_H
#define BITSHUFFLE_CORE_H

#include <stddef.h>
#include <stdint.h>

#ifndef BSHUF_VERSION_MAJOR
#define BSHUF_VERSION_MAJOR 0
#define BSHUF_VERSION_MINOR 6
#define BSHUF_VERSION_POINT 0
#endif

#ifdef __cplusplus
extern "C" {
#endif

/* CPU ISA probes of the reference.  This library runs no CPU SIMD kernels, so
 * they report 0; bshuf_using_HIP reports whether the gfx950 path is live. */
int bshuf_using_SSE2(void);
int bshuf_using_NEON(void);
int bshuf_using_AVX2(void);
int bshuf_using_AVX512(void);
int bshuf_using_HIP(void);

size_t bshuf_default_block_size(const size_t elem_size);

int64_t bshuf_bitshuffle(const void* in, void* out, const size_t size,
                         const size_t elem_size, size_t block_size);

int64_t bshuf_bitunshuffle(const void* in, void* out, const size_t size,
                           const size_t elem_size, size_t block_size);

/* ---- device-resident extensions (additive, not in the reference) ----
 * in/out are device pointers (hipMalloc / torch CUDA tensors); work is
 * enqueued on `stream` (a hipStream_t, NULL = default stream) and the call
 * returns without synchronising.  Return: size*elem_size or a negative code
 * for argument errors detected on the host. */
int64_t bshuf_bitshuffle_dev(const void* in, void* out, size_t size, size_t elem_size,
                             size_t block_size, void* stream);
int64_t bshuf_bitunshuffle_dev(const void* in, void* out, size_t size, size_t elem_size,
                               size_t block_size, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* BITSHUFFLE_CORE_H */
