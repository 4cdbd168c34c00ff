/* TEST INFRASTRUCTURE ONLY -- the drop-in C-ABI of include/bitshuffle.h served
 * by the CPU oracle (oracle/bshuf_oracle.c), so csrc/h5filter.c can be built
 * and run under AddressSanitizer on a machine without a GPU
 * (tests/asan/Makefile, tests/test_asan.py).  It checks the FILTER's buffer
 * handling (12-byte chunk header, output allocation, buffer hand-over), not
 * the codec: the product plugin links libbitshuffle_mi355x.so instead. */
#include "../../include/bitshuffle.h"
#include "../../oracle/bshuf_oracle.h"

size_t bshuf_default_block_size(const size_t elem_size) { return orc_default_block_size(elem_size); }

size_t bshuf_compress_lz4_bound(const size_t size, const size_t elem_size, size_t block_size) {
    return orc_compress_lz4_bound(size, elem_size, block_size);
}

int64_t bshuf_compress_lz4(const void* in, void* out, const size_t size, const size_t elem_size,
                           size_t block_size) {
    return orc_compress_lz4(in, out, size, elem_size, block_size);
}

int64_t bshuf_decompress_lz4(const void* in, void* out, const size_t size, const size_t elem_size,
                             size_t block_size) {
    return orc_decompress_lz4(in, out, size, elem_size, block_size);
}

int64_t bshuf_bitshuffle(const void* in, void* out, const size_t size, const size_t elem_size,
                         const size_t block_size) {
    return orc_bitshuffle(in, out, size, elem_size, block_size);
}

int64_t bshuf_bitunshuffle(const void* in, void* out, const size_t size, const size_t elem_size,
                           const size_t block_size) {
    return orc_bitunshuffle(in, out, size, elem_size, block_size);
}
