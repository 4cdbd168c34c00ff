/*
 * bshuf_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the bitshuffle + LZ4 hot path, written from the format
 * spec and checked against the reference's golden
 * vectors (tests/golden/) and against oracle/_ref (the reference C compiled
 * from /root/reference by oracle/Makefile).
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load this.  The product (bitshuffle_amd/) never links or calls it.
 *
 * Parity status: PINNED -- bit-exact vs the 42 LZ4 regression chunks of
 * tests/data/regression_{0.1.3,0.4.0}.h5 and vs oracle/_ref on correlated
 * vectors (tests/test_oracle.py).
 */
#ifndef BSHUF_ORACLE_H
#define BSHUF_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* src/bitshuffle_core.c:2038-2046 */
size_t orc_default_block_size(size_t elem_size);

/* Per-block bit transpose (src/bitshuffle_core.c:1835-1870); m % 8 == 0. */
void orc_trans_bit_elem(const uint8_t* in, uint8_t* out, size_t m, size_t elem_size);
void orc_untrans_bit_elem(const uint8_t* in, uint8_t* out, size_t m, size_t elem_size);

/* Blocked drivers (src/bitshuffle_core.c:1877-1931, 2049-2062). */
int64_t orc_bitshuffle(const void* in, void* out, size_t size, size_t elem_size, size_t block_size);
int64_t orc_bitunshuffle(const void* in, void* out, size_t size, size_t elem_size, size_t block_size);

/* LZ4 block codec as bitshuffle invokes it (lz4/lz4.c:1472, 2451). */
int orc_lz4_compress_bound(int n);
int orc_lz4_compress_block(const uint8_t* src, int n, uint8_t* dst);
int orc_lz4_decompress_block(const uint8_t* src, int csize, uint8_t* dst, int capacity);

/* Framed stream (src/bitshuffle.c:36-119, 214-247). */
size_t orc_compress_lz4_bound(size_t size, size_t elem_size, size_t block_size);
int64_t orc_compress_lz4(const void* in, void* out, size_t size, size_t elem_size, size_t block_size);
int64_t orc_decompress_lz4(const void* in, void* out, size_t size, size_t elem_size, size_t block_size);

/* Synthetic inputs of SURVEY.md 8(d) (counter based: element i depends only on i). */
void orc_gen_g0_ramp_i32(int32_t* out, size_t n, size_t first);
void orc_gen_g1_i16(int16_t* out, size_t n, size_t first, uint64_t seed);
void orc_gen_g2_f32(float* out, size_t n, size_t first, uint64_t seed);

#ifdef __cplusplus
}
#endif
#endif
