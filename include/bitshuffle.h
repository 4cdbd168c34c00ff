/*
 * bitshuffle.h -- drop-in C-ABI for bitshuffle + LZ4 (framed stream), served
 * by hand-written HIP kernels on MI355X (gfx950).
 *
 * Replaces (same names, signatures, argument meaning, return values):
 *   bshuf_compress_lz4_bound   src/bitshuffle.h:58-74  (impl src/bitshuffle.c:214-233)
 *   bshuf_compress_lz4         src/bitshuffle.h:77-98  (impl src/bitshuffle.c:236-240)
 *   bshuf_decompress_lz4       src/bitshuffle.h:101-116 (impl src/bitshuffle.c:243-247)
 * Stream format (bit-exact with the reference): for each block of block_size
 * elements (then one partial block of (size % block_size) & ~7 elements)
 *   u32 big-endian  c   ||  c bytes of LZ4 v1.10.0 block (LZ4_compress_default)
 * of the block's bit-transposed bytes, followed by (size % 8) * elem_size raw
 * bytes.  bshuf_compress_lz4 returns bytes written; bshuf_decompress_lz4
 * returns bytes CONSUMED from `in`.  ZSTD entry points are out of scope.
 */
#ifndef BITSHUFFLE_H
#define BITSHUFFLE_H

#include "bitshuffle_core.h"

#ifdef __cplusplus
extern "C" {
#endif

size_t bshuf_compress_lz4_bound(const size_t size, const size_t elem_size, size_t block_size);

int64_t bshuf_compress_lz4(const void* in, void* out, const size_t size,
                           const size_t elem_size, size_t block_size);

int64_t bshuf_decompress_lz4(const void* in, void* out, const size_t size,
                             const size_t elem_size, size_t block_size);

/* ---- device-resident extensions (additive, not in the reference) ----
 *
 * Workspace: pass ws=NULL to let the library take it from its own device
 * memory pool (stream-ordered allocate/free per call; the pool keeps up to the
 * largest workspace requested so far mapped), or
 * pre-allocate bshuf_*_dev_workspace() bytes of device memory (must be
 * 256-byte aligned) so the call performs no allocation and can be captured
 * into a hipGraph.
 *
 * Results are written to *d_result (a DEVICE int64): bytes written (compress),
 * bytes consumed (decompress), or a negative error code.  The call itself
 * returns 0 once the work is enqueued, or a negative code for host-detected
 * argument errors.  Nothing synchronises.
 *
 * bshuf_decompress_lz4_dev needs `in_nbytes`, the number of readable bytes at
 * `in` (the reference's host API walks headers through the buffer instead;
 * on the device the block index is rebuilt in parallel from the framing and
 * in_nbytes bounds every read).  `block_offsets` (optional, may be NULL) lets
 * a caller that kept the encoder's index skip that rebuild: bshuf_compress_lz4_dev
 * fills it when non-NULL (nblocks u64 entries = byte offset of each block header).
 *
 * bshuf_decompress_lz4_dev_dlen takes the stream length as a DEVICE int64
 * (d_in_nbytes, read by the kernels when they run -- e.g. the d_result word of
 * a bshuf_compress_lz4_dev enqueued before it on the same stream), so a
 * compress -> decompress chain never waits on the host.  Like the reference's
 * bshuf_decompress_lz4 (src/bitshuffle.c:243-247, which is not told the length
 * at all), the host passes no length; in_capacity bounds every read (readable
 * bytes = min(*d_in_nbytes, in_capacity)) and sizes the workspace
 * (bshuf_decompress_lz4_dev_workspace(in_capacity, ...)).  A negative
 * *d_in_nbytes (an upstream error) is written to *d_result unchanged.
 */
size_t bshuf_compress_lz4_dev_workspace(size_t size, size_t elem_size, size_t block_size);
size_t bshuf_decompress_lz4_dev_workspace(size_t in_nbytes, size_t size, size_t elem_size,
                                          size_t block_size);
size_t bshuf_lz4_dev_nblocks(size_t size, size_t elem_size, size_t block_size);

int64_t bshuf_compress_lz4_dev(const void* in, void* out, size_t size, size_t elem_size,
                               size_t block_size, void* ws, size_t ws_bytes,
                               int64_t* d_result, uint64_t* block_offsets, void* stream);

int64_t bshuf_decompress_lz4_dev(const void* in, size_t in_nbytes, void* out, size_t size,
                                 size_t elem_size, size_t block_size, void* ws,
                                 size_t ws_bytes, int64_t* d_result,
                                 const uint64_t* block_offsets, void* stream);
int64_t bshuf_decompress_lz4_dev_dlen(const void* in, const int64_t* d_in_nbytes, size_t in_capacity,
                                      void* out, size_t size, size_t elem_size, size_t block_size,
                                      void* ws, size_t ws_bytes, int64_t* d_result,
                                      const uint64_t* block_offsets, void* stream);

/* The block index of a framed stream alone (the decoder's parallel header walk,
 * replacing the reference's serial iochain walk, src/iochain.c:42-64): block k's
 * byte offset into block_offsets[k] (device, bshuf_lz4_dev_nblocks() entries;
 * ~0 for a block the walk could not place) and into *d_status 0 when the records
 * tile the stream exactly, nonzero otherwise (decoding would return -91).  The
 * workspace is bshuf_decompress_lz4_dev_workspace(in_nbytes, ...) bytes, or NULL
 * (library pool).  For splitting one stream's decode across devices. */
int64_t bshuf_lz4_block_index_dev(const void* in, size_t in_nbytes, size_t size, size_t elem_size,
                                  size_t block_size, void* ws, size_t ws_bytes,
                                  uint64_t* block_offsets, int64_t* d_status, void* stream);

/* ---- batched device entry points (additive) ----
 *
 * `count` independent framed streams per call, all with the same elem_size and
 * block_size, each with its own (device) input, output and size; one launch
 * of each kernel covers every block of every stream (the OpenMP block loop of
 * src/bitshuffle_core.c:1899-1907, widened to many buffers).  in[], out[],
 * sizes[] and in_nbytes[] are HOST arrays of device pointers / sizes;
 * d_results is a DEVICE array of `count` int64: per stream, bytes written
 * (compress) or consumed (decompress), or that stream's negative error code.
 * A corrupt stream never affects the others.  block_offsets (optional,
 * device, one u64 per block of the batch in stream order): each block's
 * header offset inside its own stream.  The per-stream table travels through a
 * per-thread pinned buffer; nothing synchronises the host.
 */
size_t bshuf_compress_lz4_batch_dev_workspace(const size_t* sizes, size_t count, size_t elem_size,
                                              size_t block_size);
int64_t bshuf_compress_lz4_batch_dev(const void* const* in, void* const* out, const size_t* sizes,
                                     size_t count, size_t elem_size, size_t block_size, void* ws,
                                     size_t ws_bytes, int64_t* d_results, uint64_t* block_offsets,
                                     void* stream);
size_t bshuf_decompress_lz4_batch_dev_workspace(const size_t* in_nbytes, const size_t* sizes,
                                                size_t count, size_t elem_size, size_t block_size);
int64_t bshuf_decompress_lz4_batch_dev(const void* const* in, const size_t* in_nbytes,
                                       void* const* out, const size_t* sizes, size_t count,
                                       size_t elem_size, size_t block_size, void* ws,
                                       size_t ws_bytes, int64_t* d_results, void* stream);
/* The same with the stream lengths as a DEVICE array d_in_nbytes[count] (e.g.
 * the d_results of a bshuf_compress_lz4_batch_dev before it on the stream);
 * in_capacity[] (host) bounds each stream's reads and sizes the workspace
 * (bshuf_decompress_lz4_batch_dev_workspace(in_capacity, ...)).  A negative
 * length is written to that stream's result unchanged. */
int64_t bshuf_decompress_lz4_batch_dev_dlen(const void* const* in, const int64_t* d_in_nbytes,
                                            const size_t* in_capacity, void* const* out,
                                            const size_t* sizes, size_t count, size_t elem_size,
                                            size_t block_size, void* ws, size_t ws_bytes,
                                            int64_t* d_results, void* stream);

/* Synthetic benchmark inputs of SURVEY.md 8(d), generated on the device
 * (counter based, identical to the CPU definition): gen 0 = int32 ramp,
 * 1 = int16 correlated noise (G1), 2 = float32 smooth field (G2). */
int64_t bshuf_synth_fill_dev(void* out, size_t n_elem, int gen, uint64_t first,
                             uint64_t seed, void* stream);

/* Per-kernel timing (HIP events on each kernel's launch stream), for
 * benchmarks: enable, run, then collect "name count total_ms" lines.
 * bshuf_prof_collect returns the buffer size needed and resets. */
void bshuf_prof_enable(int on);
/* Times only the kernel of this name (NULL: every kernel). */
void bshuf_prof_only(const char* name);
/* Selects, for the CALLING THREAD only, an alternative kernel variant for A/B
 * measurements: 0 default, 2 inline LZ4 emitter, 4 one-group-per-lane
 * transpose, 8 re-test table lookup by lane 0's returning exchange, decoder
 * record access 16 from global memory with a two-blocks-ahead touch / 32
 * without it / 64 staged in an LDS buffer of its own (default: in place at the
 * end of the block's LDS buffer), 128 insert/read-back search window.  Every
 * accepted variant produces identical bytes; anything else is rejected with -71. */
int bshuf_set_variant(int v);
size_t bshuf_prof_collect(char* buf, size_t len);

/* Host-pointer path internals (additive).  bshuf_host_poison fills every
 * cached device buffer and pinned staging slot of the CALLING thread with
 * `byte`, so a test can start the next host call from poisoned state.
 * bshuf_host_xfer_stats: out2[0] = staged pieces moved by the transfer
 * kernels, out2[1] = pieces whose completion event fired before all of their
 * flag words were set (the host waited for the flags). */
int64_t bshuf_host_poison(int byte);
void bshuf_host_xfer_stats(uint64_t* out2);

#ifdef __cplusplus
}
#endif

#endif /* BITSHUFFLE_H */
