// launch.h -- host-side launchers for the gfx950 kernels (internal to the .so).
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include <algorithm>

#include "bshuf_dev.h"

namespace bshuf {

// Per-kernel event timing (prof.hip); a no-op unless bshuf_prof_enable(1).
bool prof_on();
class ProfScope {
  public:
    ProfScope(const char* name, hipStream_t s);
    ~ProfScope();

  private:
    const char* name_;
    hipStream_t s_;
    void* a_;
};

// Kernel-variant knob for A/B measurements (bshuf_set_variant, per thread,
// byte-identical variants only); 0 = default.  The kNoPipe bit is not part of
// the variant (pipe_ctx reads it).
int tuning_variant();
#ifdef BSHUF_DIAG
int diag_variant();  // timing ablations (wrong output), diag build only
#endif

// Pipelined encode.  A long encode runs as kPipeSegs launches of the parse
// kernel on the caller's stream, and each segment's offset scan + compaction
// on a per-thread side stream as soon as that segment is parsed, so the
// HBM-bound compaction overlaps the next segment's (LDS- and latency-bound)
// parse.  pipe_ctx(s) returns the calling thread's side stream on
// the current device and its fork / join events, or nullptr: pipelining off
// (bshuf_set_variant bit kNoPipe), `s` being captured into a graph, or no
// side stream.  Every fork is joined back into `s` before the call returns,
// so callers see one stream-ordered operation as before.
constexpr int kPipeSegs = 8;
constexpr int64_t kPipeMinBlocks = 65536;  // shorter calls run unsegmented
constexpr int kPipeEvents = kPipeSegs + 2;  // fork, one per segment, join
constexpr int kNoPipe = 1 << 20;  // no pipelined encode
struct PipeCtx {
    hipStream_t side = nullptr;
    hipEvent_t ev[kPipeEvents] = {};
};
PipeCtx* pipe_ctx(hipStream_t s);
// s waits for everything enqueued on `from` so far (event ev)
hipError_t stream_after(hipStream_t s, hipStream_t from, hipEvent_t ev);

// Workgroups for a persistent launch: resident blocks per CU (occupancy API,
// dynamic LDS included) x CUs of the current device, capped by the work.
int64_t persistent_grid(const void* fn, int threads, size_t lds, int64_t work);
// hipMemsetAsync's job done by a kernel (prof.hip)
hipError_t dev_fill(void* p, int v, size_t n, hipStream_t s);
// Small host table -> device (16-aligned `dev`) on stream s, by a kernel that
// reads a per-thread pinned buffer (host.hip; no DMA engine).  Returns at once;
// the pinned buffer is reused only after that kernel's flags say it was read.
hipError_t stage_upload(const void* host, size_t bytes, void* dev, hipStream_t s);

// One independent framed stream of a batch (bshuf_*_lz4_batch_dev).  All
// streams of a batch share elem_size and block_size; global block k of the
// batch is block k - first of stream blk_seg[k].  The single-stream entry
// points run without a segment table (segs == nullptr).
struct Seg {
    const uint8_t* in;   // encoder: raw input; decoder: framed stream
    uint8_t* out;        // encoder: framed output; decoder: raw output
    int64_t first;       // first global block index
    int64_t nfull;       // full blocks
    int64_t tail;        // raw tail bytes ((size % 8) * elem_size)
    int64_t in_nbytes;   // decoder: readable bytes of the framed stream
    int64_t chunk0;      // decoder: first global index-rebuild chunk
    int64_t nchunks;     // decoder: index-rebuild chunks of this stream
    int64_t seq0;        // decoder: first u32 of this stream's token-position area
    int64_t* result;     // device: bytes written / consumed, or the error code
    int32_t last;        // elements in the partial block (0 = none)
    int32_t pad_;
};

// Fills blk_seg[segs[s].first .. + nblocks(s)) = s for every segment, or with
// chunks = true chunk_seg[segs[s].chunk0 .. + nchunks) = s.
hipError_t launch_seg_map(const Seg* segs, int nsegs, uint32_t* map, bool chunks, hipStream_t s);

// Transpose tiles: 256 groups (2048 elements) per 256-thread workgroup.
constexpr int kTileGroups = 256;

// bitshuffle / bitunshuffle of all full + partial blocks (tail not included).
hipError_t launch_transpose(const uint8_t* in, uint8_t* out, const Layout& L, bool forward,
                            hipStream_t s);

// ---- LZ4 encode --------------------------------------------------------
struct EncodeBufs {
    uint8_t* scratch;   // nblocks * slot bytes: [BE32 c][c payload] per block
    int64_t slot;       // bytes per scratch slot (16-aligned, >= 4 + lz4_bound)
    uint64_t* foot;     // nblocks + 1 u64: 4 + c per block, last = 0
    uint64_t* offs;     // nblocks + 1 u64: exclusive scan of foot
    void* scan_tmp;     // hipcub temp storage
    size_t scan_tmp_bytes;
    uint8_t* shuf = nullptr;     // large blocks: the bit-transposed input
    uint32_t* tables = nullptr;  // large blocks: kLargeTableWords per block
};
size_t encode_scan_tmp_bytes(int64_t nblocks);
int64_t encode_slot_bytes(const Layout& L);
hipError_t launch_encode(const uint8_t* in, uint8_t* out, const Layout& L, int64_t tail_bytes,
                         const EncodeBufs& b, int64_t* d_result, hipStream_t s);
// Batch of independent streams: segs (device) / hsegs (host copy) describe
// them, L carries the shared bs and E and L.nfull = total blocks.  Every
// stream's blocks must use one LZ4 table type (bs * E < 65547, or every
// block at least that long).  block_offsets (optional): per global block, the
// header offset inside its own stream.
hipError_t launch_encode_batch(const Seg* segs, const Seg* hsegs, int nsegs, const uint32_t* blk_seg,
                               const Layout& L, const EncodeBufs& b, uint64_t* block_offsets,
                               hipStream_t s);
// Largest block (bytes) the LDS-resident encoder accepts.
int64_t max_device_block_bytes();
// Blocks above these sizes take the global-memory path (lz4_large.hip).
int64_t max_lds_encode_bytes();
int64_t max_lds_decode_bytes();
constexpr int64_t kLargeTableWords = 8192;
// wave-parallel parse of blocks above max_lds_encode_bytes (lz4_encode.hip):
// shuf holds the bit-transposed blocks (64 bytes of pad behind the last)
hipError_t launch_encode_big(const uint8_t* shuf, const Layout& L, const EncodeBufs& b, hipStream_t s);
hipError_t launch_encode_large(const uint8_t* in, const Layout& L, const EncodeBufs& b,
                               uint8_t* shuf, uint32_t* tables, hipStream_t s);

// ---- LZ4 decode --------------------------------------------------------
struct DecodeBufs {
    uint64_t* offs;     // nblocks u64: header offset of each block
    int64_t* status;    // nblocks i64: consumed bytes or error code per block
    uint32_t* seq;      // token positions of the two-phase decode
    // block index rebuild (unused when offsets are supplied)
    int64_t* exits;     // nchunks
    uint64_t* cnt;      // nchunks + 1
    uint64_t* base;     // nchunks + 1
    int64_t* idx_err;   // 1 word
    long long* bad;     // 1 word: highest failing block index
    void* scan_tmp;
    size_t scan_tmp_bytes;
    int64_t chunk;      // chunk bytes for the index rebuild
    int64_t nchunks;
    uint8_t* shuf = nullptr;  // large blocks: decoded, still bit-transposed
};
int64_t index_chunk_bytes(const Layout& L);
size_t decode_scan_tmp_bytes(int64_t nchunks);
// dlen (optional): the stream length lives in device memory (read by the
// kernels); blocks_end / in_nbytes are then the CAPACITY's, tail the raw tail.
hipError_t launch_index(const uint8_t* in, int64_t blocks_end, const Layout& L,
                        const DecodeBufs& b, hipStream_t s, const int64_t* dlen = nullptr,
                        int64_t cap = 0, int64_t tail = 0);
hipError_t launch_decode(const uint8_t* in, int64_t in_nbytes, uint8_t* out, const Layout& L,
                         int64_t tail_bytes, const DecodeBufs& b, int64_t* d_result,
                         hipStream_t s, const int64_t* dlen = nullptr);
// wave-parallel execution of blocks above max_lds_decode_bytes (lz4_decode.hip)
hipError_t launch_exec_big(const uint8_t* in, const Layout& L, const DecodeBufs& b, uint8_t* shuf,
                           hipStream_t s);
hipError_t launch_decode_large(const uint8_t* in, int64_t in_nbytes, uint8_t* out, const Layout& L,
                               const DecodeBufs& b, uint8_t* shuf, hipStream_t s);
// Batch versions: L.nfull = total blocks; b.idx_err and b.bad hold one word
// per stream; chunk_seg / blk_seg map global chunks / blocks to streams.
hipError_t launch_index_batch(const Seg* segs, int nsegs, const uint32_t* chunk_seg, const Layout& L,
                              int64_t nchunks, const DecodeBufs& b, hipStream_t s);
hipError_t launch_decode_batch(const Seg* segs, const Seg* hsegs, int nsegs, const uint32_t* blk_seg,
                               const Layout& L, const DecodeBufs& b, hipStream_t s,
                               const int64_t* dlens = nullptr);
// device-held batch stream lengths: segs[i].in_nbytes (the capacity) becomes
// the readable bytes of dlens[i]; run before the index rebuild
hipError_t launch_seg_dlen(Seg* segs, const int64_t* dlens, int nsegs, hipStream_t s);

// ---- the reference's internal transpose steps (internals.hip) -------------
// out[(j * lda + i) * es + t] = in[(i * ldb + j) * es + t]  (bshuf_trans_elem)
hipError_t launch_trans_elem(const uint8_t* in, uint8_t* out, int64_t lda, int64_t ldb, int64_t es,
                             hipStream_t s);
// bshuf_shuffle_bit_eightelem_scal of `size` (multiple of 8) E-byte elements
hipError_t launch_shuffle_bit_eightelem(const uint8_t* in, uint8_t* out, int64_t size, int64_t E,
                                        hipStream_t s);

// ---- synthetic inputs ----------------------------------------------------
hipError_t launch_synth(void* out, size_t n, int gen, uint64_t first, uint64_t seed,
                        hipStream_t s);

}  // namespace bshuf
