// api.hip -- the device-resident C-ABI (include/bitshuffle.h,
// include/bitshuffle_core.h): default block size, compress bound, the *_dev
// and *_batch_dev entry points (device pointers, enqueue only).  The
// host-pointer drop-in entry points live in host.hip.  There is no CPU compute
// path: without a usable HIP device every entry point returns -70.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <mutex>
#include <vector>

#include "../../include/bitshuffle.h"
#include "launch.h"
#include "plan.h"

using namespace bshuf;

namespace {

inline size_t al256(size_t x) { return (x + 255) & ~(size_t)255; }

struct Carver {
    uint8_t* base;
    size_t off = 0;
    template <class T>
    T* take(size_t bytes) {
        T* p = reinterpret_cast<T*>(base ? base + off : nullptr);
        off += al256(bytes);
        return p;
    }
};

// ---- workspace layouts -------------------------------------------------------
size_t enc_ws(const Plan& p, EncodeBufs* b, uint8_t* base) {
    Carver c{base};
    const int64_t slot = encode_slot_bytes(p.L);
    EncodeBufs x;
    x.slot = slot;
    x.scratch = c.take<uint8_t>((size_t)(p.nb * slot));
    x.foot = c.take<uint64_t>((size_t)(p.nb + 1) * 8);
    x.offs = c.take<uint64_t>((size_t)(p.nb + 1) * 8);
    x.scan_tmp_bytes = encode_scan_tmp_bytes(p.nb);
    x.scan_tmp = c.take<void>(x.scan_tmp_bytes);
    if ((int64_t)p.L.bs * p.L.E > max_lds_encode_bytes()) {
        // large blocks: bit-transposed copy (+ over-read pad) and LZ4 tables
        x.shuf = c.take<uint8_t>((size_t)(p.L.nfull * (int64_t)p.L.bs + p.L.last) * p.L.E + 64);
        x.tables = c.take<uint32_t>((size_t)p.nb * kLargeTableWords * 4);
    }
    if (b) *b = x;
    return c.off;
}

size_t dec_ws(const Plan& p, int64_t blocks_end, int64_t in_nbytes, bool need_index, DecodeBufs* b,
              uint8_t* base) {
    Carver c{base};
    DecodeBufs x;
    x.chunk = index_chunk_bytes(p.L);
    x.nchunks = blocks_end > 0 ? (blocks_end + x.chunk - 1) / x.chunk : 0;
    x.offs = c.take<uint64_t>((size_t)p.nb * 8 + 8);
    x.status = c.take<int64_t>((size_t)p.nb * 8 + 8);
    // one u32 per 3 stream bytes (a sequence takes >= 3), + a 64-lane prefetch
    x.seq = c.take<uint32_t>(((size_t)in_nbytes / 3 + 80) * 4);
    x.exits = c.take<int64_t>((size_t)x.nchunks * 8 + 8);
    x.cnt = c.take<uint64_t>((size_t)(x.nchunks + 1) * 8);
    x.base = c.take<uint64_t>((size_t)(x.nchunks + 1) * 8);
    x.idx_err = c.take<int64_t>(8);
    x.bad = c.take<long long>(8);
    x.scan_tmp_bytes = need_index ? decode_scan_tmp_bytes(x.nchunks) : 0;
    x.scan_tmp = c.take<void>(x.scan_tmp_bytes + 8);
    if ((int64_t)p.L.bs * p.L.E > max_lds_decode_bytes())
        x.shuf = c.take<uint8_t>((size_t)(p.L.nfull * (int64_t)p.L.bs + p.L.last) * p.L.E + 64);
    if (b) *b = x;
    return c.off;
}

// Workspace of a *_dev call made with ws == NULL: stream-ordered allocation,
// freed stream-ordered when the call returns -- from the library's OWN memory
// pool, whose release threshold keeps freed memory mapped for reuse.  The
// device's default pool (release threshold 0) hands freed blocks back to the
// OS at synchronisation points and maps memory again at the next allocation;
// kernels working in such re-mapped workspaces produced wrong results early in
// a process (round-2 host-path defect, DESIGN.md §4.2: 16 of 40 fresh HDF5
// regression processes with the default pool, 0 of 40 with a pool that never
// trims).  In the diagnostic build only, BSHUF_DIAG_POOL=default brings the
// default pool back for that experiment (tools/h5_repro.sh).  This is a WORKAROUND for re-mapping
// behaviour whose mechanism is not understood, not a proven
// root cause.  What the pool keeps is capped at the largest single workspace
// requested so far (pool_keep): one call's worth stays mapped, not every
// concurrent call's.
std::atomic<uint64_t> g_pool_keep{0};
bool g_pool_is_default = false;  // BSHUF_DIAG_POOL=default: leave its threshold alone
void pool_keep(hipMemPool_t pool, size_t n) {
    if (g_pool_is_default) return;
    uint64_t cur = g_pool_keep.load(std::memory_order_relaxed);
    while (cur < n && !g_pool_keep.compare_exchange_weak(cur, (uint64_t)n, std::memory_order_relaxed)) {
    }
    if (cur < n) {
        uint64_t keep = g_pool_keep.load(std::memory_order_relaxed);
        (void)hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &keep);
    }
}
hipMemPool_t workspace_pool() {
    static hipMemPool_t pool = nullptr;
    static bool tried = false;
    static std::mutex mu;
    std::lock_guard<std::mutex> g(mu);
    if (tried) return pool;
    tried = true;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return nullptr;
#ifdef BSHUF_DIAG
    const char* e = getenv("BSHUF_DIAG_POOL");
#else
    const char* e = nullptr;
#endif
    if (e && !strcmp(e, "default")) {
        (void)hipDeviceGetDefaultMemPool(&pool, dev);
        g_pool_is_default = true;
        return pool;
    }
    hipMemPoolProps props = {};
    props.allocType = hipMemAllocationTypePinned;
    props.handleTypes = hipMemHandleTypeNone;
    props.location.type = hipMemLocationTypeDevice;
    props.location.id = dev;
    if (hipMemPoolCreate(&pool, &props) != hipSuccess) {
        pool = nullptr;
        return nullptr;
    }
    return pool;
}

struct DevBuf {
    void* p = nullptr;
    hipStream_t s = nullptr;
    hipError_t alloc(size_t n, hipStream_t st) {
        s = st;
        hipMemPool_t pool = workspace_pool();
        if (!pool) return hipErrorOutOfMemory;
        pool_keep(pool, n ? n : 1);
        return hipMallocFromPoolAsync(&p, n ? n : 1, pool, st);
    }
    ~DevBuf() {
        if (p) (void)hipFreeAsync(p, s);
    }
};

}  // namespace

extern "C" {

int bshuf_using_SSE2(void) { return 0; }
int bshuf_using_NEON(void) { return 0; }
int bshuf_using_AVX2(void) { return 0; }
int bshuf_using_AVX512(void) { return 0; }
int bshuf_using_HIP(void) { return have_device() ? 1 : 0; }

// src/bitshuffle_core.c:2038-2046 -- format-stable, never change.
size_t bshuf_default_block_size(const size_t elem_size) {
    size_t bs = 8192 / elem_size;
    bs = (bs / kBlockedMult) * kBlockedMult;
    return bs > 128 ? bs : 128;
}

// src/bitshuffle.c:214-233, including its (size_t)-81 quirk.
size_t bshuf_compress_lz4_bound(const size_t size, const size_t elem_size, size_t block_size) {
    if (block_size == 0) block_size = bshuf_default_block_size(elem_size);
    if (block_size % kBlockedMult) return (size_t)-81;
    size_t bound = ((size_t)lz4_bound((int)(block_size * elem_size)) + 4) * (size / block_size);
    size_t leftover = ((size % block_size) / kBlockedMult) * kBlockedMult;
    if (leftover) bound += (size_t)lz4_bound((int)(leftover * elem_size)) + 4;
    bound += (size % kBlockedMult) * elem_size;
    return bound;
}

size_t bshuf_lz4_dev_nblocks(size_t size, size_t elem_size, size_t block_size) {
    Plan p;
    return make_plan(size, elem_size, block_size, p) == 0 ? (size_t)p.nb : 0;
}

// ---------------------------------------------------------------------------
// device-resident entry points
// ---------------------------------------------------------------------------

static int64_t transpose_dev(const void* in, void* out, size_t size, size_t elem_size,
                             size_t block_size, void* stream, bool fwd) {
    Plan p;
    const int64_t r = make_plan(size, elem_size, block_size, p);
    if (r) return r;
    if (!have_device()) return kErrHip;
    hipStream_t s = (hipStream_t)stream;
    const uint8_t* i8 = (const uint8_t*)in;
    uint8_t* o8 = (uint8_t*)out;
    if (launch_transpose(i8, o8, p.L, fwd, s) != hipSuccess) return kErrHip;
    if (p.tail) {
        const int64_t off = (p.L.nfull * (int64_t)p.L.bs + p.L.last) * p.L.E;
        if (hipMemcpyAsync(o8 + off, i8 + off, (size_t)p.tail, hipMemcpyDeviceToDevice, s) !=
            hipSuccess)
            return kErrHip;
    }
    return (int64_t)(size * elem_size);
}

int64_t bshuf_bitshuffle_dev(const void* in, void* out, size_t size, size_t elem_size,
                             size_t block_size, void* stream) {
    return transpose_dev(in, out, size, elem_size, block_size, stream, true);
}

int64_t bshuf_bitunshuffle_dev(const void* in, void* out, size_t size, size_t elem_size,
                               size_t block_size, void* stream) {
    return transpose_dev(in, out, size, elem_size, block_size, stream, false);
}

size_t bshuf_compress_lz4_dev_workspace(size_t size, size_t elem_size, size_t block_size) {
    Plan p;
    if (make_plan(size, elem_size, block_size, p)) return 0;
    return enc_ws(p, nullptr, nullptr);
}

int64_t bshuf_compress_lz4_dev(const void* in, void* out, size_t size, size_t elem_size,
                               size_t block_size, void* ws, size_t ws_bytes, int64_t* d_result,
                               uint64_t* block_offsets, void* stream) {
    Plan p;
    const int64_t r = make_plan(size, elem_size, block_size, p);
    if (r) return r;
    if (!have_device()) return kErrHip;
    hipStream_t s = (hipStream_t)stream;
    const size_t need = enc_ws(p, nullptr, nullptr);
    DevBuf own;
    if (!ws) {
        if (own.alloc(need, s) != hipSuccess) return -1;
        ws = own.p;
    } else if (ws_bytes < need || ((uintptr_t)ws & 255)) {
        return kErrUnsupported;
    }
    EncodeBufs b;
    enc_ws(p, &b, (uint8_t*)ws);
    if (launch_encode((const uint8_t*)in, (uint8_t*)out, p.L, p.tail, b, d_result, s) !=
        hipSuccess)
        return kErrHip;
    if (block_offsets && p.nb &&
        hipMemcpyAsync(block_offsets, b.offs, (size_t)p.nb * 8, hipMemcpyDeviceToDevice, s) !=
            hipSuccess)
        return kErrHip;
    return 0;
}

size_t bshuf_decompress_lz4_dev_workspace(size_t in_nbytes, size_t size, size_t elem_size,
                                          size_t block_size) {
    Plan p;
    if (make_plan(size, elem_size, block_size, p)) return 0;
    const int64_t cb = (int64_t)in_nbytes - p.tail;
    return dec_ws(p, cb > 0 ? cb : 0, (int64_t)in_nbytes, true, nullptr, nullptr);
}

// in_nbytes: the stream's readable bytes -- or, with dlen, the capacity of
// `in`, the length itself being read by the kernels from *dlen
static int64_t decompress_dev(const void* in, size_t in_nbytes, const int64_t* dlen, void* out,
                              size_t size, size_t elem_size, size_t block_size, void* ws,
                              size_t ws_bytes, int64_t* d_result, const uint64_t* block_offsets,
                              void* stream) {
    Plan p;
    const int64_t r = make_plan(size, elem_size, block_size, p);
    if (r) return r;
    if (!have_device()) return kErrHip;
    hipStream_t s = (hipStream_t)stream;
    int64_t cb = (int64_t)in_nbytes - p.tail;
    if (cb < 0) cb = 0;
    const bool need_index = block_offsets == nullptr;
    const size_t need = dec_ws(p, cb, (int64_t)in_nbytes, need_index, nullptr, nullptr);
    DevBuf own;
    if (!ws) {
        if (own.alloc(need, s) != hipSuccess) return -1;
        ws = own.p;
    } else if (ws_bytes < need || ((uintptr_t)ws & 255)) {
        return kErrUnsupported;
    }
    DecodeBufs b;
    dec_ws(p, cb, (int64_t)in_nbytes, need_index, &b, (uint8_t*)ws);
    const uint8_t* i8 = (const uint8_t*)in;
    if (need_index) {
        if (launch_index(i8, cb, p.L, b, s, dlen, (int64_t)in_nbytes, p.tail) != hipSuccess)
            return kErrHip;
    } else {
        b.offs = const_cast<uint64_t*>(block_offsets);
        b.idx_err = nullptr;
    }
    if (launch_decode(i8, (int64_t)in_nbytes, (uint8_t*)out, p.L, p.tail, b, d_result, s, dlen) !=
        hipSuccess)
        return kErrHip;
    return 0;
}

int64_t bshuf_decompress_lz4_dev(const void* in, size_t in_nbytes, void* out, size_t size,
                                 size_t elem_size, size_t block_size, void* ws, size_t ws_bytes,
                                 int64_t* d_result, const uint64_t* block_offsets,
                                 void* stream) {
    return decompress_dev(in, in_nbytes, nullptr, out, size, elem_size, block_size, ws, ws_bytes,
                          d_result, block_offsets, stream);
}

int64_t bshuf_decompress_lz4_dev_dlen(const void* in, const int64_t* d_in_nbytes, size_t in_capacity,
                                      void* out, size_t size, size_t elem_size, size_t block_size,
                                      void* ws, size_t ws_bytes, int64_t* d_result,
                                      const uint64_t* block_offsets, void* stream) {
    if (!d_in_nbytes) return kErrUnsupported;
    return decompress_dev(in, in_capacity, d_in_nbytes, out, size, elem_size, block_size, ws,
                          ws_bytes, d_result, block_offsets, stream);
}

// The block index of a framed stream alone (K6, the decoder's parallel
// header walk): block k's byte offset in `in`, for callers that split one
// stream's decode across devices (bitshuffle_amd/split.py).  *d_status: 0 when
// the records tile the stream exactly, else the index's error word (the
// decoder would return -91); a block the walk could not place holds ~0.
// Replaces the reference's serial header walk (src/iochain.c:42-64 inside
// bshuf_blocked_wrap_fun, src/bitshuffle_core.c:1877-1931) when run alone.
int64_t bshuf_lz4_block_index_dev(const void* in, size_t in_nbytes, size_t size, size_t elem_size,
                                  size_t block_size, void* ws, size_t ws_bytes,
                                  uint64_t* block_offsets, int64_t* d_status, void* stream) {
    Plan p;
    const int64_t r = make_plan(size, elem_size, block_size, p);
    if (r) return r;
    if (!block_offsets || !d_status) return kErrUnsupported;
    if (!have_device()) return kErrHip;
    hipStream_t s = (hipStream_t)stream;
    int64_t cb = (int64_t)in_nbytes - p.tail;
    if (cb < 0) cb = 0;
    const size_t need = dec_ws(p, cb, (int64_t)in_nbytes, true, nullptr, nullptr);
    DevBuf own;
    if (!ws) {
        if (own.alloc(need, s) != hipSuccess) return -1;
        ws = own.p;
    } else if (ws_bytes < need || ((uintptr_t)ws & 255)) {
        return kErrUnsupported;
    }
    DecodeBufs b;
    dec_ws(p, cb, (int64_t)in_nbytes, true, &b, (uint8_t*)ws);
    if (launch_index((const uint8_t*)in, cb, p.L, b, s, nullptr, (int64_t)in_nbytes, p.tail) !=
        hipSuccess)
        return kErrHip;
    if (p.nb && hipMemcpyAsync(block_offsets, b.offs, (size_t)p.nb * 8, hipMemcpyDeviceToDevice, s) !=
                    hipSuccess)
        return kErrHip;
    if (hipMemcpyAsync(d_status, b.idx_err, 8, hipMemcpyDeviceToDevice, s) != hipSuccess)
        return kErrHip;
    return 0;
}

// ---------------------------------------------------------------------------
// batched device entry points: `count` independent streams per launch
// ---------------------------------------------------------------------------

namespace {

struct BatchPlan {
    std::vector<Seg> segs;
    Layout L;        // shared bs, E; L.nfull = total blocks
    int64_t nb = 0;  // total blocks
    int64_t nchunks = 0;
    int64_t seq_words = 0;
    int64_t chunk = 0;
};

// Segment table of a batch (src/bitshuffle_core.c:1877-1931 blocking per
// stream); in_nbytes == nullptr for the encoder.
int64_t make_batch(const void* const* in, void* const* out, const size_t* sizes,
                   const size_t* in_nbytes, size_t count, size_t elem_size, size_t block_size,
                   BatchPlan& bp) {
    if (count == 0 || count > (size_t)INT32_MAX) return kErrUnsupported;
    bp.segs.resize(count);
    for (size_t i = 0; i < count; i++) {
        Plan p;
        const int64_t r = make_plan(sizes[i], elem_size, block_size, p);
        if (r) return r;
        if (i == 0) {
            bp.L = p.L;
            bp.chunk = index_chunk_bytes(p.L);
        }
        Seg& g = bp.segs[i];
        g.in = in ? (const uint8_t*)in[i] : nullptr;
        g.out = out ? (uint8_t*)out[i] : nullptr;
        g.first = bp.nb;
        g.nfull = p.L.nfull;
        g.last = p.L.last;
        g.pad_ = 0;
        g.tail = p.tail;
        g.in_nbytes = in_nbytes ? (int64_t)in_nbytes[i] : 0;
        const int64_t cb = std::max<int64_t>(g.in_nbytes - g.tail, 0);
        g.chunk0 = bp.nchunks;
        g.nchunks = cb > 0 ? (cb + bp.chunk - 1) / bp.chunk : 0;
        g.seq0 = bp.seq_words;
        g.result = nullptr;
        bp.nb += p.nb;
        bp.nchunks += g.nchunks;
        bp.seq_words += g.in_nbytes / 3 + 80;
    }
    bp.L.nfull = bp.nb;
    bp.L.last = 0;
    return 0;
}

size_t enc_batch_ws(const BatchPlan& bp, EncodeBufs* b, Seg** dsegs, uint32_t** blk_seg,
                    uint8_t* base) {
    Carver c{base};
    Seg* sg = c.take<Seg>(bp.segs.size() * sizeof(Seg));
    uint32_t* bm = c.take<uint32_t>((size_t)bp.nb * 4 + 4);
    EncodeBufs x;
    x.slot = encode_slot_bytes(bp.L);
    x.scratch = c.take<uint8_t>((size_t)(bp.nb * x.slot));
    x.foot = c.take<uint64_t>((size_t)(bp.nb + 1) * 8);
    x.offs = c.take<uint64_t>((size_t)(bp.nb + 1) * 8);
    x.scan_tmp_bytes = encode_scan_tmp_bytes(bp.nb);
    x.scan_tmp = c.take<void>(x.scan_tmp_bytes);
    if (b) *b = x;
    if (dsegs) *dsegs = sg;
    if (blk_seg) *blk_seg = bm;
    return c.off;
}

size_t dec_batch_ws(const BatchPlan& bp, DecodeBufs* b, Seg** dsegs, uint32_t** blk_seg,
                    uint32_t** chunk_seg, uint8_t* base) {
    Carver c{base};
    const size_t ns = bp.segs.size();
    Seg* sg = c.take<Seg>(ns * sizeof(Seg));
    uint32_t* bm = c.take<uint32_t>((size_t)bp.nb * 4 + 4);
    uint32_t* cm = c.take<uint32_t>((size_t)bp.nchunks * 4 + 4);
    DecodeBufs x;
    x.chunk = bp.chunk;
    x.nchunks = bp.nchunks;
    x.offs = c.take<uint64_t>((size_t)bp.nb * 8 + 8);
    x.status = c.take<int64_t>((size_t)bp.nb * 8 + 8);
    x.seq = c.take<uint32_t>((size_t)bp.seq_words * 4);
    x.exits = c.take<int64_t>((size_t)bp.nchunks * 8 + 8);
    x.cnt = c.take<uint64_t>((size_t)(bp.nchunks + 1) * 8);
    x.base = c.take<uint64_t>((size_t)(bp.nchunks + 1) * 8);
    x.idx_err = c.take<int64_t>(ns * 8);
    x.bad = c.take<long long>(ns * 8);
    x.scan_tmp_bytes = decode_scan_tmp_bytes(bp.nchunks);
    x.scan_tmp = c.take<void>(x.scan_tmp_bytes + 8);
    if (b) *b = x;
    if (dsegs) *dsegs = sg;
    if (blk_seg) *blk_seg = bm;
    if (chunk_seg) *chunk_seg = cm;
    return c.off;
}

// Caller workspace, or a stream-ordered allocation owned by `own`.
int64_t get_ws(void*& ws, size_t ws_bytes, size_t need, DevBuf& own, hipStream_t s) {
    if (!ws) {
        if (own.alloc(need, s) != hipSuccess) return -1;
        ws = own.p;
    } else if (ws_bytes < need || ((uintptr_t)ws & 255)) {
        return kErrUnsupported;
    }
    return 0;
}

}  // namespace

size_t bshuf_compress_lz4_batch_dev_workspace(const size_t* sizes, size_t count, size_t elem_size,
                                              size_t block_size) {
    BatchPlan bp;
    if (make_batch(nullptr, nullptr, sizes, nullptr, count, elem_size, block_size, bp)) return 0;
    return enc_batch_ws(bp, nullptr, nullptr, nullptr, nullptr);
}

int64_t bshuf_compress_lz4_batch_dev(const void* const* in, void* const* out, const size_t* sizes,
                                     size_t count, size_t elem_size, size_t block_size, void* ws,
                                     size_t ws_bytes, int64_t* d_results, uint64_t* block_offsets,
                                     void* stream) {
    BatchPlan bp;
    const int64_t r = make_batch(in, out, sizes, nullptr, count, elem_size, block_size, bp);
    if (r) return r;
    if (!have_device()) return kErrHip;
    hipStream_t s = (hipStream_t)stream;
    for (size_t i = 0; i < count; i++) bp.segs[i].result = d_results + i;
    // blocks of both LZ4 table types in one batch (a byU32-size block_size
    // with a byU16-size partial block): one stream at a time
    const bool wide = (int64_t)bp.L.bs * bp.L.E >= kU16TableLimit;
    bool mixed = (int64_t)bp.L.bs * bp.L.E > max_lds_encode_bytes();  // large blocks: per stream
    for (const Seg& g : bp.segs) mixed = mixed || (g.last && ((int64_t)g.last * bp.L.E >= kU16TableLimit) != wide);
    if (mixed) {
        for (size_t i = 0; i < count; i++) {
            const int64_t e = bshuf_compress_lz4_dev(in[i], out[i], sizes[i], elem_size, block_size,
                                                     nullptr, 0, d_results + i,
                                                     block_offsets ? block_offsets + bp.segs[i].first : nullptr,
                                                     stream);
            if (e) return e;
        }
        return 0;
    }
    DevBuf own;
    const size_t need = enc_batch_ws(bp, nullptr, nullptr, nullptr, nullptr);
    const int64_t w = get_ws(ws, ws_bytes, need, own, s);
    if (w) return w;
    EncodeBufs b;
    Seg* dsegs = nullptr;
    uint32_t* blk_seg = nullptr;
    enc_batch_ws(bp, &b, &dsegs, &blk_seg, (uint8_t*)ws);
    if (stage_upload(bp.segs.data(), count * sizeof(Seg), dsegs, s) != hipSuccess ||
        launch_seg_map(dsegs, (int)count, blk_seg, false, s) != hipSuccess ||
        launch_encode_batch(dsegs, bp.segs.data(), (int)count, blk_seg, bp.L, b, block_offsets, s) !=
            hipSuccess)
        return kErrHip;
    return 0;
}

size_t bshuf_decompress_lz4_batch_dev_workspace(const size_t* in_nbytes, const size_t* sizes,
                                                size_t count, size_t elem_size, size_t block_size) {
    BatchPlan bp;
    if (make_batch(nullptr, nullptr, sizes, in_nbytes, count, elem_size, block_size, bp)) return 0;
    return dec_batch_ws(bp, nullptr, nullptr, nullptr, nullptr, nullptr);
}

// in_nbytes: per stream, its readable bytes -- or, with dlens (device), the
// capacity of in[i], the length itself being dlens[i]
static int64_t decompress_batch(const void* const* in, const size_t* in_nbytes, const int64_t* dlens,
                                void* const* out, const size_t* sizes, size_t count,
                                size_t elem_size, size_t block_size, void* ws, size_t ws_bytes,
                                int64_t* d_results, void* stream) {
    BatchPlan bp;
    const int64_t r = make_batch(in, out, sizes, in_nbytes, count, elem_size, block_size, bp);
    if (r) return r;
    if (!have_device()) return kErrHip;
    hipStream_t s = (hipStream_t)stream;
    for (size_t i = 0; i < count; i++) bp.segs[i].result = d_results + i;
    if ((int64_t)bp.L.bs * bp.L.E > max_lds_decode_bytes()) {
        // blocks above the LDS decoder's size: one stream at a time
        for (size_t i = 0; i < count; i++) {
            const int64_t e = decompress_dev(in[i], in_nbytes[i], dlens ? dlens + i : nullptr, out[i],
                                             sizes[i], elem_size, block_size, nullptr, 0, d_results + i,
                                             nullptr, stream);
            if (e) return e;
        }
        return 0;
    }
    DevBuf own;
    const size_t need = dec_batch_ws(bp, nullptr, nullptr, nullptr, nullptr, nullptr);
    const int64_t w = get_ws(ws, ws_bytes, need, own, s);
    if (w) return w;
    DecodeBufs b;
    Seg* dsegs = nullptr;
    uint32_t *blk_seg = nullptr, *chunk_seg = nullptr;
    dec_batch_ws(bp, &b, &dsegs, &blk_seg, &chunk_seg, (uint8_t*)ws);
    if (stage_upload(bp.segs.data(), count * sizeof(Seg), dsegs, s) != hipSuccess ||
        (dlens && launch_seg_dlen(dsegs, dlens, (int)count, s) != hipSuccess) ||
        launch_seg_map(dsegs, (int)count, blk_seg, false, s) != hipSuccess ||
        launch_seg_map(dsegs, (int)count, chunk_seg, true, s) != hipSuccess ||
        launch_index_batch(dsegs, (int)count, chunk_seg, bp.L, bp.nchunks, b, s) != hipSuccess ||
        launch_decode_batch(dsegs, bp.segs.data(), (int)count, blk_seg, bp.L, b, s, dlens) != hipSuccess)
        return kErrHip;
    return 0;
}

int64_t bshuf_decompress_lz4_batch_dev(const void* const* in, const size_t* in_nbytes,
                                       void* const* out, const size_t* sizes, size_t count,
                                       size_t elem_size, size_t block_size, void* ws,
                                       size_t ws_bytes, int64_t* d_results, void* stream) {
    return decompress_batch(in, in_nbytes, nullptr, out, sizes, count, elem_size, block_size, ws,
                            ws_bytes, d_results, stream);
}

int64_t bshuf_decompress_lz4_batch_dev_dlen(const void* const* in, const int64_t* d_in_nbytes,
                                            const size_t* in_capacity, void* const* out,
                                            const size_t* sizes, size_t count, size_t elem_size,
                                            size_t block_size, void* ws, size_t ws_bytes,
                                            int64_t* d_results, void* stream) {
    if (!d_in_nbytes) return kErrUnsupported;
    return decompress_batch(in, in_capacity, d_in_nbytes, out, sizes, count, elem_size, block_size,
                            ws, ws_bytes, d_results, stream);
}

int64_t bshuf_synth_fill_dev(void* out, size_t n_elem, int gen, uint64_t first, uint64_t seed,
                             void* stream) {
    if (gen < 0 || gen > 2) return kErrUnsupported;
    if (!have_device()) return kErrHip;
    return launch_synth(out, n_elem, gen, first, seed, (hipStream_t)stream) == hipSuccess
               ? 0
               : kErrHip;
}

}  // extern "C"
