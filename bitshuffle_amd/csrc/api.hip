// api.hip -- the drop-in C-ABI (include/bitshuffle.h, include/bitshuffle_core.h).
//
// Host-pointer entry points keep the reference's contract exactly
// (src/bitshuffle_core.c:2038-2062, src/bitshuffle.c:214-247): they stage the
// buffers through device memory on a per-thread HIP stream and run the gfx950
// kernels.  There is no CPU compute path: without a usable HIP device every
// entry point returns -70.  The *_dev entry points take device pointers and
// only enqueue work.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "../../include/bitshuffle.h"
#include "launch.h"

using namespace bshuf;

namespace {

constexpr int64_t kErrHip = -70;
constexpr int64_t kErrUnsupported = -71;

struct Plan {
    Layout L;
    int64_t tail;  // raw tail bytes
    int64_t nb;    // nblocks
};

// Blocking of src/bitshuffle_core.c:1877-1931.
int64_t make_plan(size_t size, size_t elem_size, size_t block_size, Plan& p) {
    if (elem_size == 0) return kErrUnsupported;
    if (block_size == 0) block_size = bshuf_default_block_size(elem_size);
    if (block_size % kBlockedMult) return -81;
    if (block_size * elem_size > (size_t)INT32_MAX / 2 || elem_size > 65536) return kErrUnsupported;
    p.L.bs = (int32_t)block_size;
    p.L.E = (int32_t)elem_size;
    p.L.nfull = (int64_t)(size / block_size);
    size_t last = size % block_size;
    last -= last % kBlockedMult;
    p.L.last = (int32_t)last;
    p.tail = (int64_t)((size % kBlockedMult) * elem_size);
    p.nb = p.L.nblocks();
    return 0;
}

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

bool have_device() {
    static int n = -1;
    if (n < 0) {
        int c = 0;
        n = (hipGetDeviceCount(&c) == hipSuccess) ? c : 0;
    }
    return n > 0;
}

hipStream_t thread_stream() {
    thread_local hipStream_t s = nullptr;
    if (!s && hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) s = nullptr;
    return s;
}

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

struct DevBuf {
    void* p = nullptr;
    hipStream_t s = nullptr;
    hipError_t alloc(size_t n, hipStream_t st) {
        s = st;
        return hipMallocAsync(&p, n ? n : 1, st);
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

int64_t bshuf_decompress_lz4_dev(const void* in, size_t in_nbytes, void* out, size_t size,
                                 size_t elem_size, size_t block_size, void* ws, size_t ws_bytes,
                                 int64_t* d_result, const uint64_t* block_offsets,
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
        if (launch_index(i8, cb, p.L, b, s) != hipSuccess) return kErrHip;
    } else {
        b.offs = const_cast<uint64_t*>(block_offsets);
        b.idx_err = nullptr;
    }
    if (launch_decode(i8, (int64_t)in_nbytes, (uint8_t*)out, p.L, p.tail, b, d_result, s) !=
        hipSuccess)
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

// Uploads a batch's segment table without blocking the host: the bytes go
// through a per-thread pinned staging buffer, which is reused only after the
// event of its previous copy has completed.
hipError_t upload_table(const void* host, size_t bytes, void* dev, hipStream_t s) {
    struct Stage {
        void* p = nullptr;
        size_t cap = 0;
        hipEvent_t ev = nullptr;
        bool pending = false;
    };
    thread_local Stage st;
    if (st.pending && hipEventSynchronize(st.ev) != hipSuccess) return hipErrorUnknown;
    st.pending = false;
    if (st.cap < bytes) {
        if (st.p) (void)hipHostFree(st.p);
        st.p = nullptr;
        st.cap = 0;
        if (hipHostMalloc(&st.p, bytes, hipHostMallocCoherent) != hipSuccess) return hipErrorOutOfMemory;
        st.cap = bytes;
    }
    if (!st.ev && hipEventCreateWithFlags(&st.ev, hipEventDisableTiming) != hipSuccess)
        return hipErrorUnknown;
    memcpy(st.p, host, bytes);
    hipError_t e = hipMemcpyAsync(dev, st.p, bytes, hipMemcpyHostToDevice, s);
    if (e != hipSuccess) return e;
    e = hipEventRecord(st.ev, s);
    st.pending = e == hipSuccess;
    return e;
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
    if (upload_table(bp.segs.data(), count * sizeof(Seg), dsegs, s) != hipSuccess ||
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

int64_t bshuf_decompress_lz4_batch_dev(const void* const* in, const size_t* in_nbytes,
                                       void* const* out, const size_t* sizes, size_t count,
                                       size_t elem_size, size_t block_size, void* ws,
                                       size_t ws_bytes, int64_t* d_results, void* stream) {
    BatchPlan bp;
    const int64_t r = make_batch(in, out, sizes, in_nbytes, count, elem_size, block_size, bp);
    if (r) return r;
    if (!have_device()) return kErrHip;
    hipStream_t s = (hipStream_t)stream;
    for (size_t i = 0; i < count; i++) bp.segs[i].result = d_results + i;
    if ((int64_t)bp.L.bs * bp.L.E > max_lds_decode_bytes()) {
        // blocks above the LDS decoder's size: one stream at a time
        for (size_t i = 0; i < count; i++) {
            const int64_t e = bshuf_decompress_lz4_dev(in[i], in_nbytes[i], out[i], sizes[i], elem_size,
                                                       block_size, nullptr, 0, d_results + i, nullptr,
                                                       stream);
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
    if (upload_table(bp.segs.data(), count * sizeof(Seg), dsegs, s) != hipSuccess ||
        launch_seg_map(dsegs, (int)count, blk_seg, false, s) != hipSuccess ||
        launch_seg_map(dsegs, (int)count, chunk_seg, true, s) != hipSuccess ||
        launch_index_batch(dsegs, (int)count, chunk_seg, bp.L, bp.nchunks, b, s) != hipSuccess ||
        launch_decode_batch(dsegs, bp.segs.data(), (int)count, blk_seg, bp.L, b, s) != hipSuccess)
        return kErrHip;
    return 0;
}

int64_t bshuf_synth_fill_dev(void* out, size_t n_elem, int gen, uint64_t first, uint64_t seed,
                             void* stream) {
    if (gen < 0 || gen > 2) return kErrUnsupported;
    if (!have_device()) return kErrHip;
    return launch_synth(out, n_elem, gen, first, seed, (hipStream_t)stream) == hipSuccess
               ? 0
               : kErrHip;
}

// ---------------------------------------------------------------------------
// host-pointer drop-in entry points
// ---------------------------------------------------------------------------

}  // extern "C"

namespace {

// Per-thread state of the host-pointer entry points: one HIP stream and
// grow-only device buffers, so a caller that hands over chunk after chunk (the
// HDF5 filter: one call per chunk) allocates nothing after the first call.
// The buffers live until process exit (freeing device memory from a
// thread-exit destructor could race the HIP runtime's own teardown).
struct HostCtx {
    enum { kIn, kOut, kWs, kOffs, kRes, kN };
    void* buf[kN] = {};
    size_t cap[kN] = {};
    std::vector<uint64_t> offs;
    // pinned double-buffered staging (host memcpy of piece i+1 overlaps the
    // DMA of piece i); created on first use
    void* pin[2] = {};
    hipEvent_t ev[2] = {};
    bool pending[2] = {};
    // completion of each device->host piece: a fresh event per piece from a
    // ring, never one event re-recorded while its previous recording may
    // still be waited on (observed to complete early on the ROCm 7.2 runtime)
    hipEvent_t dev_ring[8] = {};
    unsigned ring_pos = 0;
};

HostCtx& host_ctx() {
    thread_local HostCtx* c = new HostCtx();
    return *c;
}

void* ctx_buf(int i, size_t n, hipStream_t s) {
    HostCtx& c = host_ctx();
    if (n == 0) n = 1;
    if (c.buf[i] && c.cap[i] >= n) return c.buf[i];
    if (c.buf[i]) {
        (void)hipStreamSynchronize(s);
        (void)hipFree(c.buf[i]);
        c.buf[i] = nullptr;
        c.cap[i] = 0;
    }
    const size_t want = std::max(n, c.cap[i] + c.cap[i] / 4);
    if (hipMalloc(&c.buf[i], want) != hipSuccess) {
        c.buf[i] = nullptr;
        return nullptr;
    }
    c.cap[i] = want;
    return c.buf[i];
}

// Host <-> device copies go in pieces through two pinned staging buffers of
// the thread: the host memcpy of one piece overlaps the DMA of the other.
// Copying from a caller's pageable buffer directly makes the runtime pin its
// pages on every call -- for the fresh per-chunk buffers HDF5 hands a filter
// that costs more than the copy itself.  BSHUF_HOST_STAGING=0 copies directly.
constexpr size_t kStagePiece = 4u << 20;

// bit 1: host->device staged (default), bit 2: device->host staged.  The
// staged device->host copy is OFF by default: on the ROCm 7.2 runtime a
// decoded chunk read back through it came out with a ~0.5 MB stale stretch
// in about one call in ten (tools/stage_check3.py, not understood yet); the
// direct copy into the caller's pageable buffer never did.
int staging_mode() {
    static int on = -1;
    if (on < 0) {
        const char* e = getenv("BSHUF_HOST_STAGING");
        on = !e ? 1 : (e[0] == '0' ? 0 : (!strcmp(e, "h2d") ? 1 : (!strcmp(e, "d2h") ? 2 : 3)));
    }
    return on;
}

// Waits for a staging copy: its event, or (BSHUF_STAGE_SYNC=stream) the
// whole stream.
hipError_t wait_ev(hipEvent_t e, hipStream_t s) {
    static int mode = -1;
    if (mode < 0) {
        const char* v = getenv("BSHUF_STAGE_SYNC");
        mode = v && !strcmp(v, "stream") ? 1 : 0;
    }
    return mode ? hipStreamSynchronize(s) : hipEventSynchronize(e);
}

// The staging buffers are COHERENT (fine-grained) pinned memory: the default
// (coarse-grained) kind lets the GPU's device->host writes bypass the CPU
// caches, so a buffer the CPU has just read can be re-read stale after the
// next DMA into it -- observed as silently wrong decompressed pieces.
bool stage_init(HostCtx& c) {
    for (int b = 0; b < 2; b++) {
        if (!c.pin[b] && hipHostMalloc(&c.pin[b], kStagePiece, hipHostMallocCoherent) != hipSuccess) {
            c.pin[b] = nullptr;
            return false;
        }
        if (!c.ev[b] && hipEventCreateWithFlags(&c.ev[b], hipEventDisableTiming) != hipSuccess) {
            c.ev[b] = nullptr;
            return false;
        }
    }
    for (hipEvent_t& e : c.dev_ring)
        if (!e && hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) {
            e = nullptr;
            return false;
        }
    return true;
}

// Appends `n` bytes host -> device at dst (piece by piece; returns at once
// after the last memcpy, the DMA may still run).
// Every XCD's L2 written back to memory and invalidated (a system-scope
// release + acquire per workgroup; 256 workgroups reach all 8 XCDs): after the
// runtime's host->device copies into the reused per-thread buffers and before
// the device->host copy of results, so that neither side of a copy can meet a
// line an L2 kept from an earlier call.
__global__ __launch_bounds__(64) void k_host_release() { __threadfence_system(); }

hipError_t host_visible(hipStream_t s) {
    hipLaunchKernelGGL(k_host_release, dim3(256), dim3(64), 0, s);
    return hipGetLastError();
}

hipError_t h2d(uint8_t* dst, const uint8_t* src, size_t n, hipStream_t s) {
    HostCtx& c = host_ctx();
    if (!(staging_mode() & 1) || !stage_init(c)) return hipMemcpyAsync(dst, src, n, hipMemcpyHostToDevice, s);
    static thread_local int nb = 0;
    for (size_t off = 0; off < n; off += kStagePiece) {
        const size_t len = std::min(kStagePiece, n - off);
        const int b = nb;
        nb ^= 1;
        if (c.pending[b] && wait_ev(c.ev[b], s) != hipSuccess) return hipErrorUnknown;
        memcpy(c.pin[b], src + off, len);
        hipError_t e = hipMemcpyAsync(dst + off, c.pin[b], len, hipMemcpyHostToDevice, s);
        if (e == hipSuccess) e = hipEventRecord(c.ev[b], s);
        if (e != hipSuccess) return e;
        c.pending[b] = true;
    }
    return hipSuccess;
}

// n bytes device -> host, completed on return (the DMA of piece i+1 overlaps
// the host memcpy of piece i).
hipError_t d2h(uint8_t* dst, const uint8_t* src, size_t n, hipStream_t s) {
    HostCtx& c = host_ctx();
    if (!(staging_mode() & 2) || !stage_init(c)) {
        const hipError_t e = hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToHost, s);
        return e == hipSuccess ? hipStreamSynchronize(s) : e;
    }
    for (int b = 0; b < 2; b++)
        if (c.pending[b] && wait_ev(c.ev[b], s) != hipSuccess) return hipErrorUnknown;
    c.pending[0] = c.pending[1] = false;
    const size_t npieces = (n + kStagePiece - 1) / kStagePiece;
    hipEvent_t done[2] = {nullptr, nullptr};
    auto issue = [&](size_t i) -> hipError_t {
        const size_t off = i * kStagePiece, len = std::min(kStagePiece, n - off);
        done[i & 1] = c.dev_ring[c.ring_pos++ % 8];
        hipError_t e = hipMemcpyAsync(c.pin[i & 1], src + off, len, hipMemcpyDeviceToHost, s);
        return e == hipSuccess ? hipEventRecord(done[i & 1], s) : e;
    };
    if (npieces && issue(0) != hipSuccess) return hipErrorUnknown;
    for (size_t i = 0; i < npieces; i++) {
        if (i + 1 < npieces && issue(i + 1) != hipSuccess) return hipErrorUnknown;
        if (wait_ev(done[i & 1], s) != hipSuccess) return hipErrorUnknown;
        const size_t off = i * kStagePiece, len = std::min(kStagePiece, n - off);
        memcpy(dst + off, c.pin[i & 1], len);
    }
    return hipSuccess;
}

}  // namespace

extern "C" {

static int64_t transpose_host(const void* in, void* out, size_t size, size_t elem_size,
                              size_t block_size, bool fwd) {
    Plan p;
    const int64_t r = make_plan(size, elem_size, block_size, p);
    if (r) return r;
    if (!have_device()) return kErrHip;
    const size_t bytes = size * elem_size;
    if (bytes == 0) return 0;
    hipStream_t s = thread_stream();
    void* di = ctx_buf(HostCtx::kIn, bytes, s);
    void* dout = ctx_buf(HostCtx::kOut, bytes, s);
    if (!di || !dout) return -1;
    if (h2d((uint8_t*)di, (const uint8_t*)in, bytes, s) != hipSuccess || host_visible(s) != hipSuccess)
        return kErrHip;
    const int64_t n = transpose_dev(di, dout, size, elem_size, block_size, s, fwd);
    if (n < 0) return n;
    if (host_visible(s) != hipSuccess || d2h((uint8_t*)out, (const uint8_t*)dout, bytes, s) != hipSuccess)
        return kErrHip;
    return n;
}

int64_t bshuf_bitshuffle(const void* in, void* out, const size_t size, const size_t elem_size,
                         size_t block_size) {
    return transpose_host(in, out, size, elem_size, block_size, true);
}

int64_t bshuf_bitunshuffle(const void* in, void* out, const size_t size, const size_t elem_size,
                           size_t block_size) {
    return transpose_host(in, out, size, elem_size, block_size, false);
}

int64_t bshuf_compress_lz4(const void* in, void* out, const size_t size, const size_t elem_size,
                           size_t block_size) {
    Plan p;
    const int64_t r = make_plan(size, elem_size, block_size, p);
    if (r) return r;
    if (!have_device()) return kErrHip;
    const size_t bytes = size * elem_size;
    const size_t bound = bshuf_compress_lz4_bound(size, elem_size, block_size);
    const size_t wsb = bshuf_compress_lz4_dev_workspace(size, elem_size, block_size);
    hipStream_t s = thread_stream();
    void* di = ctx_buf(HostCtx::kIn, bytes, s);
    void* dout = ctx_buf(HostCtx::kOut, bound, s);
    void* ws = ctx_buf(HostCtx::kWs, wsb, s);
    int64_t* dres = (int64_t*)ctx_buf(HostCtx::kRes, 8, s);
    if (!di || !dout || !ws || !dres) return -1;
    if ((bytes && h2d((uint8_t*)di, (const uint8_t*)in, bytes, s) != hipSuccess) ||
        host_visible(s) != hipSuccess)
        return kErrHip;
    const int64_t e = bshuf_compress_lz4_dev(di, dout, size, elem_size, block_size, ws, wsb, dres,
                                             nullptr, s);
    if (e < 0) return e;
    int64_t res = 0;
    if (host_visible(s) != hipSuccess ||
        hipMemcpyAsync(&res, dres, 8, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
        return kErrHip;
    if (res > 0 && (size_t)res <= bound &&
        d2h((uint8_t*)out, (const uint8_t*)dout, (size_t)res, s) != hipSuccess)
        return kErrHip;
    return res;
}

int64_t bshuf_decompress_lz4(const void* in, void* out, const size_t size, const size_t elem_size,
                             size_t block_size) {
    Plan p;
    const int64_t r = make_plan(size, elem_size, block_size, p);
    if (r) return r;
    if (!have_device()) return kErrHip;
    const size_t bytes = size * elem_size;
    hipStream_t s = thread_stream();
    // The stream is at most the compress bound: stage into a buffer of that
    // size while the walk below finds its real length.
    const size_t max_in = bshuf_compress_lz4_bound(size, elem_size, block_size);
    uint8_t* di = (uint8_t*)ctx_buf(HostCtx::kIn, max_in, s);
    void* dout = ctx_buf(HostCtx::kOut, bytes, s);
    uint64_t* doffs = (uint64_t*)ctx_buf(HostCtx::kOffs, (size_t)p.nb * 8, s);
    int64_t* dres = (int64_t*)ctx_buf(HostCtx::kRes, 8, s);
    if (!di || !dout || !doffs || !dres) return -1;
    // Walk the BE32 headers through the host buffer (the reference's own
    // iochain walk, src/bitshuffle.c:92-95) -- this also tells how many bytes
    // of `in` belong to the stream, which the caller does not pass.  Every
    // kStagePiece bytes walked leave for the device at once, so the copy
    // overlaps the rest of the walk.
    // The walk stops at the first implausible header (length 0 or above
    // LZ4_compressBound of its block): that record is staged up to the bound,
    // the blocks behind it keep the all-ones "unresolved" offset, and the
    // device decoder assigns every error code (-1001 / -91 / -1YYY), exactly
    // as bshuf_decompress_lz4_dev does for the same bytes.
    const uint8_t* i8 = (const uint8_t*)in;
    std::vector<uint64_t>& offs = host_ctx().offs;
    offs.assign((size_t)p.nb, ~(uint64_t)0);
    uint64_t pos = 0, issued = 0;
    bool broken = false;
    for (int64_t k = 0; k < p.nb; k++) {
        offs[(size_t)k] = pos;
        const uint8_t* h = i8 + pos;
        const uint32_t len = ((uint32_t)h[0] << 24) | ((uint32_t)h[1] << 16) |
                             ((uint32_t)h[2] << 8) | h[3];
        const uint32_t bound = (uint32_t)lz4_bound((k < p.L.nfull ? p.L.bs : p.L.last) * p.L.E);
        if (len == 0 || len > bound) {
            pos += 4 + (len ? (uint64_t)bound : 0);
            broken = true;
            break;
        }
        pos += 4 + (uint64_t)len;
        if (pos - issued >= kStagePiece) {
            if (h2d(di + issued, i8 + issued, (size_t)(pos - issued), s) != hipSuccess) return kErrHip;
            issued = pos;
        }
    }
    const size_t in_nbytes = (size_t)pos + (broken ? 0 : (size_t)p.tail);
    if (in_nbytes > max_in) return -91;
    if ((in_nbytes > issued && h2d(di + issued, i8 + issued, in_nbytes - issued, s) != hipSuccess) ||
        (p.nb && hipMemcpyAsync(doffs, offs.data(), (size_t)p.nb * 8, hipMemcpyHostToDevice, s) !=
                     hipSuccess) ||
        host_visible(s) != hipSuccess)
        return kErrHip;
    // the thread's cached workspace (no stream-ordered allocation per call)
    const size_t wsb = bshuf_decompress_lz4_dev_workspace(in_nbytes, size, elem_size, block_size);
    void* ws = ctx_buf(HostCtx::kWs, wsb, s);
    if (!ws) return -1;
    const int64_t e = bshuf_decompress_lz4_dev(di, in_nbytes, dout, size, elem_size, block_size,
                                               ws, wsb, dres, doffs, s);
    if (e < 0) return e;
    int64_t res = 0;
    if (host_visible(s) != hipSuccess ||
        hipMemcpyAsync(&res, dres, 8, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
        return kErrHip;
    if (res >= 0 && bytes && d2h((uint8_t*)out, (const uint8_t*)dout, bytes, s) != hipSuccess)
        return kErrHip;
    return res;
}

}  // extern "C"
