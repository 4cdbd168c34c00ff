// host.hip -- the host-pointer drop-in entry points: bshuf_bitshuffle /
// bshuf_bitunshuffle (src/bitshuffle_core.c:2049-2062) and bshuf_compress_lz4 /
// bshuf_decompress_lz4 (src/bitshuffle.c:236-247), over the device kernels.
//
// Every calling thread owns one HIP stream, grow-only device buffers and two
// pinned staging slots; all of it is released when the thread exits.
//
// Transport.  Bytes cross PCIe ONLY through the two kernels of this file,
// k_xfer<pull> (pinned host slot -> device buffer) and k_xfer<push> (device
// buffer -> pinned host slot).  They access the pinned, fine-grained slot
// memory with system-coherent `sc0 sc1` loads and stores, and every workgroup
// publishes "my part is done" by storing the transfer's sequence number into
// its own flag word of the slot (behind a system-scope release for push).  The
// host reuses a slot, or reads the bytes of a pushed piece, only after it has
// seen EVERY flag word of that piece carry the piece's sequence number -- so no
// result depends on when a HIP event or stream query reports completion.
//
// The DMA engines and the runtime's pinning of pageable caller buffers are not
// used, so completion never rests on a copy engine's event.  (They were not the
// cause of the round-2 stale-result defect -- re-mapped stream-ordered pool
// memory was, DESIGN.md §4.2 -- but the flag protocol makes every host-visible
// byte's completion checkable.)  In the DIAGNOSTIC build only (make diag,
// -DBSHUF_DIAG), BSHUF_HOST_XFER=dma / dma_staged / dma_fenced bring DMA copies
// back for that experiment (tools/h5_repro.sh); the product has one transport.
#include <hip/hip_runtime.h>
#include <sched.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include <algorithm>
#include <atomic>
#include <vector>

#include "../../include/bitshuffle.h"
#include "plan.h"

using namespace bshuf;

namespace {

constexpr size_t kPiece = 8u << 20;   // bytes per staging slot
constexpr int kXferThreads = 256;
constexpr int kXferMaxGrid = 256;     // workgroups per piece = flag words per slot

// ---------------------------------------------------------------------------
// system-coherent global accesses (gfx950 cache policy sc0 sc1: bypass the
// CU's L1 and the XCD's L2 for this access, whatever the page's memory type)
// ---------------------------------------------------------------------------
__device__ __forceinline__ void ld_sys4(const uint8_t* p, int64_t step, u32x4& a, u32x4& b, u32x4& c,
                                        u32x4& d) {
    const uint8_t *p1 = p + step, *p2 = p + 2 * step, *p3 = p + 3 * step;
    asm volatile(
        "global_load_dwordx4 %0, %4, off sc0 sc1\n\t"
        "global_load_dwordx4 %1, %5, off sc0 sc1\n\t"
        "global_load_dwordx4 %2, %6, off sc0 sc1\n\t"
        "global_load_dwordx4 %3, %7, off sc0 sc1\n\t"
        "s_waitcnt vmcnt(0)"
        : "=&v"(a), "=&v"(b), "=&v"(c), "=&v"(d)
        : "v"(p), "v"(p1), "v"(p2), "v"(p3)
        : "memory");
}
__device__ __forceinline__ u32x4 ld_sys1(const uint8_t* p) {
    u32x4 a;
    asm volatile("global_load_dwordx4 %0, %1, off sc0 sc1\n\ts_waitcnt vmcnt(0)" : "=&v"(a) : "v"(p) : "memory");
    return a;
}
__device__ __forceinline__ uint32_t ld_sys_u8(const uint8_t* p) {
    uint32_t a;
    asm volatile("global_load_ubyte %0, %1, off sc0 sc1\n\ts_waitcnt vmcnt(0)" : "=&v"(a) : "v"(p) : "memory");
    return a;
}
__device__ __forceinline__ void st_sys(uint8_t* p, u32x4 v) {
    asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" ::"v"(p), "v"(v) : "memory");
}
__device__ __forceinline__ void st_sys_u8(uint8_t* p, uint32_t v) {
    asm volatile("global_store_byte %0, %1, off sc0 sc1" ::"v"(p), "v"(v) : "memory");
}
__device__ __forceinline__ void st_sys_u32(uint32_t* p, uint32_t v) {
    asm volatile("global_store_dword %0, %1, off sc0 sc1" ::"v"(p), "v"(v) : "memory");
}

struct XferArgs {
    uint8_t* dst;         // 16-aligned
    const uint8_t* src;   // 16-aligned
    int64_t n;
    uint32_t* flags;      // kXferMaxGrid words in pinned host memory (device view)
    uint32_t seq;         // this transfer's number, never 0
};

// kPush = false: src is pinned host memory (sc0 sc1 loads), dst a device buffer.
// kPush = true:  src is a device buffer, dst pinned host memory (sc0 sc1 stores).
template <bool kPush>
__global__ __launch_bounds__(kXferThreads) void k_xfer(XferArgs a) {
    const int64_t nch = a.n >> 4;
    const int64_t stride = (int64_t)gridDim.x * kXferThreads;
    int64_t c = (int64_t)blockIdx.x * kXferThreads + threadIdx.x;
    const gbl128c* s16 = (const gbl128c*)a.src;
    gbl128* d16 = (gbl128*)a.dst;
    for (; c + 3 * stride < nch; c += 4 * stride) {
        u32x4 v0, v1, v2, v3;
        if constexpr (kPush) {
            v0 = s16[c];
            v1 = s16[c + stride];
            v2 = s16[c + 2 * stride];
            v3 = s16[c + 3 * stride];
            st_sys(a.dst + 16 * c, v0);
            st_sys(a.dst + 16 * (c + stride), v1);
            st_sys(a.dst + 16 * (c + 2 * stride), v2);
            st_sys(a.dst + 16 * (c + 3 * stride), v3);
        } else {
            ld_sys4(a.src + 16 * c, 16 * stride, v0, v1, v2, v3);
            d16[c] = v0;
            d16[c + stride] = v1;
            d16[c + 2 * stride] = v2;
            d16[c + 3 * stride] = v3;
        }
    }
    for (; c < nch; c += stride) {
        if constexpr (kPush)
            st_sys(a.dst + 16 * c, s16[c]);
        else
            d16[c] = ld_sys1(a.src + 16 * c);
    }
    if (blockIdx.x == 0 && (int64_t)threadIdx.x < (a.n & 15)) {
        const int64_t i = nch * 16 + threadIdx.x;
        if constexpr (kPush)
            st_sys_u8(a.dst + i, a.src[i]);
        else
            a.dst[i] = (uint8_t)ld_sys_u8(a.src + i);
    }
    // publish: every wave's accesses complete, then one lane per workgroup
    // (behind a system-scope release for the host-bound data) stores the flag
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        if constexpr (kPush) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        st_sys_u32(a.flags + blockIdx.x, a.seq);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
}

#ifdef BSHUF_DIAG
// The round-2 mitigation, kept for the DMA experiment only: a system-scope
// release + acquire per workgroup (256 workgroups, hoping to meet every XCD).
__global__ __launch_bounds__(64) void k_l2_flush_all() { __threadfence_system(); }
#endif

// ---------------------------------------------------------------------------
// per-thread state
// ---------------------------------------------------------------------------
#ifdef BSHUF_DIAG
enum class Xfer { kKernel, kDma, kDmaFenced, kDmaStaged };

Xfer xfer_mode() {
    static int m = -1;
    if (m < 0) {
        const char* e = getenv("BSHUF_HOST_XFER");
        m = 0;
        if (e && !strcmp(e, "dma")) m = 1;
        if (e && !strcmp(e, "dma_fenced")) m = 2;
        if (e && !strcmp(e, "dma_staged")) m = 3;
    }
    return (Xfer)m;
}
#endif  // (the product has the kernel transport only)

std::atomic<uint64_t> g_stat_late{0};    // flags not yet all set when the event said done
std::atomic<uint64_t> g_stat_pieces{0};  // staged pieces moved

struct HostCtx {
    enum { kIn, kOut, kWs, kOffs, kRes, kN };
    hipStream_t s = nullptr;
    void* buf[kN] = {};
    size_t cap[kN] = {};
    std::vector<uint64_t> offs;
    struct Slot {
        uint8_t* host = nullptr;  // pinned, fine-grained
        uint8_t* dev = nullptr;   // its device view
        hipEvent_t ev = nullptr;
        uint32_t seq = 0;
        int nwg = 0;
        bool busy = false;
    };
    Slot slot[2];
    uint32_t* flags_host = nullptr;  // 2 x kXferMaxGrid words
    uint32_t* flags_dev = nullptr;
    int next = 0;
    bool broken = false;  // a transport wait failed: these buffers are abandoned

    ~HostCtx() {
        if (!s) return;
        // the runtime may already be gone at process exit: ignore every error
        (void)hipStreamSynchronize(s);
        for (void*& p : buf)
            if (p) (void)hipFree(p);
        for (Slot& x : slot) {
            if (x.host) (void)hipHostFree(x.host);
            if (x.ev) (void)hipEventDestroy(x.ev);
        }
        if (flags_host) (void)hipHostFree(flags_host);
        (void)hipStreamDestroy(s);
    }

    // forget every handle without releasing it (see host_ctx)
    void abandon() {
        s = nullptr;
        for (int i = 0; i < kN; i++) {
            buf[i] = nullptr;
            cap[i] = 0;
        }
        for (Slot& x : slot) x = Slot{};
        flags_host = flags_dev = nullptr;
        next = 0;
        broken = false;
    }

    bool init() {
        if (s) return true;
        if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) {
            s = nullptr;
            return false;
        }
        const unsigned fl = hipHostMallocCoherent | hipHostMallocMapped;
        void* f = nullptr;
        if (hipHostMalloc(&f, 2 * kXferMaxGrid * sizeof(uint32_t), fl) != hipSuccess) return false;
        flags_host = (uint32_t*)f;
        memset(flags_host, 0, 2 * kXferMaxGrid * sizeof(uint32_t));
        void* fd = nullptr;
        if (hipHostGetDevicePointer(&fd, f, 0) != hipSuccess) return false;
        flags_dev = (uint32_t*)fd;
        for (Slot& x : slot) {
            void* h = nullptr;
            if (hipHostMalloc(&h, kPiece + 64, fl) != hipSuccess) return false;
            x.host = (uint8_t*)h;
            void* d = nullptr;
            if (hipHostGetDevicePointer(&d, h, 0) != hipSuccess) return false;
            x.dev = (uint8_t*)d;
            if (hipEventCreateWithFlags(&x.ev, hipEventDisableTiming) != hipSuccess) return false;
        }
        return true;
    }

    void* dbuf(int i, size_t n) {
        if (n == 0) n = 1;
        if (buf[i] && cap[i] >= n) return buf[i];
        if (buf[i]) {
            (void)hipStreamSynchronize(s);
            (void)hipFree(buf[i]);
            buf[i] = nullptr;
            cap[i] = 0;
        }
        const size_t want = std::max(n, cap[i] + cap[i] / 4);
        if (hipMalloc(&buf[i], want) != hipSuccess) {
            buf[i] = nullptr;
            return nullptr;
        }
        cap[i] = want;
        return buf[i];
    }

    // Waits until every workgroup of the slot's last transfer stored its flag
    // (after the event of the kernel reported completion).
    bool settle(int k) {
        Slot& x = slot[k];
        if (!x.busy) return true;
        if (hipEventSynchronize(x.ev) != hipSuccess) return false;
        volatile uint32_t* f = flags_host + k * kXferMaxGrid;
        auto all_set = [&]() {
            for (int w = 0; w < x.nwg; w++)
                if (f[w] != x.seq) return false;
            return true;
        };
        if (!all_set()) {
            g_stat_late.fetch_add(1, std::memory_order_relaxed);
            const time_t t0 = time(nullptr);
            while (!all_set()) {
                if (time(nullptr) - t0 > 30) {
                    fprintf(stderr, "bitshuffle_mi355x: staging transfer never completed\n");
                    return false;
                }
                sched_yield();
            }
        }
        std::atomic_thread_fence(std::memory_order_acquire);
        x.busy = false;
        return true;
    }

    // Enqueues one piece through slot k (n <= kPiece; both ends 16-aligned).
    bool launch(int k, bool push, uint8_t* dst, const uint8_t* src, size_t n) {
        Slot& x = slot[k];
        x.seq = x.seq + 1 == 0 ? 1 : x.seq + 1;
        const int64_t chunks = (int64_t)(n + 15) / 16;
        x.nwg = (int)std::max<int64_t>(1, std::min<int64_t>(kXferMaxGrid, (chunks + kXferThreads * 4 - 1) /
                                                                             (kXferThreads * 4)));
        XferArgs a{dst, src, (int64_t)n, flags_dev + k * kXferMaxGrid, x.seq};
        if (push)
            hipLaunchKernelGGL(k_xfer<true>, dim3(x.nwg), dim3(kXferThreads), 0, s, a);
        else
            hipLaunchKernelGGL(k_xfer<false>, dim3(x.nwg), dim3(kXferThreads), 0, s, a);
        if (hipGetLastError() != hipSuccess || hipEventRecord(x.ev, s) != hipSuccess) return false;
        x.busy = true;
        g_stat_pieces.fetch_add(1, std::memory_order_relaxed);
        return true;
    }
};

thread_local HostCtx t_ctx;

// After a failed transfer the thread's stream, device buffers and pinned
// slots are abandoned (a lost transfer may still land in them later: they are
// never reused, and leaked rather than freed under it) and the next call
// starts over with fresh ones -- one transient fault does not disable the
// thread's later calls.
HostCtx* host_ctx() {
    if (t_ctx.broken) t_ctx.abandon();
    if (!t_ctx.init()) return nullptr;
    return &t_ctx;
}

#ifdef BSHUF_DIAG
hipError_t dma_fence(HostCtx& c) {
    if (xfer_mode() != Xfer::kDmaFenced) return hipSuccess;
    hipLaunchKernelGGL(k_l2_flush_all, dim3(256), dim3(64), 0, c.s);
    return hipGetLastError();
}

// Round-2 staged DMA transport (diagnostic mode dma_staged): SDMA copies
// between the device buffers and the pinned slots, completion by HIP events.
// After each device->host piece is copied out of its slot, the slot is
// compared with what was copied: a difference means the DMA was still writing
// the slot after its event reported completion (counted as "late").
bool h2d_staged(HostCtx& c, uint8_t* dst, const uint8_t* src, uint64_t lo, uint64_t hi) {
    for (uint64_t off = lo; off < hi; off += kPiece) {
        const size_t len = (size_t)std::min<uint64_t>(kPiece, hi - off);
        const int k = c.next;
        c.next ^= 1;
        HostCtx::Slot& x = c.slot[k];
        if (x.busy && hipEventSynchronize(x.ev) != hipSuccess) return false;
        memcpy(x.host, src + off, len);
        if (hipMemcpyAsync(dst + off, x.host, len, hipMemcpyHostToDevice, c.s) != hipSuccess ||
            hipEventRecord(x.ev, c.s) != hipSuccess)
            return false;
        x.busy = true;
    }
    return true;
}

bool d2h_staged(HostCtx& c, uint8_t* dst, const uint8_t* src, size_t n) {
    for (auto& x : c.slot)
        if (x.busy && hipEventSynchronize(x.ev) != hipSuccess) return false;
    const size_t np = (n + kPiece - 1) / kPiece;
    auto issue = [&](size_t i) {
        const size_t off = i * kPiece, len = std::min(kPiece, n - off);
        HostCtx::Slot& x = c.slot[i & 1];
        x.busy = true;
        return hipMemcpyAsync(x.host, src + off, len, hipMemcpyDeviceToHost, c.s) == hipSuccess &&
               hipEventRecord(x.ev, c.s) == hipSuccess;
    };
    if (!issue(0)) return false;
    for (size_t i = 0; i < np; i++) {
        if (i + 1 < np && !issue(i + 1)) return false;
        HostCtx::Slot& x = c.slot[i & 1];
        if (hipEventSynchronize(x.ev) != hipSuccess) return false;
        x.busy = false;
        const size_t off = i * kPiece, len = std::min(kPiece, n - off);
        memcpy(dst + off, x.host, len);
        if (memcmp(dst + off, x.host, len) != 0) g_stat_late.fetch_add(1, std::memory_order_relaxed);
    }
    return true;
}
#endif  // BSHUF_DIAG

// Host bytes [lo, hi) of `src` to the device buffer `dst` (same offsets).
// Returns once the last piece is enqueued; its slot is released later.
bool h2d(HostCtx& c, uint8_t* dst, const uint8_t* src, uint64_t lo, uint64_t hi) {
    if (hi <= lo) return true;
#ifdef BSHUF_DIAG
    if (xfer_mode() == Xfer::kDmaStaged) return h2d_staged(c, dst, src, lo, hi);
    if (xfer_mode() != Xfer::kKernel) {
        const bool ok = hipMemcpyAsync(dst + lo, src + lo, hi - lo, hipMemcpyHostToDevice, c.s) == hipSuccess;
        return ok && dma_fence(c) == hipSuccess;
    }
#endif
    lo &= ~(uint64_t)15;  // re-sending bytes already sent is harmless; keeps both ends aligned
    for (uint64_t off = lo; off < hi; off += kPiece) {
        const size_t len = (size_t)std::min<uint64_t>(kPiece, hi - off);
        const int k = c.next;
        c.next ^= 1;
        if (!c.settle(k)) return false;
        memcpy(c.slot[k].host, src + off, len);
        if (!c.launch(k, false, dst + off, c.slot[k].dev, len)) return false;
    }
    return true;
}

// n device bytes at `src` (16-aligned) to host `dst`; complete on return.
bool d2h(HostCtx& c, uint8_t* dst, const uint8_t* src, size_t n) {
    if (n == 0) return true;
#ifdef BSHUF_DIAG
    if (xfer_mode() == Xfer::kDmaStaged) return d2h_staged(c, dst, src, n);
    if (xfer_mode() != Xfer::kKernel) {
        if (dma_fence(c) != hipSuccess) return false;
        return hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToHost, c.s) == hipSuccess &&
               hipStreamSynchronize(c.s) == hipSuccess;
    }
#endif
    if (!c.settle(0) || !c.settle(1)) return false;
    const size_t np = (n + kPiece - 1) / kPiece;
    auto issue = [&](size_t i) {
        const size_t off = i * kPiece, len = std::min(kPiece, n - off);
        return c.launch((int)(i & 1), true, c.slot[i & 1].dev, src + off, len);
    };
    if (!issue(0)) return false;
    for (size_t i = 0; i < np; i++) {
        if (i + 1 < np && !issue(i + 1)) return false;
        if (!c.settle((int)(i & 1))) return false;
        const size_t off = i * kPiece, len = std::min(kPiece, n - off);
        memcpy(dst + off, c.slot[i & 1].host, len);
    }
    return true;
}

// The 8-byte device result word of the stream's last kernel.
bool read_result(HostCtx& c, const int64_t* dres, int64_t& res) {
#ifdef BSHUF_DIAG
    if (xfer_mode() != Xfer::kKernel) {
        if (dma_fence(c) != hipSuccess) return false;
        return hipMemcpyAsync(&res, dres, 8, hipMemcpyDeviceToHost, c.s) == hipSuccess &&
               hipStreamSynchronize(c.s) == hipSuccess;
    }
#endif
    return d2h(c, (uint8_t*)&res, (const uint8_t*)dres, 8);
}

// Stale-result experiment only, diagnostic build (BSHUF_DIAG_WS=alloc): the
// round-2 host path's per-call stream-ordered workspace (api.hip's DevBuf)
// instead of the thread's cached one; with BSHUF_DIAG_POOL=default it comes
// from the default pool.
bool diag_alloc_ws() {
#ifdef BSHUF_DIAG
    static const bool on = getenv("BSHUF_DIAG_WS") != nullptr;
    return on;
#else
    return false;
#endif
}

int64_t fail(HostCtx& c) {
    c.broken = true;  // a lost transfer may still land later: never reuse these buffers
    return kErrHip;
}

int64_t transpose_host(const void* in, void* out, size_t size, size_t elem_size, size_t block_size,
                       bool fwd) {
    Plan p;
    const int64_t r = make_plan(size, elem_size, block_size, p);
    if (r) return r;
    if (!have_device()) return kErrHip;
    const size_t bytes = size * elem_size;
    if (bytes == 0) return 0;
    HostCtx* c = host_ctx();
    if (!c) return kErrHip;
    uint8_t* di = (uint8_t*)c->dbuf(HostCtx::kIn, bytes);
    uint8_t* dout = (uint8_t*)c->dbuf(HostCtx::kOut, bytes);
    if (!di || !dout) return -1;
    if (!h2d(*c, di, (const uint8_t*)in, 0, bytes)) return fail(*c);
    const int64_t n = fwd ? bshuf_bitshuffle_dev(di, dout, size, elem_size, block_size, c->s)
                          : bshuf_bitunshuffle_dev(di, dout, size, elem_size, block_size, c->s);
    if (n < 0) return n;
    if (!d2h(*c, (uint8_t*)out, dout, bytes)) return fail(*c);
    return n;
}

// Per-thread pinned buffers of stage_upload (the batch segment tables), as a
// ring: a buffer is reused only once the upload kernel that read it has stored
// its flag word, so a batch call never waits for an earlier call's kernel while
// a free buffer exists (bitshuffle.h: nothing synchronises the host).  With
// kTableRing uploads still queued, the oldest one's event is waited on -- with
// no time limit, however much work is queued in front of it.  Under stream
// capture a buffer is never reused (the captured kernel reads it at every
// replay of the graph): it is kept for the life of the process.
constexpr int kTableRing = 16;
struct TableBuf {
    uint8_t* host = nullptr;
    uint8_t* dev = nullptr;
    size_t cap = 0;
    hipEvent_t ev = nullptr;
    uint32_t seq = 0;
    bool busy = false;
};
struct TableStage {
    TableBuf buf[kTableRing];
    int nbuf = 0;
    int oldest = 0;                   // the next buffer to wait for when all are busy
    uint32_t* flags_host = nullptr;   // one word per ring buffer
    uint32_t* flags_dev = nullptr;
    ~TableStage() {
        for (int i = 0; i < nbuf; i++) {
            if (buf[i].busy && buf[i].ev) (void)hipEventSynchronize(buf[i].ev);
            if (buf[i].host) (void)hipHostFree(buf[i].host);
            if (buf[i].ev) (void)hipEventDestroy(buf[i].ev);
        }
        if (flags_host) (void)hipHostFree(flags_host);
    }
    bool done(int i) const {
        const TableBuf& b = buf[i];
        return !b.busy || ((volatile const uint32_t*)flags_host)[i] == b.seq;
    }
    // a buffer whose previous upload has been read (-1: none could be made)
    int acquire() {
        for (int i = 0; i < nbuf; i++)
            if (done(i)) {
                std::atomic_thread_fence(std::memory_order_acquire);
                buf[i].busy = false;
                return i;
            }
        if (nbuf < kTableRing) {
            if (hipEventCreateWithFlags(&buf[nbuf].ev, hipEventDisableTiming) != hipSuccess) return -1;
            return nbuf++;
        }
        const int i = oldest;
        oldest = (oldest + 1) % kTableRing;
        if (hipEventSynchronize(buf[i].ev) != hipSuccess) return -1;
        // the kernel has completed: its flag store is visible (bounded wait
        // only as a guard against a transport fault)
        const time_t t0 = time(nullptr);
        while (!done(i)) {
            if (time(nullptr) - t0 > 30) return -1;
            sched_yield();
        }
        std::atomic_thread_fence(std::memory_order_acquire);
        buf[i].busy = false;
        return i;
    }
};
thread_local TableStage t_table;

// The flag word of captured uploads (written at every replay, never read).
uint32_t* t_captured_flags() {
    static uint32_t* dev = nullptr;
    static std::atomic<bool> made{false};
    static std::atomic_flag lock = ATOMIC_FLAG_INIT;
    if (made.load(std::memory_order_acquire)) return dev;
    while (lock.test_and_set(std::memory_order_acquire)) sched_yield();
    if (!made.load(std::memory_order_relaxed)) {
        void* h = nullptr;
        void* d = nullptr;
        if (hipHostMalloc(&h, 64, hipHostMallocCoherent | hipHostMallocMapped) == hipSuccess &&
            hipHostGetDevicePointer(&d, h, 0) == hipSuccess) {
            dev = (uint32_t*)d;
            made.store(true, std::memory_order_release);
        }
    }
    lock.clear(std::memory_order_release);
    return dev;
}

}  // namespace

namespace bshuf {

hipError_t stage_upload(const void* host, size_t bytes, void* dev, hipStream_t s) {
    TableStage& t = t_table;
    const unsigned fl = hipHostMallocCoherent | hipHostMallocMapped;
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(s, &cap) != hipSuccess) return hipErrorUnknown;
    if (cap != hipStreamCaptureStatusNone) {
        // captured: a buffer of its own, kept for the graph's replays
        void* h = nullptr;
        void* d = nullptr;
        if (hipHostMalloc(&h, bytes + 64, fl) != hipSuccess) return hipErrorOutOfMemory;
        if (hipHostGetDevicePointer(&d, h, 0) != hipSuccess) return hipErrorUnknown;
        memcpy(h, host, bytes);
        XferArgs a{(uint8_t*)dev, (const uint8_t*)d, (int64_t)bytes, t_captured_flags(), 1};
        if (!a.flags) return hipErrorOutOfMemory;
        hipLaunchKernelGGL(k_xfer<false>, dim3(1), dim3(kXferThreads), 0, s, a);
        return hipGetLastError();
    }
    if (!t.flags_host) {
        void* f = nullptr;
        if (hipHostMalloc(&f, kTableRing * sizeof(uint32_t), fl) != hipSuccess) return hipErrorOutOfMemory;
        t.flags_host = (uint32_t*)f;
        memset(f, 0, kTableRing * sizeof(uint32_t));
        void* fd = nullptr;
        if (hipHostGetDevicePointer(&fd, f, 0) != hipSuccess) return hipErrorUnknown;
        t.flags_dev = (uint32_t*)fd;
    }
    const int i = t.acquire();
    if (i < 0) return hipErrorUnknown;
    TableBuf& b = t.buf[i];
    if (b.cap < bytes) {
        if (b.host) (void)hipHostFree(b.host);
        b.host = b.dev = nullptr;
        b.cap = 0;
        void* h = nullptr;
        if (hipHostMalloc(&h, bytes + 64, fl) != hipSuccess) return hipErrorOutOfMemory;
        void* d = nullptr;
        if (hipHostGetDevicePointer(&d, h, 0) != hipSuccess) return hipErrorUnknown;
        b.host = (uint8_t*)h;
        b.dev = (uint8_t*)d;
        b.cap = bytes;
    }
    memcpy(b.host, host, bytes);
    b.seq = b.seq + 1 == 0 ? 1 : b.seq + 1;
    XferArgs a{(uint8_t*)dev, b.dev, (int64_t)bytes, t.flags_dev + i, b.seq};
    hipLaunchKernelGGL(k_xfer<false>, dim3(1), dim3(kXferThreads), 0, s, a);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = hipEventRecord(b.ev, s);
    if (e == hipSuccess) b.busy = true;
    return e;
}

}  // namespace bshuf

extern "C" {

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
    HostCtx* c = host_ctx();
    if (!c) return kErrHip;
    const size_t bytes = size * elem_size;
    const size_t bound = bshuf_compress_lz4_bound(size, elem_size, block_size);
    const size_t wsb = bshuf_compress_lz4_dev_workspace(size, elem_size, block_size);
    uint8_t* di = (uint8_t*)c->dbuf(HostCtx::kIn, bytes);
    uint8_t* dout = (uint8_t*)c->dbuf(HostCtx::kOut, bound);
    void* ws = c->dbuf(HostCtx::kWs, wsb);
    int64_t* dres = (int64_t*)c->dbuf(HostCtx::kRes, 8);
    if (!di || !dout || !ws || !dres) return -1;
    if (!h2d(*c, di, (const uint8_t*)in, 0, bytes)) return fail(*c);
    const bool own = diag_alloc_ws();
    const int64_t e = bshuf_compress_lz4_dev(di, dout, size, elem_size, block_size, own ? nullptr : ws,
                                             own ? 0 : wsb, dres, nullptr, c->s);
    if (e < 0) return e;
    int64_t res = 0;
    if (!read_result(*c, dres, res)) return fail(*c);
    if (res > 0 && (size_t)res <= bound && !d2h(*c, (uint8_t*)out, dout, (size_t)res)) return fail(*c);
    return res;
}

int64_t bshuf_decompress_lz4(const void* in, void* out, const size_t size, const size_t elem_size,
                             size_t block_size) {
    Plan p;
    const int64_t r = make_plan(size, elem_size, block_size, p);
    if (r) return r;
    if (!have_device()) return kErrHip;
    HostCtx* c = host_ctx();
    if (!c) return kErrHip;
    const size_t bytes = size * elem_size;
    // the stream is at most the compress bound: stage into a buffer of that
    // size while the walk below finds its real length
    const size_t max_in = bshuf_compress_lz4_bound(size, elem_size, block_size);
    uint8_t* di = (uint8_t*)c->dbuf(HostCtx::kIn, max_in);
    uint8_t* dout = (uint8_t*)c->dbuf(HostCtx::kOut, bytes);
    uint64_t* doffs = (uint64_t*)c->dbuf(HostCtx::kOffs, (size_t)p.nb * 8);
    int64_t* dres = (int64_t*)c->dbuf(HostCtx::kRes, 8);
    if (!di || !dout || !doffs || !dres) return -1;
    // Walk the BE32 headers through the host buffer (the reference's own
    // iochain walk, src/bitshuffle.c:92-95): it finds the block offsets and how
    // many bytes of `in` belong to the stream, which the caller does not pass.
    // Every kPiece bytes walked leave for the device at once, so the copy
    // overlaps the rest of the walk.  The walk stops at the first implausible
    // header (length 0 or above LZ4_compressBound of its block): that block
    // and every one behind it keep the all-ones "unresolved" offset and
    // nothing from that header on is staged, so the device decoder reports
    // -1001 -- as bshuf_decompress_lz4_dev's parallel index rebuild does for
    // the same bytes.  No byte past the last plausible record is read.
    const uint8_t* i8 = (const uint8_t*)in;
    std::vector<uint64_t>& offs = c->offs;
    offs.assign((size_t)p.nb, ~(uint64_t)0);
    uint64_t pos = 0, issued = 0;
    bool broken = false;
    for (int64_t k = 0; k < p.nb; k++) {
        const uint8_t* h = i8 + pos;
        const uint32_t len = ((uint32_t)h[0] << 24) | ((uint32_t)h[1] << 16) |
                             ((uint32_t)h[2] << 8) | h[3];
        const uint32_t bound = (uint32_t)lz4_bound((k < p.L.nfull ? p.L.bs : p.L.last) * p.L.E);
        if (len == 0 || len > bound) {
            broken = true;
            break;
        }
        offs[(size_t)k] = pos;
        pos += 4 + (uint64_t)len;
        if (pos - issued >= kPiece) {
            if (!h2d(*c, di, i8, issued, pos)) return fail(*c);
            issued = pos;
        }
    }
    const size_t in_nbytes = (size_t)pos + (broken ? 0 : (size_t)p.tail);
    if (in_nbytes > max_in) return -91;
    if (!h2d(*c, di, i8, issued, in_nbytes) ||
        !h2d(*c, (uint8_t*)doffs, (const uint8_t*)offs.data(), 0, (uint64_t)p.nb * 8))
        return fail(*c);
    const size_t wsb = bshuf_decompress_lz4_dev_workspace(in_nbytes, size, elem_size, block_size);
    void* ws = c->dbuf(HostCtx::kWs, wsb);
    if (!ws) return -1;
    const bool own = diag_alloc_ws();
    const int64_t e = bshuf_decompress_lz4_dev(di, in_nbytes, dout, size, elem_size, block_size,
                                               own ? nullptr : ws, own ? 0 : wsb, dres, doffs, c->s);
    if (e < 0) return e;
    int64_t res = 0;
    if (!read_result(*c, dres, res)) return fail(*c);
    if (res >= 0 && bytes && !d2h(*c, (uint8_t*)out, dout, bytes)) return fail(*c);
    return res;
}

// Test hook: fills every device buffer and pinned staging slot of the CALLING
// thread with `byte` (a poisoned previous state for the next host call).
int64_t bshuf_host_poison(int byte) {
    if (!have_device()) return kErrHip;
    HostCtx* c = host_ctx();
    if (!c) return kErrHip;
    if (!c->settle(0) || !c->settle(1)) return fail(*c);
    for (int i = 0; i < HostCtx::kN; i++)
        if (c->buf[i] && dev_fill(c->buf[i], byte, c->cap[i], c->s) != hipSuccess) return kErrHip;
    if (hipStreamSynchronize(c->s) != hipSuccess) return kErrHip;
    for (auto& x : c->slot) memset(x.host, byte, kPiece + 64);
    return 0;
}

// Transport counters of the process: out[0] staged pieces moved, out[1] times
// a piece's completion event fired before all of its flag words were set.
void bshuf_host_xfer_stats(uint64_t* out2) {
    out2[0] = g_stat_pieces.load();
    out2[1] = g_stat_late.load();
}

}  // extern "C"

// ---------------------------------------------------------------------------
// The reference's internal transpose steps (include/bitshuffle_internals.h,
// bitshuffle/ext.pyx:56-86): host pointers in and out, the step itself on the
// device (internals.hip, or a one-block call of the transpose kernels).
// ---------------------------------------------------------------------------
#include "../../include/bitshuffle_internals.h"

namespace {

constexpr int64_t kErrNotMult8 = -80;  // CHECK_MULT_EIGHT, src/bitshuffle_internals.h

template <class Op>
int64_t host_step(const void* in, void* out, size_t size, size_t elem_size, Op op) {
    if (!have_device()) return kErrHip;
    const size_t bytes = size * elem_size;
    if (bytes == 0) return 0;
    HostCtx* c = host_ctx();
    if (!c) return kErrHip;
    uint8_t* di = (uint8_t*)c->dbuf(HostCtx::kIn, bytes);
    uint8_t* dout = (uint8_t*)c->dbuf(HostCtx::kOut, bytes);
    if (!di || !dout) return -1;
    if (!h2d(*c, di, (const uint8_t*)in, 0, bytes)) return fail(*c);
    const int64_t r = op(di, dout, c->s);
    if (r < 0) return r;
    if (!d2h(*c, (uint8_t*)out, dout, bytes)) return fail(*c);
    return (int64_t)bytes;
}

// The one-block hooks run the whole array as ONE bitshuffle block: up to
// kMaxOneBlock bytes and elem_size <= 65536 (make_plan's device limits),
// checked before anything touches the device (bitshuffle_internals.h).
constexpr size_t kMaxOneBlock = (size_t)INT32_MAX / 2;
bool one_block_ok(size_t size, size_t elem_size) {
    return elem_size <= 65536 && (elem_size == 0 || size <= kMaxOneBlock / elem_size);
}

int64_t bit_block(const void* in, void* out, size_t size, size_t elem_size, bool fwd) {
    if (size % 8) return kErrNotMult8;
    if (!one_block_ok(size, elem_size)) return kErrUnsupported;
    return host_step(in, out, size, elem_size, [&](uint8_t* di, uint8_t* dout, hipStream_t s) {
        return fwd ? bshuf_bitshuffle_dev(di, dout, size, elem_size, size, s)
                   : bshuf_bitunshuffle_dev(di, dout, size, elem_size, size, s);
    });
}

int64_t trans_elem_step(const void* in, void* out, size_t size, size_t elem_size, int64_t lda,
                        int64_t ldb, int64_t es) {
    return host_step(in, out, size, elem_size, [&](uint8_t* di, uint8_t* dout, hipStream_t s) {
        return launch_trans_elem(di, dout, lda, ldb, es, s) == hipSuccess ? 0 : kErrHip;
    });
}

}  // namespace

extern "C" {

int64_t bshuf_copy(const void* in, void* out, const size_t size, const size_t elem_size) {
    return host_step(in, out, size, elem_size, [&](uint8_t* di, uint8_t* dout, hipStream_t s) {
        return hipMemcpyAsync(dout, di, size * elem_size, hipMemcpyDeviceToDevice, s) == hipSuccess
                   ? 0 : kErrHip;
    });
}

int64_t bshuf_trans_byte_elem_scal(const void* in, void* out, const size_t size, const size_t elem_size) {
    return trans_elem_step(in, out, size, elem_size, (int64_t)size, (int64_t)elem_size, 1);
}

int64_t bshuf_trans_bit_byte_scal(const void* in, void* out, const size_t size, const size_t elem_size) {
    const size_t nbyte = size * elem_size;
    if (nbyte % 8) return kErrNotMult8;
    if (!one_block_ok(nbyte, 1)) return kErrUnsupported;
    return host_step(in, out, size, elem_size, [&](uint8_t* di, uint8_t* dout, hipStream_t s) {
        return bshuf_bitshuffle_dev(di, dout, nbyte, 1, nbyte, s);
    });
}

int64_t bshuf_trans_bitrow_eight(const void* in, void* out, const size_t size, const size_t elem_size) {
    if (size % 8) return kErrNotMult8;
    return trans_elem_step(in, out, size, elem_size, 8, (int64_t)elem_size, (int64_t)(size / 8));
}

int64_t bshuf_trans_bit_elem_scal(const void* in, void* out, const size_t size, const size_t elem_size) {
    return bit_block(in, out, size, elem_size, true);
}

int64_t bshuf_trans_byte_bitrow_scal(const void* in, void* out, const size_t size,
                                     const size_t elem_size) {
    if (size % 8) return kErrNotMult8;
    return trans_elem_step(in, out, size, elem_size, 8 * (int64_t)elem_size, (int64_t)(size / 8), 1);
}

int64_t bshuf_shuffle_bit_eightelem_scal(const void* in, void* out, const size_t size,
                                         const size_t elem_size) {
    if (size % 8) return kErrNotMult8;
    return host_step(in, out, size, elem_size, [&](uint8_t* di, uint8_t* dout, hipStream_t s) {
        return launch_shuffle_bit_eightelem(di, dout, (int64_t)size, (int64_t)elem_size, s) == hipSuccess
                   ? 0 : kErrHip;
    });
}

int64_t bshuf_untrans_bit_elem_scal(const void* in, void* out, const size_t size, const size_t elem_size) {
    return bit_block(in, out, size, elem_size, false);
}

int64_t bshuf_trans_bit_elem(const void* in, void* out, const size_t size, const size_t elem_size) {
    return bit_block(in, out, size, elem_size, true);
}

int64_t bshuf_untrans_bit_elem(const void* in, void* out, const size_t size, const size_t elem_size) {
    return bit_block(in, out, size, elem_size, false);
}

#define BSHUF_MISSING_ISA(name, code)                                                       \
    int64_t name(const void* in, void* out, const size_t size, const size_t elem_size) {   \
        (void)in, (void)out, (void)size, (void)elem_size;                                   \
        return code;                                                                        \
    }
BSHUF_MISSING_ISA(bshuf_trans_byte_elem_SSE, -11)
BSHUF_MISSING_ISA(bshuf_trans_bit_byte_SSE, -11)
BSHUF_MISSING_ISA(bshuf_trans_bit_elem_SSE, -11)
BSHUF_MISSING_ISA(bshuf_trans_byte_bitrow_SSE, -11)
BSHUF_MISSING_ISA(bshuf_shuffle_bit_eightelem_SSE, -11)
BSHUF_MISSING_ISA(bshuf_untrans_bit_elem_SSE, -11)
BSHUF_MISSING_ISA(bshuf_trans_bit_byte_AVX, -12)
BSHUF_MISSING_ISA(bshuf_trans_bit_elem_AVX, -12)
BSHUF_MISSING_ISA(bshuf_trans_byte_bitrow_AVX, -12)
BSHUF_MISSING_ISA(bshuf_shuffle_bit_eightelem_AVX, -12)
BSHUF_MISSING_ISA(bshuf_untrans_bit_elem_AVX, -12)
BSHUF_MISSING_ISA(bshuf_trans_byte_elem_NEON, -13)
BSHUF_MISSING_ISA(bshuf_trans_bit_byte_NEON, -13)
BSHUF_MISSING_ISA(bshuf_trans_bit_elem_NEON, -13)
BSHUF_MISSING_ISA(bshuf_trans_byte_bitrow_NEON, -13)
BSHUF_MISSING_ISA(bshuf_shuffle_bit_eightelem_NEON, -13)
BSHUF_MISSING_ISA(bshuf_untrans_bit_elem_NEON, -13)
BSHUF_MISSING_ISA(bshuf_trans_bit_byte_AVX512, -14)
BSHUF_MISSING_ISA(bshuf_trans_bit_elem_AVX512, -14)
BSHUF_MISSING_ISA(bshuf_shuffle_bit_eightelem_AVX512, -14)
BSHUF_MISSING_ISA(bshuf_untrans_bit_elem_AVX512, -14)
#undef BSHUF_MISSING_ISA

}  // extern "C"
