// prof.hip -- optional per-kernel timing with HIP events on the launch stream.
//
// Off by default (one relaxed flag test per launch).  When enabled with
// bshuf_prof_enable(1), every kernel launched by the codec is bracketed by a
// pair of events recorded on ITS stream; bshuf_prof_collect() synchronises
// them and reports, per kernel name, the launch count and summed duration.
// bench.py uses this to price the dominant kernel against the HBM roofline;
// rocprofv3 --kernel-trace gives the same durations from the outside.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "launch.h"

namespace bshuf {

namespace {

struct Rec {
    const char* name;
    hipEvent_t a, b;
};

struct Prof {
    std::mutex mu;
    bool on = false;
    std::string only;  // non-empty: time only the kernel of this name
    std::vector<Rec> recs;
    std::vector<hipEvent_t> pool;
    hipEvent_t get() {
        if (!pool.empty()) {
            hipEvent_t e = pool.back();
            pool.pop_back();
            return e;
        }
        hipEvent_t e = nullptr;
        (void)hipEventCreate(&e);
        return e;
    }
};

Prof& P() {
    static Prof* p = new Prof();  // never destroyed: safe at process exit
    return *p;
}

}  // namespace

bool prof_on() { return P().on; }

// A/B knob: per calling thread, and only byte-identical variants are accepted
// (the timing ablations that change the output exist in the diag build only).
static thread_local int t_variant = 0;
int tuning_variant() { return t_variant & ~kNoPipe; }

namespace {
// The calling thread's side streams, one per device (kept for the thread's
// life; the destructor waits for them, ignoring errors at process exit).
constexpr int kPipeDevices = 16;
struct PipeSet {
    PipeCtx c[kPipeDevices];
    bool bad[kPipeDevices] = {};
    ~PipeSet() {
        for (PipeCtx& x : c) {
            if (!x.side) continue;
            (void)hipStreamSynchronize(x.side);
            for (hipEvent_t& e : x.ev)
                if (e) (void)hipEventDestroy(e);
            (void)hipStreamDestroy(x.side);
        }
    }
};
thread_local PipeSet t_pipe;
}  // namespace

PipeCtx* pipe_ctx(hipStream_t s) {
    if (t_variant & kNoPipe) return nullptr;
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(s, &cap) != hipSuccess || cap != hipStreamCaptureStatusNone) return nullptr;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kPipeDevices || t_pipe.bad[dev]) return nullptr;
    PipeCtx& x = t_pipe.c[dev];
    if (x.side) return &x;
    bool ok = hipStreamCreateWithFlags(&x.side, hipStreamNonBlocking) == hipSuccess;
    for (int i = 0; ok && i < kPipeEvents; i++)
        ok = hipEventCreateWithFlags(&x.ev[i], hipEventDisableTiming) == hipSuccess;
    if (!ok) {
        t_pipe.bad[dev] = true;  // leaked: at most once per thread and device
        x = PipeCtx{};
        return nullptr;
    }
    return &x;
}

hipError_t stream_after(hipStream_t s, hipStream_t from, hipEvent_t ev) {
    hipError_t e = hipEventRecord(ev, from);
    return e == hipSuccess ? hipStreamWaitEvent(s, ev, 0) : e;
}
#ifdef BSHUF_DIAG
static int g_diag_variant = 0;
int diag_variant() { return g_diag_variant; }
#endif

// Device memory set by a kernel (hipMemsetAsync's job).  Round 2 blamed the
// runtime memset for a stale `bad` word; the round-3 experiment (DESIGN.md
// §4.2) cleared it -- the runtime memset alone gave 0 wrong results in 40
// fresh processes -- so this is simply the codec's own fill.
__global__ __launch_bounds__(256) void k_fill(uint8_t* __restrict__ p, uint32_t v, int64_t n) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool vec = ((uintptr_t)p & 3) == 0;
    const int64_t n4 = vec ? n >> 2 : 0;
    const uint32_t w = v * 0x01010101u;
    for (int64_t i = t; i < n4; i += stride) reinterpret_cast<uint32_t*>(p)[i] = w;
    for (int64_t i = n4 * 4 + t; i < n; i += stride) p[i] = (uint8_t)v;
}

hipError_t dev_fill(void* p, int v, size_t n, hipStream_t s) {
    if (n == 0) return hipSuccess;
    const int64_t g = std::min<int64_t>(2048, ((int64_t)n / 4 + 255) / 256 + 1);
    hipLaunchKernelGGL(k_fill, dim3((unsigned)g), dim3(256), 0, s, (uint8_t*)p, (uint32_t)(v & 255),
                       (int64_t)n);
    return hipGetLastError();
}

constexpr int64_t kLdsGranule = 1280;
constexpr int64_t kLdsPerCu = 160 * 1024;

int64_t persistent_grid(const void* fn, int threads, size_t lds, int64_t work) {
    int dev = 0, cus = 256, per = 1;
    if (hipGetDevice(&dev) == hipSuccess)
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, fn, threads, lds) != hipSuccess || per < 1)
        per = 1;
    // gfx950 allocates LDS in 1,280-byte granules (measured, tools/lds_resid.hip);
    // the runtime's occupancy query assumes finer ones and can promise one
    // workgroup more per CU than fits, which leaves a second, mostly idle
    // round of persistent workgroups
    if (lds > 0) {
        const int64_t g = ((int64_t)lds + kLdsGranule - 1) / kLdsGranule * kLdsGranule;
        const int fit = (int)(kLdsPerCu / g);
        if (fit >= 1 && per > fit) per = fit;
    }
    const int64_t g = (int64_t)cus * per;
    return work < g ? (work > 0 ? work : 1) : g;
}

ProfScope::ProfScope(const char* name, hipStream_t s) : name_(name), s_(s), a_(nullptr) {
    Prof& p = P();
    if (!p.on) return;
    std::lock_guard<std::mutex> g(p.mu);
    if (!p.only.empty() && p.only != name) return;
    a_ = p.get();
    (void)hipEventRecord((hipEvent_t)a_, s);
}

ProfScope::~ProfScope() {
    if (!a_) return;
    Prof& p = P();
    std::lock_guard<std::mutex> g(p.mu);
    hipEvent_t b = p.get();
    (void)hipEventRecord(b, s_);
    p.recs.push_back(Rec{name_, (hipEvent_t)a_, b});
}

}  // namespace bshuf

using namespace bshuf;

extern "C" {

int bshuf_set_variant(int v) {
    // 2 inline LZ4 emitter, 4 one-group-per-lane transpose, 8 re-test table
    // lookup by lane 0's returning exchange, decoder record access 16 global
    // + touch / 32 global / 64 own LDS buffer (default: in place), 128
    // insert/readback search window (the fallback for devices without
    // lane-ordered LDS atomics), 512 every search window with per-lane validity
    // masks, 1024 large blocks by the lane-0 parse, 2048
    // the re-test's 4-byte test by readfirstlane before the count, 4096 record
    // copy-out at the end of its block's parse (not deferred), 8192 the
    // hand-scheduled re-test chain, 16384 the hand-scheduled search windows,
    // 24576 both, 57344 both with the shortcut (319488: + bit-sliced forward transpose), 40960 the re-test chain with its offset-2 shortcut (the
    // default for byU16 blocks), 65536 the compiled re-test chain, 172032 /
    // 450560 the 40960 / 319488 ones with the search-match hand-off in asm
    // (search_entry), 2793472 / 3072000 (the defaults) those with the whole
    // parse loop as one asm block (parse_chain) and the emission's literal
    // runs by lane_runs; any of
    // them | kNoPipe (1 << 20): no pipelined encode (launch.h)
    const int vv = v & ~kNoPipe;
    if (vv != 0 && vv != 2 && vv != 4 && vv != 8 && vv != 16 && vv != 32 && vv != 64 && vv != 128 && vv != 512 && vv != 1024 && vv != 2048 && vv != 4096 && vv != 8192 && vv != 16384 && vv != 24576 && vv != 40960 && vv != 57344 && vv != 65536 && vv != 319488 &&
        vv != 172032 && vv != 450560 &&
        vv != 2793472 && vv != 3072000)
        return -71;
    t_variant = v;
    return 0;
}

#ifdef BSHUF_DIAG
void bshuf_diag_set_ablation(int v) { g_diag_variant = v; }
#endif

void bshuf_prof_enable(int on) {
    Prof& p = P();
    std::lock_guard<std::mutex> g(p.mu);
    p.on = on != 0;
    // events made here, not per launch: hipEventCreate costs tens of us of
    // host time, which a timed region where the host is behind the GPU (after
    // a compress's result is read back) would otherwise pay per kernel
    // (measured: ~0.3 ms of GPU idle per config-2 step, r4f2 kernel trace)
    if (p.on) {
        const size_t want = 4096 + p.recs.size() * 2;
        while (p.pool.size() < want) {
            hipEvent_t e = nullptr;
            if (hipEventCreate(&e) != hipSuccess) break;
            p.pool.push_back(e);
        }
    }
}

// Restricts the timing to one kernel name (NULL or "": every kernel).  Each
// timed launch adds two event records to its stream (~0.2 ms per config-2
// step when every kernel is timed: bench.py times them all in its warmup and
// only the dominant kernel in its timed region).
void bshuf_prof_only(const char* name) {
    Prof& p = P();
    std::lock_guard<std::mutex> g(p.mu);
    p.only = name ? name : "";
}

// Writes "name count total_ms\n" lines into buf; returns the number of bytes
// needed (call again with a bigger buffer if it exceeds len).  Resets.
size_t bshuf_prof_collect(char* buf, size_t len) {
    Prof& p = P();
    std::lock_guard<std::mutex> g(p.mu);
    std::map<std::string, std::pair<long, double>> acc;
    for (auto& r : p.recs) {
        (void)hipEventSynchronize(r.b);
        float ms = 0.f;
        (void)hipEventElapsedTime(&ms, r.a, r.b);
        auto& x = acc[r.name];
        x.first += 1;
        x.second += ms;
        p.pool.push_back(r.a);
        p.pool.push_back(r.b);
    }
    p.recs.clear();
    std::string out;
    char line[256];
    for (auto& kv : acc) {
        snprintf(line, sizeof line, "%s %ld %.6f\n", kv.first.c_str(), kv.second.first,
                 kv.second.second);
        out += line;
    }
    if (buf && len) {
        const size_t n = out.size() < len - 1 ? out.size() : len - 1;
        memcpy(buf, out.data(), n);
        buf[n] = 0;
    }
    return out.size() + 1;
}

}  // extern "C"
