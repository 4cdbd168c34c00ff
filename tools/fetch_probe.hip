// fetch_probe.hip -- calibration of rocprofv3's FETCH_SIZE / WRITE_SIZE on
// gfx950 for the access shapes the codec's kernels use (VERDICT r02 item 4:
// the blanket x2 FETCH_SIZE correction is documented only for wide coalesced
// streaming reads).  Every kernel moves a known byte count over 1 GiB
// buffers (four times the 256 MiB Infinity Cache, so nothing is re-served
// on-die), once per launch; tools/fetch_probe.py divides the counters by it.
//
//   rd16     coalesced 16 B/lane loads            (encoder block prefetch,
//                                                   k_compact, decoder records)
//   rd8      coalesced 8 B/lane loads              (encoder raw prefetch, odd E)
//   rd4      coalesced 4 B/lane loads              (decoder token positions)
//   rdrec    16 B/lane loads of ~3.5 KB records at 16-B-aligned, not 128-B-
//            aligned starts, one record per wave   (decoder payload prefetch)
//   rdlane32 each lane walks its own 4 KiB region in 32-byte steps
//            (two 16-B loads; 64 lines per instruction)  (k_seq_scan windows)
//   wr16     coalesced 16 B/lane stores            (encoder records, k_compact)
//   wr16s    16-B stores, each lane 4 of them over its own 64 bytes
//            (lane stride 64 B)                    (decoder EK=2 output)
//   wr8      coalesced 8 B/lane stores             (decoder staged odd-E output)
//   wrlane16 each lane stores 16 B to its own region per step (k_seq_scan
//            token positions, SeqOut)
//
// Build: hipcc --offload-arch=gfx950 -O3 tools/fetch_probe.hip -o tools/fetch_probe
// Run:   tools/fetch_probe            (prints the known bytes per kernel, JSON)
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(1))) const u32x4 g128c;
typedef __attribute__((address_space(1))) u32x4 g128;
typedef __attribute__((address_space(1))) const u32x2 g64c;
typedef __attribute__((address_space(1))) u32x2 g64;
typedef __attribute__((address_space(1))) const uint32_t g32c;

constexpr size_t kBytes = size_t(1) << 30;
constexpr int kBlock = 256;
constexpr int kGrid = 4096;

__global__ __launch_bounds__(kBlock) void k_rd16(const uint8_t* in, uint32_t* sink) {
    const size_t n = kBytes / 16;
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * (size_t)kBlock + threadIdx.x; i < n; i += (size_t)kGrid * kBlock) {
        const u32x4 v = ((g128c*)in)[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    sink[blockIdx.x * kBlock + threadIdx.x] = acc;
}

__global__ __launch_bounds__(kBlock) void k_rd8(const uint8_t* in, uint32_t* sink) {
    const size_t n = kBytes / 8;
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * (size_t)kBlock + threadIdx.x; i < n; i += (size_t)kGrid * kBlock) {
        const u32x2 v = ((g64c*)in)[i];
        acc ^= v.x ^ v.y;
    }
    sink[blockIdx.x * kBlock + threadIdx.x] = acc;
}

__global__ __launch_bounds__(kBlock) void k_rd4(const uint8_t* in, uint32_t* sink) {
    const size_t n = kBytes / 4;
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * (size_t)kBlock + threadIdx.x; i < n; i += (size_t)kGrid * kBlock)
        acc ^= ((g32c*)in)[i];
    sink[blockIdx.x * kBlock + threadIdx.x] = acc;
}

// record r: start 4096 r + 16 ((r * 37) & 31), 3504 bytes (219 chunks)
constexpr int kRecChunks = 219;
constexpr size_t kRecs = kBytes / 4096;
__host__ __device__ inline size_t rec_start(size_t r) { return 4096 * r + 16 * ((r * 37) & 31); }

__global__ __launch_bounds__(kBlock) void k_rdrec(const uint8_t* in, uint32_t* sink) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint32_t acc = 0;
    for (size_t r = blockIdx.x * (size_t)(kBlock / 64) + wv; r < kRecs; r += (size_t)kGrid * (kBlock / 64)) {
        const g128c* p = (g128c*)(in + rec_start(r));
        for (int c = lane; c < kRecChunks; c += 64) {
            const u32x4 v = p[c];
            acc ^= v.x ^ v.y ^ v.z ^ v.w;
        }
    }
    sink[blockIdx.x * kBlock + threadIdx.x] = acc;
}

constexpr size_t kLaneRegion = 4096;
__global__ __launch_bounds__(kBlock) void k_rdlane32(const uint8_t* in, uint32_t* sink) {
    const size_t t = blockIdx.x * (size_t)kBlock + threadIdx.x;  // kGrid * kBlock regions of 1 KiB... see host
    const size_t regions = kBytes / kLaneRegion;
    uint32_t acc = 0;
    for (size_t g = t; g < regions; g += (size_t)kGrid * kBlock) {
        const g128c* p = (g128c*)(in + g * kLaneRegion);
        for (int s = 0; s < (int)(kLaneRegion / 32); s++) {
            const u32x4 a = p[2 * s], b = p[2 * s + 1];
            acc ^= a.x ^ a.y ^ a.z ^ a.w ^ b.x ^ b.y ^ b.z ^ b.w;
        }
    }
    sink[t] = acc;
}

__global__ __launch_bounds__(kBlock) void k_wr16(uint8_t* out) {
    const size_t n = kBytes / 16;
    for (size_t i = blockIdx.x * (size_t)kBlock + threadIdx.x; i < n; i += (size_t)kGrid * kBlock)
        ((g128*)out)[i] = u32x4{(uint32_t)i, 1u, 2u, 3u};
}

__global__ __launch_bounds__(kBlock) void k_wr16s(uint8_t* out) {
    const size_t n = kBytes / 64;  // 64-byte lane pieces
    for (size_t i = blockIdx.x * (size_t)kBlock + threadIdx.x; i < n; i += (size_t)kGrid * kBlock) {
        g128* p = (g128*)(out + 64 * i);
#pragma unroll
        for (int v = 0; v < 4; v++) p[v] = u32x4{(uint32_t)i, (uint32_t)v, 2u, 3u};
    }
}

__global__ __launch_bounds__(kBlock) void k_wr8(uint8_t* out) {
    const size_t n = kBytes / 8;
    for (size_t i = blockIdx.x * (size_t)kBlock + threadIdx.x; i < n; i += (size_t)kGrid * kBlock)
        ((g64*)out)[i] = u32x2{(uint32_t)i, 1u};
}

__global__ __launch_bounds__(kBlock) void k_wrlane16(uint8_t* out) {
    const size_t t = blockIdx.x * (size_t)kBlock + threadIdx.x;
    const size_t regions = kBytes / kLaneRegion;
    for (size_t g = t; g < regions; g += (size_t)kGrid * kBlock) {
        g128* p = (g128*)(out + g * kLaneRegion);
        for (int s = 0; s < (int)(kLaneRegion / 16); s++) p[s] = u32x4{(uint32_t)g, (uint32_t)s, 2u, 3u};
    }
}

#define CK(x)                                                              \
    do {                                                                   \
        hipError_t e_ = (x);                                               \
        if (e_ != hipSuccess) {                                            \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));        \
            return 1;                                                      \
        }                                                                  \
    } while (0)

int main() {
    uint8_t *a = nullptr, *b = nullptr;
    uint32_t* sink = nullptr;
    CK(hipMalloc(&a, kBytes + 4096));
    CK(hipMalloc(&b, kBytes + 4096));
    CK(hipMalloc(&sink, (size_t)kGrid * kBlock * 4));
    CK(hipMemset(a, 1, kBytes + 4096));
    CK(hipMemset(b, 0, kBytes + 4096));
    // evict a: stream 1 GiB of b through the caches first
    hipLaunchKernelGGL(k_wr16, dim3(kGrid), dim3(kBlock), 0, 0, b);
    CK(hipDeviceSynchronize());
    const size_t rec_bytes = kRecs * (size_t)kRecChunks * 16;
    hipLaunchKernelGGL(k_rd16, dim3(kGrid), dim3(kBlock), 0, 0, a, sink);
    hipLaunchKernelGGL(k_wr16, dim3(kGrid), dim3(kBlock), 0, 0, b);
    hipLaunchKernelGGL(k_rd8, dim3(kGrid), dim3(kBlock), 0, 0, a, sink);
    hipLaunchKernelGGL(k_wr16s, dim3(kGrid), dim3(kBlock), 0, 0, b);
    hipLaunchKernelGGL(k_rd4, dim3(kGrid), dim3(kBlock), 0, 0, a, sink);
    hipLaunchKernelGGL(k_wr8, dim3(kGrid), dim3(kBlock), 0, 0, b);
    hipLaunchKernelGGL(k_rdrec, dim3(kGrid), dim3(kBlock), 0, 0, a, sink);
    hipLaunchKernelGGL(k_wrlane16, dim3(kGrid), dim3(kBlock), 0, 0, b);
    hipLaunchKernelGGL(k_rdlane32, dim3(kGrid), dim3(kBlock), 0, 0, a, sink);
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    // known bytes per launch (reads: bytes loaded; the sink adds 4 MiB of
    // coalesced stores to every read kernel's WRITE_SIZE)
    printf("{\"k_rd16\": %zu, \"k_rd8\": %zu, \"k_rd4\": %zu, \"k_rdrec\": %zu, \"k_rdlane32\": %zu, "
           "\"k_wr16\": %zu, \"k_wr16s\": %zu, \"k_wr8\": %zu, \"k_wrlane16\": %zu, \"sink\": %zu}\n",
           kBytes, kBytes, kBytes, rec_bytes, kBytes, kBytes, kBytes, kBytes, kBytes,
           (size_t)kGrid * kBlock * 4);
    CK(hipFree(a));
    CK(hipFree(b));
    CK(hipFree(sink));
    return 0;
}
