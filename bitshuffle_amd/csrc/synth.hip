// synth.hip -- device generators for the benchmark inputs of SURVEY.md 8(d).
// Counter based: element i depends only on (seed, i), so the GPU produces the
// same bytes as the CPU definition without any host->device copy.
#include "launch.h"

namespace bshuf {

namespace {

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__device__ __forceinline__ uint32_t tri(uint64_t i) {
    const uint32_t p = (uint32_t)(i & 65535u);
    return p < 32768u ? p : 65536u - p;
}

__global__ __launch_bounds__(256) void k_synth(void* out, uint64_t n, int gen, uint64_t first,
                                               uint64_t seed) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += stride) {
        const uint64_t i = first + k;
        if (gen == 0) {
            reinterpret_cast<int32_t*>(out)[k] = (int32_t)i;
        } else {
            const uint64_t h = mix64(seed + (i + 1) * 0x9E3779B97F4A7C15ull);
            if (gen == 1)
                reinterpret_cast<int16_t*>(out)[k] =
                    (int16_t)((int)(tri(i) >> 3) - 2048 + (int)(h & 31u) - 16);
            else
                reinterpret_cast<float*>(out)[k] =
                    (float)(tri(i) * 64u + (uint32_t)(h & 255u)) / 1024.0f;
        }
    }
}

}  // namespace

hipError_t launch_synth(void* out, size_t n, int gen, uint64_t first, uint64_t seed,
                        hipStream_t s) {
    if (n == 0) return hipSuccess;
    const uint64_t blocks = std::min<uint64_t>((n + 255) / 256, 256 * 64);
    hipLaunchKernelGGL(k_synth, dim3((unsigned)blocks), dim3(256), 0, s, out, (uint64_t)n, gen,
                       first, seed);
    return hipGetLastError();
}

}  // namespace bshuf
