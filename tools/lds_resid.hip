// Residency probe: how many one-wave workgroups with L bytes of dynamic LDS
// are resident on a CU at once.  Every workgroup sleeps a fixed 40 us (bounded
// by s_memrealtime, so every wave exits); a grid of 256*k workgroups takes one
// period while k fit per CU and two once it does not.  Compares the measured
// residency with hipOccupancyMaxActiveBlocksPerMultiprocessor.
// Build: hipcc --offload-arch=gfx950 -O2 tools/lds_resid.hip -o tools/lds_resid
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

__global__ __launch_bounds__(64) void k_sleep(int* sink) {
    extern __shared__ int s[];
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < 4000) __builtin_amdgcn_s_sleep(8);
    if (threadIdx.x == 0) s[0] = 1;
    __builtin_amdgcn_wave_barrier();
    if (threadIdx.x == 0 && s[0] == 2) sink[0] = 1;
}

int main(int argc, char** argv) {
    int* sink;
    (void)hipMalloc(&sink, 4);
    int cus = 256;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    (void)hipFuncSetAttribute((const void*)k_sleep, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    for (int i = 1; i < argc; i++) {
        const int L = atoi(argv[i]);
        int occ = 0;
        (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, (const void*)k_sleep, 64, L);
        float base = 0;
        int fit = 0;
        for (int k = 1; k <= 24; k++) {
            hipLaunchKernelGGL(k_sleep, dim3(cus * k), dim3(64), L, 0, sink);
            (void)hipEventRecord(a, 0);
            hipLaunchKernelGGL(k_sleep, dim3(cus * k), dim3(64), L, 0, sink);
            (void)hipEventRecord(b, 0);
            (void)hipEventSynchronize(b);
            float ms = 0;
            (void)hipEventElapsedTime(&ms, a, b);
            if (k == 1) base = ms;
            if (ms < 1.5f * base) fit = k;
            else break;
        }
        printf("lds %6d  hipOccupancy %2d  measured %2d  (period %.3f ms)\n", L, occ, fit, base);
    }
    return 0;
}
