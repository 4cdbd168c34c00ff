// sq_probe.hip -- what gfx950's SQ instruction counters count (VERDICT r03
// weak #8: state the rule that turns SQ_INSTS_* into instructions per block).
// One kernel, 1024 waves of 64 lanes; every wave issues exactly, in an asm
// loop of kIters iterations: 8 VALU (v_add_u32), 4 SALU (s_add_u32, besides
// the loop's own 2 SALU), 2 LDS (ds_read_b32) and 1 branch.  Dividing the
// counters by these known totals gives the factor of each counter.
// Build: hipcc --offload-arch=gfx950 -O3 tools/sq_probe.hip -o tools/sq_probe
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int kIters = 1000;
constexpr int kWaves = 1024;

__global__ __launch_bounds__(64) void k_sq_probe(int* out) {
    __shared__ int lds[64];
    lds[threadIdx.x] = threadIdx.x;
    __syncthreads();
    int v = threadIdx.x, s = 0, cnt = kIters;
    const unsigned a = (unsigned)(uintptr_t)&lds[threadIdx.x];
    int r0, r1;
    asm volatile(
        "L_sq%=:\n\t"
        "v_add_u32 %[v], 1, %[v]\n\t"
        "v_add_u32 %[v], 1, %[v]\n\t"
        "v_add_u32 %[v], 1, %[v]\n\t"
        "v_add_u32 %[v], 1, %[v]\n\t"
        "v_add_u32 %[v], 1, %[v]\n\t"
        "v_add_u32 %[v], 1, %[v]\n\t"
        "v_add_u32 %[v], 1, %[v]\n\t"
        "v_add_u32 %[v], 1, %[v]\n\t"
        "s_add_u32 %[s], %[s], 1\n\t"
        "s_add_u32 %[s], %[s], 1\n\t"
        "s_add_u32 %[s], %[s], 1\n\t"
        "s_add_u32 %[s], %[s], 1\n\t"
        "ds_read_b32 %[r0], %[a]\n\t"
        "ds_read_b32 %[r1], %[a] offset:4\n\t"
        "s_waitcnt lgkmcnt(0)\n\t"
        "s_sub_u32 %[c], %[c], 1\n\t"
        "s_cmp_lg_u32 %[c], 0\n\t"
        "s_cbranch_scc1 L_sq%=\n\t"
        : [v] "+v"(v), [s] "+s"(s), [c] "+s"(cnt), [r0] "=&v"(r0), [r1] "=&v"(r1)
        : [a] "v"(a)
        : "scc", "memory");
    if (v == -1) out[0] = s + r0 + r1;  // keeps the results live
}

int main() {
    int* d = nullptr;
    if (hipMalloc(&d, 64) != hipSuccess) return 1;
    hipLaunchKernelGGL(k_sq_probe, dim3(kWaves), dim3(64), 0, 0, d);
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    printf("{\"waves\": %d, \"iters\": %d, \"valu_per_wave\": %d, \"salu_per_wave_loop\": %d, "
           "\"lds_per_wave\": %d, \"branch_per_wave\": %d}\n",
           kWaves, kIters, 8 * kIters, 6 * kIters, 2 * kIters, kIters);
    return 0;
}
