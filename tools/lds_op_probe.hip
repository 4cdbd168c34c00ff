// LDS op cost probe (round 6): cycles per wave instruction of ds_write_b32,
// ds_mskor_b32 (masked write, no return) and ds_write_b8, 64 lanes on
// consecutive dwords / bytes, with 1 and 8 waves per CU.  Host prints cycles
// per instruction per wave.  Build: hipcc --offload-arch=gfx950 -O3 tools/lds_op_probe.hip -o /tmp/lds_op_probe
#include <hip/hip_runtime.h>
#include <cstdio>

template <int OP>
__global__ __launch_bounds__(64) void k_probe(unsigned long long* out, int iters, int stride) {
    __shared__ uint32_t buf[64 * 65];
    const int lane = threadIdx.x;
    const uint32_t a = (uint32_t)(uintptr_t)(&buf[(blockIdx.x % 8) * 64 + lane * stride]);
    const uint32_t ab = (uint32_t)(uintptr_t)(&buf[0]) + lane;
    uint32_t v = lane;
    __syncthreads();
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int k = 0; k < 8; k++) {
            if (OP == 0) asm volatile("ds_write_b32 %0, %1" : : "v"(a), "v"(v) : "memory");
            if (OP == 1) asm volatile("ds_mskor_b32 %0, %1, %2" : : "v"(a), "v"(0xFFFFFFFFu), "v"(v) : "memory");
            if (OP == 2) asm volatile("ds_write_b8 %0, %1" : : "v"(ab), "v"(v) : "memory");
            if (OP == 3) asm volatile("ds_mskor_b32 %0, %1, %2" : : "v"(a), "v"(0x00FF00FFu), "v"(v & 0x00FF00FFu) : "memory");
        }
        v += 1;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) out[blockIdx.x] = t1 - t0;
}

int main() {
    unsigned long long* d;
    hipMalloc(&d, 8 * 4096);
    unsigned long long h[4096];
    const int iters = 4096;
    const char* names[] = {"ds_write_b32", "ds_mskor_b32 full", "ds_write_b8", "ds_mskor_b32 half"};
    for (int wpc : {1, 4, 8}) {
        const int nblk = 256 * wpc;
        for (int op = 0; op < 4; op++) {
            for (int rep = 0; rep < 2; rep++) {
                if (op == 0) hipLaunchKernelGGL(k_probe<0>, dim3(nblk), dim3(64), 0, 0, d, iters, 1);
                if (op == 1) hipLaunchKernelGGL(k_probe<1>, dim3(nblk), dim3(64), 0, 0, d, iters, 1);
                if (op == 2) hipLaunchKernelGGL(k_probe<2>, dim3(nblk), dim3(64), 0, 0, d, iters, 1);
                if (op == 3) hipLaunchKernelGGL(k_probe<3>, dim3(nblk), dim3(64), 0, 0, d, iters, 1);
                hipDeviceSynchronize();
            }
            hipMemcpy(h, d, 8 * nblk, hipMemcpyDeviceToHost);
            double s = 0;
            for (int i = 0; i < nblk; i++) s += h[i];
            // s_memtime is 100 MHz on gfx9xx? report raw ticks per instruction
            printf("waves/CU %d  %-20s %.3f ticks/instr/wave\n", wpc, names[op], s / nblk / (iters * 8.0));
        }
    }
    return 0;
}
