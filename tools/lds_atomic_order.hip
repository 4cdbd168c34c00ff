// Micro-test (tools only): in what order does the LDS serialise same-address
// lanes of ONE returning atomic (ds_mskor_rtn_b32 / ds_wrxchg_rtn_b32)?
// Each active lane sets its own value; the returned old values reveal the
// processing order.  Prints per pattern whether the order was lane order.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

__global__ void k_order(const uint64_t* masks, const uint32_t* addr_sel, int npat, uint32_t* out,
                        int mode) {
    __shared__ uint32_t S[64];
    const int lane = threadIdx.x;
    for (int p = 0; p < npat; p++) {
        S[lane] = 0;
        __syncthreads();
        const uint64_t m = masks[p];
        uint32_t ret = 0xFFFFFFFFu;
        const uint32_t a = addr_sel[p * 64 + lane];  // dword index, and half in bit 8
        const uint32_t dw = a & 63, half = (a >> 8) & 1;
        if ((m >> lane) & 1) {
            const uint32_t val = (uint32_t)(lane + 1) << (16 * half);
            const uint32_t msk = 0xFFFFu << (16 * half);
            const uint32_t lds_addr = (uint32_t)(uintptr_t)(S + dw);
            if (mode == 0)
                asm volatile("ds_mskor_rtn_b32 %0, %1, %2, %3\n s_waitcnt lgkmcnt(0)"
                             : "=v"(ret) : "v"(lds_addr), "v"(msk), "v"(val) : "memory");
            else
                asm volatile("ds_wrxchg_rtn_b32 %0, %1, %2\n s_waitcnt lgkmcnt(0)"
                             : "=v"(ret) : "v"(lds_addr), "v"(val) : "memory");
        }
        out[p * 64 + lane] = ret;
        __syncthreads();
    }
}

int main() {
    const int npat = 4000;
    uint64_t* hm = (uint64_t*)malloc(npat * 8);
    uint32_t* ha = (uint32_t*)malloc(npat * 64 * 4);
    srand(7);
    for (int p = 0; p < npat; p++) {
        uint64_t m = 0;
        const int kind = p % 4;
        for (int l = 0; l < 64; l++) {
            const int on = kind == 0 ? 1 : (rand() % 3 != 0);
            m |= (uint64_t)on << l;
            const int ndw = kind == 0 ? 1 : (kind == 1 ? 2 : (kind == 2 ? 4 : 16));
            ha[p * 64 + l] = (uint32_t)(rand() % ndw) | ((uint32_t)(rand() % 2) << 8);
        }
        hm[p] = m;
    }
    uint64_t* dm;
    uint32_t *da, *dout;
    hipMalloc(&dm, npat * 8);
    hipMalloc(&da, npat * 64 * 4);
    hipMalloc(&dout, npat * 64 * 4);
    hipMemcpy(dm, hm, npat * 8, hipMemcpyHostToDevice);
    hipMemcpy(da, ha, npat * 64 * 4, hipMemcpyHostToDevice);
    uint32_t* ho = (uint32_t*)malloc(npat * 64 * 4);
    for (int mode = 0; mode < 2; mode++) {
        for (int rep = 0; rep < 3; rep++) {
            hipLaunchKernelGGL(k_order, dim3(1), dim3(64), 0, 0, dm, da, npat, dout, mode);
            hipMemcpy(ho, dout, npat * 64 * 4, hipMemcpyDeviceToHost);
            int lane_order = 0, other = 0;
            for (int p = 0; p < npat; p++) {
                // expected under lane order: lane j sees (for its dword/half under mskor,
                // or whole dword under wrxchg) the value of the latest lower active lane
                // that wrote the same dword (and, for the half, the same half).
                int ok = 1;
                for (int l = 0; l < 64 && ok; l++) {
                    if (!((hm[p] >> l) & 1)) continue;
                    const uint32_t a = ha[p * 64 + l];
                    uint32_t exp = 0;
                    for (int q = 0; q < l; q++) {
                        if (!((hm[p] >> q) & 1)) continue;
                        const uint32_t b = ha[p * 64 + q];
                        if ((b & 63) != (a & 63)) continue;
                        const uint32_t hb = (b >> 8) & 1;
                        if (mode == 0)
                            exp = (exp & ~(0xFFFFu << (16 * hb))) | ((uint32_t)(q + 1) << (16 * hb));
                        else
                            exp = (uint32_t)(q + 1) << (16 * hb);
                    }
                    if (ho[p * 64 + l] != exp) ok = 0;
                }
                if (ok) lane_order++; else other++;
            }
            printf("%s rep %d: lane-order %d / %d patterns, other %d\n",
                   mode ? "ds_wrxchg_rtn_b32" : "ds_mskor_rtn_b32", rep, lane_order, npat, other);
        }
    }
    return 0;
}
