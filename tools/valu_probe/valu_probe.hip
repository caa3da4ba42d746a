/* valu_probe.hip -- issue model of dependent / independent v_bitop3_b32 chains on gfx950:
 * C independent chains per wave (round-robin), W waves per SIMD.  Prints cycles per VALU per SIMD. */
#include <hip/hip_runtime.h>
#include <stdio.h>

template <int C>
__global__ void chains(uint32_t *out, int iters)
{
    uint32_t a0 = threadIdx.x, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 * 9, a5 = a0 * 11, a6 = a0 * 13, a7 = a0 * 15;
    const uint32_t k = blockIdx.x;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            if (C == 1) {
                asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(a0) : "v"(k), "v"(a1));
            } else if (C == 2) {
                asm volatile("v_bitop3_b32 %0, %0, %2, %3 bitop3:0x96\n\tv_bitop3_b32 %1, %1, %2, %3 bitop3:0x96"
                             : "+v"(a0), "+v"(a1) : "v"(k), "v"(a7));
            } else if (C == 4) {
                asm volatile("v_bitop3_b32 %0, %0, %4, %5 bitop3:0x96\n\tv_bitop3_b32 %1, %1, %4, %5 bitop3:0x96\n\t"
                             "v_bitop3_b32 %2, %2, %4, %5 bitop3:0x96\n\tv_bitop3_b32 %3, %3, %4, %5 bitop3:0x96"
                             : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3) : "v"(k), "v"(a7));
            } else {
                asm volatile("v_bitop3_b32 %0, %0, %8, %9 bitop3:0x96\n\tv_bitop3_b32 %1, %1, %8, %9 bitop3:0x96\n\t"
                             "v_bitop3_b32 %2, %2, %8, %9 bitop3:0x96\n\tv_bitop3_b32 %3, %3, %8, %9 bitop3:0x96\n\t"
                             "v_bitop3_b32 %4, %4, %8, %9 bitop3:0x96\n\tv_bitop3_b32 %5, %5, %8, %9 bitop3:0x96\n\t"
                             "v_bitop3_b32 %6, %6, %8, %9 bitop3:0x96\n\tv_xor_b32 %7, %7, %8"
                             : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(k), "v"(k));
            }
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

int main()
{
    uint32_t *d;
    hipMalloc(&d, 256 * 1024 * 4 * 16);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int iters = 4096;
    for (int c : {1, 2, 4, 8}) {
        for (int w : {1, 2, 3, 4, 8}) {
            /* one workgroup of 64*4*w threads per CU: w waves per SIMD */
            const unsigned grid = 256, threads = 256 * w;
            auto launch = [&]() {
                if (c == 1) hipLaunchKernelGGL(chains<1>, dim3(grid), dim3(threads), 0, 0, d, iters);
                if (c == 2) hipLaunchKernelGGL(chains<2>, dim3(grid), dim3(threads), 0, 0, d, iters);
                if (c == 4) hipLaunchKernelGGL(chains<4>, dim3(grid), dim3(threads), 0, 0, d, iters);
                if (c == 8) hipLaunchKernelGGL(chains<8>, dim3(grid), dim3(threads), 0, 0, d, iters);
            };
            launch();
            hipDeviceSynchronize();
            hipEventRecord(e0);
            launch();
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            const double insts_per_simd = (double)iters * 16 * (c == 1 ? 1 : c) * w; /* wave-instructions per SIMD */
            printf("chains/wave=%d waves/SIMD=%d: %.3f ms, %.2f ns per VALU per SIMD (x2.4GHz = %.2f cyc)\n", c, w, ms,
                   ms * 1e6 / insts_per_simd, ms * 1e6 / insts_per_simd * 2.4);
        }
    }
    return 0;
}
