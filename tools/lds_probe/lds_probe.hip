/* lds_probe.hip -- sustained ds_read_b32 / ds_read_b128 rate on gfx950 with the T-table access pattern
 * (lane l reads bank l%32 of a 32x-replicated 256-entry table; random rows).  Reports LDS cycles per
 * wave-instruction at the measured clock (s_memtime), per CU. */
#include <hip/hip_runtime.h>
#include <stdio.h>

template <int NR, bool B128>
__global__ void __launch_bounds__(1024) lds_reads(uint32_t *out, int iters, unsigned long long *clk)
{
    __shared__ __attribute__((aligned(16))) uint32_t t[256 * 64];
    for (int i = threadIdx.x; i < 256 * 64; i += blockDim.x)
        t[i] = i * 0x9e3779b9u;
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63;
    uint32_t x[NR];
#pragma unroll
    for (int r = 0; r < NR; ++r)
        x[r] = (threadIdx.x * 131 + r * 977) & 0xff;
    const unsigned long long c0 = wall_clock64();
    const uint32_t lb = (lane & 31) * 4u;
    for (int it = 0; it < iters; ++it) {
        uint32_t v[NR][4];
        uint4 w[NR];
#pragma unroll
        for (int r = 0; r < NR; ++r) {
            if (B128) {
                const uint32_t addr = __builtin_amdgcn_perm(x[r], (lane & 15) << 4, 0x0c0c0400u);
                w[r] = *reinterpret_cast<const uint4 *>(reinterpret_cast<const uint8_t *>(t) + addr);
            } else {
                /* one v_perm per 4 lookups (offsets), as T0/T2 pairs of the kernel */
                const uint32_t addr = __builtin_amdgcn_perm(x[r], lb, 0x0c0c0400u);
                const uint8_t *p = reinterpret_cast<const uint8_t *>(t) + addr;
                v[r][0] = *reinterpret_cast<const uint32_t *>(p);
                v[r][1] = *reinterpret_cast<const uint32_t *>(p + 128);
                v[r][2] = *reinterpret_cast<const uint32_t *>(p + 32768);
                v[r][3] = *reinterpret_cast<const uint32_t *>(p + 32768 + 128);
            }
        }
#pragma unroll
        for (int r = 0; r < NR; ++r) {
            if (B128)
                x[r] = __builtin_amdgcn_bitop3_b32(__builtin_amdgcn_bitop3_b32(x[r], w[r].x, w[r].y, 0x96), w[r].z, w[r].w, 0x96);
            else
                x[r] = __builtin_amdgcn_bitop3_b32(__builtin_amdgcn_bitop3_b32(x[r], v[r][0], v[r][1], 0x96), v[r][2], v[r][3], 0x96);
        }
    }
    const unsigned long long c1 = wall_clock64();
    uint32_t acc = 0;
#pragma unroll
    for (int r = 0; r < NR; ++r)
        acc ^= x[r];
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
    if (threadIdx.x == 0 && blockIdx.x == 0)
        *clk = c1 - c0;
}

int main()
{
    uint32_t *d;
    unsigned long long *clk;
    hipMalloc(&d, 256 * 1024 * 4);
    hipMalloc(&clk, 8);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int iters = 2000;
    for (int b128 = 0; b128 < 2; ++b128)
        for (int threads : {256, 512, 768, 1024}) {
            auto launch = [&]() {
                if (b128)
                    hipLaunchKernelGGL((lds_reads<16, true>), dim3(256), dim3(threads), 0, 0, d, iters, clk);
                else
                    hipLaunchKernelGGL((lds_reads<8, false>), dim3(256), dim3(threads), 0, 0, d, iters, clk);
            };
            launch();
            hipDeviceSynchronize();
            hipEventRecord(e0);
            launch();
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            const double nr = b128 ? 16 : 32; /* 8 chains x 4 reads */
            const double winst = (double)iters * nr * (threads / 64); /* wave-instructions per CU */
            printf("%s waves/CU=%2d: %.3f ms, %.3f ns per wave-instr per CU (%.2f cyc @2.4GHz); %.1f TB/s chip\n",
                   b128 ? "ds_read_b128" : "ds_read_b32 ", threads / 64, ms, ms * 1e6 / winst, ms * 1e6 / winst * 2.4,
                   winst * 256 * 64 * (b128 ? 16 : 4) / (ms * 1e-3) / 1e12);
        }
    return 0;
}
