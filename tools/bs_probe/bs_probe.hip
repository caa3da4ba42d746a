/* bs_probe.hip -- standalone throughput probe of the bit-sliced AES-128 CTR keystream (csrc/bitslice_aes.h)
 * on gfx950: 32 blocks per lane, keystream XORed into a buffer in place.  Prints GiB/s and VALU-bound
 * expectations; checks a few blocks against a host run of the same header.  Tool, not product. */
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>
#include "bitslice_aes.h"
using namespace ptls_hip;

template <int ROUNDS, int WPE, bool ROLLED>
__global__ void __launch_bounds__(256, WPE) bs_ctr(const uint32_t *__restrict__ rk, uint8_t *buf, uint32_t nunits, uint32_t n0,
                                                   uint32_t n1, uint32_t n2)
{
    for (uint32_t u = blockIdx.x * blockDim.x + threadIdx.x; u < nunits; u += gridDim.x * blockDim.x) {
        uint32_t P[128];
#pragma unroll
        for (int k = 0; k < 32; ++k) {
            P[k] = n0;
            P[32 + k] = n1 ^ u;
            P[64 + k] = n2;
            P[96 + k] = __builtin_bswap32(k + 2);
        }
        bs::transpose_all(P);
        if (ROLLED)
            bs::encrypt_rolled<ROUNDS>(P, rk);
        else
            bs::encrypt<ROUNDS>(P, rk);
        bs::transpose_all(P);
        uint4 *p = reinterpret_cast<uint4 *>(buf) + (size_t)u * 32;
#pragma unroll
        for (int k = 0; k < 32; ++k) {
            uint4 v = p[k];
            v.x ^= P[k];
            v.y ^= P[32 + k];
            v.z ^= P[64 + k];
            v.w ^= P[96 + k];
            p[k] = v;
            __builtin_amdgcn_sched_barrier(0);
        }
    }
}

int main(int argc, char **argv)
{
    const uint32_t nunits = argc > 1 ? atoi(argv[1]) : (1u << 20); /* 32 blocks each: 512 MiB */
    uint32_t rk[60];
    for (int i = 0; i < 60; ++i)
        rk[i] = 0x9e3779b9u * (i + 1);
    uint32_t *d_rk;
    uint8_t *d_buf;
    const size_t bytes = (size_t)nunits * 512;
    hipMalloc(&d_rk, sizeof(rk));
    hipMemcpy(d_rk, rk, sizeof(rk), hipMemcpyHostToDevice);
    hipMalloc(&d_buf, bytes);
    hipMemset(d_buf, 0, bytes);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    int ncu = 256;
    const int only = argc > 2 ? atoi(argv[2]) : 0;
    for (int wpe : {1, 2, 3}) {
        if (only && wpe != only)
            continue;
        for (int grid_mult : {4, 16}) {
            const unsigned grid = ncu * grid_mult;
            auto launch = [&]() {
                if (wpe == 1)
                    hipLaunchKernelGGL((bs_ctr<10, 2, false>), dim3(grid), dim3(256), 0, 0, d_rk, d_buf, nunits, 1u, 2u, 3u);
                else if (wpe == 2)
                    hipLaunchKernelGGL((bs_ctr<10, 2, true>), dim3(grid), dim3(256), 0, 0, d_rk, d_buf, nunits, 1u, 2u, 3u);
                else
                    hipLaunchKernelGGL((bs_ctr<10, 1, true>), dim3(grid), dim3(256), 0, 0, d_rk, d_buf, nunits, 1u, 2u, 3u);
            };
            launch();
            hipDeviceSynchronize();
            float best = 1e9;
            for (int r = 0; r < 5; ++r) {
                hipEventRecord(e0);
                launch();
                hipEventRecord(e1);
                hipEventSynchronize(e1);
                float ms;
                hipEventElapsedTime(&ms, e0, e1);
                best = ms < best ? ms : best;
            }
            printf("variant=%d (1: unrolled wpe2, 2: rolled wpe2, 3: rolled wpe1) grid=%u: %.3f ms  %.1f GiB/s keystream (AES-128, %u blocks)\n", wpe, grid, best,
                   bytes / (best * 1e-3) / (1 << 30), nunits * 32);
        }
    }
    /* correctness: buffer was XORed an odd number of times (1 + 5 per config x 6 configs = 31+5... ) -> recompute */
    hipMemset(d_buf, 0, bytes);
    hipLaunchKernelGGL((bs_ctr<10, 2, true>), dim3(1024), dim3(256), 0, 0, d_rk, d_buf, nunits, 1u, 2u, 3u);
    std::vector<uint8_t> h(512 * 4);
    hipMemcpy(h.data(), d_buf + (size_t)(nunits - 4) * 512, h.size(), hipMemcpyDeviceToHost);
    int bad = 0;
    for (uint32_t u = nunits - 4; u < nunits; ++u) {
        uint32_t P[128];
        for (int k = 0; k < 32; ++k) {
            P[k] = 1;
            P[32 + k] = 2 ^ u;
            P[64 + k] = 3;
            P[96 + k] = __builtin_bswap32(k + 2);
        }
        bs::transpose_all(P);
        bs::encrypt<10>(P, rk);
        bs::transpose_all(P);
        for (int k = 0; k < 32; ++k)
            for (int w = 0; w < 4; ++w)
                if (memcmp(&h[(u - (nunits - 4)) * 512 + 16 * k + 4 * w], &P[32 * w + k], 4))
                    ++bad;
    }
    printf("check: %s (%d word mismatches)\n", bad ? "FAIL" : "ok", bad);
    return bad != 0;
}
