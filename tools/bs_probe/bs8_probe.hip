/* bs8_probe.hip -- throughput probe of the 8-blocks-per-lane bit-sliced AES-CTR keystream (tools/bs_probe/bs8_aes.h) on
 * gfx950: every lane XORs the keystream of 8 counter blocks into 8 consecutive-by-stride buffer blocks, in place.
 * Prints GiB/s per (rounds, waves per SIMD) and checks the first blocks against a host run of the same header.
 * Tool, not product:  hipcc --offload-arch=gfx950 -O3 -std=c++17 -I tools/bs_probe tools/bs_probe/bs8_probe.hip */
#include <hip/hip_runtime.h>
#pragma clang diagnostic ignored "-Wunused-result"
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>
#include "bs8_aes.h"
using namespace ptls_hip;

template <int ROUNDS, int WPS>
__global__ void __launch_bounds__(256, WPS) bs8_ctr(const uint32_t *__restrict__ K, const uint32_t *__restrict__ rk0, uint8_t *buf,
                                                    uint32_t ngroups, uint32_t n0, uint32_t n1, uint32_t n2)
{
    const uint32_t nthreads = gridDim.x * blockDim.x;
    const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
    /* lane t owns blocks t, t + T, t + 2T, ... (T = threads): group g of the lane = its blocks 8g .. 8g + 7 */
    for (uint32_t g = 0; g < ngroups; ++g) {
        uint32_t P[32];
        const uint32_t blk0 = (8 * g) * nthreads + tid;
        bs8::ctr_planes(P, rk0, n0, n1, n2, blk0, nthreads);
        bs8::rounds<ROUNDS>(P, K);
        uint32_t W[8][4];
        bs8::from_planes(P, W);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            uint4 *p = reinterpret_cast<uint4 *>(buf) + (size_t)blk0 + (size_t)k * nthreads;
            uint4 v = *p;
            v.x ^= W[k][0];
            v.y ^= W[k][1];
            v.z ^= W[k][2];
            v.w ^= W[k][3];
            *p = v;
        }
    }
}

int main(int argc, char **argv)
{
    const uint32_t ngroups = argc > 1 ? atoi(argv[1]) : 16;
    int ncu = 0;
    hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
    uint32_t rk[60], K[14 * 32];
    for (int i = 0; i < 60; ++i)
        rk[i] = 0x9e3779b9u * (i + 1);
    uint32_t *d_K, *d_rk;
    hipMalloc(&d_K, sizeof(K));
    hipMalloc(&d_rk, sizeof(rk));
    hipMemcpy(d_rk, rk, sizeof(rk), hipMemcpyHostToDevice);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    int fails = 0;
    for (int rounds : {10, 14}) {
        bs8::slice_key(rk, rounds, K);
        hipMemcpy(d_K, K, sizeof(K), hipMemcpyHostToDevice);
        for (int wps : {2, 3, 4}) {
            const unsigned block = 256, grid = ncu * wps; /* 256 threads = 1 wave per SIMD; wps blocks per CU */
            const size_t nthreads = (size_t)grid * block;
            const size_t bytes = nthreads * 8 * ngroups * 16;
            uint8_t *d_buf;
            hipMalloc(&d_buf, bytes);
            hipMemset(d_buf, 0, bytes);
            auto launch = [&]() {
#define L(R, W) hipLaunchKernelGGL((bs8_ctr<R, W>), dim3(grid), dim3(block), 0, 0, d_K, d_rk, d_buf, ngroups, 1u, 2u, 3u)
                if (rounds == 10) {
                    if (wps == 2) L(10, 2); else if (wps == 3) L(10, 3); else L(10, 4);
                } else {
                    if (wps == 2) L(14, 2); else if (wps == 3) L(14, 3); else L(14, 4);
                }
#undef L
            };
            launch(); /* buf = keystream */
            hipDeviceSynchronize();
            /* check the first 8 groups' worth of blocks of thread 0 .. 63 */
            std::vector<uint8_t> h(64 * 16);
            int bad = 0;
            for (uint32_t g = 0; g < 2; ++g)
                for (int k = 0; k < 8; ++k) {
                    const size_t blk = (size_t)(8 * g + k) * nthreads;
                    hipMemcpy(h.data(), d_buf + blk * 16, h.size(), hipMemcpyDeviceToHost);
                    for (int t = 0; t < 64; ++t) {
                        uint32_t P[32], W[8][4];
                        bs8::ctr_planes(P, rk, 1u, 2u, 3u, (uint32_t)(8 * g * nthreads + t), (uint32_t)nthreads);
                        if (rounds == 10)
                            bs8::rounds<10>(P, K);
                        else
                            bs8::rounds<14>(P, K);
                        bs8::from_planes(P, W);
                        if (memcmp(W[k], &h[16 * t], 16))
                            ++bad;
                    }
                }
            fails += bad != 0;
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
            printf("{\"rounds\": %d, \"waves_per_simd\": %d, \"ms\": %.3f, \"gibps\": %.1f, \"blocks\": %zu, \"check\": \"%s\"}\n", rounds, wps,
                   best, bytes / (best * 1e-3) / (1 << 30), nthreads * 8 * ngroups, bad ? "FAIL" : "ok");
            hipFree(d_buf);
        }
    }
    return fails != 0;
}
