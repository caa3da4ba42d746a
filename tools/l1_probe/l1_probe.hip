/* l1_probe.hip -- can the vector L1 (global_load_dword gathers from a 1 KiB table) take some of the AES
 * T-table lookups off the LDS?  Each of 8 chains per lane does NL ds_read_b32 (32x-replicated table,
 * conflict-free, as the kernel) and NG global gathers (4-B entries of a 256-entry table, random rows) per
 * iteration; reported: ns per iteration per CU and lookups per ns per CU.  768 threads per CU, as the
 * batch kernel. */
#include <hip/hip_runtime.h>
#include <stdio.h>

template <int NL, int NG>
__global__ void __launch_bounds__(768) mixed(const uint32_t *__restrict__ gt, uint32_t *out, int iters)
{
    __shared__ __attribute__((aligned(16))) uint32_t t[256 * 32];
    for (int i = threadIdx.x; i < 256 * 32; i += blockDim.x)
        t[i] = (i >> 5) * 0x9e3779b9u + 0x1234567u;
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t lb = (lane & 31) * 4u;
    constexpr int NR = 8;
    uint32_t x[NR];
#pragma unroll
    for (int r = 0; r < NR; ++r)
        x[r] = (threadIdx.x * 131 + r * 977 + blockIdx.x * 7) * 0x01010101u;
    for (int it = 0; it < iters; ++it) {
        uint32_t v[NR][8];
#pragma unroll
        for (int r = 0; r < NR; ++r) {
#pragma unroll
            for (int k = 0; k < NL; ++k) {
                const uint32_t xb = k < 4 ? x[r] : __builtin_amdgcn_alignbit(x[r], x[r], 4);
                const uint32_t addr = ((xb >> (8 * (k & 3))) & 0xff) * 128u + lb;
                v[r][k] = *reinterpret_cast<const uint32_t *>(reinterpret_cast<const uint8_t *>(t) + addr);
            }
#pragma unroll
            for (int k = 0; k < NG; ++k)
                v[r][NL + k] = gt[(x[r] >> (8 * ((k + 1) & 3))) & 0xff];
        }
#pragma unroll
        for (int r = 0; r < NR; ++r) {
            uint32_t a = x[r] * 0x9e3779b1u;
#pragma unroll
            for (int k = 0; k < NL + NG; ++k)
                a = __builtin_amdgcn_alignbit(a, a, 7) ^ v[r][k];
            x[r] = a;
        }
    }
    uint32_t acc = 0;
#pragma unroll
    for (int r = 0; r < NR; ++r)
        acc ^= x[r];
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

template <int NL, int NG>
static void run(const uint32_t *gt, uint32_t *d, int iters)
{
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipLaunchKernelGGL((mixed<NL, NG>), dim3(256), dim3(768), 0, 0, gt, d, iters);
    hipDeviceSynchronize();
    hipEventRecord(e0);
    hipLaunchKernelGGL((mixed<NL, NG>), dim3(256), dim3(768), 0, 0, gt, d, iters);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double wave_iters = (double)iters * 8 * 12; /* 8 chains x 12 waves per CU */
    const double ns = ms * 1e6 / wave_iters;
    printf("NL=%d NG=%d: %.3f ms  %.3f ns per chain-iteration per CU  -> %.3f ns per lookup (wave) ; LDS-only part %.3f ns\n", NL, NG, ms,
           ns, ns / (NL + NG), NL * 1.0);
}

int main()
{
    uint32_t *d, *gt;
    hipMalloc(&d, 256 * 1024 * 4);
    hipMalloc(&gt, 4096);
    uint32_t h[1024];
    for (int i = 0; i < 1024; ++i)
        h[i] = i * 2654435761u;
    hipMemcpy(gt, h, 4096, hipMemcpyHostToDevice);
    const int iters = 4000;
    run<4, 0>(gt, d, iters);
    run<0, 1>(gt, d, iters);
    run<0, 2>(gt, d, iters);
    run<0, 4>(gt, d, iters);
    run<4, 1>(gt, d, iters);
    run<4, 2>(gt, d, iters);
    run<4, 4>(gt, d, iters);
    run<8, 0>(gt, d, iters);
    run<8, 1>(gt, d, iters);
    run<8, 2>(gt, d, iters);
    return 0;
}
