/* copy_probe.hip -- which device-copy shape reaches the HBM rate MI355X_MICROARCH.md quotes (6.29 TB/s, "float4 copy"),
 * for bench.py's achievable-HBM reference (ptls_hip_device_copy).  Tool, not product:
 *   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/copy_probe/copy_probe.hip -o tools/copy_probe/copy_probe */
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

/* U 16-byte accesses per lane per step, grid-stride; NT: nontemporal loads and stores */
template <int U, bool NT>
__global__ void __launch_bounds__(256) copy_k(const uint4 *__restrict__ src, uint4 *__restrict__ dst, size_t n16)
{
    const size_t stride = (size_t)gridDim.x * 256 * U;
    size_t i = (size_t)blockIdx.x * 256 * U + threadIdx.x;
    for (; i + (U - 1) * 256 < n16; i += stride) {
        const u32x4 *s4 = reinterpret_cast<const u32x4 *>(src);
        u32x4 *d4 = reinterpret_cast<u32x4 *>(dst);
        u32x4 v[U];
#pragma unroll
        for (int k = 0; k < U; ++k)
            v[k] = NT ? __builtin_nontemporal_load(s4 + i + k * 256) : s4[i + k * 256];
#pragma unroll
        for (int k = 0; k < U; ++k) {
            if (NT)
                __builtin_nontemporal_store(v[k], d4 + i + k * 256);
            else
                d4[i + k * 256] = v[k];
        }
    }
    for (int k = 0; k < U; ++k)
        if (i + k * 256 < n16)
            dst[i + k * 256] = src[i + k * 256];
}

/* one contiguous slice per workgroup (no grid stride): workgroup b copies [b * per, (b + 1) * per) */
template <int U>
__global__ void __launch_bounds__(256) copy_slice(const uint4 *__restrict__ src, uint4 *__restrict__ dst, size_t per)
{
    const size_t base = (size_t)blockIdx.x * per;
    for (size_t j = threadIdx.x; j < per; j += 256 * U) {
        uint4 v[U];
#pragma unroll
        for (int k = 0; k < U; ++k)
            v[k] = src[base + j + k * 256];
#pragma unroll
        for (int k = 0; k < U; ++k)
            dst[base + j + k * 256] = v[k];
    }
}

template <class F>
static double timeit(F f, int reps = 7)
{
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    f();
    CK(hipDeviceSynchronize());
    float best = 1e30f, sum = 0;
    float t[16];
    for (int r = 0; r < reps; ++r) {
        CK(hipEventRecord(a));
        f();
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        CK(hipEventElapsedTime(&t[r], a, b));
        best = t[r] < best ? t[r] : best;
        sum += t[r];
    }
    /* median */
    for (int i = 0; i < reps; ++i)
        for (int j = i + 1; j < reps; ++j)
            if (t[j] < t[i]) { float x = t[i]; t[i] = t[j]; t[j] = x; }
    (void)best, (void)sum;
    return t[reps / 2];
}

int main(int argc, char **argv)
{
    const size_t bytes = (argc > 1 ? strtoull(argv[1], 0, 0) : (4ull << 30));
    const size_t n16 = bytes / 16;
    int ncu = 0;
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    uint4 *s, *d;
    CK(hipMalloc(&s, bytes));
    CK(hipMalloc(&d, bytes));
    CK(hipMemset(s, 1, bytes));
    CK(hipMemset(d, 0, bytes));
    auto rate = [&](double ms) { return 2.0 * bytes / (ms * 1e-3) / 1e9; };
    printf("bytes %zu, %d CUs\n", bytes, ncu);
    for (int wpc : {2, 4, 8, 16, 32, 64}) {
        const unsigned grid = ncu * wpc;
        printf("grid %5u (%2d WG/CU): U1 %.0f  U2 %.0f  U4 %.0f  U8 %.0f  U4nt %.0f  U8nt %.0f GB/s\n", grid, wpc,
               rate(timeit([&] { copy_k<1, false><<<grid, 256>>>(s, d, n16); })),
               rate(timeit([&] { copy_k<2, false><<<grid, 256>>>(s, d, n16); })),
               rate(timeit([&] { copy_k<4, false><<<grid, 256>>>(s, d, n16); })),
               rate(timeit([&] { copy_k<8, false><<<grid, 256>>>(s, d, n16); })),
               rate(timeit([&] { copy_k<4, true><<<grid, 256>>>(s, d, n16); })),
               rate(timeit([&] { copy_k<8, true><<<grid, 256>>>(s, d, n16); })));
    }
    /* one thread per 16 B, no loop (the plainest "float4 copy") */
    {
        const unsigned grid = (unsigned)((n16 + 255) / 256);
        printf("flat one-uint4-per-thread grid %u: %.0f GB/s\n", grid, rate(timeit([&] { copy_k<1, false><<<grid, 256>>>(s, d, n16); })));
    }
    for (int wpc : {4, 8, 16}) {
        const unsigned grid = ncu * wpc;
        const size_t per = n16 / grid / 1024 * 1024;
        printf("slices %u x %zu B: U4 %.0f GB/s (copies %zu of %zu bytes)\n", grid, per * 16,
               2.0 * per * grid * 16 / (timeit([&] { copy_slice<4><<<grid, 256>>>(s, d, per); }) * 1e-3) / 1e9, per * grid * 16, bytes);
    }
    CK(hipMemcpy(d, s, 64, hipMemcpyDeviceToDevice));
    printf("hipMemcpyDtoD: %.0f GB/s\n", rate(timeit([&] { CK(hipMemcpyAsync(d, s, bytes, hipMemcpyDeviceToDevice, 0)); })));
    return 0;
}
