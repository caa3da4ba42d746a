// mailbox_probe: host -> resident wave -> host ping-pong latency for the plugin worker's mailbox placement.
//   pinned : the request word in fine-grained pinned host memory, polled by the wave over PCIe (the worker today)
//   vram   : the request word in fine-grained device memory the host writes through its mapping (if the box maps it)
// The answer always goes to a pinned host word the host spins on.  One wave, bounded life, so the kernel always ends.
// Build: hipcc --offload-arch=gfx950 -O2 -o mailbox_probe mailbox_probe.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <chrono>
#include <csetjmp>
#include <csignal>
#include <cstdio>
#include <cstring>
#include <vector>

__global__ void __launch_bounds__(64) pong(const uint32_t *in, uint32_t *out, uint32_t n, uint64_t life, int polls)
{
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    uint32_t last = 0;
    while (last < n) {
        uint32_t v = __hip_atomic_load(in, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        v = __builtin_amdgcn_readfirstlane(v);
        if (v != last && v <= n) {
            last = v;
            if (threadIdx.x == 0)
                __hip_atomic_store(out, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        if (__builtin_amdgcn_s_memrealtime() - t0 > life)
            break;
        if (polls)
            __builtin_amdgcn_s_sleep(1);
    }
}

static sigjmp_buf g_jb;
static void on_segv(int) { siglongjmp(g_jb, 1); }

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

static double run(const char *name, volatile uint32_t *h_in, const uint32_t *d_in, volatile uint32_t *h_out, uint32_t *d_out, int n)
{
    *h_in = 0;
    *h_out = 0;
    hipStream_t s;
    (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    hipLaunchKernelGGL(pong, dim3(1), dim3(64), 0, s, d_in, d_out, (uint32_t)n, (uint64_t)300000000, 0);
    std::vector<double> us;
    for (int i = 1; i <= n; ++i) {
        const auto t = std::chrono::steady_clock::now();
        __atomic_store_n(h_in, (uint32_t)i, __ATOMIC_RELEASE);
        while (__atomic_load_n(h_out, __ATOMIC_ACQUIRE) != (uint32_t)i) {
            if (std::chrono::steady_clock::now() - t > std::chrono::milliseconds(200)) {
                printf("%s: no answer to %d\n", name, i);
                (void)hipStreamSynchronize(s);
                return -1;
            }
        }
        us.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t).count());
    }
    (void)hipStreamSynchronize(s);
    (void)hipStreamDestroy(s);
    std::sort(us.begin() + 10, us.end());
    const double med = us[10 + (us.size() - 10) / 2], p10 = us[10 + (us.size() - 10) / 10];
    printf("%-8s round trip: median %.2f us, p10 %.2f us\n", name, med, p10);
    return med;
}

int main()
{
    const int n = 2000;
    uint32_t *h_out = nullptr, *h_in = nullptr;
    CK(hipHostMalloc((void **)&h_out, 4096, hipHostMallocCoherent));
    CK(hipHostMalloc((void **)&h_in, 4096, hipHostMallocCoherent));
    void *d_out = nullptr, *d_in = nullptr;
    CK(hipHostGetDevicePointer(&d_out, h_out, 0));
    CK(hipHostGetDevicePointer(&d_in, h_in, 0));
    run("pinned", h_in, (const uint32_t *)d_in, h_out, (uint32_t *)d_out, n);

    const unsigned flags[2] = {hipDeviceMallocFinegrained, hipDeviceMallocUncached};
    const char *names[2] = {"vram-fg", "vram-uc"};
    for (int k = 0; k < 2; ++k) {
        void *dv = nullptr;
        if (hipExtMallocWithFlags(&dv, 4096, flags[k]) != hipSuccess) {
            printf("%s: hipExtMallocWithFlags failed\n", names[k]);
            continue;
        }
        hipPointerAttribute_t at{};
        (void)hipPointerGetAttributes(&at, dv);
        printf("%s: device %p host %p\n", names[k], at.devicePointer, at.hostPointer);
        volatile uint32_t *hv = (volatile uint32_t *)(at.hostPointer != nullptr ? at.hostPointer : dv);
        struct sigaction sa{}, old{};
        sa.sa_handler = on_segv;
        sigaction(SIGSEGV, &sa, &old);
        bool ok = false;
        if (sigsetjmp(g_jb, 1) == 0) {
            hv[0] = 7;
            ok = hv[0] == 7;
        }
        sigaction(SIGSEGV, &old, nullptr);
        if (!ok) {
            printf("%s: the host cannot write this memory\n", names[k]);
            (void)hipFree(dv);
            continue;
        }
        run(names[k], hv, (const uint32_t *)dv, h_out, (uint32_t *)d_out, n);
        (void)hipFree(dv);
    }
    return 0;
}
