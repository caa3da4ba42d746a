/*
 * engine.cpp -- host side of the MI355X AES-GCM engine, part 1: errors, the AES T-table, engines (one per device: device
 * memory pool, chunk queues, the start-up self-check).  The other host units are listed in host.h.
 *
 * There is no CPU crypto fallback: without a usable gfx950 device the constructors fail
 * (setup_crypto returns -1 so ptls_aead_new returns NULL), and a device failure inside a
 * void callback (do_encrypt has no error channel) aborts the process with a message.
 */
#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "host.h"
/* ---------------------------------------------------------------------------------------------- */
/* errors                                                                                          */
/* ---------------------------------------------------------------------------------------------- */

thread_local std::string g_err;

int fail(int code, const char *fmt, ...)
{
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

extern "C" const char *ptls_hip_last_error(void)
{
    return g_err.c_str();
}

/* ---------------------------------------------------------------------------------------------- */
/* AES T-table: T0[x] = (2s, s, s, 3s) little-endian, s = S-box(x) (FIPS-197 §5.1.1, §5.1.3)        */
/* ---------------------------------------------------------------------------------------------- */

static uint8_t gf8_mul(uint8_t a, uint8_t b)
{
    uint8_t r = 0;
    for (; b; b >>= 1) {
        if (b & 1)
            r ^= a;
        a = (uint8_t)((a << 1) ^ ((a & 0x80) ? 0x1b : 0));
    }
    return r;
}

static void make_t0(uint32_t t0[256])
{
    /* multiplicative inverse by x^254, then the affine map */
    for (int x = 0; x < 256; ++x) {
        uint8_t inv = 1, base = (uint8_t)x;
        for (int e = 254; e; e >>= 1) {
            if (e & 1)
                inv = gf8_mul(inv, base);
            base = gf8_mul(base, base);
        }
        if (x == 0)
            inv = 0;
        uint8_t s = inv;
        for (int r = 1; r < 5; ++r)
            s ^= (uint8_t)((inv << r) | (inv >> (8 - r)));
        s ^= 0x63;
        const uint8_t s2 = gf8_mul(s, 2), s3 = gf8_mul(s, 3);
        t0[x] = (uint32_t)s2 | ((uint32_t)s << 8) | ((uint32_t)s << 16) | ((uint32_t)s3 << 24);
    }
}

/* Device memory of keysets and batches.  hipFree synchronizes the whole device, so it would wait for a resident plugin
 * worker (up to its lifetime) and for other threads' work; stream-ordered allocation on the engine's own stream does
 * not (the objects' users are waited for through their launch events, Uses below).  The allocations come from the
 * engine's OWN memory pool (the device's default pool belongs to the whole process: ADVICE r04), which keeps what is freed
 * into it (release threshold: never), since otherwise every stream-ordered free returns memory to the driver at the next
 * synchronization and the next allocation maps it again, which waits for the device like hipMalloc / hipFree do.
 * hipMalloc / hipFree where the runtime has no memory pools. */
static hipMemPool_t engine_pool_new(int device)
{
    int v = 0;
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeMemoryPoolsSupported, device) != hipSuccess || v == 0) {
        (void)hipGetLastError();
        return nullptr;
    }
    hipMemPoolProps props{};
    props.allocType = hipMemAllocationTypePinned;
    props.handleTypes = hipMemHandleTypeNone;
    props.location.type = hipMemLocationTypeDevice;
    props.location.id = device;
    hipMemPool_t pool = nullptr;
    if (hipMemPoolCreate(&pool, &props) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    uint64_t keep = UINT64_MAX;
    (void)hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &keep);
    (void)hipGetLastError();
    return pool;
}

hipError_t dev_alloc(ptls_hip_engine_t *e, void **p, size_t bytes)
{
    *p = nullptr;
    if (e->pool == nullptr)
        return hipMalloc(p, bytes);
    hipError_t r = hipMallocFromPoolAsync(p, bytes, e->pool, e->util);
    if (r == hipSuccess)
        r = hipStreamSynchronize(e->util); /* usable from any stream once the call returns */
    return r;
}

void dev_free(ptls_hip_engine_t *e, void *p)
{
    if (p == nullptr)
        return;
    if (e->pool == nullptr)
        (void)hipFree(p);
    else
        (void)hipFreeAsync(p, e->util);
}

/* the chunk-queue words of one batch-kernel launch (batch_kernel.h QUEUE): zero when handed out, and the launch leaves
 * them zero (its last workgroup resets them), so slots are reused round robin without a memset; QUEUE_SLOTS launches
 * would have to be in flight at once for two to share one */
uint32_t *queue_slot(ptls_hip_engine_t *e)
{
    return e->d_queue + 2 * (size_t)(e->queue_next.fetch_add(1, std::memory_order_relaxed) % e->queue_slots);
}

/* PTLS_HIP_QUEUE_SLOTS (environment, read when an engine is created): a smaller round robin, 1 .. QUEUE_SLOTS, so that a
 * test reuses every slot within a few launches and checks that each launch leaves its words reset
 * (tests/test_gpu_queue.py).  A TEST setting: with n slots, more than n launches in flight at once (several streams or
 * threads) would share a slot, and a sharing launch would skip chunks; so the shrunken ring is announced on stderr. */
static uint32_t queue_slots_env(void)
{
    const char *v = getenv("PTLS_HIP_QUEUE_SLOTS");
    const long n = v != nullptr ? atol(v) : 0;
    if (n >= 1 && n < (long)QUEUE_SLOTS) {
        fprintf(stderr, "ptls_hip: PTLS_HIP_QUEUE_SLOTS=%ld (test setting): at most %ld batch launches may be in flight on "
                        "one engine at a time\n", n, n);
        return (uint32_t)n;
    }
    return QUEUE_SLOTS;
}

extern "C" int ptls_hip_is_supported(void)
{
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess)
        return 0;
    for (int d = 0; d < ndev; ++d) {
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, d) == hipSuccess && std::strncmp(prop.gcnArchName, "gfx950", 6) == 0)
            return 1;
    }
    return 0;
}

static int engine_self_check(ptls_hip_engine_t *e);

extern "C" ptls_hip_engine_t *ptls_hip_engine_new(int device)
{
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
        fail(PTLS_HIP_ENODEV, "no HIP device available");
        return nullptr;
    }
    if (device < 0 || device >= ndev) {
        fail(PTLS_HIP_EINVAL, "device %d out of range (%d devices)", device, ndev);
        return nullptr;
    }
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) {
        fail(PTLS_HIP_ENODEV, "hipGetDeviceProperties failed");
        return nullptr;
    }
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
        fail(PTLS_HIP_ENODEV, "device %d is %s, this engine is built for gfx950 only", device, prop.gcnArchName);
        return nullptr;
    }
    DeviceGuard g(device);
    auto *e = new st_ptls_hip_engine_t();
    e->device = device;
    e->ncu = prop.multiProcessorCount;
    uint32_t t0[256];
    make_t0(t0);
    e->d_queue = nullptr;
    e->queue_next = 0;
    e->queue_slots = queue_slots_env();
    e->util = nullptr;
    e->pool = nullptr;
    if (hipMalloc(&e->d_t0, sizeof(t0)) != hipSuccess || hipMemcpy(e->d_t0, t0, sizeof(t0), hipMemcpyHostToDevice) != hipSuccess ||
        hipMalloc(&e->d_queue, 2 * sizeof(uint32_t) * QUEUE_SLOTS) != hipSuccess ||
        hipMemset(e->d_queue, 0, 2 * sizeof(uint32_t) * QUEUE_SLOTS) != hipSuccess ||
        hipStreamCreateWithFlags(&e->util, hipStreamNonBlocking) != hipSuccess) {
        fail(PTLS_HIP_ENOMEM, "cannot allocate the AES table / chunk queues on device %d", device);
        (void)hipFree(e->d_t0);
        (void)hipFree(e->d_queue);
        if (e->util != nullptr)
            (void)hipStreamDestroy(e->util);
        delete e;
        return nullptr;
    }
    e->pool = engine_pool_new(device);
    if (engine_self_check(e) != 0) {
        const std::string why = g_err;
        ptls_hip_engine_free(e);
        fail(PTLS_HIP_ENODEV, "device %d: engine self-check failed: %s", device, why.c_str());
        return nullptr;
    }
    return e;
}

extern "C" void ptls_hip_engine_free(ptls_hip_engine_t *e)
{
    if (e == nullptr)
        return;
    DeviceGuard g(e->device);
    (void)hipStreamSynchronize(e->util);
    (void)hipStreamDestroy(e->util);
    (void)hipFree(e->d_t0);
    (void)hipFree(e->d_queue);
    if (e->pool != nullptr) /* keysets and batches are freed before their engine (their frees are stream-ordered on util) */
        (void)hipMemPoolDestroy(e->pool);
    delete e;
}

extern "C" int ptls_hip_engine_device(ptls_hip_engine_t *e)
{
    return e->device;
}

extern "C" int ptls_hip_engine_cu_count(ptls_hip_engine_t *e)
{
    return e->ncu;
}

/* the achievable-HBM reference of bench.py's roofline: one 16-byte load and store per thread */
extern "C" int ptls_hip_device_copy(ptls_hip_engine_t *eng, void *dst, const void *src, size_t bytes, void *stream)
{
    if (eng == nullptr || dst == nullptr || src == nullptr || (bytes & 15) != 0 ||
        ((reinterpret_cast<uintptr_t>(dst) | reinterpret_cast<uintptr_t>(src)) & 15) != 0)
        return fail(PTLS_HIP_EINVAL, "device_copy: 16-byte aligned pointers and a multiple of 16 bytes");
    if (bytes == 0)
        return 0;
    DeviceGuard g(eng->device);
    if (bytes / 16 > (size_t)0xffffffffu * 256)
        return fail(PTLS_HIP_EINVAL, "device_copy: at most 2^32 - 1 workgroups of 4 KiB");
    const int e = launch_copy16(dst, src, bytes / 16, stream);
    return e != 0 ? fail(PTLS_HIP_ELAUNCH, "device_copy: launch failed: %s", hipGetErrorString((hipError_t)e)) : 0;
}

/* The reference's gcm_basic #2 (t/fusion.c:251-273: key 00 11 .. ff, iv 20 .. 31, AAD 0 .. 19, the 85 bytes of
 * "hello world\n" x 7 + NUL, seq 0) sealed through the wave-per-record kernel and the batch kernel at 8 and 32 lanes per
 * record (its windowed lane combination over H^1 .. H^8 and H^1 .. H^32), and opened back, whenever an engine starts: a
 * library that computes anything else (a probe build, a broken device) fails ptls_hip_engine_new instead of serving
 * records. */
static int engine_self_check(ptls_hip_engine_t *e)
{
    static const uint8_t key[16] = {0x00, 0x11, 0x22, 0x33, 0x44, 0x55, 0x66, 0x77, 0x88, 0x99, 0xaa, 0xbb, 0xcc, 0xdd, 0xee, 0xff};
    static const uint8_t expected[101] = {
        0xd3, 0xa8, 0x1d, 0x96, 0x4c, 0x9b, 0x02, 0xd7, 0x9a, 0xb0, 0x41, 0x07, 0x4c, 0x8c, 0xe2, 0xe0, 0x2e,
        0x83, 0x54, 0x52, 0x45, 0xcb, 0xd4, 0x68, 0xc8, 0x43, 0x45, 0xca, 0x91, 0xfb, 0xa3, 0x7a, 0x67, 0xed,
        0xe8, 0xd7, 0x5e, 0xe2, 0x33, 0xd1, 0x3e, 0xbf, 0x50, 0xc2, 0x4b, 0x86, 0x83, 0x55, 0x11, 0xbb, 0x17,
        0x4f, 0xf5, 0x78, 0xb8, 0x65, 0xeb, 0x9a, 0x2b, 0x8f, 0x77, 0x08, 0xa9, 0x60, 0x17, 0x73, 0xc5, 0x07,
        0xf3, 0x04, 0xc9, 0x3f, 0x67, 0x4d, 0x12, 0xa1, 0x02, 0x93, 0xc2, 0x3c, 0xd3, 0xf8, 0x59, 0x33, 0xd5,
        0x01, 0xc3, 0xbb, 0xaa, 0xe6, 0x3f, 0xbb, 0x23, 0x66, 0x94, 0x26, 0x28, 0x43, 0xa5, 0xfd, 0x2f};
    uint8_t iv[12], aad[20], pt[85], buf[512];
    for (int i = 0; i < 12; ++i)
        iv[i] = (uint8_t)(20 + i);
    for (int i = 0; i < 20; ++i)
        aad[i] = (uint8_t)i;
    for (int i = 0; i < 84; ++i)
        pt[i] = (uint8_t)"hello world\n"[i % 12];
    pt[84] = 0;
    /* device buffer: plaintext @0, AAD @128, sealed @256 (101 B), opened @384 (85 B), result @480 */
    ptls_hip_keyset_t *ks = ptls_hip_keyset_new(e, 16, 1);
    uint8_t *d = nullptr;
    int rc = ks == nullptr ? -1 : 0;
    if (rc == 0 && ptls_hip_keyset_set(ks, 0, 1, key, iv, nullptr) != 0)
        rc = -1;
    if (rc == 0 && hipMalloc(&d, sizeof(buf)) != hipSuccess)
        rc = fail(PTLS_HIP_ENOMEM, "self-check: no device memory");
    if (rc == 0) {
        std::memset(buf, 0, sizeof(buf));
        std::memcpy(buf, pt, sizeof(pt));
        std::memcpy(buf + 128, aad, sizeof(aad));
        if (hipMemcpy(d, buf, sizeof(buf), hipMemcpyHostToDevice) != hipSuccess)
            rc = fail(PTLS_HIP_ENODEV, "self-check: upload failed");
    }
    /* the single-record kernel the plugin launches (record by value), and the batch kernel at 8 and 32 lanes per record at
     * 512 threads per workgroup: not the instantiations a 768-thread batch launch uses, so the self-check leaves no small
     * dispatch in a profile of the batch kernels */
    static const int lanes[] = {SPARSE_LANES, 8, 32};
    for (int li = 0; rc == 0 && li < 3; ++li) {
        const ptls_hip_record_t seal{0, 256, 128, 0, 85, 20, 0, 0}, open{256, 384, 128, 0, 85, 20, 0, 0};
        bool ok = hipMemset(d + 256, 0, 256) == hipSuccess;
        if (lanes[li] == SPARSE_LANES) {
            for (int o = 0; ok && o < 2; ++o) {
                KernelArgs a{};
                a.one = o ? open : seal;
                a.in = a.aad = d;
                a.out = d;
                a.result = reinterpret_cast<uint64_t *>(d + 480);
                a.slots = ks->d_slots;
                a.basis = ks->d_basis;
                a.t0 = e->d_t0;
                ok = launch_batch(SPARSE_LANES, 10, o != 0, 0, 1, nullptr, a, true) == 0 && hipStreamSynchronize(nullptr) == hipSuccess;
            }
            ok = ok && hipMemcpy(buf, d, sizeof(buf), hipMemcpyDeviceToHost) == hipSuccess;
        } else {
            ptls_hip_batch_t *bs = ptls_hip_batch_new(e, &seal, 1, nullptr), *bo = ptls_hip_batch_new(e, &open, 1, nullptr);
            ok = ok && bs != nullptr && bo != nullptr && ptls_hip_batch_set_lanes(bs, lanes[li]) == 0 &&
                 ptls_hip_batch_set_lanes(bo, lanes[li]) == 0 && ptls_hip_batch_set_workgroup(bs, 512) == 0 &&
                 ptls_hip_batch_set_workgroup(bo, 512) == 0 && ptls_hip_aesgcm_seal_batch(bs, ks, d, d, d, nullptr) == 0 &&
                 ptls_hip_aesgcm_open_batch(bo, ks, d, d, d, reinterpret_cast<uint64_t *>(d + 480), nullptr) == 0 &&
                 hipMemcpy(buf, d, sizeof(buf), hipMemcpyDeviceToHost) == hipSuccess;
            ptls_hip_batch_free(bs);
            ptls_hip_batch_free(bo);
        }
        if (!ok) {
            rc = fail(PTLS_HIP_ENODEV, "self-check: launch failed (%s)", g_err.c_str());
        } else {
            uint64_t res = 0;
            std::memcpy(&res, buf + 480, 8);
            if (std::memcmp(buf + 256, expected, sizeof(expected)) != 0 || res != 85 || std::memcmp(buf + 384, pt, sizeof(pt)) != 0)
                rc = fail(PTLS_HIP_ENODEV, "gcm_basic (t/fusion.c:251-273) sealed or opened wrong at %d lanes per record", lanes[li]);
        }
    }
    if (d != nullptr) {
        (void)hipMemset(d, 0, sizeof(buf));
        (void)hipFree(d);
    }
    ptls_hip_keyset_free(ks);
    return rc;
}
