/*
 * engine.cpp -- host side of the MI355X AES-GCM engine: the C ABI of include/ptls_hip.h.
 *
 *   engines   one per device; owns the AES T0 table in HBM and the launch geometry
 *   keysets   device-resident AEAD contexts (KeySlot + GHASH basis), expanded on the GPU
 *   batches   uploaded record descriptors + the launch plan (key-homogeneous chunks, lanes/record)
 *   plugin    ptls_hip_aes{128,256}gcm: picotls ptls_aead_algorithm_t objects whose callbacks run one
 *             record through the same kernels (setup_crypto / do_encrypt / do_encrypt_v / do_decrypt /
 *             do_get_iv / do_set_iv / dispose_crypto, mirroring lib/fusion.c:1102-1256)
 *
 * There is no CPU crypto fallback: without a usable gfx950 device the constructors fail
 * (setup_crypto returns -1 so ptls_aead_new returns NULL), and a device failure inside a
 * void callback (do_encrypt has no error channel) aborts the process with a message.
 */
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <atomic>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <chrono>
#include <mutex>
#include <string>
#include <thread>

#include <pthread.h>
#include <sched.h>
#include <sys/mman.h>
#include <sys/syscall.h>
#include <unistd.h>
#include <vector>

#include "internal.h"

using namespace ptls_hip;

/* ---------------------------------------------------------------------------------------------- */
/* errors                                                                                          */
/* ---------------------------------------------------------------------------------------------- */

static thread_local std::string g_err;

static int fail(int code, const char *fmt, ...)
{
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

#define HIP_TRY(expr, code)                                                                                                        \
    do {                                                                                                                           \
        hipError_t e_ = (expr);                                                                                                    \
        if (e_ != hipSuccess)                                                                                                      \
            return fail((code), "%s failed: %s", #expr, hipGetErrorString(e_));                                                  \
    } while (0)

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

/* ---------------------------------------------------------------------------------------------- */
/* objects                                                                                         */
/* ---------------------------------------------------------------------------------------------- */

struct st_ptls_hip_engine_t {
    int device;
    int ncu;
    uint32_t *d_t0;
    uint32_t *d_queue;                /* QUEUE_SLOTS x {next chunk, workgroups done}: the batch kernel's chunk queues */
    std::atomic<uint32_t> queue_next; /* the slot the next batch launch takes */
    uint32_t queue_slots;             /* slots in the round robin: QUEUE_SLOTS (PTLS_HIP_QUEUE_SLOTS: fewer, for tests) */
    hipStream_t util;                 /* descriptor / keyset allocation, zeroing and release (dev_alloc / dev_free) */
    hipMemPool_t pool;                /* the engine's own device memory pool (dev_alloc), or nullptr: hipMalloc */
};

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

static hipError_t dev_alloc(ptls_hip_engine_t *e, void **p, size_t bytes)
{
    *p = nullptr;
    if (e->pool == nullptr)
        return hipMalloc(p, bytes);
    hipError_t r = hipMallocFromPoolAsync(p, bytes, e->pool, e->util);
    if (r == hipSuccess)
        r = hipStreamSynchronize(e->util); /* usable from any stream once the call returns */
    return r;
}

static void dev_free(ptls_hip_engine_t *e, void *p)
{
    if (p == nullptr)
        return;
    if (e->pool == nullptr)
        (void)hipFree(p);
    else
        (void)hipFreeAsync(p, e->util);
}

/* the streams launches on an object went to, each with an event recorded after its last such launch: freeing the object
 * (or re-planning a batch) waits for exactly that work */
struct Uses {
    std::mutex mu;
    std::vector<std::pair<hipStream_t, hipEvent_t>> v;

    void note(void *stream)
    {
        hipStream_t st = static_cast<hipStream_t>(stream);
        std::lock_guard<std::mutex> lk(mu);
        for (auto &u : v)
            if (u.first == st) {
                (void)hipEventRecord(u.second, st);
                return;
            }
        hipEvent_t ev = nullptr;
        if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) == hipSuccess && hipEventRecord(ev, st) == hipSuccess)
            v.emplace_back(st, ev);
        else /* no event: the wait falls back to the whole device */
            v.emplace_back(st, nullptr);
    }

    void wait()
    {
        std::lock_guard<std::mutex> lk(mu);
        bool device_wide = false;
        for (auto &u : v) {
            if (u.second == nullptr) {
                device_wide = true;
                continue;
            }
            (void)hipEventSynchronize(u.second);
        }
        if (device_wide)
            (void)hipDeviceSynchronize();
    }

    ~Uses()
    {
        for (auto &u : v)
            if (u.second != nullptr)
                (void)hipEventDestroy(u.second);
    }
};

/* the chunk-queue words of one batch-kernel launch (batch_kernel.h QUEUE): zero when handed out, and the launch leaves
 * them zero (its last workgroup resets them), so slots are reused round robin without a memset; QUEUE_SLOTS launches
 * would have to be in flight at once for two to share one */
static uint32_t *queue_slot(ptls_hip_engine_t *e)
{
    return e->d_queue + 2 * (size_t)(e->queue_next.fetch_add(1, std::memory_order_relaxed) % e->queue_slots);
}

/* PTLS_HIP_QUEUE_SLOTS (environment, read when an engine is created): a smaller round robin, 1 .. QUEUE_SLOTS, so that a
 * test reuses every slot within a few launches and checks that each launch leaves its words reset
 * (tests/test_gpu_queue.py) */
static uint32_t queue_slots_env(void)
{
    const char *v = getenv("PTLS_HIP_QUEUE_SLOTS");
    const long n = v != nullptr ? atol(v) : 0;
    return n >= 1 && n <= (long)QUEUE_SLOTS ? (uint32_t)n : QUEUE_SLOTS;
}

struct st_ptls_hip_keyset_t {
    ptls_hip_engine_t *eng;
    size_t key_size, nslots;
    KeySlot *d_slots;
    uint32_t *d_basis;
    std::vector<uint8_t> ivs; /* host mirror of every slot's static IV (do_get_iv) */
    int64_t pool_id = -1;     /* >= 0: a plugin context's slot from the plugin pool (pool_keyset), not its own allocation */
    Uses uses; /* launches that read this keyset: keyset_free waits for exactly that work */
};

/* after a launch on `stream` that reads ks */
static void keyset_note_use(ptls_hip_keyset_t *ks, void *stream)
{
    if (ks != nullptr && ks->pool_id < 0)
        ks->uses.note(stream);
}

struct st_ptls_hip_batch_t {
    ptls_hip_engine_t *eng;
    size_t n;
    ptls_hip_record_t *d_recs;
    ptls_hip_record_t *d_recs_ord; /* descriptors in chunk order (the batch kernel's view) */
    std::vector<ptls_hip_record_t> h_recs;
    Chunk *d_chunks;
    uint32_t *d_order;
    uint32_t nchunks;
    int lanes;      /* in use */
    int wg;         /* threads per workgroup */
    int forced_wg;  /* 0 = plan_wg */
    bool all_aligned; /* every descriptor's in/out/aad offset is a multiple of 16 */
    int auto_lanes; /* chosen from the record lengths */
    bool forced;
    uint32_t max_key; /* largest key slot any record names (checked against the keyset at seal/open) */
    unsigned max_wg;  /* 0, or a cap on the workgroups of a launch (planning then sizes chunks for that many) */
    uint64_t *d_clk;  /* diagnostic clock stamps of the next launches (ptls_hip_batch_set_clock), or nullptr */
    size_t clk_bytes;
    Uses uses;        /* launches that read the descriptors and the plan: re-planning and batch_free wait for them */
};

/* CUs a batch is planned and launched for: the device's, or fewer when the batch caps its grid */
static unsigned batch_cus(const st_ptls_hip_batch_t *b)
{
    const unsigned ncu = (unsigned)b->eng->ncu;
    return b->max_wg != 0 && b->max_wg < ncu ? b->max_wg : ncu;
}

class DeviceGuard {
  public:
    explicit DeviceGuard(int dev)
    {
        (void)hipGetDevice(&prev_);
        if (prev_ != dev)
            (void)hipSetDevice(dev);
        dev_ = dev;
    }
    ~DeviceGuard()
    {
        if (prev_ != dev_)
            (void)hipSetDevice(prev_);
    }

  private:
    int prev_ = 0, dev_ = 0;
};

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

/* ---------------------------------------------------------------------------------------------- */
/* keysets                                                                                         */
/* ---------------------------------------------------------------------------------------------- */

static const size_t BASIS_WORDS_PER_SLOT = (size_t)BASIS_VECS * 4;

extern "C" ptls_hip_keyset_t *ptls_hip_keyset_new(ptls_hip_engine_t *eng, size_t key_size, size_t nslots)
{
    if (eng == nullptr || (key_size != 16 && key_size != 32) || nslots == 0 || nslots > 0xffffffffu) {
        fail(PTLS_HIP_EINVAL, "keyset_new: bad arguments (key_size %zu, nslots %zu)", key_size, nslots);
        return nullptr;
    }
    DeviceGuard g(eng->device);
    auto *ks = new st_ptls_hip_keyset_t();
    ks->eng = eng;
    ks->key_size = key_size;
    ks->nslots = nslots;
    ks->ivs.assign(nslots * 12, 0);
    if (dev_alloc(eng, reinterpret_cast<void **>(&ks->d_slots), nslots * sizeof(KeySlot)) != hipSuccess ||
        dev_alloc(eng, reinterpret_cast<void **>(&ks->d_basis), nslots * BASIS_WORDS_PER_SLOT * 4) != hipSuccess) {
        fail(PTLS_HIP_ENOMEM, "keyset_new: cannot allocate %zu key slots", nslots);
        dev_free(eng, ks->d_slots);
        dev_free(eng, ks->d_basis);
        delete ks;
        return nullptr;
    }
    (void)hipMemsetAsync(ks->d_slots, 0, nslots * sizeof(KeySlot), eng->util);
    (void)hipStreamSynchronize(eng->util);
    return ks;
}

static void pool_release(ptls_hip_keyset_t *ks); /* plugin section */

extern "C" void ptls_hip_keyset_free(ptls_hip_keyset_t *ks)
{
    if (ks == nullptr)
        return;
    DeviceGuard g(ks->eng->device);
    if (ks->pool_id >= 0) { /* a plugin context's pooled slot: zeroed and retired, nothing waits */
        pool_release(ks);
        std::fill(ks->ivs.begin(), ks->ivs.end(), 0);
        delete ks;
        return;
    }
    /* the launches that read this keyset (keyset_note_use), not the whole device: a resident plugin worker or another
     * thread's batches are not waited for */
    ks->uses.wait();
    /* zeroize key material before release (ptls_clear_memory in aesgcm_dispose_crypto, lib/fusion.c:1102-1107, :1042-1048),
     * then release in the same stream order */
    ptls_hip_engine_t *e = ks->eng;
    (void)hipMemsetAsync(ks->d_slots, 0, ks->nslots * sizeof(KeySlot), e->util);
    (void)hipMemsetAsync(ks->d_basis, 0, ks->nslots * BASIS_WORDS_PER_SLOT * 4, e->util);
    dev_free(e, ks->d_slots);
    dev_free(e, ks->d_basis);
    (void)hipStreamSynchronize(e->util);
    std::fill(ks->ivs.begin(), ks->ivs.end(), 0);
    delete ks;
}

extern "C" size_t ptls_hip_keyset_size(ptls_hip_keyset_t *ks)
{
    return ks->nslots;
}

extern "C" int ptls_hip_keyset_set(ptls_hip_keyset_t *ks, size_t first, size_t count, const void *keys, const void *ivs,
                                   void *stream)
{
    if (ks == nullptr || keys == nullptr || first + count > ks->nslots)
        return fail(PTLS_HIP_EINVAL, "keyset_set: bad arguments");
    if (count == 0)
        return 0;
    std::vector<uint8_t> zero_ivs;
    if (ivs == nullptr) { /* header-protection / ECB-only keys carry no IV */
        zero_ivs.assign(count * 12, 0);
        ivs = zero_ivs.data();
    }
    DeviceGuard g(ks->eng->device);
    hipStream_t s = static_cast<hipStream_t>(stream);
    uint8_t *d_tmp = nullptr;
    const size_t kbytes = count * ks->key_size, ibytes = count * 12;
    /* stream-ordered (dev_alloc): a hipMalloc / hipFree pair would wait for all device work, a resident plugin worker
     * included */
    HIP_TRY(dev_alloc(ks->eng, reinterpret_cast<void **>(&d_tmp), kbytes + ibytes), PTLS_HIP_ENOMEM);
    int rc = 0;
    if (hipMemcpyAsync(d_tmp, keys, kbytes, hipMemcpyHostToDevice, s) != hipSuccess ||
        hipMemcpyAsync(d_tmp + kbytes, ivs, ibytes, hipMemcpyHostToDevice, s) != hipSuccess) {
        rc = fail(PTLS_HIP_ENODEV, "keyset_set: upload failed");
    } else {
        int e = launch_keysetup(ks->d_slots, ks->d_basis, d_tmp, d_tmp + kbytes, (uint32_t)first, (uint32_t)count,
                                (int)ks->key_size, ks->eng->d_t0, stream);
        if (e != 0)
            rc = fail(PTLS_HIP_ELAUNCH, "keyset_set: key setup launch failed: %s", hipGetErrorString((hipError_t)e));
        else if (hipStreamSynchronize(s) != hipSuccess)
            rc = fail(PTLS_HIP_ENODEV, "keyset_set: key setup failed");
    }
    /* raw keys do not stay in device memory outside the expanded slots: the scrub is ordered after the
     * uploads and the key setup on the same stream, whatever path got here */
    (void)hipMemsetAsync(d_tmp, 0, kbytes + ibytes, s);
    (void)hipStreamSynchronize(s);
    dev_free(ks->eng, d_tmp); /* after the scrub: the stream was synchronized */
    if (rc == 0)
        std::memcpy(&ks->ivs[first * 12], ivs, ibytes);
    return rc;
}

/* TLS 1.3 traffic secrets -> key slots, optionally after the key-update step (keyschedule.hip) */
static int keyset_from_secrets(ptls_hip_keyset_t *ks, size_t first, size_t count, void *secrets, size_t hash_size, void *stream,
                               bool update)
{
    if (ks == nullptr || secrets == nullptr || first + count > ks->nslots || !(hash_size == 32 || hash_size == 48) ||
        count > 0xffffffffu)
        return fail(PTLS_HIP_EINVAL, "keyset_%s_secrets: bad arguments", update ? "update" : "set");
    if (count == 0)
        return 0;
    DeviceGuard g(ks->eng->device);
    hipStream_t s = static_cast<hipStream_t>(stream);
    const size_t sbytes = count * hash_size, kbytes = count * ks->key_size, ibytes = count * 12;
    uint8_t *d = nullptr;
    HIP_TRY(dev_alloc(ks->eng, reinterpret_cast<void **>(&d), 2 * sbytes + kbytes + ibytes), PTLS_HIP_ENOMEM);
    uint8_t *d_sec = d, *d_next = d + sbytes, *d_keys = d + 2 * sbytes, *d_ivs = d + 2 * sbytes + kbytes;
    std::vector<uint8_t> h_ivs(ibytes);
    int rc = 0;
    if (hipMemcpyAsync(d_sec, secrets, sbytes, hipMemcpyHostToDevice, s) != hipSuccess) {
        rc = fail(PTLS_HIP_ENODEV, "keyset secrets: upload failed");
    } else if (int e = launch_derive_traffic_keys(d_sec, update ? d_next : nullptr, (uint32_t)count, (int)hash_size,
                                                  (int)ks->key_size, update ? 1 : 0, d_keys, d_ivs, stream)) {
        rc = fail(PTLS_HIP_ELAUNCH, "keyset secrets: derive launch failed: %s", hipGetErrorString((hipError_t)e));
    } else if (int e2 = launch_keysetup(ks->d_slots, ks->d_basis, d_keys, d_ivs, (uint32_t)first, (uint32_t)count,
                                        (int)ks->key_size, ks->eng->d_t0, stream)) {
        rc = fail(PTLS_HIP_ELAUNCH, "keyset secrets: key setup launch failed: %s", hipGetErrorString((hipError_t)e2));
    } else if (hipMemcpyAsync(h_ivs.data(), d_ivs, ibytes, hipMemcpyDeviceToHost, s) != hipSuccess ||
               (update && hipMemcpyAsync(secrets, d_next, sbytes, hipMemcpyDeviceToHost, s) != hipSuccess) ||
               hipStreamSynchronize(s) != hipSuccess) {
        rc = fail(PTLS_HIP_ENODEV, "keyset secrets: derivation failed");
    }
    /* secrets and raw keys do not stay in device memory outside the expanded slots */
    (void)hipMemsetAsync(d, 0, 2 * sbytes + kbytes + ibytes, s);
    (void)hipStreamSynchronize(s);
    dev_free(ks->eng, d); /* after the scrub: the stream was synchronized */
    if (rc == 0)
        std::memcpy(&ks->ivs[first * 12], h_ivs.data(), ibytes);
    std::fill(h_ivs.begin(), h_ivs.end(), 0);
    return rc;
}

extern "C" int ptls_hip_keyset_set_secrets(ptls_hip_keyset_t *ks, size_t first, size_t count, const void *secrets, size_t hash_size,
                                           void *stream)
{
    return keyset_from_secrets(ks, first, count, const_cast<void *>(secrets), hash_size, stream, false);
}

extern "C" int ptls_hip_keyset_update_secrets(ptls_hip_keyset_t *ks, size_t first, size_t count, void *secrets, size_t hash_size,
                                              void *stream)
{
    return keyset_from_secrets(ks, first, count, secrets, hash_size, stream, true);
}

extern "C" int ptls_hip_keyset_get_iv(ptls_hip_keyset_t *ks, size_t slot, void *iv)
{
    if (ks == nullptr || slot >= ks->nslots)
        return fail(PTLS_HIP_EINVAL, "keyset_get_iv: bad slot");
    std::memcpy(iv, &ks->ivs[slot * 12], 12);
    return 0;
}

extern "C" int ptls_hip_keyset_set_iv(ptls_hip_keyset_t *ks, size_t slot, const void *iv, void *stream)
{
    if (ks == nullptr || slot >= ks->nslots)
        return fail(PTLS_HIP_EINVAL, "keyset_set_iv: bad slot");
    DeviceGuard g(ks->eng->device);
    std::memcpy(&ks->ivs[slot * 12], iv, 12);
    hipStream_t s = static_cast<hipStream_t>(stream);
    HIP_TRY(hipMemcpyAsync(&ks->d_slots[slot].iv, &ks->ivs[slot * 12], 12, hipMemcpyHostToDevice, s), PTLS_HIP_ENODEV);
    HIP_TRY(hipStreamSynchronize(s), PTLS_HIP_ENODEV);
    return 0;
}

extern "C" int ptls_hip_keyset_xor_iv(ptls_hip_keyset_t *ks, size_t slot, const void *bytes, size_t len, void *stream)
{
    if (ks == nullptr || slot >= ks->nslots || len > 12)
        return fail(PTLS_HIP_EINVAL, "keyset_xor_iv: bad arguments");
    uint8_t iv[12];
    std::memcpy(iv, &ks->ivs[slot * 12], 12);
    for (size_t i = 0; i < len; ++i)
        iv[i] ^= static_cast<const uint8_t *>(bytes)[i];
    return ptls_hip_keyset_set_iv(ks, slot, iv, stream);
}

/* ---------------------------------------------------------------------------------------------- */
/* batches                                                                                         */
/* ---------------------------------------------------------------------------------------------- */

/* lanes per record from the mean GHASH length N = ceil(A/16) + ceil(L/16) + 1: keep >= ~16 Horner
 * steps per lane so the log2(G) reduction tree stays a small fraction of the work.  Many keys with few
 * records each (a server's connections): a workgroup works on one key at a time (its GHASH tables fill
 * the LDS), so with 8 lanes a 64-record key run gives only 8 wave tasks to 12 waves; 16 lanes per
 * record doubles the tasks per key run (measured on the 64K-key BASELINE shape). */
static int choose_lanes(const ptls_hip_record_t *recs, size_t n, unsigned ncu)
{
    if (n == 0)
        return 1;
    double sum = 0;
    size_t runs = 1;
    for (size_t i = 0; i < n; ++i) {
        sum += (double)((recs[i].aad_len + 15) / 16 + (recs[i].len + 15) / 16 + 1);
        if (i != 0 && recs[i].key != recs[i - 1].key)
            ++runs;
    }
    const double mean = sum / (double)n;
    const double per_run = (double)n / (double)runs;
    /* round 4 (the windowed lane combination for every G, batch_kernel.h WIN_ALL): G = 4 is as fast as G = 8 or faster at
     * every length with long key runs (seal GiB/s G = 4 / 8, same box, tools/calls_r04/r04_call28.sh: 3 000 B 1 183 / 1 151,
     * 4 096 B 1 220 / 1 188, 8 192 B 1 215 / 1 222, c2's 16 KiB 1 258 / 1 250; 2 000 B 1 154-1 163 / 1 101; c3 G = 2 / 4
     * within 1 %).  Until then G = 8 from 128 GHASH elements (the tree's cost grew with log2 G differently) */
    const int g = mean >= 48 ? 4 : mean >= 16 ? 2 : 1;
    /* key runs too short to amortise the per-key GHASH tables: the key-independent wave-per-record kernel */
    if (per_run < SPARSE_MAX_PER_RUN)
        return SPARSE_LANES;
    /* long records, short key runs: more lanes per record give a key run more wave tasks for the workgroup's 12
     * waves, as long as the run fits one chunk (2 * 16 * 64 / G records): a run spilling into a second chunk costs up to
     * 25 %.  Measured on configs[3]'s lengths (AES-256, 64 B - 16 KiB, 4M records; tools/time_cfg.py), seal
     * GiB/s at 8 / 16 / 32 lanes, round 3 (the G = 32 window combination): 64 records per key 532 / 769 / 803, 96: 748 /
     * 813 / 620, 128: 810 / 827 / 804, 192: 838 / 644 / 806 (tools/calls_r03/r03_call17.sh); round 2 at 16 / 32 lanes
     * (sparse kernel): 8 per key 126 / 258 (503), 16: 260 / 499 (516), 24: 394 / 681 (525), 32: 518 / 715, 48: 717 / 734. */
    if (mean >= 256 && per_run <= 64)
        return 32;
    if (mean >= 256 && per_run <= 128)
        return 16;
    /* a run of up to 320 records is at most 20 wave tasks at G = 4 for 12 waves: G = 8 doubles them.  c4's lengths, seal
     * GiB/s G = 4 / 8 / 16 (tools/calls_r04/r04_call26.sh, r04_call30.sh): ~210 records per key 822 / 893 / 851, ~420 per
     * key 898 / 869 / -, one key 932 / 927 / - */
    if (mean >= 256 && per_run <= 320)
        return 8;
    /* Small batches: a launch gives each CU 12 waves that draw wave tasks of 64/G records, so a batch of fewer than
     * about two tasks per wave leaves most waves idle or waiting for one long last task.  More lanes per record make
     * more, shorter tasks, as long as each lane keeps >= 8 GHASH elements.  Round 5, same box, seal GiB/s at G = 4 / 8 /
     * 16 / 32 (tools/calls_r05/r05_call11.sh): c2's 16 KiB records, 4 096 records (64 MiB) 206 / 321 / 457 / 542,
     * 16 384 573-590 / 682-693 / 872-973 / 885-900, 65 536 981-997 / 983-989 / 974-990 / 938-966, 262 144 1 172-1 176 /
     * 1 179 / 1 173-1 176 / 1 144-1 149; c3's 1 350 B records at G = 2 / 4 / 8: 65 536 records 575 / 655-669 / 700-707,
     * 786 432 893-904 / 906-910 / 860-864. */
    int gs = g;
    const double waves = 12.0 * (double)(ncu ? ncu : 256);
    while (gs < 32 && (double)n * gs / 64.0 < 2.0 * waves && mean / (2.0 * gs) >= 8.0)
        gs *= 2;
    return gs;
}

/* grid of a launch: one workgroup per CU at most (both kernels fill the LDS); the batch kernel takes one
 * workgroup per chunk, the sparse kernel one per 12 records (a record per wave) */
static unsigned plan_grid(size_t n, size_t nchunks, int lanes, unsigned ncu)
{
    if (lanes == SPARSE_LANES)
        return (unsigned)std::max<size_t>(1, std::min<size_t>((n + 11) / 12, (size_t)ncu));
    return (unsigned)std::min<size_t>(nchunks, ncu);
}

static int plan_wg(const std::vector<Chunk> &ch, int lanes)
{
    /* Measured on MI355X (tools/tune.py, same-process sweep): 768 threads = 3 waves per SIMD at 168 VGPRs
     * (no spills for G <= 4) beats 512 (2 waves, 193 VGPRs) on every BASELINE shape: 1M x 16 KiB 1033 vs
     * 968 GiB/s seal, 4M x 1350 B 864 vs 788, 64K keys 416 vs 415; 1024 threads spills and loses to both. */
    (void)ch;
    (void)lanes;
    return WG_ALT;
}

/* Guided chunk sizes at the end of long key runs (batch_kernel.h QUEUE hands chunks out in plan order).  A workgroup's
 * last chunk ends the launch for it, so the chunks dealt last should be small: a chunk that starts when `rem` wave tasks
 * remain in the batch gets at most rem / (2 ncu) tasks (at least one), like guided self-scheduling.  Only chunks of key
 * runs longer than one full chunk are cut (configs[1], [2], [4]): a short run's pieces would each rebuild the key's GHASH
 * tables on another workgroup, and such batches already balance over many runs.  The records of a chunk stay in their
 * length-sorted order, so each piece is a contiguous, sorted range. */
static void guided_tail(std::vector<Chunk> &ch, uint32_t per_task, unsigned ncu)
{
    static const bool on = [] { /* PTLS_HIP_GUIDED=0 (environment): full-size chunks to the end (A/B measurements) */
        const char *e = getenv("PTLS_HIP_GUIDED");
        return e == nullptr || atoi(e) != 0;
    }();
    if (!on)
        return;
    size_t total = 0;
    for (const Chunk &c : ch)
        total += (c.count + per_task - 1) / per_task;
    std::vector<Chunk> out;
    out.reserve(ch.size() + 4 * (size_t)ncu);
    size_t done = 0;
    for (size_t k = 0; k < ch.size(); ++k) {
        Chunk c = ch[k];
        const bool long_run = (k > 0 && ch[k - 1].key == c.key) || (k + 1 < ch.size() && ch[k + 1].key == c.key);
        size_t tasks = (c.count + per_task - 1) / per_task;
        while (long_run && tasks > 1) {
            const size_t want = std::max<size_t>(1, (total - done) / (2 * (size_t)ncu));
            if (want >= tasks)
                break;
            Chunk piece = c;
            piece.count = (uint32_t)(want * per_task);
            out.push_back(piece);
            c.first += piece.count;
            c.count -= piece.count;
            done += want;
            tasks -= want;
        }
        done += tasks;
        out.push_back(c);
    }
    ch.swap(out);
}

/* chunk = run of records with one key slot, sized to keep all waves of a workgroup busy for a few tasks
 * (at most 32 wave tasks), but small enough that a batch of fewer tasks still spreads over every CU (the
 * grid is one workgroup per chunk up to the CU count).  Inside a chunk the records are ordered by
 * decreasing length, so the 64/lanes records a wave processes together have similar lengths (their
 * branch-free full-block stretch is limited by the shortest). */
static void build_chunks(const ptls_hip_record_t *recs, size_t n, int lanes, unsigned ncu, std::vector<Chunk> &ch,
                         std::vector<uint32_t> &order, bool &all_aligned)
{
    ch.clear();
    order.resize(n);
    all_aligned = true;
    if (lanes == SPARSE_LANES) {
        /* the sparse kernel keeps no per-key workgroup state and its waves take records grid-stride: in
         * decreasing length over the whole batch every wave gets a similar share of bytes.  One chunk holds
         * the record count (the kernel reads nothing else from it); its key field names no slot. */
        bool sorted = true;
        uint32_t max_len = 0;
        for (size_t i = 0; i < n; ++i) {
            order[i] = (uint32_t)i;
            if (((recs[i].in_off | recs[i].out_off | recs[i].aad_off) & 15) != 0)
                all_aligned = false;
            if (i != 0 && recs[i].len > recs[i - 1].len)
                sorted = false;
            max_len = std::max(max_len, recs[i].len);
        }
        /* (the host plans every slice of a host-resident pipeline while the device runs the previous one: a comparison
         * sort of ~200K QUIC records per slice took longer than the slice's kernel) */
        if (!sorted && max_len < (1u << 24)) {
            /* stable counting sort by decreasing 16-byte block count: the kernel balances GHASH elements, not bytes */
            const uint32_t nb = (max_len >> 4) + 1;
            std::vector<uint32_t> start(nb + 1, 0);
            for (size_t i = 0; i < n; ++i)
                ++start[nb - 1 - (recs[i].len >> 4) + 1];
            for (uint32_t b = 0; b < nb; ++b)
                start[b + 1] += start[b];
            for (size_t i = 0; i < n; ++i)
                order[start[nb - 1 - (recs[i].len >> 4)]++] = (uint32_t)i;
        } else if (!sorted) {
            std::stable_sort(order.begin(), order.end(), [&](uint32_t x, uint32_t y) { return recs[x].len > recs[y].len; });
        }
        if (n != 0)
            ch.push_back(Chunk{0, (uint32_t)n, 0xffffffffu, all_aligned ? 1u : 0u});
        return;
    }
    const uint32_t per_task = 64u / (uint32_t)lanes;
    const size_t tasks = (n + per_task - 1) / per_task;
    const size_t spread = (tasks + (ncu ? ncu : 1) - 1) / (ncu ? ncu : 1); /* tasks per chunk for >= ncu chunks */
    const uint32_t max_chunk = per_task * (uint32_t)std::max<size_t>(1, std::min<size_t>((WG_MAX / 64) * 2, spread));
    size_t i = 0;
    while (i < n) {
        Chunk c;
        c.first = (uint32_t)i;
        c.key = recs[i].key;
        c.count = 0;
        c.flags = 1;
        bool sorted = true;
        while (i < n && recs[i].key == c.key && c.count < max_chunk) {
            if (((recs[i].in_off | recs[i].out_off | recs[i].aad_off) & 15) != 0)
                c.flags = 0;
            if (c.count != 0 && recs[i].len > recs[i - 1].len)
                sorted = false;
            order[i] = (uint32_t)i;
            ++c.count;
            ++i;
        }
        if (!sorted)
            std::stable_sort(order.begin() + c.first, order.begin() + c.first + c.count,
                             [&](uint32_t x, uint32_t y) { return recs[x].len > recs[y].len; });
        all_aligned = all_aligned && (c.flags & 1u);
        ch.push_back(c);
    }
    guided_tail(ch, per_task, ncu ? ncu : 1);
}

static bool identity_order(const std::vector<uint32_t> &order, size_t n);

/* When the plan keeps the caller's order (equal lengths per key run, or already non-increasing: configs[1], [2], [4]),
 * the kernels read the caller-order descriptors and no order array (record index = plan position): no second copy of
 * the descriptors in HBM and 4 bytes per record less to read per launch. */
static int plan_chunks(ptls_hip_batch_t *b)
{
    std::vector<Chunk> ch;
    std::vector<uint32_t> order;
    build_chunks(b->h_recs.data(), b->n, b->lanes, batch_cus(b), ch, order, b->all_aligned);
    b->wg = b->forced_wg ? b->forced_wg : plan_wg(ch, b->lanes);
    b->uses.wait(); /* an earlier launch may still read the old plan */
    dev_free(b->eng, b->d_chunks);
    dev_free(b->eng, b->d_order);
    dev_free(b->eng, b->d_recs_ord);
    b->d_chunks = nullptr;
    b->d_order = nullptr;
    b->d_recs_ord = nullptr;
    b->nchunks = (uint32_t)ch.size();
    if (ch.empty())
        return 0;
    HIP_TRY(dev_alloc(b->eng, reinterpret_cast<void **>(&b->d_chunks), ch.size() * sizeof(Chunk)), PTLS_HIP_ENOMEM);
    HIP_TRY(hipMemcpy(b->d_chunks, ch.data(), ch.size() * sizeof(Chunk), hipMemcpyHostToDevice), PTLS_HIP_ENODEV);
    if (identity_order(order, order.size()))
        return 0; /* d_order and d_recs_ord stay null: run_batch passes d_recs and no order */
    HIP_TRY(dev_alloc(b->eng, reinterpret_cast<void **>(&b->d_order), order.size() * sizeof(uint32_t)), PTLS_HIP_ENOMEM);
    HIP_TRY(hipMemcpy(b->d_order, order.data(), order.size() * sizeof(uint32_t), hipMemcpyHostToDevice), PTLS_HIP_ENODEV);
    std::vector<ptls_hip_record_t> ord(order.size());
    for (size_t k = 0; k < order.size(); ++k)
        ord[k] = b->h_recs[order[k]];
    HIP_TRY(dev_alloc(b->eng, reinterpret_cast<void **>(&b->d_recs_ord), ord.size() * sizeof(ptls_hip_record_t)), PTLS_HIP_ENOMEM);
    HIP_TRY(hipMemcpy(b->d_recs_ord, ord.data(), ord.size() * sizeof(ptls_hip_record_t), hipMemcpyHostToDevice), PTLS_HIP_ENODEV);
    return 0;
}

extern "C" ptls_hip_batch_t *ptls_hip_batch_new(ptls_hip_engine_t *eng, const ptls_hip_record_t *recs, size_t n, void *stream)
{
    (void)stream;
    if (eng == nullptr || (recs == nullptr && n != 0) || n > 0xffffffffu) {
        fail(PTLS_HIP_EINVAL, "batch_new: bad arguments");
        return nullptr;
    }
    DeviceGuard g(eng->device);
    auto *b = new st_ptls_hip_batch_t();
    b->eng = eng;
    b->n = n;
    b->h_recs.assign(recs, recs + n);
    b->max_key = 0;
    for (size_t i = 0; i < n; ++i)
        b->max_key = std::max(b->max_key, recs[i].key);
    b->auto_lanes = b->lanes = choose_lanes(b->h_recs.data(), b->h_recs.size(), (unsigned)eng->ncu);
    if (n != 0) {
        if (dev_alloc(eng, reinterpret_cast<void **>(&b->d_recs), n * sizeof(ptls_hip_record_t)) != hipSuccess ||
            hipMemcpy(b->d_recs, recs, n * sizeof(ptls_hip_record_t), hipMemcpyHostToDevice) != hipSuccess) {
            fail(PTLS_HIP_ENOMEM, "batch_new: cannot upload %zu descriptors", n);
            dev_free(eng, b->d_recs);
            (void)hipStreamSynchronize(eng->util);
            delete b;
            return nullptr;
        }
    }
    if (plan_chunks(b) != 0) {
        ptls_hip_batch_free(b);
        return nullptr;
    }
    return b;
}

extern "C" void ptls_hip_batch_free(ptls_hip_batch_t *b)
{
    if (b == nullptr)
        return;
    DeviceGuard g(b->eng->device);
    b->uses.wait();
    dev_free(b->eng, b->d_recs);
    dev_free(b->eng, b->d_recs_ord);
    dev_free(b->eng, b->d_chunks);
    dev_free(b->eng, b->d_order);
    (void)hipStreamSynchronize(b->eng->util);
    delete b;
}

extern "C" size_t ptls_hip_batch_count(ptls_hip_batch_t *b)
{
    return b->n;
}

extern "C" int ptls_hip_batch_set_lanes(ptls_hip_batch_t *b, int lanes)
{
    if (b == nullptr ||
        !(lanes == 0 || lanes == 1 || lanes == 2 || lanes == 4 || lanes == 8 || lanes == 16 || lanes == 32 || lanes == SPARSE_LANES))
        return fail(PTLS_HIP_EINVAL, "batch_set_lanes: lanes must be 0, 1, 2, 4, 8, 16, 32 or 64");
    DeviceGuard g(b->eng->device);
    const int want = lanes == 0 ? b->auto_lanes : lanes;
    if (want == b->lanes)
        return 0;
    b->lanes = want;
    return plan_chunks(b);
}

extern "C" int ptls_hip_batch_lanes(ptls_hip_batch_t *b)
{
    return b->lanes;
}

extern "C" int ptls_hip_batch_set_workgroup(ptls_hip_batch_t *b, int threads)
{
    if (b == nullptr || !(threads == 0 || threads == 512 || threads == WG_ALT))
        return fail(PTLS_HIP_EINVAL, "batch_set_workgroup: threads must be 0, 512 or %d", WG_ALT);
    DeviceGuard g(b->eng->device);
    b->forced_wg = threads;
    return plan_chunks(b);
}

extern "C" int ptls_hip_batch_workgroup(ptls_hip_batch_t *b)
{
    return b->wg;
}

extern "C" int ptls_hip_batch_set_max_workgroups(ptls_hip_batch_t *b, int n)
{
    if (b == nullptr || n < 0)
        return fail(PTLS_HIP_EINVAL, "batch_set_max_workgroups: n must be >= 0");
    DeviceGuard g(b->eng->device);
    b->max_wg = (unsigned)n;
    return plan_chunks(b);
}

extern "C" int ptls_hip_batch_grid(ptls_hip_batch_t *b)
{
    if (b == nullptr)
        return fail(PTLS_HIP_EINVAL, "batch_grid: null batch");
    return (int)plan_grid(b->n, b->nchunks, b->lanes, batch_cus(b));
}

extern "C" int ptls_hip_batch_chunks(ptls_hip_batch_t *b)
{
    return b != nullptr ? (int)b->nchunks : fail(PTLS_HIP_EINVAL, "batch_chunks: null batch");
}

extern "C" int ptls_hip_batch_set_clock(ptls_hip_batch_t *b, void *d_buf, size_t nbytes)
{
    if (b == nullptr || (d_buf != nullptr && nbytes < (size_t)ptls_hip_batch_grid(b) * 32))
        return fail(PTLS_HIP_EINVAL, "batch_set_clock: the buffer needs 32 bytes per workgroup of the launch");
    b->d_clk = static_cast<uint64_t *>(d_buf);
    b->clk_bytes = d_buf != nullptr ? nbytes : 0;
    return 0;
}

static int run_batch(ptls_hip_batch_t *b, ptls_hip_keyset_t *ks, const void *in, const void *aad, void *out, uint64_t *result,
                     void *stream, bool open, ptls_hip_keyset_t *hp_ks = nullptr, const ptls_hip_supp_t *supp = nullptr,
                     void *mask = nullptr)
{
    if (b == nullptr || ks == nullptr || ks->eng != b->eng)
        return fail(PTLS_HIP_EINVAL, "seal/open: batch and keyset must belong to the same engine");
    if (supp != nullptr && (hp_ks == nullptr || hp_ks->eng != b->eng || hp_ks->key_size != ks->key_size || mask == nullptr))
        return fail(PTLS_HIP_EINVAL, "seal_batch_supp: the header-protection keyset must be on the same engine with the "
                                     "AEAD's key size, and mask must be given");
    if (b->n == 0)
        return 0;
    if (b->max_key >= ks->nslots)
        return fail(PTLS_HIP_EINVAL, "seal/open: a record names key slot %u, the keyset has %zu", b->max_key, ks->nslots);
    if (in == nullptr || out == nullptr || (open && result == nullptr))
        return fail(PTLS_HIP_EINVAL, "seal/open: null buffer");
    DeviceGuard g(b->eng->device);
    KernelArgs a{};
    a.recs = b->d_recs;
    a.recs_ord = b->d_recs_ord != nullptr ? b->d_recs_ord : b->d_recs;
    a.order = b->d_order;
    a.chunks = b->d_chunks;
    a.nchunks = b->nchunks;
    a.in = static_cast<const uint8_t *>(in);
    a.aad = static_cast<const uint8_t *>(aad != nullptr ? aad : in);
    a.out = static_cast<uint8_t *>(out);
    a.result = result;
    a.slots = ks->d_slots;
    a.basis = ks->d_basis;
    a.t0 = b->eng->d_t0;
    a.supp = supp;
    a.hp_slots = hp_ks != nullptr ? hp_ks->d_slots : nullptr;
    a.hp_nslots = hp_ks != nullptr ? (uint32_t)hp_ks->nslots : 0;
    a.mask = static_cast<uint8_t *>(mask);
    const bool base_aligned = ((reinterpret_cast<uintptr_t>(in) | reinterpret_cast<uintptr_t>(a.aad) |
                                reinterpret_cast<uintptr_t>(out)) & 15) == 0;
    const bool aligned = base_aligned && b->all_aligned;
    const unsigned grid = plan_grid(b->n, b->nchunks, b->lanes, batch_cus(b));
    if (b->d_clk != nullptr && b->clk_bytes < (size_t)grid * 32)
        return fail(PTLS_HIP_EINVAL, "seal/open: the clock-stamp buffer is smaller than 32 bytes x %u workgroups", grid);
    a.clk = b->d_clk;
    a.queue = queue_slot(b->eng);
    const int rounds = ks->key_size == 16 ? 10 : 14;
    int e = launch_batch(b->lanes, rounds, open, b->wg, grid, stream, a, aligned);
    if (e != 0)
        return fail(PTLS_HIP_ELAUNCH, "kernel launch failed: %s", hipGetErrorString((hipError_t)e));
    keyset_note_use(ks, stream);
    keyset_note_use(hp_ks, stream);
    b->uses.note(stream);
    return 0;
}

extern "C" int ptls_hip_aesgcm_seal_batch(ptls_hip_batch_t *b, ptls_hip_keyset_t *ks, const void *in, const void *aad, void *out,
                                          void *stream)
{
    return run_batch(b, ks, in, aad, out, nullptr, stream, false);
}

extern "C" int ptls_hip_aesgcm_seal_batch_supp(ptls_hip_batch_t *b, ptls_hip_keyset_t *ks, ptls_hip_keyset_t *hp_ks,
                                               const ptls_hip_supp_t *supp, const void *in, const void *aad, void *out, void *mask,
                                               void *stream)
{
    if (supp == nullptr)
        return fail(PTLS_HIP_EINVAL, "seal_batch_supp: supp descriptors missing");
    return run_batch(b, ks, in, aad, out, nullptr, stream, false, hp_ks, supp, mask);
}

extern "C" int ptls_hip_aesecb_batch(ptls_hip_engine_t *eng, ptls_hip_keyset_t *hp_ks, const ptls_hip_supp_t *supp, size_t n,
                                     const void *src, void *mask, void *stream)
{
    if (eng == nullptr || hp_ks == nullptr || hp_ks->eng != eng || n > 0xffffffffu ||
        (n != 0 && (supp == nullptr || src == nullptr || mask == nullptr)))
        return fail(PTLS_HIP_EINVAL, "aesecb_batch: bad arguments");
    if (n == 0)
        return 0;
    DeviceGuard g(eng->device);
    const unsigned grid = (unsigned)std::min<size_t>((n + 255) / 256, (size_t)eng->ncu * 4);
    const int e = launch_aesecb(hp_ks->key_size == 16 ? 10 : 14, supp, (uint32_t)n, static_cast<const uint8_t *>(src),
                                static_cast<uint8_t *>(mask), hp_ks->d_slots, (uint32_t)hp_ks->nslots, eng->d_t0, grid,
                                stream);
    if (e != 0)
        return fail(PTLS_HIP_ELAUNCH, "aesecb_batch: kernel launch failed: %s", hipGetErrorString((hipError_t)e));
    keyset_note_use(hp_ks, stream);
    return 0;
}

/* ---------------------------------------------------------------------------------------------- */
/* TLS 1.3 record layer                                            */
/* ---------------------------------------------------------------------------------------------- */

static const size_t TLS13_CHUNK = PTLS_HIP_TLS13_MAX_PLAINTEXT;
static const size_t TLS13_OVERHEAD = 5 + 1 + 16; /* header, content type, tag */

extern "C" size_t ptls_hip_tls13_wire_size(size_t len)
{
    const size_t full = len / TLS13_CHUNK, rest = len % TLS13_CHUNK;
    return full * (TLS13_CHUNK + TLS13_OVERHEAD) + (rest != 0 ? rest + TLS13_OVERHEAD : 0);
}

/* buffer_push_encrypted_records (lib/picotls.c:747-794), TLS 1.3 branch: chunks of <= 16384 bytes,
 * one sequence number each, records back to back */
extern "C" size_t ptls_hip_tls13_frame(const ptls_hip_tls13_message_t *msgs, size_t n, ptls_hip_record_t *recs, size_t cap)
{
    size_t k = 0;
    for (size_t m = 0; m < n; ++m) {
        const ptls_hip_tls13_message_t &g = msgs[m];
        uint64_t wire = g.out_off;
        for (size_t pos = 0, j = 0; pos < g.len; pos += TLS13_CHUNK, ++j, ++k) {
            const size_t chunk = std::min<size_t>(TLS13_CHUNK, g.len - pos);
            if (recs != nullptr && k < cap) {
                ptls_hip_record_t &r = recs[k];
                r.in_off = g.in_off + pos;
                r.aad_off = wire;
                r.out_off = wire + 5;
                r.seq = g.seq + j;
                r.len = (uint32_t)(chunk + 1);
                r.aad_len = 5;
                r.key = g.key;
                r.flags = PTLS_HIP_RECORD_TLS13_TYPE(g.type);
            }
            wire += chunk + TLS13_OVERHEAD;
        }
    }
    return k;
}

extern "C" int ptls_hip_tls13_seal_batch(ptls_hip_batch_t *b, ptls_hip_keyset_t *ks, const void *in, void *out, void *stream)
{
    if (b == nullptr || out == nullptr)
        return fail(PTLS_HIP_EINVAL, "tls13_seal_batch: bad arguments");
    if (b->n == 0)
        return 0;
    DeviceGuard g(b->eng->device);
    const unsigned grid = (unsigned)std::min<size_t>((b->n + 255) / 256, (size_t)b->eng->ncu * 4);
    const int e = launch_tls13_headers(b->d_recs, (uint32_t)b->n, static_cast<uint8_t *>(out), grid, stream);
    if (e != 0)
        return fail(PTLS_HIP_ELAUNCH, "tls13_seal_batch: header kernel launch failed: %s", hipGetErrorString((hipError_t)e));
    return run_batch(b, ks, in, out, out, nullptr, stream, false);
}

/* parse_record_header (lib/picotls.c:5020-5031) over a byte stream of TLS 1.3 application-data records */
extern "C" int ptls_hip_tls13_parse(const void *wire, size_t wire_len, uint64_t wire_off, uint32_t key, uint64_t seq,
                                    uint64_t out_base, ptls_hip_record_t *recs, size_t cap, size_t *nrecs, size_t *consumed)
{
    if ((wire == nullptr && wire_len != 0) || nrecs == nullptr || consumed == nullptr)
        return fail(PTLS_HIP_EINVAL, "tls13_parse: bad arguments");
    const uint8_t *src = static_cast<const uint8_t *>(wire);
    size_t pos = 0, k = 0;
    uint64_t out = out_base;
    int rc = 0;
    while (pos + 5 <= wire_len && k < cap) {
        const uint8_t type = src[pos];
        const size_t length = (size_t)src[pos + 3] << 8 | src[pos + 4];
        if (type != 0x17)
            break; /* not application data: left to the caller's record layer */
        if (length > PTLS_HIP_TLS13_MAX_ENCRYPTED || length < 16) {
            rc = fail(PTLS_HIP_TLS13_DECODE_ERROR, "tls13_parse: record at %zu has length %zu", pos, length);
            break;
        }
        if (pos + 5 + length > wire_len)
            break; /* incomplete */
        if (recs != nullptr) {
            ptls_hip_record_t &r = recs[k];
            r.aad_off = wire_off + pos;
            r.in_off = wire_off + pos + 5;
            r.out_off = out;
            r.seq = seq + k;
            r.len = (uint32_t)(length - 16);
            r.aad_len = 5;
            r.key = key;
            r.flags = 0;
        }
        out += length - 16;
        pos += 5 + length;
        ++k;
    }
    *nrecs = k;
    *consumed = pos;
    return rc;
}

extern "C" int ptls_hip_tls13_open_batch(ptls_hip_batch_t *b, ptls_hip_keyset_t *ks, const void *in, void *out, uint64_t *result,
                                         void *stream)
{
    int rc = run_batch(b, ks, in, in, out, result, stream, true);
    if (rc != 0 || b->n == 0)
        return rc;
    DeviceGuard g(b->eng->device);
    const unsigned grid = (unsigned)std::min<size_t>((b->n + 255) / 256, (size_t)b->eng->ncu * 4);
    const int e = launch_tls13_inner(b->d_recs, (uint32_t)b->n, static_cast<const uint8_t *>(out), result, grid, stream);
    if (e != 0)
        return fail(PTLS_HIP_ELAUNCH, "tls13_open_batch: inner-plaintext kernel launch failed: %s", hipGetErrorString((hipError_t)e));
    return 0;
}

extern "C" int ptls_hip_aesgcm_open_batch(ptls_hip_batch_t *b, ptls_hip_keyset_t *ks, const void *in, const void *aad, void *out,
                                          uint64_t *result, void *stream)
{
    return run_batch(b, ks, in, aad, out, result, stream, true);
}

extern "C" int ptls_hip_fill_records(ptls_hip_batch_t *b, void *buf, uint64_t seed, uint64_t index_base, const uint64_t *index,
                                     void *stream)
{
    if (b == nullptr || buf == nullptr)
        return fail(PTLS_HIP_EINVAL, "fill_records: bad arguments");
    if (b->n == 0)
        return 0;
    DeviceGuard g(b->eng->device);
    const unsigned grid = (unsigned)std::min<size_t>((b->n + 3) / 4, (size_t)b->eng->ncu * 16);
    int e = launch_fill(b->d_recs, (uint32_t)b->n, static_cast<uint8_t *>(buf), seed, index_base, index, grid, stream);
    if (e != 0)
        return fail(PTLS_HIP_ELAUNCH, "fill launch failed: %s", hipGetErrorString((hipError_t)e));
    b->uses.note(stream);
    return 0;
}

/* The reference's gcm_basic #2 (t/fusion.c:251-273: key 00 11 .. ff, iv 20 .. 31, AAD 0 .. 19, the 85 bytes of
 * "hello world\n" x 7 + NUL, seq 0) sealed through the wave-per-record kernel, the batch kernel's table tree (8 lanes
 * per record) and its VALU combination (32 lanes), and opened back, whenever an engine starts: a library that computes
 * anything else (a probe build, a broken device) fails ptls_hip_engine_new instead of serving records. */
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
    /* the single-record kernel the plugin launches (record by value), and the batch kernel's table tree (8 lanes) and VALU
     * combination (32 lanes) at 512 threads per workgroup: not the instantiations a 768-thread batch launch uses, so the
     * self-check leaves no small dispatch in a profile of the batch kernels */
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

/* ---------------------------------------------------------------------------------------------- */
/* host-resident pipeline: pinned H2D -> kernel -> D2H, overlapped over NSLOT streams                */
/* ---------------------------------------------------------------------------------------------- */

static const int NSLOT = 3;

struct PipeSlot {
    hipStream_t stream;
    hipEvent_t done;
    uint8_t *d_in, *d_out, *d_aad, *d_mask;
    ptls_hip_record_t *d_recs, *d_recs_ord;
    Chunk *d_chunks;
    uint32_t *d_order;
    uint64_t *d_result;
    ptls_hip_supp_t *d_supp;
    /* pinned host staging for the slice's descriptors / chunks / record order / header-protection descriptors */
    ptls_hip_record_t *h_recs, *h_recs_ord;
    Chunk *h_chunks;
    uint32_t *h_order;
    ptls_hip_supp_t *h_supp;
    bool busy;
};

struct st_ptls_hip_pipeline_t {
    ptls_hip_engine_t *eng;
    size_t slice_bytes, max_recs;
    int transport;      /* PTLS_HIP_TRANSPORT_*: what the caller asked for */
    int last_transport; /* what the last seal/open used */
    PipeSlot slot[NSLOT];
};

extern "C" ptls_hip_pipeline_t *ptls_hip_pipeline_new(ptls_hip_engine_t *eng, size_t slice_bytes)
{
    if (eng == nullptr || slice_bytes < (1u << 16)) {
        fail(PTLS_HIP_EINVAL, "pipeline_new: bad arguments");
        return nullptr;
    }
    DeviceGuard g(eng->device);
    auto *p = new st_ptls_hip_pipeline_t();
    p->eng = eng;
    p->slice_bytes = slice_bytes;
    p->max_recs = slice_bytes / 16 + 1;
    bool ok = true;
    for (auto &s : p->slot) {
        ok = ok && hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking) == hipSuccess &&
             hipEventCreateWithFlags(&s.done, hipEventDisableTiming) == hipSuccess &&
             hipMalloc(&s.d_in, slice_bytes + 64) == hipSuccess && hipMalloc(&s.d_out, slice_bytes + 64) == hipSuccess &&
             hipMalloc(&s.d_aad, slice_bytes / 4 + 64) == hipSuccess && hipMalloc(&s.d_mask, slice_bytes / 4 + 64) == hipSuccess &&
             hipMalloc(&s.d_supp, p->max_recs * sizeof(ptls_hip_supp_t)) == hipSuccess &&
             hipHostMalloc(&s.h_supp, p->max_recs * sizeof(ptls_hip_supp_t), hipHostMallocDefault) == hipSuccess &&
             hipMalloc(&s.d_recs, p->max_recs * sizeof(ptls_hip_record_t)) == hipSuccess &&
             hipMalloc(&s.d_recs_ord, p->max_recs * sizeof(ptls_hip_record_t)) == hipSuccess &&
             hipHostMalloc(&s.h_recs_ord, p->max_recs * sizeof(ptls_hip_record_t), hipHostMallocDefault) == hipSuccess &&
             hipMalloc(&s.d_chunks, p->max_recs * sizeof(Chunk)) == hipSuccess &&
             hipMalloc(&s.d_order, p->max_recs * sizeof(uint32_t)) == hipSuccess &&
             hipHostMalloc(&s.h_order, p->max_recs * sizeof(uint32_t), hipHostMallocDefault) == hipSuccess &&
             hipMalloc(&s.d_result, p->max_recs * sizeof(uint64_t)) == hipSuccess &&
             hipHostMalloc(&s.h_recs, p->max_recs * sizeof(ptls_hip_record_t), hipHostMallocDefault) == hipSuccess &&
             hipHostMalloc(&s.h_chunks, p->max_recs * sizeof(Chunk), hipHostMallocDefault) == hipSuccess;
        s.busy = false;
    }
    if (!ok) {
        fail(PTLS_HIP_ENOMEM, "pipeline_new: cannot allocate %d x %zu bytes of staging", NSLOT, slice_bytes);
        ptls_hip_pipeline_free(p);
        return nullptr;
    }
    return p;
}

extern "C" void ptls_hip_pipeline_free(ptls_hip_pipeline_t *p)
{
    if (p == nullptr)
        return;
    DeviceGuard g(p->eng->device);
    for (auto &s : p->slot) {
        if (s.stream != nullptr)
            (void)hipStreamSynchronize(s.stream);
        (void)hipFree(s.d_in);
        (void)hipFree(s.d_out);
        (void)hipFree(s.d_aad);
        (void)hipFree(s.d_mask);
        (void)hipFree(s.d_supp);
        (void)hipHostFree(s.h_supp);
        (void)hipFree(s.d_recs);
        (void)hipFree(s.d_recs_ord);
        (void)hipHostFree(s.h_recs_ord);
        (void)hipFree(s.d_chunks);
        (void)hipFree(s.d_order);
        (void)hipHostFree(s.h_order);
        (void)hipFree(s.d_result);
        (void)hipHostFree(s.h_recs);
        (void)hipHostFree(s.h_chunks);
        if (s.done != nullptr)
            (void)hipEventDestroy(s.done);
        if (s.stream != nullptr)
            (void)hipStreamDestroy(s.stream);
    }
    delete p;
}

extern "C" int ptls_hip_pipeline_set_transport(ptls_hip_pipeline_t *p, int transport)
{
    if (p == nullptr ||
        !(transport == PTLS_HIP_TRANSPORT_AUTO || transport == PTLS_HIP_TRANSPORT_COPY || transport == PTLS_HIP_TRANSPORT_MAPPED))
        return fail(PTLS_HIP_EINVAL, "pipeline_set_transport: bad arguments");
    p->transport = transport;
    return 0;
}

extern "C" int ptls_hip_pipeline_last_transport(ptls_hip_pipeline_t *p)
{
    return p->last_transport;
}

extern "C" int ptls_hip_host_register(void *ptr, size_t len)
{
    HIP_TRY(hipHostRegister(ptr, len, hipHostRegisterDefault), PTLS_HIP_ENODEV);
    return 0;
}

extern "C" int ptls_hip_host_unregister(void *ptr)
{
    HIP_TRY(hipHostUnregister(ptr), PTLS_HIP_ENODEV);
    return 0;
}

/* byte span [lo, hi) of a field over records [a, b) */
struct Span {
    uint64_t lo, hi;
};

/* what a pipeline slice runs: plain seal / open (AAD in its own buffer), or the TLS 1.3 record layer
 * (seal: the 5-byte headers are written into the output and read back as the AAD, like
 * ptls_hip_tls13_seal_batch; open: the AAD is the header in the received input, and the inner plaintext
 * is parsed after the open, like ptls_hip_tls13_open_batch) */
enum PipeMode { PIPE_SEAL, PIPE_OPEN, PIPE_TLS13_SEAL, PIPE_TLS13_OPEN };

/* the device address of pinned (hipHostMalloc'd) or registered host memory, or nullptr if it is not mapped */
static void *mapped_ptr(const void *h)
{
    if (h == nullptr)
        return nullptr;
    void *d = nullptr;
    if (hipHostGetDevicePointer(&d, const_cast<void *>(h), 0) != hipSuccess) {
        (void)hipGetLastError(); /* not an error of the pipeline: the copy transport is used */
        return nullptr;
    }
    return d;
}

/* the device address of h when pinned or registered host memory covers ALL of [h, h + need) with one mapping, else
 * nullptr; *partial = the start is mapped but not the whole span.  Such a buffer (registered only in part) must not
 * be handed to the kernels, which would touch unmapped host pages over PCIe, and the copy engines refuse it as well
 * (hipMemcpyAsync: invalid argument), so the call fails with EINVAL.  The mapping's range comes from the pointer
 * attributes; the last byte must also map, contiguously with the first. */
static void *mapped_span(const void *h, uint64_t need, bool *partial)
{
    void *d = mapped_ptr(h);
    if (d == nullptr || need <= 1)
        return d;
    const uintptr_t dp = reinterpret_cast<uintptr_t>(d);
    /* the allocation's range, queried and compared in the device address space: a span inside it is
     * mapped; otherwise the mapping of the span's last byte decides (one registration covering both ends) */
    uintptr_t start = 0;
    size_t size = 0;
    if (hipPointerGetAttribute(&start, HIP_POINTER_ATTRIBUTE_RANGE_START_ADDR, reinterpret_cast<hipDeviceptr_t>(d)) == hipSuccess &&
        hipPointerGetAttribute(&size, HIP_POINTER_ATTRIBUTE_RANGE_SIZE, reinterpret_cast<hipDeviceptr_t>(d)) == hipSuccess &&
        size != 0 && start <= dp && dp + need <= start + size)
        return d;
    (void)hipGetLastError();
    void *d_last = mapped_ptr(static_cast<const uint8_t *>(h) + (need - 1));
    if (d_last == nullptr || reinterpret_cast<uintptr_t>(d_last) != dp + (need - 1)) {
        *partial = true;
        return nullptr;
    }
    return d;
}

/* lanes per record when the kernel reads and writes host memory: the launch is PCIe-bound, not LDS-bound, and wider
 * lane groups turn each load / store instruction into longer contiguous runs per record, i.e. fewer, larger PCIe
 * requests.  Measured (tools/hostmem_probe.py, seal+open GiB/s at 4 / 8 / 16 / 32 lanes): 1350-B records 31.7 /
 * 34.8 / 36.7 / 39.5; 16-KiB records - / 36.6 / 40.2 / 41.5; 64 B - 16 KiB over 64K keys at 16 / 32: 28.6 / 36.2.
 * Records of >= 64 GHASH elements go to the wave-per-record kernel (one 1-KiB run per wave instruction): 16 / 32 / 64
 * lanes 1350-B records 36.5 / 39.2 / 40.4, 16-KiB records 40.1 / 41.5 / 42.7 (one 1-GiB batch each).
 * Batches for the sparse-key kernel keep it. */
static int mapped_lanes(const ptls_hip_record_t *recs, size_t n, unsigned ncu)
{
    const int lanes = choose_lanes(recs, n, ncu);
    if (lanes == SPARSE_LANES || n == 0)
        return lanes;
    double sum = 0;
    for (size_t i = 0; i < n; ++i)
        sum += (double)((recs[i].aad_len + 15) / 16 + (recs[i].len + 15) / 16 + 1);
    const double mean = sum / (double)n;
    return mean >= 64 ? SPARSE_LANES : mean >= 32 ? 32 : mean >= 16 ? std::max(lanes, 16) : lanes;
}

/* The kernels read the descriptors in plan order (recs_ord).  When the plan keeps the caller's order (records that
 * already come as the planner sorts them: equal lengths, non-increasing lengths within each key run), the caller-order
 * copy serves as both: no host gather and one descriptor upload less per pipeline slice (a 1 GiB slice set of QUIC
 * records is ~800K descriptors; the host plans each slice while the device runs the previous one). */
static bool identity_order(const std::vector<uint32_t> &order, size_t n)
{
    for (size_t t = 0; t < n; ++t)
        if (order[t] != (uint32_t)t)
            return false;
    return true;
}

/* PTLS_HIP_TRANSPORT_MAPPED: the batch kernel reads the records from, and writes them to, the caller's pinned host
 * buffers over PCIe itself (their device addresses); no staging copies, no copy engines.  Only the descriptors,
 * the launch plan and the header-protection descriptors go through the slots' pinned staging.  Slices of at
 * most 4 x slice_bytes of payload rotate over the slots' streams, so planning overlaps the kernels.  (tools/hostmem_probe.py, DESIGN.md §6.3: the copy
 * engines carry ~57 GB/s in both directions together, the kernel's own PCIe reads + writes ~80 GB/s.) */
static int pipeline_run_mapped(ptls_hip_pipeline_t *p, ptls_hip_keyset_t *ks, const ptls_hip_record_t *recs, size_t n,
                               const uint8_t *d_in, const uint8_t *d_aad, uint8_t *d_out, uint64_t *h_result, uint64_t *d_res,
                               PipeMode mode, ptls_hip_keyset_t *hp_ks, const ptls_hip_supp_t *supp, uint8_t *d_mask)
{
    const bool open = mode == PIPE_OPEN || mode == PIPE_TLS13_OPEN;
    const bool aad_in_out = mode == PIPE_TLS13_SEAL, aad_in_in = mode == PIPE_TLS13_OPEN;
    const int rounds = ks->key_size == 16 ? 10 : 14;
    std::vector<Chunk> ch;
    std::vector<uint32_t> order;
    int k = 0;
    for (size_t i = 0; i < n; ++k) {
        /* slices of at most slice_bytes of payload: the host plans and uploads slice k + 1 while the device runs k */
        size_t cnt = 0, bytes = 0;
        /* 4 x the staging slice: no staging is involved, and the measured best (seal+open GiB/s of 1 GiB, 64 / 128 /
         * 256 / 512 / 2048 MiB slices: 16-KiB records 35.5 / 38.6 / 39.8 / 39.9 / 39.6, 1350-B records 32.9 / 33.3 /
         * 33.4 / 30.7 / 21.9, configs[3] 34.7 / 36.3 / 37.2 / 35.8 / 33.9) */
        const size_t mslice = 4 * p->slice_bytes;
        while (i + cnt < n && cnt < p->max_recs - 1 && (cnt == 0 || bytes + recs[i + cnt].len <= mslice))
            bytes += recs[i + cnt++].len;
        PipeSlot &s = p->slot[k % NSLOT];
        if (s.busy)
            HIP_TRY(hipEventSynchronize(s.done), PTLS_HIP_ENODEV);
        std::memcpy(s.h_recs, recs + i, cnt * sizeof(ptls_hip_record_t));
        const int lanes = mapped_lanes(s.h_recs, cnt, (unsigned)p->eng->ncu);
        bool aligned;
        build_chunks(s.h_recs, cnt, lanes, (unsigned)p->eng->ncu, ch, order, aligned);
        std::memcpy(s.h_chunks, ch.data(), ch.size() * sizeof(Chunk));
        std::memcpy(s.h_order, order.data(), cnt * sizeof(uint32_t));
        const bool ident = identity_order(order, cnt);
        if (!ident) {
            for (size_t t = 0; t < cnt; ++t)
                s.h_recs_ord[t] = s.h_recs[order[t]];
            HIP_TRY(hipMemcpyAsync(s.d_recs_ord, s.h_recs_ord, cnt * sizeof(ptls_hip_record_t), hipMemcpyHostToDevice, s.stream),
                    PTLS_HIP_ENODEV);
        }
        if (!ident)
            HIP_TRY(hipMemcpyAsync(s.d_order, s.h_order, cnt * sizeof(uint32_t), hipMemcpyHostToDevice, s.stream), PTLS_HIP_ENODEV);
        HIP_TRY(hipMemcpyAsync(s.d_recs, s.h_recs, cnt * sizeof(ptls_hip_record_t), hipMemcpyHostToDevice, s.stream),
                PTLS_HIP_ENODEV);
        HIP_TRY(hipMemcpyAsync(s.d_chunks, s.h_chunks, ch.size() * sizeof(Chunk), hipMemcpyHostToDevice, s.stream), PTLS_HIP_ENODEV);
        if (supp != nullptr) {
            std::memcpy(s.h_supp, supp + i, cnt * sizeof(ptls_hip_supp_t));
            HIP_TRY(hipMemcpyAsync(s.d_supp, s.h_supp, cnt * sizeof(ptls_hip_supp_t), hipMemcpyHostToDevice, s.stream),
                    PTLS_HIP_ENODEV);
        }
        const unsigned egrid = (unsigned)std::min<size_t>((cnt + 255) / 256, (size_t)p->eng->ncu * 4);
        if (aad_in_out) {
            const int eh = launch_tls13_headers(s.d_recs, (uint32_t)cnt, d_out, egrid, s.stream);
            if (eh != 0)
                return fail(PTLS_HIP_ELAUNCH, "pipeline: header kernel launch failed: %s", hipGetErrorString((hipError_t)eh));
        }
        uint64_t *res = d_res != nullptr ? d_res + i : s.d_result;
        KernelArgs a{};
        a.recs = s.d_recs;
        a.recs_ord = ident ? s.d_recs : s.d_recs_ord;
        a.order = ident ? nullptr : s.d_order;
        a.chunks = s.d_chunks;
        a.nchunks = (uint32_t)ch.size();
        a.in = d_in;
        a.aad = aad_in_out ? d_out : aad_in_in ? d_in : d_aad;
        a.out = d_out;
        a.result = res;
        a.slots = ks->d_slots;
        a.basis = ks->d_basis;
        a.t0 = p->eng->d_t0;
        if (supp != nullptr) {
            a.supp = s.d_supp;
            a.hp_slots = hp_ks->d_slots;
            a.hp_nslots = (uint32_t)hp_ks->nslots;
            a.mask = d_mask;
        }
        const bool base_aligned =
            ((reinterpret_cast<uintptr_t>(a.in) | reinterpret_cast<uintptr_t>(a.aad) | reinterpret_cast<uintptr_t>(a.out)) & 15) == 0;
        const unsigned grid = plan_grid(cnt, ch.size(), lanes, (unsigned)p->eng->ncu);
        a.queue = queue_slot(p->eng);
        const int e = launch_batch(lanes, rounds, open, plan_wg(ch, lanes), grid, s.stream, a, aligned && base_aligned);
        if (e != 0)
            return fail(PTLS_HIP_ELAUNCH, "pipeline: kernel launch failed: %s", hipGetErrorString((hipError_t)e));
        if (mode == PIPE_TLS13_OPEN) {
            const int ei = launch_tls13_inner(s.d_recs, (uint32_t)cnt, d_out, res, egrid, s.stream);
            if (ei != 0)
                return fail(PTLS_HIP_ELAUNCH, "pipeline: inner-plaintext kernel launch failed: %s", hipGetErrorString((hipError_t)ei));
        }
        if (open && d_res == nullptr)
            HIP_TRY(hipMemcpyAsync(h_result + i, s.d_result, cnt * sizeof(uint64_t), hipMemcpyDeviceToHost, s.stream),
                    PTLS_HIP_ENODEV);
        HIP_TRY(hipEventRecord(s.done, s.stream), PTLS_HIP_ENODEV);
        s.busy = true;
        i += cnt;
    }
    for (auto &s : p->slot) {
        if (s.busy)
            HIP_TRY(hipEventSynchronize(s.done), PTLS_HIP_ENODEV);
        s.busy = false;
    }
    /* the kernel's stores to host memory are complete once its stream event has been waited for */
    p->last_transport = PTLS_HIP_TRANSPORT_MAPPED;
    return 0;
}

static int pipeline_run_copy(ptls_hip_pipeline_t *p, ptls_hip_keyset_t *ks, const ptls_hip_record_t *recs, size_t n,
                             const void *h_in, const void *h_aad, void *h_out, uint64_t *h_result, PipeMode mode,
                             ptls_hip_keyset_t *hp_ks, const ptls_hip_supp_t *supp, void *h_mask);

/* wait for every slice still in flight and free the slots: also on an error path, because an earlier slice's kernel
 * or copy may still read or write the caller's host buffers, which the caller may release once the call returned */
static void drain_slots(ptls_hip_pipeline_t *p)
{
    for (auto &s : p->slot) {
        if (s.busy)
            (void)hipStreamSynchronize(s.stream);
        s.busy = false;
    }
}

static int pipeline_run(ptls_hip_pipeline_t *p, ptls_hip_keyset_t *ks, const ptls_hip_record_t *recs, size_t n, const void *h_in,
                        const void *h_aad, void *h_out, uint64_t *h_result, PipeMode mode, ptls_hip_keyset_t *hp_ks = nullptr,
                        const ptls_hip_supp_t *supp = nullptr, void *h_mask = nullptr)
{
    if (supp != nullptr && (mode != PIPE_SEAL || hp_ks == nullptr || ks == nullptr || hp_ks->eng != ks->eng ||
                            hp_ks->key_size != ks->key_size || h_mask == nullptr))
        return fail(PTLS_HIP_EINVAL, "pipeline_seal_supp: the header-protection keyset must be on the same engine with the "
                                     "AEAD's key size, and h_mask must be given");
    const bool open = mode == PIPE_OPEN || mode == PIPE_TLS13_OPEN;
    const bool aad_in_out = mode == PIPE_TLS13_SEAL, aad_in_in = mode == PIPE_TLS13_OPEN;
    if (p == nullptr || ks == nullptr || ks->eng != p->eng || (n != 0 && (recs == nullptr || h_in == nullptr || h_out == nullptr)) ||
        (open && h_result == nullptr))
        return fail(PTLS_HIP_EINVAL, "pipeline seal/open: bad arguments");
    for (size_t i = 0; i < n; ++i)
        if (recs[i].key >= ks->nslots)
            return fail(PTLS_HIP_EINVAL, "pipeline: record %zu names key slot %u, the keyset has %zu", i, recs[i].key, ks->nslots);
    DeviceGuard g(p->eng->device);
    /* every transport checks the buffers: the copy engines refuse a buffer registered only in part as well (hipMemcpyAsync:
     * invalid argument, tests/test_gpu_node.py::test_partly_registered_input_is_refused), so such a call fails here with
     * a message that names the cause; unregistered (pageable) buffers go to the copy transport */
    if (n != 0) {
        /* the bytes the kernels would touch in each buffer: [base, base + need) */
        uint64_t need_in = 0, need_out = 0, need_aad = 0, need_mask = 0;
        for (size_t i = 0; i < n; ++i) {
            const ptls_hip_record_t &r = recs[i];
            need_in = std::max<uint64_t>(need_in, r.in_off + r.len + (open ? 16 : 0));
            need_out = std::max<uint64_t>(need_out, r.out_off + r.len + (open ? 0 : 16));
            if (r.aad_len != 0) {
                uint64_t &na = aad_in_out ? need_out : aad_in_in ? need_in : need_aad;
                na = std::max<uint64_t>(na, r.aad_off + r.aad_len);
            }
            if (supp != nullptr && (supp[i].flags & PTLS_HIP_SUPP_ENABLE))
                need_mask = std::max<uint64_t>(need_mask, supp[i].mask_off + 16);
        }
        bool partial = false;
        const uint8_t *d_in = static_cast<const uint8_t *>(mapped_span(h_in, need_in, &partial));
        uint8_t *d_out = static_cast<uint8_t *>(mapped_span(h_out, need_out, &partial));
        const uint8_t *d_aad = static_cast<const uint8_t *>(mapped_span(h_aad, need_aad, &partial));
        uint8_t *d_mask = static_cast<uint8_t *>(mapped_span(h_mask, need_mask, &partial));
        uint64_t *d_res = open ? static_cast<uint64_t *>(mapped_span(h_result, (uint64_t)n * 8, &partial)) : nullptr;
        if (partial)
            return fail(PTLS_HIP_EINVAL, "pipeline: a host buffer is pinned or registered only in part (its mapping ends before "
                                         "the last byte the records touch): neither transport can use it");
        const bool ok = d_in != nullptr && d_out != nullptr && (h_aad == nullptr || d_aad != nullptr) && (h_mask == nullptr || d_mask != nullptr);
        if (ok && p->transport != PTLS_HIP_TRANSPORT_COPY) {
            const int rc = pipeline_run_mapped(p, ks, recs, n, d_in, d_aad, d_out, h_result, d_res, mode, hp_ks, supp, d_mask);
            if (rc != 0)
                drain_slots(p);
            return rc;
        }
        if (p->transport == PTLS_HIP_TRANSPORT_MAPPED)
            return fail(PTLS_HIP_EINVAL, "pipeline: transport MAPPED needs host buffers (in, out, aad, mask) pinned or registered "
                                         "over every byte the records touch");
    }
    const int rc = pipeline_run_copy(p, ks, recs, n, h_in, h_aad, h_out, h_result, mode, hp_ks, supp, h_mask);
    if (rc != 0)
        drain_slots(p);
    return rc;
}

/* PTLS_HIP_TRANSPORT_COPY: slices staged through the slots' device buffers by the copy engines */
static int pipeline_run_copy(ptls_hip_pipeline_t *p, ptls_hip_keyset_t *ks, const ptls_hip_record_t *recs, size_t n,
                             const void *h_in, const void *h_aad, void *h_out, uint64_t *h_result, PipeMode mode,
                             ptls_hip_keyset_t *hp_ks, const ptls_hip_supp_t *supp, void *h_mask)
{
    uint8_t *hmask = static_cast<uint8_t *>(h_mask);
    const bool open = mode == PIPE_OPEN || mode == PIPE_TLS13_OPEN;
    const bool aad_in_out = mode == PIPE_TLS13_SEAL, aad_in_in = mode == PIPE_TLS13_OPEN;
    p->last_transport = PTLS_HIP_TRANSPORT_COPY;
    const int rounds = ks->key_size == 16 ? 10 : 14;
    const size_t tag_in = open ? 16 : 0, tag_out = open ? 0 : 16;
    const uint8_t *hin = static_cast<const uint8_t *>(h_in), *haad = static_cast<const uint8_t *>(h_aad);
    uint8_t *hout = static_cast<uint8_t *>(h_out);
    std::vector<Chunk> ch;
    std::vector<uint32_t> order;
    size_t i = 0;
    int k = 0;
    while (i < n) {
        /* grow the slice while every span fits the staging buffers */
        Span in{UINT64_MAX, 0}, out{UINT64_MAX, 0}, ad{UINT64_MAX, 0};
        size_t j = i;
        while (j < n && j - i < p->max_recs - 1) {
            const ptls_hip_record_t &r = recs[j];
            Span ni{std::min(in.lo, r.in_off), std::max(in.hi, r.in_off + r.len + tag_in)};
            Span no{std::min(out.lo, r.out_off), std::max(out.hi, r.out_off + r.len + tag_out)};
            Span na{std::min(ad.lo, r.aad_off), std::max(ad.hi, r.aad_off + r.aad_len)};
            if (aad_in_out) { /* the header is part of the output span */
                no = Span{std::min(no.lo, r.aad_off), std::max(no.hi, r.aad_off + r.aad_len)};
                na = Span{UINT64_MAX, 0};
            } else if (aad_in_in) { /* the header is part of the input span */
                ni = Span{std::min(ni.lo, r.aad_off), std::max(ni.hi, r.aad_off + r.aad_len)};
                na = Span{UINT64_MAX, 0};
            }
            if (j > i && (ni.hi - ni.lo > p->slice_bytes || no.hi - no.lo > p->slice_bytes || na.hi - na.lo > p->slice_bytes / 4))
                break;
            in = ni;
            out = no;
            ad = na;
            ++j;
        }
        if (in.hi - in.lo > p->slice_bytes || out.hi - out.lo > p->slice_bytes || (ad.hi > ad.lo && ad.hi - ad.lo > p->slice_bytes / 4))
            return fail(PTLS_HIP_EINVAL, "pipeline: record %zu does not fit a %zu-byte slice", i, p->slice_bytes);
        if (ad.hi <= ad.lo)
            ad = Span{0, 0};
        /* header protection: masks land in their own span; every enabled sample must lie in the slice's output */
        Span mk{UINT64_MAX, 0};
        if (supp != nullptr) {
            for (size_t t = i; t < j; ++t) {
                const ptls_hip_supp_t &sp = supp[t];
                if (!(sp.flags & PTLS_HIP_SUPP_ENABLE))
                    continue;
                if (sp.sample_off < out.lo || sp.sample_off + 16 > out.hi)
                    return fail(PTLS_HIP_EINVAL, "pipeline_seal_supp: sample of record %zu is outside the slice's output", t);
                mk = Span{std::min(mk.lo, sp.mask_off), std::max(mk.hi, sp.mask_off + 16)};
            }
            if (mk.hi > mk.lo && mk.hi - mk.lo > p->slice_bytes / 4)
                return fail(PTLS_HIP_EINVAL, "pipeline_seal_supp: masks of records %zu..%zu span more than %zu bytes", i, j,
                            p->slice_bytes / 4);
            if (mk.hi <= mk.lo)
                mk = Span{0, 0};
        }
        PipeSlot &s = p->slot[k % NSLOT];
        if (s.busy)
            HIP_TRY(hipEventSynchronize(s.done), PTLS_HIP_ENODEV);
        const size_t cnt = j - i;
        /* slice-local descriptors keep the same relative 16-byte alignment as the caller's buffers */
        const uint64_t in_base = in.lo & ~(uint64_t)15, out_base = out.lo & ~(uint64_t)15, aad_base = ad.lo & ~(uint64_t)15;
        for (size_t t = 0; t < cnt; ++t) {
            s.h_recs[t] = recs[i + t];
            s.h_recs[t].in_off -= in_base;
            s.h_recs[t].out_off -= out_base;
            s.h_recs[t].aad_off -= aad_in_out ? out_base : aad_in_in ? in_base : aad_base;
        }
        const int lanes = choose_lanes(s.h_recs, cnt, (unsigned)p->eng->ncu);
        bool aligned;
        build_chunks(s.h_recs, cnt, lanes, (unsigned)p->eng->ncu, ch, order, aligned);
        const uint64_t mask_base = mk.lo & ~(uint64_t)15;
        if (supp != nullptr) {
            for (size_t t = 0; t < cnt; ++t) {
                s.h_supp[t] = supp[i + t];
                if (s.h_supp[t].flags & PTLS_HIP_SUPP_ENABLE) {
                    s.h_supp[t].sample_off -= out_base;
                    s.h_supp[t].mask_off -= mask_base;
                }
            }
            HIP_TRY(hipMemcpyAsync(s.d_supp, s.h_supp, cnt * sizeof(ptls_hip_supp_t), hipMemcpyHostToDevice, s.stream),
                    PTLS_HIP_ENODEV);
            /* the mask span goes in as well (16 B per packet), so mask bytes of packets without header protection
             * and between masks come back unchanged */
            if (mk.hi > mk.lo)
                HIP_TRY(hipMemcpyAsync(s.d_mask + (mk.lo - mask_base), hmask + mk.lo, mk.hi - mk.lo, hipMemcpyHostToDevice, s.stream),
                        PTLS_HIP_ENODEV);
        }
        std::memcpy(s.h_chunks, ch.data(), ch.size() * sizeof(Chunk));
        std::memcpy(s.h_order, order.data(), cnt * sizeof(uint32_t));
        const bool ident = identity_order(order, cnt);
        if (!ident) {
            for (size_t t = 0; t < cnt; ++t)
                s.h_recs_ord[t] = s.h_recs[order[t]];
            HIP_TRY(hipMemcpyAsync(s.d_recs_ord, s.h_recs_ord, cnt * sizeof(ptls_hip_record_t), hipMemcpyHostToDevice, s.stream),
                    PTLS_HIP_ENODEV);
        }
        if (!ident)
            HIP_TRY(hipMemcpyAsync(s.d_order, s.h_order, cnt * sizeof(uint32_t), hipMemcpyHostToDevice, s.stream), PTLS_HIP_ENODEV);
        HIP_TRY(hipMemcpyAsync(s.d_recs, s.h_recs, cnt * sizeof(ptls_hip_record_t), hipMemcpyHostToDevice, s.stream),
                PTLS_HIP_ENODEV);
        HIP_TRY(hipMemcpyAsync(s.d_chunks, s.h_chunks, ch.size() * sizeof(Chunk), hipMemcpyHostToDevice, s.stream), PTLS_HIP_ENODEV);
        HIP_TRY(hipMemcpyAsync(s.d_in + (in.lo - in_base), hin + in.lo, in.hi - in.lo, hipMemcpyHostToDevice, s.stream),
                PTLS_HIP_ENODEV);
        if (ad.hi > ad.lo)
            HIP_TRY(hipMemcpyAsync(s.d_aad + (ad.lo - aad_base), haad + ad.lo, ad.hi - ad.lo, hipMemcpyHostToDevice, s.stream),
                    PTLS_HIP_ENODEV);
        const unsigned egrid = (unsigned)std::min<size_t>((cnt + 255) / 256, (size_t)p->eng->ncu * 4);
        if (aad_in_out) {
            const int eh = launch_tls13_headers(s.d_recs, (uint32_t)cnt, s.d_out, egrid, s.stream);
            if (eh != 0)
                return fail(PTLS_HIP_ELAUNCH, "pipeline: header kernel launch failed: %s", hipGetErrorString((hipError_t)eh));
        }
        KernelArgs a{};
        a.recs = s.d_recs;
        a.recs_ord = ident ? s.d_recs : s.d_recs_ord;
        a.order = ident ? nullptr : s.d_order;
        a.chunks = s.d_chunks;
        a.nchunks = (uint32_t)ch.size();
        a.in = s.d_in;
        a.aad = aad_in_out ? s.d_out : aad_in_in ? s.d_in : s.d_aad;
        a.out = s.d_out;
        a.result = s.d_result;
        a.slots = ks->d_slots;
        a.basis = ks->d_basis;
        a.t0 = p->eng->d_t0;
        if (supp != nullptr) {
            a.supp = s.d_supp;
            a.hp_slots = hp_ks->d_slots;
            a.hp_nslots = (uint32_t)hp_ks->nslots;
            a.mask = s.d_mask;
        }
        const unsigned grid = plan_grid(cnt, ch.size(), lanes, (unsigned)p->eng->ncu);
        a.queue = queue_slot(p->eng);
        const int e = launch_batch(lanes, rounds, open, plan_wg(ch, lanes), grid, s.stream, a, aligned);
        if (e != 0)
            return fail(PTLS_HIP_ELAUNCH, "pipeline: kernel launch failed: %s", hipGetErrorString((hipError_t)e));
        if (mode == PIPE_TLS13_OPEN) {
            const int ei = launch_tls13_inner(s.d_recs, (uint32_t)cnt, s.d_out, s.d_result, egrid, s.stream);
            if (ei != 0)
                return fail(PTLS_HIP_ELAUNCH, "pipeline: inner-plaintext kernel launch failed: %s", hipGetErrorString((hipError_t)ei));
        }
        HIP_TRY(hipMemcpyAsync(hout + out.lo, s.d_out + (out.lo - out_base), out.hi - out.lo, hipMemcpyDeviceToHost, s.stream),
                PTLS_HIP_ENODEV);
        if (supp != nullptr && mk.hi > mk.lo)
            HIP_TRY(hipMemcpyAsync(hmask + mk.lo, s.d_mask + (mk.lo - mask_base), mk.hi - mk.lo, hipMemcpyDeviceToHost, s.stream),
                    PTLS_HIP_ENODEV);
        if (open) {
            /* results come back in slice order; the caller's array is indexed like recs */
            HIP_TRY(hipMemcpyAsync(h_result + i, s.d_result, cnt * sizeof(uint64_t), hipMemcpyDeviceToHost, s.stream),
                    PTLS_HIP_ENODEV);
        }
        HIP_TRY(hipEventRecord(s.done, s.stream), PTLS_HIP_ENODEV);
        s.busy = true;
        i = j;
        ++k;
    }
    for (auto &s : p->slot) {
        if (s.busy)
            HIP_TRY(hipEventSynchronize(s.done), PTLS_HIP_ENODEV);
        s.busy = false;
    }
    return 0;
}

extern "C" int ptls_hip_pipeline_seal(ptls_hip_pipeline_t *p, ptls_hip_keyset_t *ks, const ptls_hip_record_t *recs, size_t n,
                                      const void *h_in, const void *h_aad, void *h_out)
{
    return pipeline_run(p, ks, recs, n, h_in, h_aad, h_out, nullptr, PIPE_SEAL);
}

extern "C" int ptls_hip_pipeline_seal_supp(ptls_hip_pipeline_t *p, ptls_hip_keyset_t *ks, ptls_hip_keyset_t *hp_ks,
                                           const ptls_hip_record_t *recs, const ptls_hip_supp_t *supp, size_t n, const void *h_in,
                                           const void *h_aad, void *h_out, void *h_mask)
{
    if (n != 0 && supp == nullptr)
        return fail(PTLS_HIP_EINVAL, "pipeline_seal_supp: supp descriptors missing");
    return pipeline_run(p, ks, recs, n, h_in, h_aad, h_out, nullptr, PIPE_SEAL, hp_ks, supp, h_mask);
}

extern "C" int ptls_hip_pipeline_tls13_seal(ptls_hip_pipeline_t *p, ptls_hip_keyset_t *ks, const ptls_hip_record_t *recs, size_t n,
                                            const void *h_in, void *h_wire)
{
    return pipeline_run(p, ks, recs, n, h_in, nullptr, h_wire, nullptr, PIPE_TLS13_SEAL);
}

extern "C" int ptls_hip_pipeline_tls13_open(ptls_hip_pipeline_t *p, ptls_hip_keyset_t *ks, const ptls_hip_record_t *recs, size_t n,
                                            const void *h_wire, void *h_out, uint64_t *h_result)
{
    return pipeline_run(p, ks, recs, n, h_wire, nullptr, h_out, h_result, PIPE_TLS13_OPEN);
}

extern "C" int ptls_hip_pipeline_open(ptls_hip_pipeline_t *p, ptls_hip_keyset_t *ks, const ptls_hip_record_t *recs, size_t n,
                                      const void *h_in, const void *h_aad, void *h_out, uint64_t *h_result)
{
    return pipeline_run(p, ks, recs, n, h_in, h_aad, h_out, h_result, PIPE_OPEN);
}

/* ---------------------------------------------------------------------------------------------- */
/* one batch over several devices                                                 */
/* ---------------------------------------------------------------------------------------------- */

extern "C" int ptls_hip_partition_bytes(const ptls_hip_record_t *recs, size_t n, size_t parts, size_t *bounds)
{
    if ((recs == nullptr && n != 0) || parts == 0 || bounds == nullptr)
        return fail(PTLS_HIP_EINVAL, "partition_bytes: bad arguments");
    uint64_t total = 0;
    for (size_t i = 0; i < n; ++i)
        total += recs[i].len;
    /* range r ends right after the first record whose prefix sum reaches ceil(total * (r + 1) / parts) (bench.py
     * partition_bytes is the same rule) */
    bounds[0] = 0;
    size_t i = 0;
    uint64_t csum = 0;
    for (size_t r = 1; r < parts; ++r) {
        const unsigned __int128 t = ((unsigned __int128)total * r + parts - 1) / parts;
        const uint64_t target = (uint64_t)t;
        if (total == 0) {
            bounds[r] = 0;
            continue;
        }
        while (i < n && csum < target)
            csum += recs[i++].len;
        bounds[r] = std::max(bounds[r - 1], i);
    }
    bounds[parts] = n;
    return 0;
}

struct st_ptls_hip_node_t {
    std::vector<ptls_hip_engine_t *> eng;
    std::vector<ptls_hip_keyset_t *> ks;
    std::vector<ptls_hip_pipeline_t *> pipe;
    std::vector<int> numa;       /* each device's NUMA node (-1: unknown) */
    std::vector<double> seconds; /* per device, last call */
    std::vector<size_t> bounds;  /* record ranges of the last call */
};

/* ---- NUMA placement (host buffers on each GPU's local node) ---- */

static std::vector<int> parse_cpulist(const char *text)
{
    std::vector<int> out;
    const char *p = text;
    while (*p != '\0' && *p != '\n') {
        char *end = nullptr;
        const long a = strtol(p, &end, 10);
        if (end == p)
            break;
        long b = a;
        p = end;
        if (*p == '-') {
            b = strtol(p + 1, &end, 10);
            p = end;
        }
        for (long c = a; c <= b; ++c)
            out.push_back((int)c);
        if (*p == ',')
            ++p;
    }
    return out;
}

static std::string read_small_file(const std::string &path)
{
    FILE *f = fopen(path.c_str(), "r");
    if (f == nullptr)
        return std::string();
    char buf[4096];
    const size_t n = fread(buf, 1, sizeof(buf) - 1, f);
    fclose(f);
    buf[n] = '\0';
    return std::string(buf);
}

extern "C" int ptls_hip_device_numa_node(int device)
{
    char bdf[64] = {0};
    if (hipDeviceGetPCIBusId(bdf, sizeof(bdf), device) != hipSuccess)
        return -1;
    for (char *c = bdf; *c != '\0'; ++c)
        *c = (char)tolower(*c);
    const std::string v = read_small_file(std::string("/sys/bus/pci/devices/") + bdf + "/numa_node");
    return v.empty() ? -1 : atoi(v.c_str());
}

/* the CPUs of NUMA node `node` this process may run on (empty: unknown node, or none allowed) */
static std::vector<int> node_cpus(int node)
{
    std::vector<int> out;
    if (node < 0)
        return out;
    cpu_set_t allowed;
    CPU_ZERO(&allowed);
    if (sched_getaffinity(0, sizeof(allowed), &allowed) != 0)
        return out;
    for (int c : parse_cpulist(read_small_file("/sys/devices/system/node/node" + std::to_string(node) + "/cpulist").c_str()))
        if (c >= 0 && c < CPU_SETSIZE && CPU_ISSET(c, &allowed))
            out.push_back(c);
    return out;
}

/* the calling thread runs on `node`'s CPUs (when it has any this process may use) */
static void pin_thread_to_node(int node)
{
    const std::vector<int> cpus = node_cpus(node);
    if (cpus.empty())
        return;
    cpu_set_t s;
    CPU_ZERO(&s);
    for (int c : cpus)
        CPU_SET(c, &s);
    (void)pthread_setaffinity_np(pthread_self(), sizeof(s), &s);
}

static long sys_mbind(void *addr, unsigned long len, int mode, const unsigned long *mask, unsigned long maxnode, unsigned flags)
{
    return syscall(SYS_mbind, addr, len, mode, mask, maxnode, flags);
}

extern "C" void ptls_hip_node_free(ptls_hip_node_t *node)
{
    if (node == nullptr)
        return;
    for (auto *p : node->pipe)
        ptls_hip_pipeline_free(p);
    for (auto *k : node->ks)
        ptls_hip_keyset_free(k);
    for (auto *e : node->eng)
        ptls_hip_engine_free(e);
    delete node;
}

extern "C" ptls_hip_node_t *ptls_hip_node_new(const int *devices, size_t ndev, size_t key_size, size_t nslots, size_t slice_bytes)
{
    if (devices == nullptr || ndev == 0 || ndev > 64) {
        fail(PTLS_HIP_EINVAL, "node_new: 1 to 64 devices");
        return nullptr;
    }
    auto *node = new st_ptls_hip_node_t();
    for (size_t d = 0; d < ndev; ++d) {
        ptls_hip_engine_t *e = ptls_hip_engine_new(devices[d]);
        node->eng.push_back(e);
        ptls_hip_keyset_t *k = e != nullptr ? ptls_hip_keyset_new(e, key_size, nslots) : nullptr;
        node->ks.push_back(k);
        ptls_hip_pipeline_t *p = k != nullptr ? ptls_hip_pipeline_new(e, slice_bytes) : nullptr;
        node->pipe.push_back(p);
        if (p == nullptr) {
            const std::string why = g_err;
            ptls_hip_node_free(node);
            fail(PTLS_HIP_ENODEV, "node_new: device %d: %s", devices[d], why.c_str());
            return nullptr;
        }
    }
    for (size_t d = 0; d < ndev; ++d)
        node->numa.push_back(ptls_hip_device_numa_node(devices[d]));
    node->seconds.assign(ndev, 0.0);
    node->bounds.assign(ndev + 1, 0);
    return node;
}

extern "C" int ptls_hip_node_numa(ptls_hip_node_t *node, int *numa_nodes)
{
    if (node == nullptr || numa_nodes == nullptr)
        return fail(PTLS_HIP_EINVAL, "node_numa: bad arguments");
    std::copy(node->numa.begin(), node->numa.end(), numa_nodes);
    return 0;
}

/* Host memory for a node's records: `bytes` of anonymous memory whose byte range [splits[d], splits[d + 1]) is bound
 * (mbind MPOL_BIND) to device d's NUMA node and faulted in there, then registered with every device (hipHostRegister,
 * mapped + portable) so either transport can use it.  A device whose node is unknown leaves its range to first touch. */
extern "C" void *ptls_hip_node_host_alloc(ptls_hip_node_t *node, size_t bytes, const size_t *splits)
{
    if (node == nullptr || bytes == 0 || splits == nullptr || splits[0] != 0 || splits[node->eng.size()] != bytes) {
        fail(PTLS_HIP_EINVAL, "node_host_alloc: splits must run from 0 to bytes, one range per device");
        return nullptr;
    }
    const size_t pg = (size_t)sysconf(_SC_PAGESIZE), len = (bytes + pg - 1) / pg * pg;
    void *p = mmap(nullptr, len, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (p == MAP_FAILED) {
        fail(PTLS_HIP_ENOMEM, "node_host_alloc: mmap of %zu bytes failed", bytes);
        return nullptr;
    }
    uint8_t *base = static_cast<uint8_t *>(p);
    for (size_t d = 0; d < node->eng.size(); ++d) {
        if (splits[d + 1] < splits[d]) {
            munmap(p, len);
            fail(PTLS_HIP_EINVAL, "node_host_alloc: splits must not decrease");
            return nullptr;
        }
        /* whole pages: a page shared by two ranges goes with the first */
        const size_t lo = (splits[d] + pg - 1) / pg * pg, hi = d + 1 == node->eng.size() ? len : (splits[d + 1] + pg - 1) / pg * pg;
        const int nd = node->numa[d];
        if (hi > lo && nd >= 0 && nd < 1024) {
            unsigned long mask[1024 / (8 * sizeof(unsigned long))] = {0};
            mask[nd / (8 * sizeof(unsigned long))] |= 1ul << (nd % (8 * sizeof(unsigned long)));
            (void)sys_mbind(base + lo, hi - lo, 2 /* MPOL_BIND */, mask, 1024 + 1, 0);
        }
        if (hi > lo)
            std::memset(base + lo, 0, hi - lo); /* fault the pages in on their node */
    }
    if (hipHostRegister(p, len, hipHostRegisterMapped | hipHostRegisterPortable) != hipSuccess) {
        munmap(p, len);
        fail(PTLS_HIP_ENOMEM, "node_host_alloc: hipHostRegister failed");
        return nullptr;
    }
    return p;
}

extern "C" void ptls_hip_node_host_free(void *ptr, size_t bytes)
{
    if (ptr == nullptr)
        return;
    const size_t pg = (size_t)sysconf(_SC_PAGESIZE), len = (bytes + pg - 1) / pg * pg;
    (void)hipHostUnregister(ptr);
    munmap(ptr, len);
}

/* the NUMA node of every `stride`-th page of [ptr, ptr + bytes) (move_pages query), written to nodes (-errno for a page
 * not present); returns the number of pages written */
extern "C" size_t ptls_hip_host_page_nodes(const void *ptr, size_t bytes, size_t stride, int *nodes, size_t cap)
{
    const size_t pg = (size_t)sysconf(_SC_PAGESIZE);
    std::vector<void *> pages;
    for (size_t off = 0; off < bytes && pages.size() < cap; off += pg * (stride ? stride : 1))
        pages.push_back(const_cast<uint8_t *>(static_cast<const uint8_t *>(ptr)) + off);
    if (pages.empty())
        return 0;
    if (syscall(SYS_move_pages, 0, pages.size(), pages.data(), nullptr, nodes, 0) != 0)
        return 0;
    return pages.size();
}

extern "C" size_t ptls_hip_node_size(ptls_hip_node_t *node)
{
    return node != nullptr ? node->eng.size() : 0;
}

extern "C" int ptls_hip_node_keyset_set(ptls_hip_node_t *node, size_t first, size_t count, const void *keys, const void *ivs)
{
    if (node == nullptr)
        return fail(PTLS_HIP_EINVAL, "node_keyset_set: null node");
    for (auto *k : node->ks) /* replicated: every device holds every connection's key slot */
        if (int rc = ptls_hip_keyset_set(k, first, count, keys, ivs, nullptr))
            return rc;
    return 0;
}

extern "C" int ptls_hip_node_set_transport(ptls_hip_node_t *node, int transport)
{
    if (node == nullptr)
        return fail(PTLS_HIP_EINVAL, "node_set_transport: null node");
    for (auto *p : node->pipe)
        if (int rc = ptls_hip_pipeline_set_transport(p, transport))
            return rc;
    return 0;
}

/* the records split in contiguous ranges of about equal payload bytes, one host thread per device driving its own
 * pipeline over its range (the host buffers are shared: offsets stay relative to them), no data crossing devices */
static int node_run(ptls_hip_node_t *node, const ptls_hip_record_t *recs, size_t n, const void *h_in, const void *h_aad,
                    void *h_out, uint64_t *h_result, bool open)
{
    if (node == nullptr || (n != 0 && (recs == nullptr || h_in == nullptr || h_out == nullptr)) || (open && h_result == nullptr))
        return fail(PTLS_HIP_EINVAL, "node seal/open: bad arguments");
    const size_t nd = node->eng.size();
    if (int rc = ptls_hip_partition_bytes(recs, n, nd, node->bounds.data()))
        return rc;
    std::vector<int> rcs(nd, 0);
    std::vector<std::string> errs(nd);
    std::vector<std::thread> th;
    for (size_t d = 0; d < nd; ++d) {
        th.emplace_back([&, d]() {
            pin_thread_to_node(node->numa[d]); /* the device's host thread plans and stages on the device's own node */
            const size_t lo = node->bounds[d], hi = node->bounds[d + 1];
            const auto t0 = std::chrono::steady_clock::now();
            int rc = 0;
            if (hi > lo)
                rc = open ? ptls_hip_pipeline_open(node->pipe[d], node->ks[d], recs + lo, hi - lo, h_in, h_aad, h_out, h_result + lo)
                          : ptls_hip_pipeline_seal(node->pipe[d], node->ks[d], recs + lo, hi - lo, h_in, h_aad, h_out);
            node->seconds[d] = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
            rcs[d] = rc;
            if (rc != 0)
                errs[d] = g_err; /* thread_local: carried back to the caller's thread */
        });
    }
    for (auto &t : th)
        t.join();
    for (size_t d = 0; d < nd; ++d)
        if (rcs[d] != 0)
            return fail(rcs[d], "node: device %d: %s", node->eng[d]->device, errs[d].c_str());
    return 0;
}

extern "C" int ptls_hip_node_seal(ptls_hip_node_t *node, const ptls_hip_record_t *recs, size_t n, const void *h_in, const void *h_aad,
                                  void *h_out)
{
    return node_run(node, recs, n, h_in, h_aad, h_out, nullptr, false);
}

extern "C" int ptls_hip_node_open(ptls_hip_node_t *node, const ptls_hip_record_t *recs, size_t n, const void *h_in, const void *h_aad,
                                  void *h_out, uint64_t *h_result)
{
    return node_run(node, recs, n, h_in, h_aad, h_out, h_result, true);
}

extern "C" int ptls_hip_node_last_split(ptls_hip_node_t *node, double *seconds, size_t *bounds)
{
    if (node == nullptr)
        return fail(PTLS_HIP_EINVAL, "node_last_split: null node");
    if (seconds != nullptr)
        std::copy(node->seconds.begin(), node->seconds.end(), seconds);
    if (bounds != nullptr)
        std::copy(node->bounds.begin(), node->bounds.end(), bounds);
    return 0;
}

/* ---------------------------------------------------------------------------------------------- */
/* picotls plugin: ptls_hip_aes128gcm / ptls_hip_aes256gcm                                         */
/* ---------------------------------------------------------------------------------------------- */

static std::mutex g_plugin_mu;
static ptls_hip_engine_t *g_plugin_engine = nullptr;
static int g_plugin_device = -1;

extern "C" int ptls_hip_set_default_device(int device)
{
    std::lock_guard<std::mutex> lk(g_plugin_mu);
    if (g_plugin_engine != nullptr)
        return fail(PTLS_HIP_EINVAL, "set_default_device: contexts already created on device %d", g_plugin_engine->device);
    g_plugin_device = device;
    return 0;
}

static ptls_hip_engine_t *plugin_engine(void)
{
    std::lock_guard<std::mutex> lk(g_plugin_mu);
    if (g_plugin_engine == nullptr) {
        int dev = g_plugin_device;
        if (dev < 0) {
            const char *env = getenv("PTLS_HIP_DEVICE");
            dev = env != nullptr ? atoi(env) : 0;
        }
        g_plugin_engine = ptls_hip_engine_new(dev);
    }
    return g_plugin_engine;
}

/* per-context state: one pooled key slot.  A call through the worker carries the record, the context's IV and the
 * output in a mailbox (pinned, device-mapped: the kernel reads and writes it over PCIe itself, no copy engine); the
 * context's own pinned staging exists only for records that do not fit a mailbox and for launched calls
 * (PTLS_HIP_PLUGIN_WORKER=0), and is allocated on first use. */
struct hip_aead_state {
    ptls_hip_engine_t *eng;
    ptls_hip_keyset_t *ks;
    uint8_t *h_io, *d_io; /* pinned [in: cap][out: cap + 16][aad: aad_cap] and its device address (lazy) */
    size_t cap, aad_cap;
    uint8_t *h_stage, *d_stage; /* pooled 256-B pinned piece: result, supp, mask, completion word (ST_*) (lazy) */
    uint8_t iv[12];
    bool iv_dirty;     /* launched calls: the slot's IV must be uploaded before the next launch */
    uint32_t done_seq; /* completion word sequence of the last launched call (ST_DONE) */
};

struct hip_aead_context {
    ptls_aead_context_t super;
    hip_aead_state *st; /* nullptr after an IV-only setup of a fresh context */
    uint8_t iv[12];     /* the static IV of such a context (fusion keeps it in static_iv, lib/fusion.c:1188-1189) */
};

[[noreturn]] static void plugin_die(const char *what)
{
    fprintf(stderr, "ptls_hip: fatal device error in %s: %s\n", what, g_err.c_str());
    abort();
}

static void plugin_check(hipError_t e, const char *what)
{
    if (e != hipSuccess) {
        g_err = hipGetErrorString(e);
        plugin_die(what);
    }
}

/* Wait for a plugin launch by spinning on its completion word in pinned host memory (the kernel stores the call's
 * sequence number there after everything else, system scope) instead of hipStreamSynchronize's completion path
 * (DESIGN.md §6.2).  A call whose word does not show up within 2 s falls back to the stream synchronize, which
 * reports a device fault; a kernel that completed without writing the word is a bug. */
static void plugin_wait(hipStream_t stream, const uint8_t *word_p, uint32_t seq)
{
    const uint32_t *word = reinterpret_cast<const uint32_t *>(word_p);
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t spin = 1;; ++spin) {
        if (__atomic_load_n(word, __ATOMIC_ACQUIRE) == seq)
            return;
#if defined(__x86_64__) || defined(__i386__)
        __builtin_ia32_pause();
#else
        std::this_thread::yield();
#endif
        if ((spin & 4095) == 0 && std::chrono::steady_clock::now() - t0 > std::chrono::seconds(2))
            break;
    }
    plugin_check(hipStreamSynchronize(stream), "hipStreamSynchronize");
    if (__atomic_load_n(word, __ATOMIC_ACQUIRE) != seq) {
        g_err = "kernel completed without its completion word";
        plugin_die("plugin_wait");
    }
}

static unsigned staging_flags(void);

/* ---- the plugin worker (sparse_kernel.hip plugin_worker_kernel) ------------------------------------------------- *
 * A plugin call launches nothing while the worker is resident: it writes its request into a mailbox (pinned,
 * fine-grained), then waits on its completion word as a launched call does.  The worker is ONE dispatch of `n`
 * workgroups, workgroup j serving mailbox j; a calling thread has a home mailbox (threads are spread over them round
 * robin) and takes any free one when its home is busy, so calls from different threads run side by side on different
 * CUs (lib/fusion.c contexts share no state either, :1135-1166).  The workgroups leave together after WORKER_IDLE_US
 * without a request on any of them, after WORKER_LIFE_US in any case (the dispatch must not hold its hardware queue), or
 * when asked; a call that finds its workgroup gone waits for the whole dispatch to drain and launches the next one.
 * On by default; PTLS_HIP_PLUGIN_WORKER=0 (environment) makes every call launch its own kernel instead;
 * PTLS_HIP_PLUGIN_WORKERS=n sets the number of mailboxes / workgroups (default 16, 1..64: 16 threads measured 13.6x one
 * thread's calls per second, tools/plugin_mt.py; the dispatch holds that many CUs while it is resident). */
static uint64_t worker_env_us(const char *name, uint64_t dflt)
{
    const char *e = getenv(name);
    const long long v = e != nullptr ? atoll(e) : -1;
    return v > 0 ? (uint64_t)v : dflt;
}
/* PTLS_HIP_WORKER_IDLE_US / PTLS_HIP_WORKER_LIFE_US (environment) override: a hipFree anywhere in the process synchronizes
 * the device and so waits for a resident dispatch, at most the lifetime */
static const uint64_t WORKER_IDLE_US = worker_env_us("PTLS_HIP_WORKER_IDLE_US", 200),
                      WORKER_LIFE_US = worker_env_us("PTLS_HIP_WORKER_LIFE_US", 2000);
static const unsigned WORKER_MAX = 64;

struct Mailbox {
    std::mutex mu;         /* held for a whole call */
    uint32_t seq = 0;      /* the last request number written */
    uint32_t done_seq = 0; /* the last completion-word value asked for */
};

struct PluginWorker {
    std::mutex launch_mu; /* launching / draining the dispatch */
    ptls_hip_engine_t *eng = nullptr;
    hipStream_t stream = nullptr;
    unsigned n = 0;
    WorkerSlot *h_mb = nullptr, *d_mb = nullptr;
    /* set (release) once worker_init has filled every field above; the unlocked fast paths test it (acquire) before they
     * read h_mb, n, d_mb or eng (a plain pointer store published nothing) */
    std::atomic<bool> ready{false};
    uint64_t *d_activity = nullptr;   /* the last time any workgroup served a request (100 MHz ticks) */
    std::atomic<uint32_t> epoch{0};   /* of the last dispatch launched; h_mb[j].exited == epoch: workgroup j has left */
    std::atomic<bool> launched{false};
    std::atomic<unsigned> next_home{0};
    Mailbox mbox[WORKER_MAX];
};
static PluginWorker g_worker;

static bool worker_enabled(void)
{
    static const bool on = [] {
        const char *e = getenv("PTLS_HIP_PLUGIN_WORKER");
        return e == nullptr || atoi(e) != 0;
    }();
    return on;
}

static unsigned worker_count(void)
{
    static const unsigned n = [] {
        const char *e = getenv("PTLS_HIP_PLUGIN_WORKERS");
        const int v = e != nullptr ? atoi(e) : 16;
        return (unsigned)std::max(1, std::min(v, (int)WORKER_MAX));
    }();
    return n;
}

static uint32_t load_acquire(const uint32_t *p)
{
    return __atomic_load_n(p, __ATOMIC_ACQUIRE);
}

static void cpu_relax(void)
{
#if defined(__x86_64__) || defined(__i386__)
    __builtin_ia32_pause();
#else
    std::this_thread::yield();
#endif
}

/* every workgroup of dispatch `epoch` has left (or none was launched) */
static bool worker_drained(const PluginWorker &w, uint32_t epoch)
{
    if (!w.launched.load(std::memory_order_acquire) || w.epoch.load(std::memory_order_acquire) != epoch)
        return true; /* a later dispatch exists: this one was drained before it was launched (worker_ensure) */
    for (unsigned j = 0; j < w.n; ++j)
        if (load_acquire(&w.h_mb[j].exited) != epoch)
            return false;
    return true;
}

/* at process exit (atexit: before the HIP runtime's own teardown): ask the resident workgroups to leave and wait for them,
 * with host memory only, so no kernel is running when the process ends */
static void worker_atexit(void)
{
    PluginWorker &w = g_worker;
    if (!w.ready.load(std::memory_order_acquire) || !w.launched.load())
        return;
    for (unsigned j = 0; j < w.n; ++j)
        __atomic_store_n(&w.h_mb[j].quit, 1u, __ATOMIC_RELEASE);
    const auto t0 = std::chrono::steady_clock::now();
    while (!worker_drained(w, w.epoch.load()) && std::chrono::steady_clock::now() - t0 < std::chrono::milliseconds(50))
        std::this_thread::yield();
}

/* under launch_mu: the mailboxes (fine-grained pinned host memory), the activity word and the stream, on the plugin
 * engine's device */
static void worker_init(PluginWorker &w, ptls_hip_engine_t *eng)
{
    if (w.ready.load(std::memory_order_acquire))
        return;
    DeviceGuard g(eng->device);
    const unsigned n = worker_count();
    void *d = nullptr;
    WorkerSlot *h = nullptr;
    /* the dispatch's stream at the device's greatest priority: the runtime gives each priority its own pool of hardware
     * queues (GPU_MAX_HW_QUEUES each), so no other stream of the process shares the worker's queue and waits behind the
     * resident dispatch (a key setup on a pooled stream that did: ptls_aead_new 244 us = the worker's idle exit + 44) */
    int prio_least = 0, prio_greatest = 0;
    if (hipDeviceGetStreamPriorityRange(&prio_least, &prio_greatest) != hipSuccess)
        prio_greatest = prio_least = 0;
    if (hipStreamCreateWithPriority(&w.stream, hipStreamNonBlocking, prio_greatest) != hipSuccess ||
        hipHostMalloc(reinterpret_cast<void **>(&h), n * sizeof(WorkerSlot), hipHostMallocCoherent) != hipSuccess ||
        hipHostGetDevicePointer(&d, h, 0) != hipSuccess || hipMalloc(&w.d_activity, sizeof(uint64_t)) != hipSuccess ||
        hipMemset(w.d_activity, 0, sizeof(uint64_t)) != hipSuccess) {
        g_err = "plugin worker mailboxes";
        plugin_die("worker_init");
    }
    std::memset(h, 0, n * sizeof(WorkerSlot));
    w.eng = eng;
    w.n = n;
    w.d_mb = static_cast<WorkerSlot *>(d);
    w.h_mb = h;
    atexit(worker_atexit);
    w.ready.store(true, std::memory_order_release); /* published last: the fast paths test `ready` first */
}

/* With mailbox j's lock held: a dispatch whose workgroup j has not left.  A dispatch in which it has left is drained first
 * (every workgroup asked to quit; one with a request pending serves it before it leaves), so two dispatches never serve
 * one mailbox, and a request written before the next launch is served by it (a workgroup starts from `served`). */
static void worker_ensure(PluginWorker &w, unsigned j)
{
    if (w.launched.load(std::memory_order_acquire) && load_acquire(&w.h_mb[j].exited) != w.epoch.load(std::memory_order_acquire))
        return;
    std::lock_guard<std::mutex> lk(w.launch_mu);
    DeviceGuard g(w.eng->device);
    const uint32_t ep = w.epoch.load();
    if (w.launched.load() && load_acquire(&w.h_mb[j].exited) == ep) {
        if (!worker_drained(w, ep)) {
            for (unsigned k = 0; k < w.n; ++k)
                __atomic_store_n(&w.h_mb[k].quit, 1u, __ATOMIC_RELEASE);
            const auto t0 = std::chrono::steady_clock::now();
            while (!worker_drained(w, ep)) {
                if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(2)) {
                    /* a workgroup that never started (the CUs were held by other kernels): the dispatch ends once it has
                     * run; a device fault is reported here */
                    plugin_check(hipStreamSynchronize(w.stream), "plugin worker drain");
                    if (!worker_drained(w, ep)) {
                        g_err = "the plugin worker dispatch completed with a workgroup that did not report its exit";
                        plugin_die("worker_ensure");
                    }
                    break;
                }
                std::this_thread::yield();
            }
            for (unsigned k = 0; k < w.n; ++k)
                __atomic_store_n(&w.h_mb[k].quit, 0u, __ATOMIC_RELEASE);
        }
        w.launched.store(false, std::memory_order_release);
    }
    if (!w.launched.load()) {
        const uint32_t next = ep + 1;
        const int e = launch_plugin_worker(w.d_mb, w.n, next, w.eng->d_t0, WORKER_IDLE_US * 100, WORKER_LIFE_US * 100, w.d_activity,
                                           w.stream);
        if (e != 0) {
            g_err = hipGetErrorString((hipError_t)e);
            plugin_die("plugin worker launch");
        }
        w.epoch.store(next, std::memory_order_release);
        w.launched.store(true, std::memory_order_release);
    }
}

/* a mailbox for this call, locked: the thread's home mailbox, or the first free one, or (all busy) the home one */
static unsigned worker_acquire(PluginWorker &w)
{
    static thread_local int home = -1;
    if (home < 0)
        home = (int)(w.next_home.fetch_add(1) % w.n);
    if (w.mbox[home].mu.try_lock())
        return (unsigned)home;
    for (unsigned k = 1; k < w.n; ++k) {
        const unsigned j = ((unsigned)home + k) % w.n;
        if (w.mbox[j].mu.try_lock())
            return j;
    }
    w.mbox[home].mu.lock();
    return (unsigned)home;
}

#ifndef WORKER_STAMPS
#define WORKER_STAMPS 0 /* diagnostic build only (Makefile `diag`) */
#endif
#if WORKER_STAMPS
/* diagnostic build: the worker's phase stamps of the last request on mailbox 0 and the host's wall-clock microseconds of
 * that call */
static double g_worker_call_us = 0;
extern "C" int ptls_hip_diag_worker_stamps(uint64_t *out, double *call_us)
{
    if (!g_worker.ready.load(std::memory_order_acquire))
        return -1;
    for (int i = 0; i < 5; ++i)
        out[i] = __atomic_load_n(&g_worker.h_mb->stamps[i], __ATOMIC_ACQUIRE);
    /* the record's phase stamps (shader cycles): clk[1] request loaded, clk[2..8] sparse_record's phases, clk[9] done */
    const uint64_t *clk = reinterpret_cast<const uint64_t *>(g_worker.h_mb->data + WORKER_DATA - 128);
    for (int i = 0; i < 10; ++i)
        out[5 + i] = __atomic_load_n(&clk[i], __ATOMIC_ACQUIRE);
    *call_us = g_worker_call_us;
    return 0;
}
#endif

/* one request through mailbox j (its lock held); returns once the call's completion word shows done_seq (the same
 * protocol as a launched call, plugin_wait).  A workgroup that left without serving the request is replaced (the next
 * dispatch serves it: seq != served).  A dispatch that has not started after 2 s (every CU held by other kernels) is
 * waited for with a stream synchronize, which also reports a device fault. */
static void worker_call(unsigned j, const WorkerReq &req, const uint8_t *word_p)
{
    PluginWorker &w = g_worker;
    Mailbox &m = w.mbox[j];
    WorkerSlot *mb = &w.h_mb[j];
    worker_ensure(w, j);
    mb->req = req;
    const auto tc = std::chrono::steady_clock::now();
    __atomic_store_n(&mb->seq, ++m.seq, __ATOMIC_RELEASE);
    const uint32_t *word = reinterpret_cast<const uint32_t *>(word_p);
    auto t0 = std::chrono::steady_clock::now();
    for (uint32_t spin = 1;; ++spin) {
        if (load_acquire(word) == req.done_seq) {
#if WORKER_STAMPS
            g_worker_call_us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - tc).count();
#endif
            (void)tc;
            return;
        }
        cpu_relax();
        if ((spin & 1023) != 0)
            continue;
        if (load_acquire(&mb->exited) == w.epoch.load(std::memory_order_acquire) && load_acquire(&mb->served) != m.seq) {
            worker_ensure(w, j); /* it left (idle / lifetime / drained) just before the request: the next dispatch serves it */
            t0 = std::chrono::steady_clock::now();
        } else if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(2)) {
            DeviceGuard g(w.eng->device);
            plugin_check(hipStreamSynchronize(w.stream), "plugin worker");
            if (load_acquire(word) == req.done_seq)
                return;
            if (load_acquire(&mb->served) != m.seq) { /* the dispatch ended without it: the next one serves it */
                worker_ensure(w, j);
                t0 = std::chrono::steady_clock::now();
                continue;
            }
            static char msg[256];
            snprintf(msg, sizeof(msg),
                     "the plugin worker served request %u without its completion word (mailbox %u, seen %u, epoch %u, started %u, "
                     "exited %u, word %u of %u)",
                     m.seq, j, load_acquire(&mb->seen), w.epoch.load(), load_acquire(&mb->started), load_acquire(&mb->exited),
                     load_acquire(word), req.done_seq);
            g_err = msg;
            plugin_die("worker_call");
        }
    }
}

/* ---- pooled plugin resources --------------------------------------------------------------------------------------- *
 * A picotls application creates and frees AEAD contexts per connection (lib/picotls.c:6458-6479: a malloc and a key
 * expansion for fusion, lib/fusion.c:984-1010).  Device memory, pinned host memory and streams are expensive to create
 * and to free (hipFree / hipHostFree synchronize), so the plugin keeps them in pools:
 *   - key slots: blocks of POOL_BLOCK KeySlot + GHASH basis, each with pinned staging for the raw keys the key-setup kernel
 *     reads in place.  A freed slot is zeroed on the device (async) and retired; it is handed out again only after that
 *     zeroing has completed AND every worker dispatch that could have read it has left, so the resident worker never
 *     sees a slot it has cached change under it (its key loads are vector loads after a system-scope acquire, and each
 *     dispatch starts with its caches invalidated).
 *   - streams for key setup and launched calls: taken for one operation, then returned.
 *   - 256-byte pieces of pinned staging (completion words, ECB blocks, launched calls' results). */
static const uint32_t POOL_BLOCK = 64;

struct SlotPool {
    std::mutex mu;
    struct Block {
        KeySlot *d_slots;
        uint32_t *d_basis;
        uint8_t *h_keys, *d_keys; /* pinned: [POOL_BLOCK][64] = key (32) | iv (12) */
    };
    std::vector<Block> blocks[2]; /* [AES-128, AES-256] */
    std::vector<uint32_t> free_ids[2];
    struct Retired {
        uint32_t id;
        uint32_t epoch; /* worker dispatch resident when it was freed (0: none) */
        hipEvent_t zeroed;
    };
    std::vector<Retired> retired[2];
    std::vector<hipStream_t> streams;
    std::vector<hipEvent_t> events;
    std::vector<uint8_t *> pieces; /* free 256-B pinned pieces */
};
static SlotPool g_pool;

static hipStream_t pool_stream(void)
{
    {
        std::lock_guard<std::mutex> lk(g_pool.mu);
        if (!g_pool.streams.empty()) {
            hipStream_t s = g_pool.streams.back();
            g_pool.streams.pop_back();
            return s;
        }
    }
    hipStream_t s = nullptr;
    plugin_check(hipStreamCreateWithFlags(&s, hipStreamNonBlocking), "hipStreamCreate(pool)");
    return s;
}

static void pool_stream_put(hipStream_t s)
{
    std::lock_guard<std::mutex> lk(g_pool.mu);
    g_pool.streams.push_back(s);
}

/* a 256-B piece of pinned, device-mapped staging (zeroed) */
static uint8_t *pool_piece(void)
{
    std::lock_guard<std::mutex> lk(g_pool.mu);
    if (g_pool.pieces.empty()) {
        uint8_t *h = nullptr;
        plugin_check(hipHostMalloc(reinterpret_cast<void **>(&h), 64 * 256, staging_flags()), "hipHostMalloc(pieces)");
        std::memset(h, 0, 64 * 256);
        for (int k = 63; k >= 0; --k)
            g_pool.pieces.push_back(h + 256 * k);
    }
    uint8_t *p = g_pool.pieces.back();
    g_pool.pieces.pop_back();
    return p;
}

static void pool_piece_put(uint8_t *p)
{
    std::memset(p, 0, 256);
    std::lock_guard<std::mutex> lk(g_pool.mu);
    g_pool.pieces.push_back(p);
}

/* under g_pool.mu: a slot id of key size class c (0: AES-128, 1: AES-256), recycling retired slots that are safe to reuse */
static uint32_t pool_take_locked(ptls_hip_engine_t *eng, int c)
{
    auto &ret = g_pool.retired[c];
    for (size_t k = 0; k < ret.size();) {
        /* the epoch test first: a slot of the resident dispatch costs no runtime call (the list holds at most one
         * dispatch lifetime of frees, WORKER_LIFE_US) */
        if ((ret[k].epoch == 0 || worker_drained(g_worker, ret[k].epoch)) && hipEventQuery(ret[k].zeroed) == hipSuccess) {
            g_pool.free_ids[c].push_back(ret[k].id);
            g_pool.events.push_back(ret[k].zeroed);
            ret[k] = ret.back();
            ret.pop_back();
        } else {
            ++k;
        }
    }
    if (g_pool.free_ids[c].empty()) {
        SlotPool::Block b{};
        void *dk = nullptr;
        if (hipMalloc(&b.d_slots, POOL_BLOCK * sizeof(KeySlot)) != hipSuccess ||
            hipMalloc(&b.d_basis, POOL_BLOCK * BASIS_WORDS_PER_SLOT * 4) != hipSuccess ||
            hipHostMalloc(reinterpret_cast<void **>(&b.h_keys), POOL_BLOCK * 64, staging_flags()) != hipSuccess ||
            hipHostGetDevicePointer(&dk, b.h_keys, 0) != hipSuccess) {
            g_err = "cannot allocate plugin key slots";
            return UINT32_MAX;
        }
        (void)eng;
        b.d_keys = static_cast<uint8_t *>(dk);
        std::memset(b.h_keys, 0, POOL_BLOCK * 64);
        const uint32_t base = (uint32_t)g_pool.blocks[c].size() * POOL_BLOCK;
        g_pool.blocks[c].push_back(b);
        for (uint32_t k = POOL_BLOCK; k-- > 0;)
            g_pool.free_ids[c].push_back(base + k);
    }
    const uint32_t id = g_pool.free_ids[c].back();
    g_pool.free_ids[c].pop_back();
    return id;
}

/* a one-slot keyset on a pooled slot, keyed (key setup on the device from the slot's pinned key staging) */
static ptls_hip_keyset_t *pool_keyset(ptls_hip_engine_t *eng, size_t key_size, const void *key, const void *iv)
{
    const int c = key_size == 32 ? 1 : 0;
    uint32_t id;
    SlotPool::Block b;
    {
        std::lock_guard<std::mutex> lk(g_pool.mu);
        id = pool_take_locked(eng, c);
        if (id == UINT32_MAX)
            return nullptr;
        b = g_pool.blocks[c][id / POOL_BLOCK];
    }
    const uint32_t k = id % POOL_BLOCK;
    auto *ks = new st_ptls_hip_keyset_t();
    ks->eng = eng;
    ks->key_size = key_size;
    ks->nslots = 1;
    ks->d_slots = b.d_slots + k;
    ks->d_basis = b.d_basis + (size_t)k * BASIS_WORDS_PER_SLOT;
    ks->pool_id = (int64_t)id;
    ks->ivs.assign(12, 0);
    uint8_t *hk = b.h_keys + 64 * k;
    std::memcpy(hk, key, key_size);
    if (iv != nullptr)
        std::memcpy(hk + 32, iv, 12);
    hipStream_t s = pool_stream();
    const int e = launch_keysetup(b.d_slots, b.d_basis, b.d_keys + 64 * k, b.d_keys + 64 * k + 32, k, 1, (int)key_size, eng->d_t0, s);
    const hipError_t se = e == 0 ? hipStreamSynchronize(s) : (hipError_t)e;
    pool_stream_put(s);
    std::memset(hk, 0, 64); /* the raw key does not stay in host memory */
    if (se != hipSuccess) {
        g_err = hipGetErrorString(se);
        ptls_hip_keyset_free(ks);
        return nullptr;
    }
    if (iv != nullptr)
        std::memcpy(ks->ivs.data(), iv, 12);
    return ks;
}

/* ptls_hip_keyset_free of a pooled keyset: zero the slot (async) and retire it; nothing waits */
static void pool_release(ptls_hip_keyset_t *ks)
{
    const int c = ks->key_size == 32 ? 1 : 0;
    const uint32_t id = (uint32_t)ks->pool_id;
    DeviceGuard g(ks->eng->device);
    hipStream_t s = pool_stream();
    hipEvent_t ev = nullptr;
    {
        std::lock_guard<std::mutex> lk(g_pool.mu);
        if (!g_pool.events.empty()) {
            ev = g_pool.events.back();
            g_pool.events.pop_back();
        }
    }
    if (ev == nullptr)
        plugin_check(hipEventCreateWithFlags(&ev, hipEventDisableTiming), "hipEventCreate(pool)");
    /* zeroize key material before release (ptls_clear_memory in aesgcm_dispose_crypto, lib/fusion.c:1102-1107) */
    plugin_check(hipMemsetAsync(ks->d_slots, 0, sizeof(KeySlot), s), "hipMemsetAsync(slot)");
    plugin_check(hipMemsetAsync(ks->d_basis, 0, BASIS_WORDS_PER_SLOT * 4, s), "hipMemsetAsync(basis)");
    plugin_check(hipEventRecord(ev, s), "hipEventRecord(pool)");
    pool_stream_put(s);
    const PluginWorker &w = g_worker;
    const uint32_t ep = w.ready.load(std::memory_order_acquire) && w.launched.load() ? w.epoch.load() : 0;
    std::lock_guard<std::mutex> lk(g_pool.mu);
    g_pool.retired[c].push_back(SlotPool::Retired{id, ep, ev});
}

static uint8_t *mapped_or_die(uint8_t *h);

/* ---- CTR cipher for header protection (replaces lib/fusion.c:1050-1100) ---------------------------- */

struct hip_ctr_state {
    ptls_hip_engine_t *eng;
    ptls_hip_keyset_t *ks; /* pooled slot */
    uint8_t *h_stage; /* pooled 256-B pinned piece: [output block @48][completion word @64] */
    uint8_t *d_stage; /* its device address: the kernel reads and writes it in place */
    uint8_t bits[16];
    bool ready;
    uint32_t done_seq; /* completion word sequence of the last block (ECB_DONE) */
};

struct hip_ctr_context {
    ptls_cipher_context_t super;
    hip_ctr_state *st;
};

extern "C" ptls_cipher_algorithm_t ptls_hip_aes128ctr, ptls_hip_aes256ctr;

static const hip_ctr_state *ctr_state_of(const ptls_cipher_context_t *c)
{
    if (c == nullptr || (c->algo != &ptls_hip_aes128ctr && c->algo != &ptls_hip_aes256ctr))
        return nullptr;
    return reinterpret_cast<const hip_ctr_context *>(c)->st;
}

/* ECB staging (128 B pinned): output block @48, completion word @64 (the input block travels in the kernel arguments) */
static const size_t ECB_DONE = 64;

/* one AES-ECB block on the device with the state's key (fusion: aesecb_encrypt, lib/fusion.c:322-334) */
static bool ecb_by_launch(void)
{
    static const bool on = [] { /* PTLS_HIP_ECB_LAUNCH=1 (environment): one launch per block even with the worker (A/B) */
        const char *e = getenv("PTLS_HIP_ECB_LAUNCH");
        return e != nullptr && atoi(e) != 0;
    }();
    return on;
}

static void ecb_block(hip_ctr_state *st, const void *src, uint8_t dst[16])
{
    DeviceGuard g(st->eng->device);
    if (worker_enabled() && !ecb_by_launch()) {
        /* through the worker: the block travels in the mailbox with the request (WREQ_ECB) */
        PluginWorker &w = g_worker;
        if (!w.ready.load(std::memory_order_acquire)) {
            std::lock_guard<std::mutex> lk(w.launch_mu);
            worker_init(w, st->eng);
        }
        const unsigned j = worker_acquire(w);
        WorkerSlot *h = &w.h_mb[j], *d = &w.d_mb[j];
        std::memcpy(h->data, src, 16);
        WorkerReq rq{};
        rq.in = rq.aad = d->data;
        rq.out = d->out;
        rq.result = reinterpret_cast<uint64_t *>(d->aux + WAUX_RESULT);
        rq.slots = st->ks->d_slots;
        rq.basis = st->ks->d_basis;
        rq.done = reinterpret_cast<uint32_t *>(d->aux + WAUX_DONE);
        rq.done_seq = ++w.mbox[j].done_seq;
        rq.flags = WREQ_ECB | WREQ_INLINE | (st->ks->key_size == 32 ? WREQ_AES256 : 0u);
        worker_call(j, rq, h->aux + WAUX_DONE);
        std::memcpy(dst, h->out, 16);
        std::memset(h->out, 0, 16);
        std::memset(h->data, 0, 16);
        w.mbox[j].mu.unlock();
        return;
    }
    /* one launch per block (worker off, or PTLS_HIP_ECB_LAUNCH=1): the block travels in the kernel arguments */
    /* the block goes in the kernel arguments; the result comes back through the pinned staging (@48) */
    hipStream_t stream = pool_stream();
    const int e = launch_aesecb_one(st->ks->key_size == 16 ? 10 : 14, static_cast<const uint8_t *>(src), st->ks->d_slots,
                                    st->eng->d_t0, st->d_stage + 48, reinterpret_cast<uint32_t *>(st->d_stage + ECB_DONE),
                                    ++st->done_seq, stream);
    if (e != 0) {
        g_err = hipGetErrorString((hipError_t)e);
        plugin_die("ecb launch");
    }
    plugin_wait(stream, st->h_stage + ECB_DONE, st->done_seq);
    pool_stream_put(stream);
    std::memcpy(dst, st->h_stage + 48, 16);
    std::memset(st->h_stage + 48, 0, 16);
}

/* do_init: the keystream block AES-ECB(key, iv) on the device (fusion: aesecb_encrypt, :1057-1062) */
static void ctr_init(ptls_cipher_context_t *_ctx, const void *iv)
{
    hip_ctr_state *st = reinterpret_cast<hip_ctr_context *>(_ctx)->st;
    ecb_block(st, iv, st->bits);
    st->ready = true;
}

/* do_transform: at most 16 bytes per do_init, like fusion's ctr_transform (:1064-1077) */
static void ctr_transform(ptls_cipher_context_t *_ctx, void *output, const void *input, size_t len)
{
    hip_ctr_state *st = reinterpret_cast<hip_ctr_context *>(_ctx)->st;
    if (!st->ready || len > 16) {
        fprintf(stderr, "ptls_hip: CTR transformation is supported only once per call to `init` and for at most 16 bytes\n");
        abort();
    }
    st->ready = false;
    for (size_t i = 0; i < len; ++i)
        static_cast<uint8_t *>(output)[i] = static_cast<const uint8_t *>(input)[i] ^ st->bits[i];
}

/* a one-key ECB state on the plugin engine's device: expanded key slot + 64 B of device / pinned staging */
static hip_ctr_state *ecb_state_new(const void *key, size_t key_size)
{
    ptls_hip_engine_t *eng = plugin_engine();
    if (eng == nullptr || key == nullptr)
        return nullptr;
    DeviceGuard g(eng->device);
    auto *st = new hip_ctr_state();
    st->eng = eng;
    st->ks = pool_keyset(eng, key_size, key, nullptr);
    if (st->ks == nullptr) {
        delete st;
        return nullptr;
    }
    st->h_stage = pool_piece(); /* zeroed: the completion word starts below the first block's sequence number */
    st->d_stage = mapped_or_die(st->h_stage);
    return st;
}

static void ecb_state_free(hip_ctr_state *st)
{
    /* the last block's kernel wrote its completion word after its last access to the staging or the slot (plugin_wait):
     * nothing waits here */
    ptls_hip_keyset_free(st->ks);
    pool_piece_put(st->h_stage);
    std::memset(st->bits, 0, sizeof(st->bits));
    delete st;
}

static void ctr_dispose(ptls_cipher_context_t *_ctx)
{
    auto *ctx = reinterpret_cast<hip_ctr_context *>(_ctx);
    if (ctx->st == nullptr)
        return;
    ecb_state_free(ctx->st);
    ctx->st = nullptr;
}

static int aesctr_setup(ptls_cipher_context_t *_ctx, int is_enc, const void *key, size_t key_size)
{
    (void)is_enc; /* CTR: same operation both ways */
    auto *ctx = reinterpret_cast<hip_ctr_context *>(_ctx);
    ctx->st = ecb_state_new(key, key_size);
    if (ctx->st == nullptr)
        return -1;
    ctx->super.do_dispose = ctr_dispose;
    ctx->super.do_init = ctr_init;
    ctx->super.do_transform = ctr_transform;
    return 0;
}

/* ---- fusion's public one-block ECB API (include/picotls/fusion.h:52-54, lib/fusion.c:857-928) ---- */

extern "C" int ptls_hip_aesecb_init(ptls_hip_aesecb_context_t *ctx, int is_enc, const void *key, size_t key_size, int aesni256)
{
    (void)aesni256; /* an x86 code-path choice in fusion; accepted so call sites stay the same */
    if (ctx == nullptr)
        return fail(PTLS_HIP_EINVAL, "aesecb_init: ctx is NULL");
    ctx->state = nullptr;
    ctx->rounds = 0;
    /* fusion asserts encryption-only and a 16- or 32-byte key (lib/fusion.c:859-873) */
    if (!is_enc || key == nullptr || (key_size != PTLS_AES128_KEY_SIZE && key_size != PTLS_AES256_KEY_SIZE))
        return fail(PTLS_HIP_EINVAL, "aesecb_init: encryption with a 16- or 32-byte key only");
    hip_ctr_state *st = ecb_state_new(key, key_size);
    if (st == nullptr)
        return fail(PTLS_HIP_ENODEV, "aesecb_init: %s", g_err.empty() ? "no usable gfx950 device" : g_err.c_str());
    ctx->state = st;
    ctx->rounds = key_size == PTLS_AES128_KEY_SIZE ? 10 : 14;
    return 0;
}

extern "C" void ptls_hip_aesecb_dispose(ptls_hip_aesecb_context_t *ctx)
{
    if (ctx == nullptr || ctx->state == nullptr)
        return;
    ecb_state_free(static_cast<hip_ctr_state *>(ctx->state));
    ctx->state = nullptr;
    ctx->rounds = 0;
}

extern "C" void ptls_hip_aesecb_encrypt(ptls_hip_aesecb_context_t *ctx, void *dst, const void *src)
{
    if (ctx == nullptr || ctx->state == nullptr) {
        fprintf(stderr, "ptls_hip: aesecb_encrypt on a context that init did not set up\n");
        abort();
    }
    uint8_t block[16];
    ecb_block(static_cast<hip_ctr_state *>(ctx->state), src, block);
    std::memcpy(dst, block, 16);
    std::memset(block, 0, sizeof(block));
}

static int aes128ctr_setup(ptls_cipher_context_t *ctx, int is_enc, const void *key)
{
    return aesctr_setup(ctx, is_enc, key, PTLS_AES128_KEY_SIZE);
}

static int aes256ctr_setup(ptls_cipher_context_t *ctx, int is_enc, const void *key)
{
    return aesctr_setup(ctx, is_enc, key, PTLS_AES256_KEY_SIZE);
}

/* allocation flags of the plugin's pinned staging: fine-grained (coherent) by default, whatever HIP_HOST_COHERENT says:
 * the kernel reads the record and writes its output and the completion word there, and the next call rewrites the same
 * bytes from the CPU without a stream synchronize.  PTLS_HIP_PLUGIN_STAGING=default (environment; for latency A/B
 * measurements) takes hipHostMallocDefault instead. */
static unsigned staging_flags(void)
{
    static const unsigned f = [] {
        const char *e = getenv("PTLS_HIP_PLUGIN_STAGING");
        return e != nullptr && std::strcmp(e, "default") == 0 ? (unsigned)hipHostMallocDefault : (unsigned)hipHostMallocCoherent;
    }();
    return f;
}

static uint8_t *mapped_or_die(uint8_t *h)
{
    void *d = nullptr;
    plugin_check(hipHostGetDevicePointer(&d, h, 0), "hipHostGetDevicePointer(staging)");
    return static_cast<uint8_t *>(d);
}

static void state_reserve(hip_aead_state *st, size_t len, size_t aadlen)
{
    if (st->h_io != nullptr && len <= st->cap && aadlen <= st->aad_cap)
        return;
    size_t cap = std::max(st->cap, (size_t)2048), aad_cap = std::max(st->aad_cap, (size_t)256);
    while (cap < len)
        cap *= 2;
    while (aad_cap < aadlen)
        aad_cap *= 2;
    cap = (cap + 15) & ~(size_t)15;
    aad_cap = (aad_cap + 15) & ~(size_t)15;
    /* a previous call's kernel wrote its completion word after its last access to this staging (plugin_wait) */
    if (st->h_io != nullptr) {
        std::memset(st->h_io, 0, st->cap + st->cap + 16 + st->aad_cap);
        plugin_check(hipHostFree(st->h_io), "hipHostFree");
    }
    st->h_io = nullptr;
    plugin_check(hipHostMalloc(&st->h_io, cap + (cap + 16) + aad_cap, staging_flags()), "hipHostMalloc(staging)");
    st->d_io = mapped_or_die(st->h_io);
    st->cap = cap;
    st->aad_cap = aad_cap;
}

#ifndef STAMP_PHASES
#define STAMP_PHASES 0 /* diagnostic build only (Makefile `diag`) */
#endif
#if STAMP_PHASES
/* diagnostic build (Makefile `diag`): the last plugin call's phase stamps (sparse_kernel.hip phase_stamp) */
static uint64_t *g_diag_stamps = nullptr;
extern "C" int ptls_hip_diag_plugin_stamps(uint64_t *out)
{
    return g_diag_stamps == nullptr ? -1 : (int)hipMemcpy(out, g_diag_stamps, 16 * sizeof(uint64_t), hipMemcpyDeviceToHost);
}
#endif

/* fused header protection for one plugin call: sample offset inside the record output, hp key slots */
struct PluginSupp {
    uint64_t sample_off;
    const KeySlot *hp_slots;
    uint8_t *output; /* host: supp->output */
};

/* pinned / device staging layout of a launched plugin call (256 B): result @128, supp descriptor @160, header-protection
 * mask @192, completion word @224 (the record descriptor travels in the kernel arguments) */
static const size_t ST_RESULT = 128, ST_SUPP = 160, ST_MASK = 192, ST_DONE = 224;

/* the record's input (with a detached tag: ptls_fusion_aesgcm_decrypt, lib/fusion.c:660-661) and AAD into pinned memory
 * the kernel reads */
static void stage_record(uint8_t *dst_in, uint8_t *dst_aad, const void *input, size_t len, size_t in_len, const void *tag,
                         const void *aad, size_t aadlen)
{
    if (tag != nullptr) {
        if (len != 0)
            std::memcpy(dst_in, input, len);
        std::memcpy(dst_in + len, tag, 16);
    } else if (in_len != 0) {
        std::memcpy(dst_in, input, in_len);
    }
    if (aadlen != 0)
        std::memcpy(dst_aad, aad, aadlen);
}

/* run one record: in/out/aad are the caller's (unpinned) host buffers.  The sparse kernel's single-record path (one wave
 * per record, its own 8 KiB H^64 table, none for records of <= 64 GHASH elements; two waves for longer ones) serves it
 * without building a workgroup-wide 64 KiB table; through the worker, no launch at all. */
static uint64_t plugin_run(hip_aead_state *st, bool open, void *output, const void *input, size_t len, uint64_t seq,
                           const void *aad, size_t aadlen, const PluginSupp *ps = nullptr, const void *tag = nullptr)
{
    DeviceGuard g(st->eng->device);
    const size_t in_len = open ? len + 16 : len, out_len = open ? len : len + 16;
    const size_t aad_pad = (aadlen + 15) & ~(size_t)15;
    ptls_hip_record_t rec{};
    rec.seq = seq;
    rec.len = (uint32_t)len;
    rec.aad_len = (uint32_t)aadlen;
    const ptls_hip_supp_t sp{ps != nullptr ? ps->sample_off : 0, 0, 0, PTLS_HIP_SUPP_ENABLE};
    uint64_t result = len;
    if (worker_enabled() && !STAMP_PHASES) {
        PluginWorker &w = g_worker;
        if (!w.ready.load(std::memory_order_acquire)) {
            std::lock_guard<std::mutex> lk(w.launch_mu);
            worker_init(w, st->eng);
        }
        /* the record, its output, result, mask and completion word live in the mailbox when they fit (a TLS record always
         * does: 16 KiB + 256 B); a longer one uses the context's staging */
        const bool inline_rec = aad_pad + in_len <= (size_t)WORKER_DATA && out_len <= (size_t)WORKER_DATA;
        if (!inline_rec) {
            state_reserve(st, in_len, aadlen);
            stage_record(st->h_io, st->h_io + st->cap + st->cap + 16, input, len, in_len, tag, aad, aadlen);
        }
        const unsigned j = worker_acquire(w);
        WorkerSlot *h = &w.h_mb[j], *d = &w.d_mb[j];
        WorkerReq rq{};
        rq.rec = rec;
        if (inline_rec) {
            stage_record(h->data + aad_pad, h->data, input, len, in_len, tag, aad, aadlen);
            rq.rec.aad_off = 0;
            rq.rec.in_off = aad_pad;
            rq.in = rq.aad = d->data;
            rq.out = d->out;
        } else {
            rq.in = st->d_io;
            rq.aad = st->d_io + st->cap + st->cap + 16;
            rq.out = st->d_io + st->cap;
        }
        rq.result = reinterpret_cast<uint64_t *>(d->aux + WAUX_RESULT);
        rq.slots = st->ks->d_slots;
        rq.basis = st->ks->d_basis;
        if (ps != nullptr) {
            std::memcpy(h->aux + WAUX_SUPP, &sp, sizeof(sp));
            rq.supp = reinterpret_cast<const ptls_hip_supp_t *>(d->aux + WAUX_SUPP);
            rq.hp_slots = ps->hp_slots;
            rq.mask = d->aux + WAUX_MASK;
        }
        rq.done = reinterpret_cast<uint32_t *>(d->aux + WAUX_DONE);
        rq.done_seq = ++w.mbox[j].done_seq;
        /* the context's IV travels with the request: IV changes never touch device memory the worker may have cached */
        std::memcpy(rq.iv, st->iv, 12);
        rq.flags = (open ? WREQ_OPEN : 0u) | (st->ks->key_size == 32 ? WREQ_AES256 : 0u) | WREQ_IV | (inline_rec ? WREQ_INLINE : 0u);
        worker_call(j, rq, h->aux + WAUX_DONE);
        const uint8_t *h_out = inline_rec ? h->out : st->h_io + st->cap;
        if (open)
            std::memcpy(&result, h->aux + WAUX_RESULT, 8);
        if (out_len != 0)
            std::memcpy(output, h_out, out_len);
        if (ps != nullptr)
            std::memcpy(ps->output, h->aux + WAUX_MASK, 16);
        /* the record's bytes do not stay in the mailbox or the staging */
        if (inline_rec) {
            std::memset(h->data, 0, aad_pad + in_len);
            std::memset(h->out, 0, out_len);
        } else {
            std::memset(st->h_io, 0, in_len);
            std::memset(st->h_io + st->cap, 0, out_len);
        }
        std::memset(h->aux + WAUX_MASK, 0, 16);
        w.mbox[j].mu.unlock();
        return result;
    }
    /* one launch per call (PTLS_HIP_PLUGIN_WORKER=0) */
    state_reserve(st, in_len, aadlen);
    if (st->h_stage == nullptr) {
        st->h_stage = pool_piece();
        st->d_stage = mapped_or_die(st->h_stage);
    }
    hipStream_t stream = pool_stream();
    if (st->iv_dirty) {
        if (ptls_hip_keyset_set_iv(st->ks, 0, st->iv, stream) != 0)
            plugin_die("set_iv");
        st->iv_dirty = false;
    }
    uint8_t *h_in = st->h_io, *h_out = st->h_io + st->cap, *h_aad = st->h_io + st->cap + st->cap + 16;
    uint8_t *d_in = st->d_io, *d_out = st->d_io + st->cap, *d_aad = st->d_io + st->cap + st->cap + 16;
    std::memcpy(st->h_stage + ST_SUPP, &sp, sizeof(sp));
    stage_record(h_in, h_aad, input, len, in_len, tag, aad, aadlen);
    KernelArgs a{};
    a.one = rec; /* by value in the kernel arguments (recs_ord stays null): the kernel's first dependent host read is
                    the record's own bytes */
    a.in = d_in;
    a.aad = d_aad;
    a.out = d_out;
    a.result = reinterpret_cast<uint64_t *>(st->d_stage + ST_RESULT);
    a.slots = st->ks->d_slots;
    a.basis = st->ks->d_basis;
    a.t0 = st->eng->d_t0;
    if (ps != nullptr) {
        a.supp = reinterpret_cast<const ptls_hip_supp_t *>(st->d_stage + ST_SUPP);
        a.hp_slots = ps->hp_slots;
        a.hp_nslots = 1;
        a.mask = st->d_stage + ST_MASK;
    }
    a.done = reinterpret_cast<uint32_t *>(st->d_stage + ST_DONE);
    a.done_seq = ++st->done_seq;
#if STAMP_PHASES
    if (g_diag_stamps == nullptr)
        plugin_check(hipMalloc(&g_diag_stamps, 16 * sizeof(uint64_t)), "hipMalloc(stamps)");
    a.clk = g_diag_stamps;
#endif
    const int e = launch_batch(SPARSE_LANES, st->ks->key_size == 16 ? 10 : 14, open, 0, 1, stream, a, true);
    if (e != 0) {
        g_err = hipGetErrorString((hipError_t)e);
        plugin_die("launch");
    }
    plugin_wait(stream, st->h_stage + ST_DONE, a.done_seq);
    pool_stream_put(stream);
    if (open)
        std::memcpy(&result, st->h_stage + ST_RESULT, 8);
    if (out_len != 0)
        std::memcpy(output, h_out, out_len);
    if (ps != nullptr)
        std::memcpy(ps->output, st->h_stage + ST_MASK, 16);
    /* the record's bytes do not stay in the staging */
    std::memset(h_in, 0, in_len);
    std::memset(h_out, 0, out_len);
    return result;
}

static void state_free(hip_aead_state *st)
{
    {
        DeviceGuard g(st->eng->device);
        /* the last call's kernel (or worker request) wrote its completion word after its last access to the staging and
         * the slot: nothing waits here */
        ptls_hip_keyset_free(st->ks);
        if (st->h_io != nullptr) {
            std::memset(st->h_io, 0, st->cap + st->cap + 16 + st->aad_cap);
            (void)hipHostFree(st->h_io);
        }
        if (st->h_stage != nullptr)
            pool_piece_put(st->h_stage);
    }
    std::memset(st->iv, 0, sizeof(st->iv));
    delete st;
}

static void aead_dispose(ptls_aead_context_t *_ctx)
{
    auto *ctx = reinterpret_cast<hip_aead_context *>(_ctx);
    if (ctx->st == nullptr)
        return;
    state_free(ctx->st);
    ctx->st = nullptr;
}

static void aead_get_iv(ptls_aead_context_t *_ctx, void *iv)
{
    auto *ctx = reinterpret_cast<hip_aead_context *>(_ctx);
    std::memcpy(iv, ctx->st != nullptr ? ctx->st->iv : ctx->iv, 12);
}

static void aead_set_iv(ptls_aead_context_t *_ctx, const void *iv)
{
    auto *ctx = reinterpret_cast<hip_aead_context *>(_ctx);
    if (ctx->st == nullptr) {
        std::memcpy(ctx->iv, iv, 12);
        return;
    }
    std::memcpy(ctx->st->iv, iv, 12);
    ctx->st->iv_dirty = true;
}

static void aead_encrypt_init(ptls_aead_context_t *, uint64_t, const void *, size_t)
{
    fprintf(stderr, "ptls_hip: do_encrypt_init is deprecated and not supported\n");
    abort();
}

static size_t aead_encrypt_update(ptls_aead_context_t *, void *, const void *, size_t)
{
    fprintf(stderr, "ptls_hip: do_encrypt_update is deprecated and not supported\n");
    abort();
}

static size_t aead_encrypt_final(ptls_aead_context_t *, void *)
{
    fprintf(stderr, "ptls_hip: do_encrypt_final is deprecated and not supported\n");
    abort();
}

static void encrypt_supp(hip_aead_state *st, void *output, const void *input, size_t inlen, uint64_t seq, const void *aad,
                         size_t aadlen, ptls_aead_supplementary_encryption_t *supp)
{
    if (supp != nullptr) {
        /* fused (lib/fusion.c:424-428, :636-650): our CTR context, same key size, sample inside the output */
        const hip_ctr_state *cs = ctr_state_of(supp->ctx);
        const uint8_t *in = static_cast<const uint8_t *>(supp->input), *o = static_cast<const uint8_t *>(output);
        if (cs != nullptr && cs->ks->key_size == st->ks->key_size && cs->eng == st->eng && in >= o && in + 16 <= o + inlen + 16) {
            PluginSupp ps{(uint64_t)(in - o), cs->ks->d_slots, supp->output};
            plugin_run(st, false, output, input, inlen, seq, aad, aadlen, &ps);
            return;
        }
    }
    plugin_run(st, false, output, input, inlen, seq, aad, aadlen);
    if (supp != nullptr) {
        /* header-protection mask from the caller's cipher context, computed after the AEAD output exists
         * (ptls_aead__do_encrypt, include/picotls.h:2027-2038; fusion fuses it, lib/fusion.c:636-650) */
        supp->ctx->do_init(supp->ctx, supp->input);
        std::memset(supp->output, 0, sizeof(supp->output));
        supp->ctx->do_transform(supp->ctx, supp->output, supp->output, sizeof(supp->output));
    }
}

static void aead_encrypt(ptls_aead_context_t *_ctx, void *output, const void *input, size_t inlen, uint64_t seq, const void *aad,
                         size_t aadlen, ptls_aead_supplementary_encryption_t *supp)
{
    encrypt_supp(reinterpret_cast<hip_aead_context *>(_ctx)->st, output, input, inlen, seq, aad, aadlen, supp);
}

static void aead_encrypt_v(ptls_aead_context_t *_ctx, void *output, ptls_iovec_t *input, size_t incnt, uint64_t seq,
                           const void *aad, size_t aadlen)
{
    size_t total = 0;
    for (size_t i = 0; i < incnt; ++i)
        total += input[i].len;
    std::vector<uint8_t> flat(total);
    size_t off = 0;
    for (size_t i = 0; i < incnt; ++i) {
        if (input[i].len != 0)
            std::memcpy(flat.data() + off, input[i].base, input[i].len);
        off += input[i].len;
    }
    plugin_run(reinterpret_cast<hip_aead_context *>(_ctx)->st, false, output, flat.data(), total, seq, aad, aadlen);
}

static size_t aead_decrypt(ptls_aead_context_t *_ctx, void *output, const void *input, size_t inlen, uint64_t seq, const void *aad,
                           size_t aadlen)
{
    if (inlen < 16)
        return SIZE_MAX;
    const uint64_t r = plugin_run(reinterpret_cast<hip_aead_context *>(_ctx)->st, true, output, input, inlen - 16, seq, aad, aadlen);
    return r == ~(uint64_t)0 ? SIZE_MAX : (size_t)r;
}

/* one single-record AEAD state on the plugin engine's device (shared by the plugin contexts and the
 * fusion-style low-level API) */
static hip_aead_state *state_new(const void *key, const void *iv, size_t key_size)
{
    ptls_hip_engine_t *eng = plugin_engine();
    if (eng == nullptr)
        return nullptr;
    DeviceGuard g(eng->device);
    auto *st = new hip_aead_state();
    st->eng = eng;
    st->ks = pool_keyset(eng, key_size, key, iv);
    if (st->ks == nullptr) {
        delete st;
        return nullptr;
    }
    std::memcpy(st->iv, iv, 12);
    st->iv_dirty = false;
    return st;
}

static int aesgcm_setup(ptls_aead_context_t *_ctx, int is_enc, const void *key, const void *iv, size_t key_size)
{
    (void)is_enc; /* one context seals and opens, as fusion's (lib/fusion.c:1184-1206) */
    auto *ctx = reinterpret_cast<hip_aead_context *>(_ctx);
    if (key == nullptr) {
        /* IV-only setup: fusion stores the IV and returns 0, on a fresh context as on a keyed one
         * (lib/fusion.c:1188-1191).  ptls_aead_new_direct zeroes only `super` (lib/picotls.c:6465), so a
         * fresh context is recognised by its unset dispose_crypto, never by reading the uninitialised tail.
         * Unlike fusion's, the fresh context also gets dispose / get_iv / set_iv, so ptls_aead_free and
         * ptls_aead_xor_iv work on it; encrypt / decrypt stay NULL as in fusion. */
        if (_ctx->dispose_crypto == nullptr) {
            ctx->st = nullptr;
            std::memcpy(ctx->iv, iv, 12);
            ctx->super.dispose_crypto = aead_dispose;
            ctx->super.do_get_iv = aead_get_iv;
            ctx->super.do_set_iv = aead_set_iv;
            return 0;
        }
        aead_set_iv(_ctx, iv);
        return 0;
    }
    if (_ctx->dispose_crypto != nullptr && ctx->st != nullptr) /* re-keying a keyed context: release the old key first */
        aead_dispose(_ctx);
    ctx->st = state_new(key, iv, key_size);
    if (ctx->st == nullptr)
        return -1;
    ctx->super.dispose_crypto = aead_dispose;
    ctx->super.do_get_iv = aead_get_iv;
    ctx->super.do_set_iv = aead_set_iv;
    ctx->super.do_encrypt_init = aead_encrypt_init;
    ctx->super.do_encrypt_update = aead_encrypt_update;
    ctx->super.do_encrypt_final = aead_encrypt_final;
    ctx->super.do_encrypt = aead_encrypt;
    ctx->super.do_encrypt_v = aead_encrypt_v;
    ctx->super.do_decrypt = aead_decrypt;
    return 0;
}

static int aes128gcm_setup(ptls_aead_context_t *ctx, int is_enc, const void *key, const void *iv)
{
    return aesgcm_setup(ctx, is_enc, key, iv, PTLS_AES128_KEY_SIZE);
}

static int aes256gcm_setup(ptls_aead_context_t *ctx, int is_enc, const void *key, const void *iv)
{
    return aesgcm_setup(ctx, is_enc, key, iv, PTLS_AES256_KEY_SIZE);
}

/* ptls_non_temporal_aes{128,256}gcm's contract (non_temporal_setup, lib/fusion.c:2109-2142): an encrypt
 * context has do_encrypt / do_encrypt_v and no do_decrypt, a decrypt context the reverse, and the
 * deprecated init/update/final are NULL.  The bytes are those of the fusion AEAD (the NT engine differs
 * only in its x86 store and reduction strategy), so the records run through the same kernel. */
static int non_temporal_setup(ptls_aead_context_t *_ctx, int is_enc, const void *key, const void *iv, size_t key_size)
{
    const int ret = aesgcm_setup(_ctx, is_enc, key, iv, key_size);
    if (ret != 0 || key == nullptr)
        return ret;
    _ctx->do_encrypt_init = nullptr;
    _ctx->do_encrypt_update = nullptr;
    _ctx->do_encrypt_final = nullptr;
    if (is_enc) {
        _ctx->do_decrypt = nullptr;
    } else {
        _ctx->do_encrypt = nullptr;
        _ctx->do_encrypt_v = nullptr;
    }
    return 0;
}

static int non_temporal_aes128gcm_setup(ptls_aead_context_t *ctx, int is_enc, const void *key, const void *iv)
{
    return non_temporal_setup(ctx, is_enc, key, iv, PTLS_AES128_KEY_SIZE);
}

static int non_temporal_aes256gcm_setup(ptls_aead_context_t *ctx, int is_enc, const void *key, const void *iv)
{
    return non_temporal_setup(ctx, is_enc, key, iv, PTLS_AES256_KEY_SIZE);
}

/* Field-for-field the values of ptls_fusion_aes{128,256}ctr / aes{128,256}gcm (lib/fusion.c:1219-1256). */
extern "C" {
ptls_cipher_algorithm_t ptls_hip_aes128ctr = {"AES128-CTR", PTLS_AES128_KEY_SIZE, 1, PTLS_AES_IV_SIZE, sizeof(hip_ctr_context),
                                              aes128ctr_setup};
ptls_cipher_algorithm_t ptls_hip_aes256ctr = {"AES256-CTR", PTLS_AES256_KEY_SIZE, 1, PTLS_AES_IV_SIZE, sizeof(hip_ctr_context),
                                              aes256ctr_setup};
ptls_aead_algorithm_t ptls_hip_aes128gcm = {"AES128-GCM",
                                            PTLS_AESGCM_CONFIDENTIALITY_LIMIT,
                                            PTLS_AESGCM_INTEGRITY_LIMIT,
                                            &ptls_hip_aes128ctr,
                                            nullptr,
                                            PTLS_AES128_KEY_SIZE,
                                            PTLS_AESGCM_IV_SIZE,
                                            PTLS_AESGCM_TAG_SIZE,
                                            {0, 0},
                                            0,
                                            0,
                                            sizeof(hip_aead_context),
                                            aes128gcm_setup};
ptls_aead_algorithm_t ptls_hip_aes256gcm = {"AES256-GCM",
                                            PTLS_AESGCM_CONFIDENTIALITY_LIMIT,
                                            PTLS_AESGCM_INTEGRITY_LIMIT,
                                            &ptls_hip_aes256ctr,
                                            nullptr,
                                            PTLS_AES256_KEY_SIZE,
                                            PTLS_AESGCM_IV_SIZE,
                                            PTLS_AESGCM_TAG_SIZE,
                                            {0, 0},
                                            0,
                                            0,
                                            sizeof(hip_aead_context),
                                            aes256gcm_setup};
/* the values of ptls_non_temporal_aes{128,256}gcm (lib/fusion.c:2154-2179): TLS 1.2 IV split 4 + 8,
 * non_temporal = 1, align_bits = 6 (64-byte output buffers; this engine accepts any alignment) */
ptls_aead_algorithm_t ptls_hip_non_temporal_aes128gcm = {"AES128-GCM",
                                                         PTLS_AESGCM_CONFIDENTIALITY_LIMIT,
                                                         PTLS_AESGCM_INTEGRITY_LIMIT,
                                                         &ptls_hip_aes128ctr,
                                                         nullptr,
                                                         PTLS_AES128_KEY_SIZE,
                                                         PTLS_AESGCM_IV_SIZE,
                                                         PTLS_AESGCM_TAG_SIZE,
                                                         {4, 8},
                                                         1,
                                                         6,
                                                         sizeof(hip_aead_context),
                                                         non_temporal_aes128gcm_setup};
ptls_aead_algorithm_t ptls_hip_non_temporal_aes256gcm = {"AES256-GCM",
                                                         PTLS_AESGCM_CONFIDENTIALITY_LIMIT,
                                                         PTLS_AESGCM_INTEGRITY_LIMIT,
                                                         &ptls_hip_aes256ctr,
                                                         nullptr,
                                                         PTLS_AES256_KEY_SIZE,
                                                         PTLS_AESGCM_IV_SIZE,
                                                         PTLS_AESGCM_TAG_SIZE,
                                                         {4, 8},
                                                         1,
                                                         6,
                                                         sizeof(hip_aead_context),
                                                         non_temporal_aes256gcm_setup};
}

/* ---- fusion-style low-level single-record API (include/picotls/fusion.h:56-96, lib/fusion.c:400-1048) ----
 * fusion passes the counter block as an x86 __m128i (calc_counter, lib/fusion.c:1126-1133: static IV xor
 * seq); here the caller passes the 12-byte nonce it stands for, so the state's IV is the nonce and the
 * record runs with seq 0 (nonce xor 0 == nonce). */
struct ptls_hip_aesgcm_context {
    hip_aead_state *st;
};

/* the sequence number that turns the state's IV into `nonce` (bytes 4..11 = IV xor BE64(seq), ptls_aead__build_iv,
 * lib/picotls.c:6492-6506) when bytes 0..3 agree, so a per-packet nonce needs no IV upload; otherwise the nonce
 * becomes the IV (uploaded before the launch) and the sequence number is 0 */
static uint64_t lowlevel_seq(hip_aead_state *st, const void *nonce)
{
    const uint8_t *nb = static_cast<const uint8_t *>(nonce);
    if (std::memcmp(st->iv, nb, 4) != 0) {
        std::memcpy(st->iv, nb, 12);
        st->iv_dirty = true;
        return 0;
    }
    uint64_t seq = 0;
    for (int i = 0; i < 8; ++i)
        seq = (seq << 8) | (uint8_t)(nb[4 + i] ^ st->iv[4 + i]);
    return seq;
}

extern "C" ptls_hip_aesgcm_context_t *ptls_hip_aesgcm_new(const void *key, size_t key_size, size_t capacity)
{
    if (key == nullptr || (key_size != PTLS_AES128_KEY_SIZE && key_size != PTLS_AES256_KEY_SIZE))
        return nullptr;
    static const uint8_t zero_iv[12] = {0};
    hip_aead_state *st = state_new(key, zero_iv, key_size);
    if (st == nullptr)
        return nullptr;
    auto *ctx = new ptls_hip_aesgcm_context{st};
    return ptls_hip_aesgcm_set_capacity(ctx, capacity);
}

extern "C" ptls_hip_aesgcm_context_t *ptls_hip_aesgcm_set_capacity(ptls_hip_aesgcm_context_t *ctx, size_t capacity)
{
    /* capacity = AAD + payload, as fusion's (lib/fusion.c:1017-1040); the staging also grows on demand */
    DeviceGuard g(ctx->st->eng->device);
    /* through the worker, records up to a mailbox's size need no staging of their own */
    if (!worker_enabled() || capacity + 16 > (size_t)WORKER_DATA)
        state_reserve(ctx->st, capacity + 16, 0);
    return ctx;
}

extern "C" void ptls_hip_aesgcm_free(ptls_hip_aesgcm_context_t *ctx)
{
    if (ctx == nullptr)
        return;
    state_free(ctx->st);
    delete ctx;
}

extern "C" void ptls_hip_aesgcm_encrypt(ptls_hip_aesgcm_context_t *ctx, void *output, const void *input, size_t inlen,
                                        const void *nonce, const void *aad, size_t aadlen,
                                        ptls_aead_supplementary_encryption_t *supp)
{
    encrypt_supp(ctx->st, output, input, inlen, lowlevel_seq(ctx->st, nonce), aad, aadlen, supp);
}

extern "C" int ptls_hip_aesgcm_decrypt(ptls_hip_aesgcm_context_t *ctx, void *output, const void *input, size_t inlen,
                                       const void *nonce, const void *aad, size_t aadlen, const void *tag)
{
    const uint64_t seq = lowlevel_seq(ctx->st, nonce);
    return plugin_run(ctx->st, true, output, input, inlen, seq, aad, aadlen, nullptr, tag) != ~(uint64_t)0;
}
