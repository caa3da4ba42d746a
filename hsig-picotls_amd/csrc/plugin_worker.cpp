/*
 * plugin_worker.cpp -- the picotls plugin's runtime: the resident worker dispatch that serves one-record calls from
 * mailboxes in pinned host memory, and the pools of key slots, streams and pinned staging that make a
 * ptls_aead_new / ptls_aead_free per connection cheap (lib/picotls.c:6458-6479).
 */
#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <chrono>
#include <thread>

#include "plugin.h"

void plugin_die(const char *what)
{
    fprintf(stderr, "ptls_hip: fatal device error in %s: %s\n", what, g_err.c_str());
    abort();
}

void plugin_check(hipError_t e, const char *what)
{
    if (e != hipSuccess) {
        g_err = hipGetErrorString(e);
        plugin_die(what);
    }
}


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
PluginWorker g_worker;

bool worker_enabled(void)
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
bool worker_drained(const PluginWorker &w, uint32_t epoch)
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
void worker_init(PluginWorker &w, ptls_hip_engine_t *eng)
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
unsigned worker_acquire(PluginWorker &w)
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
void worker_call(unsigned j, const WorkerReq &req, const uint8_t *word_p)
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

hipStream_t pool_stream(void)
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

void pool_stream_put(hipStream_t s)
{
    std::lock_guard<std::mutex> lk(g_pool.mu);
    g_pool.streams.push_back(s);
}

/* a 256-B piece of pinned, device-mapped staging (zeroed) */
uint8_t *pool_piece(void)
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

void pool_piece_put(uint8_t *p)
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
ptls_hip_keyset_t *pool_keyset(ptls_hip_engine_t *eng, size_t key_size, const void *key, const void *iv)
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
void pool_release(ptls_hip_keyset_t *ks)
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

/* allocation flags of the plugin's pinned staging: fine-grained (coherent) by default, whatever HIP_HOST_COHERENT says:
 * the kernel reads the record and writes its output and the completion word there, and the next call rewrites the same
 * bytes from the CPU without a stream synchronize.  PTLS_HIP_PLUGIN_STAGING=default (environment; for latency A/B
 * measurements) takes hipHostMallocDefault instead. */
unsigned staging_flags(void)
{
    static const unsigned f = [] {
        const char *e = getenv("PTLS_HIP_PLUGIN_STAGING");
        return e != nullptr && std::strcmp(e, "default") == 0 ? (unsigned)hipHostMallocDefault : (unsigned)hipHostMallocCoherent;
    }();
    return f;
}

uint8_t *mapped_or_die(uint8_t *h)
{
    void *d = nullptr;
    plugin_check(hipHostGetDevicePointer(&d, h, 0), "hipHostGetDevicePointer(staging)");
    return static_cast<uint8_t *>(d);
}
