/*
 * host.h -- what the host-side units of libptls_hip.so share (not part of the C ABI; every declaration here has hidden
 * visibility, so the library exports only include/ptls_hip.h).
 *
 *   engine.cpp         errors, the AES T-table, engines (device memory pool, chunk queues), the start-up self-check
 *   keyset.cpp         keysets: key slots + GHASH basis, keys / IVs / TLS 1.3 secrets
 *   planner.cpp        the launch planner: lanes per record, chunks, grid
 *   batch.cpp          batches and the device-resident seal / open / header-protection calls
 *   tls13.cpp          the TLS 1.3 record layer over the batch (framing, parsing)
 *   pipeline.cpp       host-resident records: the mapped and copy transports
 *   node.cpp           one batch over several devices, NUMA placement
 *   plugin_worker.cpp  the picotls plugin's runtime: the resident worker dispatch and pooled resources
 *   plugin.cpp         the picotls plugin objects (AEAD, CTR, ECB, fusion-style low-level API)
 */
#ifndef PTLS_HIP_HOST_H
#define PTLS_HIP_HOST_H

#include <hip/hip_runtime_api.h>

#include <atomic>
#include <cstdint>
#include <mutex>
#include <string>
#include <utility>
#include <vector>

#include "internal.h"

using namespace ptls_hip;

/* (the functions and variables below are hidden; the object types are plain structs without vtables) */
#pragma GCC visibility push(hidden)

/* ---- errors (engine.cpp) ---- */

/* the calling thread's last error message (ptls_hip_last_error) */
extern thread_local std::string g_err;
/* records a formatted message as the thread's last error and returns `code` */
int fail(int code, const char *fmt, ...) __attribute__((format(printf, 2, 3)));

#define HIP_TRY(expr, code)                                                                                                        \
    do {                                                                                                                           \
        hipError_t e_ = (expr);                                                                                                    \
        if (e_ != hipSuccess)                                                                                                      \
            return fail((code), "%s failed: %s", #expr, hipGetErrorString(e_));                                                  \
    } while (0)

#pragma GCC visibility pop

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
inline void keyset_note_use(ptls_hip_keyset_t *ks, void *stream)
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
inline unsigned batch_cus(const st_ptls_hip_batch_t *b)
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


#pragma GCC visibility push(hidden)

/* uint32 words of one key slot's GHASH basis (internal.h BASIS_VECS uint4) */
constexpr size_t BASIS_WORDS_PER_SLOT = (size_t)BASIS_VECS * 4;

/* ---- engine.cpp ---- */
/* stream-ordered device memory from the engine's own pool (hipMalloc / hipFree without one) */
hipError_t dev_alloc(ptls_hip_engine_t *e, void **p, size_t bytes);
void dev_free(ptls_hip_engine_t *e, void *p);
/* the chunk-queue words of one batch-kernel launch */
uint32_t *queue_slot(ptls_hip_engine_t *e);

/* ---- planner.cpp ---- */
int choose_lanes(const ptls_hip_record_t *recs, size_t n, unsigned ncu);
unsigned plan_grid(size_t n, size_t nchunks, int lanes, unsigned ncu);
int plan_wg(const std::vector<Chunk> &ch, int lanes);
void build_chunks(const ptls_hip_record_t *recs, size_t n, int lanes, unsigned ncu, std::vector<Chunk> &ch,
                  std::vector<uint32_t> &order, bool &all_aligned);
bool identity_order(const std::vector<uint32_t> &order, size_t n);

/* ---- batch.cpp ---- */
/* one asynchronous seal / open launch of a planned batch (the device-resident calls and the TLS 1.3 ones) */
int run_batch(ptls_hip_batch_t *b, ptls_hip_keyset_t *ks, const void *in, const void *aad, void *out, uint64_t *result,
              void *stream, bool open, ptls_hip_keyset_t *hp_ks = nullptr, const ptls_hip_supp_t *supp = nullptr,
              void *mask = nullptr);

/* ---- plugin_worker.cpp ---- */
/* ptls_hip_keyset_free of a plugin context's pooled slot */
void pool_release(ptls_hip_keyset_t *ks);

#pragma GCC visibility pop

#endif
