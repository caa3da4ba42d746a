/*
 * plugin.h -- shared by the picotls plugin's units: plugin_worker.cpp (the resident worker dispatch, pooled key slots,
 * streams and pinned staging) and plugin.cpp (the ptls_aead_algorithm_t / ptls_cipher_algorithm_t objects).  Hidden.
 */
#ifndef PTLS_HIP_PLUGIN_H
#define PTLS_HIP_PLUGIN_H

#include "host.h"

#pragma GCC visibility push(hidden)

/* a device failure inside a void plugin callback (do_encrypt has no error channel): message and abort */
[[noreturn]] void plugin_die(const char *what);
void plugin_check(hipError_t e, const char *what);

/* ---- the resident worker (plugin_worker.cpp) ---- */
constexpr unsigned WORKER_MAX = 64; /* mailboxes (workgroups) of the worker dispatch at most */

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
extern PluginWorker g_worker;

/* PTLS_HIP_PLUGIN_WORKER (environment): calls go through the worker (default) or launch their own kernel */
bool worker_enabled(void);
/* under w.launch_mu: mailboxes, activity word and stream on the plugin engine's device */
void worker_init(PluginWorker &w, ptls_hip_engine_t *eng);
/* a mailbox for this call, locked */
unsigned worker_acquire(PluginWorker &w);
/* one request through mailbox j (its lock held); returns once the call's completion word shows req.done_seq */
void worker_call(unsigned j, const WorkerReq &req, const uint8_t *word_p);
/* every workgroup of dispatch `epoch` has left (or none was launched) */
bool worker_drained(const PluginWorker &w, uint32_t epoch);

/* ---- pooled resources (plugin_worker.cpp) ---- */
hipStream_t pool_stream(void);
void pool_stream_put(hipStream_t s);
/* a 256-B piece of pinned, device-mapped staging (zeroed) */
uint8_t *pool_piece(void);
void pool_piece_put(uint8_t *p);
/* a one-slot keyset on a pooled slot, keyed */
ptls_hip_keyset_t *pool_keyset(ptls_hip_engine_t *eng, size_t key_size, const void *key, const void *iv);
/* allocation flags of the plugin's pinned staging */
unsigned staging_flags(void);
/* the device address of pinned staging, or abort */
uint8_t *mapped_or_die(uint8_t *h);

#pragma GCC visibility pop

#endif
