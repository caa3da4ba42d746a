/*
 * plugin.cpp -- the picotls plugin objects: ptls_hip_aes{128,256}gcm and the non-temporal variants
 * (ptls_aead_algorithm_t, lib/fusion.c:1102-1256, :2109-2179), ptls_hip_aes{128,256}ctr (:1050-1100), fusion's one-block
 * ECB API (:857-928) and its low-level single-record context (include/picotls/fusion.h:56-96).  Each call runs one record
 * through the resident worker (plugin_worker.cpp) or its own launch.
 */
#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <chrono>
#include <thread>

#include "plugin.h"

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
