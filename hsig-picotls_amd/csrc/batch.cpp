/*
 * batch.cpp -- batches (uploaded record descriptors + their launch plan) and the device-resident calls: seal / open /
 * seal with QUIC header protection / standalone ECB masks / the synthetic-record generator.  One asynchronous launch each
 * on the caller's stream (picotls has no batch API).
 */
#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "host.h"
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

int run_batch(ptls_hip_batch_t *b, ptls_hip_keyset_t *ks, const void *in, const void *aad, void *out, uint64_t *result,
              void *stream, bool open, ptls_hip_keyset_t *hp_ks, const ptls_hip_supp_t *supp, void *mask)
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
    a.clk_bytes = b->clk_bytes;
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
