/*
 * pipeline.cpp -- host-resident records (north_star: TLS records start and end in socket buffers).  A pipeline moves
 * slices of a record list through the batch kernels either by letting the kernels read and write the caller's pinned host
 * buffers over PCIe (MAPPED) or by staging through device buffers with the copy engines (COPY).
 */
#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "host.h"
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
    /* copy transport, allocated on a slice with gaps between its records: the caller's bytes of those gaps (packed) and
     * where they go in d_out, pinned and on the device */
    uint8_t *h_gap, *d_gap;
    GapPiece *h_gapd, *d_gapd;
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
        (void)hipHostFree(s.h_gap);
        (void)hipFree(s.d_gap);
        (void)hipHostFree(s.h_gapd);
        (void)hipFree(s.d_gapd);
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

/* ---- the copy transport's output: exactly the records' bytes ---------------------------------- *
 * A slice's records are written into device staging and come back by D2H copies.  Copying back the slice's whole output
 * span would also write, into the caller's buffer, whatever the staging held between the records (another call's
 * plaintext); fusion writes exactly the record's bytes (storen128 and the tag store, lib/fusion.c:388-397, :632).  So the
 * output comes back as the records' merged runs: each run by its own copy when a slice has few runs or a gap is long
 * (COPY_DIRECT_RUNS, GAP_SPLIT), and otherwise several runs by one copy, their gaps first filled in the staging with the
 * caller's own bytes of those gaps (gathered on the host into pinned memory, one upload, gap_scatter_kernel).  A gap is
 * never filled when another slice's record writes into it (records not in output order): the copy splits there. */
static const size_t COPY_DIRECT_RUNS = 8;   /* at most this many runs per slice: one copy each, no gap is written */
static const uint64_t GAP_SPLIT = 64 << 10; /* a gap this long splits the copy instead of being filled */

/* the output byte ranges of record r (its ciphertext + tag or plaintext, and a TLS 1.3 header the device writes) */
static void record_out_parts(const ptls_hip_record_t &r, PipeMode mode, std::vector<Span> &v)
{
    if (mode == PIPE_TLS13_SEAL && r.aad_len != 0)
        v.push_back(Span{r.aad_off, r.aad_off + r.aad_len});
    const uint64_t len = (uint64_t)r.len + (mode == PIPE_OPEN || mode == PIPE_TLS13_OPEN ? 0 : 16);
    if (len != 0)
        v.push_back(Span{r.out_off, r.out_off + len});
}

/* sort (unless already in order) and merge touching or overlapping ranges */
static void merge_spans(std::vector<Span> &v)
{
    bool sorted = true;
    for (size_t t = 1; t < v.size() && sorted; ++t)
        sorted = v[t].lo >= v[t - 1].lo;
    if (!sorted)
        std::sort(v.begin(), v.end(), [](const Span &a, const Span &b) { return a.lo < b.lo; });
    size_t k = 0;
    for (size_t t = 0; t < v.size(); ++t) {
        if (k != 0 && v[t].lo <= v[k - 1].hi)
            v[k - 1].hi = std::max(v[k - 1].hi, v[t].hi);
        else
            v[k++] = v[t];
    }
    v.resize(k);
}

/* some range of `uni` (sorted, merged) intersects [lo, hi) */
static bool spans_hit(const std::vector<Span> &uni, uint64_t lo, uint64_t hi)
{
    auto it = std::upper_bound(uni.begin(), uni.end(), lo, [](uint64_t x, const Span &s) { return x < s.hi; });
    return it != uni.end() && it->lo < hi;
}

static int slot_gap_buffers(ptls_hip_pipeline_t *p, PipeSlot &s)
{
    if (s.h_gap != nullptr)
        return 0;
    const size_t npieces = 2 * p->max_recs;
    if (hipHostMalloc(&s.h_gap, p->slice_bytes, hipHostMallocDefault) != hipSuccess ||
        hipMalloc(&s.d_gap, p->slice_bytes) != hipSuccess ||
        hipHostMalloc(&s.h_gapd, npieces * sizeof(GapPiece), hipHostMallocDefault) != hipSuccess ||
        hipMalloc(&s.d_gapd, npieces * sizeof(GapPiece)) != hipSuccess) {
        (void)hipHostFree(s.h_gap);
        (void)hipFree(s.d_gap);
        (void)hipHostFree(s.h_gapd);
        (void)hipFree(s.d_gapd);
        s.h_gap = s.d_gap = nullptr;
        s.h_gapd = s.d_gapd = nullptr;
        return fail(PTLS_HIP_ENOMEM, "pipeline: cannot allocate the copy transport's gap staging");
    }
    return 0;
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
    /* records in output order (each record's output range starts at or after the previous one's end, the usual layout):
     * a slice's gaps then hold no other slice's bytes.  Otherwise the union of every record's output decides. */
    std::vector<Span> uni, runs, pieces;
    bool in_order = true;
    for (size_t t = 0, prev_hi = 0; t < n && in_order; ++t) {
        runs.clear();
        record_out_parts(recs[t], mode, runs);
        for (const Span &r : runs) {
            in_order = in_order && r.lo >= prev_hi;
            prev_hi = std::max<uint64_t>(prev_hi, r.hi);
        }
    }
    if (!in_order) {
        for (size_t t = 0; t < n; ++t)
            record_out_parts(recs[t], mode, uni);
        merge_spans(uni);
    }
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
        /* the output's copies back: the records' merged runs, joined over short gaps filled with the caller's bytes */
        runs.clear();
        for (size_t t = i; t < j; ++t)
            record_out_parts(recs[t], mode, runs);
        merge_spans(runs);
        pieces.clear();
        uint32_t ngap = 0, gap_bytes = 0;
        for (size_t t = 0; t < runs.size(); ++t) {
            if (t == 0) {
                pieces.push_back(runs[0]);
                continue;
            }
            Span &cur = pieces.back();
            const uint64_t glo = cur.hi, ghi = runs[t].lo;
            if (runs.size() <= COPY_DIRECT_RUNS || ghi - glo >= GAP_SPLIT || gap_bytes + (ghi - glo) > UINT32_MAX ||
                (!in_order && spans_hit(uni, glo, ghi))) {
                pieces.push_back(runs[t]);
                continue;
            }
            if (int rc = slot_gap_buffers(p, s))
                return rc;
            std::memcpy(s.h_gap + gap_bytes, hout + glo, ghi - glo);
            s.h_gapd[ngap++] = GapPiece{glo - out_base, gap_bytes, (uint32_t)(ghi - glo)};
            gap_bytes += (uint32_t)(ghi - glo);
            cur.hi = runs[t].hi;
        }
        if (ngap != 0) {
            HIP_TRY(hipMemcpyAsync(s.d_gapd, s.h_gapd, ngap * sizeof(GapPiece), hipMemcpyHostToDevice, s.stream), PTLS_HIP_ENODEV);
            HIP_TRY(hipMemcpyAsync(s.d_gap, s.h_gap, gap_bytes, hipMemcpyHostToDevice, s.stream), PTLS_HIP_ENODEV);
            const int eg = launch_gap_scatter(s.d_gapd, ngap, s.d_gap, s.d_out, s.stream);
            if (eg != 0)
                return fail(PTLS_HIP_ELAUNCH, "pipeline: gap-fill kernel launch failed: %s", hipGetErrorString((hipError_t)eg));
        }
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
        for (const Span &pc : pieces)
            HIP_TRY(hipMemcpyAsync(hout + pc.lo, s.d_out + (pc.lo - out_base), pc.hi - pc.lo, hipMemcpyDeviceToHost, s.stream),
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

