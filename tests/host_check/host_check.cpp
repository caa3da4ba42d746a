/*
 * host_check.cpp -- the engine's host code under AddressSanitizer + UndefinedBehaviorSanitizer (the
 * reference's CI runs its tests the same way, /root/reference/.github/workflows/ci.yml:24-25).
 *
 * Built by `make -C hsig-picotls_amd asan` against the host units compiled with -fsanitize=address,undefined (the device
 * code objects are the product's, unchanged) and run by tests/test_host_sanitizers.py on a machine WITHOUT a GPU.  It
 * drives every host path that reads caller or wire bytes without needing a device:
 *   - ptls_hip_tls13_parse on 100 000 random and damaged record streams (parse_record / parse_record_header,
 *     lib/picotls.c:5020-5062), with every produced descriptor checked to lie inside the stream;
 *   - ptls_hip_tls13_frame / _wire_size on random message lists (buffer_push_encrypted_records, :747-794);
 *   - the launch planner (choose_lanes / build_chunks / plan_grid) on random descriptor sets, every plan checked to be a
 *     permutation in key runs;
 *   - ptls_hip_partition_bytes on random lengths and part counts;
 *   - the argument checks of the C ABI with NULL / out-of-range arguments, and the plugin's setup_crypto without a device
 *     (it must fail cleanly: no CPU fallback);
 *   - with a gfx950 device (argument "device", run on the GPU box): the host pipelines over random layouts -- both
 *     transports, records in and out of output order, 1-64-byte gaps, exactly-sized heap buffers -- sealed and opened
 *     back, every record compared with the CPU oracle (oracle/aesgcm_oracle.c, test infrastructure) and every byte
 *     between records checked unchanged: the slicing, gap-planning and descriptor code of pipeline.cpp under the
 *     sanitizers (the kernels are the product's).
 * Any sanitizer report aborts the process (-fno-sanitize-recover, halt_on_error); the exit status is 0 only when every
 * check held.  Test infrastructure only: nothing here ships.
 */
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <random>
#include <vector>

#include "host.h"
#include "aesgcm_oracle.h"

static int failures = 0;
#define CHECK(c)                                                                                                                   \
    do {                                                                                                                           \
        if (!(c)) {                                                                                                                \
            fprintf(stderr, "host_check: %s:%d: %s\n", __FILE__, __LINE__, #c);                                                  \
            ++failures;                                                                                                            \
        }                                                                                                                          \
    } while (0)

/* a valid TLS 1.3 application-data stream (random ciphertext bytes: the parse does not decrypt), record starts in `starts` */
static std::vector<uint8_t> valid_stream(std::mt19937_64 &rng, std::vector<size_t> &starts)
{
    std::vector<uint8_t> w;
    const int nrec = 1 + (int)(rng() % 6);
    for (int r = 0; r < nrec; ++r) {
        const size_t len = 16 + (rng() % 4 == 0 ? rng() % (16384 + 256 - 15) : rng() % 400);
        starts.push_back(w.size());
        w.push_back(0x17);
        w.push_back(0x03);
        w.push_back(0x03);
        w.push_back((uint8_t)(len >> 8));
        w.push_back((uint8_t)len);
        for (size_t i = 0; i < len; ++i)
            w.push_back((uint8_t)rng());
    }
    return w;
}

static void damage(std::mt19937_64 &rng, std::vector<uint8_t> &w, const std::vector<size_t> &starts)
{
    const int n = 1 + (int)(rng() % 3);
    for (int d = 0; d < n; ++d) {
        const size_t rec = starts.empty() ? 0 : starts[rng() % starts.size()];
        switch (rng() % 7) {
        case 0: /* truncate */
            w.resize(w.empty() ? 0 : rng() % (w.size() + 1));
            break;
        case 1: /* a length field */
            if (rec + 5 <= w.size()) {
                const uint16_t L = (uint16_t)(rng() % 4 == 0 ? rng() : ((size_t)w[rec + 3] << 8 | w[rec + 4]) + (rng() % 41) - 20);
                w[rec + 3] = (uint8_t)(L >> 8);
                w[rec + 4] = (uint8_t)L;
            }
            break;
        case 2: /* the edges of the length checks */
            if (rec + 5 <= w.size()) {
                static const uint16_t edge[] = {0, 1, 15, 16, 17, 16384 + 256, 16384 + 257, 65535};
                const uint16_t L = edge[rng() % 8];
                w[rec + 3] = (uint8_t)(L >> 8);
                w[rec + 4] = (uint8_t)L;
            }
            break;
        case 3: /* a type byte */
            if (rec < w.size())
                w[rec] = (uint8_t)rng();
            break;
        case 4: /* garbage appended */
            for (size_t i = rng() % 40; i > 0; --i)
                w.push_back((uint8_t)rng());
            break;
        case 5: /* version bytes */
            if (rec + 3 <= w.size())
                w[rec + 1 + rng() % 2] = (uint8_t)rng();
            break;
        default: /* a random byte anywhere */
            if (!w.empty())
                w[rng() % w.size()] = (uint8_t)rng();
            break;
        }
    }
}

static void check_parse(std::mt19937_64 &rng, int streams)
{
    std::vector<ptls_hip_record_t> recs;
    for (int s = 0; s < streams; ++s) {
        std::vector<size_t> starts;
        std::vector<uint8_t> w = valid_stream(rng, starts);
        if (s % 8 != 0)
            damage(rng, w, starts);
        /* the stream in an exactly-sized heap buffer, so that a read one byte past it is an ASan report */
        uint8_t *buf = w.empty() ? nullptr : static_cast<uint8_t *>(malloc(w.size()));
        if (buf != nullptr)
            memcpy(buf, w.data(), w.size());
        const size_t cap = 1 + rng() % 8;
        recs.assign(cap, ptls_hip_record_t{});
        size_t nrecs = 0, consumed = 0;
        const uint64_t wire_off = rng() % 1000, out_base = rng() % 1000, seq = rng() % 100;
        const int rc = ptls_hip_tls13_parse(buf, w.size(), wire_off, 3, seq, out_base, recs.data(), cap, &nrecs, &consumed);
        CHECK(rc == 0 || rc == PTLS_HIP_TLS13_DECODE_ERROR || rc == PTLS_HIP_TLS13_SHORT_RECORD);
        CHECK(nrecs <= cap && consumed <= w.size());
        uint64_t pos = 0, out = out_base;
        for (size_t k = 0; k < nrecs; ++k) {
            const ptls_hip_record_t &r = recs[k];
            CHECK(r.aad_off == wire_off + pos && r.aad_len == 5 && r.in_off == r.aad_off + 5 && r.out_off == out);
            CHECK(r.in_off - wire_off + r.len + 16 <= w.size() && r.seq == seq + k && r.key == 3);
            CHECK(buf[pos] == 0x17 && buf[pos + 1] == 3 && buf[pos + 2] == 3);
            CHECK(((size_t)buf[pos + 3] << 8 | buf[pos + 4]) == (size_t)r.len + 16 && r.len + 16 <= PTLS_HIP_TLS13_MAX_ENCRYPTED);
            out += r.len;
            pos += 5 + r.len + 16;
        }
        CHECK(pos == consumed);
        free(buf);
    }
    /* argument checks */
    size_t n = 0, c = 0;
    CHECK(ptls_hip_tls13_parse(nullptr, 5, 0, 0, 0, 0, recs.data(), 1, &n, &c) == PTLS_HIP_EINVAL);
    CHECK(ptls_hip_tls13_parse(nullptr, 0, 0, 0, 0, 0, nullptr, 0, &n, &c) == 0 && n == 0 && c == 0);
    CHECK(ptls_hip_tls13_parse("\x17", 1, 0, 0, 0, 0, nullptr, 4, &n, &c) == PTLS_HIP_EINVAL);
    CHECK(ptls_hip_tls13_parse("\x17", 1, 0, 0, 0, 0, recs.data(), 1, nullptr, &c) == PTLS_HIP_EINVAL);
}

static void check_frame(std::mt19937_64 &rng, int lists)
{
    for (int l = 0; l < lists; ++l) {
        std::vector<ptls_hip_tls13_message_t> msgs(rng() % 6);
        uint64_t in = 0, out = 0;
        for (auto &m : msgs) {
            m = ptls_hip_tls13_message_t{};
            m.len = (uint32_t)(rng() % 4 == 0 ? rng() % 70000 : rng() % 2000);
            m.in_off = in;
            m.out_off = out;
            m.seq = rng() % 1000;
            m.key = (uint32_t)(rng() % 4);
            m.type = 23;
            in += m.len;
            out += ptls_hip_tls13_wire_size(m.len);
        }
        const size_t need = ptls_hip_tls13_frame(msgs.data(), msgs.size(), nullptr, 0);
        const size_t cap = need == 0 ? 0 : rng() % (need + 1);
        std::vector<ptls_hip_record_t> recs(cap);
        CHECK(ptls_hip_tls13_frame(msgs.data(), msgs.size(), cap ? recs.data() : nullptr, cap) == need);
        uint64_t wire_end = 0;
        for (size_t k = 0; k < cap; ++k)
            wire_end = std::max<uint64_t>(wire_end, recs[k].out_off + recs[k].len + 16);
        CHECK(wire_end <= out);
    }
}

static void check_planner(std::mt19937_64 &rng, int sets)
{
    std::vector<Chunk> ch;
    std::vector<uint32_t> order;
    for (int s = 0; s < sets; ++s) {
        const size_t n = rng() % 3000;
        std::vector<ptls_hip_record_t> recs(n);
        uint32_t key = 0;
        for (size_t i = 0; i < n; ++i) {
            if (rng() % (1 + rng() % 200) == 0)
                key = (uint32_t)(rng() % 70000);
            recs[i] = ptls_hip_record_t{};
            recs[i].len = (uint32_t)(rng() % 4 == 0 ? rng() % 16385 : rng() % 1400);
            recs[i].aad_len = (uint32_t)(rng() % 40);
            recs[i].in_off = rng() % (1u << 30);
            recs[i].out_off = rng() % (1u << 30);
            recs[i].aad_off = rng() % (1u << 20);
            recs[i].key = key;
        }
        const unsigned ncu = 1 + (unsigned)(rng() % 300);
        const int lanes = choose_lanes(recs.data(), n, ncu);
        CHECK(lanes == 1 || lanes == 2 || lanes == 4 || lanes == 8 || lanes == 16 || lanes == 32 || lanes == SPARSE_LANES);
        bool aligned = false;
        build_chunks(recs.data(), n, lanes, ncu, ch, order, aligned);
        std::vector<uint8_t> seen(n, 0);
        size_t covered = 0;
        for (const Chunk &c : ch) {
            CHECK((size_t)c.first + c.count <= n);
            for (uint32_t t = c.first; t < c.first + c.count && t < n; ++t) {
                CHECK(order[t] < n);
                if (order[t] < n) {
                    CHECK(!seen[order[t]]);
                    seen[order[t]] = 1;
                    CHECK(lanes == SPARSE_LANES || recs[order[t]].key == c.key);
                }
            }
            covered += c.count;
        }
        CHECK(covered == n);
        CHECK(plan_grid(n, ch.size(), lanes, ncu) <= std::max<unsigned>(ncu, 1));
    }
}

static void check_partition(std::mt19937_64 &rng, int sets)
{
    for (int s = 0; s < sets; ++s) {
        const size_t n = rng() % 500, parts = 1 + rng() % 12;
        std::vector<ptls_hip_record_t> recs(n);
        for (auto &r : recs) {
            r = ptls_hip_record_t{};
            r.len = (uint32_t)(rng() % 3 == 0 ? 0 : rng() % 20000);
        }
        std::vector<size_t> b(parts + 1, ~(size_t)0);
        CHECK(ptls_hip_partition_bytes(n ? recs.data() : nullptr, n, parts, b.data()) == 0);
        CHECK(b[0] == 0 && b[parts] == n);
        for (size_t p = 0; p < parts; ++p)
            CHECK(b[p] <= b[p + 1]);
    }
    size_t b[3];
    CHECK(ptls_hip_partition_bytes(nullptr, 5, 2, b) == PTLS_HIP_EINVAL);
    CHECK(ptls_hip_partition_bytes(nullptr, 0, 0, b) == PTLS_HIP_EINVAL);
}

/* the C ABI's argument checks and the no-device paths: each must fail with an error code and a message, never crash */
static void check_abi_without_device(void)
{
    CHECK(ptls_hip_is_supported() == 0);
    CHECK(ptls_hip_engine_new(0) == nullptr && std::strlen(ptls_hip_last_error()) != 0);
    CHECK(ptls_hip_engine_new(-1) == nullptr);
    CHECK(ptls_hip_keyset_new(nullptr, 16, 4) == nullptr);
    CHECK(ptls_hip_batch_new(nullptr, nullptr, 0, nullptr) == nullptr);
    CHECK(ptls_hip_pipeline_new(nullptr, 1 << 20) == nullptr);
    const int dev[1] = {0};
    CHECK(ptls_hip_node_new(nullptr, 1, 16, 1, 1 << 20) == nullptr);
    CHECK(ptls_hip_node_new(dev, 1, 16, 1, 1 << 20) == nullptr);
    CHECK(ptls_hip_keyset_set(nullptr, 0, 1, "k", nullptr, nullptr) == PTLS_HIP_EINVAL);
    CHECK(ptls_hip_keyset_set_secrets(nullptr, 0, 1, "s", 32, nullptr) == PTLS_HIP_EINVAL);
    CHECK(ptls_hip_keyset_get_iv(nullptr, 0, nullptr) == PTLS_HIP_EINVAL);
    CHECK(ptls_hip_batch_set_lanes(nullptr, 3) == PTLS_HIP_EINVAL);
    CHECK(ptls_hip_batch_set_clock(nullptr, nullptr, 0) == PTLS_HIP_EINVAL);
    CHECK(ptls_hip_aesgcm_seal_batch(nullptr, nullptr, nullptr, nullptr, nullptr, nullptr) == PTLS_HIP_EINVAL);
    CHECK(ptls_hip_aesgcm_open_batch(nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr) == PTLS_HIP_EINVAL);
    CHECK(ptls_hip_aesecb_batch(nullptr, nullptr, nullptr, 0, nullptr, nullptr, nullptr) == PTLS_HIP_EINVAL);
    CHECK(ptls_hip_tls13_seal_batch(nullptr, nullptr, nullptr, nullptr, nullptr) == PTLS_HIP_EINVAL);
    CHECK(ptls_hip_pipeline_set_transport(nullptr, 0) == PTLS_HIP_EINVAL);
    CHECK(ptls_hip_pipeline_seal(nullptr, nullptr, nullptr, 0, nullptr, nullptr, nullptr) == PTLS_HIP_EINVAL);
    CHECK(ptls_hip_device_copy(nullptr, nullptr, nullptr, 16, nullptr) == PTLS_HIP_EINVAL);
    CHECK(ptls_hip_fill_records(nullptr, nullptr, 0, 0, nullptr, nullptr) == PTLS_HIP_EINVAL);
    /* the plugin without a device: setup_crypto fails (ptls_aead_new returns NULL), no CPU fallback */
    static const uint8_t key[32] = {0}, iv[12] = {0};
    for (ptls_aead_algorithm_t *a : {&ptls_hip_aes128gcm, &ptls_hip_aes256gcm, &ptls_hip_non_temporal_aes128gcm}) {
        std::vector<uint8_t> ctx(a->context_size, 0);
        auto *c = reinterpret_cast<ptls_aead_context_t *>(ctx.data());
        c->algo = a;
        CHECK(a->setup_crypto(c, 1, key, iv) != 0);
        /* the IV-only setup of a fresh context needs no device (fusion: lib/fusion.c:1188-1191) */
        std::vector<uint8_t> ctx2(a->context_size, 0);
        auto *c2 = reinterpret_cast<ptls_aead_context_t *>(ctx2.data());
        c2->algo = a;
        CHECK(a->setup_crypto(c2, 1, nullptr, iv) == 0 && c2->dispose_crypto != nullptr);
        uint8_t got[12];
        c2->do_get_iv(c2, got);
        CHECK(std::memcmp(got, iv, 12) == 0);
        c2->dispose_crypto(c2);
    }
    ptls_hip_aesecb_context_t ecb;
    CHECK(ptls_hip_aesecb_init(&ecb, 1, key, 16, 0) == PTLS_HIP_ENODEV && ecb.state == nullptr);
    CHECK(ptls_hip_aesecb_init(&ecb, 0, key, 16, 0) == PTLS_HIP_EINVAL);
    ptls_hip_aesecb_dispose(&ecb);
    CHECK(ptls_hip_aesgcm_new(key, 16, 1500) == nullptr);
    CHECK(ptls_hip_aesgcm_new(key, 24, 1500) == nullptr);
}

/* one pipeline seal + open over a random layout; returns false (and counts failures) on a mismatch */
static void pipeline_trial(std::mt19937_64 &rng, ptls_hip_pipeline_t *pipe, ptls_hip_keyset_t *ks, size_t key_size,
                           const std::vector<uint8_t> &keys, const std::vector<uint8_t> &ivs, int transport)
{
    const size_t n = 1 + rng() % 160;
    std::vector<uint32_t> len(n), alen(n), key(n);
    std::vector<uint64_t> in_off(n), out_off(n), aad_off(n), pt_off(n);
    size_t in_sz = 0, out_sz = 0, aad_sz = 0, pt_sz = 0;
    for (size_t i = 0; i < n; ++i) {
        len[i] = (uint32_t)(rng() % 8 == 0 ? rng() % 16385 : rng() % 3000);
        alen[i] = (uint32_t)(rng() % 41);
        key[i] = (uint32_t)((i * 3) / n);
        in_off[i] = in_sz + rng() % 4;
        in_sz = in_off[i] + len[i];
        aad_off[i] = aad_sz + rng() % 4;
        aad_sz = aad_off[i] + alen[i];
        out_off[i] = out_sz + 1 + rng() % 64;
        out_sz = out_off[i] + len[i] + 16;
        pt_off[i] = pt_sz + 1 + rng() % 64;
        pt_sz = pt_off[i] + len[i];
    }
    out_sz += 1 + rng() % 64;
    pt_sz += 1 + rng() % 64;
    const bool pinned = transport == PTLS_HIP_TRANSPORT_MAPPED;
    /* exactly-sized buffers: heap (ASan-checked) for COPY, pinned for MAPPED */
    auto alloc = [&](size_t sz) -> uint8_t * {
        void *p = nullptr;
        if (pinned) {
            if (hipHostMalloc(&p, sz ? sz : 1, hipHostMallocDefault) != hipSuccess)
                return nullptr;
        } else {
            p = malloc(sz ? sz : 1);
        }
        return static_cast<uint8_t *>(p);
    };
    auto release = [&](uint8_t *p) {
        if (pinned)
            (void)hipHostFree(p);
        else
            free(p);
    };
    uint8_t *h_in = alloc(in_sz), *h_aad = alloc(aad_sz), *h_out = alloc(out_sz), *h_pt = alloc(pt_sz);
    CHECK(h_in && h_aad && h_out && h_pt);
    if (!(h_in && h_aad && h_out && h_pt))
        return;
    for (size_t i = 0; i < in_sz; ++i)
        h_in[i] = (uint8_t)rng();
    for (size_t i = 0; i < aad_sz; ++i)
        h_aad[i] = (uint8_t)rng();
    memset(h_out, 0xA5, out_sz);
    memset(h_pt, 0x5A, pt_sz);
    /* descriptors, in output order or shuffled */
    std::vector<size_t> perm(n);
    for (size_t i = 0; i < n; ++i)
        perm[i] = i;
    if (rng() % 2)
        std::shuffle(perm.begin(), perm.end(), rng);
    std::vector<ptls_hip_record_t> rs(n), ro(n);
    for (size_t k = 0; k < n; ++k) {
        const size_t i = perm[k];
        rs[k] = ptls_hip_record_t{in_off[i], out_off[i], aad_off[i], 1000 + i, len[i], alen[i], key[i], 0};
        ro[k] = ptls_hip_record_t{out_off[i], pt_off[i], aad_off[i], 1000 + i, len[i], alen[i], key[i], 0};
    }
    CHECK(ptls_hip_pipeline_set_transport(pipe, transport) == 0);
    int rc = ptls_hip_pipeline_seal(pipe, ks, rs.data(), n, h_in, h_aad, h_out);
    CHECK(rc == 0);
    std::vector<uint8_t> exp;
    std::vector<uint8_t> touched(out_sz, 0);
    for (size_t i = 0; rc == 0 && i < n; ++i) {
        exp.resize(len[i] + 16);
        oracle_aesgcm_seal(&keys[key[i] * key_size], key_size, &ivs[key[i] * 12], 1000 + i, h_aad + aad_off[i], alen[i],
                           h_in + in_off[i], len[i], exp.data());
        CHECK(memcmp(h_out + out_off[i], exp.data(), len[i] + 16) == 0);
        memset(&touched[out_off[i]], 1, len[i] + 16);
    }
    for (size_t b = 0; b < out_sz; ++b)
        if (!touched[b] && h_out[b] != 0xA5) {
            CHECK(!"seal wrote a byte between records");
            break;
        }
    CHECK(ptls_hip_pipeline_last_transport(pipe) == transport);
    std::vector<uint64_t> res(n, 0);
    uint64_t *h_res = res.data();
    void *pres = nullptr;
    if (pinned && hipHostMalloc(&pres, n * 8, hipHostMallocDefault) == hipSuccess)
        h_res = static_cast<uint64_t *>(pres);
    rc = ptls_hip_pipeline_open(pipe, ks, ro.data(), n, h_out, h_aad, h_pt, h_res);
    CHECK(rc == 0);
    std::vector<uint8_t> ptouched(pt_sz, 0);
    for (size_t k = 0; rc == 0 && k < n; ++k) {
        const size_t i = perm[k];
        CHECK(h_res[k] == len[i]);
        CHECK(memcmp(h_pt + pt_off[i], h_in + in_off[i], len[i]) == 0);
        memset(&ptouched[pt_off[i]], 1, len[i]);
    }
    for (size_t b = 0; b < pt_sz; ++b)
        if (!ptouched[b] && h_pt[b] != 0x5A) {
            CHECK(!"open wrote a byte between records");
            break;
        }
    if (pres != nullptr)
        (void)hipHostFree(pres);
    release(h_in);
    release(h_aad);
    release(h_out);
    release(h_pt);
}

static void check_pipelines_on_device(std::mt19937_64 &rng, int trials)
{
    ptls_hip_engine_t *eng = ptls_hip_engine_new(0);
    if (eng == nullptr) {
        printf("host_check: no usable gfx950 device (%s): device paths skipped\n", ptls_hip_last_error());
        return;
    }
    for (size_t key_size : {(size_t)16, (size_t)32}) {
        std::vector<uint8_t> keys(3 * key_size), ivs(3 * 12);
        for (auto &b : keys)
            b = (uint8_t)rng();
        for (auto &b : ivs)
            b = (uint8_t)rng();
        ptls_hip_keyset_t *ks = ptls_hip_keyset_new(eng, key_size, 3);
        CHECK(ks != nullptr && ptls_hip_keyset_set(ks, 0, 3, keys.data(), ivs.data(), nullptr) == 0);
        for (size_t slice : {(size_t)64 << 10, (size_t)1 << 20}) {
            ptls_hip_pipeline_t *pipe = ptls_hip_pipeline_new(eng, slice);
            CHECK(pipe != nullptr);
            for (int t = 0; pipe != nullptr && t < trials; ++t)
                pipeline_trial(rng, pipe, ks, key_size, keys, ivs, t % 2 ? PTLS_HIP_TRANSPORT_COPY : PTLS_HIP_TRANSPORT_MAPPED);
            ptls_hip_pipeline_free(pipe);
        }
        ptls_hip_keyset_free(ks);
    }
    ptls_hip_engine_free(eng);
    printf("host_check: device paths run (%d trials x 2 key sizes x 2 slice sizes)\n", trials);
}

int main(int argc, char **argv)
{
    if (argc > 1 && std::strcmp(argv[1], "device") == 0) { /* the GPU box: the pipelines under the sanitizers */
        std::mt19937_64 rng(0x70697065ull);
        check_pipelines_on_device(rng, argc > 2 ? atoi(argv[2]) : 40);
        printf("host_check: %s (%d failed checks)\n", failures == 0 ? "ok" : "FAILED", failures);
        return failures == 0 ? 0 : 1;
    }
    const int scale = argc > 1 ? atoi(argv[1]) : 1;
    std::mt19937_64 rng(0x68737467ull);
    check_parse(rng, 100000 * scale);
    check_frame(rng, 20000 * scale);
    check_planner(rng, 300 * scale);
    check_partition(rng, 20000 * scale);
    check_abi_without_device();
    printf("host_check: %s (%d failed checks)\n", failures == 0 ? "ok" : "FAILED", failures);
    return failures == 0 ? 0 : 1;
}
