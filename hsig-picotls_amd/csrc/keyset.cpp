/*
 * keyset.cpp -- keysets: arrays of device-resident AEAD contexts (KeySlot + GHASH basis, internal.h), keyed from raw keys
 * (setup_crypto, lib/fusion.c:1184-1206) or from TLS 1.3 traffic secrets (get_traffic_keys, lib/picotls.c:1603-1622),
 * with the static-IV get / set / xor of ptls_aead_xor_iv (lib/picotls.c:6481-6490).
 */
#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "host.h"
/* ---------------------------------------------------------------------------------------------- */
/* keysets                                                                                         */
/* ---------------------------------------------------------------------------------------------- */



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
