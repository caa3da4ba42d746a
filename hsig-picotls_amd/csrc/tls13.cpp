/*
 * tls13.cpp -- the TLS 1.3 record layer over the batch: framing of messages into
 * <= 16 384-byte records (buffer_push_encrypted_records, lib/picotls.c:747-794), parsing of a received stream
 * (parse_record_header, :5020-5031), and the seal / open calls that write the headers and strip the inner padding.
 */
#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "host.h"
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

/* parse_record (lib/picotls.c:5033-5062) and parse_record_header (:5020-5031) over a byte stream of TLS 1.3 records,
 * as far as the record layer of a connection past its handshake takes them (handle_input, :5840-5883):
 *   - a first byte that is no record type (20-23) is a decode error (parse_record's check, :5040-5048);
 *   - an application-data record longer than PTLS_MAX_ENCRYPTED_RECORD_SIZE is a decode error as soon as its header is
 *     in (parse_record_header, before the fragment is complete);
 *   - a complete application-data record shorter than a tag fails as picotls's aead_decrypt fails it: fusion's
 *     aead_do_decrypt rejects inlen < 16 (lib/fusion.c:1151-1156) and aead_decrypt turns that into
 *     PTLS_ALERT_BAD_RECORD_MAC (lib/picotls.c:717-726);
 *   - an incomplete record (header or fragment) ends the parse without an error: the caller waits for more bytes;
 *   - a record of another type (change_cipher_spec, alert, handshake) ends it too: picotls's record layer decides those;
 *     so does an application-data record whose legacy_record_version is not 03 03 (TLS 1.3 senders always write 03 03,
 *     RFC 8446 §5.1; picotls ignores the field and authenticates 03 03, the device would authenticate the bytes it reads).
 * Every other application-data record becomes a descriptor; its tag is checked when the batch opens it. */
extern "C" int ptls_hip_tls13_parse(const void *wire, size_t wire_len, uint64_t wire_off, uint32_t key, uint64_t seq,
                                    uint64_t out_base, ptls_hip_record_t *recs, size_t cap, size_t *nrecs, size_t *consumed)
{
    if ((wire == nullptr && wire_len != 0) || nrecs == nullptr || consumed == nullptr || (recs == nullptr && cap != 0))
        return fail(PTLS_HIP_EINVAL, "tls13_parse: bad arguments");
    const uint8_t *src = static_cast<const uint8_t *>(wire);
    size_t pos = 0, k = 0;
    uint64_t out = out_base;
    int rc = 0;
    while (pos < wire_len && k < cap) {
        const uint8_t type = src[pos];
        if (type < 20 || type > 23) {
            rc = fail(PTLS_HIP_TLS13_DECODE_ERROR, "tls13_parse: byte %zu is not a record type (%u)", pos, type);
            break;
        }
        if (type != 0x17 || wire_len - pos < 5)
            break; /* not application data (left to the caller's record layer), or an incomplete header */
        const size_t length = (size_t)src[pos + 3] << 8 | src[pos + 4];
        if (length > PTLS_HIP_TLS13_MAX_ENCRYPTED) {
            rc = fail(PTLS_HIP_TLS13_DECODE_ERROR, "tls13_parse: record at %zu has length %zu", pos, length);
            break;
        }
        if (length > wire_len - pos - 5)
            break; /* incomplete */
        if (length < 16) {
            rc = fail(PTLS_HIP_TLS13_SHORT_RECORD, "tls13_parse: record at %zu is shorter than a tag (%zu bytes)", pos, length);
            break;
        }
        if (src[pos + 1] != 0x03 || src[pos + 2] != 0x03)
            break; /* picotls authenticates 17 03 03 length (build_aad, :696-703), whatever legacy_record_version the record
                      carries; the device reads the header as the AAD, so such a record is left to the caller as well */
        ptls_hip_record_t &r = recs[k];
        r.aad_off = wire_off + pos;
        r.in_off = wire_off + pos + 5;
        r.out_off = out;
        r.seq = seq + k;
        r.len = (uint32_t)(length - 16);
        r.aad_len = 5;
        r.key = key;
        r.flags = 0;
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
