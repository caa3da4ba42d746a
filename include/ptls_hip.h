/*
 * ptls_hip.h -- MI355X (gfx950) AES-GCM record-protection engine for picotls.
 *
 * Two faces, one library (libptls_hip.so):
 *
 * 1. The picotls plugin surface.  `ptls_hip_aes128gcm` / `ptls_hip_aes256gcm` are ordinary
 *    `ptls_aead_algorithm_t` objects, interchangeable with `ptls_fusion_aes128gcm` /
 *    `ptls_fusion_aes256gcm` (reference: lib/fusion.c:1231-1256, include/picotls/fusion.h:104).
 *    Create contexts with picotls's own `ptls_aead_new` / `ptls_aead_new_direct`
 *    (lib/picotls.c:6452-6473) and use `ptls_aead_encrypt*` / `ptls_aead_decrypt`
 *    (include/picotls.h:1993-2055).  Each call is synchronous and runs one record on the GPU.
 *
 * 2. The batch extension (picotls has no batch API).  Many independent records, each with its own
 *    key slot, sequence number, AAD, input and output, are sealed or opened by one asynchronous
 *    kernel launch on a HIP stream.  Inputs and outputs are device pointers.  This is the
 *    throughput path measured by bench.py.
 *
 * Plain C ABI: pointers, sizes, integers.  `stream` is a hipStream_t passed as void* (NULL = the
 * null stream).  Functions returning int give 0 on success and a negative PTLS_HIP_E* code on
 * failure; `ptls_hip_last_error()` describes the most recent failure on the calling thread.
 */
#ifndef PTLS_HIP_H
#define PTLS_HIP_H

#include <stddef.h>
#include <stdint.h>
#include "picotls_plugin_abi.h"

#ifdef __cplusplus
extern "C" {
#endif

#define PTLS_HIP_EINVAL (-1)   /* bad argument */
#define PTLS_HIP_ENODEV (-2)   /* no usable gfx950 device / HIP runtime failure */
#define PTLS_HIP_ENOMEM (-3)   /* device or host allocation failed */
#define PTLS_HIP_ELAUNCH (-4)  /* kernel launch failed */

const char *ptls_hip_last_error(void);

/* ------------------------------------------------------------------------------------------ *
 * 1. picotls plugin objects                                                                   *
 * ------------------------------------------------------------------------------------------ */

/* Replace ptls_fusion_aes128gcm / ptls_fusion_aes256gcm (lib/fusion.c:1231-1256).
 * setup_crypto returns non-zero (=> ptls_aead_new returns NULL) when no gfx950 device is usable;
 * key == NULL re-sets the static IV only (as fusion's aesgcm_setup, lib/fusion.c:1188-1191).
 * do_encrypt / do_encrypt_v / do_decrypt match lib/fusion.c:1135-1166 byte for byte, and in
 * addition implement do_encrypt_v (fusion asserts "FIXME" there, lib/fusion.c:1145-1149). */
extern ptls_aead_algorithm_t ptls_hip_aes128gcm, ptls_hip_aes256gcm;

/* Replace ptls_non_temporal_aes128gcm / ptls_non_temporal_aes256gcm (lib/fusion.c:2109-2179): the same
 * field values (TLS 1.2 IV sizes {4, 8}, non_temporal = 1, align_bits = 6) and the same per-direction
 * vtable (is_enc: do_encrypt + do_encrypt_v, no do_decrypt; otherwise do_decrypt only; init/update/final
 * NULL).  Output bytes equal the fusion AEAD's, as the reference's own are. */
extern ptls_aead_algorithm_t ptls_hip_non_temporal_aes128gcm, ptls_hip_non_temporal_aes256gcm;

/* Replace ptls_fusion_aes128ctr / ptls_fusion_aes256ctr (lib/fusion.c:1050-1100, :1219-1230), the
 * `ctr_cipher` of the AEAD objects above and the cipher QUIC stacks use for header protection.
 * Same contract as fusion's: do_init(iv) computes one keystream block AES-ECB(key, iv) on the GPU, and
 * the following do_transform XORs at most 16 bytes with it (fusion asserts the same, :1064-1077).
 * When such a context is passed as `supp` to ptls_hip_aes*gcm's do_encrypt (ptls_aead_encrypt_s),
 * the mask is computed inside the same kernel launch as the record, as fusion does (:636-650). */
extern ptls_cipher_algorithm_t ptls_hip_aes128ctr, ptls_hip_aes256ctr;

/* Device ordinal used by contexts created through the plugin objects (default 0; also read from
 * the environment variable PTLS_HIP_DEVICE).  Must be called before the first context is made. */
int ptls_hip_set_default_device(int device);

/* 1 when a gfx950 (MI355X) device is visible to this process, else 0: the counterpart of
 * ptls_fusion_is_supported_by_cpu (lib/fusion.c:2219-2249), for choosing the cipher suites at start-up.
 * Counts devices without creating a context. */
int ptls_hip_is_supported(void);

/* Fusion-style low-level single-record AES-GCM context (include/picotls/fusion.h:56-96,
 * lib/fusion.c:400-1048), for callers that drive fusion below the AEAD plugin (as its benchmarks and
 * tests do).  One record per call, host buffers, synchronous.
 *   nonce   the 12-byte GCM nonce (static IV xor big-endian sequence number).  Fusion takes the
 *           same value as a byte-swapped __m128i counter block (calc_counter, lib/fusion.c:1126-1133),
 *           which is x86-only; the nonce bytes are the portable form of it.
 *   capacity  maximum AAD + payload size, as fusion's; staging also grows on demand, and
 *           set_capacity returns the same context.
 * encrypt writes inlen bytes of ciphertext followed by the 16-byte tag.  supp (optional) is handled as
 * by the AEAD plugin's do_encrypt.  decrypt reads inlen bytes of ciphertext and the detached 16-byte
 * tag, always writes inlen bytes of plaintext, and returns 1 when the tag matches and 0 otherwise
 * (lib/fusion.c:660-...).  new returns NULL for a key size other than 16 or 32, or without a device. */
typedef struct ptls_hip_aesgcm_context ptls_hip_aesgcm_context_t;
ptls_hip_aesgcm_context_t *ptls_hip_aesgcm_new(const void *key, size_t key_size, size_t capacity);
ptls_hip_aesgcm_context_t *ptls_hip_aesgcm_set_capacity(ptls_hip_aesgcm_context_t *ctx, size_t capacity);
void ptls_hip_aesgcm_free(ptls_hip_aesgcm_context_t *ctx);
void ptls_hip_aesgcm_encrypt(ptls_hip_aesgcm_context_t *ctx, void *output, const void *input, size_t inlen, const void *nonce,
                             const void *aad, size_t aadlen, ptls_aead_supplementary_encryption_t *supp);
int ptls_hip_aesgcm_decrypt(ptls_hip_aesgcm_context_t *ctx, void *output, const void *input, size_t inlen, const void *nonce,
                            const void *aad, size_t aadlen, const void *tag);

/* Fusion's public one-block AES-ECB API (ptls_fusion_aesecb_init / _dispose / _encrypt,
 * include/picotls/fusion.h:52-54, lib/fusion.c:857-928): an encryption-only AES-128/256 key schedule and
 * single-block encryption, here with the key expanded into a device key slot and each block encrypted by
 * one kernel launch (synchronous, host buffers).  Same arguments as fusion's, including the trailing
 * `aesni256` (an x86 code-path switch there, ignored here).  Fusion's init returns void and asserts on
 * decryption or a key size other than 16 / 32; this one returns 0, or PTLS_HIP_EINVAL for those cases and
 * PTLS_HIP_ENODEV without a usable gfx950 device (ctx->state is then NULL and dispose is a no-op).
 * dispose zeroizes and releases the device key slot. */
typedef struct st_ptls_hip_aesecb_context_t {
    void *state;     /* engine-owned: key slot, staging, stream */
    unsigned rounds; /* 10 or 14, as fusion's ctx->rounds */
} ptls_hip_aesecb_context_t;
int ptls_hip_aesecb_init(ptls_hip_aesecb_context_t *ctx, int is_enc, const void *key, size_t key_size, int aesni256);
void ptls_hip_aesecb_dispose(ptls_hip_aesecb_context_t *ctx);
void ptls_hip_aesecb_encrypt(ptls_hip_aesecb_context_t *ctx, void *dst, const void *src);

/* ------------------------------------------------------------------------------------------ *
 * 2. batch extension                                                                          *
 * ------------------------------------------------------------------------------------------ */

typedef struct st_ptls_hip_engine_t ptls_hip_engine_t;
typedef struct st_ptls_hip_keyset_t ptls_hip_keyset_t;
typedef struct st_ptls_hip_batch_t ptls_hip_batch_t;

/* One engine per device: owns the device's AES tables and the launch configuration. */
ptls_hip_engine_t *ptls_hip_engine_new(int device);
void ptls_hip_engine_free(ptls_hip_engine_t *engine);
int ptls_hip_engine_device(ptls_hip_engine_t *engine);
int ptls_hip_engine_cu_count(ptls_hip_engine_t *engine);

/* A keyset is an array of device-resident AEAD contexts ("key slots"), all AES-128 (key_size 16)
 * or all AES-256 (key_size 32).  Slot i corresponds to one ptls_aead_context_t of the plugin
 * surface: key schedule, GHASH key powers and the 12-byte static IV. */
ptls_hip_keyset_t *ptls_hip_keyset_new(ptls_hip_engine_t *engine, size_t key_size, size_t nslots);
void ptls_hip_keyset_free(ptls_hip_keyset_t *ks); /* zeroizes device key material */
size_t ptls_hip_keyset_size(ptls_hip_keyset_t *ks);
/* Load `count` keys (count * key_size bytes) and static IVs (count * 12 bytes; NULL = zero IVs, e.g. for
 * header-protection keys) from host memory into slots [first, first + count) and expand them on the
 * device (key schedule, H = E_K(0), powers of H).
 * Equivalent to setup_crypto(ctx, is_enc, key, iv) for each slot (lib/fusion.c:1184-1206). */
int ptls_hip_keyset_set(ptls_hip_keyset_t *ks, size_t first, size_t count, const void *keys, const void *ivs, void *stream);
/* Static-IV get/set of one slot (do_get_iv / do_set_iv, lib/fusion.c:1168-1182); with
 * ptls_hip_keyset_xor_iv this gives ptls_aead_xor_iv semantics (lib/picotls.c:6481-6490). */
int ptls_hip_keyset_get_iv(ptls_hip_keyset_t *ks, size_t slot, void *iv);
int ptls_hip_keyset_set_iv(ptls_hip_keyset_t *ks, size_t slot, const void *iv, void *stream);
int ptls_hip_keyset_xor_iv(ptls_hip_keyset_t *ks, size_t slot, const void *bytes, size_t len, void *stream);

/* Many-connection key management, on the device.  `secrets` = count TLS 1.3
 * traffic secrets of hash_size bytes (32: SHA-256 suites, 48: SHA-384) in host memory.
 * set_secrets: slot i gets the record key / IV picotls derives from secret i when it creates the
 *   connection's AEAD (HKDF-Expand-Label "key" / "iv", get_traffic_keys, lib/picotls.c:1603-1622).
 * update_secrets: the TLS 1.3 key update (update_traffic_key, lib/picotls.c:4980-4996): every secret
 *   becomes HKDF-Expand-Label(secret, "traffic upd", "", hash_size) -- written back to `secrets` -- and the
 *   slots are re-keyed from the new secrets.  Both run one device thread per connection. */
int ptls_hip_keyset_set_secrets(ptls_hip_keyset_t *ks, size_t first, size_t count, const void *secrets, size_t hash_size,
                                void *stream);
int ptls_hip_keyset_update_secrets(ptls_hip_keyset_t *ks, size_t first, size_t count, void *secrets, size_t hash_size,
                                   void *stream);

/* Record descriptor (48 bytes).  Offsets are byte offsets into the buffers passed to seal/open.
 *   seal: reads len bytes at in+in_off, writes len bytes of ciphertext and the 16-byte tag at
 *         out+out_off (len + 16 bytes), like ptls_aead_encrypt (include/picotls.h:1993).
 *   open: reads len bytes of ciphertext followed by the 16-byte tag at in+in_off, writes len bytes
 *         of plaintext at out+out_off (always, like fusion's decrypt-then-verify), and sets
 *         result[i] = len on success or UINT64_MAX on authentication failure (the SIZE_MAX of
 *         ptls_aead_decrypt, lib/fusion.c:1151-1166).
 * The nonce is slot.iv with bytes 4..11 XORed with big-endian seq (ptls_aead__build_iv,
 * lib/picotls.c:6492-6506).  in == out (in place) is allowed.  For full speed keep in_off, out_off
 * 16-byte aligned and put records of the same key next to each other.  The kernels read exactly the
 * record's input (+ tag on open) and AAD bytes and write exactly its output bytes: buffers need no padding
 * past the last record (partial blocks are loaded as whole dwords + single bytes). */
typedef struct st_ptls_hip_record_t {
    uint64_t in_off;
    uint64_t out_off;
    uint64_t aad_off;
    uint64_t seq;
    uint32_t len;
    uint32_t aad_len;
    uint32_t key;   /* key slot index */
    uint32_t flags; /* 0, or PTLS_HIP_RECORD_TLS13_TYPE(type) (seal: TLS 1.3 inner content type, see 2c) */
} ptls_hip_record_t;
/* seal only: the record's plaintext is the len - 1 input bytes followed by the content-type byte `type`
 * (TLSInnerPlaintext without padding, RFC 8446 §5.2; picotls's aead_encrypt, lib/picotls.c:705-715) */
#define PTLS_HIP_RECORD_TLS13_TYPE(type) (1u | ((uint32_t)(uint8_t)(type) << 8))

/* Upload `n` host descriptors and plan the launch (runs of equal key slot, lane-group width from the
 * record lengths).  A batch is reusable for any number of seal/open calls over same-shaped buffers. */
ptls_hip_batch_t *ptls_hip_batch_new(ptls_hip_engine_t *engine, const ptls_hip_record_t *recs, size_t n, void *stream);
void ptls_hip_batch_free(ptls_hip_batch_t *batch);
size_t ptls_hip_batch_count(ptls_hip_batch_t *batch);
/* lanes cooperating on one record (1, 2, 4, 8, 16 or 32), or 64: one wave per record with key-independent
 * LDS (the kernel chosen for batches of many keys with few records each); 0 = automatic (default). */
int ptls_hip_batch_set_lanes(ptls_hip_batch_t *batch, int lanes);
int ptls_hip_batch_lanes(ptls_hip_batch_t *batch);
/* threads per workgroup of the batch kernel (512 or 768); 0 = automatic (default).  For tuning. */
int ptls_hip_batch_set_workgroup(ptls_hip_batch_t *batch, int threads);
int ptls_hip_batch_workgroup(ptls_hip_batch_t *batch);
/* at most `n` workgroups per launch, and chunks planned as for a device of n CUs (0 = the device's CU
 * count, the default).  For tests of the work distribution (a workgroup then takes several chunks of one
 * key run) and for sharing a device with other work. */
int ptls_hip_batch_set_max_workgroups(ptls_hip_batch_t *batch, int n);
/* chunks of the launch plan (runs of one key slot, at most 32 wave tasks each; the sparse kernel's plan: one) */
int ptls_hip_batch_chunks(ptls_hip_batch_t *batch);
/* workgroups one seal/open launch of the batch uses (for sizing the clock-stamp buffer below) */
int ptls_hip_batch_grid(ptls_hip_batch_t *batch);
/* Diagnostic: the following launches of the batch write, per workgroup w, the shader-cycle counter and the constant
 * 100 MHz counter at the start and at the end of its work: d_buf[4w .. 4w + 3] = {cycles0, ticks0, cycles1, ticks1}
 * (uint64, device memory of >= 32 bytes per workgroup).  delta(cycles) / delta(ticks) x 100 MHz = the clock the launch
 * ran at.  d_buf == NULL switches the stamps off (the default: then no stamp instruction executes). */
int ptls_hip_batch_set_clock(ptls_hip_batch_t *batch, void *d_buf, size_t nbytes);

/* Asynchronous on `stream`; all pointers are device (or device-accessible) memory.  Fails with
 * PTLS_HIP_EINVAL (nothing launched) when a record names a key slot outside `ks`. */
int ptls_hip_aesgcm_seal_batch(ptls_hip_batch_t *batch, ptls_hip_keyset_t *ks, const void *in, const void *aad, void *out,
                               void *stream);
int ptls_hip_aesgcm_open_batch(ptls_hip_batch_t *batch, ptls_hip_keyset_t *ks, const void *in, const void *aad, void *out,
                               uint64_t *result, void *stream);

/* QUIC header protection for a batch (RFC 9001 §5.4; fusion's `supp`, lib/fusion.c:424-428, :636-650).
 * One descriptor per record (same index as the batch's descriptors): mask + mask_off receives the
 * 16-byte AES-ECB(hp key slot `hp_key`, 16 bytes at sample_off) -- for seal the sample is read from
 * `out` AFTER the record (ciphertext and tag) is written, so it may cover the tag, exactly like
 * fusion's supplementary block.  Records with (flags & 1) == 0, or whose hp_key is outside the
 * header-protection keyset (the descriptors are device data, so this is checked on the device), are
 * skipped and their mask bytes left untouched.  The header-protection
 * keyset must have the AEAD keyset's key size (fusion runs the supp block with the AEAD's rounds). */
typedef struct st_ptls_hip_supp_t {
    uint64_t sample_off;
    uint64_t mask_off;
    uint32_t hp_key;
    uint32_t flags;
} ptls_hip_supp_t;
#define PTLS_HIP_SUPP_ENABLE 1u

/* seal_batch + header-protection masks in the same launch; `supp` is a device array of batch_count. */
int ptls_hip_aesgcm_seal_batch_supp(ptls_hip_batch_t *batch, ptls_hip_keyset_t *ks, ptls_hip_keyset_t *hp_ks,
                                    const ptls_hip_supp_t *supp, const void *in, const void *aad, void *out, void *mask,
                                    void *stream);
/* Standalone masks (receive side: the sample is ciphertext in the received packet, needed before the
 * packet number can be read and the record opened): mask + mask_off = AES-ECB(hp key, src + sample_off)
 * for n device descriptors. */
int ptls_hip_aesecb_batch(ptls_hip_engine_t *engine, ptls_hip_keyset_t *hp_ks, const ptls_hip_supp_t *supp, size_t n,
                          const void *src, void *mask, void *stream);

/* ------------------------------------------------------------------------------------------ *
 * 2b. TLS 1.3 record layer over the batch                      *
 * ------------------------------------------------------------------------------------------ */

#define PTLS_HIP_TLS13_MAX_PLAINTEXT 16384         /* PTLS_MAX_PLAINTEXT_RECORD_SIZE, lib/picotls.c:42 */
#define PTLS_HIP_TLS13_MAX_ENCRYPTED (16384 + 256) /* PTLS_MAX_ENCRYPTED_RECORD_SIZE, lib/picotls.c:43 */
/* wire bytes of one message of `len` payload bytes: ceil(len / 16384) records of 5 + chunk + 1 + 16 */
size_t ptls_hip_tls13_wire_size(size_t len);

/* Send side.  A message = `len` bytes of one content type for one connection (key slot); like
 * buffer_push_encrypted_records (lib/picotls.c:747-794) it is cut into records of at most 16384 bytes,
 * record j carrying seq + j, all written back to back at out + out_off as
 *     17 03 03 BE16(chunk + 17) || AES-GCM(chunk || type, AAD = that 5-byte header) || tag
 * (build_aad and aead_encrypt, lib/picotls.c:696-715).  len == 0 produces no record. */
typedef struct st_ptls_hip_tls13_message_t {
    uint64_t in_off;  /* payload in the `in` buffer */
    uint64_t out_off; /* first wire byte in the `out` buffer */
    uint64_t seq;     /* sequence number of the first record */
    uint32_t len;
    uint32_t key;  /* key slot */
    uint32_t type; /* content type (PTLS_CONTENT_TYPE_APPDATA = 23, handshake 22, alert 21) */
    uint32_t reserved;
} ptls_hip_tls13_message_t;
/* Host-side planning: fills up to `cap` record descriptors (aad_off = header position in `out`) and
 * returns the number of records the messages need (call with recs == NULL to size the array). */
size_t ptls_hip_tls13_frame(const ptls_hip_tls13_message_t *msgs, size_t n, ptls_hip_record_t *recs, size_t cap);
/* Writes the record headers into `out`, then seals every record (AAD read from the headers). */
int ptls_hip_tls13_seal_batch(ptls_hip_batch_t *batch, ptls_hip_keyset_t *ks, const void *in, void *out, void *stream);

/* Receive side.  Parses complete TLS records from a received byte stream on the host, like picotls's
 * parse_record / parse_record_header (lib/picotls.c:5020-5062): application-data records (type 23) of 16 to
 * 16384 + 256 bytes become descriptors {aad_off = header, in_off = header + 5, len = length - 16,
 * seq = seq + i, key, out_off = out_base + plaintext position}, at most `cap` of them (recs may be NULL
 * when cap is 0).  Stops before the first incomplete record, record of another type (change_cipher_spec,
 * alert, handshake) or record whose legacy_record_version is not 03 03: the caller's picotls record layer
 * handles those (ptls_receive from *consumed on); *consumed = wire bytes of the records
 * produced, *nrecs = their number.  Returns 0; or PTLS_HIP_TLS13_DECODE_ERROR for a byte that is no record
 * type or an oversized application-data record (as parse_record); or PTLS_HIP_TLS13_SHORT_RECORD for a
 * complete application-data record shorter than a tag (picotls's aead_decrypt fails it with
 * PTLS_ALERT_BAD_RECORD_MAC, :717-726).  The records before the error are produced either way. */
#define PTLS_HIP_TLS13_DECODE_ERROR (-50) /* -PTLS_ALERT_DECODE_ERROR */
#define PTLS_HIP_TLS13_SHORT_RECORD (-20) /* -PTLS_ALERT_BAD_RECORD_MAC */
int ptls_hip_tls13_parse(const void *wire, size_t wire_len, uint64_t wire_off, uint32_t key, uint64_t seq, uint64_t out_base,
                         ptls_hip_record_t *recs, size_t cap, size_t *nrecs, size_t *consumed);
/* Opens the records (AAD = their wire headers in `in`), strips the TLSInnerPlaintext padding and reads
 * the content type, like handle_input (lib/picotls.c:5866-5883).  result[i] = content length |
 * (uint64_t)type << 56, or PTLS_HIP_TLS13_BAD_RECORD_MAC (authentication failure), or
 * PTLS_HIP_TLS13_NO_CONTENT_TYPE (all-zero plaintext: PTLS_ALERT_UNEXPECTED_MESSAGE in picotls). */
#define PTLS_HIP_TLS13_BAD_RECORD_MAC UINT64_MAX
#define PTLS_HIP_TLS13_NO_CONTENT_TYPE (UINT64_MAX - 1)
int ptls_hip_tls13_open_batch(ptls_hip_batch_t *batch, ptls_hip_keyset_t *ks, const void *in, void *out, uint64_t *result,
                              void *stream);

/* ------------------------------------------------------------------------------------------ *
 * 2c. host-resident records (records arrive in and leave through host memory: socket buffers)  *
 * ------------------------------------------------------------------------------------------ */

/* A pipeline owns three device staging slots of `slice_bytes` each and three streams.  seal/open
 * cut the record list into slices whose input / output / AAD byte spans fit a slot and overlap, per
 * slice, H2D copy -> kernel -> D2H copy.  Offsets in `recs` are relative to the host buffers.  The
 * call returns when every output byte (and result) is in host memory.  Host buffers should be
 * pinned (hipHostMalloc'd, or ptls_hip_host_register'ed) for the copies to run asynchronously.
 * Only the records' output bytes change in the caller's output buffer (as fusion's storen128 and tag
 * store, lib/fusion.c:388-397, :632): a slice's output comes back as the records' runs, several runs
 * joined by one copy over short gaps that were first filled, on the device, with the caller's own bytes
 * of those gaps (read when the slice is planned; do not modify them during the call), never over another
 * slice's record.  The mask span of seal_supp is uploaded before and copied back after the kernel, so its
 * other bytes come back unchanged as well. */
typedef struct st_ptls_hip_pipeline_t ptls_hip_pipeline_t;
ptls_hip_pipeline_t *ptls_hip_pipeline_new(ptls_hip_engine_t *engine, size_t slice_bytes);
void ptls_hip_pipeline_free(ptls_hip_pipeline_t *p);
int ptls_hip_pipeline_seal(ptls_hip_pipeline_t *p, ptls_hip_keyset_t *ks, const ptls_hip_record_t *recs, size_t n,
                           const void *h_in, const void *h_aad, void *h_out);
int ptls_hip_pipeline_open(ptls_hip_pipeline_t *p, ptls_hip_keyset_t *ks, const ptls_hip_record_t *recs, size_t n,
                           const void *h_in, const void *h_aad, void *h_out, uint64_t *h_result);
/* seal + QUIC header-protection masks from and to host memory: `supp` is a HOST array indexed like recs
 * (offsets relative to h_out / h_mask); every enabled sample must lie inside the output of the records
 * sealed with it (QUIC: pn_offset + 4 is in the ciphertext).  Masks are written at h_mask + mask_off;
 * other bytes of h_mask are preserved. */
int ptls_hip_pipeline_seal_supp(ptls_hip_pipeline_t *p, ptls_hip_keyset_t *ks, ptls_hip_keyset_t *hp_ks,
                                const ptls_hip_record_t *recs, const ptls_hip_supp_t *supp, size_t n, const void *h_in,
                                const void *h_aad, void *h_out, void *h_mask);
/* The TLS 1.3 record layer from and to host memory (socket buffers): `recs` from ptls_hip_tls13_frame
 * (seal: h_in holds the messages, h_wire receives header + ciphertext + tag of every record) or from
 * ptls_hip_tls13_parse (open: h_wire is the received stream, h_out receives the inner content, h_result
 * is as in ptls_hip_tls13_open_batch).  Same slicing and overlap as ptls_hip_pipeline_seal/open. */
int ptls_hip_pipeline_tls13_seal(ptls_hip_pipeline_t *p, ptls_hip_keyset_t *ks, const ptls_hip_record_t *recs, size_t n,
                                 const void *h_in, void *h_wire);
int ptls_hip_pipeline_tls13_open(ptls_hip_pipeline_t *p, ptls_hip_keyset_t *ks, const ptls_hip_record_t *recs, size_t n,
                                 const void *h_wire, void *h_out, uint64_t *h_result);
/* How a pipeline moves the bytes.  AUTO (the default): MAPPED when every host buffer of the call (in, out, aad,
 * mask) is pinned or registered, COPY otherwise.  COPY: the staging described above (copy engines).  MAPPED: no
 * staging -- the kernels read the records from and write them to the host buffers over PCIe themselves (their
 * device mappings, hipHostGetDevicePointer), one launch per max-records slice; bytes between records in the
 * output are never written, as by the device-resident batch calls.  A call in MAPPED mode with an unmapped
 * buffer fails with PTLS_HIP_EINVAL.  last_transport: what the last seal/open of the pipeline used. */
#define PTLS_HIP_TRANSPORT_AUTO 0
#define PTLS_HIP_TRANSPORT_COPY 1
#define PTLS_HIP_TRANSPORT_MAPPED 2
int ptls_hip_pipeline_set_transport(ptls_hip_pipeline_t *p, int transport);
int ptls_hip_pipeline_last_transport(ptls_hip_pipeline_t *p);
int ptls_hip_host_register(void *ptr, size_t len);
int ptls_hip_host_unregister(void *ptr);

/* ------------------------------------------------------------------------------------------ *
 * 2d. one batch over several devices (records are independent, no collective)  *
 * ------------------------------------------------------------------------------------------ */

/* Host-side planning: contiguous ranges of about equal payload bytes.  bounds (parts + 1 entries): range r =
 * records [bounds[r], bounds[r + 1]), bounds[0] = 0, bounds[parts] = n; range r ends right after the first record
 * whose prefix sum of len reaches ceil(total * (r + 1) / parts).  Equal counts for equal lengths. */
int ptls_hip_partition_bytes(const ptls_hip_record_t *recs, size_t n, size_t parts, size_t *bounds);

/* A node: one engine, one keyset (nslots key slots of key_size) and one host pipeline (slice_bytes, as
 * ptls_hip_pipeline_new) per listed device; a device may be listed more than once.  seal / open split the records by
 * ptls_hip_partition_bytes and run every range on its own device from its own host thread, through that device's
 * pipeline (transport AUTO by default: the kernels read and write pinned host buffers over the device's own PCIe link),
 * and return when every device is done.  Records, offsets and buffers are as for ptls_hip_pipeline_seal / open.
 * node_keyset_set loads the same keys into every device's keyset (ptls_hip_keyset_set semantics).
 * last_split: the last call's per-device wall-clock seconds (ndev doubles) and record ranges (ndev + 1 bounds),
 * either pointer may be NULL; whole-node rate = payload bytes / the largest of the seconds. */
typedef struct st_ptls_hip_node_t ptls_hip_node_t;
ptls_hip_node_t *ptls_hip_node_new(const int *devices, size_t ndev, size_t key_size, size_t nslots, size_t slice_bytes);
void ptls_hip_node_free(ptls_hip_node_t *node);
size_t ptls_hip_node_size(ptls_hip_node_t *node);
int ptls_hip_node_keyset_set(ptls_hip_node_t *node, size_t first, size_t count, const void *keys, const void *ivs);
int ptls_hip_node_set_transport(ptls_hip_node_t *node, int transport);
int ptls_hip_node_seal(ptls_hip_node_t *node, const ptls_hip_record_t *recs, size_t n, const void *h_in, const void *h_aad,
                       void *h_out);
int ptls_hip_node_open(ptls_hip_node_t *node, const ptls_hip_record_t *recs, size_t n, const void *h_in, const void *h_aad,
                       void *h_out, uint64_t *h_result);
int ptls_hip_node_last_split(ptls_hip_node_t *node, double *seconds, size_t *bounds);
/* NUMA placement (each GPU's records in host memory on its own NUMA node).  device_numa_node: the node
 * a device's PCI function hangs off (sysfs), -1 if unknown.  node_numa: that node for every device of the node (ndev
 * ints).  Each device's host thread runs on its node's CPUs.  node_host_alloc: `bytes` of host memory whose range
 * [splits[d], splits[d + 1]) (ndev + 1 byte offsets, 0 .. bytes; whole pages, a shared page goes with the lower range)
 * is bound to device d's node and faulted in there, registered with every device (mapped, portable) so both transports
 * use it zero-copy; released with node_host_free(ptr, bytes).  host_page_nodes: the node of every stride-th page of
 * [ptr, ptr + bytes) (move_pages), at most cap of them; returns how many were written. */
int ptls_hip_device_numa_node(int device);
int ptls_hip_node_numa(ptls_hip_node_t *node, int *numa_nodes);
void *ptls_hip_node_host_alloc(ptls_hip_node_t *node, size_t bytes, const size_t *splits);
void ptls_hip_node_host_free(void *ptr, size_t bytes);
size_t ptls_hip_host_page_nodes(const void *ptr, size_t bytes, size_t stride, int *nodes, size_t cap);

/* ------------------------------------------------------------------------------------------ *
 * 3. synthetic workload (bench / tests): the payload of descriptor i is the splitmix64 stream     *
 *    seeded with seed ^ g(i), written at buf + recs[i].in_off for recs[i].len     *
 *    bytes, where g(i) = index[i] if `index` (device array of n uint64) is given, else base + i.     *
 * ------------------------------------------------------------------------------------------ */
int ptls_hip_fill_records(ptls_hip_batch_t *batch, void *buf, uint64_t seed, uint64_t index_base, const uint64_t *index,
                          void *stream);
/* The achievable-HBM reference of the roofline (bench.py): copy `bytes` (a multiple of 16; 16-byte aligned device
 * pointers) from src to dst on the engine's device, one 16-byte load and store per thread, asynchronously on `stream`. */
int ptls_hip_device_copy(ptls_hip_engine_t *engine, void *dst, const void *src, size_t bytes, void *stream);

#ifdef __cplusplus
}
#endif

#endif
