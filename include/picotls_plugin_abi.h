/*
 * picotls_plugin_abi.h -- the part of picotls's public ABI that an AEAD engine plugs into.
 *
 * The MI355X engine is a drop-in crypto engine: its algorithm objects and contexts must have exactly
 * the layout picotls expects.  When the application (or picotls itself) has already included the real
 * "picotls.h", that header is authoritative and this file declares nothing.  Otherwise it declares
 * layout-identical restatements of the handful of plugin types, so the engine builds without a picotls
 * checkout.  Field order and types follow the reference header:
 *   ptls_iovec_t                            include/picotls.h:325-328
 *   ptls_cipher_context_t / _algorithm_t    include/picotls.h:397-415
 *   ptls_aead_supplementary_encryption_t    include/picotls.h:421-436
 *   ptls_aead_context_t                     include/picotls.h:444-494
 *   ptls_aead_algorithm_t                   include/picotls.h:499-560
 *   ptls_cipher_suite_t                     include/picotls.h:624-641
 * tests/test_abi.py checks sizes/offsets against the reference build (oracle/_ref) when present.
 */
#ifndef PTLS_HIP_PLUGIN_ABI_H
#define PTLS_HIP_PLUGIN_ABI_H

#include <stddef.h>
#include <stdint.h>

#ifndef picotls_h /* include guard of the real picotls.h */

#ifdef __cplusplus
extern "C" {
#endif

#define PTLS_AES128_KEY_SIZE 16
#define PTLS_AES256_KEY_SIZE 32
#define PTLS_AES_IV_SIZE 16
#define PTLS_AESGCM_IV_SIZE 12
#define PTLS_AESGCM_TAG_SIZE 16
#define PTLS_AESGCM_CONFIDENTIALITY_LIMIT 0x2000000            /* 2^25 records */
#define PTLS_AESGCM_INTEGRITY_LIMIT UINT64_C(0x40000000000000) /* 2^54 failed opens */

/* {pointer, length} pair used for gather input */
typedef struct st_ptls_iovec_t {
    uint8_t *base;
    size_t len;
} ptls_iovec_t;

struct st_ptls_cipher_algorithm_t;

/* symmetric (CTR / ECB) cipher instance */
typedef struct st_ptls_cipher_context_t {
    const struct st_ptls_cipher_algorithm_t *algo;
    void (*do_dispose)(struct st_ptls_cipher_context_t *ctx);
    void (*do_init)(struct st_ptls_cipher_context_t *ctx, const void *iv);
    void (*do_transform)(struct st_ptls_cipher_context_t *ctx, void *output, const void *input, size_t len);
} ptls_cipher_context_t;

typedef const struct st_ptls_cipher_algorithm_t {
    const char *name;
    size_t key_size;
    size_t block_size;
    size_t iv_size;
    size_t context_size;
    int (*setup_crypto)(ptls_cipher_context_t *ctx, int is_enc, const void *key);
} ptls_cipher_algorithm_t;

/* QUIC header protection computed alongside an AEAD seal */
typedef struct st_ptls_aead_supplementary_encryption_t {
    ptls_cipher_context_t *ctx;
    const void *input;
    uint8_t output[16];
} ptls_aead_supplementary_encryption_t;

/* AEAD instance; engines append private state after these members (context_size) */
typedef struct st_ptls_aead_context_t {
    const struct st_ptls_aead_algorithm_t *algo;
    void (*dispose_crypto)(struct st_ptls_aead_context_t *ctx);
    void (*do_get_iv)(struct st_ptls_aead_context_t *ctx, void *iv);
    void (*do_set_iv)(struct st_ptls_aead_context_t *ctx, const void *iv);
    void (*do_encrypt_init)(struct st_ptls_aead_context_t *ctx, uint64_t seq, const void *aad, size_t aadlen);
    size_t (*do_encrypt_update)(struct st_ptls_aead_context_t *ctx, void *output, const void *input, size_t inlen);
    size_t (*do_encrypt_final)(struct st_ptls_aead_context_t *ctx, void *output);
    void (*do_encrypt)(struct st_ptls_aead_context_t *ctx, void *output, const void *input, size_t inlen, uint64_t seq,
                       const void *aad, size_t aadlen, ptls_aead_supplementary_encryption_t *supp);
    void (*do_encrypt_v)(struct st_ptls_aead_context_t *ctx, void *output, ptls_iovec_t *input, size_t incnt, uint64_t seq,
                         const void *aad, size_t aadlen);
    size_t (*do_decrypt)(struct st_ptls_aead_context_t *ctx, void *output, const void *input, size_t inlen, uint64_t seq,
                         const void *aad, size_t aadlen);
} ptls_aead_context_t;

/* AEAD algorithm descriptor (what a cipher suite points at) */
typedef const struct st_ptls_aead_algorithm_t {
    const char *name;
    const uint64_t confidentiality_limit;
    const uint64_t integrity_limit;
    ptls_cipher_algorithm_t *ctr_cipher;
    ptls_cipher_algorithm_t *ecb_cipher;
    size_t key_size;
    size_t iv_size;
    size_t tag_size;
    struct {
        size_t fixed_iv_size;
        size_t record_iv_size;
    } tls12;
    unsigned non_temporal : 1;
    uint8_t align_bits;
    size_t context_size;
    int (*setup_crypto)(ptls_aead_context_t *ctx, int is_enc, const void *key, const void *iv);
} ptls_aead_algorithm_t;

struct st_ptls_hash_algorithm_t; /* opaque here: suites pair our AEAD with another engine's hash */

typedef const struct st_ptls_cipher_suite_t {
    uint16_t id;
    ptls_aead_algorithm_t *aead;
    const struct st_ptls_hash_algorithm_t *hash;
    const char *name;
} ptls_cipher_suite_t;

#ifdef __cplusplus
}
#endif

#endif /* picotls_h */
#endif
