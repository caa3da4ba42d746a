/*
 * aesgcm_oracle.c -- TEST INFRASTRUCTURE ONLY (see aesgcm_oracle.h).
 *
 * Deliberately naive: byte-oriented AES with an S-box derived at start-up from the GF(2^8)
 * inverse + affine map (FIPS-197 §5.1.1), bit-serial GF(2^128) multiplication (SP 800-38D
 * Algorithm 1).  It shares no code or data layout with the HIP engine it checks.
 */
#include "aesgcm_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

static uint8_t sbox[256];
static pthread_once_t sbox_once = PTHREAD_ONCE_INIT;

static uint8_t gf8_mul(uint8_t a, uint8_t b)
{
    uint8_t p = 0;
    while (b != 0) {
        if (b & 1)
            p ^= a;
        a = (uint8_t)((a << 1) ^ ((a & 0x80) ? 0x1b : 0));
        b >>= 1;
    }
    return p;
}

static void sbox_init(void)
{
    for (int x = 0; x < 256; ++x) {
        uint8_t inv = 0;
        if (x != 0) {
            for (int y = 1; y < 256; ++y)
                if (gf8_mul((uint8_t)x, (uint8_t)y) == 1) {
                    inv = (uint8_t)y;
                    break;
                }
        }
        uint8_t s = inv;
        for (int r = 1; r <= 4; ++r)
            s ^= (uint8_t)((inv << r) | (inv >> (8 - r)));
        sbox[x] = s ^ 0x63;
    }
}

int oracle_aes_expand(const uint8_t *key, size_t key_len, uint8_t rk[240])
{
    pthread_once(&sbox_once, sbox_init);
    size_t nk = key_len / 4, rounds = nk + 6, total = 4 * (rounds + 1);
    uint8_t rcon = 1;
    if (key_len != 16 && key_len != 32)
        return -1;
    memcpy(rk, key, key_len);
    for (size_t i = nk; i < total; ++i) {
        uint8_t t[4];
        memcpy(t, rk + 4 * (i - 1), 4);
        if (i % nk == 0) {
            uint8_t u = t[0];
            t[0] = (uint8_t)(sbox[t[1]] ^ rcon);
            t[1] = sbox[t[2]];
            t[2] = sbox[t[3]];
            t[3] = sbox[u];
            rcon = gf8_mul(rcon, 2);
        } else if (nk > 6 && i % nk == 4) {
            for (int k = 0; k < 4; ++k)
                t[k] = sbox[t[k]];
        }
        for (int k = 0; k < 4; ++k)
            rk[4 * i + k] = rk[4 * (i - nk) + k] ^ t[k];
    }
    return (int)rounds;
}

void oracle_aes_encrypt(const uint8_t *rk, int rounds, const uint8_t in[16], uint8_t out[16])
{
    pthread_once(&sbox_once, sbox_init);
    uint8_t s[16], t[16];
    for (int i = 0; i < 16; ++i)
        s[i] = in[i] ^ rk[i];
    for (int r = 1; r <= rounds; ++r) {
        /* SubBytes + ShiftRows: state byte (row, col) lives at s[4*col + row] */
        for (int c = 0; c < 4; ++c)
            for (int row = 0; row < 4; ++row)
                t[4 * c + row] = sbox[s[4 * ((c + row) & 3) + row]];
        if (r != rounds) { /* MixColumns */
            for (int c = 0; c < 4; ++c) {
                uint8_t a0 = t[4 * c], a1 = t[4 * c + 1], a2 = t[4 * c + 2], a3 = t[4 * c + 3];
                s[4 * c + 0] = gf8_mul(a0, 2) ^ gf8_mul(a1, 3) ^ a2 ^ a3;
                s[4 * c + 1] = a0 ^ gf8_mul(a1, 2) ^ gf8_mul(a2, 3) ^ a3;
                s[4 * c + 2] = a0 ^ a1 ^ gf8_mul(a2, 2) ^ gf8_mul(a3, 3);
                s[4 * c + 3] = gf8_mul(a0, 3) ^ a1 ^ a2 ^ gf8_mul(a3, 2);
            }
        } else {
            memcpy(s, t, 16);
        }
        for (int i = 0; i < 16; ++i)
            s[i] ^= rk[16 * r + i];
    }
    memcpy(out, s, 16);
}

void oracle_aes_ecb(const uint8_t *key, size_t key_len, const uint8_t in[16], uint8_t out[16])
{
    uint8_t rk[240];
    int rounds = oracle_aes_expand(key, key_len, rk);
    oracle_aes_encrypt(rk, rounds, in, out);
}

void oracle_gf128_mul(const uint8_t x[16], const uint8_t y[16], uint8_t out[16])
{
    uint8_t z[16] = {0}, v[16];
    memcpy(v, y, 16);
    for (int i = 0; i < 128; ++i) {
        if (x[i / 8] & (0x80 >> (i % 8)))
            for (int k = 0; k < 16; ++k)
                z[k] ^= v[k];
        int lsb = v[15] & 1;
        for (int k = 15; k > 0; --k)
            v[k] = (uint8_t)((v[k] >> 1) | (v[k - 1] << 7));
        v[0] >>= 1;
        if (lsb)
            v[0] ^= 0xe1;
    }
    memcpy(out, z, 16);
}

static void ghash_update(uint8_t y[16], const uint8_t H[16], const uint8_t *p, size_t len)
{
    while (len != 0) {
        size_t n = len < 16 ? len : 16;
        for (size_t k = 0; k < n; ++k)
            y[k] ^= p[k];
        oracle_gf128_mul(y, H, y);
        p += n;
        len -= n;
    }
}

void oracle_ghash(const uint8_t H[16], const uint8_t *aad, size_t aadlen, const uint8_t *c, size_t clen, uint8_t out[16])
{
    uint8_t y[16] = {0}, lens[16];
    ghash_update(y, H, aad, aadlen);
    ghash_update(y, H, c, clen);
    uint64_t abits = (uint64_t)aadlen * 8, cbits = (uint64_t)clen * 8;
    for (int k = 0; k < 8; ++k) {
        lens[k] = (uint8_t)(abits >> (56 - 8 * k));
        lens[8 + k] = (uint8_t)(cbits >> (56 - 8 * k));
    }
    ghash_update(y, H, lens, 16);
    memcpy(out, y, 16);
}

void oracle_build_iv(const uint8_t static_iv[12], uint64_t seq, uint8_t nonce[12])
{
    memcpy(nonce, static_iv, 4);
    for (int k = 0; k < 8; ++k)
        nonce[4 + k] = static_iv[4 + k] ^ (uint8_t)(seq >> (56 - 8 * k));
}

/* CTR keystream from inc32(J0), J0 = nonce || 00000001 (SP 800-38D §7.1) */
static void ctr_apply(const uint8_t *rk, int rounds, const uint8_t nonce[12], const uint8_t *in, size_t len, uint8_t *out)
{
    uint8_t cb[16], ks[16];
    memcpy(cb, nonce, 12);
    uint32_t ctr = 2;
    for (size_t off = 0; off < len; off += 16, ++ctr) {
        cb[12] = (uint8_t)(ctr >> 24);
        cb[13] = (uint8_t)(ctr >> 16);
        cb[14] = (uint8_t)(ctr >> 8);
        cb[15] = (uint8_t)ctr;
        oracle_aes_encrypt(rk, rounds, cb, ks);
        size_t n = len - off < 16 ? len - off : 16;
        for (size_t k = 0; k < n; ++k)
            out[off + k] = in[off + k] ^ ks[k];
    }
}

static void compute_tag(const uint8_t *rk, int rounds, const uint8_t nonce[12], const uint8_t *aad, size_t aadlen,
                        const uint8_t *ct, size_t len, uint8_t tag[16])
{
    uint8_t zero[16] = {0}, H[16], j0[16], ekj0[16], s[16];
    oracle_aes_encrypt(rk, rounds, zero, H);
    oracle_ghash(H, aad, aadlen, ct, len, s);
    memcpy(j0, nonce, 12);
    j0[12] = j0[13] = j0[14] = 0;
    j0[15] = 1;
    oracle_aes_encrypt(rk, rounds, j0, ekj0);
    for (int k = 0; k < 16; ++k)
        tag[k] = s[k] ^ ekj0[k];
}

size_t oracle_aesgcm_seal(const uint8_t *key, size_t key_len, const uint8_t static_iv[12], uint64_t seq, const uint8_t *aad,
                          size_t aadlen, const uint8_t *in, size_t inlen, uint8_t *out)
{
    uint8_t rk[240], nonce[12], tag[16];
    int rounds = oracle_aes_expand(key, key_len, rk);
    oracle_build_iv(static_iv, seq, nonce);
    ctr_apply(rk, rounds, nonce, in, inlen, out); /* out == in allowed: byte-wise in order */
    compute_tag(rk, rounds, nonce, aad, aadlen, out, inlen, tag);
    memcpy(out + inlen, tag, 16);
    return inlen + 16;
}

size_t oracle_aesgcm_open(const uint8_t *key, size_t key_len, const uint8_t static_iv[12], uint64_t seq, const uint8_t *aad,
                          size_t aadlen, const uint8_t *in, size_t inlen, uint8_t *out)
{
    uint8_t rk[240], nonce[12], tag[16], rtag[16];
    if (inlen < 16)
        return SIZE_MAX;
    size_t len = inlen - 16;
    int rounds = oracle_aes_expand(key, key_len, rk);
    oracle_build_iv(static_iv, seq, nonce);
    memcpy(rtag, in + len, 16);
    compute_tag(rk, rounds, nonce, aad, aadlen, in, len, tag); /* GHASH over ciphertext before in-place decrypt */
    ctr_apply(rk, rounds, nonce, in, len, out);
    return memcmp(tag, rtag, 16) == 0 ? len : SIZE_MAX;
}

void oracle_fusion_domain_ghash(const uint8_t H_fusion[16], const uint8_t *blocks, size_t nblocks, uint8_t out_lo[16])
{
    /* fusion keeps H as V' = transformH(V), V = big-endian integer of E_K(0) (lib/fusion.c:996-998, :126-153):
     * V' = (V << 1) ^ (V>>127 ? 0xC2000000000000000000000000000001 : 0).  Undo it here: bit 0 of V' is the
     * shifted-out carry because V << 1 has bit 0 clear and the polynomial has bit 0 set. */
    uint8_t be[16], H[16], y[16];
    for (int k = 0; k < 16; ++k)
        be[k] = H_fusion[15 - k]; /* __m128i memory is little-endian: make it a big-endian byte string */
    int carry = be[15] & 1;
    if (carry) {
        be[15] ^= 0x01;
        be[0] ^= 0xc2;
    }
    for (int k = 15; k > 0; --k)
        H[k] = (uint8_t)((be[k] >> 1) | (be[k - 1] << 7));
    H[0] = (uint8_t)((be[0] >> 1) | (carry << 7));
    memset(y, 0, 16);
    ghash_update(y, H, blocks, nblocks * 16);
    for (int k = 0; k < 16; ++k) /* gstate.lo holds bswap(GHASH) (gfmul_get_tag128, lib/fusion.c:259-264) */
        out_lo[k] = y[15 - k];
}

/* ---------------- synthetic workload ---------------- */

static inline uint64_t splitmix_mix(uint64_t z)
{
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

uint64_t oracle_splitmix64_at(uint64_t seed, uint64_t k)
{
    return splitmix_mix(seed + (k + 1) * 0x9e3779b97f4a7c15ull);
}

void oracle_stream_bytes(uint64_t seed, uint8_t *out, size_t n)
{
    for (size_t w = 0; w * 8 < n; ++w) {
        uint64_t v = oracle_splitmix64_at(seed, w);
        for (size_t b = 0; b < 8 && w * 8 + b < n; ++b)
            out[w * 8 + b] = (uint8_t)(v >> (8 * b));
    }
}

void oracle_gen_key(uint64_t j, size_t key_len, uint8_t *key, uint8_t iv[12])
{
    uint8_t buf[48];
    oracle_stream_bytes(ORACLE_SEED_KEY ^ j, buf, key_len + 12);
    memcpy(key, buf, key_len);
    memcpy(iv, buf + key_len, 12);
}

void oracle_gen_record(uint64_t i, uint8_t *out, size_t len)
{
    oracle_stream_bytes(ORACLE_SEED_DATA ^ i, out, len);
}

void oracle_gen_quic_aad(uint64_t i, uint8_t aad[13])
{
    oracle_stream_bytes(ORACLE_SEED_AAD ^ i, aad, 13);
}

void oracle_tls_aad(size_t payload_len, uint8_t aad[5])
{
    size_t reclen = payload_len + 16; /* build_aad(aad, inlen + tag) lib/picotls.c:696-703 */
    aad[0] = 0x17;
    aad[1] = 0x03;
    aad[2] = 0x03;
    aad[3] = (uint8_t)(reclen >> 8);
    aad[4] = (uint8_t)reclen;
}

uint32_t oracle_mixed_len(uint64_t i)
{
    return 64 + (uint32_t)(oracle_splitmix64_at(ORACLE_SEED_LEN ^ i, 0) % 16321);
}

struct bench_arg {
    size_t key_len, first, count, len;
};

static void *bench_thread(void *p)
{
    struct bench_arg *a = p;
    uint8_t key[32], iv[12], aad[5];
    uint8_t *in = malloc(a->len), *out = malloc(a->len + 16);
    oracle_gen_key(0, a->key_len, key, iv);
    oracle_tls_aad(a->len, aad);
    for (size_t i = a->first; i < a->first + a->count; ++i) {
        oracle_gen_record(i, in, a->len);
        oracle_aesgcm_seal(key, a->key_len, iv, i, aad, 5, in, a->len, out);
    }
    free(in);
    free(out);
    return NULL;
}

double oracle_bench_seal(size_t key_len, size_t nrec, size_t len, int threads)
{
    pthread_t th[256];
    struct bench_arg args[256];
    struct timespec t0, t1;
    if (threads < 1)
        threads = 1;
    if (threads > 256)
        threads = 256;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (int t = 0; t < threads; ++t) {
        args[t] = (struct bench_arg){key_len, nrec * t / threads, nrec * (t + 1) / threads - nrec * t / threads, len};
        pthread_create(&th[t], NULL, bench_thread, &args[t]);
    }
    for (int t = 0; t < threads; ++t)
        pthread_join(th[t], NULL);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}
