/*
 * keyschedule.hip -- TLS 1.3 record-key derivation on the device.
 *
 * For many connections at once: record key and IV from a traffic secret, and the key-update step,
 * exactly as picotls derives them on the host for one connection:
 *   key  = HKDF-Expand-Label(secret, "key", "", key_size)      get_traffic_keys, lib/picotls.c:1603-1622
 *   iv   = HKDF-Expand-Label(secret, "iv",  "", 12)
 *   next = HKDF-Expand-Label(secret, "traffic upd", "", Nh)    update_traffic_key, lib/picotls.c:4980-4996
 * HKDF-Expand-Label (ptls_hkdf_expand_label, :6348-6371): info = BE16(L) || u8(6 + |label|) || "tls13 " ||
 * label || u8(0); HKDF-Expand (ptls_hkdf_expand, :6316-6346) with L <= Nh is ONE HMAC: T(1) =
 * HMAC(secret, info || 0x01).  SHA-256 for TLS_AES_128_GCM_SHA256, SHA-384 for TLS_AES_256_GCM_SHA384
 * (FIPS 180-4).  One thread per connection: a handful of compression-function calls, no tables.
 */
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "internal.h"

namespace ptls_hip {

/* ---------------- SHA-256 (FIPS 180-4 §6.2) ---------------- */

__device__ __constant__ uint32_t K256[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5, 0xd807aa98, 0x12835b01,
    0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174, 0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc,
    0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da, 0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147,
    0x06ca6351, 0x14292967, 0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070, 0x19a4c116, 0x1e376c08,
    0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3, 0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208,
    0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

__device__ __forceinline__ uint32_t ror32(uint32_t x, int n)
{
    return __builtin_amdgcn_alignbit(x, x, n);
}

/* state h[8] absorbs one 64-byte block given as 16 big-endian words */
__device__ void sha256_block(uint32_t h[8], const uint32_t w_in[16])
{
    uint32_t w[16];
    for (int i = 0; i < 16; ++i)
        w[i] = w_in[i];
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], k = h[7];
    for (int i = 0; i < 64; ++i) {
        uint32_t wi;
        if (i < 16) {
            wi = w[i];
        } else {
            const uint32_t w15 = w[(i + 1) & 15], w2 = w[(i + 14) & 15];
            const uint32_t s0 = ror32(w15, 7) ^ ror32(w15, 18) ^ (w15 >> 3);
            const uint32_t s1 = ror32(w2, 17) ^ ror32(w2, 19) ^ (w2 >> 10);
            wi = w[i & 15] = w[i & 15] + s0 + w[(i + 9) & 15] + s1;
        }
        const uint32_t t1 = k + (ror32(e, 6) ^ ror32(e, 11) ^ ror32(e, 25)) + ((e & f) ^ (~e & g)) + K256[i] + wi;
        const uint32_t t2 = (ror32(a, 2) ^ ror32(a, 13) ^ ror32(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
        k = g;
        g = f;
        f = e;
        e = d + t1;
        d = c;
        c = b;
        b = a;
        a = t1 + t2;
    }
    h[0] += a;
    h[1] += b;
    h[2] += c;
    h[3] += d;
    h[4] += e;
    h[5] += f;
    h[6] += g;
    h[7] += k;
}

/* ---------------- SHA-384 = SHA-512 with its own IV, truncated (FIPS 180-4 §6.4, §6.5) ---------------- */

__device__ __constant__ uint64_t K512[80] = {
    0x428a2f98d728ae22ull, 0x7137449123ef65cdull, 0xb5c0fbcfec4d3b2full, 0xe9b5dba58189dbbcull, 0x3956c25bf348b538ull,
    0x59f111f1b605d019ull, 0x923f82a4af194f9bull, 0xab1c5ed5da6d8118ull, 0xd807aa98a3030242ull, 0x12835b0145706fbeull,
    0x243185be4ee4b28cull, 0x550c7dc3d5ffb4e2ull, 0x72be5d74f27b896full, 0x80deb1fe3b1696b1ull, 0x9bdc06a725c71235ull,
    0xc19bf174cf692694ull, 0xe49b69c19ef14ad2ull, 0xefbe4786384f25e3ull, 0x0fc19dc68b8cd5b5ull, 0x240ca1cc77ac9c65ull,
    0x2de92c6f592b0275ull, 0x4a7484aa6ea6e483ull, 0x5cb0a9dcbd41fbd4ull, 0x76f988da831153b5ull, 0x983e5152ee66dfabull,
    0xa831c66d2db43210ull, 0xb00327c898fb213full, 0xbf597fc7beef0ee4ull, 0xc6e00bf33da88fc2ull, 0xd5a79147930aa725ull,
    0x06ca6351e003826full, 0x142929670a0e6e70ull, 0x27b70a8546d22ffcull, 0x2e1b21385c26c926ull, 0x4d2c6dfc5ac42aedull,
    0x53380d139d95b3dfull, 0x650a73548baf63deull, 0x766a0abb3c77b2a8ull, 0x81c2c92e47edaee6ull, 0x92722c851482353bull,
    0xa2bfe8a14cf10364ull, 0xa81a664bbc423001ull, 0xc24b8b70d0f89791ull, 0xc76c51a30654be30ull, 0xd192e819d6ef5218ull,
    0xd69906245565a910ull, 0xf40e35855771202aull, 0x106aa07032bbd1b8ull, 0x19a4c116b8d2d0c8ull, 0x1e376c085141ab53ull,
    0x2748774cdf8eeb99ull, 0x34b0bcb5e19b48a8ull, 0x391c0cb3c5c95a63ull, 0x4ed8aa4ae3418acbull, 0x5b9cca4f7763e373ull,
    0x682e6ff3d6b2b8a3ull, 0x748f82ee5defb2fcull, 0x78a5636f43172f60ull, 0x84c87814a1f0ab72ull, 0x8cc702081a6439ecull,
    0x90befffa23631e28ull, 0xa4506cebde82bde9ull, 0xbef9a3f7b2c67915ull, 0xc67178f2e372532bull, 0xca273eceea26619cull,
    0xd186b8c721c0c207ull, 0xeada7dd6cde0eb1eull, 0xf57d4f7fee6ed178ull, 0x06f067aa72176fbaull, 0x0a637dc5a2c898a6ull,
    0x113f9804bef90daeull, 0x1b710b35131c471bull, 0x28db77f523047d84ull, 0x32caab7b40c72493ull, 0x3c9ebe0a15c9bebcull,
    0x431d67c49c100d4cull, 0x4cc5d4becb3e42b6ull, 0x597f299cfc657e2aull, 0x5fcb6fab3ad6faecull, 0x6c44198c4a475817ull};

__device__ __forceinline__ uint64_t ror64(uint64_t x, int n)
{
    return (x >> n) | (x << (64 - n));
}

__device__ void sha512_block(uint64_t h[8], const uint64_t w_in[16])
{
    uint64_t w[16];
    for (int i = 0; i < 16; ++i)
        w[i] = w_in[i];
    uint64_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], k = h[7];
    for (int i = 0; i < 80; ++i) {
        uint64_t wi;
        if (i < 16) {
            wi = w[i];
        } else {
            const uint64_t w15 = w[(i + 1) & 15], w2 = w[(i + 14) & 15];
            const uint64_t s0 = ror64(w15, 1) ^ ror64(w15, 8) ^ (w15 >> 7);
            const uint64_t s1 = ror64(w2, 19) ^ ror64(w2, 61) ^ (w2 >> 6);
            wi = w[i & 15] = w[i & 15] + s0 + w[(i + 9) & 15] + s1;
        }
        const uint64_t t1 = k + (ror64(e, 14) ^ ror64(e, 18) ^ ror64(e, 41)) + ((e & f) ^ (~e & g)) + K512[i] + wi;
        const uint64_t t2 = (ror64(a, 28) ^ ror64(a, 34) ^ ror64(a, 39)) + ((a & b) ^ (a & c) ^ (b & c));
        k = g;
        g = f;
        f = e;
        e = d + t1;
        d = c;
        c = b;
        b = a;
        a = t1 + t2;
    }
    h[0] += a;
    h[1] += b;
    h[2] += c;
    h[3] += d;
    h[4] += e;
    h[5] += f;
    h[6] += g;
    h[7] += k;
}

/* ---------------- HMAC over one short message (RFC 2104) ---------------- */

/* HMAC-SHA256(key[klen <= 64], msg[mlen <= 55]) -> out[32] */
__device__ void hmac_sha256(const uint8_t *key, int klen, const uint8_t *msg, int mlen, uint8_t out[32])
{
    static const uint32_t IV[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
    uint8_t kb[64];
    for (int i = 0; i < 64; ++i)
        kb[i] = i < klen ? key[i] : 0;
    uint32_t w[16], hi[8], ho[8];
    for (int i = 0; i < 8; ++i)
        hi[i] = ho[i] = IV[i];
    for (int i = 0; i < 16; ++i)
        w[i] = ((uint32_t)kb[4 * i] << 24 | (uint32_t)kb[4 * i + 1] << 16 | (uint32_t)kb[4 * i + 2] << 8 | kb[4 * i + 3]) ^ 0x36363636u;
    sha256_block(hi, w);
    for (int i = 0; i < 16; ++i)
        w[i] ^= 0x36363636u ^ 0x5c5c5c5cu;
    sha256_block(ho, w);
    /* inner: msg || 0x80 || 0.. || BE64(8 * (64 + mlen)) */
    uint8_t blk[64];
    for (int i = 0; i < 64; ++i)
        blk[i] = i < mlen ? msg[i] : (i == mlen ? 0x80 : 0);
    const uint32_t bits = 8u * (64u + (uint32_t)mlen);
    blk[60] = (uint8_t)(bits >> 24);
    blk[61] = (uint8_t)(bits >> 16);
    blk[62] = (uint8_t)(bits >> 8);
    blk[63] = (uint8_t)bits;
    for (int i = 0; i < 16; ++i)
        w[i] = (uint32_t)blk[4 * i] << 24 | (uint32_t)blk[4 * i + 1] << 16 | (uint32_t)blk[4 * i + 2] << 8 | blk[4 * i + 3];
    sha256_block(hi, w);
    /* outer: inner digest (32 B) || 0x80 || 0.. || BE64(8 * 96) */
    for (int i = 0; i < 8; ++i)
        w[i] = hi[i];
    w[8] = 0x80000000u;
    for (int i = 9; i < 15; ++i)
        w[i] = 0;
    w[15] = 8u * 96u;
    sha256_block(ho, w);
    for (int i = 0; i < 8; ++i) {
        out[4 * i] = (uint8_t)(ho[i] >> 24);
        out[4 * i + 1] = (uint8_t)(ho[i] >> 16);
        out[4 * i + 2] = (uint8_t)(ho[i] >> 8);
        out[4 * i + 3] = (uint8_t)ho[i];
    }
}

/* HMAC-SHA384(key[klen <= 128], msg[mlen <= 111]) -> out[48] */
__device__ void hmac_sha384(const uint8_t *key, int klen, const uint8_t *msg, int mlen, uint8_t out[48])
{
    static const uint64_t IV[8] = {0xcbbb9d5dc1059ed8ull, 0x629a292a367cd507ull, 0x9159015a3070dd17ull, 0x152fecd8f70e5939ull,
                                   0x67332667ffc00b31ull, 0x8eb44a8768581511ull, 0xdb0c2e0d64f98fa7ull, 0x47b5481dbefa4fa4ull};
    uint8_t kb[128];
    for (int i = 0; i < 128; ++i)
        kb[i] = i < klen ? key[i] : 0;
    uint64_t w[16], hi[8], ho[8];
    for (int i = 0; i < 8; ++i)
        hi[i] = ho[i] = IV[i];
    for (int i = 0; i < 16; ++i) {
        uint64_t v = 0;
        for (int j = 0; j < 8; ++j)
            v = v << 8 | kb[8 * i + j];
        w[i] = v ^ 0x3636363636363636ull;
    }
    sha512_block(hi, w);
    for (int i = 0; i < 16; ++i)
        w[i] ^= 0x3636363636363636ull ^ 0x5c5c5c5c5c5c5c5cull;
    sha512_block(ho, w);
    uint8_t blk[128];
    for (int i = 0; i < 128; ++i)
        blk[i] = i < mlen ? msg[i] : (i == mlen ? 0x80 : 0);
    const uint32_t bits = 8u * (128u + (uint32_t)mlen); /* BE128 length, high words zero */
    blk[124] = (uint8_t)(bits >> 24);
    blk[125] = (uint8_t)(bits >> 16);
    blk[126] = (uint8_t)(bits >> 8);
    blk[127] = (uint8_t)bits;
    for (int i = 0; i < 16; ++i) {
        uint64_t v = 0;
        for (int j = 0; j < 8; ++j)
            v = v << 8 | blk[8 * i + j];
        w[i] = v;
    }
    sha512_block(hi, w);
    /* outer: 48-byte inner digest || 0x80 || 0.. || BE128(8 * 176) */
    for (int i = 0; i < 6; ++i)
        w[i] = hi[i];
    w[6] = 0x8000000000000000ull;
    for (int i = 7; i < 15; ++i)
        w[i] = 0;
    w[15] = 8ull * 176ull;
    sha512_block(ho, w);
    for (int i = 0; i < 6; ++i)
        for (int j = 0; j < 8; ++j)
            out[8 * i + j] = (uint8_t)(ho[i] >> (56 - 8 * j));
}

/* HKDF-Expand-Label(secret, label, "", outlen) with outlen <= Nh: one HMAC of info || 0x01 */
__device__ void hkdf_expand_label(int hash_size, const uint8_t *secret, const char *label, int label_len, int outlen, uint8_t *out)
{
    uint8_t info[64];
    int n = 0;
    info[n++] = (uint8_t)(outlen >> 8);
    info[n++] = (uint8_t)outlen;
    info[n++] = (uint8_t)(6 + label_len);
    const char prefix[6] = {'t', 'l', 's', '1', '3', ' '};
    for (int i = 0; i < 6; ++i)
        info[n++] = (uint8_t)prefix[i];
    for (int i = 0; i < label_len; ++i)
        info[n++] = (uint8_t)label[i];
    info[n++] = 0; /* empty context (hash_value) */
    info[n++] = 1; /* HKDF-Expand counter T(1) */
    uint8_t t[48];
    if (hash_size == 32)
        hmac_sha256(secret, 32, info, n, t);
    else
        hmac_sha384(secret, 48, info, n, t);
    for (int i = 0; i < outlen; ++i)
        out[i] = t[i];
}

/* per connection: (optionally) the key-update step, then the record key and IV of the secret */
__global__ void __launch_bounds__(64) derive_traffic_keys_kernel(const uint8_t *__restrict__ secrets_in, uint8_t *__restrict__ secrets_out,
                                                                 uint32_t count, int hash_size, int key_size, int update,
                                                                 uint8_t *__restrict__ keys, uint8_t *__restrict__ ivs)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= count)
        return;
    uint8_t secret[48];
    for (int j = 0; j < hash_size; ++j)
        secret[j] = secrets_in[(size_t)i * hash_size + j];
    if (update) {
        uint8_t next[48];
        hkdf_expand_label(hash_size, secret, "traffic upd", 11, hash_size, next);
        for (int j = 0; j < hash_size; ++j)
            secret[j] = next[j];
    }
    if (secrets_out != nullptr)
        for (int j = 0; j < hash_size; ++j)
            secrets_out[(size_t)i * hash_size + j] = secret[j];
    hkdf_expand_label(hash_size, secret, "key", 3, key_size, keys + (size_t)i * key_size);
    hkdf_expand_label(hash_size, secret, "iv", 2, 12, ivs + (size_t)i * 12);
    for (int j = 0; j < 48; ++j)
        secret[j] = 0;
}

int launch_derive_traffic_keys(const uint8_t *secrets_in, uint8_t *secrets_out, uint32_t count, int hash_size, int key_size,
                               int update, uint8_t *keys, uint8_t *ivs, void *stream)
{
    const unsigned grid = (count + 63) / 64;
    hipLaunchKernelGGL(derive_traffic_keys_kernel, dim3(grid), dim3(64), 0, static_cast<hipStream_t>(stream), secrets_in,
                       secrets_out, count, hash_size, key_size, update, keys, ivs);
    return (int)hipGetLastError();
}

} // namespace ptls_hip
