/*
 * aesgcm_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C, byte-at-a-time restatement of the AES-GCM record AEAD that picotls's
 * `lib/fusion.c` engine computes, used as the CPU checker for the MI355X engine.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.
 * Nothing in the product library (hsig-picotls_amd/) links or calls this code.
 *
 * Parity pin: the restatement is checked against
 *   (1) the known-answer vectors of the reference's own t/fusion.c (ECB :79,:84; gfmul :127-226;
 *       gcm_basic :238-264; gcm_capacity :278; gcm_test_vectors :309-331; gcm_iv96 :352-358),
 *   (2) fixtures produced by running the reference itself (lib/fusion.c built unmodified from
 *       /root/reference by oracle/Makefile into oracle/_ref/), see tests/golden/make_golden.py.
 */
#ifndef AESGCM_ORACLE_H
#define AESGCM_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* AES key expansion (FIPS-197 §5.2); the reference does the same with aeskeygenassist in
 * ptls_fusion_aesecb_init (lib/fusion.c:857-916).  rk receives (rounds+1)*16 bytes. */
int oracle_aes_expand(const uint8_t *key, size_t key_len, uint8_t rk[240]);

/* One AES block (FIPS-197 §5.1); reference: aesecb_encrypt (lib/fusion.c:322-334). */
void oracle_aes_encrypt(const uint8_t *rk, int rounds, const uint8_t in[16], uint8_t out[16]);

/* GF(2^128) multiply in GCM bit order (SP 800-38D Algorithm 1); reference: gfmul / gfmul_do_reduce
 * (lib/fusion.c:156-204) operate on the byte-reversed, transformH-shifted representation. */
void oracle_gf128_mul(const uint8_t x[16], const uint8_t y[16], uint8_t out[16]);

/* GHASH_H(A || 0* || C || 0* || [len(A)]64 || [len(C)]64) (SP 800-38D §6.4); reference: the
 * aggregated gfmul_*step128 chain over AAD, ciphertext and `ac` (lib/fusion.c:468, :513-632). */
void oracle_ghash(const uint8_t H[16], const uint8_t *aad, size_t aadlen, const uint8_t *c, size_t clen, uint8_t out[16]);

/* picotls nonce rule: iv[4..11] ^= BE64(seq); reference: ptls_aead__build_iv (lib/picotls.c:6492-6506),
 * fusion's calc_counter (lib/fusion.c:1126-1133). */
void oracle_build_iv(const uint8_t static_iv[12], uint64_t seq, uint8_t nonce[12]);

/* Seal: writes inlen bytes of ciphertext followed by the 16-byte tag to out; returns inlen + 16.
 * Reference: aead_do_encrypt -> ptls_fusion_aesgcm_encrypt (lib/fusion.c:1135-1143, :400-658). */
size_t oracle_aesgcm_seal(const uint8_t *key, size_t key_len, const uint8_t static_iv[12], uint64_t seq, const uint8_t *aad,
                          size_t aadlen, const uint8_t *in, size_t inlen, uint8_t *out);

/* Open: inlen includes the tag.  Plaintext is written to out even when the tag does not verify
 * (decrypt-then-verify, like ptls_fusion_aesgcm_decrypt lib/fusion.c:660-844).  Returns inlen - 16,
 * or SIZE_MAX when inlen < 16 or the tag mismatches (aead_do_decrypt lib/fusion.c:1151-1166). */
size_t oracle_aesgcm_open(const uint8_t *key, size_t key_len, const uint8_t static_iv[12], uint64_t seq, const uint8_t *aad,
                          size_t aadlen, const uint8_t *in, size_t inlen, uint8_t *out);

/* One AES-ECB block with a key (QUIC header-protection `supp` output, lib/fusion.c:636-650). */
void oracle_aes_ecb(const uint8_t *key, size_t key_len, const uint8_t in[16], uint8_t out[16]);

/* t/fusion.c:test_gfmul expresses H and the result in fusion's internal domain: H is the value held
 * in ghash[0].H (i.e. transformH(bswap(E_K(0)))) and the hash is the raw bytes of gstate.lo.
 * This maps that domain onto standard GHASH so the reference's gfmul KATs pin oracle_gf128_mul. */
void oracle_fusion_domain_ghash(const uint8_t H_fusion[16], const uint8_t *blocks, size_t nblocks, uint8_t out_lo[16]);

/* ---- synthetic workload generator; identical bytes on CPU and GPU ---- */
#define ORACLE_SEED_DATA 0x70746C7300000001ull
#define ORACLE_SEED_KEY 0x6B65790000000000ull
#define ORACLE_SEED_AAD 0x6161640000000000ull
#define ORACLE_SEED_LEN 0x00000000006C656Eull

uint64_t oracle_splitmix64_at(uint64_t seed, uint64_t k); /* k-th (0-based) output of the stream seeded with seed */
void oracle_stream_bytes(uint64_t seed, uint8_t *out, size_t n);
void oracle_gen_key(uint64_t j, size_t key_len, uint8_t *key, uint8_t iv[12]);
void oracle_gen_record(uint64_t i, uint8_t *out, size_t len);
void oracle_gen_quic_aad(uint64_t i, uint8_t aad[13]);
void oracle_tls_aad(size_t payload_len, uint8_t aad[5]);
uint32_t oracle_mixed_len(uint64_t i);

/* Multi-threaded bounded CPU baseline over synthetic records (used only when the reference build
 * in oracle/_ref is unavailable; then bench.py reports cpu_baseline.kind = "port").
 * Returns elapsed seconds for sealing nrec records of len bytes each, 5-byte TLS AAD, seq = i. */
double oracle_bench_seal(size_t key_len, size_t nrec, size_t len, int threads);

#ifdef __cplusplus
}
#endif

#endif
