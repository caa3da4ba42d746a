/*
 * ref_harness.c -- TEST / BASELINE INFRASTRUCTURE ONLY.
 *
 * Thin driver compiled together with the UNMODIFIED reference sources
 * (/root/reference/lib/{fusion,picotls,hpke}.c) into oracle/_ref/libptls_fusion_ref.so by
 * oracle/Makefile.  It reaches lib/fusion.c only through picotls's public plugin surface
 * (ptls_aead_new_direct / ptls_aead_encrypt* / ptls_aead_decrypt, include/picotls.h:1993-2055,
 * lib/picotls.c:6458-6479), exactly as a picotls application would.
 *
 * Used for: golden-vector generation (tests/golden/make_golden.py), differential CPU tests, the
 * drop-in test that instantiates the HIP engine through the reference's own ptls_aead_new_direct,
 * and bench.py's cpu_baseline leg (kind "reference").
 */
#define _GNU_SOURCE
#include <pthread.h>
#include <sched.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include "picotls.h"
#include "picotls/fusion.h"
#include "picotls/minicrypto.h"

static double now(void)
{
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

static ptls_aead_algorithm_t *pick(int bits)
{
    return bits == 256 ? &ptls_fusion_aes256gcm : &ptls_fusion_aes128gcm;
}

int ref_fusion_supported(void)
{
    return ptls_fusion_is_supported_by_cpu();
}

int ref_fusion_can_aesni256(void)
{
    return ptls_fusion_can_aesni256;
}

size_t ref_seal(int bits, const void *key, const void *iv, uint64_t seq, const void *aad, size_t aadlen, const void *in,
                size_t inlen, void *out)
{
    ptls_aead_context_t *ctx = ptls_aead_new_direct(pick(bits), 1, key, iv);
    size_t r = ptls_aead_encrypt(ctx, out, in, inlen, seq, aad, aadlen);
    ptls_aead_free(ctx);
    return r;
}

/* seal with QUIC header-protection supplementary block (ptls_aead_encrypt_s, include/picotls.h:2000) */
size_t ref_seal_supp(int bits, const void *key, const void *iv, uint64_t seq, const void *aad, size_t aadlen, const void *in,
                     size_t inlen, void *out, const void *hp_key, size_t supp_off, void *supp_out)
{
    ptls_aead_context_t *ctx = ptls_aead_new_direct(pick(bits), 1, key, iv);
    ptls_aead_supplementary_encryption_t supp;
    supp.ctx = ptls_cipher_new(bits == 256 ? &ptls_fusion_aes256ctr : &ptls_fusion_aes128ctr, 1, hp_key);
    supp.input = (uint8_t *)out + supp_off;
    ptls_aead_encrypt_s(ctx, out, in, inlen, seq, aad, aadlen, &supp);
    memcpy(supp_out, supp.output, 16);
    ptls_cipher_free(supp.ctx);
    ptls_aead_free(ctx);
    return inlen + 16;
}

size_t ref_open(int bits, const void *key, const void *iv, uint64_t seq, const void *aad, size_t aadlen, const void *in,
                size_t inlen, void *out)
{
    ptls_aead_context_t *ctx = ptls_aead_new_direct(pick(bits), 0, key, iv);
    size_t r = ptls_aead_decrypt(ctx, out, in, inlen, seq, aad, aadlen);
    ptls_aead_free(ctx);
    return r;
}

/* ptls_aead_xor_iv (lib/picotls.c:6481-6490) then seal, as in t/fusion.c:gcm_iv96 */
size_t ref_seal_iv96(int bits, const void *key, const void *iv, const void *xor_bytes, size_t xor_len, uint64_t seq,
                     const void *aad, size_t aadlen, const void *in, size_t inlen, void *out)
{
    ptls_aead_context_t *ctx = ptls_aead_new_direct(pick(bits), 1, key, iv);
    ptls_aead_xor_iv(ctx, xor_bytes, xor_len);
    size_t r = ptls_aead_encrypt(ctx, out, in, inlen, seq, aad, aadlen);
    ptls_aead_free(ctx);
    return r;
}

/* ---- IV-only setup (setup_crypto with key == NULL; fusion: lib/fusion.c:1188-1191) ---- */

/* the context ptls_aead_new_direct makes for key == NULL (lib/picotls.c:6458-6473): fusion stores the IV and
 * returns 0, leaving the vtable unset, so the caller may only release it with ref_ctx_free_raw */
void *ref_aead_new_iv_only(const ptls_aead_algorithm_t *algo, int is_enc, const void *iv)
{
    return ptls_aead_new_direct((ptls_aead_algorithm_t *)algo, is_enc, NULL, iv);
}

void ref_ctx_free_raw(void *ctx)
{
    free(ctx);
}

/* algo->setup_crypto(ctx, is_enc, NULL, iv) on a live context: IV-only re-setup */
int ref_aead_setup_iv_only(ptls_aead_context_t *ctx, int is_enc, const void *iv)
{
    return ctx->algo->setup_crypto(ctx, is_enc, NULL, iv);
}

/* lib/fusion.c: keyed context with iv, then an IV-only re-setup to iv2, then one seal */
size_t ref_seal_reiv(int bits, const void *key, const void *iv, const void *iv2, uint64_t seq, const void *aad, size_t aadlen,
                     const void *in, size_t inlen, void *out)
{
    ptls_aead_context_t *ctx = ptls_aead_new_direct(pick(bits), 1, key, iv);
    if (ref_aead_setup_iv_only(ctx, 1, iv2) != 0)
        return SIZE_MAX;
    size_t r = ptls_aead_encrypt(ctx, out, in, inlen, seq, aad, aadlen);
    ptls_aead_free(ctx);
    return r;
}

/* ---- t/ptlsbench.c bench_run_one (:88-173) over any AEAD object ----
 * The same loop: batches of up to 1000 ptls_aead_encrypt of one cache-hot zero input into 1000 distinct
 * outputs, AAD = uint64_t h[4] with h[0] = seq starting at 1, then the same records ptls_aead_decrypt-ed.
 * Contexts come from ptls_aead_new(aead, sha256, is_enc, 'z' x 64, NULL) as in bench_run_aead (:218-225).
 * Times are wall clock (CLOCK_MONOTONIC) and, like ptlsbench, process CPU time; both in microseconds. */
#define REF_BENCH_BATCH 1000
int ref_ptlsbench(const ptls_aead_algorithm_t *aead, size_t n, size_t l, double *wall_enc, double *wall_dec, double *cpu_enc,
                  double *cpu_dec)
{
    uint8_t secret[PTLS_MAX_SECRET_SIZE];
    memset(secret, 'z', sizeof(secret));
    ptls_aead_context_t *e = ptls_aead_new((ptls_aead_algorithm_t *)aead, &ptls_minicrypto_sha256, 1, secret, NULL);
    ptls_aead_context_t *d = ptls_aead_new((ptls_aead_algorithm_t *)aead, &ptls_minicrypto_sha256, 0, secret, NULL);
    uint8_t *v_in = calloc(1, l + 1), *v_dec = malloc(l + 1), *v_enc[REF_BENCH_BATCH];
    uint64_t h[4] = {0};
    int ret = 0;
    *wall_enc = *wall_dec = *cpu_enc = *cpu_dec = 0;
    for (size_t i = 0; i < REF_BENCH_BATCH; ++i)
        v_enc[i] = malloc(l + PTLS_MAX_DIGEST_SIZE);
    if (e == NULL || d == NULL) {
        ret = -1;
        goto Exit;
    }
    for (size_t k = 0; k < n;) {
        size_t e_len = 0, i_max = n - k > REF_BENCH_BATCH ? REF_BENCH_BATCH : n - k;
        uint64_t old_h = h[0];
        struct timespec c0, c1, c2;
        clock_gettime(CLOCK_PROCESS_CPUTIME_ID, &c0);
        double t0 = now();
        for (size_t i = 0; i < i_max; ++i) {
            h[0]++;
            e_len = ptls_aead_encrypt(e, v_enc[i], v_in, l, h[0], h, sizeof(h));
        }
        double t1 = now();
        clock_gettime(CLOCK_PROCESS_CPUTIME_ID, &c1);
        h[0] = old_h;
        for (size_t i = 0; i < i_max; ++i) {
            h[0]++;
            if (ptls_aead_decrypt(d, v_dec, v_enc[i], e_len, h[0], h, sizeof(h)) != l) {
                ret = -2;
                goto Exit;
            }
        }
        double t2 = now();
        clock_gettime(CLOCK_PROCESS_CPUTIME_ID, &c2);
        *wall_enc += (t1 - t0) * 1e6;
        *wall_dec += (t2 - t1) * 1e6;
        *cpu_enc += ((double)(c1.tv_sec - c0.tv_sec) * 1e9 + (double)(c1.tv_nsec - c0.tv_nsec)) * 1e-3;
        *cpu_dec += ((double)(c2.tv_sec - c1.tv_sec) * 1e9 + (double)(c2.tv_nsec - c1.tv_nsec)) * 1e-3;
        k += i_max;
    }
Exit:
    if (e != NULL)
        ptls_aead_free(e);
    if (d != NULL)
        ptls_aead_free(d);
    for (size_t i = 0; i < REF_BENCH_BATCH; ++i)
        free(v_enc[i]);
    free(v_in);
    free(v_dec);
    return ret;
}

/* ---- t/ptlsbench.c's loop on several threads at once, each with its own contexts (a server's worker threads) ----
 * Every thread makes its own encrypt and decrypt context with ptls_aead_new (bench_run_aead :218-225), then, behind a
 * barrier, runs `n` rounds of bench_run_one's body: ptls_aead_encrypt of the zero input into one of 16 outputs (AAD =
 * uint64_t h[4], h[0] = seq) and ptls_aead_decrypt of it, checking the length.  Returns calls (encrypt + decrypt) per
 * second over all threads, wall clock from the barrier to the last thread's end; -1 on a failed decrypt. */
struct mt_job {
    const ptls_aead_algorithm_t *aead;
    size_t n, l;
    pthread_barrier_t *bar;
    double t_end;
    int err;
};

static void *mt_worker(void *p)
{
    struct mt_job *j = p;
    uint8_t secret[PTLS_MAX_SECRET_SIZE];
    memset(secret, 'z', sizeof(secret));
    ptls_aead_context_t *e = ptls_aead_new((ptls_aead_algorithm_t *)j->aead, &ptls_minicrypto_sha256, 1, secret, NULL);
    ptls_aead_context_t *d = ptls_aead_new((ptls_aead_algorithm_t *)j->aead, &ptls_minicrypto_sha256, 0, secret, NULL);
    uint8_t *in = calloc(1, j->l + 1), *dec = malloc(j->l + 1), *enc = malloc(16 * (j->l + PTLS_MAX_DIGEST_SIZE));
    uint64_t h[4] = {0};
    pthread_barrier_wait(j->bar);
    j->err = e == NULL || d == NULL;
    for (size_t i = 0; i < j->n && !j->err; ++i) {
        uint8_t *o = enc + (i & 15) * (j->l + PTLS_MAX_DIGEST_SIZE);
        h[0] = i + 1;
        size_t el = ptls_aead_encrypt(e, o, in, j->l, h[0], h, sizeof(h));
        if (ptls_aead_decrypt(d, dec, o, el, h[0], h, sizeof(h)) != j->l)
            j->err = 1;
    }
    j->t_end = now();
    if (e != NULL)
        ptls_aead_free(e);
    if (d != NULL)
        ptls_aead_free(d);
    free(in);
    free(dec);
    free(enc);
    return NULL;
}

double ref_ptlsbench_mt(const ptls_aead_algorithm_t *aead, int threads, size_t n, size_t l)
{
    pthread_t th[256];
    struct mt_job jobs[256];
    pthread_barrier_t bar;
    if (threads < 1 || threads > 256)
        return -1;
    pthread_barrier_init(&bar, NULL, (unsigned)threads + 1);
    for (int t = 0; t < threads; ++t) {
        jobs[t] = (struct mt_job){aead, n, l, &bar, 0, 0};
        pthread_create(&th[t], NULL, mt_worker, &jobs[t]);
    }
    pthread_barrier_wait(&bar);
    double t0 = now(), t1 = t0;
    int err = 0;
    for (int t = 0; t < threads; ++t) {
        pthread_join(th[t], NULL);
        err |= jobs[t].err;
        if (jobs[t].t_end > t1)
            t1 = jobs[t].t_end;
    }
    pthread_barrier_destroy(&bar);
    return err ? -1 : 2.0 * (double)n * threads / (t1 - t0);
}

/* ---- context lifecycle (lib/picotls.c:6458-6479): `n` rounds of ptls_aead_new_direct, one seal, ptls_aead_free; the
 * microseconds of each new / seal / free go to the three arrays ---- */
int ref_aead_lifecycle(const ptls_aead_algorithm_t *aead, size_t n, size_t l, double *new_us, double *seal_us, double *free_us)
{
    uint8_t key[32], iv[12], *in = calloc(1, l + 1), *out = malloc(l + 16);
    memset(key, 0x42, sizeof(key));
    memset(iv, 0x24, sizeof(iv));
    int ret = 0;
    for (size_t i = 0; i < n; ++i) {
        key[0] = (uint8_t)i;
        double t0 = now();
        ptls_aead_context_t *c = ptls_aead_new_direct((ptls_aead_algorithm_t *)aead, 1, key, iv);
        double t1 = now();
        if (c == NULL) {
            ret = -1;
            break;
        }
        ptls_aead_encrypt(c, out, in, l, i, iv, sizeof(iv));
        double t2 = now();
        ptls_aead_free(c);
        double t3 = now();
        new_us[i] = (t1 - t0) * 1e6;
        seal_us[i] = (t2 - t1) * 1e6;
        free_us[i] = (t3 - t2) * 1e6;
    }
    free(in);
    free(out);
    return ret;
}

/* ---- CPU baseline: lib/fusion.c over a batch of distinct record buffers, 1..N pinned threads ---- */

struct bench_job {
    const ptls_aead_algorithm_t *aead;
    int bits, cpu, do_open;
    const uint8_t *key, *iv;
    uint8_t *in;     /* nrec * stride bytes */
    uint8_t *out;    /* nrec * stride bytes */
    size_t first, count, len, stride, aadlen;
    const uint8_t *aad; /* nrec * aadlen */
    pthread_barrier_t *bar;
    int passes;
    double secs;
};

static void *bench_worker(void *p)
{
    struct bench_job *j = p;
    if (j->cpu >= 0) {
        cpu_set_t s;
        CPU_ZERO(&s);
        CPU_SET(j->cpu, &s);
        pthread_setaffinity_np(pthread_self(), sizeof(s), &s);
    }
    /* one ptls_aead_context_t per thread per key */
    ptls_aead_context_t *ctx = ptls_aead_new_direct((ptls_aead_algorithm_t *)j->aead, !j->do_open, j->key, j->iv);
    pthread_barrier_wait(j->bar);
    double t0 = now();
    for (int pass = 0; pass < j->passes; ++pass) {
        for (size_t i = j->first; i < j->first + j->count; ++i) {
            const uint8_t *aad = j->aad + i * j->aadlen;
            if (j->do_open)
                (void)ptls_aead_decrypt(ctx, j->out + i * j->stride, j->in + i * j->stride, j->len + 16, i, aad, j->aadlen);
            else
                ptls_aead_encrypt(ctx, j->out + i * j->stride, j->in + i * j->stride, j->len, i, aad, j->aadlen);
        }
    }
    j->secs = now() - t0;
    ptls_aead_free(ctx);
    return NULL;
}

/* Seals (do_open = 0) or opens (do_open = 1) records i = 0..nrec-1 held at in + i*stride, writing to
 * out + i*stride, `passes` times over; record i uses seq = i and aad + i*aadlen.  Returns the wall time of
 * the slowest thread (all threads start behind a barrier).  cpus: cpu ids to pin to (NULL = no pinning). */
double ref_bench_algo(int nt, int bits, int do_open, const void *key, const void *iv, void *in, void *out, size_t nrec, size_t len,
                      size_t stride, const void *aad, size_t aadlen, int threads, const int *cpus, int passes);

double ref_bench(int bits, int do_open, const void *key, const void *iv, void *in, void *out, size_t nrec, size_t len,
                 size_t stride, const void *aad, size_t aadlen, int threads, const int *cpus, int passes)
{
    return ref_bench_algo(0, bits, do_open, key, iv, in, out, nrec, len, stride, aad, aadlen, threads, cpus, passes);
}

/* nt = 1: the reference's non-temporal engine, ptls_non_temporal_aes{128,256}gcm (lib/fusion.c:2109-2179): encrypt through
 * non_temporal_encrypt_v256 (VAES / VPCLMULQDQ, 256-bit lanes) when ptls_fusion_can_aesni256, decrypt through
 * non_temporal_decrypt128; the same bytes as ptls_fusion_aes*gcm.  ptls_fusion_is_supported_by_cpu() is what sets
 * ptls_fusion_can_aesni256 (:2219-2249), so it runs first. */
double ref_bench_algo(int nt, int bits, int do_open, const void *key, const void *iv, void *in, void *out, size_t nrec, size_t len,
                      size_t stride, const void *aad, size_t aadlen, int threads, const int *cpus, int passes)
{
    (void)ptls_fusion_is_supported_by_cpu();
    const ptls_aead_algorithm_t *aead =
        nt ? (bits == 256 ? &ptls_non_temporal_aes256gcm : &ptls_non_temporal_aes128gcm) : pick(bits);
    pthread_t th[512];
    struct bench_job jobs[512];
    pthread_barrier_t bar;
    if (threads < 1)
        threads = 1;
    if (threads > 512)
        threads = 512;
    pthread_barrier_init(&bar, NULL, (unsigned)threads);
    for (int t = 0; t < threads; ++t) {
        size_t a = nrec * (size_t)t / (size_t)threads, b = nrec * (size_t)(t + 1) / (size_t)threads;
        jobs[t] = (struct bench_job){aead, bits, cpus != NULL ? cpus[t] : -1, do_open, key, iv, in, out, a, b - a, len, stride, aadlen,
                                     aad, &bar, passes < 1 ? 1 : passes, 0};
        pthread_create(&th[t], NULL, bench_worker, &jobs[t]);
    }
    double mx = 0;
    for (int t = 0; t < threads; ++t) {
        pthread_join(th[t], NULL);
        if (jobs[t].secs > mx)
            mx = jobs[t].secs;
    }
    pthread_barrier_destroy(&bar);
    return mx;
}

/* ---------------------------------------------------------------------------------------------- *
 * TLS 1.3 record layer of the reference: a post-handshake ptls_t  *
 * made by ptls_import (lib/picotls.c:5334-5432) from traffic secrets, then ptls_send /            *
 * ptls_receive (:6121-6145, :6061-6097).  The AEAD is minicrypto's, or any ptls_aead_algorithm_t  *
 * the caller passes (the HIP engine's, for the drop-in test); the hash is minicrypto's SHA-256/384 *
 * (lib/cifra/aes128.c, aes256.c), compiled unmodified.                                            *
 * ---------------------------------------------------------------------------------------------- */

struct ref_tls13 {
    ptls_context_t ctx;
    struct st_ptls_cipher_suite_t suite; /* ptls_cipher_suite_t is the const-qualified typedef */
    ptls_cipher_suite_t *suites[2];
    ptls_t *tls;
};

static void ref_random_bytes(void *buf, size_t len)
{
    memset(buf, 0x5a, len); /* client_random only; irrelevant to the record layer */
}

static void put16(uint8_t **p, uint16_t v)
{
    (*p)[0] = (uint8_t)(v >> 8);
    (*p)[1] = (uint8_t)v;
    *p += 2;
}

static void put64(uint8_t **p, uint64_t v)
{
    for (int i = 0; i < 8; ++i)
        (*p)[i] = (uint8_t)(v >> (56 - 8 * i));
    *p += 8;
}

/* bits 128 -> TLS_AES_128_GCM_SHA256, 256 -> TLS_AES_256_GCM_SHA384.  aead NULL -> minicrypto's AES-GCM
 * (lib/cifra/aes{128,256}.c): fusion's own do_encrypt_v is an assert stub (lib/fusion.c:1145-1149), so
 * ptls_send cannot run on it -- the gap SURVEY.md §8(f) rank 1 names. */
void *ref_tls13_import(int bits, const void *aead, int is_server, const void *enc_secret, uint64_t enc_seq, const void *dec_secret,
                       uint64_t dec_seq)
{
    struct ref_tls13 *r = calloc(1, sizeof(*r));
    ptls_hash_algorithm_t *hash = bits == 256 ? &ptls_minicrypto_sha384 : &ptls_minicrypto_sha256;
    r->suite.id = bits == 256 ? PTLS_CIPHER_SUITE_AES_256_GCM_SHA384 : PTLS_CIPHER_SUITE_AES_128_GCM_SHA256;
    r->suite.aead = aead != NULL ? (ptls_aead_algorithm_t *)aead
                                 : (bits == 256 ? &ptls_minicrypto_aes256gcm : &ptls_minicrypto_aes128gcm);
    r->suite.hash = hash;
    r->suite.name = "ref";
    r->suites[0] = &r->suite;
    r->ctx.random_bytes = ref_random_bytes;
    r->ctx.get_time = &ptls_get_time;
    r->ctx.cipher_suites = r->suites;
    /* export_tls_params layout (lib/picotls.c:5171-5191) with the TLS 1.3 block of ptls_export (:5265-5272) */
    uint8_t params[512], *p = params + 2;
    const size_t ds = hash->digest_size;
    *p++ = (uint8_t)is_server;
    *p++ = 0; /* session_reused */
    put16(&p, PTLS_PROTOCOL_VERSION_TLS13);
    put16(&p, r->suite.id);
    memset(p, 0x11, PTLS_HELLO_RANDOM_SIZE);
    p += PTLS_HELLO_RANDOM_SIZE;
    put16(&p, 0); /* server name */
    put16(&p, 0); /* negotiated protocol */
    put16(&p, (uint16_t)(2 * (ds + 8)));
    memcpy(p, enc_secret, ds);
    p += ds;
    put64(&p, enc_seq);
    memcpy(p, dec_secret, ds);
    p += ds;
    put64(&p, dec_seq);
    put16(&p, 0); /* extensions */
    uint8_t *q = params;
    put16(&q, (uint16_t)(p - params - 2));
    if (ptls_import(&r->ctx, &r->tls, ptls_iovec_init(params, p - params)) != 0) {
        free(r);
        return NULL;
    }
    return r;
}

/* A post-handshake TLS 1.2 connection of the reference: ptls_build_tls12_export_params derives the key block
 * from a master secret and the hello randoms with the reference's PRF (lib/picotls.c:5217-5255), ptls_import
 * instantiates the AEADs through import_tls12_traffic_protection (:5291-5312), and ptls_send / ptls_receive
 * then run the TLS 1.2 record layer (buffer_push_encrypted_records :747-794 with build_tls12_aad :730-739,
 * handle_input_tls12 :5927-5990).  aead NULL -> fusion's ptls_non_temporal_aes{128,256}gcm, the objects
 * whose tls12 fields are {4, 8} (lib/fusion.c:2154-2179). */
void *ref_tls12_import(int bits, const void *aead, int is_server, const void *master_secret, const void *hello_randoms,
                       uint64_t next_send_record_iv)
{
    struct ref_tls13 *r = calloc(1, sizeof(*r));
    r->suite.id = bits == 256 ? PTLS_CIPHER_SUITE_ECDHE_RSA_WITH_AES_256_GCM_SHA384 : PTLS_CIPHER_SUITE_ECDHE_RSA_WITH_AES_128_GCM_SHA256;
    r->suite.aead = aead != NULL ? (ptls_aead_algorithm_t *)aead : (bits == 256 ? &ptls_non_temporal_aes256gcm : &ptls_non_temporal_aes128gcm);
    r->suite.hash = bits == 256 ? &ptls_minicrypto_sha384 : &ptls_minicrypto_sha256;
    r->suite.name = "ref12";
    r->suites[0] = &r->suite;
    r->ctx.random_bytes = ref_random_bytes;
    r->ctx.get_time = &ptls_get_time;
    r->ctx.tls12_cipher_suites = r->suites;
    ptls_buffer_t buf;
    ptls_buffer_init(&buf, "", 0);
    int ok = ptls_build_tls12_export_params(&r->ctx, &buf, is_server, 0, &r->suite, master_secret, hello_randoms, next_send_record_iv,
                                            NULL, ptls_iovec_init(NULL, 0)) == 0 &&
             ptls_import(&r->ctx, &r->tls, ptls_iovec_init(buf.base, buf.off)) == 0;
    ptls_buffer_dispose(&buf);
    if (!ok) {
        free(r);
        return NULL;
    }
    return r;
}

void ref_tls13_free(void *h)
{
    struct ref_tls13 *r = h;
    ptls_free(r->tls);
    free(r);
}

/* ptls_send of `len` application bytes; returns the wire bytes copied to out (or -1) */
long ref_tls13_send(void *h, const void *in, size_t len, void *out, size_t cap)
{
    struct ref_tls13 *r = h;
    ptls_buffer_t buf;
    ptls_buffer_init(&buf, "", 0);
    long n = -1;
    if (ptls_send(r->tls, &buf, in, len) == 0 && buf.off <= cap) {
        memcpy(out, buf.base, buf.off);
        n = (long)buf.off;
    }
    ptls_buffer_dispose(&buf);
    return n;
}

/* ptls_receive: returns picotls's error code; *consumed = wire bytes used, *outlen = plaintext bytes */
int ref_tls13_receive(void *h, const void *in, size_t inlen, size_t *consumed, void *out, size_t cap, size_t *outlen)
{
    struct ref_tls13 *r = h;
    ptls_buffer_t buf;
    ptls_buffer_init(&buf, "", 0);
    size_t n = inlen;
    int ret = ptls_receive(r->tls, &buf, in, &n);
    *consumed = n;
    *outlen = buf.off;
    if (buf.off <= cap)
        memcpy(out, buf.base, buf.off);
    ptls_buffer_dispose(&buf);
    return ret;
}

/* the record-protection key and IV picotls derives from a traffic secret (ptls_aead_new ->
 * get_traffic_keys, lib/picotls.c:6434-6456): HKDF-Expand-Label(secret, "key" / "iv", "", len) */
int ref_hkdf_expand_label(int bits, void *out, size_t outlen, const void *secret, const char *label, const void *hashvalue,
                          size_t hashlen)
{
    ptls_hash_algorithm_t *hash = bits == 256 ? &ptls_minicrypto_sha384 : &ptls_minicrypto_sha256;
    return ptls_hkdf_expand_label(hash, out, outlen, ptls_iovec_init(secret, hash->digest_size), label,
                                  ptls_iovec_init(hashvalue, hashlen), NULL);
}
