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

/* ---- CPU baseline: lib/fusion.c over a batch of distinct record buffers, 1..N pinned threads ---- */

struct bench_job {
    int bits, cpu, do_open;
    const uint8_t *key, *iv;
    uint8_t *in;     /* nrec * stride bytes */
    uint8_t *out;    /* nrec * stride bytes */
    size_t first, count, len, stride, aadlen;
    const uint8_t *aad; /* nrec * aadlen */
    pthread_barrier_t *bar;
    double secs;
};

static double now(void)
{
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

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
    ptls_aead_context_t *ctx = ptls_aead_new_direct(pick(j->bits), !j->do_open, j->key, j->iv);
    pthread_barrier_wait(j->bar);
    double t0 = now();
    for (size_t i = j->first; i < j->first + j->count; ++i) {
        const uint8_t *aad = j->aad + i * j->aadlen;
        if (j->do_open)
            (void)ptls_aead_decrypt(ctx, j->out + i * j->stride, j->in + i * j->stride, j->len + 16, i, aad, j->aadlen);
        else
            ptls_aead_encrypt(ctx, j->out + i * j->stride, j->in + i * j->stride, j->len, i, aad, j->aadlen);
    }
    j->secs = now() - t0;
    ptls_aead_free(ctx);
    return NULL;
}

/* Seals (do_open = 0) or opens (do_open = 1) records i = 0..nrec-1 held at in + i*stride, writing to
 * out + i*stride; record i uses seq = i and aad + i*aadlen.  Returns the wall time of the slowest
 * thread (all threads start behind a barrier).  cpus: list of cpu ids to pin to (NULL = no pinning). */
double ref_bench(int bits, int do_open, const void *key, const void *iv, void *in, void *out, size_t nrec, size_t len,
                 size_t stride, const void *aad, size_t aadlen, int threads, const int *cpus)
{
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
        jobs[t] = (struct bench_job){bits, cpus != NULL ? cpus[t] : -1, do_open, key, iv, in, out, a, b - a, len, stride, aadlen,
                                     aad, &bar, 0};
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
