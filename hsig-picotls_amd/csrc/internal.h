/*
 * internal.h -- layouts shared by the host units (host.h) and the gfx950 kernels (aesgcm_kernels.hip).
 *
 * HBM layout:
 *   key slots    KeySlot[nslots]             512 B each: round keys, static IV, H powers
 *   GHASH basis  uint4[nslots][BASIS_VECS]   18 KiB per slot: P * x^e for P in {H, H^2, ..., H^128}, then H^1..H^128
 *   records      ptls_hip_record_t[n]        48 B descriptors (caller's order)
 *   chunks       Chunk[nchunks]              runs of <= CHUNK_RECS records sharing one key slot
 *   payloads     caller's buffers, untouched layout (in / aad / out)
 */
#ifndef PTLS_HIP_INTERNAL_H
#define PTLS_HIP_INTERNAL_H

#include <stdint.h>
#include "ptls_hip.h"

/* The product build (Makefile PROD) refuses the switches that make the kernels compute something else (the TEST-ONLY
 * dealing mutants) or carry diagnostics (key-switch stamps): such objects are built only into mutants/ and diag/. */
#if defined(PTLS_HIP_PRODUCT)
#if (defined(DEAL_MUTANT) && DEAL_MUTANT) || (defined(KS_STAMPS) && KS_STAMPS)
#error "libptls_hip.so is built with a test-mutant or diagnostic switch set"
#endif
#endif

namespace ptls_hip {

constexpr int NPOW = 8; /* H^1 .. H^16 (batch kernel main tables), H^32 (batch kernel main table at G = 32), H^64 (sparse
                          kernel), H^128 (a single record on two or four waves, stride 128) */
/* GHASH basis slot: NPOW x 128 vectors P * x^e, then H^1 .. H^128 (the lane combinations' per-lane final powers H^(q+1);
 * a two-wave single record of up to 128 GHASH elements multiplies element i by H^(N - i)) */
constexpr int LANE_POWS = 128;
constexpr int BASIS_VECS = NPOW * 128 + LANE_POWS; /* uint4 per key slot: 18 KiB */
constexpr int MAX_LANES = 32;    /* lanes per record (G) of the batch kernel: 1, 2, 4, 8, 16, 32 */
constexpr int SPARSE_LANES = 64; /* "lanes" value of the wave-per-record kernel (sparse_kernel.hip) */
/* the planner picks that kernel when a batch's key runs hold fewer records than this on average */
constexpr int SPARSE_MAX_PER_RUN = 20; /* configs[3]'s lengths, seal GiB/s, sparse kernel / 32 lanes (round 3): 16 records
                                           per key 533 / 498, 24 per key 533 / 680 (tools/calls_r03/r03_call24.sh) */
/* one workgroup per CU (LDS-limited); 768 threads (3 waves per SIMD, 168 VGPRs) by default, 512 selectable
 * per batch (planner.cpp plan_wg).  WG_MAX bounds the chunk size the planner cuts key runs into. */
constexpr int WG_MAX = 1024;

struct KeySlot {
    uint32_t rk[60];      /* AES round keys, raw byte order as little-endian words (11 or 15 used) */
    uint32_t rounds;      /* 10 or 14 */
    uint32_t iv[3];       /* static IV (12 bytes, raw) */
    uint32_t hpow[NPOW][4]; /* H^(2^t), raw GCM byte order */
    uint32_t pad[(512 - 240 - 4 - 12 - 16 * NPOW) / 4];
};
static_assert(sizeof(KeySlot) == 512, "KeySlot must stay 512 bytes");

/* the second compiled workgroup size (the first is 512) */
constexpr int WG_ALT = 768;

struct Chunk {
    uint32_t first; /* position of the chunk's first record in the order array */
    uint32_t count; /* records in the chunk, all with the same key slot */
    uint32_t key;   /* key slot */
    uint32_t flags; /* bit0: every record of the chunk is 16-byte aligned (in/out/aad offsets) */
};

struct KernelArgs {
    const ptls_hip_record_t *recs;
    const ptls_hip_record_t *recs_ord; /* the same descriptors in chunk order: one dependent load per task */
    const uint32_t *order;  /* chunk positions -> record index (records of a chunk sorted by length) */
    const Chunk *chunks;
    uint32_t nchunks;
    uint32_t pad0;
    const uint8_t *in;
    const uint8_t *aad;
    uint8_t *out;
    uint64_t *result;       /* open only */
    const KeySlot *slots;
    const uint32_t *basis;  /* uint4 [slot][NPOW][128] */
    const uint32_t *t0;     /* AES T0 table, 256 words */
    /* seal only, optional: QUIC header-protection masks (ptls_hip_aesgcm_seal_batch_supp) */
    const ptls_hip_supp_t *supp; /* indexed like recs; nullptr = none */
    const KeySlot *hp_slots;
    uint32_t hp_nslots; /* supp[i].hp_key >= hp_nslots: that record's mask is left untouched */
    uint8_t *mask;
    /* sparse kernel only: with recs_ord == nullptr it runs this one record, passed by value in the kernel arguments
     * (the plugin's single-record calls: no dependent reads of host-staged descriptors) */
    ptls_hip_record_t one;
    /* optional completion word (the plugin's pinned staging): the wave that ran the by-value record stores done_seq
     * there, system scope, after all its output, tag, result and mask stores (the host spins on it instead of a
     * stream synchronize) */
    uint32_t *done;
    uint32_t done_seq;
    /* optional diagnostic clock stamps, 4 x uint64 per workgroup (ptls_hip_batch_set_clock); nullptr = none */
    uint64_t *clk;
    size_t clk_bytes; /* its size (KS_STAMPS diagnostic builds also write 16 words per wave after the workgroups' stamps) */
    /* batch kernel: this launch's chunk-queue words {next chunk - grid, workgroups done}, zero at launch and left zero by
     * the kernel (engine.cpp queue_slot); nullptr = the static grid stride */
    uint32_t *queue;
};
/* chunk-queue slots per engine: launches take them round robin, so two launches in flight never share one */
constexpr uint32_t QUEUE_SLOTS = 4096;

/* The plugin worker (sparse_kernel.hip plugin_worker_kernel, plugin_worker.cpp): a resident kernel whose workgroups each serve
 * the plugin's single-record calls from their own mailbox in fine-grained pinned host memory instead of one kernel launch
 * per call.  The host writes the request, then (release) seq; the workgroup serves it, stores the call's completion word
 * (as a launched call's kernel does), then `served`. */
enum : uint32_t { WREQ_OPEN = 1, WREQ_AES256 = 2, WREQ_INLINE = 8, WREQ_IV = 16, WREQ_ECB = 32 };
/* WREQ_ECB: one AES block (ptls_hip_aes*ctr's do_init, the fusion-style ECB API) with the request's key slot: input block at
 * data[0..16), output at out[0..16) */
/* WREQ_IV: the nonce's static IV is the request's iv[] (the context's current IV), not the key slot's: an IV change
 * (ptls_aead_set_iv / xor_iv) stays on the host. */
/* WREQ_INLINE: the record sits in the mailbox's data area (AAD padded to 16 bytes, then the input: element i of the GHASH
 * input at data + 16 i), read in the same PCIe round trip as the request.  Records that do not fit stay in the caller's
 * pinned staging. */
constexpr int WORKER_DATA = 16384 + 512;
struct WorkerReq {
    ptls_hip_record_t rec;    /* by value: offsets into in / aad / out */
    const uint8_t *in, *aad;  /* device addresses of the context's pinned staging */
    uint8_t *out;
    uint64_t *result;         /* open: the verification result */
    const KeySlot *slots;     /* the context's key slot (and its basis) */
    const uint32_t *basis;
    const ptls_hip_supp_t *supp; /* optional header protection */
    const KeySlot *hp_slots;
    uint8_t *mask;
    uint32_t *done;           /* the call's completion word */
    uint32_t done_seq;
    uint32_t flags;           /* WREQ_* */
    uint32_t iv[3];           /* WREQ_IV: the static IV (raw bytes as little-endian words, KeySlot::iv's layout) */
    uint32_t pad[11];
};
static_assert(sizeof(WorkerReq) == 192, "WorkerReq: 192 bytes");
struct WorkerSlot {
    uint32_t seq;    /* host -> worker: the request number, written after the request */
    uint32_t quit;   /* host -> worker: leave */
    uint32_t pad0[30];
    uint32_t served;  /* worker -> host: the last request served */
    uint32_t exited;  /* worker -> host: the epoch of the worker wave that left */
    uint32_t started; /* worker -> host: the epoch of the worker wave that started (diagnostics) */
    uint32_t seen;    /* worker -> host: the last request number it read (diagnostics) */
    uint32_t pad1[2];
    uint64_t stamps[13]; /* worker -> host: WORKER_STAMPS builds' phase stamps of the last request (100 MHz counter) */
    WorkerReq req;
    uint8_t data[WORKER_DATA]; /* WREQ_INLINE records */
    uint8_t out[WORKER_DATA];  /* the output of a request whose record fits (ciphertext + tag, or plaintext) */
    uint8_t aux[256];          /* the request's result @0 (8 B), header-protection descriptor @32 (ptls_hip_supp_t) and mask
                                  @64 (16 B), completion word @128 */
};
static_assert(sizeof(WorkerSlot) == 448 + 2 * WORKER_DATA + 256, "WorkerSlot: seq / quit, served / exited, request on separate 128-B lines");
constexpr uint32_t WAUX_RESULT = 0, WAUX_SUPP = 32, WAUX_MASK = 64, WAUX_DONE = 128;
static_assert(__builtin_offsetof(WorkerSlot, quit) == 4, "the worker polls {seq, quit} as one 8-byte word");

/* one run of bytes the copy transport puts back between records (pipeline.cpp): dst = offset in the slice's output
 * staging, src = offset in the packed gap buffer */
struct GapPiece {
    uint64_t dst;
    uint32_t src;
    uint32_t len;
};

/* host-side launchers, defined next to the kernels (aesgcm_kernels.hip, batch_g*.hip) */
int launch_plugin_worker(WorkerSlot *mb, unsigned nmb, uint32_t epoch, const uint32_t *t0, uint64_t idle_ticks, uint64_t life_ticks,
                         uint64_t *activity, void *stream);
int launch_batch_g1(int rounds, bool open, int wg, unsigned grid, void *stream, const KernelArgs &a, bool aligned);
int launch_batch_g2(int rounds, bool open, int wg, unsigned grid, void *stream, const KernelArgs &a, bool aligned);
int launch_batch_g4(int rounds, bool open, int wg, unsigned grid, void *stream, const KernelArgs &a, bool aligned);
int launch_batch_g8(int rounds, bool open, int wg, unsigned grid, void *stream, const KernelArgs &a, bool aligned);
int launch_batch_g16(int rounds, bool open, int wg, unsigned grid, void *stream, const KernelArgs &a, bool aligned);
int launch_batch_g32(int rounds, bool open, int wg, unsigned grid, void *stream, const KernelArgs &a, bool aligned);
int launch_batch_sparse(int rounds, bool open, unsigned grid, void *stream, const KernelArgs &a, bool aligned);
int launch_batch(int lanes, int rounds, bool open, int wg, unsigned grid, void *stream, const KernelArgs &a, bool aligned);
int launch_keysetup(KeySlot *slots, uint32_t *basis, const uint8_t *keys, const uint8_t *ivs, uint32_t first, uint32_t count,
                    int key_size, const uint32_t *t0, void *stream);
int launch_aesecb(int rounds, const ptls_hip_supp_t *supp, uint32_t n, const uint8_t *src, uint8_t *mask, const KeySlot *hp_slots,
                  uint32_t hp_nslots, const uint32_t *t0, unsigned grid, void *stream,
                  uint32_t *done = nullptr, uint32_t done_seq = 0);
int launch_aesecb_one(int rounds, const uint8_t *blk, const KeySlot *slot, const uint32_t *t0, uint8_t *out, uint32_t *done,
                      uint32_t done_seq, void *stream);
int launch_tls13_headers(const ptls_hip_record_t *recs, uint32_t n, uint8_t *hdr, unsigned grid, void *stream);
int launch_tls13_inner(const ptls_hip_record_t *recs, uint32_t n, const uint8_t *out, uint64_t *result, unsigned grid, void *stream);
int launch_derive_traffic_keys(const uint8_t *secrets_in, uint8_t *secrets_out, uint32_t count, int hash_size, int key_size,
                               int update, uint8_t *keys, uint8_t *ivs, void *stream);
int launch_fill(const ptls_hip_record_t *recs, uint32_t n, uint8_t *buf, uint64_t seed, uint64_t index_base,
                const uint64_t *index, unsigned grid, void *stream);
int launch_copy16(void *dst, const void *src, size_t n16, void *stream);
int launch_gap_scatter(const GapPiece *pieces, uint32_t n, const uint8_t *src, uint8_t *dst, void *stream);

} // namespace ptls_hip

#endif
