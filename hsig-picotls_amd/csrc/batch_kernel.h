/*
 * batch_kernel.h -- the gfx950 (MI355X) AES-GCM batch kernel template and its device helpers
 * (included by batch_g*.hip, one instantiation set per lanes-per-record G, and by aesgcm_kernels.hip).
 *
 * What is computed (bit-exact with picotls lib/fusion.c):
 *   seal  ptls_fusion_aesgcm_encrypt  lib/fusion.c:400-658
 *   open  ptls_fusion_aesgcm_decrypt  lib/fusion.c:660-844
 *   nonce calc_counter                lib/fusion.c:1126-1133 (== ptls_aead__build_iv lib/picotls.c:6492)
 *   setup new_aesgcm + setup_one_ghash_entry  lib/fusion.c:984-1010, :939-966
 * How: no AES / carry-less instructions exist on CDNA4 and north_star rules out MFMA,
 * so both halves of GCM are table work in LDS:
 *   AES   : T-table rounds.  One 256-entry table T0 (and T2 = rotl16(T0)) replicated 32x so that
 *           lane l always hits bank l%32 -> ds_read_b32 is conflict-free for any data.  The LDS
 *           address (byte << 8 | lane slot) is produced by ONE v_perm_b32 per lookup.
 *   GHASH : multiplication by a fixed power P of H is GF(2)-linear, so X*P = XOR over the 16 bytes
 *           of X of T8[p][X_p] with T8[p][v] = (v at byte p) * P.  The table is laid out row v, slot
 *           p; lane l looks up byte p = (k + l) % 16 at step k, so the 16 lanes of every ds_read_b128
 *           lane group touch 16 distinct slots -> conflict-free; X is pre-rotated per lane so the
 *           byte for step k sits at a fixed position and the address is again one v_perm_b32.
 *   Record parallelism: G lanes share one record (Horner with stride G inside a lane, then every lane multiplies its
 *           sum by its own power H^(q+1) from per-key 4-bit window tables in LDS and the record's lanes XOR their
 *           products; G = 1 multiplies by H with a nibble table), 64/G records per wave task, 12 waves per workgroup drawing
 *           tasks from an LDS counter, workgroups persist over key-homogeneous chunks taken from a device-wide queue.
 * Rejected variants (bit-sliced waves, split records, the shuffle-tree combination, probes) are measured in EXPERIMENTS.md
 * and are not in this source; the only build switches left are the TEST-ONLY dealing mutants and a diagnostic stamp.
 */
#ifndef PTLS_HIP_BATCH_KERNEL_H
#define PTLS_HIP_BATCH_KERNEL_H

#include <hip/hip_runtime.h>
#include <type_traits>
#include "internal.h"

namespace ptls_hip {

/* ---------------- LDS map (bytes) ---------------- */
constexpr uint32_t LDS_GMAIN = 0;            /* 64 KiB: row v (256 B) = 16 positions x 16 B, P = H^G       */
constexpr uint32_t LDS_AES = 65536;          /* 64 KiB: row v = [T0 x32 lane slots | T2 x32 lane slots]  */
constexpr uint32_t LDS_GTREE = 131072;       /* the lane combination's tables: G = 1 the nibble table of H ([p(32)][v(16)],
                                                8 KiB), G >= 2 the window tables of H^1 .. H^G (build_ghash_tables) */
constexpr uint32_t LDS_TREE_STRIDE = 8192;
constexpr int TREE_TABLES = 3;
__host__ __device__ constexpr uint32_t lds_bytes(int log2g)
{
    return (void)log2g, LDS_GTREE + TREE_TABLES * LDS_TREE_STRIDE;
}

/* measured constants (EXPERIMENTS.md) */
constexpr int SETPRIO = 1;     /* wave priority while a wave issues a segment's lookups: c2 +6 % */
constexpr int PURE_BLOCKS = 2; /* data blocks per lane per iteration of the branch-free loop */
#ifndef DEAL_MUTANT
#define DEAL_MUTANT 0 /* TEST-ONLY broken builds (Makefile `mutants`, tests/test_gpu_dealing.py, tests/test_gpu_c4_keyruns.py):
                         1 = the task a wave drew past one chunk is dropped at the next chunk of the key run, 2 = cbase is not
                         advanced, 3 = the workgroup's task counter is not reset at a key switch (only at its first key) */
#endif
#ifndef KS_STAMPS
#define KS_STAMPS 0 /* DIAGNOSTIC builds only (tools/keyswitch_stamps.py): every wave sums the shader cycles it spends at key
                       switches (first barrier, table build, second barrier) and in total, and within its tasks (drawing
                       the task, descriptors + AAD elements + counter-mode constants, the stretch, the generic rest, the
                       combination + tag), into clk after the 4 x grid workgroup stamps: [workgroup][wave][total,
                       barrier 1, build, barrier 2, switches, draw, setup, stretch, rest, combine] */
#endif
/* the chunk sequence a workgroup's waves walk: a ring in LDS of {sequence number, chunk} entries */
constexpr int QRING = 32;
constexpr uint32_t Q_END = 0xffffffffu;

struct V4 {
    uint32_t w0, w1, w2, w3;
};

__device__ __forceinline__ V4 v4xor(V4 a, V4 b)
{
    return V4{a.w0 ^ b.w0, a.w1 ^ b.w1, a.w2 ^ b.w2, a.w3 ^ b.w3};
}

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c)
{
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96); /* v_bitop3_b32: a ^ b ^ c in one VALU op */
}

__device__ __forceinline__ V4 v4xor3(V4 a, V4 b, V4 c)
{
    return V4{xor3(a.w0, b.w0, c.w0), xor3(a.w1, b.w1, c.w1), xor3(a.w2, b.w2, c.w2), xor3(a.w3, b.w3, c.w3)};
}

__device__ __forceinline__ uint32_t bswap32(uint32_t x)
{
    return __builtin_bswap32(x);
}

__device__ __forceinline__ uint32_t lds32(const uint8_t *lds, uint32_t addr)
{
    return *reinterpret_cast<const uint32_t *>(lds + addr);
}

__device__ __forceinline__ V4 lds128(const uint8_t *lds, uint32_t addr)
{
    const uint4 v = *reinterpret_cast<const uint4 *>(lds + addr);
    return V4{v.x, v.y, v.z, v.w};
}

__device__ __forceinline__ void lds128_store(uint8_t *lds, uint32_t addr, V4 v)
{
    *reinterpret_cast<uint4 *>(lds + addr) = make_uint4(v.w0, v.w1, v.w2, v.w3);
}

/* ======================================================================================= *
 *  AES (FIPS-197) with replicated T-tables in LDS                                          *
 * ======================================================================================= */

/* LDS byte address of T0[byte k of x] for this lane: LDS_AES | (x.byte[k] << 8) | lane_slot, from ONE
 * v_perm_b32: byte0 <- lb.byte0 (selector 0), byte1 <- x.byte[k] (selector 4+k), byte2 <- lb.byte2 (= 1,
 * i.e. the 64 KiB table base, selector 2), byte3 <- 0.  lb = (lane & 31) * 4 | LDS_AES. */
template <int K>
__device__ __forceinline__ uint32_t aes_addr(uint32_t x, uint32_t lb)
{
    static_assert(LDS_AES == 65536, "the table base is injected as byte 2 of the address");
    return __builtin_amdgcn_perm(x, lb, 0x0c020000u | ((4u + K) << 8));
}

__device__ __forceinline__ uint32_t rotl8(uint32_t x)
{
    return __builtin_amdgcn_alignbit(x, x, 24);
}

/* one output column of a full round:
 * T0[x0.b0] ^ T1[x1.b1] ^ T2[x2.b2] ^ T3[x3.b3] ^ k  with T1 = rotl8(T0), T3 = rotl8(T2) */
__device__ __forceinline__ uint32_t aes_col(const uint8_t *lds, uint32_t lb, uint32_t x0, uint32_t x1, uint32_t x2, uint32_t x3,
                                            uint32_t k)
{
    const uint32_t a0 = lds32(lds, aes_addr<0>(x0, lb));
    const uint32_t a1 = lds32(lds, aes_addr<1>(x1, lb));
    const uint32_t a2 = lds32(lds, 128 + aes_addr<2>(x2, lb));
    const uint32_t a3 = lds32(lds, 128 + aes_addr<3>(x3, lb));
    return xor3(a0, a2, rotl8(a1 ^ a3)) ^ k;
}

/* final round column: S-box bytes picked out of T2[.].b0, T0[.].b1, T0[.].b2, T2[.].b3 */
__device__ __forceinline__ uint32_t aes_col_last(const uint8_t *lds, uint32_t lb, uint32_t x0, uint32_t x1, uint32_t x2,
                                                 uint32_t x3, uint32_t k)
{
    const uint32_t u0 = lds32(lds, 128 + aes_addr<0>(x0, lb));
    const uint32_t u1 = lds32(lds, aes_addr<1>(x1, lb));
    const uint32_t u2 = lds32(lds, aes_addr<2>(x2, lb));
    const uint32_t u3 = lds32(lds, 128 + aes_addr<3>(x3, lb));
    const uint32_t lo = __builtin_amdgcn_perm(u1, u0, 0x0c0c0500u); /* u0.b0 -> b0, u1.b1 -> b1 */
    const uint32_t hi = __builtin_amdgcn_perm(u3, u2, 0x07020c0cu); /* u2.b2 -> b2, u3.b3 -> b3 */
    return xor3(lo, hi, k); /* lo and hi occupy disjoint bytes: lo ^ hi == lo | hi */
}

template <int ROUNDS>
__device__ __forceinline__ V4 aes_encrypt(const uint8_t *lds, uint32_t lb, const uint32_t *__restrict__ rk, V4 s)
{
    s.w0 ^= rk[0];
    s.w1 ^= rk[1];
    s.w2 ^= rk[2];
    s.w3 ^= rk[3];
#pragma unroll
    for (int r = 1; r < ROUNDS; ++r) {
        const uint32_t t0 = aes_col(lds, lb, s.w0, s.w1, s.w2, s.w3, rk[4 * r + 0]);
        const uint32_t t1 = aes_col(lds, lb, s.w1, s.w2, s.w3, s.w0, rk[4 * r + 1]);
        const uint32_t t2 = aes_col(lds, lb, s.w2, s.w3, s.w0, s.w1, rk[4 * r + 2]);
        const uint32_t t3 = aes_col(lds, lb, s.w3, s.w0, s.w1, s.w2, rk[4 * r + 3]);
        s = V4{t0, t1, t2, t3};
    }
    const uint32_t t0 = aes_col_last(lds, lb, s.w0, s.w1, s.w2, s.w3, rk[4 * ROUNDS + 0]);
    const uint32_t t1 = aes_col_last(lds, lb, s.w1, s.w2, s.w3, s.w0, rk[4 * ROUNDS + 1]);
    const uint32_t t2 = aes_col_last(lds, lb, s.w2, s.w3, s.w0, s.w1, rk[4 * ROUNDS + 2]);
    const uint32_t t3 = aes_col_last(lds, lb, s.w3, s.w0, s.w1, s.w2, rk[4 * ROUNDS + 3]);
    return V4{t0, t1, t2, t3};
}

/* single table lookups: T0, T1 = rotl8(T0), T2 = rotl16(T0), T3 = rotl8(T2), byte K of x */
template <int K>
__device__ __forceinline__ uint32_t lT0(const uint8_t *lds, uint32_t x, uint32_t lb)
{
    return lds32(lds, aes_addr<K>(x, lb));
}
template <int K>
__device__ __forceinline__ uint32_t lT2(const uint8_t *lds, uint32_t x, uint32_t lb)
{
    return lds32(lds, 128 + aes_addr<K>(x, lb));
}

/* Counter-mode shortcut (rounds 1-2).  For a record whose block counters stay below 2^16, the counter
 * word is 00 00 hi lo and everything else of the AES input is fixed per record, so after round 1 only
 * state columns 0 and 1 vary (they take counter bytes 15 and 14) and after round 2 every column is
 * (constant ^ two lookups).  CtrConst holds those per-record constants. */
struct CtrConst {
    uint32_t k10, k11; /* round-1 columns 0, 1 without their counter-byte term */
    uint32_t k20, k21, k22, k23; /* round-2 columns without the terms from round-1 columns 0 and 1 */
    uint32_t r03;      /* round key 0 word 3 (the counter word's whitening) */
};

__device__ __forceinline__ CtrConst ctr_const(const uint8_t *lds, uint32_t lb, const uint32_t *__restrict__ rk, uint32_t n0,
                                              uint32_t n1, uint32_t n2)
{
    const uint32_t s0 = n0 ^ rk[0], s1 = n1 ^ rk[1], s2 = n2 ^ rk[2], s3 = rk[3]; /* counter bytes 12,13 = 0 */
    CtrConst c;
    c.r03 = rk[3];
    /* round 1: t_c = T0[s_c.b0] ^ T1[s_{c+1}.b1] ^ T2[s_{c+2}.b2] ^ T3[s_{c+3}.b3] ^ rk1_c */
    c.k10 = lT0<0>(lds, s0, lb) ^ rotl8(lT0<1>(lds, s1, lb)) ^ lT2<2>(lds, s2, lb) ^ rk[4]; /* - T3[s3.b3] */
    c.k11 = lT0<0>(lds, s1, lb) ^ rotl8(lT0<1>(lds, s2, lb)) ^ rotl8(lT2<3>(lds, s0, lb)) ^ rk[5]; /* - T2[s3.b2] */
    const uint32_t t2 = lT0<0>(lds, s2, lb) ^ rotl8(lT0<1>(lds, s3, lb)) ^ lT2<2>(lds, s0, lb) ^ rotl8(lT2<3>(lds, s1, lb)) ^ rk[6];
    const uint32_t t3 = lT0<0>(lds, s3, lb) ^ rotl8(lT0<1>(lds, s0, lb)) ^ lT2<2>(lds, s1, lb) ^ rotl8(lT2<3>(lds, s2, lb)) ^ rk[7];
    /* round 2 constant parts (terms reading t2, t3) */
    c.k20 = lT2<2>(lds, t2, lb) ^ rotl8(lT2<3>(lds, t3, lb)) ^ rk[8];
    c.k21 = rotl8(lT0<1>(lds, t2, lb)) ^ lT2<2>(lds, t3, lb) ^ rk[9];
    c.k22 = lT0<0>(lds, t2, lb) ^ rotl8(lT0<1>(lds, t3, lb)) ^ rk[10];
    c.k23 = lT0<0>(lds, t3, lb) ^ rotl8(lT2<3>(lds, t2, lb)) ^ rk[11];
    return c;
}

/* ---------------- the pieces of one round, issue and finish apart ----------------
 * The compiler, left alone, consumes each T-table lookup a few instructions after issuing it (lgkmcnt(0..4) waits), so a
 * wave keeps only a handful of LDS reads in flight and the LDS array idles while the 12 waves of a CU wait on latency.
 * ctr_ghash_skewed issues a round's lookups (round_issue / last_issue), then XORs them (round_finish / last_finish) a
 * segment later. */
struct RoundLoads {
    uint32_t L[16];
};

/* the 16 lookups of a full round (column c uses bytes j of words c + j), raw T0 / T2 entries */
__device__ __forceinline__ void round_issue(const uint8_t *lds, uint32_t lb, const V4 &s, RoundLoads &r)
{
    const uint32_t w[4] = {s.w0, s.w1, s.w2, s.w3};
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        r.L[4 * c + 0] = lds32(lds, aes_addr<0>(w[c], lb));
        r.L[4 * c + 1] = lds32(lds, aes_addr<1>(w[(c + 1) & 3], lb));
        r.L[4 * c + 2] = lds32(lds, 128 + aes_addr<2>(w[(c + 2) & 3], lb));
        r.L[4 * c + 3] = lds32(lds, 128 + aes_addr<3>(w[(c + 3) & 3], lb));
    }
}

__device__ __forceinline__ V4 round_finish(const RoundLoads &r, const uint32_t *__restrict__ k)
{
    uint32_t t[4];
#pragma unroll
    for (int c = 0; c < 4; ++c)
        t[c] = xor3(r.L[4 * c + 0], r.L[4 * c + 2], rotl8(r.L[4 * c + 1] ^ r.L[4 * c + 3])) ^ k[c];
    return V4{t[0], t[1], t[2], t[3]};
}

/* final round: S-box bytes from T2[.].b0, T0[.].b1, T0[.].b2, T2[.].b3 (as aes_col_last) */
__device__ __forceinline__ void last_issue(const uint8_t *lds, uint32_t lb, const V4 &s, RoundLoads &r)
{
    const uint32_t w[4] = {s.w0, s.w1, s.w2, s.w3};
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        r.L[4 * c + 0] = lds32(lds, 128 + aes_addr<0>(w[c], lb));
        r.L[4 * c + 1] = lds32(lds, aes_addr<1>(w[(c + 1) & 3], lb));
        r.L[4 * c + 2] = lds32(lds, aes_addr<2>(w[(c + 2) & 3], lb));
        r.L[4 * c + 3] = lds32(lds, 128 + aes_addr<3>(w[(c + 3) & 3], lb));
    }
}

__device__ __forceinline__ V4 last_finish(const RoundLoads &r, const uint32_t *__restrict__ k)
{
    uint32_t t[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const uint32_t lo = __builtin_amdgcn_perm(r.L[4 * c + 1], r.L[4 * c + 0], 0x0c0c0500u);
        const uint32_t hi = __builtin_amdgcn_perm(r.L[4 * c + 3], r.L[4 * c + 2], 0x07020c0cu);
        t[c] = xor3(lo, hi, k[c]);
    }
    return V4{t[0], t[1], t[2], t[3]};
}

/* Keystream of KP counter blocks (the counter-mode shortcut for rounds 1-2, CtrConst) and, when HASH,
 * y <- (...(y * P ^ hx[0]) * P ^ ...) ^ hx[KP-1].  The lane's KP blocks run 1/KP of a round apart, so a wave always
 * has lookups in flight while it XORs.  Segment s issues a quarter GHASH multiply (s < 4 KP) and round
 * s/KP+1 of block s%KP, then finishes the round that block (s-KP+1)%KP issued KP-1 segments earlier and
 * folds in the quarter multiply (its lookups go out first, so the fold does not wait for the AES ones).
 * GH = the multiply's table, issued in GH::PARTS parts of 4 lookups: GhMain (the batch kernel's 8-bit windows,
 * 4 parts) or GhNibble (the sparse kernel's per-wave 4-bit windows, 8 parts), defined with the GHASH helpers. */
template <int ROUNDS, int KP, bool HASH, class GH>
__device__ __forceinline__ void ctr_ghash_skewed(const uint8_t *lds, uint32_t lb, const uint32_t *__restrict__ rk, const CtrConst &cc,
                                                 const uint32_t (&cw)[KP], V4 (&ks)[KP], V4 &y, const V4 (&hx)[KP], const GH &gm)
{
    constexpr int P = GH::PARTS; /* issue parts (4 lookups each) per GHASH multiply */
    static_assert(P * KP <= KP * ROUNDS, "GHASH parts must fit in the segments");
    V4 s[KP];
    uint32_t t0[KP], t1[KP];
    RoundLoads R[KP];
    uint32_t M[KP][8];
    V4 G[4];
    V4 acc = V4{0, 0, 0, 0}, xr = V4{0, 0, 0, 0};
    constexpr int NSEG = KP * ROUNDS + KP - 1;
#pragma unroll
    for (int seg = 0; seg < NSEG; ++seg) {
        const int gj = seg / P, gq = seg % P;
        const bool gh = HASH && gj < KP;
        __builtin_amdgcn_s_setprio(SETPRIO); /* a wave about to issue lookups goes first */
        /* ---- issue: GHASH quarter first, then the AES lookups (so the fold below need not wait for them) ---- */
        if (gh) {
            if (gq == 0) {
                xr = gm.prep(y);
                acc = hx[gj];
            }
            switch (gq) { /* gq is a constant once the segment loop is unrolled */
            case 0: gm.template issue<0>(lds, xr, G); break;
            case 1: gm.template issue<1>(lds, xr, G); break;
            case 2: gm.template issue<2>(lds, xr, G); break;
            case 3: gm.template issue<3 % P>(lds, xr, G); break;
            case 4: gm.template issue<4 % P>(lds, xr, G); break;
            case 5: gm.template issue<5 % P>(lds, xr, G); break;
            case 6: gm.template issue<6 % P>(lds, xr, G); break;
            default: gm.template issue<7 % P>(lds, xr, G); break;
            }
        }
        __builtin_amdgcn_sched_barrier(0);
        if (seg < KP * ROUNDS) {
            const int b = seg % KP, r = seg / KP + 1;
            if (r == 1) {
                const uint32_t x3 = cw[b] ^ cc.r03;
                M[b][0] = lT2<3>(lds, x3, lb);
                M[b][1] = lT2<2>(lds, x3, lb);
            } else if (r == 2) {
                M[b][0] = lT0<0>(lds, t0[b], lb);
                M[b][1] = lT0<1>(lds, t1[b], lb);
                M[b][2] = lT0<0>(lds, t1[b], lb);
                M[b][3] = lT2<3>(lds, t0[b], lb);
                M[b][4] = lT2<2>(lds, t0[b], lb);
                M[b][5] = lT2<3>(lds, t1[b], lb);
                M[b][6] = lT0<1>(lds, t0[b], lb);
                M[b][7] = lT2<2>(lds, t1[b], lb);
            } else if (r < ROUNDS) {
                round_issue(lds, lb, s[b], R[b]);
            } else {
                last_issue(lds, lb, s[b], R[b]);
            }
        }
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_setprio(0);
        /* ---- finish ---- */
        if (seg >= KP - 1) {
            const int fs = seg - (KP - 1); /* the segment that issued the lookups finished here */
            const int b = fs % KP, r = fs / KP + 1;
            if (r == 1) {
                t0[b] = cc.k10 ^ rotl8(M[b][0]);
                t1[b] = cc.k11 ^ M[b][1];
            } else if (r == 2) {
                s[b].w0 = xor3(cc.k20, M[b][0], rotl8(M[b][1]));
                s[b].w1 = xor3(cc.k21, M[b][2], rotl8(M[b][3]));
                s[b].w2 = xor3(cc.k22, M[b][4], rotl8(M[b][5]));
                s[b].w3 = xor3(cc.k23, rotl8(M[b][6]), M[b][7]);
            } else if (r < ROUNDS) {
                s[b] = round_finish(R[b], rk + 4 * r);
            } else {
                ks[b] = last_finish(R[b], rk + 4 * r);
            }
        }
        if (gh) {
            acc = v4xor3(acc, G[0], G[1]);
            acc = v4xor3(acc, G[2], G[3]);
            if (gq == P - 1)
                y = acc;
        }
        __builtin_amdgcn_sched_barrier(0);
    }
}

/* K independent blocks, round-interleaved */
template <int ROUNDS, int K>
__device__ __forceinline__ void aes_encrypt_n(const uint8_t *lds, uint32_t lb, const uint32_t *__restrict__ rk, V4 (&s)[K])
{
#pragma unroll
    for (int b = 0; b < K; ++b) {
        s[b].w0 ^= rk[0];
        s[b].w1 ^= rk[1];
        s[b].w2 ^= rk[2];
        s[b].w3 ^= rk[3];
    }
#pragma unroll
    for (int r = 1; r < ROUNDS; ++r) {
        const uint32_t k0 = rk[4 * r + 0], k1 = rk[4 * r + 1], k2 = rk[4 * r + 2], k3 = rk[4 * r + 3];
        V4 t[K];
#pragma unroll
        for (int b = 0; b < K; ++b) {
            t[b].w0 = aes_col(lds, lb, s[b].w0, s[b].w1, s[b].w2, s[b].w3, k0);
            t[b].w1 = aes_col(lds, lb, s[b].w1, s[b].w2, s[b].w3, s[b].w0, k1);
            t[b].w2 = aes_col(lds, lb, s[b].w2, s[b].w3, s[b].w0, s[b].w1, k2);
            t[b].w3 = aes_col(lds, lb, s[b].w3, s[b].w0, s[b].w1, s[b].w2, k3);
        }
#pragma unroll
        for (int b = 0; b < K; ++b)
            s[b] = t[b];
    }
    const uint32_t k0 = rk[4 * ROUNDS + 0], k1 = rk[4 * ROUNDS + 1], k2 = rk[4 * ROUNDS + 2], k3 = rk[4 * ROUNDS + 3];
    V4 t[K];
#pragma unroll
    for (int b = 0; b < K; ++b) {
        t[b].w0 = aes_col_last(lds, lb, s[b].w0, s[b].w1, s[b].w2, s[b].w3, k0);
        t[b].w1 = aes_col_last(lds, lb, s[b].w1, s[b].w2, s[b].w3, s[b].w0, k1);
        t[b].w2 = aes_col_last(lds, lb, s[b].w2, s[b].w3, s[b].w0, s[b].w1, k2);
        t[b].w3 = aes_col_last(lds, lb, s[b].w3, s[b].w0, s[b].w1, s[b].w2, k3);
    }
#pragma unroll
    for (int b = 0; b < K; ++b)
        s[b] = t[b];
}

/* ======================================================================================= *
 *  GHASH multiply by table                                                                 *
 * ======================================================================================= */

struct GhLane {
    uint32_t lb0, lb1, lb2, lb3; /* byte m of lbI = ((4I + m + lane) & 15) * 16 : slot of step 4I+m */
    uint32_t shift;              /* 8 * (lane & 3) */
    bool rot1, rot2;             /* word rotation by (lane >> 2) & 3 */
};

__device__ __forceinline__ GhLane gh_lane_from(uint32_t lane)
{
    GhLane g;
    /* byte m of lbI = ((lane + 4I + m) & 15) * 16: all four bytes at once (no carries: values < 256) */
    const uint32_t base = lane * 0x01010101u + 0x03020100u;
    g.lb0 = ((base + 0x00000000u) & 0x0f0f0f0fu) << 4;
    g.lb1 = ((base + 0x04040404u) & 0x0f0f0f0fu) << 4;
    g.lb2 = ((base + 0x08080808u) & 0x0f0f0f0fu) << 4;
    g.lb3 = ((base + 0x0c0c0c0cu) & 0x0f0f0f0fu) << 4;
    g.shift = 8u * (lane & 3);
    g.rot1 = ((lane >> 2) & 1) != 0;
    g.rot2 = ((lane >> 3) & 1) != 0;
    return g;
}

__device__ __forceinline__ GhLane gh_lane_init(int lane)
{
    return gh_lane_from((uint32_t)lane);
}

template <int K>
__device__ __forceinline__ V4 gh_term(const uint8_t *lds, uint32_t xw, uint32_t lbw)
{
    /* address = (xrot.byte[K] << 8) | slot(K):  byte0 <- lbw.byte[K%4], byte1 <- xw.byte[K%4] */
    const uint32_t addr = __builtin_amdgcn_perm(xw, lbw, 0x0c0c0000u | ((4u + (K & 3)) << 8) | (K & 3));
    return lds128(lds, LDS_GMAIN + addr);
}

/* returns y * P ^ x, P = the power held in the main table */
__device__ __forceinline__ V4 gh_mul_main(const uint8_t *lds, const GhLane &g, V4 y, V4 x)
{
    /* rotate y right by (lane & 15) bytes: xr.byte[k] = y.byte[(k + lane) & 15] */
    const uint32_t s0 = g.rot1 ? y.w1 : y.w0, s1 = g.rot1 ? y.w2 : y.w1, s2 = g.rot1 ? y.w3 : y.w2, s3 = g.rot1 ? y.w0 : y.w3;
    const uint32_t r0 = g.rot2 ? s2 : s0, r1 = g.rot2 ? s3 : s1, r2 = g.rot2 ? s0 : s2, r3 = g.rot2 ? s1 : s3;
    const uint32_t x0 = __builtin_amdgcn_alignbit(r1, r0, g.shift);
    const uint32_t x1 = __builtin_amdgcn_alignbit(r2, r1, g.shift);
    const uint32_t x2 = __builtin_amdgcn_alignbit(r3, r2, g.shift);
    const uint32_t x3 = __builtin_amdgcn_alignbit(r0, r3, g.shift);
    V4 acc = v4xor3(x, gh_term<0>(lds, x0, g.lb0), gh_term<1>(lds, x0, g.lb0));
    acc = v4xor3(acc, gh_term<2>(lds, x0, g.lb0), gh_term<3>(lds, x0, g.lb0));
    acc = v4xor3(acc, gh_term<4>(lds, x1, g.lb1), gh_term<5>(lds, x1, g.lb1));
    acc = v4xor3(acc, gh_term<6>(lds, x1, g.lb1), gh_term<7>(lds, x1, g.lb1));
    acc = v4xor3(acc, gh_term<8>(lds, x2, g.lb2), gh_term<9>(lds, x2, g.lb2));
    acc = v4xor3(acc, gh_term<10>(lds, x2, g.lb2), gh_term<11>(lds, x2, g.lb2));
    acc = v4xor3(acc, gh_term<12>(lds, x3, g.lb3), gh_term<13>(lds, x3, g.lb3));
    acc = v4xor3(acc, gh_term<14>(lds, x3, g.lb3), gh_term<15>(lds, x3, g.lb3));
    return acc;
}

/* gh_mul_main in pieces for ctr_ghash_skewed (GhMain): the lane rotation of y, then the lookups of words T0 / 4 .. */
__device__ __forceinline__ V4 gh_rot(const GhLane &g, V4 y)
{
    const uint32_t s0 = g.rot1 ? y.w1 : y.w0, s1 = g.rot1 ? y.w2 : y.w1, s2 = g.rot1 ? y.w3 : y.w2, s3 = g.rot1 ? y.w0 : y.w3;
    const uint32_t r0 = g.rot2 ? s2 : s0, r1 = g.rot2 ? s3 : s1, r2 = g.rot2 ? s0 : s2, r3 = g.rot2 ? s1 : s3;
    return V4{__builtin_amdgcn_alignbit(r1, r0, g.shift), __builtin_amdgcn_alignbit(r2, r1, g.shift),
              __builtin_amdgcn_alignbit(r3, r2, g.shift), __builtin_amdgcn_alignbit(r0, r3, g.shift)};
}

template <int T0, int NT, int NG>
__device__ __forceinline__ void gh_issue(const uint8_t *lds, const GhLane &g, const V4 &xr, V4 (&G)[NG])
{
    static_assert(NT <= NG, "lookups must fit the result array");
#pragma unroll
    for (int i = 0; i < NT; ++i) {
        const int t = T0 + i, q = t >> 2;
        const uint32_t xw = q == 0 ? xr.w0 : q == 1 ? xr.w1 : q == 2 ? xr.w2 : xr.w3;
        const uint32_t lbw = q == 0 ? g.lb0 : q == 1 ? g.lb1 : q == 2 ? g.lb2 : g.lb3;
        const uint32_t addr = __builtin_amdgcn_perm(xw, lbw, 0x0c0c0000u | ((4u + (t & 3)) << 8) | (t & 3));
        G[i] = lds128(lds, LDS_GMAIN + addr);
    }
}

/* GHASH-multiply policies of ctr_ghash_skewed: the issue of part Q (4 ds_read_b128) of one multiply of y */
struct GhMain { /* the batch kernel's 8-bit-window table of P at LDS_GMAIN: 16 lookups = 4 parts (one word of rotated y each) */
    const GhLane &g;
    static constexpr int PARTS = 4;
    __device__ __forceinline__ V4 prep(V4 y) const { return gh_rot(g, y); }
    template <int Q>
    __device__ __forceinline__ void issue(const uint8_t *lds, const V4 &xr, V4 (&G)[4]) const
    {
        gh_issue<4 * Q, 4>(lds, g, xr, G);
    }
};

struct GhNibble { /* a 4-bit-window table [p = 8w + j][v] at LDS offset tab (gh_mul_nibble's layout): 32 lookups = 8 parts */
    uint32_t tab;
    static constexpr int PARTS = 8;
    __device__ __forceinline__ V4 prep(V4 y) const { return y; }
    template <int Q>
    __device__ __forceinline__ void issue(const uint8_t *lds, const V4 &xr, V4 (&G)[4]) const
    {
        const uint32_t w = (Q >> 1) == 0 ? xr.w0 : (Q >> 1) == 1 ? xr.w1 : (Q >> 1) == 2 ? xr.w2 : xr.w3;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int j = 4 * (Q & 1) + i; /* nibble j of word Q / 2 */
            G[i] = lds128(lds, tab + (uint32_t)(8 * (Q >> 1) + j) * 256u + ((w >> (4 * j)) & 15u) * 16u);
        }
    }
};

template <int ROUNDS, int KP, bool HASH>
__device__ __forceinline__ void ctr_ghash(const uint8_t *lds, uint32_t lb, const uint32_t *__restrict__ rk, const CtrConst &cc,
                                          const uint32_t (&cw)[KP], V4 (&ks)[KP], V4 &y, const V4 (&hx)[KP], const GhLane &g)
{
    ctr_ghash_skewed<ROUNDS, KP, HASH>(lds, lb, rk, cc, cw, ks, y, hx, GhMain{g});
}

/* y * P with a nibble table [p = 8w + j][v] (the G = 1 multiply by H, the sparse kernel's Horner steps).  One word
 * (8 lookups) at a time: sched barriers keep the compiler from hoisting all 32 ds_read_b128 (128 VGPRs). */
__device__ __forceinline__ V4 gh_mul_nibble(const uint8_t *lds, uint32_t table, V4 y)
{
    V4 acc = V4{0, 0, 0, 0};
    const uint32_t w[4] = {y.w0, y.w1, y.w2, y.w3};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        V4 t[8];
#pragma unroll
        for (int j = 0; j < 8; ++j)
            t[j] = lds128(lds, table + (uint32_t)(8 * i + j) * 256u + ((w[i] >> (4 * j)) & 15u) * 16u);
        acc = v4xor3(acc, t[0], t[1]);
        acc = v4xor3(acc, t[2], t[3]);
        acc = v4xor3(acc, t[4], t[5]);
        acc = v4xor3(acc, t[6], t[7]);
        __builtin_amdgcn_sched_barrier(0);
    }
    return acc;
}

/* v * x in GF(2^128) on big-endian words (bit 0 of the GCM string = bit 31 of v[0]) */
__device__ __forceinline__ void mulx_be(uint32_t (&v)[4])
{
    const uint32_t c = (uint32_t)__builtin_amdgcn_sbfe((int)v[3], 0u, 1u);
    v[3] = __builtin_amdgcn_alignbit(v[2], v[3], 1);
    v[2] = __builtin_amdgcn_alignbit(v[1], v[2], 1);
    v[1] = __builtin_amdgcn_alignbit(v[0], v[1], 1);
    v[0] = (v[0] >> 1) ^ (c & 0xe1000000u);
}

/* x * y in GF(2^128), GCM bit order, both operands per lane: SP 800-38D Algorithm 1's product with 4-bit windows over x
 * (Shoup) and a per-lane table of y in LDS instead of 128 single-bit steps (11 VALU each, 1 408 in all).
 *   T[n] = n3 y + n2 y x + n1 y x^2 + n0 y x^3 (n3 = the nibble's first GCM bit); entry n of lane l at
 *   tab + n * 1024 + l * 16 (STRIDE = 1024: a row of the 64 lanes' entries n), so the 16 lanes of every ds_read_b128 /
 *   ds_write_b128 group touch 16 consecutive 16-B slots, i.e. the 64 banks once, whatever the nibbles.  (Until round 4
 *   lane l's entries were contiguous with a per-lane slot rotation: conflict-free stores but data-dependent 2-4-way
 *   conflicts on the lookups, SQ_LDS_BANK_CONFLICT 4.7 % of c4s's LDS cycles.)
 *   NT = 8 holds T[0..7] and folds n3 y in on the VALU (8 KiB per wave: the sparse kernel's per-wave table area).
 *   Z = T[nib_31]; Z = Z x^4 + T[nib_j] for j = 30 .. 0.  The 4 bits each shift drops (positions 128..131) are
 *   collected in one overflow word and folded back every 8 shifts with x^128 = 1 + x + x^2 + x^7.
 * About 500 VALU + NT ds_write_b128 + 32 ds_read_b128 against the bit-serial 1 408 VALU.  The caller owns the table
 * area; the wave's LDS operations complete in order, so no barrier is needed around it.  STRIDE = 512: the batch
 * kernel's shared G = 32 tables ([n][q], build_ghash_tables), base = the record position q's column. */
template <int NT, int STRIDE = 1024>
struct Win4 {
    uint32_t base;      /* entry n at base + n * STRIDE */
    uint32_t y[4];      /* NT = 8: y itself (big-endian words), folded in for the nibble's first bit */
};

template <int NT>
__device__ __forceinline__ Win4<NT> gf_win4_build(uint8_t *lds, uint32_t tab, int lane, V4 yr)
{
    static_assert(NT == 8 || NT == 16, "4-bit windows: 8 or 16 table entries per lane");
    uint32_t m[4][4]; /* m[k] = y x^k */
    m[0][0] = bswap32(yr.w0), m[0][1] = bswap32(yr.w1), m[0][2] = bswap32(yr.w2), m[0][3] = bswap32(yr.w3);
#pragma unroll
    for (int k = 1; k < 4; ++k) {
#pragma unroll
        for (int w = 0; w < 4; ++w)
            m[k][w] = m[k - 1][w];
        mulx_be(m[k]);
    }
    Win4<NT> t;
    /* the entries start from an opaque zero: a plain {0, 0, 0, 0} for T[0] was hoisted out of the record loop as one zero
     * vector and spilled (a 16-byte scratch reload per record in the sparse kernel) */
    uint32_t zero;
    asm volatile("v_mov_b32 %0, 0" : "=v"(zero));
    uint32_t ln = (uint32_t)lane;
    asm volatile("" : "+v"(ln)); /* keeps the lane's slot arithmetic here: hoisted out of a record loop, its values stay
                                    live across the whole kernel (the sparse batch kernel spilled 200 B per lane) */
    t.base = tab + ln * 16u;
#pragma unroll
    for (int w = 0; w < 4; ++w)
        t.y[w] = m[0][w];
#pragma unroll
    for (int n = 0; n < NT; ++n) {
        uint32_t e[4] = {zero, zero, zero, zero};
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if ((n >> (3 - k)) & 1)
#pragma unroll
                for (int w = 0; w < 4; ++w)
                    e[w] ^= m[k][w];
        lds128_store(lds, t.base + (uint32_t)n * 1024u, V4{e[0], e[1], e[2], e[3]});
    }
    return t;
}

template <int NT, int LB = 8, int STRIDE>
__device__ __forceinline__ V4 gf_win4_mul(const uint8_t *lds, const Win4<NT, STRIDE> &tb, V4 xr)
{
    static_assert(LB == 8 || LB == 4 || LB == 2, "lookups in flight: 8, 4 or 2");
    const uint32_t x[4] = {bswap32(xr.w0), bswap32(xr.w1), bswap32(xr.w2), bswap32(xr.w3)};
    uint32_t z0 = 0, z1 = 0, z2 = 0, z3 = 0, ov = 0;
#pragma unroll
    for (int g = 0; g < 32 / LB; ++g) { /* nibbles j = 31 - g LB down to 32 - (g + 1) LB */
        const int j0 = 31 - g * LB, w = j0 >> 3, i0 = 8 * w + 7 - j0;
        V4 t[LB];
#pragma unroll
        for (int ii = 0; ii < LB; ++ii) { /* nibble j = 8 w + 7 - i: bits 4 i .. 4 i + 3 from the bottom of word w */
            const int i = i0 + ii;
            const uint32_t nib = (x[w] >> (4 * i)) & 15u;
            t[ii] = lds128(lds, tb.base + (nib & (uint32_t)(NT - 1)) * (uint32_t)STRIDE);
            if (NT == 8) {
                const uint32_t mk = 0u - (nib >> 3);
                t[ii] = V4{t[ii].w0 ^ (mk & tb.y[0]), t[ii].w1 ^ (mk & tb.y[1]), t[ii].w2 ^ (mk & tb.y[2]), t[ii].w3 ^ (mk & tb.y[3])};
            }
        }
#pragma unroll
        for (int ii = 0; ii < LB; ++ii) {
            const int j = 8 * w + 7 - (i0 + ii);
            if (j != 31) { /* Z * x^4, the dropped nibble into the overflow word */
                ov = __builtin_amdgcn_alignbit(z3, ov, 4);
                z3 = __builtin_amdgcn_alignbit(z2, z3, 4);
                z2 = __builtin_amdgcn_alignbit(z1, z2, 4);
                z1 = __builtin_amdgcn_alignbit(z0, z1, 4);
                z0 >>= 4;
                if (((31 - j) & 7) == 0) { /* 8 shifts: positions 128..159 folded back */
                    z0 ^= ov ^ (ov >> 1) ^ (ov >> 2) ^ (ov >> 7);
                    z1 ^= (ov << 31) ^ (ov << 30) ^ (ov << 25);
                    ov = 0;
                }
            }
            z0 ^= t[ii].w0, z1 ^= t[ii].w1, z2 ^= t[ii].w2, z3 ^= t[ii].w3;
        }
        __builtin_amdgcn_sched_barrier(0); /* LB lookups in flight at a time (4 LB VGPRs) */
    }
    z0 ^= ov ^ (ov >> 1) ^ (ov >> 2) ^ (ov >> 7); /* the last 7 shifts' bits */
    z1 ^= (ov << 31) ^ (ov << 30) ^ (ov << 25);
    return V4{bswap32(z0), bswap32(z1), bswap32(z2), bswap32(z3)};
}

template <int NT, int LB = 8>
__device__ __forceinline__ V4 gf_mul_win4(uint8_t *lds, uint32_t tab, int lane, V4 xr, V4 yr)
{
    return gf_win4_mul<NT, LB>(lds, gf_win4_build<NT>(lds, tab, lane, yr), xr);
}

/* ---------------- table construction in LDS ---------------- */

__device__ __forceinline__ V4 ld_basis(const uint32_t *b, int e)
{
    const uint4 v = reinterpret_cast<const uint4 *>(b)[e];
    return V4{v.x, v.y, v.z, v.w};
}

/* AES tables at LDS byte offset `base`: row v = [T0[v] x 32 | rotl16(T0[v]) x 32], 256 B = 16 chunks of 16 B.
 * Thread i (of NT) writes chunks i, i + NT, ... (row c >> 4, chunk c & 15) with one ds_write_b128 each, the T0 loads
 * of all its chunks issued first (one global-load latency instead of one per entry: what a single-record launch
 * waits on); consecutive threads write consecutive 16-B chunks (conflict-free). */
template <int NT>
__device__ __forceinline__ void build_aes_tables(uint8_t *lds, uint32_t base, const uint32_t *__restrict__ t0, int tid = -1)
{
    constexpr int IT = (256 * 16 + NT - 1) / NT;
    if (tid < 0)
        tid = (int)threadIdx.x;
    uint32_t t[IT];
#pragma unroll
    for (int k = 0; k < IT; ++k) {
        const int c = tid + k * NT;
        t[k] = c < 256 * 16 ? t0[c >> 4] : 0u;
    }
#pragma unroll
    for (int k = 0; k < IT; ++k) {
        const int c = tid + k * NT;
        if (c < 256 * 16) {
            const uint32_t x = (c & 15) < 8 ? t[k] : (t[k] << 16) | (t[k] >> 16);
            lds128_store(lds, base + (uint32_t)(c >> 4) * 256u + (uint32_t)(c & 15) * 16u, V4{x, x, x, x});
        }
    }
}

/* GHASH tables of one key slot.  basis = uint4[NPOW][128], basis[t][e] = H^(2^t) * x^e (GCM bit
 * index e: byte e/8, bit 7 - e%8).  Raw byte p, bit t  <->  e = 8p + 7 - t.  tree: also the nibble tables of
 * the shuffle-tree combination (not needed when the lanes combine on the VALU).
 * Main table: thread (p = tid & 15, hv = tid >> 4) of the first 256 writes the 16 entries v = 16 hv + lv of
 * position p: 4 + popcount(hv) basis loads, the 16 low-nibble combinations in Gray-code order, and
 * stores whose 8-lane groups hold 8 different positions p, i.e. 8 different bank quads (conflict-free).
 * (Per entry from up to 8 basis loads with lanes 256 B apart cost a key switch 8x the loads and 8-way store
 * conflicts.)  The other threads build the tree tables meanwhile. */
/* the shared window tables' row width (slots) and copies per record position (build_ghash_tables, the lane combination) */
__host__ __device__ constexpr int win_row(int g) { return g > 16 ? g : 16; }
__host__ __device__ constexpr int win_copies(int g) { return g >= 16 ? 1 : 16 / g; }

__device__ void build_ghash_tables(uint8_t *lds, const uint32_t *__restrict__ basis, int log2g)
{
    const uint32_t *bm = basis + log2g * 128 * 4;
    /* the thread index made opaque: otherwise its addresses (basis vectors, table slots) are hoisted out of the kernel's
     * chunk loop and spilled, and every key switch reloads them from scratch after its barrier (round 4) */
    int tid = (int)threadIdx.x;
    asm volatile("" : "+v"(tid));
    if (tid < 256) {
        const int p = tid & 15, hv = tid >> 4;
        V4 lb[4];
        V4 hi = V4{0, 0, 0, 0};
#pragma unroll
        for (int t = 0; t < 4; ++t)
            lb[t] = ld_basis(bm, 8 * p + 7 - t);
#pragma unroll
        for (int t = 0; t < 4; ++t)
            if ((hv >> t) & 1)
                hi = v4xor(hi, ld_basis(bm, 8 * p + 7 - (4 + t)));
        /* low nibble in Gray-code order: each entry is the previous one with one basis vector toggled */
        V4 cur = hi;
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            if (k != 0)
                cur = v4xor(cur, lb[__builtin_ctz(k)]); /* bit that flips between Gray codes k - 1 and k */
            const int lv = k ^ (k >> 1);
            lds128_store(lds, LDS_GMAIN + (uint32_t)(16 * hv + lv) * 256u + (uint32_t)p * 16u, cur);
        }
    }
    const int t0 = (int)blockDim.x > 256 ? 256 : 0, nt = (int)blockDim.x - t0;
    if (log2g == 0) { /* G = 1: the nibble table of H for the record's final multiply (gh_mul_nibble's layout) */
        for (int e = tid - t0; e >= 0 && e < 512; e += nt) {
            const int p = (e >> 4) & 31, v = e & 15;
            const int w = p >> 3, j = p & 7;
            V4 acc = V4{0, 0, 0, 0};
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                if ((v >> t) & 1) {
                    const int u = 4 * j + t; /* bit u of little-endian word w = raw byte 4w + u/8, bit u%8 */
                    acc = v4xor(acc, ld_basis(basis, 8 * (4 * w + (u >> 3)) + 7 - (u & 7)));
                }
            }
            lds128_store(lds, LDS_GTREE + p * 256 + v * 16, acc);
        }
        return;
    }
    /* G >= 2: the lane combination's shared window tables, rows n < 16 of win_row(G) slots, slot
     * q * CP + c = n * H^(q + 1) for q < G (CP = win_copies(G) copies, one per record of a 16-lane group when G < 16), in
     * gf_win4_mul's big-endian words (gf_win4_build's entries, shared by every lane of the workgroup whose record position
     * is q).  A lookup's 16-lane group then reads 16 distinct slots of its row, whatever the nibbles (until round 4, for
     * G = 32 only: [q][slot (n + q) mod 16], data-dependent conflicts) */
    const int wrow = win_row(1 << log2g), wcp = win_copies(1 << log2g);
    for (int e = tid - t0; e >= 0 && e < 16 * wrow; e += nt) {
        const int sl = e % wrow, q = sl / wcp, n = e / wrow; /* consecutive threads: consecutive slots (conflict-free stores) */
        const uint32_t *hp = basis + (NPOW * 128 + q) * 4; /* H^(q + 1) */
        uint32_t m[4] = {bswap32(hp[0]), bswap32(hp[1]), bswap32(hp[2]), bswap32(hp[3])}, acc[4] = {0, 0, 0, 0};
#pragma unroll
        for (int k = 0; k < 4; ++k) { /* n3 -> y, n2 -> y x, n1 -> y x^2, n0 -> y x^3 */
            if ((n >> (3 - k)) & 1)
#pragma unroll
                for (int w = 0; w < 4; ++w)
                    acc[w] ^= m[w];
            mulx_be(m);
        }
        lds128_store(lds, LDS_GTREE + (uint32_t)(n * wrow + sl) * 16u, V4{acc[0], acc[1], acc[2], acc[3]});
    }
}

/* ---------------- global-memory block access ---------------- */

/* A whole 16-byte block at any byte address: gfx9+ global memory instructions handle unaligned
 * addresses (the ROCm default unaligned access mode), so an align(1) vector type still compiles to ONE
 * global_load/store_dwordx4.  Only whole blocks (all 16 bytes inside the record) go through these. */
struct __attribute__((packed, aligned(1))) U4u {
    uint32_t x, y, z, w;
};

__device__ __forceinline__ V4 load_full(const uint8_t *p)
{
    const U4u v = *reinterpret_cast<const U4u *>(p);
    return V4{v.x, v.y, v.z, v.w};
}

__device__ __forceinline__ void store_full(uint8_t *p, V4 v)
{
    *reinterpret_cast<U4u *>(p) = U4u{v.w0, v.w1, v.w2, v.w3};
}

/* 128-bit shifts by one byte (raw byte order: w0 holds bytes 0..3) */
__device__ __forceinline__ V4 shr8(V4 v)
{
    return V4{__builtin_amdgcn_alignbit(v.w1, v.w0, 8), __builtin_amdgcn_alignbit(v.w2, v.w1, 8),
              __builtin_amdgcn_alignbit(v.w3, v.w2, 8), v.w3 >> 8};
}

__device__ __forceinline__ V4 shl8_in(V4 v, uint8_t b)
{
    return V4{(v.w0 << 8) | b, __builtin_amdgcn_alignbit(v.w1, v.w0, 24), __builtin_amdgcn_alignbit(v.w2, v.w1, 24),
              __builtin_amdgcn_alignbit(v.w3, v.w2, 24)};
}

/* exact byte-granular access (n in 0..16), used for unaligned layouts and the first block of a record shorter than 16
 * bytes: n independent byte loads (each still behind a per-lane condition, so the compiler may wait between some of
 * them; the loop that carried the block through its shifts waited after every byte) */
__device__ __forceinline__ V4 load_bytes(const uint8_t *p, int n)
{
    uint32_t b[16];
#pragma unroll
    for (int k = 0; k < 16; ++k)
        b[k] = k < n ? (uint32_t)p[k] : 0u;
    uint32_t w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
        w[i] = b[4 * i] | (b[4 * i + 1] << 8) | (b[4 * i + 2] << 16) | (b[4 * i + 3] << 24);
    return V4{w[0], w[1], w[2], w[3]};
}

__device__ __forceinline__ void store_bytes(uint8_t *p, int n, V4 v)
{
#pragma unroll 1
    for (int k = 0; k < n; ++k) {
        p[k] = (uint8_t)v.w0;
        v = shr8(v);
    }
}

__device__ __forceinline__ V4 mask_block(V4 v, int n);

/* A (possibly partial) block of n bytes: a whole block as one 16-byte load; a partial one at a 16-byte aligned p as its
 * whole dwords, then a 16-bit and / or an 8-bit load for the last 1..3 bytes; unaligned, byte by byte.  Nothing past
 * p + n is read (fusion over-reads within the page, lib/fusion.c:345-388; a caller's allocation may end at the record's
 * last byte, SURVEY.md §5, tests/test_gpu_guard.py).  Each piece goes to a register of its own and they are combined
 * at the end (the form that combined each dword inside its branch waited there up to 4 times per block); the loads still
 * sit behind per-lane conditions, so the hot paths use tail_load / load_block_nb below, which have none. */
template <bool ALIGNED>
__device__ __forceinline__ V4 load_block(const uint8_t *p, int n)
{
    if (!ALIGNED) {
        if (n == 16)
            return load_full(p);
        return load_bytes(p, n);
    }
    V4 f = V4{0, 0, 0, 0};
    if (n == 16)
        f = load_full(p);
    const uint32_t *q = reinterpret_cast<const uint32_t *>(p);
    uint32_t d[4] = {0, 0, 0, 0}, h[4] = {0, 0, 0, 0}, b[4] = {0, 0, 0, 0};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int k = n - 4 * i;
        if (n < 16 && k >= 4)
            d[i] = q[i];
        if (k == 2 || k == 3)
            h[i] = *reinterpret_cast<const uint16_t *>(p + 4 * i);
        if (k == 1 || k == 3)
            b[i] = p[4 * i + k - 1];
    }
    uint32_t w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
        w[i] = d[i] | h[i] | (b[i] << ((n - 4 * i) == 3 ? 16 : 0));
    return V4{f.w0 | w[0], f.w1 | w[1], f.w2 | w[2], f.w3 | w[3]};
}

/* n (0..15) bytes of v to a 16-byte aligned p: whole dwords, then a 16-bit and / or an 8-bit store (nothing past p + n) */
__device__ __forceinline__ void store_partial_aligned(uint8_t *p, int n, V4 v)
{
    uint32_t *q = reinterpret_cast<uint32_t *>(p);
    const uint32_t w[4] = {v.w0, v.w1, v.w2, v.w3};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int k = n - 4 * i;
        if (k >= 4) {
            q[i] = w[i];
        } else if (k > 0) {
            if (k >= 2)
                *reinterpret_cast<uint16_t *>(p + 4 * i) = (uint16_t)w[i];
            if (k != 2)
                p[4 * i + k - 1] = (uint8_t)(w[i] >> (8 * (k - 1)));
        }
    }
}

template <bool ALIGNED>
__device__ __forceinline__ void store_block(uint8_t *p, int n, V4 v)
{
    if (n == 16) {
        store_full(p, v);
        return;
    }
    if (ALIGNED)
        store_partial_aligned(p, n, v);
    else
        store_bytes(p, n, v);
}

__device__ __forceinline__ V4 mask_block(V4 v, int n)
{
    /* keep the first n (0..16) bytes */
    const uint32_t w[4] = {v.w0, v.w1, v.w2, v.w3};
    uint32_t o[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int keep = n - 4 * i;
        o[i] = keep >= 4 ? w[i] : (keep <= 0 ? 0u : (w[i] & ((1u << (8 * keep)) - 1u)));
    }
    return V4{o[0], o[1], o[2], o[3]};
}

/* v with byte `pos` (0..15, currently zero) set to b */
__device__ __forceinline__ V4 put_byte(V4 v, int pos, uint32_t b)
{
    const uint32_t x = b << (8 * (pos & 3));
    const int w = pos >> 2;
    return V4{v.w0 | (w == 0 ? x : 0u), v.w1 | (w == 1 ? x : 0u), v.w2 | (w == 2 ? x : 0u), v.w3 | (w == 3 ? x : 0u)};
}

/* n (0..16) bytes at a 16-byte aligned p with no branch: 4 dword loads, a 16-bit and an 8-bit load, each from its place
 * in the block when it holds record bytes and from `safe` (any readable, 4-byte aligned address, e.g. the AES table's
 * global copy) when not, the unwanted results masked off.  Nothing outside [p, p + n) is read of the caller's buffers;
 * since no branch holds a load's result, the loads go out together and the wave waits once (the branchy form waited up
 * to 4 times per block: the batch kernel's AAD element at every task start). */
__device__ __forceinline__ V4 load_block_nb(const uint8_t *p, int n, const uint8_t *safe)
{
    const int nd = n >> 2, t = n & 3;
    uint32_t d[4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
        d[i] = *reinterpret_cast<const uint32_t *>(i < nd ? p + 4 * i : safe);
    const uint32_t h = *reinterpret_cast<const uint16_t *>(t >= 2 ? p + 4 * nd : safe);
    const uint32_t b = *(t & 1 ? p + n - 1 : safe);
    const uint32_t tail = (t >= 2 ? h : 0u) | (t & 1 ? b << (t == 3 ? 16 : 0) : 0u);
    uint32_t w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
        w[i] = i < nd ? d[i] : i == nd ? tail : 0u;
    return V4{w[0], w[1], w[2], w[3]};
}

/* byte k of the result = byte k + s of v (s in 0..15), zeros above byte 15 - s */
__device__ __forceinline__ V4 shr_bytes(V4 v, int s)
{
    const uint64_t lo = (uint64_t)v.w1 << 32 | v.w0, hi = (uint64_t)v.w3 << 32 | v.w2;
    const uint32_t sh = 8u * (uint32_t)s;
    const uint64_t a = sh < 64 ? lo : hi, b = sh < 64 ? hi : 0;
    const uint32_t r = sh & 63u;
    const uint64_t rlo = r ? (a >> r) | (b << (64u - r)) : a, rhi = r ? b >> r : b;
    return V4{(uint32_t)rlo, (uint32_t)(rlo >> 32), (uint32_t)rhi, (uint32_t)(rhi >> 32)};
}

/* Data block c of a record, its first nb (0..16) bytes, for the generic elements: issued as ONE 16-byte load of the 16
 * bytes that END at the block's last byte (inside the record whenever 16 c + nb >= 16), brought down by tail_shift()
 * after the AES; only the first block of a record shorter than 16 bytes is read piecewise.  No branch uses the loaded
 * value, so the loads of an element pair are all in flight during its AES (loading the partial block piecewise inside
 * divergent branches made the compiler wait there: 3.7 % of c3's wave cycles before the AES could start). */
__device__ __forceinline__ V4 tail_load(const uint8_t *blk, int c, int nb, int &shift)
{
    shift = 0;
    if (nb <= 0)
        return V4{0, 0, 0, 0};
    if (16 * c + nb >= 16) {
        shift = 16 - nb;
        return load_full(blk + nb - 16);
    }
    return load_bytes(blk, nb); /* the first block of a record of fewer than 16 bytes */
}

__device__ __forceinline__ V4 tail_shift(V4 raw, int shift)
{
    return shift ? shr_bytes(raw, shift) : raw;
}

/* Diagnostic clock stamps (ptls_hip_batch_set_clock; nothing runs unless a buffer is given): thread 0 of a workgroup
 * reads the shader-cycle counter and the constant 100 MHz counter at the start (slot 0) and the end (slot 1) of the
 * workgroup's work into clk[4 * block + 2 * slot + {0, 1}].  The host takes delta(cycles) / delta(100 MHz ticks) as the
 * clock the launch ran at (MI355X_MICROARCH.md, DVFS).  The values go only to that buffer; no output depends on them. */
__device__ __forceinline__ void clock_stamp(uint64_t *__restrict__ clk, int slot)
{
    if (clk != nullptr && threadIdx.x == 0) {
        const uint64_t t = __builtin_amdgcn_s_memtime();
        const uint64_t r = __builtin_amdgcn_s_memrealtime();
        /* the XCD this workgroup runs on (HW_REG_XCC_ID bits 3:0) rides in the top byte of the start's 100 MHz stamp */
        const uint64_t xcc = slot == 0 ? (uint64_t)(__builtin_amdgcn_s_getreg((3 << 11) | 20) & 15u) << 56 : 0;
        __builtin_amdgcn_s_waitcnt(0xC07F); /* lgkmcnt(0): the counters are back before any LDS wait is counted */
        clk[4 * blockIdx.x + 2 * slot] = t;
        clk[4 * blockIdx.x + 2 * slot + 1] = r | xcc;
    }
}

/* ---- cross-lane sums and maxima on the VALU ----
 * Over aligned groups of N = 1 .. 64 lanes: DPP row permutations pair each lane with one in the other half of its quad
 * (quad_perm [1,0,3,2], then [2,3,0,1]), of its 8 lanes (row_half_mirror: i <-> 7 - i) and of its 16-lane row
 * (row_mirror: i <-> 15 - i); gfx950's v_permlane16_swap / v_permlane32_swap pair the two rows of a 32-lane half and the
 * two halves of the wave (a swap of vdst = src = v leaves {own, partner} in the two results, in some order).  After
 * log2(N) stages every lane holds the group's total.  No LDS instruction and no per-lane partner address: the
 * ds_bpermute form cost one LDS instruction per stage and word on an LDS-bound kernel, waited an LDS round trip per
 * stage, and its partner addresses were hoisted out of the record loops into long-lived registers. */
constexpr int DPP_QUAD_XOR1 = 0xB1, DPP_QUAD_XOR2 = 0x4E, DPP_ROW_HALF_MIRROR = 0x141, DPP_ROW_MIRROR = 0x140;

template <int CTRL>
__device__ __forceinline__ uint32_t dpp_mov(uint32_t v)
{
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xf, 0xf, false);
}

/* every lane of the v's N-lane group gets op over the group (called with every lane of the wave active) */
template <int N, class OP>
__device__ __forceinline__ uint32_t group_reduce(uint32_t v, OP op)
{
    static_assert(N >= 1 && N <= 64 && (N & (N - 1)) == 0, "group of 1 .. 64 lanes");
    if constexpr (N >= 2)
        v = op(v, dpp_mov<DPP_QUAD_XOR1>(v));
    if constexpr (N >= 4)
        v = op(v, dpp_mov<DPP_QUAD_XOR2>(v));
    if constexpr (N >= 8)
        v = op(v, dpp_mov<DPP_ROW_HALF_MIRROR>(v));
    if constexpr (N >= 16)
        v = op(v, dpp_mov<DPP_ROW_MIRROR>(v));
    if constexpr (N >= 32) {
        const auto p = __builtin_amdgcn_permlane16_swap(v, v, false, false);
        v = op((uint32_t)p[0], (uint32_t)p[1]);
    }
    if constexpr (N >= 64) {
        const auto p = __builtin_amdgcn_permlane32_swap(v, v, false, false);
        v = op((uint32_t)p[0], (uint32_t)p[1]);
    }
    return v;
}

struct XorOp {
    __device__ __forceinline__ uint32_t operator()(uint32_t a, uint32_t b) const { return a ^ b; }
};
struct MaxOp {
    __device__ __forceinline__ uint32_t operator()(uint32_t a, uint32_t b) const { return (uint32_t)max((int)a, (int)b); }
};

/* the GF(2^128) sum of a V4 over each N-lane group, in every lane of the group */
template <int N>
__device__ __forceinline__ V4 group_xor(V4 z)
{
    return V4{group_reduce<N>(z.w0, XorOp{}), group_reduce<N>(z.w1, XorOp{}), group_reduce<N>(z.w2, XorOp{}),
              group_reduce<N>(z.w3, XorOp{})};
}

__device__ __forceinline__ int wave_max(int v)
{
    return (int)group_reduce<64>((uint32_t)v, MaxOp{});
}

/* ======================================================================================= *
 *  batch seal / open                                                                       *
 * ======================================================================================= */

/* one GHASH element of a lane: which of AAD / ciphertext / length block it is */
struct Elem {
    bool active, is_aad, is_c, is_len;
    int i, c, nbytes;
};

/* element i of a record of N GHASH elements (na AAD blocks, nc data blocks, the length block), as seen by a task that
 * handles the elements below `hi` (N, or the end of a split record's first part) */
__device__ __forceinline__ Elem elem_of(int i, int N, int na, int nc, int L, int hi)
{
    Elem e;
    e.i = i;
    e.active = i < hi;
    e.is_aad = e.active && i < na;
    e.is_c = e.active && !e.is_aad && i < na + nc;
    e.is_len = e.active && i == N - 1;
    e.c = i - na;
    e.nbytes = e.is_c ? min(16, L - 16 * e.c) : 0;
    return e;
}

/* AAD_IN: an AAD element's block is already in in_blk (loaded before the AES, sparse kernel); WIDE_PARTIAL = false: a
 * partial block is stored byte by byte even when aligned (the plugin worker, whose registers the wider form spills) */
template <bool OPEN, bool ALIGNED, bool AAD_IN = false, bool WIDE_PARTIAL = true>
__device__ __forceinline__ V4 finish_elem(const Elem &e, V4 in_blk, V4 ks, const uint8_t *aad_p, int A, int L, uint8_t *out_p,
                                          V4 &ek0)
{
    V4 x = V4{0, 0, 0, 0};
    if (e.is_aad) {
        x = AAD_IN ? in_blk : load_block<ALIGNED>(aad_p + 16 * e.i, min(16, A - 16 * e.i));
    } else if (e.is_c) {
        const V4 o = v4xor(in_blk, ks);
        if (OPEN) {
            store_block<ALIGNED && WIDE_PARTIAL>(out_p + 16 * (size_t)e.c, e.nbytes, o);
            x = in_blk;
        } else {
            x = mask_block(o, e.nbytes);
            store_block<ALIGNED && WIDE_PARTIAL>(out_p + 16 * (size_t)e.c, e.nbytes, x);
        }
    } else if (e.is_len) { /* [len(A)]64 || [len(C)]64 in bits, big-endian (lib/fusion.c:468) */
        x = V4{0, bswap32((uint32_t)A << 3), 0, bswap32((uint32_t)L << 3)};
        ek0 = ks;
    }
    return x;
}

/* Pointers are separate __restrict__ kernel parameters (not a struct) so the compiler can prove that
 * the key slots, tables and descriptors are never written by the kernel and read them through the
 * scalar unit (s_load into SGPRs) instead of per-lane vector loads.  in/out may alias (in place). */
template <int G, int ROUNDS, bool OPEN, bool ALIGNED, int WGT>
__global__ void __launch_bounds__(WGT)
    aesgcm_batch_kernel(const ptls_hip_record_t *__restrict__ recs_ord, const uint32_t *__restrict__ order,
                        const Chunk *__restrict__ chunks, uint32_t nchunks,
                        const uint8_t *in, const uint8_t *__restrict__ aad, uint8_t *out, uint64_t *__restrict__ result,
                        const KeySlot *__restrict__ slots, const uint32_t *__restrict__ basis, const uint32_t *__restrict__ t0,
                        const ptls_hip_supp_t *__restrict__ supp, const KeySlot *__restrict__ hp_slots, uint32_t hp_nslots,
                        uint8_t *mask, uint64_t *__restrict__ clk, uint32_t *queue)
{
    constexpr int LOG2G = G == 1 ? 0 : G == 2 ? 1 : G == 4 ? 2 : G == 8 ? 3 : G == 16 ? 4 : 5;
    static_assert(G >= 1 && G <= 32 && (G & (G - 1)) == 0, "lanes per record: 1, 2, 4, 8, 16 or 32");
    /* the workgroup's task counter sits after the tables, then the chunk ring.  The chunks come from a device-wide counter
     * (queue[0]), one at a time, each claimed by the first of the workgroup's waves that needs it; the waves walk the same
     * chunk sequence, so the claimed chunk is left in an LDS ring for the others.  A workgroup that starts late (a CU still
     * held by another kernel) or runs at a lower clock (the CUs of one XCD do not all hold the same clock under load)
     * simply takes fewer chunks.  queue[1] counts the workgroups that have drawn past the end; the last one resets both
     * words for the next launch that gets this slot (engine.cpp queue_slot).  queue == nullptr: the static grid stride. */
    constexpr uint32_t LDS_QBASE = (lds_bytes(LOG2G) + 16 + 7u) & ~7u;
    constexpr int NW = WGT / 64;
    constexpr uint32_t LDS_QRING = LDS_QBASE;              /* uint64 [QRING]: position << 32 | chunk */
    constexpr uint32_t LDS_QCLAIM = LDS_QRING + QRING * 8; /* positions claimed so far */
    constexpr uint32_t LDS_QSEQ = LDS_QCLAIM + 4;          /* uint32 [NW]: positions each wave has entered */
    constexpr uint32_t LDS_TOTAL = LDS_QSEQ + NW * 4;
    static_assert(LDS_TOTAL <= 163840, "tables + task counter + chunk ring must fit the CU's 160 KiB");
    __shared__ __attribute__((aligned(16))) uint8_t lds[LDS_TOTAL];
    uint32_t *const task_ctr = reinterpret_cast<uint32_t *>(lds + lds_bytes(LOG2G));
    constexpr int R = 64 / G; /* records per wave task */

    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const bool use_q = queue != nullptr;
    if (use_q) {
        for (int k = (int)threadIdx.x; k < QRING; k += WGT)
            reinterpret_cast<uint64_t *>(lds + LDS_QRING)[k] = ~0ull;
        if (threadIdx.x < NW)
            reinterpret_cast<uint32_t *>(lds + LDS_QSEQ)[threadIdx.x] = 0;
        if (threadIdx.x == 0)
            *reinterpret_cast<uint32_t *>(lds + LDS_QCLAIM) = 0;
        __syncthreads();
    }
    /* the chunk at the wave's next position k of the workgroup's sequence (wave-uniform; lane 0 works, the wave waits), or
     * Q_END.  The wave's position lives in LDS (LDS_QSEQ), not in a register held across the record loop. */
    auto next_chunk = [&]() -> uint32_t {
        uint32_t c = 0;
        if (lane == 0) {
            uint32_t *const entered = reinterpret_cast<uint32_t *>(lds + LDS_QSEQ);
            const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x) >> 6;
            const uint32_t k = __hip_atomic_load(entered + wv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            /* published before the entry is read: a wave that has entered e positions still reads entry e - 1 */
            __hip_atomic_store(entered + wv, k + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            uint64_t *const ent = reinterpret_cast<uint64_t *>(lds + LDS_QRING) + (k % QRING);
            if (__hip_atomic_fetch_max(reinterpret_cast<uint32_t *>(lds + LDS_QCLAIM), k + 1, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_WORKGROUP) < k + 1) {
                /* this wave claims position k.  Its ring entry last held position k - QRING, which a wave still reads while
                 * it has entered at most k - QRING + 1 positions: wait for every wave to be past that (such a wave is
                 * working on a task of an earlier chunk, and walks on without waiting for this entry) */
                if (k >= (uint32_t)QRING)
                    for (;;) {
                        uint32_t lo = 0xffffffffu;
                        for (int w = 0; w < NW; ++w)
                            lo = min(lo, __hip_atomic_load(entered + w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
                        if (lo > k + 1 - (uint32_t)QRING)
                            break;
                        __builtin_amdgcn_s_sleep(2);
                    }
                c = __hip_atomic_fetch_add(queue, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (c >= nchunks) {
                    c = Q_END;
                    if (__hip_atomic_fetch_add(queue + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1) {
                        /* every workgroup has drawn past the end: no more adds to either word in this launch */
                        __hip_atomic_store(queue, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        __hip_atomic_store(queue + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    }
                }
                __hip_atomic_store(ent, (uint64_t)k << 32 | c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            } else {
                uint64_t v;
                while (((v = __hip_atomic_load(ent, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) >> 32) != k)
                    __builtin_amdgcn_s_sleep(2);
                c = (uint32_t)v;
            }
        }
        return __builtin_amdgcn_readfirstlane(c);
    };
    const uint32_t lb_aes = (uint32_t)(lane & 31) * 4u | LDS_AES;
    const GhLane gl = gh_lane_init(lane);
    const int r = lane & (G - 1);
    const int grp = lane >> LOG2G;

    clock_stamp(clk, 0);
    build_aes_tables<WGT>(lds, LDS_AES, t0);
    uint64_t ks_acc[16] = {}; /* KS_STAMPS: see its definition */
    const uint64_t ks_t0 = KS_STAMPS ? __builtin_amdgcn_s_memtime() : 0;
    uint64_t ks_last = ks_t0;
    auto ks_phase = [&](int k) __attribute__((always_inline)) { /* the cycles since the previous mark go to phase k */
        if (KS_STAMPS) {
            const uint64_t t = __builtin_amdgcn_s_memtime();
            ks_acc[k] += t - ks_last;
            ks_last = t;
        }
    };
    uint32_t cur_key = 0xffffffffu;
    /* g = the wave's next task in the workgroup's same-key run of chunks (drawn, not yet used); cbase = tasks of the run's
     * chunks before the current one */
    uint32_t g = 0, cbase = 0;
    bool have_g = false;

    for (uint32_t ci = use_q ? next_chunk() : blockIdx.x; ci < nchunks; ci = use_q ? next_chunk() : ci + gridDim.x) {
        const Chunk ch = chunks[ci];
        if (ch.key != cur_key) { /* a key switch: every wave is done with the old key's tables before they are rebuilt */
            const uint64_t s0 = KS_STAMPS ? __builtin_amdgcn_s_memtime() : 0;
            __syncthreads();
            const uint64_t s1 = KS_STAMPS ? __builtin_amdgcn_s_memtime() : 0;
            build_ghash_tables(lds, basis + (size_t)ch.key * (BASIS_VECS * 4), LOG2G);
            if (threadIdx.x == 0 && (DEAL_MUTANT != 3 || cur_key == 0xffffffffu))
                *task_ctr = 0;
            if (KS_STAMPS)
                __builtin_amdgcn_s_waitcnt(0); /* the wave's own table stores are done: what remains is waiting for others */
            const uint64_t s2 = KS_STAMPS ? __builtin_amdgcn_s_memtime() : 0;
            __syncthreads();
            if (KS_STAMPS) {
                const uint64_t s3 = __builtin_amdgcn_s_memtime();
                ks_acc[1] += s1 - s0;
                ks_acc[2] += s2 - s1;
                ks_acc[3] += s3 - s2;
                ks_acc[4] += 1;
                ks_last = s3;
            }
            cur_key = ch.key;
            cbase = 0;
            have_g = false; /* a task drawn past the old key's run belongs to no chunk */
        }
        if (DEAL_MUTANT == 1)
            have_g = false;

        const KeySlot *__restrict__ slot = slots + ch.key;
        const uint32_t *__restrict__ rk = slot->rk;
        const int ntasks = (int)((ch.count + R - 1) / R);

        /* A wave draws its next task when it finishes one, across the chunks of a same-key run, in order (records sorted
         * by decreasing length: longest first).  Waves on one SIMD do not progress equally (issue arbitration favours the
         * older wave), so a fixed deal would leave the slowest wave on the critical path. */
        for (;;) {
            if (!have_g) {
                uint32_t v = 0;
                if (lane == 0)
                    v = __hip_atomic_fetch_add(task_ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                g = __builtin_amdgcn_readfirstlane(v);
                have_g = true;
            }
            const int t = (int)(g - cbase);
            if (t >= ntasks)
                break; /* keep g for the next chunk of the run */
            have_g = false;
            ks_phase(5);
            const uint32_t ridx = (uint32_t)t * R + grp;
            const bool valid = ridx < ch.count;
            /* descriptors in chunk order: the record is one load away (its caller index only matters for
             * result[] and supp[] at the end) */
            const uint32_t pos = ch.first + (valid ? ridx : 0);
            const ptls_hip_record_t rec = recs_ord[pos];
            const uint32_t rec_i = order != nullptr ? order[pos] : pos; /* no order array: the plan keeps the caller's order */
            const int L = valid ? (int)rec.len : 0;
            const int A = valid ? (int)rec.aad_len : 0;
            const int na = (A + 15) >> 4, nc = (L + 15) >> 4;
            const int N = valid ? na + nc + 1 : 0;
            const int i0 = (r + na) & (G - 1);
            /* the lane's elements are i0 + m G for m < my_iters */
            const int my_iters = N > i0 ? ((N - 1 - i0) >> LOG2G) + 1 : 0;

            /* seal of a TLS 1.3 record: the last plaintext byte is the content type, not input */
            const bool tflag = !OPEN && (rec.flags & 1u) != 0 && L > 0;
            const uint32_t ttype = (rec.flags >> 8) & 0xffu;
            const uint8_t *in_p = in + rec.in_off;
            uint8_t *out_p = out + rec.out_off;
            const uint8_t *aad_p = aad + rec.aad_off;
            const uint32_t n0 = slot->iv[0], n1 = slot->iv[1] ^ bswap32((uint32_t)(rec.seq >> 32)),
                           n2 = slot->iv[2] ^ bswap32((uint32_t)rec.seq);

            V4 y = V4{0, 0, 0, 0}, ek0 = V4{0, 0, 0, 0};
            /* Iterations handle two Horner elements (i and i + G) of a lane; their AES blocks are independent
             * and run interleaved.  y = y * P ^ x is exact from y = 0 (0 * P = 0), so no first-element case. */
            /* counter-mode shortcut constants of this lane's record (rounds 1-2 of every block with counter < 2^16) */
            CtrConst cc; /* computed after the AAD elements (not held through them) */

            /* elements m and m + 1 of the lane (AAD, partial or full data, length block), their two AES blocks
             * interleaved; the counter-mode shortcut unless some lane of the wave has a counter >= 2^16 */
            auto generic_pair = [&](int m) {
                Elem e[2];
                V4 in[2], ks[2];
                uint32_t cw[2];
                int big = 0;
                int sft[2];
#pragma unroll
                for (int b = 0; b < 2; ++b) {
                    e[b] = elem_of(i0 + (m + b) * G, N, na, nc, L, N);
                    in[b] = V4{0, 0, 0, 0};
                    sft[b] = 0;
                    if (e[b].is_c) {
                        const bool tb = tflag && e[b].c == nc - 1; /* the block holding the content-type byte */
                        in[b] = tail_load(in_p + 16 * (size_t)e[b].c, e[b].c, e[b].nbytes - (tb ? 1 : 0), sft[b]);
                    }
                    /* keystream for data block c (counter inc32(J0) + c), E_K(J0) for the length-block lane */
                    cw[b] = e[b].is_c ? bswap32((uint32_t)e[b].c + 2u) : 0x01000000u;
                    ks[b] = V4{n0, n1, n2, cw[b]};
                    big |= (e[b].is_c && e[b].c >= 65534) ? 1 : 0;
                }
                const int bigw = wave_max(big);
                ks_phase(10);
                if (bigw != 0) { /* wave-wide, before any lane branches off */
                    aes_encrypt_n<ROUNDS, 2>(lds, lb_aes, rk, ks);
                } else {
                    const V4 nohash[2] = {V4{0, 0, 0, 0}, V4{0, 0, 0, 0}};
                    V4 ydummy = V4{0, 0, 0, 0};
                    ctr_ghash<ROUNDS, 2, false>(lds, lb_aes, rk, cc, cw, ks, ydummy, nohash, gl);
                }
                if (KS_STAMPS)
                    __builtin_amdgcn_s_waitcnt(0xc07f); /* lgkmcnt(0): the AES lookups are back */
                ks_phase(11);
                V4 xs[2];
#pragma unroll
                for (int b = 0; b < 2; ++b) {
                    in[b] = tail_shift(in[b], sft[b]);
                    if (tflag && e[b].is_c && e[b].c == nc - 1)
                        in[b] = put_byte(in[b], e[b].nbytes - 1, ttype);
                    xs[b] = finish_elem<OPEN, ALIGNED>(e[b], in[b], ks[b], aad_p, A, L, out_p, ek0);
                }
                if (KS_STAMPS)
                    __builtin_amdgcn_s_waitcnt(0); /* the loads finish_elem used are back */
                ks_phase(12);
#pragma unroll
                for (int b = 0; b < 2; ++b)
                    if (e[b].active)
                        y = gh_mul_main(lds, gl, y, xs[b]);
                if (KS_STAMPS)
                    __builtin_amdgcn_s_waitcnt(0);
                ks_phase(13);
            };

            auto generic_iter_m = [&](int m) {
                const Elem e0 = elem_of(i0 + m * G, N, na, nc, L, N);
                V4 in0 = V4{0, 0, 0, 0};
                int sft0 = 0;
                const bool tb0 = tflag && e0.is_c && e0.c == nc - 1; /* the block holding the content-type byte */
                if (e0.is_c)
                    in0 = tail_load(in_p + 16 * (size_t)e0.c, e0.c, e0.nbytes - (tb0 ? 1 : 0), sft0);
                /* keystream for data block c (counter inc32(J0) + c), E_K(J0) for the length-block lane */
                const uint32_t cw0[1] = {e0.is_c ? bswap32((uint32_t)e0.c + 2u) : 0x01000000u};
                V4 ks0[1] = {V4{n0, n1, n2, cw0[0]}};
                if (wave_max((e0.is_c && e0.c >= 65534) ? 1 : 0) == 0) {
                    const V4 nohash[1] = {V4{0, 0, 0, 0}};
                    V4 ydummy = V4{0, 0, 0, 0};
                    ctr_ghash<ROUNDS, 1, false>(lds, lb_aes, rk, cc, cw0, ks0, ydummy, nohash, gl);
                } else {
                    aes_encrypt_n<ROUNDS, 1>(lds, lb_aes, rk, ks0);
                }
                in0 = tail_shift(in0, sft0);
                if (tb0)
                    in0 = put_byte(in0, e0.nbytes - 1, ttype);
                const V4 x0 = finish_elem<OPEN, ALIGNED>(e0, in0, ks0[0], aad_p, A, L, out_p, ek0);
                if (e0.active)
                    y = gh_mul_main(lds, gl, y, x0);
            };

            /* "pure" stretch: elements m in [pm0, pm1) of every lane of the wave are full, aligned data blocks.
             * There the body is branch-free and handles KP blocks per iteration, so their AES lookups and the
             * GHASH lookups of the previous iteration's ciphertext can all be in flight together. */
            constexpr int KP = PURE_BLOCKS;
            const int nf = (L - (tflag ? 1 : 0)) >> 4; /* full blocks that are all input bytes */
            /* the lane's AAD elements (m < pm0) */
            const int pm0 = na > i0 ? (na - i0 + G - 1) >> LOG2G : 0;
            /* full blocks only, and (for the counter-mode shortcut) block counters c + 2 < 2^16 */
            const int lastc = min(nf, 65534) - 1; /* last data block index allowed in the pure stretch */
            const int my_mhi = min((valid && na + lastc - i0 >= 0) ? ((na + lastc - i0) >> LOG2G) + 1 : 0, my_iters);
            /* Each lane starts the stretch at its own first data element (after its AAD elements), so the lanes without AAD
             * do not spend a generic step on data block 0; the stretch length is the shortest lane's. */
            const int npure = -wave_max(-max(my_mhi - pm0, 0)) / KP;
            const int pm1 = pm0 + npure * KP; /* per lane: first element after the stretch */

            /* AAD elements: GHASH only (no keystream); y = 0 * P ^ x = x for the first one */
            const int naad = wave_max(pm0);
            for (int j = 0; j < naad; ++j) {
                if (j < pm0) {
                    const int ia = i0 + j * G;
                    const V4 x = ALIGNED ? load_block_nb(aad_p + 16 * ia, min(16, A - 16 * ia), reinterpret_cast<const uint8_t *>(t0))
                                         : load_block<false>(aad_p + 16 * ia, min(16, A - 16 * ia));
                    y = j == 0 ? x : gh_mul_main(lds, gl, y, x);
                }
            }
            cc = ctr_const(lds, lb_aes, rk, n0, n1, n2);
            ks_phase(6);
            if (npure) {
                const uint8_t *src = in_p + 16 * (size_t)(i0 - na + pm0 * G);
                uint8_t *dst = out_p + 16 * (size_t)(i0 - na + pm0 * G);
                const uint32_t cbase = (uint32_t)(i0 - na + pm0 * G) + 2u;
                V4 pend[KP], bufA[KP], bufB[KP];
                /* Deferred stores (seal of 16-byte aligned records whose output does not start on a 128-byte line).  An
                 * iteration writes KP G blocks of each record; with the record at block offset lo != 0 of a line, its last
                 * lo blocks fall into a line whose first 8 - lo blocks the NEXT iteration writes, a few microseconds later,
                 * and L2 wrote such lines back as two partial lines (16-byte packed QUIC records: seal 1.21x the
                 * algorithmic bytes).  Those lanes store the block one iteration late instead, with the rest of its line:
                 * the value is `pend`, the ciphertext the next iteration hashes, so no register is added.  A task whose
                 * records all start on a line (bench.py's layout) runs the plain loop: the choice is wave-uniform, taken
                 * once per task, and each loop is its own copy of the code.  Open is not deferred: holding its plaintext
                 * one iteration spills at 768 threads (EXPERIMENTS.md). */
                constexpr bool DEFER_OK = !OPEN && ALIGNED && KP * G >= 8;
                bool spill[KP];
                int defer_any = 0;
                {
                    const int lo = DEFER_OK ? (int)(((uint32_t)(uintptr_t)out_p >> 4) & 7u) : 0; /* the record's line offset */
                    const int jr = (i0 - na) & (G - 1); /* the lane's block position in an iteration's G-block group */
#pragma unroll
                    for (int b = 0; b < KP; ++b) {
                        spill[b] = DEFER_OK && lo != 0 && jr + b * G >= KP * G - lo;
                        defer_any |= spill[b] ? 1 : 0;
                    }
                }
                /* ping-pong prefetch: iteration `it` consumes the buffer loaded one iteration earlier and refills
                 * the other one for it + 1 (clamped to the last iteration so the body stays branch-free).  Two
                 * named buffers instead of a copy keep the compiler from waiting on the fresh loads. */
#pragma unroll
                for (int b = 0; b < KP; ++b)
                    bufA[b] = load_full(src + 16 * b * G);
                /* seal's store of output block b of iteration it (c): deferred by one iteration on spilling lanes (held:
                 * the previous iteration's block) */
                auto put = [&](auto defer_tag, int it, bool first, int b, const V4 &c, const V4 &held) __attribute__((always_inline)) {
                    constexpr bool DEFER = decltype(defer_tag)::value;
                    const size_t o = (size_t)(it * KP * G) * 16;
                    if (!DEFER) {
                        store_full(dst + o + 16 * b * G, c);
                    } else if (first) { /* iteration 0: a spilling block waits for the next iteration */
                        if (!spill[b])
                            store_full(dst + o + 16 * b * G, c);
                    } else { /* a spilling lane stores the previous iteration's block, the others this one's */
                        const size_t op = (size_t)((it - 1) * KP * G) * 16;
                        store_full(dst + (spill[b] ? op : o) + 16 * b * G, spill[b] ? held : c);
                    }
                };
                auto stretch = [&](auto defer_tag) __attribute__((always_inline)) {
                    constexpr bool DEFER = decltype(defer_tag)::value;
                    /* one branch-free iteration; `hash_pending` (false: iteration 0) is a literal at every call site */
                    auto pure_iter = [&](int it, bool hash_pending, V4(&d)[KP], V4(&dn)[KP]) __attribute__((always_inline)) {
                        const size_t on = (size_t)(min(it + 1, npure - 1) * KP * G) * 16;
                        V4 k[KP];
                        uint32_t cw[KP];
#pragma unroll
                        for (int b = 0; b < KP; ++b) {
                            dn[b] = load_full(src + on + 16 * b * G);
                            cw[b] = bswap32(cbase + (uint32_t)((it * KP + b) * G));
                            k[b] = V4{n0, n1, n2, cw[b]};
                        }
                        __builtin_amdgcn_sched_barrier(0); /* keep the prefetch at the top of the iteration */
                        if (OPEN) {
                            /* the input is the ciphertext: hash it in the same iteration */
                            ctr_ghash<ROUNDS, KP, true>(lds, lb_aes, rk, cc, cw, k, y, d, gl);
#pragma unroll
                            for (int b = 0; b < KP; ++b) {
                                store_full(dst + (size_t)(it * KP * G) * 16 + 16 * b * G, v4xor(d[b], k[b]));
                            }
                        } else {
                            /* software pipelined: the ciphertext of iteration it is hashed during iteration it + 1 */
                            if (hash_pending)
                                ctr_ghash<ROUNDS, KP, true>(lds, lb_aes, rk, cc, cw, k, y, pend, gl);
                            else
                                ctr_ghash<ROUNDS, KP, false>(lds, lb_aes, rk, cc, cw, k, y, pend, gl);
#pragma unroll
                            for (int b = 0; b < KP; ++b) {
                                const V4 c = v4xor(d[b], k[b]);
                                put(defer_tag, it, !hash_pending, b, c, pend[b]);
                                pend[b] = c;
                            }
                        }
                    };
                    pure_iter(0, false, bufA, bufB);
                    int it = 1;
                    for (; it + 1 < npure; it += 2) {
                        pure_iter(it, true, bufB, bufA);
                        pure_iter(it + 1, true, bufA, bufB);
                    }
                    if (it < npure)
                        pure_iter(it, true, bufB, bufA);
                    if (DEFER) { /* the last iteration's deferred blocks */
#pragma unroll
                        for (int b = 0; b < KP; ++b)
                            if (spill[b])
                                store_full(dst + (size_t)((npure - 1) * KP * G) * 16 + 16 * b * G, pend[b]);
                    }
                };
                if (DEFER_OK && wave_max(defer_any) != 0)
                    stretch(std::true_type{});
                else
                    stretch(std::false_type{});
                if (!OPEN) {
#pragma unroll
                    for (int b = 0; b < KP; ++b)
                        y = gh_mul_main(lds, gl, y, pend[b]);
                }
            }
            ks_phase(7);
            /* the rest of each lane's elements from its own position (full blocks past the shortest lane's
             * stretch, the partial block, the length block); an element past the record is inactive */
            {
                const int rest = wave_max(max(my_iters - pm1, 0));
                int j = 0;
                for (; j + 1 < rest; j += 2)
                    generic_pair(pm1 + j);
                if (j < rest)
                    generic_iter_m(pm1 + j);
            }

            /* combine the G partial sums of each record: position q = distance of a lane's last element from the end of
             * the GHASH input; sum_q y_q * H^(q+1).  G >= 2: each lane multiplies by its own power from the key's shared
             * window tables (build_ghash_tables), then an XOR butterfly over the record's G lanes leaves the GHASH in each;
             * G = 1: the lane's sum times H (the nibble table of H) */
            ks_phase(8);
            const int q = (N - 1 - na - r) & (G - 1); /* (nc - r) mod G */
            V4 s;
            if constexpr (G >= 2) {
                constexpr int WCP = win_copies(G);
                Win4<16, 16 * win_row(G)> wt;
                wt.base = LDS_GTREE + (uint32_t)(q * WCP + (grp & (WCP - 1))) * 16u;
                s = group_xor<G>(gf_win4_mul<16, 4>(lds, wt, y));
            }
            if (valid && q == 0) {
                if constexpr (G == 1)
                    s = gh_mul_nibble(lds, LDS_GTREE, y); /* * H */
                const V4 tag = v4xor(s, ek0);
                if (OPEN) {
                    const V4 rt = load_full(in_p + L);
                    const bool ok = rt.w0 == tag.w0 && rt.w1 == tag.w1 && rt.w2 == tag.w2 && rt.w3 == tag.w3;
                    result[rec_i] = ok ? (uint64_t)L : ~(uint64_t)0;
                } else {
                    store_full(out_p + L, tag);
                }
            }
            if (!OPEN && supp != nullptr) {
                /* QUIC header protection (fusion's supp, lib/fusion.c:636-650): AES-ECB(hp key, 16 output bytes)
                 * computed after the record, because the sample may cover the tag.  The sample was written by
                 * other lanes of this wave: the release/acquire pair completes their stores before the read.  Workgroup
                 * scope: one CU, one L1 (agent scope would write back and invalidate the XCD's whole L2). */
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
                if (valid && r == 0) {
                    const ptls_hip_supp_t sp = supp[rec_i];
                    if ((sp.flags & PTLS_HIP_SUPP_ENABLE) && sp.hp_key < hp_nslots) {
                        const V4 sample = load_full(out + sp.sample_off);
                        const V4 m = aes_encrypt<ROUNDS>(lds, lb_aes, hp_slots[sp.hp_key].rk, sample);
                        store_full(mask + sp.mask_off, m);
                    }
                }
            }
            ks_phase(9);
        }
        if (DEAL_MUTANT != 2)
            cbase += (uint32_t)ntasks;
    }
    if (KS_STAMPS && clk != nullptr) {
        ks_acc[0] = __builtin_amdgcn_s_memtime() - ks_t0;
        uint64_t *o = clk + 4 * (size_t)gridDim.x + 16 * ((size_t)blockIdx.x * NW + (size_t)wave);
#pragma unroll
        for (int k = 0; k < 16; ++k)
            if (lane == k)
                o[k] = ks_acc[k];
    }
    if (clk != nullptr) { /* the workgroup's end: after its last wave */
        __syncthreads();
        clock_stamp(clk, 1);
    }
}

template <int G, int R, bool O, int W>
static hipError_t launch_one(unsigned grid, hipStream_t s, const KernelArgs &a, bool aligned)
{
    /* KS_STAMPS builds write 16 words per wave after the 4 per workgroup: refuse a smaller stamp buffer */
    if (KS_STAMPS && a.clk != nullptr && a.clk_bytes < 8 * (4 * (size_t)grid + 16 * (size_t)grid * (W / 64)))
        return hipErrorInvalidValue;
    if (aligned)
        hipLaunchKernelGGL((aesgcm_batch_kernel<G, R, O, true, W>), dim3(grid), dim3(W), 0, s, a.recs_ord, a.order, a.chunks,
                           a.nchunks, a.in, a.aad, a.out, a.result, a.slots, a.basis, a.t0, a.supp, a.hp_slots, a.hp_nslots, a.mask, a.clk,
                           a.queue);
    else
        hipLaunchKernelGGL((aesgcm_batch_kernel<G, R, O, false, W>), dim3(grid), dim3(W), 0, s, a.recs_ord, a.order, a.chunks,
                           a.nchunks, a.in, a.aad, a.out, a.result, a.slots, a.basis, a.t0, a.supp, a.hp_slots, a.hp_nslots, a.mask, a.clk,
                           a.queue);
    return hipGetLastError();
}

template <int G, int R, bool O>
static hipError_t launch_w(int wg, unsigned grid, hipStream_t s, const KernelArgs &a, bool aligned)
{
    return wg == 512 ? launch_one<G, R, O, 512>(grid, s, a, aligned) : launch_one<G, R, O, WG_ALT>(grid, s, a, aligned);
}

/* every (rounds, open, workgroup, alignment) variant of lanes-per-record G */
template <int G>
static int launch_batch_g(int rounds, bool open, int wg, unsigned grid, hipStream_t s, const KernelArgs &a, bool al)
{
    hipError_t e;
    if (rounds == 10)
        e = open ? launch_w<G, 10, true>(wg, grid, s, a, al) : launch_w<G, 10, false>(wg, grid, s, a, al);
    else
        e = open ? launch_w<G, 14, true>(wg, grid, s, a, al) : launch_w<G, 14, false>(wg, grid, s, a, al);
    return (int)e;
}

} // namespace ptls_hip

#endif
