/*
 * sparse_kernel.hip -- AES-GCM seal/open for batches whose key slots hold very few records each
 * (a server sealing one record for each of many connections).  Same bytes as lib/fusion.c
 * (ptls_fusion_aesgcm_encrypt :400-658 / _decrypt :660-844), same record descriptors and chunk plan
 * as aesgcm_batch_kernel (batch_kernel.h), selected by the planner as "64 lanes per record".
 *
 * Why a second kernel: aesgcm_batch_kernel keeps ONE key's 8-bit GHASH window tables
 * in the workgroup's LDS, so each key switch costs a table build and two workgroup barriers, and a key
 * run of one record leaves 11 of 12 waves waiting (20 GiB/s at 65 536 records over 65 536 keys).
 * Here every wave works alone on one record at a time:
 *   - 64 lanes per record: lane l takes GHASH elements e = l, l + 64, ... (Horner with P = H^64);
 *   - each wave owns an 8 KiB 4-bit-window table of H^64 in LDS ([nibble position p][value v] = v at p
 *     times H^64), rebuilt per record from the key's basis H^64 * x^e (keysetup): 4 basis loads and 8
 *     ds_write_b128 per lane, no barrier (a wave's LDS operations complete in order).  A record of at most
 *     64 GHASH elements (one per lane) needs no Horner step and skips the build;
 *   - the combination: lane l multiplies its sum by its own power H^(q+1), q = (N - 1 - l) mod 64, read from
 *     keysetup's per-key H^1..H^128 list, with 4-bit windows over a per-lane table in the wave's LDS area
 *     (gf_mul_win4), and an XOR butterfly over the 64 lanes leaves the GHASH in every lane;
 *   - a Horner multiply is 32 ds_read_b128 (gh_mul_nibble); AES-CTR uses the batch kernel's 32x-replicated
 *     T-tables (64 KiB) and round keys through the scalar unit.  64 KiB + 12 x 8 KiB = the CU's 160 KiB.
 */
#include <type_traits>

#include "batch_kernel.h"
#include "gf128.h"

namespace ptls_hip {

constexpr int SPARSE_WG = 768;  /* 12 waves: 64 KiB AES tables + 12 x 8 KiB wave tables = 160 KiB */
constexpr int SPARSE_PE = 2;    /* GHASH elements (AES blocks) per lane per main-loop iteration */
constexpr int SPARSE_TAIL = 4;  /* the last nrecs / SPARSE_TAIL records (the shortest) come from the launch's queue word */
constexpr int SPARSE_WIN_LB = 8; /* lane combination: window lookups in flight per group (c4s seal +0.3 %, open +0.7 % over 4,
                                    profiles/r04_c4s_win_lb8_ab.log) */
#ifndef STAMP_PHASES
#define STAMP_PHASES 0 /* diagnostic build only (Makefile `diag`, tools/plugin_stamps.py): the single-record (plugin) launch
                          stamps the shader clock at its phase boundaries into clk[0 .. 11] (clk[14], clk[15]: the 100 MHz
                          counter at the first and last stamp).  Its run times are not quoted, only its phase shares. */
#endif
constexpr uint32_t SP_TAB = 65536; /* per-wave nibble tables, 8 KiB each */

/* batch launches (STAMP_PHASES builds): wave 0 of workgroup 0 sums the cycles of phases 2 .. 8 over its records */
struct PhaseAcc {
    uint64_t last, acc[9], n;
};

__device__ __forceinline__ void phase_acc(PhaseAcc &pa, bool on, int k)
{
#if STAMP_PHASES
    if (on) {
        uint64_t t;
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
        __builtin_amdgcn_sched_barrier(0);
        if (k > 1)
            pa.acc[k] += t - pa.last;
        else
            ++pa.n;
        pa.last = t;
    }
#else
    (void)pa, (void)on, (void)k;
#endif
}

/* phase stamp k of the by-value record's wave (STAMP_PHASES builds; the stamp and its LDS drain in one statement) */
__device__ __forceinline__ void phase_stamp(uint64_t *__restrict__ clk, bool on, int lane, int k)
{
#if STAMP_PHASES
    if (on && clk != nullptr) {
        uint64_t t;
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
        __builtin_amdgcn_sched_barrier(0);
        if (lane == 0)
            clk[k] = t;
        if (k == 0 || k == 11) {
            const uint64_t r = __builtin_amdgcn_s_memrealtime();
            __builtin_amdgcn_s_waitcnt(0xC07F);
            if (lane == 0)
                clk[k == 0 ? 14 : 15] = r;
        }
    }
#else
    (void)clk, (void)on, (void)lane, (void)k;
#endif
}

/* the wave's LDS operations are processed in order: only the compiler must not move them across this */
__device__ __forceinline__ void wave_lds_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

/* the wave's nibble table of P (bp[e] = P * x^e, GCM bit e = byte e/8, bit 7 - e%8) at LDS offset tab,
 * laid out as gh_mul_nibble reads it: entry [p = 8w + j][v] = v at bits 4j..4j+3 of raw word w, times P.
 * Lane l writes position l/2, values 8(l&1) .. 8(l&1) + 7: load_wave_basis fetches the lane's four basis
 * vectors (issued early to hide their latency), store_wave_table writes the eight combinations. */
/* v * x in GF(2^128), GCM bit order, raw byte order words: the 128-bit big-endian string shifted right by one bit,
 * R = 0xE1 || 0^120 folded in when the last bit drops out (SP 800-38D) */
__device__ __forceinline__ V4 mulx_raw(V4 v)
{
    const uint32_t a0 = bswap32(v.w0), a1 = bswap32(v.w1), a2 = bswap32(v.w2), a3 = bswap32(v.w3);
    const uint32_t c = 0u - (a3 & 1u);
    return V4{bswap32((a0 >> 1) ^ (c & 0xe1000000u)), bswap32(__builtin_amdgcn_alignbit(a0, a1, 1)),
              bswap32(__builtin_amdgcn_alignbit(a1, a2, 1)), bswap32(__builtin_amdgcn_alignbit(a2, a3, 1))};
}

/* v * x^r for a per-lane r <= 31 (gf128.h's gf_mul_xpow31 on the raw words) */
__device__ __forceinline__ V4 mulxpow_raw(V4 v, uint32_t r)
{
    const U128 p{(uint64_t)bswap32(v.w0) << 32 | bswap32(v.w1), (uint64_t)bswap32(v.w2) << 32 | bswap32(v.w3)};
    const U128 z = gf_mul_xpow31(p, r);
    return V4{bswap32((uint32_t)(z.hi >> 32)), bswap32((uint32_t)z.hi), bswap32((uint32_t)(z.lo >> 32)), bswap32((uint32_t)z.lo)};
}

/* the lane's smallest exponent e0 - 3 = 32 w + r (below): its offset r inside the lane's 32-vector group */
__device__ __forceinline__ uint32_t basis_r(int lane)
{
    const int j = (lane >> 1) & 7;
    return (uint32_t)(8 * (j >> 1) + 4 - 4 * (j & 1));
}

__device__ __forceinline__ void load_wave_basis(const uint4 *__restrict__ bp, int lane, V4 (&b)[4])
{
    asm volatile("" : "+v"(lane)); /* the lane's basis offset computed here, not hoisted out of the record loop (scratch) */
    /* the lane's four vectors are P x^(e0), P x^(e0 - 1), P x^(e0 - 2), P x^(e0 - 3) for one e0 (bits 4j .. 4j + 3 of
     * word w lie in one byte): e0 - 3 = 32 w + basis_r(lane).  The lane loads P x^(32 w), one of four vectors (four cache
     * lines per record); store_wave_table derives the rest on the VALU (round 4: 32 vectors over 16 lines before) */
    const int w = (lane >> 1) >> 3;
    const uint4 v = bp[32 * w];
    b[3] = V4{v.x, v.y, v.z, v.w};
}

__device__ __forceinline__ void store_wave_table(uint8_t *lds, uint32_t tab, V4 (&b)[4], int lane)
{
    {
        int ln = lane;
        asm volatile("" : "+v"(ln));
        b[3] = mulxpow_raw(b[3], basis_r(ln));
    }
    b[2] = mulx_raw(b[3]);
    b[1] = mulx_raw(b[2]);
    b[0] = mulx_raw(b[1]);
    asm volatile("" : "+v"(lane)); /* the entries' masks and slots are computed here, not hoisted out of the record loop
                                      (32 lane-invariant values live across the kernel: scratch beside the lane combination) */
    const int p = lane >> 1;
    const V4 hi = (lane & 1) ? b[3] : V4{0, 0, 0, 0};
    const uint32_t row = tab + (uint32_t)p * 256u + (uint32_t)(lane & 1) * 128u;
    /* the 8 lanes of a ds_write_b128 group write rows 128 B apart, i.e. the same banks: each lane walks its eight
     * entries from its own start ((k + lane) & 7), so the group's eight addresses fall in eight distinct 16-B bank
     * quads (conflict-free); the entry's basis combination follows its low three value bits as masks */
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const uint32_t v = (uint32_t)(k + lane) & 7u;
        const uint32_t m0 = 0u - (v & 1u), m1 = 0u - ((v >> 1) & 1u), m2 = 0u - (v >> 2);
        const uint32_t hw[4] = {hi.w0, hi.w1, hi.w2, hi.w3};
        uint32_t e[4];
#pragma unroll
        for (int w = 0; w < 4; ++w) {
            const uint32_t b0 = w == 0 ? b[0].w0 : w == 1 ? b[0].w1 : w == 2 ? b[0].w2 : b[0].w3;
            const uint32_t b1 = w == 0 ? b[1].w0 : w == 1 ? b[1].w1 : w == 2 ? b[1].w2 : b[1].w3;
            const uint32_t b2 = w == 0 ? b[2].w0 : w == 1 ? b[2].w1 : w == 2 ? b[2].w2 : b[2].w3;
            uint32_t z = __builtin_amdgcn_bitop3_b32(hw[w], m0, b0, 0x78); /* z ^ (m & b) */
            z = __builtin_amdgcn_bitop3_b32(z, m1, b1, 0x78);
            e[w] = __builtin_amdgcn_bitop3_b32(z, m2, b2, 0x78);
        }
        lds128_store(lds, row + v * 16u, V4{e[0], e[1], e[2], e[3]});
    }
}

/* the wave's maximum / XOR sum in every lane: batch_kernel.h's DPP + permlane reduction (no LDS instruction, no partner
 * address; until round 4 a ds_bpermute butterfly whose partner addresses had to come from an opaque lane index, or the
 * compiler hoisted them out of the record loop into scratch) */
__device__ __forceinline__ int wave_max_sp(int v)
{
    return wave_max(v);
}

__device__ __forceinline__ V4 wave_xor(V4 z)
{
    return group_xor<64>(z);
}

/* sum over the wave of (lane's GHASH sum) * H^(q+1): one multiply by the lane's own power (keysetup's H^1..H^128 list),
 * then the XOR butterfly; every lane ends with the total.  The multiply's table is the lane's 8 multiples of H^(q+1) in
 * the wave's own 8 KiB table area (the H^64 Horner table is dead by now). */
__device__ __forceinline__ V4 ghash_combine(uint8_t *lds, uint32_t tab, int lane, const uint4 *__restrict__ bs, int q, V4 y)
{
    /* q made opaque here: the power's load and the table arithmetic stay after the record's elements instead of being
     * hoisted above the stretch (where their registers pushed the batch instantiations into scratch) */
    asm volatile("" : "+v"(q));
    const uint4 hp = bs[NPOW * 128 + q]; /* H^(q+1) */
    return wave_xor(gf_mul_win4<8, SPARSE_WIN_LB>(lds, tab, lane, y, V4{hp.x, hp.y, hp.z, hp.w}));
}

/* One record on one wave (the sparse-key kernel's per-record body, also the plugin worker's): its counter-mode
 * constants, its per-wave H^64 table, the elements (generic head / branch-free stretch / generic tail), the lane
 * combination, the tag, header protection.  pre / prefetch: a single record's first two elements per lane, read before
 * (BYVAL: the plugin's launch and the worker). */
template <int ROUNDS, bool OPEN, bool ALIGNED, bool BYVAL, int S = 64, int KPE = SPARSE_PE, bool SPLIT = false>
__device__ __forceinline__ void sparse_record(uint8_t *lds, int lane, uint32_t lb_aes, uint32_t tab, const ptls_hip_record_t &rec,
                                              uint32_t rec_i, const uint8_t *in, const uint8_t *__restrict__ aad, uint8_t *out,
                                              uint64_t *__restrict__ result, const KeySlot *__restrict__ slots,
                                              const uint32_t *__restrict__ basis, const ptls_hip_supp_t *__restrict__ supp,
                                              const KeySlot *__restrict__ hp_slots, uint32_t hp_nslots, uint8_t *mask, bool prefetch,
                                              const V4 (&pre)[2], uint64_t *__restrict__ clk, bool stamps, bool bstamps, PhaseAcc &pa,
                                              uint32_t ctab, int vw = 0, uint32_t xslot = 0, uint4 ivo = uint4{0, 0, 0, 0},
                                              int e0 = 0, int hi_split = 0, uint32_t xsplit = 0)
{
    /* S = 64: one wave per record (lane l: elements l + 64 m, Horner with H^64).  S = 128 (a single long record on two
     * waves, vw = this wave's index 0 / 1): the two waves act as one 128-lane wave, virtual lane vl = 64 vw + l takes
     * elements vl + 128 m with Horner by H^128 (basis plane 7) and multiplies its sum by H^(q+1), q = (N - 1 - vl) mod 128
     * (keysetup's list); wave 0's sum joins wave 1's through LDS (xslot) after a workgroup barrier, and the wave holding
     * the length block (q = 0) writes the tag.  Every element index below goes through vl and S.
     * SPLIT (S = 128, a long record on four waves): two such pairs, each on its own part of the record, elements
     * [e0, hi_split): pair 0 takes [0, P), pair 1 [P, N).  A lane's last element e is N - e elements from the end:
     * q_l + 1 + D with q_l = (hi - 1 - e0 - vl) mod 128 its distance from the end of its part and D = N - hi = 128 k + r
     * (0 in pair 1).  The lane weighs its sum by H^(((q_l + r) mod 128) + 1), times H^128 when q_l + r >= 128 (folded
     * into its combination table, built once the H^128 table exists); pair 0's combined sum then takes k Horner steps with the H^128 table and goes to pair 1's tag wave
     * through LDS (xsplit) after a second workgroup barrier. */
    static_assert(S == 64 || S == 128, "stride: one or two waves");
    constexpr int LOG2S = S == 64 ? 6 : 7;
    constexpr bool by_value = BYVAL;
    (void)by_value, (void)clk, (void)stamps, (void)bstamps, (void)pa;
    /* everything derived from the lane index is computed per record: hoisted out of the kernel's record loop, such values
     * (partner lanes, table slots, negative lane offsets) stayed live across the whole kernel and went to scratch, which
     * the streaming records then evicted to HBM (c4s: 84 B per lane, +4.9 KB of HBM traffic per record) */
    /* recomputed, not carried across records: a volatile asm, because the compiler hoists the mbcnt builtins out of the
     * record loop and under the register pressure spilled their value, one scratch reload and wait per record (round 4) */
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(lane));
    const int vl = 64 * vw + lane; /* the virtual lane (S = 64: the lane) */
    static_assert(!SPLIT || S == 128, "a split record: two pairs of waves at stride 128");
    const uint32_t key = __builtin_amdgcn_readfirstlane(rec.key);
    const KeySlot *__restrict__ slot = slots + key;
    const uint32_t *__restrict__ rk = slot->rk;
    const uint4 *__restrict__ bs = reinterpret_cast<const uint4 *>(basis) + (size_t)key * BASIS_VECS;
    const int L = (int)__builtin_amdgcn_readfirstlane(rec.len);
    const int A = (int)__builtin_amdgcn_readfirstlane(rec.aad_len);
    const int na = (A + 15) >> 4, nc = (L + 15) >> 4;
    const int N = na + nc + 1;
    const bool tflag = !OPEN && (rec.flags & 1u) != 0 && L > 0;
    const uint32_t ttype = (rec.flags >> 8) & 0xffu;
    const uint8_t *in_p = in + rec.in_off;
    uint8_t *out_p = out + rec.out_off;
    const uint8_t *aad_p = aad + rec.aad_off;
    const int hi = SPLIT ? hi_split : N;      /* the end of this wave's part of the record (exclusive) */
    const int vle = vl + (SPLIT ? e0 : 0);    /* the lane's first element */
    const bool last_part = !SPLIT || hi == N; /* holds the length block (the tag) */
    /* ivo.w != 0: the static IV travels in the request (the plugin worker: an IV change never writes device memory) */
    const bool ov = __builtin_amdgcn_readfirstlane(ivo.w) != 0;
    const uint32_t n0 = __builtin_amdgcn_readfirstlane(ov ? ivo.x : slot->iv[0]),
                   n1 = __builtin_amdgcn_readfirstlane((ov ? ivo.y : slot->iv[1]) ^ bswap32((uint32_t)(rec.seq >> 32))),
                   n2 = __builtin_amdgcn_readfirstlane((ov ? ivo.z : slot->iv[2]) ^ bswap32((uint32_t)rec.seq));
    const int iters = (hi - (SPLIT ? e0 : 0) + S - 1) >> LOG2S;
    const bool horner = iters > 1 || SPLIT; /* N <= S: one element per lane, no Horner step (SPLIT: pair 0's H^128 steps) */
    V4 b[4];
    /* a single record (the plugin's launch): the H^64 basis loads go out before the counter-mode constants, so their
     * memory latency overlaps that LDS chain (in batches other waves hide it; there the early loads cost c4s open
     * 2.5 %, measured) */
    const int ql = (hi - 1 - vle) & (S - 1);
    const int rsp = SPLIT ? (N - hi) & (S - 1) : 0;  /* r above (0 in pair 1 and without SPLIT) */
    const int q = (ql + rsp) & (S - 1);
    const bool qwrap = SPLIT && ql + rsp >= S;     /* the lane's extra H^128 step */
    /* batch records: the lane's first AAD block is loaded here, before the counter-mode constants and the H^64 table, so
     * its latency runs under that work (c4s seal 498-504 -> 513-519 GiB/s, profiles/r04_c4s_prefetch_ab.log) */
    V4 aad_pf = V4{0, 0, 0, 0};
    if (!BYVAL && ALIGNED)
        aad_pf = load_block_nb(vl < na ? aad_p + 16 * vl : reinterpret_cast<const uint8_t *>(slot->rk), vl < na ? min(16, A - 16 * vl) : 0,
                               reinterpret_cast<const uint8_t *>(slot->rk));
    else if (!BYVAL && vl < na)
        aad_pf = load_block<ALIGNED>(aad_p + 16 * vl, min(16, A - 16 * vl));
    (void)aad_pf;
    /* SPLIT, pair 1 (no AAD block, nothing read with the request): its first two stretch blocks go out before the
     * counter-mode constants and the tables, as pair 0's came with the request */
    const bool spre = SPLIT && !prefetch && (SPLIT ? e0 : 0) >= na;
    V4 pre1[2] = {V4{0, 0, 0, 0}, V4{0, 0, 0, 0}};
    if (spre) {
        const int lastc1 = min(min((L - (tflag ? 1 : 0)) >> 4, 65534) - 1, hi - 1 - na);
#pragma unroll
        for (int k = 0; k < 2; ++k)
            if (vle - na + S * k <= lastc1)
                pre1[k] = load_full(in_p + 16 * (size_t)(vle - na + S * k));
    }
    /* a single record builds its lane-combination table (the 16 multiples of H^(q+1)) early, in an LDS area of its own
     * (ctab), so that only the lookups remain after its last element */
    constexpr bool early_win = BYVAL;
    uint4 hpe = uint4{0, 0, 0, 0};
    if (early_win)
        hpe = bs[NPOW * 128 + q]; /* H^(q+1) */
    if (horner && by_value)
        load_wave_basis(bs + LOG2S * 128, lane, b); /* H^S */
    /* the record (and so its counter-mode constants) is the wave's alone: keep them in SGPRs */
    CtrConst cc = ctr_const(lds, lb_aes, rk, n0, n1, n2);
    cc.k10 = __builtin_amdgcn_readfirstlane(cc.k10);
    cc.k11 = __builtin_amdgcn_readfirstlane(cc.k11);
    cc.k20 = __builtin_amdgcn_readfirstlane(cc.k20);
    cc.k21 = __builtin_amdgcn_readfirstlane(cc.k21);
    cc.k22 = __builtin_amdgcn_readfirstlane(cc.k22);
    cc.k23 = __builtin_amdgcn_readfirstlane(cc.k23);
    cc.r03 = __builtin_amdgcn_readfirstlane(cc.r03);
    Win4<16> w4{};
    if (early_win && !SPLIT)
        w4 = gf_win4_build<16>(lds, ctab, lane, V4{hpe.x, hpe.y, hpe.z, hpe.w});
    (void)w4, (void)ctab;
    phase_stamp(clk, stamps, lane, 2);
    phase_acc(pa, bstamps, 2);
    wave_lds_sync(); /* the previous record's Horner reads of the table are done */
    if (horner) { /* (loading the basis during the previous record's VALU combine measured no faster: other waves hide it) */
        if (!by_value)
            load_wave_basis(bs + LOG2S * 128, lane, b); /* H^S */
        store_wave_table(lds, tab, b, lane);
    }
    wave_lds_sync();
    if (early_win && SPLIT) { /* the lane's power times H^128 where q_l + r wrapped (the H^128 table exists now) */
        const V4 hp = V4{hpe.x, hpe.y, hpe.z, hpe.w}, hs = gh_mul_nibble(lds, tab, hp);
        w4 = gf_win4_build<16>(lds, ctab, lane, qwrap ? hs : hp);
        wave_lds_sync();
    }
    phase_stamp(clk, stamps, lane, 3);
    phase_acc(pa, bstamps, 3);

    V4 y = V4{0, 0, 0, 0}, ek0 = V4{0, 0, 0, 0};
    /* generic elements m .. m + NE - 1 of the lane (past `mend`: skipped): partial / AAD / length blocks and
     * counters >= 2^16, their AES blocks interleaved (counter-mode shortcut unless a counter is that large) */
    auto generic = [&](auto ne_tag, auto pre_tag, int m, int mend) __attribute__((always_inline)) {
        constexpr int NE = decltype(ne_tag)::value;
        constexpr bool USE_PRE = decltype(pre_tag)::value; /* the head range only: pre is dead after it */
        Elem e[NE];
        V4 inb[NE], ks[NE];
        uint32_t cw[NE];
        int sft[NE];
        int big = 0;
#pragma unroll
        for (int b = 0; b < NE; ++b) {
            e[b] = elem_of(m + b < mend ? vle + (m + b) * S : N, N, na, nc, L, hi);
            inb[b] = V4{0, 0, 0, 0};
            sft[b] = 0;
            /* the lane's first two elements of a single record were read at the start (pre) */
            const bool have_pre = USE_PRE && prefetch && m + b < 2;
            const V4 pv = m + b == 0 ? pre[0] : pre[1];
            if (e[b].is_c) {
                const bool tb = tflag && e[b].c == nc - 1; /* the block holding the content-type byte */
                const int nb = e[b].nbytes - (tb ? 1 : 0);
                /* batch records: one 16-byte load ending at the block's last byte, shifted down after the AES (batch_kernel.h
                 * tail_load: no load result is combined inside a branch, so the wave does not wait before its AES) */
                if (have_pre)
                    inb[b] = mask_block(pv, nb);
                else if (!BYVAL)
                    inb[b] = tail_load(in_p + 16 * (size_t)e[b].c, e[b].c, nb, sft[b]);
                else
                    inb[b] = load_block<ALIGNED>(in_p + 16 * (size_t)e[b].c, nb);
            } else if (e[b].is_aad) { /* loaded before the AES as well, not after it in finish_elem */
                const int nb = min(16, A - 16 * e[b].i);
                inb[b] = have_pre ? mask_block(pv, nb) : load_block<ALIGNED>(aad_p + 16 * e[b].i, nb);
            }
            /* keystream for data block c (counter inc32(J0) + c), E_K(J0) for the length-block lane */
            cw[b] = e[b].is_c ? bswap32((uint32_t)e[b].c + 2u) : 0x01000000u;
            ks[b] = V4{n0, n1, n2, cw[b]};
            big |= (e[b].is_c && e[b].c >= 65534) ? 1 : 0;
        }
        if (wave_max_sp(big)) {
            aes_encrypt_n<ROUNDS, NE>(lds, lb_aes, rk, ks);
        } else {
            const V4 nohash[NE] = {};
            V4 ydummy = V4{0, 0, 0, 0};
            ctr_ghash_skewed<ROUNDS, NE, false>(lds, lb_aes, rk, cc, cw, ks, ydummy, nohash, GhNibble{tab});
        }
#pragma unroll
        for (int b = 0; b < NE; ++b) {
            if (e[b].is_c) {
                inb[b] = tail_shift(inb[b], sft[b]);
                if (tflag && e[b].c == nc - 1)
                    inb[b] = put_byte(inb[b], e[b].nbytes - 1, ttype);
            }
            const V4 x = finish_elem<OPEN, ALIGNED, true, !BYVAL>(e[b], inb[b], ks[b], aad_p, A, L, out_p, ek0);
            if (m + b == 0)
                y = x; /* 0 * P ^ x */
            else if (e[b].active)
                y = v4xor(gh_mul_nibble(lds, tab, y), x); /* y * H^64 ^ x */
        }
    };
    auto generic_range = [&](auto pre_tag, int m0, int m1) __attribute__((always_inline)) {
        int m = m0;
        for (; m + 1 < m1; m += 2)
            generic(std::integral_constant<int, 2>{}, pre_tag, m, m1);
        if (m < m1)
            generic(std::integral_constant<int, 1>{}, pre_tag, m, m1);
    };

    /* the wave's "pure" elements m in [pm0, pm1): every lane's element is a full data block with a counter below
     * 2^16 (lane l, element m = data block 64 m + l - na).  There the body is branch-free, KP blocks per lane per
     * iteration, the counter-mode AES of the blocks skewed against the H^64 multiplies of the previous iteration's
     * ciphertext (seal) or of the input ciphertext (open), the next iteration's plaintext prefetched. */
    constexpr int KP = KPE;
    const int nf = (L - (tflag ? 1 : 0)) >> 4;              /* full blocks that are all input bytes */
    const int lastc = min(min(nf, 65534) - 1, hi - 1 - na); /* last data block allowed in the stretch (of this part) */
    /* Each lane starts the stretch at its own first data element (m = 1 on the lanes holding the AAD block, 0 on the
     * others) and ends where its blocks stop being full: the stretch is the shortest lane's, the AAD elements before
     * it are hashed only, and the record's generic head (one full AES per lane for one AAD block, 17 % of a c4s
     * record, tools/sparse_stamps.py) is gone. */
    const int ml = vle < na ? (na - vle + S - 1) >> LOG2S : 0;                      /* the lane's first data element */
    const int mhl = lastc + na - vle >= 0 ? ((lastc + na - vle) >> LOG2S) + 1 : 0;  /* its elements m < mhl: full blocks */
    const int fmin = -wave_max_sp(-max(mhl - ml, 0)); /* full-block elements every lane has */
    const int npure = fmin / KP;
    /* an odd full element left over by the KP-block iterations takes one single-block step of the stretch instead of the
     * generic path */
    const int npx = npure > 0 && fmin - npure * KP > 0 ? 1 : 0;
    const int iters_l = vle < hi ? ((hi - 1 - vle) >> LOG2S) + 1 : 0;            /* the lane's elements */
    const int pm1 = ml + npure * KP + npx;                                        /* the lane's first after the stretch */
    if (!npure) { /* head and tail are one range: elements share one round trip to the record's memory (the plugin) */
        generic_range(std::integral_constant<bool, BYVAL>{}, 0, iters);
    } else { /* the lane's AAD elements: GHASH only */
        const int naad = wave_max_sp(ml);
        for (int j = 0; j < naad; ++j) {
            if (j < ml) {
                const int i = vle + S * j;
                const int nb = min(16, A - 16 * i);
                const V4 x = (BYVAL && prefetch && j < 2)       ? mask_block(j == 0 ? pre[0] : pre[1], nb)
                             : (!BYVAL && j == 0)                ? aad_pf
                                                                  : load_block<ALIGNED>(aad_p + 16 * i, nb);
                y = j == 0 ? x : v4xor(gh_mul_nibble(lds, tab, y), x);
            }
        }
    }
    phase_stamp(clk, stamps, lane, 4);
    phase_acc(pa, bstamps, 4);
    if (npure) {
        const int c0 = S * ml + vle - na; /* the lane's first data block of the stretch */
        const uint8_t *src = in_p + 16 * (size_t)c0;
        uint8_t *dst = out_p + 16 * (size_t)c0;
        V4 pend[KP], bufA[KP], bufB[KP];
        /* open hashes its input in the iteration that loads it: the next iteration's blocks are prefetched into the
         * other buffer.  Seal uses its plaintext only after the iteration's AES, so it loads at the top of the
         * iteration into one buffer (8 VGPRs fewer: the seal instantiations stay within 168 without scratch). */
#pragma unroll
        for (int b = 0; b < KP; ++b)
            bufA[b] = spre && b < 2 ? pre1[b < 2 ? b : 0] : load_full(src + 16 * S * b);
        auto pure_iter = [&](int it, bool hash_pending, V4(&d)[KP], V4(&dn)[KP]) __attribute__((always_inline)) {
            const size_t o = (size_t)it * KP * 16 * S;
            const size_t on = (size_t)min(it + 1, npure - 1) * KP * 16 * S;
            V4 k[KP];
            uint32_t cw[KP];
#pragma unroll
            for (int b = 0; b < KP; ++b) {
                if (OPEN)
                    dn[b] = load_full(src + on + 16 * S * b);
                else if (it != 0)
                    d[b] = load_full(src + o + 16 * S * b);
                cw[b] = bswap32((uint32_t)(c0 + 2 + (it * KP + b) * S));
                k[b] = V4{n0, n1, n2, cw[b]};
            }
            __builtin_amdgcn_sched_barrier(0); /* keep the loads at the top of the iteration */
            if (OPEN) {
                ctr_ghash_skewed<ROUNDS, KP, true>(lds, lb_aes, rk, cc, cw, k, y, d, GhNibble{tab});
#pragma unroll
                for (int b = 0; b < KP; ++b)
                    store_full(dst + o + 16 * S * b, v4xor(d[b], k[b]));
            } else {
                if (hash_pending)
                    ctr_ghash_skewed<ROUNDS, KP, true>(lds, lb_aes, rk, cc, cw, k, y, pend, GhNibble{tab});
                else
                    ctr_ghash_skewed<ROUNDS, KP, false>(lds, lb_aes, rk, cc, cw, k, y, pend, GhNibble{tab});
#pragma unroll
                for (int b = 0; b < KP; ++b) {
                    pend[b] = v4xor(d[b], k[b]);
                    store_full(dst + o + 16 * S * b, pend[b]);
                }
            }
        };
        /* the single-block step (npx): data block c0 + npure KP S of the lane */
        const size_t ox = (size_t)npure * KP * 16 * S;
        uint32_t cwx[1] = {bswap32((uint32_t)(c0 + 2 + npure * KP * S))};
        if (OPEN) {
            pure_iter(0, false, bufA, bufB);
            int it = 1;
            for (; it + 1 < npure; it += 2) {
                pure_iter(it, true, bufB, bufA);
                pure_iter(it + 1, true, bufA, bufB);
            }
            if (it < npure)
                pure_iter(it, true, bufB, bufA);
            if (npx) { /* hashes its own input ciphertext, as the iterations do */
                const V4 dx[1] = {load_full(src + ox)};
                V4 kx[1] = {V4{n0, n1, n2, cwx[0]}};
                ctr_ghash_skewed<ROUNDS, 1, true>(lds, lb_aes, rk, cc, cwx, kx, y, dx, GhNibble{tab});
                store_full(dst + ox, v4xor(dx[0], kx[0]));
            }
        } else {
            pure_iter(0, false, bufA, bufA);
            for (int it = 1; it < npure; ++it)
                pure_iter(it, true, bufA, bufA);
            if (npx) { /* the last iteration's ciphertext blocks hashed here but its last, which goes under the step's AES */
                const V4 dx = load_full(src + ox);
#pragma unroll
                for (int b = 0; b + 1 < KP; ++b)
                    y = v4xor(gh_mul_nibble(lds, tab, y), pend[b]);
                const V4 hx[1] = {pend[KP - 1]};
                V4 kx[1] = {V4{n0, n1, n2, cwx[0]}};
                ctr_ghash_skewed<ROUNDS, 1, true>(lds, lb_aes, rk, cc, cwx, kx, y, hx, GhNibble{tab});
                const V4 cx = v4xor(dx, kx[0]);
                store_full(dst + ox, cx);
                y = v4xor(gh_mul_nibble(lds, tab, y), cx);
            } else {
#pragma unroll
                for (int b = 0; b < KP; ++b)
                    y = v4xor(gh_mul_nibble(lds, tab, y), pend[b]);
            }
        }
    }
    phase_stamp(clk, stamps, lane, 5);
    phase_acc(pa, bstamps, 5);
    if (npure) { /* the rest of each lane's elements from its own position (partial, length and leftover blocks) */
        const int rest = wave_max_sp(max(iters_l - pm1, 0));
        int j = 0;
        for (; j + 1 < rest; j += 2)
            generic(std::integral_constant<int, 2>{}, std::false_type{}, pm1 + j, iters_l);
        if (j < rest)
            generic(std::integral_constant<int, 1>{}, std::false_type{}, pm1 + j, iters_l);
    }
    phase_stamp(clk, stamps, lane, 6);
    phase_acc(pa, bstamps, 6);

    /* lane l's sum times H^(q+1), q = distance of its last element from the end of the GHASH input; the XOR butterfly
     * then sums the 64 lanes (ghash_combine) */
    if (early_win)
        y = wave_xor(gf_win4_mul<16>(lds, w4, y));
    else
        y = ghash_combine(lds, tab, lane, bs, q, y);
    /* S = 128: the wave without the length block hands its sum over (and makes its output stores visible at system scope
     * first: the tag wave's caller stores the completion word); both waves pass the barrier */
    const int tagw = ((hi - 1 - (SPLIT ? e0 : 0)) & (S - 1)) >> 6;
    if (S > 64) {
        if (vw != tagw) {
            if (lane == 0)
                lds128_store(lds, xslot, y);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        }
        __syncthreads();
        if (vw == tagw)
            y = v4xor(y, lds128(lds, xslot));
    }
    if (SPLIT) { /* pair 0's sum times H^(N - hi) = (H^128)^k, to pair 1's tag wave */
        if (!last_part && vw == tagw) {
            for (int j = 0; j < (N - hi) >> LOG2S; ++j)
                y = gh_mul_nibble(lds, tab, y);
            if (lane == 0)
                lds128_store(lds, xsplit, y);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        }
        __syncthreads();
        if (last_part && vw == tagw)
            y = v4xor(y, lds128(lds, xsplit));
    }
    phase_stamp(clk, stamps, lane, 7);
    phase_acc(pa, bstamps, 7);
    if (q == 0 && last_part) {
        const V4 tag = v4xor(y, ek0);
        if (OPEN) {
            const V4 rt = load_block<false>(in_p + L, 16);
            const bool ok = rt.w0 == tag.w0 && rt.w1 == tag.w1 && rt.w2 == tag.w2 && rt.w3 == tag.w3;
            result[rec_i] = ok ? (uint64_t)L : ~(uint64_t)0;
        } else {
            store_full(out_p + L, tag);
        }
    }
    phase_stamp(clk, stamps, lane, 8);
    phase_acc(pa, bstamps, 8);
    if (!OPEN && supp != nullptr && vw == tagw && last_part) {
        /* QUIC header protection after the record (lib/fusion.c:636-650), as in aesgcm_batch_kernel: the
         * sample may cover the tag written by another lane of this wave */
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        if (lane == 0) {
            const ptls_hip_supp_t sp = supp[rec_i];
            if ((sp.flags & PTLS_HIP_SUPP_ENABLE) && sp.hp_key < hp_nslots) {
                const V4 sample = load_full(out + sp.sample_off);
                const V4 mk = aes_encrypt<ROUNDS>(lds, lb_aes, hp_slots[sp.hp_key].rk, sample);
                store_full(mask + sp.mask_off, mk);
            }
        }
    }
}

/* Two waves on one record of 65 .. 128 GHASH elements (a QUIC packet; the plugin's single-record launch and the worker).
 * One wave alone is bound by its own LDS issue rate (a single wave gets a fraction of the LDS's rate, MI355X_MICROARCH.md
 * §LDS), and sparse_record gives it two elements per lane plus an H^64 table and a Horner step.  Here element i = 64 w + l
 * goes to lane l of wave w: one counter-mode AES block per lane, its GHASH input times H^(N - i) (keysetup's power list;
 * the windowed multiply's table is built from the power before the AES), an XOR butterfly per wave, and wave 1 adds
 * wave 0's sum from LDS after a workgroup barrier and writes the tag.  Wave 0 makes its output stores visible at system
 * scope before the barrier, so the completion word wave 1 stores after the tag covers them.  Every wave of the workgroup
 * calls this (the barrier); waves >= 2 only take part in the barrier.  pre = the lane's element (16 bytes, read early). */
constexpr int MW_MIN_N = 65, MW_MAX_N = 2 * 64;

template <int ROUNDS, bool OPEN, bool ALIGNED>
__device__ __forceinline__ void mw_record(uint8_t *lds, int wave, int lane, uint32_t lb_aes, uint32_t ctab, uint32_t xslot,
                                          const ptls_hip_record_t &rec, const uint8_t *in, const uint8_t *__restrict__ aad,
                                          uint8_t *out, uint64_t *__restrict__ result, const KeySlot *__restrict__ slots,
                                          const uint32_t *__restrict__ basis, const ptls_hip_supp_t *__restrict__ supp,
                                          const KeySlot *__restrict__ hp_slots, uint32_t hp_nslots, uint8_t *mask, V4 pre,
                                          uint4 ivo = uint4{0, 0, 0, 0})
{
    const uint32_t key = __builtin_amdgcn_readfirstlane(rec.key);
    const KeySlot *__restrict__ slot = slots + key;
    const uint32_t *__restrict__ rk = slot->rk;
    const uint4 *__restrict__ bs = reinterpret_cast<const uint4 *>(basis) + (size_t)key * BASIS_VECS;
    const int L = (int)__builtin_amdgcn_readfirstlane(rec.len);
    const int A = (int)__builtin_amdgcn_readfirstlane(rec.aad_len);
    const int na = (A + 15) >> 4, nc = (L + 15) >> 4;
    const int N = na + nc + 1;
    const bool tflag = !OPEN && (rec.flags & 1u) != 0 && L > 0;
    const uint32_t ttype = (rec.flags >> 8) & 0xffu;
    const uint8_t *in_p = in + rec.in_off;
    uint8_t *out_p = out + rec.out_off;
    const uint8_t *aad_p = aad + rec.aad_off;
    const int i = 64 * wave + lane;
    V4 z = V4{0, 0, 0, 0}, ek0 = V4{0, 0, 0, 0};
    if (wave < 2) {
        const uint4 hp = bs[NPOW * 128 + (i < N ? N - i - 1 : 0)]; /* H^(N - i) */
        const bool ov = __builtin_amdgcn_readfirstlane(ivo.w) != 0;
        const uint32_t n0 = __builtin_amdgcn_readfirstlane(ov ? ivo.x : slot->iv[0]),
                       n1 = __builtin_amdgcn_readfirstlane((ov ? ivo.y : slot->iv[1]) ^ bswap32((uint32_t)(rec.seq >> 32))),
                       n2 = __builtin_amdgcn_readfirstlane((ov ? ivo.z : slot->iv[2]) ^ bswap32((uint32_t)rec.seq));
        CtrConst cc = ctr_const(lds, lb_aes, rk, n0, n1, n2);
        cc.k10 = __builtin_amdgcn_readfirstlane(cc.k10);
        cc.k11 = __builtin_amdgcn_readfirstlane(cc.k11);
        cc.k20 = __builtin_amdgcn_readfirstlane(cc.k20);
        cc.k21 = __builtin_amdgcn_readfirstlane(cc.k21);
        cc.k22 = __builtin_amdgcn_readfirstlane(cc.k22);
        cc.k23 = __builtin_amdgcn_readfirstlane(cc.k23);
        cc.r03 = __builtin_amdgcn_readfirstlane(cc.r03);
        const Win4<16> w4 = gf_win4_build<16>(lds, ctab, lane, V4{hp.x, hp.y, hp.z, hp.w});
        const Elem e = elem_of(i < N ? i : N, N, na, nc, L, N);
        V4 inb = V4{0, 0, 0, 0};
        if (e.is_c) {
            const bool tb = tflag && e.c == nc - 1; /* the block holding the content-type byte */
            inb = mask_block(pre, e.nbytes - (tb ? 1 : 0));
            if (tb)
                inb = put_byte(inb, e.nbytes - 1, ttype);
        } else if (e.is_aad) {
            inb = mask_block(pre, min(16, A - 16 * e.i));
        }
        uint32_t cw[1] = {e.is_c ? bswap32((uint32_t)e.c + 2u) : 0x01000000u}; /* E_K(J0) on the length-block lane */
        V4 ks[1] = {V4{n0, n1, n2, cw[0]}};
        const V4 nohash[1] = {};
        V4 ydummy = V4{0, 0, 0, 0};
        ctr_ghash_skewed<ROUNDS, 1, false>(lds, lb_aes, rk, cc, cw, ks, ydummy, nohash, GhNibble{ctab});
        const V4 x = finish_elem<OPEN, ALIGNED, true, false>(e, inb, ks[0], aad_p, A, L, out_p, ek0); /* 0 past the record */
        z = wave_xor(gf_win4_mul<16>(lds, w4, x));
        if (wave == 0) {
            if (lane == 0)
                lds128_store(lds, xslot, z);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, ""); /* this wave's output stores, before wave 1's completion word */
        }
    }
    __syncthreads();
    if (wave == 1) {
        const V4 y = v4xor(z, lds128(lds, xslot));
        if (i == N - 1) {
            const V4 tag = v4xor(y, ek0);
            if (OPEN) {
                const V4 rt = load_block<false>(in_p + L, 16);
                const bool ok = rt.w0 == tag.w0 && rt.w1 == tag.w1 && rt.w2 == tag.w2 && rt.w3 == tag.w3;
                result[0] = ok ? (uint64_t)L : ~(uint64_t)0;
            } else {
                store_full(out_p + L, tag);
            }
        }
        if (!OPEN && supp != nullptr) { /* header protection after the tag (the sample may cover it), as sparse_record */
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            if (lane == 0) {
                const ptls_hip_supp_t sp = supp[0];
                if ((sp.flags & PTLS_HIP_SUPP_ENABLE) && sp.hp_key < hp_nslots) {
                    const V4 sample = load_full(out + sp.sample_off);
                    const V4 mk = aes_encrypt<ROUNDS>(lds, lb_aes, hp_slots[sp.hp_key].rk, sample);
                    store_full(mask + sp.mask_off, mk);
                }
            }
        }
    }
}

/* BYVAL: the plugin's single-record launch (the record by value in the kernel arguments, recs_ord == nullptr); its own
 * instantiation, so the batch one carries none of its prefetch registers.  It runs 256 threads (one wave per SIMD, the
 * whole register file: no spills) since only wave 0 works on the record; the others help build the AES tables. */
constexpr int BYVAL_WG = 256;
template <int ROUNDS, bool OPEN, bool ALIGNED, bool BYVAL, int WG = BYVAL ? BYVAL_WG : SPARSE_WG>
__global__ void __launch_bounds__(WG)
    aesgcm_sparse_kernel(const ptls_hip_record_t *__restrict__ recs_ord, const uint32_t *__restrict__ order,
                         const Chunk *__restrict__ chunks, uint32_t nchunks, const uint8_t *in, const uint8_t *__restrict__ aad,
                         uint8_t *out, uint64_t *__restrict__ result, const KeySlot *__restrict__ slots,
                         const uint32_t *__restrict__ basis, const uint32_t *__restrict__ t0, const ptls_hip_supp_t *__restrict__ supp,
                         const KeySlot *__restrict__ hp_slots, uint32_t hp_nslots, uint8_t *mask, ptls_hip_record_t one,
                         uint32_t *done, uint32_t done_seq, uint64_t *__restrict__ clk, uint32_t *queue)
{
    /* BYVAL: 16 KiB more for wave 1's windowed table of a two-wave record (mw_record, or a long record at stride 128),
     * then 2 KiB for wave 1's prefetched elements of a long record and 64 B for the waves' hand-over */
    constexpr uint32_t XCH2 = SP_TAB + (WG / 64) * 8192 + 16384, XSLOT = XCH2 + 2048;
    constexpr uint32_t LDS_SIZE = SP_TAB + (WG / 64) * 8192 + (BYVAL ? 16384 + 2048 + 64 : 0);
    __shared__ __attribute__((aligned(16))) uint8_t lds[LDS_SIZE];
    static_assert(LDS_SIZE <= 163840, "AES tables + per-wave GHASH tables must fit the CU's 160 KiB");
    const int lane = threadIdx.x & 63;
    const uint32_t lb_aes = (uint32_t)(lane & 31) * 4u; /* table base 0: byte 2 of the address is 0 */
    const uint32_t tab = __builtin_amdgcn_readfirstlane(SP_TAB + (uint32_t)(threadIdx.x >> 6) * 8192u); /* wave-uniform */
    /* one record by value (recs_ord == nullptr), or build_chunks' chunks with their records contiguous from 0 */
    constexpr bool by_value = BYVAL;
    const bool stamps = STAMP_PHASES && by_value && blockIdx.x == 0 && threadIdx.x < 64;
    const bool bstamps = STAMP_PHASES && !by_value && blockIdx.x == 0 && threadIdx.x < 64;
    PhaseAcc pa{};
    uint64_t r_begin = 0, t_begin = 0;
    (void)r_begin, (void)t_begin;
#if STAMP_PHASES
    if (bstamps) {
        r_begin = __builtin_amdgcn_s_memrealtime();
        t_begin = __builtin_amdgcn_s_memtime();
    }
#endif
    phase_stamp(clk, stamps, lane, 0);
    if (!STAMP_PHASES)
        clock_stamp(clk, 0);
    /* A single record (the plugin's launch, wave 0 of the one workgroup) reads its first two elements per lane (the
     * AAD block or the data block, whole 16 bytes: the plugin's own pinned staging holds them) and touches its key slot
     * and its lane's final power before the AES tables are built, so those PCIe / HBM latencies run under the build
     * instead of after it (tools/plugin_stamps.py).  pre[m] = element lane + 64 m. */
    V4 pre[2] = {V4{0, 0, 0, 0}, V4{0, 0, 0, 0}}, pre_hi[2] = {V4{0, 0, 0, 0}, V4{0, 0, 0, 0}};
    V4 touch = V4{0, 0, 0, 0};
    const bool prefetch = by_value && blockIdx.x == 0 && threadIdx.x < 64;
    /* a single record longer than MW_MAX_N GHASH elements runs on waves 0 and 1 at stride 128 (sparse_record S = 128):
     * wave 0 reads elements lane + 64 m, m < 4; it keeps m = 0, 2 and hands m = 1, 3 to wave 1 through LDS (XCH2) */
    const int n_one = BYVAL ? (((int)one.aad_len + 15) >> 4) + (((int)one.len + 15) >> 4) + 1 : 0;
    const bool longrec = BYVAL && STAMP_PHASES == 0 && WG >= 128 && n_one > MW_MAX_N;
    if (prefetch) {
        const int na1 = ((int)one.aad_len + 15) >> 4, nc1 = ((int)one.len + 15) >> 4;
        auto elem16 = [&](int i) __attribute__((always_inline)) {
            V4 v = V4{0, 0, 0, 0};
            if (i < na1)
                v = load_full(aad + one.aad_off + 16 * (size_t)i);
            else if (i < na1 + nc1)
                v = load_full(in + one.in_off + 16 * (size_t)(i - na1));
            return v;
        };
        pre[0] = elem16(lane);
        pre[1] = elem16(lane + 64);
        if (longrec) {
            pre_hi[0] = elem16(lane + 128);
            pre_hi[1] = elem16(lane + 192);
        }
        const uint4 *bsk = reinterpret_cast<const uint4 *>(basis) + (size_t)one.key * BASIS_VECS;
        const uint4 kv = reinterpret_cast<const uint4 *>(slots + one.key)[lane & 15];       /* round keys, IV: 256 B */
        const uint4 pv = bsk[NPOW * 128 + ((na1 + nc1 - lane) & 63)];                        /* H^(q+1) of the combine */
        touch = V4{kv.x ^ pv.x, kv.y ^ pv.y, kv.z ^ pv.z, kv.w ^ pv.w};
    }
    /* the single record's wave 0 leaves the table build to the other waves: its prefetch loads are older than any T0
     * load it would issue, and vmcnt retires loads in order, so it would wait for its PCIe reads before its table stores */
    if (!BYVAL)
        build_aes_tables<WG>(lds, 0, t0); /* the batch kernel's layout at offset 0 */
    else if (threadIdx.x >= 64)
        build_aes_tables<WG - 64>(lds, 0, t0, (int)threadIdx.x - 64);
    /* a two-wave record (mw_record): wave 1's element lane + 64 was prefetched by wave 0 (pre[1]); it goes through LDS
     * (wave 3's table area, unused by a single record) */
    const bool mw = BYVAL && STAMP_PHASES == 0 && n_one >= MW_MIN_N && n_one <= MW_MAX_N;
    const uint32_t XCH = SP_TAB + 3u * 8192u;
    if (mw && threadIdx.x < 64)
        lds128_store(lds, XCH + (uint32_t)lane * 16u, pre[1]);
    if (longrec && threadIdx.x < 64) {
        lds128_store(lds, XCH2 + (uint32_t)lane * 16u, pre[1]);
        lds128_store(lds, XCH2 + 1024u + (uint32_t)lane * 16u, pre_hi[1]);
    }
    __syncthreads();
    asm volatile("" ::"v"(touch.w0), "v"(touch.w1), "v"(touch.w2), "v"(touch.w3)); /* keep the touch loads */
    if (mw) {
        const int wave = (int)(threadIdx.x >> 6);
        const V4 mine = wave == 0 ? pre[0] : wave == 1 ? lds128(lds, XCH + (uint32_t)lane * 16u) : V4{0, 0, 0, 0};
        const uint32_t ctab_w = wave == 0 ? SP_TAB + 8192u : SP_TAB + (uint32_t)(WG / 64) * 8192u;
        mw_record<ROUNDS, OPEN, ALIGNED>(lds, wave, lane, lb_aes, ctab_w, SP_TAB, one, in, aad, out, result, slots, basis, supp,
                                         hp_slots, hp_nslots, mask, mine);
        if (done != nullptr && wave == 1) { /* the tag's wave: wave 0 released its stores before the barrier */
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
            if (lane == 0)
                __hip_atomic_store(done, done_seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        return;
    }
    if (longrec) { /* waves 0 and 1 as one 128-lane wave (sparse_record S = 128); waves 2, 3 only take its barrier */
        const int wave = (int)(threadIdx.x >> 6);
        if (wave < 2) {
            V4 p2[2];
            if (wave == 0) {
                p2[0] = pre[0];
                p2[1] = pre_hi[0];
            } else {
                p2[0] = lds128(lds, XCH2 + (uint32_t)lane * 16u);
                p2[1] = lds128(lds, XCH2 + 1024u + (uint32_t)lane * 16u);
            }
            /* wave 0: its H^128 table in area 0, its combination table in areas 2-3; wave 1: area 1 and the extra 16 KiB */
            const uint32_t tab_w = SP_TAB + (uint32_t)wave * 8192u;
            const uint32_t ctab_w = wave == 0 ? SP_TAB + 2u * 8192u : SP_TAB + (uint32_t)(WG / 64) * 8192u;
            sparse_record<ROUNDS, OPEN, ALIGNED, BYVAL, 128>(lds, lane, lb_aes, tab_w, one, 0, in, aad, out, result, slots, basis,
                                                            supp, hp_slots, hp_nslots, mask, true, p2, clk, false, false, pa,
                                                            ctab_w, wave, XSLOT);
            const int tagw = ((n_one - 1) & 127) >> 6;
            if (done != nullptr && wave == tagw) { /* the other wave released its stores before sparse_record's barrier */
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
                if (lane == 0)
                    __hip_atomic_store(done, done_seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
        } else {
            __syncthreads(); /* sparse_record's hand-over barrier */
        }
        return;
    }
    phase_stamp(clk, stamps, lane, 1);
    uint32_t nrecs = 1;
    if (!by_value) {
        if (nchunks == 0)
            return;
        const Chunk last = chunks[nchunks - 1];
        nrecs = last.first + last.count;
    }
    const uint32_t waves = gridDim.x * (WG / 64);
    const uint32_t w0 = __builtin_amdgcn_readfirstlane(blockIdx.x * (WG / 64) + (threadIdx.x >> 6));
    /* The deal of records (sorted by decreasing length) to the launch's waves: a snake over the first
     * nrecs - nrecs / SPARSE_TAIL records (round k goes forward on even k and backward on odd k, so each wave's lengths
     * pair long with short), the shortest tail from the launch's queue word (a few claims per wave, taking up what the
     * waves' different speeds leave: the youngest wave on each SIMD, the slowest XCD).  A queued claim is issued when the
     * record before it starts, so its latency runs under that record; the last wave to claim past the end resets the words
     * (engine.cpp queue_slot).  Measured alternatives (EXPERIMENTS.md): a static stride, every record from the queue. */
    const bool dyn = !by_value && queue != nullptr;
    const uint32_t nstat = !dyn ? nrecs : nrecs - nrecs / SPARSE_TAIL;
    auto stat_pos = [&](uint32_t k) -> uint32_t { return k * waves + ((k & 1u) ? waves - 1u - w0 : w0); };
    auto claim = [&]() -> uint32_t { /* lane 0's returned value; read (readfirstlane) only when it is needed */
        uint32_t v = 0;
        if (lane == 0)
            v = __hip_atomic_fetch_add(queue, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return v;
    };
    uint32_t kk = 0, pos = stat_pos(0);
    bool in_dyn = dyn && pos >= nstat;
    if (in_dyn)
        pos = nstat + (uint32_t)__builtin_amdgcn_readfirstlane(claim());
    while (pos < nrecs) {
        const uint32_t sp = stat_pos(kk + 1);
        const bool nd = dyn && (in_dyn || sp >= nstat);
        const uint32_t next_v = nd ? claim() : 0u;
        phase_acc(pa, bstamps, 1);
        const ptls_hip_record_t rec = by_value ? one : recs_ord[pos];
        const uint32_t rec_i = by_value ? 0u : order != nullptr ? order[pos] : pos;
        /* a single record's wave 0 takes the unused table areas of waves 1 and 2 for its lane-combination table */
        sparse_record<ROUNDS, OPEN, ALIGNED, BYVAL>(lds, lane, lb_aes, tab, rec, rec_i, in, aad, out, result, slots, basis, supp,
                                                   hp_slots, hp_nslots, mask, prefetch, pre, clk, stamps, bstamps, pa, SP_TAB + 8192u);
        if (by_value)
            break;
        if (nd) {
            pos = nstat + (uint32_t)__builtin_amdgcn_readfirstlane(next_v);
            in_dyn = true;
        } else {
            ++kk;
            pos = sp;
        }
    }
    if (dyn && lane == 0 &&
        __hip_atomic_fetch_add(queue + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == waves - 1) {
        /* every wave has claimed past the end: no more adds to either word in this launch */
        __hip_atomic_store(queue, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(queue + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (done != nullptr && w0 == 0) {
        /* the by-value record's wave: every store above (the whole wave's, s_waitcnt is wave-wide) reaches system
         * scope before the completion word does; a vector store (global memory, never the scalar cache) */
        phase_stamp(clk, stamps, lane, 9);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        phase_stamp(clk, stamps, lane, 10);
        if (lane == 0)
            __hip_atomic_store(done, done_seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        phase_stamp(clk, stamps, lane, 11);
    }
#if STAMP_PHASES
    if (bstamps && clk != nullptr && lane == 0) { /* clk[16 + k] = cycles of phase k, [25] records, [26, 27] 100 MHz span */
        for (int k = 2; k <= 8; ++k)
            clk[16 + k] = pa.acc[k];
        clk[25] = pa.n;
        clk[26] = r_begin;
        clk[27] = __builtin_amdgcn_s_memrealtime();
        clk[28] = __builtin_amdgcn_s_memtime();
        clk[29] = t_begin;
    }
#endif
    if (!STAMP_PHASES && clk != nullptr) { /* the workgroup's end: after its last wave */
        __syncthreads();
        clock_stamp(clk, 1);
    }
}

/* The plugin worker: one workgroup stays resident per mailbox and serves it (internal.h WorkerSlot, fine-grained pinned
 * host memory): wave 0 polls seq over PCIe, waves 0 and 1 read the request, and the record runs through sparse_record (the
 * single-record path of a launched call: prefetched first elements, the wave's H^64 table, the early lane-combination
 * table; records of 65..128 GHASH elements on waves 0 and 1, mw_record; longer ones on all four waves, two pairs at stride
 * 128, waves 2 and 3 taking the request from wave 1 through LDS), then the tag's wave stores the call's completion word
 * after all its output (system scope) and then `served`.  The AES tables are built
 * once for the worker's life instead of once per call, and no launch sits between the caller and the kernel.
 *   - Polling keeps WORKER_POLLS loads of {seq, quit} in flight (a PCIe read takes ~2 us): a new request is seen about one
 *     read latency after it is written, not up to two.
 *   - A record the host put inline (WREQ_INLINE: AAD padded to 16 bytes, then the input, in the mailbox's data area) is
 *     read in the same round trip as the request: the first two elements of every lane lie at fixed offsets there.
 * The wave leaves when the host asks (quit), after idle_ticks without a request or after life_ticks (100 MHz counter) —
 * so the kernel always ends, and a stream that shares its hardware queue waits at most life_ticks — storing its epoch
 * in `exited`. */
constexpr int WORKER_POLLS = 4;

/* a pointer the worker read from its mailbox, marked as global memory: without it the compiler cannot infer the address
 * space, emits flat loads / stores and waits for every flat store's completion (a PCIe write round trip per output store
 * into pinned host memory) before the next LDS access */
template <typename T>
__device__ __forceinline__ T *as_global(T *p)
{
    uint64_t v = (uint64_t)(uintptr_t)p;
    asm volatile("" : "+v"(v)); /* an opaque integer: the global pointer made from it cannot be folded back to a flat one */
    return (T *)((__attribute__((address_space(1))) T *)v);
}
/* The key slot and basis pointers of a request are constant-address-space pointers (as_const), so the round keys come
 * through the scalar unit (s_load) as in a launched kernel (16 KiB record 28 -> 24 us per call, one ECB block 10.1 ->
 * 9.3 us; tools/calls_r04/r04_call8.sh).  Valid because a slot the resident dispatch may have read never changes while it
 * is resident (plugin_worker.cpp slot pool: a freed slot is reused only after that dispatch has left; the IV travels in the
 * request).  The round-3 attempt faulted, and so did this one's first build (r04_call7.sh): both rebuilt the 64-bit
 * pointer from two readfirstlane results, which return int, so an address with bit 31 set sign-extended over the high
 * half (s_bfe_i64 in the disassembly); as_const widens each half through uint32_t (EXPERIMENTS.md E3, "worker requests with key material through the scalar unit"). */
template <typename T>
__device__ __forceinline__ const T *as_const(const T *p)
{
    uint64_t v = (uint64_t)(uintptr_t)p;
    asm volatile("" : "+v"(v));
    /* __builtin_amdgcn_readfirstlane returns int: each half goes through uint32_t, or an address with bit 31 set would
     * sign-extend over the high half (the fault of this call's first version, tools/calls_r04/r04_call7.sh) */
    v = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(v >> 32)) << 32) |
        (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)v);
    return (const T *)((const __attribute__((address_space(4))) T *)v);
}
#ifndef WORKER_STAMPS
#define WORKER_STAMPS 0 /* diagnostic builds only (Makefile `diag`, tools/worker_stamps.py): the worker stamps the 100 MHz counter
                           at its phase boundaries into WorkerSlot::stamps (seen, request read, record done, released) */
#endif

/* a stamp of the 100 MHz counter after everything the wave issued so far has completed */
__device__ __forceinline__ uint64_t worker_stamp()
{
    __builtin_amdgcn_s_waitcnt(0);
    return __builtin_amdgcn_s_memrealtime();
}

__device__ __forceinline__ uint64_t poll_word(const WorkerSlot *ms)
{
    return __hip_atomic_load(reinterpret_cast<const uint64_t *>(&ms->seq), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

/* four waves: wave 0 polls; waves 0 and 1 serve a two-wave record (mw_record), all four a long one (two pairs) */
constexpr int WORKER_WG = 256;

__global__ void __launch_bounds__(WORKER_WG)
    plugin_worker_kernel(WorkerSlot *mb, uint32_t epoch, const uint32_t *__restrict__ t0, uint64_t idle_ticks, uint64_t life_ticks,
                         uint64_t *activity)
{
    /* AES tables | the H^128 Horner table (one key per request: the waves of a long record share it, each writing the same
     * values before it reads them) | each wave's lane-combination table | the poll's verdict | a long record's hand-overs
     * (pair 0, pair 1, pair 0 to pair 1) */
    constexpr uint32_t CTAB0 = SP_TAB + 8192, CTL = CTAB0 + (WORKER_WG / 64) * 16384, XSLOT = CTL + 16, RQ = XSLOT + 48,
                       RQW = RQ + (uint32_t)sizeof(WorkerReq);
    __shared__ __attribute__((aligned(16))) uint8_t lds[RQW + 16];
    /* wave 1 -> waves 2, 3: (request << 2) | (a two-wave record << 1) | a long record */
    uint32_t *rq_word = reinterpret_cast<uint32_t *>(lds + RQW);
    const int lane = threadIdx.x & 63, wave = (int)(threadIdx.x >> 6);
    const uint32_t lb_aes = (uint32_t)(lane & 31) * 4u;
    const uint32_t tab = SP_TAB;
    build_aes_tables<WORKER_WG>(lds, 0, t0);
    __syncthreads();
    WorkerSlot *ms = mb + blockIdx.x; /* one mailbox per workgroup (plugin.h PluginWorker: one per calling thread) */
    const uint64_t t_start = __builtin_amdgcn_s_memrealtime();
    uint64_t t_last = t_start;
    uint32_t last = __builtin_amdgcn_readfirstlane(__hip_atomic_load(&ms->served, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
    if (threadIdx.x == 0)
        __hip_atomic_store(&ms->started, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (threadIdx.x == 64) /* a request already served: never the next one's word (seen by waves 2, 3 after the first barrier) */
        __hip_atomic_store(rq_word, last << 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    PhaseAcc pa{};
    uint64_t ring[WORKER_POLLS];
    if (wave == 0) {
#pragma unroll
        for (int k = 0; k < WORKER_POLLS; ++k) {
            ring[k] = poll_word(ms);
            __builtin_amdgcn_s_sleep(8);
        }
    }
    for (;;) {
        if (wave == 0) { /* poll until a request or a reason to leave; the verdict goes to wave 1 through LDS */
            uint32_t seq = last;
            bool leave = false;
            while (!leave && seq == last) {
#pragma unroll
                for (int k = 0; k < WORKER_POLLS; ++k) { /* the oldest read in flight (vmcnt retires in order), then a new one */
                    const uint64_t v = ring[k];
                    const uint32_t sv = __builtin_amdgcn_readfirstlane((uint32_t)v),
                                   quit = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
                    /* a read issued before the last request was served may still return the one before it: only a later
                     * request number counts (the host numbers them consecutively) */
                    if (seq == last && (int32_t)(sv - last) > 0)
                        seq = sv;
                    const uint64_t now = __builtin_amdgcn_s_memrealtime();
                    if (seq == last && now - t_last > idle_ticks) {
                        /* idle here: the workgroups of the dispatch leave together, when none of them has served a request
                         * for idle_ticks (the last one served is in `activity`), so a caller rarely finds its own
                         * workgroup gone while the others still hold the dispatch */
                        const uint64_t av = __hip_atomic_load(activity, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        const uint64_t a = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(av >> 32)) << 32) |
                                           (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)av);
                        t_last = a > t_last ? a : t_last;
                    }
                    if (seq == last && (quit != 0 || now - t_last > idle_ticks || now - t_start > life_ticks))
                        leave = true;
                    /* no new read once a request is seen: the acquire below waits for every read still in flight, and
                     * one issued now would add a whole PCIe round trip (round 6) */
                    ring[k] = poll_word(ms);
                    __builtin_amdgcn_s_sleep(2);
                }
            }
            if (lane == 0)
                *reinterpret_cast<uint2 *>(lds + CTL) = make_uint2(seq, leave ? 1u : 0u);
        }
        __syncthreads();
        const uint2 verdict = *reinterpret_cast<const uint2 *>(lds + CTL);
        const uint32_t seq = __builtin_amdgcn_readfirstlane(verdict.x);
        if (__builtin_amdgcn_readfirstlane(verdict.y) != 0)
            break;
        /* Waves 0 and 1 read the request from the mailbox.  Waves 2 and 3 serve only a long record's second part: they
         * wait for wave 1's copy of the request in LDS, since two more waves reading it over PCIe (and two more
         * system-scope acquires) made every call slower by 0.3-0.9 us (measured, round 6). */
        bool serve = true;
        if (wave >= 2) {
            uint32_t lw;
            for (;;) {
                lw = __builtin_amdgcn_readfirstlane(__hip_atomic_load(rq_word, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP));
                if ((lw >> 2) == (seq & 0x3fffffffu))
                    break;
                __builtin_amdgcn_s_sleep(1);
            }
            serve = (lw & 1u) != 0;
            if (lw & 2u)
                __syncthreads(); /* mw_record's hand-over barrier */
        }
        if (serve) {
            /* the request (and the record, inline or in the caller's pinned staging) was written before seq.  Ordering the
             * loads is not enough: the vector L1 keeps the previous request's lines at the same addresses (measured: a
             * workgroup-scope acquire served request 2 with request 1's completion pointer), so the acquire is at system
             * scope, which invalidates the L1 and the L2's lines of host memory.  A key slot this dispatch may have read is never
             * rewritten while it is resident (plugin_worker.cpp slot pool: a freed slot is handed out again only after the dispatch
             * that could hold it has left), so neither the scalar nor the vector caches can hold a stale key slot. */
            uint64_t st[5] = {0, 0, 0, 0, 0};
            if (WORKER_STAMPS)
                st[0] = worker_stamp();
            if (wave < 2) /* (waves 2, 3: wave 1's acquire, then its release of the word above) */
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
            if (WORKER_STAMPS)
                st[1] = worker_stamp();
            if (threadIdx.x == 0)
                __hip_atomic_store(&ms->seen, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            const WorkerReq &rq = wave < 2 ? ms->req : *reinterpret_cast<const WorkerReq *>(lds + RQ);
            /* an inline record's elements, loaded with the request (unused otherwise): wave 0 elements l, l + 64, l + 128
             * (a two-wave record: l; a long one: l, l + 128), wave 1 elements l, l + 64, l + 192 (a one-wave record: l, l + 64;
             * a two-wave record: l + 64; a long one: l + 64, l + 192); waves 2 and 3 none (their part of a long record starts
             * where the record's length puts it) */
            /* (three named values, not an array: a wave-dependent choice between array elements became a dynamic index, i.e.
             * the array went to scratch) */
            V4 pin0 = V4{0, 0, 0, 0}, pin1 = V4{0, 0, 0, 0}, pin2 = V4{0, 0, 0, 0};
            if (wave < 2) {
                pin0 = load_full(ms->data + 16 * (size_t)lane);
                pin1 = load_full(ms->data + 16 * (size_t)(lane + 64));
                pin2 = load_full(ms->data + 16 * (size_t)(lane + 128 + 64 * wave));
            }
            V4 rqc = V4{0, 0, 0, 0}; /* wave 1: the request's bytes for waves 2, 3 */
            if (wave == 1 && lane < (int)(sizeof(WorkerReq) / 16))
                rqc = load_full(reinterpret_cast<const uint8_t *>(&ms->req) + 16 * (size_t)lane);
            const ptls_hip_record_t rec = rq.rec;
            const uint32_t flags = __builtin_amdgcn_readfirstlane(rq.flags);
            const uint4 ivo = (flags & WREQ_IV) ? uint4{rq.iv[0], rq.iv[1], rq.iv[2], 1u} : uint4{0, 0, 0, 0};
            const uint8_t *in = as_global(rq.in), *aad = as_global(rq.aad);
            uint8_t *out = as_global(rq.out);
            const KeySlot *slots = as_const(rq.slots);
            uint32_t *done = as_global(rq.done);
            const uint32_t done_seq = __builtin_amdgcn_readfirstlane(rq.done_seq);
            const ptls_hip_supp_t *supp = rq.supp != nullptr ? as_global(rq.supp) : nullptr;
            const KeySlot *hp_slots = rq.hp_slots != nullptr ? as_global(rq.hp_slots) : nullptr;
            uint8_t *mask = rq.mask != nullptr ? as_global(rq.mask) : nullptr;
            uint64_t *result = as_global(rq.result);
            const uint32_t *basis = as_const(rq.basis);
            const bool open = (flags & WREQ_OPEN) != 0, a256 = (flags & WREQ_AES256) != 0;
            const int na1 = ((int)rec.aad_len + 15) >> 4, nc1 = ((int)rec.len + 15) >> 4;
            const int n1 = na1 + nc1 + 1;
            const bool ecb = (flags & WREQ_ECB) != 0;
            const bool mw = !ecb && n1 >= MW_MIN_N && n1 <= MW_MAX_N;
            /* a long record on two pairs of waves at stride 128 (sparse_record S = 128, SPLIT): pair 1 takes the last 128 k
             * elements, about half */
            const bool longrec = !ecb && n1 > MW_MAX_N;
            /* where pair 1's part starts: pair 0 takes the AAD blocks and about 5/8 of the data blocks, a multiple of 128 (so
             * its lanes hold as many); pair 1 starts a request read later (it waits for wave 1's copy) and has no elements
             * read with the request.  16 KiB, same box: an even split 22.3 / 21.6 us seal / open, 5/8 21.1 / 21.3, 3/4
             * 21.1-22.3 / 21.2-21.6, 3/8 24.3 / 24.4 (profiles/r06_plugin/plugin_ab_split_point*.log) */
            const int n1b = na1 + min(nc1, 128 * max(1, (5 * nc1 + 512) >> 10));
            if (wave == 1) {
                if (lane < (int)(sizeof(WorkerReq) / 16))
                    lds128_store(lds, RQ + 16u * (uint32_t)lane, rqc);
                if (lane == 0)
                    __hip_atomic_store(rq_word, (seq << 2) | (mw ? 2u : 0u) | (longrec ? 1u : 0u), __ATOMIC_RELEASE,
                                       __HIP_MEMORY_SCOPE_WORKGROUP);
            }
            if (WORKER_STAMPS)
                st[2] = worker_stamp();
            /* WORKER_STAMPS builds (with STAMP_PHASES): the record's phase stamps (shader cycles) go to the end of the data area,
             * clk[1] = the request loaded, clk[9] = the record done */
            uint64_t *wclk = WORKER_STAMPS ? reinterpret_cast<uint64_t *>(ms->data + WORKER_DATA - 128) : nullptr;
            if (WORKER_STAMPS && wave == 1) {
                const uint64_t t = __builtin_amdgcn_s_memtime();
                if (lane == 0)
                    wclk[1] = t;
            }
            /* an element read from the caller's staging (records that do not fit inline) */
            auto elem_block = [&](int i) __attribute__((always_inline)) {
                V4 v = V4{0, 0, 0, 0};
                if (i < na1)
                    v = load_full(aad + rec.aad_off + 16 * (size_t)i);
                else if (i < na1 + nc1)
                    v = load_full(in + rec.in_off + 16 * (size_t)(i - na1));
                return v;
            };
            /* A record of at most MW_MIN_N - 1 elements and an ECB block run on wave 1: wave 0 polled, and it still waits for its
             * last poll reads (its acquire drains them, ~1 PCIe round trip); wave 1 has none in flight (round 6). */
            if (ecb) {
                /* one block with the slot's round keys (the block was read with the request: pin0, lane 0's element) */
                if (wave == 1) {
                    const V4 blk = V4{(uint32_t)__builtin_amdgcn_readfirstlane(pin0.w0), (uint32_t)__builtin_amdgcn_readfirstlane(pin0.w1),
                                      (uint32_t)__builtin_amdgcn_readfirstlane(pin0.w2), (uint32_t)__builtin_amdgcn_readfirstlane(pin0.w3)};
                    const V4 m = a256 ? aes_encrypt<14>(lds, lb_aes, slots->rk, blk) : aes_encrypt<10>(lds, lb_aes, slots->rk, blk);
                    if (lane == 0)
                        store_full(out, m);
                }
            } else if (longrec) {
                const int pair = wave >> 1, vw = wave & 1;
                V4 p2[2] = {V4{0, 0, 0, 0}, V4{0, 0, 0, 0}};
                if (pair == 0) { /* the first two elements of each lane of pair 0; pair 1 reads its own in the stretch */
                    if (flags & WREQ_INLINE) {
                        p2[0] = vw == 0 ? pin0 : pin1;
                        p2[1] = pin2;
                    } else {
                        p2[0] = elem_block(lane + 64 * vw);
                        p2[1] = elem_block(lane + 64 * vw + 128);
                    }
                }
                const uint32_t ctab_w = CTAB0 + 16384u * (uint32_t)wave, xs = XSLOT + 16u * (uint32_t)pair;
                const int e0 = pair == 0 ? 0 : n1b, hi = pair == 0 ? n1b : n1;
                uint64_t *lwclk = WORKER_STAMPS && wave == 1 ? wclk : nullptr; /* (diagnostic builds: wave 1's phases) */
                if (open && a256)
                    sparse_record<14, true, true, true, 128, SPARSE_PE, true>(lds, lane, lb_aes, tab, rec, 0, in, aad, out, result, slots, basis, supp, hp_slots, 1, mask,
                                                                              pair == 0, p2, lwclk, WORKER_STAMPS && wave == 1, false, pa, ctab_w, vw, xs, ivo, e0, hi, XSLOT + 32);
                else if (open)
                    sparse_record<10, true, true, true, 128, SPARSE_PE, true>(lds, lane, lb_aes, tab, rec, 0, in, aad, out, result, slots, basis, supp, hp_slots, 1, mask,
                                                                              pair == 0, p2, lwclk, WORKER_STAMPS && wave == 1, false, pa, ctab_w, vw, xs, ivo, e0, hi, XSLOT + 32);
                else if (a256)
                    sparse_record<14, false, true, true, 128, SPARSE_PE, true>(lds, lane, lb_aes, tab, rec, 0, in, aad, out, result, slots, basis, supp, hp_slots, 1, mask,
                                                                               pair == 0, p2, lwclk, WORKER_STAMPS && wave == 1, false, pa, ctab_w, vw, xs, ivo, e0, hi, XSLOT + 32);
                else
                    sparse_record<10, false, true, true, 128, SPARSE_PE, true>(lds, lane, lb_aes, tab, rec, 0, in, aad, out, result, slots, basis, supp, hp_slots, 1, mask,
                                                                               pair == 0, p2, lwclk, WORKER_STAMPS && wave == 1, false, pa, ctab_w, vw, xs, ivo, e0, hi, XSLOT + 32);
            } else if (mw) {
                const V4 mine = (flags & WREQ_INLINE) ? (wave == 0 ? pin0 : pin1) : elem_block(lane + 64 * wave);
                const uint32_t ctab_w = CTAB0 + 16384u * (uint32_t)(wave & 1);
                if (open && a256)
                    mw_record<14, true, true>(lds, wave, lane, lb_aes, ctab_w, tab, rec, in, aad, out, result, slots, basis, supp, hp_slots, 1, mask, mine, ivo);
                else if (open)
                    mw_record<10, true, true>(lds, wave, lane, lb_aes, ctab_w, tab, rec, in, aad, out, result, slots, basis, supp, hp_slots, 1, mask, mine, ivo);
                else if (a256)
                    mw_record<14, false, true>(lds, wave, lane, lb_aes, ctab_w, tab, rec, in, aad, out, result, slots, basis, supp, hp_slots, 1, mask, mine, ivo);
                else
                    mw_record<10, false, true>(lds, wave, lane, lb_aes, ctab_w, tab, rec, in, aad, out, result, slots, basis, supp, hp_slots, 1, mask, mine, ivo);
            } else if (wave == 1) {
                {
                    /* the record's first two elements per lane, as the launched single-record kernel reads them */
                    V4 pre[2];
                    if (flags & WREQ_INLINE) {
                        pre[0] = pin0;
                        pre[1] = pin1;
                    } else {
                        pre[0] = elem_block(lane);
                        pre[1] = elem_block(lane + 64);
                    }
                    const uint32_t ctab = CTAB0;
                    if (open && a256)
                        sparse_record<14, true, true, true>(lds, lane, lb_aes, tab, rec, 0, in, aad, out, result, slots, basis, supp,
                                                            hp_slots, 1, mask, true, pre, wclk, WORKER_STAMPS, false, pa, ctab, 0, 0, ivo);
                    else if (open)
                        sparse_record<10, true, true, true>(lds, lane, lb_aes, tab, rec, 0, in, aad, out, result, slots, basis, supp,
                                                            hp_slots, 1, mask, true, pre, wclk, WORKER_STAMPS, false, pa, ctab, 0, 0, ivo);
                    else if (a256)
                        sparse_record<14, false, true, true>(lds, lane, lb_aes, tab, rec, 0, in, aad, out, result, slots, basis, supp,
                                                             hp_slots, 1, mask, true, pre, wclk, WORKER_STAMPS, false, pa, ctab, 0, 0, ivo);
                    else
                        sparse_record<10, false, true, true>(lds, lane, lb_aes, tab, rec, 0, in, aad, out, result, slots, basis, supp,
                                                             hp_slots, 1, mask, true, pre, wclk, WORKER_STAMPS, false, pa, ctab, 0, 0, ivo);
                }
            }
            /* the wave holding the tag (wave 1 of a one- or two-wave record, pair 1's tag wave of a long one): every store of
             * the call reaches system scope before its completion word (the other waves released theirs before the barrier
             * that handed their sums over) */
            if (wave == (longrec ? 2 + (((n1 - 1 - n1b) & 127) >> 6) : 1)) {
                if (WORKER_STAMPS) {
                    st[3] = worker_stamp();
                    const uint64_t t = __builtin_amdgcn_s_memtime();
                    if (lane == 0)
                        wclk[9] = t;
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
                if (WORKER_STAMPS) {
                    st[4] = worker_stamp();
                    if (lane < 5)
                        __hip_atomic_store(&ms->stamps[lane], lane == 0 ? st[0] : lane == 1 ? st[1] : lane == 2 ? st[2] : lane == 3 ? st[3] : st[4],
                                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
                }
                if (lane == 0) {
                    __hip_atomic_store(done, done_seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    __hip_atomic_store(&ms->served, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
                }
            }
        }
        __syncthreads(); /* every wave is done with the request (its LDS tables, the verdict slot, the request's copy) */
        last = seq;
        t_last = __builtin_amdgcn_s_memrealtime();
        if (threadIdx.x == 0)
            __hip_atomic_fetch_max(activity, t_last, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    if (threadIdx.x == 0)
        __hip_atomic_store(&ms->exited, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

int launch_plugin_worker(WorkerSlot *mb, unsigned nmb, uint32_t epoch, const uint32_t *t0, uint64_t idle_ticks, uint64_t life_ticks,
                         uint64_t *activity, void *stream)
{
    hipLaunchKernelGGL(plugin_worker_kernel, dim3(nmb), dim3(WORKER_WG), 0, static_cast<hipStream_t>(stream), mb, epoch, t0, idle_ticks,
                       life_ticks, activity);
    return (int)hipGetLastError();
}

template <int R, bool O, bool BV>
static hipError_t launch_sparse_bv(unsigned grid, hipStream_t s, const KernelArgs &a, bool aligned)
{
    if (aligned)
        hipLaunchKernelGGL((aesgcm_sparse_kernel<R, O, true, BV>), dim3(grid), dim3(BV ? BYVAL_WG : SPARSE_WG), 0, s, a.recs_ord, a.order, a.chunks,
                           a.nchunks, a.in, a.aad, a.out, a.result, a.slots, a.basis, a.t0, a.supp, a.hp_slots, a.hp_nslots, a.mask, a.one,
                           a.done, a.done_seq, a.clk, a.queue);
    else
        hipLaunchKernelGGL((aesgcm_sparse_kernel<R, O, false, BV>), dim3(grid), dim3(BV ? BYVAL_WG : SPARSE_WG), 0, s, a.recs_ord, a.order, a.chunks,
                           a.nchunks, a.in, a.aad, a.out, a.result, a.slots, a.basis, a.t0, a.supp, a.hp_slots, a.hp_nslots, a.mask, a.one,
                           a.done, a.done_seq, a.clk, a.queue);
    return hipGetLastError();
}

template <int R, bool O>
static hipError_t launch_sparse_one(unsigned grid, hipStream_t s, const KernelArgs &a, bool aligned)
{
    return a.recs_ord == nullptr ? launch_sparse_bv<R, O, true>(grid, s, a, aligned) : launch_sparse_bv<R, O, false>(grid, s, a, aligned);
}

int launch_batch_sparse(int rounds, bool open, unsigned grid, void *stream, const KernelArgs &a, bool aligned)
{
    hipStream_t s = static_cast<hipStream_t>(stream);
    hipError_t e;
    if (rounds == 10)
        e = open ? launch_sparse_one<10, true>(grid, s, a, aligned) : launch_sparse_one<10, false>(grid, s, a, aligned);
    else
        e = open ? launch_sparse_one<14, true>(grid, s, a, aligned) : launch_sparse_one<14, false>(grid, s, a, aligned);
    return (int)e;
}

} // namespace ptls_hip
