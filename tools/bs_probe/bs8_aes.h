/*
 * bs8_aes.h -- bit-sliced AES-CTR keystream, 8 blocks per lane, on the VALU (gfx950), for the batch kernel's
 * hybrid waves (EXPERIMENTS.md E3, "hybrid waves").
 *
 * Why: the T-table path (batch_kernel.h) is bound by the LDS array (138 ds_read_b32 + 16 ds_read_b128 per
 * AES-128 block, 89 % busy on c2) while the VALU idles ~55 % of the time.  Bit-sliced AES needs no tables at
 * all, so a few waves per workgroup that run their blocks bit-sliced turn idle VALU cycles into blocks; only
 * their GHASH still reads LDS (16 ds_read_b128 per block, a fifth of a T-table block).
 *
 * Layout ("packed rows"): P[4*j + r] (j = bit 0..7, r = state row 0..3) is one 32-bit word; its byte c is state
 * column c, and bit k of that byte is bit j of state byte (row r, column c) of block k (k = 0..7).  A block in
 * the usual register form is four little-endian column words W[c] (byte r = row r), so:
 *   P[4*j + r] bit (8c + k)  ==  block k, W[c] bit (8r + j).
 * ShiftRows is a byte rotation of each row word (v_alignbit), MixColumns an XOR of plane words of the same
 * column (no data movement), SubBytes the Boyar-Peralta circuit over the 8 planes of a row (eprint 2009/191:
 * 32 AND + 81 XOR/XNOR; hipcc folds the trees into v_bitop3_b32).  Round keys are pre-sliced per key slot by
 * keysetup (bs8_slice_key): K[round][4*j + r] byte c = 0xff * bit (8r + j) of round-key word c.
 *
 * Reference semantics: the AES-CTR keystream of ptls_fusion_aesgcm_encrypt / _decrypt (lib/fusion.c:400-844,
 * round keys of ptls_fusion_aesecb_init :857-916, counter block = IV ^ seq | BE32 counter, :1126-1133).
 * Host-compilable (g++) for tools/bs_probe/bs8_check.cpp, which checks it against the oracle's AES.
 */
#ifndef PTLS_HIP_BS8_AES_H
#define PTLS_HIP_BS8_AES_H

#include <stdint.h>

#if defined(__HIPCC__)
#define BS8_INL __host__ __device__ __forceinline__
#define BS8_UNROLL _Pragma("unroll")
#else /* host (the checker): plain inline functions and loops, which g++ compiles in seconds */
#define BS8_INL static inline
#define BS8_UNROLL
#endif

namespace ptls_hip {
namespace bs8 {

/* v_perm_b32(hi, lo, sel): result byte i = byte sel_i of {hi:lo} (lo = bytes 0..3), 0x0c -> 0x00 */
BS8_INL uint32_t perm(uint32_t hi, uint32_t lo, uint32_t sel)
{
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_perm(hi, lo, sel);
#else
    const uint64_t v = ((uint64_t)hi << 32) | lo;
    uint32_t o = 0;
    for (int i = 0; i < 4; ++i) {
        const uint32_t s = (sel >> (8 * i)) & 0xff;
        const uint32_t b = s < 8 ? (uint32_t)(v >> (8 * s)) & 0xff : s == 0x0c ? 0 : 0xff;
        o |= b << (8 * i);
    }
    return o;
#endif
}

/* rotate right by n bits (0 < n < 32): one v_alignbit_b32 */
BS8_INL uint32_t rotr(uint32_t x, int n)
{
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_alignbit(x, x, (uint32_t)n);
#else
    return (x >> n) | (x << (32 - n));
#endif
}

/* in-place 4x4 byte transpose: afterwards a_r byte i = old a_i byte r (8 v_perm_b32) */
BS8_INL void bytes4x4(uint32_t &a0, uint32_t &a1, uint32_t &a2, uint32_t &a3)
{
    const uint32_t t0 = perm(a1, a0, 0x06020400u), t1 = perm(a1, a0, 0x07030501u);
    const uint32_t t2 = perm(a3, a2, 0x06020400u), t3 = perm(a3, a2, 0x07030501u);
    a0 = perm(t2, t0, 0x05040100u);
    a1 = perm(t3, t1, 0x05040100u);
    a2 = perm(t2, t0, 0x07060302u);
    a3 = perm(t3, t1, 0x07060302u);
}

/* any boolean function of three words (truth-table bit a << 2 | b << 1 | c): one v_bitop3_b32 */
template <uint32_t TT>
BS8_INL uint32_t bitop3(uint32_t a, uint32_t b, uint32_t c)
{
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_bitop3_b32(a, b, c, TT);
#else
    uint32_t o = 0;
    for (int i = 0; i < 8; ++i)
        if ((TT >> i) & 1u)
            o |= ((i & 4) ? a : ~a) & ((i & 2) ? b : ~b) & ((i & 1) ? c : ~c);
    return o;
#endif
}

BS8_INL uint32_t xor3(uint32_t a, uint32_t b, uint32_t c)
{
    return bitop3<0x96>(a, b, c);
}

/* 8x8 bit transpose inside every byte lane of T[0..7]: afterwards T[j] bit (8b + k) = old T[k] bit (8b + j).
 * Three SWAPMOVE stages (bit distance 1, 2, 4), 4 VALU each (2 shifts, 2 bit-field selects). */
BS8_INL void transpose8(uint32_t (&T)[8])
{
#define BS8_SWAP(D, M)                                                                                          \
    BS8_UNROLL                                                                                                  \
    for (int k = 0; k < 8; ++k)                                                                                 \
        if ((k & D) == 0) {                                                                                     \
            const uint32_t a = T[k], b = T[k + D];                                                              \
            T[k] = bitop3<0xca>(M, a, b << D);     /* (M & a) | (~M & b << D) */                               \
            T[k + D] = bitop3<0xca>(M, a >> D, b); /* (M & a >> D) | (~M & b) */                               \
        }
    BS8_SWAP(1, 0x55555555u)
    BS8_SWAP(2, 0x33333333u)
    BS8_SWAP(4, 0x0f0f0f0fu)
#undef BS8_SWAP
}

/* AES S-box on the planes x[0] (LSB) .. x[7], in place: the Boyar-Peralta circuit mapped onto 3-input gates */
#include "bs8_sbox.h"

/* SubBytes of state row R (the 8 plane words P[4j + R]) */
template <int R>
BS8_INL void sub_row(uint32_t (&P)[32])
{
    uint32_t x[8];
    BS8_UNROLL
    for (int j = 0; j < 8; ++j)
        x[j] = P[4 * j + R];
    sbox(x);
    BS8_UNROLL
    for (int j = 0; j < 8; ++j)
        P[4 * j + R] = x[j];
}

/* ShiftRows: row r rotates left by r columns, i.e. its word right by 8r bits */
BS8_INL void shift_rows(uint32_t (&P)[32])
{
    BS8_UNROLL
    for (int j = 0; j < 8; ++j) {
        P[4 * j + 1] = rotr(P[4 * j + 1], 8);
        P[4 * j + 2] = rotr(P[4 * j + 2], 16);
        P[4 * j + 3] = rotr(P[4 * j + 3], 24);
    }
}

/* MixColumns + AddRoundKey, in place.  out(r) = a_r ^ (a0^a1^a2^a3) ^ xtime(a_r ^ a_{r+1}) ^ k; xtime on planes:
 * bit j takes bit j-1 (0x11b: bits 0, 1, 3, 4 also take bit 7) */
BS8_INL void mix_columns_ark(uint32_t (&P)[32], const uint32_t *K)
{
    uint32_t tot[8];
    BS8_UNROLL
    for (int j = 0; j < 8; ++j)
        tot[j] = xor3(P[4 * j + 0], P[4 * j + 1], P[4 * j + 2]) ^ P[4 * j + 3];
    uint32_t N[32];
    BS8_UNROLL
    for (int r = 0; r < 4; ++r) {
        const int r1 = (r + 1) & 3;
        BS8_UNROLL
        for (int j = 0; j < 8; ++j) {
            const int jm = (j + 7) & 7; /* j - 1 (j = 0: bit 7) */
            const uint32_t v = xor3(P[4 * j + r], tot[j], P[4 * jm + r]);
            if (j == 1 || j == 3 || j == 4)
                N[4 * j + r] = xor3(xor3(v, P[4 * jm + r1], P[4 * 7 + r]), P[4 * 7 + r1], K[4 * j + r]);
            else
                N[4 * j + r] = xor3(v, P[4 * jm + r1], K[4 * j + r]);
        }
    }
    BS8_UNROLL
    for (int i = 0; i < 32; ++i)
        P[i] = N[i];
}

BS8_INL void add_round_key(uint32_t (&P)[32], const uint32_t *K)
{
    BS8_UNROLL
    for (int i = 0; i < 32; ++i)
        P[i] ^= K[i];
}

/* the planes of 8 blocks (W[k][c] = column word c of block k) -> P, and back (the transform is an involution up
 * to the order of its two steps) */
BS8_INL void to_planes(const uint32_t (&W)[8][4], uint32_t (&P)[32])
{
    uint32_t T[4][8];
    BS8_UNROLL
    for (int c = 0; c < 4; ++c) {
        BS8_UNROLL
        for (int k = 0; k < 8; ++k)
            T[c][k] = W[k][c];
        transpose8(T[c]); /* T[c][j] byte r = bits of (row r, column c, bit j) over the blocks */
    }
    BS8_UNROLL
    for (int j = 0; j < 8; ++j) {
        uint32_t a0 = T[0][j], a1 = T[1][j], a2 = T[2][j], a3 = T[3][j];
        bytes4x4(a0, a1, a2, a3);
        P[4 * j + 0] = a0, P[4 * j + 1] = a1, P[4 * j + 2] = a2, P[4 * j + 3] = a3;
    }
}

BS8_INL void from_planes(const uint32_t (&P)[32], uint32_t (&W)[8][4])
{
    uint32_t T[4][8];
    BS8_UNROLL
    for (int j = 0; j < 8; ++j) {
        uint32_t a0 = P[4 * j + 0], a1 = P[4 * j + 1], a2 = P[4 * j + 2], a3 = P[4 * j + 3];
        bytes4x4(a0, a1, a2, a3);
        T[0][j] = a0, T[1][j] = a1, T[2][j] = a2, T[3][j] = a3;
    }
    BS8_UNROLL
    for (int c = 0; c < 4; ++c) {
        transpose8(T[c]);
        BS8_UNROLL
        for (int k = 0; k < 8; ++k)
            W[k][c] = T[c][k];
    }
}

/* a whitened constant column word s (the same for all 8 blocks) in sliced form: byte r of the result is 0xff
 * where bit (8r + j) of s is set.  Bit 8r + j is moved to the sign of a byte v_perm_b32 can sign-extend
 * (selectors 8..11 = the signs of bytes 1, 3, 5, 7 of {hi:lo}). */
template <int J>
BS8_INL uint32_t splat_bits(uint32_t s)
{
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_perm(s << (15 - J), s << (7 - J), 0x090b080au);
#else
    uint32_t o = 0;
    for (int r = 0; r < 4; ++r)
        o |= ((s >> (8 * r + J)) & 1u) ? 0xffu << (8 * r) : 0u;
    return o;
#endif
}

/* counter blocks (n0, n1, n2, BE32(ctr0 + k * stride)), k = 0..7, whitened with round key 0 (rk0), in sliced
 * form.  Columns 0..2 are the same for every block: their planes come from splat_bits; only the counter column is
 * transposed. */
BS8_INL void ctr_planes(uint32_t (&P)[32], const uint32_t *rk0, uint32_t n0, uint32_t n1, uint32_t n2, uint32_t ctr0,
                        uint32_t stride)
{
    const uint32_t s0 = n0 ^ rk0[0], s1 = n1 ^ rk0[1], s2 = n2 ^ rk0[2];
    uint32_t T[8];
    BS8_UNROLL
    for (int k = 0; k < 8; ++k)
        T[k] = __builtin_bswap32(ctr0 + (uint32_t)k * stride) ^ rk0[3];
    transpose8(T);
#define BS8_PLANE(J)                                                                                            \
    {                                                                                                           \
        uint32_t a0 = splat_bits<J>(s0), a1 = splat_bits<J>(s1), a2 = splat_bits<J>(s2), a3 = T[J];             \
        bytes4x4(a0, a1, a2, a3);                                                                               \
        P[4 * J + 0] = a0, P[4 * J + 1] = a1, P[4 * J + 2] = a2, P[4 * J + 3] = a3;                             \
    }
    BS8_PLANE(0) BS8_PLANE(1) BS8_PLANE(2) BS8_PLANE(3) BS8_PLANE(4) BS8_PLANE(5) BS8_PLANE(6) BS8_PLANE(7)
#undef BS8_PLANE
}

/* rounds 1..ROUNDS on sliced state P (round 0 already applied); K = sliced round keys, 32 words per round,
 * round 1 first */
/* an offset the compiler must treat as produced here: a round's key loads stay inside the round (not hoisted out of
 * the caller's loop: hundreds of SGPRs) while the pointer keeps its kernel-argument provenance, so the loads remain
 * scalar (s_load from read-only memory) */
BS8_INL uint32_t opaque_off(uint32_t o, uint32_t after)
{
#if defined(__HIP_DEVICE_COMPILE__)
    asm volatile("" : "+s"(o) : "v"(after)); /* ... and not before `after` (the state entering the round) exists */
#else
    (void)after;
#endif
    return o;
}

template <int ROUNDS>
BS8_INL void rounds(uint32_t (&P)[32], const uint32_t *K)
{
    BS8_UNROLL
    for (int r = 1; r <= ROUNDS; ++r) {
        const uint32_t *Kr = K + opaque_off(32 * (r - 1), P[0]);
        sub_row<0>(P), sub_row<1>(P), sub_row<2>(P), sub_row<3>(P);
        shift_rows(P);
        if (r < ROUNDS)
            mix_columns_ark(P, Kr);
        else
            add_round_key(P, Kr);
    }
}

/* the sliced round keys of one key: K[32 * (r - 1) + 4j + row] byte c = 0xff * bit (8 row + j) of rk[4r + c],
 * r = 1..rounds (rk = the raw little-endian round-key words) */
BS8_INL void slice_key(const uint32_t *rk, int rounds, uint32_t *K)
{
    for (int r = 1; r <= rounds; ++r)
        for (int j = 0; j < 8; ++j)
            for (int row = 0; row < 4; ++row) {
                uint32_t v = 0;
                for (int c = 0; c < 4; ++c)
                    if ((rk[4 * r + c] >> (8 * row + j)) & 1u)
                        v |= 0xffu << (8 * c);
                K[32 * (r - 1) + 4 * j + row] = v;
            }
}

} // namespace bs8
} // namespace ptls_hip

#endif
