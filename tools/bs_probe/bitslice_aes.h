/*
 * bitslice_aes.h -- EXPERIMENT (not linked into the engine): bit-sliced AES for gfx950, 32 blocks per
 * lane, computed on the VALU.  Measured and rejected, see EXPERIMENTS.md E3 and tools/bs_probe/README.md.
 *
 * Why it was tried: the T-table path spends 138 ds_read_b32 per AES-128 block and is bound by the
 * LDS array (128 B/clk/CU), while the VALU (4 SIMD-32 = 128 lane-ops/clk/CU, v_bitop3 for any 3-input
 * boolean function) idles half the time.  Bit-sliced, AES is pure boolean logic: no tables, no LDS.
 *
 * Layout: plane P[8*i + j] holds bit j (LSB = 0) of state byte i (FIPS-197 byte order, i = 4*col + row);
 * bit k of every plane belongs to block k (k = 0..31) of this lane.  A block in the usual register form
 * is four little-endian words w0..w3 (w0 = bytes 0..3), so the planes of word w are exactly the 32x32
 * bit transpose of {word w of block k}: P[32*w + b] bit k = bit b of word w of block k.
 *
 * Reference semantics: FIPS-197 AES as used by ptls_fusion_aesgcm_encrypt's CTR keystream
 * (lib/fusion.c:400-658, round keys of ptls_fusion_aesecb_init :857-916).  The S-box is the
 * 113-gate Boyar-Peralta circuit (eprint 2009/191); tools/bs_probe/bs_check.cpp checks it on the host
 * against the plain-C oracle (all 256 S-box inputs, full AES-128/256 blocks).
 *
 * Host-compilable (g++): the same code is unit-tested on the CPU; hipcc turns the boolean trees into
 * v_bitop3_b32.
 */
#ifndef PTLS_HIP_BITSLICE_AES_H
#define PTLS_HIP_BITSLICE_AES_H

#include <stdint.h>

#if defined(__HIPCC__)
#define BS_INL __host__ __device__ __forceinline__
#define BS_UNROLL _Pragma("unroll")
#else
#define BS_INL static inline __attribute__((always_inline))
#define BS_UNROLL _Pragma("GCC unroll 64")
#endif

namespace ptls_hip {
namespace bs {

/* an SGPR value the compiler must treat as produced here: keeps per-round key-mask arithmetic inside the
 * round instead of hoisting 1408 loop-invariant masks (SGPR spills) */
BS_INL uint32_t opaque(uint32_t x)
{
#if defined(__HIP_DEVICE_COMPILE__)
    asm volatile("" : "+s"(x));
#endif
    return x;
}

/* scheduling fence: keeps the compiler from interleaving independent S-box / column work beyond what
 * the register file holds (2 waves per SIMD = 256 VGPRs) */
BS_INL void fence()
{
#if defined(__HIP_DEVICE_COMPILE__)
    __builtin_amdgcn_sched_barrier(0);
#endif
}

/* all-ones where bit b of w is set: the bit-sliced form of a key / constant bit shared by all 32 blocks */
BS_INL uint32_t bitmask(uint32_t w, int b)
{
    return (uint32_t)((int32_t)(w << (31 - b)) >> 31);
}

/* AES S-box on the 8 planes P[O..O+7] (P[O] = LSB), in place: Boyar-Peralta, 32 AND + 81 XOR/XNOR */
template <int O, int N>
BS_INL void sbox(uint32_t (&P)[N])
{
    const uint32_t x0 = P[O + 7], x1 = P[O + 6], x2 = P[O + 5], x3 = P[O + 4];
    const uint32_t x4 = P[O + 3], x5 = P[O + 2], x6 = P[O + 1], x7 = P[O + 0];
    /* top linear layer */
    const uint32_t y14 = x3 ^ x5, y13 = x0 ^ x6, y9 = x0 ^ x3, y8 = x0 ^ x5;
    const uint32_t t0 = x1 ^ x2, y1 = t0 ^ x7, y4 = y1 ^ x3, y12 = y13 ^ y14;
    const uint32_t y2 = y1 ^ x0, y5 = y1 ^ x6, y3 = y5 ^ y8, t1 = x4 ^ y12;
    const uint32_t y15 = t1 ^ x5, y20 = t1 ^ x1, y6 = y15 ^ x7, y10 = y15 ^ t0;
    const uint32_t y11 = y20 ^ y9, y7 = x7 ^ y11, y17 = y10 ^ y11, y19 = y10 ^ y8;
    const uint32_t y16 = t0 ^ y11, y21 = y13 ^ y16, y18 = x0 ^ y16;
    /* non-linear middle: inversion in GF(2^4)^2 */
    const uint32_t t2 = y12 & y15, t3 = y3 & y6, t4 = t3 ^ t2, t5 = y4 & x7;
    const uint32_t t6 = t5 ^ t2, t7 = y13 & y16, t8 = y5 & y1, t9 = t8 ^ t7;
    const uint32_t t10 = y2 & y7, t11 = t10 ^ t7, t12 = y9 & y11, t13 = y14 & y17;
    const uint32_t t14 = t13 ^ t12, t15 = y8 & y10, t16 = t15 ^ t12, t17 = t4 ^ t14;
    const uint32_t t18 = t6 ^ t16, t19 = t9 ^ t14, t20 = t11 ^ t16, t21 = t17 ^ y20;
    const uint32_t t22 = t18 ^ y19, t23 = t19 ^ y21, t24 = t20 ^ y18;
    const uint32_t t25 = t21 ^ t22, t26 = t21 & t23, t27 = t24 ^ t26, t28 = t25 & t27;
    const uint32_t t29 = t28 ^ t22, t30 = t23 ^ t24, t31 = t22 ^ t26, t32 = t31 & t30;
    const uint32_t t33 = t32 ^ t24, t34 = t23 ^ t33, t35 = t27 ^ t33, t36 = t24 & t35;
    const uint32_t t37 = t36 ^ t34, t38 = t27 ^ t36, t39 = t29 & t38, t40 = t25 ^ t39;
    const uint32_t t41 = t40 ^ t37, t42 = t29 ^ t33, t43 = t29 ^ t40, t44 = t33 ^ t37;
    const uint32_t t45 = t42 ^ t41;
    const uint32_t z0 = t44 & y15, z1 = t37 & y6, z2 = t33 & x7, z3 = t43 & y16;
    const uint32_t z4 = t40 & y1, z5 = t29 & y7, z6 = t42 & y11, z7 = t45 & y17;
    const uint32_t z8 = t41 & y10, z9 = t44 & y12, z10 = t37 & y3, z11 = t33 & y4;
    const uint32_t z12 = t43 & y13, z13 = t40 & y5, z14 = t29 & y2, z15 = t42 & y9;
    const uint32_t z16 = t45 & y14, z17 = t41 & y8;
    /* bottom linear layer */
    const uint32_t t46 = z15 ^ z16, t47 = z10 ^ z11, t48 = z5 ^ z13, t49 = z9 ^ z10;
    const uint32_t t50 = z2 ^ z12, t51 = z2 ^ z5, t52 = z7 ^ z8, t53 = z0 ^ z3;
    const uint32_t t54 = z6 ^ z7, t55 = z16 ^ z17, t56 = z12 ^ t48, t57 = t50 ^ t53;
    const uint32_t t58 = z4 ^ t46, t59 = z3 ^ t54, t60 = t46 ^ t57, t61 = z14 ^ t57;
    const uint32_t t62 = t52 ^ t58, t63 = t49 ^ t58, t64 = z4 ^ t59, t65 = t61 ^ t62;
    const uint32_t t66 = z1 ^ t63;
    const uint32_t s0 = t59 ^ t63, s6 = t56 ^ ~t62, s7 = t48 ^ ~t60, t67 = t64 ^ t65;
    const uint32_t s3 = t53 ^ t66, s4 = t51 ^ t66, s5 = t47 ^ t65, s1 = t64 ^ ~s3;
    const uint32_t s2 = t55 ^ ~t67;
    P[O + 7] = s0;
    P[O + 6] = s1;
    P[O + 5] = s2;
    P[O + 4] = s3;
    P[O + 3] = s4;
    P[O + 2] = s5;
    P[O + 1] = s6;
    P[O + 0] = s7;
}

/* SubBytes on all 16 bytes */
BS_INL void sub_bytes(uint32_t (&P)[128])
{
    sbox<0>(P), sbox<8>(P), sbox<16>(P), sbox<24>(P);
    sbox<32>(P), sbox<40>(P), sbox<48>(P), sbox<56>(P);
    sbox<64>(P), sbox<72>(P), sbox<80>(P), sbox<88>(P);
    sbox<96>(P), sbox<104>(P), sbox<112>(P), sbox<120>(P);
}

/* xtime (multiply by 02 in GF(2^8), polynomial 0x11b) of the planes d[0..7], bit j of the result */
template <int J>
BS_INL uint32_t xt(const uint32_t (&d)[8])
{
    return J == 0 ? d[7] : (J == 1 || J == 3 || J == 4) ? (d[J - 1] ^ d[7]) : d[J - 1];
}

/* one output byte of MixColumns + AddRoundKey: b = a_r ^ (a0^a1^a2^a3) ^ xtime(a_r ^ a_{r+1}) ^ k */
template <int J>
BS_INL uint32_t mix_bit(uint32_t ar, uint32_t t, const uint32_t (&d)[8], uint32_t k)
{
    return ar ^ t ^ xt<J>(d) ^ k;
}

/* output column C of a round (rk = the round's 4 key words): SubBytes of its four input bytes, ShiftRows
 * (output column c, row r takes input byte (row r, column c + r)), MixColumns, AddRoundKey */
template <bool MIX, int C>
BS_INL void column(uint32_t (&P)[128], uint32_t (&N)[128], const uint32_t *rk)
{
    {
        constexpr int c = C;
        constexpr int i0 = 8 * (4 * ((c + 0) & 3) + 0), i1 = 8 * (4 * ((c + 1) & 3) + 1);
        constexpr int i2 = 8 * (4 * ((c + 2) & 3) + 2), i3 = 8 * (4 * ((c + 3) & 3) + 3);
        sbox<i0>(P), sbox<i1>(P), sbox<i2>(P), sbox<i3>(P);
        const uint32_t kw = opaque(rk[c]);
        if (MIX) {
            uint32_t t[8], d0[8], d1[8], d2[8], d3[8];
            BS_UNROLL
            for (int j = 0; j < 8; ++j) {
                t[j] = P[i0 + j] ^ P[i1 + j] ^ P[i2 + j] ^ P[i3 + j];
                d0[j] = P[i0 + j] ^ P[i1 + j];
                d1[j] = P[i1 + j] ^ P[i2 + j];
                d2[j] = P[i2 + j] ^ P[i3 + j];
                d3[j] = P[i3 + j] ^ P[i0 + j];
            }
#define BS_MIXROW(R, IR, D)                                                                                     \
    N[8 * (4 * c + R) + 0] = mix_bit<0>(P[IR + 0], t[0], D, bitmask(kw, 8 * R + 0));                             \
    N[8 * (4 * c + R) + 1] = mix_bit<1>(P[IR + 1], t[1], D, bitmask(kw, 8 * R + 1));                             \
    N[8 * (4 * c + R) + 2] = mix_bit<2>(P[IR + 2], t[2], D, bitmask(kw, 8 * R + 2));                             \
    N[8 * (4 * c + R) + 3] = mix_bit<3>(P[IR + 3], t[3], D, bitmask(kw, 8 * R + 3));                             \
    N[8 * (4 * c + R) + 4] = mix_bit<4>(P[IR + 4], t[4], D, bitmask(kw, 8 * R + 4));                             \
    N[8 * (4 * c + R) + 5] = mix_bit<5>(P[IR + 5], t[5], D, bitmask(kw, 8 * R + 5));                             \
    N[8 * (4 * c + R) + 6] = mix_bit<6>(P[IR + 6], t[6], D, bitmask(kw, 8 * R + 6));                             \
    N[8 * (4 * c + R) + 7] = mix_bit<7>(P[IR + 7], t[7], D, bitmask(kw, 8 * R + 7));
            BS_MIXROW(0, i0, d0)
            BS_MIXROW(1, i1, d1)
            BS_MIXROW(2, i2, d2)
            BS_MIXROW(3, i3, d3)
#undef BS_MIXROW
        } else {
            BS_UNROLL
            for (int j = 0; j < 8; ++j) {
                N[8 * (4 * c + 0) + j] = P[i0 + j] ^ bitmask(kw, 0 + j);
                N[8 * (4 * c + 1) + j] = P[i1 + j] ^ bitmask(kw, 8 + j);
                N[8 * (4 * c + 2) + j] = P[i2 + j] ^ bitmask(kw, 16 + j);
                N[8 * (4 * c + 3) + j] = P[i3 + j] ^ bitmask(kw, 24 + j);
            }
        }
    }
    fence();
}

/* one round: SubBytes + ShiftRows + MixColumns (unless the last) + AddRoundKey, one output column at a
 * time (the column's four input bytes are S-boxed right before they are mixed) */
template <bool MIX>
BS_INL void round(uint32_t (&P)[128], const uint32_t *rk)
{
    uint32_t N[128];
    column<MIX, 0>(P, N, rk);
    column<MIX, 1>(P, N, rk);
    column<MIX, 2>(P, N, rk);
    column<MIX, 3>(P, N, rk);
    BS_UNROLL
    for (int i = 0; i < 128; ++i)
        P[i] = N[i];
}

BS_INL void add_round_key(uint32_t (&P)[128], const uint32_t *rk)
{
    BS_UNROLL
    for (int i = 0; i < 128; ++i)
        P[i] ^= bitmask(opaque(rk[i >> 5]), i & 31);
}

/* full AES encryption of the 32 bit-sliced blocks (rk: 4*(ROUNDS+1) raw little-endian key words) */
template <int ROUNDS>
BS_INL void encrypt(uint32_t (&P)[128], const uint32_t *rk)
{
    add_round_key(P, rk);
    BS_UNROLL
    for (int r = 1; r < ROUNDS; ++r)
        round<true>(P, rk + 4 * r);
    round<false>(P, rk + 4 * ROUNDS);
    fence();
}

/* the same with a runtime loop over the middle rounds: one round body of code instead of ROUNDS - 1
 * (instruction-cache footprint); the ShiftRows renaming costs register moves at the back edge */
template <int ROUNDS>
BS_INL void encrypt_rolled(uint32_t (&P)[128], const uint32_t *rk)
{
    add_round_key(P, rk);
#pragma unroll 1
    for (int r = 1; r < ROUNDS; ++r)
        round<true>(P, rk + 4 * r);
    round<false>(P, rk + 4 * ROUNDS);
    fence();
}

/* in-place 32x32 bit transpose of P[B..B+31]: afterwards P[B+b] bit k = old P[B+k] bit b */
template <int B>
BS_INL void transpose32(uint32_t (&P)[128])
{
#define BS_SWAP(J, M)                                                                                           \
    BS_UNROLL                                                                                                   \
    for (int k = 0; k < 32; ++k)                                                                                \
        if ((k & J) == 0) {                                                                                     \
            const uint32_t x = ((P[B + k] >> J) ^ P[B + k + J]) & M;                                            \
            P[B + k + J] ^= x;                                                                                  \
            P[B + k] ^= x << J;                                                                                 \
        }
    BS_SWAP(16, 0x0000ffffu)
    BS_SWAP(8, 0x00ff00ffu)
    BS_SWAP(4, 0x0f0f0f0fu)
    BS_SWAP(2, 0x33333333u)
    BS_SWAP(1, 0x55555555u)
#undef BS_SWAP
}

/* blocks <-> planes: on entry P[32*w + k] = word w of block k; on exit the planes (and vice versa) */
BS_INL void transpose_all(uint32_t (&P)[128])
{
    transpose32<0>(P);
    fence();
    transpose32<32>(P);
    fence();
    transpose32<64>(P);
    fence();
    transpose32<96>(P);
    fence();
}

} // namespace bs
} // namespace ptls_hip

#endif
