/*
 * gf128.h -- GF(2^128) arithmetic of GCM for key setup (keysetup_wide_kernel), in the U128 view: hi holds raw bytes 0..7
 * big-endian, lo raw bytes 8..15, so value bit 127 - i is the coefficient of x^i (SP 800-38D's bit order) and a
 * multiplication by x is a right shift by one with R = 11100001 || 0^120 folded in for the bit that falls off.
 * Written for host and device: tests/test_gf128.py compiles it on the host and checks every function against the
 * bit-serial product (SP 800-38D Algorithm 1) before the key setup relies on it.
 */
#ifndef PTLS_HIP_GF128_H
#define PTLS_HIP_GF128_H

#include <stdint.h>

#ifndef GF128_FN
#define GF128_FN __host__ __device__ __forceinline__
#endif

namespace ptls_hip {

struct U128 {
    uint64_t hi, lo; /* big-endian view: hi holds raw bytes 0..7 (byte 0 most significant) */
};

GF128_FN U128 u128_xor(U128 a, U128 b)
{
    return U128{a.hi ^ b.hi, a.lo ^ b.lo};
}

/* logical shifts of the 128-bit value, 0 <= s <= 127 */
GF128_FN U128 u128_shr(U128 a, int s)
{
    if (s == 0)
        return a;
    if (s >= 64)
        return U128{0, a.hi >> (s - 64)};
    return U128{a.hi >> s, (a.lo >> s) | (a.hi << (64 - s))};
}

GF128_FN U128 u128_shl(U128 a, int s)
{
    if (s == 0)
        return a;
    if (s >= 64)
        return U128{a.lo << (s - 64), 0};
    return U128{(a.hi << s) | (a.lo >> (64 - s)), a.lo << s};
}

/* the low s bits of the value, 0 <= s <= 127 */
GF128_FN U128 u128_low(U128 a, int s)
{
    if (s == 0)
        return U128{0, 0};
    if (s >= 64)
        return U128{s == 64 ? 0 : a.hi & ((~0ull) >> (128 - s)), a.lo};
    return U128{0, a.lo & ((~0ull) >> (64 - s))};
}

/* P * x^s for 0 <= s <= 121: the s bits shifted out (D, the coefficients of x^(128-s) .. x^127) come back as
 * D * x^(128 - s) * (x^128 mod g) = D * (1 + x + x^2 + x^7) placed at x^(128-s)..: in value bits, D << (128 - s),
 * << (127 - s), << (126 - s), << (121 - s).  None of those folds reaches past x^127 again while s <= 121. */
GF128_FN U128 gf_mul_xpow(U128 p, int s)
{
    if (s == 0)
        return p;
    const U128 d = u128_low(p, s);
    U128 r = u128_shr(p, s);
    r = u128_xor(r, u128_shl(d, 128 - s));
    r = u128_xor(r, u128_shl(d, 127 - s));
    r = u128_xor(r, u128_shl(d, 126 - s));
    return u128_xor(r, u128_shl(d, 121 - s));
}

/* P * x^s for a per-lane 0 <= s <= 31, branch-free (every shift amount stays within 0..63, where 64-bit shifts are
 * defined on host and device alike): the s dropped bits D = the low s bits of lo fold back as D << (64 - s), << (63 - s),
 * << (62 - s), << (57 - s), all inside hi.  D << (64 - s) is written (D << 1) << (63 - s) so that s = 0 shifts by 63. */
GF128_FN U128 gf_mul_xpow31(U128 p, uint32_t s)
{
    const uint64_t d = p.lo & ((1ull << s) - 1ull);
    U128 r{p.hi >> s, (p.lo >> s) | ((p.hi << 1) << (63u - s))};
    r.hi ^= ((d << 1) << (63u - s)) ^ (d << (63u - s)) ^ (d << (62u - s)) ^ (d << (57u - s));
    return r;
}

/* bit m of the 32-bit x to bit 2m of the result */
GF128_FN uint64_t spread32(uint64_t x)
{
    x &= 0xffffffffull;
    x = (x | (x << 16)) & 0x0000ffff0000ffffull;
    x = (x | (x << 8)) & 0x00ff00ff00ff00ffull;
    x = (x | (x << 4)) & 0x0f0f0f0f0f0f0f0full;
    x = (x | (x << 2)) & 0x3333333333333333ull;
    return (x | (x << 1)) & 0x5555555555555555ull;
}

/* a^2: a_i moves to x^(2i) (squaring is linear over GF(2)); the degrees 0..126 form L, the degrees 128..254 form
 * H * x^128 = H * (1 + x + x^2 + x^7) mod g.  Coefficient i of a is value bit 127 - i, and x^(2i) is value bit 127 - 2i
 * of its half, so each 32-bit quarter of a spreads to one 64-bit word, shifted up by one. */
GF128_FN U128 gf_square(U128 a)
{
    const U128 l = U128{spread32(a.hi >> 32) << 1, spread32(a.hi) << 1};
    const U128 h = U128{spread32(a.lo >> 32) << 1, spread32(a.lo) << 1};
    U128 r = u128_xor(l, h);
    r = u128_xor(r, gf_mul_xpow(h, 1));
    r = u128_xor(r, gf_mul_xpow(h, 2));
    return u128_xor(r, gf_mul_xpow(h, 7));
}

/* SP 800-38D Algorithm 1, bit-serial (the reference the fast forms are checked against; setup of many slots) */
GF128_FN U128 gf_mul_bitserial(U128 x, U128 y)
{
    U128 z{0, 0}, v = y;
    for (int i = 0; i < 128; ++i) {
        const uint64_t bit = i < 64 ? (x.hi >> (63 - i)) & 1 : (x.lo >> (127 - i)) & 1;
        if (bit)
            z = u128_xor(z, v);
        v = gf_mul_xpow(v, 1);
    }
    return z;
}

/* 4-bit window tables of a fixed multiplier P: entry [p][v] = the product of P with the element whose coefficients
 * x^(4p) .. x^(4p+3) are v's bits 3 .. 0 and zero elsewhere, i.e. the XOR of P * x^(4p + 3 - b) over the set bits b of
 * v.  A * P is then the XOR over p of [p][nibble p of A], nibble p = value bits 127 - 4p .. 124 - 4p. */
GF128_FN int gf_nibble(U128 a, int p)
{
    return p < 16 ? (int)((a.hi >> (60 - 4 * p)) & 15u) : (int)((a.lo >> (124 - 4 * p)) & 15u);
}

} // namespace ptls_hip

#endif
