// Host check of csrc/gf128.h (tests/test_gf128.py): every fast GF(2^128) form of the key setup against the textbook
// bit-serial product with an independent multiply-by-x.  Prints "ok" or the first mismatch.
#include <cstdio>
#include <cstdint>
#include <random>
#define GF128_FN static inline
#include "gf128.h"
using namespace ptls_hip;

static U128 mulx_ref(U128 v)  // SP 800-38D: V >> 1, xor R if the dropped bit was set
{
    const uint64_t c = v.lo & 1;
    U128 o{v.hi >> 1, (v.lo >> 1) | (v.hi << 63)};
    if (c)
        o.hi ^= 0xe100000000000000ull;
    return o;
}

static U128 mul_ref(U128 x, U128 y)
{
    U128 z{0, 0}, v = y;
    for (int i = 0; i < 128; ++i) {
        const uint64_t bit = i < 64 ? (x.hi >> (63 - i)) & 1 : (x.lo >> (127 - i)) & 1;
        if (bit) {
            z.hi ^= v.hi;
            z.lo ^= v.lo;
        }
        v = mulx_ref(v);
    }
    return z;
}

static bool eq(U128 a, U128 b) { return a.hi == b.hi && a.lo == b.lo; }

int main()
{
    std::mt19937_64 g(7);
    for (int it = 0; it < 3000; ++it) {
        U128 p{g(), g()}, a{g(), g()};
        if (it < 4) {  // edge values
            p = it == 0 ? U128{0, 1} : it == 1 ? U128{~0ull, ~0ull} : it == 2 ? U128{1ull << 63, 0} : U128{0, 0};
            a = p;
        }
        U128 r = p;
        for (int s = 0; s <= 121; ++s) {
            if (!eq(gf_mul_xpow(p, s), r)) {
                printf("mul_xpow s=%d it=%d\n", s, it);
                return 1;
            }
            if (s <= 31 && !eq(gf_mul_xpow31(p, (uint32_t)s), r)) {
                printf("mul_xpow31 s=%d it=%d\n", s, it);
                return 1;
            }
            r = mulx_ref(r);
        }
        if (!eq(gf_square(a), mul_ref(a, a))) {
            printf("square it=%d\n", it);
            return 1;
        }
        if (!eq(gf_mul_bitserial(a, p), mul_ref(a, p))) {
            printf("bitserial it=%d\n", it);
            return 1;
        }
        // 4-bit window product from the plane P * x^e (the key setup's LDS tables)
        U128 plane[128];
        for (int e = 0; e < 128; ++e)
            plane[e] = e < 64 ? gf_mul_xpow(p, e) : gf_mul_xpow(gf_mul_xpow(p, e - 64), 64);
        U128 acc{0, 0};
        for (int q = 0; q < 32; ++q) {
            const int v = gf_nibble(a, q);
            U128 t{0, 0};
            for (int b = 0; b < 4; ++b)
                if ((v >> b) & 1)
                    t = u128_xor(t, plane[4 * q + 3 - b]);
            acc = u128_xor(acc, t);
        }
        if (!eq(acc, mul_ref(a, p))) {
            printf("window it=%d\n", it);
            return 1;
        }
    }
    printf("ok\n");
    return 0;
}
