/* host check of tools/bs_probe/bs8_aes.h against the oracle's FIPS-197 AES:
 *   g++ -O2 -std=c++17 -I tools/bs_probe -I oracle tools/bs_probe/bs8_check.cpp oracle/aesgcm_oracle.c -o /tmp/bs8_check
 * (tests/test_bs8.py builds and runs it) */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "bs8_aes.h"
extern "C" {
#include "aesgcm_oracle.h"
}
using namespace ptls_hip;

static uint32_t rnd32()
{
    return ((uint32_t)rand() << 16) ^ (uint32_t)rand();
}

int main()
{
    int bad = 0;
    srand(7);
    /* planes round trip */
    for (int it = 0; it < 100; ++it) {
        uint32_t W[8][4], P[32], V[8][4];
        for (int k = 0; k < 8; ++k)
            for (int c = 0; c < 4; ++c)
                W[k][c] = rnd32();
        bs8::to_planes(W, P);
        /* layout: P[4j + r] bit (8c + k) == W[k][c] bit (8r + j) */
        for (int j = 0; j < 8; ++j)
            for (int r = 0; r < 4; ++r)
                for (int c = 0; c < 4; ++c)
                    for (int k = 0; k < 8; ++k)
                        if (((P[4 * j + r] >> (8 * c + k)) & 1) != ((W[k][c] >> (8 * r + j)) & 1))
                            ++bad;
        bs8::from_planes(P, V);
        bad += memcmp(W, V, sizeof W) != 0;
    }
    printf("planes: %d mismatches\n", bad);
    int kbad = 0;
    for (int kl = 16; kl <= 32; kl += 16) {
        for (int it = 0; it < 200; ++it) {
            uint8_t key[32], rkb[240];
            for (int i = 0; i < 32; ++i)
                key[i] = (uint8_t)rand();
            const int rounds = oracle_aes_expand(key, (size_t)kl, rkb);
            uint32_t rk[60], K[14 * 32];
            memcpy(rk, rkb, 240);
            bs8::slice_key(rk, rounds, K);
            const uint32_t n0 = rnd32(), n1 = rnd32(), n2 = rnd32();
            const uint32_t stride = 1u << (rand() % 6);
            const uint32_t ctr0 = it < 100 ? (uint32_t)(rand() % 70000) : rnd32(); /* wraps too */
            uint32_t P[32], W[8][4];
            bs8::ctr_planes(P, rk, n0, n1, n2, ctr0, stride);
            if (rounds == 10)
                bs8::rounds<10>(P, K);
            else
                bs8::rounds<14>(P, K);
            bs8::from_planes(P, W);
            for (int k = 0; k < 8; ++k) {
                const uint32_t blk[4] = {n0, n1, n2, __builtin_bswap32(ctr0 + (uint32_t)k * stride)};
                uint8_t in[16], exp[16];
                memcpy(in, blk, 16);
                oracle_aes_encrypt(rkb, rounds, in, exp);
                if (memcmp(exp, W[k], 16) != 0)
                    ++kbad;
            }
        }
    }
    printf("ctr keystream: %d mismatches of %d blocks\n", kbad, 2 * 200 * 8);
    return bad || kbad ? 1 : 0;
}
