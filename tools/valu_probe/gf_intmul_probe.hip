/* gf_intmul_probe.hip -- SURVEY.md §7's last GHASH candidate: a GF(2^128) multiply by a fixed
 * power computed on the VALU from INTEGER multiplies ("holes" masking, BearSSL's bmul32 idea) instead of the 8-bit window
 * table in LDS (16 ds_read_b128 per multiply, batch_kernel.h gh_mul_main).
 *
 *   32 x 32 carry-less product: x and y split into four bit classes (x & 0x11111111 << k); the 16 integer products of
 *   class pairs cannot carry into the bits of their own class (holes of 3 zero bits between every 4th bit: at most 8
 *   terms per output bit, sums < 16), so masking the XOR of the 4 products that land in class c recovers c's bits.
 *   16 v_mad_u64_u32 (32 x 32 -> 64) + masks / XORs per 32 x 32 product.
 *   128 x 128: two-level Karatsuba on 32-bit limbs (9 products of 32 x 32), the fixed operand's 9 limb combinations and
 *   their 4 bit classes precomputed per lane (36 VGPRs, as a per-key table would be), then the 256-bit product reduced
 *   modulo x^128 + x^7 + x^2 + x + 1 (the bit order is the polynomial's, not GCM's reflected one: the cost is the same).
 *
 * The probe checks the device product against a host bit-serial carry-less multiply + reduction (2 048 random pairs), then
 * times M dependent multiplies per lane (Horner: y = y * H ^ x, as the GHASH stretch runs them) with W waves per SIMD and
 * prints ns per multiply per wave and the VALU instructions of one multiply (from the loop's ISA: build with
 * --save-temps and count, see tools/valu_probe/README in DESIGN.md / EXPERIMENTS.md).
 *   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/valu_probe/gf_intmul_probe.hip -o tools/valu_probe/gf_intmul_probe */
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

struct U128 {
    uint64_t lo, hi;
};

static constexpr uint32_t M0 = 0x11111111u, M1 = 0x22222222u, M2 = 0x44444444u, M3 = 0x88888888u;
static constexpr uint64_t N0 = 0x1111111111111111ull, N1 = 0x2222222222222222ull, N2 = 0x4444444444444444ull,
                          N3 = 0x8888888888888888ull;

/* the fixed operand's limb, split in its four bit classes */
struct Split {
    uint32_t c0, c1, c2, c3;
};

__host__ __device__ inline Split split(uint32_t y)
{
    return Split{y & M0, y & M1, y & M2, y & M3};
}

__host__ __device__ inline uint64_t mul64(uint32_t a, uint32_t b)
{
    return (uint64_t)a * (uint64_t)b; /* v_mad_u64_u32 / v_mul_lo + v_mul_hi */
}

/* carry-less 32 x 32 -> 64 with y pre-split */
__host__ __device__ inline uint64_t clmul32(uint32_t x, const Split &y)
{
    const uint32_t x0 = x & M0, x1 = x & M1, x2 = x & M2, x3 = x & M3;
    const uint64_t z0 = mul64(x0, y.c0) ^ mul64(x1, y.c3) ^ mul64(x2, y.c2) ^ mul64(x3, y.c1);
    const uint64_t z1 = mul64(x0, y.c1) ^ mul64(x1, y.c0) ^ mul64(x2, y.c3) ^ mul64(x3, y.c2);
    const uint64_t z2 = mul64(x0, y.c2) ^ mul64(x1, y.c1) ^ mul64(x2, y.c0) ^ mul64(x3, y.c3);
    const uint64_t z3 = mul64(x0, y.c3) ^ mul64(x1, y.c2) ^ mul64(x2, y.c1) ^ mul64(x3, y.c0);
    return (z0 & N0) | (z1 & N1) | (z2 & N2) | (z3 & N3);
}

/* the fixed operand H = (h3 h2 h1 h0) as Karatsuba needs it: limbs and limb sums, split */
struct Fixed {
    Split l[9]; /* h0, h1, h0^h1, h2, h3, h2^h3, (h0^h2), (h1^h3), (h0^h2)^(h1^h3) */
};

__host__ __device__ inline Fixed fixed_of(U128 h)
{
    const uint32_t h0 = (uint32_t)h.lo, h1 = (uint32_t)(h.lo >> 32), h2 = (uint32_t)h.hi, h3 = (uint32_t)(h.hi >> 32);
    Fixed f;
    const uint32_t v[9] = {h0, h1, h0 ^ h1, h2, h3, h2 ^ h3, h0 ^ h2, h1 ^ h3, h0 ^ h2 ^ h1 ^ h3};
    for (int i = 0; i < 9; ++i)
        f.l[i] = split(v[i]);
    return f;
}

/* 64 x 64 -> 128 carry-less by one Karatsuba level over 32-bit limbs; y's three splits at f.l[k], l[k+1], l[k+2] */
__host__ __device__ inline U128 clmul64(uint64_t x, const Split &yl, const Split &yh, const Split &ys)
{
    const uint32_t xl = (uint32_t)x, xh = (uint32_t)(x >> 32);
    const uint64_t lo = clmul32(xl, yl), hi = clmul32(xh, yh), mid = clmul32(xl ^ xh, ys) ^ lo ^ hi;
    return U128{lo ^ (mid << 32), hi ^ (mid >> 32)};
}

/* x * H mod (x^128 + x^7 + x^2 + x + 1) */
__host__ __device__ inline U128 gf_mul_int(U128 x, const Fixed &f)
{
    const U128 lo = clmul64(x.lo, f.l[0], f.l[1], f.l[2]);
    const U128 hi = clmul64(x.hi, f.l[3], f.l[4], f.l[5]);
    U128 mid = clmul64(x.lo ^ x.hi, f.l[6], f.l[7], f.l[8]);
    mid.lo ^= lo.lo ^ hi.lo;
    mid.hi ^= lo.hi ^ hi.hi;
    /* 256-bit product p3 p2 p1 p0 (64-bit words) */
    const uint64_t p0 = lo.lo, p1 = lo.hi ^ mid.lo, p2 = hi.lo ^ mid.hi, p3 = hi.hi;
    /* fold the high 128 bits (p3 p2) down: r = hi * (x^7 + x^2 + x + 1), twice for the bits that spill past 128 */
    const uint64_t s3 = (p3 >> 63) ^ (p3 >> 62) ^ (p3 >> 57); /* bits of p3 * (x^7+x^2+x) above 2^192, into word 2 */
    const uint64_t q2 = p2 ^ s3;
    const uint64_t r0 = p0 ^ q2 ^ (q2 << 1) ^ (q2 << 2) ^ (q2 << 7);
    const uint64_t r1 = p1 ^ p3 ^ (p3 << 1) ^ (p3 << 2) ^ (p3 << 7) ^ (q2 >> 63) ^ (q2 >> 62) ^ (q2 >> 57);
    return U128{r0, r1};
}

/* host reference: bit-serial carry-less multiply and bit-serial reduction */
static U128 gf_mul_ref(U128 a, U128 b)
{
    uint64_t p[4] = {0, 0, 0, 0};
    for (int i = 0; i < 128; ++i) {
        if ((i < 64 ? a.lo >> i : a.hi >> (i - 64)) & 1) {
            /* p ^= b << i */
            for (int w = 0; w < 2; ++w) {
                const uint64_t bw = w ? b.hi : b.lo;
                const int bit = i + 64 * w, word = bit >> 6, sh = bit & 63;
                p[word] ^= bw << sh;
                if (sh)
                    p[word + 1] ^= bw >> (64 - sh);
            }
        }
    }
    for (int bit = 255; bit >= 128; --bit)
        if ((p[bit >> 6] >> (bit & 63)) & 1) {
            const int d = bit - 128; /* x^bit = x^d * (x^7 + x^2 + x + 1) */
            p[bit >> 6] ^= 1ull << (bit & 63);
            for (int t : {7, 2, 1, 0}) {
                const int b2 = d + t;
                p[b2 >> 6] ^= 1ull << (b2 & 63);
            }
        }
    return U128{p[0], p[1]};
}

__global__ void check_kernel(const U128 *a, const U128 *b, U128 *out, int n)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n)
        out[i] = gf_mul_int(a[i], fixed_of(b[i]));
}

/* m dependent Horner steps per lane: y = y * H ^ x (x varies per step so nothing folds) */
__global__ void __launch_bounds__(256) horner_kernel(const U128 *h, U128 *out, int m)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const Fixed f = fixed_of(h[i & 1023]);
    U128 y = U128{(uint64_t)i, (uint64_t)i * 0x9e3779b97f4a7c15ull};
    for (int k = 0; k < m; ++k) {
        y = gf_mul_int(y, f);
        y.lo ^= (uint64_t)k;
    }
    out[i] = y;
}

int main()
{
    const int n = 2048;
    U128 *ha = (U128 *)malloc(n * sizeof(U128)), *hb = (U128 *)malloc(n * sizeof(U128)), *hc = (U128 *)malloc(n * sizeof(U128));
    uint64_t s = 0x1234567;
    auto rnd = [&]() { s = s * 6364136223846793005ull + 1442695040888963407ull; return s ^ (s >> 29); };
    for (int i = 0; i < n; ++i) {
        ha[i] = U128{rnd(), rnd()};
        hb[i] = U128{rnd(), rnd()};
    }
    int host_bad = 0;
    for (int i = 0; i < n; ++i) { /* the integer method on the host first (same code) */
        const U128 r = gf_mul_int(ha[i], fixed_of(hb[i])), e = gf_mul_ref(ha[i], hb[i]);
        host_bad += (r.lo != e.lo || r.hi != e.hi);
    }
    printf("host: integer-multiply product vs bit-serial reference: %d mismatches of %d\n", host_bad, n);
    U128 *da, *db, *dc;
    CK(hipMalloc(&da, n * sizeof(U128)));
    CK(hipMalloc(&db, n * sizeof(U128)));
    CK(hipMalloc(&dc, n * sizeof(U128)));
    CK(hipMemcpy(da, ha, n * sizeof(U128), hipMemcpyHostToDevice));
    CK(hipMemcpy(db, hb, n * sizeof(U128), hipMemcpyHostToDevice));
    check_kernel<<<n / 256, 256>>>(da, db, dc, n);
    CK(hipMemcpy(hc, dc, n * sizeof(U128), hipMemcpyDeviceToHost));
    int dev_bad = 0;
    for (int i = 0; i < n; ++i) {
        const U128 e = gf_mul_ref(ha[i], hb[i]);
        dev_bad += (hc[i].lo != e.lo || hc[i].hi != e.hi);
    }
    printf("device: %d mismatches of %d\n", dev_bad, n);
    int ncu = 0;
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    const int m = 4096;
    U128 *dout;
    for (int wps : {1, 2, 4}) { /* waves per SIMD */
        const int grid = ncu * wps; /* 256 threads = 4 waves = one per SIMD per workgroup */
        CK(hipMalloc(&dout, (size_t)grid * 256 * sizeof(U128)));
        hipEvent_t a, b;
        CK(hipEventCreate(&a));
        CK(hipEventCreate(&b));
        horner_kernel<<<grid, 256>>>(da, dout, 16);
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(a));
        horner_kernel<<<grid, 256>>>(da, dout, m);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, a, b));
        const double per_mul_ns = ms * 1e6 / m;                    /* per wave (all waves run concurrently) */
        const double chip_muls_per_ns = (double)grid * 4 * 64 * m / (ms * 1e6); /* lane-multiplies per ns */
        printf("waves/SIMD %d: %.2f ms for %d dependent multiplies: %.1f ns per multiply per wave, %.1f G lane-multiplies/s "
               "chip-wide\n", wps, ms, m, per_mul_ns, chip_muls_per_ns);
        CK(hipFree(dout));
    }
    return host_bad || dev_bad;
}
