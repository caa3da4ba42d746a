/*
 * aesgcm_kernels.hip -- gfx950 (MI355X) kernels of the AES-GCM record engine besides the batch kernel
 * (batch_kernel.h, instantiated in batch_g*.hip): TLS 1.3 header / inner-plaintext kernels, the
 * header-protection ECB kernel, key setup, the synthetic record generator, and the host launchers.
 */
#include "batch_kernel.h"
#include "gf128.h"

namespace ptls_hip {

/* TLS 1.3 record headers (build_aad, lib/picotls.c:696-703): 17 03 03 BE16(len + 16) at hdr + aad_off of
 * every record flagged PTLS_HIP_RECORD_TLS13_TYPE; the seal kernel then reads them back as the AAD. */
__global__ void __launch_bounds__(256) tls13_header_kernel(const ptls_hip_record_t *__restrict__ recs, uint32_t n, uint8_t *hdr)
{
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const ptls_hip_record_t r = recs[i];
        if (r.flags & 1u) {
            const uint32_t reclen = r.len + 16u;
            uint8_t *h = hdr + r.aad_off;
            h[0] = 0x17;
            h[1] = 0x03;
            h[2] = 0x03;
            h[3] = (uint8_t)(reclen >> 8);
            h[4] = (uint8_t)reclen;
        }
    }
}

/* TLSInnerPlaintext of opened records (handle_input, lib/picotls.c:5877-5883): skip trailing zero padding,
 * the last non-zero byte is the content type; result = content length | type << 56. */
__global__ void __launch_bounds__(256) tls13_inner_kernel(const ptls_hip_record_t *__restrict__ recs, uint32_t n,
                                                          const uint8_t *__restrict__ out, uint64_t *__restrict__ result)
{
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        if (result[i] == ~(uint64_t)0)
            continue; /* bad record MAC */
        const ptls_hip_record_t r = recs[i];
        const uint8_t *p = out + r.out_off;
        int64_t k = (int64_t)r.len;
        uint32_t type = 0;
        /* 16 bytes at a time while a whole block lies inside the record, then byte by byte */
        while (k >= 16) {
            const V4 v = load_full(p + k - 16);
            if ((v.w0 | v.w1 | v.w2 | v.w3) != 0)
                break;
            k -= 16;
        }
        while (k > 0 && (type = p[k - 1]) == 0)
            --k;
        result[i] = k == 0 ? ~(uint64_t)1 : (uint64_t)(k - 1) | ((uint64_t)type << 56);
    }
}

/* Standalone header-protection masks (receive side): mask + mask_off = AES-ECB(hp key, src + sample_off),
 * one record per lane, grid-stride.  Same replicated T-tables as the batch kernel (at LDS_AES). */
template <int ROUNDS>
__global__ void __launch_bounds__(256) aesecb_batch_kernel(const ptls_hip_supp_t *__restrict__ supp, uint32_t n,
                                                           const uint8_t *__restrict__ src, uint8_t *__restrict__ mask,
                                                           const KeySlot *__restrict__ hp_slots, uint32_t hp_nslots,
                                                           const uint32_t *__restrict__ t0, uint32_t *done, uint32_t done_seq)
{
    __shared__ __attribute__((aligned(16))) uint8_t lds[LDS_AES + 65536];
    build_aes_tables<256>(lds, LDS_AES, t0);
    __syncthreads();
    const uint32_t lb_aes = (uint32_t)(threadIdx.x & 31) * 4u | LDS_AES;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const ptls_hip_supp_t sp = supp[i];
        if ((sp.flags & PTLS_HIP_SUPP_ENABLE) && sp.hp_key < hp_nslots) {
            const V4 m = aes_encrypt<ROUNDS>(lds, lb_aes, hp_slots[sp.hp_key].rk, load_full(src + sp.sample_off));
            store_full(mask + sp.mask_off, m);
        }
    }
    if (done != nullptr && blockIdx.x == 0 && threadIdx.x == 0) {
        /* single-block plugin call (n = 1, handled by this thread): its mask reaches system scope before the
         * completion word (a vector store) that the host spins on */
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        __hip_atomic_store(done, done_seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}


/* One AES-ECB block for the plugin's CTR / ECB objects (ptls_hip_aesecb_encrypt, the CTR cipher's do_init): the input
 * block travels in the kernel arguments (no dependent read of host staging over PCIe), one wave builds only lane slot
 * 0 of the T-tables (256 rows x {T0, T2}: every lane then reads the same slot, a broadcast), computes the block and
 * stores it into the pinned staging, then the completion word the host spins on (system scope, after the block). */
template <int ROUNDS>
__global__ void __launch_bounds__(64) aesecb_one_kernel(uint4 blk, const KeySlot *__restrict__ slot, const uint32_t *__restrict__ t0,
                                                        uint8_t *out, uint32_t *done, uint32_t done_seq)
{
    __shared__ __attribute__((aligned(16))) uint8_t lds[65536];
    const int lane = threadIdx.x;
    uint32_t t[4];
#pragma unroll
    for (int k = 0; k < 4; ++k)
        t[k] = t0[4 * lane + k];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint32_t row = (uint32_t)(4 * lane + k) * 256u;
        *reinterpret_cast<uint32_t *>(lds + row) = t[k];
        *reinterpret_cast<uint32_t *>(lds + row + 128) = (t[k] << 16) | (t[k] >> 16);
    }
    __syncthreads();
    const V4 m = aes_encrypt<ROUNDS>(lds, 0u, slot->rk, V4{blk.x, blk.y, blk.z, blk.w});
    if (lane == 0) {
        store_full(out, m);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        __hip_atomic_store(done, done_seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

constexpr uint32_t KEYSETUP_WIDE_MAX = 4096; /* slots up to which key setup runs one wave per slot (keysetup_wide_kernel) */

/* ======================================================================================= *
 *  key setup: one thread per key slot (setup_crypto, lib/fusion.c:1184-1206, :984-1010)    *
 * ======================================================================================= */

__device__ __forceinline__ U128 u128_from_raw(V4 v)
{
    return U128{__builtin_bswap64((uint64_t)v.w0 | ((uint64_t)v.w1 << 32)), __builtin_bswap64((uint64_t)v.w2 | ((uint64_t)v.w3 << 32))};
}

__device__ __forceinline__ V4 u128_to_raw(U128 u)
{
    const uint64_t a = __builtin_bswap64(u.hi), b = __builtin_bswap64(u.lo);
    return V4{(uint32_t)a, (uint32_t)(a >> 32), (uint32_t)b, (uint32_t)(b >> 32)};
}

__device__ __forceinline__ uint8_t sbox_of(const uint32_t *t0, uint8_t x)
{
    return (uint8_t)(t0[x] >> 8);
}

__device__ __forceinline__ uint8_t xtime8(uint8_t a)
{
    return (uint8_t)((a << 1) ^ ((a & 0x80) ? 0x1b : 0));
}

/* FIPS-197 key expansion (words as raw little-endian uint32, 60 entries, the unused ones 0) and H = E_K(0^128)
 * with a byte-oriented AES (setup only) */
__device__ V4 expand_key_h(const uint8_t *key, int key_size, const uint32_t *t0, uint32_t (&w)[60], int &rounds)
{
    const int nk = key_size / 4, total = 4 * (nk + 6 + 1);
    rounds = nk + 6;
    for (int i = 0; i < nk; ++i)
        w[i] = (uint32_t)key[4 * i] | ((uint32_t)key[4 * i + 1] << 8) | ((uint32_t)key[4 * i + 2] << 16) |
               ((uint32_t)key[4 * i + 3] << 24);
    uint8_t rcon = 1;
    for (int i = nk; i < 60; ++i) {
        if (i >= total) {
            w[i] = 0;
            continue;
        }
        uint32_t t = w[i - 1];
        if (i % nk == 0) {
            t = (t >> 8) | (t << 24); /* RotWord on raw bytes */
            t = (uint32_t)sbox_of(t0, t & 0xff) | ((uint32_t)sbox_of(t0, (t >> 8) & 0xff) << 8) |
                ((uint32_t)sbox_of(t0, (t >> 16) & 0xff) << 16) | ((uint32_t)sbox_of(t0, t >> 24) << 24);
            t ^= rcon;
            rcon = xtime8(rcon);
        } else if (nk > 6 && i % nk == 4) {
            t = (uint32_t)sbox_of(t0, t & 0xff) | ((uint32_t)sbox_of(t0, (t >> 8) & 0xff) << 8) |
                ((uint32_t)sbox_of(t0, (t >> 16) & 0xff) << 16) | ((uint32_t)sbox_of(t0, t >> 24) << 24);
        }
        w[i] = w[i - nk] ^ t;
    }
    uint8_t s[16], tmp[16];
    for (int i = 0; i < 16; ++i)
        s[i] = (uint8_t)(w[i >> 2] >> (8 * (i & 3)));
    for (int rr = 1; rr <= rounds; ++rr) {
        for (int c = 0; c < 4; ++c)
            for (int row = 0; row < 4; ++row)
                tmp[4 * c + row] = sbox_of(t0, s[4 * ((c + row) & 3) + row]);
        if (rr != rounds) {
            for (int c = 0; c < 4; ++c) {
                const uint8_t a0 = tmp[4 * c], a1 = tmp[4 * c + 1], a2 = tmp[4 * c + 2], a3 = tmp[4 * c + 3];
                const uint8_t all = a0 ^ a1 ^ a2 ^ a3;
                s[4 * c + 0] = a0 ^ all ^ xtime8(a0 ^ a1);
                s[4 * c + 1] = a1 ^ all ^ xtime8(a1 ^ a2);
                s[4 * c + 2] = a2 ^ all ^ xtime8(a2 ^ a3);
                s[4 * c + 3] = a3 ^ all ^ xtime8(a3 ^ a0);
            }
        } else {
            for (int i = 0; i < 16; ++i)
                s[i] = tmp[i];
        }
        for (int i = 0; i < 16; ++i)
            s[i] ^= (uint8_t)(w[4 * rr + (i >> 2)] >> (8 * (i & 3)));
    }
    V4 h;
    h.w0 = (uint32_t)s[0] | ((uint32_t)s[1] << 8) | ((uint32_t)s[2] << 16) | ((uint32_t)s[3] << 24);
    h.w1 = (uint32_t)s[4] | ((uint32_t)s[5] << 8) | ((uint32_t)s[6] << 16) | ((uint32_t)s[7] << 24);
    h.w2 = (uint32_t)s[8] | ((uint32_t)s[9] << 8) | ((uint32_t)s[10] << 16) | ((uint32_t)s[11] << 24);
    h.w3 = (uint32_t)s[12] | ((uint32_t)s[13] << 8) | ((uint32_t)s[14] << 16) | ((uint32_t)s[15] << 24);
    return h;
}

__device__ void write_slot_keys(KeySlot *slot, const uint32_t (&w)[60], int rounds, const uint8_t *iv)
{
    for (int i = 0; i < 60; ++i)
        slot->rk[i] = w[i];
    slot->rounds = (uint32_t)rounds;
    for (int i = 0; i < 3; ++i)
        slot->iv[i] = (uint32_t)iv[4 * i] | ((uint32_t)iv[4 * i + 1] << 8) | ((uint32_t)iv[4 * i + 2] << 16) |
                      ((uint32_t)iv[4 * i + 3] << 24);
}

__global__ void keysetup_kernel(KeySlot *slots, uint32_t *basis, const uint8_t *keys, const uint8_t *ivs, uint32_t first,
                                uint32_t count, int key_size, const uint32_t *t0)
{
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= count)
        return;
    KeySlot *slot = slots + first + k;
    uint32_t w[60];
    int rounds;
    const V4 h = expand_key_h(keys + (size_t)k * key_size, key_size, t0, w, rounds);
    write_slot_keys(slot, w, rounds, ivs + 12 * (size_t)k);

    U128 p = u128_from_raw(h);
    uint4 *bs = reinterpret_cast<uint4 *>(basis) + (size_t)(first + k) * BASIS_VECS;
    for (int t = 0; t < NPOW; ++t) {
        if (t != 0)
            p = gf_square(p);
        const V4 pr = u128_to_raw(p);
        slot->hpow[t][0] = pr.w0;
        slot->hpow[t][1] = pr.w1;
        slot->hpow[t][2] = pr.w2;
        slot->hpow[t][3] = pr.w3;
        U128 b = p;
        for (int e = 0; e < 128; ++e) {
            const V4 br = u128_to_raw(b);
            bs[t * 128 + e] = make_uint4(br.w0, br.w1, br.w2, br.w3);
            b = gf_mul_xpow(b, 1);
        }
    }
    /* H^1 .. H^128 (the sparse kernel's lane q multiplies its partial sum by H^(q+1); a two-wave single record element i
     * by H^(N - i)) */
    const U128 hh = u128_from_raw(h);
    U128 pk = hh;
    for (int q = 0; q < LANE_POWS; ++q) {
        const V4 pr = u128_to_raw(pk);
        bs[NPOW * 128 + q] = make_uint4(pr.w0, pr.w1, pr.w2, pr.w3);
        pk = gf_mul_bitserial(pk, hh);
    }
}

/* The same outputs with one 64-lane wave per key slot, for a few slots at a time (picotls's setup_crypto keys ONE
 * context, so this is the latency of ptls_aead_new): every lane expands the key and squares H up to H^(2^(NPOW-1))
 * itself (squaring is linear: a bit spread and one fold, gf128.h), lane j writes basis vectors e = j and j + 64 of
 * every plane (P * x^e by one shift and fold each), the planes of H^1 .. H^64 go to LDS and become 4-bit window tables
 * (32 positions x 16 values), and the lane powers H^(j+1), H^(j+65) are at most seven table products (32 lookups each)
 * of the squares.  Round 3 did the squarings and products bit-serially (1 408 VALU each) and the basis by up to 127
 * single shifts per vector: 75 us per slot. */
constexpr int KS_TABS = 7; /* window tables of H^(2^t), t < 7: the factors of H^1 .. H^128 */

__global__ void __launch_bounds__(64) keysetup_wide_kernel(KeySlot *slots, uint32_t *basis, const uint8_t *keys,
                                                           const uint8_t *ivs, uint32_t first, int key_size, const uint32_t *t0)
{
    static_assert(LANE_POWS == 128 && NPOW >= KS_TABS, "two lane powers per lane; H^(j+1), H^(j+65) from the squares H^(2^t), t < 7");
    __shared__ U128 planes[KS_TABS * 128];
    __shared__ U128 tabs[KS_TABS * 32 * 16];
    const uint32_t k = blockIdx.x;
    const int j = (int)threadIdx.x;
    KeySlot *slot = slots + first + k;
    uint4 *bs = reinterpret_cast<uint4 *>(basis) + (size_t)(first + k) * BASIS_VECS;
    uint32_t w[60];
    int rounds;
    const V4 h = expand_key_h(keys + (size_t)k * key_size, key_size, t0, w, rounds);
    U128 pw[NPOW];
    pw[0] = u128_from_raw(h);
    for (int t = 1; t < NPOW; ++t)
        pw[t] = gf_square(pw[t - 1]);
    if (j == 0) {
        write_slot_keys(slot, w, rounds, ivs + 12 * (size_t)k);
        for (int t = 0; t < NPOW; ++t) {
            const V4 r = u128_to_raw(pw[t]);
            slot->hpow[t][0] = r.w0;
            slot->hpow[t][1] = r.w1;
            slot->hpow[t][2] = r.w2;
            slot->hpow[t][3] = r.w3;
        }
    }
    for (int t = 0; t < NPOW; ++t) {
        const U128 v0 = gf_mul_xpow(pw[t], j), v1 = gf_mul_xpow(v0, 64);
        const V4 r0 = u128_to_raw(v0), r1 = u128_to_raw(v1);
        bs[t * 128 + j] = make_uint4(r0.w0, r0.w1, r0.w2, r0.w3);
        bs[t * 128 + 64 + j] = make_uint4(r1.w0, r1.w1, r1.w2, r1.w3);
        if (t < KS_TABS) {
            planes[t * 128 + j] = v0;
            planes[t * 128 + 64 + j] = v1;
        }
    }
    __syncthreads();
    /* table t, position p, value v = XOR of P * x^(4p + 3 - b) over the set bits b of v (gf128.h gf_nibble's order);
     * lane j fills position j / 2, values 8 (j & 1) .. + 7 */
    for (int t = 0; t < KS_TABS; ++t) {
        const int p = j >> 1;
        for (int v = 8 * (j & 1); v < 8 * (j & 1) + 8; ++v) {
            U128 e{0, 0};
            for (int b = 0; b < 4; ++b)
                if ((v >> b) & 1)
                    e = u128_xor(e, planes[t * 128 + 4 * p + 3 - b]);
            tabs[(t * 32 + p) * 16 + v] = e;
        }
    }
    __syncthreads();
    auto mul_tab = [&](U128 a, int t) {
        U128 z{0, 0};
        for (int p = 0; p < 32; ++p)
            z = u128_xor(z, tabs[(t * 32 + p) * 16 + gf_nibble(a, p)]);
        return z;
    };
    const int q1 = j + 1; /* 1 .. 64 */
    U128 acc{0, 0};
    bool any = false;
    for (int t = 0; t < KS_TABS; ++t) {
        if ((q1 >> t) & 1) {
            acc = any ? mul_tab(acc, t) : pw[t];
            any = true;
        }
    }
    V4 r = u128_to_raw(acc);
    bs[NPOW * 128 + j] = make_uint4(r.w0, r.w1, r.w2, r.w3);
    acc = mul_tab(acc, 6); /* H^(j + 65) = H^(j + 1) * H^64 */
    r = u128_to_raw(acc);
    bs[NPOW * 128 + 64 + j] = make_uint4(r.w0, r.w1, r.w2, r.w3);
}

/* ======================================================================================= *
 *  synthetic records: record i = splitmix64 stream seeded with seed ^ i   *
 * ======================================================================================= */

__device__ __forceinline__ uint64_t splitmix_mix(uint64_t z)
{
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

__global__ void fill_records_kernel(const ptls_hip_record_t *recs, uint32_t n, uint8_t *buf, uint64_t seed, uint64_t index_base,
                                    const uint64_t *index)
{
    /* one wave per record, 16 bytes per lane per step */
    const uint32_t lane = threadIdx.x & 63;
    for (uint32_t i = blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6); i < n; i += gridDim.x * (blockDim.x / 64)) {
        const ptls_hip_record_t rec = recs[i];
        const uint64_t sd = seed ^ (index != nullptr ? index[i] : index_base + i);
        uint8_t *p = buf + rec.in_off;
        const bool al = ((reinterpret_cast<uintptr_t>(p)) & 15) == 0;
        for (uint32_t off = lane * 16; off < rec.len; off += 64 * 16) {
            const uint64_t wi = off / 8;
            const uint64_t v0 = splitmix_mix(sd + (wi + 1) * 0x9e3779b97f4a7c15ull);
            const uint64_t v1 = splitmix_mix(sd + (wi + 2) * 0x9e3779b97f4a7c15ull);
            const int nb = (int)min(16u, rec.len - off);
            const V4 v = V4{(uint32_t)v0, (uint32_t)(v0 >> 32), (uint32_t)v1, (uint32_t)(v1 >> 32)};
            if (al)
                store_block<true>(p + off, nb, v);
            else
                store_bytes(p + off, nb, v);
        }
    }
}

/* The achievable-HBM reference of bench.py's roofline (ptls_hip_device_copy): one 16-byte load and store per thread, a
 * workgroup per 4 KiB, no loop.  Measured against grid-stride forms on one MI355X (tools/copy_probe, 4 GiB, read + write
 * counted): this flat launch 6 190 GB/s (MI355X_MICROARCH.md: 6.29 TB/s for a float4 copy); 1-8 accesses per lane in
 * a grid-stride loop over 2-64 workgroups per CU 4 460-5 400, nontemporal 4 730-5 540, one slice per workgroup
 * 5 160-5 330, hipMemcpyAsync device to device 4 980 (profiles/r05_copy_probe.log). */
__global__ void __launch_bounds__(256) copy16_kernel(const uint4 *__restrict__ src, uint4 *__restrict__ dst, size_t n16)
{
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n16)
        dst[i] = src[i];
}

/* The copy transport's gap fill (pipeline.cpp pipeline_run_copy): a slice's output span comes back from the device as a
 * few large copies, so the bytes lying between its records in that span must hold the caller's own bytes first.  The host
 * gathers them into one packed buffer; workgroup g (grid-stride) copies piece g into the device staging of the output.
 * Pieces are short (a few to a few thousand bytes): bytes, one per thread. */
__global__ void __launch_bounds__(256) gap_scatter_kernel(const GapPiece *__restrict__ pieces, uint32_t n, const uint8_t *__restrict__ src,
                                                          uint8_t *__restrict__ dst)
{
    for (uint32_t g = blockIdx.x; g < n; g += gridDim.x) {
        const GapPiece p = pieces[g];
        for (uint32_t b = threadIdx.x; b < p.len; b += 256)
            dst[p.dst + b] = src[p.src + b];
    }
}

} // namespace ptls_hip

/* ======================================================================================= *
 *  host-side launchers                                                                     *
 * ======================================================================================= */
namespace ptls_hip {

/* `aligned`: every record's in/out/aad offset and the three base pointers are 16-byte aligned.  The batch
 * kernel instantiations live in batch_g{1,2,4,8,16}.hip (one translation unit per G, built in parallel). */
int launch_batch(int lanes, int rounds, bool open, int wg, unsigned grid, void *stream, const KernelArgs &a, bool aligned)
{
    switch (lanes) {
    case 1:
        return launch_batch_g1(rounds, open, wg, grid, stream, a, aligned);
    case 2:
        return launch_batch_g2(rounds, open, wg, grid, stream, a, aligned);
    case 4:
        return launch_batch_g4(rounds, open, wg, grid, stream, a, aligned);
    case 8:
        return launch_batch_g8(rounds, open, wg, grid, stream, a, aligned);
    case 16:
        return launch_batch_g16(rounds, open, wg, grid, stream, a, aligned);
    case 32:
        return launch_batch_g32(rounds, open, wg, grid, stream, a, aligned);
    case SPARSE_LANES:
        return launch_batch_sparse(rounds, open, grid, stream, a, aligned);
    default:
        return (int)hipErrorInvalidValue;
    }
}

int launch_keysetup(KeySlot *slots, uint32_t *basis, const uint8_t *keys, const uint8_t *ivs, uint32_t first, uint32_t count,
                    int key_size, const uint32_t *t0, void *stream)
{
    /* few slots: one wave per slot (latency, ~40 us); many: one thread per slot (throughput: 64K slots in ~1 ms) */
    if (count <= KEYSETUP_WIDE_MAX) {
        hipLaunchKernelGGL(keysetup_wide_kernel, dim3(count), dim3(64), 0, static_cast<hipStream_t>(stream), slots, basis, keys,
                           ivs, first, key_size, t0);
        return (int)hipGetLastError();
    }
    const unsigned threads = 64, grid = (count + threads - 1) / threads;
    hipLaunchKernelGGL(keysetup_kernel, dim3(grid), dim3(threads), 0, static_cast<hipStream_t>(stream), slots, basis, keys, ivs,
                       first, count, key_size, t0);
    return (int)hipGetLastError();
}

int launch_fill(const ptls_hip_record_t *recs, uint32_t n, uint8_t *buf, uint64_t seed, uint64_t index_base,
                const uint64_t *index, unsigned grid, void *stream)
{
    hipLaunchKernelGGL(fill_records_kernel, dim3(grid), dim3(256), 0, static_cast<hipStream_t>(stream), recs, n, buf, seed,
                       index_base, index);
    return (int)hipGetLastError();
}

int launch_copy16(void *dst, const void *src, size_t n16, void *stream)
{
    const unsigned grid = (unsigned)((n16 + 255) / 256);
    hipLaunchKernelGGL(copy16_kernel, dim3(grid), dim3(256), 0, static_cast<hipStream_t>(stream), static_cast<const uint4 *>(src),
                       static_cast<uint4 *>(dst), n16);
    return (int)hipGetLastError();
}

int launch_gap_scatter(const GapPiece *pieces, uint32_t n, const uint8_t *src, uint8_t *dst, void *stream)
{
    if (n == 0)
        return 0;
    const unsigned grid = n < 1024 ? n : 1024;
    hipLaunchKernelGGL(gap_scatter_kernel, dim3(grid), dim3(256), 0, static_cast<hipStream_t>(stream), pieces, n, src, dst);
    return (int)hipGetLastError();
}

int launch_tls13_headers(const ptls_hip_record_t *recs, uint32_t n, uint8_t *hdr, unsigned grid, void *stream)
{
    hipLaunchKernelGGL(tls13_header_kernel, dim3(grid), dim3(256), 0, static_cast<hipStream_t>(stream), recs, n, hdr);
    return (int)hipGetLastError();
}

int launch_tls13_inner(const ptls_hip_record_t *recs, uint32_t n, const uint8_t *out, uint64_t *result, unsigned grid, void *stream)
{
    hipLaunchKernelGGL(tls13_inner_kernel, dim3(grid), dim3(256), 0, static_cast<hipStream_t>(stream), recs, n, out, result);
    return (int)hipGetLastError();
}

int launch_aesecb_one(int rounds, const uint8_t *blk, const KeySlot *slot, const uint32_t *t0, uint8_t *out, uint32_t *done,
                      uint32_t done_seq, void *stream)
{
    hipStream_t s = static_cast<hipStream_t>(stream);
    uint4 b;
    __builtin_memcpy(&b, blk, 16);
    if (rounds == 10)
        hipLaunchKernelGGL(aesecb_one_kernel<10>, dim3(1), dim3(64), 0, s, b, slot, t0, out, done, done_seq);
    else
        hipLaunchKernelGGL(aesecb_one_kernel<14>, dim3(1), dim3(64), 0, s, b, slot, t0, out, done, done_seq);
    return (int)hipGetLastError();
}

int launch_aesecb(int rounds, const ptls_hip_supp_t *supp, uint32_t n, const uint8_t *src, uint8_t *mask, const KeySlot *hp_slots,
                  uint32_t hp_nslots, const uint32_t *t0, unsigned grid, void *stream, uint32_t *done, uint32_t done_seq)
{
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (rounds == 10)
        hipLaunchKernelGGL(aesecb_batch_kernel<10>, dim3(grid), dim3(256), 0, s, supp, n, src, mask, hp_slots, hp_nslots, t0, done,
                           done_seq);
    else
        hipLaunchKernelGGL(aesecb_batch_kernel<14>, dim3(grid), dim3(256), 0, s, supp, n, src, mask, hp_slots, hp_nslots, t0, done,
                           done_seq);
    return (int)hipGetLastError();
}

} // namespace ptls_hip

