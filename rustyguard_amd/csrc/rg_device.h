// rg_device.h -- device-side building blocks for the gfx950 AEAD kernels.
//
// ChaCha20 block (RFC 8439 §2.3) and Poly1305 (RFC 8439 §2.5) written for the
// CDNA4 VALU: 32-bit ARX on VGPRs (rotates lower to v_alignbit_b32 /
// v_perm_b32), Poly1305 in radix 2^32 with v_mad_u64_u32 products.  No MFMA:
// there is no dense contraction on this path.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rg {

// ---------------------------------------------------------------- ChaCha20
__device__ __forceinline__ uint32_t rotl(uint32_t v, int n) { return __builtin_rotateleft32(v, n); }

#define RG_QR(a, b, c, d)                         \
    a += b; d ^= a; d = rotl(d, 16);              \
    c += d; b ^= c; b = rotl(b, 12);              \
    a += b; d ^= a; d = rotl(d, 8);               \
    c += d; b ^= c; b = rotl(b, 7);

struct Key8 {
    uint32_t k[8];
};

// One 64-byte keystream block: state = consts | key | block | n0 n1 n2.
// Output words are x[i] + s[i] (little-endian keystream words).
__device__ __forceinline__ void chacha_block(const Key8 &key, uint32_t block, uint32_t n0, uint32_t n1, uint32_t n2,
                                             uint32_t out[16]) {
    uint32_t x0 = 0x61707865u, x1 = 0x3320646eu, x2 = 0x79622d32u, x3 = 0x6b206574u;
    uint32_t x4 = key.k[0], x5 = key.k[1], x6 = key.k[2], x7 = key.k[3];
    uint32_t x8 = key.k[4], x9 = key.k[5], x10 = key.k[6], x11 = key.k[7];
    uint32_t x12 = block, x13 = n0, x14 = n1, x15 = n2;
#pragma unroll
    for (int i = 0; i < 10; i++) {
        RG_QR(x0, x4, x8, x12);
        RG_QR(x1, x5, x9, x13);
        RG_QR(x2, x6, x10, x14);
        RG_QR(x3, x7, x11, x15);
        RG_QR(x0, x5, x10, x15);
        RG_QR(x1, x6, x11, x12);
        RG_QR(x2, x7, x8, x13);
        RG_QR(x3, x4, x9, x14);
    }
    out[0] = x0 + 0x61707865u;
    out[1] = x1 + 0x3320646eu;
    out[2] = x2 + 0x79622d32u;
    out[3] = x3 + 0x6b206574u;
    out[4] = x4 + key.k[0];
    out[5] = x5 + key.k[1];
    out[6] = x6 + key.k[2];
    out[7] = x7 + key.k[3];
    out[8] = x8 + key.k[4];
    out[9] = x9 + key.k[5];
    out[10] = x10 + key.k[6];
    out[11] = x11 + key.k[7];
    out[12] = x12 + block;
    out[13] = x13 + n0;
    out[14] = x14 + n1;
    out[15] = x15 + n2;
}

// ---------------------------------------------------------------- Poly1305
// Accumulator h = h0 + h1 2^32 + h2 2^64 + h3 2^96 + h4 2^128, h4 small (< 8).
struct Acc {
    uint32_t h0, h1, h2, h3, h4;
};

// Clamped multiplier r (RFC 8439 §2.5: r &= 0x0ffffffc0ffffffc0ffffffc0fffffff).
// Because r1..r3 are multiples of 4, 2^128 == 5/4 (mod 2^130-5) folds exactly:
// rr_j = r_j + (r_j >> 2) = 5 r_j / 4.
struct Mul {
    uint32_t r0, r1, r2, r3, rr1, rr2, rr3;
};

__device__ __forceinline__ Mul make_mul(uint32_t k0, uint32_t k1, uint32_t k2, uint32_t k3) {
    Mul m;
    m.r0 = k0 & 0x0fffffffu;
    m.r1 = k1 & 0x0ffffffcu;
    m.r2 = k2 & 0x0ffffffcu;
    m.r3 = k3 & 0x0ffffffcu;
    m.rr1 = m.r1 + (m.r1 >> 2);
    m.rr2 = m.r2 + (m.r2 >> 2);
    m.rr3 = m.r3 + (m.r3 >> 2);
    return m;
}

__device__ __forceinline__ uint64_t mad64(uint32_t a, uint32_t b, uint64_t c) {
    return (uint64_t)a * (uint64_t)b + c;
}

// h += m + hibit * 2^128
__device__ __forceinline__ void acc_add(Acc &h, uint32_t m0, uint32_t m1, uint32_t m2, uint32_t m3, uint32_t hibit) {
    uint64_t t = (uint64_t)h.h0 + m0;
    h.h0 = (uint32_t)t;
    t = (uint64_t)h.h1 + m1 + (t >> 32);
    h.h1 = (uint32_t)t;
    t = (uint64_t)h.h2 + m2 + (t >> 32);
    h.h2 = (uint32_t)t;
    t = (uint64_t)h.h3 + m3 + (t >> 32);
    h.h3 = (uint32_t)t;
    h.h4 = h.h4 + hibit + (uint32_t)(t >> 32);
}

// h = h * r mod 2^130-5, partially reduced (h4 <= 4 on exit).
// Bounds: h_i < 2^32, h4 < 8, r_j < 2^28, rr_j < 2^28.33 -> every column sum
// < 2^62.4 fits a u64; d4 < 2^31.6 fits a u32.
__device__ __forceinline__ void acc_mul(Acc &h, const Mul &r) {
    uint64_t d0 = mad64(h.h0, r.r0, mad64(h.h1, r.rr3, mad64(h.h2, r.rr2, (uint64_t)h.h3 * r.rr1)));
    uint64_t d1 = mad64(h.h0, r.r1, mad64(h.h1, r.r0, mad64(h.h2, r.rr3, mad64(h.h3, r.rr2, (uint64_t)h.h4 * r.rr1))));
    uint64_t d2 = mad64(h.h0, r.r2, mad64(h.h1, r.r1, mad64(h.h2, r.r0, mad64(h.h3, r.rr3, (uint64_t)h.h4 * r.rr2))));
    uint64_t d3 = mad64(h.h0, r.r3, mad64(h.h1, r.r2, mad64(h.h2, r.r1, mad64(h.h3, r.r0, (uint64_t)h.h4 * r.rr3))));
    uint32_t d4 = h.h4 * r.r0;
    d1 += d0 >> 32;
    d2 += d1 >> 32;
    d3 += d2 >> 32;
    d4 += (uint32_t)(d3 >> 32);
    // 2^130 == 5: fold bits >= 130 back in
    uint32_t c = (d4 >> 2) + (d4 & ~3u);
    uint64_t t = (uint64_t)(uint32_t)d0 + c;
    h.h0 = (uint32_t)t;
    t = (uint64_t)(uint32_t)d1 + (t >> 32);
    h.h1 = (uint32_t)t;
    t = (uint64_t)(uint32_t)d2 + (t >> 32);
    h.h2 = (uint32_t)t;
    t = (uint64_t)(uint32_t)d3 + (t >> 32);
    h.h3 = (uint32_t)t;
    h.h4 = (d4 & 3u) + (uint32_t)(t >> 32);
}

// tag = (h mod p) + s mod 2^128, written as 4 little-endian words.
__device__ __forceinline__ void acc_finish(const Acc &hin, uint32_t s0, uint32_t s1, uint32_t s2, uint32_t s3,
                                           uint32_t tag[4]) {
    Acc h = hin;
    // fold h4's bits >= 2 (h < 2^131 -> h < 2^130 + 2^128)
    uint32_t c = (h.h4 >> 2) + (h.h4 & ~3u);
    uint64_t t = (uint64_t)h.h0 + c;
    h.h0 = (uint32_t)t;
    t = (uint64_t)h.h1 + (t >> 32);
    h.h1 = (uint32_t)t;
    t = (uint64_t)h.h2 + (t >> 32);
    h.h2 = (uint32_t)t;
    t = (uint64_t)h.h3 + (t >> 32);
    h.h3 = (uint32_t)t;
    h.h4 = (h.h4 & 3u) + (uint32_t)(t >> 32);
    // g = h + 5 - 2^130; take g when it does not underflow (constant time)
    t = (uint64_t)h.h0 + 5u;
    uint32_t g0 = (uint32_t)t;
    t = (uint64_t)h.h1 + (t >> 32);
    uint32_t g1 = (uint32_t)t;
    t = (uint64_t)h.h2 + (t >> 32);
    uint32_t g2 = (uint32_t)t;
    t = (uint64_t)h.h3 + (t >> 32);
    uint32_t g3 = (uint32_t)t;
    uint32_t g4 = h.h4 + (uint32_t)(t >> 32);
    uint32_t use_g = 0u - (g4 >> 2); // all-ones when h + 5 >= 2^130
    uint32_t w0 = (h.h0 & ~use_g) | (g0 & use_g);
    uint32_t w1 = (h.h1 & ~use_g) | (g1 & use_g);
    uint32_t w2 = (h.h2 & ~use_g) | (g2 & use_g);
    uint32_t w3 = (h.h3 & ~use_g) | (g3 & use_g);
    t = (uint64_t)w0 + s0;
    tag[0] = (uint32_t)t;
    t = (uint64_t)w1 + s1 + (t >> 32);
    tag[1] = (uint32_t)t;
    t = (uint64_t)w2 + s2 + (t >> 32);
    tag[2] = (uint32_t)t;
    t = (uint64_t)w3 + s3 + (t >> 32);
    tag[3] = (uint32_t)t;
}

__device__ __forceinline__ uint64_t mix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

} // namespace rg
