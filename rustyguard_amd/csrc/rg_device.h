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
// wave-uniform copies via s_readfirstlane.  The builtin works on int: go
// through uint32_t so that a set bit 31 is never sign-extended into a 64-bit
// value (byte offsets past 2 GiB).
__device__ __forceinline__ uint32_t uniform_u32(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }

// orders a wave's own LDS accesses across lanes (the compiler sees one lane; the hardware runs a
// wave's LDS instructions in order)
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
__device__ __forceinline__ uint64_t uniform_u64(uint64_t v) {
    return ((uint64_t)uniform_u32((uint32_t)(v >> 32)) << 32) | (uint64_t)uniform_u32((uint32_t)v);
}

__device__ __forceinline__ uint32_t rotl(uint32_t v, int n) { return __builtin_rotateleft32(v, n); }

// ----------------------------------------------------------- wave scans
// DPP moves (VALU, no LDS round trip; a shuffle through ds_bpermute costs an LDS
// latency per step).  update_dpp(old, src, ctrl, row_mask, bank_mask, bound_ctrl):
// with bound_ctrl a lane whose source is out of range reads 0; rows outside
// row_mask keep `old`.
template <int CTRL, int ROW_MASK = 0xF>
__device__ __forceinline__ uint32_t dpp0(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, ROW_MASK, 0xF, true);
}
// inclusive prefix sum over the 64 lanes: row_shr 1/2/4/8 inside rows of 16,
// then row_bcast:15 / row_bcast:31 carry the row totals up (GFX9 DPP)
__device__ __forceinline__ uint32_t wave_scan_incl(uint32_t x) {
    x += dpp0<0x111>(x);
    x += dpp0<0x112>(x);
    x += dpp0<0x114>(x);
    x += dpp0<0x118>(x);
    x += dpp0<0x142, 0xA>(x);
    x += dpp0<0x143, 0xC>(x);
    return x;
}
// inclusive prefix maximum over the 64 lanes (values >= 0; the same DPP steps)
__device__ __forceinline__ uint32_t wave_scan_max(uint32_t x) {
    x = max(x, dpp0<0x111>(x));
    x = max(x, dpp0<0x112>(x));
    x = max(x, dpp0<0x114>(x));
    x = max(x, dpp0<0x118>(x));
    x = max(x, dpp0<0x142, 0xA>(x));
    x = max(x, dpp0<0x143, 0xC>(x));
    return x;
}
// value of lane - 1 (0 for lane 0): wave_shr:1
__device__ __forceinline__ uint32_t wave_shr1(uint32_t x) { return dpp0<0x138>(x); }
// value of lane 63, wave-uniform
__device__ __forceinline__ uint32_t lane63(uint32_t x) { return (uint32_t)__builtin_amdgcn_readlane((int)x, 63); }

// Byte rotations as v_perm_b32 byte selects instead of v_alignbit_b32
// (tools/microbench.hip: ChaCha20 +4-5 % at one wave per SIMD, equal at eight).
// Selector byte i picks source byte sel_i of {v, v} (0-3 = bytes of src1).
__device__ __forceinline__ uint32_t rotl16(uint32_t v) { return __builtin_amdgcn_perm(v, v, 0x01000302u); }
__device__ __forceinline__ uint32_t rotl8(uint32_t v) { return __builtin_amdgcn_perm(v, v, 0x02010003u); }

#define RG_QR(a, b, c, d)                         \
    a += b; d ^= a; d = rotl16(d);                \
    c += d; b ^= c; b = rotl(b, 12);              \
    a += b; d ^= a; d = rotl8(d);                 \
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

// HChaCha20 (draft-irtf-cfrg-xchacha-03 §2.2): the ChaCha20 rounds over
// consts | key | nonce16 with no feed-forward; the subkey is words 0-3, 12-15.
__device__ __forceinline__ Key8 hchacha20(const Key8 &key, const uint32_t n[4]) {
    uint32_t x0 = 0x61707865u, x1 = 0x3320646eu, x2 = 0x79622d32u, x3 = 0x6b206574u;
    uint32_t x4 = key.k[0], x5 = key.k[1], x6 = key.k[2], x7 = key.k[3];
    uint32_t x8 = key.k[4], x9 = key.k[5], x10 = key.k[6], x11 = key.k[7];
    uint32_t x12 = n[0], x13 = n[1], x14 = n[2], x15 = n[3];
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
    return Key8{{x0, x1, x2, x3, x12, x13, x14, x15}};
}

// Per-packet ChaCha20 state with the block-counter-independent part of the
// first column round hoisted: of QR(0,4,8,12) QR(1,5,9,13) QR(2,6,10,14)
// QR(3,7,11,15) only the first reads word 12 (the block counter), so the other
// three are computed once per packet instead of once per 64-byte block.
struct Stream {
    Key8 key;
    uint32_t n0, n1, n2;
    uint32_t x0p;                  // 0x61707865 + k0: first step of QR(0,4,8,12)
    uint32_t c1[4], c2[4], c3[4];  // QR1..QR3 outputs (a, b, c, d) after the first column round
};

__device__ __forceinline__ Stream make_stream(const Key8 &key, uint32_t n0, uint32_t n1, uint32_t n2) {
    Stream st;
    st.key = key;
    st.n0 = n0;
    st.n1 = n1;
    st.n2 = n2;
    st.x0p = 0x61707865u + key.k[0];
    uint32_t a = 0x3320646eu, b = key.k[1], c = key.k[5], d = n0;
    RG_QR(a, b, c, d);
    st.c1[0] = a; st.c1[1] = b; st.c1[2] = c; st.c1[3] = d;
    a = 0x79622d32u; b = key.k[2]; c = key.k[6]; d = n1;
    RG_QR(a, b, c, d);
    st.c2[0] = a; st.c2[1] = b; st.c2[2] = c; st.c2[3] = d;
    a = 0x6b206574u; b = key.k[3]; c = key.k[7]; d = n2;
    RG_QR(a, b, c, d);
    st.c3[0] = a; st.c3[1] = b; st.c3[2] = c; st.c3[3] = d;
    return st;
}

// Keystream block `block` of a Stream (identical output to chacha_block).
__device__ __forceinline__ void stream_block(const Stream &st, uint32_t block, uint32_t out[16]) {
    // finish QR(0,4,8,12) of the first column round: a += b was hoisted (x0p)
    uint32_t x0 = st.x0p, x4 = st.key.k[0], x8 = st.key.k[4], x12 = block;
    x12 ^= x0; x12 = rotl16(x12);
    x8 += x12; x4 ^= x8; x4 = rotl(x4, 12);
    x0 += x4; x12 ^= x0; x12 = rotl8(x12);
    x8 += x12; x4 ^= x8; x4 = rotl(x4, 7);
    uint32_t x1 = st.c1[0], x5 = st.c1[1], x9 = st.c1[2], x13 = st.c1[3];
    uint32_t x2 = st.c2[0], x6 = st.c2[1], x10 = st.c2[2], x14 = st.c2[3];
    uint32_t x3 = st.c3[0], x7 = st.c3[1], x11 = st.c3[2], x15 = st.c3[3];
    // first diagonal round
    RG_QR(x0, x5, x10, x15);
    RG_QR(x1, x6, x11, x12);
    RG_QR(x2, x7, x8, x13);
    RG_QR(x3, x4, x9, x14);
#pragma unroll
    for (int i = 1; i < 10; i++) {
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
    out[4] = x4 + st.key.k[0];
    out[5] = x5 + st.key.k[1];
    out[6] = x6 + st.key.k[2];
    out[7] = x7 + st.key.k[3];
    out[8] = x8 + st.key.k[4];
    out[9] = x9 + st.key.k[5];
    out[10] = x10 + st.key.k[6];
    out[11] = x11 + st.key.k[7];
    out[12] = x12 + block;
    out[13] = x13 + st.n0;
    out[14] = x14 + st.n1;
    out[15] = x15 + st.n2;
}

// stream_block with a hook run after double-round i (i = 0..9), so that
// independent work (the previous chunk's Poly1305) is placed between the
// ARX rounds in program order: the compiler schedules close to source order,
// and the interleave fills the dependency gaps of both chains.
template <typename Hook>
__device__ __forceinline__ void stream_block_hooked(const Stream &st, uint32_t block, uint32_t out[16], Hook &&hook) {
    uint32_t x0 = st.x0p, x4 = st.key.k[0], x8 = st.key.k[4], x12 = block;
    x12 ^= x0; x12 = rotl16(x12);
    x8 += x12; x4 ^= x8; x4 = rotl(x4, 12);
    x0 += x4; x12 ^= x0; x12 = rotl8(x12);
    x8 += x12; x4 ^= x8; x4 = rotl(x4, 7);
    uint32_t x1 = st.c1[0], x5 = st.c1[1], x9 = st.c1[2], x13 = st.c1[3];
    uint32_t x2 = st.c2[0], x6 = st.c2[1], x10 = st.c2[2], x14 = st.c2[3];
    uint32_t x3 = st.c3[0], x7 = st.c3[1], x11 = st.c3[2], x15 = st.c3[3];
    RG_QR(x0, x5, x10, x15);
    RG_QR(x1, x6, x11, x12);
    RG_QR(x2, x7, x8, x13);
    RG_QR(x3, x4, x9, x14);
    hook(0);
#define RG_PIN_STATE()                                                                                 \
    asm volatile("" : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(x4), "+v"(x5), "+v"(x6), "+v"(x7), \
                 "+v"(x8), "+v"(x9), "+v"(x10), "+v"(x11), "+v"(x12), "+v"(x13), "+v"(x14), "+v"(x15))
    RG_PIN_STATE();
#pragma unroll
    for (int i = 1; i < 10; i++) {
        RG_QR(x0, x4, x8, x12);
        RG_QR(x1, x5, x9, x13);
        RG_QR(x2, x6, x10, x14);
        RG_QR(x3, x7, x11, x15);
        RG_QR(x0, x5, x10, x15);
        RG_QR(x1, x6, x11, x12);
        RG_QR(x2, x7, x8, x13);
        RG_QR(x3, x4, x9, x14);
        hook(i);
        if (i % 2 == 1) RG_PIN_STATE();
    }
#undef RG_PIN_STATE
    out[0] = x0 + 0x61707865u;
    out[1] = x1 + 0x3320646eu;
    out[2] = x2 + 0x79622d32u;
    out[3] = x3 + 0x6b206574u;
    out[4] = x4 + st.key.k[0];
    out[5] = x5 + st.key.k[1];
    out[6] = x6 + st.key.k[2];
    out[7] = x7 + st.key.k[3];
    out[8] = x8 + st.key.k[4];
    out[9] = x9 + st.key.k[5];
    out[10] = x10 + st.key.k[6];
    out[11] = x11 + st.key.k[7];
    out[12] = x12 + block;
    out[13] = x13 + st.n0;
    out[14] = x14 + st.n1;
    out[15] = x15 + st.n2;
}

// key-table row idx (8 LE words)
__device__ __forceinline__ Key8 load_key(const uint32_t *keys, uint32_t idx) {
    const uint4 *kp = reinterpret_cast<const uint4 *>(keys + 8ull * idx);
    uint4 a = kp[0], b = kp[1];
    Key8 k;
    k.k[0] = a.x; k.k[1] = a.y; k.k[2] = a.z; k.k[3] = a.w;
    k.k[4] = b.x; k.k[5] = b.y; k.k[6] = b.z; k.k[7] = b.w;
    return k;
}

__device__ __forceinline__ uint4 xor4(uint4 m, const uint32_t *ks) {
    return make_uint4(m.x ^ ks[0], m.y ^ ks[1], m.z ^ ks[2], m.w ^ ks[3]);
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

__device__ __forceinline__ uint32_t addc(uint32_t a, uint32_t b, uint32_t cin, uint32_t &cout) {
    return __builtin_addc(a, b, cin, &cout); // v_add_co_u32 / v_addc_co_u32
}

// h += m + hibit * 2^128
__device__ __forceinline__ void acc_add(Acc &h, uint32_t m0, uint32_t m1, uint32_t m2, uint32_t m3, uint32_t hibit) {
    uint32_t k;
    h.h0 = addc(h.h0, m0, 0, k);
    h.h1 = addc(h.h1, m1, k, k);
    h.h2 = addc(h.h2, m2, k, k);
    h.h3 = addc(h.h3, m3, k, k);
    h.h4 = h.h4 + hibit + k;
}

// h = h * r mod 2^130-5, partially reduced (h4 <= 4 on exit).
// Bounds: h_i < 2^32, h4 < 8, r_j < 2^28, rr_j < 2^28.33 -> every column sum
// < 2^62.4 fits a u64.  The four columns are independent v_mad_u64_u32
// chains; their 64-bit sums are then carried into 32-bit words with one
// add-with-carry chain (no 64-bit shifts, no register-pair moves).
__device__ __forceinline__ void acc_mul(Acc &h, const Mul &r) {
    const uint64_t d0 = mad64(h.h3, r.rr1, mad64(h.h2, r.rr2, mad64(h.h1, r.rr3, (uint64_t)h.h0 * r.r0)));
    const uint64_t d1 = mad64(h.h4, r.rr1, mad64(h.h3, r.rr2, mad64(h.h2, r.rr3, mad64(h.h1, r.r0, (uint64_t)h.h0 * r.r1))));
    const uint64_t d2 = mad64(h.h4, r.rr2, mad64(h.h3, r.rr3, mad64(h.h2, r.r0, mad64(h.h1, r.r1, (uint64_t)h.h0 * r.r2))));
    const uint64_t d3 = mad64(h.h4, r.rr3, mad64(h.h3, r.r0, mad64(h.h2, r.r1, mad64(h.h1, r.r2, (uint64_t)h.h0 * r.r3))));
    const uint32_t d4 = h.h4 * r.r0; // < 2^31
    uint32_t k;
    const uint32_t w0 = (uint32_t)d0;
    const uint32_t w1 = addc((uint32_t)d1, (uint32_t)(d0 >> 32), 0, k);
    const uint32_t w2 = addc((uint32_t)d2, (uint32_t)(d1 >> 32), k, k);
    const uint32_t w3 = addc((uint32_t)d3, (uint32_t)(d2 >> 32), k, k);
    const uint32_t w4 = d4 + (uint32_t)(d3 >> 32) + k; // < 2^31.6
    // 2^130 == 5: fold bits >= 130 back in
    const uint32_t c = (w4 >> 2) + (w4 & ~3u);
    h.h0 = addc(w0, c, 0, k);
    h.h1 = addc(w1, 0, k, k);
    h.h2 = addc(w2, 0, k, k);
    h.h3 = addc(w3, 0, k, k);
    h.h4 = (w4 & 3u) + k;
}

// h = valid ? (h + m + 2^128) * r : h, branch-free (v_cndmask) so that the
// block can sit in the same basic block as independent keystream work.
__device__ __forceinline__ void acc_block_pred(Acc &h, const uint4 &m, const Mul &r, bool valid) {
    Acc t = h;
    acc_add(t, m.x, m.y, m.z, m.w, 1);
    acc_mul(t, r);
    h.h0 = valid ? t.h0 : h.h0;
    h.h1 = valid ? t.h1 : h.h1;
    h.h2 = valid ? t.h2 : h.h2;
    h.h3 = valid ? t.h3 : h.h3;
    h.h4 = valid ? t.h4 : h.h4;
}

// h = valid ? h * r : h, branch-free
__device__ __forceinline__ void acc_mul_pred(Acc &h, const Mul &r, bool valid) {
    Acc t = h;
    acc_mul(t, r);
    h.h0 = valid ? t.h0 : h.h0;
    h.h1 = valid ? t.h1 : h.h1;
    h.h2 = valid ? t.h2 : h.h2;
    h.h3 = valid ? t.h3 : h.h3;
    h.h4 = valid ? t.h4 : h.h4;
}

// empty asm that makes h opaque here: later Poly work cannot move above this
// point and earlier work cannot sink below it (zero instructions)
__device__ __forceinline__ void pin_acc(Acc &h) {
    asm volatile("" : "+v"(h.h0), "+v"(h.h1), "+v"(h.h2), "+v"(h.h3), "+v"(h.h4));
}

__device__ __forceinline__ void acc_block(Acc &h, const uint4 &m, const Mul &r) {
    acc_add(h, m.x, m.y, m.z, m.w, 1);
    acc_mul(h, r);
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

// ------------------------------------------------- general multiplier
// Powers r^k are not clamped, so the rr = 5r/4 fold above does not apply.
// A general multiplier G is kept in radix 2^26 (five limbs, with 5*g_j
// precomputed, the textbook 2^130 == 5 fold); the accumulator is converted
// 2^32 -> 2^26 -> multiply -> 2^32 around the product.
struct Gen {
    uint32_t g0, g1, g2, g3, g4, s1, s2, s3, s4;
};

__device__ __forceinline__ void to26(const Acc &h, uint32_t l[5]) {
    const uint32_t M = 0x3ffffffu;
    l[0] = h.h0 & M;
    l[1] = ((h.h0 >> 26) | (h.h1 << 6)) & M;
    l[2] = ((h.h1 >> 20) | (h.h2 << 12)) & M;
    l[3] = ((h.h2 >> 14) | (h.h3 << 18)) & M;
    l[4] = (h.h3 >> 8) | (h.h4 << 24); // h4 < 8 -> l4 < 2^27
}

__device__ __forceinline__ Gen make_gen(const Acc &g) {
    uint32_t l[5];
    to26(g, l);
    Gen G;
    G.g0 = l[0]; G.g1 = l[1]; G.g2 = l[2]; G.g3 = l[3]; G.g4 = l[4];
    G.s1 = l[1] * 5; G.s2 = l[2] * 5; G.s3 = l[3] * 5; G.s4 = l[4] * 5;
    return G;
}

// h = h * G mod 2^130-5, partially reduced (h4 <= 4 on exit).
// Bounds: a_i < 2^27, g_j < 2^27, s_j < 2^29.4 -> columns < 2^59.
__device__ __forceinline__ void acc_mul_gen(Acc &h, const Gen &G) {
    uint32_t a[5];
    to26(h, a);
    uint64_t d0 = mad64(a[0], G.g0, mad64(a[1], G.s4, mad64(a[2], G.s3, mad64(a[3], G.s2, (uint64_t)a[4] * G.s1))));
    uint64_t d1 = mad64(a[0], G.g1, mad64(a[1], G.g0, mad64(a[2], G.s4, mad64(a[3], G.s3, (uint64_t)a[4] * G.s2))));
    uint64_t d2 = mad64(a[0], G.g2, mad64(a[1], G.g1, mad64(a[2], G.g0, mad64(a[3], G.s4, (uint64_t)a[4] * G.s3))));
    uint64_t d3 = mad64(a[0], G.g3, mad64(a[1], G.g2, mad64(a[2], G.g1, mad64(a[3], G.g0, (uint64_t)a[4] * G.s4))));
    uint64_t d4 = mad64(a[0], G.g4, mad64(a[1], G.g3, mad64(a[2], G.g2, mad64(a[3], G.g1, (uint64_t)a[4] * G.g0))));
    const uint64_t M = 0x3ffffffu;
    d1 += d0 >> 26;
    d2 += d1 >> 26;
    d3 += d2 >> 26;
    d4 += d3 >> 26;
    // fold bits >= 130: (d4 >> 26) * 5 into limb 0
    uint64_t t0 = (d0 & M) + (d4 >> 26) * 5;
    uint32_t l0 = (uint32_t)(t0 & M);
    uint64_t l1 = (d1 & M) + (t0 >> 26);
    // back to radix 2^32 (limbs may exceed 26 bits slightly; 64-bit packing absorbs it)
    uint64_t t = (uint64_t)l0 + (l1 << 26);
    h.h0 = (uint32_t)t;
    t = (t >> 32) + ((d2 & M) << 20);
    h.h1 = (uint32_t)t;
    t = (t >> 32) + ((d3 & M) << 14);
    h.h2 = (uint32_t)t;
    t = (t >> 32) + ((d4 & M) << 8);
    h.h3 = (uint32_t)t;
    h.h4 = (uint32_t)(t >> 32); // < 4
}

// h = h^2 mod 2^130-5 in radix 2^26 with the cross terms doubled: 15 products instead of the 25 of
// acc_mul_gen(h, make_gen(h)).  Bounds: a_i < 2^27, 2 a_i < 2^28, 5 a_i < 2^29.4 -> columns < 2^61.
__device__ __forceinline__ void acc_sqr_gen(Acc &h) {
    uint32_t a[5];
    to26(h, a);
    const uint32_t t0 = 2 * a[0], t1 = 2 * a[1], t2 = 2 * a[2], t3 = 2 * a[3];
    const uint32_t u3 = 5 * a[3], u4 = 5 * a[4];
    uint64_t d0 = mad64(a[0], a[0], mad64(t1, u4, (uint64_t)t2 * u3));
    uint64_t d1 = mad64(t0, a[1], mad64(t2, u4, (uint64_t)a[3] * u3));
    uint64_t d2 = mad64(t0, a[2], mad64(a[1], a[1], (uint64_t)t3 * u4));
    uint64_t d3 = mad64(t0, a[3], mad64(t1, a[2], (uint64_t)a[4] * u4));
    uint64_t d4 = mad64(t0, a[4], mad64(t1, a[3], (uint64_t)a[2] * a[2]));
    const uint64_t M = 0x3ffffffu;
    d1 += d0 >> 26;
    d2 += d1 >> 26;
    d3 += d2 >> 26;
    d4 += d3 >> 26;
    uint64_t r0 = (d0 & M) + (d4 >> 26) * 5;
    uint32_t l0 = (uint32_t)(r0 & M);
    uint64_t l1 = (d1 & M) + (r0 >> 26);
    uint64_t t = (uint64_t)l0 + (l1 << 26);
    h.h0 = (uint32_t)t;
    t = (t >> 32) + ((d2 & M) << 20);
    h.h1 = (uint32_t)t;
    t = (t >> 32) + ((d3 & M) << 14);
    h.h2 = (uint32_t)t;
    t = (t >> 32) + ((d4 & M) << 8);
    h.h3 = (uint32_t)t;
    h.h4 = (uint32_t)(t >> 32);
}

// h += o (both partially reduced), then fold h4 back below 5
__device__ __forceinline__ void acc_add_acc(Acc &h, const Acc &o) {
    uint32_t k;
    h.h0 = addc(h.h0, o.h0, 0, k);
    h.h1 = addc(h.h1, o.h1, k, k);
    h.h2 = addc(h.h2, o.h2, k, k);
    h.h3 = addc(h.h3, o.h3, k, k);
    h.h4 = h.h4 + o.h4 + k;
}

// partial reduction: bits >= 130 folded back (2^130 == 5), h4 <= 4 on exit
__device__ __forceinline__ void acc_fold(Acc &h) {
    const uint32_t c = (h.h4 >> 2) + (h.h4 & ~3u);
    uint32_t k;
    h.h0 = addc(h.h0, c, 0, k);
    h.h1 = addc(h.h1, 0, k, k);
    h.h2 = addc(h.h2, 0, k, k);
    h.h3 = addc(h.h3, 0, k, k);
    h.h4 = (h.h4 & 3u) + k;
}

// --------------------------------------------------- buffer / LDS-DMA access
// Raw buffer resources and LDS-DMA in inline asm: the compiler does not see these vector-memory
// operations, so it inserts no vmcnt waits for them; the kernels count them and wait with exact
// s_waitcnt vmcnt(N) (loads, stores and LDS-DMA retire in issue order on one counter).
typedef int v4i __attribute__((ext_vector_type(4)));
typedef uint32_t v4u __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) v4u g_v4u; // global memory, explicitly (not flat)

__device__ __forceinline__ v4i make_rsrc(const uint8_t *base, uint32_t num_records) {
    const uint64_t a = (uint64_t)base;
    v4i r;
    r.x = (int)uniform_u32((uint32_t)a);
    r.y = (int)uniform_u32((uint32_t)(a >> 32)); // stride 0
    r.z = (int)uniform_u32(num_records);
    r.w = 0x00020000; // raw buffer, 32-bit data format (gfx9 family)
    return r;
}

// one LDS-DMA wave-instruction: 16 bytes per lane to lds_byte + 16 * lane
__device__ __forceinline__ void dma16(const v4i &rsrc, uint32_t voff, uint32_t lds_byte) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\t"
                 "s_mov_b32 m0, %3\n\t"
                 "s_nop 0\n\t"
                 "buffer_load_dwordx4 %1, %2, 0 offen lds\n\t"
                 "s_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(voff), "s"(rsrc), "s"(lds_byte)
                 : "memory");
}

// Frame stores stay plain (write-back): a plain store leaves its line dirty in the XCD's L2 and the
// end-of-kernel release writes the dirty lines back after the last wave (tools/tailbench.hip,
// profiles/r3_tailbench.json: +2.2 us of tail at ~100 MB of coalesced stores per launch, none with sc1),
// but in the AEAD kernels write-through (sc1) stores measured no faster on configs 2, 4 and 5 and 4 %
// slower on config 3, whose 16-byte stores at a 16-byte phase then reach memory piece by piece
// (round 3, profiles/r3_sc1_ab.txt).
__device__ __forceinline__ void store16(const v4i &rsrc, uint32_t voff, const uint4 &v) {
    v4u d;
    d.x = v.x;
    d.y = v.y;
    d.z = v.z;
    d.w = v.w;
    asm volatile("buffer_store_dwordx4 %0, %1, %2, 0 offen\n\t"
                 "s_nop 1"
                 :
                 : "v"(d), "v"(voff), "s"(rsrc)
                 : "memory");
}

template <int N> __device__ __forceinline__ void wait_vm() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// ---------------------------------------------------- forged-frame restore
// Open decrypts in place before the tag is known; a frame whose tag fails is turned back into the
// ciphertext that came in (rustyguard-crypto/src/prim.rs:190-201: DecryptionError leaves the
// buffer unchanged).  The chunks of every forged lane of the wave -- chunks [c0, c0 + ceil(nb / 4))
// of its payload, pl pointing at chunk c0 -- are dealt over the wave's active lanes, 64 at a time,
// and each is re-XORed with its keystream block.  A wave holding k forged packets of C chunks thus
// pays ~k C / 64 keystream blocks instead of the one lane's C blocks for every forged lane in turn
// (the whole wave waiting): the cost is per forged packet, not per wave.  Every byte involved was
// stored by this wave: its vector-memory instructions are performed in order, so a wavefront-scope
// fence (wave_sync: no waitcnt, no cache maintenance) orders the restore's loads after the stores.
// (An agent-scope __threadfence costs a buffer_wbl2 -- the write-back of every dirty line of the
// XCD's L2 -- and a workgroup-scope one a vmcnt(0) store drain: +50 % and +37 % on config 2's open
// with 1 % of the frames forged, profiles/r3_forged_open.txt.)  Called by every active lane.
__device__ __forceinline__ void restore_forged(bool forged, const Key8 &key, uint32_t n1, uint32_t n2, uint4 *pl,
                                               uint32_t c0, uint32_t nb) {
    const uint64_t active = __ballot(true);
    uint64_t fm = __ballot(forged && nb > 0);
    if (fm == 0) return;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t nact = (uint32_t)__popcll(active);
    const uint32_t arank = (uint32_t)__popcll(active & ((1ull << lane) - 1ull)); // rank among active lanes
    const uint32_t myC = (nb + 3) >> 2;
    const uint64_t plv = reinterpret_cast<uint64_t>(pl);
    int own = -1;      // forged lane whose chunk this lane re-XORs in the current round
    uint32_t oc = 0;   // that chunk's index inside the owner's range
    uint32_t pos = 0;  // next free active-lane rank (wave-uniform)
    auto round = [&]() {
        const int src = own >= 0 ? own : (int)lane; // every active lane takes part in the shuffles
        Key8 k;
#pragma unroll
        for (int w = 0; w < 8; ++w) k.k[w] = (uint32_t)__shfl((int)key.k[w], src);
        const uint32_t m1 = (uint32_t)__shfl((int)n1, src), m2 = (uint32_t)__shfl((int)n2, src);
        const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)plv, src), hi = (uint32_t)__shfl((int)(uint32_t)(plv >> 32), src);
        const uint32_t oc0 = (uint32_t)__shfl((int)c0, src), onb = (uint32_t)__shfl((int)nb, src);
        if (own >= 0) {
            // the shuffled address as a global pointer: a generic one compiles to flat_* accesses, which
            // wait on the LDS counter too
            g_v4u *p = reinterpret_cast<g_v4u *>(((uint64_t)hi << 32) | lo) + 4 * oc;
            const uint32_t b0 = 4 * oc, last = onb - 1;
            const v4u q0 = p[min(b0, last) - b0], q1 = p[min(b0 + 1, last) - b0];
            const v4u q2 = p[min(b0 + 2, last) - b0], q3 = p[min(b0 + 3, last) - b0];
            const Stream stm = make_stream(k, 0u, m1, m2);
            uint32_t ks[16];
            stream_block(stm, oc0 + oc + 1, ks);
            if (b0 < onb) p[0] = q0 ^ v4u{ks[0], ks[1], ks[2], ks[3]};
            if (b0 + 1 < onb) p[1] = q1 ^ v4u{ks[4], ks[5], ks[6], ks[7]};
            if (b0 + 2 < onb) p[2] = q2 ^ v4u{ks[8], ks[9], ks[10], ks[11]};
            if (b0 + 3 < onb) p[3] = q3 ^ v4u{ks[12], ks[13], ks[14], ks[15]};
        }
        own = -1;
    };
    while (fm) {
        const uint32_t f = (uint32_t)__ffsll((unsigned long long)fm) - 1;
        fm &= fm - 1;
        const uint32_t Cf = (uint32_t)__builtin_amdgcn_readlane((int)myC, (int)f);
        for (uint32_t done = 0; done < Cf;) {
            const uint32_t take = min(Cf - done, nact - pos);
            if (arank >= pos && arank < pos + take) {
                own = (int)f;
                oc = done + arank - pos;
            }
            pos += take;
            done += take;
            if (pos == nact) {
                round();
                pos = 0;
            }
        }
    }
    if (pos > 0) round();
}

__device__ __forceinline__ uint64_t mix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

} // namespace rg
