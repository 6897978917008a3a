/*
 * rg_oracle.c -- CPU restatement of the WireGuard transport-data AEAD path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load this library, and only as the checker
 * (or the timed CPU baseline).  The product path (rustyguard_amd, librg_aead)
 * never links or calls it.
 *
 * What it restates
 * ----------------
 * The reference seals/opens transport packets through
 *   rustyguard-crypto/src/prim.rs:179-201   Core::chacha20poly1305_{enc,dec}
 * which forwards to the third-party crate graviola 0.2.0
 *   (Cargo.lock:370-373, rustyguard-crypto/Cargo.toml:21; NOT vendored in
 *   /root/reference, no Rust toolchain here -> reference unbuildable).
 * graviola implements RFC 8439; this file restates RFC 8439 directly:
 *   - ChaCha20 block function            RFC 8439 §2.3
 *   - Poly1305 (radix 2^26 limbs)        RFC 8439 §2.5
 *   - one-time key generation            RFC 8439 §2.6
 *   - AEAD construction                  RFC 8439 §2.8
 * plus the WireGuard-specific glue of the reference:
 *   - nonce = 00000000 || le64(counter)  rustyguard-crypto/src/prim.rs:32-36
 *   - empty AAD for transport data       prim.rs:391, prim.rs:431
 *   - header {4, receiver, counter}      rustyguard-core/src/lib.rs:286-290,
 *                                        rustyguard-types/src/lib.rs:167-179
 *   - framing hdr | ct | tag             rustyguard-core/src/lib.rs:463-469
 *   - open: len/alignment/type checks    rustyguard-core/src/lib.rs:613-629,
 *                                        rustyguard-types/src/lib.rs:181-196,
 *                                        rustyguard-crypto/src/prim.rs:427-429
 *
 * Parity pinning: the restatement is checked (tests/test_oracle_golden.py)
 * against the reference's own insta snapshots (rustyguard-crypto
 * handshake-{4,5,6,7}.snap, rustyguard-core snapshot-3.snap), the RFC 8439
 * §2.8.2 vector and OpenSSL-generated multi-block vectors (tests/golden/).
 *
 * The Poly1305 arithmetic deliberately uses a different radix (2^26) from the
 * GPU kernels (2^32) so an arithmetic slip cannot hide in both.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "rg_oracle.h"

/* ------------------------------------------------------------------------ */
/* little-endian helpers                                                     */

static uint32_t ld32(const uint8_t *p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
static void st32(uint8_t *p, uint32_t v) {
    p[0] = (uint8_t)v;
    p[1] = (uint8_t)(v >> 8);
    p[2] = (uint8_t)(v >> 16);
    p[3] = (uint8_t)(v >> 24);
}
static void st64(uint8_t *p, uint64_t v) {
    st32(p, (uint32_t)v);
    st32(p + 4, (uint32_t)(v >> 32));
}
static uint64_t ld64(const uint8_t *p) { return (uint64_t)ld32(p) | ((uint64_t)ld32(p + 4) << 32); }

static uint32_t rotl(uint32_t v, int n) { return (v << n) | (v >> (32 - n)); }

/* ------------------------------------------------------------------------ */
/* ChaCha20 (RFC 8439 §2.3)                                                  */

#define QROUND(x, a, b, c, d)                                     \
    do {                                                          \
        x[a] += x[b]; x[d] ^= x[a]; x[d] = rotl(x[d], 16);        \
        x[c] += x[d]; x[b] ^= x[c]; x[b] = rotl(x[b], 12);        \
        x[a] += x[b]; x[d] ^= x[a]; x[d] = rotl(x[d], 8);         \
        x[c] += x[d]; x[b] ^= x[c]; x[b] = rotl(x[b], 7);         \
    } while (0)

void rg_oracle_chacha20_block(const uint8_t key[32], uint32_t counter, const uint8_t nonce[12],
                              uint8_t out[64]) {
    uint32_t s[16], x[16];
    s[0] = 0x61707865u; /* "expand 32-byte k" */
    s[1] = 0x3320646eu;
    s[2] = 0x79622d32u;
    s[3] = 0x6b206574u;
    for (int i = 0; i < 8; i++) s[4 + i] = ld32(key + 4 * i);
    s[12] = counter;
    for (int i = 0; i < 3; i++) s[13 + i] = ld32(nonce + 4 * i);
    memcpy(x, s, sizeof x);
    for (int round = 0; round < 10; round++) {
        QROUND(x, 0, 4, 8, 12);
        QROUND(x, 1, 5, 9, 13);
        QROUND(x, 2, 6, 10, 14);
        QROUND(x, 3, 7, 11, 15);
        QROUND(x, 0, 5, 10, 15);
        QROUND(x, 1, 6, 11, 12);
        QROUND(x, 2, 7, 8, 13);
        QROUND(x, 3, 4, 9, 14);
    }
    for (int i = 0; i < 16; i++) st32(out + 4 * i, x[i] + s[i]);
}

/* XOR len bytes of data with the keystream starting at block `counter` (§2.4). */
static void chacha20_xor(const uint8_t key[32], uint32_t counter, const uint8_t nonce[12], uint8_t *data,
                         size_t len) {
    uint8_t ks[64];
    while (len > 0) {
        rg_oracle_chacha20_block(key, counter++, nonce, ks);
        size_t take = len < 64 ? len : 64;
        for (size_t i = 0; i < take; i++) data[i] ^= ks[i];
        data += take;
        len -= take;
    }
}

/* ------------------------------------------------------------------------ */
/* Poly1305 (RFC 8439 §2.5), five 26-bit limbs, 64-bit products.            */

typedef struct {
    uint32_t r[5];
    uint32_t h[5];
    uint32_t pad[4];
    uint8_t buf[16];
    size_t fill;
} poly_state;

static void poly_init(poly_state *st, const uint8_t otk[32]) {
    /* r = le128(otk[0..16]) & 0x0ffffffc0ffffffc0ffffffc0fffffff, split into
     * 26-bit limbs. */
    uint32_t t0 = ld32(otk + 0) & 0x0fffffffu;
    uint32_t t1 = ld32(otk + 4) & 0x0ffffffcu;
    uint32_t t2 = ld32(otk + 8) & 0x0ffffffcu;
    uint32_t t3 = ld32(otk + 12) & 0x0ffffffcu;
    st->r[0] = t0 & 0x3ffffff;
    st->r[1] = ((t0 >> 26) | (t1 << 6)) & 0x3ffffff;
    st->r[2] = ((t1 >> 20) | (t2 << 12)) & 0x3ffffff;
    st->r[3] = ((t2 >> 14) | (t3 << 18)) & 0x3ffffff;
    st->r[4] = (t3 >> 8);
    for (int i = 0; i < 5; i++) st->h[i] = 0;
    for (int i = 0; i < 4; i++) st->pad[i] = ld32(otk + 16 + 4 * i);
    st->fill = 0;
}

/* h = (h + m + hibit*2^128) * r mod 2^130-5, partially reduced. */
static void poly_block(poly_state *st, const uint8_t m[16], uint32_t hibit) {
    uint32_t m0 = ld32(m), m1 = ld32(m + 4), m2 = ld32(m + 8), m3 = ld32(m + 12);
    uint64_t h0 = st->h[0] + (m0 & 0x3ffffff);
    uint64_t h1 = st->h[1] + (((m0 >> 26) | (m1 << 6)) & 0x3ffffff);
    uint64_t h2 = st->h[2] + (((m1 >> 20) | (m2 << 12)) & 0x3ffffff);
    uint64_t h3 = st->h[3] + (((m2 >> 14) | (m3 << 18)) & 0x3ffffff);
    uint64_t h4 = st->h[4] + ((m3 >> 8) | (hibit << 24));
    const uint64_t r0 = st->r[0], r1 = st->r[1], r2 = st->r[2], r3 = st->r[3], r4 = st->r[4];
    /* 2^130 == 5 (mod p): limb products that overflow position 4 wrap with *5 */
    const uint64_t f1 = r1 * 5, f2 = r2 * 5, f3 = r3 * 5, f4 = r4 * 5;
    uint64_t d0 = h0 * r0 + h1 * f4 + h2 * f3 + h3 * f2 + h4 * f1;
    uint64_t d1 = h0 * r1 + h1 * r0 + h2 * f4 + h3 * f3 + h4 * f2;
    uint64_t d2 = h0 * r2 + h1 * r1 + h2 * r0 + h3 * f4 + h4 * f3;
    uint64_t d3 = h0 * r3 + h1 * r2 + h2 * r1 + h3 * r0 + h4 * f4;
    uint64_t d4 = h0 * r4 + h1 * r3 + h2 * r2 + h3 * r1 + h4 * r0;
    d1 += d0 >> 26; d0 &= 0x3ffffff;
    d2 += d1 >> 26; d1 &= 0x3ffffff;
    d3 += d2 >> 26; d2 &= 0x3ffffff;
    d4 += d3 >> 26; d3 &= 0x3ffffff;
    d0 += (d4 >> 26) * 5; d4 &= 0x3ffffff;
    d1 += d0 >> 26; d0 &= 0x3ffffff;
    st->h[0] = (uint32_t)d0;
    st->h[1] = (uint32_t)d1;
    st->h[2] = (uint32_t)d2;
    st->h[3] = (uint32_t)d3;
    st->h[4] = (uint32_t)d4;
}

static void poly_update(poly_state *st, const uint8_t *m, size_t len) {
    while (len > 0) {
        size_t take = 16 - st->fill;
        if (take > len) take = len;
        memcpy(st->buf + st->fill, m, take);
        st->fill += take;
        m += take;
        len -= take;
        if (st->fill == 16) {
            poly_block(st, st->buf, 1);
            st->fill = 0;
        }
    }
}

/* AEAD pads every section with zeros to a 16-byte boundary (§2.8). */
static void poly_pad16(poly_state *st) {
    if (st->fill) {
        memset(st->buf + st->fill, 0, 16 - st->fill);
        poly_block(st, st->buf, 1);
        st->fill = 0;
    }
}

static void poly_finish(poly_state *st, uint8_t tag[16]) {
    /* a trailing partial block (plain Poly1305 use) gets a 0x01 byte and no hibit */
    if (st->fill) {
        st->buf[st->fill] = 1;
        memset(st->buf + st->fill + 1, 0, 15 - st->fill);
        poly_block(st, st->buf, 0);
        st->fill = 0;
    }
    uint32_t h0 = st->h[0], h1 = st->h[1], h2 = st->h[2], h3 = st->h[3], h4 = st->h[4];
    /* full carry */
    uint32_t c;
    c = h1 >> 26; h1 &= 0x3ffffff; h2 += c;
    c = h2 >> 26; h2 &= 0x3ffffff; h3 += c;
    c = h3 >> 26; h3 &= 0x3ffffff; h4 += c;
    c = h4 >> 26; h4 &= 0x3ffffff; h0 += c * 5;
    c = h0 >> 26; h0 &= 0x3ffffff; h1 += c;
    /* g = h + 5 - 2^130; pick g when h >= p (constant time select) */
    uint32_t g0 = h0 + 5; c = g0 >> 26; g0 &= 0x3ffffff;
    uint32_t g1 = h1 + c; c = g1 >> 26; g1 &= 0x3ffffff;
    uint32_t g2 = h2 + c; c = g2 >> 26; g2 &= 0x3ffffff;
    uint32_t g3 = h3 + c; c = g3 >> 26; g3 &= 0x3ffffff;
    uint32_t g4 = h4 + c - (1u << 26);
    /* g4 wrapped negative -> h < p -> keep h; otherwise use g (all-ones mask) */
    uint32_t use_g = (g4 >> 31) - 1u;
    uint32_t keep = ~use_g;
    h0 = (h0 & keep) | (g0 & use_g);
    h1 = (h1 & keep) | (g1 & use_g);
    h2 = (h2 & keep) | (g2 & use_g);
    h3 = (h3 & keep) | (g3 & use_g);
    h4 = (h4 & keep) | (g4 & use_g);
    /* back to 4 x 32 bits, add s = pad, mod 2^128 */
    uint32_t w0 = h0 | (h1 << 26);
    uint32_t w1 = (h1 >> 6) | (h2 << 20);
    uint32_t w2 = (h2 >> 12) | (h3 << 14);
    uint32_t w3 = (h3 >> 18) | (h4 << 8);
    uint64_t f;
    f = (uint64_t)w0 + st->pad[0];             st32(tag + 0, (uint32_t)f);
    f = (uint64_t)w1 + st->pad[1] + (f >> 32); st32(tag + 4, (uint32_t)f);
    f = (uint64_t)w2 + st->pad[2] + (f >> 32); st32(tag + 8, (uint32_t)f);
    f = (uint64_t)w3 + st->pad[3] + (f >> 32); st32(tag + 12, (uint32_t)f);
}

void rg_oracle_poly1305(const uint8_t key[32], const uint8_t *msg, size_t len, uint8_t tag[16]) {
    poly_state st;
    poly_init(&st, key);
    poly_update(&st, msg, len);
    poly_finish(&st, tag);
}

/* ------------------------------------------------------------------------ */
/* AEAD (RFC 8439 §2.8)                                                      */

static void aead_tag(const uint8_t key[32], const uint8_t nonce[12], const uint8_t *aad, size_t aad_len,
                     const uint8_t *ct, size_t len, uint8_t tag[16]) {
    uint8_t block0[64];
    rg_oracle_chacha20_block(key, 0, nonce, block0); /* §2.6: otk = first 32 B of block 0 */
    poly_state st;
    poly_init(&st, block0);
    poly_update(&st, aad, aad_len);
    poly_pad16(&st);
    poly_update(&st, ct, len);
    poly_pad16(&st);
    uint8_t lens[16];
    st64(lens, (uint64_t)aad_len);
    st64(lens + 8, (uint64_t)len);
    poly_update(&st, lens, 16);
    poly_finish(&st, tag);
}

void rg_oracle_aead_seal(const uint8_t key[32], const uint8_t nonce[12], const uint8_t *aad, size_t aad_len,
                         uint8_t *payload, size_t len, uint8_t tag[16]) {
    chacha20_xor(key, 1, nonce, payload, len);
    aead_tag(key, nonce, aad, aad_len, payload, len, tag);
}

int rg_oracle_aead_open(const uint8_t key[32], const uint8_t nonce[12], const uint8_t *aad, size_t aad_len,
                        uint8_t *payload, size_t len, const uint8_t tag[16]) {
    uint8_t want[16];
    aead_tag(key, nonce, aad, aad_len, payload, len, want);
    uint8_t diff = 0;
    for (int i = 0; i < 16; i++) diff |= (uint8_t)(want[i] ^ tag[i]);
    if (diff != 0) return -1; /* CryptoError::DecryptionError, payload untouched */
    chacha20_xor(key, 1, nonce, payload, len);
    return 0;
}

/* XChaCha20-Poly1305 (draft-irtf-cfrg-xchacha-03 §2.2-2.3), the cookie AEAD of
 * Core::xchacha20poly1305_{enc,dec} (rustyguard-crypto/src/prim.rs:202-224):
 * subkey = HChaCha20(key, nonce[0..16]) -- the 20 rounds with no feed-forward,
 * words 0-3 and 12-15 -- then ChaCha20-Poly1305 with nonce 0^4 || nonce[16..24]. */
void rg_oracle_hchacha20(const uint8_t key[32], const uint8_t nonce16[16], uint8_t out[32]) {
    uint32_t x[16];
    x[0] = 0x61707865u;
    x[1] = 0x3320646eu;
    x[2] = 0x79622d32u;
    x[3] = 0x6b206574u;
    for (int i = 0; i < 8; i++) x[4 + i] = ld32(key + 4 * i);
    for (int i = 0; i < 4; i++) x[12 + i] = ld32(nonce16 + 4 * i);
    for (int round = 0; round < 10; round++) {
        QROUND(x, 0, 4, 8, 12);
        QROUND(x, 1, 5, 9, 13);
        QROUND(x, 2, 6, 10, 14);
        QROUND(x, 3, 7, 11, 15);
        QROUND(x, 0, 5, 10, 15);
        QROUND(x, 1, 6, 11, 12);
        QROUND(x, 2, 7, 8, 13);
        QROUND(x, 3, 4, 9, 14);
    }
    for (int i = 0; i < 4; i++) st32(out + 4 * i, x[i]);
    for (int i = 0; i < 4; i++) st32(out + 16 + 4 * i, x[12 + i]);
}

static void xchacha_subkey(const uint8_t key[32], const uint8_t nonce24[24], uint8_t sub[32], uint8_t n12[12]) {
    rg_oracle_hchacha20(key, nonce24, sub);
    memset(n12, 0, 4);
    memcpy(n12 + 4, nonce24 + 16, 8);
}

void rg_oracle_xaead_seal(const uint8_t key[32], const uint8_t nonce24[24], const uint8_t *aad, size_t aad_len,
                          uint8_t *payload, size_t len, uint8_t tag[16]) {
    uint8_t sub[32], n12[12];
    xchacha_subkey(key, nonce24, sub, n12);
    rg_oracle_aead_seal(sub, n12, aad, aad_len, payload, len, tag);
}

int rg_oracle_xaead_open(const uint8_t key[32], const uint8_t nonce24[24], const uint8_t *aad, size_t aad_len,
                         uint8_t *payload, size_t len, const uint8_t tag[16]) {
    uint8_t sub[32], n12[12];
    xchacha_subkey(key, nonce24, sub, n12);
    return rg_oracle_aead_open(sub, n12, aad, aad_len, payload, len, tag);
}

/* ------------------------------------------------------------------------ */
/* BLAKE2s (RFC 7693), keyed, any digest length 1..32: Core::blake2s_hash /    */
/* Core::blake2s_mac (rustyguard-crypto/src/prim.rs:118-131, blake2s_simd).   */

static const uint32_t B2S_IV[8] = {0x6A09E667u, 0xBB67AE85u, 0x3C6EF372u, 0xA54FF53Au,
                                   0x510E527Fu, 0x9B05688Cu, 0x1F83D9ABu, 0x5BE0CD19u};
static const uint8_t B2S_SIGMA[10][16] = {
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15}, {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3},
    {11, 8, 12, 0, 5, 2, 15, 13, 10, 14, 3, 6, 7, 1, 9, 4}, {7, 9, 3, 1, 13, 12, 11, 14, 2, 6, 5, 10, 4, 0, 15, 8},
    {9, 0, 5, 7, 2, 4, 10, 15, 14, 1, 11, 12, 6, 8, 3, 13}, {2, 12, 6, 10, 0, 11, 8, 3, 4, 13, 7, 5, 15, 14, 1, 9},
    {12, 5, 1, 15, 14, 13, 4, 10, 0, 7, 6, 3, 9, 2, 8, 11}, {13, 11, 7, 14, 12, 1, 3, 9, 5, 0, 15, 4, 8, 6, 2, 10},
    {6, 15, 14, 9, 11, 3, 0, 8, 12, 2, 13, 7, 1, 4, 10, 5}, {10, 2, 8, 4, 7, 6, 1, 5, 15, 11, 9, 14, 3, 12, 13, 0}};

static uint32_t rotr(uint32_t v, int n) { return (v >> n) | (v << (32 - n)); }

static void b2s_compress(uint32_t h[8], const uint8_t block[64], uint64_t t, int last) {
    uint32_t m[16], v[16];
    for (int i = 0; i < 16; i++) m[i] = ld32(block + 4 * i);
    for (int i = 0; i < 8; i++) { v[i] = h[i]; v[8 + i] = B2S_IV[i]; }
    v[12] ^= (uint32_t)t;
    v[13] ^= (uint32_t)(t >> 32);
    if (last) v[14] = ~v[14];
#define B2S_G(a, b, c, d, x, y)                                              \
    do {                                                                     \
        v[a] = v[a] + v[b] + x; v[d] = rotr(v[d] ^ v[a], 16);                \
        v[c] = v[c] + v[d]; v[b] = rotr(v[b] ^ v[c], 12);                    \
        v[a] = v[a] + v[b] + y; v[d] = rotr(v[d] ^ v[a], 8);                 \
        v[c] = v[c] + v[d]; v[b] = rotr(v[b] ^ v[c], 7);                     \
    } while (0)
    for (int r = 0; r < 10; r++) {
        const uint8_t *s = B2S_SIGMA[r];
        B2S_G(0, 4, 8, 12, m[s[0]], m[s[1]]);
        B2S_G(1, 5, 9, 13, m[s[2]], m[s[3]]);
        B2S_G(2, 6, 10, 14, m[s[4]], m[s[5]]);
        B2S_G(3, 7, 11, 15, m[s[6]], m[s[7]]);
        B2S_G(0, 5, 10, 15, m[s[8]], m[s[9]]);
        B2S_G(1, 6, 11, 12, m[s[10]], m[s[11]]);
        B2S_G(2, 7, 8, 13, m[s[12]], m[s[13]]);
        B2S_G(3, 4, 9, 14, m[s[14]], m[s[15]]);
    }
#undef B2S_G
    for (int i = 0; i < 8; i++) h[i] ^= v[i] ^ v[8 + i];
}

/* RFC 7693 §3.3: parameter block word 0 = 0x01010000 ^ (kk << 8) ^ nn; a key
 * is processed as a first, zero-padded block; the final block is flagged and
 * zero-padded (an empty unkeyed message still compresses one empty block). */
void rg_oracle_blake2s(uint8_t *out, size_t outlen, const uint8_t *key, size_t keylen, const uint8_t *msg,
                       size_t len) {
    uint32_t h[8];
    for (int i = 0; i < 8; i++) h[i] = B2S_IV[i];
    h[0] ^= 0x01010000u ^ ((uint32_t)keylen << 8) ^ (uint32_t)outlen;
    uint8_t block[64];
    uint64_t t = 0;
    if (keylen) {
        memset(block, 0, 64);
        memcpy(block, key, keylen);
        t = 64;
        b2s_compress(h, block, t, len == 0);
    }
    size_t off = 0;
    while (len - off > 64) {
        t += 64;
        b2s_compress(h, msg + off, t, 0);
        off += 64;
    }
    if (len > off || !keylen) {
        memset(block, 0, 64);
        memcpy(block, msg + off, len - off);
        t += len - off;
        b2s_compress(h, block, t, 1);
    }
    uint8_t full[32];
    for (int i = 0; i < 8; i++) st32(full + 4 * i, h[i]);
    memcpy(out, full, outlen);
}

/* HasMac::verify_mac1 / verify_mac2 (rustyguard-crypto/src/lib.rs:114-209):
 * mac1 = BLAKE2s-128(mac1_key, msg[..len-32]) must equal msg[len-32..len-16];
 * mac2 = BLAKE2s-128(cookie, msg[..len-16]) must equal msg[len-16..]; a
 * mismatch is CryptoError::Rejected.  key_idx RG_KEY_SCAN (0xFFFFFFFE) tries
 * every key in order and keeps the first match, as wg-proxy's peer scan
 * (wg-proxy/src/main.rs:217-229). */
void rg_oracle_mac_verify_batch(const uint8_t *keys, size_t key_len, size_t nkeys, int which,
                                const rg_oracle_desc *desc, size_t n, const uint8_t *buf, size_t buf_len,
                                uint8_t *status, uint32_t *key_out) {
    for (size_t i = 0; i < n; i++) {
        const rg_oracle_desc *d = &desc[i];
        key_out[i] = 0xFFFFFFFFu;
        if ((d->offset & 15) != 0) { status[i] = RG_ORACLE_UNALIGNED; continue; }
        if (d->len < 32 || d->offset > buf_len || d->len > buf_len - d->offset) {
            status[i] = RG_ORACLE_INVALID; /* framing: the message must lie in the buffer */
            continue;
        }
        const size_t covered = d->len - (which == 2 ? 16 : 32);
        const uint8_t *msg = buf + d->offset;
        size_t lo = d->key_idx, hi = d->key_idx + 1;
        if (d->key_idx == 0xFFFFFFFEu) { lo = 0; hi = nkeys; }
        status[i] = RG_ORACLE_REJECTED;
        for (size_t k = lo; k < hi && k < nkeys; k++) {
            uint8_t mac[16];
            rg_oracle_blake2s(mac, 16, keys + key_len * k, key_len, msg, covered);
            if (memcmp(mac, msg + covered, 16) == 0) {
                status[i] = RG_ORACLE_OK;
                key_out[i] = (uint32_t)k;
                break;
            }
        }
    }
}

/* prim.rs:32-36 */
void rg_oracle_wg_nonce(uint64_t counter, uint8_t nonce[12]) {
    memset(nonce, 0, 4);
    st64(nonce + 4, counter);
}

/* ------------------------------------------------------------------------ */
/* Batched transport path, same buffer contract as include/rg_aead.h         */

void rg_oracle_seal_one(const uint8_t *keys, const uint32_t *receivers, const rg_oracle_desc *d, uint64_t counter,
                        uint8_t *buf, uint8_t *status) {
    const uint8_t *key = keys + 32 * (size_t)d->key_idx;
    uint8_t *frame = buf + d->offset;
    uint8_t nonce[12];
    rg_oracle_wg_nonce(counter, nonce);
    uint8_t tag[16];
    rg_oracle_aead_seal(key, nonce, NULL, 0, frame + 16, d->len, tag);
    if (receivers) {
        /* DataHeader {type=4 LE u32, receiver LE u32, counter LE u64} */
        st32(frame + 0, 4u);
        st32(frame + 4, receivers[d->key_idx]);
        st64(frame + 8, counter);
    }
    memcpy(frame + 16 + d->len, tag, 16);
    if (status) *status = RG_ORACLE_OK;
}

void rg_oracle_open_one(const uint8_t *keys, const rg_oracle_desc *d, uint8_t *buf, uint8_t *status,
                        uint64_t *counter_out) {
    uint8_t *frame = buf + d->offset;
    uint32_t w = d->len;
    if (counter_out) *counter_out = 0;
    if ((d->offset & 15) != 0) { *status = RG_ORACLE_UNALIGNED; return; }      /* lib.rs:613-615 */
    if (w < 4) { *status = RG_ORACLE_INVALID; return; }                          /* lib.rs:619-620 */
    if (ld32(frame) != 4u) {                                                    /* lib.rs:621-628 */
        *status = ld32(frame) - 1u < 3u ? RG_ORACLE_NOT_DATA : RG_ORACLE_INVALID; /* 1-3 handshake/cookie, else :627 */
        return;
    }
    if ((w & 15) != 0 || w < 16) { *status = RG_ORACLE_INVALID; return; }        /* types lib.rs:181-196 */
    uint64_t counter = ld64(frame + 8);
    if (counter_out) *counter_out = counter;
    if (w < 32) { *status = RG_ORACLE_DECRYPT_ERR; return; }                     /* prim.rs:427-429 */
    const uint8_t *key = keys + 32 * (size_t)d->key_idx;
    uint8_t nonce[12];
    rg_oracle_wg_nonce(counter, nonce);
    size_t plen = (size_t)w - 32;
    int rc = rg_oracle_aead_open(key, nonce, NULL, 0, frame + 16, plen, frame + 16 + plen);
    *status = rc == 0 ? RG_ORACLE_OK : RG_ORACLE_DECRYPT_ERR;
}

/* Open of a frame straight off the wire (rustyguard-core/src/lib.rs:605-681):
 * the same checks as rg_oracle_open_one, with Sessions::decrypt_packet's
 * receiver -> session lookup (`peers_by_session.get_mut`, lib.rs:646-650;
 * unknown -> Error::Rejected) between the DataHeader framing check and the
 * AEAD.  Sessions are a plain list (receiver rx_rec[s], key row rx_key[s]),
 * searched linearly: deliberately not the product's hash table. */
void rg_oracle_open_one_rx(const uint8_t *keys, const uint32_t *rx_rec, const uint32_t *rx_key, size_t nrx,
                           const rg_oracle_desc *d, uint8_t *buf, uint8_t *status, uint64_t *counter_out,
                           uint32_t *key_out) {
    uint8_t *frame = buf + d->offset;
    uint32_t w = d->len;
    if (counter_out) *counter_out = 0;
    if (key_out) *key_out = 0xFFFFFFFFu;
    if ((d->offset & 15) != 0) { *status = RG_ORACLE_UNALIGNED; return; }      /* lib.rs:613-615 */
    if (w < 4) { *status = RG_ORACLE_INVALID; return; }                          /* lib.rs:619-620 */
    if (ld32(frame) != 4u) {                                                    /* lib.rs:621-628 */
        *status = ld32(frame) - 1u < 3u ? RG_ORACLE_NOT_DATA : RG_ORACLE_INVALID; /* 1-3 handshake/cookie, else :627 */
        return;
    }
    if ((w & 15) != 0 || w < 16) { *status = RG_ORACLE_INVALID; return; }        /* types lib.rs:181-196 */
    const uint32_t receiver = ld32(frame + 4);
    size_t s = 0;
    while (s < nrx && rx_rec[s] != receiver) s++;
    if (s == nrx) { *status = RG_ORACLE_REJECTED; return; }                      /* lib.rs:647-650 */
    if (key_out) *key_out = rx_key[s];
    rg_oracle_desc dk = *d;
    dk.key_idx = rx_key[s];
    rg_oracle_open_one(keys, &dk, buf, status, counter_out);
}

void rg_oracle_open_batch_rx(const uint8_t *keys, const uint32_t *rx_rec, const uint32_t *rx_key, size_t nrx,
                             const rg_oracle_desc *desc, size_t n, uint8_t *buf, uint8_t *status,
                             uint64_t *counters_out, uint32_t *key_out) {
    for (size_t i = 0; i < n; i++)
        rg_oracle_open_one_rx(keys, rx_rec, rx_key, nrx, &desc[i], buf, &status[i],
                              counters_out ? &counters_out[i] : NULL, key_out ? &key_out[i] : NULL);
}

typedef struct {
    int open;
    const uint8_t *keys;
    const uint32_t *receivers;
    const rg_oracle_desc *desc;
    const uint64_t *counters;
    uint8_t *buf;
    uint8_t *status;
    uint64_t *counters_out;
    size_t lo, hi;
} batch_job;

static void *batch_worker(void *arg) {
    batch_job *j = (batch_job *)arg;
    for (size_t i = j->lo; i < j->hi; i++) {
        if (j->open)
            rg_oracle_open_one(j->keys, &j->desc[i], j->buf, &j->status[i],
                               j->counters_out ? &j->counters_out[i] : NULL);
        else
            rg_oracle_seal_one(j->keys, j->receivers, &j->desc[i], j->counters[i], j->buf,
                               j->status ? &j->status[i] : NULL);
    }
    return NULL;
}

static void run_batch(batch_job proto, size_t n, int nthreads) {
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    if ((size_t)nthreads > n) nthreads = n ? (int)n : 1;
    pthread_t th[256];
    batch_job jobs[256];
    for (int t = 0; t < nthreads; t++) {
        jobs[t] = proto;
        jobs[t].lo = n * (size_t)t / (size_t)nthreads;
        jobs[t].hi = n * (size_t)(t + 1) / (size_t)nthreads;
    }
    if (nthreads == 1) {
        batch_worker(&jobs[0]);
        return;
    }
    for (int t = 0; t < nthreads; t++) pthread_create(&th[t], NULL, batch_worker, &jobs[t]);
    for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
}

void rg_oracle_seal_batch(const uint8_t *keys, const uint32_t *receivers, const rg_oracle_desc *desc,
                          const uint64_t *counters, size_t n, uint8_t *buf, uint8_t *status, int nthreads) {
    batch_job p = {0, keys, receivers, desc, counters, buf, status, NULL, 0, 0};
    run_batch(p, n, nthreads);
}

void rg_oracle_open_batch(const uint8_t *keys, const rg_oracle_desc *desc, size_t n, uint8_t *buf,
                          uint8_t *status, uint64_t *counters_out, int nthreads) {
    batch_job p = {1, keys, NULL, desc, NULL, buf, status, counters_out, 0, 0};
    run_batch(p, n, nthreads);
}

/* ------------------------------------------------------------------------ */
/* Synthetic plaintext generator (same formula as the product's device fill, */
/* cross-checked in tests/test_synth.py).                                    */

static uint64_t mix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

uint64_t rg_oracle_mix64(uint64_t x) { return mix64(x); }

/* Payload bytes of packet i: inner bytes [0, inner_len) are
 * le64(mix64(seed + (i << 16) + word)) bytes, bytes [inner_len, P) are the
 * zero padding of rustyguard-tun/src/lib.rs:229-238. */
void rg_oracle_synth_fill(uint8_t *buf, const rg_oracle_desc *desc, const uint32_t *inner_len, size_t n,
                          uint64_t seed) {
    for (size_t i = 0; i < n; i++) {
        uint8_t *p = buf + desc[i].offset + 16;
        uint32_t P = desc[i].len, L = inner_len[i];
        for (uint32_t w = 0; w * 8 < P; w++) {
            uint8_t tmp[8];
            st64(tmp, mix64(seed + ((uint64_t)i << 16) + w));
            for (uint32_t b = 0; b < 8 && w * 8 + b < P; b++) {
                uint32_t off = w * 8 + b;
                p[off] = off < L ? tmp[b] : 0;
            }
        }
    }
}
