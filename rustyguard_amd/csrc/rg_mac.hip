// rg_mac.hip -- batched handshake MAC checks: the
// HasMac::verify_mac1 / verify_mac2 filter of rustyguard-crypto/src/lib.rs:
// 114-209, i.e. keyed BLAKE2s-128 (Core::blake2s_mac, prim.rs:123-131,
// blake2s_simd with hash_length 16) over a handshake message up to its mac
// field, compared with that field.  One message per lane; with key index
// RG_KEY_SCAN every key is tried in order and the first match is kept, as in
// wg-proxy's peer scan (wg-proxy/src/main.rs:217-229).
//
// The keyed hash starts with the zero-padded key as its own block, so the
// state after it depends on the key alone: mac_key_state_kernel computes it
// once per key (one compression of three per 148-byte initiation saved), and
// messages are read as 16-byte vectors.
//
// BLAKE2s (RFC 7693) is 32-bit ARX like ChaCha20 -- 10 rounds of 8 G mixes
// over a 16-word state, rotations right by 16/12/8/7 -- so it runs on the
// same VALU idioms (byte rotations as v_perm_b32); the message schedule sigma
// is resolved at compile time (fully unrolled rounds, message words in VGPRs).
#include "rg_device.h"
#include "rg_internal.h"

namespace rg {
namespace {

__device__ __forceinline__ uint32_t rotr(uint32_t v, int n) { return __builtin_rotateright32(v, n); }
__device__ __forceinline__ uint32_t rotr16(uint32_t v) { return __builtin_amdgcn_perm(v, v, 0x01000302u); }
__device__ __forceinline__ uint32_t rotr8(uint32_t v) { return __builtin_amdgcn_perm(v, v, 0x00030201u); }

constexpr uint32_t kIV[8] = {0x6A09E667u, 0xBB67AE85u, 0x3C6EF372u, 0xA54FF53Au,
                             0x510E527Fu, 0x9B05688Cu, 0x1F83D9ABu, 0x5BE0CD19u};
constexpr uint8_t kSigma[10][16] = {
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15}, {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3},
    {11, 8, 12, 0, 5, 2, 15, 13, 10, 14, 3, 6, 7, 1, 9, 4}, {7, 9, 3, 1, 13, 12, 11, 14, 2, 6, 5, 10, 4, 0, 15, 8},
    {9, 0, 5, 7, 2, 4, 10, 15, 14, 1, 11, 12, 6, 8, 3, 13}, {2, 12, 6, 10, 0, 11, 8, 3, 4, 13, 7, 5, 15, 14, 1, 9},
    {12, 5, 1, 15, 14, 13, 4, 10, 0, 7, 6, 3, 9, 2, 8, 11}, {13, 11, 7, 14, 12, 1, 3, 9, 5, 0, 15, 4, 8, 6, 2, 10},
    {6, 15, 14, 9, 11, 3, 0, 8, 12, 2, 13, 7, 1, 4, 10, 5}, {10, 2, 8, 4, 7, 6, 1, 5, 15, 11, 9, 14, 3, 12, 13, 0}};

#define B2S_G(a, b, c, d, x, y)                        \
    a = a + b + (x); d = rotr16(d ^ a);                 \
    c = c + d; b = rotr(b ^ c, 12);                     \
    a = a + b + (y); d = rotr8(d ^ a);                  \
    c = c + d; b = rotr(b ^ c, 7);

// RFC 7693 §3.2 compression F; t = bytes hashed so far including this block
__device__ __forceinline__ void b2s_compress(uint32_t h[8], const uint32_t m[16], uint32_t t, bool last) {
    uint32_t v0 = h[0], v1 = h[1], v2 = h[2], v3 = h[3], v4 = h[4], v5 = h[5], v6 = h[6], v7 = h[7];
    uint32_t v8 = kIV[0], v9 = kIV[1], v10 = kIV[2], v11 = kIV[3];
    uint32_t v12 = kIV[4] ^ t, v13 = kIV[5], v14 = last ? ~kIV[6] : kIV[6], v15 = kIV[7];
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint8_t *s = kSigma[r];
        B2S_G(v0, v4, v8, v12, m[s[0]], m[s[1]]);
        B2S_G(v1, v5, v9, v13, m[s[2]], m[s[3]]);
        B2S_G(v2, v6, v10, v14, m[s[4]], m[s[5]]);
        B2S_G(v3, v7, v11, v15, m[s[6]], m[s[7]]);
        B2S_G(v0, v5, v10, v15, m[s[8]], m[s[9]]);
        B2S_G(v1, v6, v11, v12, m[s[10]], m[s[11]]);
        B2S_G(v2, v7, v8, v13, m[s[12]], m[s[13]]);
        B2S_G(v3, v4, v9, v14, m[s[14]], m[s[15]]);
    }
    h[0] ^= v0 ^ v8; h[1] ^= v1 ^ v9; h[2] ^= v2 ^ v10; h[3] ^= v3 ^ v11;
    h[4] ^= v4 ^ v12; h[5] ^= v5 ^ v13; h[6] ^= v6 ^ v14; h[7] ^= v7 ^ v15;
}
#undef B2S_G

// little-endian word at msg + byte, zero past len (byte loads: only for
// lengths or mac offsets that are not multiples of 4, which no handshake
// message has)
__device__ __forceinline__ uint32_t msg_word(const uint8_t *msg, uint32_t len, uint32_t byte) {
    uint32_t w = 0;
    for (uint32_t b = 0; b < 4; ++b)
        if (byte + b < len) w |= (uint32_t)msg[byte + b] << (8 * b);
    return w;
}

// the 16-byte piece p of a 16-byte aligned message, words past len zeroed
// (a partial last word keeps its low len % 4 bytes).  Only pieces starting
// below len are read; they end inside the frame, since the mac field follows.
__device__ __forceinline__ void msg_piece(const uint8_t *msg, uint32_t len, uint32_t p, uint32_t m[4]) {
    uint4 v = make_uint4(0, 0, 0, 0);
    if (16 * p < len) v = *reinterpret_cast<const uint4 *>(msg + 16 * p);
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint32_t byte = 16 * p + 4 * i;
        const uint32_t have = byte >= len ? 0u : min(len - byte, 4u);
        m[i] = have == 4 ? w[i] : w[i] & ((1u << (8 * have)) - 1u);
    }
}

// h after the key block (RFC 7693 §3.3: the zero-padded key is block 1 and,
// for a non-empty message, never the last block), so it depends on the key
// alone and is computed once per key by mac_key_state_kernel
__device__ __forceinline__ void b2s_key_state(const uint32_t *key, uint32_t key_len, bool last, uint32_t h[8]) {
#pragma unroll
    for (int i = 0; i < 8; ++i) h[i] = kIV[i];
    h[0] ^= 0x01010000u ^ (key_len << 8) ^ 16u;
    uint32_t m[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) m[i] = (uint32_t)(4 * i) < key_len ? key[i] : 0u;
    b2s_compress(h, m, 64, last);
}

// keyed BLAKE2s with a 16-byte digest of msg[0, len), len > 0, from the key
// state; returns the digest's first 4 words
__device__ __forceinline__ uint4 b2s_mac16(const uint32_t ks[8], const uint8_t *msg, uint32_t len) {
    uint32_t h[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) h[i] = ks[i];
    uint32_t t = 64;
    for (uint32_t off = 0; off < len; off += 64) {
        const uint32_t rem = len - off;
        const bool last = rem <= 64;
        uint32_t m[16];
#pragma unroll
        for (int p = 0; p < 4; ++p) msg_piece(msg + off, rem, p, m + 4 * p);
        t += last ? rem : 64;
        b2s_compress(h, m, t, last);
    }
    return make_uint4(h[0], h[1], h[2], h[3]);
}

__global__ __launch_bounds__(64) void mac_key_state_kernel(const uint32_t *keys, uint32_t key_len, uint32_t nkeys,
                                                          uint32_t *state) {
    const uint32_t k = blockIdx.x * 64 + threadIdx.x;
    if (k >= nkeys) return;
    uint32_t h[8];
    b2s_key_state(keys + (key_len / 4) * k, key_len, false, h);
    uint4 *o = reinterpret_cast<uint4 *>(state + 8 * k);
    o[0] = make_uint4(h[0], h[1], h[2], h[3]);
    o[1] = make_uint4(h[4], h[5], h[6], h[7]);
}

__global__ __launch_bounds__(256) void mac_verify_kernel(MacArgs a) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= a.n) return;
    const rg_pkt_desc d = a.desc[i];
    uint32_t found = RG_KEY_SKIP;
    uint8_t st;
    if ((d.offset & 15u) != 0) st = RG_PKT_UNALIGNED;
    else if (d.len < 32 || d.offset > a.buf_len || d.len > a.buf_len - d.offset) st = RG_PKT_INVALID;
    else {
        const uint8_t *msg = a.buf + d.offset;
        const uint32_t covered = d.len - (a.which == 2 ? 16u : 32u);
        uint4 want;
        if ((covered & 3u) == 0) {
            const uint32_t *w = reinterpret_cast<const uint32_t *>(msg + covered);
            want = make_uint4(w[0], w[1], w[2], w[3]);
        } else {
            want = make_uint4(msg_word(msg, d.len, covered), msg_word(msg, d.len, covered + 4),
                              msg_word(msg, d.len, covered + 8), msg_word(msg, d.len, covered + 12));
        }
        const bool scan = d.key_idx == RG_KEY_SCAN;
        const uint32_t lo = scan ? 0u : d.key_idx, hi = scan ? a.nkeys : min(d.key_idx + 1, a.nkeys);
        for (uint32_t k = lo; k < hi; ++k) {
            uint32_t ks[8];
            if (covered > 0) {
                const uint4 *s = reinterpret_cast<const uint4 *>(a.key_state + 8 * k);
                const uint4 s0 = s[0], s1 = s[1];
                ks[0] = s0.x; ks[1] = s0.y; ks[2] = s0.z; ks[3] = s0.w;
                ks[4] = s1.x; ks[5] = s1.y; ks[6] = s1.z; ks[7] = s1.w;
            } else { // empty covered part: the key block is the last block
                b2s_key_state(a.keys + (a.key_len / 4) * k, a.key_len, true, ks);
            }
            const uint4 mac = covered > 0 ? b2s_mac16(ks, msg, covered) : make_uint4(ks[0], ks[1], ks[2], ks[3]);
            const uint32_t diff = (mac.x ^ want.x) | (mac.y ^ want.y) | (mac.z ^ want.z) | (mac.w ^ want.w);
            if (diff == 0 && found == RG_KEY_SKIP) found = k; // first match, every key still hashed
        }
        st = found != RG_KEY_SKIP ? RG_PKT_OK : RG_PKT_REJECTED; // CryptoError::Rejected (lib.rs:146-152)
    }
    a.status[i] = st;
    if (a.key_out) a.key_out[i] = found;
}

} // namespace

hipError_t launch_mac_verify(const MacArgs &a, hipStream_t s) {
    if (a.n == 0) return hipSuccess;
    hipLaunchKernelGGL(mac_key_state_kernel, dim3((a.nkeys + 63) / 64), dim3(64), 0, s, a.keys, a.key_len, a.nkeys,
                       a.key_state);
    hipLaunchKernelGGL(mac_verify_kernel, dim3((a.n + 255) / 256), dim3(256), 0, s, a);
    return hipGetLastError();
}

} // namespace rg
