// rg_kernels.hip -- batched WireGuard transport-data ChaCha20-Poly1305 for
// gfx950 (MI355X).  Replaces the per-packet graviola call behind
// Core::chacha20poly1305_{enc,dec} (rustyguard-crypto/src/prim.rs:179-201)
// with one launch per batch.
//
// Mapping (v1): one packet per lane.  The lane walks its payload in 64-byte
// chunks: it issues the four 16-byte loads of the chunk, computes the chunk's
// keystream block in registers while they are in flight, XORs, stores, and
// folds the four ciphertext blocks into its Poly1305 accumulator (serial
// Horner with the clamped r; radix 2^32, v_mad_u64_u32).
#include "rg_device.h"
#include "rg_internal.h"

namespace rg {

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

// ------------------------------------------------------------------ seal
// Frame: [hdr 16][payload P][tag 16]; desc.len = P.
__global__ __launch_bounds__(256) void seal_lane_kernel(SealArgs a) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.n) return;
    const rg_pkt_desc d = a.desc[i];
    const uint32_t P = d.len;
    const bool valid = d.key_idx < a.nkeys && (P & 15u) == 0 && (d.offset & 15u) == 0 && P <= kMaxPayload &&
                       d.offset <= a.buf_len && P + 32 <= a.buf_len - d.offset;
    if (!valid) {
        if (a.status) a.status[i] = d.key_idx == RG_KEY_SKIP ? RG_PKT_REJECTED : RG_PKT_INVALID;
        return;
    }
    const Key8 key = load_key(a.keys, d.key_idx);
    const uint64_t ctr = a.counters[i];
    const uint32_t n1 = (uint32_t)ctr, n2 = (uint32_t)(ctr >> 32); // nonce = 0 || le64(ctr)
    uint32_t ks[16];
    chacha_block(key, 0, 0u, n1, n2, ks); // RFC 8439 §2.6 one-time key
    const Mul r = make_mul(ks[0], ks[1], ks[2], ks[3]);
    const uint32_t s0 = ks[4], s1 = ks[5], s2 = ks[6], s3 = ks[7];
    Acc h = {0, 0, 0, 0, 0};

    uint8_t *frame = a.buf + d.offset;
    uint4 *pl = reinterpret_cast<uint4 *>(frame + 16);
    const uint32_t nb = P >> 4; // 16-byte blocks
    for (uint32_t c = 0; 4 * c < nb; ++c) {
        const uint32_t b0 = 4 * c;
        const uint32_t cnt = nb - b0 < 4 ? nb - b0 : 4;
        uint4 m[4];
#pragma unroll
        for (int q = 0; q < 4; ++q)
            if (q < (int)cnt) m[q] = pl[b0 + q];
        chacha_block(key, c + 1, 0u, n1, n2, ks);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            if (q < (int)cnt) {
                const uint4 ct = xor4(m[q], ks + 4 * q);
                pl[b0 + q] = ct;
                acc_add(h, ct.x, ct.y, ct.z, ct.w, 1);
                acc_mul(h, r);
            }
        }
    }
    // length block: le64(aad_len = 0) || le64(P)   (RFC 8439 §2.8)
    acc_add(h, 0, 0, P, 0, 1);
    acc_mul(h, r);
    uint32_t tag[4];
    acc_finish(h, s0, s1, s2, s3, tag);
    if (a.receivers) {
        // DataHeader {4, receiver, counter} (rustyguard-core/src/lib.rs:286-290)
        *reinterpret_cast<uint4 *>(frame) = make_uint4(4u, a.receivers[d.key_idx], n1, n2);
    }
    *reinterpret_cast<uint4 *>(frame + 16 + P) = make_uint4(tag[0], tag[1], tag[2], tag[3]);
    if (a.status) a.status[i] = RG_PKT_OK;
}

// ------------------------------------------------------------------ open
// desc.len = W (frame).  Checks mirror rustyguard-core/src/lib.rs:613-629,
// rustyguard-types/src/lib.rs:181-196 and rustyguard-crypto/src/prim.rs:427-429.
__global__ __launch_bounds__(256) void open_lane_kernel(OpenArgs a) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.n) return;
    const rg_pkt_desc d = a.desc[i];
    const uint32_t W = d.len;
    if (a.counters_out) a.counters_out[i] = 0;
    uint8_t st;
    if (d.key_idx == RG_KEY_SKIP) st = RG_PKT_REJECTED;
    else if ((d.offset & 15u) != 0) st = RG_PKT_UNALIGNED;
    else if (d.key_idx >= a.nkeys || W > kMaxPayload + 32 || d.offset > a.buf_len || W > a.buf_len - d.offset ||
             W < 4)
        st = RG_PKT_INVALID;
    else st = 0xFF;
    if (st != 0xFF) {
        a.status[i] = st;
        return;
    }
    uint8_t *frame = a.buf + d.offset;
    const uint32_t type = *reinterpret_cast<const uint32_t *>(frame);
    if (type != 4u) {
        a.status[i] = RG_PKT_NOT_DATA;
        return;
    }
    if ((W & 15u) != 0 || W < 16) {
        a.status[i] = RG_PKT_INVALID;
        return;
    }
    const uint64_t ctr = *reinterpret_cast<const uint64_t *>(frame + 8);
    if (a.counters_out) a.counters_out[i] = ctr;
    if (W < 32) {
        a.status[i] = RG_PKT_DECRYPT_ERR;
        return;
    }
    const uint32_t P = W - 32;
    const Key8 key = load_key(a.keys, d.key_idx);
    const uint32_t n1 = (uint32_t)ctr, n2 = (uint32_t)(ctr >> 32);
    uint32_t ks[16];
    chacha_block(key, 0, 0u, n1, n2, ks);
    const Mul r = make_mul(ks[0], ks[1], ks[2], ks[3]);
    const uint32_t s0 = ks[4], s1 = ks[5], s2 = ks[6], s3 = ks[7];
    Acc h = {0, 0, 0, 0, 0};
    uint4 *pl = reinterpret_cast<uint4 *>(frame + 16);
    const uint32_t nb = P >> 4;
    // single pass: MAC the ciphertext and write plaintext; a failed tag
    // re-applies the keystream below so the frame is left unchanged.
    for (uint32_t c = 0; 4 * c < nb; ++c) {
        const uint32_t b0 = 4 * c;
        const uint32_t cnt = nb - b0 < 4 ? nb - b0 : 4;
        uint4 m[4];
#pragma unroll
        for (int q = 0; q < 4; ++q)
            if (q < (int)cnt) m[q] = pl[b0 + q];
        chacha_block(key, c + 1, 0u, n1, n2, ks);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            if (q < (int)cnt) {
                acc_add(h, m[q].x, m[q].y, m[q].z, m[q].w, 1);
                acc_mul(h, r);
                pl[b0 + q] = xor4(m[q], ks + 4 * q);
            }
        }
    }
    acc_add(h, 0, 0, P, 0, 1);
    acc_mul(h, r);
    uint32_t tag[4];
    acc_finish(h, s0, s1, s2, s3, tag);
    const uint4 want = *reinterpret_cast<const uint4 *>(frame + 16 + P);
    // constant-time compare (no early exit on the first differing word)
    const uint32_t diff = (tag[0] ^ want.x) | (tag[1] ^ want.y) | (tag[2] ^ want.z) | (tag[3] ^ want.w);
    if (diff != 0) {
        for (uint32_t c = 0; 4 * c < nb; ++c) {
            const uint32_t b0 = 4 * c;
            const uint32_t cnt = nb - b0 < 4 ? nb - b0 : 4;
            chacha_block(key, c + 1, 0u, n1, n2, ks);
            for (uint32_t q = 0; q < cnt; ++q) pl[b0 + q] = xor4(pl[b0 + q], ks + 4 * q);
        }
        a.status[i] = RG_PKT_DECRYPT_ERR;
    } else {
        a.status[i] = RG_PKT_OK;
    }
}

// --------------------------------------------------------------- general
// One lane per message, byte-granular: any nonce, any AAD, any length.  Used
// by the per-message CryptoPrimatives drop-in (handshake-sized messages).
__device__ void poly_bytes(Acc &h, const Mul &r, const uint8_t *p, uint64_t len) {
    for (uint64_t off = 0; off < len; off += 16) {
        uint32_t w[4] = {0, 0, 0, 0};
        for (int b = 0; b < 16; ++b)
            if (off + b < len) w[b >> 2] |= (uint32_t)p[off + b] << (8 * (b & 3));
        acc_add(h, w[0], w[1], w[2], w[3], 1); // zero-padded to 16 (RFC 8439 §2.8 pad16)
        acc_mul(h, r);
    }
}

__global__ void general_kernel(GeneralJob *jobs, uint32_t njobs, uint8_t *arena) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= njobs) return;
    GeneralJob &j = jobs[i];
    Key8 key;
    for (int t = 0; t < 8; ++t) key.k[t] = j.key[t];
    uint32_t ks[16];
    chacha_block(key, 0, j.nonce[0], j.nonce[1], j.nonce[2], ks);
    const Mul r = make_mul(ks[0], ks[1], ks[2], ks[3]);
    const uint32_t s0 = ks[4], s1 = ks[5], s2 = ks[6], s3 = ks[7];
    uint8_t *pl = arena + j.payload_off;
    const uint64_t len = j.payload_len;
    Acc h = {0, 0, 0, 0, 0};
    poly_bytes(h, r, arena + j.aad_off, j.aad_len);
    if (!j.decrypt) {
        for (uint64_t off = 0; off < len; off += 64) {
            chacha_block(key, (uint32_t)(off / 64) + 1, j.nonce[0], j.nonce[1], j.nonce[2], ks);
            for (int b = 0; b < 64 && off + b < len; ++b) pl[off + b] ^= (uint8_t)(ks[b >> 2] >> (8 * (b & 3)));
        }
    }
    poly_bytes(h, r, pl, len);
    acc_add(h, (uint32_t)j.aad_len, (uint32_t)(j.aad_len >> 32), (uint32_t)len, (uint32_t)(len >> 32), 1);
    acc_mul(h, r);
    uint32_t tag[4];
    acc_finish(h, s0, s1, s2, s3, tag);
    uint8_t *tp = arena + j.tag_off;
    if (!j.decrypt) {
        for (int b = 0; b < 16; ++b) tp[b] = (uint8_t)(tag[b >> 2] >> (8 * (b & 3)));
        j.status = RG_PKT_OK;
        return;
    }
    uint32_t diff = 0;
    for (int b = 0; b < 16; ++b) diff |= (uint32_t)(tp[b] ^ (uint8_t)(tag[b >> 2] >> (8 * (b & 3))));
    if (diff != 0) {
        j.status = RG_PKT_DECRYPT_ERR;
        return;
    }
    for (uint64_t off = 0; off < len; off += 64) {
        chacha_block(key, (uint32_t)(off / 64) + 1, j.nonce[0], j.nonce[1], j.nonce[2], ks);
        for (int b = 0; b < 64 && off + b < len; ++b) pl[off + b] ^= (uint8_t)(ks[b >> 2] >> (8 * (b & 3)));
    }
    j.status = RG_PKT_OK;
}

// ---------------------------------------------------------------- synth
__global__ __launch_bounds__(256) void synth_fill_kernel(const rg_pkt_desc *desc, const uint32_t *inner_len,
                                                         uint32_t n, uint8_t *buf, uint64_t buf_len, uint64_t seed) {
    const uint32_t i = blockIdx.x;
    if (i >= n) return;
    const rg_pkt_desc d = desc[i];
    const uint32_t P = d.len, L = inner_len[i];
    if ((d.offset & 7u) != 0 || P > kMaxPayload || d.offset > buf_len || 16 + (uint64_t)P > buf_len - d.offset) return;
    uint64_t *p = reinterpret_cast<uint64_t *>(buf + d.offset + 16);
    for (uint32_t w = threadIdx.x; 8 * w < P; w += blockDim.x) {
        uint64_t v = mix64(seed + ((uint64_t)i << 16) + w);
        const uint32_t b0 = 8 * w;
        if (b0 + 8 > L) {
            const uint32_t keep = L > b0 ? L - b0 : 0; // bytes of v kept (little-endian order)
            v = keep == 0 ? 0 : (v & (~0ull >> (64 - 8 * keep)));
        }
        if (b0 + 8 <= P) {
            p[w] = v;
        } else {
            uint8_t *pb = reinterpret_cast<uint8_t *>(p) + b0;
            for (uint32_t b = 0; b0 + b < P; ++b) pb[b] = (uint8_t)(v >> (8 * b));
        }
    }
}

// ---------------------------------------------------------------- launch
hipError_t launch_seal(const SealArgs &a, int lanes_per_packet, hipStream_t s) {
    (void)lanes_per_packet;
    if (a.n == 0) return hipSuccess;
    const uint32_t blocks = (a.n + 255) / 256;
    hipLaunchKernelGGL(seal_lane_kernel, dim3(blocks), dim3(256), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_open(const OpenArgs &a, int lanes_per_packet, hipStream_t s) {
    (void)lanes_per_packet;
    if (a.n == 0) return hipSuccess;
    const uint32_t blocks = (a.n + 255) / 256;
    hipLaunchKernelGGL(open_lane_kernel, dim3(blocks), dim3(256), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_general(GeneralJob *jobs, uint32_t njobs, uint8_t *arena, hipStream_t s) {
    if (njobs == 0) return hipSuccess;
    hipLaunchKernelGGL(general_kernel, dim3((njobs + 63) / 64), dim3(64), 0, s, jobs, njobs, arena);
    return hipGetLastError();
}

hipError_t launch_synth_fill(const rg_pkt_desc *desc, const uint32_t *inner_len, uint32_t n, uint8_t *buf,
                             uint64_t buf_len, uint64_t seed, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(synth_fill_kernel, dim3(n), dim3(256), 0, s, desc, inner_len, n, buf, buf_len, seed);
    return hipGetLastError();
}

} // namespace rg
