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

// ------------------------------------------------------------ K lanes
// K lanes cooperate on one packet (K = 1, 2, 4; groups never straddle a
// wave).  Payload chunk c (64 B, keystream block c+1) belongs to lane
// (c + shift) % K, where shift = roundup(C, K) - C pads the FRONT with empty
// chunks so that lane K-1 always owns the last chunk.  Every lane computes
// block 0 itself (r, s) -- it costs no wall time while C % K == 0.
//
// Poly1305 per lane in multiply-then-add form, acc = acc * r^d + m_b, where d
// is the block distance to the lane's previous block: 1 inside a chunk and
// 4K-3 across the K-1 chunks owned by the other lanes.  With B data blocks and
// bl blocks in the last chunk, h_B = sum_j acc_j r^{e_j}, e_{K-1} = 1,
// e_j = 4(K-2-j) + bl + 1; combined by a Horner pass over the lanes:
//   S = acc_0; S = S r^4 + acc_j (j < K-1); S = S r^bl + acc_{K-1};
//   h_B = S r;  tag = ((h_B + lenblock) r mod p) + s.
template <int K> struct Powers {
    Gen gap;   // r^(4K-3)
    Gen four;  // r^4
    Gen last;  // r^bl
};

template <int K> __device__ __forceinline__ Powers<K> make_powers(const Mul &r, uint32_t bl) {
    Powers<K> pw;
    if constexpr (K > 1) {
        const Acc r1 = {r.r0, r.r1, r.r2, r.r3, 0};
        Acc r2 = r1;
        acc_mul(r2, r);
        Acc r3 = r2;
        acc_mul(r3, r);
        Acc r4 = r2;
        acc_mul_gen(r4, make_gen(r2));
        pw.four = make_gen(r4);
        Acc rg;
        if constexpr (K == 2) {
            rg = r4;
            acc_mul(rg, r); // r^5
        } else {
            Acc r8 = r4;
            acc_mul_gen(r8, pw.four);
            Acc r12 = r8;
            acc_mul_gen(r12, pw.four);
            rg = r12;
            acc_mul(rg, r); // r^13
        }
        pw.gap = make_gen(rg);
        const Acc rb = bl == 1 ? r1 : bl == 2 ? r2 : bl == 3 ? r3 : r4;
        pw.last = make_gen(rb);
    }
    return pw;
}

__device__ __forceinline__ Acc shfl_up_acc(const Acc &a, int width) {
    Acc o;
    o.h0 = __shfl_up(a.h0, 1, width);
    o.h1 = __shfl_up(a.h1, 1, width);
    o.h2 = __shfl_up(a.h2, 1, width);
    o.h3 = __shfl_up(a.h3, 1, width);
    o.h4 = __shfl_up(a.h4, 1, width);
    return o;
}

// Combine the K per-lane accumulators into h_B on lane K-1 (other lanes: garbage).
template <int K> __device__ __forceinline__ Acc combine_lanes(Acc acc, uint32_t j, const Powers<K> &pw) {
    if constexpr (K > 1) {
        Acc S = acc;
#pragma unroll
        for (uint32_t s = 1; s < K; ++s) {
            Acc prev = shfl_up_acc(S, K);
            acc_mul_gen(prev, s == K - 1 ? pw.last : pw.four);
            acc_add(prev, acc.h0, acc.h1, acc.h2, acc.h3, acc.h4);
            if (j == s) S = prev;
        }
        return S;
    } else {
        (void)j;
        (void)pw;
        return acc;
    }
}

// Poly1305 step for one ciphertext block in multiply-then-add form.
template <int K> __device__ __forceinline__ void poly_step(Acc &acc, const Mul &r, const Powers<K> &pw, bool first,
                                                           const uint4 &ct) {
    if constexpr (K > 1) {
        if (first) acc_mul_gen(acc, pw.gap);
        else acc_mul(acc, r);
    } else {
        (void)first;
        (void)pw;
        acc_mul(acc, r);
    }
    acc_add(acc, ct.x, ct.y, ct.z, ct.w, 1);
}

// One lane's share of a packet: keystream XOR in place + Poly1305 over the
// ciphertext (seal: after XOR, open: before XOR).  Full 64-byte chunks run
// branch-free (4 loads issued before the keystream block, 4 stores after);
// the final partial chunk (bl < 4 blocks, always lane K-1's) runs after.
// MODE (diagnostics only, selected with rg_set_debug_mode): 0 = normal;
// 1 = compute only (payload loads/stores replaced by register data);
// 2 = memory only (no keystream / Poly1305, loads XORed with the block index).
template <int K, bool OPEN, int MODE = 0>
__device__ __forceinline__ Acc lane_pass(uint4 *pl, const Stream &st, const Mul &r, const Powers<K> &pw, uint32_t nb,
                                         uint32_t j) {
    const uint32_t C = (nb + 3) >> 2;
    const uint32_t T = (C + K - 1) / K; // rounds
    const uint32_t shift = T * K - C;   // empty chunks padded at the front
    const uint32_t bl = nb - 4 * (C - 1); // blocks in the last chunk (C > 0)
    const bool has_partial = C > 0 && bl < 4 && j == K - 1;
    const uint32_t t0 = j < shift ? 1 : 0;
    const uint32_t tend = has_partial ? T - 1 : T;
    Acc acc = {0, 0, 0, 0, 0};
    uint32_t ks[16];
    // Software pipeline: chunk t+1 is loaded at the top of round t, so its HBM
    // latency hides under round t's keystream block (values live across the
    // back-edge cannot be sunk to their use by the compiler).  The last round
    // re-loads its own chunk instead of running off the end (no branch).
    uint4 n0 = make_uint4(0, 0, 0, 0), n1 = n0, n2 = n0, n3 = n0;
    if (t0 < tend && MODE != 1) {
        const uint4 *src = pl + 4 * (t0 * K + j - shift);
        n0 = src[0]; n1 = src[1]; n2 = src[2]; n3 = src[3];
    }
    for (uint32_t t = t0; t < tend; ++t) {
        const uint32_t c = t * K + j - shift;
        uint4 *src = pl + 4 * c;
        const uint4 m0 = n0, m1 = n1, m2 = n2, m3 = n3;
        if constexpr (MODE != 1) {
            const uint4 *nxt = t + 1 < tend ? src + 4 * K : src;
            n0 = nxt[0]; n1 = nxt[1]; n2 = nxt[2]; n3 = nxt[3];
        } else {
            n0.x += c; n1.y ^= c; n2.z += t; n3.w ^= t; // fake data, loop-carried
        }
        if constexpr (MODE == 2) {
            const uint4 k = make_uint4(c, t, c ^ t, c + t);
            src[0] = make_uint4(m0.x ^ k.x, m0.y ^ k.y, m0.z ^ k.z, m0.w ^ k.w);
            src[1] = make_uint4(m1.x ^ k.x, m1.y ^ k.y, m1.z ^ k.z, m1.w ^ k.w);
            src[2] = make_uint4(m2.x ^ k.x, m2.y ^ k.y, m2.z ^ k.z, m2.w ^ k.w);
            src[3] = make_uint4(m3.x ^ k.x, m3.y ^ k.y, m3.z ^ k.z, m3.w ^ k.w);
            acc.h0 ^= m0.x ^ m1.y ^ m2.z ^ m3.w;
            continue;
        }
        stream_block(st, c + 1, ks);
        const uint4 x0 = xor4(m0, ks + 0), x1 = xor4(m1, ks + 4), x2 = xor4(m2, ks + 8), x3 = xor4(m3, ks + 12);
        if constexpr (MODE != 1) {
            src[0] = x0;
            src[1] = x1;
            src[2] = x2;
            src[3] = x3;
        }
        poly_step<K>(acc, r, pw, true, OPEN ? m0 : x0);
        poly_step<K>(acc, r, pw, false, OPEN ? m1 : x1);
        poly_step<K>(acc, r, pw, false, OPEN ? m2 : x2);
        poly_step<K>(acc, r, pw, false, OPEN ? m3 : x3);
    }
    if (has_partial) {
        const uint32_t c = C - 1;
        uint4 *src = pl + 4 * c;
        uint4 m[3];
#pragma unroll
        for (int q = 0; q < 3; ++q)
            if (q < (int)bl) m[q] = src[q];
        stream_block(st, c + 1, ks);
#pragma unroll
        for (int q = 0; q < 3; ++q) {
            if (q < (int)bl) {
                const uint4 x = xor4(m[q], ks + 4 * q);
                src[q] = x;
                poly_step<K>(acc, r, pw, q == 0, OPEN ? m[q] : x);
            }
        }
    }
    return acc;
}

// tag words from h_B (valid on lane K-1)
__device__ __forceinline__ void finish_tag(Acc hB, const Mul &r, uint32_t P, uint32_t s0, uint32_t s1, uint32_t s2,
                                           uint32_t s3, uint32_t tag[4]) {
    acc_mul(hB, r);           // h_B = S r
    acc_add(hB, 0, 0, P, 0, 1); // length block: le64(aad_len = 0) || le64(P)  (RFC 8439 §2.8)
    acc_mul(hB, r);
    acc_finish(hB, s0, s1, s2, s3, tag);
}

// ------------------------------------------------------------------ seal
// Frame: [hdr 16][payload P][tag 16]; desc.len = P.
template <int K, int MODE> __device__ __forceinline__ void seal_packet(const SealArgs &a, uint32_t i, uint32_t j) {
    const rg_pkt_desc d = a.desc[i];
    const uint32_t P = d.len;
    const bool valid = d.key_idx < a.nkeys && (P & 15u) == 0 && (d.offset & 15u) == 0 && P <= kMaxPayload &&
                       d.offset <= a.buf_len && P + 32 <= a.buf_len - d.offset;
    if (!valid) {
        if (a.status && j == 0) a.status[i] = d.key_idx == RG_KEY_SKIP ? RG_PKT_REJECTED : RG_PKT_INVALID;
        return;
    }
    const Key8 key = load_key(a.keys, d.key_idx);
    const uint64_t ctr = a.counters[i];
    const uint32_t n1 = (uint32_t)ctr, n2 = (uint32_t)(ctr >> 32); // nonce = 0 || le64(ctr)
    const Stream stm = make_stream(key, 0u, n1, n2);
    uint32_t ks[16];
    stream_block(stm, 0, ks); // RFC 8439 §2.6 one-time key
    const Mul r = make_mul(ks[0], ks[1], ks[2], ks[3]);
    const uint32_t s0 = ks[4], s1 = ks[5], s2 = ks[6], s3 = ks[7];
    const uint32_t nb = P >> 4;
    const uint32_t bl = nb == 0 ? 4 : nb - 4 * ((nb - 1) >> 2);
    const Powers<K> pw = make_powers<K>(r, bl);
    uint8_t *frame = a.buf + d.offset;
    Acc acc = lane_pass<K, false, MODE>(reinterpret_cast<uint4 *>(frame + 16), stm, r, pw, nb, j);
    Acc hB = combine_lanes<K>(acc, j, pw);
    if (j == K - 1) {
        uint32_t tag[4];
        finish_tag(hB, r, P, s0, s1, s2, s3, tag);
        if (a.receivers) // DataHeader {4, receiver, counter} (rustyguard-core/src/lib.rs:286-290)
            *reinterpret_cast<uint4 *>(frame) = make_uint4(4u, a.receivers[d.key_idx], n1, n2);
        *reinterpret_cast<uint4 *>(frame + 16 + P) = make_uint4(tag[0], tag[1], tag[2], tag[3]);
        if (a.status) a.status[i] = RG_PKT_OK;
    }
}

// ------------------------------------------------------------------ open
// desc.len = W (frame).  Checks mirror rustyguard-core/src/lib.rs:613-629,
// rustyguard-types/src/lib.rs:181-196 and rustyguard-crypto/src/prim.rs:427-429.
// Single pass: MAC the ciphertext and write plaintext; a failed tag re-applies
// the keystream so the frame is left unchanged (constant-time tag compare).
template <int K> __device__ __forceinline__ void open_packet(const OpenArgs &a, uint32_t i, uint32_t j) {
    const rg_pkt_desc d = a.desc[i];
    const uint32_t W = d.len;
    uint8_t st;
    if (d.key_idx == RG_KEY_SKIP) st = RG_PKT_REJECTED;
    else if ((d.offset & 15u) != 0) st = RG_PKT_UNALIGNED;
    else if (d.key_idx >= a.nkeys || W > kMaxPayload + 32 || d.offset > a.buf_len || W > a.buf_len - d.offset ||
             W < 4)
        st = RG_PKT_INVALID;
    else st = 0xFF;
    uint8_t *frame = a.buf + d.offset;
    uint64_t ctr = 0;
    if (st == 0xFF) {
        const uint4 hdr = *reinterpret_cast<const uint4 *>(frame);
        if (hdr.x != 4u) st = RG_PKT_NOT_DATA;
        else if ((W & 15u) != 0 || W < 16) st = RG_PKT_INVALID;
        else {
            ctr = ((uint64_t)hdr.w << 32) | hdr.z;
            if (W < 32) st = RG_PKT_DECRYPT_ERR;
        }
    }
    if (st != 0xFF) {
        if (j == 0) {
            a.status[i] = st;
            if (a.counters_out) a.counters_out[i] = ctr;
        }
        return;
    }
    const uint32_t P = W - 32;
    const Key8 key = load_key(a.keys, d.key_idx);
    const uint32_t n1 = (uint32_t)ctr, n2 = (uint32_t)(ctr >> 32);
    const Stream stm = make_stream(key, 0u, n1, n2);
    uint32_t ks[16];
    stream_block(stm, 0, ks);
    const Mul r = make_mul(ks[0], ks[1], ks[2], ks[3]);
    const uint32_t s0 = ks[4], s1 = ks[5], s2 = ks[6], s3 = ks[7];
    const uint32_t nb = P >> 4;
    const uint32_t bl = nb == 0 ? 4 : nb - 4 * ((nb - 1) >> 2);
    const Powers<K> pw = make_powers<K>(r, bl);
    uint4 *pl = reinterpret_cast<uint4 *>(frame + 16);
    Acc acc = lane_pass<K, true>(pl, stm, r, pw, nb, j);
    Acc hB = combine_lanes<K>(acc, j, pw);
    uint32_t ok = 0;
    if (j == K - 1) {
        uint32_t tag[4];
        finish_tag(hB, r, P, s0, s1, s2, s3, tag);
        const uint4 want = *reinterpret_cast<const uint4 *>(frame + 16 + P);
        const uint32_t diff = (tag[0] ^ want.x) | (tag[1] ^ want.y) | (tag[2] ^ want.z) | (tag[3] ^ want.w);
        ok = diff == 0;
    }
    if constexpr (K > 1) ok = __shfl(ok, K - 1, K);
    if (!ok) {
        // restore this lane's chunks: plaintext ^ keystream = ciphertext
        const uint32_t C = (nb + 3) >> 2, Cpad = (C + K - 1) / K * K, shift = Cpad - C;
        for (uint32_t v = j; v < Cpad; v += K) {
            if (v < shift) continue;
            const uint32_t c = v - shift, b0 = 4 * c, cnt = nb - b0 < 4 ? nb - b0 : 4;
            stream_block(stm, c + 1, ks);
            for (uint32_t q = 0; q < cnt; ++q) pl[b0 + q] = xor4(pl[b0 + q], ks + 4 * q);
        }
    }
    if (j == K - 1) {
        a.status[i] = ok ? RG_PKT_OK : RG_PKT_DECRYPT_ERR;
        if (a.counters_out) a.counters_out[i] = ctr;
    }
}

// ------------------------------------------------------------- kernels
// Persistent grid: the host launches at most (CUs x workgroups-per-CU)
// workgroups and reserves dynamic LDS so that exactly that many fit on each
// CU -- residency, and therefore the per-SIMD wave count, is the same on every
// CU (the dispatcher cannot stack three workgroups on one CU and one on
// another).  Lane groups then walk the packets grid-stride; a whole group
// (K lanes) always takes the same packet, so groups never diverge on i.
template <int K, int MODE = 0> __global__ __launch_bounds__(256) void seal_kernel(SealArgs a) {
    const uint32_t per_block = 256 / K;
    const uint32_t stride = gridDim.x * per_block;
    const uint32_t j = threadIdx.x % K;
    for (uint32_t i = blockIdx.x * per_block + threadIdx.x / K; i < a.n; i += stride) seal_packet<K, MODE>(a, i, j);
}

template <int K> __global__ __launch_bounds__(256) void open_kernel(OpenArgs a) {
    const uint32_t per_block = 256 / K;
    const uint32_t stride = gridDim.x * per_block;
    const uint32_t j = threadIdx.x % K;
    for (uint32_t i = blockIdx.x * per_block + threadIdx.x / K; i < a.n; i += stride) open_packet<K>(a, i, j);
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
static void grid_for(uint32_t n, int K, const Launch &L, uint32_t &blocks, uint32_t &lds) {
    const uint64_t want = ((uint64_t)n * K + 255) / 256;
    const uint64_t cap = (uint64_t)L.cus * (uint64_t)L.wg_per_cu;
    blocks = (uint32_t)(want < cap || cap == 0 ? want : cap);
    // reserve LDS so that exactly wg_per_cu workgroups are resident per CU
    lds = L.wg_per_cu > 0 ? (kLdsPerCu / L.wg_per_cu) & ~255u : 0;
}

template <typename A, void (*F1)(A), void (*F2)(A), void (*F4)(A)>
static hipError_t launch_k(const A &a, const Launch &L, hipStream_t s) {
    if (a.n == 0) return hipSuccess;
    uint32_t blocks, lds;
    grid_for(a.n, L.lanes, L, blocks, lds);
    switch (L.lanes) {
    case 1: hipLaunchKernelGGL(F1, dim3(blocks), dim3(256), lds, s, a); break;
    case 2: hipLaunchKernelGGL(F2, dim3(blocks), dim3(256), lds, s, a); break;
    case 4: hipLaunchKernelGGL(F4, dim3(blocks), dim3(256), lds, s, a); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_seal(const SealArgs &a, const Launch &L, hipStream_t s) {
    if (L.debug_mode == 1) return launch_k<SealArgs, seal_kernel<1, 1>, seal_kernel<2, 1>, seal_kernel<4, 1>>(a, L, s);
    if (L.debug_mode == 2) return launch_k<SealArgs, seal_kernel<1, 2>, seal_kernel<2, 2>, seal_kernel<4, 2>>(a, L, s);
    return launch_k<SealArgs, seal_kernel<1>, seal_kernel<2>, seal_kernel<4>>(a, L, s);
}

hipError_t launch_open(const OpenArgs &a, const Launch &L, hipStream_t s) {
    return launch_k<OpenArgs, open_kernel<1>, open_kernel<2>, open_kernel<4>>(a, L, s);
}

hipError_t prepare_kernels(int lanes_max_wg[2][3]) {
    // allow up to the whole 160 KiB LDS as dynamic shared memory, and report
    // how many 256-thread workgroups of each kernel fit on a CU (VGPR bound)
    void *seal[3] = {(void *)seal_kernel<1>, (void *)seal_kernel<2>, (void *)seal_kernel<4>};
    void *open[3] = {(void *)open_kernel<1>, (void *)open_kernel<2>, (void *)open_kernel<4>};
    for (int k = 0; k < 3; ++k) {
        for (int w = 0; w < 2; ++w) {
            const void *f = w == 0 ? seal[k] : open[k];
            hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kLdsPerCu);
            if (e != hipSuccess) return e;
            int nb = 0;
            e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, f, 256, 0);
            if (e != hipSuccess) return e;
            lanes_max_wg[w][k] = nb;
        }
    }
    return hipSuccess;
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
