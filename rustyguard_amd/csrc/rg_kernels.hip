// rg_kernels.hip -- the per-message CryptoPrimatives drop-in kernel (any
// nonce, AAD and byte length: Core::chacha20poly1305_{enc,dec} and
// Core::xchacha20poly1305_{enc,dec}, rustyguard-crypto/src/prim.rs:179-224),
// the receiver-resolution pre-pass and the synthetic-payload generator
// used by benches and tests.  The batched transport kernels live in
// rg_pipe.hip (pipelined lanes) and rg_tile.hip (LDS-staged tiles).
#include "rg_device.h"
#include "rg_internal.h"

namespace rg {

// --------------------------------------------------------------- general
// One wave per message: any nonce, any AAD, any length.  Used by the
// per-message CryptoPrimatives drop-in (handshake-sized messages).  The host
// packs each message into a job arena at 16-byte aligned offsets with zeroed
// padding, so everything moves as 16-byte vectors: the lanes generate the
// keystream blocks in parallel (lane b: blocks b + 1, b + 65, ...), lane 0
// runs the Poly1305 Horner chain (RFC 8439 §2.8, pad16 of AAD and text).
__device__ __forceinline__ uint4 mask_tail(uint4 v, uint64_t valid) { // keep bytes [0, valid) of 16
    if (valid >= 16) return v;
    uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int64_t keep = (int64_t)valid - 4 * q;
        w[q] = keep >= 4 ? w[q] : keep <= 0 ? 0u : (w[q] & (0xFFFFFFFFu >> (32 - 8 * keep)));
    }
    return make_uint4(w[0], w[1], w[2], w[3]);
}

__device__ void poly_vec(Acc &h, const Mul &r, const uint4 *p, uint64_t len) {
    const uint64_t nb = (len + 15) / 16;
    for (uint64_t b0 = 0; b0 < nb; b0 += 8) { // eight loads in flight, then the Horner chain
        uint4 m[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) m[q] = p[min(b0 + q, nb - 1)];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            if (b0 + q >= nb) break;
            const uint4 v = mask_tail(m[q], len - 16 * (b0 + q)); // zero-padded to 16 (pad16)
            acc_add(h, v.x, v.y, v.z, v.w, 1);
            acc_mul(h, r);
        }
    }
}

// lanes XOR the keystream into the text: 64-byte chunk c uses block c + 1
__device__ void xor_stream(const Key8 &key, const uint32_t nonce[3], uint4 *pl, uint64_t len, uint32_t lane) {
    const uint64_t chunks = (len + 63) / 64;
    for (uint64_t c = lane; c < chunks; c += 64) {
        uint32_t ks[16];
        chacha_block(key, (uint32_t)c + 1, nonce[0], nonce[1], nonce[2], ks);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint64_t off = 64 * c + 16 * q;
            if (off >= len) break;
            const uint4 x = xor4(pl[off / 16], ks + 4 * q);
            pl[off / 16] = mask_tail(x, len - off); // bytes past the text stay zero
        }
    }
}

__global__ __launch_bounds__(64) void general_kernel(GeneralJob *jobs, uint32_t njobs, uint8_t *arena) {
    const uint32_t i = blockIdx.x, lane = threadIdx.x;
    if (i >= njobs) return;
    GeneralJob &j = jobs[i];
    Key8 key;
    for (int t = 0; t < 8; ++t) key.k[t] = j.key[t];
    if (j.xchacha) key = hchacha20(key, j.hnonce); // XChaCha20-Poly1305 subkey (prim.rs:202-224)
    const uint32_t nonce[3] = {j.nonce[0], j.nonce[1], j.nonce[2]};
    uint4 *pl = reinterpret_cast<uint4 *>(arena + j.payload_off);
    const uint64_t len = j.payload_len;
    __shared__ uint32_t verdict;
    if (!j.decrypt) {
        xor_stream(key, nonce, pl, len, lane);
        __threadfence_block();
        __syncthreads(); // every lane's ciphertext visible to lane 0
    }
    if (lane == 0) {
        uint32_t ks[16];
        chacha_block(key, 0, nonce[0], nonce[1], nonce[2], ks); // one-time Poly1305 key
        const Mul r = make_mul(ks[0], ks[1], ks[2], ks[3]);
        Acc h = {0, 0, 0, 0, 0};
        poly_vec(h, r, reinterpret_cast<const uint4 *>(arena + j.aad_off), j.aad_len);
        poly_vec(h, r, pl, len);
        acc_add(h, (uint32_t)j.aad_len, (uint32_t)(j.aad_len >> 32), (uint32_t)len, (uint32_t)(len >> 32), 1);
        acc_mul(h, r);
        uint32_t tag[4];
        acc_finish(h, ks[4], ks[5], ks[6], ks[7], tag);
        uint4 *tp = reinterpret_cast<uint4 *>(arena + j.tag_off);
        if (!j.decrypt) {
            *tp = make_uint4(tag[0], tag[1], tag[2], tag[3]);
            verdict = RG_PKT_OK;
        } else {
            const uint4 want = *tp;
            const uint32_t diff = (tag[0] ^ want.x) | (tag[1] ^ want.y) | (tag[2] ^ want.z) | (tag[3] ^ want.w);
            verdict = diff == 0 ? RG_PKT_OK : RG_PKT_DECRYPT_ERR;
        }
        j.status = verdict;
    }
    __syncthreads();
    if (j.decrypt && verdict == RG_PKT_OK) xor_stream(key, nonce, pl, len, lane); // text only if authentic
}

// ------------------------------------------------------------ receivers
// Device half of Sessions::decrypt_packet's lookup (rustyguard-core/src/lib.rs:
// 605-650): only a frame that passes the checks the reference makes first
// (16-byte alignment, in the buffer, message type 4, whole 16-byte segments of
// at least one) is looked up; an unknown receiver becomes RG_KEY_SKIP, which
// the open kernels report as RG_PKT_REJECTED.  Frames failing an earlier check
// get key 0, so the open kernel reports that check's status.
__global__ __launch_bounds__(256) void rx_resolve_kernel(const rg_pkt_desc *desc, uint32_t n, const uint8_t *buf,
                                                         uint64_t buf_len, const rg_rx_entry *table, uint32_t cap,
                                                         rg_pkt_desc *out, uint32_t *key_out) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    rg_pkt_desc d = desc[i];
    const uint64_t W = d.len;
    uint32_t k = 0, found = RG_KEY_SKIP;
    if ((d.offset & 15u) == 0 && d.offset <= buf_len && W <= buf_len - d.offset && W >= 16 && (W & 15u) == 0) {
        const uint4 hdr = *reinterpret_cast<const uint4 *>(buf + d.offset);
        if (hdr.x == 4u) {
            uint32_t s = rx_slot(hdr.y, cap);
            for (uint32_t probe = 0; probe < cap; ++probe) {
                const rg_rx_entry e = table[s];
                if (e.key_idx == RG_KEY_SKIP) break;
                if (e.receiver == hdr.y) {
                    found = e.key_idx;
                    break;
                }
                s = (s + 1) & (cap - 1);
            }
            k = found; // RG_KEY_SKIP when unknown: Error::Rejected
        }
    }
    d.key_idx = k;
    out[i] = d;
    if (key_out) key_out[i] = found;
}

hipError_t launch_rx_resolve(const rg_pkt_desc *desc, uint32_t n, const uint8_t *buf, uint64_t buf_len,
                             const rg_rx_entry *table, uint32_t cap, rg_pkt_desc *out, uint32_t *key_out,
                             hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(rx_resolve_kernel, dim3((n + 255) / 256), dim3(256), 0, s, desc, n, buf, buf_len, table, cap,
                       out, key_out);
    return hipGetLastError();
}

// ------------------------------------------------- session device batches
// rg_send_batch_dev: the caller's descriptors (offset, len) with the key row the
// host chose for each packet (its session's send key, or RG_KEY_SKIP)
__global__ __launch_bounds__(256) void bind_keys_kernel(const rg_pkt_desc *in, const uint32_t *key_idx, uint32_t n,
                                                        rg_pkt_desc *out) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    rg_pkt_desc d = in[i];
    d.key_idx = key_idx[i];
    out[i] = d;
}

hipError_t launch_bind_keys(const rg_pkt_desc *in, const uint32_t *key_idx, uint32_t n, rg_pkt_desc *out,
                            hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(bind_keys_kernel, dim3((n + 255) / 256), dim3(256), 0, s, in, key_idx, n, out);
    return hipGetLastError();
}

// rg_recv_batch_dev_finish: frames opened on the GPU but rejected by the in-order
// anti-replay pass go back to ciphertext by a re-seal under the same key and
// nonce; their seal descriptors (P = W - 32) and counters from the open's outputs
__global__ __launch_bounds__(256) void undo_gather_kernel(const rg_pkt_desc *rd, const uint64_t *ctr,
                                                          const uint32_t *idx, uint32_t m, rg_pkt_desc *out,
                                                          uint64_t *ctr_out) {
    const uint32_t j = blockIdx.x * 256 + threadIdx.x;
    if (j >= m) return;
    const uint32_t i = idx[j];
    rg_pkt_desc d = rd[i];
    d.len -= 32;
    out[j] = d;
    ctr_out[j] = ctr[i];
}

hipError_t launch_undo_gather(const rg_pkt_desc *rd, const uint64_t *ctr, const uint32_t *idx, uint32_t m,
                              rg_pkt_desc *out, uint64_t *ctr_out, hipStream_t s) {
    if (m == 0) return hipSuccess;
    hipLaunchKernelGGL(undo_gather_kernel, dim3((m + 255) / 256), dim3(256), 0, s, rd, ctr, idx, m, out, ctr_out);
    return hipGetLastError();
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

// ---------------------------------------------------------------- preset
// Fail-closed statuses (rg_internal.h): every status of the batch reads RG_PKT_PENDING until the transport
// kernel writes the packet's verdict, and the planner's control block starts from zero.  Byte stores,
// coalesced 64 per wave instruction; workgroup 0 also clears the control words.
__global__ __launch_bounds__(256) void preset_kernel(uint8_t *status, uint32_t n, uint32_t *ctl, uint32_t done_init,
                                                     uint32_t pool_init) {
    const uint32_t t = blockIdx.x * 256 + threadIdx.x;
    if (ctl && blockIdx.x == 0)
        for (uint32_t w = threadIdx.x; w < kCtlWords; w += 256)
            ctl[w] = w == kCtlCounts + kClasses ? done_init : w == kCtlPool ? pool_init : 0u;
    if (!status) return;
    for (uint32_t i = t; i < n; i += gridDim.x * 256) status[i] = RG_PKT_PENDING;
}

// ---------------------------------------------------------------- launch
hipError_t launch_preset(uint8_t *status, uint32_t n, uint32_t *ctl, uint32_t done_init, uint32_t pool_init,
                         hipStream_t s) {
    const uint32_t blocks = status ? max(1u, min(1024u, (n + 1023) / 1024)) : 1u;
    hipLaunchKernelGGL(preset_kernel, dim3(blocks), dim3(256), 0, s, status, n, ctl, done_init, pool_init);
    return hipGetLastError();
}

hipError_t launch_general(GeneralJob *jobs, uint32_t njobs, uint8_t *arena, hipStream_t s) {
    if (njobs == 0) return hipSuccess;
    hipLaunchKernelGGL(general_kernel, dim3(njobs), dim3(64), 0, s, jobs, njobs, arena);
    return hipGetLastError();
}

hipError_t launch_synth_fill(const rg_pkt_desc *desc, const uint32_t *inner_len, uint32_t n, uint8_t *buf,
                             uint64_t buf_len, uint64_t seed, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(synth_fill_kernel, dim3(n), dim3(256), 0, s, desc, inner_len, n, buf, buf_len, seed);
    return hipGetLastError();
}

} // namespace rg
