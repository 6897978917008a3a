// rg_wave.hip -- the wave-tile kernel: batched WireGuard transport seal /
// open with coalesced frame I/O.  Replaces N x Core::chacha20poly1305_{enc,dec}
// (rustyguard-crypto/src/prim.rs:179-201) as driven by EncryptionKey::encrypt
// / DecryptionKey::decrypt (prim.rs:386-437), with the frame layout of
// EncryptedMetadata::frame_in_place (rustyguard-core/src/lib.rs:450-470).
//
// Compute is one packet per lane (16-word ChaCha20 state in VGPRs, serial
// Poly1305 Horner chain with the clamped r), as in rg_pipe.hip.  I/O is not:
// a lane-per-packet load touches 64 frames per wave instruction, and measured
// (tools/mempattern.hip) that pattern moves config-2 traffic at 3.5 TB/s
// against 4.7 TB/s when each wave instruction covers 16 frames x 64 contiguous
// bytes.  So a wave owns a tile of 64 packets and moves chunk t (64 B of each
// payload) with four coalesced instructions -- instruction k carries packets
// 16k..16k+15, lane l piece l%4 of packet 16k + l/4 -- and transposes through
// 8 KiB of wave-private LDS (no barriers: only the owning wave touches it):
//   coalesced regs R --ds_write--> in[] --ds_read (own packet)--> D
//   x = D ^ keystream --ds_write--> out[] --ds_read (coalesced)--> S --store
// Packet p keeps piece q in slot 4p + (q ^ ((p >> 2) & 3)): both the
// coalesced and the per-packet side are bank-conflict free.
//
// Every LDS and global operation of chunk t's step is placed inside its
// keystream rounds through the stream_block_hooked hook, so their latencies
// run under ARX work: after double round 0 the previous chunk's output is read
// back coalesced, after 2 it is stored; Poly1305 of chunk t-1 is absorbed
// after rounds 1, 3, 5, 7; after 8 chunk t is transposed in and chunk t+2 is
// requested, two steps ahead of its use.  Steps over
// chunks that every packet of the tile has in full run branch-free (exact
// vmcnt counts); the remaining steps (ragged tiles, the partial last chunk)
// are predicated.
#include "rg_device.h"
#include "rg_internal.h"

namespace rg {
namespace {

// Native 4 x u32 vectors throughout: HIP's uint4 is a union-based struct, and
// values of it that live across the hook's calls stay in scratch memory.
typedef uint32_t v4u __attribute__((ext_vector_type(4)));

struct Quad {
    v4u q0, q1, q2, q3;
};

__device__ __forceinline__ uint4 u4(v4u v) { return make_uint4(v.x, v.y, v.z, v.w); }
__device__ __forceinline__ v4u xorv(v4u m, const uint32_t *ks) {
    const v4u k = {ks[0], ks[1], ks[2], ks[3]};
    return m ^ k;
}

// Global-address-space 16-B blocks: the tile pointers are rebuilt from
// shuffled integers, and a generic pointer would compile to flat_* accesses,
// which count against lgkmcnt as well and make every wait a full drain.
typedef __attribute__((address_space(1))) v4u g_uint4;

// Per-lane view of the tile for coalesced I/O: instruction k reaches packet
// 16k + lane/4, piece lane%4.  Packets that are absent or invalid point at a
// harmless readable address with nbk = 0 (never stored).
struct Io {
    g_uint4 *base[4];  // payload (frame + 16) as 16-B blocks
    uint32_t last[4]; // index of the last readable block (loads clamp to it)
    uint32_t nbk[4];  // blocks (stores only below this)
};

__device__ __forceinline__ uint32_t wave_min(uint32_t v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v = min(v, (uint32_t)__shfl_xor((int)v, o));
    return v;
}
__device__ __forceinline__ uint32_t wave_max(uint32_t v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, o));
    return v;
}

// chunk t in coalesced layout (branch-free: block index clamped into the frame)
__device__ __forceinline__ void load_coal(const Io &io, Quad &R, uint32_t t, uint32_t q) {
    const uint32_t b = 4 * t + q;
    R.q0 = io.base[0][min(b, io.last[0])];
    R.q1 = io.base[1][min(b, io.last[1])];
    R.q2 = io.base[2][min(b, io.last[2])];
    R.q3 = io.base[3][min(b, io.last[3])];
}

template <bool FULL> __device__ __forceinline__ void store_coal(const Io &io, const Quad &S, uint32_t t, uint32_t q) {
    const uint32_t b = 4 * t + q;
    if (FULL || b < io.nbk[0]) io.base[0][b] = S.q0;
    if (FULL || b < io.nbk[1]) io.base[1][b] = S.q1;
    if (FULL || b < io.nbk[2]) io.base[2][b] = S.q2;
    if (FULL || b < io.nbk[3]) io.base[3][b] = S.q3;
}

// LDS slots: cb = this lane's coalesced slot in instruction 0 (+64 per k),
// own(q) = slot of this lane's packet's piece q
struct Slots {
    uint32_t cb, ob, osw;
    __device__ __forceinline__ uint32_t own(uint32_t q) const { return ob + (q ^ osw); }
};

__device__ __forceinline__ Slots make_slots(uint32_t lane) {
    Slots s;
    s.cb = 4 * (lane >> 2) + ((lane & 3) ^ ((lane >> 4) & 3));
    s.ob = 4 * lane;
    s.osw = (lane >> 2) & 3;
    return s;
}

__device__ __forceinline__ void read_coal(const v4u *L, const Slots &s, Quad &S) {
    S.q0 = L[s.cb]; S.q1 = L[64 + s.cb]; S.q2 = L[128 + s.cb]; S.q3 = L[192 + s.cb];
}

__device__ __forceinline__ void absorb_rest(Acc &h, const Quad &c, const Mul &r, uint32_t cnt) {
    acc_block_pred(h, u4(c.q0), r, cnt > 0);
    acc_block_pred(h, u4(c.q1), r, cnt > 1);
    acc_block_pred(h, u4(c.q2), r, cnt > 2);
    acc_block_pred(h, u4(c.q3), r, cnt > 3);
}

// One step over chunk t.  FIRST: nothing before it (no output to store, no
// Poly1305 to absorb).  FULL: chunks t and t-1 are whole in every packet of
// the tile -- unconditional stores and absorbs; otherwise predicated (pcnt =
// blocks of chunk t-1 in this lane's packet).  The Poly1305 input of chunk t-1
// is not kept in registers: it is re-read from this lane's own LDS slots
// (ciphertext: out[] after a seal step, in[] for open) one double round before
// each absorb, which saves 16 VGPRs and leaves the prefetch registers alone.
template <bool OPEN, bool FIRST, bool FULL>
__device__ __forceinline__ void wave_step(const Io &io, v4u *lin, v4u *lout, const Slots &sl, uint32_t q,
                                          const Stream &st, const Mul &r, Acc &h, uint32_t &pcnt, Quad &R,
                                          uint32_t t, uint32_t nb) {
    uint32_t ks[16];
    Quad D, S;
    v4u m;
    const v4u *pin = OPEN ? lin : lout;
    stream_block_hooked(st, t + 1, ks, [&](int dr) {
        if constexpr (!FIRST) {
            if (dr == 0) read_coal(lout, sl, S); // chunk t-1's output, coalesced
            if (dr == 2) store_coal<FULL>(io, S, t - 1, q);
            if (dr < 8 && dr % 2 == 0) m = pin[sl.own(dr / 2)];
            if (dr < 8 && dr % 2 == 1) {
                if constexpr (FULL) acc_block(h, u4(m), r);
                else acc_block_pred(h, u4(m), r, pcnt > (uint32_t)(dr / 2));
                pin_acc(h);
            }
        }
        if (dr == 8) { // chunk t: coalesced registers -> LDS -> this lane's packet; then chunk t+2
            lin[sl.cb] = R.q0; lin[64 + sl.cb] = R.q1; lin[128 + sl.cb] = R.q2; lin[192 + sl.cb] = R.q3;
            D.q0 = lin[sl.own(0)]; D.q1 = lin[sl.own(1)]; D.q2 = lin[sl.own(2)]; D.q3 = lin[sl.own(3)];
            load_coal(io, R, t + 2, q); // two steps ahead
        }
    });
    lout[sl.own(0)] = xorv(D.q0, ks + 0);
    lout[sl.own(1)] = xorv(D.q1, ks + 4);
    lout[sl.own(2)] = xorv(D.q2, ks + 8);
    lout[sl.own(3)] = xorv(D.q3, ks + 12);
    const uint32_t b0 = 4 * t;
    pcnt = FULL ? 4u : (nb > b0 ? min(nb - b0, 4u) : 0u);
}

// Keystream XOR + Poly1305 for this lane's packet (nb blocks) over the tile's
// chunk steps.  Fmin / Cmax: the tile's smallest full-chunk count and largest
// chunk count; R0 / R1 hold chunks 0 / 1 (loads issued).
template <bool OPEN>
__device__ __forceinline__ Acc wave_pass(const Io &io, v4u *lin, v4u *lout, const Slots &sl, uint32_t q,
                                         const Stream &st, const Mul &r, uint32_t nb, uint32_t Fmin, uint32_t Cmax,
                                         Quad &R0, Quad &R1) {
    Acc h = {0, 0, 0, 0, 0};
    uint32_t pcnt = 0;
    uint32_t t = 0;
    if (Fmin > 0) {
        wave_step<OPEN, true, true>(io, lin, lout, sl, q, st, r, h, pcnt, R0, 0, nb);
        t = 1;
        for (; t + 1 < Fmin; t += 2) { // whole pairs: exact vmcnt counts, chunk c in R(c % 2)
            wave_step<OPEN, false, true>(io, lin, lout, sl, q, st, r, h, pcnt, R1, t, nb);
            wave_step<OPEN, false, true>(io, lin, lout, sl, q, st, r, h, pcnt, R0, t + 1, nb);
        }
    }
    // predicated steps, t wave-uniform and odd from here on, so each buffer is
    // named statically (any runtime choice between R0 and R1 -- a reference
    // select, or branches the compiler merges -- puts both in scratch memory)
    if (t == 0 && Cmax > 0) {
        wave_step<OPEN, true, false>(io, lin, lout, sl, q, st, r, h, pcnt, R0, 0, nb);
        t = 1;
    }
    for (; t < Cmax; t += 2) {
        wave_step<OPEN, false, false>(io, lin, lout, sl, q, st, r, h, pcnt, R1, t, nb);
        if (t + 1 < Cmax) wave_step<OPEN, false, false>(io, lin, lout, sl, q, st, r, h, pcnt, R0, t + 1, nb);
    }
    if (Cmax > 0) { // the last chunk: output and Poly1305 input
        Quad S;
        read_coal(lout, sl, S);
        store_coal<false>(io, S, Cmax - 1, q);
        const v4u *pin = OPEN ? lin : lout;
        const Quad pi = {pin[sl.own(0)], pin[sl.own(1)], pin[sl.own(2)], pin[sl.own(3)]};
        absorb_rest(h, pi, r, pcnt);
    }
    return h;
}

// The tile's coalesced view: lane l of instruction k serves packet 16k + l/4.
// pay = this lane's payload address (or a harmless readable address when its
// packet is absent / invalid, nb = 0).
__device__ __forceinline__ Io make_io(uint64_t pay, uint32_t nb, uint32_t lane) {
    Io io;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int src = 16 * k + (int)(lane >> 2);
        const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)pay, src), hi = (uint32_t)__shfl((int)(uint32_t)(pay >> 32), src);
        io.base[k] = (g_uint4 *)(((uint64_t)hi << 32) | lo);
        io.nbk[k] = (uint32_t)__shfl((int)nb, src);
        io.last[k] = io.nbk[k] ? io.nbk[k] - 1 : 0;
    }
    return io;
}

// tag = ((h + lenblock) r mod p) + s; length block le64(aad_len = 0) || le64(P) (RFC 8439 §2.8)
__device__ __forceinline__ void wave_tag(Acc h, const Mul &r, uint32_t P, const uint32_t *s, uint32_t tag[4]) {
    acc_add(h, 0, 0, P, 0, 1);
    acc_mul(h, r);
    acc_finish(h, s[0], s[1], s[2], s[3], tag);
}

// ------------------------------------------------------------------ seal
// Frame: [hdr 16][payload P][tag 16]; desc.len = P.  Checks as seal_packet
// (rg_kernels.hip): descriptor and force_encrypt's padding assert
// (rustyguard-core/src/lib.rs:273-277).
__device__ __forceinline__ void wave_seal_tile(const SealArgs &a, uint32_t tile, v4u *lin, v4u *lout,
                                               uint32_t lane) {
    const uint32_t i = tile * 64 + lane;
    const bool present = i < a.n;
    rg_pkt_desc d = {0, 0, 0};
    if (present) d = a.desc[i];
    const uint32_t P = d.len;
    const bool valid = present && d.key_idx < a.nkeys && (P & 15u) == 0 && (d.offset & 15u) == 0 &&
                       P <= kMaxPayload && d.offset <= a.buf_len && P + 32 <= a.buf_len - d.offset;
    if (present && !valid && a.status) a.status[i] = d.key_idx == RG_KEY_SKIP ? RG_PKT_REJECTED : RG_PKT_INVALID;
    uint8_t *frame = a.buf + d.offset;
    const uint32_t nb = valid ? P >> 4 : 0;
    const Io io = make_io(valid ? (uint64_t)(frame + 16) : (uint64_t)a.keys, nb, lane);
    // invalid or absent packets give Fmin = 0: every step predicated, nothing stored for them
    const uint32_t Fmin = wave_min(nb >> 2), Cmax = wave_max((nb + 3) >> 2);
    const uint32_t q = lane & 3;
    Quad R0, R1;
    load_coal(io, R0, 0, q);
    load_coal(io, R1, 1, q);
    const Key8 key = load_key(a.keys, valid ? d.key_idx : 0);
    const uint64_t ctr = valid ? a.counters[i] : 0;
    const uint32_t n1 = (uint32_t)ctr, n2 = (uint32_t)(ctr >> 32); // nonce = 0 || le64(ctr) (prim.rs:32-36)
    const Stream stm = make_stream(key, 0u, n1, n2);
    uint32_t ks[16];
    stream_block(stm, 0, ks); // RFC 8439 §2.6 one-time key
    const Mul r = make_mul(ks[0], ks[1], ks[2], ks[3]);
    const Acc h = wave_pass<false>(io, lin, lout, make_slots(lane), q, stm, r, nb, Fmin, Cmax, R0, R1);
    if (!valid) return;
    uint32_t tag[4];
    wave_tag(h, r, P, ks + 4, tag);
    if (a.receivers) // DataHeader {4, receiver, counter} (rustyguard-core/src/lib.rs:286-290)
        *reinterpret_cast<uint4 *>(frame) = make_uint4(4u, a.receivers[d.key_idx], n1, n2);
    *reinterpret_cast<uint4 *>(frame + 16 + P) = make_uint4(tag[0], tag[1], tag[2], tag[3]);
    if (a.status) a.status[i] = RG_PKT_OK;
}

// ------------------------------------------------------------------ open
// desc.len = W.  Checks mirror rustyguard-core/src/lib.rs:613-629,
// rustyguard-types/src/lib.rs:181-196 and rustyguard-crypto/src/prim.rs:
// 427-429.  Decrypts speculatively while MACing the ciphertext; a failed tag
// (constant-time compare) re-applies the keystream, so the frame is left
// unchanged.
__device__ __forceinline__ void wave_open_tile(const OpenArgs &a, uint32_t tile, v4u *lin, v4u *lout,
                                               uint32_t lane) {
    const uint32_t i = tile * 64 + lane;
    const bool present = i < a.n;
    rg_pkt_desc d = {0, 0, 0};
    if (present) d = a.desc[i];
    const uint32_t W = d.len;
    uint32_t st;
    if (!present) st = 0;
    else if (d.key_idx == RG_KEY_SKIP) st = RG_PKT_REJECTED;
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
    if (present && st != 0xFF) {
        a.status[i] = (uint8_t)st;
        if (a.counters_out) a.counters_out[i] = ctr;
    }
    const bool valid = st == 0xFF;
    const uint32_t P = valid ? W - 32 : 0;
    const uint32_t nb = P >> 4;
    const Io io = make_io(valid ? (uint64_t)(frame + 16) : (uint64_t)a.keys, nb, lane);
    const uint32_t Fmin = wave_min(nb >> 2), Cmax = wave_max((nb + 3) >> 2);
    const uint32_t q = lane & 3;
    Quad R0, R1;
    load_coal(io, R0, 0, q);
    load_coal(io, R1, 1, q);
    uint4 want = make_uint4(0, 0, 0, 0);
    if (valid) want = *reinterpret_cast<const uint4 *>(frame + 16 + P);
    const Key8 key = load_key(a.keys, valid ? d.key_idx : 0);
    const uint32_t n1 = (uint32_t)ctr, n2 = (uint32_t)(ctr >> 32);
    const Stream stm = make_stream(key, 0u, n1, n2);
    uint32_t ks[16];
    stream_block(stm, 0, ks);
    const Mul r = make_mul(ks[0], ks[1], ks[2], ks[3]);
    const Acc h = wave_pass<true>(io, lin, lout, make_slots(lane), q, stm, r, nb, Fmin, Cmax, R0, R1);
    uint32_t tag[4];
    wave_tag(h, r, P, ks + 4, tag);
    const uint32_t diff = (tag[0] ^ want.x) | (tag[1] ^ want.y) | (tag[2] ^ want.z) | (tag[3] ^ want.w);
    const bool fail = valid && diff != 0;
    if (__any(fail)) {
        // other lanes stored this packet's plaintext: make their stores visible
        // to this lane's reads, then restore ciphertext = plaintext ^ keystream
        __threadfence();
        if (fail) {
            uint4 *pl = reinterpret_cast<uint4 *>(frame + 16);
            for (uint32_t c = 0; 4 * c < nb; ++c) {
                stream_block(stm, c + 1, ks);
                const uint32_t cnt = min(nb - 4 * c, 4u);
                for (uint32_t b = 0; b < cnt; ++b) pl[4 * c + b] = xor4(pl[4 * c + b], ks + 4 * b);
            }
        }
    }
    if (valid) {
        a.status[i] = fail ? RG_PKT_DECRYPT_ERR : RG_PKT_OK;
        if (a.counters_out) a.counters_out[i] = ctr;
    }
}

// s_memtime stamps per wave (debug buffer set): as rg_pipe.hip, kind 5
__device__ __forceinline__ void wave_stamp(uint64_t *dbg, uint64_t t0, uint64_t r0) {
    const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    if ((threadIdx.x & 63) == 0) {
        uint64_t *o = dbg + 8ull * (blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64);
        o[0] = t1 - t0; o[1] = 0; o[2] = 0; o[3] = 0;
        o[4] = r0; o[5] = 5; o[6] = 1; o[7] = r1 - r0;
    }
}

constexpr uint32_t kWaveLds = 512; // uint4 per wave: in[256] + out[256] = 8 KiB

} // namespace

// ------------------------------------------------------------- kernels
// Persistent grid of 4-wave workgroups; each wave walks tiles of 64 packets.
__global__ __launch_bounds__(256) void wave_seal_kernel(SealArgs a) {
    extern __shared__ v4u wave_lds[];
    const uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    v4u *lin = wave_lds + wv * kWaveLds, *lout = lin + 256;
    const uint32_t ntiles = (a.n + 63) / 64, nw = gridDim.x * 4;
    for (uint32_t tile = blockIdx.x * 4 + wv; tile < ntiles; tile += nw) wave_seal_tile(a, tile, lin, lout, lane);
    if (a.dbg) wave_stamp(a.dbg, t0, r0);
}

__global__ __launch_bounds__(256) void wave_open_kernel(OpenArgs a) {
    extern __shared__ v4u wave_lds[];
    const uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    v4u *lin = wave_lds + wv * kWaveLds, *lout = lin + 256;
    const uint32_t ntiles = (a.n + 63) / 64, nw = gridDim.x * 4;
    for (uint32_t tile = blockIdx.x * 4 + wv; tile < ntiles; tile += nw) wave_open_tile(a, tile, lin, lout, lane);
    if (a.dbg) wave_stamp(a.dbg, t0, r0);
}

hipError_t launch_wave(const SealArgs *sa, const OpenArgs *oa, const Launch &L, hipStream_t s) {
    const uint32_t n = sa ? sa->n : oa->n;
    if (n == 0) return hipSuccess;
    const uint64_t want = ((uint64_t)n + 255) / 256; // 4 tiles of 64 packets per workgroup
    const uint64_t cap = (uint64_t)L.cus * (uint64_t)L.wg_per_cu;
    const uint32_t blocks = (uint32_t)(want < cap || cap == 0 ? want : cap);
    // LDS: 4 waves x 8 KiB, or the residency reservation if larger
    const uint32_t need = 4 * kWaveLds * 16;
    const uint32_t resv = L.wg_per_cu > 0 ? (kLdsPerCu / L.wg_per_cu) & ~255u : 0;
    const uint32_t lds = resv > need ? resv : need;
    if (sa) hipLaunchKernelGGL(wave_seal_kernel, dim3(blocks), dim3(256), lds, s, *sa);
    else hipLaunchKernelGGL(wave_open_kernel, dim3(blocks), dim3(256), lds, s, *oa);
    return hipGetLastError();
}

hipError_t prepare_wave_kernels(int max_wg[2]) {
    const void *f[2] = {(const void *)wave_seal_kernel, (const void *)wave_open_kernel};
    for (int w = 0; w < 2; ++w) {
        hipError_t e = hipFuncSetAttribute(f[w], hipFuncAttributeMaxDynamicSharedMemorySize, (int)kLdsPerCu);
        if (e != hipSuccess) return e;
        int nb = 0;
        e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, f[w], 256, 4 * kWaveLds * 16);
        if (e != hipSuccess) return e;
        max_wg[w] = nb;
    }
    return hipSuccess;
}

} // namespace rg
