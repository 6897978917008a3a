// rg_rows.hip -- the row kernel: batched transport seal/open with
// wave-specialised workgroups.  Replaces N x Core::chacha20poly1305_{enc,dec}
// (rustyguard-crypto/src/prim.rs:179-201) as driven by EncryptionKey::encrypt
// / DecryptionKey::decrypt (prim.rs:386-437) for WireGuard data packets, with
// the frame layout of EncryptedMetadata::frame_in_place
// (rustyguard-core/src/lib.rs:450-470).
//
// Why: a packet's ChaCha20 blocks are independent, its Poly1305 chain is
// serial.  One packet per lane gives one wave per SIMD for a 64 Ki batch, and
// a single wave issues a VALU op only every ~5 cycles; splitting packets into
// segments costs more (key blocks, r^n) than it gains.  Here the keystream
// work is spread over many waves (one 64-byte block per lane per row) and the
// serial chain runs on a wave of its own:
//
//  * a tile is 64 packets: 64 consecutive packets of the batch (identity), or
//    64 entries of one size-class list of the planner (plan_kernel,
//    rg_tile.hip) when the batch mixes sizes; its rows are row 0 = ChaCha
//    block 0 of every lane's packet (the one-time Poly1305 key) and rows 1..R
//    = 64-byte chunk r-1 of every packet;
//  * a workgroup (8 waves) walks its tiles' rows as one stream in phases of 7
//    positions: ChaCha wave w (0..6) computes position 7k+w in phase k --
//    XORs each lane's chunk with keystream block r, stores it, and drops the
//    Poly1305 input (the ciphertext) into an LDS ring;
//  * wave 7 absorbs phase k-1's rows into each lane's Horner chain (lane =
//    packet, radix-2^32 clamped multiplies), finishes a tile's tags at its
//    last row, writes header + tag (seal) or verifies (open), and reports
//    every packet's status;
//  * a ChaCha wave runs a three-stage load pipeline (list entry -> descriptor
//    -> key / header / payload) ahead of its compute; the loop is unrolled
//    twice so that no register with a load in flight is ever copied (a copy
//    would make the compiler wait for it at the loop head).
//
// Open decrypts speculatively; a packet whose tag fails is re-encrypted by
// its workgroup after the last phase (all stores drained), so a rejected frame
// is left byte-for-byte unchanged (prim.rs:190-201; callers never read it on
// Err).
#include "rg_device.h"
#include "rg_internal.h"

namespace rg {

constexpr uint32_t kCWaves = 7;                    // ChaCha waves per workgroup
constexpr uint32_t kPieces = 5;                    // 16-byte pieces per lane per ring slot
constexpr uint32_t kSlotBytes = 64 * kPieces * 16; // 5 KiB
constexpr uint32_t kRingSlots = 2 * kCWaves;       // two phases in flight
constexpr uint32_t kFailCap = 256;                 // open failures remembered per workgroup
constexpr uint32_t kRingBytes = kRingSlots * kSlotBytes;
// last row of each of the workgroup's tiles, then of each tile pair (u16)
constexpr uint32_t kTableBytes = kRowMaxTilesWG * 2 + kRowMaxTilesWG;
constexpr uint32_t kRowLds = kRingBytes + kTableBytes + (kFailCap + 4) * 4;
static_assert(2 * kRowLds <= kLdsPerCu, "two row workgroups per CU");

// class c: c chunks for c <= 16; above, upper bounds 24, 32, 48, 64, ... (as rg_tile.hip)
__device__ __forceinline__ uint32_t rows_of_class(uint32_t c) {
    if (c <= 16) return c;
    const uint32_t j = c - 17;
    return (j & 1u) ? (1u << (j / 2 + 5)) : (3u << (j / 2 + 3));
}

__device__ __forceinline__ uint32_t readlane(uint32_t v, uint32_t l) {
    return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)l);
}

// ---------------------------------------------------------------- validation
// Per-packet checks, same order as the reference: seal -- the descriptor and
// force_encrypt's padding assert (rustyguard-core/src/lib.rs:273-277); open --
// alignment, message type, length, tag split (rustyguard-core/src/lib.rs:
// 613-628, rustyguard-types/src/lib.rs:181-196, rustyguard-crypto/src/prim.rs:
// 427-429).
struct Pkt {
    uint32_t st; // kWork, or the RG_PKT_* status to report
    uint32_t P, n1, n2;
};
constexpr uint32_t kWork = 0xFFu;
constexpr uint32_t kDead = 0x1FFu; // lane without a packet

template <bool OPEN>
__device__ __forceinline__ Pkt check_pkt(const rg_pkt_desc &d, uint64_t ctr, const uint4 &hdr, uint32_t nkeys,
                                         uint64_t buf_len) {
    Pkt k{kWork, 0, 0, 0};
    if constexpr (!OPEN) {
        const uint32_t P = d.len;
        const bool ok = d.key_idx < nkeys && (P & 15u) == 0 && (d.offset & 15u) == 0 && P <= kMaxPayload &&
                        d.offset <= buf_len && P + 32 <= buf_len - d.offset;
        if (!ok) k.st = d.key_idx == RG_KEY_SKIP ? RG_PKT_REJECTED : RG_PKT_INVALID;
        else {
            k.P = P;
            k.n1 = (uint32_t)ctr;
            k.n2 = (uint32_t)(ctr >> 32);
        }
    } else {
        const uint32_t W = d.len;
        if (d.key_idx == RG_KEY_SKIP) k.st = RG_PKT_REJECTED;
        else if ((d.offset & 15u) != 0) k.st = RG_PKT_UNALIGNED;
        else if (d.key_idx >= nkeys || W > kMaxPayload + 32 || d.offset > buf_len || W > buf_len - d.offset || W < 4)
            k.st = RG_PKT_INVALID;
        else if (hdr.x != 4u) k.st = RG_PKT_NOT_DATA;
        else if ((W & 15u) != 0 || W < 16) k.st = RG_PKT_INVALID;
        else {
            k.n1 = hdr.z;
            k.n2 = hdr.w;
            if (W < 32) k.st = RG_PKT_DECRYPT_ERR;
            else k.P = W - 32;
        }
    }
    return k;
}

// payload length as the size classes see it (before the header checks)
template <bool OPEN> __device__ __forceinline__ uint32_t pre_payload(const rg_pkt_desc &d) {
    const uint32_t P = OPEN ? (d.len >= 32 ? d.len - 32 : 0u) : d.len;
    return P <= kMaxPayload ? P : 0u;
}

__device__ __forceinline__ uint64_t row_stamp() {
    uint64_t t;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}
__device__ __forceinline__ uint64_t row_realtime() { // 100 MHz constant clock
    uint64_t t;
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}

__device__ __forceinline__ uint4 load_glc(const uint8_t *p) {
    uint4 v;
    asm volatile("global_load_dwordx4 %0, %1, off sc0 sc1\n\ts_waitcnt vmcnt(0)" : "=v"(v) : "v"(p) : "memory");
    return v;
}

// Re-apply the keystream to a packet whose tag failed after speculative
// decryption: its frame then holds the ciphertext again.  Called once every
// store of the workgroup has drained; payload reads bypass the L1.
__device__ void restore_packet(const OpenArgs &oa, uint32_t i) {
    const rg_pkt_desc d = oa.desc[i];
    const uint4 hdr = *reinterpret_cast<const uint4 *>(oa.buf + d.offset);
    const Pkt k = check_pkt<true>(d, 0, hdr, oa.nkeys, oa.buf_len);
    if (k.st != kWork) return;
    const Key8 key = load_key(oa.keys, d.key_idx);
    uint8_t *pl = oa.buf + d.offset + 16;
    const uint32_t nb = k.P >> 4;
    uint32_t ks[16];
    for (uint32_t c = 0; 4 * c < nb; ++c) {
        chacha_block(key, c + 1, 0u, k.n1, k.n2, ks);
        const uint32_t hi = 4 * c + 4 < nb ? 4 * c + 4 : nb;
        for (uint32_t q = 4 * c; q < hi; ++q)
            *reinterpret_cast<uint4 *>(pl + 16 * q) = xor4(load_glc(pl + 16 * q), ks + 4 * (q - 4 * c));
    }
}

// ------------------------------------------------------------ tile sources
// Planned batches: buckets of the planner's lists, largest class first; lane b
// holds bucket b.  Identical in every wave.
struct Buckets {
    uint32_t cls, cnt, tb, te; // per lane
    uint32_t tiles;            // uniform
};

__device__ __forceinline__ Buckets make_buckets(const TilePlan &tp) {
    const uint32_t b = threadIdx.x & 63;
    Buckets B;
    B.cls = b < kClasses ? kClasses - 1 - b : 0;
    B.cnt = b < kClasses ? tp.counts[B.cls] : 0;
    const uint32_t t = (B.cnt + 63) / 64;
    uint32_t x = t;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(x, d);
        if ((int)b >= d) x += y;
    }
    B.te = x;
    B.tb = x - t;
    B.tiles = uniform_u32(__shfl(x, 63));
    return B;
}

// ---------------------------------------------------------------- kernel
// ChaCha-wave pipeline registers, one set per stream position parity
struct L0 { // packet index of each lane (planned: list entry in flight)
    bool valid;
    uint32_t r, i, live;
};
struct L1 { // descriptor (+ seal counter) in flight
    bool valid;
    uint32_t r, i, live;
    rg_pkt_desc d;
    uint64_t ctr;
};
struct L2 { // key, header, payload (key row: frame tag / receiver id) in flight
    Key8 key;
    uint4 hdr;
    uint4 m[4];
    uint32_t recv;
};

template <bool OPEN, bool PLANNED>
__global__ __launch_bounds__(512, 4) void row_kernel(SealArgs sa, OpenArgs oa, TilePlan tp) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds_raw[];
    uint4 *const ring = reinterpret_cast<uint4 *>(lds_raw);
    uint16_t *const table = reinterpret_cast<uint16_t *>(lds_raw + kRingBytes);
    uint16_t *const ptable = table + kRowMaxTilesWG; // tile pairs
    uint32_t *const fails = reinterpret_cast<uint32_t *>(lds_raw + kRingBytes + kTableBytes); // [0] count, [1] total
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wave = threadIdx.x >> 6;
    const uint32_t n = OPEN ? oa.n : sa.n;
    uint8_t *const buf = OPEN ? oa.buf : sa.buf;
    const uint64_t buf_len = OPEN ? oa.buf_len : sa.buf_len;
    const uint32_t nkeys = OPEN ? oa.nkeys : sa.nkeys;
    const uint32_t *const keys = OPEN ? oa.keys : sa.keys;
    const rg_pkt_desc *const desc = OPEN ? oa.desc : sa.desc;
    constexpr bool planned = PLANNED;
    const uint32_t G = gridDim.x, bid = blockIdx.x;
    // diagnostics (debug mode 3): per-wave s_memtime section totals
    uint64_t *const dbg = OPEN ? oa.dbg : sa.dbg;
    uint64_t t_issue = 0, t_comp = 0, t_bar = 0, t_mark = 0, rt0 = 0, t_pro = 0;
    if (dbg) {
        rt0 = row_realtime();
        t_mark = row_stamp();
    }
    auto lap = [&](uint64_t &acc) {
        if (dbg) {
            const uint64_t t = row_stamp();
            acc += t - t_mark;
            t_mark = t;
        }
    };

    // ---- prologue: the last row of each of this workgroup's tiles (table),
    // and the length of its row stream
    Buckets B{};
    if constexpr (PLANNED) B = make_buckets(tp);
    const uint32_t tiles = planned ? B.tiles : (n + 63) / 64;
    const uint32_t ntw = tiles > bid ? (tiles - bid + G - 1) / G : 0u; // <= kRowMaxTilesWG (host grid sizing)
    if (threadIdx.x == 0) {
        fails[0] = 0;
        fails[1] = 0;
    }
    __syncthreads();
    for (uint32_t j = wave; j < ntw; j += 8) {
        const uint32_t T = bid + j * G;
        uint32_t R;
        if constexpr (PLANNED) {
            const uint32_t b = (uint32_t)__popcll(__ballot(B.te <= T));
            R = rows_of_class(readlane(B.cls, b < 64 ? b : 63));
        } else {
            const uint32_t i = 64 * T + lane;
            const uint32_t c = i < n ? (pre_payload<OPEN>(desc[i]) + 63) / 64 : 0u;
            uint32_t m = c;
#pragma unroll
            for (int s = 32; s >= 1; s >>= 1) {
                const uint32_t o = __shfl_xor(m, s);
                m = o > m ? o : m;
            }
            R = uniform_u32(m);
        }
        if (lane == 0) table[j] = (uint16_t)R;
    }
    __syncthreads();
    // tiles 2u, 2u+1 form pair u: its rows alternate between the two tiles in
    // the stream (positions 2 (row) + half), so that the Poly1305 wave carries
    // two independent Horner chains per lane
    const uint32_t npairs = (ntw + 1) / 2;
    uint32_t part = 0;
    for (uint32_t u = threadIdx.x; u < npairs; u += blockDim.x) {
        const uint32_t a = table[2 * u], b = 2 * u + 1 < ntw ? table[2 * u + 1] : 0u;
        const uint32_t R = a > b ? a : b;
        ptable[u] = (uint16_t)R;
        part += 2 * (R + 1);
    }
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) part += __shfl_xor(part, m);
    if (lane == 0 && part) atomicAdd(&fails[1], part);
    __syncthreads();
    const uint32_t S = fails[1];
    const uint32_t phases = (S + kCWaves - 1) / kCWaves + 1;
    lap(t_pro);

    // row-stream cursor over tile pairs (wave-uniform; positions only move forward)
    uint32_t cu = 0, cstart = 0, cR = npairs ? uniform_u32(ptable[0]) : 0u;
    auto seek = [&](uint32_t s) {
        while (s >= cstart + 2 * (cR + 1)) {
            cstart += 2 * (cR + 1);
            ++cu;
            cR = uniform_u32(ptable[cu]);
        }
    };

    if (wave < kCWaves) {
        // ------------------------------------------------ ChaCha wave
        auto issue_l0 = [&](uint32_t k) -> L0 {
            L0 a;
            const uint32_t s = kCWaves * k + wave;
            a.valid = s < S;
            a.r = a.i = a.live = 0;
            if (a.valid) {
                seek(s);
                a.r = (s - cstart) >> 1;
                const uint32_t j = 2 * cu + ((s - cstart) & 1u);
                const uint32_t T = bid + j * G;
                if (j >= ntw) {
                    a.live = 0; // odd tile count: the pair's second tile is empty
                } else if constexpr (PLANNED) {
                    const uint32_t b = (uint32_t)__popcll(__ballot(B.te <= T));
                    const uint32_t tb = readlane(B.tb, b), cls = readlane(B.cls, b), cnt = readlane(B.cnt, b);
                    const uint32_t slot = (T - tb) * 64 + lane;
                    a.live = slot < cnt;
                    a.i = tp.lists[(uint64_t)cls * tp.cap + (a.live ? slot : 0u)];
                } else {
                    a.i = 64 * T + lane;
                    a.live = a.i < n;
                }
            }
            return a;
        };
        auto issue_l1 = [&](const L0 &a) -> L1 {
            L1 b;
            b.valid = a.valid;
            b.r = a.r;
            b.live = a.valid && a.live;
            b.i = b.live ? a.i : 0u;
            b.d = desc[b.i];
            b.ctr = 0;
            if constexpr (!OPEN) b.ctr = sa.counters[b.i];
            return b;
        };
        auto issue_l2 = [&](const L1 &b) -> L2 {
            L2 c;
            const uint32_t P = pre_payload<OPEN>(b.d);
            const bool pre = b.live && b.d.key_idx < nkeys && (b.d.offset & 15u) == 0 && b.d.offset <= buf_len &&
                             (uint64_t)P + 32 <= buf_len - b.d.offset;
            // every lane issues the same loads on every row (invalid ones read a
            // harmless address): the load count per stage is fixed, so the
            // compiler's vmcnt waits stay partial
            const uint8_t *safe = reinterpret_cast<const uint8_t *>(keys);
            const uint8_t *fr = pre ? buf + b.d.offset : safe;
            c.key = load_key(keys, pre ? b.d.key_idx : 0u);
            c.hdr = make_uint4(0, 0, 0, 0);
            if constexpr (OPEN) c.hdr = *reinterpret_cast<const uint4 *>(fr);
            const uint32_t nb = pre ? P >> 4 : 0u, q0 = b.r > 0 ? 4 * (b.r - 1) : 0u;
#pragma unroll
            for (uint32_t q = 0; q < 4; ++q) {
                const bool v = b.r > 0 && q0 + q < nb;
                // key row, open: piece 0 is the frame's tag
                const bool tag = OPEN && q == 0 && b.r == 0 && pre;
                c.m[q] = *reinterpret_cast<const uint4 *>(v ? fr + 16 + 16 * (q0 + q) : tag ? fr + 16 + P : safe);
            }
            if constexpr (!OPEN) {
                // key row: the receiver id for the header
                const bool rv = sa.receivers && b.r == 0 && pre;
                c.recv = *(rv ? sa.receivers + b.d.key_idx : keys);
            }
            return c;
        };
        auto compute = [&](uint32_t k, const L1 &b, const L2 &c) {
            if (!b.valid) return;
            uint4 hdr = c.hdr;
            if constexpr (OPEN) {
                // a frame too short for the prefetch (within 48 bytes of the arena's
                // end): the header checks need what is there
                const uint32_t P = pre_payload<OPEN>(b.d);
                const bool pre = b.d.key_idx < nkeys && (b.d.offset & 15u) == 0 && b.d.offset <= buf_len &&
                                 (uint64_t)P + 32 <= buf_len - b.d.offset;
                if (b.live && !pre) {
                    hdr = make_uint4(0, 0, 0, 0);
                    if ((b.d.offset & 15u) == 0 && b.d.offset <= buf_len) {
                        const uint64_t room = buf_len - b.d.offset;
                        if (room >= 16) hdr = *reinterpret_cast<const uint4 *>(buf + b.d.offset);
                        else if (room >= 4) hdr.x = *reinterpret_cast<const uint32_t *>(buf + b.d.offset);
                    }
                }
            }
            const Pkt pk = check_pkt<OPEN>(b.d, b.ctr, hdr, nkeys, buf_len);
            const uint32_t st = b.live ? pk.st : kDead;
            uint4 *const slot = ring + ((k & 1) * kCWaves + wave) * (kSlotBytes / 16);
            uint32_t ks[16];
            chacha_block(c.key, b.r, 0u, pk.n1, pk.n2, ks);
            if (b.r == 0) {
                // key row: Poly1305 key and the packet record for the Poly1305 wave
                slot[0 * 64 + lane] = make_uint4(ks[0], ks[1], ks[2], ks[3]);
                slot[1 * 64 + lane] = make_uint4(ks[4], ks[5], ks[6], ks[7]);
                slot[2 * 64 + lane] = make_uint4((uint32_t)b.d.offset, (uint32_t)(b.d.offset >> 32), pk.P, st);
                slot[3 * 64 + lane] = make_uint4(pk.n1, pk.n2, b.i, 0);
                slot[4 * 64 + lane] = OPEN ? c.m[0] : make_uint4(c.recv, 0, 0, 0);
            } else {
                const uint32_t nb = st == kWork ? pk.P >> 4 : 0u, q0 = 4 * (b.r - 1);
                const uint32_t nblk = nb > q0 ? (nb - q0 < 4 ? nb - q0 : 4u) : 0u;
                uint4 *dst = reinterpret_cast<uint4 *>(buf + b.d.offset + 16) + q0;
#pragma unroll
                for (uint32_t q = 0; q < 4; ++q) {
                    const uint4 x = xor4(c.m[q], ks + 4 * q);
                    if (q < nblk) dst[q] = x;
                    slot[q * 64 + lane] = OPEN ? c.m[q] : x;
                }
            }
        };
        // one phase: loads for positions k+3 (list), k+2 (descriptor), k+1
        // (payload), then the compute of position k.  Register sets by parity:
        // l0/l1/l2/meta of position p live in set p % 2.
        auto phase = [&](uint32_t k, L0 &l0w, L0 &l0r, L1 &l1w, L1 &l1r, L2 &l2w, L2 &l2r, L1 &mw, L1 &mr)
                         __attribute__((always_inline)) {
            l0w = issue_l0(k + 3);
            l1w = issue_l1(l0r);
            l2w = issue_l2(l1r);
            mw = l1r;
            lap(t_issue);
            compute(k, mr, l2r);
            lap(t_comp);
            asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
            lap(t_bar);
        };
        L0 l0A, l0B;
        L1 l1A, l1B, mA, mB;
        L2 l2A, l2B;
        // prologue in stream order (the cursor only moves forward)
        l0A = issue_l0(0);
        l1A = issue_l1(l0A);
        l0B = issue_l0(1);
        l1B = issue_l1(l0B);
        l0A = issue_l0(2);
        l2A = issue_l2(l1A);
        mA = l1A;
        for (uint32_t k = 0; k < phases; k += 2) {
            phase(k, l0B, l0A, l1A, l1B, l2B, l2A, mB, mA);
            if (k + 1 >= phases) break;
            phase(k + 1, l0A, l0B, l1B, l1A, l2A, l2B, mA, mB);
        }
    } else {
        // ------------------------------------------------ Poly1305 wave
        // its serial chains bound the phase: let it issue ahead of the ChaCha waves
        __builtin_amdgcn_s_setprio(3);
        struct PState { // one lane's packet of one tile of the pair
            Mul r;
            uint32_t s0, s1, s2, s3;
            Acc acc;
            uint64_t off;
            uint32_t P, st, n1, n2, pi;
            uint4 extra;
        };
        PState pa{}, pb{};
        pa.st = pb.st = kDead;
        auto slot_at = [&](uint32_t k, uint32_t j) -> const uint4 * {
            return ring + (((k - 1) & 1) * kCWaves + j) * (kSlotBytes / 16);
        };
        auto key_row = [&](PState &x, const uint4 *slot) {
            const uint4 w0 = slot[0 * 64 + lane], w1 = slot[1 * 64 + lane], w2 = slot[2 * 64 + lane],
                        w3 = slot[3 * 64 + lane];
            x.extra = slot[4 * 64 + lane];
            x.r = make_mul(w0.x, w0.y, w0.z, w0.w);
            x.s0 = w1.x;
            x.s1 = w1.y;
            x.s2 = w1.z;
            x.s3 = w1.w;
            x.off = ((uint64_t)w2.y << 32) | w2.x;
            x.P = w2.z;
            x.st = w2.w;
            x.n1 = w3.x;
            x.n2 = w3.y;
            x.pi = w3.z;
            x.acc = Acc{0, 0, 0, 0, 0};
        };
        auto blocks_of = [&](const PState &x, uint32_t row) -> uint32_t {
            const uint32_t nb = x.st == kWork ? x.P >> 4 : 0u, q0 = 4 * (row - 1);
            return nb > q0 ? (nb - q0 < 4 ? nb - q0 : 4u) : 0u;
        };
        auto absorb = [&](PState &x, const uint4 *slot, uint32_t row) {
            const uint32_t nblk = blocks_of(x, row);
            const uint4 m0 = slot[0 * 64 + lane], m1 = slot[1 * 64 + lane], m2 = slot[2 * 64 + lane],
                        m3 = slot[3 * 64 + lane];
            acc_block_pred(x.acc, m0, x.r, nblk > 0);
            acc_block_pred(x.acc, m1, x.r, nblk > 1);
            acc_block_pred(x.acc, m2, x.r, nblk > 2);
            acc_block_pred(x.acc, m3, x.r, nblk > 3);
        };
        // the same row of both tiles: two independent chains, interleaved
        auto absorb2 = [&](const uint4 *sa_, const uint4 *sb_, uint32_t row) {
            const uint32_t na = blocks_of(pa, row), nb = blocks_of(pb, row);
            const uint4 a0 = sa_[0 * 64 + lane], a1 = sa_[1 * 64 + lane], a2 = sa_[2 * 64 + lane],
                        a3 = sa_[3 * 64 + lane];
            const uint4 b0 = sb_[0 * 64 + lane], b1 = sb_[1 * 64 + lane], b2 = sb_[2 * 64 + lane],
                        b3 = sb_[3 * 64 + lane];
            if (__ballot(na != 4 || nb != 4) == 0) { // whole chunks everywhere (all but the last rows)
                acc_block(pa.acc, a0, pa.r);
                acc_block(pb.acc, b0, pb.r);
                acc_block(pa.acc, a1, pa.r);
                acc_block(pb.acc, b1, pb.r);
                acc_block(pa.acc, a2, pa.r);
                acc_block(pb.acc, b2, pb.r);
                acc_block(pa.acc, a3, pa.r);
                acc_block(pb.acc, b3, pb.r);
            } else {
                acc_block_pred(pa.acc, a0, pa.r, na > 0);
                acc_block_pred(pb.acc, b0, pb.r, nb > 0);
                acc_block_pred(pa.acc, a1, pa.r, na > 1);
                acc_block_pred(pb.acc, b1, pb.r, nb > 1);
                acc_block_pred(pa.acc, a2, pa.r, na > 2);
                acc_block_pred(pb.acc, b2, pb.r, nb > 2);
                acc_block_pred(pa.acc, a3, pa.r, na > 3);
                acc_block_pred(pb.acc, b3, pb.r, nb > 3);
            }
        };
        // last row of a tile: status, and for packets that went through the
        // keystream the length block, tag and frame / verdict
        auto finish = [&](PState &x) {
            if (x.st == kDead) return;
            if (x.st != kWork) {
                if constexpr (!OPEN) {
                    if (sa.status) sa.status[x.pi] = (uint8_t)x.st;
                } else {
                    oa.status[x.pi] = (uint8_t)x.st;
                    if (oa.counters_out) oa.counters_out[x.pi] = ((uint64_t)x.n2 << 32) | x.n1;
                }
            } else {
                acc_add(x.acc, 0, 0, x.P, 0, 1); // le64(aad_len = 0) || le64(P)
                acc_mul(x.acc, x.r);
                uint32_t tag[4];
                acc_finish(x.acc, x.s0, x.s1, x.s2, x.s3, tag);
                uint8_t *frame = buf + x.off;
                if constexpr (!OPEN) {
                    if (sa.receivers) *reinterpret_cast<uint4 *>(frame) = make_uint4(4u, x.extra.x, x.n1, x.n2);
                    *reinterpret_cast<uint4 *>(frame + 16 + x.P) = make_uint4(tag[0], tag[1], tag[2], tag[3]);
                    if (sa.status) sa.status[x.pi] = RG_PKT_OK;
                } else {
                    const uint32_t diff =
                        (tag[0] ^ x.extra.x) | (tag[1] ^ x.extra.y) | (tag[2] ^ x.extra.z) | (tag[3] ^ x.extra.w);
                    oa.status[x.pi] = diff ? RG_PKT_DECRYPT_ERR : RG_PKT_OK;
                    if (oa.counters_out) oa.counters_out[x.pi] = ((uint64_t)x.n2 << 32) | x.n1;
                    if (diff) {
                        const uint32_t at = atomicAdd(&fails[0], 1u);
                        if (at < kFailCap) fails[2 + at] = x.pi;
                    }
                }
            }
            x.st = kDead;
        };
        auto single = [&](PState &x, const uint4 *slot, uint32_t row) {
            if (row == 0) key_row(x, slot);
            else absorb(x, slot, row);
            if (row == cR) finish(x);
        };
        for (uint32_t k = 0; k < phases; ++k) {
            if (k > 0) {
                const uint32_t s0 = kCWaves * (k - 1), se = s0 + kCWaves < S ? s0 + kCWaves : S;
                uint32_t s = s0;
                while (s < se) {
                    seek(s);
                    const uint32_t row = (s - cstart) >> 1, half = (s - cstart) & 1u;
                    if (half == 0 && s + 1 < se) {
                        const uint4 *sa_ = slot_at(k, s - s0), *sb_ = slot_at(k, s + 1 - s0);
                        if (row == 0) {
                            key_row(pa, sa_);
                            key_row(pb, sb_);
                        } else {
                            absorb2(sa_, sb_, row);
                        }
                        if (row == cR) {
                            finish(pa);
                            finish(pb);
                        }
                        s += 2;
                    } else {
                        if (half == 0) single(pa, slot_at(k, s - s0), row);
                        else single(pb, slot_at(k, s - s0), row);
                        s += 1;
                    }
                }
            }
            lap(t_comp);
            asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
            lap(t_bar);
        }
    }

    if constexpr (OPEN) {
        // forged / corrupt packets: undo the speculative decryption once every
        // store of the workgroup has landed
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
        const uint32_t nf = fails[0];
        if (nf > 0) {
            if (nf <= kFailCap) {
                for (uint32_t x = threadIdx.x; x < nf; x += blockDim.x) restore_packet(oa, fails[2 + x]);
            } else if (wave == 0) {
                // too many to list: walk this workgroup's tiles and restore by status
                for (uint32_t j = 0; j < ntw; ++j) {
                    const uint32_t T = bid + j * G;
                    uint32_t i = 64 * T + lane;
                    bool live = i < n;
                    if constexpr (PLANNED) {
                        const uint32_t b = (uint32_t)__popcll(__ballot(B.te <= T));
                        const uint32_t tb = readlane(B.tb, b), cls = readlane(B.cls, b), cnt = readlane(B.cnt, b);
                        const uint32_t slot = (T - tb) * 64 + lane;
                        live = slot < cnt;
                        if (live) i = tp.lists[(uint64_t)cls * tp.cap + slot];
                    }
                    if (live) {
                        uint32_t stv;
                        asm volatile("global_load_ubyte %0, %1, off sc0 sc1\n\ts_waitcnt vmcnt(0)"
                                     : "=v"(stv)
                                     : "v"(oa.status + i)
                                     : "memory");
                        if (stv == RG_PKT_DECRYPT_ERR) restore_packet(oa, i);
                    }
                }
            }
        }
    }

    if (dbg && lane == 0) {
        uint64_t *o = dbg + 8 * (blockIdx.x * 8 + wave);
        o[0] = t_pro;
        o[1] = t_issue;
        o[2] = t_comp;
        o[3] = t_bar;
        o[4] = rt0; // absolute start (100 MHz)
        o[5] = wave < kCWaves ? 1 : 2;
        o[6] = 1;
        o[7] = row_realtime() - rt0;
    }
    if constexpr (PLANNED) {
        // the last workgroup to finish clears the planner counters for the next
        // batch (every workgroup read them in its prologue) and reports how many
        // size classes the batch used
        __syncthreads();
        if (threadIdx.x == 0) {
            uint32_t *ctl = const_cast<uint32_t *>(tp.counts);
            __atomic_thread_fence(__ATOMIC_SEQ_CST);
            if (atomicAdd(&ctl[kClasses], 1u) == gridDim.x - 1) {
                uint32_t used = 0;
                for (uint32_t c = 0; c < kClasses; ++c) {
                    used += ctl[c] != 0;
                    ctl[c] = 0;
                }
                ctl[kClasses] = 0;
                if (tp.classes_out) *reinterpret_cast<volatile uint32_t *>(tp.classes_out) = used;
                __atomic_thread_fence(__ATOMIC_SEQ_CST);
            }
        }
    }
}

// ---------------------------------------------------------------- launch
hipError_t launch_rows(const SealArgs *sa, const OpenArgs *oa, const TilePlan &tp, const Launch &L, hipStream_t s) {
    const uint32_t n = sa ? sa->n : oa->n;
    if (n == 0) return hipSuccess;
    SealArgs a = sa ? *sa : SealArgs{};
    OpenArgs b = oa ? *oa : OpenArgs{};
    // two 8-wave workgroups per CU; more only when a workgroup's tile table
    // would overflow (then they queue).  Planned batches have at most
    // kClasses - 1 more tiles than n / 64.
    const uint64_t tiles = ((uint64_t)n + 63) / 64 + (tp.counts ? kClasses : 0);
    uint64_t blocks = (uint64_t)(L.cus > 0 ? L.cus : 1) * (uint64_t)(L.wg_per_cu > 0 ? L.wg_per_cu : 2);
    const uint64_t need = (tiles + kRowMaxTilesWG - 1) / kRowMaxTilesWG;
    if (blocks < need) blocks = need;
    const uint64_t cap = ((uint64_t)n + 63) / 64; // every workgroup gets a tile
    if (blocks > cap) blocks = cap;
    const dim3 grid((uint32_t)blocks), block(512);
    if (tp.counts) {
        if (sa) hipLaunchKernelGGL((row_kernel<false, true>), grid, block, kRowLds, s, a, b, tp);
        else hipLaunchKernelGGL((row_kernel<true, true>), grid, block, kRowLds, s, a, b, tp);
    } else {
        if (sa) hipLaunchKernelGGL((row_kernel<false, false>), grid, block, kRowLds, s, a, b, tp);
        else hipLaunchKernelGGL((row_kernel<true, false>), grid, block, kRowLds, s, a, b, tp);
    }
    return hipGetLastError();
}

hipError_t prepare_row_kernels() {
    void *fs[4] = {(void *)row_kernel<false, false>, (void *)row_kernel<true, false>, (void *)row_kernel<false, true>,
                   (void *)row_kernel<true, true>};
    for (void *f : fs) {
        hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kRowLds);
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

} // namespace rg
