// rg_flat.hip -- the flattened chunk-stream kernel (kernel family 3): batched
// WireGuard transport seal / open for batches of mixed packet sizes.  Replaces
// N x Core::chacha20poly1305_{enc,dec} (rustyguard-crypto/src/prim.rs:179-201)
// as driven by EncryptionKey::encrypt / DecryptionKey::decrypt
// (prim.rs:386-437), with the frame layout of EncryptedMetadata::frame_in_place
// (rustyguard-core/src/lib.rs:450-470).
//
// Why: with one packet per lane a wave runs as long as its longest packet, and
// a mixed batch (IMIX: 64/576/1500-byte packets at 7:4:1) leaves most lanes of
// a 64-lane wave idle.  Here every step of every lane is one 64-byte ChaCha20
// block, whichever packet it belongs to:
//
//  * The batch is cut into units of whole packets of equal work (a one-time-key
//    block + 64-byte chunks per packet), one unit per wave, inside the kernel:
//    the four waves of a workgroup scan a 4096-packet group's lengths together
//    and cut their four units by the work midpoint rule (one wave alone scans a
//    1024-packet group when the batch does not divide into such groups), so
//    nothing is sorted, no planner launch runs and no atomics sit on the data
//    path.  The 16 workgroups of a group share an XCD (its descriptors are
//    fetched into one L2).
//  * Inside a unit (processed in sub-units of <= kFlatMaxPk packets staged in
//    LDS) phase A computes every packet's one-time-key block (RFC 8439 §2.6,
//    spread over the 64 lanes: r and s go to LDS), then phase C deals the
//    concatenated 64-byte chunks of all packets evenly over the 64 lanes: lane l
//    takes chunks [l D / 64, (l + 1) D / 64).  A lane's range may end one packet,
//    hold several small ones and start another.
//  * Poly1305 runs per piece (the part of a packet inside one lane): a piece
//    that holds the packet's last chunk publishes its Horner sum to LDS; the
//    lane's last piece, when the packet continues in the next lane, publishes
//    h * r^after (after = data blocks behind it; square-and-multiply).  Phase F
//    adds a packet's pieces, the length block and s, and writes tag and status
//    (open: compares in constant time and, for a forgery, re-applies the
//    keystream so the frame is left as it came).
//
// Memory: three 64-byte chunks in flight per lane (as rg_pipe.hip), loads
// clamped inside the frame and the stores of blocks that are not payload sent
// past the arena's buffer descriptor (dropped by the range check; arenas of
// 2 GiB or more: into a per-lane sink), so every step issues the same memory
// instructions and the vmcnt waits stay exact.
#include "rg_device.h"
#include "rg_internal.h"

namespace rg {

// floor(a / b) for a < 2^46, b > 0: a * rcp(b) in double (v_rcp_f64 is good to a few ulp, so the
// estimate is off by at most one) and one branch-free correction (a 64-bit integer division is a
// long software loop on the GPU, an IEEE double division a dozen dependent instructions)
__device__ __forceinline__ uint64_t fdiv(uint64_t a, uint64_t b) {
    uint64_t q = (uint64_t)((double)a * __builtin_amdgcn_rcp((double)b));
    q = q * b > a ? q - 1 : q;
    return (q + 1) * b <= a ? q + 1 : q;
}

// ------------------------------------------------------ frame stores
// With an arena below 2 GiB (WIN) every frame store is a buffer store through one descriptor over the
// arena, and a store that is not payload gets an offset past the descriptor's range, which the
// hardware drops (no sink traffic; config 3 +1 %, profiles/r3_sc1_ab.txt).  Larger arenas store
// through 64-bit pointers, the non-payload stores into a per-lane sink.
constexpr uint32_t kDrop = 0x80000000u;    // past num_records: dropped by the range check
struct FStore {
    uint8_t *buf;
    __amdgpu_buffer_rsrc_t rs;
    uint4 *junk;
};
template <bool WIN> __device__ __forceinline__ void fstore(const FStore &S, const uint4 *p, bool keep, uint32_t j,
                                                          const uint4 &v) {
    if constexpr (WIN) {
        const uint32_t off = keep ? (uint32_t)(reinterpret_cast<const uint8_t *>(p) - S.buf) : kDrop;
        __builtin_amdgcn_raw_buffer_store_b128(v4u{v.x, v.y, v.z, v.w}, S.rs, (int)off, 0, 0);
    } else {
        *const_cast<uint4 *>(keep ? p : S.junk + j) = v;
    }
}

// ------------------------------------------------------ unit boundaries
// Work of a packet: its one-time-key block and its 64-byte chunks (from the
// descriptor alone).
__device__ __forceinline__ uint32_t flat_work_len(uint32_t len, bool open) {
    uint32_t P = open ? (len >= 32 ? len - 32 : 0u) : len;
    if (P > kMaxPayload) P = 0;
    return 1u + (P + 63) / 64;
}
__device__ __forceinline__ uint32_t flat_work(const rg_pkt_desc &d, bool open) { return flat_work_len(d.len, open); }

// -------------------------------------------------------------- LDS image
// One per wave, one record set per packet of the sub-unit, laid out so that a
// lane moving on to the next packet issues all its LDS reads at once.
constexpr uint32_t kFlatMaxPk = 128; // packets per sub-unit (phase A holds their key loads in registers; 64 measured 15 % slower)
struct FlatLds {
    uint4 rec[kFlatMaxPk + 1];    // {offset lo, offset hi, nb | kLiveBit, cs}; rec[m].w = D
    // key[8], counter lo/hi, r[4] (unclamped), desc len, desc key_idx (a 20-dword stride halves the LDS bank
    // conflicts of phase C's key reads and changes no time: round 3, profiles/r3_lds_counters.txt)
    uint32_t kr[kFlatMaxPk][16];
    // the stream's counter-independent first column round (Stream::c1..c3), made with the one-time key in
    // phase A, so that a packet switch in phase C reads it instead of recomputing three quarter-rounds
    uint32_t hq[kFlatMaxPk][12];
    uint32_t sw[kFlatMaxPk][4];   // seal: s; open: tag - s (mod 2^128)
    uint32_t fail[kFlatMaxPk];    // kFail: the tag did not verify (open)
    unsigned long long ps[kFlatMaxPk][5]; // sum of the packet's Horner pieces, radix 2^32 limbs (LDS atomics)
    uint32_t ck[64];              // scratch: the lanes' first-packet markers
    uint32_t ch[64][5];           // scratch: the lanes' last-packet markers (stride 5)
};
constexpr uint32_t kLiveBit = 0x80000000u, kFail = 2u;
// workgroup-cooperative unit search (round 3): groups of kCoopGroup packets, work of a packet
// kCoopWPkt + kCoopWChk x chunks (a key block costs less than its share of the lanes' chunk steps:
// see flat_coop_ok and DESIGN.md §4.6)
constexpr uint32_t kCoopGroup = 4096;
constexpr uint32_t kCoopWPkt = 1, kCoopWChk = 8;
// the coop search sums work in 32 bits and doubles it for the midpoint targets; the cut counts
// compare doubled sums by the sign bit of their difference, so they stay below 2^31
static_assert(kCoopGroup * (kCoopWPkt + kCoopWChk * (kMaxPayload / 64ull + 1)) * 2 < (1ull << 31),
              "coop work sums overflow 31 bits");
constexpr uint32_t kCoopLds = 256; // shared slots: wave totals
constexpr uint32_t kFlatWaves = 4; // waves per workgroup (the coop search's four quarters), one per SIMD
// the group's work prefix, quarter by quarter (each wave writes its 1024 inclusive sums once): every wave
// reads off its own two cut points after one barrier
constexpr uint32_t kCoopPrefix = kCoopGroup * 4;
constexpr uint32_t kFlatLdsBytes = kFlatWaves * sizeof(FlatLds) + kCoopLds + kCoopPrefix;
static_assert(kFlatLdsBytes <= kLdsPerCu, "flat LDS image");


struct FChunk {
    uint4 q0, q1, q2, q3;
};

// chunk t of a packet whose last 16-byte block is `last`: four loads, indices
// clamped inside the payload (always readable).  (Streaming `nt` loads cut the
// written bytes 23 % but re-read 19 % more and ran 10 % slower: round 3.)
__device__ __forceinline__ void fload(FChunk &c, const uint4 *pl, uint32_t t, uint32_t last) {
    const uint32_t b = 4 * t;
    c.q0 = pl[min(b + 0, last)];
    c.q1 = pl[min(b + 1, last)];
    c.q2 = pl[min(b + 2, last)];
    c.q3 = pl[min(b + 3, last)];
}

// a lane's position in the sub-unit's chunk stream
struct FCur {
    uint32_t k, t, c, nb;
    bool live;
    const uint4 *pl;
};

// Every packet of the stream has at least one chunk: a packet without payload blocks (P = 0, or a
// descriptor that failed its checks) holds one chunk step whose four blocks are not payload (no Horner
// block, stores dropped) and whose loads read `safe`, so that the cursors never skip packets.
__device__ __forceinline__ uint32_t flat_chunks(uint32_t nb) { return nb ? (nb + 3) >> 2 : 1u; }

__device__ __forceinline__ void fcur_from(FCur &p, const uint4 &rc, uint8_t *buf, const uint4 *safe, uint32_t k,
                                          uint32_t t) {
    p.k = k;
    p.t = t;
    p.nb = rc.z & ~kLiveBit;
    p.live = (rc.z & kLiveBit) != 0;
    p.c = flat_chunks(p.nb);
    p.pl = p.nb ? reinterpret_cast<const uint4 *>(buf + (((uint64_t)rc.y << 32) | rc.x) + 16) : safe;
}

// next chunk; returns true when it starts a new packet (one 16-byte LDS read)
__device__ __forceinline__ bool fcur_next(FCur &p, const FlatLds &L, uint8_t *buf, const uint4 *safe, uint32_t m) {
    if (++p.t < p.c) return false;
    const uint32_t k = p.k + 1;
    const uint4 rc = L.rec[k < m ? k : m];
    if (k < m) fcur_from(p, rc, buf, safe, k, 0);
    else p.k = m; // past the sub-unit (keeps pl: loads stay readable)
    return true;
}

struct FKey {
    Key8 key;
    uint32_t n1, n2;
    uint32_t r[4];
};

__device__ __forceinline__ FKey fkey(const FlatLds &L, uint32_t k) {
    const uint4 *p = reinterpret_cast<const uint4 *>(L.kr[k]);
    const uint4 a = p[0], b = p[1], c = p[2], d = p[3];
    FKey o;
    o.key = Key8{{a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w}};
    o.n1 = c.x;
    o.n2 = c.y;
    o.r[0] = c.z; o.r[1] = c.w; o.r[2] = d.x; o.r[3] = d.y;
    return o;
}

// packet k's stream (nonce 0 || counter) from its key row and the first column round phase A left in hq
__device__ __forceinline__ Stream fstream(const FlatLds &L, uint32_t k, const FKey &q) {
    const uint4 *p = reinterpret_cast<const uint4 *>(L.hq[k]);
    const uint4 a = p[0], b = p[1], c = p[2];
    Stream st;
    st.key = q.key;
    st.n0 = 0u;
    st.n1 = q.n1;
    st.n2 = q.n2;
    st.x0p = 0x61707865u + q.key.k[0];
    st.c1[0] = a.x; st.c1[1] = a.y; st.c1[2] = a.z; st.c1[3] = a.w;
    st.c2[0] = b.x; st.c2[1] = b.y; st.c2[2] = b.z; st.c2[3] = b.w;
    st.c3[0] = c.x; st.c3[1] = c.y; st.c3[2] = c.z; st.c3[3] = c.w;
    return st;
}

// per-lane state of phase C
struct FLane {
    FCur cur, f;         // compute cursor / prefetch cursor
    uint32_t nsteps, fj; // chunks of the lane; lane-relative index of the prefetch cursor
    Stream st;
    Mul r;
    Acc h;
    FChunk pi;           // seal: ciphertext chunk waiting to be absorbed (one step behind)
    uint32_t pi_cnt, pk; // its blocks and packet
    // r^e for the carry of the lane's last piece (e = data blocks of that packet after the lane),
    // square-and-multiply from bit pb down after phase C (in the keystream rounds' free slots it cost
    // 20 %: round 2)
    Acc px;
    Mul pr;
    uint32_t pe;
    int pb;
    uint32_t rn[4]; // seal: r of the compute cursor's packet, kept from its key read for the pk switch
};

// one square-and-multiply step of the carry power (pb is wave-uniform)
__device__ __forceinline__ void pow_step(FLane &s) {
    if (s.pb < 0) return;
    Acc sq = s.px;
    acc_sqr_gen(sq);
    Acc xr = sq;
    acc_mul(xr, s.pr);
    const bool bit = (s.pe >> s.pb) & 1u;
    s.px.h0 = bit ? xr.h0 : sq.h0; s.px.h1 = bit ? xr.h1 : sq.h1; s.px.h2 = bit ? xr.h2 : sq.h2;
    s.px.h3 = bit ? xr.h3 : sq.h3; s.px.h4 = bit ? xr.h4 : sq.h4;
    --s.pb;
}

// a piece of packet k's Poly1305 sum (its final piece, or a carry h r^after of an earlier lane): the
// limbs are added into the packet's 64-bit slots by LDS atomics, so phase F reads one sum per
// packet instead of walking the lanes before it (each limb < 2^32, at most 64 pieces)
__device__ __forceinline__ void add_h(FlatLds &L, uint32_t k, const Acc &h) {
    atomicAdd(&L.ps[k][0], (unsigned long long)h.h0);
    atomicAdd(&L.ps[k][1], (unsigned long long)h.h1);
    atomicAdd(&L.ps[k][2], (unsigned long long)h.h2);
    atomicAdd(&L.ps[k][3], (unsigned long long)h.h3);
    atomicAdd(&L.ps[k][4], (unsigned long long)h.h4);
}

// One step of phase C over chunk j of the lane (in buffer b).  Seal absorbs the
// previous step's ciphertext (pi) inside this step's keystream rounds, open
// absorbs this chunk's ciphertext; the pending piece is published when the
// packet changes.  Afterwards chunk j + 3 is requested into b.
template <bool OPEN, bool WIN>
__device__ __forceinline__ void flat_step(FLane &s, FChunk &b, uint32_t j, FlatLds &L, uint8_t *buf, const FStore &FS,
                                          const uint4 *safe, uint32_t m) {
    const bool active = j < s.nsteps;
    uint32_t cnt = 0;
    if (active && s.cur.live) cnt = min(4u, s.cur.nb - 4 * s.cur.t);
    uint32_t ks[16];
    stream_block_hooked(s.st, s.cur.t + 1, ks, [&](int dr) {
        if constexpr (OPEN) {
            if (dr == 1) acc_block_pred(s.h, b.q0, s.r, cnt > 0);
            if (dr == 3) acc_block_pred(s.h, b.q1, s.r, cnt > 1);
            if (dr == 5) acc_block_pred(s.h, b.q2, s.r, cnt > 2);
            if (dr == 7) acc_block_pred(s.h, b.q3, s.r, cnt > 3);
        } else {
            if (dr == 1) acc_block_pred(s.h, s.pi.q0, s.r, s.pi_cnt > 0);
            if (dr == 3) acc_block_pred(s.h, s.pi.q1, s.r, s.pi_cnt > 1);
            if (dr == 5) acc_block_pred(s.h, s.pi.q2, s.r, s.pi_cnt > 2);
            if (dr == 7) acc_block_pred(s.h, s.pi.q3, s.r, s.pi_cnt > 3);
        }
        if (dr % 2 == 1) pin_acc(s.h);
    });
    const FChunk x = {xor4(b.q0, ks + 0), xor4(b.q1, ks + 4), xor4(b.q2, ks + 8), xor4(b.q3, ks + 12)};
    uint4 *dst = const_cast<uint4 *>(s.cur.pl) + 4 * s.cur.t;
    // (segment-whole stores -- a chunk's pieces past its 64-byte seam held one step -- cut the written bytes
    // 16 % and ran 1.3 % slower: round 3, profiles/r3_cfg3_traffic_attribution.txt)
    fstore<WIN>(FS, dst + 0, cnt > 0, 0, x.q0);
    fstore<WIN>(FS, dst + 1, cnt > 1, 1, x.q1);
    fstore<WIN>(FS, dst + 2, cnt > 2, 2, x.q2);
    fstore<WIN>(FS, dst + 3, cnt > 3, 3, x.q3);
    if constexpr (OPEN) {
        if (active && s.cur.t + 1 == s.cur.c) { // the packet's last chunk: its final piece
            if (s.cur.live) add_h(L, s.cur.k, s.h);
            s.h = Acc{0, 0, 0, 0, 0};
        }
    } else {
        if (active && s.pk != s.cur.k) { // the pending packet ended in this lane: final piece
            if (s.pk < m) add_h(L, s.pk, s.h);
            s.h = Acc{0, 0, 0, 0, 0};
            s.r = make_mul(s.rn[0], s.rn[1], s.rn[2], s.rn[3]); // r of cur.k, read at its switch
            s.pk = s.cur.k;
        }
        s.pi = x;
        s.pi_cnt = cnt;
    }
    // request chunk j + 3 of the lane into b (the same chunk again past the range)
    if (s.fj + 1 < s.nsteps) {
        ++s.fj;
        fcur_next(s.f, L, buf, safe, m);
    }
    fload(b, s.f.pl, s.f.t, s.f.nb ? s.f.nb - 1 : 0);
    if (active && fcur_next(s.cur, L, buf, safe, m) && s.cur.k < m) {
        const FKey q = fkey(L, s.cur.k);
        s.st = fstream(L, s.cur.k, q);
        if constexpr (OPEN) s.r = make_mul(q.r[0], q.r[1], q.r[2], q.r[3]);
        else {
            s.rn[0] = q.r[0]; s.rn[1] = q.r[1]; s.rn[2] = q.r[2]; s.rn[3] = q.r[3];
        }
    }
}

// ------------------------------------------------ quad key blocks
// One ChaCha20 block on a lane quad: lane j holds column j (rows a, b, c, d = state words j, 4 + j,
// 8 + j, 12 + j); the diagonal rounds rotate rows b, c, d across the quad with DPP quad_perm.  Only
// the one-time key is wanted: r_j = keystream word j, s_j = word 4 + j (RFC 8439 §2.6).
template <int CTRL> __device__ __forceinline__ uint32_t quad_perm(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xF, 0xF, false);
}
template <int CTRL> __device__ __forceinline__ uint32_t quad_bcast(uint32_t v) { return quad_perm<CTRL>(v); }
__device__ __forceinline__ void quad_qr(uint32_t &a, uint32_t &b, uint32_t &c, uint32_t &d) {
    a += b; d ^= a; d = rotl(d, 16);
    c += d; b ^= c; b = rotl(b, 12);
    a += b; d ^= a; d = rotl(d, 8);
    c += d; b ^= c; b = rotl(b, 7);
}
// kw: the packet's key-record row (key[8], counter lo, hi); block 0, nonce 0 || le64(counter).  col: column j
// after the first column round (for j >= 1 the stream's counter-independent Stream::c_j)
__device__ __forceinline__ void quad_otk(const uint32_t *kw, uint32_t j, uint32_t &r_j, uint32_t &s_j, uint4 &col) {
    const uint32_t a0 = j == 0 ? 0x61707865u : j == 1 ? 0x3320646eu : j == 2 ? 0x79622d32u : 0x6b206574u;
    const uint32_t b0 = kw[j];
    uint32_t a = a0, b = b0, c = kw[4 + j], d = j < 2 ? 0u : kw[6 + j]; // words 12, 13 = 0; 14, 15 = counter
#pragma unroll
    for (int i = 0; i < 10; ++i) {
        quad_qr(a, b, c, d); // columns
        if (i == 0) col = make_uint4(a, b, c, d);
        b = quad_perm<0x39>(b); // lane j <- j + 1
        c = quad_perm<0x4E>(c); // lane j <- j + 2
        d = quad_perm<0x93>(d); // lane j <- j + 3
        quad_qr(a, b, c, d); // diagonals
        b = quad_perm<0x93>(b);
        c = quad_perm<0x4E>(c);
        d = quad_perm<0x39>(d);
    }
    r_j = a + a0;
    s_j = b + b0;
}

struct FlatArgs {
    SealArgs sa;
    OpenArgs oa;
    uint4 *junk;     // [waves][64 lanes][4] sink of the stores that are not payload
    uint32_t units;  // = waves of the grid
    uint32_t balance; // 1: units of equal work inside each group of kFlatGroup packets; 0: equal packet counts
    uint32_t coop;    // units cut by the workgroup inside groups of kCoopGroup packets (flat_coop_ok)
    uint32_t wpkt, wchk; // coop work of a packet: wpkt + wchk x its 64-byte chunks
};

// Descriptor-level checks of a packet (the reference's order, see rg_pipe.hip):
// the status (0xFF = passes) and the 16-byte blocks of its chunk stream.
template <bool OPEN>
__device__ __forceinline__ uint32_t flat_desc_check(const rg_pkt_desc &d, uint32_t nkeys, uint64_t buf_len,
                                                    uint32_t &nb) {
    nb = 0;
    if constexpr (!OPEN) {
        const uint32_t P = d.len;
        const bool valid = d.key_idx < nkeys && (P & 15u) == 0 && (d.offset & 15u) == 0 && P <= kMaxPayload &&
                           d.offset <= buf_len && P + 32 <= buf_len - d.offset;
        if (!valid) return d.key_idx == RG_KEY_SKIP ? RG_PKT_REJECTED : RG_PKT_INVALID;
        nb = P >> 4;
        return 0xFF;
    } else {
        const uint32_t W = d.len;
        if (d.key_idx == RG_KEY_SKIP) return RG_PKT_REJECTED;
        if ((d.offset & 15u) != 0) return RG_PKT_UNALIGNED; // lib.rs:613-615
        if (d.key_idx >= nkeys || W > kMaxPayload + 32 || d.offset > buf_len || W > buf_len - d.offset || W < 4)
            return RG_PKT_INVALID;
        if (W >= 32 && (W & 15u) == 0) nb = (W - 32) >> 4;
        return 0xFF;
    }
}

// stage packet k of the sub-unit: descriptor fields into LDS (rec, len, key_idx);
// returns its chunk count
template <bool OPEN>
__device__ __forceinline__ uint32_t flat_stage(FlatLds &L, uint32_t k, const rg_pkt_desc &d, uint32_t nkeys,
                                               uint64_t buf_len) {
    uint32_t nb;
    (void)flat_desc_check<OPEN>(d, nkeys, buf_len, nb);
    L.rec[k] = make_uint4((uint32_t)d.offset, (uint32_t)(d.offset >> 32), nb, 0u);
    L.kr[k][14] = d.len;
    L.kr[k][15] = d.key_idx;
    return flat_chunks(nb);
}

template <bool OPEN, bool WIN> __global__ __launch_bounds__(64 * kFlatWaves) void flat_kernel(FlatArgs A) {
    extern __shared__ __attribute__((aligned(16))) uint8_t flat_lds[];
    const uint32_t lane = threadIdx.x & 63, wv = uniform_u32(threadIdx.x >> 6);
    FlatLds &L = reinterpret_cast<FlatLds *>(flat_lds)[wv];
    // Workgroups are dealt to the 8 XCDs round-robin (blockIdx % 8, a speed-only assumption): renumbered so
    // that consecutive workgroups -- the 16 of one cooperative-search group, which all read that group's
    // descriptors -- share one XCD and its L2 (one fabric fetch of the group's descriptors, not eight)
    const uint32_t nb = gridDim.x;
    const uint32_t lb = nb % 8u == 0 ? (blockIdx.x % 8u) * (nb / 8u) + blockIdx.x / 8u : blockIdx.x;
    const uint32_t wid = uniform_u32(lb * kFlatWaves + wv);
    const uint32_t n = OPEN ? A.oa.n : A.sa.n;
    uint8_t *const buf = OPEN ? A.oa.buf : A.sa.buf;
    const uint64_t buf_len = OPEN ? A.oa.buf_len : A.sa.buf_len;
    const uint32_t nkeys = OPEN ? A.oa.nkeys : A.sa.nkeys;
    const uint32_t *const keys = OPEN ? A.oa.keys : A.sa.keys;
    const rg_pkt_desc *const desc = OPEN ? A.oa.desc : A.sa.desc;
    uint8_t *const status = OPEN ? A.oa.status : A.sa.status;
    FStore FS;
    FS.buf = buf;
    FS.rs = __builtin_amdgcn_make_buffer_rsrc(buf, (short)0, 0x7FFFFFFF, 0x00020000);
    FS.junk = WIN ? nullptr : A.junk + ((uint64_t)wid * 64 + lane) * 4;
#if RG_DIAG
    // diagnostic builds (debug mode 3): per wave, s_memtime at the end of each phase of its first sub-unit
    const uint32_t nw = gridDim.x * kFlatWaves;
    uint64_t *const dbg = OPEN ? A.oa.dbg : A.sa.dbg;
    uint64_t mk[8] = {__builtin_amdgcn_s_memtime(), 0, 0, 0, 0, 0, 0, 0};
    const uint64_t rt0 = dbg ? __builtin_amdgcn_s_memrealtime() : 0; // 100 MHz wall clock (wave start / end)
#define RG_FLAT_MARK(slot)                                                  \
    do {                                                                    \
        if (dbg && mk[slot] == 0) mk[slot] = __builtin_amdgcn_s_memtime(); \
    } while (0)
    // the cooperative search's own steps (second block of rows, slots 2..7)
    uint64_t sk[6] = {0, 0, 0, 0, 0, 0};
    uint64_t unit_info = 0; // first sub-unit: packets m | chunks D << 16 | steps S << 40 (third block of rows)
#define RG_FLAT_SUB(slot)                                                   \
    do {                                                                    \
        if (dbg && sk[slot] == 0) sk[slot] = __builtin_amdgcn_s_memtime(); \
    } while (0)
#else
#define RG_FLAT_SUB(slot) \
    do {                  \
    } while (0)
#define RG_FLAT_MARK(slot) \
    do {                   \
    } while (0)
#endif
    // one unit per wave: launch_flat sizes the grid to exactly A.units waves (a loop over units made hipcc
    // hoist every path's setup -- the one-wave search's reciprocals among them -- in front of the coop search)
    const uint32_t NU = A.units;
    {
        const uint32_t u = wid;
        // ---- this unit's packets [s, e) and, when it is read from a group, its first sub-unit staged
        uint32_t s0, e0, staged = 0;
        if (A.coop) {
            // Round 3: the four waves of a workgroup cut their four units together, inside a group of
            // kCoopGroup (4096) packets, each wave scanning 1024 of them (16 per lane, as the one-wave
            // search does with its 1024-packet group): per-group variations of the total work are
            // then averaged over four times as many packets, and the units' chunk counts stay inside
            // six 64-lane steps at config 3.  Host-checked (flat_coop_ok): one unit per wave, the
            // group's units a multiple of four, n a multiple of kCoopGroup.
            uint32_t *const sh = reinterpret_cast<uint32_t *>(flat_lds + kFlatWaves * sizeof(FlatLds));
            const uint32_t kgc = uniform_u32(A.coop);               // units per group
            const uint32_t g = uniform_u32(u / kgc), j = uniform_u32(u - g * kgc);
            const uint32_t gb = g * kCoopGroup + wv * kFlatGroup;    // this wave's 1024 packets
            RG_FLAT_SUB(0);
            // the lengths only (the work needs nothing else), as buffer loads at this lane's offset plus a
            // scalar offset per row: all 16 issue back to back, with no 64-bit address arithmetic in front
            // of them (the ILP schedule had put ~80 address instructions before the first load)
            const __amdgpu_buffer_rsrc_t drs = __builtin_amdgcn_make_buffer_rsrc(
                const_cast<rg_pkt_desc *>(desc + gb), (short)0, (int)(kFlatGroup * sizeof(rg_pkt_desc)), 0x00020000);
            uint32_t ln[16];
#pragma unroll
            for (int q = 0; q < 16; ++q)
                ln[q] = __builtin_amdgcn_raw_buffer_load_b32(drs, (int)(sizeof(rg_pkt_desc) * lane + offsetof(rg_pkt_desc, len)),
                                                              (int)(sizeof(rg_pkt_desc) * 64 * q), 0);
            uint32_t *const tw = &L.kr[0][0];
#pragma unroll
            for (int q = 0; q < 16; ++q) tw[lane + 64 * q] = A.wpkt + A.wchk * (flat_work_len(ln[q], OPEN) - 1u);
            wave_sync();
            uint32_t e[16];
            {
                const uint4 *t4 = reinterpret_cast<const uint4 *>(tw) + 4 * lane;
                const uint4 a0 = t4[0], a1 = t4[1], a2 = t4[2], a3 = t4[3];
                e[0] = a0.x; e[1] = a0.y; e[2] = a0.z; e[3] = a0.w;
                e[4] = a1.x; e[5] = a1.y; e[6] = a1.z; e[7] = a1.w;
                e[8] = a2.x; e[9] = a2.y; e[10] = a2.z; e[11] = a2.w;
                e[12] = a3.x; e[13] = a3.y; e[14] = a3.z; e[15] = a3.w;
            }
            wave_sync();
            RG_FLAT_SUB(1);
#pragma unroll
            for (int q = 1; q < 16; ++q) e[q] += e[q - 1];
            const uint32_t lsum = e[15];
            const uint32_t lx = wave_scan_incl(lsum) - lsum;
#pragma unroll
            for (int q = 0; q < 16; ++q) e[q] += lx;
            // the quarter's inclusive work prefix (packet 16 lane + q) for every wave of the workgroup
            uint32_t *const pf_all = sh + kCoopLds / 4;
            {
                uint4 *p4 = reinterpret_cast<uint4 *>(pf_all + kFlatGroup * wv) + 4 * lane;
                p4[0] = make_uint4(e[0], e[1], e[2], e[3]);
                p4[1] = make_uint4(e[4], e[5], e[6], e[7]);
                p4[2] = make_uint4(e[8], e[9], e[10], e[11]);
                p4[3] = make_uint4(e[12], e[13], e[14], e[15]);
            }
            if (lane == 0) sh[wv] = lane63(lx + lsum); // this wave's total
            RG_FLAT_SUB(2);
            __syncthreads();
            RG_FLAT_SUB(3);
            uint32_t qt[kFlatWaves], tot = 0; // the quarters' totals; the group's
#pragma unroll
            for (uint32_t w = 0; w < kFlatWaves; ++w) {
                qt[w] = uniform_u32(sh[w]);
                tot += qt[w];
            }
            // This unit's two cut points (midpoint rule: packet i goes to the unit its work midpoint falls
            // in), each wave its own: targets 2 tot j / kgc and 2 tot (j + 1) / kgc.  Any rounding is fine as
            // long as every workgroup of the group computes the same function of (tot, boundary index) --
            // they do, so a boundary shared by two workgroups lands on the same packet in both.
            // A cut = the packets of the quarters wholly below the target + the count inside the quarter
            // holding it.  Midpoints rise strictly with the packet index (every packet has work >= 1), so in
            // that quarter the 16-packet rows whose last midpoint lies below the target are a prefix (one
            // ballot), and the next row's count is a second ballot.  Sums stay below 2^31 (static_assert
            // above), so (m - t) >> 31 is m < t without a carry flag (no SGPR hazard nops).
            uint32_t cut0, cut1;
            {
                const double per = (double)tot * __builtin_amdgcn_rcp((double)kgc);
                uint32_t T[2], base[2], qw[2];
#pragma unroll
                for (int b = 0; b < 2; ++b) {
                    T[b] = uniform_u32(2 * (uint32_t)(per * (double)(j + b)));
                    // the quarter w with 2 off_w < T <= 2 (off_w + qt_w) (none: T = 0, or T past the group)
                    uint32_t off = 0, w_ = kFlatWaves, lo = 0;
#pragma unroll
                    for (uint32_t w = 0; w < kFlatWaves; ++w) {
                        if (w_ == kFlatWaves && T[b] <= 2 * (off + qt[w])) {
                            w_ = w;
                            lo = 2 * off;
                        }
                        off += qt[w];
                    }
                    qw[b] = uniform_u32(w_);
                    base[b] = uniform_u32(lo);
                }
                uint32_t full[2];
#pragma unroll
                for (int b = 0; b < 2; ++b) {
                    const uint32_t *pf = pf_all + kFlatGroup * (qw[b] < kFlatWaves ? qw[b] : 0u);
                    const uint32_t a = pf[16 * lane + 15], c = pf[16 * lane + 14];
                    full[b] = (uint32_t)__popcll(__ballot(((a + c + base[b] - T[b]) >> 31) != 0));
                }
                uint32_t cnt[2];
#pragma unroll
                for (int b = 0; b < 2; ++b) {
                    const uint32_t *pf = pf_all + kFlatGroup * (qw[b] < kFlatWaves ? qw[b] : 0u);
                    const uint32_t row = full[b] < 64 ? full[b] : 63u, q = lane & 15u;
                    const uint32_t i = 16 * row + q;
                    const uint32_t cur = pf[i], prv = i ? pf[i - 1] : 0u;
                    const uint32_t in = (uint32_t)__popcll(__ballot(lane < 16 && ((cur + prv + base[b] - T[b]) >> 31) != 0));
                    cnt[b] = qw[b] >= kFlatWaves ? kCoopGroup : kFlatGroup * qw[b] + 16u * full[b] + (full[b] < 64 ? in : 0u);
                }
                cut0 = j == 0 ? 0u : cnt[0];
                cut1 = j + 1 == kgc ? kCoopGroup : cnt[1];
            }
            RG_FLAT_SUB(4);
            RG_FLAT_SUB(5);
            // (no barrier after these reads: one unit per wave, so no wave writes the shared slots or the
            // prefix again)
            // the first sub-unit is staged from memory below (L2-resident: this workgroup just read it);
            // staging it from the four waves' registers into each other's images measured 2x slower
            s0 = g * kCoopGroup + cut0;
            e0 = g * kCoopGroup + cut1;
            wave_sync(); // the key-record scratch is read before the sub-unit is staged into it
        } else if ((uint64_t)n <= (uint64_t)kFlatGroup * NU) {
            // Units of group g (kFlatGroup packets): those whose nominal start u n / NU falls in it;
            // inside the group the cut points split its work evenly (midpoint rule).  No global
            // pass: the wave reads the group's descriptors (16 per lane) and scans them itself.
            // (wave-uniform values, pinned to scalar registers so that every test on them below is a
            // scalar branch rather than an exec-masked one)
            uint32_t g, f0, f1;
            if (NU <= 1024u) { // every operand below 2^31 (n <= 2^10 NU): 32-bit divisions
                const uint32_t gu = kFlatGroup * NU;
                g = uniform_u32(u * n / gu);
                f0 = uniform_u32((g * gu + n - 1) / n);
                f1 = uniform_u32(min(NU, ((g + 1) * gu + n - 1) / n));
            } else {
                g = uniform_u32((uint32_t)fdiv((uint64_t)u * n, (uint64_t)NU * kFlatGroup));
                f0 = uniform_u32((uint32_t)fdiv((uint64_t)g * kFlatGroup * NU + n - 1, n));
                f1 = uniform_u32((uint32_t)min((uint64_t)NU, fdiv(((uint64_t)g + 1) * kFlatGroup * NU + n - 1, n)));
            }
            const uint32_t kg = f1 - f0, j = u - f0;
            const uint32_t gb = g * kFlatGroup, gn = min(kFlatGroup, n - gb);
            // coalesced: lane l holds packets l + 64 q of the group (q = 0..15)
            rg_pkt_desc d[16];
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                const uint32_t i = lane + 64 * q;
                d[q] = desc[gb + (i < gn ? i : 0)];
            }
            // The work prefix in packet order, lane-contiguous: the per-packet work goes through LDS
            // (the key-record area, written only later) from the coalesced order (lane + 64 q) to
            // lane l holding packets 16 l .. 16 l + 15; each lane sums its 16 serially and one DPP
            // wave scan of the lane totals places them (one scan instead of one per round).  Group
            // totals stay below 2^24 (1024 packets of at most 16386 blocks), so 32 bits suffice.
            uint32_t *const tw = &L.kr[0][0];
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                const uint32_t i = lane + 64 * q;
                tw[i] = i < gn ? (A.balance ? flat_work(d[q], OPEN) : 1u) : 0u;
            }
            wave_sync();
            uint32_t e[16];
            {
                const uint4 *t4 = reinterpret_cast<const uint4 *>(tw) + 4 * lane;
                const uint4 a0 = t4[0], a1 = t4[1], a2 = t4[2], a3 = t4[3];
                e[0] = a0.x; e[1] = a0.y; e[2] = a0.z; e[3] = a0.w;
                e[4] = a1.x; e[5] = a1.y; e[6] = a1.z; e[7] = a1.w;
                e[8] = a2.x; e[9] = a2.y; e[10] = a2.z; e[11] = a2.w;
                e[12] = a3.x; e[13] = a3.y; e[14] = a3.z; e[15] = a3.w;
            }
            wave_sync(); // the reads are done before anything rewrites the area
#pragma unroll
            for (int q = 1; q < 16; ++q) e[q] += e[q - 1];
            const uint32_t lsum = e[15];
            const uint32_t lx = wave_scan_incl(lsum) - lsum; // work of the lanes before this one
#pragma unroll
            for (int q = 0; q < 16; ++q) e[q] += lx; // E_i, inclusive, of packet 16 lane + q
            const uint32_t total = lane63(lx + lsum);
            // targets j total / kg and (j + 1) total / kg without a 64-bit division
            const uint32_t t2[2] = {uniform_u32(2 * (uint32_t)fdiv((uint64_t)total * j, kg)),
                                    uniform_u32(2 * (uint32_t)fdiv((uint64_t)total * (j + 1), kg))};
            // a packet belongs to the unit its work midpoint (E_{i-1} + E_i) / 2 falls in; the midpoints
            // rise with i, so a cut is the number of packets whose midpoint lies below the target
            uint32_t c0 = 0, c1 = 0;
            {
                const uint32_t sh = wave_shr1(e[15]);
                uint32_t prev = lane ? sh : 0u; // E of the packet before 16 lane
#pragma unroll
                for (int q = 0; q < 16; ++q) {
                    const uint32_t i = 16 * lane + q;
                    const uint32_t mid2 = e[q] + prev;
                    prev = e[q];
                    c0 += (i < gn && mid2 < t2[0]) ? 1u : 0u;
                    c1 += (i < gn && mid2 < t2[1]) ? 1u : 0u;
                }
            }
            uint32_t cut[2] = {lane63(wave_scan_incl(c0)), lane63(wave_scan_incl(c1))};
            if (j == 0) cut[0] = 0;
            if (j + 1 == kg) cut[1] = gn;
            s0 = gb + cut[0];
            e0 = gb + cut[1];
            // stage the first sub-unit straight from the registers
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                if (64u * q + 63 < cut[0] || 64u * q >= min(cut[1], cut[0] + kFlatMaxPk)) continue; // uniform
                const uint32_t i = lane + 64 * q;
                if (i >= cut[0] && i < cut[1] && i - cut[0] < kFlatMaxPk) flat_stage<OPEN>(L, i - cut[0], d[q], nkeys, buf_len);
            }
            staged = 1;
        } else { // more than kFlatGroup packets per unit: whole groups
            const uint32_t G = (n + kFlatGroup - 1) / kFlatGroup;
            s0 = (uint32_t)min((uint64_t)n, fdiv((uint64_t)u * G, NU) * kFlatGroup);
            e0 = (uint32_t)min((uint64_t)n, fdiv((uint64_t)(u + 1) * G, NU) * kFlatGroup);
        }
        RG_FLAT_MARK(1);
        for (uint32_t sb = s0; sb < e0; sb += kFlatMaxPk) {
            const uint32_t m = min(kFlatMaxPk, e0 - sb);
            // ---- phase A loads, issued first so that their latency hides behind the chunk-count scan
            // and the range search (and ahead of the chunk prefetch, so that their waits stay exact)
            uint8_t dst[kFlatMaxPk / 64]; // statuses of the descriptor checks, kept for phase A
            uint4 ka[kFlatMaxPk / 64], kb[kFlatMaxPk / 64], hx[kFlatMaxPk / 64], tg[kFlatMaxPk / 64];
            uint32_t rcv[kFlatMaxPk / 64], dlen[kFlatMaxPk / 64], dkey[kFlatMaxPk / 64];
            uint64_t doff[kFlatMaxPk / 64], ctr[kFlatMaxPk / 64];
            // ---- stage (unless done above): packet k = lane + 64 q is read by the lane that works on it in
            // phase A, so its fields stay in registers (no LDS round trip before the key loads), and a
            // seal's counters are requested together with the descriptors
            if (!staged) {
#pragma unroll
                for (uint32_t q = 0; q < kFlatMaxPk / 64; ++q) {
                    const uint32_t k = lane + 64 * q;
                    if (64 * q >= m) break; // wave-uniform
                    const uint32_t i = sb + (k < m ? k : 0u);
                    const rg_pkt_desc d = desc[i];
                    if constexpr (!OPEN) ctr[q] = A.sa.counters[i];
                    if (k < m) flat_stage<OPEN>(L, k, d, nkeys, buf_len);
                    dlen[q] = d.len;
                    dkey[q] = d.key_idx;
                    doff[q] = d.offset;
                }
            } else {
                wave_sync(); // staged by the one-wave search (another lane mapping): read back
#pragma unroll
                for (uint32_t q = 0; q < kFlatMaxPk / 64; ++q) {
                    const uint32_t k = lane + 64 * q;
                    if (64 * q >= m) break; // wave-uniform
                    const uint4 rc = L.rec[k < m ? k : 0];
                    dlen[q] = L.kr[k < m ? k : 0][14];
                    dkey[q] = L.kr[k < m ? k : 0][15];
                    doff[q] = ((uint64_t)rc.y << 32) | rc.x;
                    if constexpr (!OPEN) ctr[q] = A.sa.counters[sb + (k < m ? k : 0u)];
                }
            }
            staged = 0;
            // the descriptor checks again, from the staged fields (VALU only)
#pragma unroll
            for (uint32_t q = 0; q < kFlatMaxPk / 64; ++q) {
                if (64 * q >= m) break;
                uint32_t nbx;
                const rg_pkt_desc dd = {doff[q], dlen[q], dkey[q]};
                dst[q] = (uint8_t)flat_desc_check<OPEN>(dd, nkeys, buf_len, nbx);
            }
#pragma unroll
            for (uint32_t q = 0; q < kFlatMaxPk / 64; ++q) {
                const uint32_t k = lane + 64 * q;
                if (64 * q >= m) break; // wave-uniform
                const bool ok = k < m && dst[q] == 0xFF;
                const uint4 *kp = reinterpret_cast<const uint4 *>(keys + 8ull * (ok ? dkey[q] : 0u));
                ka[q] = kp[0];
                kb[q] = kp[1];
                const uint4 *safe = reinterpret_cast<const uint4 *>(desc + sb);
                if constexpr (!OPEN) {
                    const uint64_t c = ctr[q];
                    hx[q] = make_uint4((uint32_t)c, (uint32_t)(c >> 32), 0, 0);
                    rcv[q] = A.sa.receivers ? A.sa.receivers[ok ? dkey[q] : 0u] : 0u;
                    tg[q] = make_uint4(0, 0, 0, 0);
                } else {
                    const bool go = ok && dlen[q] >= 32 && (dlen[q] & 15u) == 0; // has a tag (P >= 0)
                    const uint8_t *fr = buf + doff[q];
                    // the header as a 16-byte vector when the arena holds 16 bytes there; the type word
                    // alone otherwise (a frame of 4..15 bytes at the very end of the arena)
                    const bool room = ok && buf_len - doff[q] >= 16;
                    hx[q] = *(room ? reinterpret_cast<const uint4 *>(fr) : safe);
                    rcv[q] = *(ok ? reinterpret_cast<const uint32_t *>(fr) : reinterpret_cast<const uint32_t *>(safe));
                    tg[q] = *(go ? reinterpret_cast<const uint4 *>(fr + dlen[q] - 16) : safe);
                }
            }
            uint32_t run = 0;
            uint32_t csr[kFlatMaxPk / 64]; // chunk start of packet lane + 64 q
#pragma unroll
            for (uint32_t q = 0; q < kFlatMaxPk / 64; ++q) {
                csr[q] = 0xFFFFFFFFu;
                if (64 * q >= m) break; // wave-uniform
                const uint32_t k = lane + 64 * q;
                const uint32_t c = k < m ? flat_chunks(L.rec[k].z) : 0u;
                const uint32_t x = wave_scan_incl(c);
                if (k < m) L.rec[k].w = csr[q] = run + x - c;
                run += lane63(x);
            }
            const uint32_t D = run;
            // The lane's first packet kstart = last k with cs[k] <= c_lo(lane) and, with chunks, its last
            // packet kend = last k with cs[k] < c_hi(lane), c_lo(l) = floor(l D / 64) = c_hi(l - 1):
            // packet k qualifies for every lane from ceil(64 cs[k] / D) (resp. ceil(64 (cs[k] + 1) / D) - 1)
            // on, so each packet marks that lane (LDS max) and a running max over the lanes reads off
            // the answer -- no dependent LDS search per lane.  The carry slots serve as scratch here.
            uint32_t *const mk_lo = &L.ck[0];
            uint32_t *const mk_hi = &L.ch[0][0];
            mk_lo[lane] = 0u;
            mk_hi[5 * lane] = 0u;
            wave_sync();
            if (D) {
                const double rD = __builtin_amdgcn_rcp((double)D);
                auto fl = [&](uint32_t a) -> uint32_t { // floor(a / D), a < 2^31: estimate, then exact
                    uint32_t t = (uint32_t)((double)a * rD);
                    t = (uint64_t)t * D > a ? t - 1 : t;
                    return (uint64_t)(t + 1) * D <= a ? t + 1 : t;
                };
#pragma unroll
                for (uint32_t q = 0; q < kFlatMaxPk / 64; ++q) {
                    if (64 * q >= m) break; // wave-uniform
                    const uint32_t k = lane + 64 * q;
                    if (k >= m) continue;
                    const uint32_t l0 = fl(64 * csr[q] + D - 1);
                    const uint32_t l1 = fl(64 * (csr[q] + 1) + D - 1) - 1;
                    if (l0 < 64) atomicMax(&mk_lo[l0], k);
                    if (l1 < 64) atomicMax(&mk_hi[5 * l1], k);
                }
            }
            wave_sync();
            const uint32_t kstart_scan = wave_scan_max(mk_lo[lane]);
            const uint32_t kend_scan = wave_scan_max(mk_hi[5 * lane]);
            wave_sync(); // the scratch reads are done before the slots are used again
            if (lane == 0) L.rec[m] = make_uint4(0, 0, 0, D);
            RG_FLAT_MARK(2);
#if RG_DIAG
            if (dbg && unit_info == 0) unit_info = (uint64_t)m | ((uint64_t)D << 16) | ((uint64_t)((D + 63) / 64) << 40);
#endif
            // ---- the lane's chunk range and start packet
            const uint32_t c_lo = (uint32_t)(((uint64_t)lane * D) >> 6), c_hi = (uint32_t)(((uint64_t)(lane + 1) * D) >> 6);
            FLane s;
            s.nsteps = c_hi - c_lo;
            const uint32_t kstart = D ? kstart_scan : m - 1;
            // ---- the lane's first three chunks
            FChunk b0, b1, b2;
            const uint4 *const safe = reinterpret_cast<const uint4 *>(desc + sb); // 16 readable bytes
            if (s.nsteps) {
                fcur_from(s.cur, L.rec[kstart], buf, safe, kstart, c_lo - L.rec[kstart].w);
            } else { // no chunks: a readable dummy position
                s.cur.k = m; s.cur.t = 0; s.cur.c = 0; s.cur.nb = 1; s.cur.live = false;
                s.cur.pl = safe;
            }
            s.f = s.cur;
            s.fj = 0;
            fload(b0, s.f.pl, s.f.t, s.f.nb ? s.f.nb - 1 : 0);
            if (s.fj + 1 < s.nsteps) { ++s.fj; fcur_next(s.f, L, buf, safe, m); }
            fload(b1, s.f.pl, s.f.t, s.f.nb ? s.f.nb - 1 : 0);
            if (s.fj + 1 < s.nsteps) { ++s.fj; fcur_next(s.f, L, buf, safe, m); }
            fload(b2, s.f.pl, s.f.t, s.f.nb ? s.f.nb - 1 : 0);
            // ---- phase A: checks, one-time-key blocks, header (seal), counters_out (open)
            // Packets 64.. of a sub-unit of 65-96 get their key blocks from lane quads (16 blocks per
            // pass at ~0.36 of a full pass) instead of a second one-lane-per-packet pass.
            const bool quad = m > 64 && m <= 96; // wave-uniform
#pragma unroll
            for (uint32_t q = 0; q < kFlatMaxPk / 64; ++q) {
                const uint32_t k = lane + 64 * q;
                if (64 * q >= m) break;
                if (k >= m) continue;
                const uint32_t i = sb + k;
                uint8_t st = dst[q];
                uint32_t n1 = hx[q].x, n2 = hx[q].y; // seal: the counter
                if constexpr (OPEN) {
                    const uint32_t W = dlen[q];
                    n1 = n2 = 0;
                    if (st == 0xFF) {
                        const uint32_t type = rcv[q];
                        if (type != 4u) st = type - 1u < 3u ? RG_PKT_NOT_DATA : RG_PKT_INVALID;    // lib.rs:621-628
                        else if ((W & 15u) != 0 || W < 16) st = RG_PKT_INVALID;                   // types/lib.rs:181-196
                        else {
                            n1 = hx[q].z;
                            n2 = hx[q].w;
                            if (W < 32) st = RG_PKT_DECRYPT_ERR;                                  // prim.rs:427-429
                        }
                    }
                    if (A.oa.counters_out) A.oa.counters_out[i] = ((uint64_t)n2 << 32) | n1;
                }
                uint4 *kr = reinterpret_cast<uint4 *>(L.kr[k]);
                kr[0] = ka[q];
                kr[1] = kb[q];
                if (q == 1 && quad) {
                    // overflow packet: its one-time-key block is computed by a lane quad below
                    L.kr[k][8] = n1;
                    L.kr[k][9] = n2;
                    if constexpr (OPEN) *reinterpret_cast<uint4 *>(L.sw[k]) = tg[q]; // the tag; s is subtracted there
                } else {
                const Key8 key = {{ka[q].x, ka[q].y, ka[q].z, ka[q].w, kb[q].x, kb[q].y, kb[q].z, kb[q].w}};
                const Stream stm = make_stream(key, 0u, n1, n2); // nonce 0 || le64(counter), prim.rs:32-36
                uint32_t ks[16];
                stream_block(stm, 0, ks); // RFC 8439 §2.6 one-time key
                uint4 *hq = reinterpret_cast<uint4 *>(L.hq[k]);
                hq[0] = make_uint4(stm.c1[0], stm.c1[1], stm.c1[2], stm.c1[3]);
                hq[1] = make_uint4(stm.c2[0], stm.c2[1], stm.c2[2], stm.c2[3]);
                hq[2] = make_uint4(stm.c3[0], stm.c3[1], stm.c3[2], stm.c3[3]);
                kr[2] = make_uint4(n1, n2, ks[0], ks[1]);
                L.kr[k][12] = ks[2];
                L.kr[k][13] = ks[3];
                if constexpr (OPEN) { // tag - s (mod 2^128): phase F compares (h mod p) with it
                    uint32_t c0, w0, w1, w2, w3;
                    w0 = __builtin_subc(tg[q].x, ks[4], 0u, &c0);
                    w1 = __builtin_subc(tg[q].y, ks[5], c0, &c0);
                    w2 = __builtin_subc(tg[q].z, ks[6], c0, &c0);
                    w3 = __builtin_subc(tg[q].w, ks[7], c0, &c0);
                    *reinterpret_cast<uint4 *>(L.sw[k]) = make_uint4(w0, w1, w2, w3);
                } else {
                    *reinterpret_cast<uint4 *>(L.sw[k]) = make_uint4(ks[4], ks[5], ks[6], ks[7]);
                }
                }
                {
                    unsigned long long *z = L.ps[k];
                    z[0] = z[1] = z[2] = z[3] = z[4] = 0ull;
                    L.fail[k] = 0u;
                }
                if (st == 0xFF) {
                    L.rec[k].z |= kLiveBit;
                    if constexpr (!OPEN) {
                        // DataHeader {4, receiver, counter} (rustyguard-core/src/lib.rs:286-290)
                        if (A.sa.receivers)
                            fstore<WIN>(FS, reinterpret_cast<const uint4 *>(buf + doff[q]), true, 0, make_uint4(4u, rcv[q], n1, n2));
                    }
                } else if (status) {
                    status[i] = st;
                }
            }
            wave_sync();
            if (quad) { // the overflow packets' one-time keys: 16 per wave instruction stream (lane quads)
                for (uint32_t p0 = 64; p0 < m; p0 += 16) {
                    const uint32_t k = p0 + (lane >> 2), j = lane & 3u;
                    const uint32_t kk = k < m ? k : p0;
                    uint32_t r_j, s_j;
                    uint4 col;
                    quad_otk(L.kr[kk], j, r_j, s_j, col);
                    if constexpr (OPEN) {
                        // tag - s (mod 2^128) needs all four words of s in every lane of the quad
                        const uint32_t s0 = quad_bcast<0x00>(s_j), s1 = quad_bcast<0x55>(s_j);
                        const uint32_t s2 = quad_bcast<0xAA>(s_j), s3 = quad_bcast<0xFF>(s_j);
                        const uint4 t = *reinterpret_cast<const uint4 *>(L.sw[kk]);
                        uint32_t c0, w[4];
                        w[0] = __builtin_subc(t.x, s0, 0u, &c0);
                        w[1] = __builtin_subc(t.y, s1, c0, &c0);
                        w[2] = __builtin_subc(t.z, s2, c0, &c0);
                        w[3] = __builtin_subc(t.w, s3, c0, &c0);
                        s_j = j == 0 ? w[0] : j == 1 ? w[1] : j == 2 ? w[2] : w[3];
                    }
                    wave_sync(); // every quad has read its row before any lane writes one
                    if (k < m) {
                        L.kr[k][10 + j] = r_j;
                        L.sw[k][j] = s_j;
                        if (j) reinterpret_cast<uint4 *>(L.hq[k])[j - 1] = col;
                    }
                }
                wave_sync();
            }
            RG_FLAT_MARK(3);
            // ---- phase C: the chunk stream
            const uint32_t S = (D + 63) / 64;
            if (s.cur.k < m) {
                s.cur.live = (L.rec[s.cur.k].z & kLiveBit) != 0;
                s.f.live = s.cur.live;
                const FKey q = fkey(L, s.cur.k);
                s.st = fstream(L, s.cur.k, q);
                s.r = make_mul(q.r[0], q.r[1], q.r[2], q.r[3]);
                s.rn[0] = q.r[0]; s.rn[1] = q.r[1]; s.rn[2] = q.r[2]; s.rn[3] = q.r[3];
            } else {
                s.st = make_stream(Key8{{0, 0, 0, 0, 0, 0, 0, 0}}, 0u, 0u, 0u);
                s.r = make_mul(0, 0, 0, 0);
                s.rn[0] = s.rn[1] = s.rn[2] = s.rn[3] = 0;
            }
            s.h = Acc{0, 0, 0, 0, 0};
            s.pi = FChunk{};
            s.pi_cnt = 0;
            s.pk = s.cur.k;
            // the carry's power: the packet of the lane's last chunk, when it goes on past the lane
            {
                s.pe = 0;
                uint32_t kend = 0;
                if (s.nsteps) {
                    kend = kend_scan;
                    const uint4 rc = L.rec[kend];
                    const uint32_t nbe = rc.z & ~kLiveBit, tend = c_hi - rc.w; // chunks of kend through the lane
                    if (4 * tend < nbe) s.pe = nbe - 4 * tend;
                }
                const FKey q = fkey(L, kend);
                s.pr = make_mul(q.r[0], q.r[1], q.r[2], q.r[3]);
                s.px = Acc{1, 0, 0, 0, 0};
                uint32_t mx = s.pe;
#pragma unroll
                for (int o = 32; o >= 1; o >>= 1) mx = max(mx, (uint32_t)__shfl_xor((int)mx, o));
                s.pb = 31 - (int)__clz((int)uniform_u32(mx)); // -1 when no lane has a carry
                if (mx == 0) s.pb = -1;
            }
            {
                uint32_t j = 0;
                for (; j + 3 <= S; j += 3) {
                    flat_step<OPEN, WIN>(s, b0, j, L, buf, FS, safe, m);
                    flat_step<OPEN, WIN>(s, b1, j + 1, L, buf, FS, safe, m);
                    flat_step<OPEN, WIN>(s, b2, j + 2, L, buf, FS, safe, m);
                }
                if (j < S) flat_step<OPEN, WIN>(s, b0, j, L, buf, FS, safe, m);
                if (j + 1 < S) flat_step<OPEN, WIN>(s, b1, j + 1, L, buf, FS, safe, m);
            }
            RG_FLAT_MARK(4);
            uint32_t ck = ~0u; // the packet whose Horner sum the next lane continues (its power is s.px)
            if constexpr (!OPEN) { // the last ciphertext chunk
                // (interleaving these four blocks with the first carry-power steps, independent chains in one
                // basic block, measured no faster: round 4)
                acc_block_pred(s.h, s.pi.q0, s.r, s.pi_cnt > 0);
                acc_block_pred(s.h, s.pi.q1, s.r, s.pi_cnt > 1);
                acc_block_pred(s.h, s.pi.q2, s.r, s.pi_cnt > 2);
                acc_block_pred(s.h, s.pi.q3, s.r, s.pi_cnt > 3);
                if (s.nsteps > 0 && s.pk < m) {
                    if (s.cur.k == s.pk && s.cur.t > 0) { // the packet goes on in the next lane
                        ck = s.pk;
                    } else {
                        add_h(L, s.pk, s.h);
                    }
                }
            } else {
                if (s.nsteps > 0 && s.cur.k < m && s.cur.t > 0) {
                    ck = s.cur.k;
                }
            }
            // carry = h r^pe for the packet the next lane continues (pe: its blocks after this lane's range,
            // from the end markers before phase C; square-and-multiply over the wave's largest exponent)
            if (s.pb >= 0) { // the top bit: x = 1 squared is 1, so the first step is a choice of 1 or r
                const bool bit = (s.pe >> s.pb) & 1u;
                s.px = bit ? Acc{s.pr.r0, s.pr.r1, s.pr.r2, s.pr.r3, 0} : Acc{1, 0, 0, 0, 0};
                --s.pb;
            }
            while (s.pb >= 0) pow_step(s);
            if (ck != ~0u) {
                Acc cv = s.h;
                acc_mul_gen(cv, make_gen(s.px));
                add_h(L, ck, cv);
            }
            wave_sync();
            RG_FLAT_MARK(5);
            // ---- phase F: tags
            bool any_fail = false;
            for (uint32_t k = lane; k < m; k += 64) {
                const uint4 rc = L.rec[k];
                const unsigned long long *ps = L.ps[k];
                const unsigned long long p0 = ps[0], p1 = ps[1], p2 = ps[2], p3 = ps[3], p4 = ps[4];
                const uint4 swk = *reinterpret_cast<const uint4 *>(L.sw[k]);
                const uint4 r03 = make_uint4(L.kr[k][10], L.kr[k][11], L.kr[k][12], L.kr[k][13]);
                if (!(rc.z & kLiveBit)) continue;
                // the sum of the packet's pieces, carried into 32-bit limbs and partially reduced
                Acc h;
                unsigned long long t = p0;
                h.h0 = (uint32_t)t;
                t = (t >> 32) + p1;
                h.h1 = (uint32_t)t;
                t = (t >> 32) + p2;
                h.h2 = (uint32_t)t;
                t = (t >> 32) + p3;
                h.h3 = (uint32_t)t;
                h.h4 = (uint32_t)((t >> 32) + p4);
                acc_fold(h);
                const uint32_t P = (rc.z & ~kLiveBit) * 16;
                const Mul r = make_mul(r03.x, r03.y, r03.z, r03.w);
                acc_add(h, 0, 0, P, 0, 1); // le64(aad_len = 0) || le64(P), RFC 8439 §2.8
                acc_mul(h, r);
                const uint32_t i = sb + k;
                uint32_t tag[4];
                if constexpr (!OPEN) {
                    acc_finish(h, swk.x, swk.y, swk.z, swk.w, tag);
                    fstore<WIN>(FS, reinterpret_cast<const uint4 *>(buf + (((uint64_t)rc.y << 32) | rc.x) + 16 + P), true, 0,
                                make_uint4(tag[0], tag[1], tag[2], tag[3]));
                    if (status) status[i] = RG_PKT_OK;
                } else {
                    acc_finish(h, 0, 0, 0, 0, tag);
                    const uint32_t diff = (tag[0] ^ swk.x) | (tag[1] ^ swk.y) | (tag[2] ^ swk.z) | (tag[3] ^ swk.w);
                    status[i] = diff == 0 ? RG_PKT_OK : RG_PKT_DECRYPT_ERR;
                    if (diff != 0) {
                        L.fail[k] = kFail;
                        any_fail = true;
                    }
                }
            }
            RG_FLAT_MARK(6);
            if constexpr (OPEN) {
                // ---- forgeries: put the ciphertext back (plaintext ^ keystream), the forged packets'
                // chunks dealt over the wave's 64 lanes (as restore_forged, rg_device.h): a wave pays
                // ~chunks / 64 keystream blocks per forged packet, not the slowest lane's whole range.
                // Every byte involved was stored by this wave (in-order: wavefront-scope ordering).
                if (__ballot(any_fail)) {
                    wave_sync();
                    uint32_t cn[kFlatMaxPk / 64];
                    uint64_t fmask[kFlatMaxPk / 64];
#pragma unroll
                    for (uint32_t q = 0; q < kFlatMaxPk / 64; ++q) {
                        const uint32_t k = lane + 64 * q;
                        const bool f = k < m && L.fail[k] == kFail;
                        cn[q] = f ? ((L.rec[k].z & ~kLiveBit) + 3) >> 2 : 0u;
                        fmask[q] = __ballot(f && cn[q] > 0);
                    }
                    int own = -1;
                    uint32_t oc = 0, pos = 0;
                    auto round = [&]() {
                        if (own >= 0) {
                            const uint4 rc = L.rec[own];
                            const FKey fk = fkey(L, (uint32_t)own);
                            const uint32_t onb = rc.z & ~kLiveBit, b0 = 4 * oc, last = onb - 1;
                            uint4 *p = reinterpret_cast<uint4 *>(buf + (((uint64_t)rc.y << 32) | rc.x) + 16) + b0;
                            const uint4 m0 = p[min(b0, last) - b0], m1 = p[min(b0 + 1, last) - b0];
                            const uint4 m2 = p[min(b0 + 2, last) - b0], m3 = p[min(b0 + 3, last) - b0];
                            const Stream stm = make_stream(fk.key, 0u, fk.n1, fk.n2);
                            uint32_t ks[16];
                            stream_block(stm, oc + 1, ks);
                            if (b0 < onb) fstore<WIN>(FS, p + 0, true, 0, xor4(m0, ks + 0));
                            if (b0 + 1 < onb) fstore<WIN>(FS, p + 1, true, 0, xor4(m1, ks + 4));
                            if (b0 + 2 < onb) fstore<WIN>(FS, p + 2, true, 0, xor4(m2, ks + 8));
                            if (b0 + 3 < onb) fstore<WIN>(FS, p + 3, true, 0, xor4(m3, ks + 12));
                        }
                        own = -1;
                    };
#pragma unroll
                    for (uint32_t q = 0; q < kFlatMaxPk / 64; ++q) {
                        uint64_t fm = fmask[q];
                        while (fm) {
                            const uint32_t f = (uint32_t)__ffsll((unsigned long long)fm) - 1;
                            fm &= fm - 1;
                            const uint32_t Cf = (uint32_t)__builtin_amdgcn_readlane((int)cn[q], (int)f);
                            for (uint32_t done = 0; done < Cf;) {
                                const uint32_t take = min(Cf - done, 64u - pos);
                                if (lane >= pos && lane < pos + take) {
                                    own = (int)(64 * q + f);
                                    oc = done + lane - pos;
                                }
                                pos += take;
                                done += take;
                                if (pos == 64) {
                                    round();
                                    pos = 0;
                                }
                            }
                        }
                    }
                    if (pos > 0) round();
                }
            }
            wave_sync(); // the next sub-unit overwrites the LDS image
        }
    }
#if RG_DIAG
    if (dbg) {
        mk[7] = __builtin_amdgcn_s_memtime();
        const uint64_t rt1 = __builtin_amdgcn_s_memrealtime();
        if (lane == 0) {
            for (int q = 0; q < 8; ++q) dbg[8ull * wid + q] = mk[q];
            dbg[8ull * (nw + wid) + 0] = rt0; // second block of rows: wall-clock start and end
            dbg[8ull * (nw + wid) + 1] = rt1;
            for (int q = 0; q < 6; ++q) dbg[8ull * (nw + wid) + 2 + q] = sk[q]; // the search's steps
            dbg[8ull * (2 * nw + wid) + 0] = unit_info;
            dbg[8ull * (2 * nw + wid) + 1] =
                ((uint64_t)(uint32_t)__builtin_amdgcn_s_getreg(0xF814) << 32) | (uint32_t)__builtin_amdgcn_s_getreg(0xF804);
        }
    }
#endif
#undef RG_FLAT_MARK
#undef RG_FLAT_SUB
}

// The workgroup-cooperative unit search applies when every workgroup's four units lie in one group of
// kCoopGroup packets: n a multiple of kCoopGroup and units x kCoopGroup / n a multiple of four.
// Returns the units per group (0: the one-wave search).
static uint32_t flat_coop_ok(uint32_t n, uint32_t units, bool balance) {
    if (!balance || n < kCoopGroup || n % kCoopGroup != 0) return 0;
    const uint64_t x = (uint64_t)units * kCoopGroup;
    if (x % n != 0) return 0;
    const uint64_t kgc = x / n;
    return kgc % 4 == 0 && kgc >= 4 ? (uint32_t)kgc : 0u;
}

hipError_t launch_flat(const SealArgs *sa, const OpenArgs *oa, bool balance, uint4 *junk, int cus, hipStream_t s,
                       hipEvent_t done) {
    const uint32_t n = sa ? sa->n : oa->n;
    if (n == 0) return hipSuccess;
    FlatArgs A{};
    if (sa) A.sa = *sa;
    if (oa) A.oa = *oa;
    // one workgroup per CU (two, at two waves per SIMD, measured 5-8 % slower: profiles/r4_cfg3_twowave_ab.txt)
    const uint32_t blocks = (uint32_t)(cus > 0 ? cus : 1);
    A.units = blocks * kFlatWaves;
    A.junk = junk;
    A.balance = balance ? 1u : 0u;
    A.coop = flat_coop_ok(n, A.units, balance);
    A.wpkt = kCoopWPkt;
    A.wchk = kCoopWChk;
    const uint32_t lds = kFlatLdsBytes;
    const bool win = (sa ? sa->buf_len : oa->buf_len) < 0x7FFFFFF0ull; // frame offsets below 2 GiB
    if (sa && win) RG_LAUNCH(done, (flat_kernel<false, true>), dim3(blocks), dim3(64 * kFlatWaves), lds, s, A);
    else if (sa) RG_LAUNCH(done, (flat_kernel<false, false>), dim3(blocks), dim3(64 * kFlatWaves), lds, s, A);
    else if (win) RG_LAUNCH(done, (flat_kernel<true, true>), dim3(blocks), dim3(64 * kFlatWaves), lds, s, A);
    else RG_LAUNCH(done, (flat_kernel<true, false>), dim3(blocks), dim3(64 * kFlatWaves), lds, s, A);
    return hipGetLastError();
}

uint32_t flat_junk_bytes(int cus) { return (uint32_t)(cus > 0 ? cus : 1) * kFlatWaves * 64 * 64; }

hipError_t prepare_flat_kernels() {
    const int lds = (int)kFlatLdsBytes;
    const void *f[4] = {(const void *)flat_kernel<false, true>, (const void *)flat_kernel<false, false>,
                        (const void *)flat_kernel<true, true>, (const void *)flat_kernel<true, false>};
    hipError_t e = hipSuccess;
    for (int k = 0; k < 4 && e == hipSuccess; ++k) e = hipFuncSetAttribute(f[k], hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    return e;
}

} // namespace rg
