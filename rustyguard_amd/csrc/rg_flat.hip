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
//  * The batch is cut into units of whole packets of equal work (1 one-time-key
//    block + 64-byte chunks per packet), one unit per wave.  A planner kernel
//    writes per-1024-packet prefix sums of that work; each wave finds its own
//    unit boundaries from them (two small searches), so nothing is sorted and no
//    atomics sit on the data path.
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
// clamped inside the frame and stores redirected to a per-lane junk slot when
// a block is not part of the payload, so every step issues the same memory
// instructions and the vmcnt waits stay exact.
#include "rg_device.h"
#include "rg_internal.h"

namespace rg {

// ---------------------------------------------------------------- planner
// Work of a packet as the planner counts it: its one-time-key block and its
// 64-byte chunks (from the descriptor alone).
__device__ __forceinline__ uint32_t flat_work(const rg_pkt_desc &d, bool open) {
    uint32_t P = open ? (d.len >= 32 ? d.len - 32 : 0u) : d.len;
    if (P > kMaxPayload) P = 0;
    return 1u + (P + 63) / 64;
}

// One workgroup per kFlatGroup packets: inclusive prefix of the work inside the
// group (local_incl, padded to whole groups) and the group's total; the last
// workgroup to finish turns the totals into grp_prefix[0..G] (grp_prefix[G] =
// all work) and reports whether every packet had the same work (classes_out).
__global__ __launch_bounds__(256) void flat_plan_kernel(const rg_pkt_desc *desc, uint32_t n, uint32_t open,
                                                        FlatPlan fp) {
    __shared__ uint32_t wsum[4], wmin[4], wmax[4];
    __shared__ uint32_t is_last;
    __shared__ uint64_t carry_s;
    const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const uint64_t i0 = (uint64_t)blockIdx.x * kFlatGroup + 4 * tid;
    uint32_t w[4], lo = ~0u, hi = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint64_t i = i0 + q;
        w[q] = i < n ? flat_work(desc[i], open != 0) : 0u;
        if (i < n) {
            lo = min(lo, w[q]);
            hi = max(hi, w[q]);
        }
    }
    const uint32_t s = w[0] + w[1] + w[2] + w[3];
    uint32_t x = s;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(x, d);
        if ((int)lane >= d) x += y;
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        lo = min(lo, (uint32_t)__shfl_xor((int)lo, d));
        hi = max(hi, (uint32_t)__shfl_xor((int)hi, d));
    }
    if (lane == 63) wsum[wv] = x;
    if (lane == 0) {
        wmin[wv] = lo;
        wmax[wv] = hi;
    }
    __syncthreads();
    uint32_t base = 0;
    for (uint32_t v = 0; v < wv; ++v) base += wsum[v];
    const uint32_t e = base + x - s;
    reinterpret_cast<uint4 *>(fp.local_incl)[(uint64_t)blockIdx.x * 256 + tid] =
        make_uint4(e + w[0], e + w[0] + w[1], e + w[0] + w[1] + w[2], e + s);
    if (tid == 0) {
        const uint32_t tot = wsum[0] + wsum[1] + wsum[2] + wsum[3];
        const uint32_t gmin = min(min(wmin[0], wmin[1]), min(wmin[2], wmin[3]));
        const uint32_t gmax = max(max(wmax[0], wmax[1]), max(wmax[2], wmax[3]));
        __hip_atomic_store(&fp.grp_sum[blockIdx.x], tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&fp.grp_sum[fp.G + blockIdx.x], gmin, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&fp.grp_sum[2 * fp.G + blockIdx.x], gmax, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        is_last = __hip_atomic_fetch_add(fp.ticket, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
        carry_s = 0;
    }
    __syncthreads();
    if (!is_last) return; // block-uniform
    // last workgroup: exclusive prefix of the group totals (G <= 2^22)
    uint32_t gmin = ~0u, gmax = 0;
    for (uint32_t b = 0; b < fp.G; b += 256) {
        const uint32_t g = b + tid;
        uint32_t v = 0;
        if (g < fp.G) {
            v = __hip_atomic_load(&fp.grp_sum[g], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            gmin = min(gmin, __hip_atomic_load(&fp.grp_sum[fp.G + g], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
            gmax = max(gmax, __hip_atomic_load(&fp.grp_sum[2 * fp.G + g], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
        }
        uint32_t y = v; // 64 group totals (< 2^24 each) fit 32 bits
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t z = (uint32_t)__shfl_up((int)y, d);
            if ((int)lane >= d) y += z;
        }
        __syncthreads();
        if (lane == 63) wsum[wv] = y;
        __syncthreads();
        uint64_t pre = carry_s;
        for (uint32_t v2 = 0; v2 < wv; ++v2) pre += wsum[v2];
        if (g < fp.G) fp.grp_prefix[g] = pre + (y - v);
        __syncthreads();
        if (tid == 0) carry_s += (uint64_t)wsum[0] + wsum[1] + wsum[2] + wsum[3];
        __syncthreads();
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        gmin = min(gmin, (uint32_t)__shfl_xor((int)gmin, d));
        gmax = max(gmax, (uint32_t)__shfl_xor((int)gmax, d));
    }
    if (lane == 0) {
        wmin[wv] = gmin;
        wmax[wv] = gmax;
    }
    __syncthreads();
    if (tid == 0) {
        fp.grp_prefix[fp.G] = carry_s;
        const uint32_t mn = min(min(wmin[0], wmin[1]), min(wmin[2], wmin[3]));
        const uint32_t mx = max(max(wmax[0], wmax[1]), max(wmax[2], wmax[3]));
        if (fp.classes_out) *reinterpret_cast<volatile uint32_t *>(fp.classes_out) = mn == mx ? 1u : 2u;
        __hip_atomic_store(fp.ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// ------------------------------------------------------ unit boundaries
// First packet i whose work midpoint (B_i + E_i) / 2 lies at or past target
// (B_i / E_i: work before / through packet i), for two targets at once; a
// packet belongs to the unit its midpoint falls in.  Wave-uniform results.
__device__ __forceinline__ void flat_find2(const FlatPlan &fp, uint32_t n, const uint64_t t[2], uint32_t out[2]) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t G = fp.G;
    uint32_t stride = 1;
    while ((uint64_t)stride * 64 < G) stride *= 64;
    uint32_t base[2] = {0, 0};
    for (;;) { // last group g with grp_prefix[g] <= t (grp_prefix[0] = 0)
        uint64_t v[2];
        uint32_t gi[2];
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            gi[q] = base[q] + lane * stride;
            v[q] = fp.grp_prefix[gi[q] < G ? gi[q] : G - 1];
        }
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const uint32_t c = (uint32_t)__popcll(__ballot(gi[q] < G && v[q] <= t[q]));
            base[q] += (c - 1) * stride;
        }
        if (stride == 1) break;
        stride /= 64;
    }
    uint4 e[2][4];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        const uint4 *p = reinterpret_cast<const uint4 *>(fp.local_incl + (uint64_t)base[q] * kFlatGroup + 16 * lane);
        e[q][0] = p[0];
        e[q][1] = p[1];
        e[q][2] = p[2];
        e[q][3] = p[3];
    }
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        const uint64_t gp = fp.grp_prefix[base[q]];
        const uint32_t v[16] = {e[q][0].x, e[q][0].y, e[q][0].z, e[q][0].w, e[q][1].x, e[q][1].y, e[q][1].z, e[q][1].w,
                                e[q][2].x, e[q][2].y, e[q][2].z, e[q][2].w, e[q][3].x, e[q][3].y, e[q][3].z, e[q][3].w};
        uint32_t prev = (uint32_t)__shfl_up((int)v[15], 1);
        if (lane == 0) prev = 0;
        uint32_t first = 16;
#pragma unroll
        for (int j = 15; j >= 0; --j) {
            const uint32_t w = v[j] - (j ? v[j - 1] : prev);
            if (2 * (gp + v[j]) - w >= 2 * t[q]) first = (uint32_t)j;
        }
        const uint64_t hit = __ballot(first < 16);
        uint64_t r;
        if (hit) {
            const int fl = __ffsll((unsigned long long)hit) - 1;
            r = (uint64_t)base[q] * kFlatGroup + 16u * (uint32_t)fl + (uint32_t)__shfl((int)first, fl);
        } else {
            r = (uint64_t)(base[q] + 1) * kFlatGroup;
        }
        out[q] = uniform_u32((uint32_t)(r < n ? r : n));
        if (t[q] == 0) out[q] = 0;
        if (t[q] >= fp.grp_prefix[G]) out[q] = n;
    }
}

// -------------------------------------------------------------- LDS image
// One per wave, structure-of-arrays over the sub-unit's packets.
constexpr uint32_t kFlatMaxPk = 256;
struct FlatLds {
    uint64_t off[kFlatMaxPk];     // frame offset
    uint32_t nb[kFlatMaxPk];      // 16-byte payload blocks of the packet's chunk stream (0: none)
    uint32_t cs[kFlatMaxPk + 4];  // exclusive prefix of chunks; cs[m] = D
    uint32_t key[kFlatMaxPk][8];  // session key
    uint32_t ctr[kFlatMaxPk][2];  // nonce counter (lo, hi)
    uint32_t r[kFlatMaxPk][4];    // one-time key r (unclamped words; make_mul clamps)
    uint32_t sw[kFlatMaxPk][4];   // seal: s; open: tag - s (mod 2^128)
    uint32_t hs[kFlatMaxPk][8];   // final piece's Horner sum h0..h4, [5] = its lane (64: none)
    uint32_t flags[kFlatMaxPk];   // kLive: tag to finish in phase F; kFail: open tag mismatch
    uint32_t ck[64];              // lane's carry: packet (or ~0)
    uint32_t ch[64][5];           // lane's carry value h r^after
};
constexpr uint32_t kLive = 1u, kFail = 2u;
constexpr uint32_t kFlatWaves = 4; // one per SIMD
static_assert(kFlatWaves * sizeof(FlatLds) <= kLdsPerCu, "flat LDS image");

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

struct FChunk {
    uint4 q0, q1, q2, q3;
};

// chunk t of a packet whose last 16-byte block is `last`: four loads, indices
// clamped inside the payload (always readable)
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
    const uint4 *pl;
};

__device__ __forceinline__ void fcur_set(FCur &p, const FlatLds &L, uint8_t *buf, uint32_t k, uint32_t t) {
    p.k = k;
    p.t = t;
    p.nb = L.nb[k];
    p.c = (p.nb + 3) >> 2;
    p.pl = reinterpret_cast<const uint4 *>(buf + L.off[k] + 16);
}

// next chunk; returns true when it starts a new packet (empty packets skipped)
__device__ __forceinline__ bool fcur_next(FCur &p, const FlatLds &L, uint8_t *buf, uint32_t m) {
    if (++p.t < p.c) return false;
    uint32_t k = p.k + 1;
    while (k < m && L.cs[k + 1] == L.cs[k]) ++k;
    if (k < m) fcur_set(p, L, buf, k, 0);
    else p.k = m; // past the sub-unit (keeps pl: loads stay readable)
    return true;
}

__device__ __forceinline__ Stream fstream(const FlatLds &L, uint32_t k) {
    Key8 key;
#pragma unroll
    for (int w = 0; w < 8; ++w) key.k[w] = L.key[k][w];
    return make_stream(key, 0u, L.ctr[k][0], L.ctr[k][1]);
}

__device__ __forceinline__ Mul fmul(const FlatLds &L, uint32_t k) {
    return make_mul(L.r[k][0], L.r[k][1], L.r[k][2], L.r[k][3]);
}

// per-lane state of phase C
struct FLane {
    FCur cur, f;        // compute cursor / prefetch cursor
    uint32_t nsteps, fj; // chunks of the lane; lane-relative index of the prefetch cursor
    bool live;           // current packet's tag is computed (open: header passed)
    Stream st;
    Mul r;
    Acc h;
    FChunk pi;          // seal: ciphertext chunk waiting to be absorbed (one step behind)
    uint32_t pi_cnt, pk; // its blocks and packet
};

// One step of phase C over chunk j of the lane (in buffer b).  Seal absorbs the
// previous step's ciphertext (pi) inside this step's keystream rounds, open
// absorbs this chunk's ciphertext; the pending piece is published when the
// packet changes.  Afterwards chunk j + 3 is requested into b.
template <bool OPEN>
__device__ __forceinline__ void flat_step(FLane &s, FChunk &b, uint32_t j, FlatLds &L, uint8_t *buf, uint4 *junk,
                                          uint32_t m, uint32_t lane) {
    const bool active = j < s.nsteps;
    uint32_t cnt = 0;
    if (active && s.live) cnt = min(4u, s.cur.nb - 4 * s.cur.t);
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
    *(cnt > 0 ? dst + 0 : junk + 0) = x.q0;
    *(cnt > 1 ? dst + 1 : junk + 1) = x.q1;
    *(cnt > 2 ? dst + 2 : junk + 2) = x.q2;
    *(cnt > 3 ? dst + 3 : junk + 3) = x.q3;
    if constexpr (OPEN) {
        if (active && s.cur.t + 1 == s.cur.c) { // the packet's last chunk: its final piece
            if (s.live) {
                uint32_t *o = L.hs[s.cur.k];
                o[0] = s.h.h0; o[1] = s.h.h1; o[2] = s.h.h2; o[3] = s.h.h3; o[4] = s.h.h4; o[5] = lane;
            }
            s.h = Acc{0, 0, 0, 0, 0};
        }
    } else {
        if (active && s.pk != s.cur.k) { // the pending packet ended in this lane: final piece
            if (s.pk < m) {
                uint32_t *o = L.hs[s.pk];
                o[0] = s.h.h0; o[1] = s.h.h1; o[2] = s.h.h2; o[3] = s.h.h3; o[4] = s.h.h4; o[5] = lane;
            }
            s.h = Acc{0, 0, 0, 0, 0};
            s.r = fmul(L, s.cur.k);
            s.pk = s.cur.k;
        }
        s.pi = x;
        s.pi_cnt = cnt;
    }
    // request chunk j + 3 of the lane into b (the same chunk again past the range)
    if (s.fj + 1 < s.nsteps) {
        ++s.fj;
        fcur_next(s.f, L, buf, m);
    }
    fload(b, s.f.pl, s.f.t, s.f.nb ? s.f.nb - 1 : 0);
    if (active && fcur_next(s.cur, L, buf, m) && s.cur.k < m) {
        s.st = fstream(L, s.cur.k);
        s.live = (L.flags[s.cur.k] & kLive) != 0;
        if constexpr (OPEN) s.r = fmul(L, s.cur.k);
    }
}

// h * r^e (e < 2^21), left to right over the wave's largest exponent; lanes
// with e = 0 keep h
__device__ __forceinline__ Acc flat_pow_mul(Acc h, const Mul &r, uint32_t e) {
    uint32_t mx = e;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) mx = max(mx, (uint32_t)__shfl_xor((int)mx, o));
    const uint32_t bits = 32 - __clz((int)uniform_u32(mx));
    if (bits == 0) return h;
    Acc x = {1, 0, 0, 0, 0};
    for (int b = (int)bits - 1; b >= 0; --b) {
        Acc sq = x;
        acc_mul_gen(sq, make_gen(x));
        Acc xr = sq;
        acc_mul(xr, r);
        const bool bit = (e >> b) & 1u;
        x.h0 = bit ? xr.h0 : sq.h0; x.h1 = bit ? xr.h1 : sq.h1; x.h2 = bit ? xr.h2 : sq.h2;
        x.h3 = bit ? xr.h3 : sq.h3; x.h4 = bit ? xr.h4 : sq.h4;
    }
    Acc y = h;
    acc_mul_gen(y, make_gen(x));
    return y;
}

struct FlatArgs {
    SealArgs sa;
    OpenArgs oa;
    FlatPlan fp;     // fp.grp_prefix == nullptr: units by packet index
    uint4 *junk;     // [waves][64 lanes][4] sink of the stores that are not payload
    uint32_t units;  // = waves of the grid
};

template <bool OPEN> __global__ __launch_bounds__(256) void flat_kernel(FlatArgs A) {
    extern __shared__ __attribute__((aligned(16))) uint8_t flat_lds[];
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    FlatLds &L = reinterpret_cast<FlatLds *>(flat_lds)[wv];
    const uint32_t wid = blockIdx.x * kFlatWaves + wv, nw = gridDim.x * kFlatWaves;
    const uint32_t n = OPEN ? A.oa.n : A.sa.n;
    uint8_t *const buf = OPEN ? A.oa.buf : A.sa.buf;
    const uint64_t buf_len = OPEN ? A.oa.buf_len : A.sa.buf_len;
    const uint32_t nkeys = OPEN ? A.oa.nkeys : A.sa.nkeys;
    const uint32_t *const keys = OPEN ? A.oa.keys : A.sa.keys;
    const rg_pkt_desc *const desc = OPEN ? A.oa.desc : A.sa.desc;
    uint8_t *const status = OPEN ? A.oa.status : A.sa.status;
    uint4 *const junk = A.junk + ((uint64_t)wid * 64 + lane) * 4;
    for (uint32_t u = wid; u < A.units; u += nw) {
        // ---- this unit's packets [s, e)
        uint32_t se[2];
        if (A.fp.grp_prefix) {
            const uint64_t T = A.fp.grp_prefix[A.fp.G];
            const uint64_t q = T / A.units, rm = T % A.units;
            const uint64_t t[2] = {q * u + rm * u / A.units, q * (u + 1) + rm * (u + 1) / A.units};
            flat_find2(A.fp, n, t, se);
        } else {
            se[0] = (uint32_t)((uint64_t)n * u / A.units);
            se[1] = (uint32_t)((uint64_t)n * (u + 1) / A.units);
        }
        for (uint32_t sb = se[0]; sb < se[1]; sb += kFlatMaxPk) {
            const uint32_t m = min(kFlatMaxPk, se[1] - sb);
            // ---- A0: descriptors -> LDS, chunk counts, descriptor-level statuses
            uint32_t chunks[kFlatMaxPk / 64];
            rg_pkt_desc dk[kFlatMaxPk / 64];
            uint8_t dst[kFlatMaxPk / 64]; // 0xFF: passes the descriptor checks
#pragma unroll
            for (uint32_t q = 0; q < kFlatMaxPk / 64; ++q) {
                const uint32_t k = lane + 64 * q;
                chunks[q] = 0;
                dst[q] = 0xFF;
                dk[q] = rg_pkt_desc{0, 0, 0};
                if (k < m) {
                    const rg_pkt_desc d = desc[sb + k];
                    dk[q] = d;
                    uint32_t nb = 0;
                    if constexpr (!OPEN) {
                        const uint32_t P = d.len;
                        const bool valid = d.key_idx < nkeys && (P & 15u) == 0 && (d.offset & 15u) == 0 &&
                                           P <= kMaxPayload && d.offset <= buf_len && P + 32 <= buf_len - d.offset;
                        if (!valid) dst[q] = d.key_idx == RG_KEY_SKIP ? RG_PKT_REJECTED : RG_PKT_INVALID;
                        else nb = P >> 4;
                    } else {
                        const uint32_t W = d.len;
                        uint8_t st = 0xFF;
                        if (d.key_idx == RG_KEY_SKIP) st = RG_PKT_REJECTED;
                        else if ((d.offset & 15u) != 0) st = RG_PKT_UNALIGNED;               // lib.rs:613-615
                        else if (d.key_idx >= nkeys || W > kMaxPayload + 32 || d.offset > buf_len ||
                                 W > buf_len - d.offset || W < 4)
                            st = RG_PKT_INVALID;
                        dst[q] = st;
                        if (st == 0xFF && W >= 32 && (W & 15u) == 0) nb = (W - 32) >> 4;
                    }
                    L.off[k] = d.offset;
                    L.nb[k] = nb;
                    chunks[q] = (nb + 3) >> 2;
                }
            }
            // exclusive prefix of the chunk counts in k order (k = lane + 64 q)
            uint32_t run = 0;
#pragma unroll
            for (uint32_t q = 0; q < kFlatMaxPk / 64; ++q) {
                uint32_t x = chunks[q];
#pragma unroll
                for (int d = 1; d < 64; d <<= 1) {
                    const uint32_t y = (uint32_t)__shfl_up((int)x, d);
                    if ((int)lane >= d) x += y;
                }
                const uint32_t k = lane + 64 * q;
                if (k < m) L.cs[k] = run + x - chunks[q];
                run += uniform_u32((uint32_t)__shfl((int)x, 63));
            }
            const uint32_t D = run;
            if (lane == 0) L.cs[m] = D;
            wave_sync();
            // ---- the lane's chunk range and start packet
            const uint32_t c_lo = (uint32_t)((uint64_t)lane * D / 64), c_hi = (uint32_t)((uint64_t)(lane + 1) * D / 64);
            FLane s;
            s.nsteps = c_hi - c_lo;
            {
                uint32_t lo = 0, hi = m; // last k with cs[k] <= c_lo
                while (hi - lo > 1) {
                    const uint32_t mid = (lo + hi) >> 1;
                    if (L.cs[mid] <= c_lo) lo = mid;
                    else hi = mid;
                }
                if (s.nsteps) fcur_set(s.cur, L, buf, lo, c_lo - L.cs[lo]);
                else { // no chunks: a readable dummy position
                    s.cur.k = m; s.cur.t = 0; s.cur.c = 0; s.cur.nb = 1;
                    s.cur.pl = reinterpret_cast<const uint4 *>(desc + sb);
                }
            }
            // ---- phase A loads (issued ahead of the chunk prefetch so that their waits stay exact)
            uint4 ka[kFlatMaxPk / 64], kb[kFlatMaxPk / 64], hx[kFlatMaxPk / 64], tg[kFlatMaxPk / 64];
            uint32_t rcv[kFlatMaxPk / 64];
#pragma unroll
            for (uint32_t q = 0; q < kFlatMaxPk / 64; ++q) {
                const uint32_t k = lane + 64 * q;
                if (64 * q >= m) break; // wave-uniform
                const bool ok = k < m && dst[q] == 0xFF;
                const uint4 *kp = reinterpret_cast<const uint4 *>(keys + 8ull * (ok ? dk[q].key_idx : 0u));
                ka[q] = kp[0];
                kb[q] = kp[1];
                const uint4 *safe = reinterpret_cast<const uint4 *>(desc + sb);
                if constexpr (!OPEN) {
                    const uint64_t c = A.sa.counters[sb + (k < m ? k : 0)];
                    hx[q] = make_uint4((uint32_t)c, (uint32_t)(c >> 32), 0, 0);
                    rcv[q] = A.sa.receivers ? A.sa.receivers[ok ? dk[q].key_idx : 0u] : 0u;
                    tg[q] = make_uint4(0, 0, 0, 0);
                } else {
                    const bool go = ok && L.nb[k] > 0;
                    const uint8_t *fr = buf + dk[q].offset;
                    // the header as a 16-byte vector when the arena holds 16 bytes there; the type word
                    // alone otherwise (a frame of 4..15 bytes at the very end of the arena)
                    const bool room = ok && buf_len - dk[q].offset >= 16;
                    hx[q] = *(room ? reinterpret_cast<const uint4 *>(fr) : safe);
                    rcv[q] = *(ok ? reinterpret_cast<const uint32_t *>(fr) : reinterpret_cast<const uint32_t *>(safe));
                    tg[q] = *(go ? reinterpret_cast<const uint4 *>(fr + dk[q].len - 16) : safe);
                }
            }
            // ---- the lane's first three chunks
            FChunk b0, b1, b2;
            s.f = s.cur;
            s.fj = 0;
            fload(b0, s.f.pl, s.f.t, s.f.nb ? s.f.nb - 1 : 0);
            if (s.fj + 1 < s.nsteps) { ++s.fj; fcur_next(s.f, L, buf, m); }
            fload(b1, s.f.pl, s.f.t, s.f.nb ? s.f.nb - 1 : 0);
            if (s.fj + 1 < s.nsteps) { ++s.fj; fcur_next(s.f, L, buf, m); }
            fload(b2, s.f.pl, s.f.t, s.f.nb ? s.f.nb - 1 : 0);
            // ---- phase A: checks, one-time-key blocks, header (seal), counters_out (open)
#pragma unroll
            for (uint32_t q = 0; q < kFlatMaxPk / 64; ++q) {
                const uint32_t k = lane + 64 * q;
                if (64 * q >= m) break;
                if (k >= m) continue;
                const uint32_t i = sb + k;
                uint8_t st = dst[q];
                uint32_t n1 = hx[q].x, n2 = hx[q].y; // seal: the counter
                if constexpr (OPEN) {
                    const uint32_t W = dk[q].len;
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
                const Key8 key = {{ka[q].x, ka[q].y, ka[q].z, ka[q].w, kb[q].x, kb[q].y, kb[q].z, kb[q].w}};
                const Stream stm = make_stream(key, 0u, n1, n2); // nonce 0 || le64(counter), prim.rs:32-36
                uint32_t ks[16];
                stream_block(stm, 0, ks); // RFC 8439 §2.6 one-time key
#pragma unroll
                for (int w = 0; w < 8; ++w) L.key[k][w] = key.k[w];
                L.ctr[k][0] = n1;
                L.ctr[k][1] = n2;
                L.r[k][0] = ks[0]; L.r[k][1] = ks[1]; L.r[k][2] = ks[2]; L.r[k][3] = ks[3];
                if constexpr (OPEN) { // tag - s (mod 2^128): phase F compares (h mod p) with it
                    uint32_t c;
                    L.sw[k][0] = __builtin_subc(tg[q].x, ks[4], 0u, &c);
                    L.sw[k][1] = __builtin_subc(tg[q].y, ks[5], c, &c);
                    L.sw[k][2] = __builtin_subc(tg[q].z, ks[6], c, &c);
                    L.sw[k][3] = __builtin_subc(tg[q].w, ks[7], c, &c);
                } else {
                    L.sw[k][0] = ks[4]; L.sw[k][1] = ks[5]; L.sw[k][2] = ks[6]; L.sw[k][3] = ks[7];
                }
                L.hs[k][0] = 0; L.hs[k][1] = 0; L.hs[k][2] = 0; L.hs[k][3] = 0; L.hs[k][4] = 0; L.hs[k][5] = 64;
                L.flags[k] = st == 0xFF ? kLive : 0u;
                if (st != 0xFF) {
                    if (status) status[i] = st;
                } else if constexpr (!OPEN) {
                    // DataHeader {4, receiver, counter} (rustyguard-core/src/lib.rs:286-290)
                    if (A.sa.receivers)
                        *reinterpret_cast<uint4 *>(buf + dk[q].offset) = make_uint4(4u, rcv[q], n1, n2);
                }
            }
            wave_sync();
            // ---- phase C: the chunk stream
            const uint32_t S = (D + 63) / 64;
            if (s.cur.k < m) {
                s.st = fstream(L, s.cur.k);
                s.r = fmul(L, s.cur.k);
                s.live = (L.flags[s.cur.k] & kLive) != 0;
            } else {
                s.st = make_stream(Key8{{0, 0, 0, 0, 0, 0, 0, 0}}, 0u, 0u, 0u);
                s.r = make_mul(0, 0, 0, 0);
                s.live = false;
            }
            s.h = Acc{0, 0, 0, 0, 0};
            s.pi = FChunk{};
            s.pi_cnt = 0;
            s.pk = s.cur.k;
            {
                uint32_t j = 0;
                for (; j + 3 <= S; j += 3) {
                    flat_step<OPEN>(s, b0, j, L, buf, junk, m, lane);
                    flat_step<OPEN>(s, b1, j + 1, L, buf, junk, m, lane);
                    flat_step<OPEN>(s, b2, j + 2, L, buf, junk, m, lane);
                }
                if (j < S) flat_step<OPEN>(s, b0, j, L, buf, junk, m, lane);
                if (j + 1 < S) flat_step<OPEN>(s, b1, j + 1, L, buf, junk, m, lane);
            }
            uint32_t ck = ~0u, after = 0;
            if constexpr (!OPEN) { // the last ciphertext chunk
                acc_block_pred(s.h, s.pi.q0, s.r, s.pi_cnt > 0);
                acc_block_pred(s.h, s.pi.q1, s.r, s.pi_cnt > 1);
                acc_block_pred(s.h, s.pi.q2, s.r, s.pi_cnt > 2);
                acc_block_pred(s.h, s.pi.q3, s.r, s.pi_cnt > 3);
                if (s.nsteps > 0 && s.pk < m) {
                    if (s.cur.k == s.pk && s.cur.t > 0) { // the packet goes on in the next lane
                        ck = s.pk;
                        after = s.cur.nb - 4 * s.cur.t;
                    } else {
                        uint32_t *o = L.hs[s.pk];
                        o[0] = s.h.h0; o[1] = s.h.h1; o[2] = s.h.h2; o[3] = s.h.h3; o[4] = s.h.h4; o[5] = lane;
                    }
                }
            } else {
                if (s.nsteps > 0 && s.cur.k < m && s.cur.t > 0) {
                    ck = s.cur.k;
                    after = s.cur.nb - 4 * s.cur.t;
                }
            }
            // carry = h r^after for the packet the next lane continues
            const Acc cv = flat_pow_mul(s.h, s.r, ck != ~0u ? after : 0u);
            L.ck[lane] = ck;
            L.ch[lane][0] = cv.h0; L.ch[lane][1] = cv.h1; L.ch[lane][2] = cv.h2; L.ch[lane][3] = cv.h3;
            L.ch[lane][4] = cv.h4;
            wave_sync();
            // ---- phase F: tags
            bool any_fail = false;
            for (uint32_t k = lane; k < m; k += 64) {
                if (!(L.flags[k] & kLive)) continue;
                Acc h = {L.hs[k][0], L.hs[k][1], L.hs[k][2], L.hs[k][3], L.hs[k][4]};
                for (int l = (int)L.hs[k][5] - 1; l >= 0 && L.ck[l] == k; --l) {
                    acc_add_acc(h, Acc{L.ch[l][0], L.ch[l][1], L.ch[l][2], L.ch[l][3], L.ch[l][4]});
                    acc_fold(h);
                }
                const uint32_t P = L.nb[k] * 16;
                const Mul r = fmul(L, k);
                acc_add(h, 0, 0, P, 0, 1); // le64(aad_len = 0) || le64(P), RFC 8439 §2.8
                acc_mul(h, r);
                const uint32_t i = sb + k;
                uint32_t tag[4];
                if constexpr (!OPEN) {
                    acc_finish(h, L.sw[k][0], L.sw[k][1], L.sw[k][2], L.sw[k][3], tag);
                    *reinterpret_cast<uint4 *>(buf + L.off[k] + 16 + P) = make_uint4(tag[0], tag[1], tag[2], tag[3]);
                    if (status) status[i] = RG_PKT_OK;
                } else {
                    acc_finish(h, 0, 0, 0, 0, tag);
                    const uint32_t diff = (tag[0] ^ L.sw[k][0]) | (tag[1] ^ L.sw[k][1]) | (tag[2] ^ L.sw[k][2]) |
                                          (tag[3] ^ L.sw[k][3]);
                    status[i] = diff == 0 ? RG_PKT_OK : RG_PKT_DECRYPT_ERR;
                    if (diff != 0) {
                        L.flags[k] |= kFail;
                        any_fail = true;
                    }
                }
            }
            if constexpr (OPEN) {
                // ---- forgeries: put the ciphertext back (plaintext ^ keystream)
                if (__ballot(any_fail)) {
                    wave_sync();
                    if (s.nsteps) {
                        FCur p;
                        uint32_t lo = 0, hi = m;
                        while (hi - lo > 1) {
                            const uint32_t mid = (lo + hi) >> 1;
                            if (L.cs[mid] <= c_lo) lo = mid;
                            else hi = mid;
                        }
                        fcur_set(p, L, buf, lo, c_lo - L.cs[lo]);
                        Stream stm = fstream(L, p.k);
                        for (uint32_t j = 0; j < s.nsteps; ++j) {
                            if (L.flags[p.k] & kFail) {
                                uint32_t ks[16];
                                stream_block(stm, p.t + 1, ks);
                                uint4 *q = const_cast<uint4 *>(p.pl) + 4 * p.t;
                                const uint32_t c = min(4u, p.nb - 4 * p.t);
                                for (uint32_t b = 0; b < c; ++b) q[b] = xor4(q[b], ks + 4 * b);
                            }
                            if (fcur_next(p, L, buf, m) && p.k < m) stm = fstream(L, p.k);
                        }
                    }
                }
            }
            wave_sync(); // the next sub-unit overwrites the LDS image
        }
    }
}

hipError_t launch_flat(const SealArgs *sa, const OpenArgs *oa, const FlatPlan *fp, uint4 *junk, int cus,
                       hipStream_t s) {
    const uint32_t n = sa ? sa->n : oa->n;
    if (n == 0) return hipSuccess;
    FlatArgs A{};
    if (sa) A.sa = *sa;
    if (oa) A.oa = *oa;
    const uint32_t blocks = (uint32_t)(cus > 0 ? cus : 1);
    A.units = blocks * kFlatWaves;
    A.junk = junk;
    if (fp) {
        A.fp = *fp;
        hipLaunchKernelGGL(flat_plan_kernel, dim3(fp->G), dim3(256), 0, s, sa ? sa->desc : oa->desc, n,
                           oa ? 1u : 0u, *fp);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    const uint32_t lds = kFlatWaves * (uint32_t)sizeof(FlatLds);
    if (sa) hipLaunchKernelGGL(flat_kernel<false>, dim3(blocks), dim3(256), lds, s, A);
    else hipLaunchKernelGGL(flat_kernel<true>, dim3(blocks), dim3(256), lds, s, A);
    return hipGetLastError();
}

uint32_t flat_junk_bytes(int cus) { return (uint32_t)(cus > 0 ? cus : 1) * kFlatWaves * 64 * 64; }

hipError_t prepare_flat_kernels() {
    const int lds = (int)(kFlatWaves * sizeof(FlatLds));
    hipError_t e = hipFuncSetAttribute((const void *)flat_kernel<false>, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    if (e == hipSuccess)
        e = hipFuncSetAttribute((const void *)flat_kernel<true>, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    return e;
}

} // namespace rg
