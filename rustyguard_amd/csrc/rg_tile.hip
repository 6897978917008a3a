// rg_tile.hip -- the batched transport kernels (default path of
// rg_{seal,open}_batch_*): a size-bucketing planner and the LDS-staged tile
// kernel.  Replaces N x Core::chacha20poly1305_{enc,dec}
// (rustyguard-crypto/src/prim.rs:179-201) as driven by EncryptionKey::encrypt
// / DecryptionKey::decrypt (prim.rs:386-437) for WireGuard data packets.
//
// Planner (plan_kernel): every packet is put in the work list of its size
// class (its number of 64-byte chunks, exact up to 16, then 1.5x steps), so
// the tile kernel can build tiles of equally long packets: a 64-packet tile
// runs as long as its longest packet.
//
// Tile kernel (tile_kernel<G, OPEN>): a 256-thread workgroup (4 waves) takes
// one "group" at a time: 4 tiles of 64 packets (K = 1), 2 tiles each split
// into 2 contiguous segments on 2 waves (K = 2), or 1 tile split into 4
// segments (K = 4).  The class -> K choice comes from the class counts alone
// (target: about two waves per SIMD of work), every workgroup derives the
// same schedule from them.  Within a wave, lane l owns (a segment of) packet
// l of the tile and keeps its ChaCha state and Poly1305 accumulator in VGPRs;
// payload moves HBM -> LDS -> HBM in double-buffered windows of G chunks per
// lane with coalesced LDS-DMA loads and buffer stores (see StagedCfg).
//
// Segments: segment j of a packet covers chunks [jL, min(C, (j+1)L)),
// L = ceil(C/K), keystream blocks from jL + 1; its lane runs its own Horner
// chain A_j over its blocks.  With N_j = blocks after segment j,
//   h = sum_j A_j r^{N_j}   (RFC 8439 Poly1305 of the whole ciphertext)
//     = (..(A_0 q_1 + A_1) q_2 + ..) q_{K-1} + A_{K-1},  q_j = r^{n_j},
// so segments j > 0 also track q_j (one clamped multiply per block) and hand
// (A_j, q_j) to segment 0 through LDS.
#include "rg_device.h"
#include "rg_internal.h"

#include <type_traits>

namespace rg {

// ------------------------------------------------------------ size classes

// class_of: rg_internal.h

// Each workgroup classifies kPlanPer x 256 consecutive packets: per wave and
// class one ballot -> one LDS atomic (runs of consecutive packets stay
// together), then one global atomic per class and workgroup.  Uniform batches
// therefore keep tiles of 64 consecutive frames.
constexpr uint32_t kPlanPer = 2; // 1, 8 and 16 measured slower at config 3 (round r1e)

__global__ __launch_bounds__(256) void plan_kernel(const rg_pkt_desc *desc, uint32_t n, uint32_t open,
                                                   uint32_t *counts, uint32_t *lists, uint32_t cap, uint32_t *sched,
                                                   uint32_t simds, uint32_t *classes_out) {
    __shared__ uint32_t hist[kClasses];
    __shared__ uint32_t gbase[kClasses];
    __shared__ uint32_t last;
    const uint32_t tid = threadIdx.x, lane = tid & 63;
    if (tid < kClasses) hist[tid] = 0;
    __syncthreads();
    const uint32_t first = blockIdx.x * 256 * kPlanPer;
    uint32_t cls[kPlanPer], rank[kPlanPer];
#pragma unroll
    for (uint32_t k = 0; k < kPlanPer; ++k) {
        const uint32_t i = first + k * 256 + tid;
        uint32_t c = ~0u;
        if (i < n) {
            const uint32_t len = desc[i].len;
            uint32_t P = open ? (len >= 32 ? len - 32 : 0) : len;
            if (P > kMaxPayload) P = 0;
            c = class_of((P + 63) / 64);
        }
        cls[k] = c;
    }
#pragma unroll
    for (uint32_t k = 0; k < kPlanPer; ++k) {
        uint32_t c = cls[k], r = 0;
        uint64_t pending = __ballot(c != ~0u);
        while (pending) {
            const int leader = __ffsll((unsigned long long)pending) - 1;
            const uint32_t b = __shfl(c, leader);
            const uint64_t m = __ballot(c == b);
            uint32_t base = 0;
            if ((int)lane == leader) base = atomicAdd(&hist[b], (uint32_t)__popcll(m));
            base = __shfl(base, leader);
            if (c == b) r = base + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
            pending &= ~m;
        }
        rank[k] = r;
    }
    __syncthreads();
    if (tid < kClasses) gbase[tid] = hist[tid] ? atomicAdd(&counts[tid], hist[tid]) : 0u;
    __syncthreads();
#pragma unroll
    for (uint32_t k = 0; k < kPlanPer; ++k) {
        if (cls[k] != ~0u) lists[(uint64_t)cls[k] * cap + gbase[cls[k]] + rank[k]] = first + k * 256 + tid;
    }
    if (!sched) return; // tile kernels: every workgroup derives its schedule from the counts
    // pipelined kernel: the last planner workgroup turns the final counts into
    // its schedule (one launch fewer per batch than a separate schedule kernel)
    // No fences: this workgroup's count atomics have returned (gbase) before
    // the barrier, so they are performed at device scope before its finish
    // increment, and schedule_classes reads the counts with device-scope
    // atomic loads.  The lists reach the transport kernel at the kernel
    // boundary.
    __syncthreads();
    if (tid == 0) last = atomicAdd(&counts[kClasses], 1u) == gridDim.x - 1;
    __syncthreads();
    if (last) { // block-uniform: the whole workgroup schedules (its barrier inside)
        schedule_classes(counts, sched, simds, classes_out);
        if (tid == 0) __hip_atomic_store(&counts[kClasses], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// ------------------------------------------------------------ LDS-DMA helpers
// Pieces past a payload get an out-of-range buffer offset: the descriptor's
// range check turns such a load into zeros and drops such a store, so every
// wave issues exactly PPW DMA + PPW store instructions per window and the
// vmcnt waits are exact.
constexpr uint32_t kOOB = 0xFFFFFFF0u;

// make_rsrc / dma16 / store16 / wait_vm: rg_device.h

// segment hand-off slot per wave: rows 0-4 partial sum A_j, 5-9 q_j = r^{n_j},
// 10 the open verdict sent back by segment 0
constexpr uint32_t kSlotRows = 11;

// Window geometry: PPW 16-byte pieces per lane per window; DMA instruction q
// serves packets q*PKT_PER_INST .. +PKT_PER_INST-1, PPW lanes per packet, one
// whole contiguous 64G-byte run each (coalesced).  The LDS image is
// lane-linear, slot(p, pos) = p*PPW + pos, and an XOR swizzle on the SOURCE
// side (piece k = pos ^ swz(p)) makes the per-lane ds_read_b128 of one piece
// by 64 lanes bank-conflict free.
template <int G> struct StagedCfg {
    static constexpr uint32_t PPW = 4 * G;
    static constexpr uint32_t PKT_PER_INST = 64 / PPW;
    static constexpr uint32_t BUF = 64 * PPW * 16;  // bytes per window buffer per wave
    static constexpr uint32_t WAVE_LDS = 2 * BUF;   // double-buffered
    static constexpr uint32_t COMB = 8 * kSlotRows * 64 * 4; // segment hand-off slots, one per wave
    static constexpr uint32_t FLAGS = 2 * 8 * 4 + 16; // ready / ack generation per wave slot, work counter
    static constexpr uint32_t WG_LDS = 8 * WAVE_LDS + COMB + FLAGS;
};

template <int G> __device__ __forceinline__ uint32_t swz(uint32_t p) {
    constexpr uint32_t PPW = StagedCfg<G>::PPW;
    return (p / (16 / PPW)) % PPW;
}

// diagnostic-build stamps (STAMP kernels only)
__device__ __forceinline__ uint64_t stamp() {
    uint64_t t;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}
__device__ __forceinline__ uint64_t realtime() { // 100 MHz constant clock
    uint64_t t;
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}

constexpr uint32_t kMinSegment = 4;
constexpr uint32_t kPoolMinRounds = 8; // deal rounds from which the grid-wide pool is used (the measured regime)

__device__ __forceinline__ uint32_t pow2ceil(uint32_t x) { return x <= 1 ? 1u : 1u << (32 - __clz(x - 1)); }

// ------------------------------------------------------------ schedule
// Lane p of every wave describes bucket p of the processing order (largest
// class first).  Identical in every wave of the grid.
struct Sched {
    uint32_t cls, cnt, K, g_end; // this lane's bucket
    uint32_t total_groups;
};

__device__ __forceinline__ Sched make_sched(const TilePlan &tp, uint32_t n) {
    const uint32_t p = threadIdx.x & 63;
    Sched s;
    s.cls = 0;
    s.cnt = 0;
    s.K = 1;
    uint32_t crep = 0;
    if (tp.counts) {
        if (p < kClasses) {
            s.cls = kClasses - 1 - p;
            s.cnt = tp.counts[s.cls];
            crep = class_hi(s.cls);
        }
    } else if (p == 0) {
        s.cnt = n; // identity order: one bucket, K fixed by the host
    }
    // chunk total -> target segment length T, then K per class
    uint64_t tot = (uint64_t)s.cnt * crep;
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) tot += __shfl_xor(tot, m);
    if (tp.counts) {
        if (tp.fixed_k) {
            s.K = tp.fixed_k;
        } else {
            // segment length: the chunk total spread over target_lanes, never
            // below kMinSegment chunks (each segment pays a key block and r^N)
            const uint64_t tl = tp.target_lanes ? tp.target_lanes : 1;
            uint32_t T = (uint32_t)((tot + tl - 1) / tl);
            if (T < kMinSegment) T = kMinSegment;
            const uint32_t want = (crep + T - 1) / T;
            s.K = want >= 4 ? 4u : pow2ceil(want);
        }
    } else {
        s.K = tp.fixed_k ? tp.fixed_k : 1u;
    }
    const uint32_t tiles = (s.cnt + 63) / 64;
    const uint32_t groups = (tiles * s.K + 3) / 4;
    // inclusive prefix over lanes
    uint32_t x = groups;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(x, d);
        if ((int)p >= d) x += y;
    }
    s.g_end = x;
    s.total_groups = uniform_u32(__shfl(x, 63));
    return s;
}

// ------------------------------------------------------------ tile kernel
template <int G, bool OPEN, bool STAMP = false>
__global__ __launch_bounds__(512) void tile_kernel(SealArgs sa, OpenArgs oa, TilePlan tp) {
    using Cfg = StagedCfg<G>;
    constexpr uint32_t PPW = Cfg::PPW;
    uint64_t t_setup = 0, t_store = 0, t_issue = 0, t_wait = 0, t_chunk = 0, t_tail = 0, t_mark = 0, rt0 = 0;
    uint64_t n_pool = 0; // items taken from the grid-wide pool
    if constexpr (STAMP) {
        rt0 = realtime();
        t_mark = stamp();
    }
    extern __shared__ __attribute__((aligned(16))) uint8_t lds_raw[];
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wave = threadIdx.x >> 6; // 0..7
    const uint32_t half = wave >> 2;        // two independent 4-wave halves
    const uint32_t hw = wave & 3;           // wave within the half
    const uint32_t n = OPEN ? oa.n : sa.n;
    uint8_t *const buf = OPEN ? oa.buf : sa.buf;
    const uint64_t buf_len = OPEN ? oa.buf_len : sa.buf_len;
    const uint32_t lds_wave = (uint32_t)(uintptr_t)(lds_raw) + wave * Cfg::WAVE_LDS;
    uint4 *const lds4 = reinterpret_cast<uint4 *>(lds_raw + wave * Cfg::WAVE_LDS);
    uint32_t *const comb = reinterpret_cast<uint32_t *>(lds_raw + 8 * Cfg::WAVE_LDS); // [wave][kSlotRows][64]
    volatile uint32_t *const f_ready = reinterpret_cast<volatile uint32_t *>(lds_raw + 8 * Cfg::WAVE_LDS + Cfg::COMB);
    volatile uint32_t *const f_ack = f_ready + 8;
    uint32_t *const f_next = const_cast<uint32_t *>(f_ready) + 16; // next work item (dynamic deal)
    if (threadIdx.x < 17) f_ready[threadIdx.x] = 0;
    __syncthreads();

    // Group schedule: the groups (largest class first) are dealt to the
    // 2 x gridDim.x half-workgroup slots in snake order; slot s of round 0 is
    // half 0 of workgroup s and slot 2G-1-s half 1 of workgroup s, so every CU
    // pairs a large group with a small one and, with fewer groups than CUs,
    // gets at most one.  The halves never synchronise with each other; the K
    // segment waves of one tile hand over their Poly1305 sums through LDS slots
    // guarded by per-wave generation flags.
    //
    // Dynamic deal (every class unsegmented, 8-wave workgroups): the two halves of a SIMD are not
    // served evenly -- the older wave wins VALU issue, finishes its static share at ~60 % of the
    // launch and leaves the younger one alone on the SIMD (one wave: no latency hiding, half-rate
    // v_mad_u64_u32) for the rest (tools/stamps.py at config 4: wave ends 0.73 / 1.21 ms).  So the
    // workgroup's tiles -- the same ones the static deal gives its two halves, in the same order --
    // are taken by whichever of its waves is free, from one LDS counter: item c is round c / 8,
    // half (c / 4) % 2, tile c % 4 of that group.  With segments (K > 1) the waves of a half work
    // on one tile together and keep the static deal.
    const Sched sc = make_sched(tp, n);
    const uint32_t halves = blockDim.x / 256; // 1 when the host launched 4-wave workgroups
    const uint32_t S = halves * gridDim.x;
    const uint32_t my_slot = half == 0 ? blockIdx.x : S - 1 - blockIdx.x;
    const uint32_t rounds = (sc.total_groups + S - 1) / S;
    // (empty buckets carry a K of their own class size: only the buckets holding packets count -- round 5
    // asked every lane, so a planned batch never took the dynamic deal)
    const bool dyn = halves == 2 && __ballot(sc.cnt > 0 && sc.K > 1) == 0; // same in every wave
    // From eight deal rounds on, the last eighth of them goes to a pool shared by the whole
    // grid: the XCDs do not run at one rate (per-CU finish times at config 4 spread by 8 %, by XCD), so
    // the workgroups that run out of their own tiles first take these, one tile per device-scope atomic
    // on tp.gq[0], requested one tile ahead.  Measured: config 5 on one GPU (64 rounds) +1.5 %, config 4
    // (8 rounds) +0.7 % (with each draw waited for on the spot, config 4 lost 1 %).  Below eight rounds
    // (unmeasured: one pooled round would be half or a third of the tiles) every tile stays local.
    const uint32_t R = (dyn && tp.gq && rounds >= kPoolMinRounds) ? max(1u, rounds / 8) : 0u;
    const uint32_t rounds_local = rounds - R;
    const uint32_t pool = R ? (sc.total_groups - rounds_local * S) * 4u : 0u; // tiles in the global pool
    bool pooled = false, gq_pending = false;
    uint32_t gq_next = 0; // lane 0: the next pool item
    uint32_t next_v = 0; // the next local item, requested one item ahead (LDS atomic, lane 0)
    if (dyn && lane == 0) next_v = atomicAdd(f_next, 1u);
    uint32_t gen = 0, round_s = 0;
    for (;;) {
        uint32_t g, thw; // group, and this wave's tile (segment) slot in it
        if (dyn && !pooled) {
            const uint32_t item = uniform_u32(__shfl((int)next_v, 0));
            const uint32_t r = item >> 3;
            if (r >= rounds_local) {
                if (pool == 0) break;
                pooled = true;
                continue;
            }
            if (lane == 0) next_v = atomicAdd(f_next, 1u);
            const uint32_t sl = ((item >> 2) & 1u) == 0 ? blockIdx.x : S - 1 - blockIdx.x;
            g = r * S + ((r & 1) ? S - 1 - sl : sl);
            thw = item & 3u;
        } else if (dyn) {
            // the first draw waits for its atomic; later ones were requested one tile ahead (an atomic
            // still in flight only makes the tile's exact vmcnt waits wait for it too, never less)
            if (!gq_pending && lane == 0)
                gq_next = __hip_atomic_fetch_add(tp.gq, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const uint32_t item = uniform_u32(__shfl((int)gq_next, 0));
            gq_pending = false;
            if (item >= pool) break;
            if (lane == 0) { // requested one tile ahead (waiting for each draw on the spot: config 4 -1 %)
                gq_next = __hip_atomic_fetch_add(tp.gq, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            gq_pending = true;
            g = rounds_local * S + (item >> 2);
            thw = item & 3u;
        } else {
            if (round_s >= rounds) break;
            g = round_s * S + ((round_s & 1) ? S - 1 - my_slot : my_slot);
            thw = hw;
            ++round_s;
        }
        if (g >= sc.total_groups) continue; // uniform over the half (static deal: the last round only)
        ++gen;
        if constexpr (STAMP) {
            const uint64_t t = stamp();
            t_tail += t - t_mark;
            t_mark = t;
            if (pooled) ++n_pool;
        }
        // ---- which bucket / tile / segment this wave works on (wave-uniform)
        const uint32_t pb = (uint32_t)__popcll(__ballot(sc.g_end <= g)); // buckets fully before g
        const uint32_t cls = uniform_u32(__shfl(sc.cls, pb));
        const uint32_t cnt = uniform_u32(__shfl(sc.cnt, pb));
        const uint32_t K = uniform_u32(__shfl(sc.K, pb));
        const uint32_t g0 = pb == 0 ? 0u : uniform_u32(__shfl(sc.g_end, pb - 1));
        const uint32_t tiles_per_group = 4 / K;
        const uint32_t tile = (g - g0) * tiles_per_group + thw / K;
        const uint32_t seg = thw % K;
        const uint32_t slot = tile * 64 + lane;
        const bool live = slot < cnt;
        const uint32_t i = live ? (tp.counts ? tp.lists[(uint64_t)cls * tp.cap + slot] : slot) : 0u;

        // ---- per-lane packet setup and validation (same order as the reference)
        rg_pkt_desc d = {0, 0, 0};
        if (live) d = OPEN ? oa.desc[i] : sa.desc[i];
        uint8_t st = 0xFF;
        uint32_t P = 0;
        uint64_t ctr = 0;
        if (live) {
            if constexpr (!OPEN) {
                P = d.len;
                const bool ok = d.key_idx < sa.nkeys && (P & 15u) == 0 && (d.offset & 15u) == 0 &&
                                P <= kMaxPayload && d.offset <= buf_len && P + 32 <= buf_len - d.offset;
                if (!ok) st = d.key_idx == RG_KEY_SKIP ? RG_PKT_REJECTED : RG_PKT_INVALID;
                else ctr = sa.counters[i];
            } else {
                const uint32_t W = d.len;
                if (d.key_idx == RG_KEY_SKIP) st = RG_PKT_REJECTED;
                else if ((d.offset & 15u) != 0) st = RG_PKT_UNALIGNED;              // lib.rs:613-615
                else if (d.key_idx >= oa.nkeys || W > kMaxPayload + 32 || d.offset > buf_len ||
                         W > buf_len - d.offset || W < 4)
                    st = RG_PKT_INVALID;
                if (st == 0xFF) {
                    const uint4 hdr = *reinterpret_cast<const uint4 *>(buf + d.offset);
                    if (hdr.x != 4u) st = hdr.x - 1u < 3u ? RG_PKT_NOT_DATA : RG_PKT_INVALID; // lib.rs:621-628
                    else if ((W & 15u) != 0 || W < 16) st = RG_PKT_INVALID;             // types/lib.rs:181-196
                    else {
                        ctr = ((uint64_t)hdr.w << 32) | hdr.z;
                        if (W < 32) st = RG_PKT_DECRYPT_ERR;                            // prim.rs:427-429
                    }
                }
                if (st == 0xFF) P = W - 32;
            }
        }
        const bool work = live && st == 0xFF;
        const uint32_t nb = work ? P >> 4 : 0; // 16-byte blocks of the packet
        const uint32_t C = (nb + 3) >> 2;      // 64-byte chunks
        const uint32_t L = (C + K - 1) / K;    // segment length in chunks
        const uint32_t c0 = seg * L < C ? seg * L : C;
        const uint32_t c1 = c0 + L < C ? c0 + L : C;
        const uint32_t b0 = 4 * c0;
        const uint32_t b1 = 4 * c1 < nb ? 4 * c1 : nb;
        const uint32_t snb = b1 - b0;     // blocks of this segment
        const uint32_t segC = c1 - c0;
        // ---- tile addressing: buffer descriptor based at the 128-byte line of the lowest frame
        uint64_t lo = work ? d.offset : ~0ull;
#pragma unroll
        for (int m = 32; m >= 1; m >>= 1) {
            const uint64_t o = __shfl_xor(lo, m);
            lo = o < lo ? o : lo;
        }
        lo = uniform_u64(lo);
        if (lo == ~0ull) lo = 0;
        lo &= ~127ull;
        const uint64_t span_cap = buf_len - lo;
        const uint32_t nrec = span_cap > kOOB ? kOOB : (uint32_t)span_cap;
        const v4i rsrc = make_rsrc(buf + lo, nrec);
        const bool addressable = work && d.offset - lo + 16 + (uint64_t)P <= nrec;
        const uint32_t myC = addressable ? segC : 0;
        // Window phase: windows are PPW 16-byte pieces that start SH pieces before the segment's
        // first payload block.  When every lane's segment starts at the same phase inside a
        // PPW-piece line (fixed-stride frames: payload at +16 of a 128-byte aligned frame gives
        // SH = 1), SH is that phase and every window is whole 128-byte lines: each line is
        // fetched and written once.  Otherwise SH = 0 (windows follow the payload; lines at
        // window seams are fetched by two windows).
        const uint32_t ph = (uint32_t)((d.offset + 16 + 64ull * c0) >> 4) & (PPW - 1);
        uint32_t ph_lo = myC ? ph : PPW, ph_hi = myC ? ph : 0u;
#pragma unroll
        for (int m = 32; m >= 1; m >>= 1) {
            ph_lo = min(ph_lo, (uint32_t)__shfl_xor((int)ph_lo, m));
            ph_hi = max(ph_hi, (uint32_t)__shfl_xor((int)ph_hi, m));
        }
        const uint32_t SH = uniform_u32(ph_lo == ph_hi ? ph_lo : 0u);
        // window base of the segment relative to the descriptor (kOOB if unusable): the payload
        // base minus SH pieces, never below the tile's line base (SH > 0 is the lane's own phase)
        const uint32_t my_base = addressable ? (uint32_t)(d.offset - lo) + 16 + 64 * c0 - 16 * SH : kOOB;
        uint32_t Wl = myC ? (SH + snb + PPW - 1) / PPW : 0u;
#pragma unroll
        for (int m = 32; m >= 1; m >>= 1) {
            const uint32_t o = __shfl_xor(Wl, m);
            Wl = o > Wl ? o : Wl;
        }
        const uint32_t W = uniform_u32(Wl);
        // DMA/store address table: instruction q serves lane pq = q*PKT_PER_INST + lane/PPW,
        // piece k = (lane % PPW) ^ swz(pq) of each window; that piece is payload block
        // PPW w + k - SH of the segment, valid iff tlo <= PPW w < thi
        uint32_t tb[PPW], tlo[PPW], thi[PPW];
#pragma unroll
        for (uint32_t q = 0; q < PPW; ++q) {
            const uint32_t pq = q * Cfg::PKT_PER_INST + lane / PPW;
            const uint32_t k = (lane % PPW) ^ swz<G>(pq);
            const uint32_t b = __shfl(my_base, pq);
            const uint32_t blocks = __shfl(myC == 0 ? 0u : snb, pq);
            tb[q] = b == kOOB ? kOOB : b + 16 * k;
            tlo[q] = SH > k ? SH - k : 0u;
            thi[q] = blocks + SH > k ? blocks + SH - k : 0u;
        }
        // ---- key and one-time Poly1305 key (block 0)
        const uint32_t n1 = (uint32_t)ctr, n2 = (uint32_t)(ctr >> 32);
        const Key8 key = load_key(OPEN ? oa.keys : sa.keys, work ? d.key_idx : 0u);
        const Stream stm = make_stream(key, 0u, n1, n2);
        uint32_t ks[16];
        stream_block(stm, 0, ks);
        const Mul r = make_mul(ks[0], ks[1], ks[2], ks[3]);
        const uint32_t s0 = ks[4], s1 = ks[5], s2 = ks[6], s3 = ks[7];
        Acc acc = {0, 0, 0, 0, 0};

        auto voff_of = [&](uint32_t q, uint32_t w) -> uint32_t {
            return (tb[q] != kOOB && w * PPW >= tlo[q] && w * PPW < thi[q]) ? tb[q] + w * PPW * 16 : kOOB;
        };
        auto issue_dma = [&](uint32_t w) {
            const uint32_t lbase = lds_wave + (w & 1) * Cfg::BUF;
#pragma unroll
            for (uint32_t q = 0; q < PPW; ++q) dma16(rsrc, voff_of(q, w), uniform_u32(lbase + q * 1024));
        };
        auto store_window = [&](uint32_t w) {
            const uint4 *win = lds4 + (w & 1) * (Cfg::BUF / 16);
            uint4 v[PPW];
#pragma unroll
            for (uint32_t q = 0; q < PPW; ++q) v[q] = win[q * 64 + lane];
#pragma unroll
            for (uint32_t q = 0; q < PPW; ++q) store16(rsrc, voff_of(q, w), v[q]);
        };
        if constexpr (STAMP) {
            const uint64_t t = stamp();
            t_setup += t - t_mark;
            t_mark = t;
        }
        // ---- chunk loop, software-pipelined: the keystream block of chunk c+1
        // is generated in the same basic block as the XOR / Poly1305 of chunk c
        // iterations: the longest segment of the wave (the last window may be partial)
        uint32_t Cl = myC, Cs = myC;
#pragma unroll
        for (int m = 32; m >= 1; m >>= 1) {
            const uint32_t o = __shfl_xor(Cl, m), p = __shfl_xor(Cs, m);
            Cl = o > Cl ? o : Cl;
            Cs = p < Cs ? p : Cs;
        }
        const uint32_t Cmax = uniform_u32(Cl);
        // chunks c with c + 1 < Cmin are whole (four blocks) in every lane: their Poly1305 blocks need no
        // predicate (20 v_cndmask per chunk fewer)
        const uint32_t Cmin = uniform_u32(Cs);
        const uint32_t f = swz<G>(lane);
        // segments after the first also track q = r^{blocks absorbed} (one
        // more clamped multiply per block) for the combine below
        Acc pw = {1, 0, 0, 0, 0};
        auto run_chunks = [&](auto track_tag, auto whole_tag) {
        constexpr bool TRACK = decltype(track_tag)::value;
        // WHOLE: every lane has the wave's Cmax chunks, so every chunk before the last is whole in every
        // lane and absorbs its blocks unpredicated (a loop of its own: one body, no per-chunk choice)
        constexpr bool WHOLE = decltype(whole_tag)::value;
        uint32_t ksc[16];
        if (Cmax > 0) stream_block(stm, c0 + 1, ksc);
        // Window schedule (wave-uniform): DMA(0), DMA(1) up front; before chunk c, wait for the
        // highest window it touches; after it, each window the next chunk no longer touches is
        // stored and its buffer refilled with the window two ahead.  Issue order is therefore
        // D0 D1 S0 D2 S1 D3 ..., so the ops younger than D(w) when it is awaited are none, or
        // S(w-1) and D(w+1) once window w-1 has been released.
        int have = -1;     // highest window whose DMA has been awaited
        uint32_t low = 0;  // lowest window still held in LDS
        if (W > 0) {
            issue_dma(0);
            if (W > 1) issue_dma(1);
        }
        for (uint32_t c = 0; c < Cmax; ++c) {
            const uint32_t g0 = 4 * c + SH; // window-sequence piece of the chunk's first block
            const uint32_t need = min((g0 + 3) / PPW, W - 1);
            if constexpr (STAMP) {
                const uint64_t t = stamp();
                t_chunk += t - t_mark;
                t_mark = t;
            }
            while (have < (int)need) {
                ++have;
                const uint32_t w = (uint32_t)have;
                const uint32_t younger = w == 0 ? (W > 1 ? PPW : 0u) : (low >= w ? (w + 1 < W ? 2 * PPW : PPW) : 0u);
                if (younger == 0) wait_vm<0>();
                else if (younger == PPW) wait_vm<PPW>();
                else wait_vm<2 * PPW>();
            }
            if constexpr (STAMP) {
                const uint64_t t = stamp();
                t_wait += t - t_mark;
                t_mark = t;
            }
            // blocks of this chunk that belong to the segment (0..4)
            const uint32_t cnt4 = c < myC ? (snb - 4 * c < 4 ? snb - 4 * c : 4) : 0;
            auto slot_of = [&](uint32_t g) -> uint32_t {
                return ((g / PPW) & 1) * (Cfg::BUF / 16) + lane * PPW + ((g % PPW) ^ f);
            };
            const uint32_t sl0 = slot_of(g0), sl1 = slot_of(g0 + 1), sl2 = slot_of(g0 + 2), sl3 = slot_of(g0 + 3);
            const uint4 m0 = lds4[sl0], m1 = lds4[sl1], m2 = lds4[sl2], m3 = lds4[sl3];
            if (c + 1 == Cmax) { // last chunk: no next keystream block to overlap with
                const uint4 x0 = xor4(m0, ksc + 0), x1 = xor4(m1, ksc + 4), x2 = xor4(m2, ksc + 8),
                            x3 = xor4(m3, ksc + 12);
                lds4[sl0] = x0;
                lds4[sl1] = x1;
                lds4[sl2] = x2;
                lds4[sl3] = x3;
                acc_block_pred(acc, OPEN ? m0 : x0, r, cnt4 > 0);
                acc_block_pred(acc, OPEN ? m1 : x1, r, cnt4 > 1);
                acc_block_pred(acc, OPEN ? m2 : x2, r, cnt4 > 2);
                acc_block_pred(acc, OPEN ? m3 : x3, r, cnt4 > 3);
                if constexpr (TRACK) {
                    acc_mul_pred(pw, r, cnt4 > 0);
                    acc_mul_pred(pw, r, cnt4 > 1);
                    acc_mul_pred(pw, r, cnt4 > 2);
                    acc_mul_pred(pw, r, cnt4 > 3);
                }
            } else {
                // XOR + write-back after double round 0, Poly1305 blocks after 1, 3, 5, 7
                uint4 x0, x1, x2, x3;
                uint32_t ksn[16];
                auto body = [&](auto full_tag) {
                    constexpr bool FULL = decltype(full_tag)::value;
                    stream_block_hooked(stm, c0 + c + 2, ksn, [&](int dr) {
                        if (dr == 0) {
                            x0 = xor4(m0, ksc + 0);
                            x1 = xor4(m1, ksc + 4);
                            x2 = xor4(m2, ksc + 8);
                            x3 = xor4(m3, ksc + 12);
                            lds4[sl0] = x0; // pieces outside the payload are never stored
                            lds4[sl1] = x1;
                            lds4[sl2] = x2;
                            lds4[sl3] = x3;
                        }
                        if constexpr (FULL) {
                            if (dr == 1) acc_block(acc, OPEN ? m0 : x0, r);
                            if (dr == 3) acc_block(acc, OPEN ? m1 : x1, r);
                            if (dr == 5) acc_block(acc, OPEN ? m2 : x2, r);
                            if (dr == 7) acc_block(acc, OPEN ? m3 : x3, r);
                        } else {
                            if (dr == 1) acc_block_pred(acc, OPEN ? m0 : x0, r, cnt4 > 0);
                            if (dr == 3) acc_block_pred(acc, OPEN ? m1 : x1, r, cnt4 > 1);
                            if (dr == 5) acc_block_pred(acc, OPEN ? m2 : x2, r, cnt4 > 2);
                            if (dr == 7) acc_block_pred(acc, OPEN ? m3 : x3, r, cnt4 > 3);
                        }
                        if (dr % 2 == 1) pin_acc(acc);
                        if constexpr (TRACK) {
                            if constexpr (FULL) {
                                if (dr == 2) acc_mul(pw, r);
                                if (dr == 4) acc_mul(pw, r);
                                if (dr == 6) acc_mul(pw, r);
                                if (dr == 8) acc_mul(pw, r);
                            } else {
                                if (dr == 2) acc_mul_pred(pw, r, cnt4 > 0);
                                if (dr == 4) acc_mul_pred(pw, r, cnt4 > 1);
                                if (dr == 6) acc_mul_pred(pw, r, cnt4 > 2);
                                if (dr == 8) acc_mul_pred(pw, r, cnt4 > 3);
                            }
                            if (dr % 2 == 0 && dr > 0) pin_acc(pw);
                        }
                    });
                };
                // (seal only: the open kernel's second copy of the body spilled 9 more VGPRs)
                if constexpr (WHOLE) body(std::true_type{});
                else if (!OPEN && c + 1 < Cmin) body(std::true_type{});
                else body(std::false_type{});
#pragma unroll
                for (int t = 0; t < 16; ++t) ksc[t] = ksn[t];
            }
            if constexpr (STAMP) {
                const uint64_t t = stamp();
                t_chunk += t - t_mark;
                t_mark = t;
            }
            // release the windows the next chunk does not touch (all of them after the last)
            const uint32_t next_low = c + 1 < Cmax ? (g0 + 4) / PPW : W;
            if (c + 1 == Cmax && (int)W - 1 > have) wait_vm<0>(); // never store a window in flight
            while (low < next_low) {
                store_window(low);
                if (low + 2 < W) issue_dma(low + 2);
                ++low;
            }
            if constexpr (STAMP) {
                const uint64_t t = stamp();
                t_store += t - t_mark;
                t_mark = t;
            }
        }
        };
        const bool track = K > 1 && seg > 0; // wave-uniform
        const bool whole = Cmin == Cmax; // wave-uniform
        if (track) {
            if (whole) run_chunks(std::true_type{}, std::true_type{});
            else run_chunks(std::true_type{}, std::false_type{});
        } else {
            if (whole) run_chunks(std::false_type{}, std::true_type{});
            else run_chunks(std::false_type{}, std::false_type{});
        }
        if constexpr (STAMP) {
            const uint64_t t = stamp();
            t_chunk += t - t_mark;
            t_mark = t;
        }
        wait_vm<0>(); // this tile's stores drained before the tail touches the frames
        if (work && !addressable) {
            // frame outside the tile's 32-bit buffer window (tiles of far-apart
            // frames, e.g. mixed sizes in arenas > 4 GiB): same segment, direct
            // 16-byte global accesses
            uint4 *pl = reinterpret_cast<uint4 *>(buf + d.offset + 16);
            for (uint32_t c = c0; c < c1; ++c) {
                const uint32_t hi = 4 * c + 4 < nb ? 4 * c + 4 : nb;
                stream_block(stm, c + 1, ks);
                for (uint32_t q = 4 * c; q < hi; ++q) {
                    const uint4 m = pl[q];
                    const uint4 x = xor4(m, ks + 4 * (q - 4 * c));
                    pl[q] = x;
                    acc_block(acc, OPEN ? m : x, r);
                    if (track) acc_mul(pw, r);
                }
            }
        }

        // ---- segments: h = sum_j A_j r^{N_j}, summed by segment 0.
        // Hand-off protocol per wave slot w (hw > 0) and generation gen:
        //   segment j > 0 : wait ack[w] == gen-1, write (A_j, q_j) to the slot, ready[w] = gen
        //   segment 0     : wait ready[w+s] == gen, read, ..., ack[w+s] = gen
        //                   (open: after writing the verdict into row 10 of the slot)
        //   no hand-off   : wait ack[w] == gen-1, then ready[w] = ack[w] = gen
        // so every slot's flags advance by exactly one per generation.
        uint32_t *const mine = comb + wave * kSlotRows * 64;
        bool bad = false;
        if (hw > 0 && !dyn) {
            while (f_ack[wave] != gen - 1) __builtin_amdgcn_s_sleep(1);
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            if (K > 1 && seg > 0) {
                mine[0 * 64 + lane] = acc.h0;
                mine[1 * 64 + lane] = acc.h1;
                mine[2 * 64 + lane] = acc.h2;
                mine[3 * 64 + lane] = acc.h3;
                mine[4 * 64 + lane] = acc.h4;
                mine[5 * 64 + lane] = pw.h0;
                mine[6 * 64 + lane] = pw.h1;
                mine[7 * 64 + lane] = pw.h2;
                mine[8 * 64 + lane] = pw.h3;
                mine[9 * 64 + lane] = pw.h4;
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup"); // slot written before the flag
                if (lane == 0) f_ready[wave] = gen;
            } else if (lane == 0) {
                f_ready[wave] = gen;
                f_ack[wave] = gen;
            }
        }
        if (K > 1 && seg == 0) {
            // Horner over the segments: h = (..(A_0 q_1 + A_1) q_2 + ..) + A_{K-1}
            for (uint32_t s = 1; s < K; ++s) {
                while (f_ready[wave + s] != gen) __builtin_amdgcn_s_sleep(1);
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
                const uint32_t *o = comb + (wave + s) * kSlotRows * 64;
                const Acc a = {o[0 * 64 + lane], o[1 * 64 + lane], o[2 * 64 + lane], o[3 * 64 + lane],
                               o[4 * 64 + lane]};
                const Acc q = {o[5 * 64 + lane], o[6 * 64 + lane], o[7 * 64 + lane], o[8 * 64 + lane],
                               o[9 * 64 + lane]};
                acc_mul_gen(acc, make_gen(q));
                acc_add_acc(acc, a);
                acc_fold(acc);
            }
            if constexpr (!OPEN) {
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup"); // slots read before the ack
                if (lane == 0)
                    for (uint32_t s = 1; s < K; ++s) f_ack[wave + s] = gen;
            }
        }
        // ---- tail on segment 0: length block, finish, header/tag or verify
        uint32_t tag[4] = {0, 0, 0, 0};
        uint8_t *frame = buf + d.offset;
        if (seg == 0 && live) {
            if (st != 0xFF) {
                if constexpr (!OPEN) {
                    if (sa.status) sa.status[i] = st;
                } else {
                    oa.status[i] = st;
                    if (oa.counters_out) oa.counters_out[i] = ctr;
                }
            } else {
                acc_add(acc, 0, 0, P, 0, 1); // le64(aad_len = 0) || le64(P)
                acc_mul(acc, r);
                acc_finish(acc, s0, s1, s2, s3, tag);
                if constexpr (!OPEN) {
                    if (sa.receivers)
                        *reinterpret_cast<uint4 *>(frame) = make_uint4(4u, sa.receivers[d.key_idx], n1, n2);
                    *reinterpret_cast<uint4 *>(frame + 16 + P) = make_uint4(tag[0], tag[1], tag[2], tag[3]);
                    if (sa.status) sa.status[i] = RG_PKT_OK;
                } else {
                    const uint4 want = *reinterpret_cast<const uint4 *>(frame + 16 + P);
                    const uint32_t diff =
                        (tag[0] ^ want.x) | (tag[1] ^ want.y) | (tag[2] ^ want.z) | (tag[3] ^ want.w);
                    bad = diff != 0;
                    oa.status[i] = bad ? RG_PKT_DECRYPT_ERR : RG_PKT_OK;
                    if (oa.counters_out) oa.counters_out[i] = ctr;
                }
            }
        }
        if constexpr (OPEN) {
            // forged / corrupt: every segment re-applies its keystream so the frame is unchanged
            if (K > 1) {
                if (seg == 0) {
                    for (uint32_t s = 1; s < K; ++s) comb[(wave + s) * kSlotRows * 64 + 10 * 64 + lane] = bad ? 1u : 0u;
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                    if (lane == 0)
                        for (uint32_t s = 1; s < K; ++s) f_ack[wave + s] = gen;
                } else {
                    while (f_ack[wave] != gen) __builtin_amdgcn_s_sleep(1);
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
                    bad = mine[10 * 64 + lane] != 0;
                }
            }
            if (__ballot(bad)) {
                // the forged segments' chunks dealt over the wave's lanes (restore_forged): a lane re-XORs
                // chunks another lane's window stores wrote, so those complete and this CU's L1 goes first
                wave_sync();
                restore_forged(bad, key, n1, n2, reinterpret_cast<uint4 *>(frame + 16) + 4 * c0, c0, snb);
            }
        }
    }
    if constexpr (STAMP) {
        const uint64_t t = stamp();
        t_tail += t - t_mark;
        uint64_t *dbg = OPEN ? oa.dbg : sa.dbg;
        if (dbg && lane == 0) {
            uint64_t *o = dbg + 8 * (blockIdx.x * 8 + wave);
            const uint64_t rt1 = realtime();
            o[0] = t_setup;
            o[1] = t_store;
            o[2] = t_issue;
            o[3] = t_wait;
            o[4] = t_chunk;
            o[5] = t_tail;
            o[6] = 1;
            o[7] = rt1 - rt0;
            // second block of rows (after gridDim.x x 8 waves): wall-clock start / end (100 MHz), the
            // wave's items and XCC_ID << 32 | HW_ID (round 6: the shard-size attribution, tools/shard_attrib.py)
            uint64_t *o2 = dbg + 8 * ((uint64_t)gridDim.x * 8 + blockIdx.x * 8 + wave);
            o2[0] = rt0;
            o2[1] = rt1;
            o2[2] = gen;
            o2[3] = ((uint64_t)(uint32_t)__builtin_amdgcn_s_getreg(0xF814) << 32) | (uint32_t)__builtin_amdgcn_s_getreg(0xF804);
            o2[6] = n_pool;
        }
    }
    if (R) {
        // the last workgroup to finish clears the pool for the next launch (every wave of every
        // workgroup has taken its last item before its workgroup counts itself done)
        __syncthreads();
        if (threadIdx.x == 0) {
            __atomic_thread_fence(__ATOMIC_SEQ_CST);
            if (__hip_atomic_fetch_add(tp.gq + 32, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1) {
                __hip_atomic_store(tp.gq, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(tp.gq + 32, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __atomic_thread_fence(__ATOMIC_SEQ_CST);
            }
        }
    }
    if (tp.counts) {
        // the last workgroup to finish clears the planner counters for the next
        // batch (every workgroup read them in make_sched before getting here)
        // and reports how many size classes the batch used (auto planning)
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

// ------------------------------------------------------------ launch
template <int G> static constexpr uint32_t tile_lds() { return StagedCfg<G>::WG_LDS; }
static_assert(StagedCfg<2>::WG_LDS <= kLdsPerCu, "8 waves of G = 2 windows must fit the LDS");

hipError_t launch_plan(const rg_pkt_desc *desc, uint32_t n, bool open, const TilePlan &tp, hipStream_t s) {
    if (n == 0) return hipSuccess;
    // counters start at zero: cleared at allocation and by the last workgroup
    // of every tile kernel (or of the planner, for the pipelined kernel) that
    // consumed them
    hipLaunchKernelGGL(plan_kernel, dim3((n + 256 * kPlanPer - 1) / (256 * kPlanPer)), dim3(256), 0, s, desc, n, open ? 1u : 0u,
                       const_cast<uint32_t *>(tp.counts), const_cast<uint32_t *>(tp.lists), tp.cap, tp.sched, tp.simds,
                       tp.sched ? tp.classes_out : nullptr);
    return hipGetLastError();
}

hipError_t launch_tiles(const SealArgs *sa, const OpenArgs *oa, int G, const TilePlan &tp, const Launch &L,
                        hipStream_t s) {
    const uint32_t n = sa ? sa->n : oa->n;
    if (n == 0) return hipSuccess;
    SealArgs a = sa ? *sa : SealArgs{};
    OpenArgs b = oa ? *oa : OpenArgs{};
    // one 8-wave workgroup per CU (the whole LDS is reserved, so placement is
    // one per CU by construction)
    uint32_t blocks = (uint32_t)(L.cus > 0 ? L.cus : 1);
    uint32_t threads = 512;
    if (!tp.counts) { // identity order: the host knows the group count
        const uint64_t k = tp.fixed_k ? tp.fixed_k : 1;
        const uint64_t groups = (((uint64_t)n + 63) / 64 * k + 3) / 4;
        if (groups <= blocks) { // at most one group per CU: 4-wave workgroups
            blocks = (uint32_t)groups;
            threads = 256;
        }
    }
    if (blocks == 0) blocks = 1;
    const uint32_t need = G == 1 ? tile_lds<1>() : tile_lds<2>();
    if (G != 1 && G != 2) return hipErrorInvalidValue;
    if (need > kLdsPerCu) return hipErrorInvalidValue;
    const uint32_t lds = kLdsPerCu;
#if RG_DIAG // stamped variants (debug mode 3): diagnostic builds only
#define RG_TILES(GG)                                                                                          \
    if (L.debug_mode == 3) {                                                                                  \
        if (sa) hipLaunchKernelGGL((tile_kernel<GG, false, true>), dim3(blocks), dim3(threads), lds, s, a, b, tp); \
        else hipLaunchKernelGGL((tile_kernel<GG, true, true>), dim3(blocks), dim3(threads), lds, s, a, b, tp);     \
    } else if (sa) RG_LAUNCH(L.done, (tile_kernel<GG, false>), dim3(blocks), dim3(threads), lds, s, a, b, tp);    \
    else RG_LAUNCH(L.done, (tile_kernel<GG, true>), dim3(blocks), dim3(threads), lds, s, a, b, tp);
#else
#define RG_TILES(GG)                                                                                          \
    if (sa) RG_LAUNCH(L.done, (tile_kernel<GG, false>), dim3(blocks), dim3(threads), lds, s, a, b, tp);       \
    else RG_LAUNCH(L.done, (tile_kernel<GG, true>), dim3(blocks), dim3(threads), lds, s, a, b, tp);
#endif
    if (G == 1) {
        RG_TILES(1)
    } else {
        RG_TILES(2)
    }
#undef RG_TILES
    return hipGetLastError();
}

hipError_t prepare_tile_kernels() {
    void *fs[] = {(void *)tile_kernel<1, false>,       (void *)tile_kernel<2, false>,
                  (void *)tile_kernel<1, true>,        (void *)tile_kernel<2, true>,
#if RG_DIAG
                  (void *)tile_kernel<1, false, true>, (void *)tile_kernel<2, false, true>,
                  (void *)tile_kernel<1, true, true>,  (void *)tile_kernel<2, true, true>
#endif
    };
    for (void *f : fs) {
        hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kLdsPerCu);
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

} // namespace rg
