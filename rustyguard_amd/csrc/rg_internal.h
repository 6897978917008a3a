// rg_internal.h -- declarations shared by the kernel TU and the C-ABI TU.
#pragma once
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/rg_aead.h"

namespace rg {

// Largest payload a kernel accepts (keeps the 32-bit ChaCha block counter and
// every offset arithmetic far from overflow; WireGuard frames are <= 64 KiB).
constexpr uint32_t kMaxPayload = 1u << 20;

struct SealArgs {
    const uint32_t *keys;      // [nkeys][8] LE words
    const uint32_t *receivers; // [nkeys] or nullptr (no header written)
    const rg_pkt_desc *desc;   // [n]
    const uint64_t *counters;  // [n]
    uint8_t *buf;
    uint64_t buf_len;
    uint8_t *status; // [n] or nullptr
    uint64_t *dbg;   // diagnostics (stamp builds only), normally nullptr
    uint32_t nkeys;
    uint32_t n;
};

struct OpenArgs {
    const uint32_t *keys;
    const rg_pkt_desc *desc;
    uint8_t *buf;
    uint64_t buf_len;
    uint8_t *status;        // [n]
    uint64_t *counters_out; // [n] or nullptr
    uint64_t *dbg;          // diagnostics (stamp builds only), normally nullptr
    uint32_t nkeys;
    uint32_t n;
};

// Handshake MAC checks (rg_mac.hip)
struct MacArgs {
    const uint32_t *keys; // [nkeys][key_len / 4] LE words
    uint32_t key_len;     // 32 (mac1 key) or 16 (cookie, mac2)
    uint32_t nkeys;
    uint32_t which;       // 1 = mac1, 2 = mac2
    uint32_t n;
    const rg_pkt_desc *desc; // offset, len = whole message, key_idx or RG_KEY_SCAN
    const uint8_t *buf;
    uint64_t buf_len;
    uint8_t *status;
    uint32_t *key_out; // or nullptr
    uint32_t *key_state; // [nkeys][8] scratch: BLAKE2s state after each key block
};
hipError_t launch_mac_verify(const MacArgs &a, hipStream_t s);

// General AEAD job for the per-message drop-in (any nonce / AAD / length).
struct GeneralJob {
    uint32_t key[8];
    uint32_t nonce[3];
    uint32_t decrypt; // 0 seal, 1 open
    uint32_t xchacha; // 1: key is first replaced by HChaCha20(key, hnonce) (XChaCha20-Poly1305)
    uint32_t hnonce[4];
    uint64_t aad_off; // offsets into the job arena
    uint64_t aad_len;
    uint64_t payload_off;
    uint64_t payload_len;
    uint64_t tag_off; // seal: tag written here; open: expected tag read here
    uint32_t status;  // out: RG_PKT_OK / RG_PKT_DECRYPT_ERR
    uint32_t pad_;
};

// Launch geometry chosen by the host (rg_api.cpp): lanes per packet, CUs,
// resident 256-thread workgroups per CU (0 = plain one-shot grid).
struct Launch {
    int lanes;
    int cus;
    int wg_per_cu;
    int debug_mode; // diagnostics: 0 normal, 1/2 seal compute/memory only, 3 staged stamps
    int staged_g;   // kernel family: 0 pipelined lanes (rg_pipe.hip), 1/2 LDS-staged tiles of that window (rg_tile.hip),
                    // 3 flattened chunk stream (rg_flat.hip)
    hipEvent_t done; // recorded by the transport kernel's own dispatch (hipExtLaunchKernel's stop event: no
                     // extra queue packet; the device API's stream check, rg_api.cpp), or nullptr
};

// A transport launch, with its stop event when one is asked for: recorded as the kernel completes, by
// the dispatch itself (a separate hipEventRecord is one more queue packet between back-to-back launches:
// +3 us on an eagerly launched config-2 seal, round 6).
#define RG_LAUNCH(done, kernel, grid, block, lds, stream, ...)                                              \
    do {                                                                                                   \
        if (done) hipExtLaunchKernelGGL(kernel, grid, block, lds, stream, nullptr, done, 0u, __VA_ARGS__); \
        else hipLaunchKernelGGL(kernel, grid, block, lds, stream, __VA_ARGS__);                            \
    } while (0)
constexpr uint32_t kLdsPerCu = 160u * 1024u;

// Size-class work lists built by the planner (rg_tile.hip).  counts == nullptr:
// identity order (packet i in tile i / 64), one segment count fixed_k for all.
constexpr uint32_t kClasses = 37;
// class c: c chunks for c <= 16; above, upper bounds 24, 32, 48, 64, ..., 16384
__host__ __device__ __forceinline__ uint32_t class_hi(uint32_t c) {
    if (c <= 16) return c;
    const uint32_t j = c - 17;
    return (j & 1u) ? (1u << (j / 2 + 5)) : (3u << (j / 2 + 3));
}
// size class of a packet of `chunks` 64-byte chunks (the planner's lists; the flattened kernel's deal)
__device__ __forceinline__ uint32_t class_of(uint32_t chunks) {
    if (chunks <= 16) return chunks;
    uint32_t c = 17;
    while (c < kClasses - 1 && class_hi(c) < chunks) ++c;
    return c;
}

struct TilePlan {
    const uint32_t *counts; // [kClasses] packets per class, then [kClasses] = finished-workgroup count
    const uint32_t *lists;  // [kClasses][cap] packet indices
    uint32_t cap;
    uint32_t target_lanes; // segment sizing: aim for this many busy lanes (0 = no splitting)
    uint32_t fixed_k;      // 0 = per class from the counts, else 1 / 2 / 4 segments for every packet
    uint32_t *classes_out; // host-mapped: number of non-empty classes of the batch (or nullptr)
    uint32_t *sched;       // pipelined kernel: the planner also writes its schedule here (else nullptr)
    uint32_t simds;        // SIMDs the pipelined kernel runs on (schedule balance)
    uint32_t *gq;          // tile kernel: global pool of the last deal rounds ([0] next item, [32] workgroups
                           // done), zero between launches (the last workgroup clears it); may be nullptr
};

// Planner + LDS-staged tile kernel (rg_tile.hip); exactly one of sa / oa is non-null.
hipError_t launch_plan(const rg_pkt_desc *desc, uint32_t n, bool open, const TilePlan &tp, hipStream_t s);
hipError_t launch_tiles(const SealArgs *sa, const OpenArgs *oa, int G, const TilePlan &tp, const Launch &L,
                        hipStream_t s);
hipError_t prepare_tile_kernels();
// Pipelined lane kernel (rg_pipe.hip): one packet per lane, double-buffered
// chunk loads, Poly1305 absorbed inside the next chunk's keystream rounds.
// With a plan (planner lists, rg_tile.hip): the planner's last workgroup picks
// segments per size class by the estimated makespan (schedule_classes), then
// the waves walk tiles of 64 lanes, heaviest first, in the schedule's snake deal
// (sched[] holds the schedule; the planner zeroes its counts again).  Without
// one: lane units in array order, grid-stride.
constexpr uint32_t kSchedWords = 128;
// sched[] words: 2 total tiles, 4 + c: first tile of class c, 44 + c: log2
// segments of class c, 84 + c: packets of class c.
constexpr uint32_t kSchedStart = 4, kSchedLg = 44, kSchedCnt = 84;
static_assert(kSchedCnt + kClasses <= kSchedWords, "schedule words");

// Lane c (of each wave) owns size class c.  Segments per class: for
// a target T, the fewest (power of two) that keep a lane's slots (1
// one-time-key block + its chunks) within T.  Tiles are numbered by lane work
// w = slots (+1 for the r^N combine of split packets), heaviest first.  The
// kernel deals them in rounds of S = simds tiles, snake order (SIMD s takes
// tile s of even rounds, S-1-s of odd ones; wave slots w and w + S share a
// SIMD), so the heaviest and the lightest tiles meet on one SIMD.  The larger
// work of SIMDs 0 and S-1 is the launch's estimated makespan (it matched the
// true maximum in every mix simulated); the target is chosen among multiples of
// the batch's mean work per SIMD (1, 1.25, 1.5, 2, 3, no splitting) by the
// smallest estimate, then the least total work.  (A fixed target of the mean
// left config 3 with 1029 tiles of ~6 slots for 1024 SIMDs: five SIMDs ran two,
// 13 slots against a mean of 6.6; now at most 10, profiles/r1e_*.)
// Takes the planner's final class counts over into sched[] and zeroes them
// for the next batch.
// Called by all 256 threads of the planner's last workgroup: wave v evaluates
// candidates v and v + 4, wave 0 then writes the best one.
constexpr int kTargets = 6;
__device__ __forceinline__ void schedule_classes(uint32_t *counts, uint32_t *sched, uint32_t simds,
                                                 uint32_t *classes_out) {
    __shared__ uint32_t s_lg[kTargets][64], s_start[kTargets][64], s_est[kTargets], s_total[kTargets];
    __shared__ float s_sum[kTargets];
    const uint32_t c = threadIdx.x & 63, v = threadIdx.x >> 6;
    const uint32_t cnt =
        c < kClasses ? __hip_atomic_load(&counts[c], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0;
    const uint32_t chunks = c < kClasses ? class_hi(c) : 0;
    // Cross-lane values move by readlane (scalar) over the non-empty classes
    // and by ballots: a version with butterfly shuffle reductions (LDS
    // permutes, serially dependent) and 64-bit divisions added 4-6 us to the
    // planner; one wave evaluating all candidates ~3 us.
    const uint64_t used = __ballot(cnt > 0);
    float work = 0.0f; // lane slots with one lane per packet
    for (uint64_t m = used; m; m &= m - 1) {
        const int j = __ffsll((unsigned long long)m) - 1;
        work += (float)(uint32_t)__builtin_amdgcn_readlane((int)cnt, j) * (float)(1 + class_hi((uint32_t)j));
    }
    const uint32_t S = simds ? simds : 1;
    const float mean = work / (64.0f * (float)S);
    constexpr float kF[kTargets] = {1.0f, 1.25f, 1.5f, 2.0f, 3.0f, 0.0f}; // target = mean x f; 0: no splitting
    for (uint32_t k = v; k < (uint32_t)kTargets; k += 4) {
        const float tf = kF[k] > 0.0f ? ceilf(mean * kF[k]) : 65535.0f;
        const uint32_t target = tf < 2.0f ? 2u : tf > 65535.0f ? 65535u : (uint32_t)tf;
        uint32_t lg = 0;
        while (lg < 6 && 1 + ((chunks + (1u << lg) - 1) >> lg) > target) ++lg;
        const uint32_t tiles = cnt ? (uint32_t)((((uint64_t)cnt << lg) + 63) >> 6) : 0;
        const uint32_t w = cnt ? 1 + ((chunks + (1u << lg) - 1) >> lg) + (lg ? 1 : 0) : 0;
        // first tile: tiles of the classes ahead in (w desc, class desc) order
        uint32_t start = 0, total = 0;
        float sum = 0.0f;
        for (uint64_t m = used; m; m &= m - 1) {
            const int j = __ffsll((unsigned long long)m) - 1;
            const uint32_t wj = (uint32_t)__builtin_amdgcn_readlane((int)w, j);
            const uint32_t tj = (uint32_t)__builtin_amdgcn_readlane((int)tiles, j);
            if (wj > w || (wj == w && (uint32_t)j > c)) start += tj;
            total += tj;
            sum += (float)tj * (float)wj;
        }
        // work of SIMDs 0 and S-1 under the snake deal: round m holds tiles
        // [mS, mS + S), SIMD s takes tile mS + s in even rounds and
        // mS + S-1-s in odd ones
        uint32_t est0 = 0, est1 = 0;
        for (uint32_t t = 0, m = 0; t < total; t += S, ++m) {
            const uint32_t a = t + (m & 1u ? S - 1 : 0), b = t + (m & 1u ? 0 : S - 1);
            const uint64_t ha = __ballot(tiles > 0 && start <= a && a < start + tiles);
            const uint64_t hb = __ballot(tiles > 0 && start <= b && b < start + tiles);
            if (ha) est0 += (uint32_t)__builtin_amdgcn_readlane((int)w, __ffsll((unsigned long long)ha) - 1);
            if (hb) est1 += (uint32_t)__builtin_amdgcn_readlane((int)w, __ffsll((unsigned long long)hb) - 1);
        }
        const uint32_t est = est0 > est1 ? est0 : est1;
        s_lg[k][c] = lg;
        s_start[k][c] = start;
        if (c == 0) {
            s_est[k] = est;
            s_sum[k] = sum;
            s_total[k] = total;
        }
    }
    __syncthreads();
    if (v != 0) return;
    uint32_t best = 0;
    for (uint32_t k = 1; k < (uint32_t)kTargets; ++k) // smallest estimate, then least total work
        if (s_est[k] < s_est[best] || (s_est[k] == s_est[best] && s_sum[k] < s_sum[best])) best = k;
    if (c < kClasses) {
        __hip_atomic_store(&counts[c], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        sched[kSchedStart + c] = s_start[best][c];
        sched[kSchedLg + c] = s_lg[best][c];
        sched[kSchedCnt + c] = cnt;
    }
    if (c == 0) {
        sched[2] = s_total[best];
        if (classes_out) *reinterpret_cast<volatile uint32_t *>(classes_out) = (uint32_t)__popcll(used);
    }
}

struct PipePlan {
    uint32_t *counts;      // [kClasses] packets per class (zeroed again by the planner's last workgroup)
    const uint32_t *lists; // [kClasses][cap] packet indices
    uint32_t cap;
    uint32_t *sched;       // [kSchedWords] per-batch schedule
    uint32_t *classes_out; // host-mapped: non-empty classes of the batch (or nullptr)
    uint32_t simds;        // S of the schedule: waves w and w + S share a SIMD (grid = S x passes waves)
};
hipError_t launch_pipe(const SealArgs *sa, const OpenArgs *oa, const Launch &L, const PipePlan *plan,
                       hipStream_t s);

// Flattened chunk-stream kernel (rg_flat.hip, kernel family 3): units of
// whole packets, one per wave, cut inside groups of kFlatGroup packets at equal
// work (balance) or equal packet counts; the chunks of a unit are dealt evenly
// over the wave's 64 lanes.
constexpr uint32_t kFlatGroup = 1024;
hipError_t launch_flat(const SealArgs *sa, const OpenArgs *oa, bool balance, uint4 *junk, int cus, hipStream_t s,
                       hipEvent_t done = nullptr);
uint32_t flat_junk_bytes(int cus);
hipError_t prepare_flat_kernels();
hipError_t prepare_pipe_kernels(int max_wg[2]); // [seal, open] resident 256-thread workgroups per CU
// Receiver resolution pre-pass (rg_kernels.hip): out[i] = desc[i] with key_idx
// taken from the frame header's receiver through the rx table (see
// rg_open_batch_dev_rx); key_out may be nullptr.
hipError_t launch_rx_resolve(const rg_pkt_desc *desc, uint32_t n, const uint8_t *buf, uint64_t buf_len,
                             const rg_rx_entry *table, uint32_t cap, rg_pkt_desc *out, uint32_t *key_out,
                             hipStream_t s);
__host__ __device__ __forceinline__ uint32_t rx_slot(uint32_t receiver, uint32_t cap) {
    return cap > 1 ? (receiver * 0x9E3779B1u) >> (32 - __builtin_ctz(cap)) : 0u;
}
hipError_t launch_general(GeneralJob *jobs, uint32_t njobs, uint8_t *arena, hipStream_t s);
// device-resident session batches (rg_api.cpp): bind each packet to its key row; gather the
// frames the host's anti-replay pass rejected into a re-seal list (len W -> P = W - 32)
hipError_t launch_bind_keys(const rg_pkt_desc *in, const uint32_t *key_idx, uint32_t n, rg_pkt_desc *out,
                            hipStream_t s);
hipError_t launch_undo_gather(const rg_pkt_desc *rd, const uint64_t *ctr, const uint32_t *idx, uint32_t m,
                              rg_pkt_desc *out, uint64_t *ctr_out, hipStream_t s);
hipError_t launch_synth_fill(const rg_pkt_desc *desc, const uint32_t *inner_len, uint32_t n, uint8_t *buf,
                             uint64_t buf_len, uint64_t seed, hipStream_t s);

// Control words of one planner (rg_api.cpp PlanBuf): the planner's class counts and finished-workgroup
// count, the pipelined kernel's schedule and the tile kernel's work pool, in one block that the preset
// pass clears before every launch that hands work from one workgroup to another.
constexpr uint32_t kCtlCounts = 0;   // [kClasses] class counts, [kClasses] finished planner / tile workgroups
constexpr uint32_t kCtlSched = 64;   // [kSchedWords] pipelined kernel's schedule
constexpr uint32_t kCtlPool = 192;   // [0] next pool item, [32] workgroups done (tile kernel)
constexpr uint32_t kCtlWords = 256;
static_assert(kCtlCounts + kClasses + 1 <= kCtlSched && kCtlSched + kSchedWords <= kCtlPool &&
                  kCtlPool + 33 <= kCtlWords, "control block layout");
// Preset pass (rg_kernels.hip), ahead of every launch whose packets are handed between workgroups (the
// planned pipelined kernel, the tile kernels): status[0, n) = RG_PKT_PENDING, so a packet the transport
// kernel never reaches cannot read as RG_PKT_OK, and ctl[0, kCtlWords) = 0 except ctl[kCtlCounts +
// kClasses] = done_init and ctl[kCtlPool] = pool_init (both 0; the test library's hand-off hooks start
// them stale).  status may be nullptr.
hipError_t launch_preset(uint8_t *status, uint32_t n, uint32_t *ctl, uint32_t done_init, uint32_t pool_init,
                         hipStream_t s);

} // namespace rg
