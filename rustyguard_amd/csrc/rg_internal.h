// rg_internal.h -- declarations shared by the kernel TU and the C-ABI TU.
#pragma once
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
    int staged_g;   // kernel family: 0 pipelined lanes (rg_pipe.hip), 1/2 LDS-staged tiles of that window (rg_tile.hip)
};
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
struct TilePlan {
    const uint32_t *counts; // [kClasses] packets per class, then [kClasses] = finished-workgroup count
    const uint32_t *lists;  // [kClasses][cap] packet indices
    uint32_t cap;
    uint32_t target_lanes; // segment sizing: aim for this many busy lanes (0 = no splitting)
    uint32_t fixed_k;      // 0 = per class from the counts, else 1 / 2 / 4 segments for every packet
    uint32_t *classes_out; // host-mapped: number of non-empty classes of the batch (or nullptr)
};

// Planner + LDS-staged tile kernel (rg_tile.hip); exactly one of sa / oa is non-null.
hipError_t launch_plan(const rg_pkt_desc *desc, uint32_t n, bool open, const TilePlan &tp, hipStream_t s);
hipError_t launch_tiles(const SealArgs *sa, const OpenArgs *oa, int G, const TilePlan &tp, const Launch &L,
                        hipStream_t s);
hipError_t prepare_tile_kernels();
// Pipelined lane kernel (rg_pipe.hip): one packet per lane, double-buffered
// chunk loads, Poly1305 absorbed inside the next chunk's keystream rounds.
// With a plan (planner lists, rg_tile.hip): a schedule kernel picks segments per
// size class from the batch's mean work, then one wave per SIMD walks tiles of
// 64 lanes, largest class first, round robin (sched[] holds the schedule; the
// schedule kernel zeroes the planner's counts).  Without one: lane units in
// array order, grid-stride.
constexpr uint32_t kSchedWords = 128;
struct PipePlan {
    uint32_t *counts;      // [kClasses] packets per class (zeroed again by the schedule kernel)
    const uint32_t *lists; // [kClasses][cap] packet indices
    uint32_t cap;
    uint32_t *sched;       // [kSchedWords] per-batch schedule
    uint32_t *classes_out; // host-mapped: non-empty classes of the batch (or nullptr)
};
hipError_t launch_pipe(const SealArgs *sa, const OpenArgs *oa, const Launch &L, const PipePlan *plan,
                       hipStream_t s);
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
hipError_t launch_synth_fill(const rg_pkt_desc *desc, const uint32_t *inner_len, uint32_t n, uint8_t *buf,
                             uint64_t buf_len, uint64_t seed, hipStream_t s);

} // namespace rg
