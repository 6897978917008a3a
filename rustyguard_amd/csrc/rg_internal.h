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
    uint32_t nkeys;
    uint32_t n;
};

// General AEAD job for the per-message drop-in (any nonce / AAD / length).
struct GeneralJob {
    uint32_t key[8];
    uint32_t nonce[3];
    uint32_t decrypt; // 0 seal, 1 open
    uint64_t aad_off; // offsets into the job arena
    uint64_t aad_len;
    uint64_t payload_off;
    uint64_t payload_len;
    uint64_t tag_off; // seal: tag written here; open: expected tag read here
    uint32_t status;  // out: RG_PKT_OK / RG_PKT_DECRYPT_ERR
    uint32_t pad_;
};

hipError_t launch_seal(const SealArgs &a, int lanes_per_packet, hipStream_t s);
hipError_t launch_open(const OpenArgs &a, int lanes_per_packet, hipStream_t s);
hipError_t launch_general(GeneralJob *jobs, uint32_t njobs, uint8_t *arena, hipStream_t s);
hipError_t launch_synth_fill(const rg_pkt_desc *desc, const uint32_t *inner_len, uint32_t n, uint8_t *buf,
                             uint64_t buf_len, uint64_t seed, hipStream_t s);

} // namespace rg
