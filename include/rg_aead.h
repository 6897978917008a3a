/*
 * rg_aead.h -- C ABI of the MI355X (gfx950) WireGuard transport-data AEAD
 * engine.  Drop-in boundary for the reference's hot path:
 *
 *   trait CryptoPrimatives (rustyguard-crypto/src/prim.rs:74-111)
 *     fn chacha20poly1305_enc(key, nonce, aad, payload, tag)      prim.rs:82-88
 *     fn chacha20poly1305_dec(key, nonce, aad, payload, tag)      prim.rs:89-95
 *     fn xchacha20poly1305_enc / _dec (24-byte nonce)            prim.rs:97-110
 *   impl for Core (graviola 0.2.0 underneath)                     prim.rs:179-201
 *   EncryptionKey::encrypt  (counter++, nonce, seal)              prim.rs:376-399
 *   DecryptionKey::decrypt  (replay gate, open, mark_seen)        prim.rs:401-437
 *   AntiReplay::{would_accept, mark_seen}                         rustyguard-utils/src/anti_replay.rs:25-64
 *   PeerState::force_encrypt + EncryptedMetadata::frame_in_place  rustyguard-core/src/lib.rs:267-297, :450-470
 *   Sessions::recv_message / decrypt_packet                       rustyguard-core/src/lib.rs:605-681
 *
 * The per-packet trait shape would pay a PCIe round trip per packet, so the
 * primary entry points are BATCHED.  All calls are plain C: no exceptions or
 * panics cross the ABI, every function returns RG_OK (0) or a negative
 * rg_status; per-packet outcomes go to a caller-owned status array.
 *
 * Buffer contract (same for device and host variants)
 * ---------------------------------------------------
 *  buf            one byte arena holding wire frames; frame i starts at
 *                 desc[i].offset, which must be 16-byte aligned (mirrors
 *                 AlignedPacket, rustyguard-tun/src/lib.rs:21-24, and the
 *                 alignment check of rustyguard-core/src/lib.rs:613-615).
 *  frame layout   [DataHeader 16 B][payload P B][Tag 16 B]   (W = P + 32)
 *                 DataHeader = {u32 type=4, u32 receiver, u64 counter}, LE
 *                 (rustyguard-types/src/lib.rs:152-179).
 *  seal           desc[i].len = P (payload bytes, P % 16 == 0: the
 *                 assert of rustyguard-core/src/lib.rs:273-277).  The
 *                 payload is encrypted in place, the header (if receivers
 *                 != NULL) and the tag are written into the frame
 *                 (frame_in_place, lib.rs:463-469).  nonce =
 *                 00000000 || le64(counters[i]) (prim.rs:32-36), AAD empty.
 *  open           desc[i].len = W (whole frame).  The counter is read from
 *                 the header, the tag from the last 16 bytes; on success the
 *                 payload is decrypted in place.  On any failure the frame is
 *                 left byte-for-byte unchanged.
 *  keys           key table, nkeys rows of 32 bytes; desc[i].key_idx picks
 *                 the row (one row per session direction).
 *  frames         the frames of one call must not overlap (each is its own
 *                 datagram, as in the reference); they may come in any order.
 */
#ifndef RG_AEAD_H
#define RG_AEAD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RG_ABI_VERSION 6

typedef struct rg_ctx rg_ctx;

/* 16-byte packet descriptor; device copies must be 16-byte aligned. */
typedef struct rg_pkt_desc {
    uint64_t offset;  /* frame offset in buf, multiple of 16 */
    uint32_t len;     /* seal: payload length P; open: frame length W */
    uint32_t key_idx; /* key-table row; RG_KEY_SKIP = leave packet untouched */
} rg_pkt_desc;

#define RG_KEY_SKIP 0xFFFFFFFFu

/* call status */
typedef enum rg_status {
    RG_OK = 0,
    RG_EINVAL = -1,  /* bad argument (null pointer, n too large, ...) */
    RG_EDEVICE = -2, /* HIP runtime error; rg_last_error() has the text */
    RG_ENOMEM = -3,
    RG_ENOTFOUND = -4,
    RG_EFULL = -5,
} rg_status;

/* per-packet status (uint8_t), numbering shared with the CPU oracle.
 * Maps onto rustyguard_core::Error (rustyguard-core/src/lib.rs:416-423). */
enum rg_pkt_status {
    RG_PKT_OK = 0,
    RG_PKT_DECRYPT_ERR = 1, /* Error::DecryptionError: tag mismatch / < 16 B after header */
    RG_PKT_INVALID = 2,     /* Error::InvalidMessage: W % 16 != 0, W < 16, message type
                               not 1-4 (lib.rs:627), bad seal desc */
    RG_PKT_REJECTED = 3,    /* Error::Rejected: replayed/too old counter, no session,
                               REJECT_AFTER_MESSAGES reached, or RG_KEY_SKIP */
    RG_PKT_UNALIGNED = 4,   /* Error::Unaligned: frame not 16-byte aligned */
    RG_PKT_NOT_DATA = 5,    /* type 1, 2 or 3 (handshake init/resp, cookie): route to the
                               handshake path (lib.rs:622-624) */
    RG_PKT_PENDING = 6,     /* no verdict: the packet was never finished (the call failed, a device
                               error, or a batch still in flight).  Never an accept. */
};

/* Statuses fail closed.  A packet reads RG_PKT_OK only after the kernel that processed it wrote that
 * verdict: every launch that hands packets from one workgroup to another (the planned pipelined kernel,
 * the tile kernels) is preceded, on the same stream, by a preset pass that sets the batch's statuses to
 * RG_PKT_PENDING and clears the planner's control words; the launches without a hand-off (the pipelined
 * kernel in array order, the flattened kernel) deal every packet to a lane by its index alone, and that
 * lane writes its status.  The host-memory calls (rg_*_batch_host*, rg_send_batch, rg_recv_batch*) check
 * after the device work that no status is still RG_PKT_PENDING (RG_EDEVICE otherwise), and every host-memory
 * call that returns an error leaves all n statuses RG_PKT_PENDING: no replay window or endpoint moves on
 * a failed batch.  rg_recv_batch_dev_finish runs the replay pass only over RG_PKT_OK / RG_PKT_DECRYPT_ERR
 * verdicts and returns RG_EDEVICE when any packet is still pending. */

/* ---------------------------------------------------------------- context */

int rg_abi_version(void);
/* Create a context bound to HIP device `device` (one per process/GPU).  Every call on a context works on
 * its device and leaves the caller's current HIP device as it found it.  Key material the context keeps
 * in device memory (the host calls' key table, the MAC key states, the per-message arena) is zeroed
 * before its memory is reused or freed, in stream order: behind the launches that read it, without
 * waiting for the device or for other streams (prim.rs:227-231 zeroizes keys on drop).  A call that would
 * have to regrow such a buffer while its stream is being captured into a graph fails with RG_EDEVICE.  A
 * block that a captured launch reads is never freed under the graph: a later regrow takes a new block and
 * keeps the captured one allocated until rg_destroy (rg_sessions_destroy for a session table's rows),
 * which zeroes and frees it; such a graph must not be replayed after that.  rg_create refuses (RG_EINVAL)
 * to run under ROC_SYSTEM_SCOPE_SIGNAL=0: agent-scope completion signals hung the host pipeline's waits in
 * round 5 (profiles/r5_e2e_rtenv.txt). */
int rg_create(int device, rg_ctx **out);
void rg_destroy(rg_ctx *ctx);
/* Text of the last error on this thread ("" if none). */
const char *rg_last_error(void);

/* --------------------------------------- device-resident batch (async) */
/* Every pointer is device memory; work is enqueued on `stream`
 * (hipStream_t, NULL = legacy default stream) and the call returns without
 * synchronising.  status is required (ABI 6: it is how a caller knows a packet
 * was sealed; RG_PKT_OK is written only by the lane that sealed it), receivers /
 * counters_out may be NULL.  The kernels bounds-check every descriptor against
 * buf_len and never touch memory outside [buf, buf + buf_len).  Calls on one
 * context are ordered on one stream (they share the planner buffers and the tile
 * kernel's work pool, see rg_set_plan); use a context per concurrent stream.  A
 * call on another stream while this context's last batch is still in flight on
 * its stream fails with RG_EINVAL and enqueues nothing (the check needs no
 * wait: an event query).  Launches captured into a graph are not tracked: a
 * caller that replays such a graph orders the replays against the context's
 * other calls itself (same stream, or events). */
int rg_seal_batch_dev(rg_ctx *ctx, const uint8_t *keys, const uint32_t *receivers, uint32_t nkeys,
                      const rg_pkt_desc *desc, const uint64_t *counters, size_t n, uint8_t *buf, size_t buf_len,
                      uint8_t *status, void *stream);
int rg_open_batch_dev(rg_ctx *ctx, const uint8_t *keys, uint32_t nkeys, const rg_pkt_desc *desc, size_t n,
                      uint8_t *buf, size_t buf_len, uint8_t *status, uint64_t *counters_out, void *stream);

/* ------------------------------------ device-side receiver resolution */
/* The receiver-index -> session map of Sessions::decrypt_packet
 * (rustyguard-core/src/lib.rs:646-650, `peers_by_session`) as an
 * open-addressing table: slot = (receiver * 0x9E3779B1) >> (32 - log2 cap),
 * linear probing, key_idx == RG_KEY_SKIP marks an empty slot.  Built on the
 * host (cap a power of two >= 2 n; receivers unique), used on the device. */
typedef struct rg_rx_entry {
    uint32_t receiver;
    uint32_t key_idx;
} rg_rx_entry;
int rg_rx_table_build(const uint32_t *receivers, const uint32_t *key_idx, size_t n, rg_rx_entry *table,
                      uint32_t cap);
/* host lookup: key index, or -1 when the receiver has no session */
int64_t rg_rx_table_find(const rg_rx_entry *table, uint32_t cap, uint32_t receiver);
/* rg_open_batch_dev for frames straight off the wire: desc[i].key_idx is
 * ignored; each frame's session comes from its header's receiver index through
 * rx_table (device memory), in the reference's check order -- alignment,
 * message type and 16-byte framing first (their statuses as rg_open_batch_dev),
 * then an unknown receiver is RG_PKT_REJECTED (`Error::Rejected`, lib.rs:
 * 647-650), then the AEAD.  key_idx_out (device, may be NULL) receives the
 * resolved key index (RG_KEY_SKIP when none) for the host's anti-replay pass. */
int rg_open_batch_dev_rx(rg_ctx *ctx, const uint8_t *keys, uint32_t nkeys, const rg_rx_entry *rx_table,
                         uint32_t rx_cap, const rg_pkt_desc *desc, size_t n, uint8_t *buf, size_t buf_len,
                         uint8_t *status, uint64_t *counters_out, uint32_t *key_idx_out, void *stream);

/* ----------------------------------------- handshake MAC checks (batch) */
/* HasMac::verify_mac1 / verify_mac2 (rustyguard-crypto/src/lib.rs:114-209)
 * for n handshake messages (desc: offset, len = whole message incl. both
 * macs): mac1 = BLAKE2s-128(keys[k], msg[..len-32]) against msg[len-32..
 * len-16] (which = 1, 32-byte mac1 keys), mac2 = BLAKE2s-128(cookie,
 * msg[..len-16]) against msg[len-16..] (which = 2, 16-byte cookies).
 * status: RG_PKT_OK, RG_PKT_REJECTED (mismatch: CryptoError::Rejected),
 * RG_PKT_UNALIGNED, RG_PKT_INVALID (len < 32 or outside buf).  key_idx
 * RG_KEY_SCAN tries every key and reports the first match in key_idx_out
 * (wg-proxy's peer scan, wg-proxy/src/main.rs:217-229).  Device pointers. */
#define RG_KEY_SCAN 0xFFFFFFFEu
int rg_mac_verify_batch_dev(rg_ctx *ctx, const uint8_t *keys, uint32_t key_len, uint32_t nkeys, int which,
                            const rg_pkt_desc *desc, size_t n, const uint8_t *buf, size_t buf_len, uint8_t *status,
                            uint32_t *key_idx_out, void *stream);

/* Tuning knobs.  lanes: lanes cooperating on one packet (0 = automatic, else
 * 1/2/4).  wg_per_cu: resident 256-thread workgroups per CU of the persistent
 * grid (0 = automatic, -1 = plain one-shot grid). */
int rg_set_lanes_per_packet(rg_ctx *ctx, int lanes);
int rg_get_lanes_per_packet(rg_ctx *ctx, size_t n);
int rg_set_wg_per_cu(rg_ctx *ctx, int wg_per_cu);
/* Kernel choice: -1 (default) = automatic by batch size (rg_get_kernel);
 * 0 = pipelined lane kernel (one packet -- or one of lanes_per_packet
 * contiguous segments -- per lane, 3 chunks in flight, Poly1305 folded
 * into the keystream rounds); 1/2 = LDS-staged tiles (one packet (segment) per
 * lane, coalesced LDS-DMA windows of that many 64-byte chunks); 3 = flattened
 * chunk stream (a wave takes a run of whole packets of equal total work and
 * deals their 64-byte chunks evenly over its lanes; Poly1305 partial sums are
 * combined per packet in LDS). */
int rg_set_staged(rg_ctx *ctx, int kernel);
/* The kernel family a batch of n packets runs on (0, 1 or 2; see above).  In automatic mode a
 * small batch whose sizes are mixed (the last planned batch of the same planner -- the device API's,
 * or a host pipeline slot's -- held more than one size class) runs family 3 instead, the flattened
 * chunk stream (rg_set_staged(ctx, 3) forces it); every 32nd such call re-plans on family 0. */
int rg_get_kernel(rg_ctx *ctx, size_t n);
/* The family the most recent batched launch on this context ran (-1 before any). */
int rg_last_kernel(rg_ctx *ctx);
/* A device-side planner can first sort the batch into size classes so that
 * every 64-lane tile holds packets of similar length (both kernel families;
 * the pipelined kernel then also picks segments per class by an estimated
 * makespan and deals tiles heaviest first, in snake order over the SIMDs).
 * 0 = off (tiles take packets in array order), 1 = always, 2 (default) =
 * auto: plan unless the last planned batch of this context held a single size
 * class (re-checked every 32nd call).  Results are identical in every mode.
 * Device-API calls that share a context use one set of planner buffers and one
 * tile-kernel work pool (batches of eight or more deal rounds, CUs x 4 Ki packets =
 * 1 Mi on 256 CUs, even with the planner off): two device-API launches on one
 * context on different streams are unsupported at any batch size -- issue them on
 * one stream (or order them).  The host-memory API has its own per pipeline stream. */
int rg_set_plan(rg_ctx *ctx, int on);
/* Segments per packet for the tile kernels: 0 (default) = per size class,
 * aiming at two resident waves per SIMD; 1/2/4 = split every packet into that
 * many contiguous segments on separate waves (Poly1305 partial sums combined
 * as sum_j A_j r^{N_j}). */
int rg_set_segments(rg_ctx *ctx, int segments);
/* Diagnostics.  The product library accepts only mode 0 and a NULL stamp buffer
 * (RG_EINVAL otherwise): no context of it can emit frames that are not sealed.
 * Diagnostic builds (-DRG_DIAG, tools/build_variant.sh, never shipped) add seal
 * modes whose output is NOT a valid seal -- 1 compute only (no payload
 * loads/stores), 2 memory only, 4/5/6 non-temporal loads / stores / both,
 * 7 no payload stores, 8 line stores alternating between two lines per frame
 * (pipelined kernel) -- and mode 3, per-wave stamps of the real kernels. */
int rg_set_debug_mode(rg_ctx *ctx, int mode);
/* Diagnostic builds only: per-wave s_memtime stamps are written to this device
 * buffer, 8 x u64 per wave: mode 3 on the tile kernels (setup, store,
 * dma-issue, dma-wait, chunk, tail, valid, real-time ticks at 100 MHz); any
 * non-zero mode on the pipelined kernel (cycles, two unit marks, XCC_ID << 32 |
 * HW_ID, start tick, prologue cycles, valid, real-time ticks); mode 3 on the
 * flattened kernel (s_memtime at the end of each phase) plus a second block of
 * rows after the first CUs x 4 (wall-clock start and end, the unit search's
 * steps) and a third (the first sub-unit's packets / chunks / steps, XCC_ID << 32
 * | HW_ID), so size the buffer for 3 x CUs x 4 x 8 u64 there. */
int rg_set_debug_buffer(rg_ctx *ctx, void *dev_ptr);

/* ----------------------------------------- host-memory batch (blocking) */
/* Same contract with host pointers: frames are staged H2D, sealed/opened on
 * the GPU and copied back D2H, pipelined over three streams.  Pinned memory
 * (rg_host_alloc) gives the full PCIe rate.  rg_set_host_slice sets the byte
 * span of one pipeline slice (default 8 MiB; 64 KiB .. 1 GiB).
 *
 * Every host wait of the library is bounded: a completion the device does not
 * report within rg_set_wait_timeout's limit (default 10 000 ms per wait; 1 ..
 * 3 600 000) ends the call with RG_EDEVICE ("... timed out") and every status
 * RG_PKT_PENDING, instead of blocking forever.  Waits poll (hipEventQuery),
 * yielding the CPU between polls and sleeping once a wait has run 2 ms.  The
 * transfers of a timed-out call may still complete later: until the next host
 * call on that context returns (it waits for them, bounded, and discards them),
 * the frames of the failed call's buffer can still be written back. */
int rg_set_host_slice(rg_ctx *ctx, size_t bytes);
int rg_set_wait_timeout(rg_ctx *ctx, uint32_t ms);
int rg_seal_batch_host(rg_ctx *ctx, const uint8_t *keys, const uint32_t *receivers, uint32_t nkeys,
                       const rg_pkt_desc *desc, const uint64_t *counters, size_t n, uint8_t *buf, size_t buf_len,
                       uint8_t *status);
int rg_open_batch_host(rg_ctx *ctx, const uint8_t *keys, uint32_t nkeys, const rg_pkt_desc *desc, size_t n,
                       uint8_t *buf, size_t buf_len, uint8_t *status, uint64_t *counters_out);
void *rg_host_alloc(size_t bytes);
void rg_host_free(void *p);

/* NUMA placement (a two-socket host: half the GPUs hang off each socket).  rg_numa_node: the host NUMA
 * node closest to the context's GPU (-1 unknown).  A group's worker thread for a context runs on the CPUs
 * of that node this process may use and prefers its memory for the slice buffers it allocates.  Frames
 * are the caller's: for the full link rate a caller that owns a batch's buffer (a UDP ring, say) places
 * each context's part -- rg_split_batch's bounds -- on that context's node, by first touch from a thread
 * there or with rg_numa_bind (mbind MPOL_BIND + MPOL_MF_MOVE over the pages covering [p, p + bytes)), then
 * pins it with rg_host_register (hipHostRegister; rg_host_unregister before freeing).  Pinned pages do not
 * move: bind first. */
int rg_numa_node(rg_ctx *ctx);
int rg_numa_bind(void *p, size_t bytes, int node);
int rg_host_register(void *p, size_t bytes);
int rg_host_unregister(void *p);

/* ------------------------- per-message drop-in for CryptoPrimatives */
/* Exactly Core::chacha20poly1305_enc / _dec (prim.rs:179-201): any nonce,
 * any AAD, any length, host pointers, blocking.  dec returns RG_OK, or
 * RG_PKT_DECRYPT_ERR (positive 1) on a tag mismatch with payload untouched. */
int rg_chacha20poly1305_enc(rg_ctx *ctx, const uint8_t key[32], const uint8_t nonce[12], const uint8_t *aad,
                            size_t aad_len, uint8_t *payload, size_t len, uint8_t tag[16]);
int rg_chacha20poly1305_dec(rg_ctx *ctx, const uint8_t key[32], const uint8_t nonce[12], const uint8_t *aad,
                            size_t aad_len, uint8_t *payload, size_t len, const uint8_t tag[16]);

/* Core::xchacha20poly1305_enc / _dec (prim.rs:202-224; decl :97-110), the
 * cookie-reply AEAD (encrypt_cookie / decrypt_cookie, rustyguard-crypto/src/
 * lib.rs:50-70): HChaCha20(key, nonce[0..16]) subkey, then ChaCha20-Poly1305
 * with nonce 0^4 || nonce[16..24].  Same contract as the pair above. */
int rg_xchacha20poly1305_enc(rg_ctx *ctx, const uint8_t key[32], const uint8_t nonce[24], const uint8_t *aad,
                             size_t aad_len, uint8_t *payload, size_t len, uint8_t tag[16]);
int rg_xchacha20poly1305_dec(rg_ctx *ctx, const uint8_t key[32], const uint8_t nonce[24], const uint8_t *aad,
                             size_t aad_len, uint8_t *payload, size_t len, const uint8_t tag[16]);

/* ---------------------------------------------- host-side session layer */
/* AntiReplay: RFC 6479 window, 2048-bit bitmap, WINDOW_SIZE = 1984
 * (rustyguard-utils/src/anti_replay.rs:1-64), identical semantics. */
typedef struct rg_antireplay {
    uint64_t bitmap[32];
    uint64_t last;
} rg_antireplay;
#define RG_REPLAY_WINDOW 1984u

void rg_antireplay_init(rg_antireplay *r);
int rg_antireplay_would_accept(const rg_antireplay *r, uint64_t n);
void rg_antireplay_mark_seen(rg_antireplay *r, uint64_t n);

/* Session table: the transport half of rustyguard_core::Sessions.  Each
 * session owns an EncryptionKey {key, counter} and a DecryptionKey {key,
 * AntiReplay} (prim.rs:376-437), the peer's receiver id for outgoing
 * headers, and our local id that incoming headers name
 * (rustyguard-core/src/lib.rs:230-235, :646-650). */
typedef struct rg_sessions rg_sessions;

/* REKEY_AFTER_MESSAGES / REJECT_AFTER_MESSAGES, rustyguard-core/src/lib.rs:63-65 */
#define RG_REKEY_AFTER_MESSAGES (1ull << 60)
#define RG_REJECT_AFTER_MESSAGES (0xFFFFFFFFFFFFFFFFull - (1ull << 13))

int rg_sessions_create(rg_ctx *ctx, uint32_t capacity, rg_sessions **out);
void rg_sessions_destroy(rg_sessions *s);
/* Install a transport session (HandshakeState::split output, prim.rs:299-313);
 * returns the slot index (>= 0) or a negative rg_status.  The session is its own peer
 * (its endpoint is its own); rg_sessions_insert_peer names the peer. */
int rg_sessions_insert(rg_sessions *s, uint32_t local_id, uint32_t remote_id, const uint8_t send_key[32],
                       const uint8_t recv_key[32]);
/* rg_sessions_insert for a session of peer `peer` (any caller-chosen id but RG_PEER_NONE): the
 * peer's sessions -- its current transport and the ones a rekey leaves behind -- share one endpoint
 * record, as the reference keeps peer.endpoint per peer (PeerState, rustyguard-core/src/lib.rs:
 * 160-181, set by decrypt_packet at :670-671, read by the Keepalive timer, time.rs:135).  The
 * peer's record outlives its sessions (a new session of a known peer starts with its endpoint). */
#define RG_PEER_NONE 0xFFFFFFFFu
int rg_sessions_insert_peer(rg_sessions *s, uint32_t local_id, uint32_t remote_id, const uint8_t send_key[32],
                            const uint8_t recv_key[32], uint32_t peer);
int rg_sessions_remove(rg_sessions *s, uint32_t slot);
int rg_sessions_lookup(const rg_sessions *s, uint32_t local_id); /* slot or RG_ENOTFOUND */
/* EncryptionKey::counter() (prim.rs:396-398) / overwrite, e.g. for REKEY tests */
uint64_t rg_sessions_send_counter(const rg_sessions *s, uint32_t slot);
int rg_sessions_set_send_counter(rg_sessions *s, uint32_t slot, uint64_t counter);
rg_antireplay *rg_sessions_replay(rg_sessions *s, uint32_t slot);

/* Batched PeerState::encrypt_message + frame_in_place over host frames.
 * Packets are processed in array order: each takes the next counter of its
 * session (EncryptionKey::encrypt, prim.rs:386-394) and sets its sent time.  status[i]:
 * OK, INVALID (P % 16 != 0 / bad desc), REJECTED (counter >= REJECT_AFTER_MESSAGES or
 * the session older than REJECT_AFTER_TIME, lib.rs:204-209, 260-262).  rekey_out[i]
 * (nullable) = 1 when the session counter reached REKEY_AFTER_MESSAGES (lib.rs:564-570). */
int rg_send_batch(rg_sessions *s, const uint32_t *slots, const rg_pkt_desc *desc, size_t n, uint8_t *buf,
                  size_t buf_len, uint8_t *status, uint8_t *rekey_out);
/* Batched Sessions::recv_message for data frames: alignment/type/length
 * checks, receiver-id -> session, replay pre-filter, GPU open, then the
 * in-order anti-replay post-pass (A6 in SURVEY.md §8): packet j is accepted
 * iff its tag verifies and would_accept(n_j) holds after packets 0..j-1.
 * slots_out[i] = session slot (or 0xFFFFFFFF). */
int rg_recv_batch(rg_sessions *s, const rg_pkt_desc *desc, size_t n, uint8_t *buf, size_t buf_len,
                  uint8_t *status, uint32_t *slots_out);

/* rg_recv_batch with decrypt_packet's side effects (rustyguard-core/src/lib.rs:664-679):
 * src[i] (nullable) is an opaque tag of packet i's source address; for every packet that is
 * authenticated and accepted, in array order, the session's endpoint becomes src[i] (only
 * authenticated packets move it: whitepaper §6.5, the reference's recv_message fuzz
 * invariant) and flags_out[i] (nullable) gets RG_RECV_AUTHENTICATED, plus RG_RECV_KEEPALIVE
 * when sent + KEEPALIVE_TIMEOUT < now and no keepalive is pending yet (the caller schedules
 * the Keepalive timer; rg_sessions_keepalive_due runs it).  Other packets get flags 0. */
#define RG_RECV_AUTHENTICATED 1u
#define RG_RECV_KEEPALIVE 2u
int rg_recv_batch_ex(rg_sessions *s, const rg_pkt_desc *desc, size_t n, uint8_t *buf, size_t buf_len,
                     const uint64_t *src, uint8_t *status, uint32_t *slots_out, uint8_t *flags_out);
/* The table's clock: Sessions::turn's state.now (lib.rs:396-413) as monotonic nanoseconds.
 * Sessions take it as started / sent when inserted; rg_send_batch sets sent and rejects
 * once started + REJECT_AFTER_TIME (180 s) < now (should_expire, lib.rs:207-209). */
void rg_sessions_set_time(rg_sessions *s, uint64_t now_ns);
/* the endpoint tag of the last authenticated packet of the session's peer (any of the peer's
 * sessions, rg_sessions_insert_peer; the session itself when inserted without a peer);
 * RG_ENOTFOUND before any.  rg_peer_endpoint reads a peer's record directly. */
int rg_sessions_endpoint(const rg_sessions *s, uint32_t slot, uint64_t *src_out);
int rg_peer_endpoint(const rg_sessions *s, uint32_t peer, uint64_t *src_out);
/* the Keepalive timer entry (rustyguard-core/src/time.rs:114-141): clears keepalive_pending
 * and returns 1 when sent + KEEPALIVE_TIMEOUT < now (should_keepalive, lib.rs:201-203): the
 * caller then seals an empty payload (P = 0) for the session with rg_send_batch. */
int rg_sessions_keepalive_due(rg_sessions *s, uint32_t slot);
/* rg_sessions_keepalive_due with the address the keepalive goes to: the session's peer endpoint
 * (peer.endpoint, time.rs:135) in *dst_out when due.  Returns 1 (due, *dst_out set), 0 (not
 * due), RG_ENOTFOUND (due but the peer never authenticated a packet: the reference's
 * "should not be scheduled" expect) or another negative rg_status. */
int rg_sessions_keepalive(rg_sessions *s, uint32_t slot, uint64_t *dst_out);

/* Device-resident variants of rg_send_batch / rg_recv_batch_ex: frames, descriptors and
 * statuses in device memory, the session state on the host.  Work is enqueued on `stream`
 * (hipStream_t) and the calls return without waiting for the GPU; the table keeps device
 * mirrors of its keys, receivers and a receiver-id -> session table, refreshed (after the
 * device work that reads them has drained) on the first device call after a session change.
 *
 * rg_send_batch_dev: slots[] and rekey_out[] are host arrays; desc[i].key_idx is ignored
 * (the packet's session decides it).  Counters are reserved on the host in array order as
 * rg_send_batch does; since the lengths are on the device, a frame with P % 16 != 0 still takes
 * a counter and the kernel reports it RG_PKT_INVALID (nonces stay unique).  status (device,
 * required as for rg_seal_batch_dev) gets the per-packet statuses.  Two sends may be in flight; a
 * third waits for the first one's seal. */
int rg_send_batch_dev(rg_sessions *s, const uint32_t *slots, const rg_pkt_desc *desc, size_t n, uint8_t *buf,
                      size_t buf_len, uint8_t *status, uint8_t *rekey_out, void *stream);
/* rg_recv_batch_dev enqueues receiver resolution (rg_open_batch_dev_rx), the GPU open and
 * the copy of (status, counter, session) per packet to pinned host memory; status (device)
 * gets the GPU verdicts.  rg_recv_batch_dev_finish waits for that copy, runs the in-order
 * anti-replay pass and decrypt_packet's side effects exactly as rg_recv_batch_ex (src, flags),
 * writes the final statuses back to the device status array, and re-seals frames it rejected
 * (they go back to ciphertext), all on the batch's stream; status_out / slots_out / flags_out
 * are optional host arrays.  One device receive may be pending per table: finish it before
 * the next rg_recv_batch_dev, rg_sessions_insert or rg_sessions_remove (RG_EINVAL otherwise).
 * Replayed frames are decrypted and re-sealed (the device cannot consult the window first). */
int rg_recv_batch_dev(rg_sessions *s, const rg_pkt_desc *desc, size_t n, uint8_t *buf, size_t buf_len,
                      uint8_t *status, void *stream);
int rg_recv_batch_dev_finish(rg_sessions *s, const uint64_t *src, uint8_t *status_out, uint32_t *slots_out,
                             uint8_t *flags_out);

/* ------------------------------------------- several GPUs, one thread */
/* The reference's host is one thread owning one Sessions (RefCell, rustyguard-core/src/lib.rs:
 * 349-352; send_message / recv_message :542-583, :605-681).  A group lets that one thread drive
 * several GPUs: one context per entry of devices[] (a device may repeat: several contexts on one
 * GPU).  A batch given to a group is split into contiguous index ranges of about equal AEAD work
 * (payload bytes + one 64-byte key block per packet; rg_split_batch), one per context; every
 * context's H2D -> kernel -> D2H pipeline runs on its own streams, driven by a worker thread of the
 * library per context once some part spans more than two slices (rg_set_host_slice; smaller batches,
 * and contexts whose thread cannot be started, are stepped by the calling thread itself), and the call
 * returns when all are done.  The caller's
 * current device is left as it was.  Results are those of one context: the
 * packets are independent, counters are reserved before the split (rg_send_batch)
 * and the in-order anti-replay pass runs after the gather (rg_recv_batch_ex). */
typedef struct rg_group rg_group;
int rg_group_create(const int *devices, int n, rg_group **out);
void rg_group_destroy(rg_group *g);
int rg_group_size(const rg_group *g);
rg_ctx *rg_group_ctx(rg_group *g, int i); /* the i-th context (tuning knobs, device calls); NULL if out of range */
/* The split: bounds[0] = 0 <= bounds[1] <= ... <= bounds[parts] = n, part k = [bounds[k], bounds[k+1]),
 * cut where the running work (len, minus 32 when open, + 64 per packet) crosses k / parts of the total. */
int rg_split_batch(const rg_pkt_desc *desc, size_t n, int open, int parts, size_t *bounds);
/* rg_seal_batch_host / rg_open_batch_host over the group (same arguments and results). */
int rg_seal_batch_host_multi(rg_group *g, const uint8_t *keys, const uint32_t *receivers, uint32_t nkeys,
                             const rg_pkt_desc *desc, const uint64_t *counters, size_t n, uint8_t *buf,
                             size_t buf_len, uint8_t *status);
int rg_open_batch_host_multi(rg_group *g, const uint8_t *keys, uint32_t nkeys, const rg_pkt_desc *desc, size_t n,
                             uint8_t *buf, size_t buf_len, uint8_t *status, uint64_t *counters_out);
/* Device-resident shards: shard i lives on context i's device (its own keys, descriptors, frames,
 * statuses and stream there); rg_seal_batch_dev / rg_open_batch_dev enqueued for every shard, from
 * this thread, without waiting (counters_out and receivers may be NULL as there).  Every shard's
 * arguments are checked before any shard is enqueued: RG_EINVAL names the bad shard and nothing ran.
 * A launch that fails after the checks (a device error) returns its code with rg_last_error naming
 * the shard k; shards 0..k-1 are enqueued, k and later are not. */
typedef struct rg_dev_shard {
    const uint8_t *keys;
    const uint32_t *receivers; /* seal only */
    uint32_t nkeys;
    const rg_pkt_desc *desc;
    const uint64_t *counters; /* seal only */
    size_t n;
    uint8_t *buf;
    size_t buf_len;
    uint8_t *status;
    uint64_t *counters_out; /* open only */
    void *stream;
} rg_dev_shard;
int rg_seal_batch_dev_multi(rg_group *g, const rg_dev_shard *shards);
int rg_open_batch_dev_multi(rg_group *g, const rg_dev_shard *shards);
/* A session table whose host-frame batches (rg_send_batch, rg_recv_batch[_ex]) run on the whole
 * group; the device-frame calls (rg_send_batch_dev, rg_recv_batch_dev) refuse such a table. */
int rg_sessions_create_group(rg_group *g, uint32_t capacity, rg_sessions **out);

/* ------------------------------------------------ synthetic workloads */
/* Device fill of payload bytes: inner bytes [0, inner_len[i]) of packet i
 * are le64(mix64(seed + (i << 16) + word)), bytes [inner_len, P) are zero.
 * desc/inner_len/buf are device pointers; desc[i].len = P. */
int rg_synth_fill_dev(rg_ctx *ctx, const rg_pkt_desc *desc, const uint32_t *inner_len, size_t n, uint8_t *buf,
                      size_t buf_len, uint64_t seed, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* RG_AEAD_H */
