/*
 * rg_oracle.h -- CPU restatement of RFC 8439 ChaCha20-Poly1305 as used by
 * rustyguard transport data.  TEST INFRASTRUCTURE ONLY (see rg_oracle.c).
 */
#ifndef RG_ORACLE_H
#define RG_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* same 16-byte layout as rg_pkt_desc in include/rg_aead.h */
typedef struct {
    uint64_t offset;  /* byte offset of the frame in buf */
    uint32_t len;     /* seal: payload length P; open: frame length W */
    uint32_t key_idx; /* row of the key table */
} rg_oracle_desc;

/* per-packet status, same numbering as RG_PKT_* in include/rg_aead.h */
enum {
    RG_ORACLE_OK = 0,
    RG_ORACLE_DECRYPT_ERR = 1,
    RG_ORACLE_INVALID = 2,
    RG_ORACLE_REJECTED = 3,
    RG_ORACLE_UNALIGNED = 4,
    RG_ORACLE_NOT_DATA = 5,
};

void rg_oracle_chacha20_block(const uint8_t key[32], uint32_t counter, const uint8_t nonce[12], uint8_t out[64]);
void rg_oracle_poly1305(const uint8_t key[32], const uint8_t *msg, size_t len, uint8_t tag[16]);
void rg_oracle_aead_seal(const uint8_t key[32], const uint8_t nonce[12], const uint8_t *aad, size_t aad_len,
                         uint8_t *payload, size_t len, uint8_t tag[16]);
int rg_oracle_aead_open(const uint8_t key[32], const uint8_t nonce[12], const uint8_t *aad, size_t aad_len,
                        uint8_t *payload, size_t len, const uint8_t tag[16]);
void rg_oracle_wg_nonce(uint64_t counter, uint8_t nonce[12]);

void rg_oracle_seal_one(const uint8_t *keys, const uint32_t *receivers, const rg_oracle_desc *d, uint64_t counter,
                        uint8_t *buf, uint8_t *status);
void rg_oracle_open_one(const uint8_t *keys, const rg_oracle_desc *d, uint8_t *buf, uint8_t *status,
                        uint64_t *counter_out);
void rg_oracle_seal_batch(const uint8_t *keys, const uint32_t *receivers, const rg_oracle_desc *desc,
                          const uint64_t *counters, size_t n, uint8_t *buf, uint8_t *status, int nthreads);
/* XChaCha20-Poly1305 cookie AEAD (rustyguard-crypto/src/prim.rs:202-224) */
void rg_oracle_hchacha20(const uint8_t key[32], const uint8_t nonce16[16], uint8_t out[32]);
void rg_oracle_xaead_seal(const uint8_t key[32], const uint8_t nonce24[24], const uint8_t *aad, size_t aad_len,
                          uint8_t *payload, size_t len, uint8_t tag[16]);
int rg_oracle_xaead_open(const uint8_t key[32], const uint8_t nonce24[24], const uint8_t *aad, size_t aad_len,
                         uint8_t *payload, size_t len, const uint8_t tag[16]);
/* BLAKE2s (RFC 7693) and the handshake mac1/mac2 checks (rustyguard-crypto/src/lib.rs:114-209) */
void rg_oracle_blake2s(uint8_t *out, size_t outlen, const uint8_t *key, size_t keylen, const uint8_t *msg,
                       size_t len);
void rg_oracle_mac_verify_batch(const uint8_t *keys, size_t key_len, size_t nkeys, int which,
                                const rg_oracle_desc *desc, size_t n, const uint8_t *buf, size_t buf_len,
                                uint8_t *status, uint32_t *key_out);
void rg_oracle_open_batch(const uint8_t *keys, const rg_oracle_desc *desc, size_t n, uint8_t *buf,
                          uint8_t *status, uint64_t *counters_out, int nthreads);
/* open with the receiver -> session lookup of Sessions::decrypt_packet
 * (rustyguard-core/src/lib.rs:646-650); sessions as a plain list */
void rg_oracle_open_one_rx(const uint8_t *keys, const uint32_t *rx_rec, const uint32_t *rx_key, size_t nrx,
                           const rg_oracle_desc *d, uint8_t *buf, uint8_t *status, uint64_t *counter_out,
                           uint32_t *key_out);
void rg_oracle_open_batch_rx(const uint8_t *keys, const uint32_t *rx_rec, const uint32_t *rx_key, size_t nrx,
                             const rg_oracle_desc *desc, size_t n, uint8_t *buf, uint8_t *status,
                             uint64_t *counters_out, uint32_t *key_out);

uint64_t rg_oracle_mix64(uint64_t x);
void rg_oracle_synth_fill(uint8_t *buf, const rg_oracle_desc *desc, const uint32_t *inner_len, size_t n,
                          uint64_t seed);

#ifdef __cplusplus
}
#endif
#endif
