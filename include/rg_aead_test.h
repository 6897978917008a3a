/*
 * rg_aead_test.h -- test hooks of the MI355X WireGuard AEAD engine.
 *
 * Exported by the TEST library only (rustyguard_amd/lib/librg_aead_test.so: the product
 * kernels plus rg_api.cpp built with -DRG_TEST_HOOKS), never by the product library
 * librg_aead.so, whose ABI is include/rg_aead.h.  The GPU tests that check key wiping
 * and allocation-failure paths load the test library beside the product one.
 */
#ifndef RG_AEAD_TEST_H
#define RG_AEAD_TEST_H

#include "rg_aead.h"

#ifdef __cplusplus
extern "C" {
#endif

/* rg_debug_read_arena copies up to `bytes` of one of the context's key-bearing device buffers to
 * host memory -- which = 0: the per-message drop-in's arena (its job record holds the key while a
 * call runs and is zeroed before the call returns, on every path), 1: the batched host API's key
 * table, 2: the MAC key states -- and returns the number of bytes copied (>= 0) or a negative
 * rg_status.  Key-bearing buffers are zeroed before they are freed or regrown (rg_destroy,
 * rg_sessions_destroy), as the reference zeroizes keys on drop (rustyguard-crypto/src/prim.rs:
 * 227-231).  rg_debug_fail_reserve(n) makes the n-th following device or pinned-host buffer
 * allocation of any context of this library fail (0 = off), for error-path tests. */
int rg_debug_read_arena(rg_ctx *ctx, int which, void *dst, size_t bytes);
void rg_debug_fail_reserve(int nth);

#ifdef __cplusplus
}
#endif
#endif /* RG_AEAD_TEST_H */
