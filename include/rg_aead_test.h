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

/* Fail-closed hooks.  rg_debug_plan_handoff(1) starts the planner's finished-workgroup count
 * stale in the preset pass, so no planner workgroup finds itself last and the pipelined kernel's schedule
 * is never handed over; (2) starts the tile kernel's grid-wide pool past its end, so the pooled tiles are
 * never taken; (0) off.  Every packet such a launch never reaches must read RG_PKT_PENDING.
 * rg_debug_lose_completions(1) makes every library wait see its event as never completing (the bounded
 * waits then time out).  rg_debug_wait_selftest runs the bounded wait loop against a fake completion that
 * arrives on poll ready_after + 1 (never, for UINT32_MAX) -- no HIP call, so it runs without a GPU -- and
 * returns RG_OK or RG_EDEVICE (timed out), with the polls made and the time taken.
 * rg_debug_last_wipe copies the first bytes of the most recently wiped key block, read back from the device
 * after its wipe and before its free, and reports how many blocks were wiped so far.
 * rg_debug_secret_state reports whether a key buffer of the context is read by a captured launch (1) or
 * not (0), how many captured blocks a regrow retired, and how many stream events guard it. */
void rg_debug_plan_handoff(int mode);
void rg_debug_lose_completions(int on);
int rg_debug_wait_selftest(uint32_t timeout_ms, uint32_t ready_after, uint32_t *polls_out, uint32_t *elapsed_ms_out);
int64_t rg_debug_last_wipe(void *dst, size_t bytes, uint64_t *wipes_out);
int rg_debug_secret_state(rg_ctx *ctx, int which, uint32_t *retired_out, uint32_t *users_out);

#ifdef __cplusplus
}
#endif
#endif /* RG_AEAD_TEST_H */
