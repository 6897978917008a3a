// rg_pipe.hip -- the pipelined lane kernel: batched WireGuard transport seal /
// open, one packet per lane.  Replaces N x Core::chacha20poly1305_{enc,dec}
// (rustyguard-crypto/src/prim.rs:179-201) as driven by EncryptionKey::encrypt
// / DecryptionKey::decrypt (prim.rs:386-437), with the frame layout of
// EncryptedMetadata::frame_in_place (rustyguard-core/src/lib.rs:450-470).
//
// Why this shape (measured, tools/microbench.hip): a ChaCha20 block costs
// ~3800 cycles per wave at 1 wave/SIMD and ~3820 cycles of SIMD time per
// wave-block at 8 waves/SIMD, so one packet per lane already runs the
// keystream at the SIMD's VALU issue rate.  What the plain lane kernel loses is
// (a) HBM latency and (b) the serial Poly1305 chain, whose multiply-carry
// dependencies leave issue slots empty.  Here
//  * three chunk buffers rotate (the loop is unrolled three times, nothing in
//    flight is ever copied): chunk t+3 is requested as soon as chunk t is
//    written, so a load has three keystream periods to arrive;
//  * chunk t-1's four Poly1305 blocks (open: chunk t's ciphertext) are
//    absorbed inside chunk t's keystream rounds (after double rounds 1, 3, 5,
//    7), where the ARX chains leave the multiply chain's latency covered;
//  * payload loads of a packet are issued before its one-time-key block, so
//    that block hides the first chunks' latency.
// A partial last chunk (P % 64 != 0) runs after the loop with per-block
// predicates; the last chunk's Poly1305 blocks are absorbed after it.
//
// Round 4 measured two co-resident waves per SIMD (__launch_bounds__(256, 2),
// two lanes per packet, HW_ID stamps: profiles/r4_cfg2_twowave.txt): slower.
// The pair issues no more VALU per cycle than one wave, the memory
// instructions are not hidden either, and the split adds a one-time-key block
// and an r^N combine per packet.  One wave per SIMD stays.
//
// Diagnostic builds (-DRG_DIAG, tools/build_variant.sh; never the product
// library) add the seal modes of pipe_step and per-wave stamps.
#include "rg_device.h"
#include "rg_internal.h"

namespace rg {

struct Chunk {
    uint4 q0, q1, q2, q3;
};

// Chunks in flight per lane: while chunk t is processed, chunks t+1 .. t+2 are
// loaded or loading (the load of chunk t + 3 is issued at its end).
constexpr int kDepth = 3;

typedef unsigned v4u __attribute__((ext_vector_type(4)));
// NT (diagnostic seal modes only): 1 non-temporal loads, 2 non-temporal stores, 4 stores dropped
template <int NT> __device__ __forceinline__ uint4 ld16(const uint4 *p) {
    if constexpr (NT & 1) {
        const v4u v = __builtin_nontemporal_load(reinterpret_cast<const v4u *>(p));
        return make_uint4(v.x, v.y, v.z, v.w);
    } else return *p;
}
template <int NT> __device__ __forceinline__ void st16(uint4 *p, const uint4 &x) {
    if constexpr (NT & 4) return;
    else if constexpr (NT & 2) {
        const v4u v = {x.x, x.y, x.z, x.w};
        __builtin_nontemporal_store(v, reinterpret_cast<v4u *>(p));
    } else *p = x;
}
template <int MODE> constexpr int mode_nt() { return MODE == 7 ? 4 : (MODE >= 4 && MODE <= 6) ? MODE - 3 : 0; }

// Branch-free chunk load: piece indices are clamped to the packet's last
// 16-byte block (block 0 of an empty payload is the tag slot, also inside the
// frame), so every lane issues the same four loads and the waitcnt pass can
// count them exactly.
template <int NT = 0>
__device__ __forceinline__ void load_chunk(Chunk &c, const uint4 *pl, uint32_t t, uint32_t last) {
    const uint32_t b = 4 * t;
    c.q0 = ld16<NT>(pl + min(b + 0, last));
    c.q1 = ld16<NT>(pl + min(b + 1, last));
    c.q2 = ld16<NT>(pl + min(b + 2, last));
    c.q3 = ld16<NT>(pl + min(b + 3, last));
}

__device__ __forceinline__ void absorb_chunk(Acc &h, const Chunk &c, const Mul &r, uint32_t cnt) {
    acc_block_pred(h, c.q0, r, cnt > 0);
    acc_block_pred(h, c.q1, r, cnt > 1);
    acc_block_pred(h, c.q2, r, cnt > 2);
    acc_block_pred(h, c.q3, r, cnt > 3);
}

// ------------------------------------------------------------- line stores
// When all 64 lanes of a wave hold valid packets of one size (one lane per
// packet), the frames leave through a wave-private LDS ring in whole 128-byte
// lines: a lane-per-frame store instruction puts one 16-byte piece into each
// of 64 frames (64 cache lines per instruction, a line completed by eight
// instructions over two steps, and measured 1.29x the algorithmic write bytes
// at config 5), whereas from the ring each store instruction writes whole
// lines of 8 frames, eight lanes per line.  Step t puts its 64-byte block t
// (pieces 4t .. 4t+3 of the frame: the header, payload blocks, the tag)
// into ring set t & 3; steps 2k+2 and 2k+3 store line k (blocks 2k, 2k+1) of
// frames 0-31 and 32-63, read back at the start of the step so that the LDS
// round trip hides behind the keystream rounds.  Every step issues the same
// LDS and store instructions (no parity branch: the vmcnt waits stay exact).
// Frame p's 256 bytes hold piece j of set s in slot (4 s + j) ^ g(p & 7),
// g = {0, 1, 10, 11, 4, 5, 14, 15}: conflict-free for the frame-major
// ds_write_b128 (8-lane groups, 128-byte rows) and the line-major
// ds_read_b128 (16-lane groups, 256-byte rows).
// Alternatives measured in round 3 and dropped: a DPP quad
// transpose with 64-byte half-line stores, line stores spread over the rounds,
// an LDS-DMA staged chunk stream, lane-per-frame stores without a transpose.
constexpr uint32_t kPipeLinesFlag = 4u;      // launch flag bit (bits 0-1: log2 lanes per packet)
constexpr uint32_t kRingBytes = 64u * 256u; // per wave
// (plain vector types: HIP's uint4 has no assignment in a qualified address space)
typedef __attribute__((address_space(3))) v4u lds_u4;
__device__ __forceinline__ v4u to_v4(const uint4 &a) { return v4u{a.x, a.y, a.z, a.w}; }
__device__ __forceinline__ uint32_t ring_g(uint32_t p) { return (p & 1u) ^ (((p >> 1) & 1u) * 10u) ^ (((p >> 2) & 1u) * 4u); }

// Frame stores of a line-store wave go through a buffer resource based at the wave's lowest frame:
// 32-bit offsets (16 VGPRs fewer than 64-bit line pointers), compiler-visible, so hipcc's vmcnt
// waits stay exact.
struct Ring {
    lds_u4 *wr;          // this lane's frame record
    lds_u4 *rd;          // line-major reads: frame lane / 8 (+ 8 q + 32 h), slot base
    uint32_t fo[2][4];   // byte offset of frame 32 h + 8 q + lane / 8, + 16 (lane % 8), in the wave's window
    uint32_t self;       // byte offset of this lane's frame in the window
    uint64_t base;       // the window's base address (wave-uniform)
    __amdgpu_buffer_rsrc_t rs; // the window: the wave's frames
    uint32_t gw, gr;     // slot swizzles: this lane's frame (writes), frame lane / 8 (reads)
};

// The window of a wave whose 64 lanes all hold a frame of `len` bytes: based at the lowest frame,
// false when the frames span 2 GiB or more (the wave then stores lane by lane, without the ring).
__device__ __forceinline__ bool frame_window(const uint8_t *frame, uint32_t len, uint64_t &base) {
    const uint64_t f = reinterpret_cast<uint64_t>(frame);
    const uint64_t f0 = uniform_u64(f);
    const int64_t dlt = (int64_t)(f - f0);
    const bool near = dlt > -(int64_t)(1u << 30) && dlt < (int64_t)(1u << 30);
    if (__ballot(!near) != 0) return false;
    // biased to [0, 2^31): prefix maxima of v and of its complement give the max and the min
    const uint32_t v = (uint32_t)(dlt + (int64_t)(1u << 30));
    const uint32_t vmax = lane63(wave_scan_max(v)), vmin = 0x7FFFFFFFu - lane63(wave_scan_max(0x7FFFFFFFu - v));
    if ((uint64_t)(vmax - vmin) + len >= (1ull << 31)) return false;
    base = f0 + (uint64_t)vmin - (1ull << 30);
    return true;
}

__device__ __forceinline__ Ring make_ring(uint8_t *frame, uint64_t base) {
    extern __shared__ __attribute__((aligned(16))) uint8_t pipe_lds[];
    const uint32_t lane = threadIdx.x & 63;
    lds_u4 *lb = (lds_u4 *)(pipe_lds + (threadIdx.x >> 6) * kRingBytes);
    Ring R;
    R.wr = lb + 16 * lane;
    R.gw = ring_g(lane);
    R.rd = lb + 16 * (lane >> 3);
    R.gr = ring_g(lane >> 3);
    R.self = (uint32_t)(reinterpret_cast<uint64_t>(frame) - base);
    R.base = base;
    R.rs = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void *>(base), (short)0, 0x7FFFFFFF, 0x00020000);
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int q = 0; q < 4; ++q)
            R.fo[h][q] = (uint32_t)__shfl((int)R.self, 32 * h + 8 * q + (int)(lane >> 3)) + 16 * (lane & 7u);
    return R;
}

// the same window with its descriptor rebuilt from readfirstlane values: a descriptor that reaches its
// use through a join of branches hipcc cannot prove uniform becomes a per-lane waterfall loop
__device__ __forceinline__ Ring pin_window(const Ring &R) {
    Ring o = R;
    o.base = uniform_u64(R.base);
    o.rs = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void *>(o.base), (short)0, 0x7FFFFFFF, 0x00020000);
    return o;
}

// Cache policy of a line-store wave's last stores -- the lines stored after its final keystream step
// (the ring's last half-lines, the partial last chunk, the tag): 0 write-back (default), 16 write-through
// (sc1), 2 non-temporal.  A store-heavy launch ends with the dirty lines of the XCDs' L2s written back
// after its last wave (MI355X_MICROARCH.md, the "boundary" row); write-through final stores leave fewer of
// them (tools/l2tail.hip, round 6).  Diagnostic builds set it with -DRG_TAIL_CP.
#ifndef RG_TAIL_CP
#define RG_TAIL_CP 0
#endif
constexpr int kTailCp = RG_TAIL_CP;

// a 16-byte piece of this lane's frame at byte `off` of the frame (line-store waves)
template <int CP = 0> __device__ __forceinline__ void frame_store(const Ring &R, uint32_t off, const uint4 &x) {
    __builtin_amdgcn_raw_buffer_store_b128(to_v4(x), R.rs, (int)(R.self + off), 0, CP);
}

// block t (4 pieces) of this lane's frame into set t & 3
__device__ __forceinline__ void ring_put(const Ring &R, uint32_t t, const uint4 &a, const uint4 &b, const uint4 &c,
                                         const uint4 &d) {
    const uint32_t sw = (4 * (t & 3u)) ^ R.gw;
    R.wr[sw ^ 0] = to_v4(a);
    R.wr[sw ^ 1] = to_v4(b);
    R.wr[sw ^ 2] = to_v4(c);
    R.wr[sw ^ 3] = to_v4(d);
}

struct Ring4 {
    v4u v[4];
};
// half h of line k read back: v[q] = piece lane % 8 of line k of frame 32 h + 8 q + lane / 8
__device__ __forceinline__ Ring4 ring_get(const Ring &R, uint32_t k, uint32_t h) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t set = (2 * k + ((lane >> 2) & 1u)) & 3u;
    const lds_u4 *r = R.rd + 512 * h + ((4 * set + (lane & 3u)) ^ R.gr);
    Ring4 o;
#pragma unroll
    for (int q = 0; q < 4; ++q) o.v[q] = r[128 * q];
    return o;
}

// store it (MASK: pieces of block 2k+1 only when that block is in the ring, i.e. 2k+1 < nblk)
template <bool MASK = false, int CP = 0>
__device__ __forceinline__ void ring_store(const Ring &R, const Ring4 &x, uint32_t k, uint32_t h, uint32_t nblk = 0) {
    if constexpr (MASK) {
        const uint32_t lane = threadIdx.x & 63;
        if (((lane >> 2) & 1u) && 2 * k + 1 >= nblk) return;
    }
#pragma unroll
    for (int q = 0; q < 4; ++q)
        __builtin_amdgcn_raw_buffer_store_b128(x.v[q], R.rs, (int)((h ? R.fo[1][q] : R.fo[0][q]) + 128 * k), 0, CP);
}

// One step: keystream block t+1 -- with the previous chunk's four Poly1305
// blocks (pi, always a full chunk; open: this chunk's ciphertext) absorbed in
// its rounds when ABSORB -- XORed into chunk t (buf) and stored; then chunk
// t+3 is requested into buf.  Full steps store unconditionally: a store under
// a branch leaves the waitcnt pass a path with fewer memory operations, and
// since vmcnt counts stores as well as loads it would then also wait for the
// last step's stores to be acked.
// TAIL: the partial last chunk (cnt < 4 blocks), predicated, no prefetch.
// Stores are shifted by one block so that each step writes one 64-byte
// frame-aligned block (the payload starts 16 bytes into the frame): the
// previous chunk's last block (prev; or the header, before the first chunk of
// a sealed frame) and this chunk's first three.  Lines written piecewise across
// steps were measured at 1.66x the algorithmic write bytes (profiles/).
// LINES: the frame blocks go through the wave's LDS ring (block t goes into
// the ring; with FLUSH, half t & 1 of line (t - 2) / 2 is read back before the
// rounds and stored after them).
// MODE (seal diagnostics, RG_DIAG builds only): 0 normal; 1 compute only (no
// payload loads or stores, loop-carried fake data); 2 memory only (no
// keystream and no Poly1305); 4/5/6 non-temporal loads / stores / both; 7 no
// payload stores; 8 line stores alternate between lines 0 and 1 of each frame
// (cache-resident: the store instructions without their HBM writes).
template <bool OPEN, bool ABSORB, bool TAIL, int MODE = 0, bool LINES = false, bool FLUSH = false>
__device__ __forceinline__ void pipe_step(uint4 *pl, const Stream &st, const Mul &r, Acc &h, Chunk &pi, Chunk &buf,
                                          uint4 &prev, bool &have_prev, uint32_t t, uint32_t nb, uint32_t c0,
                                          const Ring &R) {
    uint32_t ks[16];
    static_assert(!FLUSH || (LINES && ABSORB && !TAIL), "flush steps");
    Ring4 fl;
    if constexpr (FLUSH) {
        wave_sync(); // block t - 1 was put by every lane
        fl = ring_get(R, (t - 2) >> 1, t & 1u);
    }
    if constexpr (MODE == 2) {
#pragma unroll
        for (int i = 0; i < 16; ++i) ks[i] = t * 16 + i;
        h.h0 ^= pi.q0.x ^ pi.q1.y ^ pi.q2.z ^ pi.q3.w;
    } else stream_block_hooked(st, c0 + t + 1, ks, [&](int dr) {
        if constexpr (OPEN) { // this chunk's ciphertext (TAIL: its nb % 4 blocks)
            const uint32_t bl = TAIL ? nb & 3u : 4u;
            if (dr == 1) acc_block_pred(h, buf.q0, r, bl > 0);
            if (dr == 3) acc_block_pred(h, buf.q1, r, bl > 1);
            if (dr == 5) acc_block_pred(h, buf.q2, r, bl > 2);
            if (dr == 7) acc_block_pred(h, buf.q3, r, bl > 3);
            if (dr % 2 == 1) pin_acc(h);
        } else if constexpr (ABSORB) {
            if (dr == 1) acc_block(h, pi.q0, r);
            if (dr == 3) acc_block(h, pi.q1, r);
            if (dr == 5) acc_block(h, pi.q2, r);
            if (dr == 7) acc_block(h, pi.q3, r);
            if (dr % 2 == 1) pin_acc(h);
        }
    });
    Chunk x = {xor4(buf.q0, ks + 0), xor4(buf.q1, ks + 4), xor4(buf.q2, ks + 8), xor4(buf.q3, ks + 12)};
    uint4 *dst = pl + 4 * t;
    if constexpr (MODE == 1) {
        pi = x;
        buf.q0.x += t; buf.q1.y ^= t; buf.q2.z += h.h0; buf.q3.w ^= t; // fake next chunk, loop-carried
        return;
    }
    constexpr int NT = mode_nt<MODE>();
    if constexpr (LINES && !TAIL) {
        ring_put(R, t, prev, x.q0, x.q1, x.q2); // prev: the header before the first chunk
        if constexpr (FLUSH) ring_store(R, fl, MODE == 8 ? ((t - 2) >> 1) & 1u : (t - 2) >> 1, t & 1u);
        prev = x.q3;
        have_prev = true;
    } else if constexpr (TAIL) {
        const uint32_t cnt = nb & 3u;
        if constexpr (LINES) { // one lane per packet: pl = frame + 16, dst = frame byte 16 + 64 t
            const uint32_t o = 16 + 64 * t;
            if (have_prev) frame_store<kTailCp>(R, o - 16, prev);
            frame_store<kTailCp>(R, o, x.q0); // cnt >= 1
            if (cnt > 1) frame_store<kTailCp>(R, o + 16, x.q1);
            if (cnt > 2) frame_store<kTailCp>(R, o + 32, x.q2);
        } else {
            if (have_prev) st16<NT>(dst - 1, prev);
            st16<NT>(dst + 0, x.q0); // cnt >= 1
            if (cnt > 1) st16<NT>(dst + 1, x.q1);
            if (cnt > 2) st16<NT>(dst + 2, x.q2);
        }
        have_prev = false;
    } else {
        if constexpr (ABSORB) st16<NT>(dst - 1, prev); // inside the loop there always is one
        else if (have_prev) st16<NT>(dst - 1, prev);
        st16<NT>(dst + 0, x.q0);
        st16<NT>(dst + 1, x.q1);
        st16<NT>(dst + 2, x.q2);
        prev = x.q3;
        have_prev = true;
    }
    if constexpr (!OPEN) pi = x;
    if constexpr (!TAIL) load_chunk<NT & 1>(buf, pl, t + kDepth, nb - 1);
}

// Keystream XOR in place + Poly1305 over the ciphertext of nb 16-byte blocks
// starting at chunk c0 of the payload (pl points there; keystream blocks from
// c0 + 1); b0 / b1 / b2 hold its chunks 0 / 1 / 2 (loads already issued).
// The first step is peeled (nothing to absorb yet), so that every absorb
// inside the loop is unconditional; chunk c always lives in buffer c % 3.
// head / has_head: the DataHeader a seal writes in front of the payload (only
// the lane whose segment starts the payload has one).
// LINES (a wave of valid packets of one size, has_head set): blocks through the LDS ring.
template <bool OPEN, int MODE = 0, bool LINES = false>
__device__ __forceinline__ Acc pipe_pass(uint4 *pl, const Stream &st, const Mul &r, uint32_t nb, uint32_t c0,
                                         Chunk &b0, Chunk &b1, Chunk &b2, uint4 head, bool has_head, const Ring &R0) {
    const Ring R = LINES ? pin_window(R0) : R0;
    const uint32_t F = nb >> 2, bl = nb & 3u; // full chunks, blocks in the partial last chunk
    Acc h = {0, 0, 0, 0, 0};
    Chunk pi = {};
    uint4 prev = head; // block still to be stored just in front of the current chunk
    bool have_prev = has_head;
    uint32_t pending = 0; // blocks of pi not yet absorbed
    if constexpr (LINES) wave_sync(); // the previous packet's last read-back is done
    if (F > 0) {
        pipe_step<OPEN, false, false, MODE, LINES>(pl, st, r, h, pi, b0, prev, have_prev, 0, nb, c0, R);
        uint32_t t = 1;
        // whole rounds of three steps only: a step that may be skipped would
        // leave the waitcnt pass a path without its memory operations
        // (vmcnt(0) at the next one); the remainder steps run after the loop
        if constexpr (LINES) {
            // step 1 has no complete line yet; steps 2.. each store half a line
            if (F > 1) pipe_step<OPEN, true, false, MODE, true>(pl, st, r, h, pi, b1, prev, have_prev, 1, nb, c0, R);
            for (t = 2; t + 2 < F; t += 3) {
                pipe_step<OPEN, true, false, MODE, true, true>(pl, st, r, h, pi, b2, prev, have_prev, t, nb, c0, R);
                pipe_step<OPEN, true, false, MODE, true, true>(pl, st, r, h, pi, b0, prev, have_prev, t + 1, nb, c0, R);
                pipe_step<OPEN, true, false, MODE, true, true>(pl, st, r, h, pi, b1, prev, have_prev, t + 2, nb, c0, R);
            }
            if (t < F) pipe_step<OPEN, true, false, MODE, true, true>(pl, st, r, h, pi, b2, prev, have_prev, t, nb, c0, R);
            if (t + 1 < F)
                pipe_step<OPEN, true, false, MODE, true, true>(pl, st, r, h, pi, b0, prev, have_prev, t + 1, nb, c0, R);
            // the halves not stored yet: m = F - 2 .. 2 ceil(F / 2) - 1 (k = m / 2, h = m % 2); a
            // last line of one block stores its first four pieces only
            wave_sync();
            for (uint32_t m = F >= 2 ? F - 2 : 0; m < 2 * ((F + 1) >> 1); ++m)
                ring_store<true, kTailCp>(R, ring_get(R, m >> 1, m & 1u), MODE == 8 ? (m >> 1) & 1u : m >> 1, m & 1u,
                                          F);
        } else {
            for (; t + 2 < F; t += 3) {
                pipe_step<OPEN, true, false, MODE, false>(pl, st, r, h, pi, b1, prev, have_prev, t, nb, c0, R);
                pipe_step<OPEN, true, false, MODE, false>(pl, st, r, h, pi, b2, prev, have_prev, t + 1, nb, c0, R);
                pipe_step<OPEN, true, false, MODE, false>(pl, st, r, h, pi, b0, prev, have_prev, t + 2, nb, c0, R);
            }
            if (t < F) pipe_step<OPEN, true, false, MODE, false>(pl, st, r, h, pi, b1, prev, have_prev, t, nb, c0, R);
            if (t + 1 < F) pipe_step<OPEN, true, false, MODE, false>(pl, st, r, h, pi, b2, prev, have_prev, t + 1, nb, c0, R);
        }
        pending = 4;
    }
    if (bl > 0) {
        // chunk F lives in b(F % 3); select by value (a reference select
        // between the buffers would move them to scratch memory)
        const uint32_t k = F % kDepth;
        Chunk bp = {k == 1 ? b1.q0 : k == 2 ? b2.q0 : b0.q0, k == 1 ? b1.q1 : k == 2 ? b2.q1 : b0.q1,
                    k == 1 ? b1.q2 : k == 2 ? b2.q2 : b0.q2, k == 1 ? b1.q3 : k == 2 ? b2.q3 : b0.q3};
        if (F > 0) pipe_step<OPEN, true, true, MODE, LINES>(pl, st, r, h, pi, bp, prev, have_prev, F, nb, c0, R);
        else pipe_step<OPEN, false, true, MODE, LINES>(pl, st, r, h, pi, bp, prev, have_prev, F, nb, c0, R);
        pending = bl;
    }
    if constexpr (LINES) {
        if (have_prev) frame_store<kTailCp>(R, 64 * F, prev); // pl + 4 F - 1
    } else if (have_prev && MODE != 1) st16<mode_nt<MODE>()>(pl + 4 * F - 1, prev);
    if constexpr (!OPEN) absorb_chunk(h, pi, r, pending); // the last chunk's blocks
    return h;
}

// tag = ((h + lenblock) r mod p) + s; length block le64(aad_len = 0) || le64(P) (RFC 8439 §2.8)
__device__ __forceinline__ void pipe_tag(Acc h, const Mul &r, uint32_t P, const uint32_t *s, uint32_t tag[4]) {
    acc_add(h, 0, 0, P, 0, 1);
    acc_mul(h, r);
    acc_finish(h, s[0], s[1], s[2], s[3], tag);
}

// ------------------------------------------------------------- segments
// G lanes (consecutive, G | 64) may share a packet: segment j covers chunks
// [jL, min(C, (j+1)L)), L = ceil(C / G), with its own Horner chain h_j over
// its blocks (clamped r).  With N_j = blocks after segment j,
//   Poly1305 accumulator = sum_j h_j r^{N_j},
// each lane raises r to its own N_j (left-to-right square-and-multiply: the
// squarings are general multiplies, the "times r" steps the cheap clamped
// one) and the group sums by butterfly; every lane of the group then holds
// the packet's accumulator.  Each lane also computes the one-time-key block
// itself (no cross-lane dependency before the combine).  Segments serve
// batches too small to give every SIMD a wave at one lane per packet.
struct Seg {
    uint32_t c0, nb, after; // first chunk, blocks in the segment, blocks after it
};

__device__ __forceinline__ Seg make_seg(uint32_t nb, uint32_t j, uint32_t G) {
    const uint32_t C = (nb + 3) >> 2, L = (C + G - 1) / G;
    const uint32_t c0 = min(j * L, C), c1 = min(c0 + L, C);
    const uint32_t b0 = min(4 * c0, nb), b1 = min(4 * c1, nb);
    return {c0, b1 - b0, nb - b1};
}

__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, o));
    return v;
}

__device__ __forceinline__ Acc combine_segments(Acc h, const Mul &r, uint32_t after, uint32_t G) {
    if (G == 1) return h;
    const uint32_t bits = 32 - __clz((int)wave_max_u32(after));
    if (bits > 0) {
        // r^after, left to right over the wave's bit count; every lane starts
        // from 1, so leading zero bits of a shorter exponent are harmless
        Acc x = {1, 0, 0, 0, 0};
        for (int b = (int)bits - 1; b >= 0; --b) {
            Acc sq = x;
            acc_sqr_gen(sq);
            Acc xr = sq;
            acc_mul(xr, r);
            const bool bit = (after >> b) & 1u;
            x.h0 = bit ? xr.h0 : sq.h0; x.h1 = bit ? xr.h1 : sq.h1; x.h2 = bit ? xr.h2 : sq.h2;
            x.h3 = bit ? xr.h3 : sq.h3; x.h4 = bit ? xr.h4 : sq.h4;
        }
        acc_mul_gen(h, make_gen(x));
    }
    for (uint32_t o = 1; o < G; o <<= 1) {
        Acc other;
        other.h0 = (uint32_t)__shfl_xor((int)h.h0, (int)o);
        other.h1 = (uint32_t)__shfl_xor((int)h.h1, (int)o);
        other.h2 = (uint32_t)__shfl_xor((int)h.h2, (int)o);
        other.h3 = (uint32_t)__shfl_xor((int)h.h3, (int)o);
        other.h4 = (uint32_t)__shfl_xor((int)h.h4, (int)o);
        acc_add_acc(h, other);
        acc_fold(h);
    }
    return h;
}

// ------------------------------------------------------------------ seal
// Frame: [hdr 16][payload P][tag 16]; desc.len = P.  Checks as seal_packet
// (rg_kernels.hip): descriptor and force_encrypt's padding assert
// (rustyguard-core/src/lib.rs:273-277).  Lane j of a G-lane group runs
// segment j; lane 0 writes header, tag and status.
template <int MODE>
__device__ __forceinline__ void pipe_seal_packet(const SealArgs &a, uint32_t i, const rg_pkt_desc &d, uint32_t j,
                                                 uint32_t G, bool lines_ok) {
    const uint32_t P = d.len;
    const bool valid = d.key_idx < a.nkeys && (P & 15u) == 0 && (d.offset & 15u) == 0 && P <= kMaxPayload &&
                       d.offset <= a.buf_len && P + 32 <= a.buf_len - d.offset;
    // block stores through the LDS ring: every lane of the wave a valid packet of one size
    bool lines = false;
    if constexpr (MODE == 0 || MODE == 8)
        lines = lines_ok && G == 1 && __ballot(valid && P == uniform_u32(P)) == ~0ull;
    uint64_t wbase = 0;
    if (lines) lines = frame_window(a.buf + d.offset, P + 32, wbase); // wave-uniform
    if (!valid) {
        if (a.status && j == 0) a.status[i] = d.key_idx == RG_KEY_SKIP ? RG_PKT_REJECTED : RG_PKT_INVALID;
        return;
    }
    uint8_t *frame = a.buf + d.offset;
    const uint32_t nb = P >> 4;
    const Seg sg = make_seg(nb, j, G);
    // an empty segment reads (never writes) the payload start, which is in the frame
    uint4 *pl = reinterpret_cast<uint4 *>(frame + 16) + (sg.nb ? 4 * sg.c0 : 0);
    Chunk b0, b1, b2;
    if constexpr (MODE == 1) {
        b0 = {make_uint4(i, 1, 2, 3), make_uint4(4, i, 6, 7), make_uint4(8, 9, i, 11), make_uint4(12, 13, 14, i)};
        b1 = b0;
        b2 = b0;
    } else {
        constexpr int NT = mode_nt<MODE>() & 1;
        load_chunk<NT>(b0, pl, 0, sg.nb ? sg.nb - 1 : 0);
        load_chunk<NT>(b1, pl, 1, sg.nb ? sg.nb - 1 : 0);
        load_chunk<NT>(b2, pl, 2, sg.nb ? sg.nb - 1 : 0);
    }
    const Key8 key = load_key(a.keys, d.key_idx);
    const uint64_t ctr = a.counters[i];
    const uint32_t n1 = (uint32_t)ctr, n2 = (uint32_t)(ctr >> 32); // nonce = 0 || le64(ctr) (prim.rs:32-36)
    const Stream stm = make_stream(key, 0u, n1, n2);
    uint32_t ks[16];
    stream_block(stm, 0, ks); // RFC 8439 §2.6 one-time key
    const Mul r = make_mul(ks[0], ks[1], ks[2], ks[3]);
    // DataHeader {4, receiver, counter} (rustyguard-core/src/lib.rs:286-290), stored by segment 0
    // together with the first payload blocks
    const bool head = a.receivers != nullptr && j == 0;
    uint4 hdr = make_uint4(4u, head ? a.receivers[d.key_idx] : 0u, n1, n2);
    Acc h;
    Ring R{};
    if (lines) { // wave-uniform
        if (!head) hdr = *reinterpret_cast<const uint4 *>(frame); // block 0 is stored whole: header unchanged
        R = make_ring(frame, wbase);
        h = pipe_pass<false, MODE, true>(pl, stm, r, sg.nb, sg.c0, b0, b1, b2, hdr, true, R);
    } else {
        h = pipe_pass<false, MODE, false>(pl, stm, r, sg.nb, sg.c0, b0, b1, b2, hdr, head, Ring{});
    }
    h = combine_segments(h, r, sg.after, G);
    if (j != 0) return;
    uint32_t tag[4];
    pipe_tag(h, r, P, ks + 4, tag);
    const uint4 tagv = make_uint4(tag[0], tag[1], tag[2], tag[3]);
    if (lines) frame_store<kTailCp>(pin_window(R), 16 + P, tagv);
    else *reinterpret_cast<uint4 *>(frame + 16 + P) = tagv;
    if (a.status) a.status[i] = RG_PKT_OK;
}

// ------------------------------------------------------------------ open
// desc.len = W.  Checks mirror rustyguard-core/src/lib.rs:613-629,
// rustyguard-types/src/lib.rs:181-196 and rustyguard-crypto/src/prim.rs:
// 427-429.  Decrypts speculatively while MACing the ciphertext; a failed tag
// (constant-time compare, identical on every lane of the group) makes each
// lane re-apply its segment's keystream, so the frame is left unchanged.
// (Verify-then-decrypt -- a Poly1305 pass, then the keystream pass -- makes a
// forged packet cost what a clean one does, but that Poly1305 pass runs
// latency-bound at one wave per SIMD: config 2's open +12 % in round 3,
// profiles/r3_macfirst_ab.txt.  Dropped.)
__device__ __forceinline__ void pipe_open_packet(const OpenArgs &a, uint32_t i, const rg_pkt_desc &d, uint32_t j,
                                                 uint32_t G, bool lines_ok) {
    const uint32_t W = d.len;
    uint32_t st;
    if (d.key_idx == RG_KEY_SKIP) st = RG_PKT_REJECTED;
    else if ((d.offset & 15u) != 0) st = RG_PKT_UNALIGNED;
    else if (d.key_idx >= a.nkeys || W > kMaxPayload + 32 || d.offset > a.buf_len || W > a.buf_len - d.offset ||
             W < 4)
        st = RG_PKT_INVALID;
    else st = 0xFF;
    uint8_t *frame = a.buf + d.offset;
    // Every load the lane needs is issued before the header is inspected, so
    // the header check costs no round trip of its own.  Loads stay
    // unconditional (exact waits): a frame that fails the descriptor checks
    // reads its own descriptor instead (a valid address), a length that cannot
    // decrypt reads no payload.
    const bool desc_ok = st == 0xFF;
    const bool go = desc_ok && W >= 32 && (W & 15u) == 0;
    const uint32_t P = go ? W - 32 : 0;
    const uint32_t nb = P >> 4;
    const Seg sg = make_seg(nb, j, G);
    uint4 *safe = const_cast<uint4 *>(reinterpret_cast<const uint4 *>(a.desc + i));
    uint4 *pl = go ? reinterpret_cast<uint4 *>(frame + 16) + (sg.nb ? 4 * sg.c0 : 0) : safe;
    const uint4 hdr = *(desc_ok ? reinterpret_cast<const uint4 *>(frame) : safe);
    Chunk b0, b1, b2;
    load_chunk(b0, pl, 0, sg.nb ? sg.nb - 1 : 0);
    load_chunk(b1, pl, 1, sg.nb ? sg.nb - 1 : 0);
    load_chunk(b2, pl, 2, sg.nb ? sg.nb - 1 : 0);
    const uint4 want = *(go ? reinterpret_cast<const uint4 *>(frame + 16 + P) : safe);
    const Key8 key = load_key(a.keys, go ? d.key_idx : 0);
    uint64_t ctr = 0;
    if (desc_ok) {
        if (hdr.x != 4u) st = hdr.x - 1u < 3u ? RG_PKT_NOT_DATA : RG_PKT_INVALID; // types 1-3 handshake/cookie, else lib.rs:627
        else if ((W & 15u) != 0 || W < 16) st = RG_PKT_INVALID;
        else {
            ctr = ((uint64_t)hdr.w << 32) | hdr.z;
            if (W < 32) st = RG_PKT_DECRYPT_ERR;
        }
    }
    // block stores through the LDS ring: every lane of the wave a data packet of one size
    bool lines = lines_ok && G == 1 && __ballot(st == 0xFF && W == uniform_u32(W)) == ~0ull;
    uint64_t wbase = 0;
    if (lines) lines = frame_window(frame, W, wbase); // wave-uniform
    if (st != 0xFF) {
        if (j == 0) {
            a.status[i] = (uint8_t)st;
            if (a.counters_out) a.counters_out[i] = ctr;
        }
        return;
    }
    const uint32_t n1 = (uint32_t)ctr, n2 = (uint32_t)(ctr >> 32);
    const Stream stm = make_stream(key, 0u, n1, n2);
    uint32_t ks[16];
    stream_block(stm, 0, ks);
    const Mul r = make_mul(ks[0], ks[1], ks[2], ks[3]);
    Acc h;
    Ring Ro{};
    if (lines) Ro = make_ring(frame, wbase);
    if (lines) h = pipe_pass<true, 0, true>(pl, stm, r, sg.nb, sg.c0, b0, b1, b2, hdr, true, Ro); // header unchanged
    else h = pipe_pass<true, 0, false>(pl, stm, r, sg.nb, sg.c0, b0, b1, b2, make_uint4(0, 0, 0, 0), false, Ring{});
    h = combine_segments(h, r, sg.after, G);
    uint32_t tag[4];
    pipe_tag(h, r, P, ks + 4, tag);
    const uint32_t diff = (tag[0] ^ want.x) | (tag[1] ^ want.y) | (tag[2] ^ want.z) | (tag[3] ^ want.w);
    if (__ballot(diff != 0)) {
        // restore the forged frames' segments (plaintext ^ keystream = ciphertext; callers never read
        // the buffer on Err, but the frame is left as it came), their chunks dealt over the wave's
        // lanes; with block stores other lanes wrote a lane's frame: every store completes and the
        // CU's cached lines go first
        wave_sync();
        restore_forged(diff != 0, key, n1, n2, pl, sg.c0, sg.nb);
    }
    if (j == 0) {
        a.status[i] = diff == 0 ? RG_PKT_OK : RG_PKT_DECRYPT_ERR;
        if (a.counters_out) a.counters_out[i] = ctr;
    }
}

// ------------------------------------------------------------- stamps
#if RG_DIAG
// Diagnostic builds: with a stamp buffer (debug mode 3, or any seal mode) lane 0 of every wave records
// [s_memtime delta, real-time ticks to the end of the wave's first and second unit, XCC_ID << 32 |
// HW_ID (wave slot, SIMD, CU, SH, SE), start s_memrealtime, s_memtime cycles of the prologue (entry to
// the first unit's start), 1, s_memrealtime delta]
// (tools/stamps.py, tools/coresidency.py; s_memrealtime ticks at 100 MHz).
__device__ __forceinline__ void pipe_stamp(uint64_t *dbg, uint64_t t0, uint64_t r0, const uint64_t marks[3]) {
    const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    if ((threadIdx.x & 63) == 0) {
        uint64_t *o = dbg + 8ull * (blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64);
        o[0] = t1 - t0;
        o[1] = marks[0] ? marks[0] - r0 : 0;
        o[2] = marks[1] ? marks[1] - r0 : 0;
        o[3] = ((uint64_t)(uint32_t)__builtin_amdgcn_s_getreg(0xF814) << 32) | (uint32_t)__builtin_amdgcn_s_getreg(0xF804);
        o[4] = r0;
        o[5] = marks[2] ? marks[2] - t0 : 0; // s_memtime cycles from the kernel's entry to its first unit
        o[6] = 1;
        o[7] = r1 - r0;
    }
}
#endif

// ---------------------------------------------------------------- walk
// Identity order: lane units u = G * packet + segment, grid-stride (the stride
// is a multiple of 256, so a packet's G lanes stay together in one wave);
// lg = log2(G).
// Planned order: the schedule's snake deal of the work-ordered tile list
// (schedule_classes); lane l of a tile of class c is unit (tile - first tile
// of c) * 64 + l of that class.
//
// Both orders share one loop, so the packet body has a single call site (two
// would make the compiler emit it as a real function call: stack frame, kernel
// arguments in scratch, ~250 VGPRs).
template <class Body>
__device__ __forceinline__ void pipe_walk(uint32_t n, uint32_t lg0, const PipePlan &pp, const rg_pkt_desc *desc,
                                          bool stamp, uint64_t marks[3], Body &&body) {
    const uint32_t lane = threadIdx.x & 63;
    const bool planned = pp.counts != nullptr;
    uint32_t my_cnt = 0, my_start = 0, my_lg = 0, my_tiles = 0, S = 1, simd = 0, ntiles = 0;
    uint64_t total, first, stride;
    if (planned) {
        my_cnt = lane < kClasses ? pp.sched[kSchedCnt + lane] : 0;
        my_start = lane < kClasses ? pp.sched[kSchedStart + lane] : 0;
        my_lg = lane < kClasses ? pp.sched[kSchedLg + lane] : 0;
        my_tiles = (uint32_t)((((uint64_t)my_cnt << my_lg) + 63) / 64);
        // static snake deal over the work-ordered tiles (heaviest first): rounds
        // of S tiles, SIMD s takes tile s of even rounds and S-1-s of odd ones;
        // wave slot w is SIMD w mod S in pass w / S (the grid is S x passes
        // waves), and takes rounds pass, pass + passes, ...  A shared queue
        // counter would serialise every wave on one atomic.
        S = pp.simds ? pp.simds : 1;
        const uint32_t slot = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
        simd = slot % S;
        ntiles = pp.sched[2];
        total = (ntiles + S - 1) / S; // rounds
        first = slot / S;
        stride = gridDim.x * (blockDim.x / 64) / S;
    } else { // lane units, grid-stride
        total = (uint64_t)n << lg0;
        first = blockIdx.x * 256 + threadIdx.x;
        stride = (uint64_t)gridDim.x * 256;
    }
    // unit `it` -> packet slot; the packet index itself comes from the plan's
    // list (a load) or is the unit's high bits
    struct Unit {
        uint32_t i, j, lg;
        bool live;
    };
    auto locate = [&](uint64_t it, uint32_t &list_pos) -> Unit {
        Unit o;
        list_pos = 0;
        if (planned) {
            const uint32_t tile = (uint32_t)it * S + ((it & 1u) ? S - 1 - simd : simd);
            const uint64_t hit = __ballot(lane < kClasses && my_start <= tile && tile < my_start + my_tiles);
            const uint32_t c = uniform_u32((uint32_t)(__ffsll((unsigned long long)hit) - 1));
            o.lg = uniform_u32((uint32_t)__shfl((int)my_lg, (int)c));
            const uint32_t u = (tile - uniform_u32((uint32_t)__shfl((int)my_start, (int)c))) * 64 + lane;
            const uint32_t p = u >> o.lg;
            o.live = tile < ntiles && p < uniform_u32((uint32_t)__shfl((int)my_cnt, (int)c));
            o.j = u & ((1u << o.lg) - 1);
            list_pos = o.live ? c * pp.cap + p : 0;
            o.i = 0;
        } else {
            o.lg = lg0;
            o.live = it < total;
            o.j = (uint32_t)it & ((1u << lg0) - 1);
            o.i = o.live ? (uint32_t)(it >> lg0) : 0;
        }
        return o;
    };
    // Software pipeline over a wave's units, two deep: while unit k runs, the
    // descriptor of unit k+1 and the list entry of unit k+2 are in flight, so
    // a tile starts with its descriptor in registers (the key, counter and
    // first chunks are then one round trip away, not three).  Loads are
    // unconditional (index 0 when past the end) to keep the waits exact.
    if (first >= total) return;
    uint32_t q0, q1;
    Unit cur = locate(first, q0), nxt = locate(first + stride, q1);
    if (planned) {
        cur.i = pp.lists[q0];
        nxt.i = pp.lists[q1];
    }
    rg_pkt_desc dcur = desc[cur.live ? cur.i : 0];
    for (uint64_t it = first; it < total; it += stride) {
        uint32_t q2;
        Unit far = locate(it + 2 * stride, q2);
        if (planned) far.i = pp.lists[q2];
        const rg_pkt_desc dnxt = desc[nxt.live ? nxt.i : 0];
        if (stamp && it == first) marks[2] = __builtin_amdgcn_s_memtime(); // the prologue's end
        if (cur.live) body(cur.i, dcur, cur.j, 1u << cur.lg);
        if (stamp) { // diagnostics: real-time ticks at the end of a wave's first two units
            const uint64_t now = __builtin_amdgcn_s_memrealtime();
            if (it == first) marks[0] = now;
            else if (it == first + stride) marks[1] = now;
        }
        cur = nxt;
        nxt = far;
        dcur = dnxt;
    }
}

// ------------------------------------------------------------- kernels
// Persistent grid: the host launches at most CUs x wg_per_cu workgroups with
// an LDS reservation that fixes residency.
// flags: bits 0-1 log2 lanes per packet (without a plan), kPipeLinesFlag: the LDS ring is reserved
template <int MODE> __global__ __launch_bounds__(256) void pipe_seal_kernel(SealArgs a, uint32_t flags, PipePlan pp) {
    uint64_t marks[3] = {0, 0, 0};
    const bool lines = (flags & kPipeLinesFlag) != 0;
#if RG_DIAG
    const uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    const bool stamp = a.dbg != nullptr;
#else
    constexpr bool stamp = false;
#endif
    pipe_walk(a.n, flags & 3u, pp, a.desc, stamp, marks, [=](uint32_t i, const rg_pkt_desc &d, uint32_t j, uint32_t G) {
        pipe_seal_packet<MODE>(a, i, d, j, G, lines);
    });
#if RG_DIAG
    if (stamp) pipe_stamp(a.dbg, t0, r0, marks);
#endif
}

__global__ __launch_bounds__(256) void pipe_open_kernel(OpenArgs a, uint32_t flags, PipePlan pp) {
    uint64_t marks[3] = {0, 0, 0};
    const bool lines = (flags & kPipeLinesFlag) != 0;
#if RG_DIAG
    const uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    const bool stamp = a.dbg != nullptr;
#else
    constexpr bool stamp = false;
#endif
    pipe_walk(a.n, flags & 3u, pp, a.desc, stamp, marks, [=](uint32_t i, const rg_pkt_desc &d, uint32_t j, uint32_t G) {
        pipe_open_packet(a, i, d, j, G, lines);
    });
#if RG_DIAG
    if (stamp) pipe_stamp(a.dbg, t0, r0, marks);
#endif
}

static void pipe_grid(uint64_t units, const Launch &L, uint32_t &blocks, uint32_t &lds) {
    const uint64_t want = (units + 255) / 256;
    const uint64_t cap = (uint64_t)L.cus * (uint64_t)L.wg_per_cu;
    blocks = (uint32_t)(want < cap || cap == 0 ? want : cap);
    lds = L.wg_per_cu > 0 ? (kLdsPerCu / L.wg_per_cu) & ~255u : 0;
}

hipError_t launch_pipe(const SealArgs *sa, const OpenArgs *oa, const Launch &L, const PipePlan *plan,
                       hipStream_t s) {
    const uint32_t n = sa ? sa->n : oa->n;
    if (n == 0) return hipSuccess;
    const uint32_t lg = L.lanes >= 4 ? 2 : L.lanes == 2 ? 1 : 0; // segments per packet without a plan: 1, 2, 4
    PipePlan pp{};
    uint32_t blocks, lds;
    if (plan) {
        // L.wg_per_cu 4-wave workgroups per CU, held there by the LDS reservation
        pp = *plan;
        const uint32_t wg = (uint32_t)(L.wg_per_cu > 0 ? L.wg_per_cu : 1);
        blocks = (uint32_t)(L.cus > 0 ? L.cus : 1) * wg;
        lds = (kLdsPerCu / wg) & ~255u; // sched[] was written by the planner (plan_kernel)
        // the snake deal needs the grid to be whole passes of pp.simds waves
        if (pp.simds == 0 || ((uint64_t)blocks * 4) % pp.simds != 0) return hipErrorInvalidValue;
    } else {
        pipe_grid((uint64_t)n << lg, L, blocks, lds);
    }
    const uint32_t fl = lg | (lds >= 4 * kRingBytes ? kPipeLinesFlag : 0u);
    if (oa) {
        RG_LAUNCH(L.done, pipe_open_kernel, dim3(blocks), dim3(256), lds, s, *oa, fl, pp);
        return hipGetLastError();
    }
#if RG_DIAG
    switch (L.debug_mode) { // debug mode 3 (stamps) runs the normal seal
    case 1: hipLaunchKernelGGL(pipe_seal_kernel<1>, dim3(blocks), dim3(256), lds, s, *sa, fl, pp); return hipGetLastError();
    case 2: hipLaunchKernelGGL(pipe_seal_kernel<2>, dim3(blocks), dim3(256), lds, s, *sa, fl, pp); return hipGetLastError();
    case 4: hipLaunchKernelGGL(pipe_seal_kernel<4>, dim3(blocks), dim3(256), lds, s, *sa, fl, pp); return hipGetLastError();
    case 5: hipLaunchKernelGGL(pipe_seal_kernel<5>, dim3(blocks), dim3(256), lds, s, *sa, fl, pp); return hipGetLastError();
    case 6: hipLaunchKernelGGL(pipe_seal_kernel<6>, dim3(blocks), dim3(256), lds, s, *sa, fl, pp); return hipGetLastError();
    case 7: hipLaunchKernelGGL(pipe_seal_kernel<7>, dim3(blocks), dim3(256), lds, s, *sa, fl, pp); return hipGetLastError();
    case 8: hipLaunchKernelGGL(pipe_seal_kernel<8>, dim3(blocks), dim3(256), lds, s, *sa, fl, pp); return hipGetLastError();
    default: break;
    }
#endif
    RG_LAUNCH(L.done, pipe_seal_kernel<0>, dim3(blocks), dim3(256), lds, s, *sa, fl, pp);
    return hipGetLastError();
}

hipError_t prepare_pipe_kernels(int max_wg[2]) {
    const void *f[2] = {(const void *)pipe_seal_kernel<0>, (const void *)pipe_open_kernel};
    for (int w = 0; w < 2; ++w) {
        hipError_t e = hipFuncSetAttribute(f[w], hipFuncAttributeMaxDynamicSharedMemorySize, (int)kLdsPerCu);
        if (e != hipSuccess) return e;
        int nb = 0;
        e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, f[w], 256, 0);
        if (e != hipSuccess) return e;
        max_wg[w] = nb;
    }
#if RG_DIAG
    const void *d[7] = {(const void *)pipe_seal_kernel<1>, (const void *)pipe_seal_kernel<2>,
                        (const void *)pipe_seal_kernel<4>, (const void *)pipe_seal_kernel<5>,
                        (const void *)pipe_seal_kernel<6>, (const void *)pipe_seal_kernel<7>,
                        (const void *)pipe_seal_kernel<8>};
    for (const void *k : d) {
        hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kLdsPerCu);
        if (e != hipSuccess) return e;
    }
#endif
    return hipSuccess;
}

} // namespace rg
