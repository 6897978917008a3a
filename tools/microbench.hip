// microbench.hip -- per-instruction VALU throughput on gfx950, to size the
// ChaCha20 / Poly1305 cost model in DESIGN.md.  Each kernel runs 8
// independent chains of one instruction per lane; throughput is reported as
// wave-instructions per cycle per CU relative to v_add_u32.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#include "../rustyguard_amd/csrc/rg_device.h"

#define CHECK(x)                                                              \
    do {                                                                      \
        hipError_t e = (x);                                                   \
        if (e != hipSuccess) {                                                \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));            \
            exit(1);                                                          \
        }                                                                     \
    } while (0)

constexpr int ITERS = 4096;

#define BODY8(STMT) STMT(0) STMT(1) STMT(2) STMT(3) STMT(4) STMT(5) STMT(6) STMT(7)

__global__ void k_add(uint32_t *out, uint32_t seed) {
    uint32_t a[8];
    for (int i = 0; i < 8; ++i) a[i] = seed + threadIdx.x + i;
    const uint32_t b = seed * 3;
    for (int it = 0; it < ITERS; ++it) {
#define S(i) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
        BODY8(S)
#undef S
    }
    uint32_t r = 0;
    for (int i = 0; i < 8; ++i) r ^= a[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

__global__ void k_alignbit(uint32_t *out, uint32_t seed) {
    uint32_t a[8];
    for (int i = 0; i < 8; ++i) a[i] = seed + threadIdx.x + i;
    for (int it = 0; it < ITERS; ++it) {
#define S(i) asm volatile("v_alignbit_b32 %0, %0, %0, 7" : "+v"(a[i]));
        BODY8(S)
#undef S
    }
    uint32_t r = 0;
    for (int i = 0; i < 8; ++i) r ^= a[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

__global__ void k_mad64(uint32_t *out, uint32_t seed) {
    uint64_t a[8];
    for (int i = 0; i < 8; ++i) a[i] = seed + threadIdx.x + i;
    const uint32_t x = seed | 1, y = seed * 7 + 1;
    for (int it = 0; it < ITERS; ++it) {
#define S(i) asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(a[i]) : "v"(x), "v"(y) : "vcc");
        BODY8(S)
#undef S
    }
    uint64_t r = 0;
    for (int i = 0; i < 8; ++i) r ^= a[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)(r ^ (r >> 32));
}

__global__ void k_mullo(uint32_t *out, uint32_t seed) {
    uint32_t a[8];
    for (int i = 0; i < 8; ++i) a[i] = seed + threadIdx.x + i;
    const uint32_t b = seed | 1;
    for (int it = 0; it < ITERS; ++it) {
#define S(i) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
        BODY8(S)
#undef S
    }
    uint32_t r = 0;
    for (int i = 0; i < 8; ++i) r ^= a[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

__global__ void k_mulhi(uint32_t *out, uint32_t seed) {
    uint32_t a[8];
    for (int i = 0; i < 8; ++i) a[i] = seed + threadIdx.x + i;
    const uint32_t b = seed | 1;
    for (int it = 0; it < ITERS; ++it) {
#define S(i) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
        BODY8(S)
#undef S
    }
    uint32_t r = 0;
    for (int i = 0; i < 8; ++i) r ^= a[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

__global__ void k_mul24(uint32_t *out, uint32_t seed) {
    uint32_t a[8];
    for (int i = 0; i < 8; ++i) a[i] = seed + threadIdx.x + i;
    const uint32_t b = seed | 1;
    for (int it = 0; it < ITERS; ++it) {
#define S(i) asm volatile("v_mad_u32_u24 %0, %0, %1, %0" : "+v"(a[i]) : "v"(b));
        BODY8(S)
#undef S
    }
    uint32_t r = 0;
    for (int i = 0; i < 8; ++i) r ^= a[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

__global__ void k_fma64(uint32_t *out, uint32_t seed) {
    double a[8];
    for (int i = 0; i < 8; ++i) a[i] = seed + threadIdx.x + i;
    const double b = 1.0000001, c = 0.5;
    for (int it = 0; it < ITERS; ++it) {
#define S(i) asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "v"(c));
        BODY8(S)
#undef S
    }
    double r = 0;
    for (int i = 0; i < 8; ++i) r += a[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)r;
}

__global__ void k_addco(uint32_t *out, uint32_t seed) {
    uint32_t a[8];
    for (int i = 0; i < 8; ++i) a[i] = seed + threadIdx.x + i;
    const uint32_t b = seed * 3;
    for (int it = 0; it < ITERS; ++it) {
#define S(i) asm volatile("v_add_co_u32 %0, vcc, %0, %1\n\tv_addc_co_u32 %0, vcc, %0, %1, vcc" : "+v"(a[i]) : "v"(b) : "vcc");
        BODY8(S)
#undef S
    }
    uint32_t r = 0;
    for (int i = 0; i < 8; ++i) r ^= a[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

// ChaCha20 blocks back to back (the exact device function the AEAD uses)
constexpr int CHACHA_BLOCKS = 64;
__global__ void k_chacha(uint32_t *out, uint32_t seed) {
    rg::Key8 key;
    for (int i = 0; i < 8; ++i) key.k[i] = seed * (i + 1) + threadIdx.x;
    uint32_t acc = 0, ks[16];
    for (int b = 0; b < CHACHA_BLOCKS; ++b) {
        rg::chacha_block(key, b + 1, 0u, threadIdx.x, blockIdx.x, ks);
#pragma unroll
        for (int i = 0; i < 16; ++i) acc ^= ks[i];
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

__global__ void k_chacha2(uint32_t *out, uint32_t seed) {
    rg::Key8 key;
    for (int i = 0; i < 8; ++i) key.k[i] = seed * (i + 1) + threadIdx.x;
    uint32_t acc = 0, ks[16], kt[16];
    for (int b = 0; b < CHACHA_BLOCKS; b += 2) {
        rg::chacha_block(key, b + 1, 0u, threadIdx.x, blockIdx.x, ks);
        rg::chacha_block(key, b + 2, 0u, threadIdx.x, blockIdx.x, kt);
#pragma unroll
        for (int i = 0; i < 16; ++i) acc ^= ks[i] ^ kt[i];
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

// ChaCha variants with different rotate lowerings (same arithmetic):
//  P: rot16 / rot8 as v_perm_b32 byte shuffles (rot12 / rot7 stay v_alignbit_b32)
//  S: xor + rot16 as two SDWA word-select xors, rot8 as v_perm_b32
__device__ __forceinline__ uint32_t perm_rot16(uint32_t v) { return __builtin_amdgcn_perm(v, v, 0x01000302u); }
__device__ __forceinline__ uint32_t perm_rot8(uint32_t v) { return __builtin_amdgcn_perm(v, v, 0x02010003u); }
__device__ __forceinline__ uint32_t xor_rot16_sdwa(uint32_t d, uint32_t a) {
    uint32_t t;
    asm volatile("v_xor_b32_sdwa %0, %1, %2 dst_sel:WORD_1 dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:WORD_0\n\t"
                 "v_xor_b32_sdwa %0, %1, %2 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1"
                 : "=&v"(t) : "v"(d), "v"(a));
    return t;
}
#define QR_P(a, b, c, d)                                   \
    a += b; d ^= a; d = perm_rot16(d);                      \
    c += d; b ^= c; b = rg::rotl(b, 12);                    \
    a += b; d ^= a; d = perm_rot8(d);                       \
    c += d; b ^= c; b = rg::rotl(b, 7);
#define QR_S(a, b, c, d)                                   \
    a += b; d = xor_rot16_sdwa(d, a);                       \
    c += d; b ^= c; b = rg::rotl(b, 12);                    \
    a += b; d ^= a; d = perm_rot8(d);                       \
    c += d; b ^= c; b = rg::rotl(b, 7);
#define CHACHA_VARIANT(NAME, QR)                                                       \
    __global__ void NAME(uint32_t *out, uint32_t seed) {                               \
        uint32_t k[8];                                                                 \
        for (int i = 0; i < 8; ++i) k[i] = seed * (i + 1) + threadIdx.x;              \
        uint32_t acc = 0;                                                              \
        for (int blk = 0; blk < CHACHA_BLOCKS; ++blk) {                                \
            uint32_t x0 = 0x61707865u, x1 = 0x3320646eu, x2 = 0x79622d32u, x3 = 0x6b206574u; \
            uint32_t x4 = k[0], x5 = k[1], x6 = k[2], x7 = k[3], x8 = k[4], x9 = k[5], x10 = k[6], x11 = k[7]; \
            uint32_t x12 = blk + 1, x13 = 0, x14 = threadIdx.x, x15 = blockIdx.x;       \
            _Pragma("unroll") for (int i = 0; i < 10; i++) {                           \
                QR(x0, x4, x8, x12) QR(x1, x5, x9, x13) QR(x2, x6, x10, x14) QR(x3, x7, x11, x15) \
                QR(x0, x5, x10, x15) QR(x1, x6, x11, x12) QR(x2, x7, x8, x13) QR(x3, x4, x9, x14) \
            }                                                                          \
            acc ^= (x0 + 0x61707865u) ^ (x1 + 0x3320646eu) ^ (x2 + 0x79622d32u) ^ (x3 + 0x6b206574u) ^ \
                   (x4 + k[0]) ^ (x5 + k[1]) ^ (x6 + k[2]) ^ (x7 + k[3]) ^ (x8 + k[4]) ^ (x9 + k[5]) ^ \
                   (x10 + k[6]) ^ (x11 + k[7]) ^ (x12 + blk + 1) ^ x13 ^ (x14 + threadIdx.x) ^ (x15 + blockIdx.x); \
        }                                                                              \
        out[blockIdx.x * blockDim.x + threadIdx.x] = acc;                              \
    }
CHACHA_VARIANT(k_chacha_perm, QR_P)
CHACHA_VARIANT(k_chacha_sdwa, QR_S)

// Quad ChaCha: 4 lanes per block, lane j holds column j (rows a, b, c, d =
// words j, 4+j, 8+j, 12+j); diagonal rounds rotate rows b, c, d across the
// quad with DPP quad_perm.  CHACHA_BLOCKS blocks per quad (so 4x the lanes of
// k_chacha for the same number of blocks).
template <int CTRL> __device__ __forceinline__ uint32_t qrot(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xF, 0xF, false);
}
#define QCTRL_L1 0x39 // lane j <- j+1
#define QCTRL_L2 0x4E // lane j <- j+2
#define QCTRL_L3 0x93 // lane j <- j+3
#define QQR(a, b, c, d)                                   \
    a += b; d ^= a; d = rg::rotl(d, 16);                   \
    c += d; b ^= c; b = rg::rotl(b, 12);                   \
    a += b; d ^= a; d = rg::rotl(d, 8);                    \
    c += d; b ^= c; b = rg::rotl(b, 7);
template <int ILP> __global__ void k_chacha_quad(uint32_t *out, uint32_t seed) {
    const uint32_t j = threadIdx.x & 3;
    const uint32_t k0 = seed * (j + 1) + threadIdx.x, k1 = seed * (j + 5) + threadIdx.x;
    const uint32_t a0 = 0x61707865u + j * 0x01010101u;
    uint32_t acc = 0;
    for (int blk = 0; blk < CHACHA_BLOCKS; blk += ILP) {
        uint32_t a[ILP], b[ILP], c[ILP], d[ILP];
#pragma unroll
        for (int u = 0; u < ILP; ++u) {
            a[u] = a0; b[u] = k0; c[u] = k1; d[u] = j == 0 ? (uint32_t)(blk + u + 1) : (j == 1 ? 0u : blockIdx.x + j);
        }
#pragma unroll
        for (int i = 0; i < 10; i++) {
#pragma unroll
            for (int u = 0; u < ILP; ++u) { QQR(a[u], b[u], c[u], d[u]) }
#pragma unroll
            for (int u = 0; u < ILP; ++u) {
                b[u] = qrot<QCTRL_L1>(b[u]); c[u] = qrot<QCTRL_L2>(c[u]); d[u] = qrot<QCTRL_L3>(d[u]);
            }
#pragma unroll
            for (int u = 0; u < ILP; ++u) { QQR(a[u], b[u], c[u], d[u]) }
#pragma unroll
            for (int u = 0; u < ILP; ++u) {
                b[u] = qrot<QCTRL_L3>(b[u]); c[u] = qrot<QCTRL_L2>(c[u]); d[u] = qrot<QCTRL_L1>(d[u]);
            }
        }
#pragma unroll
        for (int u = 0; u < ILP; ++u) acc ^= (a[u] + a0) ^ (b[u] + k0) ^ (c[u] + k1) ^ d[u];
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

// ChaCha with an in-kernel clock stamp: lane 0 of each wave records
// (s_memtime delta, s_memrealtime delta) into clk[wave] (100 MHz real-time).
__global__ void k_chacha_clk(uint32_t *out, uint32_t seed, unsigned long long *clk) {
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
    rg::Key8 key;
    for (int i = 0; i < 8; ++i) key.k[i] = seed * (i + 1) + threadIdx.x;
    uint32_t acc = 0, ks[16];
    for (int b = 0; b < 4 * CHACHA_BLOCKS; ++b) {
        rg::chacha_block(key, b + 1, 0u, threadIdx.x, blockIdx.x, ks);
#pragma unroll
        for (int i = 0; i < 16; ++i) acc ^= ks[i];
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
    if ((threadIdx.x & 63) == 0) {
        const uint32_t wv = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
        clk[2 * wv] = t1 - t0;
        clk[2 * wv + 1] = r1 - r0;
    }
}

// Poly1305 blocks (clamped multiply + add) back to back
constexpr int POLY_BLOCKS = 1024;
__global__ void k_poly(uint32_t *out, uint32_t seed) {
    const rg::Mul r = rg::make_mul(seed * 0x9e3779b9u, seed ^ threadIdx.x, seed + 7, seed * 3);
    rg::Acc h = {threadIdx.x, seed, 1, 2, 0};
    for (int b = 0; b < POLY_BLOCKS; ++b) {
        rg::acc_mul(h, r);
        rg::acc_add(h, b, seed, b * 3, 7, 1);
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = h.h0 ^ h.h1 ^ h.h2 ^ h.h3 ^ h.h4;
}

__global__ void k_polygen(uint32_t *out, uint32_t seed) {
    rg::Acc g = {seed * 0x9e3779b9u, seed ^ threadIdx.x, seed + 7, seed * 3, 1};
    const rg::Gen G = rg::make_gen(g);
    rg::Acc h = {threadIdx.x, seed, 1, 2, 0};
    for (int b = 0; b < POLY_BLOCKS; ++b) {
        rg::acc_mul_gen(h, G);
        rg::acc_add(h, b, seed, b * 3, 7, 1);
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = h.h0 ^ h.h1 ^ h.h2 ^ h.h3 ^ h.h4;
}


#define UNARY_KERNEL(NAME, ASM)                                                   \
    __global__ void NAME(uint32_t *out, uint32_t seed) {                          \
        uint32_t a[8];                                                            \
        for (int i = 0; i < 8; ++i) a[i] = seed + threadIdx.x + i;                \
        const uint32_t b = seed * 3 + 1, c = seed ^ 0x55;                         \
        for (int it = 0; it < ITERS; ++it) {                                      \
            _Pragma("unroll") for (int i = 0; i < 8; ++i) asm volatile(ASM : "+v"(a[i]) : "v"(b), "v"(c)); \
        }                                                                         \
        uint32_t r = 0;                                                           \
        for (int i = 0; i < 8; ++i) r ^= a[i];                                    \
        out[blockIdx.x * blockDim.x + threadIdx.x] = r;                           \
    }

UNARY_KERNEL(k_xor, "v_xor_b32 %0, %0, %1")
UNARY_KERNEL(k_and, "v_and_b32 %0, %0, %1")
UNARY_KERNEL(k_lshl, "v_lshlrev_b32 %0, 3, %0")
UNARY_KERNEL(k_perm, "v_perm_b32 %0, %0, %0, %1")
UNARY_KERNEL(k_xor3, "v_or3_b32 %0, %0, %1, %2")
UNARY_KERNEL(k_add3, "v_add3_u32 %0, %0, %1, %2")
UNARY_KERNEL(k_lshlor, "v_lshl_or_b32 %0, %0, 3, %1")
UNARY_KERNEL(k_xad, "v_xad_u32 %0, %0, %1, %2")
UNARY_KERNEL(k_alignbit2, "v_alignbit_b32 %0, %0, %1, 7")
UNARY_KERNEL(k_add_e64, "v_add_u32_e64 %0, %0, %1")
UNARY_KERNEL(k_xor_e64, "v_xor_b32_e64 %0, %0, %1")
UNARY_KERNEL(k_mov, "v_mov_b32 %0, %1")
UNARY_KERNEL(k_pkadd16, "v_pk_add_u16 %0, %0, %1")
UNARY_KERNEL(k_xor_sdwa, "v_xor_b32_sdwa %0, %0, %1 dst_sel:DWORD dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:DWORD")
UNARY_KERNEL(k_mix, "v_add_u32 %0, %0, %1\n\tv_xor_b32 %0, %0, %2\n\tv_alignbit_b32 %0, %0, %0, 16")

typedef void (*kfn)(uint32_t *, uint32_t);

// units processed per ns per CU (blocks for chacha/poly).  Dynamic LDS of
// 160 KiB / waves_per_simd per 256-thread block forces exactly that many
// blocks (= waves per SIMD) onto every CU.
static double run_units(kfn f, int waves_per_simd, uint32_t *d, double units_per_lane) {
    const int threads = 256;
    const int blocks = 256 * waves_per_simd;
    const size_t lds = (160 * 1024 / waves_per_simd) & ~255;
    CHECK(hipFuncSetAttribute((const void *)f, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    hipLaunchKernelGGL(f, dim3(blocks), dim3(threads), lds, 0, d, 1u);
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(a));
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(f, dim3(blocks), dim3(threads), lds, 0, d, 1u);
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms;
    CHECK(hipEventElapsedTime(&ms, a, b));
    return 5.0 * blocks * threads * units_per_lane / (ms * 1e6) / 256.0;
}

static double run(kfn f, int waves_per_simd, uint32_t *d, int insts_per_iter) {
    const int threads = 256;
    const int blocks = 256 * waves_per_simd; // 4 waves/block -> waves_per_simd waves per SIMD
    const size_t lds = (160 * 1024 / waves_per_simd) & ~255;
    CHECK(hipFuncSetAttribute((const void *)f, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    hipLaunchKernelGGL(f, dim3(blocks), dim3(threads), lds, 0, d, 1u);
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(a));
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(f, dim3(blocks), dim3(threads), lds, 0, d, 1u);
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms;
    CHECK(hipEventElapsedTime(&ms, a, b));
    const double wave_insts = 5.0 * blocks * (threads / 64) * (double)ITERS * 8 * insts_per_iter;
    // wave-instructions per ns per CU
    return wave_insts / (ms * 1e6) / 256.0;
}

int main() {
    uint32_t *d;
    CHECK(hipMalloc(&d, 256 * 16 * 256 * 4 * 2));
    struct {
        const char *name;
        kfn f;
        int per;
    } ks[] = {{"v_add_u32", k_add, 1},       {"v_alignbit_b32", k_alignbit, 1}, {"v_mad_u64_u32", k_mad64, 1},
              {"v_mul_lo_u32", k_mullo, 1},  {"v_mul_hi_u32", k_mulhi, 1},      {"v_mad_u32_u24", k_mul24, 1},
              {"v_fma_f64", k_fma64, 1},     {"add_co+addc", k_addco, 2},
              {"v_xor_b32", k_xor, 1}, {"v_and_b32", k_and, 1}, {"v_lshlrev_b32", k_lshl, 1},
              {"v_perm_b32", k_perm, 1}, {"v_or3_b32", k_xor3, 1}, {"v_add3_u32", k_add3, 1},
              {"v_lshl_or_b32", k_lshlor, 1}, {"v_xad_u32", k_xad, 1}, {"v_alignbit_b32(2src)", k_alignbit2, 1},
              {"v_add_u32_e64", k_add_e64, 1}, {"v_xor_b32_e64", k_xor_e64, 1}, {"v_mov_b32", k_mov, 1},
              {"v_pk_add_u16", k_pkadd16, 1}, {"v_xor_b32_sdwa", k_xor_sdwa, 1},
              {"add+xor+alignbit", k_mix, 3}};
    printf("{\"unit\": \"wave-instructions per ns per CU (x64 lanes)\", \"results\": [\n");
    bool first = true;
    for (auto &k : ks) {
        for (int w : {1, 2, 4, 8}) {
            double r = run(k.f, w, d, k.per);
            printf("%s{\"inst\": \"%s\", \"waves_per_simd\": %d, \"rate\": %.4f}\n", first ? "" : ",", k.name, w, r);
            first = false;
        }
    }
    printf("], \"kernels\": [\n");
    first = true;
    struct {
        const char *name;
        kfn f;
        double units;
    } ku[] = {{"chacha_block", k_chacha, CHACHA_BLOCKS}, {"chacha_block_x2", k_chacha2, CHACHA_BLOCKS},
              {"chacha_perm_rot", k_chacha_perm, CHACHA_BLOCKS},
              {"chacha_quad_ilp1", k_chacha_quad<1>, CHACHA_BLOCKS / 4.0}, {"chacha_quad_ilp2", k_chacha_quad<2>, CHACHA_BLOCKS / 4.0}, {"chacha_sdwa_rot16", k_chacha_sdwa, CHACHA_BLOCKS},
              {"poly_clamped_block", k_poly, POLY_BLOCKS},
              {"poly_general_block", k_polygen, POLY_BLOCKS}};
    for (auto &k : ku) {
        for (int w : {1, 2, 3, 4, 6, 8}) {
            double r = run_units(k.f, w, d, k.units);
            printf("%s{\"kernel\": \"%s\", \"waves_per_simd\": %d, \"per_ns_per_cu\": %.4f, "
                   "\"chip_GB_s\": %.1f}\n", first ? "" : ",", k.name, w, r,
                   r * 256 * ((k.f == k_chacha || k.f == k_chacha2 || k.f == k_chacha_perm || k.f == k_chacha_sdwa || k.f == k_chacha_quad<1> || k.f == k_chacha_quad<2>) ? 64 : 16));
            first = false;
        }
    }
    printf("], \"clock\": [\n");
    {
        unsigned long long *dclk;
        const int maxw = 256 * 8 * 4;
        CHECK(hipMalloc(&dclk, sizeof(unsigned long long) * 2 * maxw));
        CHECK(hipFuncSetAttribute((const void *)k_chacha_clk, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
        bool f2 = true;
        for (int w : {1, 2, 4, 8}) {
            const int blocks = 256 * w;
            const size_t lds = (160 * 1024 / w) & ~255;
            for (int rep = 0; rep < 3; ++rep)
                hipLaunchKernelGGL(k_chacha_clk, dim3(blocks), dim3(256), lds, 0, d, 1u, dclk);
            CHECK(hipDeviceSynchronize());
            static unsigned long long h[2 * 256 * 8 * 4];
            CHECK(hipMemcpy(h, dclk, sizeof(unsigned long long) * 2 * blocks * 4, hipMemcpyDeviceToHost));
            double sum = 0;
            for (int i = 0; i < blocks * 4; ++i) sum += (double)h[2 * i] / (double)h[2 * i + 1] * 0.1;
            printf("%s{\"waves_per_simd\": %d, \"clock_GHz\": %.3f, \"cycles_per_wave_block\": %.0f}\n",
                   f2 ? "" : ",", w, sum / (blocks * 4), (double)h[0] / (4 * CHACHA_BLOCKS));
            f2 = false;
        }
    }
    printf("]}\n");
    return 0;
}
