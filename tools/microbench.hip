// microbench.hip -- per-instruction VALU throughput on gfx950, to size the
// ChaCha20 / Poly1305 cost model in DESIGN.md.  Each kernel runs 8
// independent chains of one instruction per lane; throughput is reported as
// wave-instructions per cycle per CU relative to v_add_u32.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

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

typedef void (*kfn)(uint32_t *, uint32_t);

static double run(kfn f, int waves_per_simd, uint32_t *d, int insts_per_iter) {
    const int threads = 256;
    const int blocks = 256 * waves_per_simd; // 4 waves/block -> waves_per_simd waves per SIMD
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    hipLaunchKernelGGL(f, dim3(blocks), dim3(threads), 0, 0, d, 1u);
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(a));
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(f, dim3(blocks), dim3(threads), 0, 0, d, 1u);
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
    CHECK(hipMalloc(&d, 256 * 16 * 256 * 4));
    struct {
        const char *name;
        kfn f;
        int per;
    } ks[] = {{"v_add_u32", k_add, 1},       {"v_alignbit_b32", k_alignbit, 1}, {"v_mad_u64_u32", k_mad64, 1},
              {"v_mul_lo_u32", k_mullo, 1},  {"v_mul_hi_u32", k_mulhi, 1},      {"v_mad_u32_u24", k_mul24, 1},
              {"v_fma_f64", k_fma64, 1},     {"add_co+addc", k_addco, 2}};
    printf("{\"unit\": \"wave-instructions per ns per CU (x64 lanes)\", \"results\": [\n");
    bool first = true;
    for (auto &k : ks) {
        for (int w : {1, 2, 4, 8}) {
            double r = run(k.f, w, d, k.per);
            printf("%s{\"inst\": \"%s\", \"waves_per_simd\": %d, \"rate\": %.4f}\n", first ? "" : ",", k.name, w, r);
            first = false;
        }
    }
    printf("]}\n");
    return 0;
}
