// mempattern.hip -- memory-only access patterns of the transport kernels at
// config-2 geometry (64 Ki frames, 1536-B stride, payload 1504 B at +16):
// read-modify-write of every payload byte, 2-chunk-deep register prefetch,
// no cryptography.  Reports GB/s of algorithmic traffic (2 x payload).
//   scattered : lane = packet, each dwordx4 instruction touches 64 frames
//   quad      : 4 lanes per 64-B chunk, each instruction covers 16 frames
//   quad_lds  : quad loads + wave-private LDS transpose to lane = packet and back
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                      \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                  \
        }                                                                             \
    } while (0)

constexpr int N = 65536, STRIDE = 1536, NB = 94; // 16-B blocks per payload
constexpr int C = (NB + 3) / 4;                  // chunks (last one: 2 blocks)

struct Q4 {
    uint4 a, b, c, d;
};

__device__ __forceinline__ uint4 x4(uint4 v, uint32_t k) { return make_uint4(v.x ^ k, v.y ^ k, v.z ^ k, v.w ^ k); }

// lane = packet; piece q of chunk t at frame + 16 + 64 t + 16 q
__global__ __launch_bounds__(256) void k_scattered(uint8_t *buf) {
    const uint32_t p = blockIdx.x * 256 + threadIdx.x;
    uint4 *pl = reinterpret_cast<uint4 *>(buf + (size_t)p * STRIDE + 16);
    auto ld = [&](Q4 &q, int t) {
        q.a = pl[min(4 * t + 0, NB - 1)]; q.b = pl[min(4 * t + 1, NB - 1)];
        q.c = pl[min(4 * t + 2, NB - 1)]; q.d = pl[min(4 * t + 3, NB - 1)];
    };
    Q4 b0, b1;
    ld(b0, 0);
    ld(b1, 1);
    int t = 0;
    for (; t + 1 < NB / 4; t += 2) {
        uint4 *d = pl + 4 * t;
        d[0] = x4(b0.a, t); d[1] = x4(b0.b, t); d[2] = x4(b0.c, t); d[3] = x4(b0.d, t);
        ld(b0, t + 2);
        d += 4;
        d[0] = x4(b1.a, t); d[1] = x4(b1.b, t); d[2] = x4(b1.c, t); d[3] = x4(b1.d, t);
        ld(b1, t + 3);
    }
    for (; t < C; ++t) { // tail (uniform: 23 full + 1 half chunk)
        Q4 &b = (t & 1) ? b1 : b0;
        uint4 *d = pl + 4 * t;
        const int cnt = min(4, NB - 4 * t);
        d[0] = x4(b.a, t);
        if (cnt > 1) d[1] = x4(b.b, t);
        if (cnt > 2) d[2] = x4(b.c, t);
        if (cnt > 3) d[3] = x4(b.d, t);
    }
}

// scattered with a 4-chunk-deep prefetch (4 register sets)
__global__ __launch_bounds__(256) void k_scattered4(uint8_t *buf) {
    const uint32_t p = blockIdx.x * 256 + threadIdx.x;
    uint4 *pl = reinterpret_cast<uint4 *>(buf + (size_t)p * STRIDE + 16);
    auto ld = [&](Q4 &q, int t) {
        q.a = pl[min(4 * t + 0, NB - 1)]; q.b = pl[min(4 * t + 1, NB - 1)];
        q.c = pl[min(4 * t + 2, NB - 1)]; q.d = pl[min(4 * t + 3, NB - 1)];
    };
    auto st = [&](Q4 &b, int t) {
        uint4 *d = pl + 4 * t;
        d[0] = x4(b.a, t); d[1] = x4(b.b, t); d[2] = x4(b.c, t); d[3] = x4(b.d, t);
    };
    Q4 b0, b1, b2, b3;
    ld(b0, 0); ld(b1, 1); ld(b2, 2); ld(b3, 3);
    int t = 0;
    for (; t + 3 < NB / 4; t += 4) {
        st(b0, t); ld(b0, t + 4);
        st(b1, t + 1); ld(b1, t + 5);
        st(b2, t + 2); ld(b2, t + 6);
        st(b3, t + 3); ld(b3, t + 7);
    }
    for (; t < C; ++t) {
        Q4 &b = (t & 3) == 0 ? b0 : (t & 3) == 1 ? b1 : (t & 3) == 2 ? b2 : b3;
        uint4 *d = pl + 4 * t;
        const int cnt = min(4, NB - 4 * t);
        d[0] = x4(b.a, t);
        if (cnt > 1) d[1] = x4(b.b, t);
        if (cnt > 2) d[2] = x4(b.c, t);
        if (cnt > 3) d[3] = x4(b.d, t);
    }
}

// wave of 64 packets; load instruction k: lane l -> packet 16k + l/4, piece l%4
template <bool LDS> __global__ __launch_bounds__(256) void k_quad(uint8_t *buf) {
    __shared__ uint4 lds[4][64 * 4]; // [wave][packet][piece ^ swizzle]
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint32_t wave_p0 = (blockIdx.x * 4 + w) * 64;
    uint4 *pk[4];
#pragma unroll
    for (int k = 0; k < 4; ++k)
        pk[k] = reinterpret_cast<uint4 *>(buf + (size_t)(wave_p0 + 16 * k + lane / 4) * STRIDE + 16) + (lane & 3);
    auto ld = [&](Q4 &q, int t) {
        const int o = min(4 * t, NB - 4); // chunk start clamped (pieces past NB: harmless in-frame reads)
        q.a = pk[0][o]; q.b = pk[1][o]; q.c = pk[2][o]; q.d = pk[3][o];
    };
    auto process = [&](Q4 &b, int t) {
        const int o = 4 * t;
        if constexpr (LDS) {
            // transpose to lane = packet (swizzled), XOR, transpose back
            uint4 *L = lds[w];
            // packet p keeps piece q in slot q ^ ((p >> 2) & 3): conflict-free both ways
            const uint32_t sw = (lane >> 2) & 3, wsl = (lane & 3) ^ ((lane >> 4) & 3);
            L[(0 * 16 + lane / 4) * 4 + wsl] = b.a;
            L[(1 * 16 + lane / 4) * 4 + wsl] = b.b;
            L[(2 * 16 + lane / 4) * 4 + wsl] = b.c;
            L[(3 * 16 + lane / 4) * 4 + wsl] = b.d;
            uint4 m0 = L[lane * 4 + (0 ^ sw)], m1 = L[lane * 4 + (1 ^ sw)], m2 = L[lane * 4 + (2 ^ sw)],
                  m3 = L[lane * 4 + (3 ^ sw)];
            L[lane * 4 + (0 ^ sw)] = x4(m0, t);
            L[lane * 4 + (1 ^ sw)] = x4(m1, t);
            L[lane * 4 + (2 ^ sw)] = x4(m2, t);
            L[lane * 4 + (3 ^ sw)] = x4(m3, t);
            b.a = L[(0 * 16 + lane / 4) * 4 + wsl];
            b.b = L[(1 * 16 + lane / 4) * 4 + wsl];
            b.c = L[(2 * 16 + lane / 4) * 4 + wsl];
            b.d = L[(3 * 16 + lane / 4) * 4 + wsl];
        } else {
            b.a = x4(b.a, t); b.b = x4(b.b, t); b.c = x4(b.c, t); b.d = x4(b.d, t);
        }
        if (o + (int)(lane & 3) < NB) {
            pk[0][o] = b.a; pk[1][o] = b.b; pk[2][o] = b.c; pk[3][o] = b.d;
        }
    };
    Q4 b0, b1;
    ld(b0, 0);
    ld(b1, 1);
    int t = 0;
    for (; t + 1 < NB / 4; t += 2) {
        process(b0, t);
        ld(b0, t + 2);
        process(b1, t + 1);
        ld(b1, t + 3);
    }
    for (; t < C; ++t) process((t & 1) ? b1 : b0, t);
}

int main() {
    uint8_t *buf;
    const size_t bytes = (size_t)N * STRIDE;
    CHECK(hipMalloc(&buf, bytes));
    CHECK(hipMemset(buf, 1, bytes));
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    struct {
        const char *name;
        void (*f)(uint8_t *);
    } ks[] = {{"scattered", k_scattered}, {"scattered4", k_scattered4}, {"quad", k_quad<false>}, {"quad_lds", k_quad<true>}};
    printf("[\n");
    bool first = true;
    for (auto &k : ks) {
        for (int rep = 0; rep < 3; ++rep) hipLaunchKernelGGL(k.f, dim3(N / 256), dim3(256), 0, 0, buf);
        CHECK(hipDeviceSynchronize());
        const int iters = 20;
        CHECK(hipEventRecord(a));
        for (int i = 0; i < iters; ++i) hipLaunchKernelGGL(k.f, dim3(N / 256), dim3(256), 0, 0, buf);
        CHECK(hipEventRecord(b));
        CHECK(hipEventSynchronize(b));
        float ms;
        CHECK(hipEventElapsedTime(&ms, a, b));
        const double us = ms * 1e3 / iters;
        printf("%s{\"pattern\": \"%s\", \"us\": %.2f, \"GB_s\": %.1f}\n", first ? "" : ",", k.name, us,
               2.0 * N * NB * 16 / (us * 1e3));
        first = false;
    }
    printf("]\n");
    return 0;
}
