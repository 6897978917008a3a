// l2tail.hip -- VERDICT r5 item 3: does the tail after a store-heavy kernel's last wave scale with the dirty
// bytes its stores leave in the XCDs' L2s (MI355X_MICROARCH.md "boundary" row: + B / 6 TB/s when the
// predecessor leaves B bytes dirty)?  tailbench.hip's shape (1024 waves, one per SIMD, 24 steps of ~1000
// VALU instructions and four coalesced 16-B stores per lane, 100 MB per launch) with the cache policy of
// each step chosen at run time:
//   plain_last K : steps < 24 - K write-through (sc1: no dirty line), the last K steps plain (write-back):
//                  4 MiB of plain stores per step, so K steps leave up to 4 K MiB dirty (32 MiB of L2 in all)
//   sc1_last K   : the converse -- plain stores, the last K steps write-through (the lever: only the final
//                  stores of each wave made write-through)
// Reported per variant: event time per launch, the waves' wall span (s_memrealtime, 100 MHz) and
// tail = event - span, median of 7.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                   \
    do {                                                                           \
        hipError_t e_ = (x);                                                       \
        if (e_ != hipSuccess) {                                                    \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                               \
        }                                                                          \
    } while (0)

constexpr int ITERS = 24;
constexpr int WAVES = 1024;

typedef unsigned v4u __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void st_wt(v4u *p, v4u v) {
    asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
}
__device__ __forceinline__ void st_wb(v4u *p, v4u v) {
    asm volatile("global_store_dwordx4 %0, %1, off\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
}

// steps [lo, hi) store write-back, the others write-through
__global__ __launch_bounds__(256) void k_tail(v4u *buf, unsigned long long *stamps, uint32_t seed, int lo, int hi) {
    const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
    const uint32_t lane = threadIdx.x & 63, wave = blockIdx.x * 4 + threadIdx.x / 64;
    uint32_t a = seed + threadIdx.x, b = seed ^ lane, c = seed * 3 + wave, d = seed + 7;
    for (int it = 0; it < ITERS; ++it) {
        for (int k = 0; k < 250; ++k)
            asm volatile("v_add_u32 %0, %0, %1\n\tv_xor_b32 %1, %1, %2\n\tv_alignbit_b32 %2, %2, %2, 7\n\tv_add_u32 %3, %3, %0"
                         : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
        v4u *p = buf + ((size_t)(it * WAVES + wave) * 4) * 64 + lane;
        if (it >= lo && it < hi) { // wave-uniform
            st_wb(p, v4u{a, b, c, d});
            st_wb(p + 64, v4u{b, c, d, a});
            st_wb(p + 128, v4u{c, d, a, b});
            st_wb(p + 192, v4u{d, a, b, c});
        } else {
            st_wt(p, v4u{a, b, c, d});
            st_wt(p + 64, v4u{b, c, d, a});
            st_wt(p + 128, v4u{c, d, a, b});
            st_wt(p + 192, v4u{d, a, b, c});
        }
    }
    const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
    if (lane == 0) {
        stamps[2 * wave] = r0;
        stamps[2 * wave + 1] = r1;
    }
}

int main() {
    const size_t bytes = (size_t)ITERS * WAVES * 4 * 1024;
    v4u *buf;
    unsigned long long *stamps;
    CHECK(hipMalloc(&buf, bytes));
    CHECK(hipMalloc(&stamps, sizeof(unsigned long long) * 2 * WAVES));
    CHECK(hipMemset(buf, 0, bytes));
    const size_t lds = 160 * 1024; // one 4-wave workgroup per CU: one wave per SIMD
    CHECK(hipFuncSetAttribute((const void *)k_tail, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    const int ks[] = {0, 1, 2, 4, 6, 8, 12, 24};
    printf("[\n");
    bool first = true;
    for (int rep = 0; rep < 2; ++rep)
        for (int variant = 0; variant < 2; ++variant)
            for (int k : ks) {
                // plain_last k: write-back steps [24 - k, 24); sc1_last k: write-back steps [0, 24 - k)
                const int lo = variant == 0 ? ITERS - k : 0, hi = variant == 0 ? ITERS : ITERS - k;
                std::vector<float> ev;
                std::vector<double> span;
                for (int r = 0; r < 7; ++r) {
                    hipLaunchKernelGGL(k_tail, dim3(WAVES / 4), dim3(256), lds, 0, buf, stamps, 1u, 0, ITERS);
                    CHECK(hipEventRecord(e0));
                    hipLaunchKernelGGL(k_tail, dim3(WAVES / 4), dim3(256), lds, 0, buf, stamps, 2u + r, lo, hi);
                    CHECK(hipEventRecord(e1));
                    CHECK(hipEventSynchronize(e1));
                    float ms;
                    CHECK(hipEventElapsedTime(&ms, e0, e1));
                    static unsigned long long h[2 * WAVES];
                    CHECK(hipMemcpy(h, stamps, sizeof(h), hipMemcpyDeviceToHost));
                    unsigned long long a = ~0ull, b = 0;
                    for (int w = 0; w < WAVES; ++w) {
                        a = std::min(a, h[2 * w]);
                        b = std::max(b, h[2 * w + 1]);
                    }
                    ev.push_back(ms * 1000.f);
                    span.push_back((double)(b - a) / 100.0);
                }
                std::sort(ev.begin(), ev.end());
                std::sort(span.begin(), span.end());
                printf("%s{\"rep\": %d, \"variant\": \"%s\", \"k\": %d, \"wb_mib\": %d, \"event_us\": %.2f, "
                       "\"wave_span_us\": %.2f, \"tail_us\": %.2f}\n",
                       first ? "" : ",", rep, variant == 0 ? "plain_last" : "sc1_last", k,
                       4 * (hi - lo), ev[3], span[3], ev[3] - span[3]);
                first = false;
            }
    printf("]\n");
    return 0;
}
