// tailbench.hip -- what sets the ~6 us between the last wave's end and the end of a store-heavy kernel
// (config 2's seal: profiles/r2c_cfg2_experiments.txt).  1024 waves (one per SIMD, as the pipelined
// kernel), each running ITERS steps of ~4 k cycles of VALU work and four 16-byte-per-lane stores (4 KB
// per wave and step, coalesced), ~100 MB per launch like a config-2 seal.  Variants:
//   flavour: plain stores / sc1 (write-through) / nt
//   when:    every step / only in the first half of the steps (none in flight at the end) / never
// Reported: event time per launch, the waves' wall span from s_memrealtime stamps (100 MHz), and
// tail = event time - span.  If the tail follows the dirty bytes left in L2 (plain, first half) it is
// the end-of-kernel write-back; if it follows the stores in flight at the end (every step) it is the
// final burst.
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

template <int FLAVOUR> __device__ __forceinline__ void st(v4u *p, v4u v) {
    if constexpr (FLAVOUR == 1)
        asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
    else if constexpr (FLAVOUR == 2)
        asm volatile("global_store_dwordx4 %0, %1, off nt\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
    else
        asm volatile("global_store_dwordx4 %0, %1, off\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
}

// WHEN: 0 = stores every step, 1 = only in the first half of the steps, 2 = never
template <int FLAVOUR, int WHEN> __global__ __launch_bounds__(256) void k_tail(v4u *buf, unsigned long long *stamps, uint32_t seed) {
    const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
    const uint32_t lane = threadIdx.x & 63, wave = blockIdx.x * 4 + threadIdx.x / 64;
    uint32_t a = seed + threadIdx.x, b = seed ^ lane, c = seed * 3 + wave, d = seed + 7;
    for (int it = 0; it < ITERS; ++it) {
        // ~1000 VALU instructions, four independent chains (the ChaCha block's ILP)
        for (int k = 0; k < 250; ++k) {
            asm volatile("v_add_u32 %0, %0, %1\n\tv_xor_b32 %1, %1, %2\n\tv_alignbit_b32 %2, %2, %2, 7\n\tv_add_u32 %3, %3, %0"
                         : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
        }
        if (WHEN == 0 || (WHEN == 1 && it < ITERS / 2)) {
            v4u *p = buf + ((size_t)(it * WAVES + wave) * 4) * 64 + lane;
            st<FLAVOUR>(p, v4u{a, b, c, d});
            st<FLAVOUR>(p + 64, v4u{b, c, d, a});
            st<FLAVOUR>(p + 128, v4u{c, d, a, b});
            st<FLAVOUR>(p + 192, v4u{d, a, b, c});
        }
    }
    if (WHEN == 2 && (a ^ b ^ c ^ d) == 0x12345678u) buf[lane] = v4u{a, b, c, d};
    const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
    if (lane == 0) {
        stamps[2 * wave] = r0;
        stamps[2 * wave + 1] = r1;
    }
}

typedef void (*kfn)(v4u *, unsigned long long *, uint32_t);

int main() {
    const size_t bytes = (size_t)ITERS * WAVES * 4 * 1024;
    v4u *buf;
    unsigned long long *stamps;
    CHECK(hipMalloc(&buf, bytes));
    CHECK(hipMalloc(&stamps, sizeof(unsigned long long) * 2 * WAVES));
    CHECK(hipMemset(buf, 0, bytes));
    struct {
        const char *name;
        kfn f;
    } ks[] = {{"plain_every", k_tail<0, 0>}, {"plain_first_half", k_tail<0, 1>}, {"sc1_every", k_tail<1, 0>},
              {"sc1_first_half", k_tail<1, 1>}, {"nt_every", k_tail<2, 0>},          {"none", k_tail<0, 2>}};
    const size_t lds = 160 * 1024; // one 4-wave workgroup per CU: one wave per SIMD
    printf("[\n");
    bool first = true;
    for (int rep = 0; rep < 2; ++rep)
        for (auto &k : ks) {
            CHECK(hipFuncSetAttribute((const void *)k.f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
            hipEvent_t e0, e1;
            CHECK(hipEventCreate(&e0));
            CHECK(hipEventCreate(&e1));
            std::vector<float> ev;
            std::vector<double> span;
            for (int r = 0; r < 7; ++r) {
                hipLaunchKernelGGL(k.f, dim3(WAVES / 4), dim3(256), lds, 0, buf, stamps, 1u); // previous launch's lines out of the way
                CHECK(hipEventRecord(e0));
                hipLaunchKernelGGL(k.f, dim3(WAVES / 4), dim3(256), lds, 0, buf, stamps, 2u + r);
                CHECK(hipEventRecord(e1));
                CHECK(hipEventSynchronize(e1));
                float ms;
                CHECK(hipEventElapsedTime(&ms, e0, e1));
                static unsigned long long h[2 * WAVES];
                CHECK(hipMemcpy(h, stamps, sizeof(h), hipMemcpyDeviceToHost));
                unsigned long long lo = ~0ull, hi = 0;
                for (int w = 0; w < WAVES; ++w) {
                    lo = std::min(lo, h[2 * w]);
                    hi = std::max(hi, h[2 * w + 1]);
                }
                ev.push_back(ms * 1000.f);
                span.push_back((double)(hi - lo) / 100.0); // 100 MHz ticks -> us
            }
            std::sort(ev.begin(), ev.end());
            std::sort(span.begin(), span.end());
            printf("%s{\"rep\": %d, \"variant\": \"%s\", \"event_us\": %.2f, \"wave_span_us\": %.2f, \"tail_us\": %.2f, \"mb\": %.1f}\n",
                   first ? "" : ",", rep, k.name, ev[3], span[3], ev[3] - span[3], bytes / 1e6);
            first = false;
            CHECK(hipEventDestroy(e0));
            CHECK(hipEventDestroy(e1));
        }
    printf("]\n");
    return 0;
}
