// splitbench.hip -- does a ChaCha20 wave and a Poly1305 wave sharing a SIMD beat one wave doing both?
// The pipelined kernel runs one wave per SIMD and absorbs each chunk's four Poly1305 blocks inside the
// next keystream block's rounds (stream_block_hooked); there its v_mad_u64_u32 issue every 8 cycles.
// Here, with no memory traffic, ITERS steps of [one keystream block + four Poly1305 blocks] per lane:
//   fused: 1 wave per SIMD, the Poly1305 blocks in the keystream rounds (as rg_pipe.hip)
//   split: 2 waves per SIMD, waves 0-3 of a workgroup the keystream blocks, waves 4-7 the Poly1305
//          blocks (same counts, no synchronisation: the upper bound of a producer/consumer split)
//   chacha: 1 wave per SIMD, keystream only; poly: 1 wave per SIMD, Poly1305 only
//   poly2 / fused2 (round 5): the same Poly1305 blocks as two independent Horner chains
//          (even / odd blocks; the r^2 combine left out, so an upper bound on what the extra ILP saves)
// Reported: event time per launch (1024 SIMDs' worth of work in every variant).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../rustyguard_amd/csrc/rg_device.h"

#define CHECK(x)                                                                   \
    do {                                                                           \
        hipError_t e_ = (x);                                                       \
        if (e_ != hipSuccess) {                                                    \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                               \
        }                                                                          \
    } while (0)

constexpr int ITERS = 24;

__device__ __forceinline__ rg::Stream mk_stream(uint32_t seed) {
    rg::Key8 k;
    for (int i = 0; i < 8; ++i) k.k[i] = seed * (i + 3) + threadIdx.x;
    return rg::make_stream(k, 0u, seed, threadIdx.x);
}

// MODE 0 fused, 1 split, 2 chacha only, 3 poly only, 4 poly only in two chains, 5 fused with two chains
template <int MODE> __global__ __launch_bounds__(512) void k_split(uint32_t *out, uint32_t seed) {
    const uint32_t wv = threadIdx.x >> 6;
    const bool poly_wave = MODE == 1 && wv >= 4;
    const rg::Stream st = mk_stream(seed);
    const rg::Mul r = rg::make_mul(seed * 0x9e3779b9u, seed ^ threadIdx.x, seed + 7, seed * 3);
    rg::Acc h = {threadIdx.x, seed, 1, 2, 0};
    rg::Acc g = {seed, threadIdx.x, 3, 4, 0}; // the second chain (MODES 4, 5)
    uint4 m0 = make_uint4(seed, 1, 2, 3), m1 = make_uint4(4, seed, 6, 7), m2 = make_uint4(8, 9, seed, 11),
          m3 = make_uint4(12, 13, 14, seed);
    uint32_t acc = 0;
    for (int t = 0; t < ITERS; ++t) {
        if (MODE == 4) {
            rg::acc_block(h, m0, r);
            rg::acc_block(g, m1, r);
            rg::acc_block(h, m2, r);
            rg::acc_block(g, m3, r);
            m0.x += h.h0; m1.y ^= g.h1; m2.z += h.h2; m3.w ^= g.h3;
            continue;
        }
        if (MODE == 3 || poly_wave) {
            rg::acc_block(h, m0, r);
            rg::acc_block(h, m1, r);
            rg::acc_block(h, m2, r);
            rg::acc_block(h, m3, r);
            m0.x += h.h0; m1.y ^= h.h1; m2.z += h.h2; m3.w ^= h.h3;
            continue;
        }
        uint32_t ks[16];
        if (MODE == 0) {
            rg::stream_block_hooked(st, t + 1, ks, [&](int dr) {
                if (dr == 1) rg::acc_block(h, m0, r);
                if (dr == 3) rg::acc_block(h, m1, r);
                if (dr == 5) rg::acc_block(h, m2, r);
                if (dr == 7) rg::acc_block(h, m3, r);
                if (dr % 2 == 1) rg::pin_acc(h);
            });
        } else if (MODE == 5) {
            rg::stream_block_hooked(st, t + 1, ks, [&](int dr) {
                if (dr == 1) rg::acc_block(h, m0, r);
                if (dr == 3) rg::acc_block(g, m1, r);
                if (dr == 5) rg::acc_block(h, m2, r);
                if (dr == 7) rg::acc_block(g, m3, r);
                if (dr % 2 == 1) { rg::pin_acc(h); rg::pin_acc(g); }
            });
        } else {
            rg::stream_block(st, t + 1, ks);
        }
        m0 = rg::xor4(m0, ks + 0); m1 = rg::xor4(m1, ks + 4); m2 = rg::xor4(m2, ks + 8); m3 = rg::xor4(m3, ks + 12);
    }
    acc = m0.x ^ m1.y ^ m2.z ^ m3.w ^ h.h0 ^ h.h1 ^ h.h2 ^ h.h3 ^ h.h4 ^ g.h0 ^ g.h1 ^ g.h2 ^ g.h3 ^ g.h4;
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

typedef void (*kfn)(uint32_t *, uint32_t);

int main() {
    uint32_t *d;
    CHECK(hipMalloc(&d, 256 * 512 * 4));
    struct {
        const char *name;
        kfn f;
        int threads;
    } ks[] = {{"fused_1wave", k_split<0>, 256}, {"split_2waves", k_split<1>, 512},
              {"chacha_only_1wave", k_split<2>, 256}, {"poly_only_1wave", k_split<3>, 256},
              {"poly_only_2chains", k_split<4>, 256}, {"fused_2chains", k_split<5>, 256}};
    printf("[\n");
    bool first = true;
    for (int rep = 0; rep < 2; ++rep)
        for (auto &k : ks) {
            CHECK(hipFuncSetAttribute((const void *)k.f, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
            hipEvent_t a, b;
            CHECK(hipEventCreate(&a));
            CHECK(hipEventCreate(&b));
            std::vector<float> v;
            for (int r = 0; r < 7; ++r) {
                hipLaunchKernelGGL(k.f, dim3(256), dim3(k.threads), 160 * 1024, 0, d, 1u);
                CHECK(hipEventRecord(a));
                hipLaunchKernelGGL(k.f, dim3(256), dim3(k.threads), 160 * 1024, 0, d, 2u + r);
                CHECK(hipEventRecord(b));
                CHECK(hipEventSynchronize(b));
                float ms;
                CHECK(hipEventElapsedTime(&ms, a, b));
                v.push_back(ms * 1000.f);
            }
            std::sort(v.begin(), v.end());
            printf("%s{\"rep\": %d, \"variant\": \"%s\", \"us\": %.2f}\n", first ? "" : ",", rep, k.name, v[3]);
            first = false;
        }
    printf("]\n");
    return 0;
}
