// hbmcal.hip -- calibrates rocprofv3's FETCH_SIZE / WRITE_SIZE against known byte
// counts on gfx950, over a 1 GiB working set (4x the 256 MiB Infinity Cache, so
// every byte really comes from / goes to HBM).  One kernel per run (argv[1]) so
// that each counter pass sees exactly one dispatch of known traffic:
//   rd_coal   : 16 B per lane, consecutive lanes on consecutive 16 B (streaming read)
//   rd_frame  : lane = 1536-B frame, 16 B per lane per instruction (the transport
//               kernels' lane-per-packet pattern), whole frames
//   wr_coal   : streaming 16-B stores
//   wr_frame  : lane-per-frame 16-B stores, whole frames
//   wr_split  : lane-per-frame, the frame's bytes [0,16) and [16,1536) written by two
//               kernels (the header / payload split of a seal), both counted
//   ph_{wr,rd}_{0,16} [spin] : round 3 -- the flattened kernel's pattern: one wave per SIMD, each lane
//               owns 1536 contiguous bytes at phase 0 or 16 from the 64-B grid and moves 64 B per step
//               (four 16-B accesses), with `spin` x 1000 VALU instructions between steps; does a
//               16-B phase cost HBM bytes when the halves of a 64-B segment arrive one step apart?
// Prints {"kernel", "bytes_read", "bytes_written", "us"}; bytes are what the kernel
// touches, so counter / bytes is the calibration factor.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CHECK(x)                                                                      \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                  \
        }                                                                             \
    } while (0)

constexpr size_t kBytes = 1ull << 30;
constexpr uint32_t kStride = 1536, kQ = kStride / 16;
constexpr uint32_t kFrames = (uint32_t)(kBytes / kStride);

__global__ __launch_bounds__(256) void rd_coal(const uint4 *p, size_t nq, uint4 *sink) {
    uint4 acc = make_uint4(0, 0, 0, 0);
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < nq; i += (size_t)gridDim.x * 256) {
        const uint4 v = p[i];
        acc.x ^= v.x; acc.y ^= v.y; acc.z ^= v.z; acc.w ^= v.w;
    }
    if ((acc.x & acc.y & acc.z & acc.w) == 0xFFFFFFFFu) sink[0] = acc; // keeps the loads, never stores
}

__global__ __launch_bounds__(256) void rd_frame(const uint4 *p, uint4 *sink) {
    const uint32_t f = blockIdx.x * 256 + threadIdx.x;
    if (f >= kFrames) return;
    const uint4 *q = p + (size_t)f * kQ;
    uint4 acc = make_uint4(0, 0, 0, 0);
#pragma unroll 8
    for (uint32_t i = 0; i < kQ; ++i) {
        const uint4 v = q[i];
        acc.x ^= v.x; acc.y ^= v.y; acc.z ^= v.z; acc.w ^= v.w;
    }
    if ((acc.x & acc.y & acc.z & acc.w) == 0xFFFFFFFFu) sink[0] = acc;
}

__global__ __launch_bounds__(256) void wr_coal(uint4 *p, size_t nq) {
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < nq; i += (size_t)gridDim.x * 256)
        p[i] = make_uint4((uint32_t)i, 1, 2, 3);
}

__global__ __launch_bounds__(256) void wr_frame(uint4 *p, uint32_t q0, uint32_t q1) {
    const uint32_t f = blockIdx.x * 256 + threadIdx.x;
    if (f >= kFrames) return;
    uint4 *q = p + (size_t)f * kQ;
#pragma unroll 8
    for (uint32_t i = q0; i < q1; ++i) q[i] = make_uint4(f, i, 2, 3);
}

constexpr uint32_t kPhSteps = 24, kPhLanes = 65536; // 100.7 MB per launch, 1024 waves
template <uint32_t PH, bool WR> __global__ __launch_bounds__(256) void k_phase(uint4 *p, uint4 *sink, int spin) {
    const uint32_t gl = blockIdx.x * 256 + threadIdx.x;
    uint4 *q = reinterpret_cast<uint4 *>(reinterpret_cast<uint8_t *>(p) + PH + (size_t)gl * 64 * kPhSteps);
    uint32_t a = gl, b = gl ^ 7, c = gl * 3, d = 11;
    uint4 acc = make_uint4(0, 0, 0, 0);
    for (uint32_t t = 0; t < kPhSteps; ++t) {
        for (int k = 0; k < 250 * spin; ++k)
            asm volatile("v_add_u32 %0, %0, %1\n\tv_xor_b32 %1, %1, %2\n\tv_alignbit_b32 %2, %2, %2, 7\n\tv_add_u32 %3, %3, %0"
                         : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
        if (WR) {
            q[4 * t + 0] = make_uint4(a, t, 0, 1);
            q[4 * t + 1] = make_uint4(b, t, 1, 2);
            q[4 * t + 2] = make_uint4(c, t, 2, 3);
            q[4 * t + 3] = make_uint4(d, t, 3, 4);
        } else {
            for (int i = 0; i < 4; ++i) {
                const uint4 v = q[4 * t + i];
                acc.x ^= v.x; acc.y ^= v.y ^ a; acc.z ^= v.z; acc.w ^= v.w;
            }
        }
    }
    if ((acc.x & acc.y & acc.z & acc.w) == 0xFFFFFFFFu || (a ^ b ^ c ^ d) == 0x12345678u) sink[0] = acc;
}

int main(int argc, char **argv) {
    const char *k = argc > 1 ? argv[1] : "rd_coal";
    uint4 *buf, *sink;
    CHECK(hipMalloc(&buf, kBytes));
    CHECK(hipMalloc(&sink, 64));
    CHECK(hipMemset(buf, 0x5a, kBytes));
    CHECK(hipDeviceSynchronize());
    const size_t nq = kBytes / 16;
    const uint32_t fblocks = (kFrames + 255) / 256;
    size_t rd = 0, wr = 0;
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    CHECK(hipEventRecord(e0, 0));
    if (!strcmp(k, "rd_coal")) {
        hipLaunchKernelGGL(rd_coal, dim3(4096), dim3(256), 0, 0, buf, nq, sink);
        rd = kBytes;
    } else if (!strcmp(k, "rd_frame")) {
        hipLaunchKernelGGL(rd_frame, dim3(fblocks), dim3(256), 0, 0, buf, sink);
        rd = (size_t)kFrames * kStride;
    } else if (!strcmp(k, "wr_coal")) {
        hipLaunchKernelGGL(wr_coal, dim3(4096), dim3(256), 0, 0, buf, nq);
        wr = kBytes;
    } else if (!strcmp(k, "wr_frame")) {
        hipLaunchKernelGGL(wr_frame, dim3(fblocks), dim3(256), 0, 0, buf, 0u, kQ);
        wr = (size_t)kFrames * kStride;
    } else if (!strcmp(k, "wr_split")) {
        hipLaunchKernelGGL(wr_frame, dim3(fblocks), dim3(256), 0, 0, buf, 0u, 1u);
        hipLaunchKernelGGL(wr_frame, dim3(fblocks), dim3(256), 0, 0, buf, 1u, kQ);
        wr = (size_t)kFrames * kStride;
    } else if (!strncmp(k, "ph_", 3)) {
        const int spin = argc > 2 ? atoi(argv[2]) : 1;
        const bool w = !strncmp(k, "ph_wr", 5), p16 = strstr(k, "_16") != nullptr;
        void (*f)(uint4 *, uint4 *, int) = w ? (p16 ? k_phase<16, true> : k_phase<0, true>)
                                             : (p16 ? k_phase<16, false> : k_phase<0, false>);
        const int lds = 160 * 1024; // one 4-wave workgroup per CU: one wave per SIMD
        CHECK(hipFuncSetAttribute((const void *)f, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
        CHECK(hipEventRecord(e0, 0)); // (re-recorded: the attribute call is not timed)
        hipLaunchKernelGGL(f, dim3(kPhLanes / 256), dim3(256), lds, 0, buf, sink, spin);
        (w ? wr : rd) = (size_t)kPhLanes * 64 * kPhSteps;
    } else {
        fprintf(stderr, "unknown kernel %s\n", k);
        return 2;
    }
    CHECK(hipGetLastError());
    CHECK(hipEventRecord(e1, 0));
    CHECK(hipEventSynchronize(e1));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    printf("{\"kernel\": \"%s\", \"bytes_read\": %zu, \"bytes_written\": %zu, \"us\": %.1f}\n", k, rd, wr, ms * 1e3);
    CHECK(hipFree(buf));
    CHECK(hipFree(sink));
    return 0;
}
