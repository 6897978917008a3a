// Round 4: why the host path's slices run below the link's duplex rate.  rg_{seal,open}_batch_host moves
// 8 MiB slices H2D on one stream, runs a kernel per slice on a second and moves the slice back D2H on a
// third, chained by events, with three device buffers in rotation.  A copy trace of it shows each slice's
// kernel and the next slice's upload starting only when the previous slice's download ends.  This program
// times the same chain with its parts swapped out, pinned host buffers, 12 slices of 8 MiB:
//   pieces     H2D on s1 and D2H on s2 interleaved, no events (the link's duplex rate in pieces)
//   chain      H2D(k) -> event -> D2H(k), three buffers in rotation (no kernel)
//   kernel     the chain with a 30 us kernel on a third stream between the copies (the library's shape)
//   kernel_zc  the same, with D2H done by a 64-workgroup copy kernel writing host memory instead of a
//              hipMemcpyAsync (whose blit kernel has thousands of workgroups)
//   kernel_d   the same as kernel, every slice's kernel launched on the D2H stream right before its copy
// Output: one JSON line of GB/s per direction, median of 5.
//   build: hipcc --offload-arch=gfx950 -O2 tools/pipe_probe.hip -o tools/build/pipe_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                                            \
    do {                                                                                                    \
        hipError_t e_ = (x);                                                                                \
        if (e_ != hipSuccess) {                                                                             \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));               \
            exit(1);                                                                                        \
        }                                                                                                   \
    } while (0)

// a stand-in for the AEAD kernel: every workgroup touches its share of the slice and spins for `ns`
__global__ void spin(uint4 *buf, size_t n16, uint64_t ns) {
    const uint64_t t0 = wall_clock64(); // 100 MHz
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x) {
        uint4 v = buf[i];
        v.x ^= 1u;
        buf[i] = v;
    }
    while ((wall_clock64() - t0) * 10 < ns) __builtin_amdgcn_s_sleep(2);
}

__global__ void copy16(const uint4 *__restrict__ src, uint4 *__restrict__ dst, size_t n16) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x)
        dst[i] = src[i];
}

int main(int argc, char **argv) {
    const size_t piece = (argc > 1 ? strtoull(argv[1], nullptr, 0) : 8ull) << 20;
    const int pieces = 12, slots = 3;
    const size_t bytes = piece * pieces, n16 = piece / 16;
    void *h_src, *h_dst;
    CHECK(hipHostMalloc(&h_src, bytes, hipHostMallocDefault));
    CHECK(hipHostMalloc(&h_dst, bytes, hipHostMallocDefault));
    std::vector<void *> d(slots);
    for (auto &p : d) CHECK(hipMalloc(&p, piece));
    hipStream_t s1, s2, s3;
    CHECK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    CHECK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    CHECK(hipStreamCreateWithFlags(&s3, hipStreamNonBlocking));
    std::vector<hipEvent_t> e_in(slots), e_run(slots), e_out(slots);
    for (int k = 0; k < slots; ++k) {
        CHECK(hipEventCreateWithFlags(&e_in[k], hipEventDisableTiming));
        CHECK(hipEventCreateWithFlags(&e_run[k], hipEventDisableTiming));
        CHECK(hipEventCreateWithFlags(&e_out[k], hipEventDisableTiming));
    }
    int cus = 0;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    auto hs = [&](int k) { return (char *)h_src + (size_t)k * piece; };
    auto hd = [&](int k) { return (char *)h_dst + (size_t)k * piece; };

    // mode: 0 pieces, 1 chain, 2 kernel, 3 kernel_zc, 4 kernel_d
    auto run = [&](int mode) {
        std::vector<bool> used(slots, false);
        for (int k = 0; k < pieces; ++k) {
            const int s = k % slots;
            if (mode == 0) {
                CHECK(hipMemcpyAsync(d[s], hs(k), piece, hipMemcpyHostToDevice, s1));
                CHECK(hipMemcpyAsync(hd(k), d[(s + 1) % slots], piece, hipMemcpyDeviceToHost, s2));
                continue;
            }
            if (used[s]) CHECK(hipStreamWaitEvent(s1, e_out[s], 0));
            CHECK(hipMemcpyAsync(d[s], hs(k), piece, hipMemcpyHostToDevice, s1));
            CHECK(hipEventRecord(e_in[s], s1));
            hipEvent_t before_out = e_in[s];
            if (mode == 2 || mode == 3) {
                CHECK(hipStreamWaitEvent(s3, e_in[s], 0));
                hipLaunchKernelGGL(spin, dim3(cus), dim3(256), 0, s3, (uint4 *)d[s], n16, (uint64_t)30000);
                CHECK(hipEventRecord(e_run[s], s3));
                before_out = e_run[s];
            }
            CHECK(hipStreamWaitEvent(s2, before_out, 0));
            if (mode == 4) hipLaunchKernelGGL(spin, dim3(cus), dim3(256), 0, s2, (uint4 *)d[s], n16, (uint64_t)30000);
            if (mode == 3)
                hipLaunchKernelGGL(copy16, dim3(64), dim3(256), 0, s2, (const uint4 *)d[s], (uint4 *)hd(k), n16);
            else
                CHECK(hipMemcpyAsync(hd(k), d[s], piece, hipMemcpyDeviceToHost, s2));
            CHECK(hipEventRecord(e_out[s], s2));
            used[s] = true;
        }
    };
    auto timed = [&](int mode) {
        std::vector<double> ms;
        for (int r = 0; r < 6; ++r) {
            CHECK(hipDeviceSynchronize());
            hipEvent_t a, b;
            CHECK(hipEventCreate(&a));
            CHECK(hipEventCreate(&b));
            // fork s2 and s3 from s1, join them back, time on s1
            CHECK(hipEventRecord(a, s1));
            CHECK(hipStreamWaitEvent(s2, a, 0));
            CHECK(hipStreamWaitEvent(s3, a, 0));
            run(mode);
            hipEvent_t j2, j3;
            CHECK(hipEventCreateWithFlags(&j2, hipEventDisableTiming));
            CHECK(hipEventCreateWithFlags(&j3, hipEventDisableTiming));
            CHECK(hipEventRecord(j2, s2));
            CHECK(hipEventRecord(j3, s3));
            CHECK(hipStreamWaitEvent(s1, j2, 0));
            CHECK(hipStreamWaitEvent(s1, j3, 0));
            CHECK(hipEventRecord(b, s1));
            CHECK(hipEventSynchronize(b));
            float t;
            CHECK(hipEventElapsedTime(&t, a, b));
            if (r) ms.push_back(t);
            for (hipEvent_t e : {a, b, j2, j3}) CHECK(hipEventDestroy(e));
        }
        std::sort(ms.begin(), ms.end());
        return (double)bytes / 1e9 / (ms[ms.size() / 2] / 1e3);
    };
    const char *names[] = {"pieces", "chain", "kernel", "kernel_zc", "kernel_d"};
    printf("{\"piece_bytes\": %zu, \"pieces\": %d, \"gb_s_per_direction\": {", piece, pieces);
    for (int m = 0; m < 5; ++m) printf("%s\"%s\": %.2f", m ? ", " : "", names[m], timed(m));
    printf("}}\n");
    CHECK(hipGetLastError());
    return 0;
}
