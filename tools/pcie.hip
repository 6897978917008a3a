// pcie.hip -- round 4: the host <-> GPU link ceiling the end-to-end path
// (rg_{seal,open}_batch_host) is measured against.  Pinned host buffers (hipHostMalloc), 256 MiB:
//   copy engines:  H2D alone, D2H alone, and both at once on two hipStreamNonBlocking streams,
//                  whole buffers and in 16 MiB pieces alternating streams (the library's slice size);
//   zero copy:     a kernel reading pinned host memory into HBM, one writing HBM to pinned host memory,
//                  and one doing both at once (the link carries both directions from the CUs);
// each timed with HIP events over 5 repetitions (median), GB/s = 1e9 bytes per second per direction.
// Build: hipcc --offload-arch=gfx950 -O3 tools/pcie.hip -o tools/build/pcie
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CHECK(x)                                                                       \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                   \
        }                                                                              \
    } while (0)

// grid-stride 16-byte copies; `src`/`dst` may be pinned host memory (device-visible pointers)
__global__ void copy16(const uint4 *__restrict__ src, uint4 *__restrict__ dst, size_t n16) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x)
        dst[i] = src[i];
}
// both directions from one launch: even blocks pull host -> HBM, odd blocks push HBM -> host
__global__ void duplex16(const uint4 *__restrict__ hsrc, uint4 *__restrict__ dbuf, const uint4 *__restrict__ dsrc,
                         uint4 *__restrict__ hdst, size_t n16) {
    const bool up = (blockIdx.x & 1u) == 0;
    const size_t b = blockIdx.x >> 1, nb = gridDim.x >> 1;
    for (size_t i = b * blockDim.x + threadIdx.x; i < n16; i += nb * blockDim.x) {
        if (up) dbuf[i] = hsrc[i];
        else hdst[i] = dsrc[i];
    }
}

template <class F> static float timed(hipStream_t s0, F &&f) {
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    std::vector<float> ms;
    for (int r = 0; r < 6; ++r) {
        CHECK(hipDeviceSynchronize());
        CHECK(hipEventRecord(a, s0));
        f();
        CHECK(hipEventRecord(b, s0));
        CHECK(hipEventSynchronize(b));
        float t;
        CHECK(hipEventElapsedTime(&t, a, b));
        if (r) ms.push_back(t); // the first repetition warms up
    }
    std::sort(ms.begin(), ms.end());
    CHECK(hipEventDestroy(a));
    CHECK(hipEventDestroy(b));
    return ms[ms.size() / 2];
}

int main(int argc, char **argv) {
    const size_t bytes = (argc > 1 ? strtoull(argv[1], nullptr, 0) : 256ull) << 20;
    const size_t piece = 16ull << 20;
    void *h_src, *h_dst, *d_a, *d_b;
    CHECK(hipHostMalloc(&h_src, bytes, hipHostMallocDefault));
    CHECK(hipHostMalloc(&h_dst, bytes, hipHostMallocDefault));
    memset(h_src, 1, bytes);
    memset(h_dst, 2, bytes);
    CHECK(hipMalloc(&d_a, bytes));
    CHECK(hipMalloc(&d_b, bytes));
    CHECK(hipMemset(d_a, 3, bytes));
    CHECK(hipMemset(d_b, 4, bytes));
    hipStream_t s1, s2;
    CHECK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    CHECK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    hipEvent_t j1, j2, fork;
    CHECK(hipEventCreateWithFlags(&j1, hipEventDisableTiming));
    CHECK(hipEventCreateWithFlags(&j2, hipEventDisableTiming));
    CHECK(hipEventCreateWithFlags(&fork, hipEventDisableTiming));
    // the events are recorded on s1; work on s2 is forked from and joined back into s1
    auto fork_s2 = [&] {
        CHECK(hipEventRecord(fork, s1));
        CHECK(hipStreamWaitEvent(s2, fork, 0));
    };
    auto join_s2 = [&] {
        CHECK(hipEventRecord(j2, s2));
        CHECK(hipStreamWaitEvent(s1, j2, 0));
    };
    const double gb = (double)bytes / 1e9;
    auto rate = [&](float ms) { return gb / (ms / 1e3); };

    const float t_h2d = timed(s1, [&] { CHECK(hipMemcpyAsync(d_a, h_src, bytes, hipMemcpyHostToDevice, s1)); });
    const float t_d2h = timed(s1, [&] { CHECK(hipMemcpyAsync(h_dst, d_b, bytes, hipMemcpyDeviceToHost, s1)); });
    const float t_both = timed(s1, [&] {
        fork_s2();
        CHECK(hipMemcpyAsync(d_a, h_src, bytes, hipMemcpyHostToDevice, s1));
        CHECK(hipMemcpyAsync(h_dst, d_b, bytes, hipMemcpyDeviceToHost, s2));
        join_s2();
    });
    // 16 MiB pieces, H2D on s1 and D2H on s2, interleaved in issue order
    const float t_both_pieces = timed(s1, [&] {
        fork_s2();
        for (size_t o = 0; o < bytes; o += piece) {
            const size_t m = std::min(piece, bytes - o);
            CHECK(hipMemcpyAsync((char *)d_a + o, (char *)h_src + o, m, hipMemcpyHostToDevice, s1));
            CHECK(hipMemcpyAsync((char *)h_dst + o, (char *)d_b + o, m, hipMemcpyDeviceToHost, s2));
        }
        join_s2();
    });
    // zero copy: the CUs read / write pinned host memory over the link
    int cus = 0;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const size_t n16 = bytes / 16;
    const dim3 grid(cus * 8), blk(256);
    const float t_zc_up = timed(s1, [&] {
        hipLaunchKernelGGL(copy16, grid, blk, 0, s1, (const uint4 *)h_src, (uint4 *)d_a, n16);
    });
    const float t_zc_down = timed(s1, [&] {
        hipLaunchKernelGGL(copy16, grid, blk, 0, s1, (const uint4 *)d_b, (uint4 *)h_dst, n16);
    });
    const float t_zc_both = timed(s1, [&] {
        hipLaunchKernelGGL(duplex16, dim3(cus * 16), blk, 0, s1, (const uint4 *)h_src, (uint4 *)d_a,
                           (const uint4 *)d_b, (uint4 *)h_dst, n16);
    });
    // mixed: the H2D copy engine beside a zero-copy kernel writing to host
    const float t_mix = timed(s1, [&] {
        fork_s2();
        CHECK(hipMemcpyAsync(d_a, h_src, bytes, hipMemcpyHostToDevice, s1));
        hipLaunchKernelGGL(copy16, grid, blk, 0, s2, (const uint4 *)d_b, (uint4 *)h_dst, n16);
        join_s2();
    });
    CHECK(hipGetLastError());
    CHECK(hipDeviceSynchronize());
    // check: the zero-copy write reached the host buffer
    unsigned char *hd = (unsigned char *)h_dst;
    const bool ok = hd[0] == 4 && hd[bytes - 1] == 4;
    printf("{\"bytes\": %zu, \"piece_bytes\": %zu, \"gb_s_per_direction\": {"
           "\"h2d_copy\": %.2f, \"d2h_copy\": %.2f, \"both_copies\": %.2f, \"both_copies_16MiB_pieces\": %.2f, "
           "\"zero_copy_read_host\": %.2f, \"zero_copy_write_host\": %.2f, \"zero_copy_both\": %.2f, "
           "\"h2d_copy_beside_zero_copy_write\": %.2f}, \"ms\": {\"h2d\": %.3f, \"d2h\": %.3f, \"both\": %.3f, "
           "\"both_pieces\": %.3f, \"zc_up\": %.3f, \"zc_down\": %.3f, \"zc_both\": %.3f, \"mix\": %.3f}, "
           "\"zero_copy_write_checked\": %s}\n",
           bytes, piece, rate(t_h2d), rate(t_d2h), rate(t_both), rate(t_both_pieces), rate(t_zc_up), rate(t_zc_down),
           rate(t_zc_both), rate(t_mix), t_h2d, t_d2h, t_both, t_both_pieces, t_zc_up, t_zc_down, t_zc_both, t_mix,
           ok ? "true" : "false");
    return 0;
}
