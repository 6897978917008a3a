// rg_api.cpp -- the C ABI of include/rg_aead.h: device context, batched
// device/host entry points, the per-message CryptoPrimatives drop-in, and the
// host-side transport session layer (EncryptionKey / DecryptionKey /
// AntiReplay, rustyguard-crypto/src/prim.rs:376-437,
// rustyguard-utils/src/anti_replay.rs:1-64, rustyguard-core/src/lib.rs:249-681).
#include <hip/hip_runtime.h>
#include <sched.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cerrno>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <mutex>
#include <new>
#include <string>
#include <system_error>
#include <thread>
#include <unordered_map>
#include <vector>

#include "rg_internal.h"
#if RG_TEST_HOOKS
#include "../../include/rg_aead_test.h"
#endif

namespace {

thread_local std::string g_err;

int set_err(int code, const char *what, hipError_t e = hipSuccess) {
    char buf[256];
    if (e != hipSuccess)
        snprintf(buf, sizeof buf, "%s: %s", what, hipGetErrorString(e));
    else
        snprintf(buf, sizeof buf, "%s", what);
    g_err = buf;
    return code;
}

#define RG_HIP(call, what)                                                   \
    do {                                                                     \
        hipError_t e_ = (call);                                              \
        if (e_ != hipSuccess) return set_err(RG_EDEVICE, what, e_);          \
    } while (0)

#if RG_TEST_HOOKS
// test hook (rg_debug_fail_reserve, test library only): the n-th following allocation of a DevBuf /
// HostBuf fails
std::atomic<int> g_fail_reserve{0};
bool injected_failure() {
    int v = g_fail_reserve.load();
    while (v > 0)
        if (g_fail_reserve.compare_exchange_weak(v, v - 1)) return v == 1;
    return false;
}
// rg_debug_plan_handoff: the finished-workgroup count the preset pass starts the planner with (0: none)
std::atomic<uint32_t> g_stale_done{0};
std::atomic<uint32_t> g_stale_pool{0};
// rg_debug_lose_completions: every library wait sees its event as never completing
std::atomic<int> g_lose_completions{0};
#else
constexpr bool injected_failure() { return false; }
#endif

// Bounded host waits (include/rg_aead.h, rg_set_wait_timeout).  Round 5 waited with hipEventSynchronize,
// so a completion the runtime never reported -- agent-scope signals under ROC_SYSTEM_SCOPE_SIGNAL=0 hung
// the host pipeline at 16 MiB slices (profiles/r5_e2e_rtenv.txt) -- became a silent hang.  The wait polls
// query() (hipSuccess: done; hipErrorNotReady: not yet; anything else: a device error), yielding the CPU
// for the first 2 ms and sleeping 50 us between polls after that, and gives up after timeout_ms.
template <class Query> hipError_t wait_bounded(Query &&query, uint32_t timeout_ms, bool *timed_out) {
    using clk = std::chrono::steady_clock;
    const auto t0 = clk::now();
    *timed_out = false;
    for (;;) {
        const hipError_t q = query();
        if (q != hipErrorNotReady) return q;
        const auto el = clk::now() - t0;
        if (el >= std::chrono::milliseconds(timeout_ms)) {
            *timed_out = true;
            return hipErrorNotReady;
        }
        if (el < std::chrono::milliseconds(2)) std::this_thread::yield();
        else std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
}

constexpr uint32_t kDefaultWaitMs = 10000;

int wait_event(hipEvent_t e, uint32_t timeout_ms, const char *what) {
    if (!e) return RG_OK;
    bool late = false;
    const hipError_t r = wait_bounded(
        [e]() {
#if RG_TEST_HOOKS
            if (g_lose_completions.load()) return hipErrorNotReady;
#endif
            return hipEventQuery(e);
        },
        timeout_ms, &late);
    if (late) {
        char buf[160];
        snprintf(buf, sizeof buf, "%s: timed out after %u ms (the device never reported the completion)", what,
                 timeout_ms);
        return set_err(RG_EDEVICE, buf);
    }
    if (r != hipSuccess) return set_err(RG_EDEVICE, what, r);
    return RG_OK;
}

#define RG_WAIT(ev, ms, what)                                                \
    do {                                                                     \
        const int rc_ = wait_event((ev), (ms), (what));                      \
        if (rc_) return rc_;                                                 \
    } while (0)

// grow-only device allocation, freed by its owner's destructor at the latest (RAII: a context whose
// creation fails part way releases what it had allocated)
struct DevBuf {
    void *p = nullptr;
    size_t cap = 0;
    DevBuf() = default;
    DevBuf(const DevBuf &) = delete;
    DevBuf &operator=(const DevBuf &) = delete;
    ~DevBuf() { drop(); }
    void drop() {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
    hipError_t reserve(size_t bytes) {
        if (bytes <= cap) return hipSuccess;
        drop();
        if (injected_failure()) return hipErrorOutOfMemory;
        size_t want = std::max<size_t>(bytes, 4096);
        hipError_t e = hipMalloc(&p, want);
        if (e == hipSuccess) cap = want;
        return e;
    }
    void release() { drop(); }
};

bool capturing(hipStream_t s) {
    hipStreamCaptureStatus c = hipStreamCaptureStatusNone;
    return hipStreamIsCapturing(s, &c) == hipSuccess && c != hipStreamCaptureStatusNone;
}

// Device memory that holds key material: zeroed before it goes back to the allocator (the reference
// zeroizes keys on drop, prim.rs:227-231), in stream order.  Each launch that reads the buffer is
// followed by use(stream), an event recorded on that stream; reserve(bytes, s) and release(s) make s
// wait for those events, zero the old block, free it with hipFreeAsync and (reserve) take the new one
// with hipMallocAsync, all on s.  Nothing waits for the whole device -- no hipDeviceSynchronize, no
// synchronous hipFree -- so other streams (the caller's torch work) keep running and the host does not
// block (round 4 waited for the device: ADVICE r4).  A regrow inside a stream capture is refused.  A
// launch captured into a graph records no event -- the graph replays whenever its owner launches it -- so
// use() marks the block captured instead, and a block once captured is never freed under the graph: a
// later regrow retires it (it stays allocated, keys and all, until release() at rg_destroy /
// rg_sessions_destroy wipes and frees it), as ADVICE r5 asked (round 5 wiped and freed it on the next
// regrow, and a replay read freed memory).
#if RG_TEST_HOOKS
// test hook: the first bytes of the most recently wiped block, read back after its wipe (rg_debug_last_wipe)
std::mutex g_wipe_mu;
uint8_t *g_wipe_probe = nullptr; // pinned, 4 KiB, never freed (test library only)
size_t g_wipe_bytes = 0;
uint64_t g_wipes = 0;
#endif
struct SecretBuf {
    void *p = nullptr;
    size_t cap = 0;
    bool captured = false; // a captured launch reads p
    std::vector<std::pair<void *, size_t>> retired;
    std::vector<std::pair<hipStream_t, hipEvent_t>> users;
    SecretBuf() = default;
    SecretBuf(const SecretBuf &) = delete;
    SecretBuf &operator=(const SecretBuf &) = delete;
    // owners release on one of their streams first; this is the last resort (legacy stream, host wait)
    ~SecretBuf() {
        if (p || !retired.empty()) {
            (void)release(nullptr);
            (void)hipStreamSynchronize(nullptr);
        }
        forget_users();
    }
    void forget_users() {
        for (auto &u : users) (void)hipEventDestroy(u.second);
        users.clear();
    }
    // a launch on s reads the buffer (after it was enqueued)
    hipError_t use(hipStream_t s) {
        if (!p) return hipSuccess;
        if (capturing(s)) {
            captured = true;
            return hipSuccess;
        }
        for (auto &u : users)
            if (u.first == s) return hipEventRecord(u.second, s);
        // streams whose last recorded use has completed need no fence: dropped, so that a caller making a
        // new stream per call does not grow the list
        for (size_t k = 0; k < users.size();) {
            if (hipEventQuery(users[k].second) == hipSuccess) {
                (void)hipEventDestroy(users[k].second);
                users[k] = users.back();
                users.pop_back();
            } else {
                ++k;
            }
        }
        hipEvent_t e = nullptr;
        hipError_t r = hipEventCreateWithFlags(&e, hipEventDisableTiming);
        if (r != hipSuccess) return r;
        users.emplace_back(s, e);
        return hipEventRecord(e, s);
    }
    // zero one block behind every recorded use and free it, on s
    hipError_t wipe_free(void *blk, size_t n, hipStream_t s) {
        hipError_t r = hipSuccess;
        for (auto &u : users)
            if (r == hipSuccess) r = hipStreamWaitEvent(s, u.second, 0);
        if (r == hipSuccess) r = hipMemsetAsync(blk, 0, n, s);
        // a failed wait or wipe must not hand the keys back to the allocator: keep the block (freed by
        // a later release, or leaked rather than disclosed)
        if (r != hipSuccess) return r;
#if RG_TEST_HOOKS
        {
            std::lock_guard<std::mutex> g(g_wipe_mu);
            if (!g_wipe_probe) (void)hipHostMalloc(reinterpret_cast<void **>(&g_wipe_probe), 4096, hipHostMallocDefault);
            g_wipe_bytes = std::min<size_t>(n, 4096);
            if (g_wipe_probe) (void)hipMemcpyAsync(g_wipe_probe, blk, g_wipe_bytes, hipMemcpyDeviceToHost, s);
            (void)hipStreamSynchronize(s);
            ++g_wipes;
        }
#endif
        return hipFreeAsync(blk, s);
    }
    // zero and free the current block behind every recorded use, on s
    hipError_t release_current(hipStream_t s) {
        if (!p) return hipSuccess;
        hipError_t r = wipe_free(p, cap, s);
        if (r != hipSuccess) return r;
        p = nullptr;
        cap = 0;
        captured = false;
        if (retired.empty()) forget_users();
        return r;
    }
    // the owner's teardown: every retired block too (no graph may replay after it)
    hipError_t release(hipStream_t s) {
        hipError_t r = hipSuccess;
        while (r == hipSuccess && !retired.empty()) {
            r = wipe_free(retired.back().first, retired.back().second, s);
            if (r == hipSuccess) retired.pop_back();
        }
        if (r == hipSuccess) r = release_current(s);
        if (r == hipSuccess) forget_users();
        return r;
    }
    hipError_t reserve(size_t bytes, hipStream_t s) {
        if (bytes <= cap) return hipSuccess;
        if (capturing(s)) return hipErrorStreamCaptureUnsupported;
        if (captured) { // a graph reads this block: it stays until release()
            retired.emplace_back(p, cap);
            p = nullptr;
            cap = 0;
            captured = false;
        } else {
            hipError_t r = release_current(s);
            if (r != hipSuccess) return r;
        }
        if (injected_failure()) return hipErrorOutOfMemory;
        const size_t want = std::max<size_t>(bytes, 4096);
        hipError_t r = hipMallocAsync(&p, want, s);
        if (r == hipSuccess) cap = want;
        else p = nullptr;
        return r;
    }
};

// Pinned host memory.  A mapped buffer (reserve_mapped) is also read and written by kernels in place,
// through its device address d: coherent, so a kernel's stores are in host memory when it completes.
struct HostBuf {
    void *p = nullptr;
    void *d = nullptr; // device address of a mapped buffer
    size_t cap = 0;
    bool secret = false;
    HostBuf() = default;
    HostBuf(const HostBuf &) = delete;
    HostBuf &operator=(const HostBuf &) = delete;
    ~HostBuf() { drop(); }
    void drop() {
        if (p && secret) memset(p, 0, cap);
        if (p) (void)hipHostFree(p);
        p = d = nullptr;
        cap = 0;
    }
    hipError_t alloc(size_t bytes, unsigned flags) {
        if (bytes <= cap) return hipSuccess;
        drop();
        if (injected_failure()) return hipErrorOutOfMemory;
        size_t want = std::max<size_t>(bytes, 4096);
        hipError_t e = hipHostMalloc(&p, want, flags);
        if (e != hipSuccess) return e;
        cap = want;
        if (flags & hipHostMallocMapped) {
            e = hipHostGetDevicePointer(&d, p, 0);
            if (e != hipSuccess) drop();
        }
        return e;
    }
    hipError_t reserve(size_t bytes) { return alloc(bytes, hipHostMallocDefault); }
    hipError_t reserve_mapped(size_t bytes) { return alloc(bytes, hipHostMallocMapped | hipHostMallocCoherent); }
    void release() { drop(); }
};

// planner work lists (rg_tile.hip): class counts + [kClasses][cap] indices
struct PlanBuf {
    // the control block (rg_internal.h kCtl*): class counts and finished-workgroup count, the pipelined
    // kernel's schedule, the tile kernel's work pool.  Cleared by the preset pass before every launch that
    // uses it (round 5 relied on the consuming kernels to leave it zeroed, and a stale count once left a
    // whole batch unsealed: VERDICT r5 weak 3).  Allocated with the context: a launch may come inside a
    // stream capture, where allocation is not permitted.
    DevBuf ctl;
    DevBuf lists;
    hipError_t ensure_ctl() {
        if (ctl.p) return hipSuccess;
        hipError_t e = ctl.reserve(rg::kCtlWords * sizeof(uint32_t));
        if (e == hipSuccess) e = hipMemset(ctl.p, 0, rg::kCtlWords * sizeof(uint32_t));
        return e;
    }
    uint32_t *counts() const { return static_cast<uint32_t *>(ctl.p) + rg::kCtlCounts; }
    uint32_t *sched() const { return static_cast<uint32_t *>(ctl.p) + rg::kCtlSched; }
    uint32_t *pool() const { return static_cast<uint32_t *>(ctl.p) + rg::kCtlPool; }
    // statuses of the batch -> RG_PKT_PENDING, control block -> 0, on the launch stream
    hipError_t preset(uint8_t *status, uint32_t n, hipStream_t st) {
        uint32_t done0 = 0, pool0 = 0;
#if RG_TEST_HOOKS
        done0 = g_stale_done.load();
        pool0 = g_stale_pool.load();
#endif
        return rg::launch_preset(status, n, static_cast<uint32_t *>(ctl.p), done0, pool0, st);
    }
    uint32_t cap = 0;
    // auto planning: the tile kernel reports the number of size classes of the
    // last planned batch into host-mapped memory (read without synchronising;
    // a stale value only costs or saves one planner pass)
    volatile uint32_t *h_classes = nullptr;
    uint32_t *d_classes = nullptr;
    uint64_t calls = 0;
    PlanBuf() = default;
    PlanBuf(const PlanBuf &) = delete;
    PlanBuf &operator=(const PlanBuf &) = delete;
    ~PlanBuf() { release(); }
    hipError_t reserve(size_t n) {
        if (!h_classes) {
            void *hp = nullptr;
            hipError_t e = hipHostMalloc(&hp, 64, hipHostMallocMapped | hipHostMallocCoherent);
            if (e != hipSuccess) return e;
            h_classes = static_cast<volatile uint32_t *>(hp);
            *h_classes = ~0u; // unknown: plan
            void *dp = nullptr;
            e = hipHostGetDevicePointer(&dp, hp, 0);
            if (e != hipSuccess) return e;
            d_classes = static_cast<uint32_t *>(dp);
        }
        hipError_t e = hipSuccess;
        if (n <= cap) return e;
        e = lists.reserve((size_t)rg::kClasses * n * sizeof(uint32_t));
        if (e == hipSuccess) cap = (uint32_t)n;
        return e;
    }
    void release() {
        ctl.release();
        lists.release();
        cap = 0;
        if (h_classes) (void)hipHostFree(const_cast<uint32_t *>(h_classes));
        h_classes = nullptr;
        d_classes = nullptr;
    }
    // auto mode: plan unless the last planned batch held a single size class; re-check every 32nd call,
    // but never inside a stream capture (a captured graph replays the route it captured: a re-check
    // captured there would plan a uniform batch on every replay -- a bench warm-up count of 16 would
    // have put it in the timed graph)
    bool want_plan(hipStream_t st) {
        const bool check = (calls++ % 32) == 0 && !capturing(st);
        return check || !h_classes || *h_classes != 1u;
    }
};

// one slice buffer set of the host path: the slice's frames on the device, its descriptors, counters and
// statuses in mapped host memory (the kernel reads and writes them in place: round 4, one copy each way
// per slice instead of three and two), and the events that order it through the three pipeline streams
// (rg_ctx::hs_*)
struct Slot {
    PlanBuf plan;
    DevBuf d_buf;
    HostBuf h_desc, h_ctr, h_status, h_ctr_out;
    hipEvent_t ev_in = nullptr;  // the slice's inputs are on the device (recorded on hs_in)
    hipEvent_t ev_run = nullptr; // its kernel is done (recorded on hs_run)
    hipEvent_t ev_out = nullptr; // its outputs are back in host memory (recorded on hs_out)
    // bookkeeping of the slice in flight
    size_t i0 = 0, i1 = 0;
    uint64_t ticket = 0; // issue order of the slice among every context of the call (run_host)
    bool busy = false;
    // a slice left in flight by a call that failed (a timed-out wait): its results belong to no caller, and
    // the next use of the slot only waits for it (no copy into the next call's arrays)
    bool orphan = false;
};

} // namespace

struct rg_ctx {
    int device = 0;
    int lanes = 0;      // 0 = auto
    int wg_per_cu = 0;  // 0 = auto, -1 = plain one-shot grid (no LDS reservation)
    int cus = 0;
    int debug_mode = 0;
    int staged_g = -1; // -1 auto, 0 pipelined lane kernel, 1/2 LDS-staged tile windows of G chunks
    int plan = 2;     // size-class planner: 0 off (array order), 1 always, 2 auto (skip for single-class batches)
    int segments = 0; // segments per packet: 0 = automatic, else 1 / 2 / 4
    int last_kernel = -1; // kernel family of the latest batched launch (-1: none yet)
    size_t host_slice = 8ull << 20; // byte span of one host-pipeline slice (rg_set_host_slice; 8 MiB default)
    uint32_t wait_ms = kDefaultWaitMs; // limit of every host wait (rg_set_wait_timeout)
    int numa_node = -1; // host NUMA node closest to the GPU (hipDeviceAttributeHostNumaId; -1 unknown)
    PlanBuf plan_dev; // planner lists of the device API (calls on one ctx are stream-ordered)
    // the device API's last batch: its stream and an event behind it (not recorded for captured launches);
    // a call on another stream while that event is pending is refused (claim_stream)
    hipStream_t dev_stream = nullptr;
    hipEvent_t dev_ev = nullptr;
    bool dev_busy = false;
    uint64_t *dbg = nullptr; // diagnostics buffer (device), stamp builds only
    int pipe_max_wg[2] = {0, 0}; // [seal, open] resident workgroups per CU of the pipelined kernel
    std::mutex mu;
    // Host pipeline: up to kHostSlots slices in flight.  All uploads go through hs_in, all kernels through
    // hs_run and all downloads through hs_out, so that copies of one direction run one after another at
    // the link's full rate while the other direction's copy of a neighbouring slice runs beside them
    // (round 4: with one stream per slice the three slices' H2D copies ran at once and shared the
    // link, then their D2H copies -- half duplex, 27 GB/s per direction against a 48 GB/s duplex
    // ceiling; profiles/r4_e2e_probe.txt).  Three slots: a fourth (so that the upload of slice k + 1 need
    // not wait for the download of slice k - 2) measured the same at 16 MiB slices and slower at 8 MiB
    // (with the small per-slice copies that mapped host memory has since replaced).
    static constexpr int kHostSlots = 3;
    Slot slots[kHostSlots];
    hipStream_t hs_in = nullptr, hs_run = nullptr, hs_out = nullptr;
    hipEvent_t ev_in_idle = nullptr;  // behind everything on hs_in at the end of a host call (settle_host)
    hipStream_t gen_stream = nullptr; // the per-message drop-in
    hipEvent_t ev_gen = nullptr;      // its completion (bounded waits)
    SecretBuf d_keys;  // the host path's key table (rg_{seal,open}_batch_host*)
    DevBuf d_recv;
    SecretBuf d_general; // per-message drop-in arena: [job][aad][payload][tag]
    HostBuf h_general; // its pinned host image (one H2D and one D2H per call)
    DevBuf d_rx_desc;  // rg_open_batch_dev_rx: resolved descriptors
    SecretBuf d_mac_keys; // rg_mac_verify_batch_dev: per-key BLAKE2s states
    DevBuf d_junk; // flattened kernel: sink of the stores that are not payload (never read)
};

namespace {

// The caller's current HIP device, put back on the way out: every entry point selects its context's
// device (and a group call each of its contexts' in turn), while the caller -- a torch program, say --
// keeps its own device selected.
struct DeviceGuard {
    int dev = -1;
    DeviceGuard() { (void)hipGetDevice(&dev); }
    ~DeviceGuard() {
        if (dev >= 0) (void)hipSetDevice(dev);
    }
};

// The host NUMA node closest to a GPU, -1 if unknown.  HIP's attribute first; this runtime answers it with
// hipErrorInvalidValue (round 6 box), and a failed query stays the thread's last error, which the next
// launch's hipGetLastError (and PyTorch's checks) then report -- so it is cleared, and the node is read
// from the device's PCI function in sysfs instead.
int gpu_numa_node(int device) {
    int node = -1;
    if (hipDeviceGetAttribute(&node, hipDeviceAttributeHostNumaId, device) == hipSuccess && node >= 0) return node;
    (void)hipGetLastError();
    char bus[32] = {0};
    if (hipDeviceGetPCIBusId(bus, (int)sizeof bus, device) != hipSuccess) {
        (void)hipGetLastError();
        return -1;
    }
    for (char *p = bus; *p; ++p) *p = (char)((*p >= 'A' && *p <= 'F') ? *p - 'A' + 'a' : *p); // sysfs: lower case
    const std::string path = std::string("/sys/bus/pci/devices/") + bus + "/numa_node";
    FILE *f = std::fopen(path.c_str(), "r");
    if (!f) return -1;
    if (std::fscanf(f, "%d", &node) != 1) node = -1;
    std::fclose(f);
    return node >= 0 ? node : -1;
}

int check_ctx(rg_ctx *ctx) {
    if (!ctx) return set_err(RG_EINVAL, "null context");
    hipError_t e = hipSetDevice(ctx->device);
    if (e != hipSuccess) return set_err(RG_EDEVICE, "hipSetDevice", e);
    return RG_OK;
}

// One context, one stream (include/rg_aead.h): the device API's planner buffers and work pool are the
// context's, so a batch enqueued on a second stream while the first stream's batch is in flight would
// race it for them.  claim_stream refuses that call before anything is enqueued; an
// event query, no wait.  mark_stream records the event behind the call's launches.
int claim_stream(rg_ctx *ctx, hipStream_t st) {
    if (!ctx->dev_busy || ctx->dev_stream == st || capturing(st)) return RG_OK;
    const hipError_t q = hipEventQuery(ctx->dev_ev);
    if (q == hipSuccess) return RG_OK;
    if (q == hipErrorNotReady)
        return set_err(RG_EINVAL, "context busy: its last batch is still in flight on another stream (one context "
                                  "per concurrent stream; nothing enqueued)");
    return set_err(RG_EDEVICE, "context stream check", q);
}

// The event that marks a device batch's end: recorded by the transport kernel's own dispatch (RG_LAUNCH,
// no separate queue packet), or nullptr inside a stream capture (a graph is its owner's to order,
// include/rg_aead.h).  It is only queried, never used to read what the batch wrote: no system-scope fence
// (with one, the release wrote the L2s back after the kernel: +7 us on an eager config-2 seal; a separate
// fence-free hipEventRecord still cost +3 us, round 6).
hipEvent_t stream_event(rg_ctx *ctx, hipStream_t st) {
#if RG_NO_STREAM_MARK // diagnostic builds only (the A/B of the mark's cost)
    return nullptr;
#endif
    if (capturing(st)) return nullptr;
    if (!ctx->dev_ev &&
        hipEventCreateWithFlags(&ctx->dev_ev, hipEventDisableTiming | hipEventDisableSystemFence) != hipSuccess)
        ctx->dev_ev = nullptr;
    return ctx->dev_ev;
}

// after a launch that recorded ev (stream_event)
void mark_stream(rg_ctx *ctx, hipStream_t st, hipEvent_t ev) {
    if (!ev) return;
    ctx->dev_stream = st;
    ctx->dev_busy = true;
}

} // namespace

extern "C" {

int rg_abi_version(void) { return RG_ABI_VERSION; }

const char *rg_last_error(void) { return g_err.c_str(); }

int rg_create(int device, rg_ctx **out) {
    if (!out) return set_err(RG_EINVAL, "null out");
    *out = nullptr;
    // Agent-scope completion signals: the round-5 host pipeline hung under them at 16 MiB slices while 8 MiB
    // completed (profiles/r5_e2e_rtenv.txt).  The reading that fits both: a wait spins on the signal for a
    // short active-wait window, then sleeps until the signal's interrupt; a slice that finishes inside the
    // window (8 MiB) is seen by the spin, a longer one (16 MiB) leaves the host asleep on an interrupt that
    // an agent-scope signal never raises.  Waits are bounded now, but the setting would turn every slice
    // past the window into a timeout: refused.
    {
        const char *v = getenv("ROC_SYSTEM_SCOPE_SIGNAL");
        if (v && v[0] == '0' && v[1] == '\0')
            return set_err(RG_EINVAL, "ROC_SYSTEM_SCOPE_SIGNAL=0 (agent-scope signals) hangs host waits; unset it");
    }
    int ndev = 0;
    RG_HIP(hipGetDeviceCount(&ndev), "hipGetDeviceCount");
    if (device < 0 || device >= ndev) return set_err(RG_EINVAL, "no such HIP device");
    DeviceGuard dg_;
    RG_HIP(hipSetDevice(device), "hipSetDevice");
    rg_ctx *c = new (std::nothrow) rg_ctx();
    if (!c) return set_err(RG_ENOMEM, "alloc ctx");
    c->device = device;
    c->h_general.secret = true;
    {
        hipError_t e = hipDeviceGetAttribute(&c->cus, hipDeviceAttributeMultiprocessorCount, device);
        if (e == hipSuccess) c->numa_node = gpu_numa_node(device);
        if (e == hipSuccess) e = rg::prepare_tile_kernels();
        if (e == hipSuccess) e = rg::prepare_pipe_kernels(c->pipe_max_wg);
        if (e == hipSuccess) e = rg::prepare_flat_kernels();
        // the flattened kernel's store sink, allocated now: the automatic choice may first pick that
        // kernel inside a stream capture (HIP graph), where allocation is not permitted
        if (e == hipSuccess) e = c->d_junk.reserve(rg::flat_junk_bytes(c->cus));
        if (e == hipSuccess) e = c->plan_dev.ensure_ctl();
        for (auto &sl : c->slots)
            if (e == hipSuccess) e = sl.plan.ensure_ctl();
        if (e != hipSuccess) {
            rg_destroy(c); // every buffer allocated so far goes back (the owners' destructors)
            return set_err(RG_EDEVICE, "kernel setup", e);
        }
    }
    {
        hipError_t e = hipSuccess;
        for (hipStream_t *sp : {&c->hs_in, &c->hs_run, &c->hs_out, &c->gen_stream})
            if (e == hipSuccess) e = hipStreamCreateWithFlags(sp, hipStreamNonBlocking);
        for (auto &s : c->slots)
            for (hipEvent_t *ep : {&s.ev_in, &s.ev_run, &s.ev_out})
                if (e == hipSuccess) e = hipEventCreateWithFlags(ep, hipEventDisableTiming);
        if (e != hipSuccess) {
            rg_destroy(c);
            return set_err(RG_EDEVICE, "hipStreamCreate", e);
        }
    }
    // the pools zeroed above (null-stream memsets) are zero before any launch on any of the caller's streams
    {
        const hipError_t e = hipStreamSynchronize(nullptr);
        if (e != hipSuccess) {
            rg_destroy(c);
            return set_err(RG_EDEVICE, "context setup", e);
        }
    }
    *out = c;
    return RG_OK;
}

void rg_destroy(rg_ctx *ctx) {
    if (!ctx) return;
    DeviceGuard dg_;
    (void)hipSetDevice(ctx->device);
    for (hipStream_t sp : {ctx->hs_in, ctx->hs_run, ctx->hs_out, ctx->gen_stream})
        if (sp) (void)hipStreamSynchronize(sp);
    // key material: wiped behind its last readers, on the context's own stream
    {
        hipStream_t ws = ctx->gen_stream; // null while rg_create has not made it (the legacy stream then)
        (void)ctx->d_keys.release(ws);
        (void)ctx->d_general.release(ws);
        (void)ctx->d_mac_keys.release(ws);
        (void)hipStreamSynchronize(ws);
    }
    for (hipStream_t sp : {ctx->hs_in, ctx->hs_run, ctx->hs_out, ctx->gen_stream})
        if (sp) (void)hipStreamDestroy(sp);
    for (auto &s : ctx->slots) {
        for (hipEvent_t ep : {s.ev_in, s.ev_run, s.ev_out})
            if (ep) (void)hipEventDestroy(ep);
        s.plan.release();
        s.d_buf.release();
        s.h_desc.release(); s.h_ctr.release(); s.h_status.release(); s.h_ctr_out.release();
    }
    ctx->plan_dev.release();
    if (ctx->dev_ev) (void)hipEventDestroy(ctx->dev_ev);
    if (ctx->ev_in_idle) (void)hipEventDestroy(ctx->ev_in_idle);
    if (ctx->ev_gen) (void)hipEventDestroy(ctx->ev_gen);
    ctx->d_recv.release();
    ctx->d_rx_desc.release();
    ctx->h_general.release();
    ctx->d_junk.release();
    delete ctx;
}

int rg_set_lanes_per_packet(rg_ctx *ctx, int lanes) {
    if (!ctx) return set_err(RG_EINVAL, "null context");
    if (lanes != 0 && lanes != 1 && lanes != 2 && lanes != 4) return set_err(RG_EINVAL, "lanes must be 0,1,2,4");
    ctx->lanes = lanes;
    return RG_OK;
}

int rg_get_lanes_per_packet(rg_ctx *ctx, size_t n) {
    if (!ctx) return set_err(RG_EINVAL, "null context");
    if (ctx->lanes) return ctx->lanes;
    // fewest lanes per packet that still gives every SIMD one wave (n * K
    // lanes >= CUs * 256): a single wave of the pipelined kernel already keeps
    // a SIMD's VALU busy, so more segments only add combine work
    const size_t want = (size_t)(ctx->cus > 0 ? ctx->cus : 256) * 256;
    if (n >= want) return 1;
    if (2 * n >= want) return 2;
    return 4;
}

int rg_set_wg_per_cu(rg_ctx *ctx, int wg) {
    if (!ctx) return set_err(RG_EINVAL, "null context");
    if (wg < -1 || wg > 8) return set_err(RG_EINVAL, "wg_per_cu must be -1..8");
    ctx->wg_per_cu = wg;
    return RG_OK;
}

int rg_set_host_slice(rg_ctx *ctx, size_t bytes) {
    if (!ctx) return set_err(RG_EINVAL, "null context");
    if (bytes < (64u << 10) || bytes > (1ull << 30)) return set_err(RG_EINVAL, "host slice must be 64 KiB .. 1 GiB");
    ctx->host_slice = bytes;
    return RG_OK;
}

int rg_set_wait_timeout(rg_ctx *ctx, uint32_t ms) {
    if (!ctx) return set_err(RG_EINVAL, "null context");
    if (ms < 1 || ms > 3600000u) return set_err(RG_EINVAL, "wait timeout must be 1 .. 3600000 ms");
    ctx->wait_ms = ms;
    return RG_OK;
}

int rg_set_staged(rg_ctx *ctx, int g) {
    if (!ctx) return set_err(RG_EINVAL, "null context");
    if (g < -1 || g > 3)
        return set_err(RG_EINVAL, "kernel must be -1 (auto), 0 (pipelined lanes), 1/2 (tile windows) or 3 (flat)");
    ctx->staged_g = g;
    return RG_OK;
}

int rg_set_plan(rg_ctx *ctx, int on) {
    if (!ctx) return set_err(RG_EINVAL, "null context");
    if (on < 0 || on > 2) return set_err(RG_EINVAL, "plan must be 0 (off), 1 (on) or 2 (auto)");
    ctx->plan = on;
    return RG_OK;
}

int rg_set_segments(rg_ctx *ctx, int k) {
    if (!ctx) return set_err(RG_EINVAL, "null context");
    if (k != 0 && k != 1 && k != 2 && k != 4) return set_err(RG_EINVAL, "segments must be 0, 1, 2 or 4");
    ctx->segments = k;
    return RG_OK;
}

// Diagnostics exist only in diagnostic builds (-DRG_DIAG, tools/build_variant.sh): the product library
// accepts mode 0 and a null stamp buffer and refuses everything else, so no context of it can emit
// frames that are not sealed (the seal contract, prim.rs:179-188, always encrypts).
int rg_set_debug_buffer(rg_ctx *ctx, void *dev_ptr) {
    if (!ctx) return set_err(RG_EINVAL, "null context");
#if RG_DIAG
    ctx->dbg = static_cast<uint64_t *>(dev_ptr);
#else
    if (dev_ptr) return set_err(RG_EINVAL, "stamp buffers exist only in diagnostic builds (RG_DIAG)");
#endif
    return RG_OK;
}

int rg_set_debug_mode(rg_ctx *ctx, int mode) {
    if (!ctx) return set_err(RG_EINVAL, "null context");
#if RG_DIAG
    if (mode < 0 || mode > 8) return set_err(RG_EINVAL, "debug mode must be 0..8");
#else
    if (mode != 0) return set_err(RG_EINVAL, "debug modes exist only in diagnostic builds (RG_DIAG)");
#endif
    ctx->debug_mode = mode;
    return RG_OK;
}

// Kernel choice: batches that fill at most about one wave per SIMD go to the
// pipelined lane kernel (it saturates a SIMD with one wave and, with the
// planner, balances mixed sizes); larger batches go to the LDS-staged tile
// kernel, whose coalesced LDS-DMA windows win once two waves per SIMD are
// resident (measured).
int rg_get_kernel(rg_ctx *ctx, size_t n) {
    if (!ctx) return set_err(RG_EINVAL, "null context");
    if (ctx->staged_g >= 0) return ctx->staged_g;
    return n < (size_t)(ctx->cus > 0 ? ctx->cus : 256) * 512 ? 0 : 2;
}

int rg_last_kernel(rg_ctx *ctx) {
    if (!ctx) return set_err(RG_EINVAL, "null context");
    return ctx->last_kernel;
}

static rg::Launch launch_cfg(rg_ctx *ctx, size_t n, bool open) {
    rg::Launch L;
    L.done = nullptr;
    L.lanes = rg_get_lanes_per_packet(ctx, n);
    L.cus = ctx->cus;
    L.staged_g = rg_get_kernel(ctx, n);
    L.debug_mode = open ? (ctx->debug_mode == 3 ? 3 : 0) : ctx->debug_mode;
    const int cap = std::max(1, ctx->pipe_max_wg[open ? 1 : 0]);
    if (ctx->wg_per_cu < 0) {
        L.wg_per_cu = 0;
    } else if (ctx->wg_per_cu > 0) {
        L.wg_per_cu = std::min(ctx->wg_per_cu, cap);
    } else {
        // enough resident workgroups for one lane per packet segment, capped by occupancy
        const size_t need = ((size_t)n * L.lanes + 255) / 256;
        const size_t per_cu = (need + L.cus - 1) / std::max(1, L.cus);
        L.wg_per_cu = (int)std::max<size_t>(1, std::min<size_t>(per_cu, (size_t)cap));
    }
    return L;
}

// Tile kernels: persistent grid of 4-wave workgroups, two resident per CU
// (2 waves per SIMD: the VGPR budget of the kernel).  With the planner the
// work lists and the per-class segment counts are built on the device; without
// it packets stay in array order and the segment count follows from n.
static hipError_t launch_tiles_any(rg_ctx *ctx, const rg::SealArgs *sa, const rg::OpenArgs *oa, PlanBuf &pb,
                                   const rg::Launch &L0, hipStream_t st) {
    const uint32_t n = sa ? sa->n : oa->n;
    rg::Launch L = L0;
    rg::TilePlan tp{};
    tp.target_lanes = (uint32_t)std::max(1, ctx->cus) * 256u; // one wave per SIMD
    tp.fixed_k = (uint32_t)ctx->segments;
    tp.gq = pb.pool();
    bool plan = ctx->plan == 1;
    if (ctx->plan == 2) {
        hipError_t e = pb.reserve(n);
        if (e != hipSuccess) return e;
        plan = pb.want_plan(st);
    }
    // the tile kernel deals its last rounds from a grid-wide pool: statuses pending and the control block
    // cleared first, planned or not
    {
        hipError_t e = pb.preset(sa ? sa->status : oa->status, n, st);
        if (e != hipSuccess) return e;
    }
    if (plan) {
        hipError_t e = pb.reserve(n);
        if (e != hipSuccess) return e;
        tp.counts = pb.counts();
        tp.lists = static_cast<uint32_t *>(pb.lists.p);
        tp.cap = pb.cap;
        tp.classes_out = pb.d_classes;
        e = rg::launch_plan(sa ? sa->desc : oa->desc, n, oa != nullptr, tp, st);
        if (e != hipSuccess) return e;
    } else if (!tp.fixed_k) {
        tp.fixed_k = n >= tp.target_lanes ? 1u : 2ull * n >= tp.target_lanes ? 2u : 4u;
    }
    return rg::launch_tiles(sa, oa, L.staged_g, tp, L, st);
}

// Pipelined kernel: planned (size classes, per-class segments, tile queue) or
// in array order with lanes_per_packet segments.
static hipError_t launch_pipe_any(rg_ctx *ctx, const rg::SealArgs *sa, const rg::OpenArgs *oa, PlanBuf &pb,
                                  const rg::Launch &L, hipStream_t st) {
    const uint32_t n = sa ? sa->n : oa->n;
    bool plan = ctx->plan == 1;
    if (ctx->plan == 2) {
        hipError_t e = pb.reserve(n);
        if (e != hipSuccess) return e;
        plan = pb.want_plan(st);
    }
    // array order: lane unit u is packet u >> lg, by index alone -- no hand-off, no preset
    if (!plan) return rg::launch_pipe(sa, oa, L, nullptr, st);
    rg::Launch Lp = L;
    // two workgroups per CU are asked for, but the kernels' register budget (268 / 264 VGPR+AGPR, above
    // 256) admits one wave per SIMD, and the occupancy query (pipe_max_wg) caps the request at that:
    // the planned kernel runs one wave per SIMD.  Two co-resident waves, forced with
    // __launch_bounds__(256, 2), measured slower on config 2 (profiles/r4_cfg2_twowave.txt).
    const int want_wg = ctx->wg_per_cu > 0 ? ctx->wg_per_cu : 2;
    Lp.wg_per_cu = std::min(want_wg, std::max(1, ctx->pipe_max_wg[oa ? 1 : 0]));
    hipError_t e = pb.reserve(n);
    if (e != hipSuccess) return e;
    // the planner's last workgroup hands the schedule to the transport kernel: statuses pending and the
    // control block (counts, finished-workgroup count, schedule) cleared first -- a lost hand-off leaves an
    // empty schedule and every status pending
    e = pb.preset(sa ? sa->status : oa->status, n, st);
    if (e != hipSuccess) return e;
    rg::TilePlan tp{};
    tp.counts = pb.counts();
    tp.lists = static_cast<uint32_t *>(pb.lists.p);
    tp.cap = pb.cap;
    tp.sched = pb.sched();
    tp.simds = (uint32_t)std::max(1, ctx->cus) * 4u; // balance per SIMD: co-resident waves share its issue slots
    tp.classes_out = pb.d_classes;
    e = rg::launch_plan(sa ? sa->desc : oa->desc, n, oa != nullptr, tp, st);
    if (e != hipSuccess) return e;
    rg::PipePlan pp{pb.counts(), static_cast<const uint32_t *>(pb.lists.p), pb.cap, pb.sched(), pb.d_classes,
                    tp.simds};
    return rg::launch_pipe(sa, oa, Lp, &pp, st);
}

// Flattened chunk-stream kernel: units of equal work (planner on / auto) or of
// equal packet counts (planner off); the balancing runs inside the kernel.
static hipError_t launch_flat_any(rg_ctx *ctx, const rg::SealArgs *sa, const rg::OpenArgs *oa, hipStream_t st,
                                  hipEvent_t done) {
    hipError_t e = ctx->d_junk.reserve(rg::flat_junk_bytes(ctx->cus));
    if (e != hipSuccess) return e;
    return rg::launch_flat(sa, oa, ctx->plan != 0, static_cast<uint4 *>(ctx->d_junk.p), ctx->cus, st, done);
}

// Automatic choice between the two small-batch kernels: when the last planned batch of this planner
// held more than one size class (mixed sizes, e.g. IMIX), the flattened chunk stream runs -- it
// balances mixed sizes inside the kernel, without a planner pass; every 32nd call goes back to the
// planned pipelined kernel, whose planner refreshes the class count (a uniform batch returns there),
// except inside a stream capture: a captured graph replays one route, and it should be the fast one.
static int pick_family(rg_ctx *ctx, int g, PlanBuf &pb, hipStream_t st) {
    if (ctx->staged_g >= 0 || g != 0 || ctx->plan != 2 || !pb.h_classes) return g;
    const uint32_t cls = *pb.h_classes;
    if (cls < 2 || cls == ~0u) return g;
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(st, &cap) != hipSuccess) cap = hipStreamCaptureStatusNone;
    if ((pb.calls % 32) != 0 || cap != hipStreamCaptureStatusNone) {
        ++pb.calls;
        return 3;
    }
    return g;
}

// done: the event the transport kernel's dispatch records as it completes (nullptr: none)
static hipError_t launch_seal_any(rg_ctx *ctx, const rg::SealArgs &a0, PlanBuf &pb, hipStream_t st,
                                  hipEvent_t done = nullptr) {
    rg::SealArgs a = a0;
    rg::Launch L = launch_cfg(ctx, a.n, false);
    L.done = done;
    L.staged_g = pick_family(ctx, L.staged_g, pb, st);
    ctx->last_kernel = L.staged_g;
    // stamps (diagnostic builds): debug mode 3, or any diagnostic mode of the pipelined kernel
    a.dbg = L.debug_mode == 3 || (L.staged_g == 0 && L.debug_mode != 0) ? ctx->dbg : nullptr;
    if (L.staged_g == 3) return launch_flat_any(ctx, &a, nullptr, st, done);
    if (L.staged_g == 0) return launch_pipe_any(ctx, &a, nullptr, pb, L, st);
    return launch_tiles_any(ctx, &a, nullptr, pb, L, st);
}

static hipError_t launch_open_any(rg_ctx *ctx, const rg::OpenArgs &a0, PlanBuf &pb, hipStream_t st,
                                  hipEvent_t done = nullptr) {
    rg::OpenArgs a = a0;
    rg::Launch L = launch_cfg(ctx, a.n, true);
    L.done = done;
    L.staged_g = pick_family(ctx, L.staged_g, pb, st);
    ctx->last_kernel = L.staged_g;
    a.dbg = L.debug_mode == 3 ? ctx->dbg : nullptr;
    if (L.staged_g == 3) return launch_flat_any(ctx, nullptr, &a, st, done);
    if (L.staged_g == 0) return launch_pipe_any(ctx, nullptr, &a, pb, L, st);
    return launch_tiles_any(ctx, nullptr, &a, pb, L, st);
}

// --------------------------------------------------------------- device API
int rg_seal_batch_dev(rg_ctx *ctx, const uint8_t *keys, const uint32_t *receivers, uint32_t nkeys,
                      const rg_pkt_desc *desc, const uint64_t *counters, size_t n, uint8_t *buf, size_t buf_len,
                      uint8_t *status, void *stream) {
    DeviceGuard dg_;
    int rc = check_ctx(ctx);
    if (rc) return rc;
    if (n == 0) return RG_OK;
    if (!keys || !desc || !counters || !buf || !status || nkeys == 0 || n > 0xFFFFFFFFull)
        return set_err(RG_EINVAL, "seal: bad args (status is required)");
    hipStream_t st = (hipStream_t)stream;
    rc = claim_stream(ctx, st);
    if (rc) return rc;
    rg::SealArgs a{};
    a.keys = reinterpret_cast<const uint32_t *>(keys);
    a.receivers = receivers;
    a.desc = desc;
    a.counters = counters;
    a.buf = buf;
    a.buf_len = buf_len;
    a.status = status;
    a.nkeys = nkeys;
    a.n = (uint32_t)n;
    hipEvent_t ev = stream_event(ctx, st);
    RG_HIP(launch_seal_any(ctx, a, ctx->plan_dev, st, ev), "seal launch");
    mark_stream(ctx, st, ev);
    return RG_OK;
}

int rg_open_batch_dev(rg_ctx *ctx, const uint8_t *keys, uint32_t nkeys, const rg_pkt_desc *desc, size_t n,
                      uint8_t *buf, size_t buf_len, uint8_t *status, uint64_t *counters_out, void *stream) {
    DeviceGuard dg_;
    int rc = check_ctx(ctx);
    if (rc) return rc;
    if (n == 0) return RG_OK;
    if (!keys || !desc || !buf || !status || nkeys == 0 || n > 0xFFFFFFFFull)
        return set_err(RG_EINVAL, "open: bad args");
    hipStream_t st = (hipStream_t)stream;
    rc = claim_stream(ctx, st);
    if (rc) return rc;
    rg::OpenArgs a{};
    a.keys = reinterpret_cast<const uint32_t *>(keys);
    a.desc = desc;
    a.buf = buf;
    a.buf_len = buf_len;
    a.status = status;
    a.counters_out = counters_out;
    a.nkeys = nkeys;
    a.n = (uint32_t)n;
    hipEvent_t ev = stream_event(ctx, st);
    RG_HIP(launch_open_any(ctx, a, ctx->plan_dev, st, ev), "open launch");
    mark_stream(ctx, st, ev);
    return RG_OK;
}

int rg_synth_fill_dev(rg_ctx *ctx, const rg_pkt_desc *desc, const uint32_t *inner_len, size_t n, uint8_t *buf,
                      size_t buf_len, uint64_t seed, void *stream) {
    DeviceGuard dg_;
    int rc = check_ctx(ctx);
    if (rc) return rc;
    if (n == 0) return RG_OK;
    if (!desc || !inner_len || !buf || n > 0x7FFFFFFFull) return set_err(RG_EINVAL, "synth: bad args");
    RG_HIP(rg::launch_synth_fill(desc, inner_len, (uint32_t)n, buf, buf_len, seed, (hipStream_t)stream),
           "synth launch");
    return RG_OK;
}

int rg_rx_table_build(const uint32_t *receivers, const uint32_t *key_idx, size_t n, rg_rx_entry *table,
                      uint32_t cap) {
    if (!table || (n && (!receivers || !key_idx))) return set_err(RG_EINVAL, "rx table: null pointer");
    if (cap == 0 || (cap & (cap - 1)) != 0 || (uint64_t)cap < 2ull * n)
        return set_err(RG_EINVAL, "rx table: cap must be a power of two >= 2 n");
    for (uint32_t s = 0; s < cap; ++s) table[s] = rg_rx_entry{0, RG_KEY_SKIP};
    for (size_t i = 0; i < n; ++i) {
        if (key_idx[i] == RG_KEY_SKIP) return set_err(RG_EINVAL, "rx table: key index RG_KEY_SKIP is reserved");
        uint32_t s = rg::rx_slot(receivers[i], cap);
        while (table[s].key_idx != RG_KEY_SKIP) {
            if (table[s].receiver == receivers[i]) return set_err(RG_EINVAL, "rx table: duplicate receiver");
            s = (s + 1) & (cap - 1);
        }
        table[s] = rg_rx_entry{receivers[i], key_idx[i]};
    }
    return RG_OK;
}

int64_t rg_rx_table_find(const rg_rx_entry *table, uint32_t cap, uint32_t receiver) {
    if (!table || cap == 0 || (cap & (cap - 1)) != 0) return -1;
    uint32_t s = rg::rx_slot(receiver, cap);
    for (uint32_t probe = 0; probe < cap && table[s].key_idx != RG_KEY_SKIP; ++probe) {
        if (table[s].receiver == receiver) return table[s].key_idx;
        s = (s + 1) & (cap - 1);
    }
    return -1;
}

int rg_open_batch_dev_rx(rg_ctx *ctx, const uint8_t *keys, uint32_t nkeys, const rg_rx_entry *rx_table,
                         uint32_t rx_cap, const rg_pkt_desc *desc, size_t n, uint8_t *buf, size_t buf_len,
                         uint8_t *status, uint64_t *counters_out, uint32_t *key_idx_out, void *stream) {
    DeviceGuard dg_;
    int rc = check_ctx(ctx);
    if (rc) return rc;
    if (n == 0) return RG_OK;
    if (!rx_table || rx_cap == 0 || (rx_cap & (rx_cap - 1)) != 0 || !desc || n > 0xFFFFFFFFull)
        return set_err(RG_EINVAL, "open_rx: bad args");
    rc = claim_stream(ctx, (hipStream_t)stream); // before the resolve pass writes the context's descriptors
    if (rc) return rc;
    // resolved descriptors live in the context: calls on one context are stream-ordered
    RG_HIP(ctx->d_rx_desc.reserve(n * sizeof(rg_pkt_desc)), "rx descriptors");
    auto *rd = static_cast<rg_pkt_desc *>(ctx->d_rx_desc.p);
    RG_HIP(rg::launch_rx_resolve(desc, (uint32_t)n, buf, buf_len, rx_table, rx_cap, rd, key_idx_out,
                                 (hipStream_t)stream),
           "rx resolve launch");
    return rg_open_batch_dev(ctx, keys, nkeys, rd, n, buf, buf_len, status, counters_out, stream);
}

int rg_mac_verify_batch_dev(rg_ctx *ctx, const uint8_t *keys, uint32_t key_len, uint32_t nkeys, int which,
                            const rg_pkt_desc *desc, size_t n, const uint8_t *buf, size_t buf_len, uint8_t *status,
                            uint32_t *key_idx_out, void *stream) {
    DeviceGuard dg_;
    int rc = check_ctx(ctx);
    if (rc) return rc;
    if (n == 0) return RG_OK;
    if (!keys || nkeys == 0 || (key_len != 16 && key_len != 32) || (which != 1 && which != 2) || !desc || !buf ||
        !status || n > 0xFFFFFFFFull)
        return set_err(RG_EINVAL, "mac verify: bad args");
    rg::MacArgs a{};
    a.keys = reinterpret_cast<const uint32_t *>(keys);
    a.key_len = key_len;
    a.nkeys = nkeys;
    a.which = (uint32_t)which;
    a.n = (uint32_t)n;
    a.desc = desc;
    a.buf = buf;
    a.buf_len = buf_len;
    a.status = status;
    a.key_out = key_idx_out;
    // the states are key material: a regrow wipes the old block behind its readers, on this stream
    std::lock_guard<std::mutex> g(ctx->mu);
    hipStream_t st = (hipStream_t)stream;
    RG_HIP(ctx->d_mac_keys.reserve((size_t)nkeys * 32, st), "mac key states");
    a.key_state = static_cast<uint32_t *>(ctx->d_mac_keys.p);
    RG_HIP(rg::launch_mac_verify(a, st), "mac verify launch");
    RG_HIP(ctx->d_mac_keys.use(st), "mac key states event");
    return RG_OK;
}

void *rg_host_alloc(size_t bytes) {
    void *p = nullptr;
    if (hipHostMalloc(&p, bytes ? bytes : 1, hipHostMallocDefault) != hipSuccess) return nullptr;
    return p;
}

void rg_host_free(void *p) {
    if (p) (void)hipHostFree(p);
}

int rg_numa_node(rg_ctx *ctx) {
    if (!ctx) return set_err(RG_EINVAL, "null context");
    return ctx->numa_node;
}

int rg_numa_bind(void *p, size_t bytes, int node) {
    if (!p || !bytes || node < 0 || node >= 1024) return set_err(RG_EINVAL, "numa_bind: bad args");
#ifdef SYS_mbind
    const uintptr_t pg = (uintptr_t)sysconf(_SC_PAGESIZE);
    const uintptr_t a = (uintptr_t)p & ~(pg - 1), b = ((uintptr_t)p + bytes + pg - 1) & ~(pg - 1);
    unsigned long mask[16] = {0};
    mask[node / 64] = 1ul << (node % 64);
    // MPOL_BIND, MPOL_MF_MOVE: pages already touched move to the node (pinned pages cannot: bind first)
    if (syscall(SYS_mbind, a, b - a, 2 /* MPOL_BIND */, mask, 1024ul, 2u /* MPOL_MF_MOVE */) != 0) {
        char what[96];
        snprintf(what, sizeof what, "numa_bind: mbind to node %d failed (errno %d)", node, errno);
        return set_err(RG_EINVAL, what);
    }
    return RG_OK;
#else
    return set_err(RG_EINVAL, "numa_bind: no mbind on this platform");
#endif
}

int rg_host_register(void *p, size_t bytes) {
    if (!p || !bytes) return set_err(RG_EINVAL, "host_register: bad args");
    RG_HIP(hipHostRegister(p, bytes, hipHostRegisterDefault), "hipHostRegister");
    return RG_OK;
}

int rg_host_unregister(void *p) {
    if (!p) return set_err(RG_EINVAL, "host_unregister: null");
    RG_HIP(hipHostUnregister(p), "hipHostUnregister");
    return RG_OK;
}

} // extern "C"

// ------------------------------------------------------------ host pipeline
namespace {

constexpr size_t kSlicePkts = 1u << 16;
constexpr uint64_t kOutOfRange = (UINT64_MAX / 2) & ~15ull;

bool in_arena(const rg_pkt_desc &d, bool open, size_t buf_len) {
    const uint64_t need = (uint64_t)d.len + (open ? 0 : 32);
    return d.offset <= buf_len && need <= buf_len - d.offset && d.len <= rg::kMaxPayload + 32;
}

// The key table of a host call, on the upload stream ahead of the slices' frames (a slice's kernel
// waits for its frames' upload, so for the keys too).  Every host call drains its slices before it
// returns (run_host), so no kernel still reads the old table when a regrow wipes it.
int upload_keys(rg_ctx *ctx, const uint8_t *keys, const uint32_t *receivers, uint32_t nkeys) {
    RG_HIP(ctx->d_keys.reserve((size_t)nkeys * 32, ctx->hs_in), "alloc keys");
    RG_HIP(hipMemcpyAsync(ctx->d_keys.p, keys, (size_t)nkeys * 32, hipMemcpyHostToDevice, ctx->hs_in), "H2D keys");
    if (receivers) {
        RG_HIP(ctx->d_recv.reserve((size_t)nkeys * 4), "alloc receivers");
        RG_HIP(hipMemcpy(ctx->d_recv.p, receivers, (size_t)nkeys * 4, hipMemcpyHostToDevice), "H2D receivers");
    }
    return RG_OK;
}

// Drain a finished slice: copy statuses / counters back to the caller.  A status still RG_PKT_PENDING
// after the slice completed is a packet no kernel finished: the call fails (include/rg_aead.h).
int finish_slot(Slot &s, uint32_t wait_ms, uint8_t *status, uint64_t *counters_out) {
    if (!s.busy) return RG_OK;
    RG_WAIT(s.ev_out, wait_ms, "slice wait");
    if (s.orphan) {
        s.busy = s.orphan = false;
        return RG_OK;
    }
    const size_t m = s.i1 - s.i0;
    if (status) memcpy(status + s.i0, s.h_status.p, m);
    if (counters_out) memcpy(counters_out + s.i0, s.h_ctr_out.p, m * 8);
    s.busy = false;
    if (m && memchr(s.h_status.p, RG_PKT_PENDING, m)) {
        char what[128];
        snprintf(what, sizeof what, "slice [%zu, %zu): the kernel left packets unfinished (RG_PKT_PENDING)", s.i0,
                 s.i1);
        return set_err(RG_EDEVICE, what);
    }
    return RG_OK;
}

// Shared driver of the host entry points: packets [i, end) of the caller's arrays through one
// context's three-slot H2D -> kernel -> D2H pipeline, one slice per step().  A group (rg_group)
// drives one run per context (run_host_group).
struct HostRun {
    rg_ctx *ctx;
    bool open;
    uint32_t nkeys;
    const rg_pkt_desc *desc;
    const uint64_t *counters;
    size_t i, end;
    uint8_t *buf;
    size_t buf_len;
    uint8_t *status;
    uint64_t *counters_out;
    bool with_receivers;
    int which = 0;

    bool done() const { return i >= end; }
    // the slot the next step() reuses holds no slice in flight (or its download has completed): step()
    // will not block (hipEventQuery, no wait)
    bool ready() const {
        const Slot &s = ctx->slots[which];
        return !s.busy || hipEventQuery(s.ev_out) == hipSuccess;
    }
    int step(uint64_t ticket = 0); // enqueue the next slice (after draining the slot it reuses)
    // every slot's slice back (the first error is the result; the other slots still drain)
    int drain() {
        int rc = RG_OK;
        for (auto &s : ctx->slots) {
            const int r = finish_slot(s, ctx->wait_ms, status, open ? counters_out : nullptr);
            if (rc == RG_OK) rc = r;
        }
        return rc;
    }
};

int HostRun::step(uint64_t ticket) {
    RG_HIP(hipSetDevice(ctx->device), "hipSetDevice");
    // slice [i, j): bounded by packet count and by the byte span of its frames
    size_t j = i;
    uint64_t lo = UINT64_MAX, hi = 0;
    const size_t slice_bytes = ctx->host_slice;
    while (j < end && j - i < kSlicePkts) {
        const rg_pkt_desc &d = desc[j];
        if (in_arena(d, open, buf_len)) {
            const uint64_t e = d.offset + (uint64_t)d.len + (open ? 0 : 32);
            const uint64_t nlo = std::min<uint64_t>(lo, d.offset & ~15ull), nhi = std::max<uint64_t>(hi, e);
            if (j > i && nhi - nlo > slice_bytes) break;
            lo = nlo;
            hi = nhi;
        }
        ++j;
    }
    if (lo == UINT64_MAX) lo = hi = 0; // nothing in range: only statuses come back
    Slot &s = ctx->slots[which];
    int rc = finish_slot(s, ctx->wait_ms, status, counters_out);
    if (rc) return rc;
    const size_t m = j - i;
    const size_t span = hi - lo;
    RG_HIP(s.d_buf.reserve(span + 16), "alloc slice");
    RG_HIP(s.h_desc.reserve_mapped(m * sizeof(rg_pkt_desc)), "alloc h_desc");
    RG_HIP(s.h_status.reserve_mapped(m), "alloc h_status");
    // the slice's statuses start pending in host memory, whichever kernel runs (the previous slice's
    // verdicts must not stand for a packet the kernel never reaches)
    memset(s.h_status.p, RG_PKT_PENDING, m);
    rg_pkt_desc *hd = static_cast<rg_pkt_desc *>(s.h_desc.p);
    for (size_t k = 0; k < m; ++k) {
        hd[k] = desc[i + k];
        // frames outside the arena get an aligned out-of-range offset: the kernel flags them INVALID
        hd[k].offset = in_arena(desc[i + k], open, buf_len) ? desc[i + k].offset - lo : kOutOfRange;
    }
    if (!open) {
        RG_HIP(s.h_ctr.reserve_mapped(m * 8), "alloc h_ctr");
        memcpy(s.h_ctr.p, counters + i, m * 8);
    } else {
        RG_HIP(s.h_ctr_out.reserve_mapped(m * 8), "alloc h_ctr_out");
    }
    // the frames' upload on hs_in (after the previous use of this slot's buffers has been downloaded: the
    // host waited for ev_out above, so nothing of it is still in flight); descriptors, counters and
    // statuses stay in mapped host memory, which the kernel reads and writes over the link in place of
    // three small copies per slice (round 4, profiles/r4_e2e_mapped_ab.txt)
    hipStream_t sin = ctx->hs_in, srun = ctx->hs_run, sout = ctx->hs_out;
    if (span) RG_HIP(hipMemcpyAsync(s.d_buf.p, buf + lo, span, hipMemcpyHostToDevice, sin), "H2D frames");
    uint8_t *dbuf = static_cast<uint8_t *>(s.d_buf.p);
    RG_HIP(hipEventRecord(s.ev_in, sin), "slice event");
    // the kernel on hs_run, once the inputs are in
    RG_HIP(hipStreamWaitEvent(srun, s.ev_in, 0), "slice wait");
    if (!open) {
        rg::SealArgs a{};
        a.keys = static_cast<const uint32_t *>(ctx->d_keys.p);
        a.receivers = with_receivers ? static_cast<const uint32_t *>(ctx->d_recv.p) : nullptr;
        a.desc = static_cast<const rg_pkt_desc *>(s.h_desc.d);
        a.counters = static_cast<const uint64_t *>(s.h_ctr.d);
        a.buf = dbuf;
        a.buf_len = span;
        a.status = static_cast<uint8_t *>(s.h_status.d);
        a.nkeys = nkeys;
        a.n = (uint32_t)m;
        RG_HIP(launch_seal_any(ctx, a, s.plan, srun), "seal launch");
    } else {
        rg::OpenArgs a{};
        a.keys = static_cast<const uint32_t *>(ctx->d_keys.p);
        a.desc = static_cast<const rg_pkt_desc *>(s.h_desc.d);
        a.buf = dbuf;
        a.buf_len = span;
        a.status = static_cast<uint8_t *>(s.h_status.d);
        a.counters_out = static_cast<uint64_t *>(s.h_ctr_out.d);
        a.nkeys = nkeys;
        a.n = (uint32_t)m;
        RG_HIP(launch_open_any(ctx, a, s.plan, srun), "open launch");
    }
    RG_HIP(hipEventRecord(s.ev_run, srun), "slice event");
    // downloads on hs_out, once the kernel is done
    RG_HIP(hipStreamWaitEvent(sout, s.ev_run, 0), "slice wait");
    if (span) RG_HIP(hipMemcpyAsync(buf + lo, s.d_buf.p, span, hipMemcpyDeviceToHost, sout), "D2H frames");
    RG_HIP(hipEventRecord(s.ev_out, sout), "slice event");
    s.i0 = i;
    s.i1 = j;
    s.ticket = ticket;
    s.busy = true;
    i = j;
    which = (which + 1) % rg_ctx::kHostSlots;
    return RG_OK;
}

// Runs to completion from one thread (one context, or several when a group cannot start a thread per
// context, or in builds with RG_GROUP_THREADS=0).  A run is stepped
// when the slot its next slice reuses is free, so that no context waits while another's download is in
// flight (round 4 stepped round-robin and blocked in each step on the slot it reused: VERDICT r4 item 5);
// only when every unfinished run's next slot is still busy does the thread block, on the slice issued
// first of all (the oldest download).  On an error every run still drains what it has in flight (its
// slots are reused by the next call).
int run_host(HostRun *runs, size_t nruns) {
    int rc = RG_OK;
    uint64_t ticket = 0;
    while (rc == RG_OK) {
        bool more = false, moved = false;
        for (HostRun *rp = runs; rp != runs + nruns; ++rp) {
            HostRun &r = *rp;
            if (r.done()) continue;
            more = true;
            if (!r.ready()) continue;
            rc = r.step(++ticket);
            if (rc) break;
            moved = true;
        }
        if (!more || rc != RG_OK) break;
        if (!moved) {
            Slot *oldest = nullptr;
            uint32_t wait_ms = kDefaultWaitMs;
            for (HostRun *rp = runs; rp != runs + nruns; ++rp) {
                HostRun &r = *rp;
                if (r.done()) continue;
                Slot &s = r.ctx->slots[r.which];
                if (s.busy && (!oldest || s.ticket < oldest->ticket)) {
                    oldest = &s;
                    wait_ms = r.ctx->wait_ms;
                }
            }
            if (oldest) rc = wait_event(oldest->ev_out, wait_ms, "slice wait");
        }
    }
    for (HostRun *rp = runs; rp != runs + nruns; ++rp) {
        (void)hipSetDevice(rp->ctx->device);
        const int rc2 = rp->drain();
        if (rc == RG_OK) rc = rc2;
        for (auto &s : rp->ctx->slots) // still in flight after a failed wait: no longer this call's
            if (s.busy) s.orphan = true;
    }
    return rc;
}

// A group's runs, one worker thread per context (round 5).  From one thread, each slice costs ~50 us of
// HIP API calls: two copies, a launch, three event records and two stream waits
// (profiles/r5_e2e_chain.txt). At 8 MiB slices and ~45 GB/s per link, that feeds about four links.
// With a thread per context, the calls of different devices overlap, and each thread waits only for its
// own device. The caller's thread starts the workers and joins them. If a thread cannot be started, the
// caller's thread runs the remaining runs itself. The first failing run's error becomes the call's
// (rg_last_error is per thread).
// NUMA placement of a group's worker thread: on a two-socket host half the GPUs hang
// off the other socket, and a worker that drives a GPU from there crosses the socket link for every API
// call and for the slot buffers it touches.  The worker is pinned to the CPUs of its GPU's node that this
// process may use (none allowed there: left as it is), and its memory policy prefers that node, so the
// slice buffers it allocates and first-touches land there.  The caller's frames are the caller's: see
// rg_numa_bind / rg_host_register (include/rg_aead.h).
bool node_cpus(int node, cpu_set_t *out) {
    char path[96];
    snprintf(path, sizeof path, "/sys/devices/system/node/node%d/cpulist", node);
    FILE *f = fopen(path, "r");
    if (!f) return false;
    char line[4096];
    const bool got = fgets(line, sizeof line, f) != nullptr;
    fclose(f);
    if (!got) return false;
    CPU_ZERO(out);
    for (char *p = line; *p && *p != '\n';) { // "0-15,128-143"
        char *end = nullptr;
        const long a = strtol(p, &end, 10);
        if (end == p) break;
        long b = a;
        if (*end == '-') {
            p = end + 1;
            b = strtol(p, &end, 10);
        }
        for (long c = a; c <= b && c < CPU_SETSIZE; ++c) CPU_SET((int)c, out);
        p = *end == ',' ? end + 1 : end;
    }
    return true;
}

int place_thread(int node) {
    if (node < 0) return -1;
    cpu_set_t want, allowed;
    if (!node_cpus(node, &want) || sched_getaffinity(0, sizeof allowed, &allowed) != 0) return -1;
    CPU_AND(&want, &want, &allowed);
    if (CPU_COUNT(&want) == 0) return -1; // none of the node's CPUs is ours
    if (sched_setaffinity(0, sizeof want, &want) != 0) return -1;
#ifdef SYS_set_mempolicy
    unsigned long mask[16] = {0};
    if (node < 1024) {
        mask[node / 64] = 1ul << (node % 64);
        (void)syscall(SYS_set_mempolicy, 1 /* MPOL_PREFERRED */, mask, 1024ul);
    }
#endif
    return CPU_COUNT(&want);
}

#ifndef RG_GROUP_THREADS
#define RG_GROUP_THREADS 1
#endif
int run_host_group(std::vector<HostRun> &runs) {
    if (!RG_GROUP_THREADS || runs.size() < 2) return run_host(runs.data(), runs.size());
    // Threads pay off once a context has a few slices to pipeline; a small batch (every part within two
    // slices) runs from the calling thread, without starting and joining a thread per context.
    bool big = false;
    for (const HostRun &r : runs) {
        uint64_t bytes = 0;
        for (size_t k = r.i; k < r.end && !big; ++k) {
            bytes += (uint64_t)r.desc[k].len + 32;
            big = bytes > 2 * (uint64_t)r.ctx->host_slice;
        }
        if (big) break;
    }
    if (!big) return run_host(runs.data(), runs.size());
    const size_t n = runs.size();
    std::vector<int> rcs;
    std::vector<std::string> errs;
    std::vector<std::thread> workers;
    try { // (no exception may cross the C ABI: without the bookkeeping, the calling thread runs them all)
        rcs.assign(n, RG_OK);
        errs.resize(n);
        workers.reserve(n);
    } catch (const std::exception &) {
        return run_host(runs.data(), n);
    }
    size_t started = 0;
    try {
        for (; started < n; ++started)
            workers.emplace_back([&runs, &rcs, &errs, started]() {
                place_thread(runs[started].ctx->numa_node); // the CPUs (and memory) next to this GPU
                rcs[started] = run_host(&runs[started], 1);
                if (rcs[started] != RG_OK) errs[started].swap(g_err); // the worker's own message, moved out
            });
    } catch (const std::exception &) {
        // fewer threads than runs (std::system_error): the rest run here, stepped together as before
    }
    int rc_here = RG_OK;
    std::string err_here;
    if (started < n) {
        rc_here = run_host(&runs[started], n - started);
        if (rc_here != RG_OK) err_here.swap(g_err); // (swaps: no string copy that could throw)
    }
    for (auto &t : workers) t.join();
    for (size_t k = 0; k < started; ++k)
        if (rcs[k] != RG_OK) {
            g_err.swap(errs[k]);
            return rcs[k];
        }
    if (rc_here != RG_OK) g_err.swap(err_here);
    return rc_here;
}

// A slice moves the byte span of its frames H2D and back D2H, so slices must cover disjoint spans: with
// the descriptors in offset order they do (frames do not overlap), in any other order a slice's span
// would take in other slices' frames and its D2H copy could put back stale bytes over their results.
// Batches not in offset order therefore run on a sorted copy of the descriptors (and counters), their
// statuses and counters scattered back to the caller's order afterwards.
struct HostOrder {
    bool identity = true;
    std::vector<rg_pkt_desc> desc;
    std::vector<uint64_t> ctr, ctr_out;
    std::vector<uint8_t> status;
    std::vector<uint32_t> perm; // sorted position k -> caller index
};

bool in_offset_order(const rg_pkt_desc *desc, size_t n) {
    for (size_t i = 1; i < n; ++i)
        if (desc[i].offset < desc[i - 1].offset) return false;
    return true;
}

// RunFn(desc, counters, status, counters_out): the pipeline over the (possibly permuted) arrays
template <class RunFn>
int run_ordered(const rg_pkt_desc *desc, const uint64_t *counters, size_t n, uint8_t *status, uint64_t *counters_out,
                RunFn &&run) {
    if (in_offset_order(desc, n)) return run(desc, counters, status, counters_out);
    HostOrder o;
    o.perm.resize(n);
    for (size_t i = 0; i < n; ++i) o.perm[i] = (uint32_t)i;
    std::stable_sort(o.perm.begin(), o.perm.end(),
                     [&](uint32_t a, uint32_t b) { return desc[a].offset < desc[b].offset; });
    o.desc.resize(n);
    o.status.resize(n);
    for (size_t k = 0; k < n; ++k) o.desc[k] = desc[o.perm[k]];
    if (counters) {
        o.ctr.resize(n);
        for (size_t k = 0; k < n; ++k) o.ctr[k] = counters[o.perm[k]];
    }
    if (counters_out) o.ctr_out.resize(n);
    const int rc = run(o.desc.data(), counters ? o.ctr.data() : nullptr, o.status.data(),
                       counters_out ? o.ctr_out.data() : nullptr);
    for (size_t k = 0; k < n; ++k) {
        status[o.perm[k]] = o.status[k];
        if (counters_out) counters_out[o.perm[k]] = o.ctr_out[k];
    }
    return rc;
}

int host_batch(rg_ctx *ctx, bool open, uint32_t nkeys, const rg_pkt_desc *desc, const uint64_t *counters, size_t n,
               uint8_t *buf, size_t buf_len, uint8_t *status, uint64_t *counters_out, bool with_receivers) {
    return run_ordered(desc, counters, n, status, counters_out,
                       [&](const rg_pkt_desc *d, const uint64_t *c, uint8_t *st, uint64_t *co) {
                           HostRun run{ctx, open, nkeys, d, c, 0, n, buf, buf_len, st, co, with_receivers};
                           return run_host(&run, 1);
                       });
}

// The end of every host call on a context: the key table's upload on hs_in has completed (a context of a
// group that ran no slice, or a call that failed before its first slice, never waited for it, and the
// caller may reuse a pinned key buffer as soon as the call returns: ADVICE r5), and a failed call leaves
// every status pending (include/rg_aead.h).
int settle_host(rg_ctx *ctx, int rc) {
    hipError_t e = hipSuccess;
    if (!ctx->ev_in_idle) e = hipEventCreateWithFlags(&ctx->ev_in_idle, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventRecord(ctx->ev_in_idle, ctx->hs_in);
    int r2 = e == hipSuccess ? wait_event(ctx->ev_in_idle, ctx->wait_ms, "key upload") : set_err(RG_EDEVICE, "key upload", e);
    return rc != RG_OK ? rc : r2;
}

int fail_closed(int rc, uint8_t *status, size_t n) {
    if (rc < 0 && status) memset(status, RG_PKT_PENDING, n);
    return rc;
}

} // namespace

extern "C" {

int rg_seal_batch_host(rg_ctx *ctx, const uint8_t *keys, const uint32_t *receivers, uint32_t nkeys,
                       const rg_pkt_desc *desc, const uint64_t *counters, size_t n, uint8_t *buf, size_t buf_len,
                       uint8_t *status) {
    DeviceGuard dg_;
    int rc = check_ctx(ctx);
    if (rc) return fail_closed(rc, status, n);
    if (n == 0) return RG_OK;
    if (!keys || !desc || !counters || !buf || nkeys == 0)
        return fail_closed(set_err(RG_EINVAL, "seal_host: bad args"), status, n);
    std::lock_guard<std::mutex> g(ctx->mu);
    std::vector<uint8_t> tmp;
    if (!status) {
        tmp.resize(n);
        status = tmp.data();
    }
    rc = upload_keys(ctx, keys, receivers, nkeys);
    if (rc == RG_OK)
        rc = host_batch(ctx, false, nkeys, desc, counters, n, buf, buf_len, status, nullptr, receivers != nullptr);
    return fail_closed(settle_host(ctx, rc), status, n);
}

int rg_open_batch_host(rg_ctx *ctx, const uint8_t *keys, uint32_t nkeys, const rg_pkt_desc *desc, size_t n,
                       uint8_t *buf, size_t buf_len, uint8_t *status, uint64_t *counters_out) {
    DeviceGuard dg_;
    int rc = check_ctx(ctx);
    if (rc) return fail_closed(rc, status, n);
    if (n == 0) return RG_OK;
    if (!keys || !desc || !buf || !status || nkeys == 0)
        return fail_closed(set_err(RG_EINVAL, "open_host: bad args"), status, n);
    std::lock_guard<std::mutex> g(ctx->mu);
    std::vector<uint64_t> tmp;
    if (!counters_out) {
        tmp.resize(n);
        counters_out = tmp.data();
    }
    rc = upload_keys(ctx, keys, nullptr, nkeys);
    if (rc == RG_OK) rc = host_batch(ctx, true, nkeys, desc, nullptr, n, buf, buf_len, status, counters_out, false);
    return fail_closed(settle_host(ctx, rc), status, n);
}

} // extern "C"

// ------------------------------------------------------------ device group
struct rg_group {
    std::vector<rg_ctx *> ctx;
};

namespace {

// work of packet i for the split: its AEAD payload bytes plus one 64-byte one-time-key block
uint64_t split_work(const rg_pkt_desc &d, bool open) {
    const uint64_t P = open ? (d.len >= 32 ? d.len - 32 : 0) : d.len;
    return std::min<uint64_t>(P, rg::kMaxPayload) + 64;
}

void split_bounds(const rg_pkt_desc *desc, size_t n, bool open, int parts, size_t *bounds) {
    uint64_t total = 0;
    for (size_t i = 0; i < n; ++i) total += split_work(desc[i], open);
    bounds[0] = 0;
    size_t i = 0;
    uint64_t run = 0;
    for (int k = 1; k < parts; ++k) {
        // the first index whose running work before it reaches k / parts of the total
        const uint64_t target = (uint64_t)((long double)total * k / parts);
        while (i < n && run + split_work(desc[i], open) / 2 < target) run += split_work(desc[i++], open);
        bounds[k] = i;
    }
    bounds[parts] = n;
}

// every context of the group, locked in index order (a group's calls are serialised per context as
// a single context's are)
struct GroupLock {
    std::vector<std::unique_lock<std::mutex>> held;
    explicit GroupLock(rg_group *g) {
        for (rg_ctx *c : g->ctx) held.emplace_back(c->mu);
    }
};

int host_multi(rg_group *g, bool open, const uint8_t *keys, const uint32_t *receivers, uint32_t nkeys,
               const rg_pkt_desc *desc, const uint64_t *counters, size_t n, uint8_t *buf, size_t buf_len,
               uint8_t *status, uint64_t *counters_out) {
    DeviceGuard dg;
    GroupLock lk(g);
    const int parts = (int)g->ctx.size();
    int rc = RG_OK;
    int uploaded = 0; // contexts whose key upload was enqueued (each is settled below)
    for (; uploaded < parts && rc == RG_OK; ++uploaded) {
        const hipError_t e = hipSetDevice(g->ctx[uploaded]->device);
        rc = e != hipSuccess ? set_err(RG_EDEVICE, "hipSetDevice", e)
                             : upload_keys(g->ctx[uploaded], keys, receivers, nkeys);
    }
    // the split is over the batch in offset order, so the contexts' byte spans are disjoint too
    if (rc == RG_OK)
        rc = run_ordered(desc, counters, n, status, counters_out,
                         [&](const rg_pkt_desc *d, const uint64_t *c, uint8_t *st, uint64_t *co) {
                             std::vector<size_t> b(parts + 1);
                             split_bounds(d, n, open, parts, b.data());
                             std::vector<HostRun> runs;
                             for (int k = 0; k < parts; ++k)
                                 if (b[k] < b[k + 1])
                                     runs.push_back(HostRun{g->ctx[k], open, nkeys, d, c, b[k], b[k + 1], buf,
                                                            buf_len, st, co, receivers != nullptr});
                             return run_host_group(runs);
                         });
    for (int k = 0; k < uploaded; ++k) {
        (void)hipSetDevice(g->ctx[k]->device);
        rc = settle_host(g->ctx[k], rc);
    }
    return fail_closed(rc, status, n);
}

} // namespace

extern "C" {

int rg_group_create(const int *devices, int n, rg_group **out) {
    if (!out) return set_err(RG_EINVAL, "group: null out");
    *out = nullptr;
    if (!devices || n <= 0 || n > 64) return set_err(RG_EINVAL, "group: 1..64 devices");
    rg_group *g = new (std::nothrow) rg_group();
    if (!g) return set_err(RG_ENOMEM, "alloc group");
    DeviceGuard dg;
    for (int i = 0; i < n; ++i) {
        rg_ctx *c = nullptr;
        int rc = rg_create(devices[i], &c);
        if (rc) {
            rg_group_destroy(g);
            return rc;
        }
        g->ctx.push_back(c);
    }
    *out = g;
    return RG_OK;
}

void rg_group_destroy(rg_group *g) {
    if (!g) return;
    DeviceGuard dg;
    for (rg_ctx *c : g->ctx) rg_destroy(c);
    delete g;
}

int rg_group_size(const rg_group *g) { return g ? (int)g->ctx.size() : set_err(RG_EINVAL, "group: null"); }

rg_ctx *rg_group_ctx(rg_group *g, int i) {
    if (!g || i < 0 || i >= (int)g->ctx.size()) return nullptr;
    return g->ctx[i];
}

int rg_split_batch(const rg_pkt_desc *desc, size_t n, int open, int parts, size_t *bounds) {
    if (!bounds || parts <= 0 || (n && !desc)) return set_err(RG_EINVAL, "split: bad args");
    split_bounds(desc, n, open != 0, parts, bounds);
    return RG_OK;
}

int rg_seal_batch_host_multi(rg_group *g, const uint8_t *keys, const uint32_t *receivers, uint32_t nkeys,
                             const rg_pkt_desc *desc, const uint64_t *counters, size_t n, uint8_t *buf,
                             size_t buf_len, uint8_t *status) {
    if (!g || g->ctx.empty()) return fail_closed(set_err(RG_EINVAL, "seal_host_multi: null group"), status, n);
    if (n == 0) return RG_OK;
    if (!keys || !desc || !counters || !buf || nkeys == 0)
        return fail_closed(set_err(RG_EINVAL, "seal_host_multi: bad args"), status, n);
    std::vector<uint8_t> tmp;
    if (!status) {
        tmp.resize(n);
        status = tmp.data();
    }
    return host_multi(g, false, keys, receivers, nkeys, desc, counters, n, buf, buf_len, status, nullptr);
}

int rg_open_batch_host_multi(rg_group *g, const uint8_t *keys, uint32_t nkeys, const rg_pkt_desc *desc, size_t n,
                             uint8_t *buf, size_t buf_len, uint8_t *status, uint64_t *counters_out) {
    if (!g || g->ctx.empty()) return fail_closed(set_err(RG_EINVAL, "open_host_multi: null group"), status, n);
    if (n == 0) return RG_OK;
    if (!keys || !desc || !buf || !status || nkeys == 0)
        return fail_closed(set_err(RG_EINVAL, "open_host_multi: bad args"), status, n);
    std::vector<uint64_t> tmp;
    if (!counters_out) {
        tmp.resize(n);
        counters_out = tmp.data();
    }
    return host_multi(g, true, keys, nullptr, nkeys, desc, nullptr, n, buf, buf_len, status, counters_out);
}

// Every shard's arguments are checked before any shard is enqueued (a call that failed on
// shard k after enqueuing shards 0..k-1 left the caller unable to tell which frames were sealed, and a
// retry would seal those again under new counters).  A launch that fails after the checks names its
// shard in rg_last_error; the shards before it are enqueued (include/rg_aead.h).
static int check_shards(rg_group *g, const rg_dev_shard *sh, bool open) {
    for (size_t k = 0; k < g->ctx.size(); ++k) {
        const rg_dev_shard &x = sh[k];
        if (x.n == 0) continue;
        const bool bad = !g->ctx[k] || !x.keys || !x.desc || !x.buf || !x.status || x.nkeys == 0 ||
                         x.n > 0xFFFFFFFFull || (!open && !x.counters);
        if (bad) {
            char what[96];
            snprintf(what, sizeof what, "%s_dev_multi: bad args in shard %zu (nothing enqueued)", open ? "open" : "seal", k);
            return set_err(RG_EINVAL, what);
        }
    }
    return RG_OK;
}

static int shard_failed(int rc, const char *op, size_t k) {
    const std::string inner = g_err;
    char what[384];
    if (k == 0)
        snprintf(what, sizeof what, "%s_dev_multi: shard 0 failed (nothing enqueued): %s", op, inner.c_str());
    else
        snprintf(what, sizeof what, "%s_dev_multi: shard %zu failed (shards 0..%zu enqueued): %s", op, k, k - 1,
                 inner.c_str());
    return set_err(rc, what);
}

int rg_seal_batch_dev_multi(rg_group *g, const rg_dev_shard *sh) {
    if (!g || !sh) return set_err(RG_EINVAL, "seal_dev_multi: bad args");
    int rc = check_shards(g, sh, false);
    if (rc) return rc;
    DeviceGuard dg;
    for (size_t k = 0; k < g->ctx.size(); ++k) {
        const rg_dev_shard &x = sh[k];
        rc = rg_seal_batch_dev(g->ctx[k], x.keys, x.receivers, x.nkeys, x.desc, x.counters, x.n, x.buf, x.buf_len,
                               x.status, x.stream);
        if (rc) return shard_failed(rc, "seal", k);
    }
    return RG_OK;
}

int rg_open_batch_dev_multi(rg_group *g, const rg_dev_shard *sh) {
    if (!g || !sh) return set_err(RG_EINVAL, "open_dev_multi: bad args");
    int rc = check_shards(g, sh, true);
    if (rc) return rc;
    DeviceGuard dg;
    for (size_t k = 0; k < g->ctx.size(); ++k) {
        const rg_dev_shard &x = sh[k];
        rc = rg_open_batch_dev(g->ctx[k], x.keys, x.nkeys, x.desc, x.n, x.buf, x.buf_len, x.status, x.counters_out,
                               x.stream);
        if (rc) return shard_failed(rc, "open", k);
    }
    return RG_OK;
}

// ---------------------------------------------------- per-message drop-in
// nonce: 12 bytes, or 24 for XChaCha20-Poly1305 (xchacha)
static int general_one(rg_ctx *ctx, bool dec, const uint8_t key[32], const uint8_t *nonce, const uint8_t *aad,
                       size_t aad_len, uint8_t *payload, size_t len, uint8_t tag[16], bool xchacha = false) {
    DeviceGuard dg_;
    int rc = check_ctx(ctx);
    if (rc) return rc;
    if (!key || !nonce || !tag || (aad_len && !aad) || (len && !payload))
        return set_err(RG_EINVAL, "aead: bad args");
    if (len > (64ull << 32)) return set_err(RG_EINVAL, "aead: message too long for a 32-bit block counter");
    std::lock_guard<std::mutex> g(ctx->mu);
    // one pinned image of the device arena: the inputs are packed into it on the host, moved by one
    // H2D copy, and the results come back by one D2H copy (pageable copies of each piece cost tens of
    // microseconds apiece)
    const size_t job_bytes = (sizeof(rg::GeneralJob) + 15) & ~15ull;
    const size_t aad_off = 0, pay_off = (aad_len + 15) & ~15ull, tag_off = pay_off + ((len + 15) & ~15ull);
    const size_t arena = job_bytes + tag_off + 16;
    RG_HIP(ctx->d_general.reserve(arena, ctx->gen_stream), "alloc arena");
    RG_HIP(ctx->h_general.reserve(arena), "alloc pinned arena");
    uint8_t *d = static_cast<uint8_t *>(ctx->d_general.p);
    uint8_t *h = static_cast<uint8_t *>(ctx->h_general.p);
    rg::GeneralJob job;
    memset(&job, 0, sizeof job);
    memcpy(job.key, key, 32);
    if (xchacha) { // HChaCha20 input nonce[0..16]; ChaCha20-Poly1305 nonce 0^4 || nonce[16..24]
        job.xchacha = 1;
        memcpy(job.hnonce, nonce, 16);
        memcpy(reinterpret_cast<uint8_t *>(job.nonce) + 4, nonce + 16, 8);
    } else {
        memcpy(job.nonce, nonce, 12);
    }
    job.decrypt = dec ? 1 : 0;
    job.aad_off = aad_off;
    job.aad_len = aad_len;
    job.payload_off = pay_off;
    job.payload_len = len;
    job.tag_off = tag_off;
    job.status = RG_PKT_PENDING; // fail closed: only the kernel's verdict accepts
    if (!ctx->ev_gen) {
        const hipError_t e = hipEventCreateWithFlags(&ctx->ev_gen, hipEventDisableTiming);
        if (e != hipSuccess) {
            memset(&job, 0, sizeof job);
            return set_err(RG_EDEVICE, "general event", e);
        }
    }
    memcpy(h, &job, sizeof job);
    // from here on the key sits in the pinned image (and, after the H2D copy, in the device arena):
    // wiped on every way out, errors included (the reference zeroizes keys on drop, prim.rs:227-231); the
    // waits are bounded, and a device that never completes keeps its arena (only the host image is wiped)
    struct Wipe {
        uint8_t *h, *d;
        size_t n;
        hipStream_t st;
        hipEvent_t ev;
        uint32_t ms;
        bool settled() { return hipEventRecord(ev, st) == hipSuccess && wait_event(ev, ms, "general wipe") == RG_OK; }
        ~Wipe() {
            const std::string keep = g_err; // the call's own error stays the one reported
            if (settled()) { // nothing of this call is still reading the job
                (void)hipMemsetAsync(d, 0, n, st);
                (void)settled();
            }
            memset(h, 0, n);
            g_err = keep;
        }
    } wipe{h, d, job_bytes, ctx->gen_stream, ctx->ev_gen, ctx->wait_ms};
    memset(&job.key, 0, sizeof job.key); // the stack copy
    uint8_t *hb = h + job_bytes; // arena base as the kernel sees it; padding zeroed (pad16)
    memset(hb, 0, tag_off + 16);
    if (aad_len) memcpy(hb + aad_off, aad, aad_len);
    if (len) memcpy(hb + pay_off, payload, len);
    if (dec) memcpy(hb + tag_off, tag, 16);
    hipStream_t st = ctx->gen_stream;
    RG_HIP(hipMemcpyAsync(d, h, arena, hipMemcpyHostToDevice, st), "H2D arena");
    RG_HIP(rg::launch_general(reinterpret_cast<rg::GeneralJob *>(d), 1, d + job_bytes, st), "general launch");
    RG_HIP(hipMemcpyAsync(h, d, arena, hipMemcpyDeviceToHost, st), "D2H arena");
    RG_HIP(hipEventRecord(ctx->ev_gen, st), "general event");
    RG_WAIT(ctx->ev_gen, ctx->wait_ms, "general wait");
    const uint32_t status = reinterpret_cast<const rg::GeneralJob *>(h)->status;
    if (status != RG_PKT_OK && status != RG_PKT_DECRYPT_ERR)
        return set_err(RG_EDEVICE, "aead: the kernel left the message unfinished");
    if (dec && status != RG_PKT_OK) return RG_PKT_DECRYPT_ERR; // payload untouched
    if (len) memcpy(payload, hb + pay_off, len);
    if (!dec) memcpy(tag, hb + tag_off, 16);
    return RG_OK;
}

int rg_chacha20poly1305_enc(rg_ctx *ctx, const uint8_t key[32], const uint8_t nonce[12], const uint8_t *aad,
                            size_t aad_len, uint8_t *payload, size_t len, uint8_t tag[16]) {
    return general_one(ctx, false, key, nonce, aad, aad_len, payload, len, tag);
}

int rg_chacha20poly1305_dec(rg_ctx *ctx, const uint8_t key[32], const uint8_t nonce[12], const uint8_t *aad,
                            size_t aad_len, uint8_t *payload, size_t len, const uint8_t tag[16]) {
    return general_one(ctx, true, key, nonce, aad, aad_len, payload, len, const_cast<uint8_t *>(tag));
}

int rg_xchacha20poly1305_enc(rg_ctx *ctx, const uint8_t key[32], const uint8_t nonce[24], const uint8_t *aad,
                             size_t aad_len, uint8_t *payload, size_t len, uint8_t tag[16]) {
    return general_one(ctx, false, key, nonce, aad, aad_len, payload, len, tag, true);
}

int rg_xchacha20poly1305_dec(rg_ctx *ctx, const uint8_t key[32], const uint8_t nonce[24], const uint8_t *aad,
                             size_t aad_len, uint8_t *payload, size_t len, const uint8_t tag[16]) {
    return general_one(ctx, true, key, nonce, aad, aad_len, payload, len, const_cast<uint8_t *>(tag), true);
}

// ------------------------------------------------------------ test hooks
// Built into the test library only (librg_aead_test.so, -DRG_TEST_HOOKS; include/rg_aead_test.h),
// never into the product library.
#if RG_TEST_HOOKS
int rg_debug_read_arena(rg_ctx *ctx, int which, void *dst, size_t bytes) {
    DeviceGuard dg_;
    int rc = check_ctx(ctx);
    if (rc) return rc;
    if (!dst) return set_err(RG_EINVAL, "debug_read_arena: null dst");
    const SecretBuf *b = which == 0 ? &ctx->d_general : which == 1 ? &ctx->d_keys : which == 2 ? &ctx->d_mac_keys : nullptr;
    if (!b) return set_err(RG_EINVAL, "debug_read_arena: which must be 0, 1 or 2");
    std::lock_guard<std::mutex> g(ctx->mu);
    RG_HIP(hipDeviceSynchronize(), "debug_read_arena sync"); // test hook: the buffer's writers are done
    const size_t m = std::min(bytes, b->cap);
    if (m) RG_HIP(hipMemcpy(dst, b->p, m, hipMemcpyDeviceToHost), "debug_read_arena copy");
    return (int)std::min<size_t>(m, 0x7FFFFFFF);
}

void rg_debug_fail_reserve(int nth) { g_fail_reserve.store(nth > 0 ? nth : 0); }

void rg_debug_plan_handoff(int mode) {
    g_stale_done.store(mode == 1 ? 0x40000000u : 0u);
    g_stale_pool.store(mode == 2 ? 0x40000000u : 0u);
}

void rg_debug_lose_completions(int on) { g_lose_completions.store(on ? 1 : 0); }

int rg_debug_wait_selftest(uint32_t timeout_ms, uint32_t ready_after, uint32_t *polls_out, uint32_t *elapsed_ms_out) {
    uint32_t polls = 0;
    bool late = false;
    const auto t0 = std::chrono::steady_clock::now();
    const hipError_t r = wait_bounded(
        [&]() { return ++polls > ready_after ? hipSuccess : hipErrorNotReady; }, timeout_ms, &late);
    const auto el = std::chrono::steady_clock::now() - t0;
    if (polls_out) *polls_out = polls;
    if (elapsed_ms_out) *elapsed_ms_out = (uint32_t)std::chrono::duration_cast<std::chrono::milliseconds>(el).count();
    if (late) return set_err(RG_EDEVICE, "wait selftest: timed out");
    return r == hipSuccess ? RG_OK : set_err(RG_EDEVICE, "wait selftest: error");
}

int64_t rg_debug_last_wipe(void *dst, size_t bytes, uint64_t *wipes_out) {
    std::lock_guard<std::mutex> g(g_wipe_mu);
    if (wipes_out) *wipes_out = g_wipes;
    if (!g_wipe_probe || !dst) return 0;
    const size_t m = std::min(bytes, g_wipe_bytes);
    memcpy(dst, g_wipe_probe, m);
    return (int64_t)m;
}

int rg_debug_secret_state(rg_ctx *ctx, int which, uint32_t *retired_out, uint32_t *users_out) {
    if (!ctx) return set_err(RG_EINVAL, "null context");
    const SecretBuf *b = which == 0 ? &ctx->d_general : which == 1 ? &ctx->d_keys : which == 2 ? &ctx->d_mac_keys : nullptr;
    if (!b) return set_err(RG_EINVAL, "debug_secret_state: which must be 0, 1 or 2");
    if (retired_out) *retired_out = (uint32_t)b->retired.size();
    if (users_out) *users_out = (uint32_t)b->users.size();
    return b->captured ? 1 : 0;
}
#endif

// ------------------------------------------------------------- AntiReplay
// rustyguard-utils/src/anti_replay.rs:1-64 with usize = u64:
// BITMAP_LEN = 32 words, REDUNDANT_BIT_SHIFTS = 6, WINDOW_SIZE = 2048 - 64.
void rg_antireplay_init(rg_antireplay *r) {
    if (r) memset(r, 0, sizeof *r);
}

int rg_antireplay_would_accept(const rg_antireplay *r, uint64_t n) {
    if (n > r->last) return 1;
    const uint64_t d = r->last - n;
    if (d >= RG_REPLAY_WINDOW) return 0;
    const uint64_t index = n >> 6, shift = n & 63;
    return ((r->bitmap[index & 31] >> shift) & 1) == 0;
}

void rg_antireplay_mark_seen(rg_antireplay *r, uint64_t n) {
    const uint64_t index = n >> 6, shift = n & 63;
    if (n > r->last) {
        const uint64_t next_index = (r->last >> 6) + 1;
        if (index > next_index && index - next_index > 32) {
            memset(r->bitmap, 0, sizeof r->bitmap); // the window skipped entirely ahead
        } else {
            for (uint64_t i = next_index; i <= index; ++i) r->bitmap[i & 31] = 0;
        }
        r->last = n;
    }
    r->bitmap[index & 31] |= 1ull << shift;
}

} // extern "C"

// ----------------------------------------------------------- session table
namespace {
struct Session {
    bool used = false;
    uint32_t local_id = 0, remote_id = 0;
    uint64_t send_ctr = 0;
    rg_antireplay replay{};
    // rustyguard-core/src/lib.rs:185-191: when the session started and last sent, whether a
    // keepalive is already scheduled; plus the peer endpoint learned from authenticated packets
    uint64_t started = 0, sent = 0;
    bool keepalive_pending = false;
    bool has_endpoint = false; // sessions without a peer (rg_sessions_insert) keep their own endpoint
    uint64_t endpoint = 0;
    uint32_t peer = RG_PEER_NONE;
};
// PeerState's endpoint (rustyguard-core/src/lib.rs:160-181, :670-671): shared by the peer's sessions
struct Peer {
    bool has_endpoint = false;
    uint64_t endpoint = 0;
};
constexpr uint64_t kNsPerSec = 1000000000ull;
constexpr uint64_t kKeepaliveTimeout = 10 * kNsPerSec; // KEEPALIVE_TIMEOUT, lib.rs:70
constexpr uint64_t kRejectAfterTime = 180 * kNsPerSec; // REJECT_AFTER_TIME, lib.rs:67
} // namespace

namespace {
// Device half of the session table for rg_send_batch_dev / rg_recv_batch_dev: mirrors of the key
// rows, the receivers and a receiver-id -> recv-row table, refreshed before the next device call
// after a session change (once the device work that reads them has drained).
struct SendStage { // one device send in flight per stage; two stages alternate
    DevBuf d_desc, d_kidx, d_ctr;
    HostBuf h_kidx, h_ctr;
    hipEvent_t ev = nullptr; // the stage's seal has consumed its buffers
};
struct RecvStage { // the device receive between rg_recv_batch_dev and rg_recv_batch_dev_finish
    DevBuf d_rdesc, d_ctr, d_key, d_idx, d_udesc, d_uctr, d_ustatus;
    HostBuf h_status, h_ctr, h_key, h_fix, h_idx;
    hipEvent_t ev_meta = nullptr, ev_done = nullptr;
    bool pending = false;
    size_t n = 0;
    hipStream_t st = nullptr;
    uint8_t *buf = nullptr, *status = nullptr;
    size_t buf_len = 0;
};
hipError_t ensure_event(hipEvent_t &e) {
    return e ? hipSuccess : hipEventCreateWithFlags(&e, hipEventDisableTiming);
}
struct SessDev {
    SecretBuf keys; // send rows [0, cap), recv rows [cap, 2 cap)
    HostBuf h_keys; // their pinned staging copy (zeroed when freed)
    hipEvent_t ev_keys = nullptr; // the staging copy's upload is done
    DevBuf recv, rx;
    uint32_t rx_cap = 0;
    bool dirty = true;
    SendStage send[2];
    int send_next = 0;
    RecvStage rv;
};
} // namespace

struct rg_sessions {
    rg_ctx *ctx = nullptr;
    rg_group *group = nullptr; // host-frame batches on every context of the group (ctx = its first)
    uint32_t cap = 0;
    uint64_t now = 0; // Sessions' clock (state.now, advanced by turn: lib.rs:396-413), nanoseconds
    std::vector<Session> s;
    std::vector<uint8_t> keys;       // rows [0,cap): send keys, [cap,2cap): recv keys
    std::vector<uint32_t> receivers; // remote ids for send rows
    std::unordered_map<uint32_t, uint32_t> by_local;
    std::unordered_map<uint32_t, Peer> peers;
    SessDev dev;
};

namespace {

// The in-order tail of DecryptionKey::decrypt (prim.rs:414-437) and decrypt_packet
// (rustyguard-core/src/lib.rs:655-679) for packet i of session `slot`, whose GPU verdict
// `st` is RG_PKT_OK or RG_PKT_DECRYPT_ERR: would_accept comes first (Error::Rejected, also
// for a frame too short or with a bad tag), then the AEAD's verdict; an accepted packet
// advances the window (only authenticated counters do, RFC 6479 §3.4.3), may move the
// endpoint (whitepaper §6.5) and may ask for a keepalive.  *undo: the GPU left plaintext in
// a frame the reference would not have decrypted.
uint8_t replay_step(rg_sessions *s, uint32_t slot, uint64_t ctr, uint8_t st, const uint64_t *src, size_t i,
                    uint8_t *fl, bool *undo) {
    Session &x = s->s[slot];
    *undo = false;
    *fl = 0;
    if (!rg_antireplay_would_accept(&x.replay, ctr)) {
        *undo = st == RG_PKT_OK;
        return RG_PKT_REJECTED;
    }
    if (st != RG_PKT_OK) return st;
    rg_antireplay_mark_seen(&x.replay, ctr);
    uint8_t f = RG_RECV_AUTHENTICATED;
    if (x.sent + kKeepaliveTimeout < s->now && !x.keepalive_pending) {
        x.keepalive_pending = true;
        f |= RG_RECV_KEEPALIVE;
    }
    if (src) { // the peer's endpoint moves (the session's own without a peer)
        if (x.peer != RG_PEER_NONE) {
            Peer &p = s->peers[x.peer];
            p.endpoint = src[i];
            p.has_endpoint = true;
        } else {
            x.endpoint = src[i];
            x.has_endpoint = true;
        }
    }
    *fl = f;
    return RG_PKT_OK;
}

// every device batch of the table has finished with its tables (bounded waits)
int drain_device_work(rg_sessions *s) {
    SessDev &D = s->dev;
    const uint32_t ms = s->ctx->wait_ms;
    for (auto &g : D.send) RG_WAIT(g.ev, ms, "session tables in use");
    RG_WAIT(D.rv.ev_meta, ms, "session tables in use");
    RG_WAIT(D.rv.ev_done, ms, "session tables in use");
    RG_WAIT(D.ev_keys, ms, "session key upload");
    return RG_OK;
}

// refresh the device mirrors after session changes, on the call's stream st (the key rows are
// rewritten in place; a regrow wipes the old rows behind their last readers, SecretBuf).  The key rows
// go through a pinned staging copy whose upload is fenced by an event (round 5 synchronised the caller's
// stream here, waiting for all of the caller's queued work: ADVICE r5); the next refresh waits for that
// event before it rewrites the staging copy.  Inside a stream capture the refresh would be replayed by the
// graph from a staging copy that changes under it: refused.
int sync_tables(rg_sessions *s, hipStream_t st) {
    SessDev &D = s->dev;
    if (!D.dirty) return RG_OK;
    if (capturing(st))
        return set_err(RG_EDEVICE, "session tables changed since the last device call: refresh them (one device "
                                   "call) outside the stream capture");
    int rc = drain_device_work(s);
    if (rc) return rc;
    RG_HIP(ensure_event(D.ev_keys), "session key event");
    RG_HIP(D.keys.reserve(s->keys.size(), st), "alloc session keys");
    D.h_keys.secret = true;
    RG_HIP(D.h_keys.reserve(s->keys.size()), "alloc session key staging");
    memcpy(D.h_keys.p, s->keys.data(), s->keys.size());
    RG_HIP(hipMemcpyAsync(D.keys.p, D.h_keys.p, s->keys.size(), hipMemcpyHostToDevice, st), "H2D session keys");
    RG_HIP(hipEventRecord(D.ev_keys, st), "session key event");
    RG_HIP(D.recv.reserve((size_t)s->cap * 4), "alloc session receivers");
    RG_HIP(hipMemcpy(D.recv.p, s->receivers.data(), (size_t)s->cap * 4, hipMemcpyHostToDevice),
           "H2D session receivers");
    std::vector<uint32_t> ids, rows;
    for (uint32_t i = 0; i < s->cap; ++i)
        if (s->s[i].used) {
            ids.push_back(s->s[i].local_id);
            rows.push_back(s->cap + i); // the session's recv-key row
        }
    uint32_t rx_cap = 2;
    while (rx_cap < 2 * ids.size()) rx_cap <<= 1;
    std::vector<rg_rx_entry> t(rx_cap);
    rc = rg_rx_table_build(ids.data(), rows.data(), ids.size(), t.data(), rx_cap);
    if (rc) return rc;
    RG_HIP(D.rx.reserve((size_t)rx_cap * sizeof(rg_rx_entry)), "alloc rx table");
    RG_HIP(hipMemcpy(D.rx.p, t.data(), (size_t)rx_cap * sizeof(rg_rx_entry), hipMemcpyHostToDevice), "H2D rx table");
    D.rx_cap = rx_cap;
    D.dirty = false;
    return RG_OK;
}


} // namespace

extern "C" {

int rg_sessions_create(rg_ctx *ctx, uint32_t capacity, rg_sessions **out) {
    if (!ctx || !out || capacity == 0 || capacity > (1u << 24)) return set_err(RG_EINVAL, "sessions: bad args");
    rg_sessions *s = new (std::nothrow) rg_sessions();
    if (!s) return set_err(RG_ENOMEM, "alloc sessions");
    s->ctx = ctx;
    s->cap = capacity;
    s->s.resize(capacity);
    s->keys.assign((size_t)capacity * 64, 0);
    s->receivers.assign((size_t)capacity * 2, 0);
    *out = s;
    return RG_OK;
}

int rg_sessions_create_group(rg_group *g, uint32_t capacity, rg_sessions **out) {
    if (!g || g->ctx.empty()) return set_err(RG_EINVAL, "sessions: null group");
    int rc = rg_sessions_create(g->ctx[0], capacity, out);
    if (rc == RG_OK) (*out)->group = g;
    return rc;
}

void rg_sessions_destroy(rg_sessions *s) {
    if (!s) return;
    std::fill(s->keys.begin(), s->keys.end(), 0); // zeroize, as prim.rs:227-231 / lib.rs:216-228
    SessDev &D = s->dev;
    DeviceGuard dg_;
    (void)hipSetDevice(s->ctx->device);
    (void)drain_device_work(s);
    (void)D.keys.release(s->ctx->gen_stream); // zeroed behind its last readers, then freed
    (void)hipStreamSynchronize(s->ctx->gen_stream);
    D.h_keys.release();
    if (D.ev_keys) (void)hipEventDestroy(D.ev_keys);
    D.recv.release(); D.rx.release();
    for (auto &g : D.send) {
        g.d_desc.release(); g.d_kidx.release(); g.d_ctr.release(); g.h_kidx.release(); g.h_ctr.release();
        if (g.ev) (void)hipEventDestroy(g.ev);
    }
    RecvStage &R = D.rv;
    R.d_rdesc.release(); R.d_ctr.release(); R.d_key.release(); R.d_idx.release(); R.d_udesc.release();
    R.d_uctr.release(); R.d_ustatus.release(); R.h_status.release(); R.h_ctr.release(); R.h_key.release(); R.h_fix.release();
    R.h_idx.release();
    if (R.ev_meta) (void)hipEventDestroy(R.ev_meta);
    if (R.ev_done) (void)hipEventDestroy(R.ev_done);
    delete s;
}

int rg_sessions_insert(rg_sessions *s, uint32_t local_id, uint32_t remote_id, const uint8_t send_key[32],
                       const uint8_t recv_key[32]) {
    return rg_sessions_insert_peer(s, local_id, remote_id, send_key, recv_key, RG_PEER_NONE);
}

int rg_sessions_insert_peer(rg_sessions *s, uint32_t local_id, uint32_t remote_id, const uint8_t send_key[32],
                            const uint8_t recv_key[32], uint32_t peer) {
    if (!s || !send_key || !recv_key) return set_err(RG_EINVAL, "insert: bad args");
    if (s->dev.rv.pending) return set_err(RG_EINVAL, "insert: a device receive batch is pending");
    if (s->by_local.count(local_id)) return set_err(RG_EINVAL, "insert: local id in use");
    for (uint32_t i = 0; i < s->cap; ++i) {
        Session &x = s->s[i];
        if (x.used) continue;
        x = Session();
        x.used = true;
        x.local_id = local_id;
        x.remote_id = remote_id;
        x.started = x.sent = s->now; // handshake.rs:119-124, :215-216
        x.peer = peer;
        if (peer != RG_PEER_NONE) (void)s->peers[peer]; // the record exists from the peer's first session
        memcpy(&s->keys[(size_t)i * 32], send_key, 32);
        memcpy(&s->keys[((size_t)s->cap + i) * 32], recv_key, 32);
        s->receivers[i] = remote_id;
        s->by_local[local_id] = i;
        s->dev.dirty = true;
        return (int)i;
    }
    return set_err(RG_EFULL, "insert: table full");
}

int rg_sessions_remove(rg_sessions *s, uint32_t slot) {
    if (!s || slot >= s->cap || !s->s[slot].used) return set_err(RG_EINVAL, "remove: bad slot");
    if (s->dev.rv.pending) return set_err(RG_EINVAL, "remove: a device receive batch is pending");
    s->dev.dirty = true;
    s->by_local.erase(s->s[slot].local_id);
    s->s[slot] = Session();
    memset(&s->keys[(size_t)slot * 32], 0, 32);
    memset(&s->keys[((size_t)s->cap + slot) * 32], 0, 32);
    return RG_OK;
}

int rg_sessions_lookup(const rg_sessions *s, uint32_t local_id) {
    if (!s) return set_err(RG_EINVAL, "lookup: null");
    auto it = s->by_local.find(local_id);
    return it == s->by_local.end() ? RG_ENOTFOUND : (int)it->second;
}

uint64_t rg_sessions_send_counter(const rg_sessions *s, uint32_t slot) {
    if (!s || slot >= s->cap) return 0;
    return s->s[slot].send_ctr;
}

int rg_sessions_set_send_counter(rg_sessions *s, uint32_t slot, uint64_t counter) {
    if (!s || slot >= s->cap || !s->s[slot].used) return set_err(RG_EINVAL, "set_counter: bad slot");
    s->s[slot].send_ctr = counter;
    return RG_OK;
}

rg_antireplay *rg_sessions_replay(rg_sessions *s, uint32_t slot) {
    if (!s || slot >= s->cap) return nullptr;
    return &s->s[slot].replay;
}

void rg_sessions_set_time(rg_sessions *s, uint64_t now_ns) {
    if (s) s->now = now_ns;
}

int rg_peer_endpoint(const rg_sessions *s, uint32_t peer, uint64_t *src_out) {
    if (!s || !src_out || peer == RG_PEER_NONE) return set_err(RG_EINVAL, "peer_endpoint: bad args");
    auto it = s->peers.find(peer);
    if (it == s->peers.end() || !it->second.has_endpoint) return RG_ENOTFOUND;
    *src_out = it->second.endpoint;
    return RG_OK;
}

int rg_sessions_endpoint(const rg_sessions *s, uint32_t slot, uint64_t *src_out) {
    if (!s || slot >= s->cap || !s->s[slot].used || !src_out) return set_err(RG_EINVAL, "endpoint: bad slot");
    const Session &x = s->s[slot];
    if (x.peer != RG_PEER_NONE) return rg_peer_endpoint(s, x.peer, src_out);
    if (!x.has_endpoint) return RG_ENOTFOUND;
    *src_out = x.endpoint;
    return RG_OK;
}

int rg_sessions_keepalive_due(rg_sessions *s, uint32_t slot) {
    if (!s || slot >= s->cap || !s->s[slot].used) return set_err(RG_EINVAL, "keepalive: bad slot");
    Session &x = s->s[slot];
    x.keepalive_pending = false;                     // time.rs:118
    return x.sent + kKeepaliveTimeout < s->now ? 1 : 0; // should_keepalive, lib.rs:201-203
}

int rg_sessions_keepalive(rg_sessions *s, uint32_t slot, uint64_t *dst_out) {
    if (!dst_out) return set_err(RG_EINVAL, "keepalive: null dst");
    const int due = rg_sessions_keepalive_due(s, slot);
    if (due <= 0) return due;
    const int rc = rg_sessions_endpoint(s, slot, dst_out); // peer.endpoint, time.rs:135
    return rc == RG_OK ? 1 : rc;
}

int rg_send_batch(rg_sessions *s, const uint32_t *slots, const rg_pkt_desc *desc, size_t n, uint8_t *buf,
                  size_t buf_len, uint8_t *status, uint8_t *rekey_out) {
    if (!s || !slots || !desc || !buf || !status) return fail_closed(set_err(RG_EINVAL, "send_batch: bad args"), status, n);
    if (n == 0) return RG_OK;
    std::vector<rg_pkt_desc> d(desc, desc + n);
    std::vector<uint64_t> ctr(n, 0);
    std::vector<uint8_t> host_status(n, RG_PKT_OK);
    for (size_t i = 0; i < n; ++i) {
        if (rekey_out) rekey_out[i] = 0;
        const uint32_t slot = slots[i];
        if (slot >= s->cap || !s->s[slot].used) {
            host_status[i] = RG_PKT_REJECTED; // no transport session: caller must handshake
        } else if (d[i].len % 16 != 0) {
            host_status[i] = RG_PKT_INVALID; // force_encrypt's padding assert, lib.rs:273-277
        } else if (s->s[slot].send_ctr >= RG_REJECT_AFTER_MESSAGES ||
                   s->s[slot].started + kRejectAfterTime < s->now) {
            host_status[i] = RG_PKT_REJECTED; // should_reject / should_expire, lib.rs:204-209
        }
        if (host_status[i] != RG_PKT_OK) {
            d[i].key_idx = RG_KEY_SKIP;
            continue;
        }
        Session &x = s->s[slot];
        ctr[i] = x.send_ctr++; // EncryptionKey::encrypt, prim.rs:387-388
        x.sent = s->now;        // force_encrypt, lib.rs:285
        d[i].key_idx = slot;
        if (rekey_out && x.send_ctr >= RG_REKEY_AFTER_MESSAGES) rekey_out[i] = 1; // lib.rs:564-570
    }
    int rc = s->group ? rg_seal_batch_host_multi(s->group, s->keys.data(), s->receivers.data(), s->cap, d.data(),
                                                 ctr.data(), n, buf, buf_len, status)
                      : rg_seal_batch_host(s->ctx, s->keys.data(), s->receivers.data(), s->cap, d.data(), ctr.data(),
                                           n, buf, buf_len, status);
    if (rc) return rc;
    for (size_t i = 0; i < n; ++i)
        if (host_status[i] != RG_PKT_OK) status[i] = host_status[i];
    return RG_OK;
}

int rg_recv_batch(rg_sessions *s, const rg_pkt_desc *desc, size_t n, uint8_t *buf, size_t buf_len,
                  uint8_t *status, uint32_t *slots_out) {
    return rg_recv_batch_ex(s, desc, n, buf, buf_len, nullptr, status, slots_out, nullptr);
}

int rg_recv_batch_ex(rg_sessions *s, const rg_pkt_desc *desc, size_t n, uint8_t *buf, size_t buf_len,
                     const uint64_t *src, uint8_t *status, uint32_t *slots_out, uint8_t *flags_out) {
    if (!s || !desc || !buf || !status) return fail_closed(set_err(RG_EINVAL, "recv_batch: bad args"), status, n);
    if (n == 0) return RG_OK;
    std::vector<rg_pkt_desc> d(desc, desc + n);
    std::vector<uint8_t> host_status(n, 0xFF);
    std::vector<uint32_t> slot_of(n, 0xFFFFFFFFu);
    std::vector<uint64_t> ctr(n, 0);
    for (size_t i = 0; i < n; ++i) {
        const uint64_t off = d[i].offset;
        const uint32_t w = d[i].len;
        uint8_t st = 0xFF;
        if (off > buf_len || buf_len - off < w) st = RG_PKT_INVALID;
        else if (((uintptr_t)(buf + off) & 15) != 0) st = RG_PKT_UNALIGNED; // lib.rs:613-615
        else if (w < 4) st = RG_PKT_INVALID;
        else {
            uint32_t type, recv;
            memcpy(&type, buf + off, 4);
            if (type != 4u) st = type - 1u < 3u ? RG_PKT_NOT_DATA : RG_PKT_INVALID; // 1-3: control plane; else lib.rs:627
            else if (w % 16 != 0 || w < 16) st = RG_PKT_INVALID; // message_mut_from
            else {
                memcpy(&recv, buf + off + 4, 4);
                memcpy(&ctr[i], buf + off + 8, 8);
                auto it = s->by_local.find(recv);
                if (it == s->by_local.end()) st = RG_PKT_REJECTED; // lib.rs:646-650
                else {
                    slot_of[i] = it->second;
                    // replay pre-filter with the pre-batch window: a counter rejected now is
                    // rejected by any later window state too (the window only advances)
                    if (!rg_antireplay_would_accept(&s->s[it->second].replay, ctr[i])) st = RG_PKT_REJECTED;
                    else if (w < 32) st = RG_PKT_DECRYPT_ERR; // prim.rs:427-429
                }
            }
        }
        host_status[i] = st;
        d[i].key_idx = st == 0xFF ? s->cap + slot_of[i] : RG_KEY_SKIP;
    }
    int rc = s->group ? rg_open_batch_host_multi(s->group, s->keys.data(), 2 * s->cap, d.data(), n, buf, buf_len,
                                                 status, nullptr)
                      : rg_open_batch_host(s->ctx, s->keys.data(), 2 * s->cap, d.data(), n, buf, buf_len, status,
                                           nullptr);
    if (rc) { // statuses pending (the open call's fail-closed contract); no packet is flagged either
        if (flags_out) memset(flags_out, 0, n);
        return rc;
    }
    // in-order post-pass (RFC 6479 §3.4.3: only authenticated counters advance the window)
    std::vector<rg_pkt_desc> undo;
    std::vector<uint64_t> undo_ctr;
    if (flags_out) memset(flags_out, 0, n);
    for (size_t i = 0; i < n; ++i) {
        uint8_t st = host_status[i] != 0xFF ? host_status[i] : status[i];
        // a frame that reached the session (GPU verdict, or too short for a tag) takes the
        // in-order window check first: a second copy of a counter accepted earlier in this
        // batch, or one the window has moved past since, is Rejected before decrypting
        // (prim.rs:420-423), and a GPU plaintext there is put back to ciphertext
        if (slot_of[i] != 0xFFFFFFFFu && (st == RG_PKT_OK || st == RG_PKT_DECRYPT_ERR)) {
            uint8_t fl;
            bool back;
            st = replay_step(s, slot_of[i], ctr[i], st, src, i, &fl, &back);
            if (flags_out) flags_out[i] = fl;
            if (back) {
                undo.push_back(rg_pkt_desc{d[i].offset, d[i].len - 32, d[i].key_idx});
                undo_ctr.push_back(ctr[i]);
            }
        }
        status[i] = st;
        if (slots_out) slots_out[i] = slot_of[i];
    }
    if (!undo.empty()) {
        // Re-sealing the plaintext under the same key and nonce reproduces the ciphertext and,
        // since the tag is the MAC of that ciphertext, the frame's own (verified) tag; without
        // receivers the header is not rewritten.  The frame is byte-for-byte what arrived.
        std::vector<uint8_t> st2(undo.size());
        rc = s->group ? rg_seal_batch_host_multi(s->group, s->keys.data(), nullptr, 2 * s->cap, undo.data(),
                                                 undo_ctr.data(), undo.size(), buf, buf_len, st2.data())
                      : rg_seal_batch_host(s->ctx, s->keys.data(), nullptr, 2 * s->cap, undo.data(), undo_ctr.data(),
                                           undo.size(), buf, buf_len, st2.data());
        for (uint8_t x : st2)
            if (rc == RG_OK && x != RG_PKT_OK) rc = set_err(RG_EDEVICE, "recv_batch: restoring a replayed frame failed");
        if (rc) { // a failed batch hands nothing up (include/rg_aead.h)
            if (flags_out) memset(flags_out, 0, n);
            return fail_closed(rc, status, n);
        }
    }
    return RG_OK;
}

int rg_send_batch_dev(rg_sessions *s, const uint32_t *slots, const rg_pkt_desc *desc, size_t n, uint8_t *buf,
                      size_t buf_len, uint8_t *status, uint8_t *rekey_out, void *stream) {
    if (!s || !slots || !desc || !buf || !status) return set_err(RG_EINVAL, "send_batch_dev: bad args (status is required)");
    if (s->group) return set_err(RG_EINVAL, "send_batch_dev: a group's table takes host frames (rg_send_batch)");
    if (n > 0xFFFFFFFFull) return set_err(RG_EINVAL, "send_batch_dev: too many packets");
    if (n == 0) return RG_OK;
    DeviceGuard dg_;
    int rc = check_ctx(s->ctx);
    if (rc) return rc;
    rc = claim_stream(s->ctx, static_cast<hipStream_t>(stream)); // before any counter is taken
    if (rc) return rc;
    rc = sync_tables(s, static_cast<hipStream_t>(stream));
    if (rc) return rc;
    SessDev &D = s->dev;
    SendStage &g = D.send[D.send_next];
    RG_HIP(ensure_event(g.ev), "send event");
    RG_WAIT(g.ev, s->ctx->wait_ms, "send staging"); // the stage's previous batch has been sealed
    D.send_next ^= 1;
    RG_HIP(g.h_kidx.reserve(n * 4), "alloc send staging");
    RG_HIP(g.h_ctr.reserve(n * 8), "alloc send staging");
    RG_HIP(g.d_kidx.reserve(n * 4), "alloc send key rows");
    RG_HIP(g.d_ctr.reserve(n * 8), "alloc send counters");
    RG_HIP(g.d_desc.reserve(n * sizeof(rg_pkt_desc)), "alloc send descriptors");
    uint32_t *kx = static_cast<uint32_t *>(g.h_kidx.p);
    uint64_t *cx = static_cast<uint64_t *>(g.h_ctr.p);
    // rg_send_batch's session checks, in array order; the lengths live on the device, so a
    // frame with P % 16 != 0 takes its counter and the kernel reports it RG_PKT_INVALID
    for (size_t i = 0; i < n; ++i) {
        if (rekey_out) rekey_out[i] = 0;
        const uint32_t slot = slots[i];
        kx[i] = RG_KEY_SKIP; // the kernel reports RG_PKT_REJECTED
        cx[i] = 0;
        if (slot >= s->cap || !s->s[slot].used) continue;
        Session &x = s->s[slot];
        if (x.send_ctr >= RG_REJECT_AFTER_MESSAGES || x.started + kRejectAfterTime < s->now) continue;
        cx[i] = x.send_ctr++; // EncryptionKey::encrypt, prim.rs:387-388
        x.sent = s->now;      // force_encrypt, lib.rs:285
        kx[i] = slot;
        if (rekey_out && x.send_ctr >= RG_REKEY_AFTER_MESSAGES) rekey_out[i] = 1; // lib.rs:564-570
    }
    hipStream_t st = static_cast<hipStream_t>(stream);
    RG_HIP(hipMemcpyAsync(g.d_kidx.p, kx, n * 4, hipMemcpyHostToDevice, st), "H2D send key rows");
    RG_HIP(hipMemcpyAsync(g.d_ctr.p, cx, n * 8, hipMemcpyHostToDevice, st), "H2D send counters");
    auto *bd = static_cast<rg_pkt_desc *>(g.d_desc.p);
    RG_HIP(rg::launch_bind_keys(desc, static_cast<const uint32_t *>(g.d_kidx.p), (uint32_t)n, bd, st), "bind launch");
    rc = rg_seal_batch_dev(s->ctx, static_cast<const uint8_t *>(D.keys.p), static_cast<const uint32_t *>(D.recv.p),
                           s->cap, bd, static_cast<const uint64_t *>(g.d_ctr.p), n, buf, buf_len, status, stream);
    if (rc) return rc;
    RG_HIP(D.keys.use(st), "session keys event");
    RG_HIP(hipEventRecord(g.ev, st), "send event record");
    return RG_OK;
}

int rg_recv_batch_dev(rg_sessions *s, const rg_pkt_desc *desc, size_t n, uint8_t *buf, size_t buf_len,
                      uint8_t *status, void *stream) {
    if (!s || !desc || !buf || !status) return set_err(RG_EINVAL, "recv_batch_dev: bad args");
    if (s->group) return set_err(RG_EINVAL, "recv_batch_dev: a group's table takes host frames (rg_recv_batch_ex)");
    if (n > 0xFFFFFFFFull) return set_err(RG_EINVAL, "recv_batch_dev: too many packets");
    RecvStage &R = s->dev.rv;
    if (R.pending) return set_err(RG_EINVAL, "recv_batch_dev: finish the pending batch first");
    DeviceGuard dg_;
    int rc = check_ctx(s->ctx);
    if (rc) return rc;
    rc = claim_stream(s->ctx, static_cast<hipStream_t>(stream));
    if (rc) return rc;
    rc = sync_tables(s, static_cast<hipStream_t>(stream));
    if (rc) return rc;
    SessDev &D = s->dev;
    RG_HIP(ensure_event(R.ev_meta), "recv event");
    RG_HIP(ensure_event(R.ev_done), "recv event");
    RG_WAIT(R.ev_done, s->ctx->wait_ms, "recv staging"); // the previous batch's fix-ups are done
    hipStream_t st = static_cast<hipStream_t>(stream);
    // The batch becomes pending only once every buffer is reserved and every step is enqueued: a
    // failure leaves no pending batch (finish then reports none), and work already enqueued is
    // fenced by ev_done, which the next call waits for before it reuses the staging buffers.
    if (n > 0) {
        RG_HIP(R.d_rdesc.reserve(n * sizeof(rg_pkt_desc)), "alloc recv descriptors");
        RG_HIP(R.d_ctr.reserve(n * 8), "alloc recv counters");
        RG_HIP(R.d_key.reserve(n * 4), "alloc recv key rows");
        RG_HIP(R.h_status.reserve(n), "alloc recv staging");
        RG_HIP(R.h_ctr.reserve(n * 8), "alloc recv staging");
        RG_HIP(R.h_key.reserve(n * 4), "alloc recv staging");
        auto fenced = [&](int code) {
            (void)hipEventRecord(R.ev_done, st);
            return code;
        };
        auto *rd = static_cast<rg_pkt_desc *>(R.d_rdesc.p);
        hipError_t e = rg::launch_rx_resolve(desc, (uint32_t)n, buf, buf_len, static_cast<const rg_rx_entry *>(D.rx.p),
                                             D.rx_cap, rd, static_cast<uint32_t *>(R.d_key.p), st);
        if (e != hipSuccess) return fenced(set_err(RG_EDEVICE, "rx resolve launch", e));
        rc = rg_open_batch_dev(s->ctx, static_cast<const uint8_t *>(D.keys.p), 2 * s->cap, rd, n, buf, buf_len, status,
                               static_cast<uint64_t *>(R.d_ctr.p), stream);
        if (rc) return fenced(rc);
        e = D.keys.use(st);
        if (e == hipSuccess) e = hipMemcpyAsync(R.h_status.p, status, n, hipMemcpyDeviceToHost, st);
        if (e == hipSuccess) e = hipMemcpyAsync(R.h_ctr.p, R.d_ctr.p, n * 8, hipMemcpyDeviceToHost, st);
        if (e == hipSuccess) e = hipMemcpyAsync(R.h_key.p, R.d_key.p, n * 4, hipMemcpyDeviceToHost, st);
        if (e == hipSuccess) e = hipEventRecord(R.ev_meta, st);
        if (e != hipSuccess) return fenced(set_err(RG_EDEVICE, "recv metadata copies", e));
    }
    R.n = n;
    R.st = st;
    R.buf = buf;
    R.buf_len = buf_len;
    R.status = status;
    R.pending = true;
    return RG_OK;
}

int rg_recv_batch_dev_finish(rg_sessions *s, const uint64_t *src, uint8_t *status_out, uint32_t *slots_out,
                             uint8_t *flags_out) {
    if (!s) return set_err(RG_EINVAL, "recv_batch_dev_finish: null");
    RecvStage &R = s->dev.rv;
    if (!R.pending) return set_err(RG_EINVAL, "recv_batch_dev_finish: no pending batch");
    R.pending = false;
    const size_t n = R.n;
    if (n == 0) return RG_OK;
    DeviceGuard dg_;
    int rc = check_ctx(s->ctx);
    if (rc) return rc;
    RG_WAIT(R.ev_meta, s->ctx->wait_ms, "recv metadata");
    RG_HIP(R.h_fix.reserve(n), "alloc recv staging");
    RG_HIP(R.h_idx.reserve(n * 4), "alloc recv staging");
    const uint8_t *gs = static_cast<const uint8_t *>(R.h_status.p);
    const uint64_t *cx = static_cast<const uint64_t *>(R.h_ctr.p);
    const uint32_t *kx = static_cast<const uint32_t *>(R.h_key.p);
    uint8_t *fx = static_cast<uint8_t *>(R.h_fix.p);
    uint32_t *ix = static_cast<uint32_t *>(R.h_idx.p);
    size_t m = 0, pending = 0;
    bool changed = false;
    for (size_t i = 0; i < n; ++i) {
        uint8_t st = gs[i], fl = 0;
        pending += st == RG_PKT_PENDING; // never reached by the kernel: no replay step, no side effect
        const uint32_t k = kx[i];
        const uint32_t slot = k != RG_KEY_SKIP && k >= s->cap && k < 2 * s->cap ? k - s->cap : 0xFFFFFFFFu;
        if (slot != 0xFFFFFFFFu && (st == RG_PKT_OK || st == RG_PKT_DECRYPT_ERR)) {
            bool back;
            const uint8_t st2 = replay_step(s, slot, cx[i], st, src, i, &fl, &back);
            if (back) ix[m++] = (uint32_t)i;
            changed |= st2 != st;
            st = st2;
        }
        fx[i] = st;
        if (status_out) status_out[i] = st;
        if (slots_out) slots_out[i] = slot;
        if (flags_out) flags_out[i] = fl;
    }
    hipStream_t st = R.st;
    if (changed) RG_HIP(hipMemcpyAsync(R.status, fx, n, hipMemcpyHostToDevice, st), "H2D recv status");
    if (m) {
        // re-seal under the same key and nonce: ciphertext and tag come back byte for byte
        RG_HIP(R.d_idx.reserve(m * 4), "alloc undo list");
        RG_HIP(R.d_udesc.reserve(m * sizeof(rg_pkt_desc)), "alloc undo list");
        RG_HIP(R.d_uctr.reserve(m * 8), "alloc undo list");
        RG_HIP(hipMemcpyAsync(R.d_idx.p, ix, m * 4, hipMemcpyHostToDevice, st), "H2D undo list");
        auto *ud = static_cast<rg_pkt_desc *>(R.d_udesc.p);
        RG_HIP(rg::launch_undo_gather(static_cast<const rg_pkt_desc *>(R.d_rdesc.p),
                                      static_cast<const uint64_t *>(R.d_ctr.p), static_cast<const uint32_t *>(R.d_idx.p),
                                      (uint32_t)m, ud, static_cast<uint64_t *>(R.d_uctr.p), st),
               "undo gather launch");
        RG_HIP(R.d_ustatus.reserve(m), "alloc undo list");
        rc = rg_seal_batch_dev(s->ctx, static_cast<const uint8_t *>(s->dev.keys.p), nullptr, 2 * s->cap, ud,
                               static_cast<const uint64_t *>(R.d_uctr.p), m, R.buf, R.buf_len,
                               static_cast<uint8_t *>(R.d_ustatus.p), st);
        if (rc) return rc;
        RG_HIP(s->dev.keys.use(st), "session keys event");
    }
    RG_HIP(hipEventRecord(R.ev_done, st), "recv event record");
    if (pending) {
        char what[128];
        snprintf(what, sizeof what, "recv_batch_dev_finish: %zu of %zu packets were never finished (RG_PKT_PENDING)",
                 pending, n);
        return set_err(RG_EDEVICE, what);
    }
    return RG_OK;
}

} // extern "C"
