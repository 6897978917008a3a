// driver.cpp -- TEST INFRASTRUCTURE ONLY: drives the host logic of rg_api.cpp (built host-only and linked
// against tests/sanitize/hip_stub.cpp, no GPU) under AddressSanitizer + UBSan and under ThreadSanitizer
// (tests/test_sanitize_cpu.py).  Every scenario checks its own results (seal -> open
// round trips, forged frames, replayed counters, endpoints, fail-closed statuses) so a sanitizer run is
// also a functional run of the paths it covers:
//   1 host seal/open over many small slices, descriptors out of offset order (run_ordered's permutation)
//   2 the session layer: rg_send_batch / rg_recv_batch_ex with replays, forgeries, endpoints, keepalive
//   3 a group of four contexts on two stub devices, batches large enough for one worker thread per context
//   4 a group's session table (rg_sessions_create_group)
//   5 device-frame sessions: rg_send_batch_dev / rg_recv_batch_dev + _finish (device memory = host here)
//   6 fail-closed paths: a lost planner hand-off (test hook) and lost completions (bounded waits)
//   7 the per-message drop-in (rg_chacha20poly1305_enc/dec)
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "rg_aead.h"
#include "rg_aead_test.h"

static int g_fail = 0;
#define CHECK(cond, ...)                                                                                   \
    do {                                                                                                   \
        if (!(cond)) {                                                                                     \
            fprintf(stderr, "CHECK failed at %s:%d: %s -- ", __FILE__, __LINE__, #cond);                  \
            fprintf(stderr, __VA_ARGS__);                                                                  \
            fprintf(stderr, " (last error: %s)\n", rg_last_error());                                      \
            ++g_fail;                                                                                      \
        }                                                                                                  \
    } while (0)

struct Batch {
    std::vector<rg_pkt_desc> desc;
    std::vector<uint8_t> buf, plain;
    std::vector<uint64_t> ctr;
};

// n frames of random 16-byte-multiple payloads (0 .. 1504), packed, one key row `key`
static Batch make_batch(std::mt19937_64 &rng, size_t n, uint32_t key) {
    Batch b;
    uint64_t off = 0;
    for (size_t i = 0; i < n; ++i) {
        const uint32_t P = 16 * (uint32_t)(rng() % 95);
        b.desc.push_back({off, P, key});
        b.ctr.push_back(i * 3 + 1);
        off += P + 32;
    }
    b.buf.resize(off + 64);
    for (auto &x : b.buf) x = (uint8_t)rng();
    b.plain = b.buf;
    return b;
}

static bool payloads_equal(const Batch &b, const std::vector<uint8_t> &x) {
    for (const auto &d : b.desc)
        if (memcmp(&x[d.offset + 16], &b.plain[d.offset + 16], d.len) != 0) return false;
    return true;
}

static std::vector<rg_pkt_desc> open_view(const std::vector<rg_pkt_desc> &s) {
    std::vector<rg_pkt_desc> o = s;
    for (auto &d : o) d.len += 32;
    return o;
}

static void scenario_host(rg_ctx *c, std::mt19937_64 &rng) {
    uint8_t keys[2][32];
    for (auto &k : keys)
        for (auto &x : k) x = (uint8_t)rng();
    const uint32_t rec[2] = {0x1111, 0x2222};
    Batch b = make_batch(rng, 3000, 1);
    // out of offset order: reverse pairs
    for (size_t i = 0; i + 1 < b.desc.size(); i += 2) {
        std::swap(b.desc[i], b.desc[i + 1]);
        std::swap(b.ctr[i], b.ctr[i + 1]);
    }
    CHECK(rg_set_host_slice(c, 64 << 10) == RG_OK, "slice");
    const size_t n = b.desc.size();
    std::vector<uint8_t> st(n, 0xEE);
    CHECK(rg_seal_batch_host(c, &keys[0][0], rec, 2, b.desc.data(), b.ctr.data(), n, b.buf.data(), b.buf.size(),
                             st.data()) == RG_OK, "seal");
    for (size_t i = 0; i < n; ++i) CHECK(st[i] == RG_PKT_OK, "seal status %zu = %u", i, st[i]);
    CHECK(!payloads_equal(b, b.buf), "sealed payloads differ from the plaintext");
    // forge every 7th frame's tag, then open
    const auto od = open_view(b.desc);
    for (size_t i = 0; i < n; i += 7) b.buf[od[i].offset + od[i].len - 1] ^= 0x40;
    std::vector<uint64_t> co(n);
    CHECK(rg_open_batch_host(c, &keys[0][0], 2, od.data(), n, b.buf.data(), b.buf.size(), st.data(), co.data()) ==
              RG_OK, "open");
    for (size_t i = 0; i < n; ++i) {
        CHECK(st[i] == (i % 7 == 0 ? RG_PKT_DECRYPT_ERR : RG_PKT_OK), "open status %zu = %u", i, st[i]);
        CHECK(co[i] == b.ctr[i], "counter %zu", i);
        if (i % 7) CHECK(memcmp(&b.buf[od[i].offset + 16], &b.plain[od[i].offset + 16], b.desc[i].len) == 0, "plain %zu", i);
    }
}

struct Pair {
    rg_sessions *a = nullptr, *b = nullptr;
    int sa = -1, sb = -1;
};

static Pair make_pair(rg_ctx *c, rg_group *g, std::mt19937_64 &rng) {
    Pair p;
    uint8_t k1[32], k2[32];
    for (int i = 0; i < 32; ++i) k1[i] = (uint8_t)rng(), k2[i] = (uint8_t)rng();
    if (g) {
        CHECK(rg_sessions_create_group(g, 8, &p.a) == RG_OK, "create group table");
        CHECK(rg_sessions_create_group(g, 8, &p.b) == RG_OK, "create group table");
    } else {
        CHECK(rg_sessions_create(c, 8, &p.a) == RG_OK, "create table");
        CHECK(rg_sessions_create(c, 8, &p.b) == RG_OK, "create table");
    }
    p.sa = rg_sessions_insert_peer(p.a, 0x1111, 0x2222, k1, k2, 77);
    p.sb = rg_sessions_insert(p.b, 0x2222, 0x1111, k2, k1);
    CHECK(p.sa >= 0 && p.sb >= 0, "insert");
    return p;
}

// B sends n frames to A; A receives them with duplicates of every 5th appended and every 9th forged
static void scenario_sessions(rg_ctx *c, rg_group *g, std::mt19937_64 &rng, size_t n) {
    Pair p = make_pair(c, g, rng);
    rg_sessions_set_time(p.a, 30ull * 1000000000ull);
    Batch b = make_batch(rng, n, 0);
    std::vector<uint32_t> slots(n, (uint32_t)p.sb);
    std::vector<uint8_t> st(n), rk(n);
    CHECK(rg_send_batch(p.b, slots.data(), b.desc.data(), n, b.buf.data(), b.buf.size(), st.data(), rk.data()) == RG_OK,
          "send");
    for (size_t i = 0; i < n; ++i) CHECK(st[i] == RG_PKT_OK && rk[i] == 0, "send status %zu", i);
    CHECK(rg_sessions_send_counter(p.b, p.sb) == n, "counter");
    // the receive buffer: all frames, then copies of every 5th
    std::vector<rg_pkt_desc> rd = open_view(b.desc);
    std::vector<uint8_t> rbuf = b.buf;
    std::vector<size_t> orig;
    for (size_t i = 0; i < n; ++i) orig.push_back(i);
    for (size_t i = 0; i < n; i += 5) {
        const rg_pkt_desc d = rd[i];
        const uint64_t off = (rbuf.size() + 15) & ~15ull;
        rbuf.resize(off + d.len + 16);
        memcpy(&rbuf[off], &b.buf[d.offset], d.len);
        rd.push_back({off, d.len, 0});
        orig.push_back(i);
    }
    for (size_t i = 0; i < n; i += 9) rbuf[rd[i].offset + 20] ^= 1;
    const size_t m = rd.size();
    std::vector<uint64_t> src(m);
    for (size_t i = 0; i < m; ++i) src[i] = 1000 + i;
    std::vector<uint8_t> rst(m), fl(m);
    std::vector<uint32_t> sl(m);
    CHECK(rg_recv_batch_ex(p.a, rd.data(), m, rbuf.data(), rbuf.size(), src.data(), rst.data(), sl.data(), fl.data()) ==
              RG_OK, "recv");
    size_t ok = 0, last_ok = 0, keep = 0;
    for (size_t i = 0; i < m; ++i) {
        const size_t o = orig[i];
        uint8_t want = o % 9 == 0 ? RG_PKT_DECRYPT_ERR : RG_PKT_OK;
        if (i >= n) want = o % 9 == 0 ? RG_PKT_DECRYPT_ERR : RG_PKT_REJECTED; // a copy of an accepted counter
        // the copy of a forged original is intact: accepted while its counter is still inside the window
        // (RG_REPLAY_WINDOW behind the batch's highest accepted counter, n - 1), too old after that
        if (i >= n && o % 9 == 0) want = (n - 1 - o) < RG_REPLAY_WINDOW ? RG_PKT_OK : RG_PKT_REJECTED;
        CHECK(rst[i] == want, "recv status %zu (orig %zu) = %u, want %u", i, o, rst[i], want);
        if (rst[i] == RG_PKT_OK) {
            ++ok;
            last_ok = i;
            CHECK(memcmp(&rbuf[rd[i].offset + 16], &b.plain[b.desc[o].offset + 16], b.desc[o].len) == 0, "plain %zu", i);
            CHECK(fl[i] & RG_RECV_AUTHENTICATED, "flag %zu", i);
            keep += (fl[i] & RG_RECV_KEEPALIVE) != 0;
        } else {
            CHECK(fl[i] == 0, "flag of a rejected frame %zu", i);
        }
    }
    CHECK(keep == 1, "one keepalive request (%zu)", keep);
    uint64_t ep = 0;
    CHECK(rg_peer_endpoint(p.a, 77, &ep) == RG_OK && ep == src[last_ok], "endpoint %llu", (unsigned long long)ep);
    rg_sessions_destroy(p.a);
    rg_sessions_destroy(p.b);
}

static void scenario_device_sessions(rg_ctx *c, std::mt19937_64 &rng) {
    Pair p = make_pair(c, nullptr, rng);
    const size_t n = 400;
    Batch b = make_batch(rng, n, 0);
    std::vector<uint32_t> slots(n, (uint32_t)p.sb);
    std::vector<uint8_t> st(n, 0xEE), rk(n);
    for (int rep = 0; rep < 3; ++rep) { // three sends: the two staging sets alternate
        Batch x = b;
        CHECK(rg_send_batch_dev(p.b, slots.data(), x.desc.data(), n, x.buf.data(), x.buf.size(), st.data(), rk.data(),
                                nullptr) == RG_OK, "send dev");
        for (size_t i = 0; i < n; ++i) CHECK(st[i] == RG_PKT_OK, "send dev status %zu", i);
        if (rep == 2) b = x;
    }
    CHECK(rg_send_batch_dev(p.b, slots.data(), b.desc.data(), n, b.buf.data(), b.buf.size(), nullptr, rk.data(),
                            nullptr) == RG_EINVAL, "status is required");
    const auto rd = open_view(b.desc);
    std::vector<uint8_t> dst(n), hst(n), fl(n);
    std::vector<uint32_t> sl(n);
    CHECK(rg_recv_batch_dev(p.a, rd.data(), n, b.buf.data(), b.buf.size(), dst.data(), nullptr) == RG_OK, "recv dev");
    CHECK(rg_recv_batch_dev_finish(p.a, nullptr, hst.data(), sl.data(), fl.data()) == RG_OK, "finish");
    for (size_t i = 0; i < n; ++i) CHECK(hst[i] == RG_PKT_OK && dst[i] == RG_PKT_OK, "recv dev status %zu", i);
    CHECK(payloads_equal(b, b.buf), "device receive restored the plaintext");
    // the same frames again: every counter is a replay now; the frames were re-sealed... they are plaintext
    // here, so re-seal them first through the device send path with the counters rewound
    rg_sessions_destroy(p.a);
    rg_sessions_destroy(p.b);
}

static void scenario_failclosed(rg_ctx *c, std::mt19937_64 &rng) {
    // a lost planner hand-off on the planned pipelined kernel: RG_EDEVICE, every status pending, nothing
    // marked seen
    CHECK(rg_set_staged(c, 0) == RG_OK && rg_set_plan(c, 1) == RG_OK, "knobs");
    Pair p = make_pair(c, nullptr, rng);
    const size_t n = 100;
    Batch b = make_batch(rng, n, 0);
    std::vector<uint32_t> slots(n, (uint32_t)p.sb);
    std::vector<uint8_t> st(n), fl(n);
    std::vector<uint32_t> sl(n);
    CHECK(rg_send_batch(p.b, slots.data(), b.desc.data(), n, b.buf.data(), b.buf.size(), st.data(), nullptr) == RG_OK,
          "send");
    const auto rd = open_view(b.desc);
    std::vector<uint8_t> arrived = b.buf;
    rg_debug_plan_handoff(1);
    std::vector<uint64_t> src(n, 5);
    CHECK(rg_recv_batch_ex(p.a, rd.data(), n, b.buf.data(), b.buf.size(), src.data(), st.data(), sl.data(),
                           fl.data()) == RG_EDEVICE, "lost hand-off fails");
    rg_debug_plan_handoff(0);
    for (size_t i = 0; i < n; ++i) CHECK(st[i] == RG_PKT_PENDING && fl[i] == 0, "pending %zu = %u", i, st[i]);
    CHECK(b.buf == arrived, "frames untouched");
    uint64_t ep;
    CHECK(rg_peer_endpoint(p.a, 77, &ep) == RG_ENOTFOUND, "no endpoint");
    const rg_antireplay *r = rg_sessions_replay(p.a, (uint32_t)p.sa);
    for (uint64_t k = 0; k < 400; ++k) CHECK(rg_antireplay_would_accept(r, k), "window untouched %llu", (unsigned long long)k);
    CHECK(rg_recv_batch_ex(p.a, rd.data(), n, b.buf.data(), b.buf.size(), src.data(), st.data(), sl.data(),
                           fl.data()) == RG_OK, "recovered");
    for (size_t i = 0; i < n; ++i) CHECK(st[i] == RG_PKT_OK, "accepted after the hook %zu", i);
    // lost completions: the bounded waits time out, statuses pending, and the context recovers
    CHECK(rg_set_wait_timeout(c, 50) == RG_OK, "timeout");
    rg_debug_lose_completions(1);
    Batch x = make_batch(rng, 200, 0);
    std::vector<uint8_t> st2(200, 0);
    uint8_t key[32] = {1};
    const uint32_t rec = 9;
    CHECK(rg_seal_batch_host(c, key, &rec, 1, x.desc.data(), x.ctr.data(), 200, x.buf.data(), x.buf.size(),
                             st2.data()) == RG_EDEVICE, "lost completion times out");
    for (auto s : st2) CHECK(s == RG_PKT_PENDING, "pending after timeout");
    rg_debug_lose_completions(0);
    CHECK(rg_seal_batch_host(c, key, &rec, 1, x.desc.data(), x.ctr.data(), 200, x.buf.data(), x.buf.size(),
                             st2.data()) == RG_OK, "recovered after timeout");
    CHECK(rg_set_staged(c, -1) == RG_OK && rg_set_plan(c, 2) == RG_OK, "knobs back");
    rg_sessions_destroy(p.a);
    rg_sessions_destroy(p.b);
}

static void scenario_group(std::mt19937_64 &rng) {
    const int devs[4] = {0, 1, 0, 1};
    rg_group *g = nullptr;
    CHECK(rg_group_create(devs, 4, &g) == RG_OK, "group");
    if (!g) return;
    for (int k = 0; k < 4; ++k) CHECK(rg_set_host_slice(rg_group_ctx(g, k), 64 << 10) == RG_OK, "slice");
    uint8_t keys[32 * 3];
    for (auto &x : keys) x = (uint8_t)rng();
    const uint32_t rec[3] = {1, 2, 3};
    Batch b = make_batch(rng, 6000, 2); // ~4.5 MB: every part spans more than two 64 KiB slices (threads)
    const size_t n = b.desc.size();
    std::vector<uint8_t> st(n, 0xEE);
    CHECK(rg_seal_batch_host_multi(g, keys, rec, 3, b.desc.data(), b.ctr.data(), n, b.buf.data(), b.buf.size(),
                                   st.data()) == RG_OK, "seal multi");
    for (size_t i = 0; i < n; ++i) CHECK(st[i] == RG_PKT_OK, "seal multi %zu", i);
    const auto od = open_view(b.desc);
    CHECK(rg_open_batch_host_multi(g, keys, 3, od.data(), n, b.buf.data(), b.buf.size(), st.data(), nullptr) == RG_OK,
          "open multi");
    for (size_t i = 0; i < n; ++i) CHECK(st[i] == RG_PKT_OK, "open multi %zu", i);
    CHECK(payloads_equal(b, b.buf), "group round trip");
    std::vector<size_t> bounds(5);
    CHECK(rg_split_batch(b.desc.data(), n, 0, 4, bounds.data()) == RG_OK && bounds[0] == 0 && bounds[4] == n, "split");
    for (int k = 0; k < 4; ++k) CHECK(bounds[k] <= bounds[k + 1], "split order");
    scenario_sessions(nullptr, g, rng, 3000);
    rg_group_destroy(g);
}

static void scenario_per_message(rg_ctx *c) {
    uint8_t key[32], nonce[12] = {0, 0, 0, 0, 7}, aad[5] = {1, 2, 3, 4, 5}, msg[100], ref[100], tag[16];
    for (int i = 0; i < 32; ++i) key[i] = (uint8_t)(3 * i);
    for (int i = 0; i < 100; ++i) msg[i] = ref[i] = (uint8_t)i;
    CHECK(rg_chacha20poly1305_enc(c, key, nonce, aad, 5, msg, 100, tag) == RG_OK, "enc");
    CHECK(memcmp(msg, ref, 100) != 0, "enc changed the text");
    CHECK(rg_chacha20poly1305_dec(c, key, nonce, aad, 5, msg, 100, tag) == RG_OK && memcmp(msg, ref, 100) == 0, "dec");
    CHECK(rg_chacha20poly1305_enc(c, key, nonce, aad, 5, msg, 100, tag) == RG_OK, "enc again");
    tag[3] ^= 1;
    uint8_t before[100];
    memcpy(before, msg, 100);
    CHECK(rg_chacha20poly1305_dec(c, key, nonce, aad, 5, msg, 100, tag) == RG_PKT_DECRYPT_ERR, "forged");
    CHECK(memcmp(msg, before, 100) == 0, "forged message untouched");
}

int main() {
    std::mt19937_64 rng(12345);
    rg_ctx *c = nullptr;
    CHECK(rg_create(0, &c) == RG_OK, "create");
    if (!c) return 1;
    scenario_host(c, rng);
    scenario_sessions(c, nullptr, rng, 500);
    scenario_device_sessions(c, rng);
    scenario_failclosed(c, rng);
    scenario_per_message(c);
    rg_destroy(c);
    scenario_group(rng);
    if (g_fail) {
        fprintf(stderr, "%d checks failed\n", g_fail);
        return 1;
    }
    printf("sanitize driver: all scenarios passed\n");
    return 0;
}
