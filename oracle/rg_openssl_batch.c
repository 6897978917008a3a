/* TEST / BASELINE INFRASTRUCTURE ONLY -- never linked into the product.
 *
 * Multi-threaded batch seal/open through OpenSSL's EVP ChaCha20-Poly1305
 * (libcrypto.so.3, dlopen'ed), the CPU baseline "CPU-B" of BASELINE.md §2: an
 * assembly-optimised RFC 8439 implementation standing in for the reference's
 * graviola 0.2.0 AEAD (Cargo.lock:370-373), which cannot be built here.  Same
 * buffer contract as rg_oracle_seal_batch / rg_oracle_open_batch; like the
 * reference (rustyguard-crypto/src/prim.rs:186-200, ChaCha20Poly1305::new per
 * call) every packet re-keys the cipher context (key setup only: the cipher
 * object is fetched once per worker thread).
 */
#define _GNU_SOURCE
#include <dlfcn.h>
#include <pthread.h>
#include <stddef.h>
#include <stdint.h>
#include <string.h>

#include "rg_oracle.h"

typedef void EVP_CIPHER_CTX;
typedef void EVP_CIPHER;

static struct {
    int ok;
    EVP_CIPHER_CTX *(*ctx_new)(void);
    void (*ctx_free)(EVP_CIPHER_CTX *);
    const EVP_CIPHER *(*chacha)(void);
    int (*cipher_init)(EVP_CIPHER_CTX *, const EVP_CIPHER *, void *, const uint8_t *, const uint8_t *, int);
    int (*cipher_update)(EVP_CIPHER_CTX *, uint8_t *, int *, const uint8_t *, int);
    int (*cipher_final)(EVP_CIPHER_CTX *, uint8_t *, int *);
    int (*ctrl)(EVP_CIPHER_CTX *, int, int, void *);
    const char *(*version)(int);
} ssl;

static pthread_once_t ssl_once = PTHREAD_ONCE_INIT;

static void ssl_load(void) {
    void *h = dlopen("libcrypto.so.3", RTLD_NOW | RTLD_LOCAL);
    if (!h) return;
    ssl.ctx_new = (EVP_CIPHER_CTX * (*)(void)) dlsym(h, "EVP_CIPHER_CTX_new");
    ssl.ctx_free = (void (*)(EVP_CIPHER_CTX *))dlsym(h, "EVP_CIPHER_CTX_free");
    ssl.chacha = (const EVP_CIPHER *(*)(void))dlsym(h, "EVP_chacha20_poly1305");
    ssl.cipher_init = (int (*)(EVP_CIPHER_CTX *, const EVP_CIPHER *, void *, const uint8_t *, const uint8_t *, int))dlsym(
        h, "EVP_CipherInit_ex");
    ssl.cipher_update = (int (*)(EVP_CIPHER_CTX *, uint8_t *, int *, const uint8_t *, int))dlsym(h, "EVP_CipherUpdate");
    ssl.cipher_final = (int (*)(EVP_CIPHER_CTX *, uint8_t *, int *))dlsym(h, "EVP_CipherFinal_ex");
    ssl.ctrl = (int (*)(EVP_CIPHER_CTX *, int, int, void *))dlsym(h, "EVP_CIPHER_CTX_ctrl");
    ssl.version = (const char *(*)(int))dlsym(h, "OpenSSL_version");
    ssl.ok = ssl.ctx_new && ssl.ctx_free && ssl.chacha && ssl.cipher_init && ssl.cipher_update && ssl.cipher_final &&
             ssl.ctrl;
}

/* 1 when libcrypto.so.3 with EVP_chacha20_poly1305 is available */
int rg_openssl_available(void) {
    pthread_once(&ssl_once, ssl_load);
    return ssl.ok;
}

const char *rg_openssl_version(void) {
    if (!rg_openssl_available() || !ssl.version) return "";
    return ssl.version(0);
}

enum { CTRL_AEAD_GET_TAG = 0x10, CTRL_AEAD_SET_TAG = 0x11 };

typedef struct {
    int open;
    const uint8_t *keys;
    const uint32_t *receivers;
    const rg_oracle_desc *desc;
    const uint64_t *counters;
    uint8_t *buf;
    uint8_t *status;
    size_t lo, hi;
} job_t;

static void put32(uint8_t *p, uint32_t v) {
    for (int i = 0; i < 4; i++) p[i] = (uint8_t)(v >> (8 * i));
}
static void put64(uint8_t *p, uint64_t v) {
    for (int i = 0; i < 8; i++) p[i] = (uint8_t)(v >> (8 * i));
}
static uint64_t get64(const uint8_t *p) {
    uint64_t v = 0;
    for (int i = 7; i >= 0; i--) v = (v << 8) | p[i];
    return v;
}

static void *worker(void *arg) {
    job_t *j = (job_t *)arg;
    EVP_CIPHER_CTX *c = ssl.ctx_new();
    uint8_t nonce[12];
    /* the cipher is fetched and bound once per context; each packet then only re-keys it
     * (EVP_CipherInit_ex with a NULL cipher), the equivalent of graviola's per-call
     * ChaCha20Poly1305::new(key) key setup */
    ssl.cipher_init(c, ssl.chacha(), NULL, NULL, NULL, j->open ? 0 : 1);
    for (size_t i = j->lo; i < j->hi; i++) {
        const rg_oracle_desc *d = &j->desc[i];
        uint8_t *frame = j->buf + d->offset;
        const uint8_t *key = j->keys + 32 * (size_t)d->key_idx;
        int outl = 0, ok = 1;
        if (!j->open) {
            const uint64_t ctr = j->counters[i];
            rg_oracle_wg_nonce(ctr, nonce);
            ok &= ssl.cipher_init(c, NULL, NULL, key, nonce, 1);
            ok &= ssl.cipher_update(c, frame + 16, &outl, frame + 16, (int)d->len);
            ok &= ssl.cipher_final(c, frame + 16 + d->len, &outl);
            ok &= ssl.ctrl(c, CTRL_AEAD_GET_TAG, 16, frame + 16 + d->len);
            if (j->receivers) {
                put32(frame, 4u);
                put32(frame + 4, j->receivers[d->key_idx]);
                put64(frame + 8, ctr);
            }
        } else {
            if (d->len < 32) { /* no room for header + tag: prim.rs:427-429 */
                if (j->status) j->status[i] = RG_ORACLE_DECRYPT_ERR;
                continue;
            }
            const uint32_t P = d->len - 32;
            rg_oracle_wg_nonce(get64(frame + 8), nonce);
            ok &= ssl.cipher_init(c, NULL, NULL, key, nonce, 0);
            ok &= ssl.ctrl(c, CTRL_AEAD_SET_TAG, 16, frame + 16 + P);
            ok &= ssl.cipher_update(c, frame + 16, &outl, frame + 16, (int)P);
            ok &= ssl.cipher_final(c, frame + 16 + P, &outl) > 0;
        }
        if (j->status) j->status[i] = ok ? RG_ORACLE_OK : RG_ORACLE_DECRYPT_ERR;
    }
    ssl.ctx_free(c);
    return NULL;
}

static int run(job_t proto, size_t n, int nthreads) {
    if (!rg_openssl_available()) return -1;
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    pthread_t th[256];
    job_t jobs[256];
    for (int t = 0; t < nthreads; t++) {
        jobs[t] = proto;
        jobs[t].lo = n * (size_t)t / (size_t)nthreads;
        jobs[t].hi = n * (size_t)(t + 1) / (size_t)nthreads;
    }
    for (int t = 0; t < nthreads; t++) pthread_create(&th[t], NULL, worker, &jobs[t]);
    for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
    return 0;
}

/* seal: desc.len = P; open: desc.len = W = P + 32 (seal output, ciphertext framed) */
int rg_openssl_seal_batch(const uint8_t *keys, const uint32_t *receivers, const rg_oracle_desc *desc,
                          const uint64_t *counters, size_t n, uint8_t *buf, uint8_t *status, int nthreads) {
    job_t p = {0, keys, receivers, desc, counters, buf, status, 0, 0};
    return run(p, n, nthreads);
}

int rg_openssl_open_batch(const uint8_t *keys, const rg_oracle_desc *desc, size_t n, uint8_t *buf, uint8_t *status,
                          int nthreads) {
    job_t p = {1, keys, NULL, desc, NULL, buf, status, 0, 0};
    return run(p, n, nthreads);
}

/* ---- BASELINE config 1: one transport packet, one thread (bench.py --workload cfg1) ----
 * Seals then opens one frame of payload P `iters` times (counter i for round i, so every seal is a
 * fresh nonce, as EncryptionKey::encrypt would use it) and returns the mean wall-clock ns of one
 * seal and of one open.  impl 0: the C restatement (rg_oracle_seal_one / _open_one); impl 1:
 * OpenSSL EVP, re-keyed per packet like graviola's ChaCha20Poly1305::new per call. */
#include <stdlib.h>
#include <time.h>

static double now_ns(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (double)t.tv_sec * 1e9 + (double)t.tv_nsec;
}

int rg_cpu_time_one(int impl, const uint8_t key[32], uint32_t P, uint64_t iters, double out_ns[2]) {
    if (impl == 1 && !rg_openssl_available()) return -1;
    uint8_t *frame = aligned_alloc(64, ((size_t)P + 32 + 63) & ~(size_t)63);
    if (!frame) return -2;
    for (uint32_t b = 0; b < P + 32; b++) frame[b] = (uint8_t)(b * 131u + 7u);
    const uint32_t recv = 0x12345678u;
    rg_oracle_desc ds = {0, P, 0}, dopen = {0, P + 32, 0};
    EVP_CIPHER_CTX *c = NULL;
    if (impl == 1) c = ssl.ctx_new();
    uint8_t nonce[12], status = 0;
    double t_seal = 0, t_open = 0;
    int ok = 1, outl = 0;
    for (uint64_t i = 0; i < iters; i++) {
        double t0 = now_ns();
        if (impl == 0) {
            rg_oracle_seal_one(key, &recv, &ds, i, frame, &status);
            ok &= status == RG_ORACLE_OK;
        } else {
            rg_oracle_wg_nonce(i, nonce);
            ok &= ssl.cipher_init(c, i == 0 ? ssl.chacha() : NULL, NULL, key, nonce, 1);
            ok &= ssl.cipher_update(c, frame + 16, &outl, frame + 16, (int)P);
            ok &= ssl.cipher_final(c, frame + 16 + P, &outl);
            ok &= ssl.ctrl(c, CTRL_AEAD_GET_TAG, 16, frame + 16 + P);
            put32(frame, 4u);
            put32(frame + 4, recv);
            put64(frame + 8, i);
        }
        double t1 = now_ns();
        if (impl == 0) {
            rg_oracle_open_one(key, &dopen, frame, &status, NULL);
            ok &= status == RG_ORACLE_OK;
        } else {
            rg_oracle_wg_nonce(get64(frame + 8), nonce);
            ok &= ssl.cipher_init(c, NULL, NULL, key, nonce, 0);
            ok &= ssl.ctrl(c, CTRL_AEAD_SET_TAG, 16, frame + 16 + P);
            ok &= ssl.cipher_update(c, frame + 16, &outl, frame + 16, (int)P);
            ok &= ssl.cipher_final(c, frame + 16 + P, &outl) > 0;
        }
        double t2 = now_ns();
        t_seal += t1 - t0;
        t_open += t2 - t1;
    }
    if (c) ssl.ctx_free(c);
    free(frame);
    out_ns[0] = t_seal / (double)(iters ? iters : 1);
    out_ns[1] = t_open / (double)(iters ? iters : 1);
    return ok ? 0 : -3;
}

/* ---- CPU baseline harness (bench.py cpu_baseline) ----
 * Round 5 timed the baselines through rg_*_batch above, which start fresh threads -- and, for OpenSSL, a
 * fresh EVP_CIPHER_CTX and cipher fetch -- per call, on a 4096-packet sample: 256 packets (~200 us) per
 * thread per call, so thread start-up and joins dominated the all-core figure (OpenSSL 3.3x on 16 threads).
 * rg_cpu_bench keeps one pool for the whole measurement: nthreads workers, each owning a fixed slice of
 * the sample and (OpenSSL) one cipher context for its lifetime, run in rounds between two barriers; a
 * round seals the slice then opens it again (the frames return to plaintext, so every round does the same
 * work).  One untimed round first; then rounds until `seconds` have passed.
 * impl 0: the C restatement (rg_oracle_seal_one / _open_one); 1: OpenSSL EVP, re-keyed per packet; 2: OpenSSL
 * EVP with the key installed only when it changes (bench.py --cpu-study only).
 * cpus (optional, nthreads entries): worker t runs on CPU cpus[t] only.  local != 0: each worker works on a
 * private copy of its slice's frames, allocated and first-touched by itself (its NUMA node, its caches),
 * copied back into buf at the end.
 * out[0] = elapsed seconds of the timed rounds, out[1] = timed rounds, out[2] = packets whose seal or open
 * failed (0 expected). */
#include <sched.h>

typedef struct {
    int impl;
    const uint8_t *keys;
    const uint32_t *receivers;
    const rg_oracle_desc *desc;
    const uint64_t *counters;
    uint8_t *buf;
    size_t n;
    int nthreads;
    const int *cpus;
    int local;
    pthread_barrier_t start, done;
    volatile int stop;
    volatile uint64_t bad;
    pthread_mutex_t mu;
} pool_t;

typedef struct {
    pool_t *p;
    int t;
} pool_arg_t;

static uint64_t pool_round(pool_t *p, uint8_t *bufp, EVP_CIPHER_CTX *c, size_t lo, size_t hi) {
    uint64_t bad = 0;
    uint8_t nonce[12], st = 0;
    int outl = 0;
    /* impl 2 (study only): the key is installed only when it changes from the previous packet's, the nonce
     * per packet -- what per-packet re-keying costs beyond the cipher itself */
    const uint8_t *cur_key = NULL;
    int cur_enc = -1;
    for (size_t i = lo; i < hi; i++) { /* seal: desc.len = P */
        const rg_oracle_desc *d = &p->desc[i];
        uint8_t *frame = bufp + d->offset;
        if (p->impl == 0) {
            rg_oracle_seal_one(p->keys, p->receivers, d, p->counters[i], bufp, &st);
            bad += st != RG_ORACLE_OK;
        } else {
            int ok = 1;
            const uint8_t *key = p->keys + 32 * (size_t)d->key_idx;
            rg_oracle_wg_nonce(p->counters[i], nonce);
            if (p->impl == 2 && key == cur_key && cur_enc == 1) ok &= ssl.cipher_init(c, NULL, NULL, NULL, nonce, 1);
            else ok &= ssl.cipher_init(c, NULL, NULL, key, nonce, 1);
            cur_key = key;
            cur_enc = 1;
            ok &= ssl.cipher_update(c, frame + 16, &outl, frame + 16, (int)d->len);
            ok &= ssl.cipher_final(c, frame + 16 + d->len, &outl);
            ok &= ssl.ctrl(c, CTRL_AEAD_GET_TAG, 16, frame + 16 + d->len);
            put32(frame, 4u);
            put32(frame + 4, p->receivers ? p->receivers[d->key_idx] : 0u);
            put64(frame + 8, p->counters[i]);
            bad += !ok;
        }
    }
    for (size_t i = lo; i < hi; i++) { /* open the frames just sealed: W = P + 32 */
        rg_oracle_desc d = p->desc[i];
        d.len += 32;
        uint8_t *frame = bufp + d.offset;
        if (p->impl == 0) {
            rg_oracle_open_one(p->keys, &d, bufp, &st, NULL);
            bad += st != RG_ORACLE_OK;
        } else {
            int ok = 1;
            const uint32_t P = d.len - 32;
            const uint8_t *key = p->keys + 32 * (size_t)d.key_idx;
            rg_oracle_wg_nonce(get64(frame + 8), nonce);
            if (p->impl == 2 && key == cur_key && cur_enc == 0) ok &= ssl.cipher_init(c, NULL, NULL, NULL, nonce, 0);
            else ok &= ssl.cipher_init(c, NULL, NULL, key, nonce, 0);
            cur_key = key;
            cur_enc = 0;
            ok &= ssl.ctrl(c, CTRL_AEAD_SET_TAG, 16, frame + 16 + P);
            ok &= ssl.cipher_update(c, frame + 16, &outl, frame + 16, (int)P);
            ok &= ssl.cipher_final(c, frame + 16 + P, &outl) > 0;
            bad += !ok;
        }
    }
    return bad;
}

static void *pool_worker(void *arg) {
    pool_arg_t *a = (pool_arg_t *)arg;
    pool_t *p = a->p;
    const size_t lo = p->n * (size_t)a->t / (size_t)p->nthreads, hi = p->n * (size_t)(a->t + 1) / (size_t)p->nthreads;
    if (p->cpus) {
        cpu_set_t set;
        CPU_ZERO(&set);
        CPU_SET(p->cpus[a->t], &set);
        (void)pthread_setaffinity_np(pthread_self(), sizeof set, &set);
    }
    /* the frames this worker touches: [desc[lo].offset, end of desc[hi - 1]'s frame) when the slice is in
     * offset order (the workloads' layout); a private copy rebases the same offsets onto it */
    uint8_t *bufp = p->buf, *priv = NULL;
    size_t base = 0, span = 0;
    if (p->local && hi > lo) {
        base = (size_t)p->desc[lo].offset;
        size_t end = base;
        for (size_t i = lo; i < hi; i++) {
            const size_t e = (size_t)p->desc[i].offset + p->desc[i].len + 32;
            if ((size_t)p->desc[i].offset < base) base = (size_t)p->desc[i].offset;
            if (e > end) end = e;
        }
        span = end - base;
        priv = (uint8_t *)malloc(span);
        if (priv) {
            memcpy(priv, p->buf + base, span); /* first touch by this worker */
            bufp = priv - base;
        }
    }
    EVP_CIPHER_CTX *c = NULL;
    if (p->impl >= 1) { /* one context for the worker's lifetime, the cipher bound once */
        c = ssl.ctx_new();
        ssl.cipher_init(c, ssl.chacha(), NULL, NULL, NULL, 1);
    }
    uint64_t bad = 0;
    for (;;) {
        pthread_barrier_wait(&p->start);
        if (p->stop) break;
        bad += pool_round(p, bufp, c, lo, hi);
        pthread_barrier_wait(&p->done);
    }
    if (c) ssl.ctx_free(c);
    if (priv) { /* the slices do not overlap: each worker writes back its own frames */
        memcpy(p->buf + base, priv, span);
        free(priv);
    }
    pthread_mutex_lock(&p->mu);
    p->bad += bad;
    pthread_mutex_unlock(&p->mu);
    return NULL;
}

int rg_cpu_bench(int impl, int nthreads, const uint8_t *keys, const uint32_t *receivers, const rg_oracle_desc *desc,
                 const uint64_t *counters, size_t n, uint8_t *buf, double seconds, const int *cpus, int local,
                 double out[3]) {
    if (impl >= 1 && !rg_openssl_available()) return -1;
    if (nthreads < 1 || nthreads > 256 || n == 0) return -2;
    pool_t p;
    memset(&p, 0, sizeof p);
    p.impl = impl;
    p.keys = keys;
    p.receivers = receivers;
    p.desc = desc;
    p.counters = counters;
    p.buf = buf;
    p.n = n;
    p.nthreads = nthreads;
    p.cpus = cpus;
    p.local = local;
    if (local) { /* private copies are written back whole: the slices' frame spans must not overlap */
        size_t prev_end = 0;
        for (int t = 0; t < nthreads; t++) {
            const size_t lo = n * (size_t)t / (size_t)nthreads, hi = n * (size_t)(t + 1) / (size_t)nthreads;
            if (hi <= lo) continue;
            size_t b = (size_t)desc[lo].offset, e = b;
            for (size_t i = lo; i < hi; i++) {
                if ((size_t)desc[i].offset < b) b = (size_t)desc[i].offset;
                if ((size_t)desc[i].offset + desc[i].len + 32 > e) e = (size_t)desc[i].offset + desc[i].len + 32;
            }
            if (b < prev_end) return -4;
            prev_end = e;
        }
    }
    pthread_barrier_init(&p.start, NULL, (unsigned)nthreads + 1);
    pthread_barrier_init(&p.done, NULL, (unsigned)nthreads + 1);
    pthread_mutex_init(&p.mu, NULL);
    pthread_t th[256];
    pool_arg_t args[256];
    int started = 0;
    for (; started < nthreads; started++) {
        args[started].p = &p;
        args[started].t = started;
        if (pthread_create(&th[started], NULL, pool_worker, &args[started]) != 0) break;
    }
    if (started < nthreads) { /* cannot run the measurement as asked: release the ones that started */
        /* the barriers count nthreads + 1: a short pool would block forever, so nothing ran yet */
        for (int t = 0; t < started; t++) pthread_cancel(th[t]);
        for (int t = 0; t < started; t++) pthread_join(th[t], NULL);
        return -3;
    }
    /* one untimed round (first-touch, caches, frequency ramp) */
    pthread_barrier_wait(&p.start);
    pthread_barrier_wait(&p.done);
    uint64_t rounds = 0;
    const double t0 = now_ns();
    double el = 0;
    do {
        pthread_barrier_wait(&p.start);
        pthread_barrier_wait(&p.done);
        rounds++;
        el = (now_ns() - t0) * 1e-9;
    } while (el < seconds);
    p.stop = 1;
    pthread_barrier_wait(&p.start);
    for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
    pthread_barrier_destroy(&p.start);
    pthread_barrier_destroy(&p.done);
    pthread_mutex_destroy(&p.mu);
    out[0] = el;
    out[1] = (double)rounds;
    out[2] = (double)p.bad;
    return 0;
}
