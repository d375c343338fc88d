/* host_calls.c -- the config-1 serving shape driven from native threads.
 *
 * Weaviate calls the scan once per query from a goroutine
 * (adapters/repos/db/index_queue.go:575-586); through cgo a call costs ~0.1 us
 * on top of the C function.  bench.py's Python caller threads add ~2-4 us of
 * interpreter and ctypes per call, so the per-call latency of the ABI itself
 * is measured here: T POSIX threads each call wvg_search (passed in as a
 * function pointer, so this file links nothing of the library) back to back
 * for a fixed time and record every call's latency.  Benchmark tooling only:
 * built by __graft_entry__.build() into tools/libhostcalls.so, loaded by
 * bench.py's host-API leg.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

typedef int (*search_fn)(void *corpus, const float *query, uint32_t nq, uint32_t k, const uint64_t *allow,
                         uint64_t allow_words, uint64_t *ids, float *dists, uint32_t *counts);

typedef struct {
    search_fn fn;
    void *corpus;
    const float *queries; /* nqs x dim */
    uint32_t nqs, dim, k, threads, t;
    const uint64_t *const *allows; /* nallow lists (NULL: unfiltered) */
    const uint64_t *allow_words;
    uint32_t nallow;
    double stop_at;
    double *lat; /* this thread's latency slots (us) */
    uint64_t cap, n;
    int rc;
    pthread_barrier_t *start;
} worker_t;

static double now_s(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

static void *worker(void *p)
{
    worker_t *w = (worker_t *)p;
    uint64_t ids[256];
    float dists[256];
    uint32_t cnt;
    uint64_t i = w->t;
    pthread_barrier_wait(w->start);
    for (;;) {
        const double t0 = now_s();
        if (t0 >= w->stop_at || w->n >= w->cap) break;
        const float *q = w->queries + (size_t)(i % w->nqs) * w->dim;
        const uint64_t *a = w->nallow ? w->allows[i % w->nallow] : NULL;
        const uint64_t aw = w->nallow ? w->allow_words[i % w->nallow] : 0;
        const int rc = w->fn(w->corpus, q, 1, w->k, a, aw, ids, dists, &cnt);
        const double t1 = now_s();
        if (rc != 0) {
            w->rc = rc;
            break;
        }
        w->lat[w->n++] = (t1 - t0) * 1e6;
        i += w->threads;
    }
    return NULL;
}

/* Returns 0, or the first nonzero wvg_search return code, or -100 on a setup
 * failure.  lat_us holds threads x cap_per_thread slots; counts[t] = calls of
 * thread t (its latencies at lat_us[t * cap_per_thread ...]); *elapsed_s = wall
 * time from the common start to the last thread's end. */
int wvgb_call_loop(void *fn, void *corpus, const float *queries, uint32_t nqs, uint32_t dim, uint32_t k,
                   const uint64_t *const *allows, const uint64_t *allow_words, uint32_t nallow, uint32_t threads,
                   double seconds, double *lat_us, uint64_t cap_per_thread, uint64_t *counts, double *elapsed_s)
{
    if (!fn || threads == 0 || threads > 256 || k > 256 || nqs == 0) return -100;
    pthread_t th[256];
    worker_t ws[256];
    pthread_barrier_t start;
    if (pthread_barrier_init(&start, NULL, threads + 1) != 0) return -100;
    memset(ws, 0, sizeof(worker_t) * threads);
    uint32_t made = 0;
    for (uint32_t t = 0; t < threads; t++) {
        worker_t *w = &ws[t];
        w->fn = (search_fn)fn;
        w->corpus = corpus;
        w->queries = queries;
        w->nqs = nqs;
        w->dim = dim;
        w->k = k;
        w->threads = threads;
        w->t = t;
        w->allows = allows;
        w->allow_words = allow_words;
        w->nallow = nallow;
        w->stop_at = 1e300;
        w->lat = lat_us + (size_t)t * cap_per_thread;
        w->cap = cap_per_thread;
        w->start = &start;
        if (pthread_create(&th[t], NULL, worker, w) != 0) break;
        made++;
    }
    if (made < threads) { /* release the started threads at once and report */
        for (uint32_t t = 0; t < made; t++) ws[t].stop_at = 0.0;
        /* the barrier counts threads + 1: the missing threads never arrive, so
           destroy nothing and detach; a setup failure ends the bench */
        for (uint32_t t = 0; t < made; t++) pthread_detach(th[t]);
        return -100;
    }
    const double t0 = now_s();
    for (uint32_t t = 0; t < threads; t++) ws[t].stop_at = t0 + seconds;
    __atomic_thread_fence(__ATOMIC_SEQ_CST);
    pthread_barrier_wait(&start);
    const double ts = now_s();
    int rc = 0;
    for (uint32_t t = 0; t < threads; t++) {
        pthread_join(th[t], NULL);
        counts[t] = ws[t].n;
        if (ws[t].rc && !rc) rc = ws[t].rc;
    }
    *elapsed_s = now_s() - ts;
    pthread_barrier_destroy(&start);
    return rc;
}
