/* host_calls.c -- the config-1 serving shape driven from native threads.
 *
 * Weaviate calls the scan once per query from a goroutine
 * (adapters/repos/db/index_queue.go:575-586); through cgo a call costs ~0.1 us
 * on top of the C function.  bench.py's Python caller threads add ~2-4 us of
 * interpreter and ctypes per call, so the per-call latency of the ABI itself
 * is measured here: T POSIX threads each call wvg_search (passed in as a
 * function pointer, so this file links nothing of the library) back to back
 * for a fixed time and record every call's latency (optionally with a
 * different k per call, the mixed-k traffic the coalescer batches together).
 * Benchmark tooling only: built by __graft_entry__.build() into
 * tools/libhostcalls.so, loaded by bench.py's host-API leg.
 */
#include <pthread.h>
#include <sched.h>
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
    const uint32_t *ks; /* nks per-call k values (call i: ks[i % nks]); NULL: k */
    uint32_t nks;
    const uint64_t *const *allows; /* nallow lists (NULL: unfiltered) */
    const uint64_t *allow_words;
    uint32_t nallow;
    double stop_at;
    double *lat; /* this thread's latency slots (us) */
    uint64_t cap, n;
    int rc;
    const int *go; /* the common start: 0 until every thread exists */
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
    while (!__atomic_load_n(w->go, __ATOMIC_ACQUIRE)) sched_yield();
    for (;;) {
        const double t0 = now_s();
        if (t0 >= w->stop_at || w->n >= w->cap) break;
        const float *q = w->queries + (size_t)(i % w->nqs) * w->dim;
        const uint64_t *a = w->nallow ? w->allows[i % w->nallow] : NULL;
        const uint64_t aw = w->nallow ? w->allow_words[i % w->nallow] : 0;
        const uint32_t k = w->nks ? w->ks[i % w->nks] : w->k;
        const int rc = w->fn(w->corpus, q, 1, k, a, aw, ids, dists, &cnt);
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
                   const uint32_t *ks, uint32_t nks, const uint64_t *const *allows, const uint64_t *allow_words,
                   uint32_t nallow, uint32_t threads, double seconds, double *lat_us, uint64_t cap_per_thread,
                   uint64_t *counts, double *elapsed_s)
{
    if (!fn || threads == 0 || threads > 256 || k > 256 || nqs == 0) return -100;
    for (uint32_t i = 0; i < nks; i++)
        if (ks[i] == 0 || ks[i] > 256) return -100;
    pthread_t th[256];
    worker_t ws[256];
    int go = 0;
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
        w->ks = ks;
        w->nks = nks;
        w->threads = threads;
        w->t = t;
        w->allows = allows;
        w->allow_words = allow_words;
        w->nallow = nallow;
        w->stop_at = 0.0; /* set below, before the start */
        w->lat = lat_us + (size_t)t * cap_per_thread;
        w->cap = cap_per_thread;
        w->go = &go;
        if (pthread_create(&th[t], NULL, worker, w) != 0) break;
        made++;
    }
    const double t0 = now_s();
    /* a thread that could not be created: the others start with stop_at = 0 and
       end at once */
    if (made == threads)
        for (uint32_t t = 0; t < threads; t++) ws[t].stop_at = t0 + seconds;
    __atomic_store_n(&go, 1, __ATOMIC_RELEASE);
    const double ts = now_s();
    int rc = 0;
    for (uint32_t t = 0; t < made; t++) {
        pthread_join(th[t], NULL);
        counts[t] = ws[t].n;
        if (ws[t].rc && !rc) rc = ws[t].rc;
    }
    *elapsed_s = now_s() - ts;
    return made == threads ? rc : -100;
}
