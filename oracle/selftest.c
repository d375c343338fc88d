/*
 * selftest.c -- memory / UB self-check of the oracle (TEST INFRASTRUCTURE).
 *
 * Built by `make -C oracle asan` together with wv_oracle.c under
 * -fsanitize=address,undefined and run by tests/test_oracle.py: every entry
 * point is driven over the edge sizes the parity tests use (empty inputs,
 * lengths around the 8/32-float blocks of l2_256 / dot_256 and the 16/64-float
 * blocks of the 512-bit kernels, k = 0, k > n, deletions, ragged BQ words) so
 * an out-of-bounds read or an overflow in the checker cannot hide a kernel
 * bug.  Prints "selftest ok" and exits 0 when every check holds.
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

float orc_l2_256(const float *a, const float *b, long len);
float orc_dot_256(const float *a, const float *b, long len);
float orc_l2_512(const float *a, const float *b, long len);
float orc_dot_512(const float *a, const float *b, long len);
float orc_l2_step(const float *a, const float *b, long n);
float orc_dot_step(const float *a, const float *b, long n);
float orc_single_dist(int metric, const float *a, const float *b, long n);
void orc_normalize(const float *v, long n, float *out);
void orc_bq_encode(const float *v, long d, uint64_t *code);
float orc_bq_distance(const uint64_t *x, const uint64_t *y, long w);
void orc_pq_lut(int metric, const float *q, const float *centers, long m, long ks, long ds, float *lut);
float orc_pq_adc(int metric, const float *lut, const uint8_t *code, long m, long ks);
void orc_pq_global_distances(int metric, const float *centers, long m, long ks, long ds, float *table);
float orc_pq_sdc(int metric, const float *table, const uint8_t *x, const uint8_t *y, long m, long ks);
void orc_pq_encode(const float *x, long n, long d, const float *centers, long m, long ks, uint8_t *codes);
long orc_pq_fit(const float *x, long n, long d, long m, long ks, long training_limit, uint64_t seed,
                float *centers, uint32_t *iterations);
long orc_heap_topk(const float *dists, const uint64_t *ids, const uint8_t *valid, long n, long k,
                   uint64_t *out_ids, float *out_dists);
long orc_flat_search(const float *rows, long n, long d, long pitch, const uint8_t *valid, const float *q,
                     long k, int metric, void *fn, uint64_t *out_ids, float *out_dists);
long orc_flat_search_bq(const float *rows, const uint64_t *codes, long n, long d, long pitch,
                        const uint8_t *valid, const float *query, long k, long rescore_limit, int metric,
                        uint64_t *out_ids, float *out_dists, uint64_t *cand_ids);
void orc_synth_rows(uint64_t seed, uint64_t row0, long n, long d, long pitch, int dist, float *out);

static int failures = 0;
#define CHECK(cond, ...)                                                                                   \
    do {                                                                                                   \
        if (!(cond)) {                                                                                     \
            failures++;                                                                                    \
            fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__);                                          \
            fprintf(stderr, __VA_ARGS__);                                                                  \
            fputc('\n', stderr);                                                                           \
        }                                                                                                  \
    } while (0)

/* exact-size heap buffers so ASan sees any read past the logical end */
static float *frows(uint64_t seed, long n, long d)
{
    float *p = (float *)malloc(sizeof(float) * (size_t)(n * d > 0 ? n * d : 1));
    if (n * d > 0) orc_synth_rows(seed, 0, n, d, d, 0, p);
    return p;
}

static void distances(void)
{
    static const long lens[] = {0, 1, 7, 8, 9, 15, 16, 17, 31, 32, 33, 63, 64, 65, 127, 128, 129, 255, 256, 257,
                                767, 768, 1535, 1536};
    for (size_t t = 0; t < sizeof(lens) / sizeof(lens[0]); t++) {
        long n = lens[t];
        float *a = frows(1 + t, 1, n), *b = frows(100 + t, 1, n);
        float *na = (float *)malloc(sizeof(float) * (size_t)(n > 0 ? n : 1));
        CHECK(orc_l2_256(a, a, n) == 0.0f, "l2_256(a,a) len %ld", n);
        CHECK(orc_l2_512(a, a, n) == 0.0f, "l2_512(a,a) len %ld", n);
        CHECK(orc_l2_step(a, a, n) == 0.0f, "l2_step(a,a) len %ld", n);
        CHECK(orc_l2_256(a, b, n) == orc_l2_256(b, a, n), "l2_256 symmetric len %ld", n);
        CHECK(orc_dot_256(a, b, n) == orc_dot_256(b, a, n), "dot_256 symmetric len %ld", n);
        CHECK(orc_dot_512(a, b, n) == orc_dot_512(b, a, n), "dot_512 symmetric len %ld", n);
        CHECK(orc_l2_256(a, b, n) >= 0.0f, "l2_256 >= 0 len %ld", n);
        (void)orc_dot_step(a, b, n);
        for (int m = 0; m < 3; m++) (void)orc_single_dist(m, a, b, n);
        if (n > 0) {
            orc_normalize(a, n, na);
            float s = orc_dot_step(na, na, n);
            CHECK(fabsf(s - 1.0f) < 1e-4f, "normalize len %ld: |v|^2 = %g", n, (double)s);
        }
        free(a);
        free(b);
        free(na);
    }
}

static void bq(void)
{
    static const long dims[] = {1, 63, 64, 65, 127, 128, 129, 1536};
    for (size_t t = 0; t < sizeof(dims) / sizeof(dims[0]); t++) {
        long d = dims[t], w = (d + 63) / 64;
        float *x = frows(7 + t, 1, d), *y = frows(70 + t, 1, d);
        uint64_t *cx = (uint64_t *)malloc(sizeof(uint64_t) * (size_t)w);
        uint64_t *cy = (uint64_t *)malloc(sizeof(uint64_t) * (size_t)w);
        orc_bq_encode(x, d, cx);
        orc_bq_encode(y, d, cy);
        CHECK(orc_bq_distance(cx, cx, w) == 0.0f, "bq self distance d %ld", d);
        float h = orc_bq_distance(cx, cy, w);
        CHECK(h >= 0.0f && h <= (float)d, "bq distance range d %ld: %g", d, (double)h);
        free(x);
        free(y);
        free(cx);
        free(cy);
    }
}

static void pq(void)
{
    const long n = 300, d = 16, m = 4, ks = 16, ds = d / m;
    float *x = frows(11, n, d);
    float *centers = (float *)malloc(sizeof(float) * (size_t)(m * ks * ds));
    uint32_t it[4];
    CHECK(orc_pq_fit(x, n, d, m, ks, 0, 3, centers, it) == 0, "pq_fit");
    CHECK(orc_pq_fit(x, ks - 1, d, m, ks, 0, 3, centers, it) != 0, "pq_fit must refuse n < ks");
    CHECK(orc_pq_fit(x, n, d, m, ks, 0, 3, centers, it) == 0, "pq_fit again");
    uint8_t *codes = (uint8_t *)malloc((size_t)(n * m));
    orc_pq_encode(x, n, d, centers, m, ks, codes);
    float *lut = (float *)malloc(sizeof(float) * (size_t)(m * ks));
    float *table = (float *)malloc(sizeof(float) * (size_t)(m * ks * ks));
    orc_pq_global_distances(0, centers, m, ks, ds, table);
    for (int metric = 0; metric < 3; metric++) {
        orc_pq_lut(metric, x, centers, m, ks, ds, lut);
        for (long i = 0; i < n; i++) (void)orc_pq_adc(metric, lut, codes + i * m, m, ks);
    }
    for (long i = 0; i < n; i++) {
        CHECK(codes[i * m] < ks, "code range");
        CHECK(orc_pq_sdc(0, table, codes + i * m, codes + i * m, m, ks) == 0.0f, "sdc self distance");
    }
    free(x);
    free(centers);
    free(codes);
    free(lut);
    free(table);
}

static void topk(void)
{
    static const long ns[] = {0, 1, 5, 64, 65, 1000};
    static const long ks[] = {0, 1, 3, 10, 64, 300, 2000};
    for (size_t a = 0; a < sizeof(ns) / sizeof(ns[0]); a++) {
        long n = ns[a], d = 33;
        float *rows = frows(21 + a, n, d), *q = frows(5, 1, d);
        float *dists = (float *)malloc(sizeof(float) * (size_t)(n > 0 ? n : 1));
        uint64_t *ids = (uint64_t *)malloc(sizeof(uint64_t) * (size_t)(n > 0 ? n : 1));
        uint8_t *valid = (uint8_t *)malloc((size_t)(n > 0 ? n : 1));
        long live = 0;
        for (long i = 0; i < n; i++) {
            dists[i] = orc_l2_256(q, rows + i * d, d);
            ids[i] = (uint64_t)i;
            valid[i] = (uint8_t)(i % 3 != 1);
            live += valid[i];
        }
        uint64_t *codes = (uint64_t *)malloc(sizeof(uint64_t) * (size_t)(n > 0 ? n : 1));
        for (long i = 0; i < n; i++) orc_bq_encode(rows + i * d, d, codes + i);
        for (size_t b = 0; b < sizeof(ks) / sizeof(ks[0]); b++) {
            long k = ks[b], want = k < live ? k : live;
            uint64_t *oid = (uint64_t *)malloc(sizeof(uint64_t) * (size_t)(k > 0 ? k : 1));
            float *od = (float *)malloc(sizeof(float) * (size_t)(k > 0 ? k : 1));
            uint64_t *cand = (uint64_t *)malloc(sizeof(uint64_t) * (size_t)(k > 500 ? k : 500));
            long c = orc_heap_topk(dists, ids, valid, n, k, oid, od);
            CHECK(c == want, "heap_topk n %ld k %ld: %ld != %ld", n, k, c, want);
            for (long i = 1; i < c; i++) CHECK(od[i - 1] <= od[i], "heap_topk order");
            for (long i = 0; i < c; i++) CHECK(valid[oid[i]], "heap_topk returned a deleted row");
            c = orc_flat_search(rows, n, d, d, valid, q, k, 0, NULL, oid, od);
            CHECK(c == want, "flat_search n %ld k %ld: %ld != %ld", n, k, c, want);
            c = orc_flat_search_bq(rows, codes, n, d, d, valid, q, k, 500, 0, oid, od, cand);
            CHECK(c == want, "flat_search_bq n %ld k %ld: %ld != %ld", n, k, c, want);
            free(oid);
            free(od);
            free(cand);
        }
        free(rows);
        free(q);
        free(dists);
        free(ids);
        free(valid);
        free(codes);
    }
}

int main(void)
{
    distances();
    bq();
    pq();
    topk();
    if (failures) {
        fprintf(stderr, "selftest: %d failure(s)\n", failures);
        return 1;
    }
    printf("selftest ok\n");
    return 0;
}
