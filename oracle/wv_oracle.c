/*
 * wv_oracle.c -- CPU restatement of Weaviate's vector-scoring hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in weaviate_amd/ links, loads or calls
 * this file.  It is used by tests/ (as the parity checker), by
 * __graft_entry__.smoke() (as the checker) and by bench.py's cpu_baseline leg
 * (as the timed CPU baseline).  The product path is the HIP library
 * weaviate_amd/libwvgpu.so and fails loudly when it is missing.
 *
 * Parity pinning: the float kernels below are checked bit-for-bit against the
 * reference's own C kernels compiled from /root/reference into oracle/_ref/
 * (oracle/Makefile, target `ref`), and against the hand-vector known answers of
 * the reference's Go tests (tests/golden/).  See DESIGN.md "Oracle".
 *
 * Every function cites the reference file:line it restates.  Abbreviations:
 *   D/  = adapters/repos/db/vector/hnsw/distancer/
 *   CH/ = adapters/repos/db/vector/compressionhelpers/
 *   V/  = adapters/repos/db/vector/
 *
 * Build: gcc -O2 -ffp-contract=off (no fusing except the explicit fmaf calls
 * that mirror the reference's _mm256_fmadd_ps / vfmadd231ss instructions).
 */
#include <float.h>
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#define ORC_API __attribute__((visibility("default")))

/* ------------------------------------------------------------------------ */
/* Float distance kernels                                                    */
/* ------------------------------------------------------------------------ */

/* Reduction tail shared by l2_256 / dot_256: D/c/l2_avx256_amd64.c:96-104.
 * acc[0] = acc1+acc0; acc[2] = acc3+acc2; acc[0] = acc2+acc0; two hadds give
 * lane0 = (s0+s1)+(s2+s3) and lane4 = (s4+s5)+(s6+s7); lo128+hi128; sum += . */
static float avx256_reduce(float acc[4][8], float sum)
{
    float s[8];
    for (int l = 0; l < 8; l++) {
        float a01 = acc[1][l] + acc[0][l];
        float a23 = acc[3][l] + acc[2][l];
        s[l] = a23 + a01;
    }
    float lo = (s[0] + s[1]) + (s[2] + s[3]);
    float hi = (s[4] + s[5]) + (s[6] + s[7]);
    float t4 = lo + hi;
    return sum + t4;
}

/* l2_256: D/c/l2_avx256_amd64.c:14-107 (shipped as D/asm/l2_avx256_amd64.s).
 * n<8: sequential unfused diff*diff (:20-34, asm vmulss+vaddss).
 * n>=8: 4 accumulators x 8 lanes, acc[j] = fma(diff,diff,acc[j]) per 32-float
 * block (:43-69); leftover 8-blocks into acc0 (:72-83); scalar unfused tail
 * into sum (:86-94); fixed reduction tree (:97-104).
 * Note: the reference loops forever for len==0 (do/while); we return 0. */
ORC_API float orc_l2_256(const float *a, const float *b, long len)
{
    int n = (int)len;
    float sum = 0.0f;
    if (n <= 0) return 0.0f;
    if (n < 8) {
        do {
            float diff = a[0] - b[0];
            float sq = diff * diff;
            sum += sq;
            n--; a++; b++;
        } while (n);
        return sum;
    }
    float acc[4][8];
    memset(acc, 0, sizeof(acc));
    while (n >= 32) {
        for (int j = 0; j < 4; j++)
            for (int l = 0; l < 8; l++) {
                float diff = a[8 * j + l] - b[8 * j + l];
                acc[j][l] = fmaf(diff, diff, acc[j][l]);
            }
        n -= 32; a += 32; b += 32;
    }
    while (n >= 8) {
        for (int l = 0; l < 8; l++) {
            float diff = a[l] - b[l];
            acc[0][l] = fmaf(diff, diff, acc[0][l]);
        }
        n -= 8; a += 8; b += 8;
    }
    while (n) {
        float diff = a[0] - b[0];
        float sq = diff * diff;
        sum += sq;
        n--; a++; b++;
    }
    return avx256_reduce(acc, sum);
}

/* dot_256: D/c/dot_avx256_amd64.c:14-104 (shipped D/asm/dot_avx256_amd64.s).
 * Same structure as l2_256 with acc = fma(a,b,acc).  The scalar paths are
 * FUSED in the shipped asm (vfmadd231ss, dot_avx256_amd64.s:25,82-87,155):
 * clang contracts `sum += a[0] * b[0]` (one expression). */
ORC_API float orc_dot_256(const float *a, const float *b, long len)
{
    int n = (int)len;
    float sum = 0.0f;
    if (n <= 0) return 0.0f;
    if (n < 8) {
        do {
            sum = fmaf(a[0], b[0], sum);
            n--; a++; b++;
        } while (n);
        return sum;
    }
    float acc[4][8];
    memset(acc, 0, sizeof(acc));
    while (n >= 32) {
        for (int j = 0; j < 4; j++)
            for (int l = 0; l < 8; l++)
                acc[j][l] = fmaf(a[8 * j + l], b[8 * j + l], acc[j][l]);
        n -= 32; a += 32; b += 32;
    }
    while (n >= 8) {
        for (int l = 0; l < 8; l++)
            acc[0][l] = fmaf(a[l], b[l], acc[0][l]);
        n -= 8; a += 8; b += 8;
    }
    while (n) {
        sum = fmaf(a[0], b[0], sum);
        n--; a++; b++;
    }
    return avx256_reduce(acc, sum);
}

/* l2_512: D/c/l2_avx512_amd64.c:14-178.  Selected only on AMX+AVX512 hosts
 * (D/l2_amd64.go:19-25).  For n>=128: 8 x 16-lane accumulators per 128-block,
 * tree-reduced to one 512 register, folded lo256 then hi256 into acc0. */
static float l2_or_dot_512(const float *a, const float *b, long len, int is_dot)
{
    int n = (int)len;
    float sum = 0.0f;
    if (n <= 0) return 0.0f;
    if (n < 8) {
        do {
            if (is_dot) sum = fmaf(a[0], b[0], sum);
            else { float diff = a[0] - b[0]; float sq = diff * diff; sum += sq; }
            n--; a++; b++;
        } while (n);
        return sum;
    }
    float acc[4][8];
    memset(acc, 0, sizeof(acc));
    if (n >= 128) {
        float a5[8][16];
        memset(a5, 0, sizeof(a5));
        do {
            for (int j = 0; j < 8; j++)
                for (int l = 0; l < 16; l++) {
                    float x = a[16 * j + l], y = b[16 * j + l];
                    if (is_dot) a5[j][l] = fmaf(x, y, a5[j][l]);
                    else { float diff = x - y; a5[j][l] = fmaf(diff, diff, a5[j][l]); }
                }
            n -= 128; a += 128; b += 128;
        } while (n >= 128);
        float r[16];
        for (int l = 0; l < 16; l++) {
            float x0 = a5[1][l] + a5[0][l];
            float x2 = a5[3][l] + a5[2][l];
            float x4 = a5[5][l] + a5[4][l];
            float x6 = a5[7][l] + a5[6][l];
            x0 = x2 + x0;
            x4 = x6 + x4;
            r[l] = x4 + x0;
        }
        for (int l = 0; l < 8; l++) acc[0][l] = r[l] + acc[0][l];
        for (int l = 0; l < 8; l++) acc[0][l] = r[8 + l] + acc[0][l];
        if (!n) return avx256_reduce(acc, sum);
    }
    while (n >= 32) {
        for (int j = 0; j < 4; j++)
            for (int l = 0; l < 8; l++) {
                float x = a[8 * j + l], y = b[8 * j + l];
                if (is_dot) acc[j][l] = fmaf(x, y, acc[j][l]);
                else { float diff = x - y; acc[j][l] = fmaf(diff, diff, acc[j][l]); }
            }
        n -= 32; a += 32; b += 32;
    }
    while (n >= 8) {
        for (int l = 0; l < 8; l++) {
            float x = a[l], y = b[l];
            if (is_dot) acc[0][l] = fmaf(x, y, acc[0][l]);
            else { float diff = x - y; acc[0][l] = fmaf(diff, diff, acc[0][l]); }
        }
        n -= 8; a += 8; b += 8;
    }
    while (n) {
        if (is_dot) sum = fmaf(a[0], b[0], sum);
        else { float diff = a[0] - b[0]; float sq = diff * diff; sum += sq; }
        n--; a++; b++;
    }
    return avx256_reduce(acc, sum);
}
ORC_API float orc_l2_512(const float *a, const float *b, long len) { return l2_or_dot_512(a, b, len, 0); }
/* dot_512: D/c/dot_avx512_amd64.c:14 (same structure, fused products). */
ORC_API float orc_dot_512(const float *a, const float *b, long len) { return l2_or_dot_512(a, b, len, 1); }

/* Pure-Go Step loops, amd64 GOAMD64=v1 => no FMA fusion.
 * L2 Step: D/l2.go:79-88; dot/cosine Step: D/dot_product.go:87-94,
 * D/cosine_dist.go:57-64. */
ORC_API float orc_l2_step(const float *a, const float *b, long n)
{
    float sum = 0.0f;
    for (long i = 0; i < n; i++) {
        float diff = a[i] - b[i];
        float sq = diff * diff;
        sum += sq;
    }
    return sum;
}
ORC_API float orc_dot_step(const float *a, const float *b, long n)
{
    float sum = 0.0f;
    for (long i = 0; i < n; i++) {
        float p = a[i] * b[i];
        sum += p;
    }
    return sum;
}

enum { ORC_L2 = 0, ORC_DOT = 1, ORC_COSINE = 2, ORC_MANHATTAN = 3, ORC_HAMMING = 4 };

/* manhattanImpl: D/manhattan.go:20-30 -- pure Go on every host (no SIMD
 * kernel): sum += float32(math.Abs(float64(a[i] - b[i]))) in element order.
 * The float64 round trip is exact, so this is fabsf of the fp32 difference.
 * ManhattanProvider.Step (:68-78) is the same loop. */
ORC_API float orc_manhattan(const float *a, const float *b, long n)
{
    float sum = 0.0f;
    for (long i = 0; i < n; i++) {
        float diff = a[i] - b[i];
        sum += fabsf(diff);
    }
    return sum;
}

/* hamming_256: D/c/hamming_avx256_amd64.c:14-144, dispatched on AVX2 hosts by
 * D/hamming_amd64.go:18-24 (hamming_512, D/c/hamming_avx512_amd64.c, counts
 * the same elements with the same comparisons).  An int count, stored as
 * float.  n < 8 (:20-32): `a[0] != b[0]` per element (C's !=: a NaN counts).
 * n >= 8: the 32- and 8-blocks (:59-119) compare with _CMP_NEQ_OQ (ordered
 * not-equal: a NaN does NOT count); the tail (:121-131) with != again.
 * Note: the reference loops forever for len == 0 (do/while); we return 0. */
ORC_API float orc_hamming_256(const float *a, const float *b, long len)
{
    int n = (int)len;
    int sum = 0;
    if (n <= 0) return 0.0f;
    int nord = n >= 8 ? (n & ~7) : 0;
    for (int i = 0; i < n; i++) {
        if (i < nord)
            sum += (a[i] < b[i] || a[i] > b[i]) ? 1 : 0; /* _CMP_NEQ_OQ */
        else
            sum += a[i] != b[i] ? 1 : 0;
    }
    return (float)sum;
}

/* HammingProvider.Step: D/hamming.go:76-86 -- pure Go: sum += float32(1)
 * where x[i] != y[i] (Go's !=: a NaN counts). */
ORC_API float orc_hamming_step(const float *a, const float *b, long n)
{
    float sum = 0.0f;
    for (long i = 0; i < n; i++)
        if (a[i] != b[i]) sum += 1.0f;
    return sum;
}

/* Provider.SingleDist on an AVX2 (non-AMX) amd64 host:
 * L2 D/l2.go:46-53 -> l2_256; dot D/dot_product.go:68-76 -> -dot_256;
 * cosine-dot D/cosine_dist.go:38-45 -> 1 - dot_256. */
ORC_API float orc_single_dist(int metric, const float *a, const float *b, long n)
{
    switch (metric) {
    case ORC_L2: return orc_l2_256(a, b, n);
    case ORC_DOT: return -orc_dot_256(a, b, n);
    case ORC_MANHATTAN: return orc_manhattan(a, b, n);      /* D/manhattan.go:51-58 */
    case ORC_HAMMING: return orc_hamming_256(a, b, n);      /* D/hamming.go:59-66 */
    default: return 1.0f - orc_dot_256(a, b, n);
    }
}

/* SingleDist as dispatched on AMX + AVX-512 hosts (D/l2_amd64.go:19-25,
 * D/dot_product_amd64.go:19-25): the 512 kernels, same Wrap. */
ORC_API float orc_single_dist_512(int metric, const float *a, const float *b, long n)
{
    switch (metric) {
    case ORC_L2: return orc_l2_512(a, b, n);
    case ORC_DOT: return -orc_dot_512(a, b, n);
    case ORC_MANHATTAN: return orc_manhattan(a, b, n);
    case ORC_HAMMING: return orc_hamming_256(a, b, n);  /* hamming_512 counts identically */
    default: return 1.0f - orc_dot_512(a, b, n);
    }
}

ORC_API void orc_dist_all_512(int metric, const float *q, const float *rows, long n, long d, float *out)
{
    for (long i = 0; i < n; i++) out[i] = orc_single_dist_512(metric, q, rows + i * d, d);
}

/* Provider.Wrap: L2 identity (D/l2.go:90-92), dot -x (D/dot_product.go:96-98),
 * cosine 1-x (D/cosine_dist.go:66-68), manhattan / hamming identity
 * (D/manhattan.go:80-82, D/hamming.go:88-90). */
ORC_API float orc_wrap(int metric, float x)
{
    switch (metric) {
    case ORC_DOT: return -x;
    case ORC_COSINE: return 1.0f - x;
    default: return x;
    }
}

ORC_API float orc_step(int metric, const float *a, const float *b, long n)
{
    switch (metric) {
    case ORC_L2: return orc_l2_step(a, b, n);
    case ORC_MANHATTAN: return orc_manhattan(a, b, n);
    case ORC_HAMMING: return orc_hamming_step(a, b, n);
    default: return orc_dot_step(a, b, n);
    }
}

/* distancer.Normalize: D/normalize.go:16-32.  Sequential unfused sum of
 * squares, float32(math.Sqrt(float64(norm))), element-wise division; zero
 * norm returns a zero vector. */
ORC_API void orc_normalize(const float *v, long n, float *out)
{
    float norm = 0.0f;
    for (long i = 0; i < n; i++) {
        float p = v[i] * v[i];
        norm += p;
    }
    if (norm == 0.0f) {
        for (long i = 0; i < n; i++) out[i] = 0.0f;
        return;
    }
    norm = (float)sqrt((double)norm);
    for (long i = 0; i < n; i++) out[i] = v[i] / norm;
}

/* ------------------------------------------------------------------------ */
/* Binary quantization                                                       */
/* ------------------------------------------------------------------------ */

/* BinaryQuantizer.Encode: CH/binary_quantization.go:32-45.  W = ceil(d/64)
 * words; bit j%64 of word j/64 set iff v[j] < 0 (the reference adds
 * uint64(math.Pow(2, j%64)), i.e. sets that bit once). */
ORC_API void orc_bq_encode(const float *v, long d, uint64_t *code)
{
    long w = (d + 63) / 64;
    for (long i = 0; i < w; i++) code[i] = 0;
    for (long j = 0; j < d; j++)
        if (v[j] < 0.0f) code[j / 64] += (uint64_t)1 << (j % 64);
}

/* BinaryQuantizer.DistanceBetweenCompressedVectors: CH/binary_quantization.go:47-56.
 * total += float32(bits.OnesCount64(x^y)) -- an exact small integer. */
ORC_API float orc_bq_distance(const uint64_t *x, const uint64_t *y, long w)
{
    float total = 0.0f;
    for (long i = 0; i < w; i++) total += (float)__builtin_popcountll(x[i] ^ y[i]);
    return total;
}

/* ------------------------------------------------------------------------ */
/* Product quantization                                                      */
/* ------------------------------------------------------------------------ */

/* DistanceLookUpTable filled for every (segment, code): CH/product_quantization.go:85-104
 * computes lut[i][c] = distance.Step(center_i, centroid_i[c]) lazily; the
 * values are identical whether filled lazily or eagerly.
 * centers layout: [m][ks][ds]. */
ORC_API void orc_pq_lut(int metric, const float *q, const float *centers,
                        long m, long ks, long ds, float *lut)
{
    for (long i = 0; i < m; i++)
        for (long c = 0; c < ks; c++)
            lut[i * ks + c] = orc_step(metric, q + i * ds, centers + (i * ks + c) * ds, ds);
}

/* LookUp / PQDistancer.Distance: CH/product_quantization.go:85-104, :352-361.
 * Sequential fp32 sum over segments, then Wrap. */
ORC_API float orc_pq_adc(int metric, const float *lut, const uint8_t *code, long m, long ks)
{
    float sum = 0.0f;
    for (long i = 0; i < m; i++) sum += lut[i * ks + code[i]];
    return orc_wrap(metric, sum);
}

/* ProductQuantizer.DistanceBetweenCompressedVectors (SDC): CH/product_quantization.go:297-311,
 * table from buildGlobalDistances :236-251 (Step(cX,cY), mirrored). */
ORC_API void orc_pq_global_distances(int metric, const float *centers, long m, long ks,
                                     long ds, float *table)
{
    for (long s = 0; s < m; s++)
        for (long i = 0; i < ks; i++)
            for (long j = 0; j <= i; j++) {
                float v = orc_step(metric, centers + (s * ks + i) * ds, centers + (s * ks + j) * ds, ds);
                table[s * ks * ks + i * ks + j] = v;
                table[s * ks * ks + j * ks + i] = v;
            }
}
ORC_API float orc_pq_sdc(int metric, const float *table, const uint8_t *x, const uint8_t *y,
                         long m, long ks)
{
    float dist = 0.0f;
    for (long i = 0; i < m; i++) dist += table[i * ks * ks + (long)x[i] * ks + y[i]];
    return orc_wrap(metric, dist);
}

/* KMeans.nNearest with n=1: CH/kmeans.go:111-135.  Distance is
 * L2SquaredProvider.SingleDist (kmeans.go:72,120) -> l2_256.  The candidate
 * replaces the best unless best < d, so ties go to the highest index and a
 * NaN distance replaces. */
ORC_API uint32_t orc_kmeans_nearest(const float *point_seg, const float *centers, long ks, long ds)
{
    uint32_t best = 0;
    float minD = FLT_MAX;
    for (long c = 0; c < ks; c++) {
        float d = orc_l2_256(point_seg, centers + c * ds, ds);
        if (!(minD < d)) {
            minD = d;
            best = (uint32_t)c;
        }
    }
    return best;
}

/* ProductQuantizer.Encode: CH/product_quantization.go:420-426 -> KMeans.Encode
 * per segment (kmeans.go:103-109). */
ORC_API void orc_pq_encode(const float *x, long n, long d, const float *centers,
                           long m, long ks, uint8_t *codes)
{
    long ds = d / m;
    for (long r = 0; r < n; r++)
        for (long s = 0; s < m; s++)
            codes[r * m + s] = (uint8_t)orc_kmeans_nearest(x + r * d + s * ds, centers + s * ks * ds, ks, ds);
}

/* The random draws of KMeans (rand.Intn(len(data)) at CH/kmeans.go:153,182).
 * Go's global math/rand is unseeded and shared by the concurrently fitted
 * segments, so the reference is not reproducible; both sides use this
 * counter stream keyed by (seed, segment) instead
 * (weaviate_amd/csrc/wvg_capi.hip kmeans_draw). */
static uint64_t mix64(uint64_t z);
static uint64_t orc_kmeans_draw(uint64_t seed, long s, uint64_t *ctr, uint64_t n)
{
    uint64_t h = mix64(mix64(seed + 0x632BE59BD9B4E019ull * (uint64_t)(s + 1)) + (*ctr)++);
    return h % n;
}

/* KMeans.Fit for one segment: CH/kmeans.go:220-250, with initCenters :146-160,
 * recluster :162-175, resortOnEmptySets :177-198, recalcCenters :200-213,
 * stopCondition :215-219.  cc[] is kept as append-only member lists exactly
 * like m.data.cc (a reseeded row stays in its old cluster's list).
 * centers: [ks][ds] out.  Returns the number of loop passes. */
static long orc_kmeans_fit_segment(const float *x, long n, long d, long seg, long ks, long ds, uint64_t seed,
                                   float *centers)
{
    uint64_t ctr = 0;
    for (long c = 0; c < ks; c++) { /* initCenters */
        uint64_t r = orc_kmeans_draw(seed, seg, &ctr, (uint64_t)n);
        memcpy(centers + c * ds, x + r * d + seg * ds, ds * sizeof(float));
    }
    uint64_t *points = calloc(n, sizeof(uint64_t));
    long *cc_len = malloc(ks * sizeof(long));
    long *cc_cap = malloc(ks * sizeof(long));
    uint64_t **cc = malloc(ks * sizeof(uint64_t *));
    for (long c = 0; c < ks; c++) { cc_cap[c] = 16; cc[c] = malloc(16 * sizeof(uint64_t)); }
#define CC_APPEND(ci, v) do { if (cc_len[ci] == cc_cap[ci]) { cc_cap[ci] *= 2; \
        cc[ci] = realloc(cc[ci], cc_cap[ci] * sizeof(uint64_t)); } cc[ci][cc_len[ci]++] = (v); } while (0)
    long changes = 1, passes = 0;
    for (long i = 0; changes > 0; i++) {
        passes++;
        changes = 0;
        for (long c = 0; c < ks; c++) cc_len[c] = 0;
        for (long p = 0; p < n; p++) { /* recluster */
            uint64_t ci = orc_kmeans_nearest(x + p * d + seg * ds, centers, ks, ds);
            CC_APPEND(ci, (uint64_t)p);
            if (points[p] != ci) { points[p] = ci; changes++; }
        }
        for (long ci = 0; ci < ks; ci++) { /* resortOnEmptySets */
            if (cc_len[ci] == 0) {
                uint64_t ri;
                for (;;) {
                    ri = orc_kmeans_draw(seed, seg, &ctr, (uint64_t)n);
                    if (cc_len[points[ri]] > 1) break;
                }
                CC_APPEND(ci, ri);
                points[ri] = (uint64_t)ci;
                changes = n;
            }
        }
        if (changes > 0) { /* recalcCenters */
            for (long c = 0; c < ks; c++) {
                for (long j = 0; j < ds; j++) centers[c * ds + j] = 0.0f;
                long size = cc_len[c];
                for (long t = 0; t < size; t++) {
                    const float *v = x + cc[c][t] * d + seg * ds;
                    for (long j = 0; j < ds; j++) centers[c * ds + j] += v[j];
                }
                for (long j = 0; j < ds; j++) centers[c * ds + j] /= (float)size;
            }
        }
        if (i >= 10 || changes < (long)((float)n * 0.01f)) break; /* stopCondition */
    }
#undef CC_APPEND
    for (long c = 0; c < ks; c++) free(cc[c]);
    free(cc); free(cc_len); free(cc_cap); free(points);
    return passes;
}

/* ProductQuantizer.Fit, k-means encoder: CH/product_quantization.go:372-418
 * (data truncated to trainingLimit; one KMeans per segment). */
ORC_API long orc_pq_fit(const float *x, long n, long d, long m, long ks, long training_limit, uint64_t seed,
                        float *centers, uint32_t *iterations)
{
    if (training_limit > 0 && n > training_limit) n = training_limit;
    if (n < ks) return -1; /* "not enough data to fit kmeans" */
    long ds = d / m;
    for (long s = 0; s < m; s++) {
        long it = orc_kmeans_fit_segment(x, n, d, s, ks, ds, seed, centers + s * ks * ds);
        if (iterations) iterations[s] = (uint32_t)it;
    }
    return 0;
}

/* ------------------------------------------------------------------------ */
/* Top-k: the reference's bounded max-heap                                   */
/* ------------------------------------------------------------------------ */

/* priorityqueue.Queue with NewMax less (a.Dist > b.Dist):
 * adapters/repos/db/priorityqueue/queue.go:43-147. */
typedef struct { uint64_t id; float dist; } orc_item;
typedef struct { orc_item *items; long len; } orc_heap;

static int heap_less(const orc_heap *h, long i, long j) { return h->items[i].dist > h->items[j].dist; }
static void heap_swap(orc_heap *h, long i, long j)
{
    orc_item t = h->items[i]; h->items[i] = h->items[j]; h->items[j] = t;
}
static void heap_insert(orc_heap *h, uint64_t id, float dist) /* queue.go:104-112 */
{
    h->items[h->len].id = id;
    h->items[h->len].dist = dist;
    long i = h->len++;
    while (i != 0 && heap_less(h, i, (i - 1) / 2)) {
        heap_swap(h, i, (i - 1) / 2);
        i = (i - 1) / 2;
    }
}
static void heap_heapify(orc_heap *h, long i) /* queue.go:130-147 */
{
    for (;;) {
        long left = 2 * i + 1, right = 2 * i + 2, smallest = i;
        if (left < h->len && heap_less(h, left, i)) smallest = left;
        if (right < h->len && heap_less(h, right, smallest)) smallest = right;
        if (smallest == i) return;
        heap_swap(h, i, smallest);
        i = smallest;
    }
}
static orc_item heap_pop(orc_heap *h) /* queue.go:53-59 */
{
    orc_item out = h->items[0];
    h->items[0] = h->items[h->len - 1];
    h->len--;
    heap_heapify(h, 0);
    return out;
}
/* flat.insertToHeap: V/flat/index.go:497-506 */
static void insert_to_heap(orc_heap *h, long limit, uint64_t id, float dist)
{
    if (h->len < limit) heap_insert(h, id, dist);
    else if (h->items[0].dist > dist) {
        heap_pop(h);
        heap_insert(h, id, dist);
    }
}
/* flat.extractHeap: V/flat/index.go:508-520 (ascending output). */
static long extract_heap(orc_heap *h, uint64_t *ids, float *dists)
{
    long len = h->len;
    for (long i = len - 1; i >= 0; i--) {
        orc_item it = heap_pop(h);
        ids[i] = it.id;
        dists[i] = it.dist;
    }
    return len;
}

/* Heap top-k over a precomputed distance stream visited in the given order
 * (ascending docID in the reference: V/flat/index.go:441-450).  valid[i]==0
 * rows are skipped (deleted / not allowed).  Returns the result count. */
ORC_API long orc_heap_topk(const float *dists, const uint64_t *ids, const uint8_t *valid,
                           long n, long k, uint64_t *out_ids, float *out_dists)
{
    if (k <= 0) return 0;
    orc_heap h = { (orc_item *)malloc(sizeof(orc_item) * (size_t)(k + 1)), 0 };
    for (long i = 0; i < n; i++)
        if (!valid || valid[i]) insert_to_heap(&h, k, ids[i], dists[i]);
    long cnt = extract_heap(&h, out_ids, out_dists);
    free(h.items);
    return cnt;
}

/* ------------------------------------------------------------------------ */
/* Flat scans (the CPU baseline and the search-level oracle)                 */
/* ------------------------------------------------------------------------ */

/* The reference kernels' own ABI (D/asm/l2_amd64.go:19-30 passes
 * x=query, y=candidate, &res, &len). */
typedef void (*orc_dist_fn)(float *, float *, float *, long *);

/* flat.searchByVector -> findTopVectors (V/flat/index.go:319-334, 411-452)
 * over a dense resident matrix (no LSM cursor / LE decode: favourable to the
 * CPU).  `fn` is the distance kernel (oracle restatement, or the reference's
 * own l2_256 / dot_256 / hamming_256 loaded from oracle/_ref); the metric's
 * Wrap is applied to its result (orc_wrap). */
ORC_API long orc_flat_search(const float *rows, long n, long d, long pitch, const uint8_t *valid,
                             const float *q, long k, int metric, orc_dist_fn fn,
                             uint64_t *out_ids, float *out_dists)
{
    if (k <= 0) return 0;
    orc_heap h = { (orc_item *)malloc(sizeof(orc_item) * (size_t)(k + 1)), 0 };
    for (long i = 0; i < n; i++) {
        if (valid && !valid[i]) continue;
        float dist;
        if (fn) {
            float r = 0.0f;
            long len = d;
            fn((float *)q, (float *)(rows + i * pitch), &r, &len);
            dist = orc_wrap(metric, r);
        } else {
            dist = orc_single_dist(metric, q, rows + i * pitch, d);
        }
        insert_to_heap(&h, k, (uint64_t)i, dist);
    }
    long cnt = extract_heap(&h, out_ids, out_dists);
    free(h.items);
    return cnt;
}

/* flat.searchByVectorBQ with the BQ cache path: V/flat/index.go:347-389,
 * findTopVectorsCached :456-495.  Hamming top-`rescore` heap over ascending
 * ids, pop all (descending Hamming order), exact distance for each popped id
 * and insertToHeap(k), then extractHeap.  `query` must already be normalized
 * for cosine (index.go:352).  Returns count. */
static long flat_search_bq_fn(const float *rows, const uint64_t *codes, long n, long d, long pitch,
                              const uint8_t *valid, const float *query, long k, long rescore_limit, int metric,
                              orc_dist_fn fn, uint64_t *out_ids, float *out_dists, uint64_t *cand_ids);

ORC_API long orc_flat_search_bq(const float *rows, const uint64_t *codes, long n, long d,
                                long pitch, const uint8_t *valid, const float *query,
                                long k, long rescore_limit, int metric,
                                uint64_t *out_ids, float *out_dists,
                                uint64_t *cand_ids /* optional, len >= rescore */)
{
    return flat_search_bq_fn(rows, codes, n, d, pitch, valid, query, k, rescore_limit, metric, NULL, out_ids,
                             out_dists, cand_ids);
}

/* The candidate half of searchByVectorBQ alone, over precomputed Hamming
 * distances of ids 0..n-1 (so a caller can stream a corpus too large for
 * one buffer of codes through orc_bq_dist_all): findTopVectorsCached's heap
 * of `rescore` over ascending ids (V/flat/index.go:456-495) and the pop loop
 * (:369-374).  Writes the ids / distances in pop order; returns the count. */
ORC_API long orc_heap_pops(const float *dists, long n, const uint8_t *valid, long rescore, uint64_t *out_ids,
                           float *out_dists)
{
    if (rescore <= 0) return 0;
    orc_heap h = { (orc_item *)malloc(sizeof(orc_item) * (size_t)(rescore + 1)), 0 };
    for (long i = 0; i < n; i++) {
        if (valid && !valid[i]) continue;
        insert_to_heap(&h, rescore, (uint64_t)i, dists[i]);
    }
    long nc = h.len;
    for (long i = 0; i < nc; i++) {
        orc_item it = heap_pop(&h);
        out_ids[i] = it.id;
        out_dists[i] = it.dist;
    }
    free(h.items);
    return nc;
}

/* The same with the rescore distance from `fn` (the reference's own l2_256 /
 * dot_256 from oracle/_ref in the CPU baseline), else the restatement. */
static long flat_search_bq_fn(const float *rows, const uint64_t *codes, long n, long d, long pitch,
                              const uint8_t *valid, const float *query, long k, long rescore_limit, int metric,
                              orc_dist_fn fn, uint64_t *out_ids, float *out_dists, uint64_t *cand_ids)
{
    long w = (d + 63) / 64;
    long rescore = rescore_limit > k ? rescore_limit : k; /* index.go:297-305 */
    if (k <= 0) return 0;
    uint64_t *qc = (uint64_t *)malloc(sizeof(uint64_t) * (size_t)w);
    orc_bq_encode(query, d, qc);
    orc_heap h = { (orc_item *)malloc(sizeof(orc_item) * (size_t)(rescore + 1)), 0 };
    for (long i = 0; i < n; i++) {
        if (valid && !valid[i]) continue;
        insert_to_heap(&h, rescore, (uint64_t)i, orc_bq_distance(codes + i * w, qc, w));
    }
    long nc = h.len;
    uint64_t *ids = (uint64_t *)malloc(sizeof(uint64_t) * (size_t)(nc + 1));
    for (long i = 0; i < nc; i++) ids[i] = heap_pop(&h).id;
    if (cand_ids) memcpy(cand_ids, ids, sizeof(uint64_t) * (size_t)nc);
    for (long i = 0; i < nc; i++) {
        float dist;
        if (fn) {
            float r = 0.0f;
            long len = d;
            fn((float *)query, (float *)(rows + ids[i] * pitch), &r, &len);
            dist = orc_wrap(metric, r);
        } else {
            dist = orc_single_dist(metric, query, rows + ids[i] * pitch, d);
        }
        insert_to_heap(&h, k, ids[i], dist);
    }
    long cnt = extract_heap(&h, out_ids, out_dists);
    free(ids); free(h.items); free(qc);
    return cnt;
}

/* ------------------------------------------------------------------------ */
/* Synthetic data: counter-based generator keyed by (seed, row, col).        */
/* Mirrors weaviate_amd/csrc/wvg_common.hpp wv_synth_value (product side);   */
/* tests check the GPU generator against this one bit-for-bit.               */
/* Distribution 0: uniform [-1,1) like V/testinghelpers/helpers.go:125-133;   */
/* 1: integers in [0,255] (SIFT-like, frequent ties).                         */
/* ------------------------------------------------------------------------ */
static uint64_t mix64(uint64_t z)
{
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
ORC_API float orc_synth_value(uint64_t seed, uint64_t row, uint64_t col, int dist)
{
    uint64_t h = mix64(mix64(seed) ^ ((row << 20) | (col & 0xFFFFF)));
    uint32_t u24 = (uint32_t)(h >> 40);
    if (dist == 1) return (float)(u24 >> 16);            /* 0..255 */
    return (float)u24 * (1.0f / 8388608.0f) - 1.0f;     /* k*2^-23 - 1, exact */
}
ORC_API void orc_synth_rows(uint64_t seed, uint64_t row0, long n, long d, long pitch, int dist,
                            float *out)
{
    for (long r = 0; r < n; r++)
        for (long c = 0; c < pitch; c++)
            out[r * pitch + c] = c < d ? orc_synth_value(seed, row0 + (uint64_t)r, (uint64_t)c, dist) : 0.0f;
}

/* ------------------------------------------------------------------------ */
/* CPU baseline driver: Q queries, one query per thread (CH/utils.go:25-42   */
/* Concurrently splits the index range across GOMAXPROCS workers).           */
/* ------------------------------------------------------------------------ */
typedef struct {
    const float *rows; const uint64_t *codes; long n, d, pitch; const float *qs; long k, rescore;
    int metric; orc_dist_fn fn;
    long q0, q1; uint64_t *out_ids; float *out_dists;
} orc_job;

static void *orc_worker(void *arg)
{
    orc_job *j = (orc_job *)arg;
    for (long q = j->q0; q < j->q1; q++) {
        if (j->codes)  /* BQ cache flow: Hamming top-R, exact rescore, top-k */
            flat_search_bq_fn(j->rows, j->codes, j->n, j->d, j->pitch, NULL, j->qs + q * j->d, j->k, j->rescore,
                              j->metric, j->fn, j->out_ids + q * j->k, j->out_dists + q * j->k, NULL);
        else
            orc_flat_search(j->rows, j->n, j->d, j->pitch, NULL, j->qs + q * j->d, j->k, j->metric,
                            j->fn, j->out_ids + q * j->k, j->out_dists + q * j->k);
    }
    return NULL;
}

static double run_jobs(orc_job proto, long nq, int threads)
{
    if (threads < 1) threads = 1;
    pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * (size_t)threads);
    orc_job *jobs = (orc_job *)malloc(sizeof(orc_job) * (size_t)threads);
    long split = (nq + threads - 1) / threads;
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (int t = 0; t < threads; t++) {
        long q0 = t * split, q1 = q0 + split;
        if (q1 > nq) q1 = nq;
        if (q0 > nq) q0 = nq;
        jobs[t] = proto;
        jobs[t].q0 = q0;
        jobs[t].q1 = q1;
        pthread_create(&th[t], NULL, orc_worker, &jobs[t]);
    }
    for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    free(th); free(jobs);
    return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}

/* Runs nq flat searches on `threads` threads; returns wall seconds. */
ORC_API double orc_bench_flat(const float *rows, long n, long d, long pitch, const float *qs,
                              long nq, long k, int metric, orc_dist_fn fn, int threads,
                              uint64_t *out_ids, float *out_dists)
{
    orc_job p = { rows, NULL, n, d, pitch, qs, k, 0, metric, fn, 0, 0, out_ids, out_dists };
    return run_jobs(p, nq, threads);
}

/* Runs nq flat BQ searches (findTopVectorsCached + rescore, V/flat/index.go:
 * 347-389, 456-495) over prebuilt codes [n][ceil(d/64)] (the BQ cache) on
 * `threads` threads; queries already normalized for cosine.  Wall seconds. */
ORC_API double orc_bench_flat_bq(const float *rows, const uint64_t *codes, long n, long d, long pitch,
                                 const float *qs, long nq, long k, long rescore_limit, int metric,
                                 orc_dist_fn fn, int threads, uint64_t *out_ids, float *out_dists)
{
    orc_job p = { rows, codes, n, d, pitch, qs, k, rescore_limit, metric, fn, 0, 0, out_ids, out_dists };
    return run_jobs(p, nq, threads);
}

/* PQ ADC top-k over a code matrix [n][m] for one query: the distancer's
 * LookUp table (CH/product_quantization.go:85-104, filled eagerly -- the
 * same values as the lazy fill), one ADC sum per row + Wrap (:352-361) in
 * ascending id order, insertToHeap(k), extractHeap (V/flat/index.go:441-452).
 * `lut` is caller scratch of m*ks floats.  Returns count. */
ORC_API long orc_pq_search(const uint8_t *codes, long n, long m, long ks, long ds, const float *centers,
                           const float *q, long k, int metric, float *lut, uint64_t *out_ids, float *out_dists)
{
    if (k <= 0) return 0;
    orc_pq_lut(metric, q, centers, m, ks, ds, lut);
    orc_heap h = { (orc_item *)malloc(sizeof(orc_item) * (size_t)(k + 1)), 0 };
    for (long i = 0; i < n; i++) insert_to_heap(&h, k, (uint64_t)i, orc_pq_adc(metric, lut, codes + i * m, m, ks));
    long cnt = extract_heap(&h, out_ids, out_dists);
    free(h.items);
    return cnt;
}

typedef struct {
    const uint8_t *codes; long n, m, ks, ds; const float *centers, *qs; long d, k; int metric;
    long q0, q1; uint64_t *out_ids; float *out_dists;
} orc_pq_job;

static void *orc_pq_worker(void *arg)
{
    orc_pq_job *j = (orc_pq_job *)arg;
    float *lut = (float *)malloc(sizeof(float) * (size_t)(j->m * j->ks));
    for (long q = j->q0; q < j->q1; q++)
        orc_pq_search(j->codes, j->n, j->m, j->ks, j->ds, j->centers, j->qs + q * j->d, j->k, j->metric, lut,
                      j->out_ids + q * j->k, j->out_dists + q * j->k);
    free(lut);
    return NULL;
}

/* Runs nq PQ ADC searches (orc_pq_search) on `threads` threads, one query per
 * thread at a time; returns wall seconds (the CPU leg of BASELINE configs[3]). */
ORC_API double orc_bench_pq(const uint8_t *codes, long n, long m, long ks, long ds, const float *centers,
                            const float *qs, long nq, long k, int metric, int threads, uint64_t *out_ids,
                            float *out_dists)
{
    if (threads < 1) threads = 1;
    pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * (size_t)threads);
    orc_pq_job *jobs = (orc_pq_job *)malloc(sizeof(orc_pq_job) * (size_t)threads);
    long split = (nq + threads - 1) / threads;
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (int t = 0; t < threads; t++) {
        long q0 = t * split, q1 = q0 + split;
        if (q1 > nq) q1 = nq;
        if (q0 > nq) q0 = nq;
        orc_pq_job p = { codes, n, m, ks, ds, centers, qs, m * ds, k, metric, q0, q1, out_ids, out_dists };
        jobs[t] = p;
        pthread_create(&th[t], NULL, orc_pq_worker, &jobs[t]);
    }
    for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    free(th); free(jobs);
    return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}

/* BinaryQuantizer.Encode of n rows into codes [n][ceil(d/64)] (test helper). */
ORC_API void orc_bq_encode_rows(const float *rows, long n, long d, uint64_t *codes)
{
    long w = (d + 63) / 64;
    for (long i = 0; i < n; i++) orc_bq_encode(rows + i * d, d, codes + i * w);
}

/* Provider.SingleDist(q, rows[i]) for every row (test helper; AVX2-order
 * kernels as dispatched on non-AMX amd64, D/l2_amd64.go:19-25). */
ORC_API void orc_dist_all(int metric, const float *q, const float *rows, long n, long d, float *out)
{
    for (long i = 0; i < n; i++) out[i] = orc_single_dist(metric, q, rows + i * d, d);
}

/* BinaryQuantizer Hamming of q against every code row (test helper). */
ORC_API void orc_bq_dist_all(const uint64_t *q, const uint64_t *codes, long n, long w, float *out)
{
    for (long i = 0; i < n; i++) out[i] = orc_bq_distance(codes + i * w, q, w);
}
