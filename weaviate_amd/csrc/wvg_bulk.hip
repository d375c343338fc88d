// wvg_bulk.hip -- bulk primitives of the C ABI over host buffers
// (distancer.Provider / compressionhelpers bulk ops): distances, normalize,
// BQ / PQ encode and distances, the BQ rescore over host rows, the SDC table
// and the synthetic-row generator.

#include "wvg_host.hpp"

namespace wvg {

int pq_validate(uint32_t m, uint32_t ks, uint32_t dim)
{
    if (m == 0) return fail(WVG_ERR_INVALID, "segments cannot be 0 nor negative");
    if (ks > 256)
        return fail(WVG_ERR_INVALID,
                    "centroids should not be higher than 256. Attempting to use " + std::to_string(ks));
    if (ks == 0) return fail(WVG_ERR_INVALID, "centroids must be > 0");
    if (dim % m != 0) return fail(WVG_ERR_INVALID, "segments should be an integer divisor of dimensions");
    return WVG_OK;
}

}  // namespace wvg

using namespace wvg;

extern "C" {

int wvg_rescore(wvg_ctx *ctx, int metric, const float *q, const float *rows, const uint64_t *ids, uint64_t n,
                uint32_t dim, uint32_t k, uint64_t *out_ids, float *out_dists, uint32_t *out_count)
{
    if (!ctx || !q || (n && (!rows || !ids))) return fail(WVG_ERR_INVALID, "null argument");
    if (metric < WVG_METRIC_L2 || metric > WVG_METRIC_HAMMING) return fail(WVG_ERR_INVALID, "unknown metric");
    if (n > 0xFFFFFFFFull) return fail(WVG_ERR_INVALID, "too many rows");
    if (out_count) *out_count = 0;
    if (n == 0 || k == 0 || dim == 0) return WVG_OK;
    WVG_HIP(hipSetDevice(ctx->device));
    const uint32_t nch = f32_chunks(dim);
    Carver cv;
    const size_t o_x = cv.take(n * dim * 4), o_t = cv.take(tiles_of(n) * 64 * (size_t)nch * 16),
                 o_q = cv.take((size_t)nch * 16), o_k = cv.take(n * 8), o_i = cv.take((size_t)k * 8),
                 o_d = cv.take((size_t)k * 4), o_c = cv.take(4);
    const bool large = !ctx->opt.heap_replay && k > MAX_K;  // beyond the fused top-k: sort the n keys
    const size_t temp_bytes = large ? sort_temp_bytes(n) : 0;
    const size_t o_s = cv.take(large ? n * 8 : 0), o_tmp = cv.take(temp_bytes);
    Bulk bk(ctx);
    int rc = bk.begin(cv.off);
    if (rc) return rc;
    // host rows, query and results go through the slot's pinned staging: a
    // pageable hipMemcpyAsync is a staged, blocking copy (the caller's R rows
    // are the rescore's only sizeable transfer)
    const size_t rows_b = n * dim * 4, q_b = (size_t)nch * 16, out_b = o_c + 4 - o_i;
    const bool rows_pinned = host_pinned_ptr(rows);  // a wvg_host_alloc buffer: copied from directly
    Staging st;
    rc = st.reserve(bk.g.slot, (rows_pinned ? 0 : stage_bytes(rows_b)) + stage_bytes(q_b) + stage_bytes(out_b));
    if (rc) return rc;
    WVG_HIP(st.h2d(bk.b + o_x, rows, rows_b, bk.s()));
    std::vector<float> qp((size_t)nch * 4, 0.0f);
    std::memcpy(qp.data(), q, (size_t)dim * 4);
    WVG_HIP(st.h2d(bk.b + o_q, qp.data(), q_b, bk.s()));
    WVG_HIP(launch_f32_store((const float *)(bk.b + o_x), nullptr, n, dim, nch, 0, (float *)(bk.b + o_t), bk.s()));
    WVG_HIP(launch_dist_keys(metric, (const float *)(bk.b + o_q), (const float *)(bk.b + o_t), n, dim,
                             (uint64_t *)(bk.b + o_k), bk.s(), ctx->order512));
    if (ctx->opt.heap_replay) {
        // the rescore loop's own heap (V/flat/index.go:375-387): every distance back,
        // inserted in input order into a heap of k on the host, then extracted
        std::vector<uint64_t> keys(n);
        WVG_HIP(hipMemcpyAsync(keys.data(), bk.b + o_k, n * 8, hipMemcpyDeviceToHost, bk.s()));
        WVG_HIP(hipStreamSynchronize(bk.s()));
        GoMaxHeap h(std::min<uint64_t>(k, n));
        for (uint64_t i = 0; i < n; i++) insert_to_heap(h, k, ids[i], wvg_unord_f32((uint32_t)(keys[i] >> 32)));
        std::vector<uint64_t> oi(h.len());
        std::vector<float> od(h.len());
        const size_t cnt = extract_heap(h, oi.data(), od.data());
        for (uint32_t i = 0; i < k; i++) {
            if (out_ids) out_ids[i] = i < cnt ? oi[i] : WVG_KEY_NONE;
            if (out_dists) out_dists[i] = i < cnt ? od[i] : INFINITY;
        }
        if (out_count) *out_count = (uint32_t)cnt;
        return WVG_OK;
    }
    if (large) {
        const uint32_t kk = (uint32_t)std::min<uint64_t>(k, n);
        WVG_HIP(sort_keys64(bk.b + o_tmp, temp_bytes, (const uint64_t *)(bk.b + o_k), (uint64_t *)(bk.b + o_s), n,
                            bk.s()));
        WVG_HIP(launch_emit_sorted((const uint64_t *)(bk.b + o_s), kk, 0, (uint64_t *)(bk.b + o_i),
                                   (float *)(bk.b + o_d), bk.s()));
        std::vector<float> inf(k - kk, INFINITY);  // tail: no entry (KEY_NONE id, +inf)
        WVG_HIP(hipMemcpyAsync(bk.b + o_c, &kk, 4, hipMemcpyHostToDevice, bk.s()));
        if (kk < k) {
            WVG_HIP(hipMemsetAsync(bk.b + o_i + (size_t)kk * 8, 0xFF, (size_t)(k - kk) * 8, bk.s()));
            WVG_HIP(hipMemcpyAsync(bk.b + o_d + (size_t)kk * 4, inf.data(), inf.size() * 4, hipMemcpyHostToDevice,
                                   bk.s()));
        }
        WVG_HIP(hipStreamSynchronize(bk.s()));  // the host sources above are stack buffers
    } else {
        WVG_HIP(launch_merge_keys((const uint64_t *)(bk.b + o_k), 1, (uint32_t)n, k, 0, (uint64_t *)(bk.b + o_i),
                                  (float *)(bk.b + o_d), (uint32_t *)(bk.b + o_c), bk.s()));
    }
    // one copy of the [ids | dists | count] span back through the staging
    char *pin = st.take(out_b);
    WVG_HIP(hipMemcpyAsync(pin, bk.b + o_i, out_b, hipMemcpyDeviceToHost, bk.s()));
    WVG_HIP(hipStreamSynchronize(bk.s()));
    const uint64_t *idx = (const uint64_t *)pin;
    uint32_t cnt = 0;
    std::memcpy(&cnt, pin + (o_c - o_i), 4);
    if (out_dists) std::memcpy(out_dists, pin + (o_d - o_i), (size_t)k * 4);
    for (uint32_t i = 0; i < k; i++)  // row index -> caller's docID
        if (out_ids) out_ids[i] = i < cnt ? ids[idx[i]] : WVG_KEY_NONE;
    if (out_count) *out_count = cnt;
    return WVG_OK;
}

int wvg_synthetic_rows(wvg_ctx *ctx, uint64_t seed, const uint64_t *ids, uint64_t n, uint32_t dim, int distribution,
                       int normalize, float *out)
{
    if (!ctx || (n && (!ids || !out))) return fail(WVG_ERR_INVALID, "null argument");
    if (n == 0 || dim == 0) return WVG_OK;
    WVG_HIP(hipSetDevice(ctx->device));
    Carver cv;
    const size_t o_i = cv.take(n * 8), o_o = cv.take(n * dim * 4);
    Bulk bk(ctx);
    int rc = bk.begin(cv.off);
    if (rc) return rc;
    Staging st;
    rc = st.reserve(bk.g.slot, stage_bytes(n * 8));
    if (rc) return rc;
    WVG_HIP(st.h2d(bk.b + o_i, ids, n * 8, bk.s()));
    WVG_HIP(launch_synth_rows(seed, distribution, (const uint64_t *)(bk.b + o_i), n, dim, normalize,
                              (float *)(bk.b + o_o), bk.s()));
    WVG_HIP(hipMemcpyAsync(out, bk.b + o_o, n * dim * 4, hipMemcpyDeviceToHost, bk.s()));
    WVG_HIP(hipStreamSynchronize(bk.s()));
    return WVG_OK;
}

// ---------------------------------------------------------------------------
// Bulk primitives
// ---------------------------------------------------------------------------

int wvg_distance_batch(wvg_ctx *ctx, int metric, const float *q, const float *X, uint64_t n, uint32_t dim, float *out)
{
    if (!ctx || !q || (n && (!X || !out))) return fail(WVG_ERR_INVALID, "null argument");
    if (metric < WVG_METRIC_L2 || metric > WVG_METRIC_HAMMING) return fail(WVG_ERR_INVALID, "unknown metric");
    if (n == 0 || dim == 0) return WVG_OK;
    WVG_HIP(hipSetDevice(ctx->device));
    const uint32_t nch = f32_chunks(dim);
    Carver cv;
    const size_t o_x = cv.take(n * dim * 4), o_t = cv.take(tiles_of(n) * 64 * (size_t)nch * 16),
                 o_q = cv.take((size_t)nch * 16), o_o = cv.take(n * 4);
    Bulk bk(ctx);
    int rc = bk.begin(cv.off);
    if (rc) return rc;
    std::vector<float> qp((size_t)nch * 4, 0.0f);
    std::memcpy(qp.data(), q, (size_t)dim * 4);
    Staging st;  // rows (up to STAGE_MAX), query and distances through the slot's pinned staging
    rc = st.reserve(bk.g.slot, stage_bytes(n * dim * 4) + stage_bytes(qp.size() * 4) + stage_bytes(n * 4));
    if (rc) return rc;
    WVG_HIP(st.h2d(bk.b + o_x, X, n * dim * 4, bk.s()));
    WVG_HIP(st.h2d(bk.b + o_q, qp.data(), qp.size() * 4, bk.s()));
    WVG_HIP(launch_f32_store((const float *)(bk.b + o_x), nullptr, n, dim, nch, 0, (float *)(bk.b + o_t), bk.s()));
    WVG_HIP(launch_distance_rows(metric, (const float *)(bk.b + o_q), (const float *)(bk.b + o_t), n, dim,
                                 (float *)(bk.b + o_o), bk.s(), ctx->order512));
    char *pin = n * 4 <= STAGE_MAX ? st.take(n * 4) : nullptr;
    WVG_HIP(hipMemcpyAsync(pin ? (void *)pin : (void *)out, bk.b + o_o, n * 4, hipMemcpyDeviceToHost, bk.s()));
    WVG_HIP(hipStreamSynchronize(bk.s()));
    if (pin) std::memcpy(out, pin, n * 4);
    return WVG_OK;
}

int wvg_normalize_batch(wvg_ctx *ctx, const float *X, uint64_t n, uint32_t dim, float *out)
{
    if (!ctx || (n && (!X || !out))) return fail(WVG_ERR_INVALID, "null argument");
    if (n == 0 || dim == 0) return WVG_OK;
    WVG_HIP(hipSetDevice(ctx->device));
    Carver cv;
    const size_t o_x = cv.take(n * dim * 4), o_o = cv.take(n * dim * 4);
    Bulk bk(ctx);
    int rc = bk.begin(cv.off);
    if (rc) return rc;
    // in and out through the slot's pinned staging (see wvg_rescore) up to
    // STAGE_MAX; larger inputs are copied straight from / to the caller's
    // buffers (pageable copies), so a bulk normalize never pins its whole
    // input for the life of the context
    const size_t bytes = n * dim * 4;
    const bool direct = stage_bytes(bytes) == 0 || host_pinned_ptr(X);
    Staging st;
    rc = st.reserve(bk.g.slot, direct ? 0 : stage_bytes(bytes));
    if (rc) return rc;
    WVG_HIP(st.h2d(bk.b + o_x, X, bytes, bk.s()));
    WVG_HIP(launch_normalize_rows((const float *)(bk.b + o_x), n, dim, (float *)(bk.b + o_o), bk.s()));
    if (direct || host_pinned_ptr(out)) {
        WVG_HIP(hipMemcpyAsync(out, bk.b + o_o, bytes, hipMemcpyDeviceToHost, bk.s()));
        WVG_HIP(hipStreamSynchronize(bk.s()));
        return WVG_OK;
    }
    char *pin = st.p;  // the input's staging piece, free again once the input copy has run
    WVG_HIP(hipMemcpyAsync(pin, bk.b + o_o, bytes, hipMemcpyDeviceToHost, bk.s()));
    WVG_HIP(hipStreamSynchronize(bk.s()));
    std::memcpy(out, pin, bytes);
    return WVG_OK;
}

int wvg_bq_encode(wvg_ctx *ctx, const float *X, uint64_t n, uint32_t dim, uint64_t *out_words)
{
    if (!ctx || (n && (!X || !out_words))) return fail(WVG_ERR_INVALID, "null argument");
    if (n == 0 || dim == 0) return WVG_OK;
    WVG_HIP(hipSetDevice(ctx->device));
    const uint32_t w = bq_words(dim);
    Carver cv;
    const size_t o_x = cv.take(n * dim * 4), o_o = cv.take(n * w * 8);
    Bulk bk(ctx);
    int rc = bk.begin(cv.off);
    if (rc) return rc;
    WVG_HIP(hipMemcpyAsync(bk.b + o_x, X, n * dim * 4, hipMemcpyHostToDevice, bk.s()));
    WVG_HIP(launch_bq_encode_rows((const float *)(bk.b + o_x), n, dim, 0, (uint64_t *)(bk.b + o_o), bk.s()));
    WVG_HIP(hipMemcpyAsync(out_words, bk.b + o_o, n * w * 8, hipMemcpyDeviceToHost, bk.s()));
    WVG_HIP(hipStreamSynchronize(bk.s()));
    return WVG_OK;
}

int wvg_bq_distance_batch(wvg_ctx *ctx, const uint64_t *q, const uint64_t *codes, uint64_t n, uint32_t words,
                          float *out)
{
    if (!ctx || !q || (n && (!codes || !out))) return fail(WVG_ERR_INVALID, "null argument");
    if (n == 0) return WVG_OK;
    WVG_HIP(hipSetDevice(ctx->device));
    Carver cv;
    const size_t o_q = cv.take((size_t)words * 8), o_c = cv.take(n * words * 8), o_o = cv.take(n * 4);
    Bulk bk(ctx);
    int rc = bk.begin(cv.off);
    if (rc) return rc;
    WVG_HIP(hipMemcpyAsync(bk.b + o_q, q, (size_t)words * 8, hipMemcpyHostToDevice, bk.s()));
    WVG_HIP(hipMemcpyAsync(bk.b + o_c, codes, n * words * 8, hipMemcpyHostToDevice, bk.s()));
    WVG_HIP(launch_bq_distance_rows((const uint64_t *)(bk.b + o_q), (const uint64_t *)(bk.b + o_c), n, words,
                                    (float *)(bk.b + o_o), bk.s()));
    WVG_HIP(hipMemcpyAsync(out, bk.b + o_o, n * 4, hipMemcpyDeviceToHost, bk.s()));
    WVG_HIP(hipStreamSynchronize(bk.s()));
    return WVG_OK;
}

int wvg_pq_encode(wvg_ctx *ctx, const float *centers, uint32_t m, uint32_t ks, const float *X, uint64_t n,
                  uint32_t dim, uint8_t *out_codes)
{
    if (!ctx || !centers || (n && (!X || !out_codes))) return fail(WVG_ERR_INVALID, "null argument");
    int rc = pq_validate(m, ks, dim);
    if (rc) return rc;
    if (n == 0) return WVG_OK;
    WVG_HIP(hipSetDevice(ctx->device));
    const uint32_t nch = f32_chunks(dim), ds = dim / m;
    Carver cv;
    const size_t o_x = cv.take(n * dim * 4), o_t = cv.take(tiles_of(n) * 64 * (size_t)nch * 16),
                 o_c = cv.take(pq_centers_alloc_bytes(m, ks, ds)), o_o = cv.take(n * m);
    Bulk bk(ctx);
    rc = bk.begin(cv.off);
    if (rc) return rc;
    std::vector<float> pairs(pq_has_pairs(ks, ds) ? (size_t)m * ks * ds : 0);
    if (!pairs.empty()) pq_pair_layout(centers, m, ks, pairs.data());
    WVG_HIP(hipMemcpyAsync(bk.b + o_x, X, n * dim * 4, hipMemcpyHostToDevice, bk.s()));
    WVG_HIP(hipMemcpyAsync(bk.b + o_c, centers, (size_t)m * ks * ds * 4, hipMemcpyHostToDevice, bk.s()));
    if (!pairs.empty())
        WVG_HIP(hipMemcpyAsync(bk.b + o_c + (size_t)m * ks * ds * 4, pairs.data(), pairs.size() * 4,
                               hipMemcpyHostToDevice, bk.s()));
    WVG_HIP(launch_f32_store((const float *)(bk.b + o_x), nullptr, n, dim, nch, 0, (float *)(bk.b + o_t), bk.s()));
    WVG_HIP(launch_pq_encode((const float *)(bk.b + o_t), n, dim, (const float *)(bk.b + o_c), m, ks,
                             (uint8_t *)(bk.b + o_o), bk.s(), false, pq_nan_free(centers, (size_t)m * ks * ds)));
    WVG_HIP(hipMemcpyAsync(out_codes, bk.b + o_o, n * m, hipMemcpyDeviceToHost, bk.s()));
    WVG_HIP(hipStreamSynchronize(bk.s()));
    return WVG_OK;
}

int wvg_pq_lut(wvg_ctx *ctx, int metric, const float *centers, uint32_t m, uint32_t ks, uint32_t dim, const float *q,
               float *out_lut)
{
    if (!ctx || !centers || !q || !out_lut) return fail(WVG_ERR_INVALID, "null argument");
    int rc = pq_validate(m, ks, dim);
    if (rc) return rc;
    WVG_HIP(hipSetDevice(ctx->device));
    const uint32_t ds = dim / m;
    Carver cv;
    const size_t o_q = cv.take((size_t)dim * 4), o_c = cv.take((size_t)m * ks * ds * 4),
                 o_o = cv.take((size_t)m * ks * 4);
    Bulk bk(ctx);
    rc = bk.begin(cv.off);
    if (rc) return rc;
    WVG_HIP(hipMemcpyAsync(bk.b + o_q, q, (size_t)dim * 4, hipMemcpyHostToDevice, bk.s()));
    WVG_HIP(hipMemcpyAsync(bk.b + o_c, centers, (size_t)m * ks * ds * 4, hipMemcpyHostToDevice, bk.s()));
    WVG_HIP(launch_pq_lut(metric, (const float *)(bk.b + o_q), 1, dim, (const float *)(bk.b + o_c), m, ks, ds,
                          (float *)(bk.b + o_o), bk.s()));
    WVG_HIP(hipMemcpyAsync(out_lut, bk.b + o_o, (size_t)m * ks * 4, hipMemcpyDeviceToHost, bk.s()));
    WVG_HIP(hipStreamSynchronize(bk.s()));
    return WVG_OK;
}

int wvg_pq_adc_batch(wvg_ctx *ctx, int metric, const float *lut, uint32_t m, uint32_t ks, const uint8_t *codes,
                     uint64_t n, float *out)
{
    if (!ctx || !lut || (n && (!codes || !out))) return fail(WVG_ERR_INVALID, "null argument");
    if (n == 0) return WVG_OK;
    WVG_HIP(hipSetDevice(ctx->device));
    Carver cv;
    const size_t o_l = cv.take((size_t)m * ks * 4), o_c = cv.take(n * m), o_o = cv.take(n * 4);
    Bulk bk(ctx);
    int rc = bk.begin(cv.off);
    if (rc) return rc;
    WVG_HIP(hipMemcpyAsync(bk.b + o_l, lut, (size_t)m * ks * 4, hipMemcpyHostToDevice, bk.s()));
    WVG_HIP(hipMemcpyAsync(bk.b + o_c, codes, n * m, hipMemcpyHostToDevice, bk.s()));
    WVG_HIP(launch_pq_adc_rows(metric, (const float *)(bk.b + o_l), m, ks, (const uint8_t *)(bk.b + o_c), n,
                               (float *)(bk.b + o_o), bk.s()));
    WVG_HIP(hipMemcpyAsync(out, bk.b + o_o, n * 4, hipMemcpyDeviceToHost, bk.s()));
    WVG_HIP(hipStreamSynchronize(bk.s()));
    return WVG_OK;
}

int wvg_pq_global_distances(wvg_ctx *ctx, int metric, const float *centers, uint32_t m, uint32_t ks, uint32_t dim,
                            float *out_table)
{
    if (!ctx || !centers || !out_table) return fail(WVG_ERR_INVALID, "null argument");
    int rc = pq_validate(m, ks, dim);
    if (rc) return rc;
    WVG_HIP(hipSetDevice(ctx->device));
    const uint32_t ds = dim / m;
    const size_t tab = (size_t)m * ks * ks;
    Carver cv;
    const size_t o_c = cv.take((size_t)m * ks * ds * 4), o_t = cv.take(tab * 4);
    Bulk bk(ctx);
    rc = bk.begin(cv.off);
    if (rc) return rc;
    WVG_HIP(hipMemcpyAsync(bk.b + o_c, centers, (size_t)m * ks * ds * 4, hipMemcpyHostToDevice, bk.s()));
    WVG_HIP(launch_pq_sdc_table(metric, (const float *)(bk.b + o_c), m, ks, ds, (float *)(bk.b + o_t), bk.s()));
    WVG_HIP(hipMemcpyAsync(out_table, bk.b + o_t, tab * 4, hipMemcpyDeviceToHost, bk.s()));
    WVG_HIP(hipStreamSynchronize(bk.s()));
    return WVG_OK;
}

int wvg_pq_sdc_batch(wvg_ctx *ctx, int metric, const float *table, uint32_t m, uint32_t ks, const uint8_t *x,
                     const uint8_t *codes, uint64_t n, float *out)
{
    if (!ctx || !table || !x || (n && (!codes || !out))) return fail(WVG_ERR_INVALID, "null argument");
    if (n == 0) return WVG_OK;
    WVG_HIP(hipSetDevice(ctx->device));
    const size_t tab = (size_t)m * ks * ks;
    Carver cv;
    const size_t o_t = cv.take(tab * 4), o_x = cv.take(m), o_c = cv.take(n * m), o_o = cv.take(n * 4);
    Bulk bk(ctx);
    int rc = bk.begin(cv.off);
    if (rc) return rc;
    WVG_HIP(hipMemcpyAsync(bk.b + o_t, table, tab * 4, hipMemcpyHostToDevice, bk.s()));
    WVG_HIP(hipMemcpyAsync(bk.b + o_x, x, m, hipMemcpyHostToDevice, bk.s()));
    WVG_HIP(hipMemcpyAsync(bk.b + o_c, codes, n * m, hipMemcpyHostToDevice, bk.s()));
    WVG_HIP(launch_pq_sdc_rows(metric, (const float *)(bk.b + o_t), m, ks, (const uint8_t *)(bk.b + o_x),
                               (const uint8_t *)(bk.b + o_c), n, (float *)(bk.b + o_o), bk.s()));
    WVG_HIP(hipMemcpyAsync(out, bk.b + o_o, n * 4, hipMemcpyDeviceToHost, bk.s()));
    WVG_HIP(hipStreamSynchronize(bk.s()));
    return WVG_OK;
}

}  // extern "C"
