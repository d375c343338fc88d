// wvg_pqfit.hip -- ProductQuantizer.Fit (CH/product_quantization.go:372-418):
// per segment KMeans.Fit (CH/kmeans.go:146-250) with the Lloyd passes on
// the device (K9 assignment + K10 count / members / sums, wvg_pq.hip) and
// the reseeding / stop control on the host.

#include "wvg_host.hpp"

namespace wvg {

// Draw j of segment s's random stream: stands in for Go's global math/rand
// (rand.Intn(len(data)) at CH/kmeans.go:153,182), which is unseeded and shared
// by the concurrently fitted segments, so no run of the reference is
// reproducible.  oracle/wv_oracle.c orc_kmeans_draw is the same function.
static uint64_t kmeans_draw(uint64_t seed, uint32_t s, uint64_t &ctr, uint64_t n)
{
    const uint64_t h = wvg_mix64(wvg_mix64(seed + 0x632BE59BD9B4E019ull * (uint64_t)(s + 1)) + ctr++);
    return h % n;
}

}  // namespace wvg

using namespace wvg;

extern "C" {

int wvg_pq_fit(wvg_ctx *ctx, const float *X, uint64_t n, uint32_t dim, uint32_t m, uint32_t ks,
               uint64_t training_limit, uint64_t seed, float *out_centers, uint32_t *out_iterations)
{
    if (!ctx || !out_centers || (n && !X)) return fail(WVG_ERR_INVALID, "null argument");
    int rc = pq_validate(m, ks, dim);
    if (rc) return rc;
    if (training_limit > 0 && n > training_limit) n = training_limit;  // product_quantization.go:373-375
    if (n < ks) return fail(WVG_ERR_INVALID, "not enough data to fit kmeans");  // kmeans.go:222-224
    if (n > 0xFFFFFFFFull) return fail(WVG_ERR_INVALID, "too many training rows");
    WVG_HIP(hipSetDevice(ctx->device));
    const uint32_t ds = dim / m, nch = f32_chunks(dim);
    const size_t nc = (size_t)m * ks * ds;
    Carver cv;
    const size_t o_x = cv.take(n * dim * 4), o_xt = cv.take(tiles_of(n) * 64 * (size_t)nch * 16),
                 o_c = cv.take(pq_centers_alloc_bytes(m, ks, ds)), o_p = cv.take(n * m), o_code = cv.take(n * m),
                 o_mem = cv.take(n * m * 4), o_off = cv.take((size_t)m * ks * 4),
                 o_cnt = cv.take((size_t)m * ks * 4), o_chg = cv.take((size_t)m * 4), o_act = cv.take(m),
                 o_rec = cv.take(m), o_skip = cv.take((size_t)m * ks),
                 o_bh = cv.take((size_t)m * kmeans_blocks(n) * ks * 4), o_nan = cv.take((size_t)m * 4);
    Bulk bk(ctx);
    rc = bk.begin(cv.off);
    if (rc) return rc;
    hipStream_t s = bk.s();
    float *dX = (float *)(bk.b + o_x), *dXt = (float *)(bk.b + o_xt), *dC = (float *)(bk.b + o_c);
    uint8_t *dP = (uint8_t *)(bk.b + o_p), *dCode = (uint8_t *)(bk.b + o_code);
    uint32_t *dMem = (uint32_t *)(bk.b + o_mem), *dOff = (uint32_t *)(bk.b + o_off);
    uint32_t *dCnt = (uint32_t *)(bk.b + o_cnt), *dChg = (uint32_t *)(bk.b + o_chg);
    uint8_t *dAct = (uint8_t *)(bk.b + o_act), *dRec = (uint8_t *)(bk.b + o_rec), *dSkip = (uint8_t *)(bk.b + o_skip);
    uint32_t *dBh = (uint32_t *)(bk.b + o_bh), *dNan = (uint32_t *)(bk.b + o_nan);
    WVG_HIP(hipMemcpyAsync(dX, X, n * dim * 4, hipMemcpyHostToDevice, s));
    // the training rows in the tiled layout K9 (the assignment) reads
    WVG_HIP(hipMemsetAsync(dXt, 0, tiles_of(n) * 64 * (size_t)nch * 16, s));
    WVG_HIP(launch_f32_store(dX, nullptr, n, dim, nch, 0, dXt, s));
    const bool pairs = pq_has_pairs(ks, ds);
    // K9's ds = 4 pair copy of the current centers and their per-segment NaN flags (a segment
    // without NaN centroids takes K9's min3 argmin; its rows' NaNs are checked per wave)
    WVG_HIP(hipMemsetAsync(dNan, 0xFF, (size_t)m * 4, s));
    auto refresh_pairs = [&]() -> hipError_t {
        return pairs ? launch_pq_pairs(dC, m, ks, dC + nc, s, dNan) : hipSuccess;
    };
    // initCenters (kmeans.go:146-160): ks random rows (with replacement) per segment
    std::vector<float> C(nc);
    std::vector<uint64_t> ctr(m, 0);
    for (uint32_t sg = 0; sg < m; sg++)
        for (uint32_t c = 0; c < ks; c++) {
            const uint64_t r = kmeans_draw(seed, sg, ctr[sg], n);
            std::memcpy(&C[((size_t)sg * ks + c) * ds], X + r * dim + (size_t)sg * ds, ds * 4);
        }
    WVG_HIP(hipMemcpyAsync(dC, C.data(), nc * 4, hipMemcpyHostToDevice, s));
    WVG_HIP(refresh_pairs());
    WVG_HIP(hipMemsetAsync(dP, 0, n * m, s));  // data.points = make([]uint64, n): all zero (kept [m][n])
    std::vector<uint8_t> active(m, 1), rec(m), skip((size_t)m * ks);
    std::vector<uint32_t> cnt((size_t)m * ks), chg(m), iters(m, 0);
    std::vector<uint8_t> hp;  // host copy of points ([m][n]), only when a reseed needs it
    const int thresh = (int)((float)n * 0.01f);  // int(float32(dataSize) * DeltaThreshold), kmeans.go:217-219
    for (uint32_t it = 0;; it++) {
        bool any = false;
        for (uint32_t sg = 0; sg < m; sg++) any |= active[sg] != 0;
        if (!any) break;
        WVG_HIP(hipMemcpyAsync(dAct, active.data(), m, hipMemcpyHostToDevice, s));
        WVG_HIP(hipMemsetAsync(dCnt, 0, (size_t)m * ks * 4, s));
        WVG_HIP(hipMemsetAsync(dChg, 0, (size_t)m * 4, s));
        // nNearest for every (row, segment): K9, the encoder (kmeans.go:103-135; ties to the
        // highest index); then changes and cluster sizes of the active segments
        WVG_HIP(launch_pq_encode(dXt, n, dim, dC, m, ks, dCode, s, false, false, pairs ? dNan : nullptr));
        WVG_HIP(launch_kmeans_count(dCode, n, m, ks, dAct, dP, dChg, dCnt, dBh, s));
        WVG_HIP(hipMemcpyAsync(cnt.data(), dCnt, cnt.size() * 4, hipMemcpyDeviceToHost, s));
        WVG_HIP(hipMemcpyAsync(chg.data(), dChg, chg.size() * 4, hipMemcpyDeviceToHost, s));
        WVG_HIP(hipStreamSynchronize(s));
        // resortOnEmptySets (kmeans.go:177-198): an empty cluster takes a random
        // row whose cluster has more than one member; the row stays counted in
        // its old cluster's sum (cc is append-only) but points[ri] moves.
        std::fill(skip.begin(), skip.end(), 0);
        std::vector<std::pair<uint64_t, std::pair<uint32_t, uint32_t>>> moves;  // (row, (segment, cluster))
        bool fetched = false;
        for (uint32_t sg = 0; sg < m; sg++) {
            if (!active[sg]) continue;
            uint32_t *sz = &cnt[(size_t)sg * ks];
            std::vector<uint32_t> size(sz, sz + ks);
            for (uint32_t ci = 0; ci < ks; ci++) {
                if (size[ci] != 0) continue;
                if (!fetched) {
                    hp.resize(n * m);
                    WVG_HIP(hipMemcpy(hp.data(), dP, n * m, hipMemcpyDeviceToHost));
                    fetched = true;
                }
                uint64_t ri;
                for (;;) {
                    ri = kmeans_draw(seed, sg, ctr[sg], n);
                    if (size[hp[(size_t)sg * n + ri]] > 1) break;
                }
                size[ci] = 1;
                hp[(size_t)sg * n + ri] = (uint8_t)ci;
                skip[(size_t)sg * ks + ci] = 1;
                moves.push_back({ri, {sg, ci}});
                for (uint32_t j = 0; j < ds; j++)  // recalcCenters over cc[ci] = {ri}: (0 + x) / float32(1)
                    C[((size_t)sg * ks + ci) * ds + j] = (0.0f + X[ri * dim + (size_t)sg * ds + j]) / 1.0f;
                chg[sg] = (uint32_t)n;  // data.changes = dataSize
            }
        }
        for (uint32_t sg = 0; sg < m; sg++) rec[sg] = active[sg] && chg[sg] > 0;
        WVG_HIP(hipMemcpyAsync(dRec, rec.data(), m, hipMemcpyHostToDevice, s));
        WVG_HIP(hipMemcpyAsync(dSkip, skip.data(), skip.size(), hipMemcpyHostToDevice, s));
        // recalcCenters with the recluster assignment (the reseeded rows still
        // in their old clusters), then the reseeded clusters = their one row
        WVG_HIP(launch_kmeans_recalc2(dX, n, dim, dP, m, ks, ds, dRec, dCnt, dBh, dSkip, dMem, dOff, dC, s));
        for (auto &mv : moves) {
            const uint32_t sg = mv.second.first, ci = mv.second.second;
            const uint8_t code = (uint8_t)ci;
            WVG_HIP(hipMemcpyAsync(dC + ((size_t)sg * ks + ci) * ds, &C[((size_t)sg * ks + ci) * ds], ds * 4,
                                   hipMemcpyHostToDevice, s));
            WVG_HIP(hipMemcpyAsync(dP + (size_t)sg * n + mv.first, &code, 1, hipMemcpyHostToDevice, s));
            WVG_HIP(hipStreamSynchronize(s));  // `code` is a stack byte
        }
        WVG_HIP(refresh_pairs());
        for (uint32_t sg = 0; sg < m; sg++) {
            if (!active[sg]) continue;
            iters[sg] = it + 1;
            // stopCondition (kmeans.go:215-219) or the loop test changes > 0 (:232)
            if (it >= 10 || (int)chg[sg] < thresh || chg[sg] == 0) active[sg] = 0;
        }
    }
    WVG_HIP(hipMemcpyAsync(out_centers, dC, nc * 4, hipMemcpyDeviceToHost, s));
    WVG_HIP(hipStreamSynchronize(s));
    if (out_iterations) std::memcpy(out_iterations, iters.data(), m * 4);
    return WVG_OK;
}

}  // extern "C"
