// wvg_range.hip -- unbounded selections (wvg_select.hip kernels S1-S4): top-k
// for k > 256, BQ rescore windows above 256 and the range search of
// SearchByVectorDistance (V/flat/index.go:531-591, V/hnsw/search.go:85-151).
// One query at a time; every phase in HBM.

#include "wvg_host.hpp"

namespace wvg {


// Device buffers of the selection flow over `nslots` slots.
struct SelectBufs {
    uint32_t *keys = nullptr;           // [nslots] ordered distance keys
    void *st = nullptr;                 // radix-select state
    uint32_t *hist = nullptr;           // 4096 bins
    unsigned long long *cnt = nullptr;  // [4] counters
    uint64_t *cmp = nullptr;            // [nslots] compacted keys
    uint64_t *sorted = nullptr;         // [nslots] sorted keys
    void *temp = nullptr;
    size_t temp_bytes = 0;
    static void layout(Carver &cv, uint64_t nslots, size_t o[6], size_t &temp_bytes)
    {
        temp_bytes = sort_temp_bytes(nslots);
        o[0] = cv.take(nslots * 4);
        o[1] = cv.take(select_state_bytes());
        o[2] = cv.take(4096 * 4);
        o[3] = cv.take(4 * 8);
        o[4] = cv.take(nslots * 8);
        o[5] = cv.take(nslots * 8);
    }
    void bind(char *b, const size_t o[6], size_t o_temp, size_t tb)
    {
        keys = (uint32_t *)(b + o[0]);
        st = b + o[1];
        hist = (uint32_t *)(b + o[2]);
        cnt = (unsigned long long *)(b + o[3]);
        cmp = (uint64_t *)(b + o[4]);
        sorted = (uint64_t *)(b + o[5]);
        temp = b + o_temp;
        temp_bytes = tb;
    }
};

// Compacts live keys <= threshold (st_dev: the radix-select result, else thr)
// and sorts them; returns how many there are.
static int compact_sort(const SelectBufs &sb, uint64_t nslots, const void *st_dev, uint32_t thr, uint32_t slot0,
                        int num_cus, hipStream_t s, uint64_t *n_out)
{
    WVG_HIP(launch_key_compact(sb.keys, nslots, st_dev, thr, slot0, num_cus, sb.cmp, sb.cnt, s));
    unsigned long long n = 0;
    WVG_HIP(hipMemcpyAsync(&n, sb.cnt, 8, hipMemcpyDeviceToHost, s));
    WVG_HIP(hipStreamSynchronize(s));
    WVG_HIP(sort_keys64(sb.temp, sb.temp_bytes, sb.cmp, sb.sorted, n, s));
    *n_out = n;
    return WVG_OK;
}

// The `want` smallest (distance, slot) keys of one prepared query, ascending,
// in sb.sorted; *n_out = min(want, live allowed rows).
static int select_smallest(const wvg_corpus *c, const ScanArgs &a1, uint64_t want, const SelectBufs &sb,
                           hipStream_t s, uint64_t *n_out)
{
    const int cus = c->ctx->num_cus;
    const uint64_t nslots = (a1.tile_end - a1.tile_begin) * 64;
    WVG_HIP(launch_ordkeys(a1, c->kind, cus, sb.keys, s));
    uint64_t n = 0;
    int rc;
    if (want >= nslots) {
        rc = compact_sort(sb, nslots, nullptr, 0xFFFFFFFEu, (uint32_t)(a1.tile_begin * 64), cus, s, &n);
    } else {
        WVG_HIP(launch_select_kth(sb.keys, nslots, want, cus, sb.st, sb.hist, s));
        rc = compact_sort(sb, nslots, sb.st, 0u, (uint32_t)(a1.tile_begin * 64), cus, s, &n);
    }
    if (rc) return rc;
    *n_out = std::min<uint64_t>(n, want);
    return WVG_OK;
}

// Element size of one prepared query row (F32 / PQ LUT floats, BQ words).
static size_t query_elem_bytes(const wvg_corpus *c) { return c->kind == WVG_KIND_BQ ? 8 : 4; }

// wvg_search for k > 256: S1-S4 per query.
int search_large_k(wvg_corpus *c, const float *queries, uint32_t nq, uint32_t k, const uint64_t *allow_bits,
                          uint64_t allow_words, const SearchPlan &p, uint64_t *out_ids, float *out_dists,
                          uint32_t *out_counts)
{
    SlotGuard g(c->ctx);
    int rc = c->ctx->acquire(&g.slot);
    if (rc) return rc;
    const uint64_t nslots = (p.te - p.tb) * 64;
    Carver cv;
    const size_t o_q = cv.take(query_bytes(c, nq));
    const size_t o_qtmp = cv.take(c->kind == WVG_KIND_PQ ? (size_t)nq * c->dim * 4 : 0);
    const size_t o_allow = cv.take(p.allow_bytes());
    size_t o_sel[6], temp_bytes = 0;
    SelectBufs::layout(cv, nslots, o_sel, temp_bytes);
    const size_t o_temp = cv.take(temp_bytes);
    const size_t o_ids = cv.take((size_t)k * 8), o_d = cv.take((size_t)k * 4);
    void *base = nullptr;
    rc = g.slot->device_scratch(cv.off, &base);
    if (rc) return rc;
    char *b = (char *)base;
    hipStream_t s = g.slot->stream;
    uint32_t qpitch = 0;
    rc = stage_queries(c, g.slot, queries, nq, b + o_q, qpitch, (float *)(b + o_q), b + o_qtmp);
    if (rc) return rc;
    const uint64_t *d_allow = nullptr;
    if (p.allow_host) {
        WVG_HIP(hipMemcpyAsync(b + o_allow, p.allow_host, p.allow_bytes(), hipMemcpyHostToDevice, s));
        d_allow = (const uint64_t *)(b + o_allow);
    }
    SelectBufs sb;
    sb.bind(b, o_sel, o_temp, temp_bytes);
    for (uint32_t qi = 0; qi < nq; qi++) {
        const void *dq = b + o_q + (size_t)qi * qpitch * query_elem_bytes(c);
        ScanArgs a1 = scan_args_for(c, dq, qpitch, 1, k, d_allow, p.tb, p.te);
        uint64_t n = 0;
        rc = select_smallest(c, a1, k, sb, s, &n);
        if (rc) return rc;
        WVG_HIP(launch_emit_sorted(sb.sorted, n, c->id_base, (uint64_t *)(b + o_ids), (float *)(b + o_d), s));
        if (out_ids && n) WVG_HIP(hipMemcpyAsync(out_ids + (size_t)qi * k, b + o_ids, n * 8, hipMemcpyDeviceToHost, s));
        if (out_dists && n)
            WVG_HIP(hipMemcpyAsync(out_dists + (size_t)qi * k, b + o_d, n * 4, hipMemcpyDeviceToHost, s));
        WVG_HIP(hipStreamSynchronize(s));
        for (uint64_t i = n; i < k; i++) {
            if (out_ids) out_ids[(size_t)qi * k + i] = WVG_KEY_NONE;
            if (out_dists) out_dists[(size_t)qi * k + i] = INFINITY;
        }
        if (out_counts) out_counts[qi] = (uint32_t)n;
    }
    return WVG_OK;
}

// Largest ordered key o in [ord(-inf), ord(+inf)] with pred(unord(o)), for a
// predicate that is true up to some distance and false above it; 0 (below
// every real key) if it holds nowhere.
template <typename Pred>
static uint32_t max_ord_where(Pred pred)
{
    uint32_t lo = wvg_ord_f32(-INFINITY), hi = wvg_ord_f32(INFINITY);
    if (!pred(wvg_unord_f32(lo))) return 0u;
    while (lo < hi) {
        const uint32_t mid = lo + (hi - lo + 1) / 2;
        if (pred(wvg_unord_f32(mid)))
            lo = mid;
        else
            hi = mid - 1;
    }
    return lo;
}

// flat.searchByVectorBQ with a rescore window above 256: per query the
// Hamming top-R by S1-S4, the exact rescore of those R rows, a sort, top-k.
int bq_rescore_large(wvg_corpus *bq, wvg_corpus *f32, const float *queries, uint32_t nq, uint32_t k,
                            uint32_t R, const uint64_t *allow_bits, uint64_t allow_words, const SearchPlan &p,
                            uint64_t *out_ids, float *out_dists, uint32_t *out_counts)
{
    SlotGuard g(bq->ctx);
    int rc = bq->ctx->acquire(&g.slot);
    if (rc) return rc;
    const uint32_t fpitch = f32_chunks(bq->dim) * 4;
    const uint64_t nslots = (p.te - p.tb) * 64;
    Carver cv;
    const size_t o_qb = cv.take(query_bytes(bq, nq));
    const size_t o_qf = cv.take((size_t)nq * fpitch * 4);
    const size_t o_allow = cv.take(p.allow_bytes());
    size_t o_sel[6], temp_bytes = 0;
    SelectBufs::layout(cv, nslots, o_sel, temp_bytes);
    const size_t o_temp = cv.take(temp_bytes);
    const size_t o_resc = cv.take((size_t)R * 8), o_rs = cv.take((size_t)R * 8);
    const size_t o_ids = cv.take((size_t)k * 8), o_d = cv.take((size_t)k * 4);
    void *base = nullptr;
    rc = g.slot->device_scratch(cv.off, &base);
    if (rc) return rc;
    char *b = (char *)base;
    hipStream_t s = g.slot->stream;
    uint32_t qpb = 0, qpf = 0;
    rc = stage_queries(bq, g.slot, queries, nq, b + o_qb, qpb, nullptr, nullptr);
    if (rc) return rc;
    rc = stage_queries(f32, g.slot, queries, nq, b + o_qf, qpf, nullptr, nullptr);
    if (rc) return rc;
    const uint64_t *d_allow = nullptr;
    if (p.allow_host) {
        WVG_HIP(hipMemcpyAsync(b + o_allow, p.allow_host, p.allow_bytes(), hipMemcpyHostToDevice, s));
        d_allow = (const uint64_t *)(b + o_allow);
    }
    SelectBufs sb;
    sb.bind(b, o_sel, o_temp, temp_bytes);
    for (uint32_t qi = 0; qi < nq; qi++) {
        ScanArgs a1 = scan_args_for(bq, b + o_qb + (size_t)qi * qpb * 8, qpb, 1, R, d_allow, p.tb, p.te);
        uint64_t n = 0;
        rc = select_smallest(bq, a1, R, sb, s, &n);
        if (rc) return rc;
        // sb.sorted[0..n) = Hamming top-R keys (slot in the low 32 bits)
        WVG_HIP(launch_rescore_keys(f32->metric, (const float *)(b + o_qf) + (size_t)qi * qpf, qpf,
                                    (const float *)f32->d_data, f32->dim, f32->nchunks, sb.sorted, 1, (uint32_t)n,
                                    (uint32_t)n, (uint64_t *)(b + o_resc), s, f32->ctx->order512));
        WVG_HIP(sort_keys64(sb.temp, sb.temp_bytes, (uint64_t *)(b + o_resc), (uint64_t *)(b + o_rs), n, s));
        const uint64_t kk = std::min<uint64_t>(k, n);
        WVG_HIP(launch_emit_sorted((uint64_t *)(b + o_rs), kk, f32->id_base, (uint64_t *)(b + o_ids),
                                   (float *)(b + o_d), s));
        if (out_ids && kk) WVG_HIP(hipMemcpyAsync(out_ids + (size_t)qi * k, b + o_ids, kk * 8, hipMemcpyDeviceToHost, s));
        if (out_dists && kk)
            WVG_HIP(hipMemcpyAsync(out_dists + (size_t)qi * k, b + o_d, kk * 4, hipMemcpyDeviceToHost, s));
        WVG_HIP(hipStreamSynchronize(s));
        for (uint64_t i = kk; i < k; i++) {
            if (out_ids) out_ids[(size_t)qi * k + i] = WVG_KEY_NONE;
            if (out_dists) out_dists[(size_t)qi * k + i] = INFINITY;
        }
        if (out_counts) out_counts[qi] = (uint32_t)kk;
    }
    return WVG_OK;
}

// findTopVectorsCached's heap of R > 256 and its pop order (V/flat/index.go:
// 355-374), exactly (the heap replay of wvg_replay.hip for windows the scan's
// register top-k cannot hold): S1 keys of every slot; chunks of the slot
// window doubling from R (chunk 0 = [0, R), chunk j = [R 2^(j-1), R 2^j)), each
// with thr[j] = the R-th smallest key before it (a radix select over the
// prefix; no threshold while fewer than R live rows precede); the slots of
// chunk j below thr[j] are a superset of the rows the heap inserts there
// (about R per chunk, R (1 + log2(rows / R)) in all), compacted, sorted into
// docID order, copied back and replayed through the heap on the host.
size_t select_replay_bytes(const SearchPlan &p)
{
    const uint64_t nslots = (p.te - p.tb) * 64;
    Carver cv;
    size_t o[6], temp_bytes = 0;
    SelectBufs::layout(cv, nslots, o, temp_bytes);
    cv.take(temp_bytes);
    cv.take(65 * 4);
    return cv.off;
}

int bq_heap_candidates_select(wvg_corpus *bq, StreamSlot *sl, const void *d_qb, uint32_t qpb, uint32_t nq,
                              uint32_t R, const uint64_t *d_allow, const SearchPlan &p, char *ws,
                              std::vector<std::vector<GoItem>> &pops)
{
    hipStream_t s = sl->stream;
    const int cus = bq->ctx->num_cus;
    const uint64_t nslots = (p.te - p.tb) * 64;
    Carver cv;
    size_t o_sel[6], temp_bytes = 0;
    SelectBufs::layout(cv, nslots, o_sel, temp_bytes);
    const size_t o_temp = cv.take(temp_bytes), o_thr = cv.take(65 * 4);
    SelectBufs sb;
    sb.bind(ws, o_sel, o_temp, temp_bytes);
    uint32_t *d_thr = (uint32_t *)(ws + o_thr);
    pops.assign(nq, {});
    std::vector<uint64_t> keys;
    for (uint32_t qi = 0; qi < nq; qi++) {
        ScanArgs a1 = scan_args_for(bq, (const uint64_t *)d_qb + (size_t)qi * qpb, qpb, 1, R, d_allow, p.tb, p.te);
        WVG_HIP(launch_ordkeys(a1, bq->kind, cus, sb.keys, s));
        uint32_t thr[65];
        thr[0] = 0xFFFFFFFFu;  // chunk 0: no row precedes -- keep every live one
        bool enough = false;   // R live rows precede the chunk (then for every later chunk too)
        int J = 1;
        for (; J < 64 && ((uint64_t)R << (J - 1)) < nslots; J++) {
            const uint64_t b = (uint64_t)R << (J - 1);
            if (!enough) {
                WVG_HIP(launch_key_count(sb.keys, b, 0u, 0u, cus, sb.cnt, s));
                unsigned long long cnt[3] = {0, 0, 0};
                WVG_HIP(hipMemcpyAsync(cnt, sb.cnt, sizeof(cnt), hipMemcpyDeviceToHost, s));
                WVG_HIP(hipStreamSynchronize(s));
                enough = cnt[2] >= R;
            }
            thr[J] = 0xFFFFFFFFu;
            if (enough) {
                WVG_HIP(launch_select_kth(sb.keys, b, R, cus, sb.st, sb.hist, s));
                WVG_HIP(read_select_kth(sb.st, &thr[J], s));
            }
        }
        WVG_HIP(hipMemcpyAsync(d_thr, thr, (size_t)J * 4, hipMemcpyHostToDevice, s));
        WVG_HIP(launch_key_compact_chunks(sb.keys, nslots, d_thr, R, (uint32_t)(p.tb * 64), cus, sb.cmp, sb.cnt, s));
        unsigned long long n = 0;
        WVG_HIP(hipMemcpyAsync(&n, sb.cnt, 8, hipMemcpyDeviceToHost, s));
        WVG_HIP(hipStreamSynchronize(s));  // (also keeps `thr` alive until its copy is done)
        WVG_HIP(sort_keys64(sb.temp, sb.temp_bytes, sb.cmp, sb.sorted, n, s));
        keys.resize(n);
        if (n) WVG_HIP(hipMemcpyAsync(keys.data(), sb.sorted, n * 8, hipMemcpyDeviceToHost, s));
        WVG_HIP(hipStreamSynchronize(s));
        GoMaxHeap h(R);
        for (uint64_t i = 0; i < n; i++)
            insert_to_heap(h, R, (uint32_t)(keys[i] >> 32), wvg_unord_f32((uint32_t)keys[i]));
        pops[qi].reserve(h.len());
        while (h.len()) pops[qi].push_back(h.pop());
    }
    return WVG_OK;
}

// How many of the ascending results SearchByVectorDistance returns, given
// p_le = #rows with dist <= target, p_q = #rows kept by the threshold test
// (dist <= target || InDelta 1e-6), live = #rows.  Restates the growing-limit
// loop: limits 100, 1100, 11100, ... (V/common/search_by_dist_params.go:14-83),
// continue while the last row of the window is <= target, stop before a
// limit above max_limit (V/hnsw/search.go:85-151, the loop flat's
// V/flat/index.go:531-591 intends).
uint64_t range_result_count(uint64_t p_le, uint64_t p_q, uint64_t live, int64_t max_limit)
{
    uint64_t offset = 0, limit = 100, total = 100, searched = 100;
    for (;;) {
        const uint64_t hi = std::min(total, live), lo = std::min(offset, live);
        if (lo == hi) break;                  // empty window
        if (!(hi - 1 < p_le)) break;          // last found > target
        offset = total;
        limit *= 10;
        total = offset + limit;
        if (max_limit >= 0 && (int64_t)total > max_limit) break;
        searched = total;
    }
    return std::min(p_q, std::min(searched, live));
}

}  // namespace wvg

using namespace wvg;

extern "C" {

int wvg_search_by_distance(wvg_corpus *c, const float *query, float target_distance, int64_t max_limit,
                           const uint64_t *allow_bits, uint64_t allow_words, uint64_t *out_ids, float *out_dists,
                           uint64_t out_capacity, uint64_t *out_count)
{
    int rc = check_corpus(c);
    if (rc) return rc;
    if (!query || !out_count) return fail(WVG_ERR_INVALID, "null argument");
    if (c->kind == WVG_KIND_PQ && !c->d_centers) return fail(WVG_ERR_INVALID, "PQ corpus has no codebook");
    *out_count = 0;
    std::shared_lock<std::shared_mutex> lk(c->rw);
    SearchPlan p = plan_search(c, 1, 1, allow_bits, allow_words);
    if (p.empty) return WVG_OK;
    SlotGuard g(c->ctx);
    rc = c->ctx->acquire(&g.slot);
    if (rc) return rc;
    const uint64_t nslots = (p.te - p.tb) * 64;
    Carver cv;
    const size_t o_q = cv.take(query_bytes(c, 1));
    const size_t o_qtmp = cv.take(c->kind == WVG_KIND_PQ ? (size_t)c->dim * 4 : 0);
    const size_t o_allow = cv.take(p.allow_bytes());
    size_t o_sel[6], temp_bytes = 0;
    SelectBufs::layout(cv, nslots, o_sel, temp_bytes);
    const size_t o_temp = cv.take(temp_bytes);
    const size_t o_ids = cv.take(nslots * 8), o_d = cv.take(nslots * 4);
    void *base = nullptr;
    rc = g.slot->device_scratch(cv.off, &base);
    if (rc) return rc;
    char *b = (char *)base;
    hipStream_t s = g.slot->stream;
    uint32_t qpitch = 0;
    rc = stage_queries(c, g.slot, query, 1, b + o_q, qpitch, (float *)(b + o_q), b + o_qtmp);
    if (rc) return rc;
    const uint64_t *d_allow = nullptr;
    if (p.allow_host) {
        WVG_HIP(hipMemcpyAsync(b + o_allow, p.allow_host, p.allow_bytes(), hipMemcpyHostToDevice, s));
        d_allow = (const uint64_t *)(b + o_allow);
    }
    SelectBufs sb;
    sb.bind(b, o_sel, o_temp, temp_bytes);
    const int cus = c->ctx->num_cus;
    ScanArgs a1 = scan_args_for(c, b + o_q, qpitch, 1, 1, d_allow, p.tb, p.te);
    WVG_HIP(launch_ordkeys(a1, c->kind, cus, sb.keys, s));
    const float t = target_distance;
    const uint32_t t_le = max_ord_where([t](float d) { return d <= t; });
    const uint32_t t_q = max_ord_where([t](float d) {
        return d <= t || std::fabs((double)d - (double)t) <= 1e-6;  // floatcomp.InDelta
    });
    WVG_HIP(launch_key_count(sb.keys, nslots, t_le, t_q, cus, sb.cnt, s));
    unsigned long long cnt[3] = {0, 0, 0};
    WVG_HIP(hipMemcpyAsync(cnt, sb.cnt, sizeof(cnt), hipMemcpyDeviceToHost, s));
    WVG_HIP(hipStreamSynchronize(s));
    const uint64_t R = range_result_count(cnt[0], cnt[1], cnt[2], max_limit);
    *out_count = R;
    if (R == 0) return WVG_OK;
    uint64_t n = 0;
    rc = compact_sort(sb, nslots, nullptr, t_q, (uint32_t)(p.tb * 64), cus, s, &n);
    if (rc) return rc;
    const uint64_t ncopy = std::min<uint64_t>(R, out_capacity);
    if (ncopy == 0) return WVG_OK;
    WVG_HIP(launch_emit_sorted(sb.sorted, ncopy, c->id_base, (uint64_t *)(b + o_ids), (float *)(b + o_d), s));
    if (out_ids) WVG_HIP(hipMemcpyAsync(out_ids, b + o_ids, ncopy * 8, hipMemcpyDeviceToHost, s));
    if (out_dists) WVG_HIP(hipMemcpyAsync(out_dists, b + o_d, ncopy * 4, hipMemcpyDeviceToHost, s));
    WVG_HIP(hipStreamSynchronize(s));
    return WVG_OK;
}

int wvg_search_by_distance_window(wvg_corpus *c, const float *query, float target_distance, uint32_t window,
                                  const uint64_t *allow_bits, uint64_t allow_words, uint64_t *out_ids,
                                  float *out_dists, uint64_t out_capacity, uint64_t *out_count)
{
    if (!c || !query || !out_count) return fail(WVG_ERR_INVALID, "null argument");
    *out_count = 0;
    if (window == 0) return WVG_OK;
    // the first window of flat.SearchByVectorDistance's loop: SearchByVector(q, window)
    // (V/flat/index.go:539-542), then the rows up to the first beyond the target (:555-567)
    std::vector<uint64_t> ids(window);
    std::vector<float> d(window);
    uint32_t cnt = 0;
    int rc = wvg_search(c, query, 1, window, allow_bits, allow_words, ids.data(), d.data(), &cnt);
    if (rc) return rc;
    uint64_t n = 0;
    for (uint32_t i = 0; i < cnt; i++) {
        const bool keep = d[i] <= target_distance || std::fabs((double)d[i] - (double)target_distance) <= 1e-6;
        if (!keep) break;  // floatcomp.InDelta (usecases/floatcomp/delta.go:16-19)
        if (n < out_capacity) {
            if (out_ids) out_ids[n] = ids[i];
            if (out_dists) out_dists[n] = d[i];
        }
        n++;
    }
    *out_count = n;
    return WVG_OK;
}

}  // extern "C"
