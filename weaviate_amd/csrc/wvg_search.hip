// wvg_search.hip -- search planning and dispatch: flat.SearchByVector /
// searchByVector (V/flat/index.go:307-334), searchByVectorBQ + rescore
// (:347-389), the device-pointer and query-stream searches, the shard merge
// (adapters/repos/db/index.go:1644-1648) and DistanceToNode by docID
// (CH/compression.go:306-325).

#include <atomic>
#include <chrono>

#include "wvg_host.hpp"

namespace wvg {

// distancer.Normalize (D/normalize.go:16-32) on the host for queries; this
// translation unit is compiled with -ffp-contract=off.
static void normalize_host(const float *v, uint32_t n, float *out)
{
    float norm = 0.0f;
    for (uint32_t i = 0; i < n; i++) {
        float p = v[i] * v[i];
        norm = norm + p;
    }
    if (norm == 0.0f) {
        for (uint32_t i = 0; i < n; i++) out[i] = 0.0f;
        return;
    }
    norm = (float)std::sqrt((double)norm);
    for (uint32_t i = 0; i < n; i++) out[i] = v[i] / norm;
}

// normalize_host over nq rows (out pitch `pitch`), eight rows at a time: each
// row's sum of squares is still its own sequential chain, but eight chains run
// side by side (one chain of d dependent adds per query bounded a 1024 x 768
// batch's host preparation at ~0.5 ms).
static void normalize_host_rows(const float *v, uint32_t nq, uint32_t d, float *out, uint32_t pitch)
{
    constexpr uint32_t B = 8;
    uint32_t i = 0;
    for (; i + B <= nq; i += B) {
        const float *r = v + (size_t)i * d;
        float norm[B];
        for (uint32_t j = 0; j < B; j++) norm[j] = 0.0f;
        for (uint32_t e = 0; e < d; e++)
            for (uint32_t j = 0; j < B; j++) {
                const float x = r[(size_t)j * d + e];
                const float p = x * x;
                norm[j] = norm[j] + p;
            }
        for (uint32_t j = 0; j < B; j++) {
            const float *src = r + (size_t)j * d;
            float *dst = out + (size_t)(i + j) * pitch;
            if (norm[j] == 0.0f) {
                for (uint32_t e = 0; e < d; e++) dst[e] = 0.0f;
                continue;
            }
            const float n = (float)std::sqrt((double)norm[j]);
            for (uint32_t e = 0; e < d; e++) dst[e] = src[e] / n;
        }
    }
    for (; i < nq; i++) normalize_host(v + (size_t)i * d, d, out + (size_t)i * pitch);
}

// BinaryQuantizer.Encode (CH/binary_quantization.go:32-45).
static void bq_encode_host(const float *v, uint32_t d, uint64_t *code, uint32_t words)
{
    for (uint32_t i = 0; i < words; i++) code[i] = 0;
    for (uint32_t j = 0; j < d; j++)
        if (v[j] < 0.0f) code[j / 64] |= 1ull << (j % 64);
}

// Allow bitmap -> tile range [tb, te) of slots that can be allowed; false if
// empty.  Only the words of this corpus's own docID window are read (the
// bitmap is over global docIDs and word w covers docIDs 64w..64w+63, so the
// word of tile t is id_base/64 + t): O(corpus tiles) host work however large
// the docID space is; the scan then gets the words of [tb, te) only.
bool allow_tile_range(const wvg_corpus *c, const uint64_t *allow, uint64_t allow_words, uint64_t &tb,
                             uint64_t &te)
{
    const uint64_t hw_tiles = tiles_of(c->high_water);
    tb = 0;
    te = hw_tiles;
    if (!allow) return hw_tiles > 0;
    const uint64_t wb = c->id_base / 64;
    if (allow_words <= wb) return false;
    const uint64_t n = std::min(allow_words - wb, hw_tiles);
    const uint64_t *w = allow + wb;
    uint64_t first = 0;
    while (first < n && !w[first]) first++;
    if (first == n) return false;  // allow.IsEmpty() (here: for this corpus) -> nothing (V/flat/index.go:425-427)
    uint64_t last = n - 1;
    while (!w[last]) last--;
    tb = first;
    te = last + 1;
    return true;
}

// Queries -> the device-side representation the scan of this corpus reads.
// F32: [nq][qpitch] floats (normalized for cosine).  BQ: [nq][qpitch] words.
// PQ: raw floats are staged at qf and turned into LUTs by the caller.
void prepare_queries_host(const wvg_corpus *c, const float *queries, uint32_t nq, std::vector<float> &qf,
                                 std::vector<uint64_t> &qb, uint32_t &qpitch)
{
    const uint32_t d = c->dim;
    std::vector<float> tmp(d);
    if (c->kind == WVG_KIND_BQ) {
        const uint32_t words = bq_words(d);
        qpitch = bq_chunks(d) * 2;
        qb.assign((size_t)nq * qpitch, 0ull);
        for (uint32_t i = 0; i < nq; i++) {
            const float *q = queries + (size_t)i * d;
            if (c->metric == WVG_METRIC_COSINE) {
                normalize_host(q, d, tmp.data());
                q = tmp.data();
            }
            bq_encode_host(q, d, qb.data() + (size_t)i * qpitch, words);
        }
        return;
    }
    qpitch = c->kind == WVG_KIND_F32 ? f32_chunks(d) * 4 : d;
    qf.assign((size_t)nq * qpitch, 0.0f);
    if (c->metric == WVG_METRIC_COSINE) {
        normalize_host_rows(queries, nq, d, qf.data(), qpitch);
        return;
    }
    for (uint32_t i = 0; i < nq; i++) std::memcpy(qf.data() + (size_t)i * qpitch, queries + (size_t)i * d, sizeof(float) * d);
}

static hipError_t launch_scan(const ScanArgs &a, int kind, uint64_t *partials, int groups, hipStream_t s)
{
    switch (kind) {
    case WVG_KIND_F32: return launch_scan_f32(a, partials, groups, s);
    case WVG_KIND_BQ: return launch_scan_bq(a, partials, groups, s);
    default: return launch_scan_pq(a, partials, groups, s);
    }
}

// Direction of the next scan of `c`: consecutive scans alternate (serpentine),
// so a scan starts on the rows the previous one read last -- the part of the
// corpus still in the 256 MiB Infinity Cache.  `nq` scans are reserved (the
// query-stream kernel alternates per query from the returned start).
uint32_t next_direction(wvg_corpus *c, uint32_t nq)
{
    if (!c->ctx->opt.cache_reuse || !tuning().serpentine) return 0u;
    return (uint32_t)(c->scan_serial.fetch_add(nq, std::memory_order_relaxed) & 1u);
}

// PQ m = 32 scans without an allow list on a corpus with >= 3/4 of its slots
// live run K8c, which loads every tile instead of skipping dead ones.
int pq_dense(const wvg_corpus *c, const uint64_t *d_allow)
{
    return !d_allow && c->count * 4 >= c->high_water * 3;
}

// K1 row loads: non-temporal for scans far past the 256 MiB Infinity Cache,
// the default policy up to 800 MiB of scanned rows, where consecutive scans
// of the same rows find part of them in the cache (1M x 128 = 512 MB: 4 %
// faster; 2M x 128: 2 % slower; profiles/r02/bench/load_policy_ab.jsonl).
static int plain_loads(const wvg_corpus *c, uint64_t tb, uint64_t te)
{
    const int v = tuning().k1_loads;
    if (v) return v == 2;
    if (!c->ctx->opt.cache_reuse) return 0;  // streaming: every row load non-temporal
    return c->kind == WVG_KIND_F32 && (te - tb) * (uint64_t)c->nchunks * 1024ull <= (800ull << 20);
}

// K1 cache tail: with serpentine scans (consecutive scans alternate
// direction) the next scan starts on the rows this one read last, so each
// wave reads the last ~320 MB worth of its pass with the default policy (the
// 256 MiB Infinity Cache plus the L2s keep them) and the rest non-temporal
// (which does not evict them).  1M x 128 (512 MB): tail 160/256 -> 13.95k ->
// 14.80k QPS; 128/256: 14.74k; all default-policy: 13.95k
// (profiles/r02/bench/k1_cache_tail_ab.txt).  Scans that fit are all default
// policy (plain_loads).
constexpr uint64_t K1_CACHE_BYTES = 320000000ull;
static uint32_t k1_cache_tail(const wvg_corpus *c, uint64_t tb, uint64_t te)
{
    const int v = tuning().k1_tail;
    // F32 scans only: the same split in K8e's PQ code loads (tail 25/256 at 100M
    // codes) measured no gain -- that scan is not purely memory-bound
    if (c->kind != WVG_KIND_F32 || v < 0 || !c->ctx->opt.cache_reuse) return 0u;
    if (v > 0) return (uint32_t)std::min(v, 256);
    if (!tuning().serpentine || tuning().k1_loads) return 0u;  // no reversal / a forced policy (A/B)
    const uint64_t bytes = (te - tb) * (uint64_t)c->nchunks * 1024ull;
    if (bytes <= K1_CACHE_BYTES) return 0u;
    return (uint32_t)std::max<uint64_t>(1, (256ull * K1_CACHE_BYTES) / bytes);
}

ScreenWs screen_ws(uint32_t nq, uint32_t k, uint32_t nrr, uint32_t kbn, uint32_t fb_groups)
{
    ScreenWs w;
    Carver cv;
    const size_t nq_pad = (size_t)(nq + 127) / 128 * 128, ncand = (size_t)nrr * SCREEN_M;
    w.part = cv.take(nq * ncand * 8);
    w.cand = cv.take(nq * ncand * 8);
    w.keys = cv.take(nq * ncand * 8);
    w.gb = cv.take((size_t)nq * 4);
    w.qf = cv.take(nq_pad / 16 * kbn * 1024);
    w.k1 = cv.take(nq_pad * 4);
    w.k2 = cv.take(nq_pad * 4);
    w.em = cv.take(nq_pad * 4);
    w.fl = cv.take((size_t)nq * 4);
    w.nf = cv.take(4);
    w.fbp = cv.take((size_t)nq * fb_groups * k * 8);
    w.pids = cv.take((size_t)nq * k * 8);  // the pilot's own results (the caller's arrays may be null)
    w.pd = cv.take((size_t)nq * k * 4);
    w.pc = cv.take((size_t)nq * 4);
    w.kb = cv.take(nq_pad * 4);  // K3i's per-query constants
    w.css = cv.take(nq_pad * 4);
    w.qinv = cv.take(nq_pad * 4);
    w.total = cv.off;
    return w;
}

SearchPlan plan_search(wvg_corpus *c, uint32_t nq, uint32_t k, const uint64_t *allow, uint64_t allow_words,
                       bool mq_ok, bool gemm_ok)
{
    SearchPlan p;
    p.empty = !allow_tile_range(c, allow, allow_words, p.tb, p.te) || k == 0 || nq == 0;
    if (allow && !p.empty) p.allow_host = allow + c->id_base / 64 + p.tb;
    ScanArgs a{};
    a.tile_begin = p.tb;
    a.tile_end = p.te;
    a.nq = nq;
    a.dim = c->kind == WVG_KIND_F32 ? c->dim : 0;  // K1 grid depends on the row size and metric
    a.metric = c->metric;
    const uint32_t mn = c->ctx->opt.mfma_min_queries;
    p.gemm = gemm_ok && c->kind == WVG_KIND_F32 && mn > 0 && nq >= mn && gemm_supported(c->dim, c->metric) &&
             !c->ctx->order512;  // K3's 32 MFMA slices are the AVX2 order's chains
    if (p.gemm)
        p.groups = (int)gemm_row_ranges(nq, std::max<uint64_t>(1, p.te - p.tb), c->ctx->num_cus, c->dim, k);
    else
        p.groups = scan_groups_for(a, c->ctx->num_cus);
    // K5 (BQ) single-query scans: three 4-wave workgroups per CU, not K8e's one 8-wave one
    // (100M x 1536: 2.80 / 2.87 -> 2.78 / 2.82 ms, profiles/r06/bq/bq_groups_per_cu*.jsonl)
    if (c->kind == WVG_KIND_BQ && nq == 1 && tuning().groups_per_cu <= 0)  // (each wave >= 2 tiles)
        p.groups = (int)std::min<uint64_t>(3ull * (uint64_t)c->ctx->num_cus, std::max<uint64_t>(1, (p.te - p.tb) / 8));
    // bf16 screen + exact rescore for the batches it applies to (results identical to K3b)
    if (p.gemm && c->ctx->opt.batch_screen && screen_supported(c->dim, c->metric, k) && c->dim % 4 == 0 &&
        !c->sh_failed) {
        p.screen = true;
        p.exact_groups = p.groups;
        p.groups = (int)screen_row_ranges(nq, std::max<uint64_t>(1, p.te - p.tb), c->ctx->num_cus);
        ScanArgs a1 = a;
        a1.nq = 1;
        p.fb_groups = (uint32_t)std::min(scan_groups_for(a1, c->ctx->num_cus), c->ctx->num_cus);
        p.kbn = screen_kblocks(c->dim);
    }
    // PQ batches: the nq queries of one row range run side by side on one XCD and share its L2
    const bool pq_cos = c->kind == WVG_KIND_PQ && c->pq_m == 32 && c->pq_ks == 256 && pq_dense(c, nullptr) &&
                        (tuning().pq_variant == 0 || tuning().pq_variant == 48 || tuning().pq_variant == 49);
    const bool bq_cos = c->kind == WVG_KIND_BQ;  // K5 COS (wvg_bq.hip)
    p.cosched = nq > 1 && !allow && tuning().pq_cosched != 0 && (pq_cos || bq_cos);
    if (p.cosched)  // BQ: K5 workgroups are 4 waves, so bq_cos_gpc of them per CU
        p.groups = pq_cosched_groups(nq, c->ctx->num_cus * (bq_cos ? std::max(1, tuning().bq_cos_gpc) : 1));
    // flat batches below the MFMA threshold: K1 COS, the nq queries of one row
    // range side by side on one XCD (K1's workgroups per CU as for one query)
    if (c->kind == WVG_KIND_F32 && nq > 1 && !p.gemm && tuning().pq_cosched != 0) {
        ScanArgs a1 = a;
        a1.nq = 1;
        p.cosched = true;
        // K1Q (unfiltered L2 / dot / cosine at d = 128 / 768): Q queries per workgroup, so the
        // grid is sized for the nq / Q query groups (profiles/r05/k1q/)
        const int q = tuning().k1_mq;
        p.mq = mq_ok && !allow && (q == 2 || q == 4) && !c->ctx->order512 && (c->dim == 128 || c->dim == 768) &&
                       (c->metric == WVG_METRIC_L2 || c->metric == WVG_METRIC_DOT || c->metric == WVG_METRIC_COSINE)
                   ? q
                   : 0;
        p.groups = pq_cosched_groups(p.mq ? (nq + p.mq - 1) / p.mq : nq,
                                     std::max(scan_groups_for(a1, c->ctx->num_cus), 8));
    }
    return p;
}

// K3c: screen, exact rescore of the candidates, top-k; the flagged queries
// (a range list overflowed below tau) are rescanned exactly with K1.
static int run_screen(wvg_corpus *c, const ScanArgs &a, const SearchPlan &p, char *ws, uint64_t *ids, float *dists,
                      uint32_t *counts, hipStream_t s)
{
    const uint32_t nq = a.nq, k = a.k, nrr = (uint32_t)p.groups, ncand = nrr * SCREEN_M;
    const ScreenWs w = screen_ws(nq, k, nrr, p.kbn, p.fb_groups);
    ScreenLaunch L{};
    L.shadow = c->d_shadow;
    L.norms = c->d_norms;
    L.nmax = c->d_nmax;
    L.valid = a.valid;
    L.allow = a.allow;
    L.allow_words = a.allow_words;
    L.allow_t0 = a.allow_t0;
    L.tile_begin = a.tile_begin;
    L.tile_end = a.tile_end;
    L.dim = c->dim;
    L.queries = (const float *)a.queries;
    L.qpitch = a.qpitch;
    L.nq = nq;
    L.k = k;
    L.nrr = nrr;
    L.cosine = c->metric == WVG_METRIC_COSINE;
    L.num_cus = c->ctx->num_cus;
    L.qfrag = ws + w.qf;
    L.k1 = (float *)(ws + w.k1);
    L.k2 = (float *)(ws + w.k2);
    L.emax = (float *)(ws + w.em);
    L.gbound = (uint32_t *)(ws + w.gb);
    L.partials = (uint64_t *)(ws + w.part);
    L.cand = (uint64_t *)(ws + w.cand);
    L.flist = (uint32_t *)(ws + w.fl);
    L.nflag = (uint32_t *)(ws + w.nf);
    L.pilot = &a;                             // exact K1 over the first tiles (the fallback's partials are
    L.pilot_part = (uint64_t *)(ws + w.fbp);  // free until the rescan)
    L.pilot_groups = std::max<uint32_t>(1, std::min<uint32_t>(p.fb_groups, 4));
    L.pilot_part_lists = p.fb_groups;
    L.pilot_ids = (uint64_t *)(ws + w.pids);
    L.pilot_dists = (float *)(ws + w.pd);
    L.pilot_counts = (uint32_t *)(ws + w.pc);
    L.i8 = c->sh_i8;
    L.errs = c->d_errs;
    L.kb = (float *)(ws + w.kb);
    L.css = (float *)(ws + w.css);
    L.qinv = (float *)(ws + w.qinv);
    uint64_t *keys = (uint64_t *)(ws + w.keys);
    L.metric = c->metric;
    L.data = (const float *)c->d_data;
    L.nchunks = c->nchunks;
    WVG_HIP(launch_screen(L, s));
    WVG_HIP(launch_rescore_keys(c->metric, (const float *)a.queries, a.qpitch, (const float *)c->d_data, c->dim,
                                c->nchunks, L.cand, nq, ncand, ncand, keys, s, 0));
    WVG_HIP(launch_merge_keys(keys, nq, ncand, k, c->id_base, ids, dists, counts, s));
    ScanArgs f = a;
    f.nq = 1;
    f.cosched = 0;
    f.reverse = 0;
    uint64_t *fbp = (uint64_t *)(ws + w.fbp);
    WVG_HIP(launch_scan_f32_qlist(f, fbp, (int)p.fb_groups, L.flist, L.nflag, std::min<uint32_t>(nq, 8), s));
    WVG_HIP(launch_merge_lists_qlist(fbp, nq, p.fb_groups, k, k, c->id_base, ids, dists, counts, L.flist, L.nflag, s));
    return WVG_OK;
}

// Runs phase 1 + phase 2 for one corpus with device-resident prepared queries.
// One query of a host call on the query-stream kernel with its in-launch merge
// (run_search); its results can then go straight to host memory.
// (a filtered query too: its allow window is copied with the call, the scan masks tiles with it)
static bool inlaunch_single(const wvg_corpus *c, uint32_t nq, const SearchPlan &p)
{
    return nq == 1 && !p.gemm && !p.cosched && c->kind == WVG_KIND_F32 && tuning().pipeline_mode == 1;
}

int run_search(wvg_corpus *c, const void *d_q, uint32_t qpitch, uint32_t nq, uint32_t k, const uint64_t *d_allow,
               const SearchPlan &p, uint64_t *partials, uint64_t *ids, float *dists, uint32_t *counts, hipStream_t s,
               StreamSlot *sl, const float *qhost, const SingleOut *so)
{
    ScanArgs a{};
    a.data = c->d_data;
    a.valid = c->d_valid;
    a.allow = d_allow;
    a.allow_words = d_allow ? p.te - p.tb : 0;
    a.allow_t0 = p.tb;
    a.allow_qstride = d_allow ? p.allow_qstride : 0;
    a.id_base = c->id_base;
    a.tile_begin = p.tb;
    a.tile_end = p.te;
    a.dim = c->dim;
    a.nchunks = c->nchunks;
    a.metric = c->metric;
    a.queries = d_q;
    a.qpitch = qpitch;
    a.nq = nq;
    a.k = k;
    a.pq_m = c->pq_m;
    a.pq_ks = c->pq_ks;
    a.dense = pq_dense(c, d_allow);
    a.cosched = p.cosched ? (p.mq >= 2 ? p.mq : 1) : 0;  // (K1Q: queries per workgroup)
    a.order512 = c->ctx->order512;
    a.plain = plain_loads(c, p.tb, p.te);
    a.cache_tail256 = k1_cache_tail(c, p.tb, p.te);
    if (!p.gemm) a.reverse = next_direction(c, 1);
    if (p.cosched && c->kind == WVG_KIND_F32) {  // K1 COS: partners read the rows from L2
        a.plain = 1;
        a.cache_tail256 = 0;
    }
    if (p.screen) {
        if (ensure_shadow(c, s)) {
            ProfArm arm(c->ctx);
            if (arm.rc) return arm.rc;
            return run_screen(c, a, p, reinterpret_cast<char *>(partials), ids, dists, counts, s);
        }
        SearchPlan pe = p;  // no shadow: the exact MFMA path over the same workspace
        pe.screen = false;
        pe.groups = p.exact_groups;
        return run_search(c, d_q, qpitch, nq, k, d_allow, pe, partials, ids, dists, counts, s, sl, nullptr, so);
    }
    if (sl && inlaunch_single(c, nq, p)) {
        // One query of a host call: the query-stream kernel, whose extra workgroup merges
        // the partial lists in the same launch (no second kernel, no gap between them);
        // its arrival counter is the slot's persistent one, counted from the slot's base
        // (no per-call memset).  A merge that gives up (4 s) writes empty entries and the
        // header count WVG_RECORDS_TIMEOUT: search_batch reports it as WVG_ERR_DEVICE.
        uint32_t *ctl = nullptr;
        int rc = sl->control(&ctl);
        if (rc) return rc;
        StreamJob j{};
        j.partials = partials;
        j.arrivals = ctl;
        j.arrival_base = sl->arrival_base;
        j.status = ctl + 1;
        j.wait_limit = 400000000ull;
        j.groups = (uint32_t)p.groups;
        j.ids = ids;
        j.dists = dists;
        j.counts = counts;
        if (so) {
            j.records = so->records;
            j.tag = so->tag;
            j.legacy_poll = so->legacy_poll ? 1u : 0u;
        }
        j.row_split = (tuning().stream_variant & 1) == 0;
        // per-list hand-offs: the slot's ready words (zeroed once), tagged with the call's tag
        const bool ready = (tuning().stream_variant & 2) == 0 && so && so->tag && (uint32_t)p.groups <= SLOT_READY_MAX;
        if (ready) {
            j.ready = ctl + SLOT_READY_OFF;
            j.ready_tag = so->tag;
        }
        if (!d_q) {  // the query in the kernel arguments
            if (!qhost || qpitch > STREAM_QIN_FLOATS) return fail(WVG_ERR_INVALID, "inline query missing or too long");
            std::memcpy(j.qin, qhost, (size_t)qpitch * 4);
            a.queries = nullptr;
        }
        ProfArm arm(c->ctx);
        if (arm.rc) return arm.rc;
        WVG_HIP(launch_scan_f32_stream(a, j, s));
        if (!ready) sl->arrival_base += (uint32_t)p.groups;
        return WVG_OK;
    }
    ProfArm arm(c->ctx);
    if (arm.rc) return arm.rc;
    if (p.gemm) {
        uint32_t *prog = reinterpret_cast<uint32_t *>(partials + (size_t)nq * p.groups * k);
        WVG_HIP(launch_gemm_topk(a, (uint32_t)p.groups, partials, prog, prog + (size_t)p.groups * ((nq + 15) / 16),
                                 c->ctx->num_cus, s));
    }
    else
        WVG_HIP(launch_scan(a, c->kind, partials, p.groups, s));
    WVG_HIP(launch_merge_lists(partials, nq, (uint32_t)p.groups, k, k, c->id_base, ids, dists, counts, s));
    return WVG_OK;
}

void write_empty(uint32_t nq, uint32_t k, uint64_t *ids, float *dists, uint32_t *counts)
{
    for (uint64_t i = 0; i < (uint64_t)nq * k; i++) {
        if (ids) ids[i] = WVG_KEY_NONE;
        if (dists) dists[i] = INFINITY;
    }
    if (counts)
        for (uint32_t i = 0; i < nq; i++) counts[i] = 0;
}

int stage_queries(wvg_corpus *c, StreamSlot *sl, const float *queries, uint32_t nq, char *dst, uint32_t &qpitch,
                         float *d_lut_or_null, char *d_qtmp, Staging *st)
{
    std::vector<float> qf;
    std::vector<uint64_t> qb;
    if (c->kind == WVG_KIND_F32 && c->metric != WVG_METRIC_COSINE && f32_chunks(c->dim) * 4 == c->dim) {
        // the prepared queries are the caller's rows as they are: one copy, no host pass
        qpitch = c->dim;
        hipStream_t s = sl->stream;
        WVG_HIP(st ? st->h2d(dst, queries, (size_t)nq * c->dim * 4, s)
                   : hipMemcpyAsync(dst, queries, (size_t)nq * c->dim * 4, hipMemcpyHostToDevice, s));
        return WVG_OK;
    }
    prepare_queries_host(c, queries, nq, qf, qb, qpitch);
    // A copy from pageable memory returns once the source has been staged, so
    // qf / qb may go out of scope without a stream sync (which would put a host
    // round trip between the PQ LUT kernel and the scan).
    hipStream_t s = sl->stream;
    auto h2d = [&](void *d, const void *h, size_t bytes) {
        return st ? st->h2d(d, h, bytes, s) : hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, s);
    };
    if (c->kind == WVG_KIND_BQ) {
        WVG_HIP(h2d(dst, qb.data(), qb.size() * 8));
        return WVG_OK;
    }
    if (c->kind == WVG_KIND_F32) {
        WVG_HIP(h2d(dst, qf.data(), qf.size() * 4));
        return WVG_OK;
    }
    // PQ: queries -> LUTs [nq][m*ks] (CH/product_quantization.go:329-337)
    WVG_HIP(h2d(d_qtmp, qf.data(), qf.size() * 4));
    WVG_HIP(launch_pq_lut(c->metric, (const float *)d_qtmp, nq, qpitch, c->d_centers, c->pq_m, c->pq_ks, c->pq_ds,
                          d_lut_or_null, s));
    qpitch = c->pq_m * c->pq_ks;
    return WVG_OK;
}

// wvg_search_device's prepared queries after the partial lists: PQ LUTs, or
// BQ codes at the scan's pitch plus the encoder's dense output.
size_t device_query_bytes(const wvg_corpus *c, uint32_t nq)
{
    switch (c->kind) {
    case WVG_KIND_PQ: return align_up((size_t)nq * c->pq_m * c->pq_ks * 4, 256);
    case WVG_KIND_BQ:
        return align_up((size_t)nq * bq_chunks(c->dim) * 16, 256) + align_up((size_t)nq * bq_words(c->dim) * 8, 256);
    default: return 0;
    }
}

size_t query_bytes(const wvg_corpus *c, uint32_t nq)
{
    switch (c->kind) {
    case WVG_KIND_F32: return (size_t)nq * f32_chunks(c->dim) * 16;
    case WVG_KIND_BQ: return (size_t)nq * bq_chunks(c->dim) * 16;
    default: return (size_t)nq * c->pq_m * c->pq_ks * 4;
    }
}

// Upper bound of the host bytes stage_queries copies (a Staging reservation).
size_t staged_query_bytes(const wvg_corpus *c, uint32_t nq)
{
    return std::max(query_bytes(c, nq), (size_t)nq * c->dim * 4);
}


ScanArgs scan_args_for(const wvg_corpus *c, const void *d_q, uint32_t qpitch, uint32_t nq, uint32_t k,
                              const uint64_t *d_allow, uint64_t tb, uint64_t te)
{
    ScanArgs a{};
    a.data = c->d_data;
    a.valid = c->d_valid;
    a.allow = d_allow;
    a.allow_words = d_allow ? te - tb : 0;
    a.allow_t0 = tb;
    a.id_base = c->id_base;
    a.tile_begin = tb;
    a.tile_end = te;
    a.dim = c->dim;
    a.nchunks = c->nchunks;
    a.metric = c->metric;
    a.queries = d_q;
    a.qpitch = qpitch;
    a.nq = nq;
    a.k = k;
    a.pq_m = c->pq_m;
    a.pq_ks = c->pq_ks;
    a.dense = pq_dense(c, d_allow);
    a.order512 = c->ctx->order512;
    return a;
}

}  // namespace wvg

using namespace wvg;

// One caller's single-query search waiting in a corpus's coalescer.
struct wvg_search_request {
    const float *q;
    uint32_t k;
    const uint64_t *allow = nullptr;  // the caller's allow list (helpers.AllowList bitmap), or null
    uint64_t allow_words = 0;
    uint64_t tb = 0, te = 0;          // its tile window (allow_tile_range), for filtered requests
    uint64_t *ids;
    float *dists;
    uint32_t *counts;
    int rc = WVG_OK;
    std::string err;
    bool done = false;
};

namespace wvg {

#ifdef WVG_TOOLS
// tools-build counters of the single-query host path (wvgx_single_counters):
// [0] tagged calls, [1] calls whose header carried the tag before every entry did
// (out-of-order arrival observed), [2] calls that fell back to a stream sync,
// [3] round-4 layout: ids that changed after the polled count was seen
static std::atomic<uint64_t> g_single[4];
void single_counter(int i, bool hit)
{
    if (hit) g_single[i].fetch_add(1, std::memory_order_relaxed);
}
void single_counters(uint64_t out[4], bool reset)
{
    for (int i = 0; i < 4; i++) out[i] = reset ? g_single[i].exchange(0) : g_single[i].load();
}
// the coalescer's batches (wvgx_coalesce_counters): [0] batches, [1] requests,
// [2] ns spent running batches, [3] the largest batch
static std::atomic<uint64_t> g_coal[4];
static void coalesce_counter(size_t reqs, uint64_t ns)
{
    g_coal[0].fetch_add(1, std::memory_order_relaxed);
    g_coal[1].fetch_add(reqs, std::memory_order_relaxed);
    g_coal[2].fetch_add(ns, std::memory_order_relaxed);
    uint64_t m = g_coal[3].load();
    while (reqs > m && !g_coal[3].compare_exchange_weak(m, reqs)) {
    }
}
void coalesce_counters(uint64_t out[4], bool reset)
{
    for (int i = 0; i < 4; i++) out[i] = reset ? g_coal[i].exchange(0) : g_coal[i].load();
}
// host time of the in-launch single-query path (wvgx_single_timing): ns summed over
// calls -- [0] search_batch entry -> launch call, [1] the launch call (run_search),
// [2] polling for the tagged records, [3] copying them out; [4] calls
static std::atomic<uint64_t> g_stime[5];
static void single_timing(const std::chrono::steady_clock::time_point (&t)[5])
{
    for (int i = 0; i < 4; i++)
        g_stime[i].fetch_add((uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(t[i + 1] - t[i]).count(),
                             std::memory_order_relaxed);
    g_stime[4].fetch_add(1, std::memory_order_relaxed);
}
void single_timing_read(uint64_t out[5], bool reset)
{
    for (int i = 0; i < 5; i++) out[i] = reset ? g_stime[i].exchange(0) : g_stime[i].load();
}
#define WVG_STAMP(i) tstamp[i] = std::chrono::steady_clock::now()
// host time of filtered coalesced batches (wvgx_filtered_timing): ns summed over
// batches -- [0] entry -> queries staged, [1] windows filled (+ copies issued),
// [2] the launch call, [3] the wait for the results; [4] batches
static std::atomic<uint64_t> g_ftime[5];
static void filtered_timing(const std::chrono::steady_clock::time_point (&t)[5])
{
    for (int i = 0; i < 4; i++)
        g_ftime[i].fetch_add((uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(t[i + 1] - t[i]).count(),
                             std::memory_order_relaxed);
    g_ftime[4].fetch_add(1, std::memory_order_relaxed);
}
void filtered_timing_read(uint64_t out[5], bool reset)
{
    for (int i = 0; i < 5; i++) out[i] = reset ? g_ftime[i].exchange(0) : g_ftime[i].load();
}
#else
inline void single_counter(int, bool) {}
inline void coalesce_counter(size_t, uint64_t) {}
#define WVG_STAMP(i) ((void)0)
#endif

// Waits until a single query's tagged records (StreamJob::records) have all
// landed in host memory: the header and every one of the k entries carry this
// call's tag.  GPU stores to host memory may become visible out of order -- the
// round-4 layout (ids / dists, a system-scope release, then a count the host
// polled) returned the slot's PREVIOUS result in ~1 of 1000 concurrent calls
// (profiles/r04/single_query_stress/, profiles/r05/single_query/): the count had
// landed, the ids of this call not yet.  Checking the tag in every entry makes
// acceptance independent of the arrival order.  An entry is {slot, tag, dist,
// tag} (the slot, not the 64-bit docID: id_base is the host's), so BOTH 8-byte
// halves carry the tag and acceptance does not assume that a 16-byte store
// reaches host memory as one unit -- only that an aligned 8-byte one does (a
// single PCIe / xGMI write of it is never split).  sync: synchronize the
// stream first (tools A/B); a poll that has not seen the tags after 50 ms (long
// scans, a fault) synchronizes too, and the tags must then arrive within 1 s.
static int wait_records(const SingleOut &so, uint32_t k, hipStream_t s, bool sync)
{
    const volatile uint32_t *w = reinterpret_cast<const volatile uint32_t *>(so.records);
    bool early = false;
    auto landed = [&]() {
        if (w[4 * k + 1] != so.tag) return false;
        for (uint32_t i = 0; i < k; i++)
            if (w[4 * i + 1] != so.tag || w[4 * i + 3] != so.tag) {
                early = true;
                return false;
            }
        return true;
    };
    single_counter(0, true);
    bool ok = false;
    if (!sync) {
        const auto t0 = std::chrono::steady_clock::now();
        for (uint32_t spin = 0;; spin++) {
            if (landed()) {
                ok = true;
                break;
            }
            if ((spin & 1023u) == 1023u && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(50))
                break;
        }
    }
    if (!ok) {
        single_counter(2, !sync);
        WVG_HIP(hipStreamSynchronize(s));
        const auto t0 = std::chrono::steady_clock::now();
        while (!landed())
            if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(1))
                return fail(WVG_ERR_DEVICE, "single-query results did not arrive in host memory (tag mismatch)");
    }
    std::atomic_thread_fence(std::memory_order_acquire);
    single_counter(1, early);
    return WVG_OK;
}

// flat.SearchByVector for nq queries (the caller holds the corpus lock shared).
static int search_batch(wvg_corpus *c, const float *queries, uint32_t nq, uint32_t k, const uint64_t *allow_bits,
                        uint64_t allow_words, uint64_t *out_ids, float *out_dists, uint32_t *out_counts);

// Queries a coalesced batch may take: K1 co-scheduled batches gain up to ~31
// queries on one corpus (profiles/r03/measure_1/small.log.txt), dot / cosine
// batches of >= mfma_min_queries go to the matrix cores.
constexpr size_t COALESCE_MAX = 256;
// A filtered batch's per-query allow windows (B x union width x 8 bytes) stay
// within this (256 callers over a 125M-row slab would need 4 GB).
constexpr size_t FILTER_BATCH_BYTES = (size_t)8 << 20;
// k classes of coalesced batches: the bf16 screen takes k <= 16, the register
// top-k holds 64 / 128 / 256 keys per wave (a k = 256 caller put
// every k = 10 caller of its batch on the E = 4 top-k and off the screen).
static int coalesce_kclass(uint32_t k) { return k <= 16 ? 0 : k <= 64 ? 1 : k <= 128 ? 2 : 3; }

// Filtered single queries of one coalesced batch (F32): one co-scheduled K1
// launch over the union of their allow windows, every query masked by its
// own window (ScanArgs::allow_qstride).
static int search_batch_filtered(wvg_corpus *c, const std::vector<wvg_search_request *> &batch, uint32_t k,
                                 uint64_t *out_ids, float *out_dists, uint32_t *out_counts);

// Runs one coalesced batch at k = the largest k of its requests and hands every
// request the first r->k rows of its result: the top-k order is a strict total
// order on (distance, docID) keys, so a smaller k's result is exactly a prefix of
// a larger k's (counts: min(count, r->k)); a failure is every request's failure.
static void run_coalesced(wvg_corpus *c, const std::vector<wvg_search_request *> &batch, uint32_t k)
{
    const size_t B = batch.size();
    if (B == 1) {
        wvg_search_request *r = batch[0];
        r->rc = search_batch(c, r->q, 1, r->k, r->allow, r->allow_words, r->ids, r->dists, r->counts);
        if (r->rc) r->err = wvg_last_error();
        return;
    }
    const uint32_t d = c->dim;
    std::vector<float> q(B * d), dists(B * k);
    std::vector<uint64_t> ids(B * k);
    std::vector<uint32_t> counts(B);
    for (size_t i = 0; i < B; i++) std::memcpy(q.data() + i * d, batch[i]->q, (size_t)d * 4);
    const int rc = batch[0]->allow
                       ? search_batch_filtered(c, batch, k, ids.data(), dists.data(), counts.data())
                       : search_batch(c, q.data(), (uint32_t)B, k, nullptr, 0, ids.data(), dists.data(), counts.data());
    const std::string err = rc ? wvg_last_error() : std::string();
    for (size_t i = 0; i < B; i++) {
        wvg_search_request *r = batch[i];
        r->rc = rc;
        r->err = err;
        if (rc) continue;
        if (r->ids) std::memcpy(r->ids, ids.data() + i * k, (size_t)r->k * 8);
        if (r->dists) std::memcpy(r->dists, dists.data() + i * k, (size_t)r->k * 4);
        if (r->counts) *r->counts = std::min(counts[i], r->k);
    }
}

// A single-query search through the corpus's coalescer: the request queues;
// while no batch of this corpus executes, the first waiter takes every queued
// request of the head's class (filtered or not; any k, the batch runs at the
// largest; up to COALESCE_MAX) and runs them as one batch (results identical to
// separate calls: tests/test_gpu_coalesce.py), then wakes the others.  A lone
// call finds the coalescer idle and runs at once; under load a batch forms from
// the calls that arrive while the previous one runs, so the batch size follows
// the arrival rate.
static int search_coalesced(wvg_corpus *c, const float *query, uint32_t k, const uint64_t *allow,
                            uint64_t allow_words, uint64_t tb, uint64_t te, uint64_t *out_ids, float *out_dists,
                            uint32_t *out_counts)
{
    wvg_search_request r;
    r.q = query;
    r.k = k;
    r.allow = allow;
    r.allow_words = allow_words;
    r.tb = tb;
    r.te = te;
    r.ids = out_ids;
    r.dists = out_dists;
    r.counts = out_counts;
    wvg_coalescer &co = c->co;
    std::unique_lock<std::mutex> g(co.mu);
    co.pending.push_back(&r);
    if (co.gathering) co.gather_cv.notify_one();
    while (!r.done) {
        if (co.busy) {
            co.cv.wait(g);
            continue;
        }
        co.busy = true;
        // Gathering: callers come back right after their batch returns, so the batch
        // that starts next would otherwise hold only those that queued meanwhile --
        // with T closed-loop callers the batches settled at T / 2, alternating halves
        // (profiles/r05/coalesce/).  When the last batch (of more than one request)
        // ended moments ago, the runner waits a short window until its callers are back
        // too: the requests that were waiting when it ended + as many as it held.  The
        // window is at most a quarter of that batch's run time (tuning gather_div) and
        // 50 us + 3 us per caller to wake (64 callers on 16 cores take ~200 us), at least 10
        // us.  Only after batches of 4 or more: a lone caller never waits, and two or
        // three callers gain little from merged batches (2 queries: 0.10 ms vs 0.08 ms
        // for one) but would pay the window whenever one of them does not come back.
        const size_t want = std::min(co.carry + co.last_n, COALESCE_MAX);
        if (co.last_n >= 4 && co.pending.size() < want) {
            const auto window = std::max<std::chrono::nanoseconds>(
                std::chrono::microseconds(10),
                std::min<std::chrono::nanoseconds>(std::chrono::microseconds(50 + 3 * (int64_t)co.last_n),
                                                   co.last_run / tuning().gather_div));
            const auto until = co.last_done + window;
            if (std::chrono::steady_clock::now() < until) {
                co.gathering = true;
                while (co.pending.size() < want && co.gather_cv.wait_until(g, until) != std::cv_status::timeout) {
                }
                co.gathering = false;
            }
        }
        std::vector<wvg_search_request *> batch;
        uint32_t kk = 0;  // the batch's k: the largest of its requests' (round 4: the head's k only)
        // filtered and unfiltered requests form separate batches.  A filtered batch
        // holds every query's allow words over the union of their windows (B x W
        // words on the host, in scratch and over the bus), so it stops growing at
        // FILTER_BATCH_BYTES; the requests left over run in the next batch.
        // Requests of one batch also share a k class (coalesce_kclass), so a large-k
        // caller never moves small-k callers to a larger register top-k or off the screen.
        const bool filt = co.pending.front()->allow != nullptr;
        const int kcl = coalesce_kclass(co.pending.front()->k);
        uint64_t TB = UINT64_MAX, TE = 0;
        for (auto it = co.pending.begin(); it != co.pending.end() && batch.size() < COALESCE_MAX;) {
            if (((*it)->allow != nullptr) != filt || coalesce_kclass((*it)->k) != kcl) {
                ++it;
                continue;
            }
            if (filt) {
                const uint64_t nb = std::min(TB, (*it)->tb), ne = std::max(TE, (*it)->te);
                if (!batch.empty() && (batch.size() + 1) * (ne - nb) * 8 > FILTER_BATCH_BYTES) break;
                TB = nb;
                TE = ne;
            }
            kk = std::max(kk, (*it)->k);
            batch.push_back(*it);
            it = co.pending.erase(it);
        }
        g.unlock();
        const auto tb0 = std::chrono::steady_clock::now();
        run_coalesced(c, batch, kk);
        const auto tb1 = std::chrono::steady_clock::now();
        coalesce_counter(batch.size(), (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(tb1 - tb0).count());
        g.lock();
        co.last_n = batch.size();
        co.carry = co.pending.size();
        co.last_done = tb1;
        co.last_run = std::chrono::duration_cast<std::chrono::nanoseconds>(tb1 - tb0);
        for (wvg_search_request *b : batch) b->done = true;
        co.busy = false;
        co.cv.notify_all();
    }
    if (r.rc) set_error(r.err);
    return r.rc;
}

}  // namespace wvg

extern "C" {

int wvg_search(wvg_corpus *c, const float *queries, uint32_t nq, uint32_t k, const uint64_t *allow_bits,
               uint64_t allow_words, uint64_t *out_ids, float *out_dists, uint32_t *out_counts)
{
    int rc = check_corpus(c);
    if (rc) return rc;
    if (nq > 0 && !queries) return fail(WVG_ERR_INVALID, "null queries");
    if (c->kind == WVG_KIND_PQ && !c->d_centers) return fail(WVG_ERR_INVALID, "PQ corpus has no codebook");
    std::shared_lock<std::shared_mutex> lk(c->rw);
    if (nq == 1 && k > 0 && k <= MAX_K && c->ctx->opt.coalesce && (!allow_bits || c->kind == WVG_KIND_F32)) {
        uint64_t tb = 0, te = 0;
        if (allow_bits && !allow_tile_range(c, allow_bits, allow_words, tb, te)) {  // nothing allowed here
            write_empty(1, k, out_ids, out_dists, out_counts);
            return WVG_OK;
        }
        return search_coalesced(c, queries, k, allow_bits, allow_words, tb, te, out_ids, out_dists, out_counts);
    }
    return search_batch(c, queries, nq, k, allow_bits, allow_words, out_ids, out_dists, out_counts);
}

}  // extern "C"

static int wvg::search_batch(wvg_corpus *c, const float *queries, uint32_t nq, uint32_t k, const uint64_t *allow_bits,
                             uint64_t allow_words, uint64_t *out_ids, float *out_dists, uint32_t *out_counts)
{
#ifdef WVG_TOOLS
    std::chrono::steady_clock::time_point tstamp[5];
#endif
    WVG_STAMP(0);
    int rc;
    SearchPlan p = plan_search(c, nq, std::min(k, MAX_K), allow_bits, allow_words);
    if (p.empty) {
        write_empty(nq, k, out_ids, out_dists, out_counts);
        return WVG_OK;
    }
    if (k > MAX_K)  // beyond the fused register top-k: select + sort in HBM
        return search_large_k(c, queries, nq, k, allow_bits, allow_words, p, out_ids, out_dists, out_counts);
    SlotGuard g(c->ctx);
    rc = c->ctx->acquire(&g.slot);
    if (rc) return rc;
    Carver cv;
    const size_t o_q = cv.take(query_bytes(c, nq));
    const size_t o_qtmp = cv.take(c->kind == WVG_KIND_PQ ? (size_t)nq * c->dim * 4 : 0);
    const size_t o_allow = cv.take(p.allow_bytes());
    const size_t o_part = cv.take(p.workspace_bytes(nq, k));
    const size_t o_ids = cv.take((size_t)nq * k * 8);
    const size_t o_d = cv.take((size_t)nq * k * 4);
    const size_t o_cnt = cv.take((size_t)nq * 4);
    void *base = nullptr;
    rc = g.slot->device_scratch(cv.off, &base);
    if (rc) return rc;
    char *b = (char *)base;
    hipStream_t s = g.slot->stream;
    // queries, allow words and the [ids | dists | counts] result span through
    // the slot's pinned staging: one copy each way, no pageable round trips
    const size_t out_b = o_cnt + (size_t)nq * 4 - o_ids;
    Staging st;
    rc = st.reserve(g.slot, stage_bytes(staged_query_bytes(c, nq)) +
                                (p.allow_host ? stage_bytes(p.allow_bytes()) : 0) + stage_bytes(out_b));
    if (rc) return rc;
    uint32_t qpitch = 0;
    // a single in-launch F32 query of up to STREAM_QIN_FLOATS floats goes in the kernel arguments
    alignas(16) float qinl[STREAM_QIN_FLOATS];  // (no heap allocation on the single-query path)
    const bool qin = inlaunch_single(c, nq, p) &&
                     (size_t)f32_chunks(c->dim) * 4 <= STREAM_QIN_FLOATS && (tuning().single_path & 1) == 0;
    if (qin) {  // prepare_queries_host for one F32 query, into the kernel-argument buffer
        qpitch = f32_chunks(c->dim) * 4;
        for (uint32_t i = c->dim; i < qpitch; i++) qinl[i] = 0.0f;
        if (c->metric == WVG_METRIC_COSINE)
            normalize_host(queries, c->dim, qinl);
        else
            std::memcpy(qinl, queries, (size_t)c->dim * 4);
    } else {
        rc = stage_queries(c, g.slot, queries, nq, b + o_q, qpitch, (float *)(b + o_q), b + o_qtmp, &st);
        if (rc) return rc;
    }
    const uint64_t *d_allow = nullptr;
    if (p.allow_host && inlaunch_single(c, nq, p) && p.allow_bytes() <= STAGE_MAX) {
        // a single in-launch query reads its allow window straight from the slot's pinned
        // staging over the bus (each wave's next tile word is prefetched a tile ahead): no
        // host-to-device copy (~10 us of a 125 KB window's copy and its API time)
        char *h = st.take(p.allow_bytes());
        std::memcpy(h, p.allow_host, p.allow_bytes());
        d_allow = reinterpret_cast<const uint64_t *>(h);
    } else if (p.allow_host) {
        WVG_HIP(st.h2d(b + o_allow, p.allow_host, p.allow_bytes(), s));
        d_allow = (const uint64_t *)(b + o_allow);
    }
    // a single query merged in-launch writes its results straight into the slot's
    // coherent host buffer as tagged records: no device-to-host copy (and its ~10 us)
    // and no stream synchronization per call (the host polls the tags)
    const bool zc = inlaunch_single(c, nq, p);
    const int sp = tuning().single_path;
    const bool legacy = zc && (sp & 4) != 0;  // tools A/B: round 4's untagged layout
    SingleOut so;
    char *hc = nullptr;
    if (zc) {
        void *v = nullptr;
        rc = g.slot->host_coherent(legacy ? out_b : (size_t)(k + 1) * 16, &v);
        if (rc) return rc;
        hc = (char *)v;
        if (!legacy) {
            so.records = reinterpret_cast<uint4 *>(hc);
            so.tag = ++g.slot->tag ? g.slot->tag : ++g.slot->tag;  // never 0
        }
    }
    if (zc && !legacy) {
        WVG_STAMP(1);
        rc = run_search(c, qin ? nullptr : b + o_q, qpitch, nq, k, d_allow, p, (uint64_t *)(b + o_part), nullptr,
                        nullptr, nullptr, s, g.slot, qin ? qinl : nullptr, &so);
        if (rc) return rc;
        WVG_STAMP(2);
        rc = wait_records(so, k, s, (sp & 2) != 0);
        if (rc) return rc;
        WVG_STAMP(3);
        const uint4 *r = so.records;
        for (uint32_t i = 0; i < k; i++) {
            if (out_ids) out_ids[i] = r[i].x == 0xFFFFFFFFu ? WVG_KEY_NONE : c->id_base + r[i].x;
            if (out_dists) std::memcpy(out_dists + i, &r[i].z, 4);
        }
#ifdef WVG_TOOLS
        WVG_STAMP(4);
        single_timing(tstamp);
#endif
        const uint32_t c0 = r[k].x;
        if (c0 == WVG_RECORDS_TIMEOUT) {  // the in-launch merge gave up (empty entries were written)
            if (out_counts) *out_counts = 0;
            return fail(WVG_ERR_DEVICE, "single-query merge timed out waiting for the scan workgroups");
        }
        if (out_counts) *out_counts = c0;
        return WVG_OK;
    }
    char *rspan = zc ? hc : b + o_ids;  // the result span [ids | dists | counts]
    // tools A/B (single_path bit 2): round 4's polled untagged layout -- the host polls the count
    // word (preset to a sentinel) that the merge writes last, after a system-scope release
    volatile uint32_t *cflag = legacy && (sp & 2) == 0
                                   ? reinterpret_cast<volatile uint32_t *>(rspan + (o_cnt - o_ids))
                                   : nullptr;
    if (legacy) so.legacy_poll = cflag != nullptr;
    if (cflag) *cflag = 0xFFFFFFFFu;
    rc = run_search(c, qin ? nullptr : b + o_q, qpitch, nq, k, d_allow, p, (uint64_t *)(b + o_part), (uint64_t *)rspan,
                    (float *)(rspan + (o_d - o_ids)), (uint32_t *)(rspan + (o_cnt - o_ids)), s, g.slot,
                    qin ? qinl : nullptr, &so);
    if (rc) return rc;
    const char *pin = zc ? hc : out_b <= STAGE_MAX ? st.take(out_b) : nullptr;
    std::vector<char> big(pin ? 0 : out_b);
    if (!pin) pin = big.data();
    if (!zc) WVG_HIP(hipMemcpyAsync((void *)pin, b + o_ids, out_b, hipMemcpyDeviceToHost, s));
    bool polled = false;
    if (cflag) {
        const auto t0 = std::chrono::steady_clock::now();
        for (uint32_t spin = 0;; spin++) {
            if (*cflag != 0xFFFFFFFFu) {
                polled = true;
                break;
            }
            if ((spin & 1023u) == 1023u && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(50))
                break;  // long scans (or a fault): the stream synchronization below decides
        }
        std::atomic_thread_fence(std::memory_order_acquire);
    }
    if (!polled) WVG_HIP(hipStreamSynchronize(s));
    if (out_ids) std::memcpy(out_ids, pin, (size_t)nq * k * 8);
    if (out_dists) std::memcpy(out_dists, pin + (o_d - o_ids), (size_t)nq * k * 4);
    if (out_counts) std::memcpy(out_counts, pin + (o_cnt - o_ids), (size_t)nq * 4);
#ifdef WVG_TOOLS
    if (polled && out_ids) {  // diagnostic: did ids land in host memory AFTER the polled count?
        WVG_HIP(hipStreamSynchronize(s));
        single_counter(3, std::memcmp(out_ids, hc, (size_t)k * 8) != 0);
    }
#endif
    if (nq == 1 && !d_allow && c->count > 0) {  // a live row exists: 0 results = the in-launch merge gave up
        uint32_t c0 = 0;
        std::memcpy(&c0, pin + (o_cnt - o_ids), 4);
        if (c0 == 0) return fail(WVG_ERR_DEVICE, "single-query merge timed out waiting for the scan workgroups");
    }
    return WVG_OK;
}

static int wvg::search_batch_filtered(wvg_corpus *c, const std::vector<wvg_search_request *> &batch, uint32_t k,
                                      uint64_t *out_ids, float *out_dists, uint32_t *out_counts)
{
#ifdef WVG_TOOLS
    std::chrono::steady_clock::time_point tstamp[5];
#endif
    WVG_STAMP(0);
    const uint32_t B = (uint32_t)batch.size(), d = c->dim;
    // every query's window [tb_i, te_i) and their union [TB, TE)
    std::vector<uint64_t> tb(B), te(B);
    std::vector<char> live(B);
    uint64_t TB = UINT64_MAX, TE = 0;
    for (uint32_t i = 0; i < B; i++) {  // (windows found by wvg_search: a request with none never queues)
        tb[i] = batch[i]->tb;
        te[i] = batch[i]->te;
        live[i] = te[i] > tb[i];
        if (!live[i]) continue;
        TB = std::min(TB, tb[i]);
        TE = std::max(TE, te[i]);
    }
    write_empty(B, k, out_ids, out_dists, out_counts);
    if (TE <= TB) return WVG_OK;
    const uint64_t W = TE - TB, wb = c->id_base / 64;
    // query i's allow words of tiles [TB, TE) (0 outside its own), written straight into
    // the pinned staging (below): one pass over the callers' words, zeros only outside
    // each window (round 5 filled a zeroed vector, then staged it: three passes)
    auto fill_window = [&](uint64_t *win, uint32_t i) {
        uint64_t *row = win + (size_t)i * W;
        if (!live[i]) {
            std::memset(row, 0, W * 8);
            return;
        }
        std::memset(row, 0, (tb[i] - TB) * 8);
        std::memcpy(row + (tb[i] - TB), batch[i]->allow + wb + tb[i], (te[i] - tb[i]) * 8);
        std::memset(row + (te[i] - TB), 0, (TE - te[i]) * 8);
    };
    // windows of queries [i0, i1); large ones (e.g. 16 x 125 KB for 10 % lists over 1M rows)
    // on several host threads
    auto fill_windows = [&](uint64_t *win, uint32_t i0, uint32_t i1) {
        if ((size_t)(i1 - i0) * W * 8 >= ((size_t)128 << 10) && i1 - i0 > 1)
            parallel_for(i1 - i0, [&](uint32_t i) { fill_window(win, i0 + i); });
        else
            for (uint32_t i = i0; i < i1; i++) fill_window(win, i);
    };
    // per-query allow windows: K1Q's filtered variant (d = 128 / 768, L2 / dot / cosine) or the COS K1
    SearchPlan p = plan_search(c, B, k, nullptr, 0, true, false);
    if (p.empty) return WVG_OK;
    if (p.gemm || !p.cosched) return fail(WVG_ERR_INVALID, "filtered coalesced batch needs the co-scheduled K1");
    p.tb = TB;
    p.te = TE;
    p.allow_qstride = W;
    std::vector<float> q((size_t)B * d);
    for (uint32_t i = 0; i < B; i++) std::memcpy(q.data() + (size_t)i * d, batch[i]->q, (size_t)d * 4);
    SlotGuard g(c->ctx);
    int rc = c->ctx->acquire(&g.slot);
    if (rc) return rc;
    Carver cv;
    const size_t o_q = cv.take(query_bytes(c, B));
    const size_t o_allow = cv.take((size_t)B * W * 8);
    const size_t o_part = cv.take(p.workspace_bytes(B, k));
    const size_t o_ids = cv.take((size_t)B * k * 8);
    const size_t o_d = cv.take((size_t)B * k * 4);
    const size_t o_cnt = cv.take((size_t)B * 4);
    void *base = nullptr;
    rc = g.slot->device_scratch(cv.off, &base);
    if (rc) return rc;
    char *b = (char *)base;
    hipStream_t s = g.slot->stream;
    const size_t out_b = o_cnt + (size_t)B * 4 - o_ids;
    Staging st;
    rc = st.reserve(g.slot, stage_bytes(staged_query_bytes(c, B)) + stage_bytes((size_t)B * W * 8) + stage_bytes(out_b));
    if (rc) return rc;
    uint32_t qpitch = 0;
    rc = stage_queries(c, g.slot, q.data(), B, b + o_q, qpitch, nullptr, nullptr, &st);
    if (rc) return rc;
    std::vector<uint64_t> wbig;  // (beyond the staging: pageable, copied by HIP)
    uint64_t *win = nullptr;
    if ((size_t)B * W * 8 <= STAGE_MAX) {
        win = reinterpret_cast<uint64_t *>(st.take((size_t)B * W * 8));
    } else {
        wbig.resize((size_t)B * W);
        win = wbig.data();
    }
    WVG_STAMP(1);
    const uint64_t *d_allow = (const uint64_t *)(b + o_allow);
    if (!wbig.empty() || (tuning().filter_zc & 1) == 0) {
        // two halves: the first half's copy runs while the second half is filled
        const uint32_t hB = (size_t)B * W * 8 >= ((size_t)512 << 10) ? B / 2 : 0;
        if (hB > 0) {
            fill_windows(win, 0, hB);
            WVG_HIP(hipMemcpyAsync(b + o_allow, win, (size_t)hB * W * 8, hipMemcpyHostToDevice, s));
        }
        fill_windows(win, hB, B);
        WVG_HIP(hipMemcpyAsync(b + o_allow + (size_t)hB * W * 8, win + (size_t)hB * W, (size_t)(B - hB) * W * 8,
                               hipMemcpyHostToDevice, s));
    } else {
        // the windows stay in the slot's pinned staging and K1Q reads them over the bus (each
        // wave's next tile words prefetched a tile ahead, as a lone filtered query's): no
        // host-to-device copy in front of the scan (16 x 125 KB: ~45 us of copy)
        fill_windows(win, 0, B);
        d_allow = win;
    }
    WVG_STAMP(2);
    rc = run_search(c, b + o_q, qpitch, B, k, d_allow, p, (uint64_t *)(b + o_part), (uint64_t *)(b + o_ids),
                    (float *)(b + o_d), (uint32_t *)(b + o_cnt), s);
    if (rc) return rc;
    const char *pin = out_b <= STAGE_MAX ? st.take(out_b) : nullptr;
    std::vector<char> big(pin ? 0 : out_b);
    if (!pin) pin = big.data();
    WVG_HIP(hipMemcpyAsync((void *)pin, b + o_ids, out_b, hipMemcpyDeviceToHost, s));
    WVG_STAMP(3);
    WVG_HIP(hipStreamSynchronize(s));  // also keeps q / win alive until their copies are done
#ifdef WVG_TOOLS
    WVG_STAMP(4);
    filtered_timing(tstamp);
#endif
    std::memcpy(out_ids, pin, (size_t)B * k * 8);
    std::memcpy(out_dists, pin + (o_d - o_ids), (size_t)B * k * 4);
    std::memcpy(out_counts, pin + (o_cnt - o_ids), (size_t)B * 4);
    return WVG_OK;
}

extern "C" {

int wvg_search_bq_rescore(wvg_corpus *bq, wvg_corpus *f32, const float *queries, uint32_t nq, uint32_t k,
                          uint32_t rescore_limit, const uint64_t *allow_bits, uint64_t allow_words, uint64_t *out_ids,
                          float *out_dists, uint32_t *out_counts)
{
    int rc = check_corpus(bq);
    if (rc) return rc;
    if (!f32 || bq->kind != WVG_KIND_BQ || f32->kind != WVG_KIND_F32)
        return fail(WVG_ERR_INVALID, "need a BQ corpus and an F32 corpus");
    if (bq->dim != f32->dim || bq->id_base != f32->id_base || bq->metric != f32->metric)
        return fail(WVG_ERR_INVALID, "BQ and F32 corpora disagree on dim/id_base/metric");
    if (nq > 0 && !queries) return fail(WVG_ERR_INVALID, "null queries");
    const uint32_t R = std::max(rescore_limit, k);  // searchTimeRescore (V/flat/index.go:297-305)
    std::shared_lock<std::shared_mutex> lk1(bq->rw);
    std::shared_lock<std::shared_mutex> lk2(f32->rw);
    SearchPlan p = plan_search(bq, nq, std::min(R, MAX_K), allow_bits, allow_words);
    if (p.empty || k == 0) {
        write_empty(nq, k, out_ids, out_dists, out_counts);
        return WVG_OK;
    }
    if (bq->ctx->opt.heap_replay)  // the reference heaps' exact result (wvg_replay.hip), any R
        return bq_rescore_replay(bq, f32, queries, nq, k, R, p, out_ids, out_dists, out_counts);
    if (R > MAX_K)
        return bq_rescore_large(bq, f32, queries, nq, k, R, allow_bits, allow_words, p, out_ids, out_dists,
                                out_counts);
    SlotGuard g(bq->ctx);
    rc = bq->ctx->acquire(&g.slot);
    if (rc) return rc;
    const uint32_t d = bq->dim;
    const uint32_t fpitch = f32_chunks(d) * 4;
    Carver cv;
    const size_t o_qb = cv.take(query_bytes(bq, nq));
    const size_t o_qf = cv.take((size_t)nq * fpitch * 4);
    const size_t o_allow = cv.take(p.allow_bytes());
    const size_t o_part = cv.take(p.workspace_bytes(nq, R));
    const size_t o_cand = cv.take((size_t)nq * R * 8);
    const size_t o_resc = cv.take((size_t)nq * R * 8);
    const size_t o_ids = cv.take((size_t)nq * k * 8);
    const size_t o_d = cv.take((size_t)nq * k * 4);
    const size_t o_cnt = cv.take((size_t)nq * 4);
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
    // Hamming top-R keys (slot in the low 32 bits): phase 1 + a keys-only phase 2
    ScanArgs a{};
    a.data = bq->d_data;
    a.valid = bq->d_valid;
    a.allow = d_allow;
    a.allow_words = d_allow ? p.te - p.tb : 0;
    a.allow_t0 = p.tb;
    a.id_base = bq->id_base;
    a.tile_begin = p.tb;
    a.tile_end = p.te;
    a.dim = d;
    a.nchunks = bq->nchunks;
    a.metric = bq->metric;
    a.queries = b + o_qb;
    a.qpitch = qpb;
    a.nq = nq;
    a.k = R;
    a.cosched = p.cosched;  // the plan's group count assumes the co-scheduled K5 grid (nq > 1)
    a.reverse = next_direction(bq, 1);
    uint64_t *part = (uint64_t *)(b + o_part);
    WVG_HIP(launch_scan_bq(a, part, p.groups, s));
    // Hamming top-R; ids are id_base + slot, so id_base = 0 keeps the slots
    uint64_t *cand_ids = (uint64_t *)(b + o_cand);
    WVG_HIP(launch_merge_lists(part, nq, (uint32_t)p.groups, R, R, 0, cand_ids, (float *)(b + o_resc), nullptr, s));
    // cand_ids now hold slots (or KEY_NONE); rescore them exactly against the f32 rows
    WVG_HIP(launch_rescore_keys(f32->metric, (const float *)(b + o_qf), qpf, (const float *)f32->d_data, d,
                                f32->nchunks, cand_ids, nq, R, R, (uint64_t *)(b + o_resc), s, f32->ctx->order512));
    WVG_HIP(launch_merge_keys((uint64_t *)(b + o_resc), nq, R, k, f32->id_base, (uint64_t *)(b + o_ids),
                              (float *)(b + o_d), (uint32_t *)(b + o_cnt), s));
    if (out_ids) WVG_HIP(hipMemcpyAsync(out_ids, b + o_ids, (size_t)nq * k * 8, hipMemcpyDeviceToHost, s));
    if (out_dists) WVG_HIP(hipMemcpyAsync(out_dists, b + o_d, (size_t)nq * k * 4, hipMemcpyDeviceToHost, s));
    if (out_counts) WVG_HIP(hipMemcpyAsync(out_counts, b + o_cnt, (size_t)nq * 4, hipMemcpyDeviceToHost, s));
    WVG_HIP(hipStreamSynchronize(s));
    return WVG_OK;
}

int wvg_search_bq_candidates(wvg_corpus *bq, const float *queries, uint32_t nq, uint32_t rescore_limit,
                             const uint64_t *allow_bits, uint64_t allow_words, uint64_t *out_ids, float *out_dists,
                             uint32_t *out_counts)
{
    int rc = check_corpus(bq);
    if (rc) return rc;
    if (bq->kind != WVG_KIND_BQ) return fail(WVG_ERR_INVALID, "need a BQ corpus");
    if (nq > 0 && !queries) return fail(WVG_ERR_INVALID, "null queries");
    const uint32_t R = rescore_limit;
    if (!bq->ctx->opt.heap_replay) {  // the lexicographic top-R, in pop (descending) order
        rc = wvg_search(bq, queries, nq, R, allow_bits, allow_words, out_ids, out_dists, out_counts);
        if (rc) return rc;
        for (uint32_t q = 0; q < nq; q++) {
            const uint32_t c = out_counts ? out_counts[q] : R;
            if (out_ids) std::reverse(out_ids + (size_t)q * R, out_ids + (size_t)q * R + c);
            if (out_dists) std::reverse(out_dists + (size_t)q * R, out_dists + (size_t)q * R + c);
        }
        return WVG_OK;
    }
    std::shared_lock<std::shared_mutex> lk(bq->rw);
    SearchPlan p = plan_search(bq, nq, std::min(R, MAX_K), allow_bits, allow_words);
    if (p.empty || R == 0) {
        write_empty(nq, R, out_ids, out_dists, out_counts);
        return WVG_OK;
    }
    return bq_rescore_replay(bq, nullptr, queries, nq, R, R, p, out_ids, out_dists, out_counts);
}

// Device-search workspaces start with a 256-byte status block (the sticky
// status word read by wvg_search_device_check); the scan workspace follows.
static const size_t WS_STATUS_BYTES = 256;

// Workspace of the query-stream scan (after the status block): partial lists
// [nq][groups][k], then the per-query arrival counters and the per-list ready
// words [nq][groups] (both zeroed per call by one memset).
struct StreamLayout {
    size_t partials = 0, arrivals = 0, ready = 0, total = 0;
};
static StreamLayout stream_layout(const SearchPlan &p1, uint32_t nq, uint32_t k)
{
    StreamLayout l;
    l.partials = WS_STATUS_BYTES;
    l.arrivals = l.partials + align_up((size_t)nq * p1.groups * k * 8, 256);
    l.ready = l.arrivals + align_up((size_t)nq * 4, 256);
    l.total = l.ready + align_up((size_t)nq * p1.groups * 4, 256);  // memset block: 16-B multiple
    return l;
}

size_t wvg_search_workspace_size(wvg_corpus *c, uint32_t nq, uint32_t k)
{
    if (!c) return 0;
    const uint32_t kk = std::max<uint32_t>(k, 1);
    SearchPlan p = plan_search(c, nq, k, nullptr, 0);
    const size_t dev = WS_STATUS_BYTES + align_up(p.workspace_bytes(nq, kk), 256) + device_query_bytes(c, nq);
    if (c->kind != WVG_KIND_F32) return dev;  // no pipelined mode
    SearchPlan p1 = plan_search(c, 1, k, nullptr, 0);  // pipelined: two single-query buffers, or the stream layout
    const size_t chain = 2 * align_up(p1.workspace_bytes(1, kk), 256);
    const size_t stream = stream_layout(p1, nq, kk).total;
    return std::max({dev, WS_STATUS_BYTES + chain, stream});
}

int wvg_search_device_check(wvg_ctx *ctx, void *d_workspace, void *stream)
{
    if (!ctx || !d_workspace) return fail(WVG_ERR_INVALID, "null ctx/workspace");
    WVG_HIP(hipSetDevice(ctx->device));
    hipStream_t s = (hipStream_t)stream;
    uint32_t st = 0;
    WVG_HIP(hipMemcpyAsync(&st, d_workspace, 4, hipMemcpyDeviceToHost, s));
    WVG_HIP(hipStreamSynchronize(s));
    if (st == 0) return WVG_OK;
    WVG_HIP(hipMemsetAsync(d_workspace, 0, 4, s));
    WVG_HIP(hipStreamSynchronize(s));
    if (st & WVG_STATUS_MERGE_TIMEOUT)
        return fail(WVG_ERR_DEVICE, "query-stream merge timed out waiting for the scan workgroups; "
                                    "the affected queries returned empty results");
    return fail(WVG_ERR_DEVICE, "device search status " + std::to_string(st));
}

int wvg_search_device_pipelined(wvg_corpus *c, const float *d_queries, uint32_t nq, uint32_t k, uint64_t *d_ids,
                                float *d_dists, uint32_t *d_counts, void *d_workspace, size_t workspace_bytes,
                                void *stream)
{
    if (!c) return fail(WVG_ERR_INVALID, "null corpus");
    if (k > MAX_K) return fail(WVG_ERR_UNSUPPORTED, "k above 256 is not supported by the fused top-k");
    if (c->kind != WVG_KIND_F32) return fail(WVG_ERR_UNSUPPORTED, "pipelined search supports F32 corpora");
    if (c->dim % 4 != 0) return fail(WVG_ERR_UNSUPPORTED, "device search needs dim % 4 == 0");
    if (nq == 0 || k == 0) return WVG_OK;
    hipStream_t s = (hipStream_t)stream;
    std::shared_lock<std::shared_mutex> lk(c->rw);
    SearchPlan p = plan_search(c, 1, k, nullptr, 0);
    if (p.empty) {  // empty corpus / slab: empty results, as wvg_search's write_empty
        WVG_HIP(launch_fill_empty(d_ids, d_dists, d_counts, nq, k, s));
        return WVG_OK;
    }
    if (tuning().pipeline_mode == 1) {  // query-stream kernel: one launch for all nq queries (the product path)
        const StreamLayout l = stream_layout(p, nq, k);
        if (!d_workspace || workspace_bytes < l.total) return fail(WVG_ERR_INVALID, "workspace too small");
        char *w = (char *)d_workspace;
        StreamJob j{};
        j.partials = (uint64_t *)(w + l.partials);
        j.arrivals = (uint32_t *)(w + l.arrivals);
        j.status = (uint32_t *)w;
        const uint32_t wait_us = tuning().merge_wait_us > 0 ? (uint32_t)tuning().merge_wait_us : c->ctx->opt.merge_wait_us;
        j.wait_limit = wait_us > 0 ? (uint64_t)wait_us * 100ull : 400000000ull;
        j.groups = (uint32_t)p.groups;
        j.ids = d_ids;
        j.dists = d_dists;
        j.counts = d_counts;
        ScanArgs a{};
        a.data = c->d_data;
        a.valid = c->d_valid;
        a.id_base = c->id_base;
        a.tile_begin = p.tb;
        a.tile_end = p.te;
        a.dim = c->dim;
        a.nchunks = c->nchunks;
        a.metric = c->metric;
        a.queries = d_queries;
        a.qpitch = c->dim;
        a.nq = nq;
        a.k = k;
        a.reverse = next_direction(c, nq);
        a.order512 = c->ctx->order512;
        a.plain = plain_loads(c, p.tb, p.te);
        a.cache_tail256 = k1_cache_tail(c, p.tb, p.te);
        j.row_split = (tuning().stream_variant & 1) == 0;
        if ((tuning().stream_variant & 2) == 0) {  // per-list hand-offs; the words are zeroed with the counters
            j.ready = (uint32_t *)(w + l.ready);
            j.ready_tag = 1;
        }
        WVG_HIP(hipMemsetAsync(j.arrivals, 0, l.total - l.arrivals, s));
        ProfArm arm(c->ctx);
        if (arm.rc) return arm.rc;
        WVG_HIP(launch_scan_f32_stream(a, j, s));
        return WVG_OK;
    }
#ifdef WVG_TOOLS
    // A/B (pipeline_mode 0): one scan launch per query, query i's launch merging query i-1
    const size_t half = align_up(p.workspace_bytes(1, k), 256);
    if (!d_workspace || workspace_bytes < WS_STATUS_BYTES + 2 * half) return fail(WVG_ERR_INVALID, "workspace too small");
    char *w0 = (char *)d_workspace + WS_STATUS_BYTES;
    uint64_t *buf[2] = {(uint64_t *)w0, (uint64_t *)(w0 + half)};
    ScanArgs a{};
    a.data = c->d_data;
    a.valid = c->d_valid;
    a.id_base = c->id_base;
    a.tile_begin = p.tb;
    a.tile_end = p.te;
    a.dim = c->dim;
    a.nchunks = c->nchunks;
    a.metric = c->metric;
    a.qpitch = c->dim;
    a.nq = 1;
    a.k = k;
    a.order512 = c->ctx->order512;
    a.plain = plain_loads(c, p.tb, p.te);
    a.cache_tail256 = k1_cache_tail(c, p.tb, p.te);
    const uint32_t dir0 = next_direction(c, nq);
    for (uint32_t i = 0; i < nq; i++) {
        a.queries = d_queries + (size_t)i * c->dim;
        a.reverse = (dir0 + i) & 1u;
        a.side = MergeJob{};
        if (i > 0) {
            a.side = MergeJob{buf[(i - 1) & 1], (uint32_t)p.groups, k, k, c->id_base, d_ids + (size_t)(i - 1) * k,
                              d_dists + (size_t)(i - 1) * k, d_counts ? d_counts + (i - 1) : nullptr, 1};
        }
        ProfArm arm(c->ctx);
        if (arm.rc) return arm.rc;
        WVG_HIP(launch_scan_f32(a, buf[i & 1], p.groups, s));
    }
    const uint32_t last = nq - 1;
    WVG_HIP(launch_merge_lists(buf[last & 1], 1, (uint32_t)p.groups, k, k, c->id_base, d_ids + (size_t)last * k,
                               d_dists + (size_t)last * k, d_counts ? d_counts + last : nullptr, s));
    return WVG_OK;
#else
    return fail(WVG_ERR_UNSUPPORTED, "pipeline mode");
#endif
}

int wvg_search_device(wvg_corpus *c, const float *d_queries, uint32_t nq, uint32_t k, uint64_t *d_ids, float *d_dists,
                      uint32_t *d_counts, void *d_workspace, size_t workspace_bytes, void *stream)
{
    if (!c) return fail(WVG_ERR_INVALID, "null corpus");
    if (k > MAX_K) return fail(WVG_ERR_UNSUPPORTED, "k above 256 is not supported by the fused top-k");
    if (c->kind == WVG_KIND_F32 && c->dim % 4 != 0)
        return fail(WVG_ERR_UNSUPPORTED, "device search needs dim % 4 == 0");
    if (c->kind == WVG_KIND_PQ && !c->d_centers) return fail(WVG_ERR_INVALID, "PQ corpus has no codebook");
    if (nq == 0 || k == 0) return WVG_OK;
    hipStream_t s = (hipStream_t)stream;
    std::shared_lock<std::shared_mutex> lk(c->rw);
    SearchPlan p = plan_search(c, nq, k, nullptr, 0);
    if (p.empty) {  // empty corpus / slab (e.g. a rank with no rows): empty results
        WVG_HIP(launch_fill_empty(d_ids, d_dists, d_counts, nq, k, s));
        return WVG_OK;
    }
    const size_t part = align_up(p.workspace_bytes(nq, k), 256);
    if (!d_workspace || workspace_bytes < WS_STATUS_BYTES + part + device_query_bytes(c, nq))
        return fail(WVG_ERR_INVALID, "workspace too small");
    uint64_t *partials = (uint64_t *)((char *)d_workspace + WS_STATUS_BYTES);
    char *qbuf = (char *)d_workspace + WS_STATUS_BYTES + part;
    if (c->kind == WVG_KIND_PQ) {  // the queries' LUTs on the device (CH/product_quantization.go:329-337)
        WVG_HIP(launch_pq_lut(c->metric, d_queries, nq, c->dim, c->d_centers, c->pq_m, c->pq_ks, c->pq_ds,
                              (float *)qbuf, s));
        return run_search(c, qbuf, c->pq_m * c->pq_ks, nq, k, nullptr, p, partials, d_ids, d_dists, d_counts, s);
    }
    if (c->kind == WVG_KIND_BQ) {  // sign bits (CH/binary_quantization.go:32-45) at the scan's query pitch
        const uint32_t words = bq_words(c->dim), qpitch = bq_chunks(c->dim) * 2;
        uint64_t *codes = (uint64_t *)(qbuf + align_up((size_t)nq * qpitch * 8, 256));
        WVG_HIP(launch_bq_encode_rows(d_queries, nq, c->dim, 0, codes, s));
        WVG_HIP(hipMemsetAsync(qbuf, 0, (size_t)nq * qpitch * 8, s));
        WVG_HIP(hipMemcpy2DAsync(qbuf, (size_t)qpitch * 8, codes, (size_t)words * 8, (size_t)words * 8, nq,
                                 hipMemcpyDeviceToDevice, s));
        return run_search(c, qbuf, qpitch, nq, k, nullptr, p, partials, d_ids, d_dists, d_counts, s);
    }
    return run_search(c, d_queries, c->dim, nq, k, nullptr, p, partials, d_ids, d_dists, d_counts, s);
}

int wvg_topk_merge_device(wvg_ctx *ctx, const float *d_dists, const uint64_t *d_ids, uint32_t nq, uint32_t nlists,
                          uint32_t k_in, uint32_t k, uint64_t *d_out_ids, float *d_out_dists, uint32_t *d_out_counts,
                          void *stream)
{
    if (!ctx) return fail(WVG_ERR_INVALID, "null ctx");
    if ((uint64_t)nlists * k_in > 8192) return fail(WVG_ERR_UNSUPPORTED, "merge input above 8192 pairs per query");
    if (nq == 0 || k == 0) return WVG_OK;
    const uint64_t stride = (uint64_t)nq * k_in;
    WVG_HIP(launch_merge_pairs(d_dists, d_ids, stride, stride, nq, nlists, k_in, k, d_out_ids, d_out_dists,
                               d_out_counts, (hipStream_t)stream));
    return WVG_OK;
}

size_t wvg_topk_packed_bytes(uint32_t nq, uint32_t k) { return align_up((size_t)nq * k * 12, 16); }

int wvg_topk_merge_packed(wvg_ctx *ctx, const void *d_packed, uint32_t nq, uint32_t nlists, uint32_t k_in, uint32_t k,
                          uint64_t *d_out_ids, float *d_out_dists, uint32_t *d_out_counts, void *stream)
{
    if (!ctx || !d_packed) return fail(WVG_ERR_INVALID, "null ctx/input");
    if ((uint64_t)nlists * k_in > 8192) return fail(WVG_ERR_UNSUPPORTED, "merge input above 8192 pairs per query");
    if (nq == 0 || k == 0) return WVG_OK;
    const size_t block = wvg_topk_packed_bytes(nq, k_in);
    const char *b = (const char *)d_packed;
    WVG_HIP(launch_merge_pairs((const float *)(b + (size_t)nq * k_in * 8), (const uint64_t *)b, block / 8, block / 4,
                               nq, nlists, k_in, k, d_out_ids, d_out_dists, d_out_counts, (hipStream_t)stream));
    return WVG_OK;
}

int wvg_corpus_distance_by_ids(wvg_corpus *c, const float *query, const uint64_t *ids, uint64_t n, float *out_dists,
                               uint8_t *out_ok)
{
    int rc = check_corpus(c);
    if (rc) return rc;
    if (!query || (n && (!ids || !out_dists || !out_ok))) return fail(WVG_ERR_INVALID, "null argument");
    if (c->kind == WVG_KIND_PQ && !c->d_centers) return fail(WVG_ERR_INVALID, "PQ corpus has no codebook");
    if (n == 0) return WVG_OK;
    std::shared_lock<std::shared_mutex> lk(c->rw);
    SlotGuard g(c->ctx);
    rc = c->ctx->acquire(&g.slot);
    if (rc) return rc;
    Carver cv;
    const size_t o_q = cv.take(query_bytes(c, 1));
    const size_t o_qtmp = cv.take(c->kind == WVG_KIND_PQ ? (size_t)c->dim * 4 : 0);
    const size_t o_ids = cv.take(n * 8), o_d = cv.take(n * 4), o_ok = cv.take(n);
    void *base = nullptr;
    rc = g.slot->device_scratch(cv.off, &base);
    if (rc) return rc;
    char *b = (char *)base;
    hipStream_t s = g.slot->stream;
    const size_t out_b = o_ok + n - o_d;  // [dists | ok]
    Staging st;
    rc = st.reserve(g.slot, stage_bytes(staged_query_bytes(c, 1)) + stage_bytes(n * 8) + stage_bytes(out_b));
    if (rc) return rc;
    uint32_t qpitch = 0;
    rc = stage_queries(c, g.slot, query, 1, b + o_q, qpitch, (float *)(b + o_q), b + o_qtmp, &st);
    if (rc) return rc;
    WVG_HIP(st.h2d(b + o_ids, ids, n * 8, s));
    ScanArgs a = scan_args_for(c, b + o_q, qpitch, 1, 1, nullptr, 0, tiles_of(c->high_water));
    WVG_HIP(launch_dist_by_ids(a, c->kind, c->capacity, (const uint64_t *)(b + o_ids), n, (float *)(b + o_d),
                               (uint8_t *)(b + o_ok), s));
    if (out_b <= STAGE_MAX) {
        char *pin = st.take(out_b);
        WVG_HIP(hipMemcpyAsync(pin, b + o_d, out_b, hipMemcpyDeviceToHost, s));
        WVG_HIP(hipStreamSynchronize(s));
        std::memcpy(out_dists, pin, n * 4);
        std::memcpy(out_ok, pin + (o_ok - o_d), n);
        return WVG_OK;
    }
    WVG_HIP(hipMemcpyAsync(out_dists, b + o_d, n * 4, hipMemcpyDeviceToHost, s));
    WVG_HIP(hipMemcpyAsync(out_ok, b + o_ok, n, hipMemcpyDeviceToHost, s));
    WVG_HIP(hipStreamSynchronize(s));
    return WVG_OK;
}

int wvg_corpus_distance_by_ids_batch(wvg_corpus *c, const float *queries, uint32_t nq, const uint64_t *offsets,
                                     const uint64_t *ids, float *out_dists, uint8_t *out_ok)
{
    int rc = check_corpus(c);
    if (rc) return rc;
    if (nq == 0) return WVG_OK;
    if (!queries || !offsets) return fail(WVG_ERR_INVALID, "null argument");
    if (offsets[0] != 0) return fail(WVG_ERR_INVALID, "offsets[0] must be 0");
    for (uint32_t q = 0; q < nq; q++)
        if (offsets[q + 1] < offsets[q]) return fail(WVG_ERR_INVALID, "offsets must be non-decreasing");
    const uint64_t n = offsets[nq];
    if (n && (!ids || !out_dists || !out_ok)) return fail(WVG_ERR_INVALID, "null argument");
    if (c->kind == WVG_KIND_PQ && !c->d_centers) return fail(WVG_ERR_INVALID, "PQ corpus has no codebook");
    if (n == 0) return WVG_OK;
    std::vector<uint32_t> qidx(n);
    for (uint32_t q = 0; q < nq; q++)
        for (uint64_t i = offsets[q]; i < offsets[q + 1]; i++) qidx[i] = q;
    std::shared_lock<std::shared_mutex> lk(c->rw);
    SlotGuard g(c->ctx);
    rc = c->ctx->acquire(&g.slot);
    if (rc) return rc;
    Carver cv;
    const size_t o_q = cv.take(query_bytes(c, nq));
    const size_t o_qtmp = cv.take(c->kind == WVG_KIND_PQ ? (size_t)nq * c->dim * 4 : 0);
    const size_t o_ids = cv.take(n * 8), o_qi = cv.take(n * 4), o_d = cv.take(n * 4), o_ok = cv.take(n);
    void *base = nullptr;
    rc = g.slot->device_scratch(cv.off, &base);
    if (rc) return rc;
    char *b = (char *)base;
    hipStream_t s = g.slot->stream;
    uint32_t qpitch = 0;
    rc = stage_queries(c, g.slot, queries, nq, b + o_q, qpitch, (float *)(b + o_q), b + o_qtmp);
    if (rc) return rc;
    WVG_HIP(hipMemcpyAsync(b + o_ids, ids, n * 8, hipMemcpyHostToDevice, s));
    WVG_HIP(hipMemcpyAsync(b + o_qi, qidx.data(), n * 4, hipMemcpyHostToDevice, s));
    ScanArgs a = scan_args_for(c, b + o_q, qpitch, nq, 1, nullptr, 0, tiles_of(c->high_water));
    WVG_HIP(launch_dist_by_ids(a, c->kind, c->capacity, (const uint64_t *)(b + o_ids), n, (float *)(b + o_d),
                               (uint8_t *)(b + o_ok), s, (const uint32_t *)(b + o_qi)));
    WVG_HIP(hipMemcpyAsync(out_dists, b + o_d, n * 4, hipMemcpyDeviceToHost, s));
    WVG_HIP(hipMemcpyAsync(out_ok, b + o_ok, n, hipMemcpyDeviceToHost, s));
    WVG_HIP(hipStreamSynchronize(s));  // also keeps qidx alive until its copy is done
    return WVG_OK;
}

}  // extern "C"
