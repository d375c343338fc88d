// wvg_corpus.hip -- device-resident corpora: allocation and growth, writes
// (flat.Add / AddBatch / Delete, V/flat/index.go:197-295; the PostStartup
// bulk load, :640-681), reads by id (vectorById, :401-407), the PQ codebook
// (NewProductQuantizer validation, CH/product_quantization.go:187-197) and
// the bf16 shadow state of F32 dot / cosine corpora (K3c / K3d).

#include <cstring>

#include "wvg_host.hpp"

namespace wvg {

size_t corpus_row_bytes(int kind, uint32_t dim, uint32_t pq_m)
{
    switch (kind) {
    case WVG_KIND_F32: return (size_t)f32_chunks(dim) * 16;
    case WVG_KIND_BQ: return (size_t)bq_chunks(dim) * 16;
    default: return (size_t)pq_chunks(pq_m) * 16;
    }
}

// Bytes of one row as the caller hands it over (and as the LSM buckets store
// it): F32 dim float32, BQ ceil(dim/64) uint64 words, PQ m code bytes.
static size_t host_row_bytes(const wvg_corpus *c)
{
    switch (c->kind) {
    case WVG_KIND_F32: return (size_t)c->dim * 4;
    case WVG_KIND_BQ: return (size_t)bq_words(c->dim) * 8;
    default: return c->pq_m;
    }
}

static uint32_t corpus_nchunks(const wvg_corpus *c)
{
    switch (c->kind) {
    case WVG_KIND_F32: return f32_chunks(c->dim);
    case WVG_KIND_BQ: return bq_chunks(c->dim);
    default: return pq_chunks(c->pq_m);
    }
}

// Rows of tiles [t0, t1) were (re)written: the shadow rebuilds them at the
// next screened search.  Callers hold the corpus lock exclusively.
void shadow_mark(wvg_corpus *c, uint64_t t0, uint64_t t1)
{
    if (!c->d_shadow || t1 <= t0) return;
    if (c->sh_dirty_lo >= c->sh_dirty_hi) {
        c->sh_dirty_lo = t0;
        c->sh_dirty_hi = t1;
    } else {
        c->sh_dirty_lo = std::min(c->sh_dirty_lo, t0);
        c->sh_dirty_hi = std::max(c->sh_dirty_hi, t1);
    }
}

void shadow_free(wvg_corpus *c)
{
    if (c->d_shadow) (void)hipFree(c->d_shadow);
    if (c->d_norms) (void)hipFree(c->d_norms);
    if (c->d_nmax) (void)hipFree(c->d_nmax);
    if (c->d_errs) (void)hipFree(c->d_errs);
    c->d_shadow = nullptr;
    c->d_norms = nullptr;
    c->d_nmax = nullptr;
    c->d_errs = nullptr;
    c->sh_i8 = false;
    c->sh_dirty_lo = c->sh_dirty_hi = 0;
    c->sh_failed = false;  // a failed allocation is retried at the next screened search
}

// The bf16 shadow (fragments + row norms) of an F32 dot / cosine corpus,
// allocated on first use and rebuilt over the tiles written since the last
// build; ordered before the caller's screen on stream s.  False when it
// cannot be allocated (the batch then runs the exact path).  Under stream
// capture (a device search recorded into a hipGraph) nothing is allocated,
// built or waited for on the stream: a shadow that is not built and clean
// gives false (the exact path, sh_failed untouched), a clean one is waited
// for on the host -- a wait on an event recorded outside the capture would
// invalidate it.
bool ensure_shadow(wvg_corpus *c, hipStream_t s)
{
    std::lock_guard<std::mutex> g(c->sh_mu);
    if (c->sh_failed) return false;
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(s, &cs) != hipSuccess) {
        (void)hipGetLastError();
        cs = hipStreamCaptureStatusNone;
    }
    if (cs != hipStreamCaptureStatusNone) {
        if (!c->d_shadow || c->sh_dirty_lo < c->sh_dirty_hi || !c->sh_ready) return false;
        return hipEventSynchronize(c->sh_ready) == hipSuccess;
    }
    const uint64_t tiles = tiles_of(c->capacity);
    if (!c->d_shadow) {
        void *sh = nullptr, *nr = nullptr, *mx = nullptr, *er = nullptr;
        auto fail = [&]() {
            (void)hipGetLastError();
            (void)hipStreamSynchronize(s);
            if (sh) (void)hipFree(sh);
            if (nr) (void)hipFree(nr);
            if (mx) (void)hipFree(mx);
            if (er) (void)hipFree(er);
            c->sh_failed = true;
            return false;
        };
        if (hipMalloc(&mx, 256) != hipSuccess || hipMemsetAsync(mx, 0, 256, s) != hipSuccess) return fail();
        // K3i (the int8 screen, option batch_screen = 2) where its dims apply: the corpus
        // scale S = the largest finite |x| / 127 of the rows written so far (one pass and
        // one host wait, at the shadow's first build); no rows / all zeros / an extreme
        // scale keep the bf16 shadow
        bool i8 = c->ctx->opt.batch_screen == 2 && screen_i8_supported(c->dim) && c->high_water > 0;
        float sc[2] = {1.f, 1.f};
        if (i8) {
            uint32_t amax_bits = 0;
            if (launch_shadow_maxabs((const float *)c->d_data, c->dim, tiles_of(c->high_water), (uint32_t *)mx, s) !=
                    hipSuccess ||
                hipMemcpyAsync(&amax_bits, mx, 4, hipMemcpyDeviceToHost, s) != hipSuccess ||
                hipStreamSynchronize(s) != hipSuccess || hipMemsetAsync(mx, 0, 256, s) != hipSuccess)
                return fail();
            float amax;
            std::memcpy(&amax, &amax_bits, 4);
            sc[0] = amax / 127.f;
            sc[1] = 1.f / sc[0];
            i8 = sc[0] >= 0x1p-100f && sc[0] <= 0x1p100f;
            if (i8 && hipMemcpyAsync((uint32_t *)mx + 2, sc, 8, hipMemcpyHostToDevice, s) != hipSuccess) return fail();
            if (i8 && hipStreamSynchronize(s) != hipSuccess) return fail();  // (sc is on this stack)
        }
        const uint32_t kbn = i8 ? c->dim / 64 : screen_kblocks(c->dim);
        const size_t sbytes = (size_t)(tiles + 4) * kbn * 4 * 1024, nbytes = (size_t)(tiles + 4) * 64 * 4;
        if (hipMalloc(&sh, sbytes) != hipSuccess || hipMalloc(&nr, nbytes) != hipSuccess ||
            (i8 && hipMalloc(&er, nbytes) != hipSuccess) || hipMemsetAsync(sh, 0, sbytes, s) != hipSuccess ||
            hipMemsetAsync(nr, 0, nbytes, s) != hipSuccess || (er && hipMemsetAsync(er, 0, nbytes, s) != hipSuccess) ||
            (!c->sh_ready && hipEventCreateWithFlags(&c->sh_ready, hipEventDisableTiming) != hipSuccess))
            return fail();
        c->d_shadow = sh;
        c->d_norms = (float *)nr;
        c->d_nmax = (uint32_t *)mx;
        c->d_errs = (float *)er;
        c->sh_i8 = i8;
        c->sh_dirty_lo = 0;
        c->sh_dirty_hi = tiles_of(c->high_water);
    }
    if (c->sh_dirty_lo < c->sh_dirty_hi) {
        const hipError_t e =
            c->sh_i8 ? launch_shadow_build_i8((const float *)c->d_data, c->dim, c->sh_dirty_lo, c->sh_dirty_hi,
                                              c->d_shadow, c->d_norms, c->d_errs, c->d_nmax, s)
                     : launch_shadow_build((const float *)c->d_data, c->dim, c->sh_dirty_lo, c->sh_dirty_hi,
                                           c->d_shadow, c->d_norms, c->d_nmax, s);
        if (e != hipSuccess || hipEventRecord(c->sh_ready, s) != hipSuccess) return false;
        c->sh_dirty_lo = c->sh_dirty_hi = 0;
        return true;
    }
    return hipStreamWaitEvent(s, c->sh_ready, 0) == hipSuccess;
}

}  // namespace wvg

using namespace wvg;

extern "C" {

// ---------------------------------------------------------------------------
// (Re)allocates the row tiles and validity words for `capacity` rows, keeping
// the rows of the old allocation.  The zero fill and the copy of the old rows
// run on a pool stream and complete before this returns: every later writer
// (upsert, synthetic fill, load_kv) runs on a non-blocking pool stream, which
// does not order against the legacy null stream, so a null-stream memset
// could land after -- and wipe -- rows written right after creation.  On any
// failure the new buffers are freed and the corpus keeps its old storage.
static int corpus_alloc(wvg_corpus *c, uint64_t capacity)
{
    const uint64_t tiles = tiles_of(capacity);
    const size_t row_bytes = corpus_row_bytes(c->kind, c->dim, c->pq_m);
    void *data = nullptr;
    uint64_t *valid = nullptr;
    auto drop = [&](int code, const char *what, hipError_t e) {
        if (data) (void)hipFree(data);
        if (valid) (void)hipFree(valid);
        return fail(code, std::string(what) + ": " + hipGetErrorString(e));
    };
    shadow_free(c);  // sized by the capacity (rebuilt at the next screened search): never beside the new rows
    if (tiles > 0) {
        hipError_t e;
        if (row_bytes > 0 && (e = hipMalloc(&data, tiles * 64 * row_bytes)) != hipSuccess) {
            data = nullptr;
            return drop(WVG_ERR_NOMEM, "corpus hipMalloc", e);
        }
        if ((e = hipMalloc(&valid, tiles * 8)) != hipSuccess) {
            valid = nullptr;
            return drop(WVG_ERR_NOMEM, "validity hipMalloc", e);
        }
        SlotGuard g(c->ctx);
        int rc = c->ctx->acquire(&g.slot);
        if (rc) {
            if (data) (void)hipFree(data);
            (void)hipFree(valid);
            return rc;
        }
        const hipStream_t s = g.slot->stream;
        const uint64_t keep = std::min(tiles_of(c->capacity), tiles);
        const size_t keep_data = (c->d_data && data) ? keep * 64 * row_bytes : 0;
        const size_t keep_valid = c->d_valid ? keep * 8 : 0;
        if (data && keep_data && (e = hipMemcpyAsync(data, c->d_data, keep_data, hipMemcpyDeviceToDevice, s)) != hipSuccess)
            return drop(WVG_ERR_DEVICE, "corpus row copy", e);
        if (data && (e = hipMemsetAsync((char *)data + keep_data, 0, tiles * 64 * row_bytes - keep_data, s)) != hipSuccess)
            return drop(WVG_ERR_DEVICE, "corpus zero fill", e);
        if (keep_valid && (e = hipMemcpyAsync(valid, c->d_valid, keep_valid, hipMemcpyDeviceToDevice, s)) != hipSuccess)
            return drop(WVG_ERR_DEVICE, "validity copy", e);
        if ((e = hipMemsetAsync((char *)valid + keep_valid, 0, tiles * 8 - keep_valid, s)) != hipSuccess)
            return drop(WVG_ERR_DEVICE, "validity zero fill", e);
        if ((e = hipStreamSynchronize(s)) != hipSuccess) return drop(WVG_ERR_DEVICE, "corpus alloc sync", e);
    }
    if (c->d_data) (void)hipFree(c->d_data);
    if (c->d_valid) (void)hipFree(c->d_valid);
    c->d_data = data;
    c->d_valid = valid;
    c->capacity = tiles * 64;
    c->h_valid.resize(tiles, 0ull);
    return WVG_OK;
}

int wvg_corpus_create(wvg_ctx *ctx, int kind, int metric, uint32_t dim, uint64_t id_base, uint64_t capacity,
                      wvg_corpus **out)
{
    if (!ctx || !out) return fail(WVG_ERR_INVALID, "null ctx/out");
    *out = nullptr;
    if (kind < WVG_KIND_F32 || kind > WVG_KIND_PQ) return fail(WVG_ERR_INVALID, "unknown corpus kind");
    if (metric < WVG_METRIC_L2 || metric > WVG_METRIC_HAMMING) return fail(WVG_ERR_INVALID, "unknown metric");
    if (dim == 0) return fail(WVG_ERR_INVALID, "dim must be > 0");
    if (id_base % 64 != 0) return fail(WVG_ERR_INVALID, "id_base must be a multiple of 64");
    if (capacity > (1ull << 32)) return fail(WVG_ERR_INVALID, "capacity above 2^32 rows per corpus");
    WVG_HIP(hipSetDevice(ctx->device));
    wvg_corpus *c = new wvg_corpus();
    c->ctx = ctx;
    c->kind = kind;
    c->metric = metric;
    c->dim = dim;
    c->id_base = id_base;
    c->nchunks = kind == WVG_KIND_PQ ? 0 : corpus_nchunks(c);
    int rc = corpus_alloc(c, capacity);
    if (rc != WVG_OK) {
        delete c;
        return rc;
    }
    *out = c;
    return WVG_OK;
}

int wvg_corpus_destroy(wvg_corpus *c)
{
    if (!c) return WVG_OK;
    (void)hipSetDevice(c->ctx->device);
    if (c->d_data) (void)hipFree(c->d_data);
    if (c->d_valid) (void)hipFree(c->d_valid);
    if (c->d_centers) (void)hipFree(c->d_centers);
    shadow_free(c);
    if (c->sh_ready) (void)hipEventDestroy(c->sh_ready);
    delete c;
    return WVG_OK;
}

int wvg_corpus_reserve(wvg_corpus *c, uint64_t capacity)
{
    int rc = check_corpus(c);
    if (rc) return rc;
    std::unique_lock<std::shared_mutex> lk(c->rw);
    if (capacity <= c->capacity) return WVG_OK;
    if (capacity > (1ull << 32)) return fail(WVG_ERR_INVALID, "capacity above 2^32 rows per corpus");
    return corpus_alloc(c, capacity);
}

int wvg_corpus_info(wvg_corpus *c, uint64_t *count, uint64_t *high_water, uint64_t *capacity)
{
    if (!c) return fail(WVG_ERR_INVALID, "null corpus");
    std::shared_lock<std::shared_mutex> lk(c->rw);
    if (count) *count = c->count;
    if (high_water) *high_water = c->high_water;
    if (capacity) *capacity = c->capacity;
    return WVG_OK;
}

// Maps ids to slots, dedups (last occurrence wins, as sequential flat.Add
// calls would) and updates the host validity mirror.  Returns the row
// indices to store, in input order.
static int map_slots(wvg_corpus *c, const uint64_t *ids, uint64_t n, std::vector<uint64_t> &rows,
                     std::vector<uint64_t> &slots)
{
    std::vector<std::pair<uint64_t, uint64_t>> v;
    v.reserve(n);
    for (uint64_t i = 0; i < n; i++) {
        if (ids[i] < c->id_base || ids[i] - c->id_base >= c->capacity)
            return fail(WVG_ERR_CAPACITY, "id " + std::to_string(ids[i]) + " outside corpus [" +
                                              std::to_string(c->id_base) + ", " +
                                              std::to_string(c->id_base + c->capacity) + ")");
        v.emplace_back(ids[i] - c->id_base, i);
    }
    std::stable_sort(v.begin(), v.end(), [](auto &a, auto &b) { return a.first < b.first; });
    rows.clear();
    slots.clear();
    for (size_t j = 0; j < v.size(); j++) {
        if (j + 1 < v.size() && v[j + 1].first == v[j].first) continue;  // a later duplicate wins
        rows.push_back(v[j].second);
        slots.push_back(v[j].first);
    }
    return WVG_OK;
}

static void mark_valid_host(wvg_corpus *c, const std::vector<uint64_t> &slots)
{
    for (uint64_t s : slots) {
        uint64_t &w = c->h_valid[s >> 6];
        const uint64_t bit = 1ull << (s & 63);
        if (!(w & bit)) {
            w |= bit;
            c->count++;
        }
        c->high_water = std::max(c->high_water, s + 1);
    }
}

// Stores `nr` rows (host floats, gathered by rows[]) into the corpus.
static int store_rows(wvg_corpus *c, StreamSlot *sl, const float *vectors, const std::vector<uint64_t> &rows,
                      const std::vector<uint64_t> &slots, uint64_t r0, uint64_t r1)
{
    const uint64_t nr = r1 - r0;
    const uint32_t d = c->dim;
    hipStream_t s = sl->stream;
    Carver cv;
    const size_t o_rows = cv.take(nr * d * 4);
    const size_t o_norm = cv.take(nr * d * 4);
    const size_t o_slots = cv.take(nr * 8);
    const size_t o_codes = cv.take(nr * std::max<size_t>(bq_words(d) * 8, c->pq_m));
    const size_t o_tile = cv.take(tiles_of(nr) * 64 * (size_t)f32_chunks(d) * 16);
    void *base = nullptr;
    int rc = sl->device_scratch(cv.off, &base);
    if (rc) return rc;
    char *b = (char *)base;
    float *d_rows = (float *)(b + o_rows);
    float *d_norm = (float *)(b + o_norm);
    uint64_t *d_slots = (uint64_t *)(b + o_slots);
    // gather the selected host rows into pinned staging
    void *pin = nullptr;
    rc = sl->host_pinned(nr * d * 4 + nr * 8, &pin);
    if (rc) return rc;
    float *hrows = (float *)pin;
    uint64_t *hslots = (uint64_t *)((char *)pin + nr * d * 4);
    for (uint64_t i = 0; i < nr; i++) {
        std::memcpy(hrows + i * d, vectors + rows[r0 + i] * d, (size_t)d * 4);
        hslots[i] = slots[r0 + i];
    }
    WVG_HIP(hipMemcpyAsync(d_rows, hrows, nr * d * 4, hipMemcpyHostToDevice, s));
    WVG_HIP(hipMemcpyAsync(d_slots, hslots, nr * 8, hipMemcpyHostToDevice, s));
    const float *src = d_rows;
    if (c->metric == WVG_METRIC_COSINE) {  // flat.Add normalizes (V/flat/index.go:258)
        WVG_HIP(launch_normalize_rows(d_rows, nr, d, d_norm, s));
        src = d_norm;
    }
    switch (c->kind) {
    case WVG_KIND_F32:
        WVG_HIP(launch_f32_store(src, d_slots, nr, d, c->nchunks, 0, (float *)c->d_data, s));
        break;
    case WVG_KIND_BQ: {
        uint64_t *codes = (uint64_t *)(b + o_codes);
        WVG_HIP(launch_bq_encode_rows(src, nr, d, 0, codes, s));
        WVG_HIP(launch_bq_store(codes, d_slots, nr, bq_words(d), c->nchunks, (uint64_t *)c->d_data, s));
        break;
    }
    default: {
        uint8_t *codes = (uint8_t *)(b + o_codes);
        float *tile = (float *)(b + o_tile);
        WVG_HIP(launch_f32_store(src, nullptr, nr, d, f32_chunks(d), 0, tile, s));
        WVG_HIP(launch_pq_encode(tile, nr, d, c->d_centers, c->pq_m, c->pq_ks, codes, s, false, c->pq_nan_free));
        WVG_HIP(launch_pq_store(codes, d_slots, nr, c->pq_m, c->nchunks, (uint8_t *)c->d_data, s));
        break;
    }
    }
    WVG_HIP(launch_set_valid(c->d_valid, d_slots, nr, 1, s));
    WVG_HIP(hipStreamSynchronize(s));
    return WVG_OK;
}

static const uint64_t UPSERT_BATCH = 1u << 18;

int wvg_corpus_upsert(wvg_corpus *c, const uint64_t *ids, const float *vectors, uint64_t n, uint32_t dim)
{
    int rc = check_corpus(c);
    if (rc) return rc;
    if (n == 0) return WVG_OK;
    if (!ids || !vectors) return fail(WVG_ERR_INVALID, "null ids/vectors");
    if (dim != c->dim) return fail(WVG_ERR_DIM_MISMATCH, "insert called with a vector of the wrong size");
    if (c->kind == WVG_KIND_PQ && !c->d_centers) return fail(WVG_ERR_INVALID, "PQ corpus has no codebook");
    std::unique_lock<std::shared_mutex> lk(c->rw);
    std::vector<uint64_t> rows, slots;
    rc = map_slots(c, ids, n, rows, slots);
    if (rc) return rc;
    SlotGuard g(c->ctx);
    rc = c->ctx->acquire(&g.slot);
    if (rc) return rc;
    if (!slots.empty()) shadow_mark(c, slots.front() >> 6, (slots.back() >> 6) + 1);  // slots ascend
    for (uint64_t r0 = 0; r0 < rows.size(); r0 += UPSERT_BATCH) {
        const uint64_t r1 = std::min<uint64_t>(rows.size(), r0 + UPSERT_BATCH);
        rc = store_rows(c, g.slot, vectors, rows, slots, r0, r1);
        if (rc) return rc;
    }
    mark_valid_host(c, slots);
    return WVG_OK;
}

int wvg_corpus_upsert_codes(wvg_corpus *c, const uint64_t *ids, const void *codes, uint64_t n)
{
    int rc = check_corpus(c);
    if (rc) return rc;
    if (n == 0) return WVG_OK;
    if (!ids || !codes) return fail(WVG_ERR_INVALID, "null ids/codes");
    if (c->kind == WVG_KIND_PQ && !c->d_centers) return fail(WVG_ERR_INVALID, "PQ corpus has no codebook");
    std::unique_lock<std::shared_mutex> lk(c->rw);
    std::vector<uint64_t> rows, slots;
    rc = map_slots(c, ids, n, rows, slots);
    if (rc) return rc;
    SlotGuard g(c->ctx);
    rc = c->ctx->acquire(&g.slot);
    if (rc) return rc;
    const size_t rb = host_row_bytes(c);
    const uint64_t nr = rows.size();
    if (c->kind == WVG_KIND_PQ && c->pq_ks < 256) {  // a code indexes the m x ks LUT
        const unsigned char *cb = (const unsigned char *)codes;
        for (uint64_t i = 0; i < n * rb; i++)
            if (cb[i] >= c->pq_ks)
                return fail(WVG_ERR_INVALID, "PQ code " + std::to_string(cb[i]) + " of row " +
                                                 std::to_string(i / rb) + " is not below centroids (" +
                                                 std::to_string(c->pq_ks) + ")");
    }
    Carver cv;
    const size_t o_codes = cv.take(nr * rb), o_slots = cv.take(nr * 8);
    void *base = nullptr;
    rc = g.slot->device_scratch(cv.off, &base);
    if (rc) return rc;
    std::vector<unsigned char> hc(nr * rb);
    for (uint64_t i = 0; i < nr; i++) std::memcpy(hc.data() + i * rb, (const char *)codes + rows[i] * rb, rb);
    hipStream_t s = g.slot->stream;
    char *b = (char *)base;
    WVG_HIP(hipMemcpyAsync(b + o_codes, hc.data(), nr * rb, hipMemcpyHostToDevice, s));
    WVG_HIP(hipMemcpyAsync(b + o_slots, slots.data(), nr * 8, hipMemcpyHostToDevice, s));
    if (c->kind == WVG_KIND_F32)  // stored rows: already normalized at Add, kept bit for bit
        WVG_HIP(launch_f32_store((const float *)(b + o_codes), (uint64_t *)(b + o_slots), nr, c->dim, c->nchunks, 0,
                                 (float *)c->d_data, s));
    else if (c->kind == WVG_KIND_BQ)
        WVG_HIP(launch_bq_store((uint64_t *)(b + o_codes), (uint64_t *)(b + o_slots), nr, bq_words(c->dim), c->nchunks,
                                (uint64_t *)c->d_data, s));
    else
        WVG_HIP(launch_pq_store((uint8_t *)(b + o_codes), (uint64_t *)(b + o_slots), nr, c->pq_m, c->nchunks,
                                (uint8_t *)c->d_data, s));
    WVG_HIP(launch_set_valid(c->d_valid, (uint64_t *)(b + o_slots), nr, 1, s));
    WVG_HIP(hipStreamSynchronize(s));
    if (!slots.empty()) shadow_mark(c, slots.front() >> 6, (slots.back() >> 6) + 1);
    mark_valid_host(c, slots);
    return WVG_OK;
}

int wvg_corpus_delete(wvg_corpus *c, const uint64_t *ids, uint64_t n)
{
    int rc = check_corpus(c);
    if (rc) return rc;
    if (n == 0) return WVG_OK;
    if (!ids) return fail(WVG_ERR_INVALID, "null ids");
    std::unique_lock<std::shared_mutex> lk(c->rw);
    std::vector<uint64_t> slots;
    for (uint64_t i = 0; i < n; i++) {
        if (ids[i] < c->id_base || ids[i] - c->id_base >= c->capacity) continue;  // absent: no-op like an LSM delete
        const uint64_t s = ids[i] - c->id_base;
        uint64_t &w = c->h_valid[s >> 6];
        const uint64_t bit = 1ull << (s & 63);
        if (w & bit) {
            w &= ~bit;
            c->count--;
        }
        slots.push_back(s);
    }
    if (slots.empty()) return WVG_OK;
    SlotGuard g(c->ctx);
    rc = c->ctx->acquire(&g.slot);
    if (rc) return rc;
    void *base = nullptr;
    rc = g.slot->device_scratch(slots.size() * 8, &base);
    if (rc) return rc;
    WVG_HIP(hipMemcpyAsync(base, slots.data(), slots.size() * 8, hipMemcpyHostToDevice, g.slot->stream));
    WVG_HIP(launch_set_valid(c->d_valid, (uint64_t *)base, slots.size(), 0, g.slot->stream));
    WVG_HIP(hipStreamSynchronize(g.slot->stream));
    return WVG_OK;
}

int wvg_corpus_get(wvg_corpus *c, uint64_t id, void *out)
{
    int rc = check_corpus(c);
    if (rc) return rc;
    if (!out) return fail(WVG_ERR_INVALID, "null out");
    std::shared_lock<std::shared_mutex> lk(c->rw);
    if (id < c->id_base || id - c->id_base >= c->capacity) return fail(WVG_ERR_NOT_FOUND, "id not found");
    const uint64_t s = id - c->id_base;
    if (!((c->h_valid[s >> 6] >> (s & 63)) & 1ull)) return fail(WVG_ERR_NOT_FOUND, "id not found");
    const uint32_t nch = c->nchunks;
    std::vector<unsigned char> buf((size_t)nch * 16);
    const unsigned char *tile = (const unsigned char *)c->d_data + (s >> 6) * (size_t)nch * 64 * 16;
    WVG_HIP(hipMemcpy2D(buf.data(), 16, tile + (s & 63) * 16, 64 * 16, 16, nch, hipMemcpyDeviceToHost));
    size_t bytes = c->kind == WVG_KIND_F32 ? (size_t)c->dim * 4
                   : c->kind == WVG_KIND_BQ ? (size_t)bq_words(c->dim) * 8
                                            : (size_t)c->pq_m;
    if (c->kind == WVG_KIND_PQ && pq_rotated(c->pq_m)) {  // stored byte b = code[(b + slot) mod 32]
        unsigned char *o = (unsigned char *)out;
        for (uint32_t b = 0; b < 32; b++) o[(b + (uint32_t)(s & 31)) & 31u] = buf[b];
        return WVG_OK;
    }
    std::memcpy(out, buf.data(), bytes);
    return WVG_OK;
}

int wvg_corpus_get_batch(wvg_corpus *c, const uint64_t *ids, uint64_t n, void *out, uint8_t *out_ok)
{
    int rc = check_corpus(c);
    if (rc) return rc;
    if (n == 0) return WVG_OK;
    if (!ids || !out || !out_ok) return fail(WVG_ERR_INVALID, "null argument");
    std::shared_lock<std::shared_mutex> lk(c->rw);
    const size_t rb = host_row_bytes(c), cb = (size_t)c->nchunks * 16;
    std::vector<uint64_t> slots, where;  // live rows: slot, output index
    slots.reserve(n);
    where.reserve(n);
    for (uint64_t i = 0; i < n; i++) {
        const bool in = ids[i] >= c->id_base && ids[i] - c->id_base < c->capacity;
        const uint64_t s = in ? ids[i] - c->id_base : 0;
        const bool live = in && ((c->h_valid[s >> 6] >> (s & 63)) & 1ull);
        out_ok[i] = live ? 1 : 0;
        if (live) {
            slots.push_back(s);
            where.push_back(i);
        } else {
            std::memset((char *)out + i * rb, 0, rb);
        }
    }
    if (slots.empty()) return WVG_OK;
    SlotGuard g(c->ctx);
    rc = c->ctx->acquire(&g.slot);
    if (rc) return rc;
    const hipStream_t st = g.slot->stream;
    const uint64_t batch = std::max<uint64_t>(1, ((size_t)256 << 20) / (cb + 8));
    std::vector<unsigned char> buf;
    for (uint64_t r0 = 0; r0 < slots.size(); r0 += batch) {
        const uint64_t nr = std::min<uint64_t>(batch, slots.size() - r0);
        Carver cv;
        const size_t o_s = cv.take(nr * 8), o_o = cv.take(nr * cb);
        void *base = nullptr;
        rc = g.slot->device_scratch(cv.off, &base);
        if (rc) return rc;
        char *b = (char *)base;
        buf.resize(nr * cb);
        WVG_HIP(hipMemcpyAsync(b + o_s, slots.data() + r0, nr * 8, hipMemcpyHostToDevice, st));
        WVG_HIP(launch_gather_chunks(c->d_data, (const uint64_t *)(b + o_s), nr, c->nchunks, b + o_o, st));
        WVG_HIP(hipMemcpyAsync(buf.data(), b + o_o, nr * cb, hipMemcpyDeviceToHost, st));
        WVG_HIP(hipStreamSynchronize(st));
        for (uint64_t j = 0; j < nr; j++) {
            unsigned char *o = (unsigned char *)out + where[r0 + j] * rb;
            const unsigned char *src = buf.data() + j * cb;
            if (c->kind == WVG_KIND_PQ && pq_rotated(c->pq_m)) {  // stored byte b = code[(b + slot) mod 32]
                const uint32_t rot = (uint32_t)(slots[r0 + j] & 31);
                for (uint32_t q = 0; q < 32; q++) o[(q + rot) & 31u] = src[q];
            } else {
                std::memcpy(o, src, rb);
            }
        }
    }
    return WVG_OK;
}

int wvg_corpus_fill_synthetic(wvg_corpus *c, uint64_t seed, uint64_t n, int distribution)
{
    int rc = check_corpus(c);
    if (rc) return rc;
    if (c->kind == WVG_KIND_PQ) return fail(WVG_ERR_UNSUPPORTED, "synthetic fill supports F32 and BQ corpora");
    if (distribution < 0 || distribution > 1) return fail(WVG_ERR_INVALID, "distribution must be 0 or 1");
    std::unique_lock<std::shared_mutex> lk(c->rw);
    if (n > c->capacity) return fail(WVG_ERR_CAPACITY, "n exceeds corpus capacity");
    SlotGuard g(c->ctx);
    rc = c->ctx->acquire(&g.slot);
    if (rc) return rc;
    hipStream_t s = g.slot->stream;
    const int norm = c->metric == WVG_METRIC_COSINE;
    const uint64_t step = 1ull << 24;
    for (uint64_t r0 = 0; r0 < n; r0 += step) {
        const uint64_t nr = std::min(step, n - r0);
        if (c->kind == WVG_KIND_F32)
            WVG_HIP(launch_f32_synth(seed, distribution, c->id_base + r0, nr, r0, c->dim, c->nchunks, norm,
                                     (float *)c->d_data, s));
        else
            WVG_HIP(launch_bq_synth(seed, distribution, c->id_base + r0, nr, r0, c->dim, c->nchunks, norm,
                                    (uint64_t *)c->d_data, s));
    }
    // validity: full words for [0, n)
    std::vector<uint64_t> &hv = c->h_valid;
    for (uint64_t t = 0; t < tiles_of(n); t++) {
        const uint64_t lo = t * 64, hi = std::min(n, lo + 64);
        const uint64_t word = hi - lo == 64 ? ~0ull : ((1ull << (hi - lo)) - 1);
        c->count += (uint64_t)__builtin_popcountll(word & ~hv[t]);
        hv[t] |= word;
    }
    c->high_water = std::max(c->high_water, n);
    shadow_mark(c, 0, tiles_of(n));
    WVG_HIP(hipMemcpyAsync(c->d_valid, hv.data(), tiles_of(n) * 8, hipMemcpyHostToDevice, s));
    WVG_HIP(hipStreamSynchronize(s));
    return WVG_OK;
}

int wvg_pq_set_codebook(wvg_corpus *c, const float *centers, uint32_t m, uint32_t ks)
{
    int rc = check_corpus(c);
    if (rc) return rc;
    if (c->kind != WVG_KIND_PQ) return fail(WVG_ERR_INVALID, "not a PQ corpus");
    if (!centers) return fail(WVG_ERR_INVALID, "null centers");
    // NewProductQuantizer (CH/product_quantization.go:187-197)
    if (m == 0) return fail(WVG_ERR_INVALID, "segments cannot be 0 nor negative");
    if (ks > 256)
        return fail(WVG_ERR_INVALID,
                    "centroids should not be higher than 256. Attempting to use " + std::to_string(ks));
    if (ks == 0) return fail(WVG_ERR_INVALID, "centroids must be > 0");
    if (c->dim % m != 0) return fail(WVG_ERR_INVALID, "segments should be an integer divisor of dimensions");
    std::unique_lock<std::shared_mutex> lk(c->rw);
    // stored codes index the codebook: a non-empty corpus keeps its shape
    if (c->count > 0 && m != c->pq_m) return fail(WVG_ERR_INVALID, "cannot change segments of a non-empty PQ corpus");
    if (c->count > 0 && ks != c->pq_ks)
        return fail(WVG_ERR_INVALID, "cannot change centroids of a non-empty PQ corpus");
    const uint32_t ds = c->dim / m;
    float *dc = nullptr;
    WVG_HIP(hipMalloc(&dc, pq_centers_alloc_bytes(m, ks, ds)));
    {
        std::vector<float> pairs(pq_has_pairs(ks, ds) ? (size_t)m * ks * ds : 0);
        if (!pairs.empty()) pq_pair_layout(centers, m, ks, pairs.data());
        SlotGuard g(c->ctx);
        rc = c->ctx->acquire(&g.slot);
        hipError_t e = hipSuccess;
        if (!rc) {
            const hipStream_t s = g.slot->stream;
            e = hipMemcpyAsync(dc, centers, (size_t)m * ks * ds * 4, hipMemcpyHostToDevice, s);
            if (e == hipSuccess && !pairs.empty())
                e = hipMemcpyAsync(dc + (size_t)m * ks * ds, pairs.data(), pairs.size() * 4, hipMemcpyHostToDevice, s);
            const hipError_t e2 = hipStreamSynchronize(s);  // `pairs` is a host temporary
            if (e == hipSuccess) e = e2;
        }
        if (rc || e != hipSuccess) {
            (void)hipFree(dc);
            return rc ? rc : fail(WVG_ERR_DEVICE, std::string("codebook copy: ") + hipGetErrorString(e));
        }
    }
    if (c->d_centers) (void)hipFree(c->d_centers);
    c->d_centers = dc;
    const bool realloc = c->pq_m != m;
    c->pq_m = m;
    c->pq_ks = ks;
    c->pq_ds = ds;
    c->pq_nan_free = pq_nan_free(centers, (size_t)m * ks * ds);
    c->nchunks = pq_chunks(m);
    if (realloc) {
        const uint64_t cap = c->capacity;
        if (c->d_data) (void)hipFree(c->d_data);
        if (c->d_valid) (void)hipFree(c->d_valid);
        c->d_data = nullptr;
        c->d_valid = nullptr;
        c->capacity = 0;
        c->h_valid.clear();
        return corpus_alloc(c, cap);
    }
    return WVG_OK;
}

int wvg_pq_encode_corpus(wvg_corpus *pq, wvg_corpus *f32)
{
    int rc = check_corpus(pq);
    if (rc) return rc;
    if (!f32 || pq->kind != WVG_KIND_PQ || f32->kind != WVG_KIND_F32)
        return fail(WVG_ERR_INVALID, "need a PQ corpus and an F32 corpus");
    if (!pq->d_centers) return fail(WVG_ERR_INVALID, "PQ corpus has no codebook");
    if (pq->dim != f32->dim || pq->id_base != f32->id_base) return fail(WVG_ERR_INVALID, "dim / id_base mismatch");
    std::unique_lock<std::shared_mutex> lk1(pq->rw);
    std::shared_lock<std::shared_mutex> lk2(f32->rw);
    const uint64_t hw = f32->high_water;
    if (hw > pq->capacity) return fail(WVG_ERR_CAPACITY, "PQ corpus capacity below the float corpus");
    if (hw == 0) return WVG_OK;
    SlotGuard g(pq->ctx);
    rc = pq->ctx->acquire(&g.slot);
    if (rc) return rc;
    hipStream_t s = g.slot->stream;
    WVG_HIP(launch_pq_encode((const float *)f32->d_data, tiles_of(hw) * 64, pq->dim, pq->d_centers, pq->pq_m,
                             pq->pq_ks, (uint8_t *)pq->d_data, s, true, pq->pq_nan_free));
    const uint64_t tiles = tiles_of(hw);
    WVG_HIP(hipMemcpyAsync(pq->d_valid, f32->d_valid, tiles * 8, hipMemcpyDeviceToDevice, s));
    WVG_HIP(hipStreamSynchronize(s));
    pq->count = 0;
    for (uint64_t t = 0; t < tiles; t++) {
        pq->h_valid[t] = f32->h_valid[t];
        pq->count += (uint64_t)__builtin_popcountll(pq->h_valid[t]);
    }
    pq->high_water = std::max(pq->high_water, hw);
    return WVG_OK;
}

int wvg_corpus_load_kv(wvg_corpus *c, const uint8_t *keys, const uint8_t *values, uint64_t n, uint64_t value_bytes)
{
    int rc = check_corpus(c);
    if (rc) return rc;
    if (n == 0) return WVG_OK;
    if (!keys || !values) return fail(WVG_ERR_INVALID, "null keys/values");
    if (c->kind == WVG_KIND_PQ && !c->d_centers) return fail(WVG_ERR_INVALID, "PQ corpus has no codebook");
    if (value_bytes != host_row_bytes(c))
        return fail(WVG_ERR_DIM_MISMATCH, "vector lengths don't match: " + std::to_string(value_bytes) + " vs " +
                                              std::to_string(host_row_bytes(c)) + " bytes");
    // keys: 8-byte big-endian docIDs (binary.BigEndian.PutUint64, V/flat/index.go:218-224)
    std::vector<uint64_t> ids(n);
    uint64_t max_id = 0;
    for (uint64_t i = 0; i < n; i++) {
        uint64_t v = 0;
        for (int j = 0; j < 8; j++) v = (v << 8) | keys[i * 8 + j];
        ids[i] = v;
        max_id = std::max(max_id, v);
    }
    if (max_id < c->id_base) return fail(WVG_ERR_CAPACITY, "id below the corpus id_base");
    if (max_id - c->id_base >= c->capacity) {  // bqCache.Grow(maxID) (V/flat/index.go:671)
        rc = wvg_corpus_reserve(c, max_id - c->id_base + 1);
        if (rc) return rc;
    }
    // values: little-endian payloads (binary.LittleEndian, index.go:226-245) == the
    // host layout on little-endian machines, so they load as stored rows
    return wvg_corpus_upsert_codes(c, ids.data(), values, n);
}

}  // extern "C"
