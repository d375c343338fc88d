// wvg_capi.hip -- the C ABI (include/wvgpu.h): device context, stream pool,
// device-resident corpora and the search flows of the flat index.
//
// Host-side semantics mirrored from the reference:
//   flat.Add / AddBatch / Delete          V/flat/index.go:197-295
//   flat.SearchByVector / searchByVector  V/flat/index.go:307-334
//   flat.searchByVectorBQ (+ rescore)     V/flat/index.go:347-389
//   flat.normalized / distancer.Normalize V/flat/index.go:522-529, D/normalize.go:16-32
//   BinaryQuantizer.Encode                CH/binary_quantization.go:32-45
//   NewProductQuantizer validation        CH/product_quantization.go:187-197
// Errors are returned as negative codes with a thread-local message; no HIP
// failure aborts the process (no panics across cgo).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include "wvg_internal.hpp"

namespace wvg {

static thread_local std::string g_last_error;

void set_error(const std::string &msg) { g_last_error = msg; }

int fail(int code, const std::string &msg)
{
    g_last_error = msg;
    return code;
}

static size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

int StreamSlot::device_scratch(size_t bytes, void **out)
{
    if (bytes > dscratch_bytes) {
        if (dscratch) (void)hipFree(dscratch);
        dscratch = nullptr;
        dscratch_bytes = 0;
        size_t want = std::max(bytes, (size_t)1 << 20);
        hipError_t e = hipMalloc(&dscratch, want);
        if (e != hipSuccess) return fail(WVG_ERR_NOMEM, std::string("scratch hipMalloc: ") + hipGetErrorString(e));
        dscratch_bytes = want;
    }
    *out = dscratch;
    return WVG_OK;
}

int StreamSlot::host_pinned(size_t bytes, void **out)
{
    if (bytes > hpinned_bytes) {
        if (hpinned) (void)hipHostFree(hpinned);
        hpinned = nullptr;
        hpinned_bytes = 0;
        size_t want = std::max(bytes, (size_t)1 << 16);
        hipError_t e = hipHostMalloc(&hpinned, want, hipHostMallocDefault);
        if (e != hipSuccess) return fail(WVG_ERR_NOMEM, std::string("hipHostMalloc: ") + hipGetErrorString(e));
        hpinned_bytes = want;
    }
    *out = hpinned;
    return WVG_OK;
}

// Carves 256-byte aligned regions out of one scratch allocation.
struct Carver {
    size_t off = 0;
    size_t take(size_t bytes)
    {
        size_t o = off;
        off = align_up(off + bytes, 256);
        return o;
    }
};

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

// BinaryQuantizer.Encode (CH/binary_quantization.go:32-45).
static void bq_encode_host(const float *v, uint32_t d, uint64_t *code, uint32_t words)
{
    for (uint32_t i = 0; i < words; i++) code[i] = 0;
    for (uint32_t j = 0; j < d; j++)
        if (v[j] < 0.0f) code[j / 64] |= 1ull << (j % 64);
}

struct SlotGuard {
    wvg_ctx *ctx;
    StreamSlot *slot = nullptr;
    explicit SlotGuard(wvg_ctx *c) : ctx(c) {}
    ~SlotGuard()
    {
        if (slot) ctx->release(slot);
    }
};

// Host bytes of one call in the slot's pinned buffer.  A copy from pageable
// memory is a staged, blocking round trip (~16 us each for a few hundred
// bytes on MI355X: tools/latency_probe.py), so a call's small inputs and its
// results go through here.  The call reserves every piece up front (the
// buffer may only move before the first copy is queued) and the region is
// not reused before the call's closing stream sync.  Pieces above
// STAGE_MAX stay pageable (their fixed cost is noise; pinned memory is not).
constexpr size_t STAGE_MAX = (size_t)8 << 20;
static size_t stage_bytes(size_t bytes) { return bytes <= STAGE_MAX ? align_up(bytes, 64) : 0; }
// True for page-locked host memory (wvg_host_alloc / hipHostMalloc): a copy
// from it needs no staging.
static bool host_pinned_ptr(const void *p)
{
    hipPointerAttribute_t at{};
    if (hipPointerGetAttributes(&at, p) != hipSuccess) {
        (void)hipGetLastError();  // an unregistered pointer reports an error: clear it
        return false;
    }
    return at.type == hipMemoryTypeHost;
}

struct Staging {
    char *p = nullptr;
    size_t off = 0, cap = 0;
    int reserve(StreamSlot *sl, size_t bytes)
    {
        void *v = nullptr;
        const int rc = sl->host_pinned(std::max<size_t>(bytes, 64), &v);
        p = (char *)v;
        cap = bytes;
        off = 0;
        return rc;
    }
    char *take(size_t bytes)  // a reserved piece (stage_bytes(bytes) of it)
    {
        char *r = p + off;
        off += align_up(bytes, 64);
        return r;
    }
    hipError_t h2d(void *dst, const void *src, size_t bytes, hipStream_t s)
    {
        if (bytes > STAGE_MAX || host_pinned_ptr(src)) return hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, s);
        char *r = take(bytes);
        std::memcpy(r, src, bytes);
        return hipMemcpyAsync(dst, r, bytes, hipMemcpyHostToDevice, s);
    }
};

struct Bulk {
    SlotGuard g;
    char *b = nullptr;
    explicit Bulk(wvg_ctx *ctx) : g(ctx) {}
    int begin(size_t bytes)
    {
        int rc = g.ctx->acquire(&g.slot);
        if (rc) return rc;
        void *p = nullptr;
        rc = g.slot->device_scratch(bytes, &p);
        b = (char *)p;
        return rc;
    }
    hipStream_t s() const { return g.slot->stream; }
};

// Allow bitmap -> tile range [tb, te) of slots that can be allowed; false if
// empty.  Only the words of this corpus's own docID window are read (the
// bitmap is over global docIDs and word w covers docIDs 64w..64w+63, so the
// word of tile t is id_base/64 + t): O(corpus tiles) host work however large
// the docID space is; the scan then gets the words of [tb, te) only.
static bool allow_tile_range(const wvg_corpus *c, const uint64_t *allow, uint64_t allow_words, uint64_t &tb,
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

// Rows of tiles [t0, t1) were (re)written: the shadow rebuilds them at the
// next screened search.  Callers hold the corpus lock exclusively.
static void shadow_mark(wvg_corpus *c, uint64_t t0, uint64_t t1)
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

static void shadow_free(wvg_corpus *c)
{
    if (c->d_shadow) (void)hipFree(c->d_shadow);
    if (c->d_norms) (void)hipFree(c->d_norms);
    if (c->d_nmax) (void)hipFree(c->d_nmax);
    c->d_shadow = nullptr;
    c->d_norms = nullptr;
    c->d_nmax = nullptr;
    c->sh_dirty_lo = c->sh_dirty_hi = 0;
}

static int check_corpus(wvg_corpus *c)
{
    if (!c || !c->ctx) return fail(WVG_ERR_INVALID, "null corpus");
    WVG_HIP(hipSetDevice(c->ctx->device));
    return WVG_OK;
}

// Queries -> the device-side representation the scan of this corpus reads.
// F32: [nq][qpitch] floats (normalized for cosine).  BQ: [nq][qpitch] words.
// PQ: raw floats are staged at qf and turned into LUTs by the caller.
static void prepare_queries_host(const wvg_corpus *c, const float *queries, uint32_t nq, std::vector<float> &qf,
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
    for (uint32_t i = 0; i < nq; i++) {
        const float *q = queries + (size_t)i * d;
        float *dst = qf.data() + (size_t)i * qpitch;
        if (c->metric == WVG_METRIC_COSINE)
            normalize_host(q, d, dst);
        else
            std::memcpy(dst, q, sizeof(float) * d);
    }
}

static hipError_t launch_scan(const ScanArgs &a, int kind, uint64_t *partials, int groups, hipStream_t s)
{
    switch (kind) {
    case WVG_KIND_F32: return launch_scan_f32(a, partials, groups, s);
    case WVG_KIND_BQ: return launch_scan_bq(a, partials, groups, s);
    default: return launch_scan_pq(a, partials, groups, s);
    }
}

static const uint32_t MAX_K = 256;

}  // namespace wvg

using namespace wvg;

// ---------------------------------------------------------------------------
int wvg_ctx::acquire(StreamSlot **out)
{
    {
        std::lock_guard<std::mutex> g(pool_mu);
        if (!free_slots.empty()) {
            *out = free_slots.back();
            free_slots.pop_back();
            return WVG_OK;
        }
    }
    StreamSlot *s = new StreamSlot();
    hipError_t e = hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking);
    if (e != hipSuccess) {
        delete s;
        return fail(WVG_ERR_DEVICE, std::string("hipStreamCreate: ") + hipGetErrorString(e));
    }
    std::lock_guard<std::mutex> g(pool_mu);
    all_slots.push_back(s);
    *out = s;
    return WVG_OK;
}

void wvg_ctx::release(StreamSlot *s)
{
    std::lock_guard<std::mutex> g(pool_mu);
    free_slots.push_back(s);
}

extern "C" {

int wvg_abi_version(void) { return WVG_ABI_VERSION; }

const char *wvg_last_error(void) { return g_last_error.c_str(); }

int wvg_device_count(int *out)
{
    if (!out) return fail(WVG_ERR_INVALID, "null out");
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess) {
        *out = 0;
        return fail(WVG_ERR_DEVICE, std::string("hipGetDeviceCount: ") + hipGetErrorString(e));
    }
    *out = n;
    return WVG_OK;
}

void wvg_options_default(wvg_options *o)
{
    if (!o) return;
    *o = wvg_options{};
    o->size = (uint32_t)sizeof(wvg_options);
    o->mfma_min_queries = 32;
    o->cache_reuse = 1;
    o->merge_wait_us = 0;
    o->batch_screen = 1;
}

int wvg_open(int device, wvg_ctx **out) { return wvg_open_ex(device, nullptr, out); }

int wvg_open_ex(int device, const wvg_options *opts, wvg_ctx **out)
{
    if (!out) return fail(WVG_ERR_INVALID, "null out");
    *out = nullptr;
    wvg_options o;
    wvg_options_default(&o);
    if (opts) {
        if (opts->size != sizeof(wvg_options)) return fail(WVG_ERR_INVALID, "wvg_options.size mismatch");
        o = *opts;
    }
    int n = 0;
    WVG_HIP(hipGetDeviceCount(&n));
    if (device < 0 || device >= n) return fail(WVG_ERR_INVALID, "device index out of range");
    WVG_HIP(hipSetDevice(device));
    hipDeviceProp_t prop;
    WVG_HIP(hipGetDeviceProperties(&prop, device));
    wvg_ctx *c = new wvg_ctx();
    c->device = device;
    c->num_cus = prop.multiProcessorCount > 0 ? prop.multiProcessorCount : 256;
    c->opt = o;
#ifdef WVG_TOOLS
    if (const char *e = getenv("WVG_MFMA_MIN_QUERIES")) c->opt.mfma_min_queries = (uint32_t)strtoul(e, nullptr, 10);
    if (const char *e = getenv("WVG_SERPENTINE")) tuning().serpentine = (int)strtol(e, nullptr, 10);  // A/B runs
    if (const char *e = getenv("WVG_K1_TAIL")) tuning().k1_tail = (int)strtol(e, nullptr, 10);        // A/B runs
    if (const char *e = getenv("WVG_K1_LOADS")) tuning().k1_loads = (int)strtol(e, nullptr, 10);        // A/B runs
#endif
    *out = c;
    return WVG_OK;
}

int wvg_close(wvg_ctx *ctx)
{
    if (!ctx) return WVG_OK;
    (void)hipSetDevice(ctx->device);
    for (auto &e : ctx->prof_events) {
        (void)hipEventDestroy(e.first);
        (void)hipEventDestroy(e.second);
    }
    for (StreamSlot *s : ctx->all_slots) {
        (void)hipStreamSynchronize(s->stream);
        if (s->dscratch) (void)hipFree(s->dscratch);
        if (s->hpinned) (void)hipHostFree(s->hpinned);
        (void)hipStreamDestroy(s->stream);
        delete s;
    }
    delete ctx;
    return WVG_OK;
}

int wvg_set_distance_order(wvg_ctx *ctx, int order)
{
    if (!ctx) return fail(WVG_ERR_INVALID, "null ctx");
    if (order != WVG_ORDER_AVX256 && order != WVG_ORDER_AVX512) return fail(WVG_ERR_INVALID, "unknown distance order");
    ctx->order512 = order == WVG_ORDER_AVX512;
    return WVG_OK;
}

int wvg_synchronize(wvg_ctx *ctx)
{
    if (!ctx) return fail(WVG_ERR_INVALID, "null ctx");
    WVG_HIP(hipSetDevice(ctx->device));
    WVG_HIP(hipDeviceSynchronize());
    return WVG_OK;
}

int wvg_host_alloc(wvg_ctx *ctx, uint64_t bytes, void **out)
{
    if (!ctx || !out) return fail(WVG_ERR_INVALID, "null argument");
    *out = nullptr;
    if (bytes == 0) return WVG_OK;
    WVG_HIP(hipSetDevice(ctx->device));
    hipError_t e = hipHostMalloc(out, bytes, hipHostMallocDefault);
    if (e != hipSuccess) {
        *out = nullptr;
        return fail(WVG_ERR_NOMEM, std::string("hipHostMalloc: ") + hipGetErrorString(e));
    }
    return WVG_OK;
}

int wvg_host_free(wvg_ctx *ctx, void *p)
{
    if (!ctx) return fail(WVG_ERR_INVALID, "null context");
    if (!p) return WVG_OK;
    WVG_HIP(hipSetDevice(ctx->device));
    WVG_HIP(hipHostFree(p));
    return WVG_OK;
}

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
    shadow_free(c);  // sized by the capacity: rebuilt at the next screened search
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

// ---------------------------------------------------------------------------
// Search
// ---------------------------------------------------------------------------

// Next free profiling event pair of the context (grown on demand).
static int prof_pair(wvg_ctx *ctx, std::pair<hipEvent_t, hipEvent_t> *out)
{
    std::lock_guard<std::mutex> g(ctx->prof_mu);
    if (ctx->prof_used == ctx->prof_events.size()) {
        hipEvent_t a, b;
        WVG_HIP(hipEventCreate(&a));
        WVG_HIP(hipEventCreate(&b));
        ctx->prof_events.emplace_back(a, b);
    }
    *out = ctx->prof_events[ctx->prof_used++];
    return WVG_OK;
}

// Arms a profiling event pair for the next scan dispatch on this thread
// (launch_timed binds it to the dispatch); a pair the launch path did not
// consume is handed back on scope exit.
struct ProfArm {
    wvg_ctx *ctx = nullptr;
    int rc = WVG_OK;
    explicit ProfArm(wvg_ctx *c)
    {
        if (!c->profiling.load(std::memory_order_relaxed)) return;
        std::pair<hipEvent_t, hipEvent_t> ev;
        rc = prof_pair(c, &ev);
        if (rc) return;
        ctx = c;
        armed_events() = LaunchEvents{ev.first, ev.second};
    }
    ~ProfArm()
    {
        if (!ctx) return;
        if (armed_events().start) {
            armed_events() = LaunchEvents{};
            std::lock_guard<std::mutex> g(ctx->prof_mu);
            if (ctx->prof_used) ctx->prof_used--;
        }
    }
};

// Direction of the next scan of `c`: consecutive scans alternate (serpentine),
// so a scan starts on the rows the previous one read last -- the part of the
// corpus still in the 256 MiB Infinity Cache.  `nq` scans are reserved (the
// query-stream kernel alternates per query from the returned start).
static uint32_t next_direction(wvg_corpus *c, uint32_t nq)
{
    if (!c->ctx->opt.cache_reuse || !tuning().serpentine) return 0u;
    return (uint32_t)(c->scan_serial.fetch_add(nq, std::memory_order_relaxed) & 1u);
}

// PQ m = 32 scans without an allow list on a corpus with >= 3/4 of its slots
// live run K8c, which loads every tile instead of skipping dead ones.
static int pq_dense(const wvg_corpus *c, const uint64_t *d_allow)
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

// Workspace of a K3c screen (wvg_screen.hip): range lists, candidates,
// rescored keys, per-query bounds, query fragments and constants, the
// flagged-query list and the rescan's partial lists.
struct ScreenWs {
    size_t part = 0, cand = 0, keys = 0, gb = 0, qf = 0, k1 = 0, k2 = 0, em = 0, fl = 0, nf = 0, fbp = 0, total = 0;
};
static ScreenWs screen_ws(uint32_t nq, uint32_t k, uint32_t nrr, uint32_t kbn, uint32_t fb_groups)
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
    w.total = cv.off;
    return w;
}

struct SearchPlan {
    uint64_t tb = 0, te = 0;
    int groups = 1;      // scan: workgroups per query; gemm: row ranges (screen: K3c row ranges)
    bool gemm = false;   // K3 batched MFMA path
    bool screen = false; // gemm via the K3c bf16 screen + exact rescore
    int exact_groups = 1;   // screen: K3b's row ranges, if the shadow cannot be built
    uint32_t fb_groups = 0; // screen: K1 workgroups per flagged query's rescan
    uint32_t kbn = 0;       // screen: 32-element K blocks
    bool cosched = false; // PQ batch: co-scheduled K8e (ScanArgs::cosched)
    bool empty = false;
    const uint64_t *allow_host = nullptr;  // the caller's allow words of tiles [tb, te), or null
    size_t allow_bytes() const { return allow_host ? (size_t)(te - tb) * 8 : 0; }
    size_t partial_keys(uint32_t nq, uint32_t k) const { return (size_t)nq * groups * k; }
    // K3b's per-row-range progress counters, then its per-query distance
    // bounds, follow the partial lists (gemm only)
    static size_t gemm_bytes(uint32_t nq, uint32_t k, int groups, bool gemm)
    {
        return (size_t)nq * groups * k * 8 + (gemm ? (size_t)groups * ((nq + 15) / 16) * 4 + (size_t)nq * 4 + 256 : 0);
    }
    size_t workspace_bytes(uint32_t nq, uint32_t k) const
    {
        if (screen) return std::max(screen_ws(nq, k, (uint32_t)groups, kbn, fb_groups).total, gemm_bytes(nq, k, exact_groups, true));
        return gemm_bytes(nq, k, groups, gemm);
    }
};

static SearchPlan plan_search(wvg_corpus *c, uint32_t nq, uint32_t k, const uint64_t *allow, uint64_t allow_words)
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
    p.gemm = c->kind == WVG_KIND_F32 && mn > 0 && nq >= mn && gemm_supported(c->dim, c->metric) &&
             !c->ctx->order512;  // K3's 32 MFMA slices are the AVX2 order's chains
    if (p.gemm)
        p.groups = (int)gemm_row_ranges(nq, std::max<uint64_t>(1, p.te - p.tb), c->ctx->num_cus, c->dim, k);
    else
        p.groups = scan_groups_for(a, c->ctx->num_cus);
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
        p.groups = pq_cosched_groups(nq, std::max(scan_groups_for(a1, c->ctx->num_cus), 8));
    }
    return p;
}

// The bf16 shadow (fragments + row norms) of an F32 dot / cosine corpus,
// allocated on first use and rebuilt over the tiles written since the last
// build; ordered before the caller's screen on stream s.  False when it
// cannot be allocated (the batch then runs the exact path).
static bool ensure_shadow(wvg_corpus *c, hipStream_t s)
{
    std::lock_guard<std::mutex> g(c->sh_mu);
    if (c->sh_failed) return false;
    const uint64_t tiles = tiles_of(c->capacity);
    const uint32_t kbn = screen_kblocks(c->dim);
    if (!c->d_shadow) {
        const size_t sbytes = (size_t)(tiles + 4) * kbn * 4 * 1024, nbytes = (size_t)(tiles + 4) * 64 * 4;
        void *sh = nullptr, *nr = nullptr, *mx = nullptr;
        if (hipMalloc(&sh, sbytes) != hipSuccess || hipMalloc(&nr, nbytes) != hipSuccess ||
            hipMalloc(&mx, 256) != hipSuccess || hipMemsetAsync(sh, 0, sbytes, s) != hipSuccess ||
            hipMemsetAsync(nr, 0, nbytes, s) != hipSuccess || hipMemsetAsync(mx, 0, 256, s) != hipSuccess ||
            (!c->sh_ready && hipEventCreateWithFlags(&c->sh_ready, hipEventDisableTiming) != hipSuccess)) {
            (void)hipGetLastError();
            (void)hipStreamSynchronize(s);
            if (sh) (void)hipFree(sh);
            if (nr) (void)hipFree(nr);
            if (mx) (void)hipFree(mx);
            c->sh_failed = true;
            return false;
        }
        c->d_shadow = sh;
        c->d_norms = (float *)nr;
        c->d_nmax = (uint32_t *)mx;
        c->sh_dirty_lo = 0;
        c->sh_dirty_hi = tiles_of(c->high_water);
    }
    if (c->sh_dirty_lo < c->sh_dirty_hi) {
        if (launch_shadow_build((const float *)c->d_data, c->dim, c->sh_dirty_lo, c->sh_dirty_hi, c->d_shadow,
                                c->d_norms, c->d_nmax, s) != hipSuccess ||
            hipEventRecord(c->sh_ready, s) != hipSuccess)
            return false;
        c->sh_dirty_lo = c->sh_dirty_hi = 0;
        return true;
    }
    return hipStreamWaitEvent(s, c->sh_ready, 0) == hipSuccess;
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
    L.pilot = &a;                             // exact K1 over the first tiles (the fallback's partials and
    L.pilot_part = (uint64_t *)(ws + w.fbp);  // the result arrays are free until the rescan / final merge)
    L.pilot_groups = std::max<uint32_t>(1, std::min<uint32_t>(p.fb_groups, 4));
    L.pilot_ids = ids;
    L.pilot_dists = dists;
    L.pilot_counts = counts;
    WVG_HIP(launch_screen(L, s));
    uint64_t *keys = (uint64_t *)(ws + w.keys);
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
static int run_search(wvg_corpus *c, const void *d_q, uint32_t qpitch, uint32_t nq, uint32_t k, const uint64_t *d_allow,
                      const SearchPlan &p, uint64_t *partials, uint64_t *ids, float *dists, uint32_t *counts,
                      hipStream_t s)
{
    ScanArgs a{};
    a.data = c->d_data;
    a.valid = c->d_valid;
    a.allow = d_allow;
    a.allow_words = d_allow ? p.te - p.tb : 0;
    a.allow_t0 = p.tb;
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
    a.cosched = p.cosched;
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
        return run_search(c, d_q, qpitch, nq, k, d_allow, pe, partials, ids, dists, counts, s);
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


static void write_empty(uint32_t nq, uint32_t k, uint64_t *ids, float *dists, uint32_t *counts)
{
    for (uint64_t i = 0; i < (uint64_t)nq * k; i++) {
        if (ids) ids[i] = WVG_KEY_NONE;
        if (dists) dists[i] = INFINITY;
    }
    if (counts)
        for (uint32_t i = 0; i < nq; i++) counts[i] = 0;
}

static int stage_queries(wvg_corpus *c, StreamSlot *sl, const float *queries, uint32_t nq, char *dst, uint32_t &qpitch,
                         float *d_lut_or_null, char *d_qtmp, Staging *st = nullptr)
{
    std::vector<float> qf;
    std::vector<uint64_t> qb;
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
static size_t device_query_bytes(const wvg_corpus *c, uint32_t nq)
{
    switch (c->kind) {
    case WVG_KIND_PQ: return align_up((size_t)nq * c->pq_m * c->pq_ks * 4, 256);
    case WVG_KIND_BQ:
        return align_up((size_t)nq * bq_chunks(c->dim) * 16, 256) + align_up((size_t)nq * bq_words(c->dim) * 8, 256);
    default: return 0;
    }
}

static size_t query_bytes(const wvg_corpus *c, uint32_t nq)
{
    switch (c->kind) {
    case WVG_KIND_F32: return (size_t)nq * f32_chunks(c->dim) * 16;
    case WVG_KIND_BQ: return (size_t)nq * bq_chunks(c->dim) * 16;
    default: return (size_t)nq * c->pq_m * c->pq_ks * 4;
    }
}

// Upper bound of the host bytes stage_queries copies (a Staging reservation).
static size_t staged_query_bytes(const wvg_corpus *c, uint32_t nq)
{
    return std::max(query_bytes(c, nq), (size_t)nq * c->dim * 4);
}

}  // extern "C"
namespace wvg {
static int search_large_k(wvg_corpus *c, const float *queries, uint32_t nq, uint32_t k, const uint64_t *allow_bits,
                          uint64_t allow_words, const SearchPlan &p, uint64_t *out_ids, float *out_dists,
                          uint32_t *out_counts);
static int bq_rescore_large(wvg_corpus *bq, wvg_corpus *f32, const float *queries, uint32_t nq, uint32_t k,
                            uint32_t R, const uint64_t *allow_bits, uint64_t allow_words, const SearchPlan &p,
                            uint64_t *out_ids, float *out_dists, uint32_t *out_counts);
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
    rc = stage_queries(c, g.slot, queries, nq, b + o_q, qpitch, (float *)(b + o_q), b + o_qtmp, &st);
    if (rc) return rc;
    const uint64_t *d_allow = nullptr;
    if (p.allow_host) {
        WVG_HIP(st.h2d(b + o_allow, p.allow_host, p.allow_bytes(), s));
        d_allow = (const uint64_t *)(b + o_allow);
    }
    rc = run_search(c, b + o_q, qpitch, nq, k, d_allow, p, (uint64_t *)(b + o_part), (uint64_t *)(b + o_ids),
                    (float *)(b + o_d), (uint32_t *)(b + o_cnt), s);
    if (rc) return rc;
    const char *pin = out_b <= STAGE_MAX ? st.take(out_b) : nullptr;
    std::vector<char> big(pin ? 0 : out_b);
    if (!pin) pin = big.data();
    WVG_HIP(hipMemcpyAsync((void *)pin, b + o_ids, out_b, hipMemcpyDeviceToHost, s));
    WVG_HIP(hipStreamSynchronize(s));
    if (out_ids) std::memcpy(out_ids, pin, (size_t)nq * k * 8);
    if (out_dists) std::memcpy(out_dists, pin + (o_d - o_ids), (size_t)nq * k * 4);
    if (out_counts) std::memcpy(out_counts, pin + (o_cnt - o_ids), (size_t)nq * 4);
    return WVG_OK;
}

}  // extern "C"

// ---------------------------------------------------------------------------
// Unbounded selections (wvg_select.hip): top-k for k > 256 and the range
// search of SearchByVectorDistance.  One query at a time; every phase in HBM.
// ---------------------------------------------------------------------------
namespace wvg {

static ScanArgs scan_args_for(const wvg_corpus *c, const void *d_q, uint32_t qpitch, uint32_t nq, uint32_t k,
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
static int search_large_k(wvg_corpus *c, const float *queries, uint32_t nq, uint32_t k, const uint64_t *allow_bits,
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
static int bq_rescore_large(wvg_corpus *bq, wvg_corpus *f32, const float *queries, uint32_t nq, uint32_t k,
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

// Device-search workspaces start with a 256-byte status block (the sticky
// status word read by wvg_search_device_check); the scan workspace follows.
static const size_t WS_STATUS_BYTES = 256;

// Workspace of the query-stream scan (after the status block): partial lists
// [nq][groups][k], then the per-query arrival counters.
struct StreamLayout {
    size_t partials = 0, arrivals = 0, total = 0;
};
static StreamLayout stream_layout(const SearchPlan &p1, uint32_t nq, uint32_t k)
{
    StreamLayout l;
    l.partials = WS_STATUS_BYTES;
    l.arrivals = l.partials + align_up((size_t)nq * p1.groups * k * 8, 256);
    l.total = l.arrivals + align_up((size_t)nq * 4, 256);  // memset block: 16-B multiple
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
        WVG_HIP(hipMemsetAsync(j.arrivals, 0, align_up((size_t)nq * 4, 16), s));
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
    const bool large = k > MAX_K;  // beyond the fused top-k: sort the n keys
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

#ifdef WVG_TOOLS
// tools build: K3c counters [row-block epilogues (per wave), slow-path entries, insert calls, 0]
int wvgx_screen_counters(uint64_t *out4, int reset)
{
    if (!out4) return WVG_ERR_INVALID;
    wvg::screen_counters(out4, reset != 0);
    return WVG_OK;
}

// A/B knob of the tools build (not part of include/wvgpu.h): 0 = K1 scan variant,
// 1 = K1 resident workgroups per CU, ... 7 = K8 ADC variant, 8 = query-stream merge wait (us),
// 9 = serpentine scan order, 10 = K3b row-range length, 11 = K1 load policy, 12 = K3b SIMD pairing,
// 13 = K3b partner priority, 14 = PQ encode min3 argmin, 15 = co-scheduled PQ / BQ batches, 16 = co-scheduled BQ workgroups per CU, 17 = K3c row-range length,
// 18 = K3c diagnostics (results not distances), 19 = K3c split launch,
// 20 = screen kernel (0 K3d where it applies, 1 K3c), 21 = screen pilot seed.  Returns the previous value.
int wvgx_set_tuning(int key, int value)
{
    Tuning &t = tuning();
    int old = -1;
    if (key == 0) {
        old = t.scan_variant;
        t.scan_variant = value;
    } else if (key == 1) {
        old = t.groups_per_cu;
        t.groups_per_cu = value;
    } else if (key == 2) {
        old = t.pipeline_mode;
        t.pipeline_mode = value;
    } else if (key == 3) {
        old = t.gemm_pf;
        t.gemm_pf = value;
    } else if (key == 4) {
        old = t.gemm_kernel;
        t.gemm_kernel = value;
    } else if (key == 5) {
        old = t.gemm_skew;
        t.gemm_skew = value;
    } else if (key == 6) {
        old = t.gemm_lockstep;
        t.gemm_lockstep = value;
    } else if (key == 7) {
        old = t.pq_variant;
        t.pq_variant = value;
    } else if (key == 8) {
        old = t.merge_wait_us;
        t.merge_wait_us = value;
    } else if (key == 9) {
        old = t.serpentine;
        t.serpentine = value;
    } else if (key == 10) {
        old = t.gemm_range_tiles;
        t.gemm_range_tiles = value;
    } else if (key == 11) {
        old = t.k1_loads;
        t.k1_loads = value;
    } else if (key == 12) {
        old = t.gemm_pairing;
        t.gemm_pairing = value;
    } else if (key == 13) {
        old = t.gemm_prio;
        t.gemm_prio = value;
    } else if (key == 14) {
        old = t.pq_encode_min3;
        t.pq_encode_min3 = value;
    } else if (key == 15) {
        old = t.pq_cosched;
        t.pq_cosched = value;
    } else if (key == 16) {
        old = t.bq_cos_gpc;
        t.bq_cos_gpc = value;
    } else if (key == 17) {
        old = t.screen_range_blocks;
        t.screen_range_blocks = value;
    } else if (key == 18) {
        old = t.screen_diag;
        t.screen_diag = value;
    } else if (key == 19) {
        old = t.screen_split;
        t.screen_split = value;
    } else if (key == 20) {
        old = t.screen_variant;
        t.screen_variant = value;
    } else if (key == 21) {
        old = t.screen_pilot;
        t.screen_pilot = value;
    }
    return old;
}
#endif

int wvg_measure_hbm_read(wvg_ctx *ctx, uint64_t bytes, uint32_t reps, double *out_gbps)
{
    if (!ctx || !out_gbps) return fail(WVG_ERR_INVALID, "null argument");
    *out_gbps = 0.0;
    bytes = bytes / 4096 * 4096;
    if (bytes == 0 || reps == 0) return fail(WVG_ERR_INVALID, "bytes and reps must be > 0");
    WVG_HIP(hipSetDevice(ctx->device));
    void *buf = nullptr;
    if (hipMalloc(&buf, bytes + 256) != hipSuccess) return fail(WVG_ERR_NOMEM, "probe buffer hipMalloc");
    SlotGuard g(ctx);
    hipEvent_t a = nullptr, b = nullptr;
    auto done = [&](int rc) {
        if (g.slot) (void)hipStreamSynchronize(g.slot->stream);
        if (a) (void)hipEventDestroy(a);
        if (b) (void)hipEventDestroy(b);
        (void)hipFree(buf);
        return rc;
    };
    int rc = ctx->acquire(&g.slot);
    if (rc) return done(rc);
    const hipStream_t s = g.slot->stream;
    float *sink = (float *)((char *)buf + bytes);
    if (hipMemsetAsync(buf, 0, bytes + 256, s) != hipSuccess || hipEventCreate(&a) != hipSuccess ||
        hipEventCreate(&b) != hipSuccess)
        return done(fail(WVG_ERR_DEVICE, "probe setup"));
    double best = 0.0;
    // grid-stride forms, then the scans' contiguous-chunk form (negative = chunk workgroups)
    for (int blocks : {1024, 2048, 4096, 8192, -256, -512, -1024, -2048}) {
        for (int w = 0; w < 2; w++)
            if (launch_hbm_read(buf, bytes, blocks, sink, s) != hipSuccess) return done(fail(WVG_ERR_DEVICE, "probe"));
        (void)hipEventRecord(a, s);
        for (uint32_t r = 0; r < reps; r++)
            if (launch_hbm_read(buf, bytes, blocks, sink, s) != hipSuccess) return done(fail(WVG_ERR_DEVICE, "probe"));
        (void)hipEventRecord(b, s);
        float ms = 0.f;
        if (hipEventSynchronize(b) != hipSuccess || hipEventElapsedTime(&ms, a, b) != hipSuccess || ms <= 0.f)
            return done(fail(WVG_ERR_DEVICE, "probe timing"));
        best = std::max(best, (double)bytes * reps / (ms * 1e-3) / 1e9);
    }
    *out_gbps = best;
    return done(WVG_OK);
}

int wvg_profile_start(wvg_ctx *ctx)
{
    if (!ctx) return fail(WVG_ERR_INVALID, "null ctx");
    std::lock_guard<std::mutex> g(ctx->prof_mu);
    ctx->prof_used = 0;
    ctx->profiling.store(true);
    return WVG_OK;
}

int wvg_profile_stop(wvg_ctx *ctx, double *scan_ms_total, uint64_t *scan_launches)
{
    if (!ctx) return fail(WVG_ERR_INVALID, "null ctx");
    WVG_HIP(hipSetDevice(ctx->device));
    ctx->profiling.store(false);
    std::lock_guard<std::mutex> g(ctx->prof_mu);
    double total = 0.0;
    for (size_t i = 0; i < ctx->prof_used; i++) {
        WVG_HIP(hipEventSynchronize(ctx->prof_events[i].second));
        float ms = 0.0f;
        WVG_HIP(hipEventElapsedTime(&ms, ctx->prof_events[i].first, ctx->prof_events[i].second));
        total += ms;
    }
    if (scan_ms_total) *scan_ms_total = total;
    if (scan_launches) *scan_launches = ctx->prof_used;
    ctx->prof_used = 0;
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

static int pq_validate(uint32_t m, uint32_t ks, uint32_t dim)
{
    if (m == 0) return fail(WVG_ERR_INVALID, "segments cannot be 0 nor negative");
    if (ks > 256)
        return fail(WVG_ERR_INVALID,
                    "centroids should not be higher than 256. Attempting to use " + std::to_string(ks));
    if (ks == 0) return fail(WVG_ERR_INVALID, "centroids must be > 0");
    if (dim % m != 0) return fail(WVG_ERR_INVALID, "segments should be an integer divisor of dimensions");
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

// Draw j of segment s's random stream: stands in for Go's global math/rand
// (rand.Intn(len(data)) at CH/kmeans.go:153,182), which is unseeded and shared
// by the concurrently fitted segments, so no run of the reference is
// reproducible.  oracle/wv_oracle.c orc_kmeans_draw is the same function.
static uint64_t kmeans_draw(uint64_t seed, uint32_t s, uint64_t &ctr, uint64_t n)
{
    const uint64_t h = wvg_mix64(wvg_mix64(seed + 0x632BE59BD9B4E019ull * (uint64_t)(s + 1)) + ctr++);
    return h % n;
}

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
                 o_bh = cv.take((size_t)m * kmeans_blocks(n) * ks * 4);
    Bulk bk(ctx);
    rc = bk.begin(cv.off);
    if (rc) return rc;
    hipStream_t s = bk.s();
    float *dX = (float *)(bk.b + o_x), *dXt = (float *)(bk.b + o_xt), *dC = (float *)(bk.b + o_c);
    uint8_t *dP = (uint8_t *)(bk.b + o_p), *dCode = (uint8_t *)(bk.b + o_code);
    uint32_t *dMem = (uint32_t *)(bk.b + o_mem), *dOff = (uint32_t *)(bk.b + o_off);
    uint32_t *dCnt = (uint32_t *)(bk.b + o_cnt), *dChg = (uint32_t *)(bk.b + o_chg);
    uint8_t *dAct = (uint8_t *)(bk.b + o_act), *dRec = (uint8_t *)(bk.b + o_rec), *dSkip = (uint8_t *)(bk.b + o_skip);
    uint32_t *dBh = (uint32_t *)(bk.b + o_bh);
    WVG_HIP(hipMemcpyAsync(dX, X, n * dim * 4, hipMemcpyHostToDevice, s));
    // the training rows in the tiled layout K9 (the assignment) reads
    WVG_HIP(hipMemsetAsync(dXt, 0, tiles_of(n) * 64 * (size_t)nch * 16, s));
    WVG_HIP(launch_f32_store(dX, nullptr, n, dim, nch, 0, dXt, s));
    const bool pairs = pq_has_pairs(ks, ds);
    auto refresh_pairs = [&]() -> hipError_t {  // K9's ds = 4 pair copy of the current centers
        return pairs ? launch_pq_pairs(dC, m, ks, dC + nc, s) : hipSuccess;
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
        WVG_HIP(launch_pq_encode(dXt, n, dim, dC, m, ks, dCode, s, false, false));
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
