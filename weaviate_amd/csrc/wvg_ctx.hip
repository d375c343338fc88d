// wvg_ctx.hip -- context, stream pool, errors, profiling and the tools-build
// tuning knobs of the C ABI (include/wvgpu.h).  Errors are returned as
// negative codes with a thread-local message; no HIP failure aborts the
// process (no panics across cgo).

#include <condition_variable>
#include <thread>
#include <functional>
#include <atomic>
#include <mutex>
#include "wvg_host.hpp"

namespace wvg {

static thread_local std::string g_last_error;

void set_error(const std::string &msg) { g_last_error = msg; }

int fail(int code, const std::string &msg)
{
    g_last_error = msg;
    return code;
}

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

int StreamSlot::control(uint32_t **out)
{
    if (!dctl) {
        void *p = nullptr;
        const size_t bytes = 4 * (SLOT_READY_OFF + SLOT_READY_MAX);
        hipError_t e = hipMalloc(&p, bytes);
        if (e == hipSuccess) e = hipMemsetAsync(p, 0, bytes, stream);
        if (e == hipSuccess) e = hipStreamSynchronize(stream);
        if (e != hipSuccess) {
            if (p) (void)hipFree(p);
            return fail(WVG_ERR_NOMEM, std::string("slot control block: ") + hipGetErrorString(e));
        }
        dctl = (uint32_t *)p;
        arrival_base = 0;
    }
    *out = dctl;
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

int StreamSlot::host_coherent(size_t bytes, void **out)
{
    if (bytes > hcoh_bytes) {
        if (hcoh) (void)hipHostFree(hcoh);
        hcoh = nullptr;
        hcoh_bytes = 0;
        size_t want = std::max(bytes, (size_t)1 << 12);
        hipError_t e = hipHostMalloc(&hcoh, want, hipHostMallocCoherent);
        if (e != hipSuccess) return fail(WVG_ERR_NOMEM, std::string("hipHostMalloc (coherent): ") + hipGetErrorString(e));
        hcoh_bytes = want;
    }
    *out = hcoh;
    return WVG_OK;
}

// Next free profiling event pair of the context (grown on demand).
int prof_pair(wvg_ctx *ctx, std::pair<hipEvent_t, hipEvent_t> *out)
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

}  // namespace wvg

namespace wvg {
namespace {
// parallel_for's workers: a job is open from its post until the caller has run
// out of items and closed it; a worker joins only an open job (active + 1), so
// once the job is closed and active is 0, no worker can touch it again.
struct HostPool {
    std::mutex mu;
    std::condition_variable cv, done_cv;
    const std::function<void(uint32_t)> *job = nullptr;
    uint32_t n = 0, active = 0;
    std::atomic<uint32_t> next{0};
    uint64_t gen = 0;
    bool closed = true;
    explicit HostPool(int threads)
    {
        for (int t = 0; t < threads; t++) std::thread([this] { run(); }).detach();  // process lifetime
    }
    void run()
    {
        uint64_t seen = 0;
        std::unique_lock<std::mutex> lk(mu);
        for (;;) {
            cv.wait(lk, [&] { return gen != seen; });
            seen = gen;
            if (closed) continue;
            const std::function<void(uint32_t)> *f = job;
            const uint32_t total = n;
            active++;
            lk.unlock();
            for (uint32_t i; (i = next.fetch_add(1, std::memory_order_relaxed)) < total;) (*f)(i);
            lk.lock();
            if (--active == 0) done_cv.notify_all();
        }
    }
};
}  // namespace

void parallel_for(uint32_t n, const std::function<void(uint32_t)> &f)
{
    static HostPool *pool = new HostPool(7);  // (never destroyed: its threads are detached)
    static std::mutex call_mu;                // one job at a time
    std::lock_guard<std::mutex> one(call_mu);
    {
        std::lock_guard<std::mutex> lk(pool->mu);
        pool->job = &f;
        pool->n = n;
        pool->next.store(0, std::memory_order_relaxed);
        pool->closed = false;
        pool->gen++;
    }
    pool->cv.notify_all();
    for (uint32_t i; (i = pool->next.fetch_add(1, std::memory_order_relaxed)) < n;) f(i);
    std::unique_lock<std::mutex> lk(pool->mu);
    pool->closed = true;
    pool->done_cv.wait(lk, [&] { return pool->active == 0; });
}
}  // namespace wvg

using namespace wvg;

extern "C" {

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
    o->batch_screen = 2;
    o->coalesce = 1;
    o->heap_replay = 1;
}

int wvg_open(int device, wvg_ctx **out) { return wvg_open_ex(device, nullptr, out); }

#ifdef WVG_TOOLS
int wvgx_set_tuning(int key, int value);  // (tools A/B knobs, below)
#endif
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
    if (const char *e = getenv("WVG_SCREEN_VARIANT")) tuning().screen_variant = (int)strtol(e, nullptr, 10);  // A/B
    if (const char *e = getenv("WVG_STREAM_VARIANT")) tuning().stream_variant = (int)strtol(e, nullptr, 10);  // A/B
    if (const char *e = getenv("WVG_SCREEN_SP")) tuning().screen_pilot_screen = (int)strtol(e, nullptr, 10);  // A/B
    if (const char *e = getenv("WVG_GROUPS_PER_CU")) tuning().groups_per_cu = (int)strtol(e, nullptr, 10);  // A/B
    if (const char *e = getenv("WVG_TUNING")) {  // A/B: "key:value,key:value" -- any wvgx_set_tuning key
        for (const char *p = e; *p;) {
            char *end = nullptr;
            const long key = strtol(p, &end, 10);
            if (end == p || *end != ':') break;
            p = end + 1;
            const long val = strtol(p, &end, 10);
            if (end == p) break;
            (void)wvgx_set_tuning((int)key, (int)val);
            p = *end == ',' ? end + 1 : end;
        }
    }
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
        if (s->hcoh) (void)hipHostFree(s->hcoh);
        if (s->dctl) (void)hipFree(s->dctl);
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

int wvg_device_alloc(wvg_ctx *ctx, uint64_t bytes, int zero, void **out)
{
    if (!ctx || !out) return fail(WVG_ERR_INVALID, "null argument");
    *out = nullptr;
    if (bytes == 0) return WVG_OK;
    WVG_HIP(hipSetDevice(ctx->device));
    void *p = nullptr;
    hipError_t e = hipMalloc(&p, bytes);
    if (e != hipSuccess) return fail(WVG_ERR_NOMEM, std::string("hipMalloc: ") + hipGetErrorString(e));
    if (zero) {
        e = hipMemset(p, 0, bytes);  // synchronous: the memory is ready for any stream on return
        if (e != hipSuccess) {
            (void)hipFree(p);
            return fail(WVG_ERR_DEVICE, std::string("hipMemset: ") + hipGetErrorString(e));
        }
    }
    *out = p;
    return WVG_OK;
}

int wvg_device_free(wvg_ctx *ctx, void *p)
{
    if (!ctx) return fail(WVG_ERR_INVALID, "null context");
    if (!p) return WVG_OK;
    WVG_HIP(hipSetDevice(ctx->device));
    WVG_HIP(hipFree(p));
    return WVG_OK;
}

int wvg_stream_create(wvg_ctx *ctx, void **out)
{
    if (!ctx || !out) return fail(WVG_ERR_INVALID, "null argument");
    *out = nullptr;
    WVG_HIP(hipSetDevice(ctx->device));
    hipStream_t s = nullptr;
    WVG_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    *out = (void *)s;
    return WVG_OK;
}

int wvg_stream_destroy(wvg_ctx *ctx, void *stream)
{
    if (!ctx) return fail(WVG_ERR_INVALID, "null context");
    if (!stream) return WVG_OK;
    WVG_HIP(hipSetDevice(ctx->device));
    WVG_HIP(hipStreamDestroy((hipStream_t)stream));
    return WVG_OK;
}

int wvg_stream_synchronize(wvg_ctx *ctx, void *stream)
{
    if (!ctx) return fail(WVG_ERR_INVALID, "null context");
    WVG_HIP(hipSetDevice(ctx->device));
    WVG_HIP(hipStreamSynchronize((hipStream_t)stream));
    return WVG_OK;
}

int wvg_memcpy_h2d(wvg_ctx *ctx, void *d_dst, const void *src, uint64_t bytes, void *stream)
{
    if (!ctx || ((!d_dst || !src) && bytes)) return fail(WVG_ERR_INVALID, "null argument");
    if (!bytes) return WVG_OK;
    WVG_HIP(hipSetDevice(ctx->device));
    WVG_HIP(hipMemcpyAsync(d_dst, src, bytes, hipMemcpyHostToDevice, (hipStream_t)stream));
    WVG_HIP(hipStreamSynchronize((hipStream_t)stream));  // src may be Go memory: not retained past the call
    return WVG_OK;
}

int wvg_memcpy_d2h(wvg_ctx *ctx, void *dst, const void *d_src, uint64_t bytes, void *stream)
{
    if (!ctx || ((!dst || !d_src) && bytes)) return fail(WVG_ERR_INVALID, "null argument");
    if (!bytes) return WVG_OK;
    WVG_HIP(hipSetDevice(ctx->device));
    WVG_HIP(hipMemcpyAsync(dst, d_src, bytes, hipMemcpyDeviceToHost, (hipStream_t)stream));
    WVG_HIP(hipStreamSynchronize((hipStream_t)stream));
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

// tools build: single-query host path counters (wvg_search.hip, single_counters)
int wvgx_single_counters(uint64_t *out4, int reset)
{
    if (!out4) return WVG_ERR_INVALID;
    wvg::single_counters(out4, reset != 0);
    return WVG_OK;
}

int wvgx_coalesce_counters(uint64_t *out4, int reset)
{
    if (!out4) return WVG_ERR_INVALID;
    wvg::coalesce_counters(out4, reset != 0);
    return WVG_OK;
}

int wvgx_single_timing(uint64_t *out5, int reset)
{
    if (!out5) return WVG_ERR_INVALID;
    wvg::single_timing_read(out5, reset != 0);
    return WVG_OK;
}

int wvgx_filtered_timing(uint64_t *out5, int reset)
{
    if (!out5) return WVG_ERR_INVALID;
    wvg::filtered_timing_read(out5, reset != 0);
    return WVG_OK;
}

// A/B knob of the tools build (not part of include/wvgpu.h): 0 = K1 scan variant,
// 1 = K1 resident workgroups per CU, ... 7 = K8 ADC variant, 8 = query-stream merge wait (us),
// 9 = serpentine scan order, 10 = K3b row-range length, 11 = K1 load policy, 12 = K3b SIMD pairing,
// 13 = K3b partner priority, 14 = PQ encode min3 argmin, 15 = co-scheduled PQ / BQ batches, 16 = co-scheduled BQ workgroups per CU, 17 = K3c row-range length,
// 18 = K3c diagnostics (results not distances), 19 = K3c split launch,
// 20 = screen kernel (0 K3d where it applies, 1 K3c), 21 = screen pilot seed, 22 = exact seeds between
// screen phases, 23 = K3b pilot tiles, 24 = single-query host path, ..., 29 / 30 = K3i warm-up range
// blocks (first / second phase), 31 = filtered batches' windows from pinned staging, 32 = K3i's K3b pilot tiles,
// 33 = screen ranges in whole rounds of the CUs.  Returns the previous value.
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
    } else if (key == 22) {
        old = t.screen_seed;
        t.screen_seed = value;
    } else if (key == 23) {
        old = t.screen_pilot_gemm;
        t.screen_pilot_gemm = value;
    } else if (key == 24) {
        old = t.single_path;
        t.single_path = value;
    } else if (key == 25) {
        old = t.stream_variant;
        t.stream_variant = value;
    } else if (key == 26) {
        old = t.screen_pilot_screen;
        t.screen_pilot_screen = value;
    } else if (key == 27) {
        old = t.k1_mq;
        t.k1_mq = value;
    } else if (key == 28 && value > 0) {
        old = t.gather_div;
        t.gather_div = value;
    } else if (key == 29) {
        old = t.screen_warm;
        t.screen_warm = value;
    } else if (key == 30) {
        old = t.screen_warm2;
        t.screen_warm2 = value;
    } else if (key == 31) {
        old = t.filter_zc;
        t.filter_zc = value;
    } else if (key == 32) {
        old = t.screen_pilot_gemm_i8;
        t.screen_pilot_gemm_i8 = value;
    } else if (key == 33) {
        old = t.screen_round;
        t.screen_round = value;
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

}  // extern "C"
