// wvg_host.hpp -- host-runtime pieces shared by the C-ABI translation units
// (wvg_ctx / wvg_corpus / wvg_search / wvg_range / wvg_bulk / wvg_pqfit.hip):
// scratch carving, pooled-stream guards, pinned staging, the search plan and
// the corpus-state hooks (bf16 shadow) the search path calls.
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

#include "wvg_heap.hpp"
#include "wvg_internal.hpp"

namespace wvg {

inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

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
inline size_t stage_bytes(size_t bytes) { return bytes <= STAGE_MAX ? align_up(bytes, 64) : 0; }
// True for page-locked host memory (wvg_host_alloc / hipHostMalloc): a copy
// from it needs no staging.
inline bool host_pinned_ptr(const void *p)
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

// A small process-wide pool of host threads for bulk memory work on a call's
// critical path (the filtered batch's allow windows: ~2 MB of caller words per
// 16-query batch).  parallel_for(n, f) runs f(0) .. f(n - 1) on the pool and
// the calling thread and returns when all are done.
void parallel_for(uint32_t n, const std::function<void(uint32_t)> &f);

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

inline int check_corpus(wvg_corpus *c)
{
    if (!c || !c->ctx) return fail(WVG_ERR_INVALID, "null corpus");
    WVG_HIP(hipSetDevice(c->ctx->device));
    return WVG_OK;
}

constexpr uint32_t MAX_K = 256;  // the fused register top-k; above: select + sort in HBM

// NewProductQuantizer's argument checks (CH/product_quantization.go:187-197).
int pq_validate(uint32_t m, uint32_t ks, uint32_t dim);

// ---- profiling (wvg_ctx.hip) ------------------------------------------------
// Next free profiling event pair of the context (grown on demand).
int prof_pair(wvg_ctx *ctx, std::pair<hipEvent_t, hipEvent_t> *out);

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

// ---- corpus state (wvg_corpus.hip) -------------------------------------------
// Rows of tiles [t0, t1) were (re)written: the shadow rebuilds them at the
// next screened search.  Callers hold the corpus lock exclusively.
void shadow_mark(wvg_corpus *c, uint64_t t0, uint64_t t1);
void shadow_free(wvg_corpus *c);
// The bf16 shadow of an F32 dot / cosine corpus, ready for a screen on stream
// s (built or refreshed there, or waited for).  False: run the exact path.
bool ensure_shadow(wvg_corpus *c, hipStream_t s);

// ---- search planning (wvg_search.hip) ------------------------------------------
// Workspace of a K3c / K3d screen (wvg_screen.hip): range lists, candidates,
// rescored keys, per-query bounds, query fragments and constants, the
// flagged-query list, the rescan's partial lists and the pilot's results.
struct ScreenWs {
    size_t part = 0, cand = 0, keys = 0, gb = 0, qf = 0, k1 = 0, k2 = 0, em = 0, fl = 0, nf = 0, fbp = 0;
    size_t pids = 0, pd = 0, pc = 0, kb = 0, css = 0, qinv = 0, total = 0;
};
ScreenWs screen_ws(uint32_t nq, uint32_t k, uint32_t nrr, uint32_t kbn, uint32_t fb_groups);

struct SearchPlan {
    uint64_t tb = 0, te = 0;
    int groups = 1;      // scan: workgroups per query; gemm: row ranges (screen: K3c row ranges)
    bool gemm = false;   // K3 batched MFMA path
    bool screen = false; // gemm via the K3c bf16 screen + exact rescore
    int exact_groups = 1;   // screen: K3b's row ranges, if the shadow cannot be built
    uint32_t fb_groups = 0; // screen: K1 workgroups per flagged query's rescan
    uint32_t kbn = 0;       // screen: 32-element K blocks
    bool cosched = false; // PQ batch: co-scheduled K8e (ScanArgs::cosched)
    int mq = 0;           // F32 co-scheduled batch: queries per K1Q workgroup (0 = one, the COS K1)
    bool empty = false;
    const uint64_t *allow_host = nullptr;  // the caller's allow words of tiles [tb, te), or null
    uint64_t allow_qstride = 0;            // per-query allow windows (ScanArgs::allow_qstride)
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

bool allow_tile_range(const wvg_corpus *c, const uint64_t *allow, uint64_t allow_words, uint64_t &tb, uint64_t &te);
// mq_ok: K1Q may take the batch; gemm_ok: the MFMA kernels may (neither takes
// per-query allow windows, ScanArgs::allow_qstride)
SearchPlan plan_search(wvg_corpus *c, uint32_t nq, uint32_t k, const uint64_t *allow, uint64_t allow_words,
                       bool mq_ok = true, bool gemm_ok = true);
uint32_t next_direction(wvg_corpus *c, uint32_t nq);
int pq_dense(const wvg_corpus *c, const uint64_t *d_allow);
void prepare_queries_host(const wvg_corpus *c, const float *queries, uint32_t nq, std::vector<float> &qf,
                          std::vector<uint64_t> &qb, uint32_t &qpitch);
// A single host query merged in-launch straight into host memory (StreamJob::records).
struct SingleOut {
    uint4 *records = nullptr;  // [k + 1] in the slot's coherent host buffer, or null (ids / dists / counts)
    uint32_t tag = 0;
    bool legacy_poll = false;  // tools A/B: round 4's untagged layout in host memory
};
// sl: the calling host API's stream slot (a single query then merges in-launch), or null
// qhost: the prepared host query of a single in-launch search (d_q null), passed in the kernel arguments
int run_search(wvg_corpus *c, const void *d_q, uint32_t qpitch, uint32_t nq, uint32_t k, const uint64_t *d_allow,
               const SearchPlan &p, uint64_t *partials, uint64_t *ids, float *dists, uint32_t *counts, hipStream_t s,
               StreamSlot *sl = nullptr, const float *qhost = nullptr, const SingleOut *so = nullptr);
void write_empty(uint32_t nq, uint32_t k, uint64_t *ids, float *dists, uint32_t *counts);
int stage_queries(wvg_corpus *c, StreamSlot *sl, const float *queries, uint32_t nq, char *dst, uint32_t &qpitch,
                  float *d_lut_or_null, char *d_qtmp, Staging *st = nullptr);
size_t device_query_bytes(const wvg_corpus *c, uint32_t nq);
size_t query_bytes(const wvg_corpus *c, uint32_t nq);
size_t staged_query_bytes(const wvg_corpus *c, uint32_t nq);
ScanArgs scan_args_for(const wvg_corpus *c, const void *d_q, uint32_t qpitch, uint32_t nq, uint32_t k,
                       const uint64_t *d_allow, uint64_t tb, uint64_t te);

// ---- the reference heap's exact result (wvg_replay.hip) -------------------------
// Device workspace of bq_heap_candidates (per-wave emission buffers, the kept rows).
size_t replay_workspace_bytes(const wvg_corpus *bq, uint32_t nq, uint32_t R, const SearchPlan &p);
// findTopVectorsCached into a heap of R + the pop loop (V/flat/index.go:355-374)
// for nq prepared BQ queries: pops[q] = (slot, Hamming distance) in pop order.
int bq_heap_candidates(wvg_corpus *bq, StreamSlot *sl, const void *d_qb, uint32_t qpb, uint32_t nq, uint32_t R,
                       const uint64_t *d_allow, const SearchPlan &p, char *ws, std::vector<std::vector<GoItem>> &pops);
// The same for windows above MAX_K (wvg_range.hip): S1 keys, doubling chunks
// with prefix-select thresholds, compaction, sort, the host heap.
size_t select_replay_bytes(const SearchPlan &p);
int bq_heap_candidates_select(wvg_corpus *bq, StreamSlot *sl, const void *d_qb, uint32_t qpb, uint32_t nq,
                              uint32_t R, const uint64_t *d_allow, const SearchPlan &p, char *ws,
                              std::vector<std::vector<GoItem>> &pops);
// searchByVectorBQ exactly (any R): the candidates above, their exact
// distances on the device, the k-heap in pop order on the host.  f32 null:
// outputs are the candidates themselves ([nq][R], pop order).
int bq_rescore_replay(wvg_corpus *bq, wvg_corpus *f32, const float *queries, uint32_t nq, uint32_t k, uint32_t R,
                      const SearchPlan &p, uint64_t *out_ids, float *out_dists, uint32_t *out_counts);

// ---- unbounded selections (wvg_range.hip) ---------------------------------------
int search_large_k(wvg_corpus *c, const float *queries, uint32_t nq, uint32_t k, const uint64_t *allow_bits,
                   uint64_t allow_words, const SearchPlan &p, uint64_t *out_ids, float *out_dists, uint32_t *out_counts);
int bq_rescore_large(wvg_corpus *bq, wvg_corpus *f32, const float *queries, uint32_t nq, uint32_t k, uint32_t R,
                     const uint64_t *allow_bits, uint64_t allow_words, const SearchPlan &p, uint64_t *out_ids,
                     float *out_dists, uint32_t *out_counts);

}  // namespace wvg
