// wvg_multi.hip -- several GPUs in ONE process behind the C ABI.
//
// Weaviate serves a class from one Go process whose Index fans a search out
// over its shards and merges their results (Index.objectVectorSearch,
// adapters/repos/db/index.go:1567-1648: errgroup over shards, :1577; merge by
// distance, :1644-1648).  The single-process equivalent here: a multi handle
// owns one context per device and, when the devices are distinct, one RCCL
// communicator per device from ncclCommInitAll; a multi corpus deals docIDs
// to the devices in contiguous slabs (slab i = docIDs [i * slab, (i+1) *
// slab), a multiple of 64 rows); a search runs every slab's scan on its own
// device stream into a packed block (ids [nq][k] | dists [nq][k]), moves the
// blocks with ONE grouped ncclAllGather (xGMI), and merges them on device 0
// (wvg_topk_merge_packed's kernel) -- the only collective on the data path.
// Without distinct devices (a rehearsal on one GPU, devices = {0, 0}) or
// without RCCL the blocks travel by peer copies to device 0 instead; results
// are identical either way.  RCCL is opened with dlopen (librccl.so.1, the
// copy a host process such as torch already loaded, else the system one), so
// the library itself does not depend on it.
#include <dlfcn.h>

#include <rccl/rccl.h>  // types and prototypes only: the symbols come from dlopen

#include <memory>
#include <thread>

#include "wvg_host.hpp"

struct wvg_multi {
    std::vector<int> devices;
    std::vector<wvg_ctx *> ctx;
    std::vector<ncclComm_t> comms;  // empty: the peer-copy exchange
    std::mutex coll_mu;             // grouped collectives are issued one search at a time
    std::atomic<int> corpora{0};
};

struct wvg_multi_corpus {
    wvg_multi *m = nullptr;
    int kind = 0, metric = 0;
    uint32_t dim = 0;
    uint64_t slab = 0, rows = 0;
    std::vector<wvg_corpus *> shards;  // shard i holds docIDs [i * slab, (i + 1) * slab)
};

namespace wvg {
namespace {

struct Rccl {
    decltype(&ncclCommInitAll) init_all = nullptr;
    decltype(&ncclCommDestroy) destroy = nullptr;
    decltype(&ncclAllGather) all_gather = nullptr;
    decltype(&ncclGroupStart) group_start = nullptr;
    decltype(&ncclGroupEnd) group_end = nullptr;
    decltype(&ncclGetErrorString) error_string = nullptr;
    bool ok() const { return init_all && destroy && all_gather && group_start && group_end && error_string; }
};

const Rccl &rccl()
{
    static const Rccl r = [] {
        Rccl x;
        void *h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) return x;
        x.init_all = (decltype(x.init_all))dlsym(h, "ncclCommInitAll");
        x.destroy = (decltype(x.destroy))dlsym(h, "ncclCommDestroy");
        x.all_gather = (decltype(x.all_gather))dlsym(h, "ncclAllGather");
        x.group_start = (decltype(x.group_start))dlsym(h, "ncclGroupStart");
        x.group_end = (decltype(x.group_end))dlsym(h, "ncclGroupEnd");
        x.error_string = (decltype(x.error_string))dlsym(h, "ncclGetErrorString");
        return x;
    }();
    return r;
}

int nccl_fail(ncclResult_t r, const char *what)
{
    return fail(WVG_ERR_DEVICE, std::string(what) + ": " + rccl().error_string(r));
}

// Runs f(i) for every shard, one thread per shard when there is more than one
// (each thread sets its own current device); the first failure is returned.
template <typename F>
int for_shards(size_t n, F &&f)
{
    if (n == 1) return f(0);
    std::vector<int> rcs(n, WVG_OK);
    std::vector<std::string> errs(n);
    std::vector<std::thread> th;
    for (size_t i = 0; i < n; i++)
        th.emplace_back([&, i] {
            rcs[i] = f(i);
            if (rcs[i]) errs[i] = wvg_last_error();
        });
    for (auto &t : th) t.join();
    for (size_t i = 0; i < n; i++)
        if (rcs[i]) {
            set_error(errs[i]);
            return rcs[i];
        }
    return WVG_OK;
}

}  // namespace
}  // namespace wvg

using namespace wvg;

extern "C" {

int wvg_multi_open(const int *devices, int ndev, const wvg_options *opts, wvg_multi **out)
{
    if (!out) return fail(WVG_ERR_INVALID, "null out");
    *out = nullptr;
    if (!devices || ndev <= 0) return fail(WVG_ERR_INVALID, "need at least one device");
    int n = 0;
    WVG_HIP(hipGetDeviceCount(&n));
    for (int i = 0; i < ndev; i++)
        if (devices[i] < 0 || devices[i] >= n) return fail(WVG_ERR_INVALID, "device index out of range");
    wvg_multi *m = new wvg_multi();
    m->devices.assign(devices, devices + ndev);
    for (int i = 0; i < ndev; i++) {
        wvg_ctx *c = nullptr;
        const int rc = wvg_open_ex(devices[i], opts, &c);
        if (rc) {
            for (wvg_ctx *o : m->ctx) wvg_close(o);
            delete m;
            return rc;
        }
        m->ctx.push_back(c);
    }
    std::vector<int> sorted(m->devices);
    std::sort(sorted.begin(), sorted.end());
    const bool distinct = std::adjacent_find(sorted.begin(), sorted.end()) == sorted.end();
    if (distinct && rccl().ok()) {
        m->comms.resize(ndev);
        const ncclResult_t r = rccl().init_all(m->comms.data(), ndev, m->devices.data());
        if (r != ncclSuccess) {
            m->comms.clear();
            for (wvg_ctx *o : m->ctx) wvg_close(o);
            delete m;
            return nccl_fail(r, "ncclCommInitAll");
        }
    }
    *out = m;
    return WVG_OK;
}

int wvg_multi_close(wvg_multi *m)
{
    if (!m) return WVG_OK;
    if (m->corpora.load()) return fail(WVG_ERR_INVALID, "multi corpora still open");
    for (ncclComm_t c : m->comms) rccl().destroy(c);
    for (wvg_ctx *c : m->ctx) wvg_close(c);
    delete m;
    return WVG_OK;
}

int wvg_multi_info(wvg_multi *m, int *ndev, int *uses_rccl)
{
    if (!m) return fail(WVG_ERR_INVALID, "null multi");
    if (ndev) *ndev = (int)m->ctx.size();
    if (uses_rccl) *uses_rccl = m->comms.empty() ? 0 : 1;
    return WVG_OK;
}

int wvg_multi_ctx(wvg_multi *m, int i, wvg_ctx **out)
{
    if (!m || !out || i < 0 || i >= (int)m->ctx.size()) return fail(WVG_ERR_INVALID, "bad multi / index");
    *out = m->ctx[i];
    return WVG_OK;
}

int wvg_multi_corpus_create(wvg_multi *m, int kind, int metric, uint32_t dim, uint64_t rows, wvg_multi_corpus **out)
{
    if (!m || !out) return fail(WVG_ERR_INVALID, "null argument");
    *out = nullptr;
    const size_t nd = m->ctx.size();
    wvg_multi_corpus *mc = new wvg_multi_corpus();
    mc->m = m;
    mc->kind = kind;
    mc->metric = metric;
    mc->dim = dim;
    mc->rows = rows;
    mc->slab = std::max<uint64_t>(64, align_up((rows + nd - 1) / nd, 64));
    mc->shards.assign(nd, nullptr);
    const int rc = for_shards(nd, [&](size_t i) {
        return wvg_corpus_create(m->ctx[i], kind, metric, dim, i * mc->slab, mc->slab, &mc->shards[i]);
    });
    if (rc) {
        for (wvg_corpus *c : mc->shards)
            if (c) wvg_corpus_destroy(c);
        delete mc;
        return rc;
    }
    m->corpora++;
    *out = mc;
    return WVG_OK;
}

int wvg_multi_corpus_destroy(wvg_multi_corpus *mc)
{
    if (!mc) return WVG_OK;
    for (wvg_corpus *c : mc->shards)
        if (c) wvg_corpus_destroy(c);
    mc->m->corpora--;
    delete mc;
    return WVG_OK;
}

int wvg_multi_corpus_shard(wvg_multi_corpus *mc, int i, wvg_corpus **out, uint64_t *id_base, uint64_t *slab_rows)
{
    if (!mc || i < 0 || i >= (int)mc->shards.size()) return fail(WVG_ERR_INVALID, "bad multi corpus / index");
    if (out) *out = mc->shards[i];
    if (id_base) *id_base = (uint64_t)i * mc->slab;
    if (slab_rows) *slab_rows = mc->slab;
    return WVG_OK;
}

int wvg_multi_corpus_upsert(wvg_multi_corpus *mc, const uint64_t *ids, const float *vectors, uint64_t n, uint32_t dim)
{
    if (!mc || (n && (!ids || !vectors))) return fail(WVG_ERR_INVALID, "null argument");
    if (dim != mc->dim) return fail(WVG_ERR_DIM_MISMATCH, "insert called with a vector of the wrong size");
    const size_t nd = mc->shards.size();
    std::vector<std::vector<uint64_t>> sid(nd);
    for (uint64_t i = 0; i < n; i++) {
        const uint64_t s = ids[i] / mc->slab;
        if (s >= nd) return fail(WVG_ERR_CAPACITY, "id " + std::to_string(ids[i]) + " beyond the multi corpus");
        sid[s].push_back(i);
    }
    return for_shards(nd, [&](size_t s) {
        if (sid[s].empty()) return WVG_OK;
        std::vector<uint64_t> id(sid[s].size());
        std::vector<float> v(sid[s].size() * (size_t)dim);
        for (size_t j = 0; j < sid[s].size(); j++) {
            id[j] = ids[sid[s][j]];
            std::memcpy(v.data() + j * dim, vectors + sid[s][j] * dim, (size_t)dim * 4);
        }
        return wvg_corpus_upsert(mc->shards[s], id.data(), v.data(), id.size(), dim);
    });
}

int wvg_multi_corpus_delete(wvg_multi_corpus *mc, const uint64_t *ids, uint64_t n)
{
    if (!mc || (n && !ids)) return fail(WVG_ERR_INVALID, "null argument");
    const size_t nd = mc->shards.size();
    std::vector<std::vector<uint64_t>> sid(nd);
    for (uint64_t i = 0; i < n; i++) {
        const uint64_t s = ids[i] / mc->slab;
        if (s < nd) sid[s].push_back(ids[i]);  // ids beyond every slab are not present: nothing to delete
    }
    return for_shards(nd, [&](size_t s) {
        return sid[s].empty() ? WVG_OK : wvg_corpus_delete(mc->shards[s], sid[s].data(), sid[s].size());
    });
}

int wvg_multi_corpus_fill_synthetic(wvg_multi_corpus *mc, uint64_t seed, uint64_t n, int distribution)
{
    if (!mc) return fail(WVG_ERR_INVALID, "null multi corpus");
    return for_shards(mc->shards.size(), [&](size_t s) {
        const uint64_t b = s * mc->slab;
        const uint64_t cnt = n > b ? std::min(mc->slab, n - b) : 0;
        return cnt ? wvg_corpus_fill_synthetic(mc->shards[s], seed, cnt, distribution) : WVG_OK;
    });
}

int wvg_multi_corpus_set_codebook(wvg_multi_corpus *mc, const float *centers, uint32_t m, uint32_t ks)
{
    if (!mc) return fail(WVG_ERR_INVALID, "null multi corpus");
    return for_shards(mc->shards.size(), [&](size_t s) { return wvg_pq_set_codebook(mc->shards[s], centers, m, ks); });
}

int wvg_multi_search(wvg_multi_corpus *mc, const float *queries, uint32_t nq, uint32_t k, const uint64_t *allow_bits,
                     uint64_t allow_words, uint64_t *out_ids, float *out_dists, uint32_t *out_counts)
{
    if (!mc) return fail(WVG_ERR_INVALID, "null multi corpus");
    if (nq > 0 && !queries) return fail(WVG_ERR_INVALID, "null queries");
    if (k > MAX_K) return fail(WVG_ERR_UNSUPPORTED, "multi-GPU search: k above 256");
    if (nq == 0 || k == 0) return WVG_OK;
    wvg_multi *m = mc->m;
    const size_t nd = mc->shards.size();
    const size_t blk = wvg_topk_packed_bytes(nq, k);
    // per shard: a pooled stream slot of its context, its scratch carve and the scan's done-event
    struct Shard {
        SlotGuard g;
        char *b = nullptr;
        size_t o_q = 0, o_qtmp = 0, o_allow = 0, o_part = 0, o_send = 0, o_cnt = 0, o_recv = 0, o_ids = 0, o_d = 0,
               o_c = 0;
        hipEvent_t done = nullptr;
        explicit Shard(wvg_ctx *c) : g(c) {}
    };
    std::vector<std::unique_ptr<Shard>> sh;
    for (size_t i = 0; i < nd; i++) sh.emplace_back(new Shard(m->ctx[i]));
    std::vector<std::shared_lock<std::shared_mutex>> locks;
    for (wvg_corpus *c : mc->shards) locks.emplace_back(c->rw);
    auto cleanup = [&] {
        for (auto &x : sh) {
            if (!x->g.slot) continue;
            (void)hipSetDevice(x->g.ctx->device);
            (void)hipStreamSynchronize(x->g.slot->stream);
            if (x->done) (void)hipEventDestroy(x->done);
        }
    };
    // 1. every shard's scan into its packed block, on its own device stream
    int rc = for_shards(nd, [&](size_t i) -> int {
        Shard &x = *sh[i];
        wvg_corpus *c = mc->shards[i];
        WVG_HIP(hipSetDevice(c->ctx->device));
        int r = c->ctx->acquire(&x.g.slot);
        if (r) return r;
        SearchPlan p = plan_search(c, nq, k, allow_bits, allow_words, true, true);
        Carver cv;
        x.o_q = cv.take(query_bytes(c, nq));
        x.o_qtmp = cv.take(c->kind == WVG_KIND_PQ ? (size_t)nq * c->dim * 4 : 0);
        x.o_allow = cv.take(p.allow_bytes());
        x.o_part = cv.take(p.workspace_bytes(nq, k));
        x.o_send = cv.take(blk);
        x.o_cnt = cv.take((size_t)nq * 4);
        x.o_recv = cv.take(i == 0 ? blk * nd : (m->comms.empty() ? 0 : blk * nd));
        x.o_ids = cv.take(i == 0 ? (size_t)nq * k * 8 : 0);
        x.o_d = cv.take(i == 0 ? (size_t)nq * k * 4 : 0);
        x.o_c = cv.take(i == 0 ? (size_t)nq * 4 : 0);
        void *base = nullptr;
        r = x.g.slot->device_scratch(cv.off, &base);
        if (r) return r;
        x.b = (char *)base;
        hipStream_t s = x.g.slot->stream;
        WVG_HIP(hipEventCreateWithFlags(&x.done, hipEventDisableTiming));
        uint64_t *ids = (uint64_t *)(x.b + x.o_send);
        float *dists = (float *)(x.b + x.o_send + (size_t)nq * k * 8);
        uint32_t *cnt = (uint32_t *)(x.b + x.o_cnt);
        if (p.empty) {  // an empty slab (or nothing allowed in it): an all-empty block
            WVG_HIP(launch_fill_empty(ids, dists, cnt, nq, k, s));
        } else {
            uint32_t qpitch = 0;
            r = stage_queries(c, x.g.slot, queries, nq, x.b + x.o_q, qpitch, (float *)(x.b + x.o_q), x.b + x.o_qtmp);
            if (r) return r;
            const uint64_t *d_allow = nullptr;
            if (p.allow_host) {
                WVG_HIP(hipMemcpyAsync(x.b + x.o_allow, p.allow_host, p.allow_bytes(), hipMemcpyHostToDevice, s));
                d_allow = (const uint64_t *)(x.b + x.o_allow);
            }
            r = run_search(c, x.b + x.o_q, qpitch, nq, k, d_allow, p, (uint64_t *)(x.b + x.o_part), ids, dists, cnt,
                           s);
            if (r) return r;
        }
        WVG_HIP(hipEventRecord(x.done, s));
        return WVG_OK;
    });
    if (rc) {
        cleanup();
        return rc;
    }
    // 2. the exchange: one grouped all-gather over the communicators, or peer copies to device 0
    Shard &s0 = *sh[0];
    hipStream_t st0 = s0.g.slot->stream;
    if (!m->comms.empty()) {
        std::lock_guard<std::mutex> lk(m->coll_mu);
        ncclResult_t r = rccl().group_start();
        for (size_t i = 0; r == ncclSuccess && i < nd; i++)
            r = rccl().all_gather(sh[i]->b + sh[i]->o_send, sh[i]->b + sh[i]->o_recv, blk, ncclUint8, m->comms[i],
                                  sh[i]->g.slot->stream);
        const ncclResult_t r2 = rccl().group_end();
        if (r != ncclSuccess || r2 != ncclSuccess) {
            cleanup();
            return nccl_fail(r != ncclSuccess ? r : r2, "ncclAllGather");
        }
    } else {
        WVG_HIP(hipSetDevice(s0.g.ctx->device));
        for (size_t i = 0; i < nd; i++) {
            WVG_HIP(hipStreamWaitEvent(st0, sh[i]->done, 0));
            WVG_HIP(hipMemcpyPeerAsync(s0.b + s0.o_recv + i * blk, m->devices[0], sh[i]->b + sh[i]->o_send,
                                       m->devices[i], blk, st0));
        }
    }
    // 3. the merge on device 0 (index.go:1644-1648) and one copy of the results back
    WVG_HIP(hipSetDevice(s0.g.ctx->device));
    const size_t out_b = s0.o_c + (size_t)nq * 4 - s0.o_ids;
    Staging stg;
    rc = stg.reserve(s0.g.slot, stage_bytes(out_b));
    if (rc) {
        cleanup();
        return rc;
    }
    rc = wvg_topk_merge_packed(m->ctx[0], s0.b + s0.o_recv, nq, (uint32_t)nd, k, k, (uint64_t *)(s0.b + s0.o_ids),
                               (float *)(s0.b + s0.o_d), (uint32_t *)(s0.b + s0.o_c), st0);
    if (rc) {
        cleanup();
        return rc;
    }
    std::vector<char> big(out_b > STAGE_MAX ? out_b : 0);
    char *pin = out_b <= STAGE_MAX ? stg.take(out_b) : big.data();
    WVG_HIP(hipMemcpyAsync(pin, s0.b + s0.o_ids, out_b, hipMemcpyDeviceToHost, st0));
    cleanup();  // every shard's stream drained (the all-gather used them all)
    if (out_ids) std::memcpy(out_ids, pin, (size_t)nq * k * 8);
    if (out_dists) std::memcpy(out_dists, pin + (s0.o_d - s0.o_ids), (size_t)nq * k * 4);
    if (out_counts) std::memcpy(out_counts, pin + (s0.o_c - s0.o_ids), (size_t)nq * 4);
    return WVG_OK;
}

}  // extern "C"
