// wvg_scan.hip -- K1 fp32 flat scan fused with wave-level top-k (phase 1),
// K2 top-k merge (phase 2), and the tiled-layout helpers for F32 corpora.
//
// Reference path replaced: flat.searchByVector -> findTopVectors
// (V/flat/index.go:319-334, 411-452): for every live (and allowed) docID in
// ascending order, SingleDist(query, row) and insertToHeap(k).
//
// Phase 1: each wave owns a contiguous range of 64-row tiles.  Lane = row.
// One global_load_dwordx4 per chunk reads 1 KiB of the tile; the lane folds
// its row in the AVX2 order (wvg_rowdist.hpp) and offers (dist, slot) to the
// wave's register top-k.  The workgroup merges its waves' lists in LDS and
// writes K keys per (query, workgroup).  Phase 2 merges those lists.
// Roofline: HBM, N*d*4 bytes per query.
#include <type_traits>

#include "wvg_internal.hpp"
#include "wvg_rowdist.hpp"
#include "wvg_topk.hpp"

namespace wvg {

#ifdef WVG_TOOLS
Tuning &tuning()
{
    static Tuning t;
    return t;
}
#else
const Tuning &tuning()
{
    static const Tuning t;
    return t;
}
#endif

LaunchEvents &armed_events()
{
    static thread_local LaunchEvents e;
    return e;
}

// Wave index as a wave-uniform (SGPR) value, so per-wave loops, the tile mask
// loads and the skip branch are scalar.
__device__ __forceinline__ int wave_id() { return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); }

// Per-tile mask of live, allowed rows (one 64-bit word per tile = one bit per lane);
// qi: the query whose allow window applies (ScanArgs::allow_qstride).
__device__ __forceinline__ uint64_t tile_mask(const ScanArgs &a, uint64_t t, uint32_t qi = 0)
{
    uint64_t m = a.valid[t];
    if (a.allow) {
        uint64_t w = t - a.allow_t0;  // allow[0] is tile allow_t0's word
        m &= w < a.allow_words ? a.allow[(uint64_t)qi * a.allow_qstride + w] : 0ull;
    }
    return m;
}

__device__ __forceinline__ void wave_range(const ScanArgs &a, int waves_per_group, uint64_t &t0,
                                           uint64_t &t1)
{
    const uint64_t ntiles = a.tile_end - a.tile_begin;
    const uint64_t groups = gridDim.x - (a.side.active ? 1u : 0u);
    const uint64_t total = groups * waves_per_group;
    const uint64_t gw = (uint64_t)blockIdx.x * waves_per_group + wave_id();
    t0 = a.tile_begin + ntiles * gw / total;
    t1 = a.tile_begin + ntiles * (gw + 1) / total;
}

// Phase-2 merge body for one query (see merge_keys_kernel): WAVES waves read
// `nlists` ascending lists transposed, then tree-merge in LDS; wave 0 writes.
// rec (host-read results, see StreamJob::records): entry i goes to rec[i] as ONE
// 16-byte store {id lo, id hi, dist bits, tag}, then the header {count, tag}
// at rec[k] -- the host accepts only entries carrying its call's tag.
template <int E, int WAVES>
__device__ __forceinline__ void merge_finish(WaveTopK<E> &tk, uint32_t k, uint64_t id_base, uint64_t *ids,
                                             float *dists, uint32_t *count, uint4 *rec, uint32_t tag, bool sys_release);

template <int E, int WAVES>
__device__ __forceinline__ void merge_lists_body(const uint64_t *src, uint32_t nlists, uint32_t list_len, uint32_t k,
                                                 uint64_t id_base, uint64_t *ids, float *dists, uint32_t *count,
                                                 uint4 *rec = nullptr, uint32_t tag = 0, bool sys_release = false)
{
    const int lane = threadIdx.x & 63, wave = wave_id();
    WaveTopK<E> tk;
    tk.init((int)k);
    for (uint32_t g0 = (uint32_t)wave * 64; g0 < nlists; g0 += WAVES * 64) {
        const uint32_t list = g0 + lane;
        const uint64_t *lp = src + (size_t)list * list_len;
        // four entries per lane in flight at a time (independent loads): a one-query
        // merge sits on the launch's critical path, where one dependent load per entry
        // (~1 us each from L2) was most of its time
        bool done = false;
        for (uint32_t r0 = 0; r0 < list_len && !done; r0 += 4) {
            uint64_t c4[4];
#pragma unroll
            for (int i = 0; i < 4; i++)
                c4[i] = (r0 + i < list_len && list < nlists) ? lp[r0 + i] : WVG_KEY_NONE;
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const uint32_t r = r0 + (uint32_t)i;
                if (r >= list_len) break;
                if (list_len > 1 && r > 0 && __ballot(c4[i] < tk.tau) == 0ull) {  // sorted lists: done
                    done = true;
                    break;
                }
                tk.offer(c4[i]);
            }
        }
    }
    merge_finish<E, WAVES>(tk, k, id_base, ids, dists, count, rec, tag, sys_release);
}

// The merge's end: the WAVES waves' lists tree-merged in LDS, wave 0 writes
// ids / dists / count, or the tagged records (rec) for a host-read result.
template <int E, int WAVES>
__device__ __forceinline__ void merge_finish(WaveTopK<E> &tk, uint32_t k, uint64_t id_base, uint64_t *ids,
                                             float *dists, uint32_t *count, uint4 *rec, uint32_t tag, bool sys_release)
{
    __shared__ uint64_t msh[WAVES][64 * E];
    const int lane = threadIdx.x & 63, wave = wave_id();
#pragma unroll
    for (int e = 0; e < E; e++) msh[wave][e * 64 + lane] = tk.l[e];
    for (int step = 1; step < WAVES; step <<= 1) {
        __syncthreads();
        if ((wave & (2 * step - 1)) == 0) {
            uint64_t o[E];
#pragma unroll
            for (int e = 0; e < E; e++) o[e] = msh[wave + step][e * 64 + lane];
            merge_lists<E>(tk.l, o);
#pragma unroll
            for (int e = 0; e < E; e++) msh[wave][e * 64 + lane] = tk.l[e];
        }
    }
    if (wave != 0) return;
    uint32_t cnt = 0;
#pragma unroll
    for (int e = 0; e < E; e++) {
        const uint32_t i = e * 64 + lane;
        const uint64_t key = tk.l[e];
        const bool live = i < k && key != WVG_KEY_NONE;
        cnt += (uint32_t)__popcll(__ballot(live));
        if (i < k) {
            const uint64_t id = live ? id_base + (key & 0xFFFFFFFFull) : WVG_KEY_NONE;
            const float dv = live ? wvg_unord_f32((uint32_t)(key >> 32)) : __builtin_inff();
            if (rec)  // {slot, tag, dist, tag}: each 8-byte half carries the tag (the host adds id_base)
                rec[i] = make_uint4(live ? (uint32_t)key : 0xFFFFFFFFu, tag, __float_as_uint(dv), tag);
            else {
                ids[i] = id;
                dists[i] = dv;
            }
        }
    }
    if (rec) {
        if (lane == 0)
            __hip_atomic_store(reinterpret_cast<uint64_t *>(rec + k), ((uint64_t)tag << 32) | cnt, __ATOMIC_RELEASE,
                               __HIP_MEMORY_SCOPE_SYSTEM);
        return;
    }
    // sys_release (tools A/B of the round-4 polled layout): a system-scope release between
    // the ids / dists stores and the count the host polls
    if (sys_release) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    if (lane == 0 && count) *count = cnt;
}

__device__ __forceinline__ uint64_t lane_key(uint64_t m, float dist, uint64_t t, int lane)
{
    return ((m >> lane) & 1ull) ? wvg_make_key(dist, (uint32_t)(t * 64 + lane)) : WVG_KEY_NONE;
}

typedef __attribute__((address_space(1))) uint32_t gu32;
typedef __attribute__((address_space(1))) uint64_t gu64;

// The query-stream merge of one query as its lists ARRIVE (StreamJob::ready):
// scan workgroup g stores its list sc1, drains it, then sc1-stores `tag` into
// ready[g]; lane l of merge wave w owns list g = 64 w + l (+ 64 WAVES ...),
// polls its ready word (sc1 load) and, once it matches, reads the list with sc1
// loads (MI355X_MICROARCH.md correctness boundaries: the valid hand-off form
// without an acquire) and offers it to the wave's top-k -- lists that arrive
// early are merged while the scan's stragglers still run, so after the last
// arrival only its own list is left to read.  False after `limit` ticks of
// s_memrealtime without every list.
template <int E, int WAVES>
__device__ __forceinline__ bool merge_lists_ready(const uint64_t *src, const uint32_t *ready, uint32_t tag,
                                                  uint32_t nlists, uint32_t k, uint64_t limit, uint64_t id_base,
                                                  uint64_t *ids, float *dists, uint32_t *count, uint4 *rec,
                                                  uint32_t rtag)
{
    __shared__ int ok_sh;
    const int lane = threadIdx.x & 63, wave = wave_id();
    WaveTopK<E> tk;
    tk.init((int)k);
    const uint64_t start = __builtin_amdgcn_s_memrealtime();
    bool ok = true;
    for (uint32_t g0 = (uint32_t)wave * 64; g0 < nlists && ok; g0 += WAVES * 64) {
        const uint32_t list = g0 + lane;
        bool done = list >= nlists;
        const gu64 *lp = (const gu64 *)(src + (size_t)list * k);
        while (true) {
            const bool rdy = !done && __hip_atomic_load((const gu32 *)(ready + list), __ATOMIC_RELAXED,
                                                        __HIP_MEMORY_SCOPE_AGENT) == tag;
            if (__ballot(rdy)) {
                for (uint32_t r0 = 0; r0 < k; r0 += 4) {
                    uint64_t c4[4];
#pragma unroll
                    for (int i = 0; i < 4; i++)
                        c4[i] = rdy && r0 + i < k ? __hip_atomic_load(lp + r0 + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                                  : WVG_KEY_NONE;
                    bool stop = false;
#pragma unroll
                    for (int i = 0; i < 4; i++) {
                        const uint32_t r = r0 + (uint32_t)i;
                        if (r >= k) break;
                        if (r > 0 && __ballot(c4[i] < tk.tau) == 0ull) {  // sorted lists: the rest cannot enter
                            stop = true;
                            break;
                        }
                        tk.offer(c4[i]);
                    }
                    if (stop) break;
                }
                done = done || rdy;
            }
            if (__ballot(!done) == 0ull) break;
            if (__builtin_amdgcn_s_memrealtime() - start > limit) {
                ok = false;
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
    }
    if (threadIdx.x == 0) ok_sh = 1;
    __syncthreads();
    if (!ok && lane == 0) ok_sh = 0;
    __syncthreads();
    if (!ok_sh) return false;
    merge_finish<E, WAVES>(tk, k, id_base, ids, dists, count, rec, rtag, false);
    return true;
}

// One wave's tiles [t0, t1) for one query: one tile's loads in flight per
// wave; tiles with no live/allowed row are skipped without touching their rows.
// rev: walk the range downwards (t1-1 .. t0); the result does not depend on
// the order (lexicographic keys), only the cache state the next scan finds.
// first_mask / last_mask: lanes of tiles t0 / t1 - 1 this wave owns (a
// row-granular split of the range, see scan_f32_stream_kernel); on such a
// partial tile only the owned lanes load, so two waves sharing a tile fetch it
// once between them.
template <int METRIC, int D, int E>
__device__ __forceinline__ void scan_tiles(const ScanArgs &a, const float4 *q4, uint64_t t0, uint64_t t1,
                                           WaveTopK<E> &tk, bool rev = false, uint32_t qi = 0,
                                           uint64_t first_mask = ~0ull, uint64_t last_mask = ~0ull)
{
    const int lane = threadIdx.x & 63;
    const float4 *data = reinterpret_cast<const float4 *>(a.data);
    const uint64_t n = t1 - t0;
    // passes i >= split load with the default policy (cache_tail256: only the tail of the pass)
    const uint64_t split = a.cache_tail256 ? n - ((n * a.cache_tail256) >> 8) : (a.plain ? 0 : n);
    uint64_t m_next = n ? tile_mask(a, rev ? t1 - 1 : t0, qi) : 0ull;
    for (uint64_t i = 0; i < n; ++i) {
        const uint64_t t = rev ? t1 - 1 - i : t0 + i;
        uint64_t m = m_next;
        if (i + 1 < n) m_next = tile_mask(a, rev ? t - 1 : t + 1, qi);  // scalar prefetch of the next mask
        const uint64_t own = (t == t0 ? first_mask : ~0ull) & (t == t1 - 1 ? last_mask : ~0ull);
        m &= own;
        if (m == 0ull) continue;  // wave-uniform: nothing live/allowed in this tile
        const float4 *rp = data + (size_t)t * a.nchunks * 64 + lane;
        // ONE call site of the distance (a lambda called from two branches was not
        // inlined: its captures then forced the kernel arguments into scratch); on a
        // shared edge tile only this wave's lanes are active, so only they load
        float r = 0.0f;
        if ((own >> lane) & 1ull) {
            if (a.order512)  // wave-uniform: the AVX-512 kernels' order (generic length)
                r = row_dist_512<METRIC, 64>(rp, q4, (int)a.dim);
            else if constexpr (D > 0)
                r = i >= split ? row_dot_or_l2_fixed<METRIC, D, 64, false>(rp, q4)
                               : row_dot_or_l2_fixed<METRIC, D, 64>(rp, q4);
            else
                r = row_dot_or_l2_generic<METRIC, 64>(rp, q4, (int)a.dim);
        }
        tk.offer(lane_key(m, wrap_metric(a.metric, r), t, lane));
    }
}

// COS (a batch of 1 < nq < the MFMA threshold, ScanArgs::cosched): a 1D grid
// of G row ranges x nq queries where workgroup id -> (range, query) puts the
// nq queries of one range at consecutive ids on ONE XCD (equal id mod 8; K5 /
// K8e use the same map).  They run side by side and each wave walks the same
// rows as its partners, so all but the first read of a line hit that XCD's
// L2 (the host sets default-policy loads for this).  Results are those of
// single-query scans: the keys are lexicographic, the visiting order free.
template <int METRIC, int D, int E, bool COS = false>
__global__ __launch_bounds__(SCAN_WAVES * 64) void scan_f32_kernel(ScanArgs a, uint64_t *partials)
{
    if (a.side.active && blockIdx.x == gridDim.x - 1) {  // the previous query's merge (uniform branch)
        if (blockIdx.y == 0)
            merge_lists_body<E, SCAN_WAVES>(a.side.partials, a.side.nlists, a.side.list_len, a.side.k,
                                            a.side.id_base, a.side.ids, a.side.dists, a.side.counts);
        return;
    }
    uint32_t qi = blockIdx.y, rng = blockIdx.x, G = gridDim.x;
    uint64_t t0, t1;
    if constexpr (COS) {
        G = gridDim.x / a.nq;
        const uint32_t kk = blockIdx.x >> 3;
        rng = (kk / a.nq) * 8u + (blockIdx.x & 7u);
        qi = kk % a.nq;
        const uint64_t ntiles = a.tile_end - a.tile_begin, total = (uint64_t)G * SCAN_WAVES;
        const uint64_t gw = (uint64_t)rng * SCAN_WAVES + wave_id();
        t0 = a.tile_begin + ntiles * gw / total;
        t1 = a.tile_begin + ntiles * (gw + 1) / total;
    } else {
        wave_range(a, SCAN_WAVES, t0, t1);
    }
    const float4 *q4 = reinterpret_cast<const float4 *>(a.queries) + (size_t)qi * (a.qpitch / 4);
    WaveTopK<E> tk;
    tk.init((int)a.k);
    scan_tiles<METRIC, D, E>(a, q4, t0, t1, tk, a.reverse & 1u, qi);
    group_combine_store<E, SCAN_WAVES>(tk, partials + ((size_t)qi * G + rng) * a.k);
}

// K1Q's tile masks: the validity word for each of the Q queries (FILT ANDs each
// query's own allow word, mq_allow_chunk) -- a function, not a lambda: an
// out-of-line lambda once moved a kernel's arguments to scratch, DESIGN.md section 5.
template <int Q>
__device__ __forceinline__ void mq_tile_masks(const ScanArgs &a, uint64_t t, uint64_t (&mq)[Q])
{
    const uint64_t v = a.valid[t];
#pragma unroll
    for (int j = 0; j < Q; j++) mq[j] = v;
}

// K1Q FILT's allow words of iterations [c0, c0 + 64) of a wave's tile loop: lane
// l holds (lo, hi) of query j's word for iteration c0 + l (0 past the range or the
// window), one vector load per query for up to 64 tiles -- the windows may sit in
// pinned host memory (ScanArgs::allow over the bus), where a tile-ahead scalar
// prefetch left most of the bus latency exposed (profiles/r06/host_api/)
template <int Q>
__device__ __forceinline__ void mq_allow_chunk(const ScanArgs &a, uint64_t t0, uint64_t t1, bool rev, uint64_t c0,
                                               int lane, const uint32_t (&qix)[Q], uint32_t (&lo)[Q],
                                               uint32_t (&hi)[Q])
{
    const uint64_t idx = c0 + (uint64_t)lane;
    const uint64_t t = rev ? t1 - 1 - idx : t0 + idx;
    const uint64_t w = t - a.allow_t0;
    const bool ok = idx < t1 - t0 && w < a.allow_words;
#pragma unroll
    for (int j = 0; j < Q; j++) {
        const uint64_t v = ok ? a.allow[(uint64_t)qix[j] * a.allow_qstride + w] : 0ull;
        lo[j] = (uint32_t)v;
        hi[j] = (uint32_t)(v >> 32);
    }
}

// K1Q (round 5): co-scheduled small batches with Q queries per workgroup.  The
// COS grid gives each (row range, query) its own workgroup; the nq workgroups of a
// range read the same rows side by side, so every row crosses from L2 to the CUs
// nq times and the batch is L2-bound (64 queries over 1M x 128: 32 GB of L2 reads,
// ~2 ms).  Here a wave loads each 32-float block of its row once and folds it into
// the Q queries' AVX2-order chains (acc[Q][4][8]: every query's distance is the
// same chain as a scan of its own, so results are bit-identical), then offers each
// query its key: a quarter of the L2 traffic at Q = 4.  L2 / dot / cosine, fixed D.
// FILT (round 6): coalesced filtered single queries, each with its own allow
// window (ScanArgs::allow_qstride): a tile is loaded if any of the Q queries
// may see a row of it, every query offers only its own rows.
template <int METRIC, int D, int E, int Q, bool FILT = false>
__global__ __launch_bounds__(SCAN_WAVES * 64) void scan_f32_mq_kernel(ScanArgs a, uint64_t *partials)
{
    static_assert(D % 32 == 0 && D > 0 && !is_abs_or_neq<METRIC>, "K1Q: fixed D, the AVX2 chains");
    const uint32_t nqg = (a.nq + Q - 1) / Q;
    const uint32_t G = gridDim.x / nqg;
    const uint32_t kk = blockIdx.x >> 3;
    const uint32_t rng = (kk / nqg) * 8u + (blockIdx.x & 7u), qg = kk % nqg;
    const uint64_t ntiles = a.tile_end - a.tile_begin, total = (uint64_t)G * SCAN_WAVES;
    const uint64_t gw = (uint64_t)rng * SCAN_WAVES + wave_id();
    const uint64_t t0 = a.tile_begin + ntiles * gw / total, t1 = a.tile_begin + ntiles * (gw + 1) / total;
    const int lane = threadIdx.x & 63;
    const float4 *q4[Q];
    uint32_t qix[Q];
#pragma unroll
    for (int j = 0; j < Q; j++) {  // (a short last group repeats its last query and stores nothing for it)
        qix[j] = qg * Q + j < a.nq ? qg * Q + j : a.nq - 1;
        q4[j] = reinterpret_cast<const float4 *>(a.queries) + (size_t)qix[j] * (a.qpitch / 4);
    }
    WaveTopK<E> tk[Q];
#pragma unroll
    for (int j = 0; j < Q; j++) tk[j].init((int)a.k);
    const float4 *data = reinterpret_cast<const float4 *>(a.data);
    const bool rev = (a.reverse & 1u) != 0;
    const uint64_t n = t1 - t0;
    // per-query tile masks (scalar; the next tile's prefetched): the validity word, and with
    // FILT each query's own allow word
    // (FILT: the validity words so, the allow words 64 tiles at a time from mq_allow_chunk)
    uint64_t mq_next[Q];
    if (n) mq_tile_masks<Q>(a, rev ? t1 - 1 : t0, mq_next);
    uint32_t alo[Q], ahi[Q];
    if (FILT && n) mq_allow_chunk<Q>(a, t0, t1, rev, 0, lane, qix, alo, ahi);
    for (uint64_t i = 0; i < n; ++i) {
        const uint64_t t = rev ? t1 - 1 - i : t0 + i;
        uint64_t mq[Q];
#pragma unroll
        for (int j = 0; j < Q; j++) mq[j] = mq_next[j];
        if (i + 1 < n) mq_tile_masks<Q>(a, rev ? t - 1 : t + 1, mq_next);
        if (FILT) {
            const int il = (int)(i & 63u);
            if (il == 0 && i > 0) mq_allow_chunk<Q>(a, t0, t1, rev, i, lane, qix, alo, ahi);
#pragma unroll
            for (int j = 0; j < Q; j++)
                mq[j] &= ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)ahi[j], il) << 32) |
                         (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)alo[j], il);
        }
        uint64_t m = 0ull;
#pragma unroll
        for (int j = 0; j < Q; j++) m |= mq[j];
        if (m == 0ull) continue;
        const float4 *rp = data + (size_t)t * a.nchunks * 64 + lane;
        float acc[Q][4][8];
#pragma unroll
        for (int j = 0; j < Q; j++)
#pragma unroll
            for (int r = 0; r < 4; r++)
#pragma unroll
                for (int l = 0; l < 8; l++) acc[j][r][l] = 0.0f;
        constexpr int NB = D / 32;
#pragma unroll 2
        for (int b = 0; b < NB; b++) {
            float4 xs[8];
#pragma unroll
            for (int cc = 0; cc < 8; cc++) xs[cc] = rp[(size_t)(b * 8 + cc) * 64];
#pragma unroll
            for (int j = 0; j < Q; j++)
#pragma unroll
                for (int cc = 0; cc < 8; cc++) chunk_update<METRIC>(acc[j], cc, q4[j][b * 8 + cc], xs[cc]);
        }
#pragma unroll
        for (int j = 0; j < Q; j++)
            tk[j].offer(lane_key(mq[j], wrap_metric(a.metric, avx256_reduce(acc[j], 0.0f)), t, lane));
    }
#pragma unroll
    for (int j = 0; j < Q; j++) {
        const uint32_t qi = qg * Q + j;
        if (qi < a.nq) group_combine_store<E, SCAN_WAVES>(tk[j], partials + ((size_t)qi * G + rng) * a.k);
        __syncthreads();  // the combine's LDS is reused by the next query
    }
}

// The exact rescan of a query list (the K3c screen's flagged queries, whose
// candidate lists overflowed): block (g, f) scans slice g for the listed
// queries f, f + gridDim.y, ... < *nlist; partials [f][groups][k].
template <int METRIC, int D, int E>
__global__ __launch_bounds__(SCAN_WAVES * 64) void scan_f32_qlist_kernel(ScanArgs a, uint64_t *partials,
                                                                          const uint32_t *qlist, const uint32_t *nlist)
{
    const uint32_t nl = *nlist;
    uint64_t t0, t1;
    wave_range(a, SCAN_WAVES, t0, t1);
    for (uint32_t f = blockIdx.y; f < nl; f += gridDim.y) {
        const uint32_t qi = qlist[f];
        const float4 *q4 = reinterpret_cast<const float4 *>(a.queries) + (size_t)qi * (a.qpitch / 4);
        WaveTopK<E> tk;
        tk.init((int)a.k);
        scan_tiles<METRIC, D, E>(a, q4, t0, t1, tk);
        group_combine_store<E, SCAN_WAVES>(tk, partials + ((size_t)f * gridDim.x + blockIdx.x) * a.k);
        __syncthreads();  // the combine's LDS is reused by the next listed query
    }
}

// Empty results for queries [q0, nq): ids KEY_NONE, dists +inf, counts 0
// (what the host path's write_empty returns for an empty corpus / slab).
__device__ __forceinline__ void fill_empty_body(uint64_t *ids, float *dists, uint32_t *counts, uint32_t q0,
                                                uint32_t nq, uint32_t k)
{
    const uint64_t n = (uint64_t)(nq - q0) * k, off = (uint64_t)q0 * k;
    for (uint64_t i = threadIdx.x; i < n; i += blockDim.x) {
        if (ids) ids[off + i] = WVG_KEY_NONE;
        if (dists) dists[off + i] = __builtin_inff();
    }
    if (counts)
        for (uint32_t q = q0 + threadIdx.x; q < nq; q += blockDim.x) counts[q] = 0;
}

__global__ __launch_bounds__(256) void fill_empty_kernel(uint64_t *ids, float *dists, uint32_t *counts, uint32_t nq,
                                                         uint32_t k)
{
    fill_empty_body(ids, dists, counts, 0, nq, k);
}

hipError_t launch_fill_empty(uint64_t *ids, float *dists, uint32_t *counts, uint32_t nq, uint32_t k, hipStream_t s)
{
    if (nq == 0) return hipSuccess;
    hipLaunchKernelGGL(fill_empty_kernel, dim3(1), dim3(256), 0, s, ids, dists, counts, nq, k);
    return hipGetLastError();
}

// In-launch hand-off (cdna_hip_programming.md §6 Guideline 16, form R1): the
// producer stores its list write-through (agent-scope relaxed atomic stores =
// sc1), drains them (s_waitcnt vmcnt(0)) and adds to an arrival counter; no
// release fence, so no per-query L2 writeback.  The consumer polls the counter
// relaxed with s_sleep, then ONE agent-scope acquire drops its stale L1 lines.
// Thread 0 polls; false after `limit` ticks of s_memrealtime (100 MHz; 4 s
// by default), so a waiting workgroup always exits.
// The counter counts up from `base` (0 for a workspace zeroed per call; a
// stream slot's persistent counter otherwise: the unsigned difference is
// exact across the 2^32 wrap).
__device__ __forceinline__ bool wait_arrivals(uint32_t *ctr, uint32_t base, uint32_t target, uint64_t limit)
{
    __shared__ int ok;
    if (threadIdx.x == 0) {
        const uint64_t start = __builtin_amdgcn_s_memrealtime();
        int r = 1;
        while (__hip_atomic_load((gu32 *)ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - base < target) {
            if (__builtin_amdgcn_s_memrealtime() - start > limit) {
                r = 0;
                break;
            }
            __builtin_amdgcn_s_sleep(4);
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        ok = r;
    }
    __syncthreads();
    return ok != 0;
}

// group_combine_store with write-through stores, then the storing wave drains
// and publishes one arrival.
template <int E, int WAVES>
__device__ __forceinline__ void group_combine_publish(WaveTopK<E> &tk, uint64_t *out, uint32_t *arrivals,
                                                      uint32_t *ready = nullptr, uint32_t tag = 0)
{
    __shared__ uint64_t sh[WAVES][64 * E];
    const int lane = threadIdx.x & 63;
    const int wave = wave_id();
#pragma unroll
    for (int e = 0; e < E; e++) sh[wave][e * 64 + lane] = tk.l[e];
    __syncthreads();
    // pairwise tree, as group_combine_store
#pragma unroll
    for (int half = WAVES / 2; half >= 2; half /= 2) {
        if (wave < half) {
            uint64_t o[E];
#pragma unroll
            for (int e = 0; e < E; e++) o[e] = sh[wave + half][e * 64 + lane];
            merge_lists<E>(tk.l, o);
#pragma unroll
            for (int e = 0; e < E; e++) sh[wave][e * 64 + lane] = tk.l[e];
        }
        __syncthreads();
    }
    if (wave == 0) {
        if (WAVES > 1) {
            uint64_t o[E];
#pragma unroll
            for (int e = 0; e < E; e++) o[e] = sh[1][e * 64 + lane];
            merge_lists<E>(tk.l, o);
        }
#pragma unroll
        for (int e = 0; e < E; e++) {
            const int i = e * 64 + lane;
            if (i < tk.k) __hip_atomic_store((gu64 *)(out + i), tk.l[e], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (lane == 0) {
            if (ready)  // StreamJob::ready: this list's own flag
                __hip_atomic_store((gu32 *)ready, tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            else
                __hip_atomic_fetch_add((gu32 *)arrivals, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    __syncthreads();  // sh is reused by the next query
}

// Query-stream scan (see StreamJob).  Workgroups 0..groups-1 scan; workgroup
// `groups` merges.  Scan workgroups never wait on anything, so the merge
// workgroup's wait always ends.
template <int METRIC, int D, int E>
__global__ __launch_bounds__(SCAN_WAVES * 64) void scan_f32_stream_kernel(ScanArgs a, StreamJob j)
{
    const uint32_t G = j.groups;
    if (blockIdx.x == G) {
        for (uint32_t q = 0; q < a.nq; q++) {
            const bool got = j.ready
                                 ? merge_lists_ready<E, SCAN_WAVES>(
                                       j.partials + (size_t)q * G * a.k, j.ready + (size_t)q * G, j.ready_tag + q, G,
                                       a.k, j.wait_limit, a.id_base, j.ids ? j.ids + (size_t)q * a.k : nullptr,
                                       j.dists ? j.dists + (size_t)q * a.k : nullptr, j.counts ? j.counts + q : nullptr,
                                       j.records ? j.records + (size_t)q * (a.k + 1) : nullptr, j.tag)
                                 : wait_arrivals(j.arrivals + q, j.arrival_base, G, j.wait_limit);
            if (!got) {
                // gave up: queries q.. get empty results (never stale ones) and
                // the sticky status word tells wvg_search_device_check
                if (threadIdx.x == 0) atomicOr(j.status, WVG_STATUS_MERGE_TIMEOUT);
                if (j.records) {  // tagged empty entries and count 0: the host reports the timeout
                    for (uint32_t qq = q; qq < a.nq; qq++) {
                        uint4 *r = j.records + (size_t)qq * (a.k + 1);
                        for (uint32_t i = threadIdx.x; i < a.k; i += blockDim.x)
                            r[i] = make_uint4(0xFFFFFFFFu, j.tag, 0x7F800000u, j.tag);
                        __syncthreads();
                        if (threadIdx.x == 0)
                            __hip_atomic_store(reinterpret_cast<uint64_t *>(r + a.k),
                                               (uint64_t)j.tag << 32 | WVG_RECORDS_TIMEOUT, __ATOMIC_RELEASE,
                                               __HIP_MEMORY_SCOPE_SYSTEM);
                    }
                } else {
                    fill_empty_body(j.ids, j.dists, j.counts, q, a.nq, a.k);
                }
                return;
            }
            if (!j.ready)
                merge_lists_body<E, SCAN_WAVES>(j.partials + (size_t)q * G * a.k, G, a.k, a.k, a.id_base,
                                                j.ids ? j.ids + (size_t)q * a.k : nullptr,
                                                j.dists ? j.dists + (size_t)q * a.k : nullptr,
                                                j.counts ? j.counts + q : nullptr,
                                                j.records ? j.records + (size_t)q * (a.k + 1) : nullptr, j.tag,
                                                j.legacy_poll != 0);
            __syncthreads();  // merge LDS reused by the next query
        }
        return;
    }
    const uint64_t ntiles = a.tile_end - a.tile_begin;
    const uint64_t total = (uint64_t)G * SCAN_WAVES;
    const uint64_t gw = (uint64_t)blockIdx.x * SCAN_WAVES + wave_id();
    uint64_t t0, t1, fmask = ~0ull, lmask = ~0ull;
    if (j.row_split) {
        // row-granular: every wave gets the same number of rows (+-1), so none ends a
        // whole tile after the others (tile-granular: 15 or 16 tiles per wave at 1M rows)
        const uint64_t nrows = ntiles * 64, r0 = nrows * gw / total, r1 = nrows * (gw + 1) / total;
        t0 = a.tile_begin + r0 / 64;
        t1 = a.tile_begin + (r1 + 63) / 64;
        fmask = ~0ull << (r0 % 64);
        const uint32_t hi = (uint32_t)(r1 - (t1 - 1 - a.tile_begin) * 64);  // 1..64 lanes of the last tile
        lmask = hi >= 64 ? ~0ull : (1ull << hi) - 1ull;
        if (r0 == r1) t1 = t0;
    } else {
        t0 = a.tile_begin + ntiles * gw / total;
        t1 = a.tile_begin + ntiles * (gw + 1) / total;
    }
    // (queries null: one query inline in the kernel arguments, StreamJob::qin)
    const float4 *qsrc = a.queries ? reinterpret_cast<const float4 *>(a.queries) : reinterpret_cast<const float4 *>(j.qin);
    for (uint32_t q = 0; q < a.nq; q++) {
        const float4 *q4 = qsrc + (size_t)q * (a.qpitch / 4);
        WaveTopK<E> tk;
        tk.init((int)a.k);
        scan_tiles<METRIC, D, E>(a, q4, t0, t1, tk, (a.reverse + q) & 1u, 0, fmask, lmask);  // serpentine
        group_combine_publish<E, SCAN_WAVES>(tk, j.partials + ((size_t)q * G + blockIdx.x) * a.k, j.arrivals + q,
                                             j.ready ? j.ready + (size_t)q * G + blockIdx.x : nullptr,
                                             j.ready_tag + q);
    }
}

#ifdef WVG_TOOLS
// Tools-build A/B variants of K1 (tuning key 0; profiles/r01/scan_ab_*.jsonl):
// none beat scan_f32_kernel, so the product library does not carry them.
// Variant 1: block-granular software pipeline.  The wave's tile range is a
// flat sequence of 32-float blocks (8 chunks = 8 KiB per wave); the loads of
// the next two blocks are in flight while a block is folded, across tile
// boundaries, so a wave never idles the memory system between tiles.  Every
// tile is loaded (no skip): used when there is no allow list.
template <int METRIC, int D, int E>
__global__ __launch_bounds__(SCAN_WAVES * 64) void scan_f32_pipe_kernel(ScanArgs a, uint64_t *partials)
{
    static_assert(D % 32 == 0 && D > 0, "pipelined scan needs a fixed D % 32 == 0");
    constexpr int NB = D / 32;
    const int lane = threadIdx.x & 63;
    const uint32_t qi = blockIdx.y;
    const float4 *q4 = reinterpret_cast<const float4 *>(a.queries) + (size_t)qi * (a.qpitch / 4);
    const float4 *data = reinterpret_cast<const float4 *>(a.data) + lane;
    uint64_t t0, t1;
    wave_range(a, SCAN_WAVES, t0, t1);
    WaveTopK<E> tk;
    tk.init((int)a.k);
    const uint64_t nunits = (t1 - t0) * NB;
    float acc[4][8];
    uint64_t m = 0;
    float4 b0[8], b1[8], b2[8];
    auto load_unit = [&](float4 (&buf)[8], uint64_t u) {
        if (u < nunits) {
            const uint64_t t = t0 + u / NB;
            const uint32_t b = (uint32_t)(u % NB);
            const float4 *p = data + ((size_t)t * (D / 4) + b * 8) * 64;
#pragma unroll
            for (int cc = 0; cc < 8; cc++) buf[cc] = ld_stream(p + cc * 64);
        }
    };
    auto consume = [&](const float4 (&buf)[8], uint64_t u) {
        const uint64_t t = t0 + u / NB;
        const uint32_t b = (uint32_t)(u % NB);
        if (b == 0) {
            m = tile_mask(a, t);
#pragma unroll
            for (int j = 0; j < 4; j++)
#pragma unroll
                for (int l = 0; l < 8; l++) acc[j][l] = 0.0f;
        }
#pragma unroll
        for (int cc = 0; cc < 8; cc++) chunk_update<METRIC>(acc, cc, q4[b * 8 + cc], buf[cc]);
        if (b == NB - 1) tk.offer(lane_key(m, wrap_metric(a.metric, avx256_reduce(acc, 0.0f)), t, lane));
    };
    load_unit(b0, 0);
    load_unit(b1, 1);
    for (uint64_t u = 0; u < nunits; u += 3) {
        load_unit(b2, u + 2);
        consume(b0, u);
        if (u + 1 >= nunits) break;
        load_unit(b0, u + 3);
        consume(b1, u + 1);
        if (u + 2 >= nunits) break;
        load_unit(b1, u + 4);
        consume(b2, u + 2);
    }
    group_combine_store<E, SCAN_WAVES>(tk, partials + ((size_t)qi * gridDim.x + blockIdx.x) * a.k);
}

// Variant 3: as variant 0, but tiles are dealt round-robin to the waves of
// the whole grid (wave g takes tiles g, g + G, g + 2G, ...), so at any moment
// all waves read neighbouring tiles: one sweeping front through HBM instead of
// thousands of separate streams (DRAM row-buffer locality).
template <int METRIC, int D, int E>
__global__ __launch_bounds__(SCAN_WAVES * 64) void scan_f32_sweep_kernel(ScanArgs a, uint64_t *partials)
{
    const int lane = threadIdx.x & 63;
    const uint32_t qi = blockIdx.y;
    const float4 *q4 = reinterpret_cast<const float4 *>(a.queries) + (size_t)qi * (a.qpitch / 4);
    const float4 *data = reinterpret_cast<const float4 *>(a.data);
    const uint64_t G = (uint64_t)gridDim.x * SCAN_WAVES;
    const uint64_t t0 = a.tile_begin + (uint64_t)blockIdx.x * SCAN_WAVES + wave_id();
    WaveTopK<E> tk;
    tk.init((int)a.k);
    uint64_t m_next = t0 < a.tile_end ? tile_mask(a, t0) : 0ull;
    for (uint64_t t = t0; t < a.tile_end; t += G) {
        const uint64_t m = m_next;
        if (t + G < a.tile_end) m_next = tile_mask(a, t + G);
        if (m == 0ull) continue;
        const float4 *rp = data + (size_t)t * a.nchunks * 64 + lane;
        float r;
        if (a.order512)
            r = row_dist_512<METRIC, 64>(rp, q4, (int)a.dim);
        else if constexpr (D > 0)
            r = row_dot_or_l2_fixed<METRIC, D, 64>(rp, q4);
        else
            r = row_dot_or_l2_generic<METRIC, 64>(rp, q4, (int)a.dim);
        tk.offer(lane_key(m, wrap_metric(a.metric, r), t, lane));
    }
    group_combine_store<E, SCAN_WAVES>(tk, partials + ((size_t)qi * gridDim.x + blockIdx.x) * a.k);
}

// Plain-load twin of variant 0 for A/B (variant 2).
template <int METRIC, int D, int E>
__global__ __launch_bounds__(SCAN_WAVES * 64) void scan_f32_plain_kernel(ScanArgs a, uint64_t *partials)
{
    const int lane = threadIdx.x & 63;
    const uint32_t qi = blockIdx.y;
    const float4 *q4 = reinterpret_cast<const float4 *>(a.queries) + (size_t)qi * (a.qpitch / 4);
    const float4 *data = reinterpret_cast<const float4 *>(a.data);
    uint64_t t0, t1;
    wave_range(a, SCAN_WAVES, t0, t1);
    WaveTopK<E> tk;
    tk.init((int)a.k);
    for (uint64_t t = t0; t < t1; ++t) {
        const uint64_t m = tile_mask(a, t);
        if (m == 0ull) continue;
        const float4 *rp = data + (size_t)t * a.nchunks * 64 + lane;
        const float r = row_dist<METRIC, 64>(rp, q4, D, a.order512);
        tk.offer(lane_key(m, wrap_metric(a.metric, r), t, lane));
    }
    group_combine_store<E, SCAN_WAVES>(tk, partials + ((size_t)qi * gridDim.x + blockIdx.x) * a.k);
}
#endif  // WVG_TOOLS

// Grid: `groups_per_cu` resident workgroups of 4 waves per CU (3 at the d=128
// kernel's 167 VGPRs), each wave owning a contiguous tile range of at least 2
// tiles.  For nq > 1 the queries share the machine.
int scan_groups_for(const ScanArgs &a, int num_cus)
{
    const uint64_t ntiles = a.tile_end > a.tile_begin ? a.tile_end - a.tile_begin : 0;
    uint64_t g = (ntiles + SCAN_WAVES * 2 - 1) / (SCAN_WAVES * 2);
    // groups_per_cu 0 = auto (tools/k1_dim_ab.py, profiles/r01/k1_grid/,
    // profiles/r05/headline_gpc/):
    // - d <= 128: two per CU (round 1 measured L2 3-6 % slower with two on
    //   its kernel; with round 5's query-stream kernel -- tile ranges, per-list
    //   hand-offs -- the 16-query headline launch is 8 % faster with two:
    //   1126 -> 1041 us, and a lone query 82.6 -> 80.4 us; dot / cosine: one
    //   ran 20M x 128 cosine at 4.2 TB/s, two at 6.7);
    // - d > 128 (F32 only; a.dim is 0 for BQ / PQ): three (a d = 768 row is
    //   loaded 16 KiB at a time per wave: 4.2 -> 7.15 TB/s at 10M x 768,
    //   4.2 -> 7.0 at 3M x 1536).
    int gpc = tuning().groups_per_cu;
    if (gpc <= 0) gpc = a.dim > 128 ? 3 : (a.dim > 0 ? 2 : 1);
    uint64_t cap = (uint64_t)num_cus * (uint64_t)gpc;
    if (a.nq > 1) cap = std::max<uint64_t>((uint64_t)num_cus / 4, cap / a.nq);
    if (g > cap) g = cap;
    if (g < 1) g = 1;
    return (int)g;
}

template <int METRIC, int D, int E>
static void launch_fixed(const ScanArgs &a, uint64_t *partials, dim3 grid, dim3 block, hipStream_t s)
{
#ifdef WVG_TOOLS
    // variants 1-3: AVX2 order only, and L2 / dot (their chain sets)
    const int v = a.side.active || a.order512 || is_abs_or_neq<METRIC> ? 0 : tuning().scan_variant;
    if constexpr (!is_abs_or_neq<METRIC>) {
        if (v == 1 && !a.allow)
            return launch_timed((scan_f32_pipe_kernel<METRIC, D, E>), grid, block, 0, s, a, partials);
        if (v == 2) return launch_timed((scan_f32_plain_kernel<METRIC, D, E>), grid, block, 0, s, a, partials);
        if (v == 3) return launch_timed((scan_f32_sweep_kernel<METRIC, D, E>), grid, block, 0, s, a, partials);
    }
#endif
    launch_timed((scan_f32_kernel<METRIC, D, E>), grid, block, 0, s, a, partials);
}

template <int METRIC, int E>
static hipError_t launch_f32_e(const ScanArgs &a, uint64_t *partials, int groups, hipStream_t s)
{
    if constexpr (!is_abs_or_neq<METRIC>) {
        // K1Q: ScanArgs::cosched = Q >= 2 queries per workgroup (plan_search sets it for L2 / dot /
        // cosine batches at d = 128 / 768 without a shared allow window; groups = its row ranges);
        // coalesced filtered queries (per-query windows, allow_qstride) take the FILT variant
        const bool filt = a.allow && a.allow_qstride;
        if ((a.cosched == 2 || a.cosched == 4) && a.nq > 1 && groups % 8 == 0 && !a.side.active &&
            (!a.allow || filt) && !a.order512 && (a.dim == 128 || a.dim == 768)) {
            const uint32_t nqg = (a.nq + (uint32_t)a.cosched - 1) / (uint32_t)a.cosched;
            dim3 grid((unsigned)groups * nqg), block(SCAN_WAVES * 64);
            auto go = [&](auto fq) {
                constexpr bool F = decltype(fq)::value;
                if (a.cosched == 4) {
                    if (a.dim == 128) launch_timed((scan_f32_mq_kernel<METRIC, 128, E, 4, F>), grid, block, 0, s, a, partials);
                    else launch_timed((scan_f32_mq_kernel<METRIC, 768, E, 4, F>), grid, block, 0, s, a, partials);
                } else {
                    if (a.dim == 128) launch_timed((scan_f32_mq_kernel<METRIC, 128, E, 2, F>), grid, block, 0, s, a, partials);
                    else launch_timed((scan_f32_mq_kernel<METRIC, 768, E, 2, F>), grid, block, 0, s, a, partials);
                }
            };
            if (filt) go(std::true_type{});
            else go(std::false_type{});
            return hipGetLastError();
        }
    }
    if (a.cosched && a.nq > 1 && groups % 8 == 0 && !a.side.active) {
        dim3 grid((unsigned)groups * a.nq), block(SCAN_WAVES * 64);
        switch (a.dim) {
        case 128: launch_timed((scan_f32_kernel<METRIC, 128, E, true>), grid, block, 0, s, a, partials); break;
        case 768: launch_timed((scan_f32_kernel<METRIC, 768, E, true>), grid, block, 0, s, a, partials); break;
        case 1536: launch_timed((scan_f32_kernel<METRIC, 1536, E, true>), grid, block, 0, s, a, partials); break;
        default: launch_timed((scan_f32_kernel<METRIC, 0, E, true>), grid, block, 0, s, a, partials); break;
        }
        return hipGetLastError();
    }
    dim3 grid(groups + (a.side.active ? 1 : 0), a.nq), block(SCAN_WAVES * 64);
    switch (a.dim) {
    case 128: launch_fixed<METRIC, 128, E>(a, partials, grid, block, s); break;
    case 768: launch_fixed<METRIC, 768, E>(a, partials, grid, block, s); break;
    case 1536: launch_fixed<METRIC, 1536, E>(a, partials, grid, block, s); break;
    default: launch_timed((scan_f32_kernel<METRIC, 0, E>), grid, block, 0, s, a, partials); break;
    }
    return hipGetLastError();
}

template <int METRIC, int E>
static hipError_t launch_stream_e(const ScanArgs &a, const StreamJob &j, hipStream_t s)
{
    dim3 grid(j.groups + 1), block(SCAN_WAVES * 64);
    switch (a.dim) {
    case 128: launch_timed((scan_f32_stream_kernel<METRIC, 128, E>), grid, block, 0, s, a, j); break;
    case 768: launch_timed((scan_f32_stream_kernel<METRIC, 768, E>), grid, block, 0, s, a, j); break;
    case 1536: launch_timed((scan_f32_stream_kernel<METRIC, 1536, E>), grid, block, 0, s, a, j); break;
    default: launch_timed((scan_f32_stream_kernel<METRIC, 0, E>), grid, block, 0, s, a, j); break;
    }
    return hipGetLastError();
}

template <int METRIC>
static hipError_t launch_stream_m(const ScanArgs &a, const StreamJob &j, hipStream_t s)
{
    if (a.k <= 64) return launch_stream_e<METRIC, 1>(a, j, s);
    if (a.k <= 128) return launch_stream_e<METRIC, 2>(a, j, s);
    return launch_stream_e<METRIC, 4>(a, j, s);
}

hipError_t launch_scan_f32_stream(const ScanArgs &a, const StreamJob &j, hipStream_t s)
{
    return with_metric(a.metric, [&](auto M) { return launch_stream_m<decltype(M)::value>(a, j, s); });
}

template <int METRIC>
static hipError_t launch_f32_m(const ScanArgs &a, uint64_t *partials, int groups, hipStream_t s)
{
    if (a.k <= 64) return launch_f32_e<METRIC, 1>(a, partials, groups, s);
    if (a.k <= 128) return launch_f32_e<METRIC, 2>(a, partials, groups, s);
    return launch_f32_e<METRIC, 4>(a, partials, groups, s);
}

template <int METRIC, int E>
static hipError_t launch_qlist_e(const ScanArgs &a, uint64_t *partials, int groups, const uint32_t *qlist,
                                 const uint32_t *nlist, uint32_t slots, hipStream_t s)
{
    dim3 grid(groups, slots), block(SCAN_WAVES * 64);
    switch (a.dim) {
    case 128: hipLaunchKernelGGL((scan_f32_qlist_kernel<METRIC, 128, E>), grid, block, 0, s, a, partials, qlist, nlist); break;
    case 768: hipLaunchKernelGGL((scan_f32_qlist_kernel<METRIC, 768, E>), grid, block, 0, s, a, partials, qlist, nlist); break;
    default: hipLaunchKernelGGL((scan_f32_qlist_kernel<METRIC, 0, E>), grid, block, 0, s, a, partials, qlist, nlist); break;
    }
    return hipGetLastError();
}

hipError_t launch_scan_f32_qlist(const ScanArgs &a, uint64_t *partials, int groups, const uint32_t *qlist,
                                 const uint32_t *nlist, uint32_t slots, hipStream_t s)
{
    return with_metric(a.metric, [&](auto M) -> hipError_t {
        constexpr int MM = decltype(M)::value;
        if (a.k <= 64) return launch_qlist_e<MM, 1>(a, partials, groups, qlist, nlist, slots, s);
        if (a.k <= 128) return launch_qlist_e<MM, 2>(a, partials, groups, qlist, nlist, slots, s);
        return launch_qlist_e<MM, 4>(a, partials, groups, qlist, nlist, slots, s);
    });
}

hipError_t launch_scan_f32(const ScanArgs &a, uint64_t *partials, int groups, hipStream_t s)
{
    return with_metric(a.metric, [&](auto M) { return launch_f32_m<decltype(M)::value>(a, partials, groups, s); });
}

// ---------------------------------------------------------------------------
// Phase 2: per query, `nlists` ascending lists of `list_len` keys -> final ids
// / dists / counts.  The lists are read TRANSPOSED: a wave takes 64 lists and
// offers batch r = the r-th key of each; batch 0 (the 64 list heads) is
// sorted once, after which almost every lane is rejected by one compare, and
// the first batch with no key below the threshold ends the group (every later
// key of those lists is larger).  Unsorted input: list_len = 1.
// ---------------------------------------------------------------------------
constexpr int MERGE_WAVES = 8;

template <int E>
__global__ __launch_bounds__(MERGE_WAVES * 64) void merge_keys_kernel(const uint64_t *partials, uint32_t nlists,
                                                                      uint32_t list_len, uint32_t k, uint64_t id_base,
                                                                      uint64_t *ids, float *dists, uint32_t *counts)
{
    const uint32_t qi = blockIdx.x;
    merge_lists_body<E, MERGE_WAVES>(partials + (size_t)qi * nlists * list_len, nlists, list_len, k, id_base,
                                     ids + (size_t)qi * k, dists + (size_t)qi * k, counts ? counts + qi : nullptr);
}

hipError_t launch_merge_lists(const uint64_t *partials, uint32_t nq, uint32_t nlists, uint32_t list_len, uint32_t k,
                              uint64_t id_base, uint64_t *ids, float *dists, uint32_t *counts, hipStream_t s)
{
    dim3 grid(nq), block(MERGE_WAVES * 64);
    if (k <= 64)
        hipLaunchKernelGGL((merge_keys_kernel<1>), grid, block, 0, s, partials, nlists, list_len, k, id_base, ids,
                           dists, counts);
    else if (k <= 128)
        hipLaunchKernelGGL((merge_keys_kernel<2>), grid, block, 0, s, partials, nlists, list_len, k, id_base, ids,
                           dists, counts);
    else
        hipLaunchKernelGGL((merge_keys_kernel<4>), grid, block, 0, s, partials, nlists, list_len, k, id_base, ids,
                           dists, counts);
    return hipGetLastError();
}

// Phase 2 for a query list: block f merges listed query qlist[f]'s lists
// (partials [f][nlists][list_len]) into that query's outputs.
template <int E>
__global__ __launch_bounds__(MERGE_WAVES * 64) void merge_keys_qlist_kernel(const uint64_t *partials, uint32_t nlists,
                                                                            uint32_t list_len, uint32_t k,
                                                                            uint64_t id_base, uint64_t *ids,
                                                                            float *dists, uint32_t *counts,
                                                                            const uint32_t *qlist,
                                                                            const uint32_t *nlist)
{
    const uint32_t f = blockIdx.x;
    if (f >= *nlist) return;
    const uint32_t qi = qlist[f];
    merge_lists_body<E, MERGE_WAVES>(partials + (size_t)f * nlists * list_len, nlists, list_len, k, id_base,
                                     ids + (size_t)qi * k, dists + (size_t)qi * k, counts ? counts + qi : nullptr);
}

hipError_t launch_merge_lists_qlist(const uint64_t *partials, uint32_t nq, uint32_t nlists, uint32_t list_len,
                                    uint32_t k, uint64_t id_base, uint64_t *ids, float *dists, uint32_t *counts,
                                    const uint32_t *qlist, const uint32_t *nlist, hipStream_t s)
{
    dim3 grid(nq), block(MERGE_WAVES * 64);
    if (k <= 64)
        hipLaunchKernelGGL((merge_keys_qlist_kernel<1>), grid, block, 0, s, partials, nlists, list_len, k, id_base, ids,
                           dists, counts, qlist, nlist);
    else if (k <= 128)
        hipLaunchKernelGGL((merge_keys_qlist_kernel<2>), grid, block, 0, s, partials, nlists, list_len, k, id_base, ids,
                           dists, counts, qlist, nlist);
    else
        hipLaunchKernelGGL((merge_keys_qlist_kernel<4>), grid, block, 0, s, partials, nlists, list_len, k, id_base, ids,
                           dists, counts, qlist, nlist);
    return hipGetLastError();
}

hipError_t launch_merge_keys(const uint64_t *partials, uint32_t nq, uint32_t n_per_query, uint32_t k,
                             uint64_t id_base, uint64_t *ids, float *dists, uint32_t *counts, hipStream_t s)
{
    return launch_merge_lists(partials, nq, n_per_query, 1, k, id_base, ids, dists, counts, s);
}

// ---------------------------------------------------------------------------
// Multi-shard merge of (dist, id64) lists: one workgroup per query, bitonic
// sort in LDS of all nlists*k_in pairs ordered by (dist, id).  Used after the
// RCCL all-gather of per-GPU top-k (adapters/repos/db/index.go:1644-1648).
// ---------------------------------------------------------------------------
constexpr int MERGE_PAIRS_MAX = 8192;

// List l of query qi starts at ids + l * ids_stride + qi * k_in (and likewise
// for dists): strides of nq * k_in for the plain [nlists][nq][k_in] arrays,
// the packed block size for all-gathered wvg_topk_packed blocks.
__global__ __launch_bounds__(1024) void merge_pairs_kernel(const float *dists, const uint64_t *ids,
                                                           uint64_t ids_stride, uint64_t d_stride,
                                                           uint32_t nlists, uint32_t k_in, uint32_t k,
                                                           uint32_t pow2, uint64_t *out_ids,
                                                           float *out_dists, uint32_t *out_counts)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    uint64_t *sid = reinterpret_cast<uint64_t *>(smem);
    uint32_t *sd = reinterpret_cast<uint32_t *>(smem + (size_t)pow2 * 8);
    const uint32_t qi = blockIdx.x;
    const uint32_t n = nlists * k_in;
    for (uint32_t i = threadIdx.x; i < pow2; i += blockDim.x) {
        if (i < n) {
            const uint32_t l = i / k_in, j = i % k_in;
            const size_t q_off = (size_t)qi * k_in + j;
            const uint64_t id = ids[l * ids_stride + q_off];
            sid[i] = id;
            sd[i] = id == WVG_KEY_NONE ? 0xFFFFFFFFu : wvg_ord_f32(dists[l * d_stride + q_off]);
        } else {
            sid[i] = WVG_KEY_NONE;
            sd[i] = 0xFFFFFFFFu;
        }
    }
    __syncthreads();
    for (uint32_t size = 2; size <= pow2; size <<= 1) {
        for (uint32_t stride = size >> 1; stride > 0; stride >>= 1) {
            for (uint32_t i = threadIdx.x; i < pow2; i += blockDim.x) {
                const uint32_t j = i ^ stride;
                if (j > i) {
                    const bool asc = (i & size) == 0;
                    const bool gt = sd[i] > sd[j] || (sd[i] == sd[j] && sid[i] > sid[j]);
                    if (gt == asc) {
                        uint32_t td = sd[i]; sd[i] = sd[j]; sd[j] = td;
                        uint64_t ti = sid[i]; sid[i] = sid[j]; sid[j] = ti;
                    }
                }
            }
            __syncthreads();
        }
    }
    __shared__ uint32_t live_count;
    if (threadIdx.x == 0) live_count = 0;
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < k; i += blockDim.x) {
        const bool live = i < n && sid[i] != WVG_KEY_NONE;
        out_ids[(size_t)qi * k + i] = live ? sid[i] : WVG_KEY_NONE;
        out_dists[(size_t)qi * k + i] = live ? wvg_unord_f32(sd[i]) : __builtin_inff();
        if (live) atomicAdd(&live_count, 1u);
    }
    __syncthreads();
    if (threadIdx.x == 0 && out_counts) out_counts[qi] = live_count;
}

hipError_t launch_merge_pairs(const float *dists, const uint64_t *ids, uint64_t ids_stride, uint64_t d_stride,
                              uint32_t nq, uint32_t nlists, uint32_t k_in, uint32_t k, uint64_t *out_ids,
                              float *out_dists, uint32_t *out_counts, hipStream_t s)
{
    uint32_t n = nlists * k_in, pow2 = 1;
    while (pow2 < n) pow2 <<= 1;
    if (pow2 > (uint32_t)MERGE_PAIRS_MAX) return hipErrorInvalidValue;
    const size_t lds = (size_t)pow2 * 12;
    hipLaunchKernelGGL(merge_pairs_kernel, dim3(nq), dim3(1024), lds, s, dists, ids, ids_stride, d_stride, nlists,
                       k_in, k, pow2, out_ids, out_dists, out_counts);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Layout helpers
// ---------------------------------------------------------------------------

// distancer.Normalize (D/normalize.go:16-32), one lane per row: sequential
// unfused fp32 sum of squares, float32(sqrt(float64)), element-wise divide.
// The sequential fp32 sum of Normalize (D/normalize.go:16-32) over 64 values
// a wave holds at once (lane l: element b + l): the wave folds them in element
// order through v_readlane, so every lane ends with the same, in-order sum.
// One wave per row: the loads are coalesced and the 1536-long dependent add
// chain runs on registers (one thread per row waited on a load per element).
// Round 6: the 64 values go through the wave's 256 bytes of LDS and every lane
// adds them in element order from broadcast reads -- a readlane per element
// made each add wait on a VALU -> SGPR -> VALU round trip (45 us per 1536-float
// row, profiles/r06/final/trace: normalize_rows_kernel); the adds and their
// order are unchanged, so the sum is the same bits.
__device__ __forceinline__ float wave_seq_sum(float acc, float p, uint32_t cnt, float *lds)
{
    const uint32_t lane = threadIdx.x & 63u;
    __builtin_amdgcn_wave_barrier();  // (the previous block's reads of lds are done)
    lds[lane] = p;
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's write landed
    if (cnt == 64) {
#pragma unroll
        for (uint32_t l = 0; l < 64; l += 4) {
            const float4 v = *reinterpret_cast<const float4 *>(lds + l);
            acc = acc + v.x;
            acc = acc + v.y;
            acc = acc + v.z;
            acc = acc + v.w;
        }
    } else {
        for (uint32_t l = 0; l < cnt; l++) acc = acc + lds[l];
    }
    return acc;
}

__global__ __launch_bounds__(256) void normalize_rows_kernel(const float *in, uint64_t n, uint32_t dim, float *out)
{
    const uint32_t lane = threadIdx.x & 63u;
    __shared__ __attribute__((aligned(16))) float sh[4][64];
    const uint64_t r = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);  // one row per wave
    if (r >= n) return;
    const float *v = in + r * dim;
    float *o = out + r * dim;
    float norm = 0.0f;
    for (uint32_t b = 0; b < dim; b += 64) {
        const uint32_t i = b + lane;
        const float x = i < dim ? v[i] : 0.0f;
        const float p = x * x;
        norm = wave_seq_sum(norm, p, dim - b < 64u ? dim - b : 64u, sh[threadIdx.x >> 6]);
    }
    if (norm == 0.0f) {
        for (uint32_t i = lane; i < dim; i += 64) o[i] = 0.0f;
        return;
    }
    norm = (float)__builtin_sqrt((double)norm);
    for (uint32_t i = lane; i < dim; i += 64) o[i] = v[i] / norm;
}

hipError_t launch_normalize_rows(const float *in, uint64_t n, uint32_t dim, float *out, hipStream_t s)
{
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(normalize_rows_kernel, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, s, in, n, dim, out);
    return hipGetLastError();
}

// Row-major [n][dim] -> tiled chunks at slots[i] (identity when slots == null).
__global__ void f32_store_kernel(const float *rows, const uint64_t *slots, uint64_t n, uint32_t dim,
                                 uint32_t nchunks, float4 *tiled)
{
    const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= n * nchunks) return;
    const uint64_t i = g / nchunks;
    const uint32_t c = (uint32_t)(g % nchunks);
    const uint64_t slot = slots ? slots[i] : i;
    const float *src = rows + i * dim;
    float v[4];
#pragma unroll
    for (int e = 0; e < 4; e++) {
        const uint32_t p = c * 4 + e;
        v[e] = p < dim ? src[p] : 0.0f;
    }
    tiled[((slot >> 6) * nchunks + c) * 64 + (slot & 63)] = make_float4(v[0], v[1], v[2], v[3]);
}

hipError_t launch_f32_store(const float *rows, const uint64_t *slots, uint64_t n, uint32_t dim,
                            uint32_t nchunks, int normalize, float *tiled, hipStream_t s)
{
    (void)normalize;  // rows are normalized by the caller (launch_normalize_rows)
    const uint64_t total = n * nchunks;
    if (total == 0) return hipSuccess;
    hipLaunchKernelGGL(f32_store_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, rows, slots, n,
                       dim, nchunks, reinterpret_cast<float4 *>(tiled));
    return hipGetLastError();
}

// Synthetic rows generated in place; for cosine the row is normalized with
// the same sequential order as Normalize (two passes over the generator).
__global__ void f32_synth_kernel(uint64_t seed_mixed, int dist, uint64_t row0, uint64_t n, uint64_t slot0,
                                 uint32_t dim, uint32_t nchunks, int normalize, float4 *tiled)
{
    const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    const uint64_t row = row0 + r, slot = slot0 + r;
    float norm = 1.0f;
    bool zero = false;
    if (normalize) {
        float acc = 0.0f;
        for (uint32_t i = 0; i < dim; i++) {
            float v = wvg_synth_value(seed_mixed, row, i, dist);
            float p = v * v;
            acc = acc + p;
        }
        zero = acc == 0.0f;
        norm = (float)__builtin_sqrt((double)acc);
    }
    float4 *dst = tiled + ((slot >> 6) * nchunks) * 64 + (slot & 63);
    for (uint32_t c = 0; c < nchunks; c++) {
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; e++) {
            const uint32_t p = c * 4 + e;
            float x = p < dim ? wvg_synth_value(seed_mixed, row, p, dist) : 0.0f;
            if (normalize) x = zero ? 0.0f : x / norm;
            v[e] = x;
        }
        dst[(size_t)c * 64] = make_float4(v[0], v[1], v[2], v[3]);
    }
}

hipError_t launch_f32_synth(uint64_t seed, int dist, uint64_t row0, uint64_t n, uint64_t slot0, uint32_t dim,
                            uint32_t nchunks, int normalize, float *tiled, hipStream_t s)
{
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(f32_synth_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, wvg_mix64(seed), dist,
                       row0, n, slot0, dim, nchunks, normalize, reinterpret_cast<float4 *>(tiled));
    return hipGetLastError();
}

__global__ void f32_gather_kernel(const float4 *tiled, const uint64_t *slots, uint64_t n, uint32_t dim,
                                  uint32_t nchunks, float *rows)
{
    const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= n * dim) return;
    const uint64_t i = g / dim;
    const uint32_t p = (uint32_t)(g % dim);
    const uint64_t slot = slots[i];
    const float4 *row = tiled + ((slot >> 6) * nchunks) * 64 + (slot & 63);
    rows[g] = elem_at<64>(row, (int)p);
}

hipError_t launch_f32_gather(const float *tiled, const uint64_t *slots, uint64_t n, uint32_t dim,
                             uint32_t nchunks, float *rows, hipStream_t s)
{
    const uint64_t total = n * dim;
    if (total == 0) return hipSuccess;
    hipLaunchKernelGGL(f32_gather_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s,
                       reinterpret_cast<const float4 *>(tiled), slots, n, dim, nchunks, rows);
    return hipGetLastError();
}

// Stored rows by slot, as raw 16-byte chunks: out[i] = the nchunks chunks of
// slots[i] (any corpus kind; the host trims / un-rotates).
__global__ void gather_chunks_kernel(const uint4 *tiled, const uint64_t *slots, uint64_t n, uint32_t nchunks,
                                     uint4 *out)
{
    const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= n * nchunks) return;
    const uint64_t i = g / nchunks;
    const uint32_t c = (uint32_t)(g % nchunks);
    const uint64_t slot = slots[i];
    out[g] = tiled[((slot >> 6) * nchunks + c) * 64 + (slot & 63)];
}

hipError_t launch_gather_chunks(const void *tiled, const uint64_t *slots, uint64_t n, uint32_t nchunks, void *out,
                                hipStream_t s)
{
    const uint64_t total = n * nchunks;
    if (total == 0) return hipSuccess;
    hipLaunchKernelGGL(gather_chunks_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s,
                       reinterpret_cast<const uint4 *>(tiled), slots, n, nchunks, reinterpret_cast<uint4 *>(out));
    return hipGetLastError();
}

// Provider.SingleDist(q, X[i]) for a tiled temporary (distancer.BatchProvider).
template <int METRIC>
__global__ void distance_tiled_kernel(int metric, const float4 *q4, const float4 *tiled, uint64_t n, uint32_t dim,
                                      uint32_t nchunks, float *out, int o512)
{
    const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    const float4 *rp = tiled + ((r >> 6) * nchunks) * 64 + (r & 63);
    out[r] = wrap_metric(metric, row_dist<METRIC, 64>(rp, q4, (int)dim, o512));
}

hipError_t launch_distance_rows(int metric, const float *q, const float *tiled, uint64_t n, uint32_t dim,
                                float *out, hipStream_t s, int o512)
{
    if (n == 0) return hipSuccess;
    const uint32_t nchunks = f32_chunks(dim);
    dim3 grid((unsigned)((n + 255) / 256)), block(256);
    with_metric(metric, [&](auto M) {
        hipLaunchKernelGGL((distance_tiled_kernel<decltype(M)::value>), grid, block, 0, s, metric,
                           reinterpret_cast<const float4 *>(q), reinterpret_cast<const float4 *>(tiled), n, dim,
                           nchunks, out, o512);
    });
    return hipGetLastError();
}

template <int METRIC>
__global__ void dist_keys_kernel(int metric, const float4 *q4, const float4 *tiled, uint64_t n, uint32_t dim,
                                 uint32_t nchunks, uint64_t *keys, int o512)
{
    const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    const float4 *rp = tiled + ((r >> 6) * nchunks) * 64 + (r & 63);
    keys[r] = wvg_make_key(wrap_metric(metric, row_dist<METRIC, 64>(rp, q4, (int)dim, o512)), (uint32_t)r);
}

hipError_t launch_dist_keys(int metric, const float *q, const float *tiled, uint64_t n, uint32_t dim, uint64_t *keys,
                            hipStream_t s, int o512)
{
    if (n == 0) return hipSuccess;
    const uint32_t nchunks = f32_chunks(dim);
    dim3 grid((unsigned)((n + 255) / 256)), block(256);
    with_metric(metric, [&](auto M) {
        hipLaunchKernelGGL((dist_keys_kernel<decltype(M)::value>), grid, block, 0, s, metric,
                           reinterpret_cast<const float4 *>(q), reinterpret_cast<const float4 *>(tiled), n, dim,
                           nchunks, keys, o512);
    });
    return hipGetLastError();
}

// Synthetic rows for arbitrary ids, row-major (bench / test helper); one
// wave per row, the normalize sum as in normalize_rows_kernel.
__global__ __launch_bounds__(256) void synth_rows_kernel(uint64_t seed_mixed, int dist, const uint64_t *ids,
                                                         uint64_t n, uint32_t dim, int normalize, float *out)
{
    __shared__ __attribute__((aligned(16))) float sh[4][64];
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t r = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (r >= n) return;
    const uint64_t row = ids[r];
    float norm = 1.0f;
    bool zero = false;
    if (normalize) {
        float acc = 0.0f;
        for (uint32_t b = 0; b < dim; b += 64) {
            const uint32_t i = b + lane;
            const float v = i < dim ? wvg_synth_value(seed_mixed, row, i, dist) : 0.0f;
            const float p = v * v;
            acc = wave_seq_sum(acc, p, dim - b < 64u ? dim - b : 64u, sh[threadIdx.x >> 6]);
        }
        zero = acc == 0.0f;
        norm = (float)__builtin_sqrt((double)acc);
    }
    for (uint32_t i = lane; i < dim; i += 64) {
        float x = wvg_synth_value(seed_mixed, row, i, dist);
        if (normalize) x = zero ? 0.0f : x / norm;
        out[r * dim + i] = x;
    }
}

hipError_t launch_synth_rows(uint64_t seed, int dist, const uint64_t *ids, uint64_t n, uint32_t dim, int normalize,
                             float *out, hipStream_t s)
{
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(synth_rows_kernel, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, s, wvg_mix64(seed), dist,
                       ids, n, dim, normalize, out);
    return hipGetLastError();
}

// Exact rescore of candidate keys (slot in the low 32 bits) against the tiled
// float rows: the rescore loop of flat.searchByVectorBQ (V/flat/index.go:375-385).
template <int METRIC>
__global__ void rescore_keys_kernel(int metric, const float4 *q4, uint32_t qpitch, const float4 *tiled, uint32_t dim,
                                    uint32_t nchunks, const uint64_t *cand, uint32_t ncand, uint32_t cand_stride,
                                    uint64_t *out, int o512, int qmajor)
{
    // qmajor: grid (nq, chunks), so consecutive workgroups -- on different XCDs -- are different
    // queries whatever ncand is (grid (chunks, nq) put chunk x of every query on XCD x mod 8 when
    // the chunk count was a multiple of 8: the screen's rescore at 5120 candidates per query ran
    // 0.95 ms instead of 0.24); the other order only for more than 65535 chunks (grid y's limit)
    const uint32_t qi = qmajor ? blockIdx.x : blockIdx.y;
    const uint32_t j = (qmajor ? blockIdx.y : blockIdx.x) * blockDim.x + threadIdx.x;
    if (j >= ncand) return;
    const uint64_t key = cand[(size_t)qi * cand_stride + j];
    uint64_t res = WVG_KEY_NONE;
    if (key != WVG_KEY_NONE) {
        const uint32_t slot = (uint32_t)key;
        const float4 *rp = tiled + ((size_t)(slot >> 6) * nchunks) * 64 + (slot & 63);
        const float4 *q = q4 + (size_t)qi * (qpitch / 4);
        const float d = wrap_metric(metric, row_dist<METRIC, 64>(rp, q, (int)dim, o512));
        res = wvg_make_key(d, slot);
    }
    out[(size_t)qi * ncand + j] = res;
}

hipError_t launch_rescore_keys(int metric, const float *q, uint32_t qpitch, const float *tiled, uint32_t dim,
                               uint32_t nchunks, const uint64_t *cand_keys, uint32_t nq, uint32_t ncand,
                               uint32_t cand_stride, uint64_t *out_keys, hipStream_t s, int o512)
{
    if (nq == 0 || ncand == 0) return hipSuccess;
    const uint32_t chunks = (ncand + 63) / 64;
    const int qmajor = chunks <= 65535 ? 1 : 0;
    dim3 grid(qmajor ? nq : chunks, qmajor ? chunks : nq), block(64);
    with_metric(metric, [&](auto M) {
        hipLaunchKernelGGL((rescore_keys_kernel<decltype(M)::value>), grid, block, 0, s, metric,
                           reinterpret_cast<const float4 *>(q), qpitch, reinterpret_cast<const float4 *>(tiled), dim,
                           nchunks, cand_keys, ncand, cand_stride, out_keys, o512, qmajor);
    });
    return hipGetLastError();
}

// Screen seed (wvg_screen.hip): per query, the k smallest lower-bound keys of
// the first `nlists` range lists (ascending, so only their first k entries
// can be among them; a wave top-k over those), rescored exactly with the
// final rescore's distance, and their k-th distance -- k real rows at or
// below it -- folded into gbound.  One wave per query, rank by shuffles.
template <int METRIC>
__global__ __launch_bounds__(64) void seed_exact_kernel(int metric, const float4 *q4, uint32_t qpitch,
                                                        const float4 *tiled, uint32_t dim, uint32_t nchunks,
                                                        const uint64_t *partials, uint32_t list_stride,
                                                        uint32_t list_len, uint32_t nlists, uint32_t k,
                                                        uint32_t *gbound)
{
    const uint32_t qi = blockIdx.x, lane = threadIdx.x;
    const uint64_t *src = partials + (size_t)qi * list_stride;
    WaveTopK<1> tk;
    tk.init((int)k);
    const uint32_t n = nlists * k;
    for (uint32_t i0 = 0; i0 < n; i0 += 64) {
        const uint32_t i = i0 + lane;
        tk.offer(i < n ? src[(size_t)(i / k) * list_len + i % k] : WVG_KEY_NONE);
    }
    const uint64_t key = lane < k ? tk.l[0] : WVG_KEY_NONE;
    uint32_t v = 0xFFFFFFFFu;
    if (key != WVG_KEY_NONE) {
        const uint32_t slot = (uint32_t)key;
        const float4 *rp = tiled + ((size_t)(slot >> 6) * nchunks) * 64 + (slot & 63);
        v = wvg_ord_f32(wrap_metric(metric, row_dist<METRIC, 64>(rp, q4 + (size_t)qi * (qpitch / 4), (int)dim, 0)));
    }
    const uint64_t live = __ballot(key != WVG_KEY_NONE);
    if ((uint32_t)__popcll(live) < k) return;
    uint32_t rank = 0;
    for (int j = 0; j < 64; j++) {
        const uint32_t o = (uint32_t)__shfl((int)v, j);
        rank += (o < v) || (o == v && (uint32_t)j < lane);
    }
    if (key != WVG_KEY_NONE && rank == k - 1 && wvg_unord_f32(v) < __builtin_inff()) atomicMin(gbound + qi, v);
}

hipError_t launch_seed_exact(int metric, const float *q, uint32_t qpitch, const float *tiled, uint32_t dim,
                             uint32_t nchunks, const uint64_t *partials, uint32_t list_stride, uint32_t list_len,
                             uint32_t nlists, uint32_t nq, uint32_t k, uint32_t *gbound, hipStream_t s)
{
    if (nq == 0 || nlists == 0) return hipSuccess;
    if (k == 0 || k > 64 || k > list_len) return hipErrorInvalidValue;
    with_metric(metric, [&](auto M) {
        hipLaunchKernelGGL((seed_exact_kernel<decltype(M)::value>), dim3(nq), dim3(64), 0, s, metric,
                           reinterpret_cast<const float4 *>(q), qpitch, reinterpret_cast<const float4 *>(tiled), dim,
                           nchunks, partials, list_stride, list_len, nlists, k, gbound);
    });
    return hipGetLastError();
}

// Streaming-read probe behind wvg_measure_hbm_read: the HBM read ceiling the
// scans are judged against, measured in-process (tools/hbm_read.hip's best
// form: grid-stride 16-byte non-temporal loads, 8 in flight per lane).
__global__ __launch_bounds__(256) void hbm_read_kernel(const float4 *__restrict__ p, uint64_t n4, float *out)
{
    typedef float f4v __attribute__((ext_vector_type(4)));
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    const f4v *q = reinterpret_cast<const f4v *>(p);
    float acc = 0.f;
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i + 7 * stride < n4; i += 8 * stride) {
        f4v v[8];
#pragma unroll
        for (int u = 0; u < 8; u++) v[u] = __builtin_nontemporal_load(q + i + u * stride);
#pragma unroll
        for (int u = 0; u < 8; u++) acc += v[u].x + v[u].y + v[u].z + v[u].w;
    }
    for (; i < n4; i += stride) acc += q[i].x;
    if (acc == 12345.678f) out[0] = acc;  // keeps the loads live; never true for the zero-filled buffer
}

// The scans' own access shape: each workgroup streams one contiguous chunk,
// each wave 8 consecutive KiB per step (8 non-temporal 16-byte loads per lane
// in flight), so a DRAM page is read by one wave at a time.
__global__ __launch_bounds__(256) void hbm_read_chunk_kernel(const float4 *__restrict__ p, uint64_t n4, float *out)
{
    typedef float f4v __attribute__((ext_vector_type(4)));
    const uint64_t per = (n4 + gridDim.x - 1) / gridDim.x;
    const uint64_t lo = (uint64_t)blockIdx.x * per;
    const uint64_t hi = lo + per < n4 ? lo + per : n4;
    const f4v *q = reinterpret_cast<const f4v *>(p);
    const unsigned wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    float acc = 0.f;
    uint64_t i = lo + wave * 512 + lane;
    for (; i + 7 * 64 < hi; i += 4 * 512) {
        f4v v[8];
#pragma unroll
        for (int u = 0; u < 8; u++) v[u] = __builtin_nontemporal_load(q + i + u * 64);
#pragma unroll
        for (int u = 0; u < 8; u++) acc += v[u].x + v[u].y + v[u].z + v[u].w;
    }
    for (; i < hi; i += 64) acc += q[i].x;
    if (acc == 12345.678f) out[0] = acc;
}

hipError_t launch_hbm_read(const void *p, uint64_t bytes, int blocks, float *out, hipStream_t s)
{
    // blocks < 0: the contiguous-chunk form with -blocks workgroups
    if (blocks < 0)
        hipLaunchKernelGGL(hbm_read_chunk_kernel, dim3(-blocks), dim3(256), 0, s, reinterpret_cast<const float4 *>(p),
                           bytes / 16, out);
    else
        hipLaunchKernelGGL(hbm_read_kernel, dim3(blocks), dim3(256), 0, s, reinterpret_cast<const float4 *>(p),
                           bytes / 16, out);
    return hipGetLastError();
}

// Validity bits (flat.Add sets, flat.Delete clears; V/flat/index.go:247-295).
__global__ void set_valid_kernel(unsigned long long *valid, const uint64_t *slots, uint64_t n, int set)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t s = slots[i];
    const unsigned long long bit = 1ull << (s & 63);
    if (set)
        atomicOr(valid + (s >> 6), bit);
    else
        atomicAnd(valid + (s >> 6), ~bit);
}

hipError_t launch_set_valid(uint64_t *valid, const uint64_t *slots, uint64_t n, int set, hipStream_t s)
{
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(set_valid_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s,
                       reinterpret_cast<unsigned long long *>(valid), slots, n, set);
    return hipGetLastError();
}

}  // namespace wvg
