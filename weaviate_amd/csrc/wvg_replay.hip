// wvg_replay.hip -- the reference's heap, reproduced exactly, for the BQ flow
// (flat.searchByVectorBQ, V/flat/index.go:347-389).
//
// Why.  findTopVectorsCached (index.go:456-495) walks the docIDs in ascending
// order through a bounded max-heap (insertToHeap, :497-506; priorityqueue,
// adapters/repos/db/priorityqueue/queue.go).  Hamming distances are small
// integers, so at R = 200 over millions of rows the R-th distance is shared
// by many rows, and WHICH of them the heap keeps -- and the order it pops
// them in, which is the order the rescore inserts them into the k-heap
// (:368-385) -- follows from the heap's insertion history, not from any
// ordering of (distance, docID).  A lexicographic top-R can therefore hand
// the rescore a different candidate set and change the final top-k.
//
// How.  The heap inserts row i iff fewer than R rows precede it or d_i <
// T_i, the R-th smallest distance of all rows before i; every other row is a
// no-op.  So replaying the heap over any superset of the inserted rows, in
// docID order, reproduces it exactly.  The device finds a small superset:
//  1. K5 EMIT (wvg_bq.hip): each wave keeps d_i < its own running R-th
//     distance (T_i can only be lower: the wave sees a subset of the prefix);
//  2. emit_prefix: per query, thr[g] = the R-th smallest distance of all
//     ranges before range g (from the ranges' top-R lists);
//  3. emit_filter: drop the kept rows with d_i >= thr[g] (T_i <= thr[g]);
//  4. emit_gather: the survivors of all waves in wave = docID order.
// About R (1 + ln G) rows per query survive (~1.5k for R = 200), which the
// host replays through the heap (wvg_heap.hpp), pops, rescores exactly on the
// device (K6) and replays again into the k-heap.  A wave whose buffer
// overflows (adversarial orders: distances falling with the docID) reruns its
// query with full-size buffers, seeded with the first pass's thr.
#include "wvg_heap.hpp"
#include "wvg_host.hpp"
#include "wvg_topk.hpp"

namespace wvg {

// ---- device -------------------------------------------------------------------

// key of list element k-1 (wave-uniform); the select runs on the scalar side
template <int E>
__device__ __forceinline__ uint64_t kth_key(const uint64_t (&l)[E], uint32_t k)
{
    const int idx = (int)k - 1, hi = idx >> 6, lo = idx & 63;
    uint64_t t = readlane64(l[0], lo);
#pragma unroll
    for (int e = 1; e < E; e++) {
        const uint64_t te = readlane64(l[e], lo);
        t = hi == e ? te : t;
    }
    return t;
}

// l <- the k smallest of (l U the ascending list o); entries past k are don't-care.
template <int E>
__device__ __forceinline__ void fold_list(uint64_t (&l)[E], const uint64_t (&o)[E], uint32_t k)
{
    uint64_t t = kth_key<E>(l, k);
    uint32_t c = 0;
#pragma unroll
    for (int e = 0; e < E; e++) c += (uint32_t)__popcll(__ballot(o[e] < t));
    if (c == 0) return;
    if (c > (uint32_t)TOPK_INSERT_MAX) {
        merge_lists<E>(l, o);
        return;
    }
    // the c entries below the k-th are o's first c (o ascending, c <= 12 < 64)
    for (uint32_t i = 0; i < c; i++) {
        const uint64_t x = readlane64(o[0], (int)i);
        if (x >= t) break;
        insert_one<E>(l, x);
        t = kth_key<E>(l, k);
    }
}

template <int E>
__device__ __forceinline__ void load_list(uint64_t (&o)[E], const uint64_t *p, uint32_t k, int lane)
{
#pragma unroll
    for (int e = 0; e < E; e++) {
        const uint32_t i = (uint32_t)(e * 64 + lane);
        o[e] = i < k ? p[i] : WVG_KEY_NONE;
    }
}

__device__ __forceinline__ float key_dist(uint64_t key)
{
    return key == WVG_KEY_NONE ? __builtin_inff() : wvg_unord_f32((uint32_t)(key >> 32));
}

// thr[q][g] = R-th smallest distance of ranges 0..g-1 (their top-R lists).
// One 16-wave workgroup per query, in three phases so the serial chain is
// ~3 * groups / 16 folds instead of `groups`: (A) wave w folds the lists of
// its block of ranges; (B) wave 0 turns the block lists into exclusive
// prefixes; (C) wave w folds its block's lists again, starting from its
// prefix, and records the threshold before each.
constexpr int PREFIX_WAVES = 16;
template <int E>
__global__ __launch_bounds__(PREFIX_WAVES * 64) void emit_prefix_kernel(const uint64_t *partials, uint32_t groups,
                                                                        uint32_t k, float *thr)
{
    __shared__ uint64_t blk[PREFIX_WAVES][64 * E];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t qi = blockIdx.x;
    const uint64_t *pq = partials + (size_t)qi * groups * k;
    const uint32_t per = (groups + PREFIX_WAVES - 1) / PREFIX_WAVES;
    const uint32_t g0 = min(groups, (uint32_t)wave * per), g1 = min(groups, g0 + per);
    uint64_t l[E], o[E];
#pragma unroll
    for (int e = 0; e < E; e++) l[e] = WVG_KEY_NONE;
    for (uint32_t g = g0; g < g1; g++) {  // (A)
        load_list<E>(o, pq + (size_t)g * k, k, lane);
        fold_list<E>(l, o, k);
    }
#pragma unroll
    for (int e = 0; e < E; e++) blk[wave][e * 64 + lane] = l[e];
    __syncthreads();
    if (wave == 0) {  // (B)
        uint64_t pre[E];
#pragma unroll
        for (int e = 0; e < E; e++) pre[e] = WVG_KEY_NONE;
        for (int w = 0; w < PREFIX_WAVES; w++) {
#pragma unroll
            for (int e = 0; e < E; e++) o[e] = blk[w][e * 64 + lane];
#pragma unroll
            for (int e = 0; e < E; e++) blk[w][e * 64 + lane] = pre[e];
            fold_list<E>(pre, o, k);
        }
    }
    __syncthreads();
#pragma unroll
    for (int e = 0; e < E; e++) l[e] = blk[wave][e * 64 + lane];
    for (uint32_t g = g0; g < g1; g++) {  // (C)
        const float t = key_dist(kth_key<E>(l, k));
        if (lane == 0) thr[(size_t)qi * groups + g] = t;
        load_list<E>(o, pq + (size_t)g * k, k, lane);
        fold_list<E>(l, o, k);
    }
}

// The same thresholds from distance histograms (round 6): Hamming distances are
// integers in [0, max_dist], and thr[g] needs only the R-th smallest DISTANCE of
// ranges 0..g-1, not their keys.  (A) wave w counts its block's list entries
// into its own LDS histogram; (B) each bin becomes the exclusive prefix over
// the blocks (the counts of every range before the wave's block); (C) wave w
// walks its block in order: v = the smallest bin whose cumulative count
// reaches R (+inf while fewer than R), thr[g] = v, then list g's entries below
// v join the histogram and v steps down while the count at or below v - 1
// still reaches R.  The chain is the block's 16 lists, not ~3 x groups / 16
// key-list merges (emit_prefix_kernel: 114 us per query at 100M x 1536,
// profiles/r06/final/trace).  Identical thresholds: the R-th smallest
// distance of the prefix, +inf below R entries.
__global__ __launch_bounds__(PREFIX_WAVES * 64) void emit_prefix_hist_kernel(const uint64_t *partials, uint32_t groups,
                                                                             uint32_t k, uint32_t nbins, float *thr)
{
    extern __shared__ uint32_t hist[];  // [PREFIX_WAVES][nbins]
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t qi = blockIdx.x;
    const uint64_t *pq = partials + (size_t)qi * groups * k;
    const uint32_t per = (groups + PREFIX_WAVES - 1) / PREFIX_WAVES;
    const uint32_t g0 = min(groups, (uint32_t)wave * per), g1 = min(groups, g0 + per);
    for (uint32_t i = threadIdx.x; i < PREFIX_WAVES * nbins; i += PREFIX_WAVES * 64) hist[i] = 0u;
    __syncthreads();
    uint32_t *h = hist + (size_t)wave * nbins;
    auto bin_of = [&](uint64_t key) -> uint32_t {  // KEY_NONE -> nbins (no bin)
        if (key == WVG_KEY_NONE) return nbins;
        const float d = wvg_unord_f32((uint32_t)(key >> 32));
        return d >= 0.f && d < (float)nbins ? (uint32_t)d : nbins;
    };
    // the block's lists as bins in registers when it has at most 16 (one range per CU:
    // 256 ranges = 16 per wave), all loads issued at once; larger blocks read them twice
    constexpr int CL = 16;
    const uint32_t nl = g1 - g0;
    const bool cached = nl <= (uint32_t)CL && k <= 256;
    uint32_t rb[CL][4];
    if (cached) {
#pragma unroll
        for (int L = 0; L < CL; L++)
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const uint32_t i = (uint32_t)lane + 64u * (uint32_t)j;
                rb[L][j] = ((uint32_t)L < nl && i < k) ? bin_of(pq[(size_t)(g0 + L) * k + i]) : nbins;
            }
#pragma unroll
        for (int L = 0; L < CL; L++)  // (A)
#pragma unroll
            for (int j = 0; j < 4; j++)
                if (rb[L][j] < nbins) atomicAdd(&h[rb[L][j]], 1u);
    } else {
        for (uint32_t g = g0; g < g1; g++)  // (A)
            for (uint32_t i = (uint32_t)lane; i < k; i += 64) {
                const uint32_t b = bin_of(pq[(size_t)g * k + i]);
                if (b < nbins) atomicAdd(&h[b], 1u);
            }
    }
    __syncthreads();
    for (uint32_t b = threadIdx.x; b < nbins; b += PREFIX_WAVES * 64) {  // (B)
        uint32_t run = 0;
        for (int w = 0; w < PREFIX_WAVES; w++) {
            const uint32_t c = hist[(size_t)w * nbins + b];
            hist[(size_t)w * nbins + b] = run;
            run += c;
        }
    }
    __syncthreads();
    // (C) v = the smallest bin whose cumulative count reaches k (nbins: none yet); cnt = the
    // count at or below v (while v = nbins: every entry counted so far)
    uint32_t v = nbins, cnt = 0;
    auto find_v = [&]() {  // the first bin with cumulative count >= k, from scratch (wave-wide)
        uint32_t base = 0;
        v = nbins;
        for (uint32_t b0 = 0; b0 < nbins; b0 += 64) {
            const uint32_t b = b0 + (uint32_t)lane;
            uint32_t c = b < nbins ? h[b] : 0u;
#pragma unroll
            for (int off = 1; off < 64; off <<= 1) {  // inclusive prefix sum over the 64 lanes
                const uint32_t o = (uint32_t)__shfl_up((int)c, off, 64);
                if (lane >= off) c += o;
            }
            const uint64_t hit = __ballot(base + c >= k);
            if (hit) {
                const int l = __builtin_ctzll(hit);
                v = b0 + (uint32_t)l;
                cnt = base + (uint32_t)__shfl((int)c, l, 64);
                return;
            }
            base += (uint32_t)__shfl((int)c, 63, 64);
        }
        cnt = base;
    };
    find_v();
    auto step = [&](uint32_t g, auto &&bin_at) {  // thr[g], then range g's entries below v join
        if (lane == 0) thr[(size_t)qi * groups + g] = v < nbins ? (float)v : __builtin_inff();
        uint32_t added = 0;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const uint32_t b = bin_at(j);
            const bool take = b < v;  // (v = nbins: every entry)
            if (take) atomicAdd(&h[b], 1u);
            added += (uint32_t)__popcll(__ballot(take));
        }
        __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): the wave's atomics landed
        __builtin_amdgcn_wave_barrier();
        if (v == nbins) {
            if (cnt + added >= k) find_v();
            else cnt += added;
        } else {
            cnt += added;
            while (v > 0 && cnt - h[v] >= k) {  // (uniform: every lane reads the same words)
                cnt -= h[v];
                --v;
            }
        }
    };
    if (cached) {
#pragma unroll
        for (int L = 0; L < CL; L++)
            if ((uint32_t)L < nl) step(g0 + (uint32_t)L, [&](int j) { return rb[L][j]; });
    } else {
        for (uint32_t g = g0; g < g1; g++)
            step(g, [&](int j) {
                const uint32_t i = (uint32_t)lane + 64u * (uint32_t)j;
                return i < k ? bin_of(pq[(size_t)g * k + i]) : nbins;
            });
    }
}

hipError_t launch_emit_prefix(const uint64_t *partials, uint32_t nq, uint32_t groups, uint32_t k, float *thr,
                              hipStream_t s, uint32_t max_dist)
{
    if (nq == 0 || groups == 0 || k == 0 || k > 256) return hipSuccess;
    const dim3 grid(nq), block(PREFIX_WAVES * 64);
    const uint32_t nbins = max_dist + 1;
    const size_t lds = (size_t)PREFIX_WAVES * nbins * 4;
    if (max_dist > 0 && lds <= (size_t)(120u << 10)) {
        static const bool attr = hipFuncSetAttribute(reinterpret_cast<const void *>(&emit_prefix_hist_kernel),
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, 120 << 10) == hipSuccess;
        (void)attr;
        hipLaunchKernelGGL(emit_prefix_hist_kernel, grid, block, lds, s, partials, groups, k, nbins, thr);
        return hipGetLastError();
    }
    if (k <= 64)
        hipLaunchKernelGGL(emit_prefix_kernel<1>, grid, block, 0, s, partials, groups, k, thr);
    else if (k <= 128)
        hipLaunchKernelGGL(emit_prefix_kernel<2>, grid, block, 0, s, partials, groups, k, thr);
    else
        hipLaunchKernelGGL(emit_prefix_kernel<4>, grid, block, 0, s, partials, groups, k, thr);
    return hipGetLastError();
}

// One wave per emitting wave: keep the keys with distance < thr of its range,
// compacted in place (a chunk is read whole before any of it is overwritten,
// and writes never pass the read position).
__global__ __launch_bounds__(256) void emit_filter_kernel(uint64_t *emit, const uint32_t *emit_cnt, uint32_t cap,
                                                          const float *thr, uint32_t groups, uint32_t wpg,
                                                          uint32_t *fcnt, uint32_t *oflow)
{
    const int lane = threadIdx.x & 63;
    const uint32_t waves = groups * wpg;
    const uint32_t w = blockIdx.x * 4 + (threadIdx.x >> 6), qi = blockIdx.y;
    if (w >= waves) return;
    const size_t src = (size_t)qi * waves + w;
    const uint32_t cnt = emit_cnt[src], n = min(cnt, cap);
    const float tv = thr[(size_t)qi * groups + w / wpg];
    uint64_t *buf = emit + src * cap;
    uint32_t out = 0;
    for (uint32_t i = 0; i < n; i += 64) {
        const uint64_t key = i + lane < n ? buf[i + lane] : WVG_KEY_NONE;
        const bool keep = key != WVG_KEY_NONE && key_dist(key) < tv;
        const uint64_t m = __ballot(keep);
        const uint32_t pos = out + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
        if (keep) buf[pos] = key;
        out += (uint32_t)__popcll(m);
    }
    if (lane == 0) {
        fcnt[src] = out;
        if (cnt > cap) oflow[qi] = 1u;
    }
}

hipError_t launch_emit_filter(uint64_t *emit, const uint32_t *emit_cnt, uint32_t emit_cap, const float *thr,
                              uint32_t nq, uint32_t groups, uint32_t waves_per_group, uint32_t *fcnt, uint32_t *oflow,
                              hipStream_t s)
{
    const uint32_t waves = groups * waves_per_group;
    if (nq == 0 || waves == 0) return hipSuccess;
    hipLaunchKernelGGL(emit_filter_kernel, dim3((waves + 3) / 4, nq), dim3(256), 0, s, emit, emit_cnt, emit_cap, thr,
                       groups, waves_per_group, fcnt, oflow);
    return hipGetLastError();
}

// One wave per emitting wave: its offset is the sum of the earlier waves'
// kept counts (<= a few thousand words, read from L2), then a coalesced copy.
__global__ __launch_bounds__(256) void emit_gather_kernel(const uint64_t *emit, const uint32_t *fcnt, uint32_t cap,
                                                          uint32_t waves, uint64_t *out, uint32_t out_cap,
                                                          uint32_t *totals)
{
    const int lane = threadIdx.x & 63;
    const uint32_t w = blockIdx.x * 4 + (threadIdx.x >> 6), qi = blockIdx.y;
    if (w >= waves) return;
    const uint32_t *fc = fcnt + (size_t)qi * waves;
    uint32_t part = 0;
    for (uint32_t v = (uint32_t)lane; v < w; v += 64) part += fc[v];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) part += __shfl_xor(part, off, 64);
    const uint32_t base = part, n = fc[w];
    const uint64_t *src = emit + ((size_t)qi * waves + w) * cap;
    uint64_t *dst = out + (size_t)qi * out_cap;
    for (uint32_t i = (uint32_t)lane; i < n; i += 64)
        if (base + i < out_cap) dst[base + i] = src[i];
    if (w == waves - 1 && lane == 0) totals[qi] = base + n;
}

hipError_t launch_emit_gather(const uint64_t *emit, const uint32_t *fcnt, uint32_t emit_cap, uint32_t nq,
                              uint32_t waves, uint64_t *out, uint32_t out_cap, uint32_t *totals, hipStream_t s)
{
    if (nq == 0 || waves == 0) return hipSuccess;
    hipLaunchKernelGGL(emit_gather_kernel, dim3((waves + 3) / 4, nq), dim3(256), 0, s, emit, fcnt, emit_cap, waves,
                       out, out_cap, totals);
    return hipGetLastError();
}

// ---- host ---------------------------------------------------------------------

namespace {

constexpr uint32_t REPLAY_OUT_CAP = 65536;  // kept rows per query held on the device (more: the rerun)
constexpr uint32_t REPLAY_HEAD = 4096;      // kept rows per query copied back with the totals

// Per-wave record buffer.  On a random docID order the wave-local filter
// keeps about R (1 + ln(n / R)) of a wave's n rows (~1.4k of 98k at 100M x
// 1536, R = 200; a sum of independent Bernoulli(R / i), so its variance is
// at most its mean).  Fast mode records into LDS (no global store in the scan
// loop): as many keys as the LDS left by the workgroups sharing a CU holds,
// used when that is the wave's whole range or 6 standard deviations above the
// estimate; otherwise the keys go straight to HBM with twice the estimate.
// Either way a wave that overflows reruns its query (rerun_full).
struct EmitPlan {
    uint32_t cap = 0;
    bool lds = false;
};
EmitPlan emit_plan_for(uint64_t ntiles, int groups, uint32_t nq, uint32_t R, int num_cus)
{
    const uint32_t waves = (uint32_t)groups * BQ_SCAN_WAVES;
    const uint64_t rows = align_up((ntiles / std::max<uint32_t>(waves, 1) + 2) * 64, 64);
    const double est = (double)R * (1.0 + std::log(std::max(1.0, (double)rows / std::max<uint32_t>(R, 1))));
    const uint64_t wg_per_cu = std::max<uint64_t>(1, ((uint64_t)groups * nq + num_cus - 1) / num_cus);
    const size_t lds_wg = std::min<size_t>(BQ_EMIT_LDS_MAX, std::max<size_t>(16u << 10, (160u << 10) / wg_per_cu -
                                                                                            (16u << 10)));
    const uint64_t lcap = std::min<uint64_t>(rows, lds_wg / (BQ_SCAN_WAVES * 8) / 64 * 64);
    EmitPlan e;
    if (lcap >= rows || (double)lcap >= est + 6.0 * std::sqrt(est) + 64) {  // the count's variance <= its mean
        e.cap = (uint32_t)lcap;
        e.lds = true;
        return e;
    }
    e.cap = (uint32_t)std::min<uint64_t>(rows, align_up((uint64_t)(2.0 * est) + 256, 64));
    return e;
}

struct ReplayWs {
    size_t part = 0, emit = 0, ecnt = 0, thr = 0, fcnt = 0, out = 0, tot = 0, total = 0;
};

ReplayWs replay_ws(uint32_t nq, uint32_t groups, uint32_t R, uint32_t cap, uint32_t out_cap)
{
    ReplayWs w;
    Carver cv;
    const size_t waves = (size_t)groups * BQ_SCAN_WAVES;
    w.part = cv.take((size_t)nq * groups * R * 8);
    w.emit = cv.take((size_t)nq * waves * cap * 8);
    w.ecnt = cv.take((size_t)nq * waves * 4);
    w.thr = cv.take((size_t)nq * groups * 4);
    w.fcnt = cv.take((size_t)nq * waves * 4);
    w.out = cv.take((size_t)nq * out_cap * 8);
    w.tot = cv.take((size_t)nq * 8);  // totals [nq], then overflow flags [nq]
    w.total = cv.off;
    return w;
}

// The four device steps over ScanArgs `a` (queries, allow window, k = R set),
// into `ws` laid out by `w`; no host synchronization.
int run_emit(wvg_ctx *ctx, const ScanArgs &a0, int groups, uint32_t cap, bool lds, uint32_t out_cap, char *ws,
             const ReplayWs &w, const float *seed, hipStream_t s)
{
    ScanArgs a = a0;
    a.emit = (uint64_t *)(ws + w.emit);
    a.emit_cnt = (uint32_t *)(ws + w.ecnt);
    a.emit_cap = cap;
    a.emit_seed = seed;
    const uint32_t nq = a.nq, R = a.k, waves = (uint32_t)groups * BQ_SCAN_WAVES;
    uint32_t *tot = (uint32_t *)(ws + w.tot);
    WVG_HIP(hipMemsetAsync(tot, 0, (size_t)nq * 8, s));
    uint64_t *part = (uint64_t *)(ws + w.part);
    {
        ProfArm arm(ctx);  // wvg_profile_*: the scan dispatch's own events
        if (arm.rc) return arm.rc;
        WVG_HIP(launch_scan_bq_emit(a, part, groups, lds, s));
    }
    WVG_HIP(launch_emit_prefix(part, nq, (uint32_t)groups, R, (float *)(ws + w.thr), s, 128u * a.nchunks));
    WVG_HIP(launch_emit_filter(a.emit, a.emit_cnt, cap, (const float *)(ws + w.thr), nq, (uint32_t)groups,
                               BQ_SCAN_WAVES, (uint32_t *)(ws + w.fcnt), tot + nq, s));
    WVG_HIP(launch_emit_gather(a.emit, (const uint32_t *)(ws + w.fcnt), cap, nq, waves, (uint64_t *)(ws + w.out),
                               out_cap, tot, s));
    return WVG_OK;
}

// The heap replay of one query's kept rows (ascending docID): findTopVectorsCached
// into a heap of R, then the pop loop of searchByVectorBQ (index.go:369-374).
void replay_pops(const uint64_t *keys, size_t n, uint32_t R, std::vector<GoItem> &pops)
{
    GoMaxHeap h(R);
    for (size_t i = 0; i < n; i++) {
        const uint64_t key = keys[i];
        insert_to_heap(h, R, (uint32_t)key, wvg_unord_f32((uint32_t)(key >> 32)));
    }
    pops.clear();
    pops.reserve(h.len());
    while (h.len()) pops.push_back(h.pop());
}

// One query again with buffers that cannot overflow (every row of a wave),
// seeded with the first pass's thresholds: its own device allocation (this
// path is for adversarial docID orders only).
int rerun_full(wvg_ctx *ctx, const ScanArgs &a0, int groups, const float *d_thr_q, hipStream_t s,
               std::vector<uint64_t> &keys)
{
    const uint64_t ntiles = a0.tile_end - a0.tile_begin;
    const uint32_t waves = (uint32_t)groups * BQ_SCAN_WAVES;
    const uint32_t cap = (uint32_t)align_up((ntiles / waves + 2) * 64, 64);
    const uint64_t out_cap64 = ntiles * 64;
    if (out_cap64 > 0xFFFFFFFFull) return fail(WVG_ERR_UNSUPPORTED, "heap replay rerun: corpus window too large");
    const uint32_t out_cap = (uint32_t)out_cap64;
    const ReplayWs w = replay_ws(1, (uint32_t)groups, a0.k, cap, out_cap);
    const size_t seed_off = align_up(w.total, 256);
    void *mem = nullptr;
    if (hipMalloc(&mem, seed_off + (size_t)groups * 4) != hipSuccess) {
        (void)hipGetLastError();
        return fail(WVG_ERR_NOMEM, "heap replay rerun: out of device memory");
    }
    char *ws = (char *)mem;
    int rc = WVG_OK;
    do {
        if (hipMemcpyAsync(ws + seed_off, d_thr_q, (size_t)groups * 4, hipMemcpyDeviceToDevice, s) != hipSuccess) {
            rc = fail(WVG_ERR_DEVICE, "heap replay rerun: seed copy");
            break;
        }
        ScanArgs a = a0;
        a.nq = 1;
        a.cosched = 0;  // same groups, so the same ranges as the first pass
        rc = run_emit(ctx, a, groups, cap, false, out_cap, ws, w, (const float *)(ws + seed_off), s);
        if (rc) break;
        uint32_t tot[2] = {0, 0};
        if (hipMemcpyAsync(tot, ws + w.tot, 8, hipMemcpyDeviceToHost, s) != hipSuccess ||
            hipStreamSynchronize(s) != hipSuccess) {
            rc = fail(WVG_ERR_DEVICE, "heap replay rerun: totals");
            break;
        }
        if (tot[1] || tot[0] > out_cap) {
            rc = fail(WVG_ERR_DEVICE, "heap replay rerun overflowed");
            break;
        }
        keys.resize(tot[0]);
        if (tot[0] && (hipMemcpyAsync(keys.data(), ws + w.out, (size_t)tot[0] * 8, hipMemcpyDeviceToHost, s) !=
                           hipSuccess ||
                       hipStreamSynchronize(s) != hipSuccess)) {
            rc = fail(WVG_ERR_DEVICE, "heap replay rerun: keys");
            break;
        }
    } while (0);
    (void)hipStreamSynchronize(s);
    (void)hipFree(mem);
    return rc;
}

// The recording scan's grid: one 4-wave workgroup per CU for a lone query (the
// plain K5 scan runs three, which would leave each wave too little LDS for its
// records); a batch keeps the co-scheduled grid of the plan.
int replay_groups(const wvg_corpus *bq, uint32_t nq, const SearchPlan &p)
{
    if (nq != 1) return p.groups;
    return (int)std::min<uint64_t>((uint64_t)bq->ctx->num_cus, std::max<uint64_t>(1, (p.te - p.tb + 7) / 8));
}

}  // namespace

size_t replay_workspace_bytes(const wvg_corpus *bq, uint32_t nq, uint32_t R, const SearchPlan &p)
{
    const int groups = replay_groups(bq, nq, p);
    const EmitPlan e = emit_plan_for(p.te - p.tb, groups, nq, R, bq->ctx->num_cus);
    return replay_ws(nq, (uint32_t)groups, R, e.cap, REPLAY_OUT_CAP).total;
}

int bq_heap_candidates(wvg_corpus *bq, StreamSlot *sl, const void *d_qb, uint32_t qpb, uint32_t nq, uint32_t R,
                       const uint64_t *d_allow, const SearchPlan &p, char *ws, std::vector<std::vector<GoItem>> &pops)
{
    hipStream_t s = sl->stream;
    const int groups = replay_groups(bq, nq, p);
    const EmitPlan e = emit_plan_for(p.te - p.tb, groups, nq, R, bq->ctx->num_cus);
    const ReplayWs w = replay_ws(nq, (uint32_t)groups, R, e.cap, REPLAY_OUT_CAP);
    ScanArgs a{};
    a.data = bq->d_data;
    a.valid = bq->d_valid;
    a.allow = d_allow;
    a.allow_words = d_allow ? p.te - p.tb : 0;
    a.allow_t0 = p.tb;
    a.id_base = bq->id_base;
    a.tile_begin = p.tb;
    a.tile_end = p.te;
    a.dim = bq->dim;
    a.nchunks = bq->nchunks;
    a.metric = bq->metric;
    a.queries = d_qb;
    a.qpitch = qpb;
    a.nq = nq;
    a.k = R;
    a.cosched = p.cosched;
    int rc = run_emit(bq->ctx, a, groups, e.cap, e.lds, REPLAY_OUT_CAP, ws, w, nullptr, s);
    if (rc) return rc;
    // totals, overflow flags and the first REPLAY_HEAD kept rows of every query in one round trip
    const uint32_t head = REPLAY_HEAD;
    const size_t tot_b = (size_t)nq * 8, head_b = (size_t)nq * head * 8;
    Staging st;
    rc = st.reserve(sl, stage_bytes(tot_b) + stage_bytes(head_b));
    if (rc) return rc;
    std::vector<char> big(head_b > STAGE_MAX ? head_b : 0);
    char *pin_tot = st.take(tot_b);
    char *pin_head = head_b <= STAGE_MAX ? st.take(head_b) : big.data();
    WVG_HIP(hipMemcpyAsync(pin_tot, ws + w.tot, tot_b, hipMemcpyDeviceToHost, s));
    WVG_HIP(hipMemcpy2DAsync(pin_head, (size_t)head * 8, ws + w.out, (size_t)REPLAY_OUT_CAP * 8, (size_t)head * 8, nq,
                             hipMemcpyDeviceToHost, s));
    WVG_HIP(hipStreamSynchronize(s));
    const uint32_t *tot = (const uint32_t *)pin_tot, *oflow = tot + nq;
    pops.assign(nq, {});
    std::vector<uint64_t> keys;
    for (uint32_t q = 0; q < nq; q++) {
        const uint64_t *qk = (const uint64_t *)pin_head + (size_t)q * head;
        size_t n = tot[q];
        if (oflow[q] || n > REPLAY_OUT_CAP) {
            ScanArgs aq = a;
            aq.queries = (const uint64_t *)d_qb + (size_t)q * qpb;
            aq.allow = d_allow;  // filtered batches use one shared window (no per-query stride here)
            rc = rerun_full(bq->ctx, aq, groups, (const float *)(ws + w.thr) + (size_t)q * groups, s, keys);
            if (rc) return rc;
            qk = keys.data();
            n = keys.size();
        } else if (n > head) {
            keys.resize(n);
            WVG_HIP(hipMemcpyAsync(keys.data(), ws + w.out + (size_t)q * REPLAY_OUT_CAP * 8, n * 8,
                                   hipMemcpyDeviceToHost, s));
            WVG_HIP(hipStreamSynchronize(s));
            qk = keys.data();
        }
        replay_pops(qk, n, R, pops[q]);
    }
    return WVG_OK;
}

int bq_rescore_replay(wvg_corpus *bq, wvg_corpus *f32, const float *queries, uint32_t nq, uint32_t k, uint32_t R,
                      const SearchPlan &p, uint64_t *out_ids, float *out_dists, uint32_t *out_counts)
{
    SlotGuard g(bq->ctx);
    int rc = bq->ctx->acquire(&g.slot);
    if (rc) return rc;
    const uint32_t d = bq->dim;
    const uint32_t fpitch = f32_chunks(d) * 4;
    Carver cv;
    const size_t o_qb = cv.take(query_bytes(bq, nq));
    const size_t o_qf = cv.take(f32 ? (size_t)nq * fpitch * 4 : 0);
    const size_t o_allow = cv.take(p.allow_bytes());
    const bool large = R > MAX_K;  // beyond the scan's register top-k: the select-based superset
    const size_t o_rep = cv.take(large ? select_replay_bytes(p) : replay_workspace_bytes(bq, nq, R, p));
    const size_t o_cand = cv.take(f32 ? (size_t)nq * R * 8 : 0);
    const size_t o_resc = cv.take(f32 ? (size_t)nq * R * 8 : 0);
    void *base = nullptr;
    rc = g.slot->device_scratch(cv.off, &base);
    if (rc) return rc;
    char *b = (char *)base;
    hipStream_t s = g.slot->stream;
    uint32_t qpb = 0, qpf = 0;
    rc = stage_queries(bq, g.slot, queries, nq, b + o_qb, qpb, nullptr, nullptr);
    if (rc) return rc;
    if (f32) {
        rc = stage_queries(f32, g.slot, queries, nq, b + o_qf, qpf, nullptr, nullptr);
        if (rc) return rc;
    }
    const uint64_t *d_allow = nullptr;
    if (p.allow_host) {
        WVG_HIP(hipMemcpyAsync(b + o_allow, p.allow_host, p.allow_bytes(), hipMemcpyHostToDevice, s));
        d_allow = (const uint64_t *)(b + o_allow);
    }
    std::vector<std::vector<GoItem>> pops;
    rc = large ? bq_heap_candidates_select(bq, g.slot, b + o_qb, qpb, nq, R, d_allow, p, b + o_rep, pops)
               : bq_heap_candidates(bq, g.slot, b + o_qb, qpb, nq, R, d_allow, p, b + o_rep, pops);
    if (rc) return rc;
    if (!f32) {  // the candidates themselves, in pop order
        for (uint32_t q = 0; q < nq; q++) {
            const std::vector<GoItem> &v = pops[q];
            for (uint32_t i = 0; i < R; i++) {
                const bool has = i < v.size();
                if (out_ids) out_ids[(size_t)q * R + i] = has ? bq->id_base + v[i].id : WVG_KEY_NONE;
                if (out_dists) out_dists[(size_t)q * R + i] = has ? v[i].dist : INFINITY;
            }
            if (out_counts) out_counts[q] = (uint32_t)v.size();
        }
        return WVG_OK;
    }
    // the rescore loop (index.go:368-385): exact distances of the popped ids on the
    // device, inserted into a heap of k in pop order on the host
    const size_t ck_b = (size_t)nq * R * 8;
    std::vector<uint64_t> ck((size_t)nq * R, WVG_KEY_NONE);
    for (uint32_t q = 0; q < nq; q++)
        for (size_t i = 0; i < pops[q].size(); i++) ck[(size_t)q * R + i] = pops[q][i].id;
    Staging st;
    rc = st.reserve(g.slot, stage_bytes(ck_b) * 2);
    if (rc) return rc;
    WVG_HIP(st.h2d(b + o_cand, ck.data(), ck_b, s));
    WVG_HIP(launch_rescore_keys(f32->metric, (const float *)(b + o_qf), qpf, (const float *)f32->d_data, d,
                                f32->nchunks, (const uint64_t *)(b + o_cand), nq, R, R, (uint64_t *)(b + o_resc), s,
                                f32->ctx->order512));
    std::vector<uint64_t> big(ck_b > STAGE_MAX ? (size_t)nq * R : 0);
    uint64_t *resc = ck_b <= STAGE_MAX ? (uint64_t *)st.take(ck_b) : big.data();
    WVG_HIP(hipMemcpyAsync(resc, b + o_resc, ck_b, hipMemcpyDeviceToHost, s));
    WVG_HIP(hipStreamSynchronize(s));
    std::vector<uint64_t> ids(k);
    std::vector<float> dists(k);
    for (uint32_t q = 0; q < nq; q++) {
        GoMaxHeap h(k);
        for (size_t i = 0; i < pops[q].size(); i++)
            insert_to_heap(h, k, bq->id_base + pops[q][i].id,
                           wvg_unord_f32((uint32_t)(resc[(size_t)q * R + i] >> 32)));
        const size_t cnt = extract_heap(h, ids.data(), dists.data());
        for (uint32_t i = 0; i < k; i++) {
            if (out_ids) out_ids[(size_t)q * k + i] = i < cnt ? ids[i] : WVG_KEY_NONE;
            if (out_dists) out_dists[(size_t)q * k + i] = i < cnt ? dists[i] : INFINITY;
        }
        if (out_counts) out_counts[q] = (uint32_t)cnt;
    }
    return WVG_OK;
}

}  // namespace wvg
