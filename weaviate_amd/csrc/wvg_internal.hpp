// wvg_internal.hpp -- host-side internals shared by the HIP translation units.
#pragma once

#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <mutex>
#include <shared_mutex>
#include <string>
#include <vector>

#include "../../include/wvgpu.h"
#include "wvg_common.hpp"

namespace wvg {

// thread-local last-error message (wvg_last_error)
void set_error(const std::string &msg);
int fail(int code, const std::string &msg);

#define WVG_HIP(expr)                                                                   \
    do {                                                                                \
        hipError_t _e = (expr);                                                         \
        if (_e != hipSuccess)                                                           \
            return ::wvg::fail(WVG_ERR_DEVICE, std::string(#expr ": ") + hipGetErrorString(_e)); \
    } while (0)

constexpr uint32_t SLOT_READY_OFF = 64;     // words
constexpr uint32_t SLOT_READY_MAX = 4032;   // lists (scan workgroups) of a single query with per-list hand-offs
// A pooled HIP stream with its own grow-only device scratch and pinned host
// staging, borrowed by one C-ABI call at a time (callers are many goroutines).
struct StreamSlot {
    hipStream_t stream = nullptr;
    void *dscratch = nullptr;
    size_t dscratch_bytes = 0;
    void *hpinned = nullptr;
    size_t hpinned_bytes = 0;
    // a single-query host search's in-launch merge: a persistent arrival counter
    // (and the merge's status word) on the device, and the count the next
    // launch starts from -- no per-call memset
    uint32_t *dctl = nullptr;
    uint32_t arrival_base = 0;
    uint32_t tag = 0;  // the slot's last single-query call tag (StreamJob::tag; never 0)
    // and its results: written by the merge workgroup straight into coherent
    // (uncached, fine-grained) host memory -- no device-to-host copy per call
    void *hcoh = nullptr;
    size_t hcoh_bytes = 0;
    int device_scratch(size_t bytes, void **out);
    int host_pinned(size_t bytes, void **out);
    int host_coherent(size_t bytes, void **out);
    int control(uint32_t **out);  // dctl, allocated and zeroed on first use: [0] arrivals, [1] status,
                                  // [SLOT_READY_OFF ..) the single query's per-list ready words
};

}  // namespace wvg

struct wvg_ctx {
    int device = 0;
    int num_cus = 256;
    wvg_options opt{};          // fixed at wvg_open / wvg_open_ex
    int order512 = 0;           // distancer kernels of an AMX + AVX-512 host (wvg_set_distance_order)
    std::mutex pool_mu;
    std::vector<wvg::StreamSlot *> free_slots;
    std::vector<wvg::StreamSlot *> all_slots;
    int acquire(wvg::StreamSlot **out);
    void release(wvg::StreamSlot *s);
    // profiling (wvg_profile_start/stop): event pairs around scan launches
    std::atomic<bool> profiling{false};
    std::mutex prof_mu;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> prof_events;
    size_t prof_used = 0;
};

// Concurrent single-query wvg_search calls on one corpus (one goroutine per
// Weaviate query) join one batched launch: a request queue, and at most one
// batch of it executing at a time (wvg_search.hip, search_coalesced).
struct wvg_search_request;
struct wvg_coalescer {
    std::mutex mu;
    std::condition_variable cv;
    std::condition_variable gather_cv;  // arrivals wake a runner that is gathering its batch
    std::deque<wvg_search_request *> pending;
    bool busy = false;       // a batch is executing (or its runner is gathering)
    bool gathering = false;
    size_t last_n = 0;       // requests of the last batch
    size_t carry = 0;        // requests that were waiting when it ended (not its own callers)
    std::chrono::steady_clock::time_point last_done{};
    std::chrono::nanoseconds last_run{0};
};

struct wvg_corpus {
    wvg_ctx *ctx = nullptr;
    int kind = WVG_KIND_F32;
    int metric = WVG_METRIC_L2;
    uint32_t dim = 0;       // vector dimensions
    uint32_t nchunks = 0;   // 16-byte chunks per row in the tiled layout
    uint64_t id_base = 0;   // global docID of slot 0 (multiple of 64)
    uint64_t capacity = 0;  // rows, multiple of 64
    uint64_t high_water = 0;
    uint64_t count = 0;
    void *d_data = nullptr;        // tiled rows
    uint64_t *d_valid = nullptr;   // one word per tile
    std::vector<uint64_t> h_valid; // host mirror of d_valid
    // PQ codebook (kind == PQ)
    float *d_centers = nullptr;    // [m][ks][ds]
    uint32_t pq_m = 0, pq_ks = 0, pq_ds = 0;
    bool pq_nan_free = false;      // the codebook has no NaN (launch_pq_encode)
    // K3c's bf16 shadow of an F32 dot / cosine corpus (wvg_screen.hip), built on
    // the first batched search that uses it and kept in step with later writes
    void *d_shadow = nullptr;      // [tiles + 4][screen_kblocks][4][64] 16-B bf16 fragments
    float *d_norms = nullptr;      // [(tiles + 4) * 64] row-norm upper bounds
    uint32_t *d_nmax = nullptr;    // {max of d_norms, max of d_errs (float bits), S, 1 / S (K3i's row scale)}
    float *d_errs = nullptr;       // K3i: [(tiles + 4) * 64] row quantization-error bounds
    bool sh_i8 = false;            // the shadow is K3i's int8 one (d_shadow: [tiles + 4][dim / 64][4][64] 16 B)
    uint64_t sh_dirty_lo = 0, sh_dirty_hi = 0;  // tiles written since the last build
    bool sh_failed = false;        // the shadow could not be allocated: batches stay on the exact path
    std::mutex sh_mu;              // builds (searches hold rw shared)
    hipEvent_t sh_ready = nullptr; // the last build, for searches on other streams
    std::shared_mutex rw;          // shared: search; exclusive: upsert/delete/grow
    std::atomic<uint64_t> scan_serial{0};  // query scans issued so far (parity = next scan direction)
    wvg_coalescer co;                      // single-query searches batched across callers
};

namespace wvg {

__host__ __device__ inline uint64_t tiles_of(uint64_t rows) { return (rows + WVG_TILE - 1) / WVG_TILE; }
__host__ __device__ inline uint32_t f32_chunks(uint32_t dim) { return (dim + 3) / 4; }
__host__ __device__ inline uint32_t bq_words(uint32_t dim) { return (dim + 63) / 64; }
__host__ __device__ inline uint32_t bq_chunks(uint32_t dim) { return (bq_words(dim) + 1) / 2; }
__host__ __device__ inline uint32_t pq_chunks(uint32_t m) { return (m + 15) / 16; }
// PQ corpora with m = 32 store each row's 32 codes rotated by its slot:
// stored byte b = code[(b + slot mod 32) mod 32].  K8b then reads the bytes
// it needs at step j straight from the stored words (no per-tile barrel
// shift); every other reader undoes the rotation with pq32_window.
__host__ __device__ inline bool pq_rotated(uint32_t m) { return m == 32; }
// Codebook buffers handed to launch_pq_encode: the [m][ks][ds] table and, for
// ds == 4 with even ks, the pair-interleaved copy [m][ks/2][4][2] right after
// it (pq_pair_layout) for the packed two-centroid encoder.
inline bool pq_has_pairs(uint32_t ks, uint32_t ds) { return ds == 4 && ks % 2 == 0; }
inline size_t pq_centers_alloc_bytes(uint32_t m, uint32_t ks, uint32_t ds)
{
    return (size_t)m * ks * ds * 4 * (pq_has_pairs(ks, ds) ? 2 : 1);
}
inline void pq_pair_layout(const float *centers, uint32_t m, uint32_t ks, float *out)
{
    for (uint32_t s = 0; s < m; s++)
        for (uint32_t p = 0; p < ks / 2; p++)
            for (uint32_t k = 0; k < 4; k++)
                for (uint32_t h = 0; h < 2; h++)
                    out[(((size_t)s * (ks / 2) + p) * 4 + k) * 2 + h] = centers[((size_t)s * ks + 2 * p + h) * 4 + k];
}
// out byte i = in byte (off + i) mod 32 (off per lane: v_cndmask stages + v_alignbyte)
__device__ __forceinline__ void pq32_window(const uint32_t (&in)[8], uint32_t off, uint32_t (&out)[8])
{
    uint32_t d[8];
#pragma unroll
    for (int i = 0; i < 8; i++) d[i] = in[i];
    const uint32_t q = (off >> 2) & 7u, r = off & 3u;
#pragma unroll
    for (int b = 0; b < 3; b++) {
        const bool sb = (q >> b) & 1u;
        uint32_t e[8];
#pragma unroll
        for (int i = 0; i < 8; i++) e[i] = sb ? d[(i + (1 << b)) & 7] : d[i];
#pragma unroll
        for (int i = 0; i < 8; i++) d[i] = e[i];
    }
#pragma unroll
    for (int w = 0; w < 8; w++) out[w] = __builtin_amdgcn_alignbyte(d[(w + 1) & 7], d[w], r);
}
// One row's ADC sum in segment order (CH/product_quantization.go:85-104) from
// its tiled code chunks (rp = chunk 0 of the row, chunks 64 uint4 apart), for
// the non-streaming readers (dist by id, unbounded selection, K8 generic).
__device__ __forceinline__ float pq_row_sum(const uint4 *rp, uint32_t nch, uint32_t m, uint32_t ks, const float *lut,
                                            uint64_t slot)
{
    float sum = 0.0f;
    if (pq_rotated(m)) {
        const uint4 lo = rp[0], hi = rp[64];
        const uint32_t w[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
        uint32_t o[8];
        pq32_window(w, (32u - (uint32_t)(slot & 31)) & 31u, o);
#pragma unroll
        for (int i = 0; i < 32; i++) sum = sum + lut[i * ks + ((o[i >> 2] >> (8 * (i & 3))) & 0xFFu)];
        return sum;
    }
    for (uint32_t c = 0; c < nch; c++) {
        const uint4 x = rp[(size_t)c * 64];
        const uint32_t ws[4] = {x.x, x.y, x.z, x.w};
        for (uint32_t b = 0; b < 16; b++) {
            const uint32_t s = c * 16 + b;
            if (s < m) sum = sum + lut[s * ks + ((ws[b >> 2] >> (8 * (b & 3))) & 0xFFu)];
        }
    }
    return sum;
}
size_t corpus_row_bytes(int kind, uint32_t dim, uint32_t pq_m);

// f(std::integral_constant<int, M>{}) for the kernel template metric M of a
// runtime metric: L2, MANHATTAN, HAMMING as themselves; dot and cosine share
// the raw dot product (DOT), the Wrap (-x / 1-x) is applied at run time.
template <int M>
struct MetricTag {
    static constexpr int value = M;
};
template <typename F>
inline auto with_metric(int metric, F &&f)
{
    switch (metric) {
    case WVG_M_L2: return f(MetricTag<WVG_M_L2>{});
    case WVG_M_MANHATTAN: return f(MetricTag<WVG_M_MANHATTAN>{});
    case WVG_M_HAMMING: return f(MetricTag<WVG_M_HAMMING>{});
    default: return f(MetricTag<WVG_M_DOT>{});
    }
}

// ---- kernel launchers (wvg_scan.hip / wvg_bq.hip / wvg_pq.hip) -----------
// Scan phase 1: per (query, workgroup) top-K keys into `partials`
//   [nq][groups][K].  Returns the number of groups used.
// A finished query's phase-2 merge, run by one extra workgroup of the next
// query's scan launch (inputs complete by stream order): the merge costs no
// launch of its own and overlaps the scan.
struct MergeJob {
    const uint64_t *partials;  // [nlists][list_len] ascending lists
    uint32_t nlists, list_len, k;
    uint64_t id_base;
    uint64_t *ids;
    float *dists;
    uint32_t *counts;
    int active;
};

struct ScanArgs {
    const void *data;          // tiled corpus
    const uint64_t *valid;     // one word per tile
    const uint64_t *allow;     // allow bitmap window, may be null: allow[i] masks tile allow_t0 + i
    uint64_t allow_words;      // tiles covered by the window (tiles outside it are not allowed)
    uint64_t allow_t0;
    uint64_t allow_qstride;    // K1: words between consecutive queries' windows (coalesced filtered
                               // single queries, each with its own allow list); 0 = one shared window
    uint64_t id_base;
    uint64_t tile_begin, tile_end;
    uint32_t dim, nchunks;
    int metric;
    const void *queries;       // F32: [nq][qpitch] floats; BQ: [nq][2*nchunks] u64; PQ: luts [nq][m*ks]
    uint32_t qpitch;           // elements per query in `queries`
    uint32_t nq, k;
    uint32_t pq_m, pq_ks;
    MergeJob side;             // F32 scan only; gridDim.x includes its workgroup
    uint32_t reverse;          // scan direction: 1 = every wave walks its tile range downwards.  The
                               // query-stream kernel alternates per query from this start, and the host
                               // alternates between calls (wvg_corpus::scan_serial): consecutive scans then
                               // begin where the previous one ended, on rows still in the Infinity Cache
    int dense;                 // PQ m = 32: no allow list and mostly-live rows -> K8c (no tile skipping)
    int cosched;               // PQ m = 32 dense, nq > 1: K8e with a 1D grid whose consecutive workgroups
                               // on one XCD are the nq queries of one row range (pq_cosched_groups)
    int order512;              // F32 distances in the AVX-512 kernels' order (wvg_set_distance_order)
    int plain;                 // F32 K1 row loads with the default cache policy instead of non-temporal
                               // (scanned bytes within a few x the Infinity Cache: plain_loads())
    uint32_t cache_tail256;    // K1 (A/B): if > 0, each wave reads the last cache_tail256/256 of its pass
                               // with the default policy and the rest non-temporal -- the serpentine's
                               // next pass starts on exactly those rows
    // Reference-heap replay (K5 EMIT, wvg_replay.hip): every wave also writes the
    // keys of the rows the reference's sequential heap could insert -- those
    // strictly below min(the wave's own running k-th distance, its range's
    // prefix seed) -- in docID order, [nq][groups * 4][emit_cap]; emit_cnt
    // [nq][groups * 4] holds each wave's full count (> emit_cap: overflowed).
    uint64_t *emit;
    uint32_t *emit_cnt;
    uint32_t emit_cap;
    const float *emit_seed;    // [nq][groups] thresholds (a rerun seeded from the first pass), or null
};
// Phase 1 writes dense partials [nq][groups][K] (keys, KEY_NONE = empty).
int scan_groups_for(const ScanArgs &a, int num_cus);
// Row ranges per query of a co-scheduled PQ batch: a multiple of 8 (XCDs) with
// ranges x nq ~ one workgroup per CU.
inline int pq_cosched_groups(uint32_t nq, int num_cus)
{
    const int g = num_cus / (int)(nq ? nq : 1) / 8;
    return 8 * (g > 0 ? g : 1);
}
hipError_t launch_scan_f32(const ScanArgs &a, uint64_t *partials, int groups, hipStream_t s);
// Query-stream K1 (wvg_search_device_pipelined): ONE launch scans a.nq queries
// back to back, every query a full scan of the corpus.  `groups` scan
// workgroups loop over the queries, publishing each query's partial list with
// a release + arrival count; one more workgroup waits for each query's
// `groups` arrivals and merges it while the scan proceeds to the next query.
// Sticky status word of a device-search workspace (its first bytes; read and
// cleared by wvg_search_device_check).
constexpr uint32_t WVG_STATUS_MERGE_TIMEOUT = 1u;
constexpr uint32_t WVG_RECORDS_TIMEOUT = 0xFFFFFFFFu;  // header count of a merge that gave up (StreamJob::records)
constexpr uint32_t STREAM_QIN_FLOATS = 256;  // a query of up to 256 dims (f32 chunks) inline in StreamJob
constexpr int SCAN_WAVES = 4;  // waves per K1 / query-stream scan workgroup
struct StreamJob {
    uint64_t *partials;  // [nq][groups][k]
    uint32_t *arrivals;  // [nq], arrival_base at launch
    uint32_t arrival_base;  // 0 for a zeroed workspace; a stream slot's running count otherwise
    uint32_t *status;    // WVG_STATUS_MERGE_TIMEOUT set if the merge workgroup gave up waiting
    uint64_t wait_limit; // merge workgroup's wait per query, s_memrealtime ticks (100 MHz)
    uint32_t groups;
    uint64_t *ids;
    float *dists;
    uint32_t *counts;
    // Single host queries: the results go to host memory as tagged 16-byte records
    // [nq][k + 1] (entries {slot, tag, dist, tag} -- the host adds id_base -- then the header {count, tag}),
    // ids / dists / counts unused.  GPU writes to host memory can become visible
    // out of order (a later header before earlier entries), so the host accepts a
    // result only when the header AND every entry carry its call's tag.
    uint4 *records;
    uint32_t tag;
    uint32_t legacy_poll;  // tools A/B: round 4's layout (ids / dists, a release, then the polled count)
    // per-list hand-off (instead of the arrival counter): scan workgroup g of query q
    // sc1-stores ready_tag + q into ready[q * groups + g] after its list; the merge
    // workgroup merges each list as soon as its word matches (merge_lists_ready)
    uint32_t *ready;
    uint32_t ready_tag;
    uint32_t row_split;    // row-granular wave ranges (scan_f32_stream_kernel)
    // a single host query rides in the kernel arguments (ScanArgs::queries null):
    // no host-to-device copy (a blit dispatch + ~10 us of API time) per call
    alignas(16) float qin[STREAM_QIN_FLOATS];
};
hipError_t launch_scan_f32_stream(const ScanArgs &a, const StreamJob &j, hipStream_t s);
// ids KEY_NONE, dists +inf, counts 0 for nq queries (empty corpus / slab).
hipError_t launch_fill_empty(uint64_t *ids, float *dists, uint32_t *counts, uint32_t nq, uint32_t k, hipStream_t s);
hipError_t launch_scan_bq(const ScanArgs &a, uint64_t *partials, int groups, hipStream_t s);
// K5 with the heap-replay emission (a.emit set; groups * BQ_SCAN_WAVES waves per query):
// lds = record into LDS (4 * emit_cap * 8 <= BQ_EMIT_LDS_MAX bytes), else straight to HBM.
constexpr int BQ_SCAN_WAVES = 4;
constexpr size_t BQ_EMIT_LDS_MAX = 128u << 10;
hipError_t launch_scan_bq_emit(const ScanArgs &a, uint64_t *partials, int groups, bool lds, hipStream_t s);
// Heap replay (wvg_replay.hip).  prefix: per query, thr[q][g] = the k-th smallest
// distance of ranges 0..g-1's lists (partials [nq][groups][k], ascending; +inf
// while fewer than k rows precede range g).  filter: each wave's emitted keys
// with distance < its range's thr, compacted in place (fcnt [nq][waves]; a wave
// whose count exceeded emit_cap sets oflow[q]).  gather: per query the kept keys
// of all waves in wave (= docID) order into out [nq][out_cap], totals [nq].
hipError_t launch_emit_prefix(const uint64_t *partials, uint32_t nq, uint32_t groups, uint32_t k, float *thr,
                              hipStream_t s, uint32_t max_dist = 0);  // max_dist > 0: integer distances <= it
hipError_t launch_emit_filter(uint64_t *emit, const uint32_t *emit_cnt, uint32_t emit_cap, const float *thr,
                              uint32_t nq, uint32_t groups, uint32_t waves_per_group, uint32_t *fcnt, uint32_t *oflow,
                              hipStream_t s);
hipError_t launch_emit_gather(const uint64_t *emit, const uint32_t *fcnt, uint32_t emit_cap, uint32_t nq,
                              uint32_t waves, uint64_t *out, uint32_t out_cap, uint32_t *totals, hipStream_t s);
hipError_t launch_scan_pq(const ScanArgs &a, uint64_t *partials, int groups, hipStream_t s);
// The exact K1 rescan of a device-resident query list (qlist[0 .. *nlist)),
// `slots` queries in flight: partials [f][groups][k]; and its merge.
hipError_t launch_scan_f32_qlist(const ScanArgs &a, uint64_t *partials, int groups, const uint32_t *qlist,
                                 const uint32_t *nlist, uint32_t slots, hipStream_t s);
hipError_t launch_merge_lists_qlist(const uint64_t *partials, uint32_t nq, uint32_t nlists, uint32_t list_len,
                                    uint32_t k, uint64_t id_base, uint64_t *ids, float *dists, uint32_t *counts,
                                    const uint32_t *qlist, const uint32_t *nlist, hipStream_t s);
// K3c bf16 MFMA screen + exact rescore (wvg_screen.hip).
constexpr int SCREEN_M = 16;  // lower bounds kept per (wave, query) and per (row range, query)
inline uint32_t screen_kblocks(uint32_t dim) { return (dim + 63) / 64 * 2; }
bool screen_supported(uint32_t dim, int metric, uint32_t k);
uint32_t screen_row_ranges(uint32_t nq, uint64_t ntiles, int num_cus);
#ifdef WVG_TOOLS
void screen_counters(uint64_t out[4], bool reset);
void single_counters(uint64_t out[4], bool reset);
void coalesce_counters(uint64_t out[4], bool reset);
void single_timing_read(uint64_t out[5], bool reset);
void filtered_timing_read(uint64_t out[5], bool reset);
#endif
hipError_t launch_shadow_build(const float *tiled, uint32_t dim, uint64_t t0, uint64_t t1, void *shadow, float *norms,
                               uint32_t *nmax, hipStream_t s);
// K3i (the int8 screen): dims it runs, the corpus scale's pass (largest finite
// |x| of tiles [0, tiles) as float bits into *out) and the shadow build
// (mx = {max norm, max error, S, 1 / S})
inline bool screen_i8_supported(uint32_t dim) { return dim == 512 || dim == 768 || dim == 1024; }
hipError_t launch_shadow_maxabs(const float *tiled, uint32_t dim, uint64_t tiles, uint32_t *out, hipStream_t s);
hipError_t launch_shadow_build_i8(const float *tiled, uint32_t dim, uint64_t t0, uint64_t t1, void *shadow,
                                  float *norms, float *errs, uint32_t *mx, hipStream_t s);
struct ScreenLaunch {
    const void *shadow;
    const float *norms;
    const uint32_t *nmax;
    const uint64_t *valid;
    const uint64_t *allow;
    uint64_t allow_words, allow_t0;
    uint64_t tile_begin, tile_end;
    uint32_t dim;
    const float *queries;  // [nq][qpitch] (normalized for cosine)
    uint32_t qpitch, nq, k, nrr;
    int cosine;
    int num_cus;           // sizes the split screen's first launch
    void *qfrag;           // [nq_pad / 16][kblocks][64] x 16 B
    float *k1, *k2, *emax; // [nq_pad]
    // K3i (int8 shadow): the rows' error bounds, the corpus scale ({.., .., S, 1 / S}
    // after the two maxima in nmax's words) and per-query B, score scale, 1 / Sq
    bool i8 = false;
    const float *errs = nullptr;
    float *kb = nullptr, *css = nullptr, *qinv = nullptr;  // [nq_pad]
    uint32_t *gbound;      // [nq]
    uint64_t *partials;    // [nq][nrr][SCREEN_M]
    uint64_t *cand;        // [nq][nrr * SCREEN_M]
    uint32_t *flist;       // [nq] flagged queries
    uint32_t *nflag;       // count
    // exact seeds (optional): the rows and distance the final rescore uses
    int metric = 0;
    const float *data = nullptr;  // tiled fp32 rows
    uint32_t nchunks = 0;
    // pilot (optional): the exact K1 top-k of every query over the range's
    // first tiles seeds the bound before the first phase
    const ScanArgs *pilot = nullptr;
    uint64_t *pilot_part = nullptr;  // [nq][pilot_groups][k] K1 partials ([nq][rr][k] K3b partials)
    uint32_t pilot_groups = 1;
    uint32_t pilot_part_lists = 0;   // pilot_part's capacity in k-lists per query
    uint64_t *pilot_ids = nullptr;   // [nq][k] scratch (the caller's result arrays)
    float *pilot_dists = nullptr;
    uint32_t *pilot_counts = nullptr;
};
// screen + collect (the rescore, merge and rescan are launched by the host)
hipError_t launch_screen(const ScreenLaunch &L, hipStream_t s);
// K3 batched MFMA scoring (wvg_gemm.hip): partials [nq][nrr][K].
bool gemm_supported(uint32_t dim, int metric);
uint32_t gemm_row_ranges(uint32_t nq, uint64_t ntiles, int num_cus, uint32_t dim, uint32_t k);
// prog: [nrr][query blocks] u32 workspace (zeroed here) for K3b's soft lockstep;
// gbound: [nq] u32 workspace (set to 0xFF.. here) for K3b's per-query distance bounds.
hipError_t launch_gemm_topk(const ScanArgs &a, uint32_t nrr, uint64_t *partials, uint32_t *prog, uint32_t *gbound,
                            int num_cus, hipStream_t s);
// A/B knobs of the tools build (make -C weaviate_amd/csrc tools ->
// tools/libwvgpu_tools.so, -DWVG_TOOLS, which exports wvgx_set_tuning and
// compiles the tuning / diagnostic kernel variants).  In the product library
// tuning() is a constant holding these defaults: nothing here can change at
// run time, and every per-deployment choice is a context option (wvg_options).
struct Tuning {
    int scan_variant = 0;    // K1 variant (see wvg_scan.hip)
    int groups_per_cu = 0;   // K1 workgroups per CU; 0 = auto by row size (scan_groups_for)
    int gemm_pf = 0;         // K3 register prefetch depth: 0 = by top-k size (2 for k <= 64), 1 = force 1
    int gemm_kernel = 0;     // K3 variant: 0 = K3b (queries resident, rows streamed; 2 waves per SIMD)
                             // where it applies, 2 = K3b with 2 query tiles per wave, 1 = K3
    int gemm_lockstep = 0;   // K3b soft lockstep of the workgroups sharing a row range:
                             // allowed lead in tiles, 0 = off (A/B)
    int gemm_skew = 0;       // K3b two-waves-per-SIMD: start delay of the second query half (x ~512 cycles)
    int pipeline_mode = 1;   // wvg_search_device_pipelined: 0 = one launch per query (merge folded into the
                             // next launch), 1 = one query-stream launch
    int pq_variant = 0;      // K8: 0 = rotated-segment ADC (K8b) where it applies (m = 32, ks = 256),
                             // 1 = K8 gather in segment order everywhere
    int merge_wait_us = 0;   // query-stream merge workgroup's wait per query in us; 0 = 4 s (test knob)
    int serpentine = 1;      // alternate the scan direction between consecutive scans (0 = always upwards; A/B)
    int k1_loads = 0;        // K1 row-load policy: 0 = by scanned bytes (plain_loads), 1 = non-temporal,
                             // 2 = default policy (A/B)
    int gemm_range_tiles = 0;  // K3b row-range length in tiles: 0 = auto (512), > 0 = that many,
                               // -1 = one long range per workgroup (one wave of workgroups; A/B)
    int gemm_pairing = 0;    // K3b QH = 2: SIMD partners share rows (0) or queries (1) (A/B)
    int gemm_prio = 0;       // K3b: s_setprio 1 for the second wave of each SIMD (A/B)
    int pq_cosched = 1;      // PQ / BQ batches (nq > 1): co-scheduled K8e / K5 (1) or one range set per
                             // query (0; A/B)
    int bq_cos_gpc = 2;      // co-scheduled K5: 4-wave workgroups per CU (2: 1.01 ms per query of an 8-query
                             // 100M x 1536 batch; 1: 1.49, 4: 1.34; A/B)
    int k1_tail = 0;         // K1 cache_tail256: 0 = auto (k1_cache_tail), -1 = off (plain_loads() policy
                             // for the whole pass), 1..256 = forced (A/B; env WVG_K1_TAIL)
    int pq_encode_min3 = 1;  // PQ encode pair path: min3 argmin on NaN-free codebooks (1) or the
                             // reference's compare-and-select loop everywhere (0; A/B and parity)
    int screen_pilot = 16;   // K3c/K3d: tiles of the exact pilot scan that seeds the bound (0 = none; A/B)
    int screen_pilot_gemm = 512;  // K3c/K3d: tiles of the K3b (exact fp32 MFMA) pilot, which replaces the K1
                                  // pilot (0 = the K1 pilot; A/B)
    int screen_round = 1;    // screen row ranges (tuning key 33): 1 = nrr * query blocks a multiple of the CUs
    int screen_pilot_gemm_i8 = 256;  // the same for K3i (tuning key 32): with its warm-up ranges half the
                                     // pilot is ~1 % faster per batch (profiles/r06/screen_i8/pilot_tiles_ab*.jsonl)
    int screen_variant = 0;  // batched screen kernel: 0 = K3d where it applies (d = 512, 768), 1 = K3c,
                             // 2 = K3e (K3d with 32x32x16 MFMAs), 3 = K3f (two waves per SIMD); 2 and 3
                             // exist in the tools build only (profiles/r05/k3e, k3f)
    int stream_variant = 1;  // query-stream K1 (tuning key 25): bit 0 = tile-granular wave ranges (the default:
                             // row-granular ranges let every wave touch one more, shared tile, and a wave's time
                             // follows its tile count -- 85.1 vs 82.5 us per 1M-row query, profiles/r05/stream_ab/),
                             // bit 1 = the arrival-counter merge after all lists (round 4) instead of the per-list
                             // hand-offs (83.7 vs 82.5 us)
    int single_path = 0;     // single-query host calls: bit 0 = query staged by copy instead of in the kernel
                             // arguments, bit 1 = stream synchronization instead of polling, bit 2 = round 4's
                             // untagged layout (ids / dists + a polled count: returned the slot's previous result
                             // in ~1 of 1000 concurrent calls, profiles/r04/single_query_stress/; A/B only)
    int screen_split = 1;    // K3c/K3d phases seeded from the earlier ones: 1 = up to three, 2 = two, 0 = one launch,
                             // 3 = doubling (r1, 2 r1, 4 r1, ...; A/B)
    int screen_seed = 3;     // K3c/K3d exact seeds (the exact k-th of the rescored k smallest lower bounds):
                             // bit 0 between phases (else the lists' k-th lower bound + 2 Emax), bit 1 before
                             // the final collect (A/B)
    int screen_range_blocks = 0;  // K3c row-range length in 256-row blocks (0 = auto, ~128; A/B)
    int gather_div = 4;      // coalescer gathering window: at most the last batch's run time / this (key 28;
                             // with K1Q batches 4 beat 8: 16 callers 47.6-54.7k -> 64.7k QPS,
                             // profiles/r05/coalesce/gather_window_k1q.txt)
    int screen_warm = 32;    // K3i (tuning key 29): row blocks per first-phase range (short warm-up ranges
                             // screened against the pilot's bound); 0 = equal ranges (A/B)
    int filter_zc = 1;       // filtered coalesced batches (tuning key 31): bit 0 = K1Q reads the allow
                             // windows from pinned staging (no copy); 0 = copied to HBM first (A/B)
    int screen_warm2 = 0;    // K3i (tuning key 30): row blocks per second-phase range; 0 = the rest uniform
    int k1_mq = 4;           // F32 co-scheduled batches (tuning key 27): queries per K1Q workgroup, 2 or 4
                             // (0 = the COS K1, one query per workgroup)
    int screen_pilot_screen = 0;  // K3c/K3d (tuning key 26): tiles of the SCREEN pilot -- the bf16 screen itself over
                                  // the first tiles in short ranges + one exact seed from their lists -- which
                                  // replaces the K3b pilot (0 = the K3b pilot; A/B)
    int screen_diag = 0;     // K3c diagnostics (tools build only; results are NOT distances): bit 0 = no
                             // wait for the stage loads, bit 1 = no epilogue, bit 2 = no list insertions, bit 3 = no query-fragment loads (K3c); K3d: 1, 2, 4 or 16 (= counters) select compiled variants
};
#ifdef WVG_TOOLS
Tuning &tuning();
#else
const Tuning &tuning();
#endif
// Profiling: events armed by the host runtime (wvg_profile_start) are bound to
// the next scan-kernel dispatch itself (hipExtLaunchKernel), so timing adds no
// marker packets -- a hipEventRecord pair around each launch cost ~5 us of idle
// GPU per record between back-to-back scans.
struct LaunchEvents {
    hipEvent_t start = nullptr, stop = nullptr;
};
LaunchEvents &armed_events();  // thread-local
template <typename... KArgs, typename... Args>
inline void launch_timed(void (*kernel)(KArgs...), dim3 grid, dim3 block, uint32_t lds, hipStream_t s, Args... args)
{
    LaunchEvents &e = armed_events();
    if (e.start) {
        hipExtLaunchKernelGGL(kernel, grid, block, lds, s, e.start, e.stop, 0u, args...);
        e = LaunchEvents{};
    } else {
        hipLaunchKernelGGL(kernel, grid, block, lds, s, args...);
    }
}
// Phase 2: per query `nlists` ascending lists of `list_len` keys -> final
// (ids = id_base + slot, dists, counts).
hipError_t launch_merge_lists(const uint64_t *partials, uint32_t nq, uint32_t nlists, uint32_t list_len, uint32_t k,
                              uint64_t id_base, uint64_t *ids, float *dists, uint32_t *counts, hipStream_t s);
// Unsorted [nq][n_per_query] keys (list_len = 1).
hipError_t launch_merge_keys(const uint64_t *partials, uint32_t nq, uint32_t n_per_query, uint32_t k,
                             uint64_t id_base, uint64_t *ids, float *dists, uint32_t *counts,
                             hipStream_t s);
// Merge (dist, id64) lists -> [nq][k]: list l of query q starts at
// ids + l * ids_stride + q * k_in (dists likewise with d_stride).
hipError_t launch_merge_pairs(const float *dists, const uint64_t *ids, uint64_t ids_stride, uint64_t d_stride,
                              uint32_t nq, uint32_t nlists, uint32_t k_in, uint32_t k, uint64_t *out_ids,
                              float *out_dists, uint32_t *out_counts, hipStream_t s);

// Row-major -> tiled scatter (with optional normalize for cosine) of F32 rows.
hipError_t launch_f32_store(const float *rows, const uint64_t *slots, uint64_t n, uint32_t dim,
                            uint32_t nchunks, int normalize, float *tiled, hipStream_t s);
hipError_t launch_f32_synth(uint64_t seed, int dist, uint64_t row0, uint64_t n, uint64_t slot0,
                            uint32_t dim, uint32_t nchunks, int normalize, float *tiled,
                            hipStream_t s);
hipError_t launch_f32_gather(const float *tiled, const uint64_t *slots, uint64_t n, uint32_t dim,
                             uint32_t nchunks, float *rows, hipStream_t s);
// out[i] = the raw nchunks 16-byte chunks of slots[i] (any corpus kind).
hipError_t launch_gather_chunks(const void *tiled, const uint64_t *slots, uint64_t n, uint32_t nchunks, void *out,
                                hipStream_t s);
hipError_t launch_normalize_rows(const float *in, uint64_t n, uint32_t dim, float *out,
                                 hipStream_t s);
hipError_t launch_distance_rows(int metric, const float *q, const float *rows, uint64_t n,
                                uint32_t dim, float *out, hipStream_t s, int o512 = 0);
// keys[i] = (SingleDist(q, row i), i) over a tiled temporary of n rows.
hipError_t launch_dist_keys(int metric, const float *q, const float *tiled, uint64_t n, uint32_t dim,
                            uint64_t *keys, hipStream_t s, int o512 = 0);
hipError_t launch_synth_rows(uint64_t seed, int dist, const uint64_t *ids, uint64_t n, uint32_t dim,
                             int normalize, float *out, hipStream_t s);
// The screen's exact seed: per query, the k smallest keys of its first `nlists`
// ascending range lists (partials [nq][list_stride], lists of list_len keys)
// rescored exactly; their k-th distance into gbound (atomicMin).
hipError_t launch_seed_exact(int metric, const float *q, uint32_t qpitch, const float *tiled, uint32_t dim,
                             uint32_t nchunks, const uint64_t *partials, uint32_t list_stride, uint32_t list_len,
                             uint32_t nlists, uint32_t nq, uint32_t k, uint32_t *gbound, hipStream_t s);
hipError_t launch_rescore_keys(int metric, const float *q, uint32_t qpitch, const float *tiled,
                               uint32_t dim, uint32_t nchunks, const uint64_t *cand_keys,
                               uint32_t nq, uint32_t ncand, uint32_t cand_stride,
                               uint64_t *out_keys, hipStream_t s, int o512 = 0);
// BQ
hipError_t launch_bq_encode_rows(const float *rows, uint64_t n, uint32_t dim, int normalize,
                                 uint64_t *codes, hipStream_t s);
hipError_t launch_bq_store(const uint64_t *codes, const uint64_t *slots, uint64_t n, uint32_t words,
                           uint32_t nchunks, uint64_t *tiled, hipStream_t s);
hipError_t launch_bq_synth(uint64_t seed, int dist, uint64_t row0, uint64_t n, uint64_t slot0,
                           uint32_t dim, uint32_t nchunks, int normalize, uint64_t *tiled,
                           hipStream_t s);
hipError_t launch_bq_distance_rows(const uint64_t *q, const uint64_t *codes, uint64_t n,
                                   uint32_t words, float *out, hipStream_t s);
// PQ
hipError_t launch_pq_lut(int metric, const float *q, uint32_t nq, uint32_t qpitch,
                         const float *centers, uint32_t m, uint32_t ks, uint32_t ds, float *lut,
                         hipStream_t s);
// codes: row-major [n][m] bytes, or (tiled_out) the PQ corpus layout at slots 0..n-1.
// nan_free: the codebook holds no NaN (enables the pair path's min3 argmin, pq_encode_kernel);
// seg_nan: per-segment NaN flags on the device (launch_pq_pairs), the same per segment.
// Row-major codes of fewer rows than fill the chip split the segments over the grid.
hipError_t launch_pq_encode(const float *tiled_rows, uint64_t n, uint32_t dim, const float *centers,
                            uint32_t m, uint32_t ks, uint8_t *codes, hipStream_t s, bool tiled_out = false,
                            bool nan_free = false, const uint32_t *seg_nan = nullptr);
inline bool pq_nan_free(const float *centers, size_t count)
{
    for (size_t i = 0; i < count; i++)
        if (centers[i] != centers[i]) return false;
    return true;
}
hipError_t launch_pq_store(const uint8_t *codes, const uint64_t *slots, uint64_t n, uint32_t m,
                           uint32_t nchunks, uint8_t *tiled, hipStream_t s);
hipError_t launch_pq_adc_rows(int metric, const float *lut, uint32_t m, uint32_t ks,
                              const uint8_t *codes, uint64_t n, float *out, hipStream_t s);
// Unbounded selection (wvg_select.hip): S1 per-row ordered distance keys for
// one prepared query over [tile_begin, tile_end); S2 radix select of the k-th
// smallest key; S3 compaction of keys <= threshold into (key << 32 | slot);
// S4 rocPRIM sort.
hipError_t launch_ordkeys(const ScanArgs &a, int kind, int num_cus, uint32_t *keys, hipStream_t s);
size_t select_state_bytes();
hipError_t launch_select_kth(const uint32_t *keys, uint64_t n, uint64_t k, int num_cus, void *st_dev,
                             uint32_t *hist, hipStream_t s);
hipError_t launch_key_count(const uint32_t *keys, uint64_t n, uint32_t t_le, uint32_t t_q, int num_cus,
                            unsigned long long *counts, hipStream_t s);
hipError_t launch_key_compact(const uint32_t *keys, uint64_t n, const void *st_dev, uint32_t thr,
                              uint32_t slot0, int num_cus, uint64_t *out, unsigned long long *count,
                              hipStream_t s);
hipError_t read_select_kth(const void *st_dev, uint32_t *kth, hipStream_t s);  // synchronizes s
// The heap replay's superset above 256 (key_compact_chunks_kernel): slot i of
// chunk j kept iff keys[i] < thr[j]; out (slot << 32 | key), unordered.
hipError_t launch_key_compact_chunks(const uint32_t *keys, uint64_t n, const uint32_t *thr, uint64_t R, uint32_t slot0,
                                     int num_cus, uint64_t *out, unsigned long long *count, hipStream_t s);
size_t sort_temp_bytes(uint64_t n);
hipError_t sort_keys64(void *temp, size_t temp_bytes, const uint64_t *in, uint64_t *out, uint64_t n,
                       hipStream_t s);
hipError_t launch_emit_sorted(const uint64_t *sorted, uint64_t n, uint64_t id_base, uint64_t *ids,
                              float *dists, hipStream_t s);
// k-means training (wvg_pq.hip K10) and the PQ symmetric-distance table.
// K10 (wvg_pq.hip): one Lloyd pass = K9 assignment, count, members, sums;
// points segment-major [m][n]
// seg_nan (optional): m words, nonzero where a segment's centroids hold a NaN
hipError_t launch_pq_pairs(const float *centers, uint32_t m, uint32_t ks, float *out, hipStream_t s,
                           uint32_t *seg_nan = nullptr);
// row blocks per segment of the count / member kernels; bhist = [m][blocks][ks]
uint32_t kmeans_blocks(uint64_t n);
hipError_t launch_kmeans_count(const uint8_t *codes, uint64_t n, uint32_t m, uint32_t ks, const uint8_t *active,
                               uint8_t *points, uint32_t *changes, uint32_t *counts, uint32_t *bhist, hipStream_t s);
hipError_t launch_kmeans_recalc2(const float *X, uint64_t n, uint32_t dim, const uint8_t *points, uint32_t m,
                                 uint32_t ks, uint32_t ds, const uint8_t *recalc, const uint32_t *counts,
                                 const uint32_t *bhist, const uint8_t *skip, uint32_t *members, uint32_t *offsets,
                                 float *centers, hipStream_t s);
hipError_t launch_pq_sdc_table(int metric, const float *centers, uint32_t m, uint32_t ks, uint32_t ds,
                               float *table, hipStream_t s);
hipError_t launch_pq_sdc_rows(int metric, const float *table, uint32_t m, uint32_t ks, const uint8_t *x,
                              const uint8_t *codes, uint64_t n, float *out, hipStream_t s);
hipError_t launch_dist_by_ids(const ScanArgs &a, int kind, uint64_t capacity, const uint64_t *ids, uint64_t n,
                              float *out, uint8_t *ok, hipStream_t s,
                              const uint32_t *qidx = nullptr);
hipError_t launch_hbm_read(const void *p, uint64_t bytes, int blocks, float *out, hipStream_t s);
hipError_t launch_set_valid(uint64_t *valid, const uint64_t *slots, uint64_t n, int set,
                            hipStream_t s);

}  // namespace wvg
