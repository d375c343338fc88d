/*
 * wvgpu.h -- C ABI of the MI355X (gfx950) vector-scoring backend for
 * Weaviate's flat / BQ / PQ hot path.  Go binds it through cgo (see
 * INTEGRATION.md); the test and bench harness binds it through ctypes.
 *
 * Citations are relative to the reference tree (antas-marcin/weaviate):
 *   D/  = adapters/repos/db/vector/hnsw/distancer/
 *   CH/ = adapters/repos/db/vector/compressionhelpers/
 *   V/  = adapters/repos/db/vector/
 *
 * Conventions:
 *  - every function returns WVG_OK (0) or a negative WVG_ERR_*; the message is
 *    available from wvg_last_error() on the calling thread.  Nothing aborts.
 *  - host buffers are borrowed for the duration of the call only and never
 *    retained (cgo pointer rules); device memory belongs to the handles.
 *  - distances are float32, smaller is closer; results are ascending by
 *    (distance, id); ids are uint64 docIDs.
 *  - handles are safe for concurrent searches; upsert/delete/reserve take an
 *    exclusive lock on the corpus.
 */
#ifndef WVGPU_H
#define WVGPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 2: wvg_options gained `coalesce` (round 4) and the device-memory / stream
 * entry points were added (wvg_device_alloc ... wvg_memcpy_d2h).
 * 3: wvg_options gained `heap_replay`; wvg_search_bq_candidates; the
 * multi-GPU handle (wvg_multi_*). */
#define WVG_ABI_VERSION 3

#define WVG_OK 0
#define WVG_ERR_INVALID -1       /* bad argument (null, k < 0 analogue, bad kind) */
#define WVG_ERR_DIM_MISMATCH -2  /* "vector lengths don't match" (D/l2.go:47-50) */
#define WVG_ERR_NOMEM -3
#define WVG_ERR_DEVICE -4        /* HIP runtime error */
#define WVG_ERR_NOT_FOUND -5     /* id not present (deleted / never added) */
#define WVG_ERR_UNSUPPORTED -6
#define WVG_ERR_CAPACITY -7      /* id outside [id_base, id_base + capacity) */

/* corpus kinds */
#define WVG_KIND_F32 0 /* float32 rows (flat "vectors" bucket, V/flat/index.go:259-260) */
#define WVG_KIND_BQ 1  /* sign-bit codes (CH/binary_quantization.go:32) */
#define WVG_KIND_PQ 2  /* PQ byte codes (CH/product_quantization.go:420) */

/* metrics: entities/vectorindex/common/config.go:22-31 */
#define WVG_METRIC_L2 0     /* "l2-squared" D/l2.go */
#define WVG_METRIC_DOT 1    /* "dot"        D/dot_product.go */
#define WVG_METRIC_COSINE 2 /* "cosine-dot" D/cosine_dist.go (rows/queries normalized) */
#define WVG_METRIC_MANHATTAN 3 /* "manhattan" D/manhattan.go (pure Go on every host) */
#define WVG_METRIC_HAMMING 4   /* "hamming"   D/hamming.go -> hamming_256 / hamming_512
                                  (D/hamming_amd64.go:18-24); selected by name in
                                  adapters/repos/db/shard.go:406-421 like the others */

typedef struct wvg_ctx wvg_ctx;
typedef struct wvg_corpus wvg_corpus;

/* ---- library / device ---------------------------------------------------- */
int wvg_abi_version(void);
const char *wvg_last_error(void);
int wvg_device_count(int *out);
/* One context per GPU (one process per GPU in the multi-GPU deployment). */
int wvg_open(int device, wvg_ctx **out);
/* Context options, fixed for the life of the context (wvg_open uses the
 * defaults).  Fill with wvg_options_default, change fields, then open.     */
typedef struct wvg_options {
    uint32_t size;             /* sizeof(wvg_options) (ABI guard; set by wvg_options_default) */
    uint32_t mfma_min_queries; /* dot / cosine batches of at least this many queries are scored on the
                                  matrix cores (bf16 screen + exact fp32 rescore, or exact fp32 MFMA);
                                  smaller ones run one HBM-bound scan per query.  0 = never.  Default 32. */
    int32_t cache_reuse;       /* 1 (default): consecutive scans of a corpus alternate direction and read
                                  the last ~320 MB of each pass with the default cache policy, so the next
                                  scan starts on rows still in the 256 MiB Infinity Cache.  0: streaming --
                                  one direction, non-temporal loads, no reuse between scans (e.g. next to
                                  other memory-heavy work, or to measure the DRAM-bound rate). */
    uint32_t merge_wait_us;    /* bound on the in-launch merge's wait for one query's scan workgroups
                                  (wvg_search_device_pipelined); 0 = the default, 4 s.  On expiry the
                                  query gets empty results and wvg_search_device_check fails. */
    int32_t batch_screen;      /* 2 (default): batched dot / cosine searches screen every row with int8
                                  MFMA (d = 512 / 768 / 1024; other d: bf16) and a per-row error bound,
                                  then rescore the candidates exactly in fp32 (results identical to the
                                  exact path); 1: the bf16 screen for every d; 0: exact fp32 MFMA only.
                                  The first screened search of a corpus allocates its shadow: int8 = dim
                                  + 8 bytes per row of capacity (7.7 GB at 10M x 768; its first build
                                  also takes one pass over the rows for the corpus scale and one host
                                  wait), bf16 = 2 * dim + 4 bytes per row (15.4 GB), kept until the
                                  corpus is destroyed or grows. */
    int32_t coalesce;          /* 1 (default): concurrent single-query wvg_search calls on one corpus
                                  join one batched launch -- while a batch runs, the calls that arrive
                                  queue up and the next batch takes them all (filtered calls, each with its
                                  own allow list, in batches of their own; any mix of k, run at the
                                  largest); right after a batch of 4 or more the next one waits a short window
                                  (at most a quarter of that batch's run time) for the callers just answered; each
                                  caller gets exactly its own results (identical to a call of its own); a
                                  lone call does not wait.  0: every call launches on its own. */
    int32_t heap_replay;       /* 1 (default): wvg_search_bq_rescore / wvg_search_bq_candidates return
                                  exactly what Weaviate's heaps return (V/flat/index.go:347-389,
                                  497-520): which rows of a tie at the R-th Hamming distance become
                                  candidates, their pop order, and the k-heap's choice and order among
                                  equal exact distances.  The scan also records the rows the heap could
                                  insert and the host replays the heap over them (~R ln(rows) per query).
                                  0: candidates = the (distance, docID)-lexicographic top-R, results
                                  ascending by (distance, docID) -- identical except at such ties. */
} wvg_options;
void wvg_options_default(wvg_options *opts);
int wvg_open_ex(int device, const wvg_options *opts, wvg_ctx **out);
int wvg_close(wvg_ctx *ctx);
int wvg_synchronize(wvg_ctx *ctx);
/* Page-locked host memory for a caller's reusable staging buffers (e.g. the
 * R rows flat.searchByVectorBQ gathers for its rescore, V/flat/index.go:375-385):
 * every entry point copies from / to such a buffer directly, without its own
 * staging copy.  Any other host pointer keeps working (copied through the
 * call's staging).  Free with wvg_host_free on the same context. */
int wvg_host_alloc(wvg_ctx *ctx, uint64_t bytes, void **out);
int wvg_host_free(wvg_ctx *ctx, void *p);
/* Device memory and streams of the context's GPU for the device-pointer
 * entry points below (wvg_search_device*, wvg_topk_merge_*), so a caller
 * without a HIP binding of its own (the Go backend) can hold queries,
 * results and workspaces in HBM: wvg_device_alloc returns `bytes` of HBM,
 * zero-filled when `zero` != 0 (a search workspace must be); free it with
 * wvg_device_free after the work using it has finished (wvg_stream_synchronize).
 * wvg_stream_create makes a non-blocking stream (a hipStream_t) for `stream`
 * arguments.  wvg_memcpy_h2d / _d2h copy on `stream` and return when the copy
 * is complete (so `src` / `dst` host memory may be a Go slice); `stream` NULL
 * = the default stream.  Replaces the cgo-side HIP plumbing a serving loop
 * would need (adapters/repos/db/vector_index.go:24-45 callers hold no HIP). */
int wvg_device_alloc(wvg_ctx *ctx, uint64_t bytes, int zero, void **out);
int wvg_device_free(wvg_ctx *ctx, void *p);
int wvg_stream_create(wvg_ctx *ctx, void **out);
int wvg_stream_destroy(wvg_ctx *ctx, void *stream);
int wvg_stream_synchronize(wvg_ctx *ctx, void *stream);
int wvg_memcpy_h2d(wvg_ctx *ctx, void *d_dst, const void *src, uint64_t bytes, void *stream);
int wvg_memcpy_d2h(wvg_ctx *ctx, void *dst, const void *d_src, uint64_t bytes, void *stream);
/* The reduction order of the fp32 distances (l2 / dot / cosine), i.e. which
 * of the reference's SIMD kernels the results must match bit for bit: its
 * init() picks l2_512 / dot_512 on hosts with AMX-BF16 and AVX-512, else
 * l2_256 / dot_256 (D/l2_amd64.go:19-25, D/dot_product_amd64.go:19-25).
 * Default WVG_ORDER_AVX256 (AMD EPYC hosts, which have no AMX).  Applies to
 * every fp32 distance of the context (scans, rescoring, DistanceToNode,
 * wvg_distance_batch); batched dot/cosine then scans with K1 instead of the
 * MFMA kernel, whose slices are the AVX2 order's chains.                  */
#define WVG_ORDER_AVX256 0
#define WVG_ORDER_AVX512 1
int wvg_set_distance_order(wvg_ctx *ctx, int order);

/* ---- corpus: the device-resident copy of a flat index's rows --------------
 * Replaces the LSM cursor scan of V/flat/index.go:411-452 and the BQ cache of
 * V/cache/sharded_lock_cache.go:29-60 (docID-indexed).  Slot = id - id_base.
 * id_base must be a multiple of 64; capacity is rounded up to 64 rows.      */
int wvg_corpus_create(wvg_ctx *ctx, int kind, int metric, uint32_t dim, uint64_t id_base,
                      uint64_t capacity, wvg_corpus **out);
int wvg_corpus_destroy(wvg_corpus *c);
/* cache.Grow analogue (V/cache/sharded_lock_cache.go:251): keeps contents. */
int wvg_corpus_reserve(wvg_corpus *c, uint64_t capacity);
int wvg_corpus_info(wvg_corpus *c, uint64_t *count, uint64_t *high_water, uint64_t *capacity);
/* flat.Add / AddBatch (V/flat/index.go:247-274): validates the dimension
 * ("insert called with a vector of the wrong size"), normalizes for cosine,
 * and for kind BQ encodes on device (index.go:262-270), for PQ encodes with
 * the codebook (CH/product_quantization.go:420).  vectors: [n][dim] float32. */
int wvg_corpus_upsert(wvg_corpus *c, const uint64_t *ids, const float *vectors, uint64_t n,
                      uint32_t dim);
/* Load already-stored rows (restart from the "vectors" / "vectors_compressed"
 * buckets, V/flat/index.go:640-681): F32 = [n][dim] float32 (already
 * normalized at Add for cosine), BQ = [n][ceil(dim/64)] uint64 LE words,
 * PQ = [n][m] bytes.  Stored as given (no normalization / encoding). */
int wvg_corpus_upsert_codes(wvg_corpus *c, const uint64_t *ids, const void *codes, uint64_t n);
/* Restart / PostStartup bulk load from an LSM cursor (V/flat/index.go:640-681):
 * keys [n][8] big-endian docIDs, values [n][value_bytes] little-endian rows as
 * the "vectors" (F32: dim float32) or "vectors_compressed" (BQ: uint64 words)
 * bucket stores them, or PQ codes (m bytes).  Stored as given; the capacity
 * grows to the largest id (bqCache.Grow(maxID)).                           */
int wvg_corpus_load_kv(wvg_corpus *c, const uint8_t *keys, const uint8_t *values, uint64_t n,
                       uint64_t value_bytes);
/* Batched Distance / CompressorDistancer.DistanceToNode(id) (CH/compression.go:306-325,
 * the HNSW rescore loop V/hnsw/search.go:564-581): the query's distance to
 * the rows with docIDs ids[n] (F32: SingleDist, BQ: Hamming, PQ: ADC);
 * out_ok[i] = 0 (and out_dists[i] = 0) where the id is not live, like the
 * reference's ok=false for deleted nodes.                                  */
int wvg_corpus_distance_by_ids(wvg_corpus *c, const float *query, const uint64_t *ids, uint64_t n,
                               float *out_dists, uint8_t *out_ok);
/* The same for many queries in ONE launch (batched HNSW rescore: every
 * query's ef candidates, V/hnsw/search.go:564-581, for concurrent queries):
 * queries [nq][dim]; query q's ids are ids[offsets[q] .. offsets[q+1]),
 * offsets[nq+1] non-decreasing from 0; outputs parallel to ids.            */
int wvg_corpus_distance_by_ids_batch(wvg_corpus *c, const float *queries, uint32_t nq, const uint64_t *offsets,
                                     const uint64_t *ids, float *out_dists, uint8_t *out_ok);
/* flat.Delete (V/flat/index.go:276-295): clears the validity bit. */
int wvg_corpus_delete(wvg_corpus *c, const uint64_t *ids, uint64_t n);
/* flat.vectorById (V/flat/index.go:401-407): copies the stored row
 * (F32: dim floats, BQ: words u64, PQ: m bytes); WVG_ERR_NOT_FOUND if absent. */
int wvg_corpus_get(wvg_corpus *c, uint64_t id, void *out);
/* vectorById for many ids in one call (the rescore loop's row fetches,
 * V/flat/index.go:375-385): out [n][row bytes as wvg_corpus_get];
 * out_ok[i] = 0 (row zero-filled) where ids[i] is not live.               */
int wvg_corpus_get_batch(wvg_corpus *c, const uint64_t *ids, uint64_t n, void *out, uint8_t *out_ok);
/* Bench / test helper: fills slots [0, n) with synthetic rows generated in
 * place from a counter-based RNG keyed by (seed, id_base + slot, column);
 * distribution 0 = uniform [-1,1), 1 = integers 0..255.  F32 and BQ only.  */
int wvg_corpus_fill_synthetic(wvg_corpus *c, uint64_t seed, uint64_t n, int distribution);
/* PQ codebook: centers [m][ks][dim/m] float32 (KMeans centers, CH/kmeans.go:85-93).
 * Validation as NewProductQuantizer (CH/product_quantization.go:187-197).  */
int wvg_pq_set_codebook(wvg_corpus *c, const float *centers, uint32_t m, uint32_t ks);

/* ---- search ---------------------------------------------------------------
 * flat.SearchByVector (V/flat/index.go:307-334) for F32 corpora; for BQ the
 * Hamming top-k of findTopVectorsCached (index.go:456-495); for PQ the ADC
 * top-k (PQDistancer.Distance, CH/product_quantization.go:352-361).
 * queries: [nq][dim] float32 (normalized internally for cosine, index.go:323).
 * allow_bits: optional bitmap over global docIDs (helpers.AllowList), bit i of
 * word i/64; an empty allow list yields empty results (index.go:425-427).
 * Outputs: [nq][k] ids/dists, counts[nq] = min(k, live allowed rows).
 * Any k: up to 256 the fused register top-k of the scan; above, a radix
 * select + sort over per-row distance keys in HBM (the same distances).    */
int wvg_search(wvg_corpus *c, const float *queries, uint32_t nq, uint32_t k,
               const uint64_t *allow_bits, uint64_t allow_words, uint64_t *out_ids,
               float *out_dists, uint32_t *out_counts);
/* flat.searchByVectorBQ (V/flat/index.go:347-389): Hamming top-R over `bq`,
 * R = max(rescore_limit, k) (index.go:297-305), exact rescore of the R
 * candidates against the device-resident float rows of `f32`, top-k.      */
int wvg_search_bq_rescore(wvg_corpus *bq, wvg_corpus *f32, const float *queries, uint32_t nq,
                          uint32_t k, uint32_t rescore_limit, const uint64_t *allow_bits,
                          uint64_t allow_words, uint64_t *out_ids, float *out_dists,
                          uint32_t *out_counts);
/* The first half of searchByVectorBQ for callers whose float rows are not on
 * the GPU (the LSM "vectors" bucket, V/flat/index.go:375-380): the candidates
 * findTopVectorsCached leaves in its heap of R = rescore_limit (index.go:
 * 355-357, 456-495) in the order heap.Pop() returns them (:369-374), i.e.
 * descending Hamming distance with the heap's own order among ties.  Outputs
 * [nq][R] ids / Hamming distances, counts[nq]; feed them in this order to
 * wvg_rescore (which inserts in input order, as :375-385 does).  With
 * heap_replay = 0: the lexicographic top-R, descending.  Any R.           */
int wvg_search_bq_candidates(wvg_corpus *bq, const float *queries, uint32_t nq, uint32_t rescore_limit,
                             const uint64_t *allow_bits, uint64_t allow_words, uint64_t *out_ids,
                             float *out_dists, uint32_t *out_counts);

/* flat.SearchByVectorDistance (V/flat/index.go:531-591): every row with
 * dist <= target_distance or |dist - target| <= 1e-6 (floatcomp.InDelta,
 * usecases/floatcomp/delta.go:16-19), ascending, as far as the growing-limit
 * loop reaches (limits 100, 1100, 11100, ...; V/common/search_by_dist_params.go:
 * 14-83): it stops at the first window whose last row is above the target,
 * and before a limit above max_limit (max_limit < 0: unlimited).  One pass
 * over the corpus regardless of how many windows the loop takes.
 * *out_count = number of results; min(count, out_capacity) are written. */
int wvg_search_by_distance(wvg_corpus *c, const float *query, float target_distance, int64_t max_limit,
                           const uint64_t *allow_bits, uint64_t allow_words, uint64_t *out_ids,
                           float *out_dists, uint64_t out_capacity, uint64_t *out_count);
/* The flat index's own SearchByVectorDistance result (V/flat/index.go:
 * 531-591 as written): its loop calls recursiveSearch once -- the post
 * statement of the `for` is empty, so later iterations only grow the limit
 * until max_limit stops them (and never stop when max_limit < 0) -- so the
 * result is the first window: among the `window` (100:
 * V/common/search_by_dist_params.go:17) nearest rows, those with dist <=
 * target or within 1e-6 of it, up to the first row beyond.  HNSW callers use
 * wvg_search_by_distance (V/hnsw/search.go:85-151 re-searches).            */
int wvg_search_by_distance_window(wvg_corpus *c, const float *query, float target_distance, uint32_t window,
                                  const uint64_t *allow_bits, uint64_t allow_words, uint64_t *out_ids,
                                  float *out_dists, uint64_t out_capacity, uint64_t *out_count);

/* Device-pointer variants: inputs/outputs in HBM, asynchronous on `stream`
 * (a hipStream_t, NULL = default stream); no host synchronization, no
 * allocation (caller supplies a workspace of wvg_search_workspace_size bytes,
 * zero-filled once before its first use), so a call can be captured in a
 * hipGraph.  Exception: the first screened dot / cosine batch of a corpus
 * (batch_screen) allocates and builds the corpus's shadow on `stream`;
 * under capture that never happens -- a corpus without a current shadow takes
 * the exact path, one with a shadow waits for it before the capture (run one
 * uncaptured batch first to warm it).  d_counts may be NULL.  One workspace
 * serves any number of calls issued in order on one stream.  An empty corpus
 * (e.g. a rank whose slab holds no rows) yields empty results: ids
 * UINT64_MAX, dists +inf, counts 0 (as wvg_search).  wvg_search_device
 * takes F32, BQ and PQ corpora (d_queries: float [nq][dim]; BQ codes and PQ
 * LUTs are built on the device -- size the workspace after the PQ codebook
 * is set); wvg_search_device_pipelined takes F32 corpora.                  */
size_t wvg_search_workspace_size(wvg_corpus *c, uint32_t nq, uint32_t k);
int wvg_search_device(wvg_corpus *c, const float *d_queries, uint32_t nq, uint32_t k,
                      uint64_t *d_ids, float *d_dists, uint32_t *d_counts, void *d_workspace,
                      size_t workspace_bytes, void *stream);
/* nq independent single-query searches (each one full scan of the corpus:
 * flat.SearchByVector per query, as concurrent Weaviate queries issue them)
 * in ONE launch: the scan workgroups walk the queries back to back and one
 * extra workgroup merges each query's partial lists while the scan moves
 * on, so the merges cost no launches of their own.  F32 corpora; same
 * workspace size rule; outputs as wvg_search_device.                       */
int wvg_search_device_pipelined(wvg_corpus *c, const float *d_queries, uint32_t nq, uint32_t k,
                                uint64_t *d_ids, float *d_dists, uint32_t *d_counts,
                                void *d_workspace, size_t workspace_bytes, void *stream);
/* Synchronizes `stream` and reads (and clears) the workspace's sticky status
 * word: WVG_ERR_DEVICE if any device search on this workspace since the last
 * check could not complete -- the query-stream merge workgroup of
 * wvg_search_device_pipelined gave up waiting for the scan (bounded at 4 s);
 * the queries it could not merge were given empty results, never stale ones. */
int wvg_search_device_check(wvg_ctx *ctx, void *d_workspace, void *stream);
/* Multi-shard merge (Index.objectVectorSearch, adapters/repos/db/index.go:1644-1648):
 * [nlists][nq][k_in] (dist, id) lists (the layout an all-gather of per-GPU
 * [nq][k_in] results produces) -> [nq][k] ascending, ties by id; missing
 * entries carry id UINT64_MAX.                                            */
int wvg_topk_merge_device(wvg_ctx *ctx, const float *d_dists, const uint64_t *d_ids, uint32_t nq,
                          uint32_t nlists, uint32_t k_in, uint32_t k, uint64_t *d_out_ids,
                          float *d_out_dists, uint32_t *d_out_counts, void *stream);
/* The same merge over packed blocks, so one all-gather moves both halves of
 * every rank's result: a block holds ids [nq][k] uint64 at byte 0 and dists
 * [nq][k] float32 at byte nq*k*8, and is wvg_topk_packed_bytes(nq, k) bytes
 * (a multiple of 16); d_packed holds nlists consecutive blocks.  Write a
 * block directly with wvg_search_device*(..., d_ids = block,
 * d_dists = block + nq*k*8, ...).                                          */
size_t wvg_topk_packed_bytes(uint32_t nq, uint32_t k);
int wvg_topk_merge_packed(wvg_ctx *ctx, const void *d_packed, uint32_t nq, uint32_t nlists, uint32_t k_in,
                          uint32_t k, uint64_t *d_out_ids, float *d_out_dists, uint32_t *d_out_counts,
                          void *stream);

/* ---- several GPUs in one process ------------------------------------------
 * Index.objectVectorSearch (adapters/repos/db/index.go:1567-1648) fans a
 * search out over the shards of one process and merges their results by
 * distance.  A multi handle holds one context per device (opts as
 * wvg_open_ex) and, when the devices are distinct and RCCL loads, one
 * communicator per device (ncclCommInitAll).  A multi corpus deals docIDs to
 * the devices in contiguous slabs: shard i holds [i * slab, (i + 1) * slab),
 * slab = rows / ndev rounded up to 64.  wvg_multi_search runs every shard's
 * scan on its own device stream into a packed block, ONE grouped RCCL
 * all-gather of the blocks over xGMI (peer copies to device 0 when devices
 * repeat, e.g. a one-GPU rehearsal {0, 0}), the merge on device 0, and returns
 * [nq][k] ascending by (distance, docID) -- identical to one corpus holding
 * every row.  Per-shard operations (PQ codebooks, other search kinds) take
 * the shard's own handle from wvg_multi_corpus_shard.                      */
typedef struct wvg_multi wvg_multi;
typedef struct wvg_multi_corpus wvg_multi_corpus;
int wvg_multi_open(const int *devices, int ndev, const wvg_options *opts, wvg_multi **out);
int wvg_multi_close(wvg_multi *m);  /* after every multi corpus is destroyed */
int wvg_multi_info(wvg_multi *m, int *ndev, int *uses_rccl);
int wvg_multi_ctx(wvg_multi *m, int i, wvg_ctx **out);
int wvg_multi_corpus_create(wvg_multi *m, int kind, int metric, uint32_t dim, uint64_t rows,
                            wvg_multi_corpus **out);
int wvg_multi_corpus_destroy(wvg_multi_corpus *mc);
int wvg_multi_corpus_shard(wvg_multi_corpus *mc, int i, wvg_corpus **out, uint64_t *id_base, uint64_t *slab_rows);
/* flat.Add / Delete routed to the shard owning each docID (WVG_ERR_CAPACITY
 * for an id beyond the last slab). */
int wvg_multi_corpus_upsert(wvg_multi_corpus *mc, const uint64_t *ids, const float *vectors, uint64_t n,
                            uint32_t dim);
int wvg_multi_corpus_delete(wvg_multi_corpus *mc, const uint64_t *ids, uint64_t n);
/* As wvg_corpus_fill_synthetic over docIDs [0, n) of the whole corpus. */
int wvg_multi_corpus_fill_synthetic(wvg_multi_corpus *mc, uint64_t seed, uint64_t n, int distribution);
int wvg_multi_corpus_set_codebook(wvg_multi_corpus *mc, const float *centers, uint32_t m, uint32_t ks);
/* wvg_search over all shards (any kind; k <= 256; allow_bits over global docIDs). */
int wvg_multi_search(wvg_multi_corpus *mc, const float *queries, uint32_t nq, uint32_t k,
                     const uint64_t *allow_bits, uint64_t allow_words, uint64_t *out_ids, float *out_dists,
                     uint32_t *out_counts);

/* The rescore loop of flat.searchByVectorBQ (V/flat/index.go:375-385) when
 * the candidate rows come from the host (LSM point gets): exact SingleDist of
 * q against rows [n][dim] (q used as given: normalize it first for cosine,
 * as index.go:352 does), each inserted into a heap of k in input order
 * (insertToHeap, :384) and extracted (extractHeap, :508-520), so ties among
 * equal distances resolve exactly as the reference's heap resolves them
 * (heap_replay = 0: ascending by (dist, input position)).  out_count = min(k, n). */
int wvg_rescore(wvg_ctx *ctx, int metric, const float *q, const float *rows, const uint64_t *ids,
                uint64_t n, uint32_t dim, uint32_t k, uint64_t *out_ids, float *out_dists,
                uint32_t *out_count);
/* Bulk PQ compression of a resident float corpus (hnsw.compress ->
 * compressor.Preload per vector, V/hnsw/compress.go:98-104): every live row
 * of `f32` is encoded with `pq`'s codebook into the same slot of `pq`.  Both
 * corpora must share dim and id_base. */
int wvg_pq_encode_corpus(wvg_corpus *pq, wvg_corpus *f32);
/* Bench / test helper: the synthetic generator of wvg_corpus_fill_synthetic
 * for arbitrary row ids: out [n][dim] (normalized if `normalize`). */
int wvg_synthetic_rows(wvg_ctx *ctx, uint64_t seed, const uint64_t *ids, uint64_t n, uint32_t dim,
                       int distribution, int normalize, float *out);

/* Profiling: while enabled, every scan-kernel launch of this context is
 * bracketed by a pair of HIP events on its stream; stop() synchronizes and
 * returns the summed scan-kernel time and the launch count (feeds the
 * vector_index_durations_ms metric, usecases/monitoring/prometheus.go:292). */
int wvg_profile_start(wvg_ctx *ctx);
int wvg_profile_stop(wvg_ctx *ctx, double *scan_ms_total, uint64_t *scan_launches);
/* Measurement helper: the HBM streaming-read rate of this GPU, in GB/s -- the
 * best of 16-byte non-temporal reads of a `bytes` buffer (its own
 * allocation, freed again) in two shapes -- grid-stride over 1024..8192
 * workgroups, and the scans' contiguous chunk per workgroup (8 KiB per wave
 * per step) over 256..2048 workgroups -- `reps` passes each.  The ceiling
 * the HBM-bound scans are compared with (roofline).                       */
int wvg_measure_hbm_read(wvg_ctx *ctx, uint64_t bytes, uint32_t reps, double *out_gbps);

/* ---- bulk primitives (distancer.BatchProvider / compressionhelpers bulk) --- */
/* Provider.SingleDist of q against n rows X [n][dim] (D/provider.go:14-20). */
int wvg_distance_batch(wvg_ctx *ctx, int metric, const float *q, const float *X, uint64_t n,
                       uint32_t dim, float *out);
/* distancer.Normalize of n rows (D/normalize.go:16-32). */
int wvg_normalize_batch(wvg_ctx *ctx, const float *X, uint64_t n, uint32_t dim, float *out);
/* BinaryQuantizer.Encode of n rows -> [n][ceil(dim/64)] words (CH/binary_quantization.go:32-45). */
int wvg_bq_encode(wvg_ctx *ctx, const float *X, uint64_t n, uint32_t dim, uint64_t *out_words);
/* BinaryQuantizer.DistanceBetweenCompressedVectors of q against n codes (:47-56). */
int wvg_bq_distance_batch(wvg_ctx *ctx, const uint64_t *q, const uint64_t *codes, uint64_t n,
                          uint32_t words, float *out);
/* ProductQuantizer.Encode of n rows (CH/product_quantization.go:420-426,
 * CH/kmeans.go:103-135; ties to the highest centroid index). */
int wvg_pq_encode(wvg_ctx *ctx, const float *centers, uint32_t m, uint32_t ks, const float *X,
                  uint64_t n, uint32_t dim, uint8_t *out_codes);
/* DistanceLookUpTable for one query (CH/product_quantization.go:62-104): [m][ks]. */
int wvg_pq_lut(wvg_ctx *ctx, int metric, const float *centers, uint32_t m, uint32_t ks,
               uint32_t dim, const float *q, float *out_lut);
/* PQDistancer.Distance of n codes against a LUT (CH/product_quantization.go:352-361). */
int wvg_pq_adc_batch(wvg_ctx *ctx, int metric, const float *lut, uint32_t m, uint32_t ks,
                     const uint8_t *codes, uint64_t n, float *out);

/* ProductQuantizer.Fit with the k-means encoder (CH/product_quantization.go:372-418):
 * the first training_limit rows (0 = all) of X [n][dim]; per segment
 * KMeans.Fit (CH/kmeans.go:220-250): ks initial centers drawn (with
 * replacement) from the rows, Lloyd iterations -- nNearest assignment (ties to
 * the highest index), empty clusters reseeded from a random row of a cluster
 * with more than one member, centers = sequential fp32 sums / size -- until
 * fewer than int(float32(n) * 0.01) rows change or after 11 passes.  The
 * random draws come from a counter RNG keyed by (seed, segment) instead of
 * Go's unseeded global math/rand.  out_centers: [m][ks][dim/m];
 * out_iterations (nullable): [m] Lloyd passes per segment.  "not enough data
 * to fit kmeans" if fewer than ks rows.                                    */
int wvg_pq_fit(wvg_ctx *ctx, const float *X, uint64_t n, uint32_t dim, uint32_t m, uint32_t ks,
               uint64_t training_limit, uint64_t seed, float *out_centers, uint32_t *out_iterations);
/* buildGlobalDistances (CH/product_quantization.go:236-251): [m][ks][ks]
 * table of Step(C_s[i], C_s[j]) (the symmetric-distance table of HNSW's
 * node-to-node PQ distances). */
int wvg_pq_global_distances(wvg_ctx *ctx, int metric, const float *centers, uint32_t m, uint32_t ks, uint32_t dim,
                            float *out_table);
/* DistanceBetweenCompressedVectors (CH/product_quantization.go:297-311) of
 * code x against n codes [n][m], from the table above. */
int wvg_pq_sdc_batch(wvg_ctx *ctx, int metric, const float *table, uint32_t m, uint32_t ks, const uint8_t *x,
                     const uint8_t *codes, uint64_t n, float *out);

#ifdef __cplusplus
}
#endif

#endif /* WVGPU_H */
