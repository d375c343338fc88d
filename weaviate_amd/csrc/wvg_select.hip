// wvg_select.hip -- the unbounded selections of the flat index: top-k for any
// k (the fused register top-k of K1/K5/K8 stops at k = 256) and the range
// search of SearchByVectorDistance.
//
// Reference paths:
//   flat.SearchByVector with a large limit       V/flat/index.go:307-334 (heap of size k)
//   flat.SearchByVectorDistance                  V/flat/index.go:531-591, growing limits
//     100, 1100, 11100, ... (V/common/search_by_dist_params.go:14-83), kept rows
//     dist <= target || InDelta(dist, target, 1e-6) (usecases/floatcomp/delta.go:16-19)
//
// Flow (one query at a time, all in HBM):
//   S1 ordkeys  : one pass over the corpus writes the order-preserving u32 of
//                 every row's distance (0xFFFFFFFF = dead / not allowed), lane
//                 = row, the same per-lane distance code as the scans, so the
//                 values are bit-identical to K1/K5/K8.  HBM: row bytes + 4 B/row.
//   S2 select   : radix select of the k-th smallest key over the 4-byte keys
//                 (12 + 12 + 8 bit digits; LDS histograms, one pick workgroup
//                 per digit) -- or, for range search, a count of the keys under
//                 the two host-computed thresholds.
//   S3 compact  : keys <= threshold -> (key << 32 | slot) u64, wave-aggregated
//                 atomic append (order restored by S4).
//   S4 sort     : rocPRIM radix sort of the compacted u64 keys, i.e. ascending
//                 (distance, docID); the first k (or R) are emitted.
#include <cstring>

#include <rocprim/device/device_radix_sort.hpp>

#include "wvg_internal.hpp"
#include "wvg_rowdist.hpp"

namespace wvg {

constexpr uint32_t ORD_NONE = 0xFFFFFFFFu;  // never an ordered distance (NaN canonicalises below it)

__device__ __forceinline__ uint64_t sel_tile_mask(const ScanArgs &a, uint64_t t)
{
    uint64_t m = a.valid[t];
    if (a.allow) {
        const uint64_t w = t - a.allow_t0;  // allow[0] is tile allow_t0's word
        m &= w < a.allow_words ? a.allow[w] : 0ull;
    }
    return m;
}

// S1, F32: keys[slot - 64*tile_begin] for the query at a.queries (padded to 4).
template <int METRIC>
__global__ __launch_bounds__(256) void ordkeys_f32_kernel(ScanArgs a, uint32_t *keys)
{
    const int lane = threadIdx.x & 63;
    const uint64_t ntiles = a.tile_end - a.tile_begin;
    const uint64_t gw = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint64_t nw = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    const float4 *q4 = reinterpret_cast<const float4 *>(a.queries);
    const float4 *data = reinterpret_cast<const float4 *>(a.data);
    for (uint64_t i = gw; i < ntiles; i += nw) {
        const uint64_t t = a.tile_begin + i;
        const uint64_t m = sel_tile_mask(a, t);
        uint32_t key = ORD_NONE;
        if ((m >> lane) & 1ull) {
            const float4 *rp = data + (size_t)t * a.nchunks * 64 + lane;
            key = wvg_ord_f32(wrap_metric(a.metric, row_dist<METRIC, 64>(rp, q4, (int)a.dim, a.order512)));
        }
        keys[i * 64 + lane] = key;
    }
}

// S1, BQ: Hamming distance (CH/binary_quantization.go:47-56) as in K5.
__global__ __launch_bounds__(256) void ordkeys_bq_kernel(ScanArgs a, uint32_t *keys)
{
    const int lane = threadIdx.x & 63;
    const uint64_t ntiles = a.tile_end - a.tile_begin;
    const uint64_t gw = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint64_t nw = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    const uint64_t *q = reinterpret_cast<const uint64_t *>(a.queries);
    const ulonglong2 *data = reinterpret_cast<const ulonglong2 *>(a.data);
    for (uint64_t i = gw; i < ntiles; i += nw) {
        const uint64_t t = a.tile_begin + i;
        const uint64_t m = sel_tile_mask(a, t);
        uint32_t key = ORD_NONE;
        if ((m >> lane) & 1ull) {
            const ulonglong2 *rp = data + (size_t)t * a.nchunks * 64 + lane;
            uint32_t tot = 0;
            for (uint32_t c = 0; c < a.nchunks; c++) {
                const ulonglong2 x = rp[(size_t)c * 64];
                tot += (uint32_t)__popcll(x.x ^ q[2 * c]) + (uint32_t)__popcll(x.y ^ q[2 * c + 1]);
            }
            key = wvg_ord_f32((float)tot);
        }
        keys[i * 64 + lane] = key;
    }
}

// S1, PQ: ADC with the query's LUT in LDS (CH/product_quantization.go:85-104), as K8.
__global__ __launch_bounds__(256) void ordkeys_pq_kernel(ScanArgs a, uint32_t *keys)
{
    extern __shared__ float lut[];
    const uint32_t m = a.pq_m, ks = a.pq_ks;
    const float *glut = reinterpret_cast<const float *>(a.queries);
    for (uint32_t i = threadIdx.x; i < m * ks; i += blockDim.x) lut[i] = glut[i];
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const uint64_t ntiles = a.tile_end - a.tile_begin;
    const uint64_t gw = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint64_t nw = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    const uint4 *data = reinterpret_cast<const uint4 *>(a.data);
    for (uint64_t i = gw; i < ntiles; i += nw) {
        const uint64_t t = a.tile_begin + i;
        const uint64_t msk = sel_tile_mask(a, t);
        uint32_t key = ORD_NONE;
        if ((msk >> lane) & 1ull) {
            const uint4 *rp = data + (size_t)t * a.nchunks * 64 + lane;
            const float sum = pq_row_sum(rp, a.nchunks, m, ks, lut, (uint64_t)lane);
            key = wvg_ord_f32(wrap_metric(a.metric, sum));
        }
        keys[i * 64 + lane] = key;
    }
}

static unsigned sel_grid(uint64_t ntiles, int num_cus)
{
    const uint64_t want = (ntiles + 3) / 4;  // 4 waves per 256-thread block
    return (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(want, (uint64_t)num_cus * 8));
}

hipError_t launch_ordkeys(const ScanArgs &a, int kind, int num_cus, uint32_t *keys, hipStream_t s)
{
    const uint64_t ntiles = a.tile_end - a.tile_begin;
    if (ntiles == 0) return hipSuccess;
    dim3 grid(sel_grid(ntiles, num_cus)), block(256);
    if (kind == WVG_KIND_F32) {
        with_metric(a.metric, [&](auto M) {
            hipLaunchKernelGGL((ordkeys_f32_kernel<decltype(M)::value>), grid, block, 0, s, a, keys);
        });
    } else if (kind == WVG_KIND_BQ) {
        hipLaunchKernelGGL(ordkeys_bq_kernel, grid, block, 0, s, a, keys);
    } else {
        hipLaunchKernelGGL(ordkeys_pq_kernel, grid, block, (size_t)a.pq_m * a.pq_ks * 4, s, a, keys);
    }
    return hipGetLastError();
}

// ---- S2: radix select -------------------------------------------------------
// State: keys whose bits under `mask` equal `prefix` are the live candidates;
// `krem` = rank (1-based) of the wanted key among them.
struct SelState {
    uint32_t prefix, mask;
    unsigned long long krem;
};

constexpr int HIST_BITS = 12;
constexpr int HIST_BINS = 1 << HIST_BITS;

__global__ __launch_bounds__(256) void key_hist_kernel(const uint32_t *keys, uint64_t n, const SelState *st, int shift,
                                                       int bits, uint32_t *hist)
{
    __shared__ uint32_t h[HIST_BINS];
    for (int i = threadIdx.x; i < HIST_BINS; i += blockDim.x) h[i] = 0;
    __syncthreads();
    const uint32_t prefix = st->prefix, mask = st->mask;
    const uint32_t dmask = (1u << bits) - 1u;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t k = keys[i];
        if ((k & mask) == prefix) atomicAdd(&h[(k >> shift) & dmask], 1u);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < HIST_BINS; i += blockDim.x)
        if (h[i]) atomicAdd(&hist[i], h[i]);
}

// One workgroup: the digit whose cumulative count reaches krem; clears hist
// for the next pass.
__global__ __launch_bounds__(256) void key_pick_kernel(SelState *st, uint32_t *hist, int shift, int bits)
{
    __shared__ unsigned long long part[256];
    const int tid = threadIdx.x;
    const int nb = 1 << bits, per = nb / 256;
    unsigned long long loc = 0;
    for (int j = 0; j < per; j++) loc += hist[tid * per + j];
    part[tid] = loc;
    __syncthreads();
    if (tid == 0) {
        unsigned long long krem = st->krem, cum = 0;
        int t = 0;
        while (t < 255 && cum + part[t] < krem) cum += part[t++];
        int d = t * per;
        for (;; d++) {
            const unsigned long long c = hist[d];
            if (cum + c >= krem || d == t * per + per - 1) break;
            cum += c;
        }
        st->krem = krem - cum;
        st->prefix |= (uint32_t)d << shift;
        st->mask |= (uint32_t)(nb - 1) << shift;
    }
    __syncthreads();
    for (int i = tid; i < HIST_BINS; i += 256) hist[i] = 0;
}

// st/hist: device scratch (hist HIST_BINS u32).  After the call st->prefix is
// the k-th smallest key (1 <= k <= n).
hipError_t launch_select_kth(const uint32_t *keys, uint64_t n, uint64_t k, int num_cus, void *st_dev, uint32_t *hist,
                             hipStream_t s)
{
    SelState init{0u, 0u, (unsigned long long)k};
    SelState *st = reinterpret_cast<SelState *>(st_dev);
    hipError_t e = hipMemcpyAsync(st, &init, sizeof(init), hipMemcpyHostToDevice, s);
    if (e != hipSuccess) return e;
    e = hipMemsetAsync(hist, 0, HIST_BINS * 4, s);
    if (e != hipSuccess) return e;
    const unsigned grid = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((n + 1023) / 1024, (uint64_t)num_cus * 4));
    const int shifts[3] = {20, 8, 0}, bits[3] = {12, 12, 8};
    for (int p = 0; p < 3; p++) {
        hipLaunchKernelGGL(key_hist_kernel, dim3(grid), dim3(256), 0, s, keys, n, st, shifts[p], bits[p], hist);
        hipLaunchKernelGGL(key_pick_kernel, dim3(1), dim3(256), 0, s, st, hist, shifts[p], bits[p]);
    }
    return hipGetLastError();
}

hipError_t read_select_kth(const void *st_dev, uint32_t *kth, hipStream_t s)
{
    SelState h{};
    hipError_t e = hipMemcpyAsync(&h, st_dev, sizeof(h), hipMemcpyDeviceToHost, s);
    if (e != hipSuccess) return e;
    e = hipStreamSynchronize(s);
    *kth = h.prefix;
    return e;
}

size_t select_state_bytes() { return sizeof(SelState); }

// counts[0] = #keys <= t_le, counts[1] = #keys <= t_q, counts[2] = #live keys.
__global__ __launch_bounds__(256) void key_count_kernel(const uint32_t *keys, uint64_t n, uint32_t t_le, uint32_t t_q,
                                                        unsigned long long *counts)
{
    unsigned long long c0 = 0, c1 = 0, c2 = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t k = keys[i];
        c2 += k != ORD_NONE;
        c0 += k != ORD_NONE && k <= t_le;
        c1 += k != ORD_NONE && k <= t_q;
    }
    for (int off = 32; off > 0; off >>= 1) {
        c0 += __shfl_down(c0, off);
        c1 += __shfl_down(c1, off);
        c2 += __shfl_down(c2, off);
    }
    if ((threadIdx.x & 63) == 0) {
        atomicAdd(&counts[0], c0);
        atomicAdd(&counts[1], c1);
        atomicAdd(&counts[2], c2);
    }
}

hipError_t launch_key_count(const uint32_t *keys, uint64_t n, uint32_t t_le, uint32_t t_q, int num_cus,
                            unsigned long long *counts, hipStream_t s)
{
    hipError_t e = hipMemsetAsync(counts, 0, 3 * 8, s);
    if (e != hipSuccess || n == 0) return e;
    const unsigned grid = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((n + 1023) / 1024, (uint64_t)num_cus * 4));
    hipLaunchKernelGGL(key_count_kernel, dim3(grid), dim3(256), 0, s, keys, n, t_le, t_q, counts);
    return hipGetLastError();
}

// ---- S3: compaction -----------------------------------------------------------
// Live keys <= thr (thr from the select state when st != null) ->
// out[atomic] = key << 32 | (slot0 + i).
__global__ __launch_bounds__(256) void key_compact_kernel(const uint32_t *keys, uint64_t n, const SelState *st,
                                                          uint32_t thr, uint32_t slot0, uint64_t *out,
                                                          unsigned long long *count)
{
    if (st) thr = st->prefix;
    const int lane = threadIdx.x & 63;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    // wave-uniform trip count so the ballot sees all 64 lanes
    const uint64_t base0 = (uint64_t)blockIdx.x * blockDim.x + (threadIdx.x & ~63u);
    for (uint64_t base = base0; base < n; base += stride) {
        const uint64_t i = base + lane;
        const uint32_t k = i < n ? keys[i] : ORD_NONE;
        const bool take = k != ORD_NONE && k <= thr;
        const uint64_t bal = __ballot(take);
        if (!bal) continue;
        unsigned long long pos0 = 0;
        if (lane == 0) pos0 = atomicAdd(count, (unsigned long long)__popcll(bal));
        pos0 = __shfl(pos0, 0);
        if (take) {
            const uint64_t below = lane ? (bal & ((1ull << lane) - 1ull)) : 0ull;
            out[pos0 + __popcll(below)] = ((uint64_t)k << 32) | (uint32_t)(slot0 + i);
        }
    }
}

hipError_t launch_key_compact(const uint32_t *keys, uint64_t n, const void *st_dev, uint32_t thr, uint32_t slot0,
                              int num_cus, uint64_t *out, unsigned long long *count, hipStream_t s)
{
    hipError_t e = hipMemsetAsync(count, 0, 8, s);
    if (e != hipSuccess || n == 0) return e;
    const unsigned grid = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((n + 255) / 256, (uint64_t)num_cus * 8));
    hipLaunchKernelGGL(key_compact_kernel, dim3(grid), dim3(256), 0, s, keys, n,
                       reinterpret_cast<const SelState *>(st_dev), thr, slot0, out, count);
    return hipGetLastError();
}

// The heap replay's superset for windows above 256 (wvg_range.hip,
// bq_heap_candidates_select): slot i of chunk j (chunk 0 = [0, R), chunk j >= 1
// = [R 2^(j-1), R 2^j)) is kept iff its key is below thr[j], the R-th smallest
// key of every slot before the chunk (ORD_NONE: fewer than R rows precede, keep
// all) -- a row the reference heap inserts is below the R-th of ITS prefix,
// which is at most thr[j].  Output (slot << 32 | key): sorted, docID order.
__global__ __launch_bounds__(256) void key_compact_chunks_kernel(const uint32_t *keys, uint64_t n, const uint32_t *thr,
                                                                 uint64_t R, uint32_t slot0, uint64_t *out,
                                                                 unsigned long long *count)
{
    const int lane = threadIdx.x & 63;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    const uint64_t base0 = (uint64_t)blockIdx.x * blockDim.x + (threadIdx.x & ~63u);
    for (uint64_t base = base0; base < n; base += stride) {
        const uint64_t i = base + lane;
        const uint32_t k = i < n ? keys[i] : ORD_NONE;
        const uint32_t j = i < R ? 0u : 64u - (uint32_t)__clzll((unsigned long long)(i / R));
        const bool take = k != ORD_NONE && k < thr[j];
        const uint64_t m = __ballot(take);
        if (m == 0ull) continue;
        unsigned long long pos = 0;
        if (lane == 0) pos = atomicAdd(count, (unsigned long long)__popcll(m));
        pos = __shfl(pos, 0, 64);
        const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
        if (take) out[pos + below] = ((uint64_t)(slot0 + (uint32_t)i) << 32) | k;
    }
}

hipError_t launch_key_compact_chunks(const uint32_t *keys, uint64_t n, const uint32_t *thr, uint64_t R, uint32_t slot0,
                                     int num_cus, uint64_t *out, unsigned long long *count, hipStream_t s)
{
    hipError_t e = hipMemsetAsync(count, 0, 8, s);
    if (e != hipSuccess || n == 0) return e;
    const unsigned grid = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((n + 255) / 256, (uint64_t)num_cus * 8));
    hipLaunchKernelGGL(key_compact_chunks_kernel, dim3(grid), dim3(256), 0, s, keys, n, thr, R, slot0, out, count);
    return hipGetLastError();
}

// ---- S4: sort + emit ----------------------------------------------------------
size_t sort_temp_bytes(uint64_t n)
{
    size_t bytes = 0;
    (void)rocprim::radix_sort_keys(nullptr, bytes, (const unsigned long long *)nullptr,
                                   (unsigned long long *)nullptr, (size_t)n, 0, 64, (hipStream_t)0);
    return bytes;
}

hipError_t sort_keys64(void *temp, size_t temp_bytes, const uint64_t *in, uint64_t *out, uint64_t n, hipStream_t s)
{
    if (n == 0) return hipSuccess;
    return rocprim::radix_sort_keys(temp, temp_bytes, reinterpret_cast<const unsigned long long *>(in),
                                    reinterpret_cast<unsigned long long *>(out), (size_t)n, 0, 64, s);
}

__global__ void emit_sorted_kernel(const uint64_t *sorted, uint64_t n, uint64_t id_base, uint64_t *ids, float *dists)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t key = sorted[i];
    ids[i] = id_base + (uint32_t)key;
    dists[i] = wvg_unord_f32((uint32_t)(key >> 32));
}

hipError_t launch_emit_sorted(const uint64_t *sorted, uint64_t n, uint64_t id_base, uint64_t *ids, float *dists,
                              hipStream_t s)
{
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(emit_sorted_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, sorted, n, id_base, ids,
                       dists);
    return hipGetLastError();
}

}  // namespace wvg

// ---------------------------------------------------------------------------
// Distances of one prepared query to corpus rows named by docID: the batched
// form of distancer.Distance / CompressorDistancer.DistanceToNode(id)
// (CH/compression.go:306-325) that HNSW's rescore loop
// (V/hnsw/search.go:564-581) and filtered flat search issue one id at a time.
// One thread per id (a gather); ok[i] = 0 for ids that are not live.
// ---------------------------------------------------------------------------
namespace wvg {

// qidx (nullable): query index of every id -- many queries' candidate lists
// in one launch (a.queries holds nq prepared queries, a.qpitch elements apart).
template <int KIND, int METRIC>
__global__ void dist_by_ids_kernel(ScanArgs a, uint64_t capacity, const uint64_t *ids, uint64_t n, float *out,
                                   uint8_t *ok, const uint32_t *qidx)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    if (qidx)
        a.queries = reinterpret_cast<const char *>(a.queries) +
                    (size_t)qidx[i] * a.qpitch * (KIND == WVG_KIND_BQ ? 8u : 4u);
    const uint64_t id = ids[i];
    const uint64_t slot = id - a.id_base;
    const bool live = id >= a.id_base && slot < capacity && ((a.valid[slot >> 6] >> (slot & 63)) & 1ull);
    float d = 0.0f;
    if (live) {
        const uint64_t t = slot >> 6, lane = slot & 63;
        if constexpr (KIND == WVG_KIND_F32) {
            const float4 *rp = reinterpret_cast<const float4 *>(a.data) + (size_t)t * a.nchunks * 64 + lane;
            d = wrap_metric(a.metric, row_dist<METRIC, 64>(rp, reinterpret_cast<const float4 *>(a.queries),
                                                           (int)a.dim, a.order512));
        } else if constexpr (KIND == WVG_KIND_BQ) {
            const ulonglong2 *rp = reinterpret_cast<const ulonglong2 *>(a.data) + (size_t)t * a.nchunks * 64 + lane;
            const uint64_t *q = reinterpret_cast<const uint64_t *>(a.queries);
            uint32_t tot = 0;
            for (uint32_t c = 0; c < a.nchunks; c++) {
                const ulonglong2 x = rp[(size_t)c * 64];
                tot += (uint32_t)__popcll(x.x ^ q[2 * c]) + (uint32_t)__popcll(x.y ^ q[2 * c + 1]);
            }
            d = (float)tot;
        } else {
            const uint4 *rp = reinterpret_cast<const uint4 *>(a.data) + (size_t)t * a.nchunks * 64 + lane;
            const float *lut = reinterpret_cast<const float *>(a.queries);
            d = wrap_metric(a.metric, pq_row_sum(rp, a.nchunks, a.pq_m, a.pq_ks, lut, slot));
        }
    }
    out[i] = d;
    ok[i] = live ? 1 : 0;
}

hipError_t launch_dist_by_ids(const ScanArgs &a, int kind, uint64_t capacity, const uint64_t *ids, uint64_t n,
                              float *out, uint8_t *ok, hipStream_t s, const uint32_t *qidx)
{
    if (n == 0) return hipSuccess;
    dim3 grid((unsigned)((n + 255) / 256)), block(256);
    if (kind == WVG_KIND_F32) {
        with_metric(a.metric, [&](auto M) {
            hipLaunchKernelGGL((dist_by_ids_kernel<WVG_KIND_F32, decltype(M)::value>), grid, block, 0, s, a, capacity,
                               ids, n, out, ok, qidx);
        });
    } else if (kind == WVG_KIND_BQ) {
        hipLaunchKernelGGL((dist_by_ids_kernel<WVG_KIND_BQ, 0>), grid, block, 0, s, a, capacity, ids, n, out, ok, qidx);
    } else {
        hipLaunchKernelGGL((dist_by_ids_kernel<WVG_KIND_PQ, 0>), grid, block, 0, s, a, capacity, ids, n, out, ok, qidx);
    }
    return hipGetLastError();
}

}  // namespace wvg
