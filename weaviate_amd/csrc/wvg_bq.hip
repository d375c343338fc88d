// wvg_bq.hip -- binary quantization on MI355X.
//
// K4 encode: BinaryQuantizer.Encode (CH/binary_quantization.go:32-45): bit j%64
//   of word j/64 is set iff v[j] < 0 (of the normalized vector for cosine,
//   V/flat/index.go:258,262-263).
// K5 scan:   DistanceBetweenCompressedVectors (CH/binary_quantization.go:47-56)
//   = sum of popcount(x ^ q) over words, fused with the wave top-k (the
//   findTopVectorsCached heap, V/flat/index.go:456-495).  Roofline: HBM,
//   N * 8 * ceil(d/64) bytes per query.
// Tiled layout: [tile][pair c][lane][2 x u64] -- one 16-byte load per lane per
// word pair, 1 KiB per wave-instruction; the query code is wave-uniform.
#include "wvg_internal.hpp"
#include "wvg_topk.hpp"

namespace wvg {

constexpr int BQ_WAVES = BQ_SCAN_WAVES;

__device__ __forceinline__ uint64_t bq_tile_mask(const ScanArgs &a, uint64_t t)
{
    uint64_t m = a.valid[t];
    if (a.allow) {
        uint64_t w = t - a.allow_t0;  // allow[0] is tile allow_t0's word
        m &= w < a.allow_words ? a.allow[w] : 0ull;
    }
    return m;
}

typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ u64x2 ld_codes(const u64x2 *p) { return __builtin_nontemporal_load(p); }

// K5: one wave per 64-row tile at a time (lane = row), XOR + popcount over
// the tile's 16-byte chunks.  Fixed NCH: the next live tile's chunks are
// loaded (non-temporal) while the current tile is reduced and offered, so a
// wave keeps two tiles' codes in flight; tile masks are scalar and prefetched.
// COS (a batch, ScanArgs::cosched): the 1D grid's consecutive ids on one XCD
// are the nq queries of one row range, which read the same codes side by side
// from that XCD's L2 (default-policy loads; K8e COS in wvg_pq.hip).
// EMIT (the heap replay, wvg_replay.hip): each wave also records the keys of
// the rows the reference's heap could insert (WaveTopK::offer_dist_emit):
// 1 = into an LDS buffer of emit_cap keys per wave (dynamic shared memory),
// copied to a.emit after the scan loop; 2 = straight into a.emit (the rerun
// with buffers as large as the wave's rows).
template <int E, int NCH, bool COS = false, int EMIT = 0>
__global__ __launch_bounds__(BQ_WAVES * 64) void scan_bq_kernel(ScanArgs a, uint64_t *partials)
{
    extern __shared__ uint64_t emit_lds[];
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint32_t qi = blockIdx.y, rng = blockIdx.x, G = gridDim.x;
    if constexpr (COS) {
        G = gridDim.x / a.nq;
        const uint32_t kk = blockIdx.x >> 3;
        rng = (kk / a.nq) * 8u + (blockIdx.x & 7u);
        qi = kk % a.nq;
    }
    auto ld = [](const u64x2 *p) -> u64x2 {
        if constexpr (COS)
            return *p;
        else
            return ld_codes(p);
    };
    const uint64_t *q = reinterpret_cast<const uint64_t *>(a.queries) + (size_t)qi * a.qpitch;
    const u64x2 *data = reinterpret_cast<const u64x2 *>(a.data);
    const uint32_t nch = NCH > 0 ? (uint32_t)NCH : a.nchunks;
    const uint64_t ntiles = a.tile_end - a.tile_begin;
    const uint64_t total = (uint64_t)G * BQ_WAVES;
    const uint64_t gw = (uint64_t)rng * BQ_WAVES + wave;
    const uint64_t t0 = a.tile_begin + ntiles * gw / total, t1 = a.tile_begin + ntiles * (gw + 1) / total;
    WaveTopK<E> tk;
    tk.init((int)a.k);
    tk.init_fast();
    uint64_t *ebuf = nullptr;
    uint32_t ecnt = 0;
    float eseed = __builtin_inff();
    if constexpr (EMIT != 0) {
        ebuf = EMIT == 1 ? emit_lds + (size_t)wave * a.emit_cap : a.emit + ((size_t)qi * total + gw) * a.emit_cap;
        if (a.emit_seed) eseed = a.emit_seed[(size_t)qi * G + rng];
    }
    if constexpr (NCH > 0) {
        // next live tile at or after t (wave-uniform), its mask in m
        auto next_live = [&](uint64_t t, uint64_t &m) {
            for (; t < t1; ++t) {
                m = bq_tile_mask(a, t);
                if (m) break;
            }
            return t;
        };
        uint64_t m_cur = 0, m_nxt = 0;
        uint64_t t = next_live(t0, m_cur);
        u64x2 cur[NCH], nxt[NCH];
        if (t < t1) {
            const u64x2 *rp = data + (size_t)t * NCH * 64 + lane;
#pragma unroll
            for (int c = 0; c < NCH; c++) cur[c] = ld(rp + (size_t)c * 64);
        }
        while (t < t1) {
            const uint64_t tn = next_live(t + 1, m_nxt);
            if (tn < t1) {
                const u64x2 *rp = data + (size_t)tn * NCH * 64 + lane;
#pragma unroll
                for (int c = 0; c < NCH; c++) nxt[c] = ld(rp + (size_t)c * 64);
            }
            uint32_t tot = 0;
#pragma unroll
            for (int c = 0; c < NCH; c++)
                tot += (uint32_t)__popcll(cur[c].x ^ q[2 * c]) + (uint32_t)__popcll(cur[c].y ^ q[2 * c + 1]);
            const float dist = (float)tot;  // exact: sum of float32(popcount) is an integer < 2^24
            // rejection on the float distance first: the key is built only when some lane passes
            if constexpr (EMIT != 0)
                tk.offer_dist_emit(dist, (uint32_t)(t * 64 + lane), m_cur, eseed, ebuf, ecnt, a.emit_cap);
            else
                tk.offer_dist_fast(dist, (uint32_t)(t * 64 + lane), m_cur);
#pragma unroll
            for (int c = 0; c < NCH; c++) cur[c] = nxt[c];
            t = tn;
            m_cur = m_nxt;
        }
    } else {
        for (uint64_t t = t0; t < t1; ++t) {
            const uint64_t m = bq_tile_mask(a, t);
            if (m == 0ull) continue;
            const u64x2 *rp = data + (size_t)t * nch * 64 + lane;
            uint32_t tot = 0;
            for (uint32_t c = 0; c < nch; c++) {
                const u64x2 x = ld(rp + (size_t)c * 64);
                tot += (uint32_t)__popcll(x.x ^ q[2 * c]) + (uint32_t)__popcll(x.y ^ q[2 * c + 1]);
            }
            const float dist = (float)tot;
            if constexpr (EMIT != 0)
                tk.offer_dist_emit(dist, (uint32_t)(t * 64 + lane), m, eseed, ebuf, ecnt, a.emit_cap);
            else
                tk.offer_dist_fast(dist, (uint32_t)(t * 64 + lane), m);
        }
    }
    if constexpr (EMIT != 0) {
        if constexpr (EMIT == 1) {  // the wave's LDS record to its global buffer (after every load)
            uint64_t *g = a.emit + ((size_t)qi * total + gw) * a.emit_cap;
            const uint32_t n = min(ecnt, a.emit_cap);
            for (uint32_t i = (uint32_t)lane; i < n; i += 64) g[i] = ebuf[i];
        }
        if (lane == 0) a.emit_cnt[(size_t)qi * total + gw] = ecnt;
    }
    group_combine_store<E, BQ_WAVES>(tk, partials + ((size_t)qi * G + rng) * a.k);
}

template <int E, bool COS, int EMIT>
static hipError_t launch_bq_ec(const ScanArgs &a, uint64_t *partials, int groups, hipStream_t s)
{
    const dim3 grid = COS ? dim3((unsigned)groups * a.nq) : dim3(groups, a.nq), block(BQ_WAVES * 64);
    const uint32_t lds = EMIT == 1 ? (uint32_t)(BQ_WAVES * a.emit_cap * 8) : 0u;
    switch (a.nchunks) {
    case 1: launch_timed((scan_bq_kernel<E, 1, COS, EMIT>), grid, block, lds, s, a, partials); break;   // d <= 128
    case 6: launch_timed((scan_bq_kernel<E, 6, COS, EMIT>), grid, block, lds, s, a, partials); break;   // d = 768
    case 12: launch_timed((scan_bq_kernel<E, 12, COS, EMIT>), grid, block, lds, s, a, partials); break; // d = 1536
    default: launch_timed((scan_bq_kernel<E, 0, COS, EMIT>), grid, block, lds, s, a, partials); break;
    }
    return hipGetLastError();
}

template <int E, int EMIT>
static hipError_t launch_bq_e(const ScanArgs &a, uint64_t *partials, int groups, hipStream_t s)
{
    if (a.cosched && a.nq > 1 && groups % 8 == 0) return launch_bq_ec<E, true, EMIT>(a, partials, groups, s);
    return launch_bq_ec<E, false, EMIT>(a, partials, groups, s);
}

template <int EMIT>
static hipError_t launch_bq_k(const ScanArgs &a, uint64_t *partials, int groups, hipStream_t s)
{
    if (a.k <= 64) return launch_bq_e<1, EMIT>(a, partials, groups, s);
    if (a.k <= 128) return launch_bq_e<2, EMIT>(a, partials, groups, s);
    return launch_bq_e<4, EMIT>(a, partials, groups, s);
}

hipError_t launch_scan_bq(const ScanArgs &a, uint64_t *partials, int groups, hipStream_t s)
{
    return launch_bq_k<0>(a, partials, groups, s);
}

hipError_t launch_scan_bq_emit(const ScanArgs &a, uint64_t *partials, int groups, bool lds, hipStream_t s)
{
    if (!a.emit || !a.emit_cnt || a.k == 0 || a.k > 256) return hipErrorInvalidValue;
    if (lds && (size_t)BQ_WAVES * a.emit_cap * 8 > BQ_EMIT_LDS_MAX) return hipErrorInvalidValue;
    return lds ? launch_bq_k<1>(a, partials, groups, s) : launch_bq_k<2>(a, partials, groups, s);
}

// Encode row-major float rows; `normalize` is applied per row first (cosine).
// One thread per (row, word).  Rows must already be normalized by the caller
// when normalize == 0 is passed for cosine corpora.
__global__ void bq_encode_kernel(const float *rows, uint64_t n, uint32_t dim, uint64_t *codes)
{
    const uint32_t w = bq_words(dim);
    const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= n * w) return;
    const uint64_t i = g / w;
    const uint32_t word = (uint32_t)(g % w);
    const float *v = rows + i * dim;
    uint64_t code = 0;
    const uint32_t j0 = word * 64, j1 = min(dim, j0 + 64);
    for (uint32_t j = j0; j < j1; j++)
        if (v[j] < 0.0f) code |= 1ull << (j & 63);
    codes[g] = code;
}

hipError_t launch_bq_encode_rows(const float *rows, uint64_t n, uint32_t dim, int normalize, uint64_t *codes,
                                 hipStream_t s)
{
    (void)normalize;
    const uint64_t total = n * bq_words(dim);
    if (total == 0) return hipSuccess;
    hipLaunchKernelGGL(bq_encode_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, rows, n, dim, codes);
    return hipGetLastError();
}

__global__ void bq_store_kernel(const uint64_t *codes, const uint64_t *slots, uint64_t n, uint32_t words,
                                uint32_t nchunks, ulonglong2 *tiled)
{
    const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= n * nchunks) return;
    const uint64_t i = g / nchunks;
    const uint32_t c = (uint32_t)(g % nchunks);
    const uint64_t slot = slots ? slots[i] : i;
    const uint64_t *src = codes + i * words;
    ulonglong2 v;
    v.x = 2 * c < words ? src[2 * c] : 0ull;
    v.y = 2 * c + 1 < words ? src[2 * c + 1] : 0ull;
    tiled[((slot >> 6) * nchunks + c) * 64 + (slot & 63)] = v;
}

hipError_t launch_bq_store(const uint64_t *codes, const uint64_t *slots, uint64_t n, uint32_t words,
                           uint32_t nchunks, uint64_t *tiled, hipStream_t s)
{
    const uint64_t total = n * nchunks;
    if (total == 0) return hipSuccess;
    hipLaunchKernelGGL(bq_store_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, codes, slots, n,
                       words, nchunks, reinterpret_cast<ulonglong2 *>(tiled));
    return hipGetLastError();
}

// Synthetic BQ rows: encode(normalize?(synth row)) generated in place.
__global__ void bq_synth_kernel(uint64_t seed_mixed, int dist, uint64_t row0, uint64_t n, uint64_t slot0,
                                uint32_t dim, uint32_t nchunks, int normalize, ulonglong2 *tiled)
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
    ulonglong2 *dst = tiled + ((slot >> 6) * nchunks) * 64 + (slot & 63);
    for (uint32_t c = 0; c < nchunks; c++) {
        uint64_t w2[2] = {0ull, 0ull};
        for (int h = 0; h < 2; h++) {
            const uint32_t j0 = (2 * c + h) * 64;
            for (uint32_t j = j0; j < j0 + 64 && j < dim; j++) {
                float x = wvg_synth_value(seed_mixed, row, j, dist);
                if (normalize) x = zero ? 0.0f : x / norm;
                if (x < 0.0f) w2[h] |= 1ull << (j & 63);
            }
        }
        ulonglong2 v;
        v.x = w2[0];
        v.y = w2[1];
        dst[(size_t)c * 64] = v;
    }
}

hipError_t launch_bq_synth(uint64_t seed, int dist, uint64_t row0, uint64_t n, uint64_t slot0, uint32_t dim,
                           uint32_t nchunks, int normalize, uint64_t *tiled, hipStream_t s)
{
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(bq_synth_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, wvg_mix64(seed), dist,
                       row0, n, slot0, dim, nchunks, normalize, reinterpret_cast<ulonglong2 *>(tiled));
    return hipGetLastError();
}

__global__ void bq_distance_rows_kernel(const uint64_t *q, const uint64_t *codes, uint64_t n, uint32_t words,
                                        float *out)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t *x = codes + i * words;
    float total = 0.0f;
    for (uint32_t w = 0; w < words; w++) total += (float)__popcll(x[w] ^ q[w]);
    out[i] = total;
}

hipError_t launch_bq_distance_rows(const uint64_t *q, const uint64_t *codes, uint64_t n, uint32_t words,
                                   float *out, hipStream_t s)
{
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(bq_distance_rows_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, q, codes, n,
                       words, out);
    return hipGetLastError();
}

}  // namespace wvg
