// wvg_gemm.hip -- K3: batched multi-query scoring on fp32 MFMA, fused with
// per-query top-k.
//
// Reference path: Q independent flat.searchByVector calls (V/flat/index.go:319)
// over the same rows, each SingleDist = dot_256 (D/c/dot_avx256_amd64.c:14) or
// l2_256.  Scoring Q queries against N rows is the dense contraction
// S = Q_mat * X^T (2*Q*N*d FLOP); it runs on v_mfma_f32_16x16x4_f32, whose
// result is bit-for-bit a k-ordered fp32 fmaf chain (MI355X_MICROARCH.md,
// Matrix cores).  The AVX2 kernel keeps 32 independent fma chains ("slices"
// s = 8j + l: elements 32b + s, b = 0..d/32-1) and folds them with a fixed
// tree; here every slice gets its own 16x16 accumulator, the MFMA's K = 4
// steps are 4 consecutive blocks b of that slice, and the epilogue applies the
// same tree -- so dot products are bit-identical to the CPU distancer.
// Squared L2 is not a plain contraction in the reference's order (it squares
// differences), so this kernel serves dot and cosine-dot (BASELINE config 2);
// L2 batches use K1.
//
// Workgroup: 8 waves, tile = 32 queries x 64 rows (one corpus tile); each
// wave owns a 16x16 sub-tile with 32 slice accumulators (128 acc VGPRs).
// K is staged in 128-position chunks (4 blocks x 32 slices) through LDS,
// double-buffered with register prefetch.  After each row tile the 32x64
// distance keys go through LDS to the per-query wave top-k (4 queries/wave).
// Roofline: MFMA fp32 (157.3 TFLOP/s dense), 2*Q*N*d FLOP per batch.
#include "wvg_internal.hpp"
#include "wvg_topk.hpp"

namespace wvg {

typedef float floatx4 __attribute__((ext_vector_type(4)));

constexpr int GQ = 32;        // queries per workgroup tile
constexpr int GR = 64;        // rows per workgroup tile (one corpus tile)
constexpr int GWAVES = 8;     // 2 (query) x 4 (row) sub-tiles of 16x16
constexpr int GCH = 128;      // positions per K chunk (4 blocks x 32 slices)
constexpr int GSTRIDE = 132;  // LDS row stride in floats (pad: conflict-free ds_read_b128)

struct GemmArgs {
    const float4 *data;     // tiled corpus
    const uint64_t *valid;  // one word per tile
    const uint64_t *allow;
    uint64_t allow_words;
    uint64_t id_base;
    uint64_t tile_begin, tile_end;
    uint32_t dim, nchunks;  // nchunks: float4 chunks per row in the corpus layout
    int metric;
    const float *queries;   // [nq][dim] row-major, 16-byte aligned rows (dim % 32 == 0)
    uint32_t nq, k;
    uint32_t nqb, nrr;      // query blocks, row ranges
};

template <int E>
__global__ __launch_bounds__(GWAVES * 64) void gemm_topk_kernel(GemmArgs a, uint64_t *partials)
{
    extern __shared__ __attribute__((aligned(16))) float smem[];
    // buffer b: queries at smem + b*(GQ+GR)*GSTRIDE, rows right after them
    uint64_t *keys = reinterpret_cast<uint64_t *>(smem + 2 * (GQ + GR) * GSTRIDE);  // [GQ][GR]

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wq = wave & 1, wr = wave >> 1;

    // XCD-aware mapping: the nqb query blocks of one row range share an XCD
    // (blocks b and b+8 share one), so a row tile is fetched from HBM once per XCD.
    const uint32_t b = blockIdx.x;
    uint32_t qb, rr;
    if (a.nrr % 8 == 0) {
        const uint32_t xcd = b % 8, w = b / 8;
        qb = w % a.nqb;
        rr = (w / a.nqb) * 8 + xcd;
    } else {
        qb = b % a.nqb;
        rr = b / a.nqb;
    }
    const uint64_t ntiles = a.tile_end - a.tile_begin;
    const uint64_t t0 = a.tile_begin + ntiles * rr / a.nrr, t1 = a.tile_begin + ntiles * (rr + 1) / a.nrr;
    const uint32_t q0 = qb * GQ;
    const uint32_t nb = a.dim / 32;               // 32-float blocks
    const uint32_t nk = (nb + 3) / 4;             // K chunks of 4 blocks

    WaveTopK<E> tk[4];
#pragma unroll
    for (int i = 0; i < 4; i++) tk[i].init((int)a.k);

    // staging: (GQ + GR) rows x 32 float4 per chunk = 3072 float4 / 512 threads = 6 per thread
    constexpr int PER = (GQ + GR) * (GCH / 4) / (GWAVES * 64);
    float4 pf[PER];
    auto load_chunk = [&](uint64_t t, uint32_t kc) {
#pragma unroll
        for (int i = 0; i < PER; i++) {
            const int idx = tid + i * GWAVES * 64;  // 0 .. 3071
            const int row = idx >> 5, c4 = idx & 31;  // row within (queries ++ rows), float4 within chunk
            const uint32_t pos = kc * GCH + c4 * 4;
            float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
            if (pos < a.dim) {
                if (row < GQ) {
                    const uint32_t q = q0 + row;
                    if (q < a.nq) v = *reinterpret_cast<const float4 *>(a.queries + (size_t)q * a.dim + pos);
                } else {
                    const int r = row - GQ;
                    v = a.data[((size_t)t * a.nchunks + (pos >> 2)) * 64 + r];
                }
            }
            pf[i] = v;
        }
    };
    auto store_chunk = [&](int buf) {
#pragma unroll
        for (int i = 0; i < PER; i++) {
            const int idx = tid + i * GWAVES * 64;
            const int row = idx >> 5, c4 = idx & 31;
            float *dst = smem + buf * (GQ + GR) * GSTRIDE + row * GSTRIDE;
            *reinterpret_cast<float4 *>(dst + c4 * 4) = pf[i];
        }
    };

    const int qrow = wq * 16 + (lane & 15);  // A operand row (query) in the tile
    const int rrow = wr * 16 + (lane & 15);  // B operand row (corpus row) in the tile
    const int kk = lane >> 4;                // K index within an MFMA = block within the chunk

    for (uint64_t t = t0; t < t1; ++t) {
        uint64_t m = a.valid[t];
        if (a.allow) {
            const uint64_t w = (a.id_base >> 6) + t;
            m &= w < a.allow_words ? a.allow[w] : 0ull;
        }
        if (m == 0ull) continue;  // uniform
        floatx4 acc[32];
#pragma unroll
        for (int s = 0; s < 32; s++) acc[s] = (floatx4){0.f, 0.f, 0.f, 0.f};
        load_chunk(t, 0);
        store_chunk(0);
        __syncthreads();
        for (uint32_t kc = 0; kc < nk; kc++) {
            const int cur = kc & 1;
            if (kc + 1 < nk) load_chunk(t, kc + 1);  // prefetch into registers
            const float *qa = smem + cur * (GQ + GR) * GSTRIDE + qrow * GSTRIDE + kk * 32;
            const float *rb = smem + cur * (GQ + GR) * GSTRIDE + (GQ + rrow) * GSTRIDE + kk * 32;
#pragma unroll
            for (int g = 0; g < 8; g++) {
                const float4 av = *reinterpret_cast<const float4 *>(qa + g * 4);
                const float4 bv = *reinterpret_cast<const float4 *>(rb + g * 4);
                acc[4 * g + 0] = __builtin_amdgcn_mfma_f32_16x16x4f32(av.x, bv.x, acc[4 * g + 0], 0, 0, 0);
                acc[4 * g + 1] = __builtin_amdgcn_mfma_f32_16x16x4f32(av.y, bv.y, acc[4 * g + 1], 0, 0, 0);
                acc[4 * g + 2] = __builtin_amdgcn_mfma_f32_16x16x4f32(av.z, bv.z, acc[4 * g + 2], 0, 0, 0);
                acc[4 * g + 3] = __builtin_amdgcn_mfma_f32_16x16x4f32(av.w, bv.w, acc[4 * g + 3], 0, 0, 0);
            }
            if (kc + 1 < nk) store_chunk(cur ^ 1);
            __syncthreads();
        }
        // epilogue: AVX2 reduction tree per output element (D/c/dot_avx256_amd64.c:94-103)
        // C/D layout: col = lane & 15 (row j), row = (lane >> 4) * 4 + r (query i)
#pragma unroll
        for (int r = 0; r < 4; r++) {
            float s[8];
#pragma unroll
            for (int l = 0; l < 8; l++) {
                const float a01 = acc[8 + l][r] + acc[l][r];
                const float a23 = acc[24 + l][r] + acc[16 + l][r];
                s[l] = a23 + a01;
            }
            const float lo = (s[0] + s[1]) + (s[2] + s[3]);
            const float hi = (s[4] + s[5]) + (s[6] + s[7]);
            const float dot = 0.0f + (lo + hi);
            const float dist = a.metric == WVG_M_DOT ? -dot : 1.0f - dot;
            const int qi = wq * 16 + (lane >> 4) * 4 + r;
            const int j = wr * 16 + (lane & 15);
            keys[qi * GR + j] = ((m >> j) & 1ull) ? wvg_make_key(dist, (uint32_t)(t * 64 + j)) : WVG_KEY_NONE;
        }
        __syncthreads();
#pragma unroll
        for (int i = 0; i < 4; i++) tk[i].offer(keys[(wave * 4 + i) * GR + lane]);
        __syncthreads();
    }
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const uint32_t q = q0 + wave * 4 + i;
        if (q >= a.nq) continue;
        uint64_t *out = partials + ((size_t)q * a.nrr + rr) * a.k;
#pragma unroll
        for (int e = 0; e < E; e++) {
            const int idx = e * 64 + lane;
            if (idx < (int)a.k) out[idx] = tk[i].l[e];
        }
    }
}

bool gemm_supported(uint32_t dim, int metric) { return dim % 32 == 0 && dim > 0 && metric != WVG_M_L2; }

uint32_t gemm_row_ranges(uint32_t nq, uint64_t ntiles, int num_cus)
{
    const uint32_t nqb = (nq + GQ - 1) / GQ;
    uint64_t want = ((uint64_t)num_cus + nqb - 1) / nqb;  // about one workgroup per CU
    want = (want + 7) / 8 * 8;
    if (want > ntiles) want = ntiles;
    if (want < 1) want = 1;
    return (uint32_t)want;
}

hipError_t launch_gemm_topk(const ScanArgs &s, uint32_t nrr, uint64_t *partials, hipStream_t st)
{
    GemmArgs a{};
    a.data = reinterpret_cast<const float4 *>(s.data);
    a.valid = s.valid;
    a.allow = s.allow;
    a.allow_words = s.allow_words;
    a.id_base = s.id_base;
    a.tile_begin = s.tile_begin;
    a.tile_end = s.tile_end;
    a.dim = s.dim;
    a.nchunks = s.nchunks;
    a.metric = s.metric;
    a.queries = reinterpret_cast<const float *>(s.queries);
    a.nq = s.nq;
    a.k = s.k;
    a.nqb = (s.nq + GQ - 1) / GQ;
    a.nrr = nrr;
    const size_t lds = (size_t)2 * (GQ + GR) * GSTRIDE * 4 + (size_t)GQ * GR * 8;
    dim3 grid(a.nqb * a.nrr), block(GWAVES * 64);
    if (s.k <= 64)
        launch_timed((gemm_topk_kernel<1>), grid, block, lds, st, a, partials);
    else if (s.k <= 128)
        launch_timed((gemm_topk_kernel<2>), grid, block, lds, st, a, partials);
    else
        launch_timed((gemm_topk_kernel<4>), grid, block, lds, st, a, partials);
    return hipGetLastError();
}

}  // namespace wvg
