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
// double-buffered, fed by a register prefetch two chunks deep that runs across
// row-tile boundaries.  After each row tile the 32x64
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
constexpr int GBLK = 36;      // LDS floats per 32-position block (4 pad)
constexpr int GSTRIDE = 152;  // LDS row stride in floats: with GBLK, the MFMA operand ds_read_b128s
                              // of every lane group hit 16 distinct 4-bank sets (conflict-free)

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

// PF = chunks of prefetch in registers (2: 48 staging VGPRs; E > 1 top-k
// lists leave room for 1 only).
// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS ops,
// not for its global loads, so the chunk prefetch stays in flight across it
// (__syncthreads() would also drain vmcnt; cdna_hip_programming.md "step-3
// structure" ceiling).
__device__ __forceinline__ void lds_barrier()
{
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

__device__ __forceinline__ uint64_t sload64(const uint64_t *p)
{
    uint64_t v;
    asm volatile("s_load_dwordx2 %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v) : "s"(p) : "memory");
    return v;
}

template <int E, int PF>
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
    static_assert(GQ * (GCH / 4) == 2 * GWAVES * 64, "staging slots 0-1 are query rows, 2.. corpus rows");
    // Branch-free: every address is valid (positions past dim read position 0,
    // query rows past nq read the last query, units past the range read tile
    // t0) and the out-of-range values are zeroed at store time, so the
    // compiler's vmcnt tracking stays exact and chunk u+2's loads stay in
    // flight while chunk u+1 is parked.
    auto load_chunk = [&](float4 (&pf)[PER], uint64_t t, uint32_t kc) {
#pragma unroll
        for (int i = 0; i < PER; i++) {
            const int idx = tid + i * GWAVES * 64;  // 0 .. 3071
            const int row = idx >> 5, c4 = idx & 31;  // row within (queries ++ rows), float4 within chunk
            uint32_t pos = kc * GCH + c4 * 4;
            pos = pos < a.dim ? pos : 0u;
            if (i < 2) {
                const uint32_t q = min(q0 + (uint32_t)row, a.nq - 1);
                pf[i] = *reinterpret_cast<const float4 *>(a.queries + (size_t)q * a.dim + pos);
            } else {
                pf[i] = a.data[((size_t)t * a.nchunks + (pos >> 2)) * 64 + (row - GQ)];
            }
        }
    };
    auto store_chunk = [&](const float4 (&pf)[PER], int buf, uint32_t kc) {
#pragma unroll
        for (int i = 0; i < PER; i++) {
            const int idx = tid + i * GWAVES * 64;
            const int row = idx >> 5, c4 = idx & 31;
            const bool in = kc * GCH + c4 * 4 < a.dim;
            float *dst = smem + buf * (GQ + GR) * GSTRIDE + row * GSTRIDE;
            *reinterpret_cast<float4 *>(dst + (c4 >> 3) * GBLK + (c4 & 7) * 4) =
                in ? pf[i] : make_float4(0.f, 0.f, 0.f, 0.f);
        }
    };
    // Tile masks through the scalar cache (the words are read-only in this
    // launch): a vector load here would make the compiler drain vmcnt(0), and
    // with it the chunk prefetch, at every tile boundary.
    auto tile_live = [&](uint64_t t) {
        uint64_t m = sload64(a.valid + t);
        if (a.allow) {
            const uint64_t w = (a.id_base >> 6) + t;
            m &= w < a.allow_words ? sload64(a.allow + w) : 0ull;
        }
        return m;
    };
    // The (tile, chunk) units of this workgroup form one stream: chunk u is
    // computed from LDS while chunk u+1 waits in registers and chunk u+2's
    // loads are in flight, across tile boundaries (two chunks of cover for
    // the global-load latency).  Tiles with no live/allowed row are skipped.
    auto next_live = [&](uint64_t t, uint64_t &m) {
        for (; t < t1; ++t) {
            m = tile_live(t);
            if (m) break;
        }
        return t;
    };
    struct Unit {
        uint64_t t, m;
        uint32_t kc;
    };
    auto advance = [&](Unit u) {
        if (u.t >= t1) return u;
        if (u.kc + 1 < nk) {
            u.kc++;
            return u;
        }
        u.kc = 0;
        u.t = next_live(u.t + 1, u.m);
        return u;
    };

    const int qrow = wq * 16 + (lane & 15);  // A operand row (query) in the tile
    const int rrow = wr * 16 + (lane & 15);  // B operand row (corpus row) in the tile
    const int kk = lane >> 4;                // K index within an MFMA = block within the chunk

    Unit u0;
    u0.kc = 0;
    u0.m = 0;
    u0.t = next_live(t0, u0.m);
    if (u0.t < t1) {
        float4 pa[PER], pb[PER];
        Unit u1 = advance(u0), u2 = advance(u1);
        auto load_unit = [&](float4 (&pf)[PER], const Unit &u) {
            load_chunk(pf, u.t < t1 ? u.t : t0, u.t < t1 ? u.kc : 0u);
        };
        load_chunk(pa, u0.t, u0.kc);
        store_chunk(pa, 0, u0.kc);
        load_unit(pa, u1);
        if (PF == 2) load_unit(pb, u2);
        __syncthreads();
        floatx4 acc[32];
        int cur = 0;
        // 32 MFMAs of one chunk; the operand fragments of step g+1 are read
        // from LDS before the MFMAs of step g issue (register double buffer).
        auto mfma_chunk = [&]() {
            const float *qa = smem + cur * (GQ + GR) * GSTRIDE + qrow * GSTRIDE + kk * GBLK;
            const float *rb = smem + cur * (GQ + GR) * GSTRIDE + (GQ + rrow) * GSTRIDE + kk * GBLK;
            float4 av[2], bv[2];
            av[0] = *reinterpret_cast<const float4 *>(qa);
            bv[0] = *reinterpret_cast<const float4 *>(rb);
#pragma unroll
            for (int g = 0; g < 8; g++) {
                if (g + 1 < 8) {
                    av[(g + 1) & 1] = *reinterpret_cast<const float4 *>(qa + (g + 1) * 4);
                    bv[(g + 1) & 1] = *reinterpret_cast<const float4 *>(rb + (g + 1) * 4);
                }
                const float4 x = av[g & 1], y = bv[g & 1];
                acc[4 * g + 0] = __builtin_amdgcn_mfma_f32_16x16x4f32(x.x, y.x, acc[4 * g + 0], 0, 0, 0);
                acc[4 * g + 1] = __builtin_amdgcn_mfma_f32_16x16x4f32(x.y, y.y, acc[4 * g + 1], 0, 0, 0);
                acc[4 * g + 2] = __builtin_amdgcn_mfma_f32_16x16x4f32(x.z, y.z, acc[4 * g + 2], 0, 0, 0);
                acc[4 * g + 3] = __builtin_amdgcn_mfma_f32_16x16x4f32(x.w, y.w, acc[4 * g + 3], 0, 0, 0);
            }
        };
        // One chunk: compute from LDS[cur], park the registers of chunk u+1
        // in LDS[cur^1], refill the freed registers (PF = 2: with chunk u+2;
        // the two register sets alternate roles, so nothing is copied).
        auto body = [&](float4 (&rnow)[PER]) -> bool {
            if (u0.kc == 0) {
#pragma unroll
                for (int sl = 0; sl < 32; sl++) acc[sl] = (floatx4){0.f, 0.f, 0.f, 0.f};
            }
            mfma_chunk();
            const bool more = u1.t < t1;
            if (more) store_chunk(rnow, cur ^ 1, u1.kc);  // chunk u+1 -> the other buffer
            if (u0.kc + 1 == nk) {
                // epilogue: AVX2 reduction tree per output element (D/c/dot_avx256_amd64.c:94-103)
                // C/D layout: col = lane & 15 (row j), row = (lane >> 4) * 4 + r (query i)
                const uint64_t t = u0.t, m = u0.m;
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    float sv[8];
#pragma unroll
                    for (int l = 0; l < 8; l++) {
                        const float a01 = acc[8 + l][r] + acc[l][r];
                        const float a23 = acc[24 + l][r] + acc[16 + l][r];
                        sv[l] = a23 + a01;
                    }
                    const float lo = (sv[0] + sv[1]) + (sv[2] + sv[3]);
                    const float hi = (sv[4] + sv[5]) + (sv[6] + sv[7]);
                    const float dot = 0.0f + (lo + hi);
                    const float dist = a.metric == WVG_M_DOT ? -dot : 1.0f - dot;
                    const int qi = wq * 16 + (lane >> 4) * 4 + r;
                    const int j = wr * 16 + (lane & 15);
                    keys[qi * GR + j] = ((m >> j) & 1ull) ? wvg_make_key(dist, (uint32_t)(t * 64 + j)) : WVG_KEY_NONE;
                }
                lds_barrier();
#pragma unroll
                for (int i = 0; i < 4; i++) tk[i].offer(keys[(wave * 4 + i) * GR + lane]);
            }
            lds_barrier();
            if (!more) return false;
            u0 = u1;
            u1 = u2;
            u2 = advance(u2);
            if constexpr (PF == 2)
                load_unit(rnow, u2);
            else
                load_unit(rnow, u1);
            __builtin_amdgcn_sched_barrier(0);  // keep the prefetch issued here, ahead of the next chunk
            cur ^= 1;
            return true;
        };
        if constexpr (PF == 2) {
            while (body(pa) && body(pb)) {
            }
        } else {
            while (body(pa)) {
            }
        }
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
        if (tuning().gemm_pf == 1)
            launch_timed((gemm_topk_kernel<1, 1>), grid, block, lds, st, a, partials);
        else
            launch_timed((gemm_topk_kernel<1, 2>), grid, block, lds, st, a, partials);
    else if (s.k <= 128)
        launch_timed((gemm_topk_kernel<2, 1>), grid, block, lds, st, a, partials);
    else
        launch_timed((gemm_topk_kernel<4, 1>), grid, block, lds, st, a, partials);
    return hipGetLastError();
}

}  // namespace wvg
