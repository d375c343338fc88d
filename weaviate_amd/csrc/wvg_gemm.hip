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
    uint64_t allow_t0;      // tile whose validity word allow[0] masks (allow covers tiles [t0, t0 + words))
    uint64_t id_base;
    uint64_t tile_begin, tile_end;
    uint32_t dim, nchunks;  // nchunks: float4 chunks per row in the corpus layout
    int metric;
    const float *queries;   // [nq][dim] row-major, 16-byte aligned rows (dim % 32 == 0)
    uint32_t nq, k;
    uint32_t nqb, nrr;      // query blocks, row ranges
    int skew;               // K3b: start delay of waves NW/2.. (units of s_sleep(8))
    int pairing;            // K3b (QH = 2): 0 = SIMD partners share rows (query halves), 1 = share queries
    int prio;               // K3b: s_setprio 1 for waves NW/2.. (the second wave on each SIMD)
    uint32_t *prog;         // K3b: [nrr][nqb] tiles done per workgroup (null: no lockstep)
    uint32_t lag;           // K3b: allowed lead over the group's slowest workgroup, in tiles
    uint32_t *gbound;       // K3b: [nq] ordered distance of a finished workgroup's k-th key (min over them)
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
            const uint64_t w = t - a.allow_t0;  // allow[0] is tile allow_t0's word
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

// ---------------------------------------------------------------------------
// K3b: the same contraction with the QUERIES resident and the ROWS streamed
// straight into MFMA operand registers.  A workgroup = 4 waves (one per SIMD,
// 512-register budget) and QB = 16*QT queries held in LDS for the whole
// launch; wave w scores rows 16w..16w+15 of every 64-row tile of the
// workgroup's row range against all QB queries (QT 16x16 output tiles
// sharing one B operand).  No workgroup barrier in the main loop: each wave
// streams its own rows (B: lane (kk, j) loads the 128 contiguous bytes of
// block 4g+kk of row j, 8 x 16-byte loads per K step, double-buffered in
// registers one K step ahead), reads the query operands from LDS (XOR-
// swizzled so every ds_read_b128 is conflict-free) and keeps a per-query
// top-k list in LDS that a candidate enters only if it beats the list's
// current k-th key (a rare wave-uniform insertion).  The four waves' lists
// are merged by rank at the end.  Same slice accumulators and AVX2 reduction
// tree as K3, so the distances are the same bits.
// ---------------------------------------------------------------------------
constexpr int RS_RG = 4;     // row groups of 16 per 64-row tile
constexpr uint32_t RS_SYNC = 1;  // lockstep check at least every RS_SYNC tiles

// QH query halves x 4 row groups = 4*QH waves; wave (qg, rg) scores rows
// 16*rg..16*rg+15 of every tile against queries qg*16*QT .. +16*QT.
template <int D, int QT, int QH, int NBUF>
__global__ __launch_bounds__(RS_RG * QH * 64, 1) void gemm_rs_kernel(GemmArgs a, uint64_t *partials)
{
    constexpr int NW = RS_RG * QH;    // waves per workgroup
    constexpr int NB = D / 32;        // 32-float blocks per row
    constexpr int NK = NB / 4;        // K steps of 4 blocks (D % 128 == 0)
    static_assert(NB % 4 == 0 && NK % NBUF == 0 && NBUF >= 2, "K3b: the B ring must divide the K steps");
    constexpr int QW = 16 * QT;       // queries per wave
    constexpr int QB = QW * QH;       // queries per workgroup
    constexpr int QROW = NB * 8;      // float4 per query row in LDS
    extern __shared__ __attribute__((aligned(16))) float4 smem4[];
    float4 *qs = smem4;                                                  // [QB][QROW]
    const int K = (int)a.k;
    uint64_t *lists = reinterpret_cast<uint64_t *>(smem4 + QB * QROW);  // [NW][QW][K]
    uint64_t *thr = lists + NW * QW * K;                                 // [NW][QW]
    uint64_t *tmp = thr + NW * QW;                                       // [NW][64]
    float *thrf = reinterpret_cast<float *>(tmp + NW * 64);              // [NW][QW]: rejection distance
    uint32_t *gord = reinterpret_cast<uint32_t *>(thrf + NW * QW);       // [NW][QW]: bound read at start

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    // waves w and w + 4 share a SIMD.  pairing 0: they score the same rows
    // against the two query halves; pairing 1 (QH = 2): the same queries
    // against different row groups, so their loads are independent.
    const int rg = QH == 2 && a.pairing ? wave >> 1 : wave % RS_RG;
    const int qg = QH == 2 && a.pairing ? wave & 1 : wave / RS_RG;
    const int slot = qg * RS_RG + rg;  // this wave's list / bound slot
    const uint32_t b = blockIdx.x;
    uint32_t qb, rr;
    if (a.nrr % 8 == 0) {  // the query blocks of one row range share an XCD (blocks b, b+8, ...)
        const uint32_t xcd = b % 8, w = b / 8;
        qb = w % a.nqb;
        rr = (w / a.nqb) * 8 + xcd;
    } else {
        qb = b % a.nqb;
        rr = b / a.nqb;
    }
    const uint64_t ntiles = a.tile_end - a.tile_begin;
    const uint64_t t0 = a.tile_begin + ntiles * rr / a.nrr, t1 = a.tile_begin + ntiles * (rr + 1) / a.nrr;
    const uint32_t q0 = qb * QB;

    // queries -> LDS: chunk cc of block bk of query i at i*QROW + bk*8 + (cc ^ (i & 7))
    for (int idx = tid; idx < QB * NB * 8; idx += NW * 64) {
        const int i = idx / (NB * 8), rem = idx % (NB * 8), bk = rem >> 3, cc = rem & 7;
        const uint32_t q = q0 + (uint32_t)i;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (q < a.nq) v = *reinterpret_cast<const float4 *>(a.queries + (size_t)q * a.dim + bk * 32 + cc * 4);
        qs[i * QROW + bk * 8 + (cc ^ (i & 7))] = v;
    }
    for (int idx = tid; idx < NW * QW * K; idx += NW * 64) lists[idx] = WVG_KEY_NONE;
    // Cross-workgroup bound: a workgroup that finished a row range published,
    // per query, the ordered distance of its k-th key -- k rows at or below
    // it exist, so no row above it can be in the final top-k.  Read once at
    // start (a stale value is a larger, still valid bound); 0xFFFFFFFF = none.
    for (int idx = tid; idx < NW * QW; idx += NW * 64) {
        const uint32_t q = q0 + (uint32_t)((idx / QW) / RS_RG * QW + idx % QW);
        const uint32_t g = a.gbound && q < a.nq ? a.gbound[q] : 0xFFFFFFFFu;
        thr[idx] = WVG_KEY_NONE;
        gord[idx] = g;
        thrf[idx] = wvg_unord_f32(g);  // no bound: a NaN, and !(dist > NaN) admits every row
    }
    __syncthreads();

    const int kk = lane >> 4, j = lane & 15;
    // A operand: lane (i = j, kk) reads chunk cc of block 4g+kk of query qg*QW + 16*tq + j
    const float4 *qa = qs + (qg * QW + j) * QROW + kk * 8;
    const int hsw = j & 7;
    // B operand: lane (kk, j) reads chunk 8*(4g+kk)+cc of row 16*rg + j
    const float4 *rbase = reinterpret_cast<const float4 *>(a.data) + (size_t)(8 * kk) * 64 + 16 * rg + j;
    const uint32_t nch = a.nchunks;
    uint64_t *wl = lists + (size_t)slot * QW * K;
    uint64_t *wthr = thr + slot * QW;
    float *wthrf = thrf + slot * QW;
    const uint32_t *wgord = gord + slot * QW;
    // lanes of query rows past nq, per (query tile, r): C row i = 4*(lane >> 4) + r
    uint64_t qlive[QT][4];
#pragma unroll
    for (int tq = 0; tq < QT; tq++)
#pragma unroll
        for (int r = 0; r < 4; r++)
            qlive[tq][r] = __ballot(q0 + qg * QW + tq * 16 + (lane >> 4) * 4 + r < a.nq);

    auto tile_live = [&](uint64_t t) -> uint64_t {
        uint64_t m = sload64(a.valid + t);
        if (a.allow) {
            const uint64_t w = t - a.allow_t0;  // allow[0] is tile allow_t0's word
            m &= w < a.allow_words ? sload64(a.allow + w) : 0ull;
        }
        return (m >> (16 * rg)) & 0xFFFFull;
    };
    auto next_live = [&](uint64_t t, uint64_t &m) {
        for (; t < t1; ++t) {
            m = tile_live(t);
            if (m) break;
        }
        return t;
    };
    auto load_b = [&](float4 (&bb)[8], uint64_t t, int g) {
        const float4 *rp = rbase + ((size_t)t * nch + 32 * g) * 64;
#pragma unroll
        for (int cc = 0; cc < 8; cc++) bb[cc] = rp[(size_t)cc * 64];
    };
    // per-wave top-k list insertion (wave-uniform qi, key)
    auto insert = [&](int qi, uint64_t key) {
        uint64_t *L = wl + qi * K;
        const uint64_t v = lane < K ? L[lane] : WVG_KEY_NONE;
        const uint64_t last = __shfl(v, K - 1);
        if (!(key < last)) return;
        const uint64_t below = __ballot(lane < K && v < key);
        const int pos = __popcll(below);
        if (lane < K - 1 && lane >= pos) L[lane + 1] = v;
        if (lane == pos) L[pos] = key;
        const uint64_t prev = K >= 2 ? __shfl(v, K - 2) : key;
        if (lane == 0) {
            const uint64_t th = pos <= K - 2 ? prev : key;
            wthr[qi] = th;
            wthrf[qi] = wvg_unord_f32(min((uint32_t)(th >> 32), wgord[qi]));
        }
    };

    floatx4 acc[QT][32];
    float4 bb[NBUF][8];  // ring of K-step operand buffers: step g lives in bb[g % NBUF]

    // MFMAs of one K step for query tile tq: 8 groups of 4 (4 slices each);
    // the A operand of group cc+2 is read from LDS while group cc issues.
    auto mfma_half = [&](int tq, int g, const float4 (&bq)[8]) {
        const float4 *qp = qa + tq * 16 * QROW + g * 32;
        float4 a0 = qp[0 ^ hsw], a1 = qp[1 ^ hsw];
#pragma unroll
        for (int cc = 0; cc < 8; cc++) {
            float4 a2 = a1;
            if (cc + 2 < 8) a2 = qp[(cc + 2) ^ hsw];
            const float4 y = bq[cc];
            floatx4 *ac = &acc[tq][4 * cc];
            const floatx4 z = (floatx4){0.f, 0.f, 0.f, 0.f};
            ac[0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.x, y.x, g == 0 ? z : ac[0], 0, 0, 0);
            ac[1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.y, y.y, g == 0 ? z : ac[1], 0, 0, 0);
            ac[2] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.z, y.z, g == 0 ? z : ac[2], 0, 0, 0);
            ac[3] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.w, y.w, g == 0 ? z : ac[3], 0, 0, 0);
            a0 = a1;
            a1 = a2;
        }
    };
    // Issue order of one half (cdna_hip_programming.md T19; masks: MFMA 0x8,
    // VALU 0x2, DS read 0x100): A reads two groups ahead of their MFMAs, and
    // with an epilogue in the region, ~40 of its VALU after each MFMA group.
    auto pin_plain = [&]() {
        __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
#pragma unroll
        for (int cc = 0; cc < 8; cc++) {
            __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
            if (cc + 2 < 8) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        }
    };
    auto pin_epi = [&]() {
        __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
#pragma unroll
        for (int cc = 0; cc < 8; cc++) {
            __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
            if (cc + 2 < 8) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x002, 40, 0);
        }
    };
    // Epilogue of query tile tq of row tile (t, m): AVX2 reduction tree
    // (D/c/dot_avx256_amd64.c:94-103) per output element; C layout: row j =
    // lane & 15, query 4*(lane >> 4) + r.  Straight-line VALU, so it can run
    // under the other query tile's MFMAs.
    auto reduce_keys = [&](int tq, float (&dd)[4]) {
#pragma unroll
        for (int r = 0; r < 4; r++) {
            float sv[8];
#pragma unroll
            for (int l = 0; l < 8; l++) {
                const float a01 = acc[tq][8 + l][r] + acc[tq][l][r];
                const float a23 = acc[tq][24 + l][r] + acc[tq][16 + l][r];
                sv[l] = a23 + a01;
            }
            const float lo = (sv[0] + sv[1]) + (sv[2] + sv[3]);
            const float hi = (sv[4] + sv[5]) + (sv[6] + sv[7]);
            const float dot = 0.0f + (lo + hi);
            dd[r] = a.metric == WVG_M_DOT ? -dot : 1.0f - dot;
        }
    };
    // Rejection on the float distance against the list's K-th distance
    // (a superset test: !(dist > tau) also admits NaN rows, ties and -0 vs
    // +0, and a NaN tau -- a list not yet full -- admits all); the 64-bit key
    // is built only for the survivors, and insert() decides exactly.
    auto candidates = [&](int tq, uint64_t t, uint64_t m, const float (&dd)[4]) {
        const uint64_t m4 = m * 0x0001000100010001ull;  // the row group's 16 live bits, once per 16-lane group
#pragma unroll
        for (int r = 0; r < 4; r++) {
            const int qi = tq * 16 + (lane >> 4) * 4 + r;
            uint64_t pend = __ballot(!(dd[r] > wthrf[qi])) & m4 & qlive[tq][r];
            if (!pend) continue;  // rare after the first tiles: wave-uniform insertions
            const uint64_t key = wvg_make_key(dd[r], (uint32_t)(t * 64 + 16 * rg + j));
            while (pend) {
                const int src = __builtin_ctzll(pend);
                pend &= pend - 1;
                const int qsrc = tq * 16 + (src >> 4) * 4 + r;
                const uint64_t ks = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(key >> 32), src) << 32) |
                                    (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)key, src);
                insert(qsrc, ks);
            }
        }
    };

    uint64_t m_cur = 0, m_nxt = 0;
    uint64_t t = next_live(t0, m_cur);
    if (t < t1) {
#pragma unroll
        for (int g = 0; g + 1 < NBUF; g++) load_b(bb[g], t, g);
    }
    // Software pipeline over the two query tiles (QT == 2): tile 0's epilogue
    // runs under tile 1's last-step MFMAs, tile 1's under the next row tile's
    // first-step tile-0 MFMAs -- one wave per SIMD, so nothing else would
    // fill the matrix pipe while a wave reduces.
    bool have_prev = false;
    uint64_t t_prev = 0, m_prev = 0;
    if (QH == 2 && wave >= NW / 2) {  // A/B knobs: de-phase / prioritise the SIMD partner
        if (a.prio) __builtin_amdgcn_s_setprio(1);
        for (int i = 0; i < a.skew; i++) __builtin_amdgcn_s_sleep(8);
    }
    // Soft lockstep of the nqb workgroups that stream one row range (they share
    // an XCD and its 4 MiB L2, ~20 row tiles at d = 768): every RS_SYNC tiles a
    // wave that is more than `lag` tiles ahead of the slowest workgroup of its
    // group sleeps, so the group's rows come from HBM once and from L2 for the
    // rest.  Without it the two-waves-per-SIMD variant drifted apart and read
    // 684 GB from HBM per 1024-query batch (22 x the corpus).  Bounded: a wave
    // that waits too long (a group member not resident) stops syncing.
    uint32_t tiles_done = 0;
    bool lockstep = a.prog != nullptr;
    const uint32_t sync_every = a.lag / 4 > RS_SYNC ? a.lag / 4 : RS_SYNC;  // check a quarter of the lead
    uint32_t *grp = a.prog ? a.prog + (size_t)rr * a.nqb : nullptr;
    auto keep_pace = [&]() {
        if (wave == 0 && lane == 0)
            __hip_atomic_store(grp + qb, tiles_done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        for (int spin = 0; spin < 2048; spin++) {
            uint32_t mn = 0xFFFFFFFFu;
            for (uint32_t i = lane; i < a.nqb; i += 64)
                mn = min(mn, __hip_atomic_load(grp + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) mn = min(mn, (uint32_t)__shfl_xor((int)mn, off));
            if (tiles_done <= mn + a.lag) return;
            __builtin_amdgcn_s_sleep(16);
        }
        lockstep = false;
    };
    while (t < t1) {
        const uint64_t tn = next_live(t + 1, m_nxt);
#pragma unroll
        for (int g = 0; g < NK; g++) {
            // NBUF-1 K steps ahead: a later step of this tile, or an early step of
            // the next live tile (the last tile re-reads itself into the dead slot)
            constexpr int AHEAD = NBUF - 1;
            const int gp = g + AHEAD;
            if (gp < NK)
                load_b(bb[gp % NBUF], t, gp);
            else
                load_b(bb[gp % NBUF], tn < t1 ? tn : t, gp - NK);
            // keep the prefetch issued here, ahead of this step's MFMAs (left
            // alone, the scheduler sinks each load next to its consumer and the
            // prefetch distance collapses to one MFMA group)
            __builtin_amdgcn_sched_barrier(0);
            const float4 (&bq)[8] = bb[g % NBUF];
            if constexpr (QT == 2) {
                if (g == 0 && have_prev) {
                    float kp[4];
                    mfma_half(0, g, bq);
                    reduce_keys(1, kp);
                    pin_epi();
                    __builtin_amdgcn_sched_barrier(0);
                    candidates(1, t_prev, m_prev, kp);
                } else {
                    mfma_half(0, g, bq);
                    pin_plain();
                }
                __builtin_amdgcn_sched_barrier(0);
                if (g == NK - 1) {
                    float k0[4];
                    mfma_half(1, g, bq);
                    reduce_keys(0, k0);
                    pin_epi();
                    __builtin_amdgcn_sched_barrier(0);
                    candidates(0, t, m_cur, k0);
                } else {
                    mfma_half(1, g, bq);
                    pin_plain();
                }
                __builtin_amdgcn_sched_barrier(0);
            } else {
#pragma unroll
                for (int tq = 0; tq < QT; tq++) {
                    mfma_half(tq, g, bq);
                    pin_plain();
                    __builtin_amdgcn_sched_barrier(0);
                }
            }
        }
        if constexpr (QT != 2) {
#pragma unroll
            for (int tq = 0; tq < QT; tq++) {
                float kq[4];
                reduce_keys(tq, kq);
                candidates(tq, t, m_cur, kq);
            }
        }
        have_prev = true;
        t_prev = t;
        m_prev = m_cur;
        t = tn;
        m_cur = m_nxt;
        if (lockstep && (++tiles_done % sync_every) == 0) keep_pace();
    }
    if (a.prog && wave == 0 && lane == 0)  // done: never hold the group back
        __hip_atomic_store(grp + qb, 0xFFFFFFFFu, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if constexpr (QT == 2) {
        if (have_prev) {  // the last row tile's query tile 1
            float kp[4];
            reduce_keys(1, kp);
            candidates(1, t_prev, m_prev, kp);
        }
    }
    __syncthreads();
    // merge the four row groups' lists by rank: wave w takes queries w, w+NW, ...
    uint64_t *tw = tmp + wave * 64;
    for (int qi = wave; qi < QB; qi += NW) {
        const uint32_t q = q0 + (uint32_t)qi;
        if (q >= a.nq) break;
        const int g = qi / QW, ql = qi % QW;
        uint64_t mine[RS_RG];
#pragma unroll
        for (int v = 0; v < RS_RG; v++)
            mine[v] = lane < K ? lists[((size_t)(g * RS_RG + v) * QW + ql) * K + lane] : WVG_KEY_NONE;
        int rank[RS_RG] = {0, 0, 0, 0};
        for (int v = 0; v < RS_RG; v++)
            for (int p = 0; p < K; p++) {
                const uint64_t o = lists[((size_t)(g * RS_RG + v) * QW + ql) * K + p];
#pragma unroll
                for (int e = 0; e < RS_RG; e++) rank[e] += o < mine[e];
            }
        if (lane < K) tw[lane] = WVG_KEY_NONE;
#pragma unroll
        for (int e = 0; e < RS_RG; e++)
            if (mine[e] != WVG_KEY_NONE && rank[e] < K) tw[rank[e]] = mine[e];
        if (lane < K) partials[((size_t)q * a.nrr + rr) * K + lane] = tw[lane];
        if (a.gbound && lane == K - 1 && tw[lane] != WVG_KEY_NONE)  // publish this range's k-th distance
            atomicMin(a.gbound + q, (uint32_t)(tw[lane] >> 32));
    }
}

// K3b applies when the queries of a workgroup fit in LDS next to the lists.
struct RsConfig {
    int qt = 1, qh = 1;
    size_t lds = 0;
};
static bool rs_config(uint32_t dim, uint32_t k, RsConfig &c)
{
    if (k == 0 || k > 64) return false;
    if (dim != 256 && dim != 512 && dim != 768 && dim != 1024 && dim != 1536) return false;
    // 0: QT=1 x QH=2 (two waves per SIMD: one wave's epilogue runs under the
    //    other's MFMAs; measured best), 2: QT=2 x QH=1 (one wave per SIMD, the
    //    two query tiles' epilogues software-pipelined in the wave)
    const int mode = tuning().gemm_kernel;
    c.qt = mode == 2 && dim <= 768 ? 2 : 1;  // two query tiles spill registers above d = 768
    c.qh = mode == 2 ? 1 : 2;
    for (;;) {  // shrink the query block until it fits LDS
        const size_t qw = 16 * (size_t)c.qt, nw = (size_t)RS_RG * c.qh, qb = qw * c.qh;
        c.lds = qb * dim * 4 + nw * qw * k * 8 + nw * qw * 8 + nw * 64 * 8 + nw * qw * 8;
        if (c.lds <= 160 * 1024) return true;
        if (c.qh == 2)
            c.qh = 1;
        else if (c.qt == 2)
            c.qt = 1;
        else
            return false;
    }
}

bool gemm_supported(uint32_t dim, int metric)
{
    return dim % 32 == 0 && dim > 0 && (metric == WVG_M_DOT || metric == WVG_M_COSINE);
}

uint32_t gemm_queries_per_block(uint32_t dim, uint32_t k)
{
    RsConfig c;
    if (tuning().gemm_kernel != 1 && rs_config(dim, k, c)) return 16u * (uint32_t)(c.qt * c.qh);
    return GQ;
}

uint32_t gemm_row_ranges(uint32_t nq, uint64_t ntiles, int num_cus, uint32_t dim, uint32_t k)
{
    const uint32_t qpb = gemm_queries_per_block(dim, k);
    const uint32_t nqb = (nq + qpb - 1) / qpb;
    uint64_t want = ((uint64_t)num_cus + nqb - 1) / nqb;  // about one workgroup per CU
    // Short row ranges dispatched range-major: the nqb workgroups of one range
    // start together on one XCD and stay within a few tiles of each other, so
    // each row tile comes from HBM about once per XCD and from L2 for the rest;
    // a long range per workgroup lets them drift apart (~1.1 TB of fabric reads
    // per 10M x 768 batch instead of 0.2 TB).  The per-query bounds published by
    // finished ranges keep the restarted top-k lists cheap.
    const int rt = tuning().gemm_range_tiles == 0 ? 512 : tuning().gemm_range_tiles;
    if (rt > 0) want = std::max<uint64_t>(want, (ntiles + rt - 1) / rt);
    want = (want + 7) / 8 * 8;
    if (want > ntiles) want = ntiles;
    if (want < 1) want = 1;
    return (uint32_t)want;
}

hipError_t launch_gemm_topk(const ScanArgs &s, uint32_t nrr, uint64_t *partials, uint32_t *prog, uint32_t *gbound,
                            int num_cus, hipStream_t st)
{
    GemmArgs a{};
    a.data = reinterpret_cast<const float4 *>(s.data);
    a.valid = s.valid;
    a.allow = s.allow;
    a.allow_words = s.allow_words;
    a.allow_t0 = s.allow_t0;
    a.id_base = s.id_base;
    a.tile_begin = s.tile_begin;
    a.tile_end = s.tile_end;
    a.dim = s.dim;
    a.nchunks = s.nchunks;
    a.metric = s.metric;
    a.queries = reinterpret_cast<const float *>(s.queries);
    a.nq = s.nq;
    a.k = s.k;
    a.nrr = nrr;
    a.skew = tuning().gemm_skew;
    a.pairing = tuning().gemm_pairing;
    a.prio = tuning().gemm_prio;
    RsConfig rc;
    if (tuning().gemm_kernel != 1 && rs_config(s.dim, s.k, rc) && s.nchunks == s.dim / 4) {
        const uint32_t qb = 16u * (uint32_t)(rc.qt * rc.qh);
        a.nqb = (s.nq + qb - 1) / qb;
        dim3 grid(a.nqb * a.nrr), block(RS_RG * rc.qh * 64);
        // lockstep only when every workgroup of the grid is resident (one per CU)
        a.lag = (uint32_t)tuning().gemm_lockstep;
        a.prog = prog && a.lag && a.nqb * a.nrr <= (uint32_t)num_cus ? prog : nullptr;
        if (a.prog) {
            hipError_t e = hipMemsetAsync(a.prog, 0, (size_t)a.nqb * a.nrr * 4, st);
            if (e != hipSuccess) return e;
        }
        a.gbound = gbound;
        if (a.gbound) {
            hipError_t e = hipMemsetAsync(a.gbound, 0xFF, (size_t)s.nq * 4, st);
            if (e != hipSuccess) return e;
        }
        const uint32_t lds = (uint32_t)rc.lds;
#ifdef WVG_TOOLS
#define WVG_RS_QT2(DD, NBF)                                                                            \
        if (rc.qt == 2) {                                                                              \
            launch_timed((gemm_rs_kernel<DD, 2, 1, NBF>), grid, block, lds, st, a, partials);          \
            return hipGetLastError();                                                                  \
        }
#else
#define WVG_RS_QT2(DD, NBF)
#endif
#define WVG_RS(DD, NBF)                                                                                \
    case DD:                                                                                           \
        WVG_RS_QT2(DD, NBF)                                                                            \
        if (rc.qh == 2)                                                                                \
            launch_timed((gemm_rs_kernel<DD, 1, 2, 2>), grid, block, lds, st, a, partials);            \
        else                                                                                           \
            launch_timed((gemm_rs_kernel<DD, 1, 1, NBF>), grid, block, lds, st, a, partials);          \
        return hipGetLastError();
        switch (s.dim) {
            WVG_RS(256, 2)
            WVG_RS(512, 2)
            WVG_RS(768, 2)
            WVG_RS(1024, 2)
            WVG_RS(1536, 3)
        default: break;
        }
#undef WVG_RS
#undef WVG_RS_QT2
    }
    a.nqb = (s.nq + GQ - 1) / GQ;
    const size_t lds = (size_t)2 * (GQ + GR) * GSTRIDE * 4 + (size_t)GQ * GR * 8;
    dim3 grid(a.nqb * a.nrr), block(GWAVES * 64);
    if (s.k <= 64)
#ifdef WVG_TOOLS
        if (tuning().gemm_pf == 1)
            launch_timed((gemm_topk_kernel<1, 1>), grid, block, lds, st, a, partials);
        else
#endif
            launch_timed((gemm_topk_kernel<1, 2>), grid, block, lds, st, a, partials);
    else if (s.k <= 128)
        launch_timed((gemm_topk_kernel<2, 1>), grid, block, lds, st, a, partials);
    else
        launch_timed((gemm_topk_kernel<4, 1>), grid, block, lds, st, a, partials);
    return hipGetLastError();
}

}  // namespace wvg
