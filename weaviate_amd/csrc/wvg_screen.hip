// wvg_screen.hip -- K3c: batched dot / cosine scoring as a bf16 MFMA screen
// with a rigorous per-(query, row) error bound, followed by the exact fp32
// rescore of every row the bound cannot rule out.  Results are bit-identical
// to the exact path (K3b / K1, the reference's AVX2-order dot_256):
//
//   Reference: Q independent flat.searchByVector calls (V/flat/index.go:319)
//   over the same rows, SingleDist = dot_256 (D/dot_product.go:68-98,
//   D/c/dot_avx256_amd64.c) or its cosine Wrap (D/cosine_dist.go:38-68).
//
// The bound.  r = the exact fp32 dot of (q, x) in the AVX2 order; s = the
// bf16 MFMA dot of (bf16(q), bf16(x)) (round to nearest: |x - bf16(x)| <=
// 2^-8 |x|, products exact in fp32, fp32 accumulation).  Then
//   |r - s| <= (2^-7 + 2^-16 + 3 d 2^-24) sum |q_i x_i| + (denormal terms)
//           <= c Nq Nx + 2^-120 (Nq + Nx) + 2^-110,
// Nq, Nx upper bounds of the L2 norms (Cauchy-Schwarz), c = 2^-7 + 2^-15 +
// d 2^-21 (the extra terms absorb the fp32 roundings of the bound itself).
// Cosine adds 2^-19 for the 1 - r roundings.  Per element: E = fma(Nx, K1q,
// K2q), u = s + E >= r, so lower = -u (dot) / 1 - u (cosine) <= the exact
// distance.  A row can be in the top-k only if lower <= tau, for any tau
// with k rows at or below it: tau = (k-th smallest lower) + 2 Emax_q, taken
// per wave from its lists and across workgroups from finished row ranges.
//
// K3c.  A workgroup owns 128 queries x one range of 256-row blocks; per
// 32-deep K stage it stages 8 KiB of query fragments, 16 KiB of row
// fragments and the block's row norms into LDS with global_load_lds (both
// operands pre-laid out in HBM in MFMA operand order: 1 KiB = one 16 x 32
// bf16 fragment, lane l = item l & 15, k 8 (l >> 4) .. +7), a ring of four
// stage buffers with three stages in flight (counted vmcnt, raw s_barrier:
// a __syncthreads would drain the DMA), one barrier per stage; 8 waves as
// 4 (queries) x 2 (rows), each wave a 32 x 128 tile of 16x16x32 bf16 MFMAs.
// After a row block: u per element, one compare with the query's threshold;
// the rare survivors enter the wave's per-query list of the SC_M smallest
// lower bounds (LDS).  A finished range merges its two waves' lists per query
// into partials and publishes tau (atomicMin); collect keeps the entries with
// lower <= the final tau -- a superset of the exact top-k and its ties -- and
// flags a query whose range list was full below tau (rows may have been
// dropped): it is rescanned exactly (K1).
// Roofline: bf16 MFMA, 2 Q N d FLOP per batch (2.5 PFLOP/s dense).
#include <numeric>
#include <type_traits>
#include <utility>

#include "wvg_internal.hpp"

namespace wvg {

typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

constexpr int SC_BQ = 128;                 // queries per workgroup
constexpr int SC_WAVES = 8;                // 4 (query quarters) x 2 (row halves)
constexpr int SC_AFR = 8;                  // query fragments per stage (8 groups of 16, one 32-deep K block)
constexpr int SC_BFR = 16;                 // row fragments per stage (16 groups of 16)
constexpr int SC_STAGE = (SC_AFR + SC_BFR + 1) * 1024 + 256;  // + the row block's 256 norms and tile words
constexpr int SC_NBUF = 4;                 // stages in LDS: three in flight while one is computed
constexpr int SC_LISTS = SC_WAVES * 32 * SCREEN_M * 8;
constexpr int SC_LDS = SC_NBUF * SC_STAGE + SC_LISTS + SC_WAVES * 32 * 4 * 2 + SC_BQ * 4 * 3;

// A wave-uniform 64-bit value from a VGPR.
__device__ __forceinline__ uint64_t readfirstlane64(uint64_t v)
{
    return ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(v >> 32)) << 32) |
           (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
}

// ---------------------------------------------------------------------------
// Shadow build: bf16 fragments + row-norm upper bounds of tiles [t0, t1).
// One thread per (fragment, lane): fragment (t, kb, rg), lane l -> row
// 16 rg + (l & 15) of tile t, elements 32 kb + 8 (l >> 4) .. + 7.
__global__ __launch_bounds__(256) void shadow_frag_kernel(const float4 *__restrict__ tiled, uint32_t nchunks,
                                                          uint32_t kbn, uint64_t t0, uint64_t nfrag, uint4 *shadow)
{
    const uint64_t g = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (g >= nfrag * 64) return;
    const uint32_t lane = (uint32_t)(g & 63);
    const uint64_t f = g >> 6;                 // fragment index relative to tile t0
    const uint32_t rg = (uint32_t)(f & 3);
    const uint64_t tk = f >> 2;
    const uint32_t kb = (uint32_t)(tk % kbn);
    const uint64_t t = t0 + tk / kbn;
    const uint32_t row = 16 * rg + (lane & 15);
    const uint32_t c0 = (32 * kb + 8 * (lane >> 4)) / 4;  // first float4 chunk
    float v[8];
#pragma unroll
    for (int h = 0; h < 2; h++) {
        const uint32_t c = c0 + h;
        const float4 x = c < nchunks ? tiled[((size_t)t * nchunks + c) * 64 + row] : make_float4(0.f, 0.f, 0.f, 0.f);
        v[4 * h + 0] = x.x;
        v[4 * h + 1] = x.y;
        v[4 * h + 2] = x.z;
        v[4 * h + 3] = x.w;
    }
    bf16x8 o;
#pragma unroll
    for (int e = 0; e < 8; e++) o[e] = (__bf16)v[e];  // v_cvt_pk_bf16_f32: round to nearest even
    shadow[((t * kbn + kb) * 4 + rg) * 64 + lane] = *reinterpret_cast<const uint4 *>(&o);
}

// An upper bound of the L2 norm from the exact square sum in double:
// rounded up past the float cast; +inf for a non-finite row.
__device__ __forceinline__ float norm_upper(double ss)
{
    if (!(ss < 1e300)) return __builtin_inff();  // inf / NaN components
    return (float)(__builtin_sqrt(ss) * (1.0 + 1e-6));
}

__global__ __launch_bounds__(256) void shadow_norm_kernel(const float4 *__restrict__ tiled, uint32_t nchunks,
                                                          uint64_t slot0, uint64_t n, float *norms, uint32_t *nmax)
{
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    float nv = 0.f;
    if (i < n) {
        const uint64_t slot = slot0 + i;
        const float4 *rp = tiled + (slot >> 6) * nchunks * 64 + (slot & 63);
        double ss = 0.0;
        for (uint32_t c = 0; c < nchunks; c++) {
            const float4 x = rp[(size_t)c * 64];
            ss += (double)x.x * x.x + (double)x.y * x.y + (double)x.z * x.z + (double)x.w * x.w;
        }
        nv = norm_upper(ss);
        norms[slot] = nv;
    }
    // the block's maximum, then one atomic (non-negative floats order as their bits)
    uint32_t b = __float_as_uint(nv);
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) b = max(b, (uint32_t)__shfl_xor((int)b, off));
    if ((threadIdx.x & 63) == 0) atomicMax(nmax, b);
}

hipError_t launch_shadow_build(const float *tiled, uint32_t dim, uint64_t t0, uint64_t t1, void *shadow, float *norms,
                               uint32_t *nmax, hipStream_t s)
{
    if (t1 <= t0) return hipSuccess;
    const uint32_t nch = f32_chunks(dim), kbn = screen_kblocks(dim);
    const uint64_t nfrag = (t1 - t0) * kbn * 4;
    hipLaunchKernelGGL(shadow_frag_kernel, dim3((unsigned)((nfrag * 64 + 255) / 256)), dim3(256), 0, s,
                       reinterpret_cast<const float4 *>(tiled), nch, kbn, t0, nfrag, reinterpret_cast<uint4 *>(shadow));
    const uint64_t n = (t1 - t0) * 64;
    hipLaunchKernelGGL(shadow_norm_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s,
                       reinterpret_cast<const float4 *>(tiled), nch, t0 * 64, n, norms, nmax);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Query preparation: fragments [nq16][kbn][64] and the bound constants.
__global__ __launch_bounds__(256) void screen_qfrag_kernel(const float *q, uint32_t nq, uint32_t qpitch, uint32_t dim,
                                                           uint32_t kbn, uint32_t nq16, uint4 *qfrag)
{
    const uint64_t g = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (g >= (uint64_t)nq16 * kbn * 64) return;
    const uint32_t lane = (uint32_t)(g & 63);
    const uint32_t kb = (uint32_t)((g >> 6) % kbn);
    const uint32_t qg = (uint32_t)((g >> 6) / kbn);
    const uint32_t qi = 16 * qg + (lane & 15);
    const uint32_t e0 = 32 * kb + 8 * (lane >> 4);
    bf16x8 o;
#pragma unroll
    for (int e = 0; e < 8; e++) {
        const uint32_t p = e0 + e;
        o[e] = (__bf16)(qi < nq && p < dim ? q[(size_t)qi * qpitch + p] : 0.0f);
    }
    qfrag[g] = *reinterpret_cast<const uint4 *>(&o);
}

__global__ __launch_bounds__(256) void screen_qconst_kernel(const float *q, uint32_t nq, uint32_t qpitch,
                                                            uint32_t dim, uint32_t nq_pad, int cosine,
                                                            const uint32_t *nmax, float *k1, float *k2, float *emax)
{
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t qi = blockIdx.x * 4 + (threadIdx.x >> 6);  // one wave per query
    if (qi >= nq_pad) return;
    double ss = 0.0;
    if (qi < nq)
        for (uint32_t i = lane; i < dim; i += 64) {
            const double x = q[(size_t)qi * qpitch + i];
            ss += x * x;
        }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) ss += __shfl_xor(ss, off);
    if (lane) return;
    const float nq_up = norm_upper(ss);
    const float c = 0x1p-7f + 0x1p-15f + (float)dim * 0x1p-21f;
    const float a = cosine ? 0x1p-19f : 0x1p-110f;
    float K1 = c * nq_up + 0x1p-120f, K2 = 0x1p-120f * nq_up + a;
    if (qi >= nq) K1 = K2 = 0.f;
    k1[qi] = K1;
    k2[qi] = K2;
    emax[qi] = __builtin_fmaf(__uint_as_float(*nmax), K1, K2);
}

// ---------------------------------------------------------------------------
// The int8 screen (K3i, round 6).  bf16 MFMA runs at 2.5 PFLOP/s, int8 at
// twice that; K3d's time is almost all per K block (10M x 768 / 512 cosine:
// 15.34 / 10.83 ms per 1024-query batch = 1.8 ms + 0.56 ms per K block,
// profiles/r06/screen_i8/), and an int8 K block is 64 deep for the same
// instructions and the same 16 KiB stage.  The rows get one corpus-wide
// scale S (the largest |x| / 127 at the shadow's first build; later rows
// clamp at +-127), each query its own Sq; codes x8 = clamp(rint(x / S)),
// q8 = clamp(rint(q / Sq)); the MFMA sums q8 . x8 exactly in int32 (|sum| <=
// d 127^2 < 2^24 for d <= 1024, so its float is exact too).  With xt = S x8,
// qt = Sq q8 and r the exact fp32 dot in the AVX2 order:
//   q.x = qt.xt + qt.(x - xt) + (q - qt).x
//   |qt.(x - xt)| <= |qt| Ex,  |(q - qt).x| <= Eq |x|   (Cauchy-Schwarz)
//   |r - q.x| <= 4 d 2^-24 |q| |x|    (fp32 dot: ~(d / 32 + 5) 2^-24 for its 32 chains)
//   s = fl(fl(acc) fl(S Sq)) = qt.xt (1 + <= 2^-22.9)
// with per-row Ex >= |x - xt| and Nx >= |x| (fp64 sums rounded up, +inf for
// a non-finite row) and per-query Nqt >= |qt|, Eq >= |q - qt|, Nq >= |q|:
//   u = s + fma(Ex, A, fma(Nx, B, K2)) >= r,
//   A = Nqt (1 + 2^-19),  B = Eq (1 + 2^-19) + 4 d 2^-24 Nq + 2^-19 Nqt,
// the 2^-19 terms absorbing s's and u's own fp32 roundings (relative, all
// terms >= 0), K2 = K3c's (2^-120 Nq + 2^-110; cosine + 2^-19).  The bound is
// two-sided, so tau = (k-th smallest lower) + 2 Emax holds as in K3c, Emax_q
// = fma(max Ex, A, fma(max Nx, B, K2)).  A query that is not finite or whose
// scale underflows gets A = +inf: every row is a candidate (the flag path).
typedef int i32x4 __attribute__((ext_vector_type(4)));

// x's int8 code at 1 / inv: nearest, clamped to +-127 (NaN -> 0: a non-finite
// row's error bound is +inf, so its codes decide nothing)
__device__ __forceinline__ int si_code(float x, float inv)
{
    const float r = __builtin_rintf(x * inv);
    return r >= 127.f ? 127 : (r <= -127.f ? -127 : (r == r ? (int)r : 0));
}
__device__ __forceinline__ uint32_t si_pack4(float4 x, float inv)
{
    return (uint32_t)(si_code(x.x, inv) & 255) | (uint32_t)(si_code(x.y, inv) & 255) << 8 |
           (uint32_t)(si_code(x.z, inv) & 255) << 16 | (uint32_t)(si_code(x.w, inv) & 255) << 24;
}

// The largest finite |x| of rows [0, n) (tiled layout, whole tiles: the zero
// fill of a partial tile does not change it), as float bits into *out.
__global__ __launch_bounds__(256) void shadow_maxabs_kernel(const float4 *__restrict__ tiled, uint64_t count,
                                                            uint32_t *out)
{
    float m = 0.f;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < count; i += (uint64_t)gridDim.x * 256) {
        const float4 x = tiled[i];
        const float v[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
        for (int e = 0; e < 4; e++) {
            const float a = __builtin_fabsf(v[e]);
            if (a <= 3.4028235e38f) m = __builtin_fmaxf(m, a);  // (NaN / inf skipped)
        }
    }
    uint32_t b = __float_as_uint(m);
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) b = max(b, (uint32_t)__shfl_xor((int)b, off));
    if ((threadIdx.x & 63) == 0) atomicMax(out, b);
}

// int8 fragments of tiles [t0, t1): fragment (t, kb, rg), lane l -> row
// 16 rg + (l & 15), elements 64 kb + 16 (l >> 4) .. + 15 (byte e = element e).
// scale = {S, 1 / S}.
__global__ __launch_bounds__(256) void shadow_i8_frag_kernel(const float4 *__restrict__ tiled, uint32_t nchunks,
                                                             uint32_t kbn, uint64_t t0, uint64_t nfrag,
                                                             const float *scale, uint4 *shadow)
{
    const uint64_t g = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (g >= nfrag * 64) return;
    const uint32_t lane = (uint32_t)(g & 63);
    const uint64_t f = g >> 6;
    const uint32_t rg = (uint32_t)(f & 3);
    const uint64_t tk = f >> 2;
    const uint32_t kb = (uint32_t)(tk % kbn);
    const uint64_t t = t0 + tk / kbn;
    const uint32_t row = 16 * rg + (lane & 15);
    const uint32_t c0 = (64 * kb + 16 * (lane >> 4)) / 4;
    const float inv = scale[1];
    uint32_t wv[4];
#pragma unroll
    for (int h = 0; h < 4; h++) {
        const uint32_t c = c0 + h;
        const float4 x = c < nchunks ? tiled[((size_t)t * nchunks + c) * 64 + row] : make_float4(0.f, 0.f, 0.f, 0.f);
        wv[h] = si_pack4(x, inv);
    }
    shadow[((t * kbn + kb) * 4 + rg) * 64 + lane] = make_uint4(wv[0], wv[1], wv[2], wv[3]);
}

// Per row: Nx >= |x| and Ex >= |x - S x8| (fp64 sums, rounded up); their
// maxima into mx[0], mx[1] (float bits; only ever raised).
__global__ __launch_bounds__(256) void shadow_i8_norm_kernel(const float4 *__restrict__ tiled, uint32_t nchunks,
                                                             uint64_t slot0, uint64_t n, const float *scale,
                                                             float *norms, float *errs, uint32_t *mx)
{
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    float nv = 0.f, ev = 0.f;
    if (i < n) {
        const uint64_t slot = slot0 + i;
        const float4 *rp = tiled + (slot >> 6) * nchunks * 64 + (slot & 63);
        const double S = scale[0];
        const float inv = scale[1];
        double ss = 0.0, se = 0.0;
        for (uint32_t c = 0; c < nchunks; c++) {
            const float4 x = rp[(size_t)c * 64];
            const float v[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
            for (int e = 0; e < 4; e++) {
                const double d = (double)v[e] - S * (double)si_code(v[e], inv);
                ss += (double)v[e] * v[e];
                se += d * d;
            }
        }
        nv = norm_upper(ss);
        ev = norm_upper(se);
        norms[slot] = nv;
        errs[slot] = ev;
    }
    uint32_t b = __float_as_uint(nv), c = __float_as_uint(ev);
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        b = max(b, (uint32_t)__shfl_xor((int)b, off));
        c = max(c, (uint32_t)__shfl_xor((int)c, off));
    }
    if ((threadIdx.x & 63) == 0) {
        atomicMax(mx, b);
        atomicMax(mx + 1, c);
    }
}

// Per query (one wave each): Sq, the bound constants A (k1), B (kb), K2 (k2),
// Emax, the score scale fl(S Sq) (css) and 1 / Sq (qinv, for the fragments).
__global__ __launch_bounds__(256) void screen_qconst_i8_kernel(const float *q, uint32_t nq, uint32_t qpitch,
                                                               uint32_t dim, uint32_t nq_pad, int cosine,
                                                               const uint32_t *mx, const float *scale, float *k1,
                                                               float *k2, float *kb, float *css, float *qinv,
                                                               float *emax)
{
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t qi = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (qi >= nq_pad) return;
    float amax = 0.f;
    bool bad = false;
    if (qi < nq)
        for (uint32_t i = lane; i < dim; i += 64) {
            const float a = __builtin_fabsf(q[(size_t)qi * qpitch + i]);
            if (a <= 3.4028235e38f) amax = __builtin_fmaxf(amax, a);
            else bad = true;
        }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) amax = __builtin_fmaxf(amax, __shfl_xor(amax, off));
    bad = __ballot(bad) != 0;
    const float sq = amax > 0.f ? amax / 127.f : 1.f, inv = 1.f / sq;
    double st = 0.0, se = 0.0, sn = 0.0;
    if (qi < nq)
        for (uint32_t i = lane; i < dim; i += 64) {
            const float x = q[(size_t)qi * qpitch + i];
            const double t = (double)sq * (double)si_code(x, inv);
            st += t * t;
            se += ((double)x - t) * ((double)x - t);
            sn += (double)x * x;
        }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        st += __shfl_xor(st, off);
        se += __shfl_xor(se, off);
        sn += __shfl_xor(sn, off);
    }
    if (lane) return;
    const double nqt = norm_upper(st), eq = norm_upper(se), nqu = norm_upper(sn);
    const float S = scale[0];
    float A = (float)(nqt * (1.0 + 0x1p-19) + 0x1p-120);
    float B = (float)(eq * (1.0 + 0x1p-19) + 4.0 * dim * 0x1p-24 * nqu + 0x1p-19 * nqt + 0x1p-120);
    float K2 = (float)(0x1p-120 * nqu + (cosine ? 0x1p-19 : 0x1p-110));
    float cs = S * sq;
    // non-finite query or a scale outside the normal range: no fast rejection
    if (bad || !(cs >= 0x1p-100f && cs <= 0x1p100f) || !(A < __builtin_inff())) A = __builtin_inff();
    if (qi >= nq) A = B = K2 = cs = 0.f;
    k1[qi] = A;
    k2[qi] = K2;
    kb[qi] = B;
    css[qi] = cs;
    qinv[qi] = inv;
    emax[qi] = __builtin_fmaf(__uint_as_float(mx[1]), A, __builtin_fmaf(__uint_as_float(mx[0]), B, K2));
}

hipError_t launch_shadow_maxabs(const float *tiled, uint32_t dim, uint64_t tiles, uint32_t *out, hipStream_t s)
{
    const uint64_t count = tiles * f32_chunks(dim) * 64;
    if (count == 0) return hipSuccess;
    const uint64_t blocks = std::min<uint64_t>(4096, (count + 255) / 256);
    hipLaunchKernelGGL(shadow_maxabs_kernel, dim3((unsigned)blocks), dim3(256), 0, s,
                       reinterpret_cast<const float4 *>(tiled), count, out);
    return hipGetLastError();
}

hipError_t launch_shadow_build_i8(const float *tiled, uint32_t dim, uint64_t t0, uint64_t t1, void *shadow,
                                  float *norms, float *errs, uint32_t *mx, hipStream_t s)
{
    if (t1 <= t0) return hipSuccess;
    const uint32_t nch = f32_chunks(dim), kbn = dim / 64;
    const float *scale = reinterpret_cast<const float *>(mx + 2);
    const uint64_t nfrag = (t1 - t0) * kbn * 4;
    hipLaunchKernelGGL(shadow_i8_frag_kernel, dim3((unsigned)((nfrag * 64 + 255) / 256)), dim3(256), 0, s,
                       reinterpret_cast<const float4 *>(tiled), nch, kbn, t0, nfrag, scale,
                       reinterpret_cast<uint4 *>(shadow));
    const uint64_t n = (t1 - t0) * 64;
    hipLaunchKernelGGL(shadow_i8_norm_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s,
                       reinterpret_cast<const float4 *>(tiled), nch, t0 * 64, n, scale, norms, errs, mx);
    return hipGetLastError();
}

// int8 query fragments [nq16][kbn][64]: lane l -> query 16 qg + (l & 15),
// elements 64 kb + 16 (l >> 4) .. + 15 (the rows' element map)
__global__ __launch_bounds__(256) void screen_qfrag_i8_kernel(const float *q, uint32_t nq, uint32_t qpitch,
                                                              uint32_t dim, uint32_t kbn, uint32_t nq16,
                                                              const float *qinv, uint4 *qfrag)
{
    const uint64_t g = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (g >= (uint64_t)nq16 * kbn * 64) return;
    const uint32_t lane = (uint32_t)(g & 63);
    const uint32_t kb = (uint32_t)((g >> 6) % kbn);
    const uint32_t qg = (uint32_t)((g >> 6) / kbn);
    const uint32_t qi = 16 * qg + (lane & 15);
    const uint32_t e0 = 64 * kb + 16 * (lane >> 4);
    const float inv = qi < nq ? qinv[qi] : 0.f;
    uint32_t wv[4];
#pragma unroll
    for (int h = 0; h < 4; h++) {
        float4 x = make_float4(0.f, 0.f, 0.f, 0.f);
        if (qi < nq && e0 + 4 * h + 3 < dim) {
            const float *p = q + (size_t)qi * qpitch + e0 + 4 * h;
            x = make_float4(p[0], p[1], p[2], p[3]);
        }
        wv[h] = si_pack4(x, inv);
    }
    qfrag[g] = make_uint4(wv[0], wv[1], wv[2], wv[3]);
}

// ---------------------------------------------------------------------------
// K3c
struct ScreenArgs {
    const uint4 *shadow;      // [tiles][kbn][4][64]
    const float *norms;       // [slots]
    const uint64_t *valid;
    const uint64_t *allow;
    uint64_t allow_words, allow_t0;
    uint64_t tile_begin, tile_end;
    uint32_t kbn;             // 32-element K blocks (even)
    const uint4 *qfrag;       // [nq16][kbn][64]
    const float *k1, *k2, *emax;  // [nq_pad]
    const float *errs;        // K3i: [slots] row quantization-error norms (upper bounds)
    const float *kb, *css;    // K3i: [nq_pad] row-norm coefficient B, score scale S * Sq
    uint32_t nq, k, nqb, nrr;
    uint32_t rr0, nrr_l;      // this launch's ranges: [rr0, rr0 + nrr_l) of nrr
    uint32_t rsplit[2];       // (K3i) ranges [0, rsplit[0]) split row blocks [0, bsplit[0]), ranges
    uint64_t bsplit[2];       // [rsplit[0], rsplit[1]) blocks [bsplit[0], bsplit[1]) (short warm-up
                              // ranges), the others the rest; rsplit[0] = 0: nrr equal ranges
    int cosine;
#ifdef WVG_TOOLS
    int diag;                 // Tuning::screen_diag
#endif
    uint32_t *gbound;         // [nq] ordered tau; 0xFFFFFFFF = none yet
    uint64_t *partials;       // [nq][nrr][SCREEN_M]
};

// Row blocks [b0, b1) of range rr (ScreenArgs::rsplit; the host checks
// 0 < rsplit[0] <= rsplit[1] < nrr and 0 < bsplit[0] <= bsplit[1] < nblk)
__device__ __forceinline__ void sc_range(const ScreenArgs &a, uint64_t nblk, uint32_t rr, uint64_t &b0, uint64_t &b1)
{
    uint64_t lo = 0, hi = nblk, r = rr, n = a.nrr;
    if (a.rsplit[0] != 0) {
        if (rr < a.rsplit[0]) {
            hi = a.bsplit[0];
            n = a.rsplit[0];
        } else if (rr < a.rsplit[1]) {
            lo = a.bsplit[0];
            hi = a.bsplit[1];
            r = rr - a.rsplit[0];
            n = a.rsplit[1] - a.rsplit[0];
        } else {
            lo = a.bsplit[1];
            r = rr - a.rsplit[1];
            n = a.nrr - a.rsplit[1];
        }
    }
    b0 = lo + (hi - lo) * r / n;
    b1 = lo + (hi - lo) * (r + 1) / n;
}

// lower bound (distance space) of a survivor's u; NaN u (a non-finite row or
// query) -> -inf: always a candidate, rescored exactly
__device__ __forceinline__ float sc_lower(float u, int cosine)
{
    if (u != u) return -__builtin_inff();
    return cosine ? 1.0f - u : -u;
}

// u-space threshold of a distance threshold tau (a superset for cosine)
__device__ __forceinline__ float sc_sigma(float tau, int cosine)
{
    if (!(tau < __builtin_inff())) return -__builtin_inff();
    return cosine ? (1.0f - tau) - 0x1p-20f : -tau;
}

// tau from the k-th smallest lower bound of a list: every one of those k rows
// has its exact distance <= lower + 2 E <= lower_k + 2 Emax.  Not a number
// (-inf + inf: a non-finite query) means no bound: +inf.
__device__ __forceinline__ float sc_tau_k(float lower_k, float emax, int cosine)
{
    const float t = lower_k + 2.0f * emax * (1.0f + 0x1p-10f) + (cosine ? 0x1p-20f : 0.0f);
    return t == t ? t : __builtin_inff();
}

__device__ __forceinline__ float key_lower(uint64_t key) { return wvg_unord_f32((uint32_t)(key >> 32)); }

// Exact insertion of one survivor (wave-uniform arguments) into a wave's list
// L of the SCREEN_M smallest (lower, slot) keys of one query, then the
// query's thresholds: WT (distance space) = min(tau, k-th lower + 2 Emax,
// M-th lower), WS its u-space form.  Returns the query's current WS, so the
// caller drops the other candidates of that query it no longer admits.
// Out of line (it is reached from 64 / 128 unrolled epilogue sites; inlined,
// the kernel spilled inside its main loop) with LDS-typed pointers: through
// generic pointers every list access was a flat load / store, each followed by
// a vmcnt(0) + lgkmcnt(0) wait.  (A call still begins with the ABI's full
// wait, which drains the stage prefetch once per exact-path row block.)
typedef __attribute__((address_space(3))) uint64_t lds_u64;
typedef __attribute__((address_space(3))) float lds_f32;
__device__ __attribute__((noinline)) float sc_insert(lds_u64 *L, lds_f32 *WT, lds_f32 *WS, float emax, int K,
                                                     int cosine, float u, uint32_t slot)
{
    const int lane = threadIdx.x & 63, M = SCREEN_M;
    const float lower = sc_lower(u, cosine);
    if (!(lower <= *WT)) return *WS;
    const uint64_t key = ((uint64_t)wvg_ord_f32(lower) << 32) | slot;
    const uint64_t v = lane < M ? L[lane] : WVG_KEY_NONE;
    const uint64_t last = __shfl(v, M - 1);
    if (!(key < last)) return *WS;
    const int pos = __popcll(__ballot(lane < M && v < key));
    if (lane >= pos && lane < M - 1) L[lane + 1] = v;
    if (lane == pos) L[pos] = key;
    __builtin_amdgcn_wave_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const uint64_t nk = L[K - 1], nm = L[M - 1];
    float t = *WT;
    if (nk != WVG_KEY_NONE) t = fminf(t, sc_tau_k(key_lower(nk), emax, cosine));
    if (nm != WVG_KEY_NONE) t = fminf(t, key_lower(nm));
    const float ws = sc_sigma(t, cosine);
    if (lane == 0) {
        *WT = t;
        *WS = ws;
    }
    __builtin_amdgcn_wave_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    return ws;
}

#ifdef WVG_TOOLS
__device__ unsigned long long g_screen_ctr[4];  // tools build: [0] row blocks, [1] slow-path entries, [2] insert calls
#endif

__global__ __launch_bounds__(SC_WAVES * 64, 1) void screen_kernel(ScreenArgs a)
{
#ifdef WVG_TOOLS
    uint32_t n_blk = 0, n_slow = 0, n_call = 0;
#endif
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    uint64_t *lists = reinterpret_cast<uint64_t *>(smem + SC_NBUF * SC_STAGE);  // [8][32][M]
    float *tau = reinterpret_cast<float *>(smem + SC_NBUF * SC_STAGE + SC_LISTS);  // [8][32] distance-space threshold
    float *sig = tau + SC_WAVES * 32;                                      // [8][32] u-space threshold
    float *ck1 = sig + SC_WAVES * 32;                                      // [128]
    float *ck2 = ck1 + SC_BQ;
    float *cem = ck2 + SC_BQ;

    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wq = w & 3, wr = w >> 2;
    const int K = (int)a.k, M = SCREEN_M;
    const int cosine = a.cosine;
    // the nqb query blocks of one row range share an XCD (blocks b, b+8, ...)
    const uint32_t b = blockIdx.x;
    uint32_t qb, rr;
    if (a.nrr_l % 8 == 0) {
        const uint32_t xcd = b % 8, wv = b / 8;
        qb = wv % a.nqb;
        rr = a.rr0 + (wv / a.nqb) * 8 + xcd;
    } else {
        qb = b % a.nqb;
        rr = a.rr0 + b / a.nqb;
    }
    const uint64_t ntiles = a.tile_end - a.tile_begin;
    const uint64_t nblk = (ntiles + 3) / 4;  // 256-row blocks
    const uint64_t blk0 = nblk * rr / a.nrr, blk1 = nblk * (rr + 1) / a.nrr;
    const uint32_t q0 = qb * SC_BQ;
    const uint32_t NK = a.kbn;  // 32-deep stages per row block

    // per-query constants and thresholds
    for (int i = tid; i < SC_BQ; i += SC_WAVES * 64) {
        const uint32_t q = q0 + (uint32_t)i;
        ck1[i] = a.k1[q];
        ck2[i] = a.k2[q];
        cem[i] = a.emax[q];
    }
    for (int i = tid; i < SC_WAVES * 32; i += SC_WAVES * 64) {
        const int ww = i / 32, ql = i % 32;
        const uint32_t q = q0 + (uint32_t)((ww & 3) * 32 + ql);
        // agent-scope load (L1 bypassed): the bounds are atomicMin'd by ranges that
        // finished on any XCD; a plain load could return a stale line
        const uint32_t g = q < a.nq ? __hip_atomic_load(a.gbound + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
        const float t = q >= a.nq ? -__builtin_inff() : (g == 0xFFFFFFFFu ? __builtin_inff() : wvg_unord_f32(g));
        tau[i] = t;
        sig[i] = q >= a.nq ? __builtin_inff() : sc_sigma(t, cosine);
    }
    for (int i = tid; i < SC_WAVES * 32 * M; i += SC_WAVES * 64) lists[i] = WVG_KEY_NONE;
    __syncthreads();
    if (blk0 >= blk1) goto publish;
    {
        // stage loader: wave w moves fragments 3w .. 3w+2 of a stage (A 0..7, B 8..23);
        // waves 0-3 also one 256-byte quarter of the block's norms, wave 4 the
        // block's validity and allow words (so a wave's loads per stage: 4 for
        // waves 0-4, 3 for 5-7)
        // Per-lane source pointers of this wave's three fragments at stage 0 of
        // the load cursor's row block: a stage adds one K block (A: 1 KiB,
        // B: 4 KiB), a row block four tiles of B (the shadow is padded by 4
        // tiles); the norms pointer moves by a row block.
        const uint4 *lsrc[3];
        uint32_t lstep[3];
        uint64_t lblkstep[3];
#pragma unroll
        for (int j = 0; j < 3; j++) {
            const int f = 3 * w + j;
            if (f < SC_AFR) {
                lsrc[j] = a.qfrag + (size_t)(qb * 8 + f) * a.kbn * 64 + lane;
                lstep[j] = 64;
                lblkstep[j] = 0;
            } else {
                const int r16 = f - SC_AFR, tt = r16 >> 2, rg = r16 & 3;
                const uint64_t t = a.tile_begin + blk0 * 4 + tt;
                lsrc[j] = a.shadow + ((size_t)t * a.kbn * 4 + rg) * 64 + lane;
                lstep[j] = 256;
                lblkstep[j] = (uint64_t)4 * a.kbn * 256;
            }
        }
        const float *lnorm = a.norms + (a.tile_begin + blk0 * 4 + (w & 3)) * 64 + lane;
        auto load_stage = [&](unsigned char *dst, uint32_t ks, uint64_t lb) {
#pragma unroll
            for (int j = 0; j < 3; j++) {
#ifdef WVG_TOOLS
                if ((a.diag & 8) && 3 * w + j < SC_AFR) continue;  // diagnostic: no query-fragment loads
#endif
                __builtin_amdgcn_global_load_lds(lsrc[j] + (size_t)ks * lstep[j],
                                                 reinterpret_cast<uint4 *>(dst + (3 * w + j) * 1024), 16, 0, 0);
            }
            if (w < 4)
                __builtin_amdgcn_global_load_lds(lnorm, reinterpret_cast<float *>(dst + (SC_AFR + SC_BFR) * 1024 + w * 256),
                                                 4, 0, 0);
            if (w == 4) {
                // the block's tile words as dwords: lanes 0-7 validity (tile
                // lane >> 1, half lane & 1), 8-15 allow; the epilogue reads them
                // from LDS (a scalar load there waited the full memory latency:
                // the words fall out of L2 behind the row stream)
                const uint32_t wi = (uint32_t)(lane & 7) >> 1, half = lane & 1;
                const uint64_t t = a.tile_begin + lb * 4 + wi;
                const uint32_t *src = reinterpret_cast<const uint32_t *>(a.valid + (t < a.tile_end ? t : a.tile_end - 1)) + half;
                if (lane >= 8 && lane < 16 && a.allow) {
                    const uint64_t aw = t - a.allow_t0;
                    src = reinterpret_cast<const uint32_t *>(a.allow + (aw < a.allow_words ? aw : 0)) + half;
                }
                __builtin_amdgcn_global_load_lds(src, reinterpret_cast<uint32_t *>(dst + (SC_AFR + SC_BFR + 1) * 1024),
                                                 4, 0, 0);
            }
        };
        auto next_block = [&]() {  // the load cursor moves to the next row block
#pragma unroll
            for (int j = 0; j < 3; j++) lsrc[j] += lblkstep[j];
            lnorm += 256;
        };
        // wait until at most `younger` stages' loads of this wave are in flight
        auto wait_stages = [&](int younger) {
#ifdef WVG_TOOLS
            if (a.diag & 1) return;
#endif
            if (w < 5) {
                if (younger >= 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
                else if (younger == 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
                else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            } else {
                if (younger >= 2) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
                else if (younger == 1) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
                else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
        };
        auto raw_barrier = [&]() {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");
        };
        const int qlane = 4 * (lane >> 4);
        uint64_t qlive[2][4];
#pragma unroll
        for (int mq = 0; mq < 2; mq++)
#pragma unroll
            for (int r = 0; r < 4; r++)
                qlive[mq][r] = __ballot(q0 + 32 * wq + 16 * mq + qlane + r < a.nq);
        uint64_t *WL = lists + (size_t)w * 32 * M;
        float *WT = tau + w * 32, *WS = sig + w * 32;
        // +inf when one of this lane's queries is not fast-eligible (K1 > 2^50: a
        // huge or non-finite query), so its elements always take the exact test
        float lane_force = -__builtin_inff();
#pragma unroll
        for (int mq = 0; mq < 2; mq++)
#pragma unroll
            for (int r = 0; r < 4; r++)
                if (!(ck1[32 * wq + 16 * mq + qlane + r] <= 0x1p50f)) lane_force = __builtin_inff();

        floatx4 acc[2][8];
#pragma unroll
        for (int mq = 0; mq < 2; mq++)
#pragma unroll
            for (int nr = 0; nr < 8; nr++) acc[mq][nr] = (floatx4){0.f, 0.f, 0.f, 0.f};
        // the (row block, stage) units of the range form one stream: unit u in
        // buffer u % 4, loaded three units ahead
        const uint64_t U = (blk1 - blk0) * NK;
        uint64_t lblk = blk0, blk = blk0;  // load cursor (three units ahead), compute cursor
        uint32_t lks = 0, ks = 0;
        auto unit_load = [&](uint64_t u) {
            load_stage(smem + (u & (SC_NBUF - 1)) * SC_STAGE, lks, lblk);
            if (++lks == NK) {
                lks = 0;
                ++lblk;
                next_block();
            }
        };
        for (uint64_t u = 0; u < 3 && u < U; u++) unit_load(u);
        wait_stages(U >= 3 ? 2 : (int)U - 1);
        raw_barrier();
        for (uint64_t u = 0;; u++) {
            if (u + 3 < U) unit_load(u + 3);  // buffer (u + 3) % 4 was last read in unit u - 1
            const unsigned char *sb = smem + (u & (SC_NBUF - 1)) * SC_STAGE;
            {
                bf16x8 av[2], bv[8];
#pragma unroll
                for (int mq = 0; mq < 2; mq++)
                    av[mq] = *reinterpret_cast<const bf16x8 *>(sb + (2 * wq + mq) * 1024 + lane * 16);
#pragma unroll
                for (int nr = 0; nr < 8; nr++)
                    bv[nr] = *reinterpret_cast<const bf16x8 *>(sb + (SC_AFR + 8 * wr + nr) * 1024 + lane * 16);
#pragma unroll
                for (int mq = 0; mq < 2; mq++)
#pragma unroll
                    for (int nr = 0; nr < 8; nr++)
                        acc[mq][nr] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[mq], bv[nr], acc[mq][nr], 0, 0, 0);
            }
#ifdef WVG_TOOLS
            const bool epi = ks == NK - 1 && !(a.diag & 2);
#else
            const bool epi = ks == NK - 1;
#endif
            if (epi) {
                // epilogue of row block blk: C layout row (query) qlane + r, column (row) lane & 15
                // The epilogue's LDS reads go through inline asm: the compiler's
                // wait pass cannot tell them from reads of an in-flight LDS DMA
                // buffer and would drain the whole prefetch (vmcnt(0)) first.
                // None of them touches a buffer with a DMA in flight (the norms
                // sit in this unit's buffer, which landed before the barrier).
                float nrm[8];
                const uint32_t nrs = (uint32_t)(uintptr_t)(sb + (SC_AFR + SC_BFR) * 1024) +
                                     4u * (uint32_t)((2 * wr) * 64 + (lane & 15));
                asm volatile("ds_read_b32 %0, %8\n\t"
                             "ds_read_b32 %1, %8 offset:64\n\t"
                             "ds_read_b32 %2, %8 offset:128\n\t"
                             "ds_read_b32 %3, %8 offset:192\n\t"
                             "ds_read_b32 %4, %8 offset:256\n\t"
                             "ds_read_b32 %5, %8 offset:320\n\t"
                             "ds_read_b32 %6, %8 offset:384\n\t"
                             "ds_read_b32 %7, %8 offset:448\n\t"
                             "s_waitcnt lgkmcnt(0)"
                             : "=v"(nrm[0]), "=v"(nrm[1]), "=v"(nrm[2]), "=v"(nrm[3]), "=v"(nrm[4]), "=v"(nrm[5]),
                               "=v"(nrm[6]), "=v"(nrm[7])
                             : "v"(nrs)
                             : "memory");
                uint64_t vm[2];
                {
                    uint4 vw, aw4;
                    const uint32_t wa = (uint32_t)(uintptr_t)(sb + (SC_AFR + SC_BFR + 1) * 1024) + 16u * (uint32_t)wr;
                    asm volatile("ds_read_b128 %0, %2\n\t"
                                 "ds_read_b128 %1, %2 offset:32\n\t"
                                 "s_waitcnt lgkmcnt(0)"
                                 : "=v"(vw), "=v"(aw4)
                                 : "v"(wa)
                                 : "memory");
                    const uint64_t words[2] = {((uint64_t)vw.y << 32) | vw.x, ((uint64_t)vw.w << 32) | vw.z};
                    const uint64_t allows[2] = {((uint64_t)aw4.y << 32) | aw4.x, ((uint64_t)aw4.w << 32) | aw4.z};
#pragma unroll
                    for (int h = 0; h < 2; h++) {
                        const uint64_t t = a.tile_begin + blk * 4 + 2 * wr + h;
                        uint64_t m = t < a.tile_end ? readfirstlane64(words[h]) : 0ull;
                        if (a.allow) {
                            const uint64_t aw = t - a.allow_t0;
                            m &= aw < a.allow_words ? readfirstlane64(allows[h]) : 0ull;
                        }
                        vm[h] = m;
                    }
                }
                float k1r[2][4], k2r[2][4], svr[2][4];
#pragma unroll
                for (int mq = 0; mq < 2; mq++) {
                    float4 k1v, k2v, sv;
                    asm volatile("ds_read_b128 %0, %3\n\t"
                                 "ds_read_b128 %1, %4\n\t"
                                 "ds_read_b128 %2, %5\n\t"
                                 "s_waitcnt lgkmcnt(0)"
                                 : "=v"(k1v), "=v"(k2v), "=v"(sv)
                                 : "v"((uint32_t)(uintptr_t)(ck1 + 32 * wq + 16 * mq + qlane)),
                                   "v"((uint32_t)(uintptr_t)(ck2 + 32 * wq + 16 * mq + qlane)),
                                   "v"((uint32_t)(uintptr_t)(WS + 16 * mq + qlane))
                                 : "memory");
                    k1r[mq][0] = k1v.x, k1r[mq][1] = k1v.y, k1r[mq][2] = k1v.z, k1r[mq][3] = k1v.w;
                    k2r[mq][0] = k2v.x, k2r[mq][1] = k2v.y, k2r[mq][2] = k2v.z, k2r[mq][3] = k2v.w;
                    svr[mq][0] = sv.x, svr[mq][1] = sv.y, svr[mq][2] = sv.z, svr[mq][3] = sv.w;
                }
                // Fast check, branch-free: the largest u - sigma over this
                // lane's 64 elements.  On the fast-eligible inputs (query K1 <=
                // 2^50, row norm bound <= 2^60) every u is finite and sigma is
                // finite or +-inf, so u - sigma is never NaN and its sign is
                // exactly that of u - sigma; a huge / non-finite query
                // (lane_force = +inf) or row forces the exact path below, which
                // is the per-element test (NaN-safe) with the list insertions.
                const bool all_valid = (vm[0] & vm[1]) == ~0ull;
                float mx = -__builtin_inff(), mnr_a[8];
#pragma unroll
                for (int nr = 0; nr < 8; nr++) {
                    float mnr = lane_force;
#pragma unroll
                    for (int mq = 0; mq < 2; mq++)
#pragma unroll
                        for (int r = 0; r < 4; r++) {
                            const float u = acc[mq][nr][r] + __builtin_fmaf(nrm[nr], k1r[mq][r], k2r[mq][r]);
                            mnr = __builtin_fmaxf(mnr, u - svr[mq][r]);
                        }
                    mnr = nrm[nr] <= 0x1p60f ? mnr : __builtin_inff();
                    if (!all_valid) {
                        const uint32_t m16 = (uint32_t)(vm[nr >> 2] >> (16 * (nr & 3)));
                        mnr = (m16 >> (lane & 15)) & 1u ? mnr : -__builtin_inff();
                    }
                    mnr_a[nr] = mnr;
                    mx = __builtin_fmaxf(mx, mnr);
                }
#ifdef WVG_TOOLS
                n_blk++;
                const bool slow = __ballot(mx >= 0.f) && !(a.diag & 4);
                n_slow += slow;
#else
                const bool slow = __ballot(mx >= 0.f);
#endif
                if (slow) {
                // only the row groups where some lane passed the fast check (their
                // elements' exact tests are the only ones that can pass)
#pragma unroll
                for (int nr = 0; nr < 8; nr++) {
                    if (!__ballot(mnr_a[nr] >= 0.f)) continue;
#pragma unroll
                    for (int mq = 0; mq < 2; mq++) {
                        const uint64_t m16 = (vm[nr >> 2] >> (16 * (nr & 3))) & 0xFFFFull;
                        const uint64_t m64 = m16 * 0x0001000100010001ull;
#pragma unroll
                        for (int r = 0; r < 4; r++) {
                            const float u = acc[mq][nr][r] + __builtin_fmaf(nrm[nr], k1r[mq][r], k2r[mq][r]);
                            uint64_t pass = __ballot(!(u < svr[mq][r])) & m64 & qlive[mq][r];
                            while (pass) {  // rare after the first row blocks of a range
                                const int src = __builtin_ctzll(pass);
                                pass &= pass - 1;
                                const int ql = 16 * mq + 4 * (src >> 4) + r;
                                const float us = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(u), src));
                                const uint32_t slot = (uint32_t)((a.tile_begin + blk * 4) * 64 + 128 * wr + 16 * nr +
                                                                 (src & 15));
#ifdef WVG_TOOLS
                                n_call++;
#endif
                                const float ws_now =
                                    sc_insert((lds_u64 *)(WL + ql * M), (lds_f32 *)(WT + ql), (lds_f32 *)(WS + ql), cem[32 * wq + ql], K, cosine, us, slot);
                                // the other lanes of this 16-lane group hold the same query
                                const uint64_t grp = 0xFFFFull << (16 * (src >> 4));
                                pass &= ~grp | __ballot(!(u < ws_now));
                            }
                        }
                    }
                }
                }
#pragma unroll
                for (int mq = 0; mq < 2; mq++)
#pragma unroll
                    for (int nr = 0; nr < 8; nr++) acc[mq][nr] = (floatx4){0.f, 0.f, 0.f, 0.f};
            }
            if (u + 1 >= U) break;
            if (++ks == NK) {
                ks = 0;
                ++blk;
            }
            // unit u + 1 landed (its loads are the oldest in flight), then everyone's
            wait_stages(u + 3 < U ? 2 : (u + 2 < U ? 1 : 0));
            raw_barrier();
        }
    }
publish:
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#ifdef WVG_TOOLS
    if (lane == 0) {
        atomicAdd(&g_screen_ctr[0], (unsigned long long)n_blk);
        atomicAdd(&g_screen_ctr[1], (unsigned long long)n_slow);
        atomicAdd(&g_screen_ctr[2], (unsigned long long)n_call);
    }
#endif
    __syncthreads();
    // merge the two row halves' lists per query (waves wq and wq + 4), by rank:
    // wave w takes queries w, w + 8, ... of the workgroup
    for (int qw = w; qw < SC_BQ; qw += SC_WAVES) {
        const uint32_t q = q0 + (uint32_t)qw;
        if (q >= a.nq) break;
        const int qq = qw >> 5, ql = qw & 31;
        const uint64_t x = lane < M ? lists[((size_t)qq * 32 + ql) * M + lane]
                                    : (lane < 2 * M ? lists[((size_t)(qq + 4) * 32 + ql) * M + lane - M] : WVG_KEY_NONE);
        int rank = 0;
        for (int j = 0; j < 2 * M; j++) {
            const uint64_t y = __shfl(x, j);
            rank += (y < x) || (y == x && j < lane);
        }
        uint64_t *out = a.partials + ((size_t)q * a.nrr + rr) * M;
        if (lane < 2 * M && rank < M) out[rank] = x;
        if (lane < 2 * M && rank == K - 1 && x != WVG_KEY_NONE) {
            const float t = sc_tau_k(key_lower(x), cem[qw], cosine);
            atomicMin(a.gbound + q, wvg_ord_f32(t));
        }
    }
}

// ---------------------------------------------------------------------------
// K3d: K3c with the queries resident in registers (d = 32 KBN, KBN in {16, 24}).
// A workgroup = 4 waves, one per SIMD, 128 queries (32 per wave) whose bf16
// fragments for every K block are loaded once into VGPRs / AGPRs; only the row
// fragments stream through LDS: per 32-deep stage 16 KiB (256 rows) by LDS DMA
// into a ring of 8 stage buffers, six stages in flight (loads past the range
// end re-read its last block, so every stage issues the same loads and the
// vmcnt waits are constants).  Per stage and wave: the first half of the rows'
// fragments (read one stage ahead) feeds 16 MFMAs while the second half is
// read; the barrier for the next stage sits between the halves; the next
// stage's first half is read during the second half's MFMAs.  Against K3c per
// 128 x 256 x 32 tile: 16 KiB instead of 25 KiB from L2 (no query fragments,
// one norm copy) and 64 KiB instead of 80 KiB of LDS reads.  The bound and
// the partials are K3c's.
//
// Survivors (round 4).  The epilogue of a row block only APPENDS its
// survivors -- (u, query, row) -- to a per-wave LDS queue (one ballot, one
// mbcnt and one ds_write per element group with a survivor); after the
// epilogue ONE code site drains the queue into the wave's lists, which live
// in registers (SurvivorLists), and refreshes the query thresholds the next
// block's fast check reads.  The round-3 kernel called an out-of-line
// insertion at each of the 128 unrolled epilogue sites: the call ABI spilled
// registers around the main loop, and every spill reload is a scratch load
// counted in vmcnt, so each epilogue ended in vmcnt(0) -- a drain of the six
// stages in flight (profiles/r03/k3d_ab: the stage loop alone ran at 75% of
// the bf16 peak, the product kernel at 32%).  Nothing in the loop now waits on
// vmcnt except the ring's constant waits.
constexpr int SD_WAVES = 4;
constexpr int SD_BQ = 128;
constexpr int SD_BFR = 16;
constexpr int SD_STAGE = SD_BFR * 1024;
constexpr int SD_NBUF = 8;
constexpr int SD_NSLOT = 1280;
constexpr int SD_RING = SD_NBUF * SD_STAGE + 2 * SD_NSLOT;
constexpr int SD_LISTS = SD_WAVES * 32 * SCREEN_M * 8;
constexpr int SD_LDS = SD_RING + SD_LISTS + SD_WAVES * 32 * 4 * 2 + SD_BQ * 4 * 3;
static_assert(SD_LDS <= 160 * 1024, "K3d's LDS");

// K3i (round 6): K3d on an int8 shadow (below, "The int8 screen").  Its LDS:
// the ring holds NB stages (KBN % NB == 0: 6 for d = 768's 12 K blocks, else
// 8), a norm slot holds the block's row norms, tile words and row errors, and
// the per-query constants gain B (the row-norm coefficient) and the score scale.
constexpr int si_nbuf(int kbn) { return kbn % 8 == 0 ? 8 : 6; }
constexpr int SI_NSLOT = 2304;  // norms [0, 1024), tile words [1024, 1088), row errors [1280, 2304)
constexpr int si_ring(int nb) { return nb * SD_STAGE + 2 * SI_NSLOT; }
constexpr int si_lds(int nb) { return si_ring(nb) + SD_LISTS + SD_WAVES * 32 * 4 * 2 + SD_BQ * 4 * 5; }
static_assert(si_lds(8) <= 160 * 1024, "K3i's LDS");

// One accumulator element read where it is used.  Through C++ the compiler
// copies the whole accumulator tile into VGPRs at the top of the epilogue (~100
// live VGPRs next to the resident queries: spills); the asm names the element
// in its AGPR, and asm statements keep their program order.
__device__ __forceinline__ float agpr_read(float x)
{
    float r;
    asm volatile("v_accvgpr_read_b32 %0, %1" : "=v"(r) : "a"(x));
    return r;
}
// (K3i) an int32 accumulator element
__device__ __forceinline__ int agpr_read(int x)
{
    int r;
    asm volatile("v_accvgpr_read_b32 %0, %1" : "=v"(r) : "a"(x));
    return r;
}

__device__ __forceinline__ uint64_t readlane64(uint64_t v, int l)
{
    return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l) << 32) |
           (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
}

// lane i of each 16-lane row takes lane i - 1's value (DPP row_shr:1; lane 0 keeps its own)
__device__ __forceinline__ uint64_t row_shr1_64(uint64_t v)
{
    const int lo = __builtin_amdgcn_update_dpp((int)(uint32_t)v, (int)(uint32_t)v, 0x111, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp((int)(uint32_t)(v >> 32), (int)(uint32_t)(v >> 32), 0x111, 0xF, 0xF,
                                               false);
    return ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo;
}

// A wave's survivor lists: the SCREEN_M smallest (lower, slot) keys of each of
// its 32 queries, ascending, in LDS (32 x 16 keys); a group of the epilogue
// holds four of them in one register (see the slow path).
struct SurvivorLists {
    uint32_t laddr;  // LDS byte address of the wave's 32 lists
};

// Compile-time loop (the K-block loop of K3d): the body sees its index as a
// constant, so per-unit load counts and vmcnt waits are immediates.
template <typename F, int... I>
__device__ __forceinline__ void sd_static_for(F &f, std::integer_sequence<int, I...>)
{
    (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void sd_static_for(F &&f)
{
    sd_static_for(f, std::make_integer_sequence<int, N>{});
}

// Vector-memory loads one K3d wave issues for unit u (K block u of a row
// block): its 4 row-fragment pieces, and with unit 0 the block's row norms of
// its tile (+ wave 0: the block's tile words).  DIAG 256 (tools): round 3's
// norms / words with every unit.
template <int DIAG, bool I8 = false>
constexpr int sd_unit_loads(int u, bool w0)
{
    if ((DIAG & 128) != 0) return 0;
    if ((DIAG & 32) != 0) return 4;
    if ((DIAG & 256) != 0) return 5 + (w0 ? 1 : 0);
    return 4 + (u == 0 ? 1 + (I8 ? 1 : 0) + (w0 ? 1 : 0) : 0);  // (K3i: + the row errors)
}
// The loads issued after unit `first`'s, over units first + 1 .. first + n (mod KBN)
template <int KBN, int DIAG, bool I8 = false>
constexpr int sd_younger(int first, int n, bool w0)
{
    int c = 0;
    for (int i = 1; i <= n; i++) c += sd_unit_loads<DIAG, I8>((first + i) % KBN, w0);
    return c;
}

// DIAG (tools build only; 0 in the product): bit 0 = no wait for the stage
// loads, bit 1 = no epilogue (alone it lets the compiler delete the MFMAs, as
// the round-3 "stage loop alone" diagnostics did: their 8.3 ms had no MFMA),
// bit 1 + bit 3 (10) = the stage loop with its MFMAs and a one-sum consumer,
// bit 2 = tests but no survivor queue, bit 4 = count row blocks / blocks with
// survivors / queued survivors.  Compile-time, so the tools build's DIAG = 0
// kernel is the product kernel, register allocation included.
//
// I8 (K3i, round 6): the same kernel on the int8 shadow -- 64-deep K blocks
// of v_mfma_i32_16x16x64_i8 (twice the bf16 rate: a K block is the same
// instruction count and the same 16 KiB stage for twice the depth), exact
// int32 scores scaled once per element, and the two-term bound of "The int8
// screen" below (row norm and row quantization error).
template <int KBN, int DIAG = 0, bool I8 = false>
__global__ __launch_bounds__(SD_WAVES * 64, 1) void screen_ar_kernel(ScreenArgs a)
{
    constexpr int NB = I8 ? si_nbuf(KBN) : SD_NBUF;  // stage buffers
    constexpr int NSLOT = I8 ? SI_NSLOT : SD_NSLOT;
    constexpr int RING = NB * SD_STAGE + 2 * NSLOT;
    static_assert(KBN % NB == 0, "the stage buffer of a K block must be a compile-time constant");
    static_assert(!I8 || (DIAG & ~(2 | 8)) == 0, "K3i: only the stage-loop diagnostic");
    using frag_t = std::conditional_t<I8, i32x4, bf16x8>;
    using acc_t = std::conditional_t<I8, i32x4, floatx4>;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    uint64_t *lists = reinterpret_cast<uint64_t *>(smem + RING);  // [4][32][M]
    float *tau = reinterpret_cast<float *>(smem + RING + SD_LISTS);
    float *sig = tau + SD_WAVES * 32;
    float *ck1 = sig + SD_WAVES * 32;
    float *ck2 = ck1 + SD_BQ;
    float *cem = ck2 + SD_BQ;
    float *ckb = cem + SD_BQ;  // (I8) B
    float *ccs = ckb + SD_BQ;  // (I8) score scale
    uint32_t n_blk = 0, n_slow = 0, n_call = 0, n_grp = 0;  // (DIAG & 16)
    (void)n_blk, (void)n_slow, (void)n_call, (void)n_grp;
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int K = (int)a.k, M = SCREEN_M;
    const int cosine = a.cosine;
    const uint32_t b = blockIdx.x;
    uint32_t qb, rr;
    if (a.nrr_l % 8 == 0) {
        const uint32_t xcd = b % 8, wv = b / 8;
        qb = wv % a.nqb;
        rr = a.rr0 + (wv / a.nqb) * 8 + xcd;
    } else {
        qb = b % a.nqb;
        rr = a.rr0 + b / a.nqb;
    }
    const uint64_t ntiles = a.tile_end - a.tile_begin;
    const uint64_t nblk = (ntiles + 3) / 4;
    uint64_t blk0, blk1;
    sc_range(a, nblk, rr, blk0, blk1);
    const uint32_t q0 = qb * SD_BQ;

    for (int i = tid; i < SD_BQ; i += SD_WAVES * 64) {
        const uint32_t q = q0 + (uint32_t)i;
        ck1[i] = a.k1[q];
        ck2[i] = a.k2[q];
        cem[i] = a.emax[q];
        if constexpr (I8) {
            ckb[i] = a.kb[q];
            ccs[i] = a.css[q];
        }
    }
    for (int i = tid; i < SD_WAVES * 32; i += SD_WAVES * 64) {
        const uint32_t q = q0 + (uint32_t)i;
        const uint32_t g = q < a.nq ? __hip_atomic_load(a.gbound + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
        const float t = q >= a.nq ? -__builtin_inff() : (g == 0xFFFFFFFFu ? __builtin_inff() : wvg_unord_f32(g));
        tau[i] = t;
        sig[i] = q >= a.nq ? __builtin_inff() : sc_sigma(t, cosine);
    }
    for (int i = tid; i < SD_WAVES * 32 * M; i += SD_WAVES * 64) lists[i] = WVG_KEY_NONE;
    __syncthreads();
    SurvivorLists S;
    S.laddr = (uint32_t)(uintptr_t)(lists + (size_t)w * 32 * M);
    // the wave's per-query thresholds WT (tau), their u-space form WS (sig) and Emax
    // (cem): LDS byte address of tau[w][0]; sig, ck1, ck2, cem at + 512, + 1024, + 1536,
    // + 2048 (I8: ckb, ccs at + 2560, + 3072)
    const uint32_t tbase = (uint32_t)(uintptr_t)(tau + w * 32);
    if (blk0 < blk1) {
        // the wave's 32 queries, every K block, resident for the whole range
        frag_t areg[KBN][2];
        // The first SD_AKB K blocks' fragments live in AGPRs (an MFMA A operand may be
        // an AGPR), the rest in VGPRs: 128 accumulator + 64 B-fragment + 48 such AGPRs,
        // which leaves the epilogue ~100 VGPRs -- with all 192 in VGPRs the compiler
        // spilled query fragments around the epilogue, and a scratch reload before the
        // loop costs a vmcnt(0) (a drain of the stage ring) at every row block.
        constexpr int SD_AKB = 6;
        const uint4 *qsrc = a.qfrag + (size_t)(qb * 8 + 2 * w) * KBN * 64 + lane;
#pragma unroll
        for (int ks = 0; ks < KBN; ks++)
#pragma unroll
            for (int mq = 0; mq < 2; mq++) {
                const uint4 *src = qsrc + ((size_t)mq * KBN + ks) * 64;
                if (ks < SD_AKB)
                    asm volatile("global_load_dwordx4 %0, %1, off" : "=a"(areg[ks][mq]) : "v"(src) : "memory");
                else
                    asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(areg[ks][mq]) : "v"(src) : "memory");
            }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
        for (int ks = 0; ks < KBN; ks++)
#pragma unroll
            for (int mq = 0; mq < 2; mq++) {
                if (ks < SD_AKB)
                    asm volatile("" : "+a"(areg[ks][mq]));
                else
                    asm volatile("" : "+v"(areg[ks][mq]));
            }

        // loads of one stage: wave w moves row fragments 4w .. 4w+3 (tile w,
        // row groups 0..3); with unit 0 also the norms of tile w, and wave 0
        // the block's tile words (sd_unit_loads).  Round 3 reloaded the norms
        // and words with every unit: 25 % more LDS-DMA issues per unit.
        const uint4 *lsrc = a.shadow + ((size_t)(a.tile_begin + blk0 * 4 + w) * KBN * 4) * 64 + lane;
        const float *lnorm = a.norms + (a.tile_begin + blk0 * 4 + w) * 64 + lane;
        const float *lerr = I8 ? a.errs + (a.tile_begin + blk0 * 4 + w) * 64 + lane : nullptr;
        uint64_t lblk = blk0;
        auto load_stage = [&](int ks) {
            if constexpr ((DIAG & 128) != 0) return;
            unsigned char *dst = smem + (ks % NB) * SD_STAGE;
#pragma unroll
            for (int rg = 0; rg < 4; rg++)
                __builtin_amdgcn_global_load_lds(lsrc + ((size_t)ks * 4 + rg) * 64,
                                                 reinterpret_cast<uint4 *>(dst + (4 * w + rg) * 1024), 16, 0, 0);
            unsigned char *nslot = smem + NB * SD_STAGE + (lblk & 1) * NSLOT;
            // the block's norms / tile words with its unit 0 (sd_unit_loads: the waits count them)
            const bool with_norms = (DIAG & 32) == 0 && ((DIAG & 256) != 0 || ks == 0);
            if (with_norms)
                __builtin_amdgcn_global_load_lds(lnorm, reinterpret_cast<float *>(nslot + w * 256), 4, 0, 0);
            if (I8 && with_norms)
                __builtin_amdgcn_global_load_lds(lerr, reinterpret_cast<float *>(nslot + 1280 + w * 256), 4, 0, 0);
            if (with_norms && w == 0) {
                const uint32_t wi = (uint32_t)(lane & 7) >> 1, half = lane & 1;
                const uint64_t t = a.tile_begin + lblk * 4 + wi;
                const uint32_t *src =
                    reinterpret_cast<const uint32_t *>(a.valid + (t < a.tile_end ? t : a.tile_end - 1)) + half;
                if (lane >= 8 && lane < 16 && a.allow) {
                    const uint64_t aw = t - a.allow_t0;
                    src = reinterpret_cast<const uint32_t *>(a.allow + (aw < a.allow_words ? aw : 0)) + half;
                }
                __builtin_amdgcn_global_load_lds(src, reinterpret_cast<uint32_t *>(nslot + 1024), 4, 0, 0);
            }
            if (ks == KBN - 1 && lblk + 1 < blk1) {  // the load cursor moves on; past the end it stays
                ++lblk;
                lsrc += (size_t)4 * KBN * 4 * 64;
                lnorm += 256;
                if constexpr (I8) lerr += 256;
            }
        };
        // six stages in flight at every wait: unit ks + 1 (waited for at K block ks) + the 5
        // younger units ks + 2 .. ks + 6, whose loads the wait leaves outstanding
        // PAIR (tools A/B, DIAG 1024): one wait + barrier per two K blocks -- at even ks for
        // unit ks + 2 (units ks + 3 .. ks + 6 outstanding), which also covers the odd
        // iteration's reads of unit ks + 1; the two units ks + 7, ks + 8 load after it
        // (K3i with NB = 6: four stages in flight, three left outstanding)
        constexpr bool PAIR = (DIAG & 1024) != 0;
        auto wait_next = [&](auto KS) {
            if constexpr ((DIAG & 129) != 0) return;
            constexpr int ks = decltype(KS)::value;
            if constexpr (PAIR && (ks & 1) != 0) return;
            constexpr int first = PAIR ? ks + 2 : ks + 1, n = PAIR ? NB - 4 : NB - 3;
            constexpr int n0 = sd_younger<KBN, DIAG, I8>(first, n, true);
            constexpr int n1 = sd_younger<KBN, DIAG, I8>(first, n, false);
            if (w == 0) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(n0) : "memory");
            else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(n1) : "memory");
        };
        auto raw_barrier = [&]() {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            if constexpr ((DIAG & 64) == 0) __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");
        };
        // Half a stage's row fragments straight into AGPRs (the MFMA B operand may
        // be an AGPR): the 512 registers hold the resident queries (192 VGPRs), the
        // accumulators (128 AGPRs) and both halves (64 AGPRs), which leaves the
        // VGPRs the epilogue needs.  The reads are asynchronous to the compiler:
        // every consumer first passes a wait that names the registers (wait_b0,
        // and the barrier's lgkmcnt(0) + the "+a" fence for the second half).
        // One lane base address for every read: the stage / half offset is added
        // inside the asm from an SGPR (16 precomputed addresses cost 16 VGPRs).
        const uint32_t rbase = (uint32_t)(uintptr_t)smem + 16u * lane;
        auto read_half = [&](int ks, int h, frag_t (&br)[8]) {
            const uint32_t soff = (uint32_t)((ks % NB) * SD_STAGE + h * 8 * 1024);
            uint32_t tmp;
            asm volatile("v_add_u32 %8, %9, %10\n\t"
                         "ds_read_b128 %0, %8\n\t"
                         "ds_read_b128 %1, %8 offset:1024\n\t"
                         "ds_read_b128 %2, %8 offset:2048\n\t"
                         "ds_read_b128 %3, %8 offset:3072\n\t"
                         "ds_read_b128 %4, %8 offset:4096\n\t"
                         "ds_read_b128 %5, %8 offset:5120\n\t"
                         "ds_read_b128 %6, %8 offset:6144\n\t"
                         "ds_read_b128 %7, %8 offset:7168"
                         : "=a"(br[0]), "=a"(br[1]), "=a"(br[2]), "=a"(br[3]), "=a"(br[4]), "=a"(br[5]), "=a"(br[6]),
                           "=a"(br[7]), "=&v"(tmp)
                         : "s"(soff), "v"(rbase)
                         : "memory");
        };
        // the first half landed (the second half's eight reads may still be in flight)
        auto wait_b0 = [&](frag_t (&br)[8]) {
            asm volatile("s_waitcnt lgkmcnt(8)"
                         : "+a"(br[0]), "+a"(br[1]), "+a"(br[2]), "+a"(br[3]), "+a"(br[4]), "+a"(br[5]), "+a"(br[6]),
                           "+a"(br[7])
                         :
                         : "memory");
        };
        const int qlane = 4 * (lane >> 4);
        // epilogue lane bases: smem (+ the tile-word bytes, lane-independent), the
        // row norm of this lane's column, this lane's first query in sig / ck1 / ck2
        const uint32_t sbase = (uint32_t)(uintptr_t)smem;
        const uint32_t nbase = sbase + 4u * (uint32_t)(lane & 15);
        const uint32_t qbase = sbase + 4u * (uint32_t)qlane;
        const uint32_t csoff = (uint32_t)((uintptr_t)sig - (uintptr_t)smem);
        // +inf when one of this lane's queries is not fast-eligible (K1 > 2^50: a huge or
        // non-finite query), so its elements always take the exact test
        bool lane_force = false;
#pragma unroll
        for (int mq = 0; mq < 2; mq++)
#pragma unroll
            for (int r = 0; r < 4; r++)
                if (!(ck1[32 * w + 16 * mq + qlane + r] <= 0x1p50f)) lane_force = true;

        acc_t acc[2][16];
#pragma unroll
        for (int mq = 0; mq < 2; mq++)
#pragma unroll
            for (int nr = 0; nr < 16; nr++) acc[mq][nr] = acc_t{0, 0, 0, 0};
        frag_t b0[8], b1[8];
        // one K block of one 16 x 16 tile: bf16 16x16x32, or (I8) int8 16x16x64 with exact int32 sums
        auto mfma = [](const frag_t &x, const frag_t &y, const acc_t &c) -> acc_t {
            if constexpr (I8)
                return __builtin_amdgcn_mfma_i32_16x16x64_i8(x, y, c, 0, 0, 0);
            else
                return __builtin_amdgcn_mfma_f32_16x16x32_bf16(x, y, c, 0, 0, 0);
        };
        // prologue: units 0 .. NB - 2 of the range (a unit = one K block of one row
        // block; the ring holds K block ks of any row block in buffer ks % NB)
#pragma unroll
        for (int ks = 0; ks < NB - 1; ks++) load_stage(ks);
        // unit 0 landed: the NB - 2 younger units outstanding
        if (w == 0) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(sd_younger<KBN, DIAG, I8>(0, NB - 2, true)) : "memory");
        else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(sd_younger<KBN, DIAG, I8>(0, NB - 2, false)) : "memory");
        raw_barrier();
        read_half(0, 0, b0);
        for (uint64_t blk = blk0; blk < blk1; blk++) {
            sd_static_for<KBN>([&](auto KS) {
                constexpr int ks = decltype(KS)::value;
                read_half(ks, 1, b1);
                wait_b0(b0);
#pragma unroll
                for (int mq = 0; mq < 2; mq++)
#pragma unroll
                    for (int nr = 0; nr < 8; nr++) acc[mq][nr] = mfma(areg[ks][mq], b0[nr], acc[mq][nr]);
                wait_next(KS);  // the next unit landed
                if constexpr (!PAIR || (ks & 1) == 0)
                    raw_barrier();  // (lgkmcnt(0): this wave's second-half reads done)
                else
                    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
                for (int j = 0; j < 8; j++) asm volatile("" : "+a"(b1[j]));
                // unit + 7 into the buffer of unit - 1 (fully read before this barrier); PAIR:
                // also unit + 8 into the buffer of this unit (its reads done: the barrier's wait)
                if constexpr (!PAIR) {
                    load_stage((ks + NB - 1) % KBN);
                } else if constexpr ((ks & 1) == 0) {
                    load_stage((ks + NB - 1) % KBN);
                    load_stage((ks + NB) % KBN);
                }
                if (ks + 1 < KBN) read_half(ks + 1, 0, b0);  // (the next block's first half: after the epilogue)
#pragma unroll
                for (int mq = 0; mq < 2; mq++)
#pragma unroll
                    for (int nr = 0; nr < 8; nr++) acc[mq][8 + nr] = mfma(areg[ks][mq], b1[nr], acc[mq][8 + nr]);
            });
            // The epilogue reads the accumulators through inline asm (agpr_read), which the
            // compiler's hazard recognizer does not see: an MFMA's result may be read by a
            // VALU op only after its passes + 2 wait states (XDL write -> VALU read; 11 for an
            // 8-pass, 19 for a 16-pass op), so the block's last MFMAs get 24 here (the norm
            // reads that come first usually cover them; this makes it unconditional).
            __builtin_amdgcn_sched_barrier(0);
            asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
            __builtin_amdgcn_sched_barrier(0);
            // epilogue of row block blk (K3c's, over 16 row groups): C layout row
            // (query) qlane + r, column (row) 16 nr + (lane & 15)
            if constexpr ((DIAG & 2) == 0) {
                // Fast check per query group, then the exact test !(u < WS) (NaN-safe: a
                // non-finite row or query always passes) on the groups the check could not
                // rule out, survivors inserted into register-held lists (the slow path
                // below).  Accumulators are read where they are used (agpr_read); every
                // epilogue LDS access is inline asm with its own lgkmcnt wait (through C++
                // the compiler cannot tell them from the stage ring's LDS DMA and waits
                // vmcnt(0), draining the prefetch), at a lane base + an SGPR offset.
                const uint32_t nsoff = (uint32_t)(NB * SD_STAGE + (blk & 1) * NSLOT);  // the block's norms
                // row norms of row groups 8 hh .. 8 hh + 7 (hh 2, 3: I8's row errors, slot bytes 1280 ..)
                auto read_norms8 = [&](int hh, float (&nrm)[8]) {
                    uint32_t tmp;
                    asm volatile("v_add_u32 %8, %9, %10\n\t"
                                 "ds_read_b32 %0, %8\n\t"
                                 "ds_read_b32 %1, %8 offset:64\n\t"
                                 "ds_read_b32 %2, %8 offset:128\n\t"
                                 "ds_read_b32 %3, %8 offset:192\n\t"
                                 "ds_read_b32 %4, %8 offset:256\n\t"
                                 "ds_read_b32 %5, %8 offset:320\n\t"
                                 "ds_read_b32 %6, %8 offset:384\n\t"
                                 "ds_read_b32 %7, %8 offset:448\n\t"
                                 "s_waitcnt lgkmcnt(0)"
                                 : "=v"(nrm[0]), "=v"(nrm[1]), "=v"(nrm[2]), "=v"(nrm[3]), "=v"(nrm[4]),
                                   "=v"(nrm[5]), "=v"(nrm[6]), "=v"(nrm[7]), "=&v"(tmp)
                                 : "s"(nsoff + (hh < 2 ? 512u * hh : 1280u + 512u * (hh - 2))), "v"(nbase)
                                 : "memory");
                };
                auto read_consts = [&](int mq, float (&k1r)[4], float (&k2r)[4], float (&svr)[4]) {
                    // sig, ck1, ck2 are consecutive 128-float arrays: one address, offsets 0 / 512 / 1024
                    const uint32_t coff = (uint32_t)(csoff + 4 * (32 * w + 16 * mq));
                    float4 k1v, k2v, sv;
                    uint32_t tmp;
                    asm volatile("v_add_u32 %3, %4, %5\n\t"
                                 "ds_read_b128 %0, %3 offset:512\n\t"
                                 "ds_read_b128 %1, %3 offset:1024\n\t"
                                 "ds_read_b128 %2, %3\n\t"
                                 "s_waitcnt lgkmcnt(0)"
                                 : "=v"(k1v), "=v"(k2v), "=v"(sv), "=&v"(tmp)
                                 : "s"(coff), "v"(qbase)
                                 : "memory");
                    k1r[0] = k1v.x, k1r[1] = k1v.y, k1r[2] = k1v.z, k1r[3] = k1v.w;
                    k2r[0] = k2v.x, k2r[1] = k2v.y, k2r[2] = k2v.z, k2r[3] = k2v.w;
                    svr[0] = sv.x, svr[1] = sv.y, svr[2] = sv.z, svr[3] = sv.w;
                };
                // (I8) B and the score scale of the lane's four queries of half mq: ckb, ccs at
                // sig + 2048, + 2560
                auto read_consts_i8 = [&](int mq, float (&kbr)[4], float (&csr)[4]) {
                    const uint32_t coff = (uint32_t)(csoff + 4 * (32 * w + 16 * mq));
                    float4 kbv, csv;
                    uint32_t tmp;
                    asm volatile("v_add_u32 %2, %3, %4\n\t"
                                 "ds_read_b128 %0, %2 offset:2048\n\t"
                                 "ds_read_b128 %1, %2 offset:2560\n\t"
                                 "s_waitcnt lgkmcnt(0)"
                                 : "=v"(kbv), "=v"(csv), "=&v"(tmp)
                                 : "s"(coff), "v"(qbase)
                                 : "memory");
                    kbr[0] = kbv.x, kbr[1] = kbv.y, kbr[2] = kbv.z, kbr[3] = kbv.w;
                    csr[0] = csv.x, csr[1] = csv.y, csr[2] = csv.z, csr[3] = csv.w;
                };
                (void)read_consts_i8;
                if constexpr ((DIAG & 16) != 0) n_blk++;
                // fast check: the lane's 16 rows' largest norm bound bounds each of their E
                // (E = fma(norm, K1q, K2q) is monotone in the norm), so per query the largest
                // raw score of the lane's rows + that E against WS is a superset test of
                // every element (monotone roundings); finite on the fast-eligible inputs
                // (query K1 <= 2^50, row norms <= 2^60), else the exact test runs
                // TIGHT (tools A/B, DIAG 2048): the check on each element's own u (its row's E),
                // i.e. exactly the exact test's verdict per group, at 32 more VALU per group
                constexpr bool TIGHT = (DIAG & 2048) != 0;
                float nmax, nsum;  // (nsum: NaN when a norm is -- fmaxf would drop it)
                float nrmt[TIGHT ? 16 : 1];
                {
                    float n0[8], n1[8];
                    read_norms8(0, n0);
                    read_norms8(1, n1);
                    nmax = n0[0];
                    nsum = n0[0];
#pragma unroll
                    for (int j2 = 1; j2 < 8; j2++) nmax = __builtin_fmaxf(nmax, n0[j2]), nsum += n0[j2];
#pragma unroll
                    for (int j2 = 0; j2 < 8; j2++) nmax = __builtin_fmaxf(nmax, n1[j2]), nsum += n1[j2];
                    if constexpr (TIGHT) {
#pragma unroll
                        for (int j2 = 0; j2 < 8; j2++) nrmt[j2] = n0[j2], nrmt[8 + j2] = n1[j2];
                    }
                }
                // (I8) the lane's 16 rows' largest error bound: E = fma(err, A, fma(norm, B, K2))
                // is monotone in both
                float emx = 0.f, esum = 0.f;
                if constexpr (I8) {
                    float e0[8], e1[8];
                    read_norms8(2, e0);
                    read_norms8(3, e1);
                    emx = e0[0];
                    esum = e0[0];
#pragma unroll
                    for (int j2 = 1; j2 < 8; j2++) emx = __builtin_fmaxf(emx, e0[j2]), esum += e0[j2];
#pragma unroll
                    for (int j2 = 0; j2 < 8; j2++) emx = __builtin_fmaxf(emx, e1[j2]), esum += e1[j2];
                }
                // per (query half mq, query r of the lane's four): whether some lane cannot rule
                // out its 16 elements -- only those groups run the exact test (a wave-uniform
                // bit each; typically one or two of the eight)
                const bool force = lane_force || !(nmax <= 0x1p60f) || nsum != nsum || !(emx <= 0x1p60f) || esum != esum;
                uint32_t wact = 0;
#pragma unroll
                for (int mq = 0; mq < 2; mq++) {
                    float k1r[4], k2r[4], svr[4];
                    read_consts(mq, k1r, k2r, svr);
                    if constexpr (I8) {
                        // the largest exact int32 score, scaled once (rounding is monotone)
                        float kbr[4], csr[4];
                        read_consts_i8(mq, kbr, csr);
#pragma unroll
                        for (int r = 0; r < 4; r++) {
                            int mi = agpr_read(acc[mq][0][r]);
#pragma unroll
                            for (int nr = 1; nr < 16; nr++) mi = max(mi, agpr_read(acc[mq][nr][r]));
                            const float m = (float)mi * csr[r];
                            const float t =
                                (m + __builtin_fmaf(emx, k1r[r], __builtin_fmaf(nmax, kbr[r], k2r[r]))) - svr[r];
                            if (__ballot(force || t >= 0.f)) wact |= 1u << (4 * mq + r);
                        }
                        continue;
                    }
#pragma unroll
                    for (int r = 0; r < 4; r++) {
                        float t;
                        if constexpr (TIGHT) {
                            float m = -__builtin_inff();
#pragma unroll
                            for (int nr = 0; nr < 16; nr++)
                                m = __builtin_fmaxf(m, agpr_read(acc[mq][nr][r]) + __builtin_fmaf(nrmt[nr], k1r[r], k2r[r]));
                            t = m - svr[r];
                        } else {
                            float m = agpr_read(acc[mq][0][r]);
#pragma unroll
                            for (int nr = 1; nr < 16; nr++) m = __builtin_fmaxf(m, agpr_read(acc[mq][nr][r]));
                            t = (m + __builtin_fmaf(nmax, k1r[r], k2r[r])) - svr[r];
                        }
                        if (__ballot(force || t >= 0.f)) wact |= 1u << (4 * mq + r);
                    }
                }
                const bool slow = wact != 0 && (DIAG & 4) == 0;
                if (slow) {
                    uint64_t vm[4];
                    {
                        uint4 vw0, vw1, aw0, aw1;
                        uint32_t tmp;
                        asm volatile("v_add_u32 %4, %5, %6\n\t"
                                     "ds_read_b128 %0, %4 offset:1024\n\t"
                                     "ds_read_b128 %1, %4 offset:1040\n\t"
                                     "ds_read_b128 %2, %4 offset:1056\n\t"
                                     "ds_read_b128 %3, %4 offset:1072\n\t"
                                     "s_waitcnt lgkmcnt(0)"
                                     : "=v"(vw0), "=v"(vw1), "=v"(aw0), "=v"(aw1), "=&v"(tmp)
                                     : "s"(nsoff), "v"(sbase)
                                     : "memory");
                        const uint64_t words[4] = {((uint64_t)vw0.y << 32) | vw0.x, ((uint64_t)vw0.w << 32) | vw0.z,
                                                   ((uint64_t)vw1.y << 32) | vw1.x, ((uint64_t)vw1.w << 32) | vw1.z};
                        const uint64_t allows[4] = {((uint64_t)aw0.y << 32) | aw0.x, ((uint64_t)aw0.w << 32) | aw0.z,
                                                    ((uint64_t)aw1.y << 32) | aw1.x, ((uint64_t)aw1.w << 32) | aw1.z};
#pragma unroll
                        for (int h = 0; h < 4; h++) {
                            const uint64_t t = a.tile_begin + blk * 4 + h;
                            uint64_t m = t < a.tile_end ? readfirstlane64(words[h]) : 0ull;
                            if (a.allow) {
                                const uint64_t aw = t - a.allow_t0;
                                m &= aw < a.allow_words ? readfirstlane64(allows[h]) : 0ull;
                            }
                            vm[h] = m;
                        }
                    }
                    const uint64_t slot0 = (a.tile_begin + blk * 4) * 64;
                    if constexpr ((DIAG & 16) != 0) n_slow++;
                    // Per active group gi = (mq, r): lane l tests its column's 16 rows against
                    // query ql = 16 mq + r + qlane (C layout), and row l >> 4 of the register v
                    // holds that same query's list (lane l: entry l & 15) -- the four queries of
                    // the group, one per 16-lane row.  A survivor is inserted into its own row in
                    // registers (DPP shift), the row's thresholds tighten at once, and the lists
                    // and thresholds go back to LDS once per group.  The group loop is not
                    // unrolled (the code would not fit the unroller's budget); its 16
                    // accumulator elements come out of the AGPRs through one switch.
                    float nrm16[16];
                    read_norms8(0, *reinterpret_cast<float(*)[8]>(&nrm16[0]));
                    read_norms8(1, *reinterpret_cast<float(*)[8]>(&nrm16[8]));
                    float err16[I8 ? 16 : 1];  // (I8) the rows' error bounds
                    if constexpr (I8) {
                        read_norms8(2, *reinterpret_cast<float(*)[8]>(&err16[0]));
                        read_norms8(3, *reinterpret_cast<float(*)[8]>(&err16[8]));
                    }
                    for (uint32_t gw = wact; gw; gw &= gw - 1) {
                        const int gi = __builtin_ctz(gw);
                        if constexpr ((DIAG & 16) != 0) n_grp++;
                        float uv[16];  // (I8: the exact int32 scores, exactly as floats: |score| < 2^24)
                        switch (gi) {
#define WVG_SD_GROUP(G)                                                                        \
    case G:                                                                                    \
        _Pragma("unroll") for (int nr = 0; nr < 16; nr++) uv[nr] = (float)agpr_read(acc[(G) >> 2][nr][(G) & 3]); \
        break;
                        WVG_SD_GROUP(0) WVG_SD_GROUP(1) WVG_SD_GROUP(2) WVG_SD_GROUP(3)
                        WVG_SD_GROUP(4) WVG_SD_GROUP(5) WVG_SD_GROUP(6) WVG_SD_GROUP(7)
#undef WVG_SD_GROUP
                        default: break;
                        }
                        const uint32_t ql = 16u * (uint32_t)(gi >> 2) + (uint32_t)(gi & 3) + (uint32_t)qlane;
                        const uint32_t la = S.laddr + ql * (SCREEN_M * 8) + 8u * (uint32_t)(lane & 15);
                        const uint32_t ta = tbase + 4u * ql;  // tau; sig + 512, ck1 + 1024, ck2 + 1536, cem + 2048
                        uint2 v2;
                        float wt, ws, em, k1, k2;
                        asm volatile("ds_read_b64 %0, %6\n\t"
                                     "ds_read_b32 %1, %7\n\t"
                                     "ds_read_b32 %2, %7 offset:512\n\t"
                                     "ds_read_b32 %3, %7 offset:2048\n\t"
                                     "ds_read_b32 %4, %7 offset:1024\n\t"
                                     "ds_read_b32 %5, %7 offset:1536\n\t"
                                     "s_waitcnt lgkmcnt(0)"
                                     : "=v"(v2), "=v"(wt), "=v"(ws), "=v"(em), "=v"(k1), "=v"(k2)
                                     : "v"(la), "v"(ta)
                                     : "memory");
                        float kbq = 0.f, csq = 1.f;  // (I8) B and the score scale: ckb + 2560, ccs + 3072
                        if constexpr (I8)
                            asm volatile("ds_read_b32 %0, %2 offset:2560\n\t"
                                         "ds_read_b32 %1, %2 offset:3072\n\t"
                                         "s_waitcnt lgkmcnt(0)"
                                         : "=v"(kbq), "=v"(csq)
                                         : "v"(ta)
                                         : "memory");
                        uint64_t v = ((uint64_t)v2.y << 32) | v2.x;
                        const int li = lane & 15;
#pragma unroll
                        for (int nr = 0; nr < 16; nr++) {
                            const uint64_t m64 = ((vm[nr >> 2] >> (16 * (nr & 3))) & 0xFFFFull) * 0x0001000100010001ull;
                            float u;
                            if constexpr (I8)
                                u = uv[nr] * csq + __builtin_fmaf(err16[nr], k1, __builtin_fmaf(nrm16[nr], kbq, k2));
                            else
                                u = uv[nr] + __builtin_fmaf(nrm16[nr], k1, k2);
                            uint64_t pass = __ballot(!(u < ws)) & m64;
                            while (pass) {
                                const int j = __builtin_ctzll(pass);
                                pass &= pass - 1;
                                const int g = j >> 4;
                                const float lower =
                                    sc_lower(__int_as_float(__builtin_amdgcn_readlane(__float_as_int(u), j)), cosine);
                                float wtg = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(wt), j));
                                if (!(lower <= wtg)) continue;
                                if constexpr ((DIAG & 16) != 0) n_call++;
                                const uint64_t key = ((uint64_t)wvg_ord_f32(lower) << 32) |
                                                     (uint32_t)(slot0 + 16u * (uint32_t)nr + (uint32_t)(j & 15));
                                if (!(key < readlane64(v, 16 * g + SCREEN_M - 1))) continue;
                                const bool inrow = (lane >> 4) == g;
                                const int pos = __popcll(__ballot(inrow && v < key));
                                const uint64_t sh = row_shr1_64(v);
                                v = inrow ? (li > pos ? sh : (li == pos ? key : v)) : v;
                                const uint64_t nk = readlane64(v, 16 * g + K - 1);
                                const uint64_t nm = readlane64(v, 16 * g + SCREEN_M - 1);
                                const float emg = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(em), j));
                                if (nk != WVG_KEY_NONE) wtg = fminf(wtg, sc_tau_k(key_lower(nk), emg, cosine));
                                if (nm != WVG_KEY_NONE) wtg = fminf(wtg, key_lower(nm));
                                const float wsg = sc_sigma(wtg, cosine);
                                wt = inrow ? wtg : wt;
                                ws = inrow ? wsg : ws;
                                // the row's other survivors of this element group meet the new threshold
                                pass &= ~(0xFFFFull << (16 * g)) | __ballot(!(u < ws));
                            }
                        }
                        const uint2 o2 = make_uint2((uint32_t)v, (uint32_t)(v >> 32));
                        asm volatile("ds_write_b64 %0, %1" ::"v"(la), "v"(o2) : "memory");
                        if (li == 0)
                            asm volatile("ds_write_b32 %0, %1\n\t"
                                         "ds_write_b32 %0, %2 offset:512" ::"v"(ta), "v"(wt), "v"(ws)
                                         : "memory");
                    }
                    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                }
            } else if constexpr ((DIAG & 8) != 0) {
                // diagnostic (DIAG 10): the stage loop alone -- the accumulators are consumed by
                // one sum, so the MFMAs stay (without any consumer the compiler removes them)
                float x = 0.f;
#pragma unroll
                for (int mq = 0; mq < 2; mq++)
#pragma unroll
                    for (int nr = 0; nr < 16; nr++) x += (float)agpr_read(acc[mq][nr][0]);
                if (x == 0x1p-120f) a.partials[0] = 0;
            }
#pragma unroll
            for (int mq = 0; mq < 2; mq++)
#pragma unroll
                for (int nr = 0; nr < 16; nr++) acc[mq][nr] = acc_t{0, 0, 0, 0};
            // the next block's first K block: its stage landed before the last barrier and is not
            // overwritten before the next block's second barrier
            read_half(0, 0, b0);
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#ifdef WVG_TOOLS
    if constexpr ((DIAG & 16) != 0) {
        if (lane == 0) {
            atomicAdd(&g_screen_ctr[0], (unsigned long long)n_blk);
            atomicAdd(&g_screen_ctr[1], (unsigned long long)n_slow);
            atomicAdd(&g_screen_ctr[2], (unsigned long long)n_call);
            atomicAdd(&g_screen_ctr[3], (unsigned long long)n_grp);
        }
    }
#endif
    __syncthreads();
    // each wave owns whole lists: its 32 queries' range lists go straight to partials
    for (int ql = 0; ql < 32; ql++) {
        const uint32_t q = q0 + (uint32_t)(32 * w + ql);
        if (q >= a.nq) break;
        const uint64_t x = lane < M ? lists[((size_t)w * 32 + ql) * M + lane] : WVG_KEY_NONE;
        uint64_t *out = a.partials + ((size_t)q * a.nrr + rr) * M;
        if (lane < M) out[lane] = x;
        if (lane == K - 1 && x != WVG_KEY_NONE) {
            const float t = sc_tau_k(key_lower(x), cem[32 * w + ql], cosine);
            atomicMin(a.gbound + q, wvg_ord_f32(t));
        }
    }
}

// ---------------------------------------------------------------------------
// K3i (round 6) for d = 512 / 768: the int8 screen with 2 x 2 waves.  K3d's
// waves each own 32 queries x all 256 rows of a block, so every wave reads the
// whole 16 KiB stage from LDS: 64 KiB of LDS reads per K block and CU for 32
// MFMAs per wave, the loop's bound (profiles/r06/screen_i8: the stage loop
// alone ran the matrix pipe ~44 % busy).  int8 queries take half the registers
// of bf16 ones, so here a wave owns 64 queries (4 groups, resident) x 128 rows
// (one half of the block: its own 8 KiB of the stage): the same 32 MFMAs per
// K block from half the LDS reads.  The two row halves keep separate survivor
// lists per query (K3c's rule: each list holds its half's smallest lower
// bounds, its thresholds are valid for its rows); the kernel merges each
// query's two lists at the end.  The ring has 7 stages for every KBN (the
// buffer of a unit is (block * KBN + ks) % 7, a scalar); LDS = 7 x 16 KiB
// ring + 2 norm / error slots + 4 x 64 lists + thresholds and constants.
constexpr int SJ_NB = 7;
constexpr int SJ_LISTS = SD_WAVES * 64 * SCREEN_M * 8;
constexpr int SJ_RING = SJ_NB * SD_STAGE + 2 * SI_NSLOT;
constexpr int SJ_LDS = SJ_RING + SJ_LISTS + SD_WAVES * 64 * 4 * 2 + SD_BQ * 4 * 5;
static_assert(SJ_LDS <= 160 * 1024, "K3i 2x2's LDS");

// DIAG (tools build only; 0 in the product): 16 = counters (wave row blocks, active groups,
// inserts, groups with a passing element), 4 = fast check but no slow path, 10 = no epilogue
// (the accumulators consumed by one sum) -- timing only, results are not search results.
template <int KBN, int DIAG = 0>
__global__ __launch_bounds__(SD_WAVES * 64, 1) void screen_i8_kernel(ScreenArgs a)
{
    static_assert(KBN <= 12, "64 resident queries x KBN K blocks must fit the registers");
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    uint64_t *lists = reinterpret_cast<uint64_t *>(smem + SJ_RING);  // [4 waves][64][M]
    float *tau = reinterpret_cast<float *>(smem + SJ_RING + SJ_LISTS);  // [4 waves][64]
    float *sig = tau + SD_WAVES * 64;                                     // [4 waves][64]
    float *ck1 = sig + SD_WAVES * 64;                                     // [128]: A
    float *ck2 = ck1 + SD_BQ;                                             // K2
    float *cem = ck2 + SD_BQ;                                             // Emax
    float *ckb = cem + SD_BQ;                                             // B
    float *ccs = ckb + SD_BQ;                                             // score scale
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    uint32_t n_blk = 0, n_grp = 0, n_pass = 0, n_ins = 0;  // (DIAG 16, tools)
    (void)n_blk, (void)n_grp, (void)n_pass, (void)n_ins;
    const int wq = w & 1, wr = w >> 1;  // query half (64 queries), row half (tiles 2 wr, 2 wr + 1)
    const int K = (int)a.k, M = SCREEN_M;
    const int cosine = a.cosine;
    const uint32_t b = blockIdx.x;
    uint32_t qb, rr;
    if (a.nrr_l % 8 == 0) {
        const uint32_t xcd = b % 8, wv = b / 8;
        qb = wv % a.nqb;
        rr = a.rr0 + (wv / a.nqb) * 8 + xcd;
    } else {
        qb = b % a.nqb;
        rr = a.rr0 + b / a.nqb;
    }
    const uint64_t ntiles = a.tile_end - a.tile_begin;
    const uint64_t nblk = (ntiles + 3) / 4;
    uint64_t blk0, blk1;
    sc_range(a, nblk, rr, blk0, blk1);
    const uint32_t q0 = qb * SD_BQ;

    for (int i = tid; i < SD_BQ; i += SD_WAVES * 64) {
        const uint32_t q = q0 + (uint32_t)i;
        ck1[i] = a.k1[q];
        ck2[i] = a.k2[q];
        cem[i] = a.emax[q];
        ckb[i] = a.kb[q];
        ccs[i] = a.css[q];
    }
    for (int i = tid; i < SD_WAVES * 64; i += SD_WAVES * 64) {  // (wave v, query ql) = (i / 64, i % 64)
        const uint32_t q = q0 + (uint32_t)(64 * ((i >> 6) & 1) + (i & 63));
        const uint32_t g = q < a.nq ? __hip_atomic_load(a.gbound + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
        const float t = q >= a.nq ? -__builtin_inff() : (g == 0xFFFFFFFFu ? __builtin_inff() : wvg_unord_f32(g));
        tau[i] = t;
        sig[i] = q >= a.nq ? __builtin_inff() : sc_sigma(t, cosine);
    }
    for (int i = tid; i < SD_WAVES * 64 * M; i += SD_WAVES * 64) lists[i] = WVG_KEY_NONE;
    __syncthreads();
    SurvivorLists S;
    S.laddr = (uint32_t)(uintptr_t)(lists + (size_t)w * 64 * M);
    // LDS byte addresses: tau[w][0] (sig at + 1024) and ck1[64 wq] (ck2, cem, ckb, ccs at
    // + 512, + 1024, + 1536, + 2048)
    const uint32_t tbase = (uint32_t)(uintptr_t)(tau + w * 64);
    const uint32_t cbase = (uint32_t)(uintptr_t)(ck1 + 64 * wq);
    if (blk0 < blk1) {
        // the wave's 64 queries (4 groups of 16), every K block, resident: the first
        // 6 K blocks in AGPRs (128 accumulator + 32 B-fragment + 96 such AGPRs), the
        // rest in VGPRs
        constexpr int AKB = 6;
        i32x4 areg[KBN][4];
        const uint4 *qsrc = a.qfrag + (size_t)(qb * 8 + 4 * wq) * KBN * 64 + lane;
#pragma unroll
        for (int ks = 0; ks < KBN; ks++)
#pragma unroll
            for (int g = 0; g < 4; g++) {
                const uint4 *src = qsrc + ((size_t)g * KBN + ks) * 64;
                if (ks < AKB)
                    asm volatile("global_load_dwordx4 %0, %1, off" : "=a"(areg[ks][g]) : "v"(src) : "memory");
                else
                    asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(areg[ks][g]) : "v"(src) : "memory");
            }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
        for (int ks = 0; ks < KBN; ks++)
#pragma unroll
            for (int g = 0; g < 4; g++) {
                if (ks < AKB)
                    asm volatile("" : "+a"(areg[ks][g]));
                else
                    asm volatile("" : "+v"(areg[ks][g]));
            }

        // loads of one unit (K block ks of a row block): wave w moves the 4 fragments of
        // the block's tile w; with ks = 0 also tile w's norms and errors, and wave 0 the
        // block's tile words (sd_unit_loads<.., true>)
        const uint4 *lsrc = a.shadow + ((size_t)(a.tile_begin + blk0 * 4 + w) * KBN * 4) * 64 + lane;
        const float *lnorm = a.norms + (a.tile_begin + blk0 * 4 + w) * 64 + lane;
        const float *lerr = a.errs + (a.tile_begin + blk0 * 4 + w) * 64 + lane;
        uint64_t lblk = blk0;
        uint32_t lbuf = 0;  // ring buffer of the next unit to load (the units run in order)
        auto load_stage = [&](int ks) {
            unsigned char *dst = smem + lbuf * SD_STAGE;
            lbuf = lbuf + 1 == (uint32_t)SJ_NB ? 0u : lbuf + 1;
#pragma unroll
            for (int rg = 0; rg < 4; rg++)
                __builtin_amdgcn_global_load_lds(lsrc + ((size_t)ks * 4 + rg) * 64,
                                                 reinterpret_cast<uint4 *>(dst + (4 * w + rg) * 1024), 16, 0, 0);
            unsigned char *nslot = smem + SJ_NB * SD_STAGE + (lblk & 1) * SI_NSLOT;
            if (ks == 0) {
                __builtin_amdgcn_global_load_lds(lnorm, reinterpret_cast<float *>(nslot + w * 256), 4, 0, 0);
                __builtin_amdgcn_global_load_lds(lerr, reinterpret_cast<float *>(nslot + 1280 + w * 256), 4, 0, 0);
                if (w == 0) {
                    const uint32_t wi = (uint32_t)(lane & 7) >> 1, half = lane & 1;
                    const uint64_t t = a.tile_begin + lblk * 4 + wi;
                    const uint32_t *src =
                        reinterpret_cast<const uint32_t *>(a.valid + (t < a.tile_end ? t : a.tile_end - 1)) + half;
                    if (lane >= 8 && lane < 16 && a.allow) {
                        const uint64_t aw = t - a.allow_t0;
                        src = reinterpret_cast<const uint32_t *>(a.allow + (aw < a.allow_words ? aw : 0)) + half;
                    }
                    __builtin_amdgcn_global_load_lds(src, reinterpret_cast<uint32_t *>(nslot + 1024), 4, 0, 0);
                }
            }
            if (ks == KBN - 1 && lblk + 1 < blk1) {  // the load cursor moves on; past the end it stays
                ++lblk;
                lsrc += (size_t)4 * KBN * 4 * 64;
                lnorm += 256;
                lerr += 256;
            }
        };
        // NB - 2 = 5 units in flight at every wait: unit ks + 1 (waited for at K block ks)
        // and the NB - 3 younger ones
        auto wait_next = [&](auto KS) {
            constexpr int ks = decltype(KS)::value;
            constexpr int n0 = sd_younger<KBN, 0, true>(ks + 1, SJ_NB - 3, true);
            constexpr int n1 = sd_younger<KBN, 0, true>(ks + 1, SJ_NB - 3, false);
            if (w == 0) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(n0) : "memory");
            else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(n1) : "memory");
        };
        auto raw_barrier = [&]() {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");
        };
        // Half of the wave's row fragments of a unit (tile 2 wr + h: row groups 4 h .. 4 h + 3)
        // straight into AGPRs, from the unit's ring buffer rb (a scalar)
        const uint32_t rbase = (uint32_t)(uintptr_t)smem + 16u * lane + 8192u * (uint32_t)wr;
        auto read_half = [&](uint32_t rb, int h, i32x4 (&br)[4]) {
            const uint32_t soff = rb * (uint32_t)SD_STAGE + (uint32_t)h * 4096u;
            uint32_t tmp;
            asm volatile("v_add_u32 %4, %5, %6\n\t"
                         "ds_read_b128 %0, %4\n\t"
                         "ds_read_b128 %1, %4 offset:1024\n\t"
                         "ds_read_b128 %2, %4 offset:2048\n\t"
                         "ds_read_b128 %3, %4 offset:3072"
                         : "=a"(br[0]), "=a"(br[1]), "=a"(br[2]), "=a"(br[3]), "=&v"(tmp)
                         : "s"(soff), "v"(rbase)
                         : "memory");
        };
        auto wait_b0 = [&](i32x4 (&br)[4]) {  // the first half landed (the second half's 4 reads may not)
            asm volatile("s_waitcnt lgkmcnt(4)" : "+a"(br[0]), "+a"(br[1]), "+a"(br[2]), "+a"(br[3]) : : "memory");
        };
        const int qlane = 4 * (lane >> 4);
        const uint32_t sbase = (uint32_t)(uintptr_t)smem;
        const uint32_t nbase = sbase + 4u * (uint32_t)(lane & 15);
        // +inf when one of this lane's queries is not fast-eligible (A > 2^50)
        bool lane_force = false;
#pragma unroll
        for (int g = 0; g < 4; g++)
#pragma unroll
            for (int r = 0; r < 4; r++)
                if (!(ck1[64 * wq + 16 * g + qlane + r] <= 0x1p50f)) lane_force = true;

        i32x4 acc[4][8];
#pragma unroll
        for (int g = 0; g < 4; g++)
#pragma unroll
            for (int nr = 0; nr < 8; nr++) acc[g][nr] = i32x4{0, 0, 0, 0};
        i32x4 b0[4], b1[4];
        // prologue: units 0 .. NB - 2 of the range into buffers 0 .. NB - 2
#pragma unroll
        for (int ks = 0; ks < SJ_NB - 1; ks++) load_stage(ks % KBN);
        if (w == 0) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(sd_younger<KBN, 0, true>(0, SJ_NB - 2, true)) : "memory");
        else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(sd_younger<KBN, 0, true>(0, SJ_NB - 2, false)) : "memory");
        raw_barrier();
        uint32_t cbuf = 0;  // ring buffer of K block 0 of the current row block
        read_half(0u, 0, b0);
        for (uint64_t blk = blk0; blk < blk1; blk++) {
            sd_static_for<KBN>([&](auto KS) {
                constexpr int ks = decltype(KS)::value;
                const uint32_t ub = __builtin_amdgcn_readfirstlane((cbuf + (uint32_t)ks) % (uint32_t)SJ_NB);  // its buffer
                read_half(ub, 1, b1);
                wait_b0(b0);
#pragma unroll
                for (int g = 0; g < 4; g++)
#pragma unroll
                    for (int nr = 0; nr < 4; nr++)
                        acc[g][nr] = __builtin_amdgcn_mfma_i32_16x16x64_i8(areg[ks][g], b0[nr], acc[g][nr], 0, 0, 0);
                wait_next(KS);  // the next unit landed
                raw_barrier();  // (lgkmcnt(0): this wave's second-half reads done)
#pragma unroll
                for (int j = 0; j < 4; j++) asm volatile("" : "+a"(b1[j]));
                // unit + NB - 1 into the buffer of unit - 1 (fully read before this barrier)
                load_stage((ks + SJ_NB - 1) % KBN);
                if (ks + 1 < KBN) {
                    uint32_t nb = ub + 1 == (uint32_t)SJ_NB ? 0u : ub + 1;
                    read_half(__builtin_amdgcn_readfirstlane(nb), 0, b0);
                }
#pragma unroll
                for (int g = 0; g < 4; g++)
#pragma unroll
                    for (int nr = 0; nr < 4; nr++)
                        acc[g][4 + nr] =
                            __builtin_amdgcn_mfma_i32_16x16x64_i8(areg[ks][g], b1[nr], acc[g][4 + nr], 0, 0, 0);
            });
            cbuf = (cbuf + (uint32_t)KBN) % (uint32_t)SJ_NB;
            // (the XDL write -> VALU read hazard of the block's last MFMAs: see K3d)
            __builtin_amdgcn_sched_barrier(0);
            asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
            __builtin_amdgcn_sched_barrier(0);
            // epilogue of row block blk: C layout row (query) 16 g + qlane + r, column (row)
            // 128 wr + 16 nr + (lane & 15)
            if constexpr (DIAG == 10) {
                int x = 0;
#pragma unroll
                for (int g = 0; g < 4; g++)
#pragma unroll
                    for (int nr = 0; nr < 8; nr++) x += agpr_read(acc[g][nr][0]);
                if (x == 0x7FFFFFF1) a.partials[0] = 0;
            } else {
            const uint32_t nsoff = (uint32_t)(SJ_NB * SD_STAGE + (blk & 1) * SI_NSLOT);
            auto read8 = [&](uint32_t off, float (&v)[8]) {  // 8 row groups of the wave's half at off
                uint32_t tmp;
                asm volatile("v_add_u32 %8, %9, %10\n\t"
                             "ds_read_b32 %0, %8\n\t"
                             "ds_read_b32 %1, %8 offset:64\n\t"
                             "ds_read_b32 %2, %8 offset:128\n\t"
                             "ds_read_b32 %3, %8 offset:192\n\t"
                             "ds_read_b32 %4, %8 offset:256\n\t"
                             "ds_read_b32 %5, %8 offset:320\n\t"
                             "ds_read_b32 %6, %8 offset:384\n\t"
                             "ds_read_b32 %7, %8 offset:448\n\t"
                             "s_waitcnt lgkmcnt(0)"
                             : "=v"(v[0]), "=v"(v[1]), "=v"(v[2]), "=v"(v[3]), "=v"(v[4]), "=v"(v[5]), "=v"(v[6]),
                               "=v"(v[7]), "=&v"(tmp)
                             : "s"(off), "v"(nbase)
                             : "memory");
            };
            float nrm[8], err[8];
            read8(nsoff + 512u * (uint32_t)wr, nrm);
            read8(nsoff + 1280u + 512u * (uint32_t)wr, err);
            float nmax = nrm[0], nsum = nrm[0], emx = err[0], esum = err[0];
#pragma unroll
            for (int j = 1; j < 8; j++) {
                nmax = __builtin_fmaxf(nmax, nrm[j]), nsum += nrm[j];
                emx = __builtin_fmaxf(emx, err[j]), esum += err[j];
            }
            const bool force = lane_force || !(nmax <= 0x1p60f) || nsum != nsum || !(emx <= 0x1p60f) || esum != esum;
            if constexpr (DIAG == 16) n_blk++;
            // fast check per (query group g, query r of the lane's four): the largest exact
            // int32 score of the lane's 8 rows, scaled once, + the bound of the lane's largest
            // error and norm, against WS -- a superset test of every element (monotone roundings)
            // (query groups two at a time, their 8 (g, r) maxima as independent chains: with
            // one wave per SIMD a group-by-group chain of dependent reads and maxima exposes
            // every VALU latency; all 16 at once spill)
            uint32_t wact = 0;
#pragma unroll
            for (int gp = 0; gp < 2; gp++) {
                int mi[2][4];
#pragma unroll
                for (int h = 0; h < 2; h++)
#pragma unroll
                    for (int r = 0; r < 4; r++) mi[h][r] = agpr_read(acc[2 * gp + h][0][r]);
#pragma unroll
                for (int nr = 1; nr < 8; nr++)
#pragma unroll
                    for (int h = 0; h < 2; h++)
#pragma unroll
                        for (int r = 0; r < 4; r++) mi[h][r] = max(mi[h][r], agpr_read(acc[2 * gp + h][nr][r]));
#pragma unroll
                for (int h = 0; h < 2; h++) {
                    const int g = 2 * gp + h;
                    float4 k1v, k2v, kbv, csv, sv;
                    {
                        const uint32_t ca = cbase + 4u * (uint32_t)(16 * g + qlane);
                        const uint32_t sa = tbase + 1024u + 4u * (uint32_t)(16 * g + qlane);
                        asm volatile("ds_read_b128 %0, %5\n\t"
                                     "ds_read_b128 %1, %5 offset:512\n\t"
                                     "ds_read_b128 %2, %5 offset:1536\n\t"
                                     "ds_read_b128 %3, %5 offset:2048\n\t"
                                     "ds_read_b128 %4, %6\n\t"
                                     "s_waitcnt lgkmcnt(0)"
                                     : "=v"(k1v), "=v"(k2v), "=v"(kbv), "=v"(csv), "=v"(sv)
                                     : "v"(ca), "v"(sa)
                                     : "memory");
                    }
                    const float k1r[4] = {k1v.x, k1v.y, k1v.z, k1v.w}, k2r[4] = {k2v.x, k2v.y, k2v.z, k2v.w};
                    const float kbr[4] = {kbv.x, kbv.y, kbv.z, kbv.w}, csr[4] = {csv.x, csv.y, csv.z, csv.w};
                    const float svr[4] = {sv.x, sv.y, sv.z, sv.w};
#pragma unroll
                    for (int r = 0; r < 4; r++) {
                        const float t = ((float)mi[h][r] * csr[r] +
                                         __builtin_fmaf(emx, k1r[r], __builtin_fmaf(nmax, kbr[r], k2r[r]))) -
                                        svr[r];
                        if (__ballot(force || t >= 0.f)) wact |= 1u << (4 * g + r);
                    }
                }
            }
            if (DIAG != 4 && wact != 0) {
                // the wave's two tiles' live words (valid & allow)
                uint64_t vm[2];
                {
                    uint4 vw, aw;
                    uint32_t tmp;
                    asm volatile("v_add_u32 %2, %3, %4\n\t"
                                 "ds_read_b128 %0, %2 offset:1024\n\t"
                                 "ds_read_b128 %1, %2 offset:1056\n\t"
                                 "s_waitcnt lgkmcnt(0)"
                                 : "=v"(vw), "=v"(aw), "=&v"(tmp)
                                 : "s"(nsoff + 16u * (uint32_t)wr), "v"(sbase)
                                 : "memory");
                    const uint64_t words[2] = {((uint64_t)vw.y << 32) | vw.x, ((uint64_t)vw.w << 32) | vw.z};
                    const uint64_t allows[2] = {((uint64_t)aw.y << 32) | aw.x, ((uint64_t)aw.w << 32) | aw.z};
#pragma unroll
                    for (int h = 0; h < 2; h++) {
                        const uint64_t t = a.tile_begin + blk * 4 + 2 * wr + h;
                        uint64_t m = t < a.tile_end ? readfirstlane64(words[h]) : 0ull;
                        if (a.allow) {
                            const uint64_t aw2 = t - a.allow_t0;
                            m &= aw2 < a.allow_words ? readfirstlane64(allows[h]) : 0ull;
                        }
                        vm[h] = m;
                    }
                }
                const uint64_t slot0 = (a.tile_begin + blk * 4 + 2 * wr) * 64;
                // per active group gi = (g, r): lane l tests its column's 8 rows against query
                // ql = 16 g + r + qlane of the wave, whose list is row l >> 4 of v (K3d's slow path)
                for (uint32_t gw = wact; gw; gw &= gw - 1) {
                    const int gi = __builtin_ctz(gw);
                    if constexpr (DIAG == 16) n_grp++;
                    float uv[8];  // the exact int32 scores as floats (|score| < 2^24)
                    switch (gi) {
#define WVG_SJ_GROUP(G)                                                                               \
    case G:                                                                                           \
        _Pragma("unroll") for (int nr = 0; nr < 8; nr++) uv[nr] = (float)agpr_read(acc[(G) >> 2][nr][(G) & 3]); \
        break;
                    WVG_SJ_GROUP(0) WVG_SJ_GROUP(1) WVG_SJ_GROUP(2) WVG_SJ_GROUP(3)
                    WVG_SJ_GROUP(4) WVG_SJ_GROUP(5) WVG_SJ_GROUP(6) WVG_SJ_GROUP(7)
                    WVG_SJ_GROUP(8) WVG_SJ_GROUP(9) WVG_SJ_GROUP(10) WVG_SJ_GROUP(11)
                    WVG_SJ_GROUP(12) WVG_SJ_GROUP(13) WVG_SJ_GROUP(14) WVG_SJ_GROUP(15)
#undef WVG_SJ_GROUP
                    default: break;
                    }
                    const uint32_t ql = 16u * (uint32_t)(gi >> 2) + (uint32_t)(gi & 3) + (uint32_t)qlane;
                    const uint32_t la = S.laddr + ql * (SCREEN_M * 8) + 8u * (uint32_t)(lane & 15);
                    const uint32_t ta = tbase + 4u * ql;  // tau; sig + 1024
                    const uint32_t ca = cbase + 4u * ql;  // A; K2 + 512, Emax + 1024, B + 1536, scale + 2048
                    // u of the group's 8 row groups first: a group the coarse fast check let
                    // through often has no element at or above WS, and then its list and
                    // thresholds are neither read nor written back
                    float ws, k1, k2, kbq, csq;
                    asm volatile("ds_read_b32 %0, %5 offset:1024\n\t"
                                 "ds_read_b32 %1, %6\n\t"
                                 "ds_read_b32 %2, %6 offset:512\n\t"
                                 "ds_read_b32 %3, %6 offset:1536\n\t"
                                 "ds_read_b32 %4, %6 offset:2048\n\t"
                                 "s_waitcnt lgkmcnt(0)"
                                 : "=v"(ws), "=v"(k1), "=v"(k2), "=v"(kbq), "=v"(csq)
                                 : "v"(ta), "v"(ca)
                                 : "memory");
                    float uu[8];
                    uint64_t any = 0;
#pragma unroll
                    for (int nr = 0; nr < 8; nr++) {
                        const uint64_t m64 = ((vm[nr >> 2] >> (16 * (nr & 3))) & 0xFFFFull) * 0x0001000100010001ull;
                        uu[nr] = uv[nr] * csq + __builtin_fmaf(err[nr], k1, __builtin_fmaf(nrm[nr], kbq, k2));
                        any |= __ballot(!(uu[nr] < ws)) & m64;
                    }
                    if (!any) continue;
                    if constexpr (DIAG == 16) n_pass++;
                    uint2 v2;
                    float wt, em;
                    asm volatile("ds_read_b64 %0, %3\n\t"
                                 "ds_read_b32 %1, %4\n\t"
                                 "ds_read_b32 %2, %5 offset:1024\n\t"
                                 "s_waitcnt lgkmcnt(0)"
                                 : "=v"(v2), "=v"(wt), "=v"(em)
                                 : "v"(la), "v"(ta), "v"(ca)
                                 : "memory");
                    uint64_t v = ((uint64_t)v2.y << 32) | v2.x;
                    const int li = lane & 15;
#pragma unroll
                    for (int nr = 0; nr < 8; nr++) {
                        const uint64_t m64 = ((vm[nr >> 2] >> (16 * (nr & 3))) & 0xFFFFull) * 0x0001000100010001ull;
                        const float u = uu[nr];
                        uint64_t pass = __ballot(!(u < ws)) & m64;
                        while (pass) {
                            const int j = __builtin_ctzll(pass);
                            pass &= pass - 1;
                            const int gq = j >> 4;
                            const float lower =
                                sc_lower(__int_as_float(__builtin_amdgcn_readlane(__float_as_int(u), j)), cosine);
                            float wtg = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(wt), j));
                            if (!(lower <= wtg)) continue;
                            const uint64_t key = ((uint64_t)wvg_ord_f32(lower) << 32) |
                                                 (uint32_t)(slot0 + 16u * (uint32_t)nr + (uint32_t)(j & 15));
                            if (!(key < readlane64(v, 16 * gq + SCREEN_M - 1))) continue;
                            if constexpr (DIAG == 16) n_ins++;
                            const bool inrow = (lane >> 4) == gq;
                            const int pos = __popcll(__ballot(inrow && v < key));
                            const uint64_t sh = row_shr1_64(v);
                            v = inrow ? (li > pos ? sh : (li == pos ? key : v)) : v;
                            const uint64_t nk = readlane64(v, 16 * gq + K - 1);
                            const uint64_t nm = readlane64(v, 16 * gq + SCREEN_M - 1);
                            const float emg = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(em), j));
                            if (nk != WVG_KEY_NONE) wtg = fminf(wtg, sc_tau_k(key_lower(nk), emg, cosine));
                            if (nm != WVG_KEY_NONE) wtg = fminf(wtg, key_lower(nm));
                            const float wsg = sc_sigma(wtg, cosine);
                            wt = inrow ? wtg : wt;
                            ws = inrow ? wsg : ws;
                            pass &= ~(0xFFFFull << (16 * gq)) | __ballot(!(u < ws));
                        }
                    }
                    const uint2 o2 = make_uint2((uint32_t)v, (uint32_t)(v >> 32));
                    asm volatile("ds_write_b64 %0, %1" ::"v"(la), "v"(o2) : "memory");
                    if (li == 0)
                        asm volatile("ds_write_b32 %0, %1\n\t"
                                     "ds_write_b32 %0, %2 offset:1024" ::"v"(ta), "v"(wt), "v"(ws)
                                     : "memory");
                }
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            }
            }  // (DIAG != 10)
#pragma unroll
            for (int g = 0; g < 4; g++)
#pragma unroll
                for (int nr = 0; nr < 8; nr++) acc[g][nr] = i32x4{0, 0, 0, 0};
            // the next block's first K block: landed before the last barrier, not overwritten
            // before the next block's second barrier
            read_half(__builtin_amdgcn_readfirstlane(cbuf), 0, b0);
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#ifdef WVG_TOOLS
    if constexpr (DIAG == 16) {
        if (lane == 0) {
            atomicAdd(&g_screen_ctr[0], (unsigned long long)n_blk);
            atomicAdd(&g_screen_ctr[1], (unsigned long long)n_grp);
            atomicAdd(&g_screen_ctr[2], (unsigned long long)n_ins);
            atomicAdd(&g_screen_ctr[3], (unsigned long long)n_pass);
        }
    }
#endif
    __syncthreads();
    // per query of the block: the merge of its two row halves' lists (waves wq and wq + 2),
    // the 16 smallest of 32 distinct-or-empty keys by rank (A's before B's on equal keys),
    // straight to partials; wave w takes block queries 32 w .. 32 w + 31
    for (int i = 0; i < 32; i++) {
        const uint32_t bq = (uint32_t)(32 * w + i), q = q0 + bq;
        if (q >= a.nq) break;
        const uint32_t hq = bq >> 6, ql = bq & 63;
        const uint64_t *la_ = lists + ((size_t)hq * 64 + ql) * M;        // wave hq (row half 0)
        const uint64_t *lb_ = lists + ((size_t)(hq + 2) * 64 + ql) * M;  // wave hq + 2 (row half 1)
        const int li = lane & 15;
        const uint64_t x = lane < 16 ? la_[li] : (lane < 32 ? lb_[li] : WVG_KEY_NONE);
        uint32_t rank = (uint32_t)li;
#pragma unroll
        for (int j = 0; j < 16; j++) {
            const uint64_t ya = readlane64(x, j), yb = readlane64(x, 16 + j);
            if (lane < 16) rank += yb < x ? 1u : 0u;
            else if (lane < 32) rank += ya <= x ? 1u : 0u;
        }
        uint64_t *out = a.partials + ((size_t)q * a.nrr + rr) * M;
        if (lane < 32 && rank < (uint32_t)M) out[rank] = x;
        if (lane < 32 && rank == (uint32_t)(K - 1) && x != WVG_KEY_NONE) {
            const float t = sc_tau_k(key_lower(x), cem[bq], cosine);
            atomicMin(a.gbound + q, wvg_ord_f32(t));
        }
    }
}

constexpr int SF_WAVES = 8;  // K3f's waves per workgroup

#ifdef WVG_TOOLS  // K3e and K3f: round-5 A/B variants (tools build only; the product runs K3d)
// ---------------------------------------------------------------------------
// K3e (round 5): K3d with 32x32x16 bf16 MFMAs.  K3d's 16x16x32 MFMA takes 16
// cycles of the matrix pipe and holds the wave's issue for 8 of them, so per
// 32-deep unit (32 MFMAs, 512 pipe cycles) only ~256 issue cycles are left for
// the unit's 16 ds_read_b128, 4 LDS-DMA pieces (~60 cycles each among MFMAs,
// MI355X_MICROARCH.md) and the barrier: one wave per SIMD cannot keep the pipe
// busy (K3d counters: MFMA busy 40 %).  v_mfma_f32_32x32x16_bf16 does the same
// work in half the instructions -- 16 per unit, 32 pipe cycles each, 8 of them
// issue -- which leaves ~384 issue cycles per unit for the same reads, DMA and
// barrier.  Registers, LDS ring, loads, waits and barriers are K3d's.
//   A operand = the wave's 32 queries (resident; lane l: query l % 32, k 8 (l / 32) + 0..7
//   of each 16-deep step -- gathered once from qfrag's 16 x 32 fragments);
//   B operand = 32 rows of the row block (lane l: row l % 32 of the group, same k),
//   read straight from the ring's 16 x 32 fragments with a per-lane address
//   (conflict-free: the 16 lanes of each ds_read_b128 group hit 16 distinct
//   16-byte bank groups);
//   C: lane l holds row n = 32 g + (l & 31) of row group g and queries
//   m = 8 (r >> 2) + 4 (l >> 5) + (r & 3), r = 0..15.
// Epilogue: per lane and query slot r the largest raw score of its 8 rows +
// E(its rows' largest norm) against WS (a superset test of every element);
// one ballot per slot gives 16 wave-uniform bits, each covering two queries
// (lanes 0-31 and 32-63) x 256 rows; an active slot's two lists sit in lanes
// 0-15 and 32-47 of one register and survivors are inserted as in K3d.
typedef float floatx16 __attribute__((ext_vector_type(16)));

template <int KBN, int DIAG = 0>
__global__ __launch_bounds__(SD_WAVES * 64, 1) void screen_ar32_kernel(ScreenArgs a)
{
    static_assert(KBN % SD_NBUF == 0, "the stage buffer of a K block must be a compile-time constant");
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    uint64_t *lists = reinterpret_cast<uint64_t *>(smem + SD_RING);  // [4][32][M]
    float *tau = reinterpret_cast<float *>(smem + SD_RING + SD_LISTS);
    float *sig = tau + SD_WAVES * 32;
    float *ck1 = sig + SD_WAVES * 32;
    float *ck2 = ck1 + SD_BQ;
    float *cem = ck2 + SD_BQ;
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int K = (int)a.k, M = SCREEN_M;
    const int cosine = a.cosine;
    const uint32_t b = blockIdx.x;
    uint32_t qb, rr;
    if (a.nrr_l % 8 == 0) {
        const uint32_t xcd = b % 8, wv = b / 8;
        qb = wv % a.nqb;
        rr = a.rr0 + (wv / a.nqb) * 8 + xcd;
    } else {
        qb = b % a.nqb;
        rr = a.rr0 + b / a.nqb;
    }
    const uint64_t ntiles = a.tile_end - a.tile_begin;
    const uint64_t nblk = (ntiles + 3) / 4;
    const uint64_t blk0 = nblk * rr / a.nrr, blk1 = nblk * (rr + 1) / a.nrr;
    const uint32_t q0 = qb * SD_BQ;

    for (int i = tid; i < SD_BQ; i += SD_WAVES * 64) {
        const uint32_t q = q0 + (uint32_t)i;
        ck1[i] = a.k1[q];
        ck2[i] = a.k2[q];
        cem[i] = a.emax[q];
    }
    for (int i = tid; i < SD_WAVES * 32; i += SD_WAVES * 64) {
        const uint32_t q = q0 + (uint32_t)i;
        const uint32_t g = q < a.nq ? __hip_atomic_load(a.gbound + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
        const float t = q >= a.nq ? -__builtin_inff() : (g == 0xFFFFFFFFu ? __builtin_inff() : wvg_unord_f32(g));
        tau[i] = t;
        sig[i] = q >= a.nq ? __builtin_inff() : sc_sigma(t, cosine);
    }
    for (int i = tid; i < SD_WAVES * 32 * M; i += SD_WAVES * 64) lists[i] = WVG_KEY_NONE;
    __syncthreads();
    const uint32_t laddr = (uint32_t)(uintptr_t)(lists + (size_t)w * 32 * M);
    const uint32_t tbase = (uint32_t)(uintptr_t)(tau + w * 32);
    if (blk0 < blk1) {
        // the wave's 32 queries, every K block and step, resident for the whole range
        bf16x8 areg[KBN][2];
        constexpr int SD_AKB = 6;  // K blocks whose fragments live in AGPRs (as K3d)
        {
            const uint32_t ql = (uint32_t)lane & 31u;
            const uint4 *qsrc = a.qfrag + (size_t)(qb * 8 + 2 * w + (ql >> 4)) * KBN * 64 + (ql & 15u);
#pragma unroll
            for (int ks = 0; ks < KBN; ks++)
#pragma unroll
                for (int st = 0; st < 2; st++) {
                    const uint4 *src = qsrc + (size_t)ks * 64 + (2 * st + (lane >> 5)) * 16;
                    if (ks < SD_AKB)
                        asm volatile("global_load_dwordx4 %0, %1, off" : "=a"(areg[ks][st]) : "v"(src) : "memory");
                    else
                        asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(areg[ks][st]) : "v"(src) : "memory");
                }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
        for (int ks = 0; ks < KBN; ks++)
#pragma unroll
            for (int st = 0; st < 2; st++) {
                if (ks < SD_AKB)
                    asm volatile("" : "+a"(areg[ks][st]));
                else
                    asm volatile("" : "+v"(areg[ks][st]));
            }

        // the stage loads: K3d's (wave w moves tile w's four 16-row fragments; unit 0 also
        // its norms, wave 0 the block's tile words)
        const uint4 *lsrc = a.shadow + ((size_t)(a.tile_begin + blk0 * 4 + w) * KBN * 4) * 64 + lane;
        const float *lnorm = a.norms + (a.tile_begin + blk0 * 4 + w) * 64 + lane;
        uint64_t lblk = blk0;
        auto load_stage = [&](int ks) {
            unsigned char *dst = smem + (ks % SD_NBUF) * SD_STAGE;
#pragma unroll
            for (int rg = 0; rg < 4; rg++)
                __builtin_amdgcn_global_load_lds(lsrc + ((size_t)ks * 4 + rg) * 64,
                                                 reinterpret_cast<uint4 *>(dst + (4 * w + rg) * 1024), 16, 0, 0);
            unsigned char *nslot = smem + SD_NBUF * SD_STAGE + (lblk & 1) * SD_NSLOT;
            if (ks == 0)
                __builtin_amdgcn_global_load_lds(lnorm, reinterpret_cast<float *>(nslot + w * 256), 4, 0, 0);
            if (ks == 0 && w == 0) {
                const uint32_t wi = (uint32_t)(lane & 7) >> 1, half = lane & 1;
                const uint64_t t = a.tile_begin + lblk * 4 + wi;
                const uint32_t *src =
                    reinterpret_cast<const uint32_t *>(a.valid + (t < a.tile_end ? t : a.tile_end - 1)) + half;
                if (lane >= 8 && lane < 16 && a.allow) {
                    const uint64_t aw = t - a.allow_t0;
                    src = reinterpret_cast<const uint32_t *>(a.allow + (aw < a.allow_words ? aw : 0)) + half;
                }
                __builtin_amdgcn_global_load_lds(src, reinterpret_cast<uint32_t *>(nslot + 1024), 4, 0, 0);
            }
            if (ks == KBN - 1 && lblk + 1 < blk1) {
                ++lblk;
                lsrc += (size_t)4 * KBN * 4 * 64;
                lnorm += 256;
            }
        };
        auto wait_next = [&](auto KS) {
            constexpr int ks = decltype(KS)::value;
            constexpr int n0 = sd_younger<KBN, 0>(ks + 1, SD_NBUF - 3, true);
            constexpr int n1 = sd_younger<KBN, 0>(ks + 1, SD_NBUF - 3, false);
            if (w == 0) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(n0) : "memory");
            else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(n1) : "memory");
        };
        auto raw_barrier = [&]() {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");
        };
        // B fragments of step st (8 row groups of 32) straight into AGPRs: lane l reads row
        // l % 32 of group g, k 8 (2 st + l / 32) .. + 7 of the unit, i.e. 16-row fragment
        // 2 g + ((l & 31) >> 4), lane (2 st + l / 32) * 16 + (l & 15) of it
        const uint32_t rbase = (uint32_t)(uintptr_t)smem + (uint32_t)(lane >> 5) * 256u +
                               (uint32_t)((lane & 31) >> 4) * 1024u + (uint32_t)(lane & 15) * 16u;
        auto read_half = [&](int ks, int st, bf16x8 (&br)[8]) {
            const uint32_t soff = (uint32_t)((ks % SD_NBUF) * SD_STAGE + st * 512);
            uint32_t tmp;
            asm volatile("v_add_u32 %8, %9, %10\n\t"
                         "ds_read_b128 %0, %8\n\t"
                         "ds_read_b128 %1, %8 offset:2048\n\t"
                         "ds_read_b128 %2, %8 offset:4096\n\t"
                         "ds_read_b128 %3, %8 offset:6144\n\t"
                         "ds_read_b128 %4, %8 offset:8192\n\t"
                         "ds_read_b128 %5, %8 offset:10240\n\t"
                         "ds_read_b128 %6, %8 offset:12288\n\t"
                         "ds_read_b128 %7, %8 offset:14336"
                         : "=a"(br[0]), "=a"(br[1]), "=a"(br[2]), "=a"(br[3]), "=a"(br[4]), "=a"(br[5]), "=a"(br[6]),
                           "=a"(br[7]), "=&v"(tmp)
                         : "s"(soff), "v"(rbase)
                         : "memory");
        };
        auto wait_b0 = [&](bf16x8 (&br)[8]) {
            asm volatile("s_waitcnt lgkmcnt(8)"
                         : "+a"(br[0]), "+a"(br[1]), "+a"(br[2]), "+a"(br[3]), "+a"(br[4]), "+a"(br[5]), "+a"(br[6]),
                           "+a"(br[7])
                         :
                         : "memory");
        };
        // this lane's queries: m(r) = 8 (r >> 2) + qh + (r & 3), qh = 4 (l >> 5)
        const int qh = 4 * (lane >> 5);
        const uint32_t sbase = (uint32_t)(uintptr_t)smem;
        const uint32_t nbase = sbase + 4u * (uint32_t)(lane & 31);  // norm of row 32 g + (l & 31): + 128 g
        const uint32_t csoff = (uint32_t)((uintptr_t)sig - (uintptr_t)smem);
        bool lane_force = false;
#pragma unroll
        for (int r = 0; r < 16; r++)
            if (!(ck1[32 * w + 8 * (r >> 2) + qh + (r & 3)] <= 0x1p50f)) lane_force = true;

        floatx16 acc[8];
#pragma unroll
        for (int g = 0; g < 8; g++)
#pragma unroll
            for (int e = 0; e < 16; e++) acc[g][e] = 0.f;
        bf16x8 b0[8], b1[8];
#pragma unroll
        for (int ks = 0; ks < SD_NBUF - 1; ks++) load_stage(ks);
        if (w == 0) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(sd_younger<KBN, 0>(0, SD_NBUF - 2, true)) : "memory");
        else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(sd_younger<KBN, 0>(0, SD_NBUF - 2, false)) : "memory");
        raw_barrier();
        read_half(0, 0, b0);
        for (uint64_t blk = blk0; blk < blk1; blk++) {
            sd_static_for<KBN>([&](auto KS) {
                constexpr int ks = decltype(KS)::value;
                read_half(ks, 1, b1);
                wait_b0(b0);
#pragma unroll
                for (int g = 0; g < 8; g++)
                    acc[g] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(areg[ks][0], b0[g], acc[g], 0, 0, 0);
                wait_next(KS);
                raw_barrier();  // (lgkmcnt(0): this wave's second-step reads done)
#pragma unroll
                for (int j = 0; j < 8; j++) asm volatile("" : "+a"(b1[j]));
                load_stage((ks + SD_NBUF - 1) % KBN);  // unit + 7 into the buffer of unit - 1
                if (ks + 1 < KBN) read_half(ks + 1, 0, b0);
#pragma unroll
                for (int g = 0; g < 8; g++)
                    acc[g] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(areg[ks][1], b1[g], acc[g], 0, 0, 0);
            });
            // 32x32x16: 16 passes, 18 wait states before a VALU reads its result (agpr_read
            // is inline asm the hazard recognizer does not see)
            __builtin_amdgcn_sched_barrier(0);
            asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
            __builtin_amdgcn_sched_barrier(0);
            if constexpr ((DIAG & 2) == 0) {
                const uint32_t nsoff = (uint32_t)(SD_NBUF * SD_STAGE + (blk & 1) * SD_NSLOT);
                float nrm[8];
                {
                    uint32_t tmp;
                    asm volatile("v_add_u32 %8, %9, %10\n\t"
                                 "ds_read_b32 %0, %8\n\t"
                                 "ds_read_b32 %1, %8 offset:128\n\t"
                                 "ds_read_b32 %2, %8 offset:256\n\t"
                                 "ds_read_b32 %3, %8 offset:384\n\t"
                                 "ds_read_b32 %4, %8 offset:512\n\t"
                                 "ds_read_b32 %5, %8 offset:640\n\t"
                                 "ds_read_b32 %6, %8 offset:768\n\t"
                                 "ds_read_b32 %7, %8 offset:896\n\t"
                                 "s_waitcnt lgkmcnt(0)"
                                 : "=v"(nrm[0]), "=v"(nrm[1]), "=v"(nrm[2]), "=v"(nrm[3]), "=v"(nrm[4]),
                                   "=v"(nrm[5]), "=v"(nrm[6]), "=v"(nrm[7]), "=&v"(tmp)
                                 : "s"(nsoff), "v"(nbase)
                                 : "memory");
                }
                float nmax = nrm[0], nsum = nrm[0];
#pragma unroll
                for (int g = 1; g < 8; g++) nmax = __builtin_fmaxf(nmax, nrm[g]), nsum += nrm[g];
                const bool force = lane_force || !(nmax <= 0x1p60f) || nsum != nsum;
                uint32_t wact = 0;
#pragma unroll
                for (int i = 0; i < 4; i++) {
                    // queries 32 w + 8 i + qh + 0..3: sig, ck1, ck2 (128-float arrays, +512 / +1024 B)
                    const uint32_t coff = (uint32_t)(csoff + 4 * (32 * w + 8 * i));
                    const uint32_t qbase = sbase + 4u * (uint32_t)qh;
                    float4 k1v, k2v, sv;
                    uint32_t tmp;
                    asm volatile("v_add_u32 %3, %4, %5\n\t"
                                 "ds_read_b128 %0, %3 offset:512\n\t"
                                 "ds_read_b128 %1, %3 offset:1024\n\t"
                                 "ds_read_b128 %2, %3\n\t"
                                 "s_waitcnt lgkmcnt(0)"
                                 : "=v"(k1v), "=v"(k2v), "=v"(sv), "=&v"(tmp)
                                 : "s"(coff), "v"(qbase)
                                 : "memory");
                    const float k1r[4] = {k1v.x, k1v.y, k1v.z, k1v.w}, k2r[4] = {k2v.x, k2v.y, k2v.z, k2v.w};
                    const float svr[4] = {sv.x, sv.y, sv.z, sv.w};
#pragma unroll
                    for (int j = 0; j < 4; j++) {
                        const int r = 4 * i + j;
                        float m = agpr_read(acc[0][r]);
#pragma unroll
                        for (int g = 1; g < 8; g++) m = __builtin_fmaxf(m, agpr_read(acc[g][r]));
                        const float t = (m + __builtin_fmaf(nmax, k1r[j], k2r[j])) - svr[j];
                        if (__ballot(force || t >= 0.f)) wact |= 1u << r;
                    }
                }
                if (wact != 0 && (DIAG & 4) == 0) {
                    uint64_t vm[4];
                    {
                        uint4 vw0, vw1, aw0, aw1;
                        uint32_t tmp;
                        asm volatile("v_add_u32 %4, %5, %6\n\t"
                                     "ds_read_b128 %0, %4 offset:1024\n\t"
                                     "ds_read_b128 %1, %4 offset:1040\n\t"
                                     "ds_read_b128 %2, %4 offset:1056\n\t"
                                     "ds_read_b128 %3, %4 offset:1072\n\t"
                                     "s_waitcnt lgkmcnt(0)"
                                     : "=v"(vw0), "=v"(vw1), "=v"(aw0), "=v"(aw1), "=&v"(tmp)
                                     : "s"(nsoff), "v"(sbase)
                                     : "memory");
                        const uint64_t words[4] = {((uint64_t)vw0.y << 32) | vw0.x, ((uint64_t)vw0.w << 32) | vw0.z,
                                                   ((uint64_t)vw1.y << 32) | vw1.x, ((uint64_t)vw1.w << 32) | vw1.z};
                        const uint64_t allows[4] = {((uint64_t)aw0.y << 32) | aw0.x, ((uint64_t)aw0.w << 32) | aw0.z,
                                                    ((uint64_t)aw1.y << 32) | aw1.x, ((uint64_t)aw1.w << 32) | aw1.z};
#pragma unroll
                        for (int h = 0; h < 4; h++) {
                            const uint64_t t = a.tile_begin + blk * 4 + h;
                            uint64_t m = t < a.tile_end ? readfirstlane64(words[h]) : 0ull;
                            if (a.allow) {
                                const uint64_t aw = t - a.allow_t0;
                                m &= aw < a.allow_words ? readfirstlane64(allows[h]) : 0ull;
                            }
                            vm[h] = m;
                        }
                    }
                    const uint64_t slot0 = (a.tile_begin + blk * 4) * 64;
                    // live rows of each row group g (lane l: row 32 g + (l & 31))
                    uint64_t live[8];
#pragma unroll
                    for (int g = 0; g < 8; g++)
                        live[g] = __ballot((vm[g >> 1] >> (32 * (g & 1) + (lane & 31))) & 1ull);
                    const int li = lane & 15;
                    for (uint32_t gw = wact; gw; gw &= gw - 1) {
                        const int r = __builtin_ctz(gw);
                        float uv[8];
                        switch (r) {
#define WVG_SE_SLOT(R)                                                                          \
    case R:                                                                                     \
        _Pragma("unroll") for (int g = 0; g < 8; g++) uv[g] = agpr_read(acc[g][R]);           \
        break;
                        WVG_SE_SLOT(0) WVG_SE_SLOT(1) WVG_SE_SLOT(2) WVG_SE_SLOT(3)
                        WVG_SE_SLOT(4) WVG_SE_SLOT(5) WVG_SE_SLOT(6) WVG_SE_SLOT(7)
                        WVG_SE_SLOT(8) WVG_SE_SLOT(9) WVG_SE_SLOT(10) WVG_SE_SLOT(11)
                        WVG_SE_SLOT(12) WVG_SE_SLOT(13) WVG_SE_SLOT(14) WVG_SE_SLOT(15)
#undef WVG_SE_SLOT
                        default: break;
                        }
                        const uint32_t ql = 8u * (uint32_t)(r >> 2) + (uint32_t)qh + (uint32_t)(r & 3);
                        const uint32_t la = laddr + ql * (SCREEN_M * 8) + 8u * (uint32_t)li;
                        const uint32_t ta = tbase + 4u * ql;  // tau; sig + 512, ck1 + 1024, ck2 + 1536, cem + 2048
                        uint2 v2;
                        float wt, ws, em, k1, k2;
                        asm volatile("ds_read_b64 %0, %6\n\t"
                                     "ds_read_b32 %1, %7\n\t"
                                     "ds_read_b32 %2, %7 offset:512\n\t"
                                     "ds_read_b32 %3, %7 offset:2048\n\t"
                                     "ds_read_b32 %4, %7 offset:1024\n\t"
                                     "ds_read_b32 %5, %7 offset:1536\n\t"
                                     "s_waitcnt lgkmcnt(0)"
                                     : "=v"(v2), "=v"(wt), "=v"(ws), "=v"(em), "=v"(k1), "=v"(k2)
                                     : "v"(la), "v"(ta)
                                     : "memory");
                        uint64_t v = ((uint64_t)v2.y << 32) | v2.x;
#pragma unroll
                        for (int g = 0; g < 8; g++) {
                            const float u = uv[g] + __builtin_fmaf(nrm[g], k1, k2);
                            uint64_t pass = __ballot(!(u < ws)) & live[g];
                            while (pass) {
                                const int j = __builtin_ctzll(pass);
                                pass &= pass - 1;
                                const int gr = 2 * (j >> 5);  // the survivor's query's list row
                                const float lower =
                                    sc_lower(__int_as_float(__builtin_amdgcn_readlane(__float_as_int(u), j)), cosine);
                                float wtg = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(wt), j));
                                if (!(lower <= wtg)) continue;
                                const uint64_t key = ((uint64_t)wvg_ord_f32(lower) << 32) |
                                                     (uint32_t)(slot0 + 32u * (uint32_t)g + (uint32_t)(j & 31));
                                if (!(key < readlane64(v, 16 * gr + SCREEN_M - 1))) continue;
                                const bool inrow = (lane >> 4) == gr;
                                const int pos = __popcll(__ballot(inrow && v < key));
                                const uint64_t sh = row_shr1_64(v);
                                v = inrow ? (li > pos ? sh : (li == pos ? key : v)) : v;
                                const uint64_t nk = readlane64(v, 16 * gr + K - 1);
                                const uint64_t nm = readlane64(v, 16 * gr + SCREEN_M - 1);
                                const float emg = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(em), j));
                                if (nk != WVG_KEY_NONE) wtg = fminf(wtg, sc_tau_k(key_lower(nk), emg, cosine));
                                if (nm != WVG_KEY_NONE) wtg = fminf(wtg, key_lower(nm));
                                const float wsg = sc_sigma(wtg, cosine);
                                const bool mine = (lane >> 5) == (j >> 5);  // lanes of the survivor's query
                                wt = mine ? wtg : wt;
                                ws = mine ? wsg : ws;
                                // that query's other survivors of this row group meet the new threshold
                                pass &= ~(0xFFFFFFFFull << (32 * (j >> 5))) | __ballot(!(u < ws));
                            }
                        }
                        const uint2 o2 = make_uint2((uint32_t)v, (uint32_t)(v >> 32));
                        if (((lane >> 4) & 1) == 0) asm volatile("ds_write_b64 %0, %1" ::"v"(la), "v"(o2) : "memory");
                        if ((lane & 31) == 0)
                            asm volatile("ds_write_b32 %0, %1\n\t"
                                         "ds_write_b32 %0, %2 offset:512" ::"v"(ta), "v"(wt), "v"(ws)
                                         : "memory");
                    }
                    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                }
            } else if constexpr ((DIAG & 8) != 0) {
                float x = 0.f;
#pragma unroll
                for (int g = 0; g < 8; g++) x += agpr_read(acc[g][0]);
                if (x == 0x1p-120f) a.partials[0] = 0;
            }
#pragma unroll
            for (int g = 0; g < 8; g++)
#pragma unroll
                for (int e = 0; e < 16; e++) acc[g][e] = 0.f;
            read_half(0, 0, b0);
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int ql = 0; ql < 32; ql++) {
        const uint32_t q = q0 + (uint32_t)(32 * w + ql);
        if (q >= a.nq) break;
        const uint64_t x = lane < M ? lists[((size_t)w * 32 + ql) * M + lane] : WVG_KEY_NONE;
        uint64_t *out = a.partials + ((size_t)q * a.nrr + rr) * M;
        if (lane < M) out[lane] = x;
        if (lane == K - 1 && x != WVG_KEY_NONE) {
            const float t = sc_tau_k(key_lower(x), cem[32 * w + ql], cosine);
            atomicMin(a.gbound + q, wvg_ord_f32(t));
        }
    }
}

// ---------------------------------------------------------------------------
// K3f (round 5): K3d at two waves per SIMD.  K3d's counters (profiles/r05/k3e)
// put the matrix pipe at 43 % busy: per 32-deep unit its one wave per SIMD
// spends 512 cycles issuing MFMAs and, serially after them, the barrier, four
// LDS-DMA pieces (~60 cycles of issue each) and 16 ds_read_b128 -- ~1180
// cycles per unit.  K3e's fewer, longer MFMAs left that unchanged.  K3f keeps
// 128 queries per workgroup but gives each of 8 waves 16 of them (96 resident
// AGPRs, 64 accumulator AGPRs, 32 for a quarter-stage double buffer), so a SIMD
// holds two waves and one wave's DMA issue, barrier wait and reads overlap the
// other's MFMAs.  The price is LDS traffic: every wave reads the whole stage,
// 128 KiB of ds_read_b128 + 16 KiB of DMA per unit per CU = 576 LDS-array
// cycles at 256 B/clk against 512 MFMA cycles per SIMD -- the LDS, not the
// issue stream, bounds the loop.  Ring, loads (2 pieces per wave), waits,
// epilogue tests and lists are K3d's; lists and thresholds keep K3d's LDS
// layout (wave w owns queries 16 w .. 16 w + 15 of the workgroup's 128).
static_assert(SF_WAVES * 16 == SD_BQ && SD_WAVES * 32 == SD_BQ, "K3f keeps K3d's 128-query LDS layout");

// Vector-memory loads one K3f wave issues for unit u: its 2 row-fragment
// pieces; with unit 0 waves 4..7 also the norms of tile w - 4 and wave 0 the
// block's tile words (ex: a wave with that extra load).
constexpr int sf_unit_loads(int u, bool ex)
{
    return 2 + (u == 0 && ex ? 1 : 0);
}
template <int KBN>
constexpr int sf_younger(int first, int n, bool ex)
{
    int c = 0;
    for (int i = 1; i <= n; i++) c += sf_unit_loads((first + i) % KBN, ex);
    return c;
}

template <int KBN, int DIAG = 0>
__global__ __launch_bounds__(SF_WAVES * 64) void screen_ar16_kernel(ScreenArgs a)
{
    static_assert(KBN % SD_NBUF == 0, "the stage buffer of a K block must be a compile-time constant");
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    uint64_t *lists = reinterpret_cast<uint64_t *>(smem + SD_RING);  // [8][16][M]
    float *tau = reinterpret_cast<float *>(smem + SD_RING + SD_LISTS);
    float *sig = tau + SD_BQ;
    float *ck1 = sig + SD_BQ;
    float *ck2 = ck1 + SD_BQ;
    float *cem = ck2 + SD_BQ;
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int K = (int)a.k, M = SCREEN_M;
    const int cosine = a.cosine;
    const uint32_t b = blockIdx.x;
    uint32_t qb, rr;
    if (a.nrr_l % 8 == 0) {
        const uint32_t xcd = b % 8, wv = b / 8;
        qb = wv % a.nqb;
        rr = a.rr0 + (wv / a.nqb) * 8 + xcd;
    } else {
        qb = b % a.nqb;
        rr = a.rr0 + b / a.nqb;
    }
    const uint64_t ntiles = a.tile_end - a.tile_begin;
    const uint64_t nblk = (ntiles + 3) / 4;
    const uint64_t blk0 = nblk * rr / a.nrr, blk1 = nblk * (rr + 1) / a.nrr;
    const uint32_t q0 = qb * SD_BQ;

    for (int i = tid; i < SD_BQ; i += SF_WAVES * 64) {
        const uint32_t q = q0 + (uint32_t)i;
        ck1[i] = a.k1[q];
        ck2[i] = a.k2[q];
        cem[i] = a.emax[q];
        const uint32_t g = q < a.nq ? __hip_atomic_load(a.gbound + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
        const float t = q >= a.nq ? -__builtin_inff() : (g == 0xFFFFFFFFu ? __builtin_inff() : wvg_unord_f32(g));
        tau[i] = t;
        sig[i] = q >= a.nq ? __builtin_inff() : sc_sigma(t, cosine);
    }
    for (int i = tid; i < SD_BQ * M; i += SF_WAVES * 64) lists[i] = WVG_KEY_NONE;
    __syncthreads();
    const uint32_t laddr = (uint32_t)(uintptr_t)(lists + (size_t)w * 16 * M);
    const uint32_t tbase = (uint32_t)(uintptr_t)(tau + w * 16);  // sig + 512, ck1 + 1024, ck2 + 1536, cem + 2048
    const bool ex = w == 0 || w >= 4;
    if (blk0 < blk1) {
        // the wave's 16 queries, every K block, resident for the whole range: the
        // compiler splits a 256-register wave's file 128 / 128 between VGPRs and
        // AGPRs, so the first SF_AKB K blocks sit next to the accumulators (64) and
        // the quarter buffers (32) in AGPRs, the rest in VGPRs
        constexpr int SF_AKB = 8;
        bf16x8 areg[KBN];
        {
            const uint4 *qsrc = a.qfrag + (size_t)(qb * 8 + w) * KBN * 64 + lane;
#pragma unroll
            for (int ks = 0; ks < KBN; ks++) {
                if (ks < SF_AKB)
                    asm volatile("global_load_dwordx4 %0, %1, off" : "=a"(areg[ks]) : "v"(qsrc + (size_t)ks * 64) : "memory");
                else
                    asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(areg[ks]) : "v"(qsrc + (size_t)ks * 64) : "memory");
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
            for (int ks = 0; ks < KBN; ks++) {
                if (ks < SF_AKB)
                    asm volatile("" : "+a"(areg[ks]));
                else
                    asm volatile("" : "+v"(areg[ks]));
            }
        }
        // loads of one stage: wave w moves row fragments 2 w, 2 w + 1 (tile w / 2, row
        // groups 2 (w & 1) + 0, 1); with unit 0 waves 4..7 the norms of tile w - 4 and
        // wave 0 the block's tile words (sf_unit_loads)
        // (wave-uniform bases + the lane: SGPR base + lane offset, no per-lane 64-bit pointers)
        const uint4 *lsrc = a.shadow + ((size_t)(a.tile_begin + blk0 * 4 + (w >> 1)) * KBN * 4) * 64;
        const float *lnorm = a.norms + (a.tile_begin + blk0 * 4 + (w & 3)) * 64;
        const int rg0 = 2 * (w & 1);
        uint64_t lblk = blk0;
        auto load_stage = [&](int ks) {
            unsigned char *dst = smem + (ks % SD_NBUF) * SD_STAGE;
#pragma unroll
            for (int j = 0; j < 2; j++)
                __builtin_amdgcn_global_load_lds(lsrc + ((size_t)ks * 4 + rg0 + j) * 64 + lane,
                                                 reinterpret_cast<uint4 *>(dst + (2 * w + j) * 1024), 16, 0, 0);
            unsigned char *nslot = smem + SD_NBUF * SD_STAGE + (lblk & 1) * SD_NSLOT;
            if (ks == 0 && w >= 4)
                __builtin_amdgcn_global_load_lds(lnorm + lane, reinterpret_cast<float *>(nslot + (w - 4) * 256), 4, 0,
                                                 0);
            if (ks == 0 && w == 0) {
                const uint32_t wi = (uint32_t)(lane & 7) >> 1, half = lane & 1;
                const uint64_t t = a.tile_begin + lblk * 4 + wi;
                const uint32_t *src =
                    reinterpret_cast<const uint32_t *>(a.valid + (t < a.tile_end ? t : a.tile_end - 1)) + half;
                if (lane >= 8 && lane < 16 && a.allow) {
                    const uint64_t aw = t - a.allow_t0;
                    src = reinterpret_cast<const uint32_t *>(a.allow + (aw < a.allow_words ? aw : 0)) + half;
                }
                __builtin_amdgcn_global_load_lds(src, reinterpret_cast<uint32_t *>(nslot + 1024), 4, 0, 0);
            }
            if (ks == KBN - 1 && lblk + 1 < blk1) {  // the load cursor moves on; past the end it stays
                ++lblk;
                lsrc += (size_t)4 * KBN * 4 * 64;
                lnorm += 256;
            }
        };
        // six stages in flight at every wait (K3d's ring): unit ks + 1 landed, the
        // loads of units ks + 2 .. ks + 6 left outstanding
        auto wait_next = [&](auto KS) {
            constexpr int ks = decltype(KS)::value;
            constexpr int n1 = sf_younger<KBN>(ks + 1, SD_NBUF - 3, true);
            constexpr int n0 = sf_younger<KBN>(ks + 1, SD_NBUF - 3, false);
            if (ex) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(n1) : "memory");
            else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(n0) : "memory");
        };
        auto raw_barrier = [&]() {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");
        };
        // A quarter stage (row fragments 4 qq .. 4 qq + 3) straight into AGPRs, in
        // flight while the previous quarter's MFMAs issue; consumers pass wait_q
        // (lgkmcnt(4): every read but the 4 younger ones landed) or the barrier.
        // The stage / quarter offset is an instruction literal (as SGPR operands the
        // 32 distinct offsets were hoisted into SGPRs and spilled).
        const uint32_t rbase = (uint32_t)(uintptr_t)smem + 16u * lane;
        auto read_q = [](auto KS, auto QQ, bf16x8 (&br)[4], uint32_t rb) {
            constexpr uint32_t soff =
                (uint32_t)((decltype(KS)::value % SD_NBUF) * SD_STAGE + decltype(QQ)::value * 4 * 1024);
            uint32_t tmp;
            asm volatile("v_add_u32 %4, %5, %6\n\t"
                         "ds_read_b128 %0, %4\n\t"
                         "ds_read_b128 %1, %4 offset:1024\n\t"
                         "ds_read_b128 %2, %4 offset:2048\n\t"
                         "ds_read_b128 %3, %4 offset:3072"
                         : "=a"(br[0]), "=a"(br[1]), "=a"(br[2]), "=a"(br[3]), "=&v"(tmp)
                         : "n"(soff), "v"(rb)
                         : "memory");
        };
        using I0 = std::integral_constant<int, 0>;
        using I1 = std::integral_constant<int, 1>;
        using I2 = std::integral_constant<int, 2>;
        using I3 = std::integral_constant<int, 3>;
        auto wait_q = [&](bf16x8 (&br)[4]) {
            asm volatile("s_waitcnt lgkmcnt(4)" : "+a"(br[0]), "+a"(br[1]), "+a"(br[2]), "+a"(br[3]) : : "memory");
        };
        const int qlane = 4 * (lane >> 4);
        const uint32_t sbase = (uint32_t)(uintptr_t)smem;
        const uint32_t nbase = sbase + 4u * (uint32_t)(lane & 15);
        const uint32_t qbase = sbase + 4u * (uint32_t)qlane;
        const uint32_t csoff = (uint32_t)((uintptr_t)sig - (uintptr_t)smem);
        bool lane_force = false;
#pragma unroll
        for (int r = 0; r < 4; r++)
            if (!(ck1[16 * w + qlane + r] <= 0x1p50f)) lane_force = true;

        floatx4 acc[16];
#pragma unroll
        for (int nr = 0; nr < 16; nr++) acc[nr] = (floatx4){0.f, 0.f, 0.f, 0.f};
        bf16x8 bq0[4], bq1[4];
        auto mfma4 = [&](int ks, int qq, bf16x8 (&br)[4]) {
#pragma unroll
            for (int j = 0; j < 4; j++)
                acc[4 * qq + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(areg[ks], br[j], acc[4 * qq + j], 0, 0, 0);
        };
#pragma unroll
        for (int ks = 0; ks < SD_NBUF - 1; ks++) load_stage(ks);
        if (ex) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(sf_younger<KBN>(0, SD_NBUF - 2, true)) : "memory");
        else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(sf_younger<KBN>(0, SD_NBUF - 2, false)) : "memory");
        raw_barrier();
        read_q(I0{}, I0{}, bq0, rbase);
        for (uint64_t blk = blk0; blk < blk1; blk++) {
            sd_static_for<KBN>([&](auto KS) {
                constexpr int ks = decltype(KS)::value;
                read_q(KS, I1{}, bq1, rbase);
                wait_q(bq0);
                mfma4(ks, 0, bq0);
                read_q(KS, I2{}, bq0, rbase);
                wait_q(bq1);
                mfma4(ks, 1, bq1);
                read_q(KS, I3{}, bq1, rbase);
                wait_q(bq0);
                mfma4(ks, 2, bq0);
                wait_next(KS);  // the next unit landed
                raw_barrier();  // (lgkmcnt(0): quarter 3 landed)
#pragma unroll
                for (int j = 0; j < 4; j++) asm volatile("" : "+a"(bq1[j]));
                load_stage((ks + SD_NBUF - 1) % KBN);  // into the buffer of unit - 1, read before the barrier
                if constexpr (ks + 1 < KBN) read_q(std::integral_constant<int, ks + 1>{}, I0{}, bq0, rbase);
                mfma4(ks, 3, bq1);
            });
            // XDL write -> VALU read of the accumulators through agpr_read: see K3d
            __builtin_amdgcn_sched_barrier(0);
            asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
            __builtin_amdgcn_sched_barrier(0);
            if constexpr ((DIAG & 2) == 0) {
                // K3d's epilogue over the wave's 16 queries: C layout row (query) qlane + r,
                // column (row) 16 nr + (lane & 15); fast check per query r, exact test on
                // the groups it could not rule out
                const uint32_t nsoff = (uint32_t)(SD_NBUF * SD_STAGE + (blk & 1) * SD_NSLOT);
                auto read_norms8 = [&](int hh, float (&nrm)[8]) {
                    uint32_t tmp;
                    asm volatile("v_add_u32 %8, %9, %10\n\t"
                                 "ds_read_b32 %0, %8\n\t"
                                 "ds_read_b32 %1, %8 offset:64\n\t"
                                 "ds_read_b32 %2, %8 offset:128\n\t"
                                 "ds_read_b32 %3, %8 offset:192\n\t"
                                 "ds_read_b32 %4, %8 offset:256\n\t"
                                 "ds_read_b32 %5, %8 offset:320\n\t"
                                 "ds_read_b32 %6, %8 offset:384\n\t"
                                 "ds_read_b32 %7, %8 offset:448\n\t"
                                 "s_waitcnt lgkmcnt(0)"
                                 : "=v"(nrm[0]), "=v"(nrm[1]), "=v"(nrm[2]), "=v"(nrm[3]), "=v"(nrm[4]),
                                   "=v"(nrm[5]), "=v"(nrm[6]), "=v"(nrm[7]), "=&v"(tmp)
                                 : "s"(nsoff + 512u * hh), "v"(nbase)
                                 : "memory");
                };
                float nmax, nsum;
                {
                    float n0[8], n1[8];
                    read_norms8(0, n0);
                    read_norms8(1, n1);
                    nmax = n0[0];
                    nsum = n0[0];
#pragma unroll
                    for (int j2 = 1; j2 < 8; j2++) nmax = __builtin_fmaxf(nmax, n0[j2]), nsum += n0[j2];
#pragma unroll
                    for (int j2 = 0; j2 < 8; j2++) nmax = __builtin_fmaxf(nmax, n1[j2]), nsum += n1[j2];
                }
                const bool force = lane_force || !(nmax <= 0x1p60f) || nsum != nsum;
                uint32_t wact = 0;
                {
                    const uint32_t coff = (uint32_t)(csoff + 4 * (16 * w));
                    float4 k1v, k2v, sv;
                    uint32_t tmp;
                    asm volatile("v_add_u32 %3, %4, %5\n\t"
                                 "ds_read_b128 %0, %3 offset:512\n\t"
                                 "ds_read_b128 %1, %3 offset:1024\n\t"
                                 "ds_read_b128 %2, %3\n\t"
                                 "s_waitcnt lgkmcnt(0)"
                                 : "=v"(k1v), "=v"(k2v), "=v"(sv), "=&v"(tmp)
                                 : "s"(coff), "v"(qbase)
                                 : "memory");
                    const float k1r[4] = {k1v.x, k1v.y, k1v.z, k1v.w};
                    const float k2r[4] = {k2v.x, k2v.y, k2v.z, k2v.w};
                    const float svr[4] = {sv.x, sv.y, sv.z, sv.w};
#pragma unroll
                    for (int r = 0; r < 4; r++) {
                        float m = agpr_read(acc[0][r]);
#pragma unroll
                        for (int nr = 1; nr < 16; nr++) m = __builtin_fmaxf(m, agpr_read(acc[nr][r]));
                        const float t = (m + __builtin_fmaf(nmax, k1r[r], k2r[r])) - svr[r];
                        if (__ballot(force || t >= 0.f)) wact |= 1u << r;
                    }
                }
                if (wact != 0) {
                    uint64_t vm[4];
                    {
                        uint4 vw0, vw1, aw0, aw1;
                        uint32_t tmp;
                        asm volatile("v_add_u32 %4, %5, %6\n\t"
                                     "ds_read_b128 %0, %4 offset:1024\n\t"
                                     "ds_read_b128 %1, %4 offset:1040\n\t"
                                     "ds_read_b128 %2, %4 offset:1056\n\t"
                                     "ds_read_b128 %3, %4 offset:1072\n\t"
                                     "s_waitcnt lgkmcnt(0)"
                                     : "=v"(vw0), "=v"(vw1), "=v"(aw0), "=v"(aw1), "=&v"(tmp)
                                     : "s"(nsoff), "v"(sbase)
                                     : "memory");
                        const uint64_t words[4] = {((uint64_t)vw0.y << 32) | vw0.x, ((uint64_t)vw0.w << 32) | vw0.z,
                                                   ((uint64_t)vw1.y << 32) | vw1.x, ((uint64_t)vw1.w << 32) | vw1.z};
                        const uint64_t allows[4] = {((uint64_t)aw0.y << 32) | aw0.x, ((uint64_t)aw0.w << 32) | aw0.z,
                                                    ((uint64_t)aw1.y << 32) | aw1.x, ((uint64_t)aw1.w << 32) | aw1.z};
#pragma unroll
                        for (int h = 0; h < 4; h++) {
                            const uint64_t t = a.tile_begin + blk * 4 + h;
                            uint64_t m = t < a.tile_end ? readfirstlane64(words[h]) : 0ull;
                            if (a.allow) {
                                const uint64_t aw = t - a.allow_t0;
                                m &= aw < a.allow_words ? readfirstlane64(allows[h]) : 0ull;
                            }
                            vm[h] = m;
                        }
                    }
                    const uint64_t slot0 = (a.tile_begin + blk * 4) * 64;
                    // per active query slot gi: lane l tests its column's 16 rows against query
                    // qlane + gi, and row l >> 4 of v holds that query's list (K3d's slow path;
                    // four groups, each its own unrolled copy reading its accumulators in place)
                    sd_static_for<4>([&](auto G) {
                        constexpr int gi = decltype(G)::value;
                        if (((wact >> gi) & 1u) == 0) return;
                        const uint32_t ql = (uint32_t)gi + (uint32_t)qlane;
                        const uint32_t la = laddr + ql * (SCREEN_M * 8) + 8u * (uint32_t)(lane & 15);
                        const uint32_t ta = tbase + 4u * ql;
                        uint2 v2;
                        float wt, ws, em, k1, k2;
                        asm volatile("ds_read_b64 %0, %6\n\t"
                                     "ds_read_b32 %1, %7\n\t"
                                     "ds_read_b32 %2, %7 offset:512\n\t"
                                     "ds_read_b32 %3, %7 offset:2048\n\t"
                                     "ds_read_b32 %4, %7 offset:1024\n\t"
                                     "ds_read_b32 %5, %7 offset:1536\n\t"
                                     "s_waitcnt lgkmcnt(0)"
                                     : "=v"(v2), "=v"(wt), "=v"(ws), "=v"(em), "=v"(k1), "=v"(k2)
                                     : "v"(la), "v"(ta)
                                     : "memory");
                        uint64_t v = ((uint64_t)v2.y << 32) | v2.x;
                        const int li = lane & 15;
#pragma unroll
                        for (int nr = 0; nr < 16; nr++) {
                            const uint64_t m64 = ((vm[nr >> 2] >> (16 * (nr & 3))) & 0xFFFFull) * 0x0001000100010001ull;
                            float nrm;  // the row norm of this lane's column (read here: 16 fewer live VGPRs)
                            asm volatile("ds_read_b32 %0, %1 offset:%2\n\t"
                                         "s_waitcnt lgkmcnt(0)"
                                         : "=v"(nrm)
                                         : "v"(nbase + nsoff), "n"(64 * nr)
                                         : "memory");
                            const float u = agpr_read(acc[nr][gi]) + __builtin_fmaf(nrm, k1, k2);
                            uint64_t pass = __ballot(!(u < ws)) & m64;
                            while (pass) {
                                const int j = __builtin_ctzll(pass);
                                pass &= pass - 1;
                                const int g = j >> 4;
                                const float lower =
                                    sc_lower(__int_as_float(__builtin_amdgcn_readlane(__float_as_int(u), j)), cosine);
                                float wtg = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(wt), j));
                                if (!(lower <= wtg)) continue;
                                const uint64_t key = ((uint64_t)wvg_ord_f32(lower) << 32) |
                                                     (uint32_t)(slot0 + 16u * (uint32_t)nr + (uint32_t)(j & 15));
                                if (!(key < readlane64(v, 16 * g + SCREEN_M - 1))) continue;
                                const bool inrow = (lane >> 4) == g;
                                const int pos = __popcll(__ballot(inrow && v < key));
                                const uint64_t sh = row_shr1_64(v);
                                v = inrow ? (li > pos ? sh : (li == pos ? key : v)) : v;
                                const uint64_t nk = readlane64(v, 16 * g + K - 1);
                                const uint64_t nm = readlane64(v, 16 * g + SCREEN_M - 1);
                                const float emg = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(em), j));
                                if (nk != WVG_KEY_NONE) wtg = fminf(wtg, sc_tau_k(key_lower(nk), emg, cosine));
                                if (nm != WVG_KEY_NONE) wtg = fminf(wtg, key_lower(nm));
                                const float wsg = sc_sigma(wtg, cosine);
                                wt = inrow ? wtg : wt;
                                ws = inrow ? wsg : ws;
                                pass &= ~(0xFFFFull << (16 * g)) | __ballot(!(u < ws));
                            }
                        }
                        const uint2 o2 = make_uint2((uint32_t)v, (uint32_t)(v >> 32));
                        asm volatile("ds_write_b64 %0, %1" ::"v"(la), "v"(o2) : "memory");
                        if (li == 0)
                            asm volatile("ds_write_b32 %0, %1\n\t"
                                         "ds_write_b32 %0, %2 offset:512" ::"v"(ta), "v"(wt), "v"(ws)
                                         : "memory");
                        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                    });
                }
            } else if constexpr ((DIAG & 8) != 0) {
                // diagnostic (DIAG 10): the stage loop alone, the accumulators consumed by one sum
                float x = 0.f;
#pragma unroll
                for (int nr = 0; nr < 16; nr++) x += agpr_read(acc[nr][0]);
                if (x == 0x1p-120f) a.partials[0] = 0;
            }
#pragma unroll
            for (int nr = 0; nr < 16; nr++) acc[nr] = (floatx4){0.f, 0.f, 0.f, 0.f};
            read_q(I0{}, I0{}, bq0, rbase);
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int ql = 0; ql < 16; ql++) {
        const uint32_t q = q0 + (uint32_t)(16 * w + ql);
        if (q >= a.nq) break;
        const uint64_t x = lane < M ? lists[((size_t)w * 16 + ql) * M + lane] : WVG_KEY_NONE;
        uint64_t *out = a.partials + ((size_t)q * a.nrr + rr) * M;
        if (lane < M) out[lane] = x;
        if (lane == K - 1 && x != WVG_KEY_NONE) {
            const float t = sc_tau_k(key_lower(x), cem[16 * w + ql], cosine);
            atomicMin(a.gbound + q, wvg_ord_f32(t));
        }
    }
}

// ---------------------------------------------------------------------------
// K3g (round 5, tools variant 4): K3f's 16-query waves in 4-wave workgroups of
// 64 queries, TWO workgroups per CU, each with its own 4-stage ring and its
// own barrier.  K3f's 8 waves shared one barrier per unit, so the two waves of
// a SIMD issued MFMAs, DMA and reads in the same phase; two independent
// workgroups drift apart, so one wave's DMA issue and barrier wait can fall in
// the other's MFMA stream.  Costs: every CU streams each row block twice (once
// per 64-query workgroup; L2 hits) and the ring holds 2 stages in flight
// instead of 6.
constexpr int SG_WAVES = 4;
constexpr int SG_BQ = 64;
constexpr int SG_NBUF = 4;
constexpr int SG_RING = SG_NBUF * SD_STAGE + 2 * SD_NSLOT;
constexpr int SG_LISTS = SG_BQ * SCREEN_M * 8;
constexpr int SG_LDS = SG_RING + SG_LISTS + SG_BQ * 4 * 5;
static_assert(2 * SG_LDS <= 160 * 1024, "K3g: two workgroups per CU");
static_assert(SG_WAVES * 16 == SG_BQ, "K3g: 16 queries per wave");

template <int KBN, int DIAG = 0>
__global__ __launch_bounds__(SG_WAVES * 64, 2) void screen_ar16x2_kernel(ScreenArgs a)
{
    static_assert(KBN % SG_NBUF == 0, "the stage buffer of a K block must be a compile-time constant");
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    uint64_t *lists = reinterpret_cast<uint64_t *>(smem + SG_RING);  // [4][16][M]
    float *tau = reinterpret_cast<float *>(smem + SG_RING + SG_LISTS);
    float *sig = tau + SG_BQ;
    float *ck1 = sig + SG_BQ;
    float *ck2 = ck1 + SG_BQ;
    float *cem = ck2 + SG_BQ;
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int K = (int)a.k, M = SCREEN_M;
    const int cosine = a.cosine;
    const uint32_t b = blockIdx.x;
    uint32_t qb, rr;
    if (a.nrr_l % 8 == 0) {
        const uint32_t xcd = b % 8, wv = b / 8;
        qb = wv % a.nqb;
        rr = a.rr0 + (wv / a.nqb) * 8 + xcd;
    } else {
        qb = b % a.nqb;
        rr = a.rr0 + b / a.nqb;
    }
    const uint64_t ntiles = a.tile_end - a.tile_begin;
    const uint64_t nblk = (ntiles + 3) / 4;
    const uint64_t blk0 = nblk * rr / a.nrr, blk1 = nblk * (rr + 1) / a.nrr;
    const uint32_t q0 = qb * SG_BQ;

    for (int i = tid; i < SG_BQ; i += SG_WAVES * 64) {
        const uint32_t q = q0 + (uint32_t)i;
        ck1[i] = a.k1[q];
        ck2[i] = a.k2[q];
        cem[i] = a.emax[q];
        const uint32_t g = q < a.nq ? __hip_atomic_load(a.gbound + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
        const float t = q >= a.nq ? -__builtin_inff() : (g == 0xFFFFFFFFu ? __builtin_inff() : wvg_unord_f32(g));
        tau[i] = t;
        sig[i] = q >= a.nq ? __builtin_inff() : sc_sigma(t, cosine);
    }
    for (int i = tid; i < SG_BQ * M; i += SG_WAVES * 64) lists[i] = WVG_KEY_NONE;
    __syncthreads();
    const uint32_t laddr = (uint32_t)(uintptr_t)(lists + (size_t)w * 16 * M);
    const uint32_t tbase = (uint32_t)(uintptr_t)(tau + w * 16);  // sig + 256, ck1 + 512, ck2 + 768, cem + 1024
    if (blk0 < blk1) {
        // the wave's 16 queries, every K block, resident for the whole range: the
        // compiler splits a 256-register wave's file 128 / 128 between VGPRs and
        // AGPRs, so the first SF_AKB K blocks sit next to the accumulators (64) and
        // the quarter buffers (32) in AGPRs, the rest in VGPRs
        constexpr int SF_AKB = 8;
        bf16x8 areg[KBN];
        {
            const uint4 *qsrc = a.qfrag + (size_t)(qb * 4 + w) * KBN * 64 + lane;
#pragma unroll
            for (int ks = 0; ks < KBN; ks++) {
                if (ks < SF_AKB)
                    asm volatile("global_load_dwordx4 %0, %1, off" : "=a"(areg[ks]) : "v"(qsrc + (size_t)ks * 64) : "memory");
                else
                    asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(areg[ks]) : "v"(qsrc + (size_t)ks * 64) : "memory");
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
            for (int ks = 0; ks < KBN; ks++) {
                if (ks < SF_AKB)
                    asm volatile("" : "+a"(areg[ks]));
                else
                    asm volatile("" : "+v"(areg[ks]));
            }
        }
        // loads of one stage (K3d's): wave w moves row fragments 4 w .. 4 w + 3 (tile w),
        // with unit 0 also the norms of tile w, and wave 0 the block's tile words
        const uint4 *lsrc = a.shadow + ((size_t)(a.tile_begin + blk0 * 4 + w) * KBN * 4) * 64;
        const float *lnorm = a.norms + (a.tile_begin + blk0 * 4 + w) * 64;
        uint64_t lblk = blk0;
        auto load_stage = [&](int ks) {
            unsigned char *dst = smem + (ks % SG_NBUF) * SD_STAGE;
#pragma unroll
            for (int rg = 0; rg < 4; rg++)
                __builtin_amdgcn_global_load_lds(lsrc + ((size_t)ks * 4 + rg) * 64 + lane,
                                                 reinterpret_cast<uint4 *>(dst + (4 * w + rg) * 1024), 16, 0, 0);
            unsigned char *nslot = smem + SG_NBUF * SD_STAGE + (lblk & 1) * SD_NSLOT;
            if (ks == 0)
                __builtin_amdgcn_global_load_lds(lnorm + lane, reinterpret_cast<float *>(nslot + w * 256), 4, 0, 0);
            if (ks == 0 && w == 0) {
                const uint32_t wi = (uint32_t)(lane & 7) >> 1, half = lane & 1;
                const uint64_t t = a.tile_begin + lblk * 4 + wi;
                const uint32_t *src =
                    reinterpret_cast<const uint32_t *>(a.valid + (t < a.tile_end ? t : a.tile_end - 1)) + half;
                if (lane >= 8 && lane < 16 && a.allow) {
                    const uint64_t aw = t - a.allow_t0;
                    src = reinterpret_cast<const uint32_t *>(a.allow + (aw < a.allow_words ? aw : 0)) + half;
                }
                __builtin_amdgcn_global_load_lds(src, reinterpret_cast<uint32_t *>(nslot + 1024), 4, 0, 0);
            }
            if (ks == KBN - 1 && lblk + 1 < blk1) {  // the load cursor moves on; past the end it stays
                ++lblk;
                lsrc += (size_t)4 * KBN * 4 * 64;
                lnorm += 256;
            }
        };
        // SG_NBUF - 2 stages in flight at every wait: unit ks + 1 landed, the loads of
        // units ks + 2 .. ks + SG_NBUF - 2 left outstanding (K3d's per-unit load counts)
        auto wait_next = [&](auto KS) {
            constexpr int ks = decltype(KS)::value;
            constexpr int n0 = sd_younger<KBN, 0>(ks + 1, SG_NBUF - 3, true);
            constexpr int n1 = sd_younger<KBN, 0>(ks + 1, SG_NBUF - 3, false);
            if (w == 0) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(n0) : "memory");
            else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(n1) : "memory");
        };
        auto raw_barrier = [&]() {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");
        };
        // A quarter stage (row fragments 4 qq .. 4 qq + 3) straight into AGPRs, in
        // flight while the previous quarter's MFMAs issue; consumers pass wait_q
        // (lgkmcnt(4): every read but the 4 younger ones landed) or the barrier.
        // The stage / quarter offset is an instruction literal (as SGPR operands the
        // 32 distinct offsets were hoisted into SGPRs and spilled).
        const uint32_t rbase = (uint32_t)(uintptr_t)smem + 16u * lane;
        auto read_q = [](auto KS, auto QQ, bf16x8 (&br)[4], uint32_t rb) {
            constexpr uint32_t soff =
                (uint32_t)((decltype(KS)::value % SG_NBUF) * SD_STAGE + decltype(QQ)::value * 4 * 1024);
            uint32_t tmp;
            asm volatile("v_add_u32 %4, %5, %6\n\t"
                         "ds_read_b128 %0, %4\n\t"
                         "ds_read_b128 %1, %4 offset:1024\n\t"
                         "ds_read_b128 %2, %4 offset:2048\n\t"
                         "ds_read_b128 %3, %4 offset:3072"
                         : "=a"(br[0]), "=a"(br[1]), "=a"(br[2]), "=a"(br[3]), "=&v"(tmp)
                         : "n"(soff), "v"(rb)
                         : "memory");
        };
        using I0 = std::integral_constant<int, 0>;
        using I1 = std::integral_constant<int, 1>;
        using I2 = std::integral_constant<int, 2>;
        using I3 = std::integral_constant<int, 3>;
        auto wait_q = [&](bf16x8 (&br)[4]) {
            asm volatile("s_waitcnt lgkmcnt(4)" : "+a"(br[0]), "+a"(br[1]), "+a"(br[2]), "+a"(br[3]) : : "memory");
        };
        const int qlane = 4 * (lane >> 4);
        const uint32_t sbase = (uint32_t)(uintptr_t)smem;
        const uint32_t nbase = sbase + 4u * (uint32_t)(lane & 15);
        const uint32_t qbase = sbase + 4u * (uint32_t)qlane;
        const uint32_t csoff = (uint32_t)((uintptr_t)sig - (uintptr_t)smem);
        bool lane_force = false;
#pragma unroll
        for (int r = 0; r < 4; r++)
            if (!(ck1[16 * w + qlane + r] <= 0x1p50f)) lane_force = true;

        floatx4 acc[16];
#pragma unroll
        for (int nr = 0; nr < 16; nr++) acc[nr] = (floatx4){0.f, 0.f, 0.f, 0.f};
        bf16x8 bq0[4], bq1[4];
        auto mfma4 = [&](int ks, int qq, bf16x8 (&br)[4]) {
#pragma unroll
            for (int j = 0; j < 4; j++)
                acc[4 * qq + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(areg[ks], br[j], acc[4 * qq + j], 0, 0, 0);
        };
#pragma unroll
        for (int ks = 0; ks < SG_NBUF - 1; ks++) load_stage(ks);
        if (w == 0) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(sd_younger<KBN, 0>(0, SG_NBUF - 2, true)) : "memory");
        else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(sd_younger<KBN, 0>(0, SG_NBUF - 2, false)) : "memory");
        raw_barrier();
        read_q(I0{}, I0{}, bq0, rbase);
        for (uint64_t blk = blk0; blk < blk1; blk++) {
            sd_static_for<KBN>([&](auto KS) {
                constexpr int ks = decltype(KS)::value;
                read_q(KS, I1{}, bq1, rbase);
                wait_q(bq0);
                mfma4(ks, 0, bq0);
                read_q(KS, I2{}, bq0, rbase);
                wait_q(bq1);
                mfma4(ks, 1, bq1);
                read_q(KS, I3{}, bq1, rbase);
                wait_q(bq0);
                mfma4(ks, 2, bq0);
                wait_next(KS);  // the next unit landed
                raw_barrier();  // (lgkmcnt(0): quarter 3 landed)
#pragma unroll
                for (int j = 0; j < 4; j++) asm volatile("" : "+a"(bq1[j]));
                load_stage((ks + SG_NBUF - 1) % KBN);  // into the buffer of unit - 1, read before the barrier
                if constexpr (ks + 1 < KBN) read_q(std::integral_constant<int, ks + 1>{}, I0{}, bq0, rbase);
                mfma4(ks, 3, bq1);
            });
            // XDL write -> VALU read of the accumulators through agpr_read: see K3d
            __builtin_amdgcn_sched_barrier(0);
            asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
            __builtin_amdgcn_sched_barrier(0);
            if constexpr ((DIAG & 2) == 0) {
                // K3d's epilogue over the wave's 16 queries: C layout row (query) qlane + r,
                // column (row) 16 nr + (lane & 15); fast check per query r, exact test on
                // the groups it could not rule out
                const uint32_t nsoff = (uint32_t)(SG_NBUF * SD_STAGE + (blk & 1) * SD_NSLOT);
                auto read_norms8 = [&](int hh, float (&nrm)[8]) {
                    uint32_t tmp;
                    asm volatile("v_add_u32 %8, %9, %10\n\t"
                                 "ds_read_b32 %0, %8\n\t"
                                 "ds_read_b32 %1, %8 offset:64\n\t"
                                 "ds_read_b32 %2, %8 offset:128\n\t"
                                 "ds_read_b32 %3, %8 offset:192\n\t"
                                 "ds_read_b32 %4, %8 offset:256\n\t"
                                 "ds_read_b32 %5, %8 offset:320\n\t"
                                 "ds_read_b32 %6, %8 offset:384\n\t"
                                 "ds_read_b32 %7, %8 offset:448\n\t"
                                 "s_waitcnt lgkmcnt(0)"
                                 : "=v"(nrm[0]), "=v"(nrm[1]), "=v"(nrm[2]), "=v"(nrm[3]), "=v"(nrm[4]),
                                   "=v"(nrm[5]), "=v"(nrm[6]), "=v"(nrm[7]), "=&v"(tmp)
                                 : "s"(nsoff + 512u * hh), "v"(nbase)
                                 : "memory");
                };
                float nmax, nsum;
                {
                    float n0[8], n1[8];
                    read_norms8(0, n0);
                    read_norms8(1, n1);
                    nmax = n0[0];
                    nsum = n0[0];
#pragma unroll
                    for (int j2 = 1; j2 < 8; j2++) nmax = __builtin_fmaxf(nmax, n0[j2]), nsum += n0[j2];
#pragma unroll
                    for (int j2 = 0; j2 < 8; j2++) nmax = __builtin_fmaxf(nmax, n1[j2]), nsum += n1[j2];
                }
                const bool force = lane_force || !(nmax <= 0x1p60f) || nsum != nsum;
                uint32_t wact = 0;
                {
                    const uint32_t coff = (uint32_t)(csoff + 4 * (16 * w));
                    float4 k1v, k2v, sv;
                    uint32_t tmp;
                    asm volatile("v_add_u32 %3, %4, %5\n\t"
                                 "ds_read_b128 %0, %3 offset:256\n\t"
                                 "ds_read_b128 %1, %3 offset:512\n\t"
                                 "ds_read_b128 %2, %3\n\t"
                                 "s_waitcnt lgkmcnt(0)"
                                 : "=v"(k1v), "=v"(k2v), "=v"(sv), "=&v"(tmp)
                                 : "s"(coff), "v"(qbase)
                                 : "memory");
                    const float k1r[4] = {k1v.x, k1v.y, k1v.z, k1v.w};
                    const float k2r[4] = {k2v.x, k2v.y, k2v.z, k2v.w};
                    const float svr[4] = {sv.x, sv.y, sv.z, sv.w};
#pragma unroll
                    for (int r = 0; r < 4; r++) {
                        float m = agpr_read(acc[0][r]);
#pragma unroll
                        for (int nr = 1; nr < 16; nr++) m = __builtin_fmaxf(m, agpr_read(acc[nr][r]));
                        const float t = (m + __builtin_fmaf(nmax, k1r[r], k2r[r])) - svr[r];
                        if (__ballot(force || t >= 0.f)) wact |= 1u << r;
                    }
                }
                if (wact != 0) {
                    uint64_t vm[4];
                    {
                        uint4 vw0, vw1, aw0, aw1;
                        uint32_t tmp;
                        asm volatile("v_add_u32 %4, %5, %6\n\t"
                                     "ds_read_b128 %0, %4 offset:1024\n\t"
                                     "ds_read_b128 %1, %4 offset:1040\n\t"
                                     "ds_read_b128 %2, %4 offset:1056\n\t"
                                     "ds_read_b128 %3, %4 offset:1072\n\t"
                                     "s_waitcnt lgkmcnt(0)"
                                     : "=v"(vw0), "=v"(vw1), "=v"(aw0), "=v"(aw1), "=&v"(tmp)
                                     : "s"(nsoff), "v"(sbase)
                                     : "memory");
                        const uint64_t words[4] = {((uint64_t)vw0.y << 32) | vw0.x, ((uint64_t)vw0.w << 32) | vw0.z,
                                                   ((uint64_t)vw1.y << 32) | vw1.x, ((uint64_t)vw1.w << 32) | vw1.z};
                        const uint64_t allows[4] = {((uint64_t)aw0.y << 32) | aw0.x, ((uint64_t)aw0.w << 32) | aw0.z,
                                                    ((uint64_t)aw1.y << 32) | aw1.x, ((uint64_t)aw1.w << 32) | aw1.z};
#pragma unroll
                        for (int h = 0; h < 4; h++) {
                            const uint64_t t = a.tile_begin + blk * 4 + h;
                            uint64_t m = t < a.tile_end ? readfirstlane64(words[h]) : 0ull;
                            if (a.allow) {
                                const uint64_t aw = t - a.allow_t0;
                                m &= aw < a.allow_words ? readfirstlane64(allows[h]) : 0ull;
                            }
                            vm[h] = m;
                        }
                    }
                    const uint64_t slot0 = (a.tile_begin + blk * 4) * 64;
                    // per active query slot gi: lane l tests its column's 16 rows against query
                    // qlane + gi, and row l >> 4 of v holds that query's list (K3d's slow path;
                    // four groups, each its own unrolled copy reading its accumulators in place)
                    sd_static_for<4>([&](auto G) {
                        constexpr int gi = decltype(G)::value;
                        if (((wact >> gi) & 1u) == 0) return;
                        const uint32_t ql = (uint32_t)gi + (uint32_t)qlane;
                        const uint32_t la = laddr + ql * (SCREEN_M * 8) + 8u * (uint32_t)(lane & 15);
                        const uint32_t ta = tbase + 4u * ql;
                        uint2 v2;
                        float wt, ws, em, k1, k2;
                        asm volatile("ds_read_b64 %0, %6\n\t"
                                     "ds_read_b32 %1, %7\n\t"
                                     "ds_read_b32 %2, %7 offset:256\n\t"
                                     "ds_read_b32 %3, %7 offset:1024\n\t"
                                     "ds_read_b32 %4, %7 offset:512\n\t"
                                     "ds_read_b32 %5, %7 offset:768\n\t"
                                     "s_waitcnt lgkmcnt(0)"
                                     : "=v"(v2), "=v"(wt), "=v"(ws), "=v"(em), "=v"(k1), "=v"(k2)
                                     : "v"(la), "v"(ta)
                                     : "memory");
                        uint64_t v = ((uint64_t)v2.y << 32) | v2.x;
                        const int li = lane & 15;
#pragma unroll
                        for (int nr = 0; nr < 16; nr++) {
                            const uint64_t m64 = ((vm[nr >> 2] >> (16 * (nr & 3))) & 0xFFFFull) * 0x0001000100010001ull;
                            float nrm;  // the row norm of this lane's column (read here: 16 fewer live VGPRs)
                            asm volatile("ds_read_b32 %0, %1 offset:%2\n\t"
                                         "s_waitcnt lgkmcnt(0)"
                                         : "=v"(nrm)
                                         : "v"(nbase + nsoff), "n"(64 * nr)
                                         : "memory");
                            const float u = agpr_read(acc[nr][gi]) + __builtin_fmaf(nrm, k1, k2);
                            uint64_t pass = __ballot(!(u < ws)) & m64;
                            while (pass) {
                                const int j = __builtin_ctzll(pass);
                                pass &= pass - 1;
                                const int g = j >> 4;
                                const float lower =
                                    sc_lower(__int_as_float(__builtin_amdgcn_readlane(__float_as_int(u), j)), cosine);
                                float wtg = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(wt), j));
                                if (!(lower <= wtg)) continue;
                                const uint64_t key = ((uint64_t)wvg_ord_f32(lower) << 32) |
                                                     (uint32_t)(slot0 + 16u * (uint32_t)nr + (uint32_t)(j & 15));
                                if (!(key < readlane64(v, 16 * g + SCREEN_M - 1))) continue;
                                const bool inrow = (lane >> 4) == g;
                                const int pos = __popcll(__ballot(inrow && v < key));
                                const uint64_t sh = row_shr1_64(v);
                                v = inrow ? (li > pos ? sh : (li == pos ? key : v)) : v;
                                const uint64_t nk = readlane64(v, 16 * g + K - 1);
                                const uint64_t nm = readlane64(v, 16 * g + SCREEN_M - 1);
                                const float emg = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(em), j));
                                if (nk != WVG_KEY_NONE) wtg = fminf(wtg, sc_tau_k(key_lower(nk), emg, cosine));
                                if (nm != WVG_KEY_NONE) wtg = fminf(wtg, key_lower(nm));
                                const float wsg = sc_sigma(wtg, cosine);
                                wt = inrow ? wtg : wt;
                                ws = inrow ? wsg : ws;
                                pass &= ~(0xFFFFull << (16 * g)) | __ballot(!(u < ws));
                            }
                        }
                        const uint2 o2 = make_uint2((uint32_t)v, (uint32_t)(v >> 32));
                        asm volatile("ds_write_b64 %0, %1" ::"v"(la), "v"(o2) : "memory");
                        if (li == 0)
                            asm volatile("ds_write_b32 %0, %1\n\t"
                                         "ds_write_b32 %0, %2 offset:256" ::"v"(ta), "v"(wt), "v"(ws)
                                         : "memory");
                        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                    });
                }
            } else if constexpr ((DIAG & 8) != 0) {
                // diagnostic (DIAG 10): the stage loop alone, the accumulators consumed by one sum
                float x = 0.f;
#pragma unroll
                for (int nr = 0; nr < 16; nr++) x += agpr_read(acc[nr][0]);
                if (x == 0x1p-120f) a.partials[0] = 0;
            }
#pragma unroll
            for (int nr = 0; nr < 16; nr++) acc[nr] = (floatx4){0.f, 0.f, 0.f, 0.f};
            read_q(I0{}, I0{}, bq0, rbase);
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int ql = 0; ql < 16; ql++) {
        const uint32_t q = q0 + (uint32_t)(16 * w + ql);
        if (q >= a.nq) break;
        const uint64_t x = lane < M ? lists[((size_t)w * 16 + ql) * M + lane] : WVG_KEY_NONE;
        uint64_t *out = a.partials + ((size_t)q * a.nrr + rr) * M;
        if (lane < M) out[lane] = x;
        if (lane == K - 1 && x != WVG_KEY_NONE) {
            const float t = sc_tau_k(key_lower(x), cem[16 * w + ql], cosine);
            atomicMin(a.gbound + q, wvg_ord_f32(t));
        }
    }
}

#endif  // WVG_TOOLS

// ---------------------------------------------------------------------------
// Collect, per query.  Every range list holds its range's SCREEN_M smallest
// lower bounds, so their union holds the global k smallest: tau* = the k-th
// smallest lower of the union + 2 Emax is a valid bound (k rows at or below
// it) and the tightest the lists give -- far below the per-range bounds the
// screen published.  Entries with lower <= tau* become the rescore
// candidates (KEY_NONE elsewhere); a range list that is full with its last
// entry <= tau* may have dropped a row below tau*: the query is flagged for
// the exact rescan.  The k-th smallest is a 4-pass radix select (8-bit
// digits) over the entries' ordered lower bounds in LDS.
constexpr uint32_t SC_COLLECT_MAX = 8192;  // nrr * SCREEN_M (screen_row_ranges caps nrr at 512)

// The k-th smallest (k >= 1) of the ordered values hv[0, n) in LDS, of which
// at least k are not 0xFFFFFFFF: a 4-pass radix select over 8-bit digits.
// Block-wide (every thread calls it); every thread gets the value.
__device__ uint32_t block_kth_ordered(const uint32_t *hv, uint32_t n, uint32_t k, uint32_t *hist, uint32_t &sh_prefix,
                                      uint32_t &sh_need)
{
    if (threadIdx.x == 0) {
        sh_prefix = 0;
        sh_need = k;
    }
    __syncthreads();
    for (int shift = 24; shift >= 0; shift -= 8) {
        for (uint32_t i = threadIdx.x; i < 256; i += blockDim.x) hist[i] = 0;
        __syncthreads();
        const uint32_t hi_mask = shift == 24 ? 0u : (0xFFFFFFFFu << (shift + 8));
        const uint32_t pre = sh_prefix;
        for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
            const uint32_t v = hv[i];
            if (v != 0xFFFFFFFFu && (v & hi_mask) == (pre & hi_mask)) atomicAdd(&hist[(v >> shift) & 255u], 1u);
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            uint32_t need = sh_need, cum = 0, dg = 255;
            for (uint32_t d = 0; d < 256; d++) {
                if (cum + hist[d] >= need) {
                    dg = d;
                    break;
                }
                cum += hist[d];
            }
            sh_need = need - cum;
            sh_prefix = pre | (dg << shift);
        }
        __syncthreads();
    }
    return sh_prefix;
}

// seed (cand == nullptr): the same tau* over the lists of the first nrr_use
// ranges only, folded into gbound (atomicMin) -- the bound the later ranges
// of a split screen start from (without exact seeds; launch_seed_exact's
// k-th exact distance drops that bound's error term, about one Emax).
// Final (cand != nullptr): candidates within min(tau*, gbound).
__global__ __launch_bounds__(256) void screen_collect_kernel(const uint64_t *partials, uint32_t nrr, uint32_t nrr_use,
                                                             uint32_t k, const float *emax, int cosine, uint64_t *cand,
                                                             uint32_t *flist, uint32_t *nflag, uint32_t *gbound)
{
    __shared__ uint32_t hv[SC_COLLECT_MAX];
    __shared__ uint32_t hist[256];
    __shared__ uint32_t sh_prefix, sh_need, sh_total;
    __shared__ int ovf;
    const uint32_t q = blockIdx.x, n = nrr_use * SCREEN_M;
    const uint64_t *src = partials + (size_t)q * nrr * SCREEN_M;
    uint64_t *dst = cand + (size_t)q * n;
    if (threadIdx.x == 0) {
        ovf = 0;
        sh_total = 0;
    }
    __syncthreads();
    uint32_t live = 0;
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
        const uint64_t e = src[i];
        hv[i] = (uint32_t)(e >> 32);  // KEY_NONE -> 0xFFFFFFFF, above every real ordered distance
        live += e != WVG_KEY_NONE;
    }
    atomicAdd(&sh_total, live);
    __syncthreads();
    float t = __builtin_inff();
    if (sh_total >= k) t = sc_tau_k(wvg_unord_f32(block_kth_ordered(hv, n, k, hist, sh_prefix, sh_need)), emax[q], cosine);
    // the candidates: gbound may hold a tighter valid bound than tau* (an exact seed)
    const uint32_t gb = gbound[q];
    if (cand && gb != 0xFFFFFFFFu) t = fminf(t, wvg_unord_f32(gb));
    if (!cand) {
        if (threadIdx.x == 0 && t < __builtin_inff()) atomicMin(gbound + q, wvg_ord_f32(t));
        return;
    }
    __syncthreads();
    if (threadIdx.x == 0) sh_total = 0;
    __syncthreads();
    // the kept keys are packed at the front of the query's row (the rescore's
    // waves then run full; the merge reads an unordered key set), the rest is
    // KEY_NONE
    const uint32_t lane = threadIdx.x & 63;
    for (uint32_t i0 = 0; i0 < n; i0 += blockDim.x) {
        const uint32_t i = i0 + threadIdx.x;
        const uint64_t e = i < n ? src[i] : WVG_KEY_NONE;
        const bool keep = e != WVG_KEY_NONE && key_lower(e) <= t;
        if (keep && (i % SCREEN_M) == SCREEN_M - 1) ovf = 1;  // full list, last entry within tau*
        const uint64_t bal = __ballot(keep);
        uint32_t base = 0;
        if (lane == 0 && bal) base = atomicAdd(&sh_total, (uint32_t)__popcll(bal));
        base = __shfl(base, 0);
        if (keep) dst[base + __popcll(bal & ((1ull << lane) - 1ull))] = e;
    }
    __syncthreads();
    for (uint32_t i = sh_total + threadIdx.x; i < n; i += blockDim.x) dst[i] = WVG_KEY_NONE;
    if (threadIdx.x == 0 && ovf) flist[atomicAdd(nflag, 1u)] = q;
}


__global__ __launch_bounds__(256) void screen_pilot_list_kernel(uint32_t *flist, uint32_t nq, uint32_t *nflag)
{
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i < nq) flist[i] = i;
    if (i == 0) *nflag = nq;
}

// gbound[q] = the ordered k-th exact distance of the pilot (when it found k rows)
__global__ __launch_bounds__(256) void screen_pilot_seed_kernel(const float *dists, const uint32_t *counts, uint32_t nq,
                                                               uint32_t k, uint32_t *gbound)
{
    const uint32_t q = blockIdx.x * 256 + threadIdx.x;
    if (q >= nq || counts[q] < k) return;
    const float t = dists[(size_t)q * k + k - 1];
    if (t < __builtin_inff()) atomicMin(gbound + q, wvg_ord_f32(t));
}

// Whether K3c applies (the bound needs dim % 32 == 0 only for the fragment
// layout; k <= SCREEN_M for the list to hold the k-th key).
bool screen_supported(uint32_t dim, int metric, uint32_t k)
{
    return dim % 32 == 0 && dim > 0 && k > 0 && k <= (uint32_t)SCREEN_M &&
           (metric == WVG_M_DOT || metric == WVG_M_COSINE);
}

#ifdef WVG_TOOLS
// tools build: the K3c counters summed over every launch since the last reset
void screen_counters(uint64_t out[4], bool reset)
{
    unsigned long long v[4] = {0, 0, 0, 0};
    (void)hipDeviceSynchronize();
    (void)hipMemcpyFromSymbol(v, HIP_SYMBOL(g_screen_ctr), sizeof(v));
    for (int i = 0; i < 4; i++) out[i] = v[i];
    if (reset) {
        const unsigned long long z[4] = {0, 0, 0, 0};
        (void)hipMemcpyToSymbol(HIP_SYMBOL(g_screen_ctr), z, sizeof(z));
    }
}
#endif

uint32_t screen_row_ranges(uint32_t nq, uint64_t ntiles, int num_cus)
{
    const uint32_t nqb = (nq + SC_BQ - 1) / SC_BQ;
    const uint64_t nblk = (ntiles + 3) / 4;
    // ranges of ~128 row blocks dispatched range-major (the nqb workgroups of a
    // range start together on one XCD and share its L2 for the row fragments),
    // at least one workgroup per CU
    uint64_t want = std::max<uint64_t>(((uint64_t)num_cus + nqb - 1) / nqb, (nblk + 127) / 128);
#ifdef WVG_TOOLS
    if (tuning().screen_range_blocks > 0)
        want = std::max<uint64_t>(want, (nblk + tuning().screen_range_blocks - 1) / tuning().screen_range_blocks);
#endif
    want = std::min<uint64_t>((want + 7) / 8 * 8, SC_COLLECT_MAX / SCREEN_M);
    // whole rounds of workgroups (the screens run one workgroup per CU): nrr * nqb a multiple of
    // num_cus where that adds at most 1/8 more ranges -- 10M rows, 1024 queries: 312 ranges left
    // the last phase's 3968 workgroups at 15.5 per CU, so its last round ran half empty
    if (tuning().screen_round && num_cus > 0) {
        const uint64_t step = std::lcm<uint64_t>(8, (uint64_t)num_cus / std::gcd<uint64_t>((uint64_t)num_cus, nqb));
        const uint64_t w2 = (want + step - 1) / step * step;
        if (w2 <= SC_COLLECT_MAX / SCREEN_M && w2 * 8 <= want * 9) want = w2;
    }
    if (want > nblk) want = nblk;
    if (want < 1) want = 1;
    return (uint32_t)want;
}

hipError_t launch_screen(const ScreenLaunch &L, hipStream_t s)
{
    const bool i8 = L.i8 && screen_i8_supported(L.dim);
    const uint32_t kbn = i8 ? L.dim / 64 : screen_kblocks(L.dim);  // (K3i: 64-deep int8 K blocks)
    const uint32_t nq16 = (L.nq + 15) / 16, nq_pad = (L.nq + SC_BQ - 1) / SC_BQ * SC_BQ;
    uint32_t nqb = nq_pad / SC_BQ;  // (K3g, tools: 64-query blocks)
    hipError_t e;
    (void)nq16;
    if (i8) {
        // K3i: per-query scale and bound constants first, then the int8 fragments at that scale
        hipLaunchKernelGGL(screen_qconst_i8_kernel, dim3(nq_pad / 4), dim3(256), 0, s, L.queries, L.nq, L.qpitch,
                           L.dim, nq_pad, L.cosine, L.nmax, reinterpret_cast<const float *>(L.nmax + 2), L.k1, L.k2,
                           L.kb, L.css, L.qinv, L.emax);
        hipLaunchKernelGGL(screen_qfrag_i8_kernel, dim3((unsigned)(((uint64_t)nq_pad / 16 * kbn * 64 + 255) / 256)),
                           dim3(256), 0, s, L.queries, L.nq, L.qpitch, L.dim, kbn, nq_pad / 16, L.qinv,
                           reinterpret_cast<uint4 *>(L.qfrag));
    } else {
        // query fragments for every 16-query group of the padded batch
        hipLaunchKernelGGL(screen_qfrag_kernel, dim3((unsigned)(((uint64_t)nq_pad / 16 * kbn * 64 + 255) / 256)),
                           dim3(256), 0, s, L.queries, L.nq, L.qpitch, L.dim, kbn, nq_pad / 16,
                           reinterpret_cast<uint4 *>(L.qfrag));
        hipLaunchKernelGGL(screen_qconst_kernel, dim3(nq_pad / 4), dim3(256), 0, s, L.queries, L.nq, L.qpitch, L.dim,
                           nq_pad, L.cosine, L.nmax, L.k1, L.k2, L.emax);
    }
    if ((e = hipMemsetAsync(L.gbound, 0xFF, (size_t)L.nq * 4, s)) != hipSuccess) return e;
    // profiling: one event pair spans every phase and the seeds between them (taken
    // before the pilot, whose K3b launch would otherwise bind them)
    const LaunchEvents ev = armed_events();
    armed_events() = LaunchEvents{};
    const uint64_t pilot_tiles = (uint64_t)std::max(tuning().screen_pilot, 0);
    const uint64_t pilot_gemm_tiles = (uint64_t)std::max(L.i8 ? tuning().screen_pilot_gemm_i8 : tuning().screen_pilot_gemm, 0);
    // Screen pilot: short ranges of the screen itself over the first sp_tiles tiles
    // (one workgroup per CU), lists into the pilot scratch ([nq][sp_rr][SCREEN_M]),
    // then one exact seed from them (below, once the kernel is chosen)
    const uint64_t sp_tiles = std::min<uint64_t>((uint64_t)std::max(tuning().screen_pilot_screen, 0),
                                                 L.tile_end - L.tile_begin);
    uint32_t sp_rr = 0;
    if (sp_tiles > 0 && L.pilot_part && L.data && L.pilot_part_lists > 0) {
        const uint64_t nb = (sp_tiles + 3) / 4;
        uint64_t want = std::min<uint64_t>(((uint64_t)L.num_cus / nqb + 7) / 8 * 8, nb);
        want = std::min<uint64_t>(want, (uint64_t)L.pilot_part_lists * L.k / SCREEN_M);  // the scratch's capacity
        sp_rr = want >= 8 ? (uint32_t)(want / 8 * 8) : 0;
    }
    uint32_t pilot_rr = 0;  // K3b pilot: its row ranges (0: the K1 pilot)
    if (sp_rr > 0) {
        // (the screen pilot replaces the K3b / K1 pilots)
    } else if (L.pilot && pilot_gemm_tiles > 0) {
        const uint64_t nt = std::min<uint64_t>(L.pilot->tile_end - L.pilot->tile_begin, pilot_gemm_tiles);
        pilot_rr = nt ? gemm_row_ranges(L.nq, nt, L.num_cus, L.dim, L.k) : 0;
        if (pilot_rr > L.pilot_part_lists) pilot_rr = 0;
    }
    if (pilot_rr > 0) {
        // Pilot (K3b): the exact top-k of every query over the first pilot_gemm_tiles
        // tiles (16k rows), exact fp32 MFMA -- per row ~16x cheaper than K1's
        // per-query scans, so 16x the rows of the K1 pilot at about its cost; its
        // k-th distance bounds the final k-th and seeds gbound before the first phase
        ScanArgs f = *L.pilot;
        f.cosched = 0;
        f.reverse = 0;
        f.tile_end = std::min<uint64_t>(f.tile_end, f.tile_begin + pilot_gemm_tiles);
        if ((e = launch_gemm_topk(f, pilot_rr, L.pilot_part, nullptr, nullptr, L.num_cus, s)) != hipSuccess) return e;
        if ((e = launch_merge_lists(L.pilot_part, L.nq, pilot_rr, L.k, L.k, 0, L.pilot_ids, L.pilot_dists,
                                    L.pilot_counts, s)) != hipSuccess)
            return e;
        hipLaunchKernelGGL(screen_pilot_seed_kernel, dim3((L.nq + 255) / 256), dim3(256), 0, s, L.pilot_dists,
                           L.pilot_counts, L.nq, L.k, L.gbound);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    } else if (sp_rr == 0 && L.pilot && pilot_tiles > 0) {
        // Pilot: every query's exact top-k (K1, AVX2-order distances) over the
        // range's first 16 tiles (1024 rows); its k-th distance bounds the final k-th
        // (k real rows lie at or below it), so it seeds gbound before the
        // first phase, whose lists otherwise start empty with no threshold
        // and take an insertion for nearly every row of their first blocks.
        ScanArgs f = *L.pilot;
        f.nq = 1;
        f.cosched = 0;
        f.reverse = 0;
        f.tile_end = std::min<uint64_t>(f.tile_end, f.tile_begin + pilot_tiles);
        hipLaunchKernelGGL(screen_pilot_list_kernel, dim3((L.nq + 255) / 256), dim3(256), 0, s, L.flist, L.nq, L.nflag);
        if ((e = hipGetLastError()) != hipSuccess) return e;
        if ((e = launch_scan_f32_qlist(f, L.pilot_part, (int)L.pilot_groups, L.flist, L.nflag, L.nq, s)) !=
            hipSuccess)
            return e;
        if ((e = launch_merge_lists_qlist(L.pilot_part, L.nq, L.pilot_groups, L.k, L.k, 0, L.pilot_ids, L.pilot_dists,
                                          L.pilot_counts, L.flist, L.nflag, s)) != hipSuccess)
            return e;
        hipLaunchKernelGGL(screen_pilot_seed_kernel, dim3((L.nq + 255) / 256), dim3(256), 0, s, L.pilot_dists,
                           L.pilot_counts, L.nq, L.k, L.gbound);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    if ((e = hipMemsetAsync(L.nflag, 0, 4, s)) != hipSuccess) return e;
    ScreenArgs a{};
    a.shadow = reinterpret_cast<const uint4 *>(L.shadow);
    a.norms = L.norms;
    a.valid = L.valid;
    a.allow = L.allow;
    a.allow_words = L.allow_words;
    a.allow_t0 = L.allow_t0;
    a.tile_begin = L.tile_begin;
    a.tile_end = L.tile_end;
    a.kbn = kbn;
    a.qfrag = reinterpret_cast<const uint4 *>(L.qfrag);
    a.k1 = L.k1;
    a.k2 = L.k2;
    a.emax = L.emax;
    a.nq = L.nq;
    a.k = L.k;
    a.nqb = nqb;
    a.nrr = L.nrr;
    a.cosine = L.cosine;
#ifdef WVG_TOOLS
    a.diag = tuning().screen_diag;
#endif
    a.gbound = L.gbound;
    a.partials = L.partials;
    a.errs = L.errs;
    a.kb = L.kb;
    a.css = L.css;
    static bool attr = [] {
        return hipFuncSetAttribute(reinterpret_cast<const void *>(&screen_kernel),
                                   hipFuncAttributeMaxDynamicSharedMemorySize, SC_LDS) == hipSuccess &&
               hipFuncSetAttribute(reinterpret_cast<const void *>(&screen_ar_kernel<16>),
                                   hipFuncAttributeMaxDynamicSharedMemorySize, SD_LDS) == hipSuccess &&
               hipFuncSetAttribute(reinterpret_cast<const void *>(&screen_ar_kernel<24>),
                                   hipFuncAttributeMaxDynamicSharedMemorySize, SD_LDS) == hipSuccess &&
               hipFuncSetAttribute(reinterpret_cast<const void *>(&screen_ar_kernel<8, 0, true>),
                                   hipFuncAttributeMaxDynamicSharedMemorySize, si_lds(si_nbuf(8))) == hipSuccess &&
               hipFuncSetAttribute(reinterpret_cast<const void *>(&screen_ar_kernel<12, 0, true>),
                                   hipFuncAttributeMaxDynamicSharedMemorySize, si_lds(si_nbuf(12))) == hipSuccess &&
               hipFuncSetAttribute(reinterpret_cast<const void *>(&screen_ar_kernel<16, 0, true>),
                                   hipFuncAttributeMaxDynamicSharedMemorySize, si_lds(si_nbuf(16))) == hipSuccess &&
               hipFuncSetAttribute(reinterpret_cast<const void *>(&screen_i8_kernel<8>),
                                   hipFuncAttributeMaxDynamicSharedMemorySize, SJ_LDS) == hipSuccess &&
               hipFuncSetAttribute(reinterpret_cast<const void *>(&screen_i8_kernel<12>),
                                   hipFuncAttributeMaxDynamicSharedMemorySize, SJ_LDS) == hipSuccess;
    }();
    (void)attr;
    // K3i on an int8 shadow; else K3d (queries resident in registers) where its template applies, else K3c
    void (*kern)(ScreenArgs) = kbn == 24 ? &screen_ar_kernel<24> : kbn == 16 ? &screen_ar_kernel<16> : nullptr;
    // (d = 512 / 768: the 2 x 2-wave layout; d = 1024: 64 resident queries would not fit the
    // registers, K3d's layout)
    bool i8_22 = i8 && kbn <= 12;
#ifdef WVG_TOOLS
    if (tuning().screen_variant == 5) i8_22 = false;  // A/B: K3i on K3d's 1 x 4 layout
#endif
    if (i8)
        kern = i8_22 ? (kbn == 8 ? &screen_i8_kernel<8> : &screen_i8_kernel<12>)
                     : (kbn == 8 ? &screen_ar_kernel<8, 0, true>
                                 : (kbn == 12 ? &screen_ar_kernel<12, 0, true> : &screen_ar_kernel<16, 0, true>));
#ifdef WVG_TOOLS
    if (i8_22 && kbn == 12 && (tuning().screen_diag == 4 || tuning().screen_diag == 10 || tuning().screen_diag == 16)) {
        kern = tuning().screen_diag == 4    ? &screen_i8_kernel<12, 4>
               : tuning().screen_diag == 10 ? &screen_i8_kernel<12, 10>
                                            : &screen_i8_kernel<12, 16>;  // K3i diagnostics
        (void)hipFuncSetAttribute(reinterpret_cast<const void *>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                                  SJ_LDS);
    }
#endif
    bool k3f = false;
#ifdef WVG_TOOLS
    bool k3g = false;
    if (i8 && tuning().screen_diag == 10 && kbn == 12) {  // K3i's stage loop alone (A/B)
        kern = &screen_ar_kernel<12, 10, true>;
        (void)hipFuncSetAttribute(reinterpret_cast<const void *>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                                  si_lds(si_nbuf(12)));
    }
    if (!i8) {
    if (tuning().screen_variant == 2 && kern)  // K3e (32x32x16 MFMAs)
        kern = kbn == 24 ? &screen_ar32_kernel<24> : &screen_ar32_kernel<16>;
    if (tuning().screen_variant == 3 && kern)  // K3f (two waves per SIMD)
        kern = kbn == 24 ? &screen_ar16_kernel<24> : &screen_ar16_kernel<16>;
    k3g = tuning().screen_variant == 4 && kern;  // K3g (two 4-wave workgroups per CU)
    if (k3g) kern = kbn == 24 ? &screen_ar16x2_kernel<24> : &screen_ar16x2_kernel<16>;
    if (tuning().screen_variant >= 2 && kern)
        (void)hipFuncSetAttribute(reinterpret_cast<const void *>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                                  k3g ? SG_LDS : SD_LDS);
    if (kbn == 24) {  // K3d diagnostics: separately compiled instantiations
        switch (tuning().screen_diag) {
        case 1: kern = &screen_ar_kernel<24, 1>; break;
        case 2: kern = &screen_ar_kernel<24, 2>; break;
        case 4: kern = &screen_ar_kernel<24, 4>; break;
        case 16: kern = &screen_ar_kernel<24, 16>; break;
        case 10: kern = &screen_ar_kernel<24, 10>; break;
        case 42: kern = &screen_ar_kernel<24, 42>; break;    // 10 without the norm / tile-word loads
        case 106: kern = &screen_ar_kernel<24, 106>; break;  // 42 without the per-unit s_barrier
        case 138: kern = &screen_ar_kernel<24, 138>; break;  // 10 without any stage load
        case 202: kern = &screen_ar_kernel<24, 202>; break;  // 138 without the s_barrier
        case 32: kern = &screen_ar_kernel<24, 32>; break;    // the product without the norm / tile-word loads
        case 256: kern = &screen_ar_kernel<24, 256>; break;  // round 3's norms / words with every unit
        case 266: kern = &screen_ar_kernel<24, 266>; break;  // 10 with round 3's per-unit norms / words
        case 1024: kern = &screen_ar_kernel<24, 1024>; break;  // one barrier per two K blocks
        case 2048: kern = &screen_ar_kernel<24, 2048>; break;  // the per-element (tight) fast check
        case 2064: kern = &screen_ar_kernel<24, 2064>; break;  // 2048 with the counters (16)
        case 1034: kern = &screen_ar_kernel<24, 1034>; break;  // 10 with one barrier per two K blocks
        default: break;
        }
        if (tuning().screen_variant == 2 && tuning().screen_diag == 10) kern = &screen_ar32_kernel<24, 10>;
        if (tuning().screen_variant == 3 && tuning().screen_diag == 10) kern = &screen_ar16_kernel<24, 10>;
        if (kern != &screen_ar_kernel<24> && kern != &screen_ar32_kernel<24> && kern != &screen_ar16_kernel<24>)
            (void)hipFuncSetAttribute(reinterpret_cast<const void *>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                                      SD_LDS);
    }
    if (tuning().screen_variant == 1) kern = nullptr;
    k3f = kern == &screen_ar16_kernel<24> || kern == &screen_ar16_kernel<16> || kern == &screen_ar16_kernel<24, 10>;
    }  // (!i8)
#endif
#ifdef WVG_TOOLS
    if (k3g) {  // 64-query workgroups: twice the query blocks
        nqb = nq_pad / SG_BQ;
        a.nqb = nqb;
    }
    const uint32_t lds = i8_22 ? SJ_LDS : i8 ? si_lds(si_nbuf(kbn)) : k3g ? SG_LDS : kern ? SD_LDS : SC_LDS;
#else
    const uint32_t lds = i8_22 ? SJ_LDS : i8 ? si_lds(si_nbuf(kbn)) : kern ? SD_LDS : SC_LDS;
#endif
    const uint32_t threads = k3f ? SF_WAVES * 64 : kern ? SD_WAVES * 64 : SC_WAVES * 64;
    if (!kern) kern = &screen_kernel;
    // Phased screen: the first r1 ranges (one workgroup per CU) run alone; their
    // lists' joint tau* (k-th smallest lower bound over ~10 % of the rows,
    // + 2 Emax) seeds the next phase's thresholds, the next r2 - r1 ranges
    // (~30 %) run, and the joint tau* over the first r2 seeds the rest.
    // Without it a range starts from the k-th bound of single finished
    // ranges (rows in the top-k of 1 % of the corpus), and most row blocks
    // took the exact per-element path with list insertions.
    if (sp_rr > 0) {
        // Screen pilot (round 5): the bf16 screen over the first sp_tiles tiles in sp_rr
        // short ranges (a few row blocks each, every CU busy), its lists into the pilot
        // scratch, then the exact seed over them: the k smallest lower bounds rescored
        // exactly, their k-th distance into gbound -- k real rows at or below it, so a
        // valid bound, as the K3b pilot's exact k-th over its rows (which cost ~0.76 ms
        // per 1024-query batch: K3b's start-up on a short range)
        ScreenArgs f = a;
        f.rsplit[0] = 0;
        f.tile_end = L.tile_begin + sp_tiles;
        f.nrr = sp_rr;
        f.rr0 = 0;
        f.nrr_l = sp_rr;
        f.partials = L.pilot_part;
        hipLaunchKernelGGL(kern, dim3(nqb * sp_rr), dim3(threads), lds, s, f);
        if ((e = hipGetLastError()) != hipSuccess) return e;
        if ((e = launch_seed_exact(L.metric, L.queries, L.qpitch, L.data, L.dim, L.nchunks, L.pilot_part,
                                   sp_rr * SCREEN_M, SCREEN_M, sp_rr, L.nq, L.k, L.gbound, s)) != hipSuccess)
            return e;
    }
    uint32_t bounds[12] = {0}, nph = 0;
    bounds[nph++] = 0;
    const int split = tuning().screen_split;
    if (L.nrr % 8 == 0) {
        const uint32_t r1 = std::max<uint32_t>(8, ((uint32_t)L.num_cus / nqb + 7) / 8 * 8);
        if (r1 <= L.nrr / 4) {
            bounds[nph++] = r1;
            if (split == 3) {  // doubling phases (tools A/B)
                for (uint32_t b = 2 * r1; b <= L.nrr / 2 && nph < 10; b *= 2) bounds[nph++] = b;
            } else if (4 * r1 <= L.nrr / 2) {
                bounds[nph++] = 4 * r1;
            }
        }
    }
    if (split == 0) nph = 1;
    if (split == 2 && nph > 2) nph = 2;
    bounds[nph] = L.nrr;
    // K3i warm-up (round 6): the first phase's ranges cover only screen_warm row blocks each
    // (8k rows at 32), so few rows are screened against the pilot's loose bound before the
    // first exact seed -- the survivors of that phase were most of the screen's list
    // insertions (tools counters: ~1.1k of ~1.2k per query at 10M x 768)
    const uint64_t nblk_all = (L.tile_end - L.tile_begin + 3) / 4;
    if (i8 && nph >= 2 && tuning().screen_warm > 0 && (uint64_t)bounds[1] * tuning().screen_warm * 4 <= nblk_all) {
        a.rsplit[0] = a.rsplit[1] = bounds[1];
        a.bsplit[0] = a.bsplit[1] = (uint64_t)bounds[1] * (uint64_t)tuning().screen_warm;
        // the second phase's ranges: screen_warm2 row blocks each
        const uint64_t b2 = nph >= 3 ? a.bsplit[0] + (uint64_t)(bounds[2] - bounds[1]) * (uint64_t)tuning().screen_warm2 : 0;
        if (nph >= 3 && tuning().screen_warm2 > 0 && bounds[2] < L.nrr && b2 * 2 <= nblk_all) {
            a.rsplit[1] = bounds[2];
            a.bsplit[1] = b2;
        }
    }
    // seeds between phases: the exact k-th over the earlier ranges' candidates
    // (rescored with the final rescore's distances) where the rows are at hand
    const bool rows = L.data != nullptr;
    const bool seed_exact = rows && (tuning().screen_seed & 1) != 0, seed_final = rows && (tuning().screen_seed & 2) != 0;
    // an exact seed over the lists of ranges [0, nr_use)
    auto exact_seed = [&](uint32_t nr_use) -> hipError_t {
        return launch_seed_exact(L.metric, L.queries, L.qpitch, L.data, L.dim, L.nchunks, L.partials,
                                 L.nrr * SCREEN_M, SCREEN_M, nr_use, L.nq, L.k, L.gbound, s);
    };
    for (uint32_t ph = 0; ph < nph; ph++) {
        a.rr0 = bounds[ph];
        a.nrr_l = bounds[ph + 1] - bounds[ph];
        const hipEvent_t e0 = ph == 0 ? ev.start : nullptr, e1 = ph + 1 == nph ? ev.stop : nullptr;
        if (e0 || e1)
            hipExtLaunchKernelGGL(kern, dim3(nqb * a.nrr_l), dim3(threads), lds, s, e0, e1, 0u, a);
        else
            hipLaunchKernelGGL(kern, dim3(nqb * a.nrr_l), dim3(threads), lds, s, a);
        if ((e = hipGetLastError()) != hipSuccess) return e;
        if (ph + 1 < nph) {
            if (seed_exact) {
                if ((e = exact_seed(bounds[ph + 1])) != hipSuccess) return e;
            } else {
                hipLaunchKernelGGL(screen_collect_kernel, dim3(L.nq), dim3(256), 0, s, L.partials, L.nrr,
                                   bounds[ph + 1], L.k, L.emax, L.cosine, (uint64_t *)nullptr, L.flist, L.nflag,
                                   L.gbound);
            }
            if ((e = hipGetLastError()) != hipSuccess) return e;
        }
    }
    if ((e = hipGetLastError()) != hipSuccess) return e;
    // the final candidates: lower <= min(tau*, gbound); with the exact seed over every
    // range, gbound ~ the k-th exact distance, about one Emax below tau* -- a third of
    // the rows to rescore on 10M x 768 cosine
    if (seed_final && (e = exact_seed(L.nrr)) != hipSuccess) return e;
    hipLaunchKernelGGL(screen_collect_kernel, dim3(L.nq), dim3(256), 0, s, L.partials, L.nrr, L.nrr, L.k, L.emax,
                       L.cosine, L.cand, L.flist, L.nflag, L.gbound);
    return hipGetLastError();
}

}  // namespace wvg
