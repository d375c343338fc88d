// wvg_rowdist.hpp -- one lane computes Provider.SingleDist(query, row) for its
// own row, in exactly the reference's AVX2 reduction order, so the fp32 result
// is bit-identical to Weaviate's CPU distancer on non-AMX amd64 hosts
// (dispatch D/l2_amd64.go:19-25, D/dot_product_amd64.go:19-25).
//
// Order restated (D/c/l2_avx256_amd64.c:14-107, D/c/dot_avx256_amd64.c:14-104):
//   n < 8      : sequential scalar loop into `sum` (L2 unfused mul+add,
//                dot fused vfmadd231ss per the shipped asm)
//   32-blocks  : acc[j][l] = fma(.., acc[j][l]) for element 32b + 8j + l
//   8-blocks   : acc[0][l] for element 32nb + 8t + l
//   tail (<8)  : scalar into `sum`
//   reduce     : s_l = (acc3+acc2)+(acc1+acc0); ((s0+s1)+(s2+s3)) + ((s4+s5)+(s6+s7)); sum += .
//
// The compilation unit must be built with -ffp-contract=off: every fused
// operation below is an explicit __builtin_fmaf.
#pragma once

#include "wvg_common.hpp"

namespace wvg {

template <int METRIC>
__device__ __forceinline__ void acc_update(float &acc, float q, float x)
{
    if constexpr (METRIC == WVG_M_L2) {
        float diff = q - x;
        acc = __builtin_fmaf(diff, diff, acc);
    } else {
        acc = __builtin_fmaf(q, x, acc);
    }
}

template <int METRIC>
__device__ __forceinline__ void scalar_update(float &sum, float q, float x)
{
    if constexpr (METRIC == WVG_M_L2) {
        float diff = q - x;
        float sq = diff * diff;
        sum = sum + sq;
    } else {
        sum = __builtin_fmaf(q, x, sum);
    }
}

__device__ __forceinline__ float avx256_reduce(const float (&acc)[4][8], float sum)
{
    float s[8];
#pragma unroll
    for (int l = 0; l < 8; l++) {
        float a01 = acc[1][l] + acc[0][l];
        float a23 = acc[3][l] + acc[2][l];
        s[l] = a23 + a01;
    }
    float lo = (s[0] + s[1]) + (s[2] + s[3]);
    float hi = (s[4] + s[5]) + (s[6] + s[7]);
    return sum + (lo + hi);
}

typedef float f4v __attribute__((ext_vector_type(4)));

// Streaming 16-byte load.  NT: non-temporal -- for a corpus well past the
// 256 MiB Infinity Cache, read once per query (measured: 6.9 vs 6.2-6.4 TB/s
// over 3.2 GB, profiles/r02/pq_adc/mall_reuse_policies.jsonl); at or below
// ~800 MiB the default policy lets consecutive scans of the same rows
// find part of them there (1M x 128: 1150 vs 1197 us per 16 scans,
// profiles/r02/bench/load_policy_ab.jsonl).  The host picks (ScanArgs.plain).
template <bool NT = true>
__device__ __forceinline__ float4 ld_stream(const float4 *p)
{
    if constexpr (NT) {
        const f4v v = __builtin_nontemporal_load(reinterpret_cast<const f4v *>(p));
        return make_float4(v.x, v.y, v.z, v.w);
    } else {
        return *p;
    }
}

template <int METRIC>
__device__ __forceinline__ void chunk_update(float (&acc)[4][8], int cc, float4 q, float4 x)
{
    const int j = cc >> 1, l0 = (cc & 1) * 4;
    acc_update<METRIC>(acc[j][l0 + 0], q.x, x.x);
    acc_update<METRIC>(acc[j][l0 + 1], q.y, x.y);
    acc_update<METRIC>(acc[j][l0 + 2], q.z, x.z);
    acc_update<METRIC>(acc[j][l0 + 3], q.w, x.w);
}

// p: chunk 0 of this lane's row; consecutive chunks are CSTRIDE float4 apart
// (64 in the tiled corpus).  q: the query, 16-byte aligned, padded to 4.
template <int CSTRIDE>
__device__ __forceinline__ float elem_at(const float4 *__restrict__ p, int pos)
{
    const float *c = reinterpret_cast<const float *>(p + (size_t)(pos >> 2) * CSTRIDE);
    return c[pos & 3];
}

// Manhattan and Hamming: the two metrics whose sum is not an AVX2 chain set.
//  - Manhattan (D/manhattan.go:20-30): pure Go on every host (no SIMD kernel
//    exists): sum += float32(math.Abs(float64(a_i - b_i))) in element order.
//    The float64 round trip is exact, so it is |q - x| in fp32 added in order.
//  - Hamming (D/hamming_amd64.go:18-24 -> D/c/hamming_avx256_amd64.c:14-144;
//    hamming_512 counts the same elements the same way): an integer count
//    converted to float once.  n < 8: `a != b` per element (C's unordered !=,
//    a NaN counts); n >= 8: the first n & ~7 elements by _CMP_NEQ_OQ (ordered:
//    a NaN does NOT count), the rest by !=.  A count is order-free, so only
//    which comparison an element gets matters.
// Whole 16-byte chunks are read 8 at a time (loads in flight), the tail of a
// dimension that is not a multiple of 4 element by element.
__device__ __forceinline__ uint32_t neq_oq(float a, float b) { return (a < b) || (a > b) ? 1u : 0u; }
__device__ __forceinline__ uint32_t neq_uo(float a, float b) { return a != b ? 1u : 0u; }

template <int METRIC>
constexpr bool is_abs_or_neq = METRIC == WVG_M_MANHATTAN || METRIC == WVG_M_HAMMING;

template <int METRIC, int CSTRIDE, bool NT = false>
__device__ __forceinline__ float row_abs_or_neq(const float4 *__restrict__ p, const float4 *__restrict__ q4, int n)
{
    static_assert(is_abs_or_neq<METRIC>, "manhattan / hamming only");
    const float *q = reinterpret_cast<const float *>(q4);
    float sum = 0.0f;
    uint32_t cnt = 0u;
    const int nord = METRIC == WVG_M_HAMMING && n >= 8 ? (n & ~7) : 0;  // elements under _CMP_NEQ_OQ
    auto upd = [&](int c, float4 qq, float4 x) {
        if constexpr (METRIC == WVG_M_MANHATTAN) {
            sum = sum + __builtin_fabsf(qq.x - x.x);
            sum = sum + __builtin_fabsf(qq.y - x.y);
            sum = sum + __builtin_fabsf(qq.z - x.z);
            sum = sum + __builtin_fabsf(qq.w - x.w);
        } else if (4 * c < nord) {  // nord is a multiple of 8: a chunk is wholly inside or outside
            cnt += neq_oq(qq.x, x.x) + neq_oq(qq.y, x.y) + neq_oq(qq.z, x.z) + neq_oq(qq.w, x.w);
        } else {
            cnt += neq_uo(qq.x, x.x) + neq_uo(qq.y, x.y) + neq_uo(qq.z, x.z) + neq_uo(qq.w, x.w);
        }
    };
    const int nc = n >> 2;
    int c = 0;
    for (; c + 8 <= nc; c += 8) {
        float4 xs[8];
#pragma unroll
        for (int cc = 0; cc < 8; cc++) xs[cc] = ld_stream<NT>(p + (size_t)(c + cc) * CSTRIDE);
#pragma unroll
        for (int cc = 0; cc < 8; cc++) upd(c + cc, q4[c + cc], xs[cc]);
    }
    for (; c < nc; c++) upd(c, q4[c], p[(size_t)c * CSTRIDE]);
    for (int i = nc * 4; i < n; i++) {
        const float x = elem_at<CSTRIDE>(p, i);
        if constexpr (METRIC == WVG_M_MANHATTAN)
            sum = sum + __builtin_fabsf(q[i] - x);
        else
            cnt += i < nord ? neq_oq(q[i], x) : neq_uo(q[i], x);
    }
    if constexpr (METRIC == WVG_M_HAMMING)
        return (float)cnt;
    else
        return sum;
}

template <int METRIC, int D, int CSTRIDE, bool NT = true>
__device__ __forceinline__ float row_dot_or_l2_fixed(const float4 *__restrict__ p,
                                                     const float4 *__restrict__ q)
{
    static_assert(D % 32 == 0 && D >= 32, "fixed path needs D % 32 == 0");
    if constexpr (is_abs_or_neq<METRIC>) {
        return row_abs_or_neq<METRIC, CSTRIDE, NT>(p, q, D);
    } else {
    float acc[4][8];
#pragma unroll
    for (int j = 0; j < 4; j++)
#pragma unroll
        for (int l = 0; l < 8; l++) acc[j][l] = 0.0f;
    constexpr int NB = D / 32;
    constexpr int UNROLL = NB <= 4 ? NB : 2;
#pragma unroll UNROLL
    for (int b = 0; b < NB; b++) {
        float4 xs[8];
#pragma unroll
        for (int cc = 0; cc < 8; cc++) xs[cc] = ld_stream<NT>(p + (size_t)(b * 8 + cc) * CSTRIDE);
#pragma unroll
        for (int cc = 0; cc < 8; cc++) chunk_update<METRIC>(acc, cc, q[b * 8 + cc], xs[cc]);
    }
    return avx256_reduce(acc, 0.0f);
    }
}

template <int METRIC, int CSTRIDE>
__device__ __forceinline__ float row_dot_or_l2_generic(const float4 *__restrict__ p,
                                                       const float4 *__restrict__ q4, int n)
{
    if constexpr (is_abs_or_neq<METRIC>) return row_abs_or_neq<METRIC, CSTRIDE>(p, q4, n);
    const float *q = reinterpret_cast<const float *>(q4);
    float sum = 0.0f;
    if (n < 8) {
        for (int i = 0; i < n; i++) scalar_update<METRIC>(sum, q[i], elem_at<CSTRIDE>(p, i));
        return sum;
    }
    float acc[4][8];
#pragma unroll
    for (int j = 0; j < 4; j++)
#pragma unroll
        for (int l = 0; l < 8; l++) acc[j][l] = 0.0f;
    const int nb = n >> 5;
    for (int b = 0; b < nb; b++) {
        float4 xs[8];
#pragma unroll
        for (int cc = 0; cc < 8; cc++) xs[cc] = p[(size_t)(b * 8 + cc) * CSTRIDE];
#pragma unroll
        for (int cc = 0; cc < 8; cc++) chunk_update<METRIC>(acc, cc, q4[b * 8 + cc], xs[cc]);
    }
    int pos = nb * 32;
    int rem = n - pos;
    while (rem >= 8) {
        const int c = pos >> 2;
        float4 x0 = p[(size_t)c * CSTRIDE], x1 = p[(size_t)(c + 1) * CSTRIDE];
        chunk_update<METRIC>(acc, 0, q4[c], x0);  // acc[0][0..3]
        chunk_update<METRIC>(acc, 1, q4[c + 1], x1);  // acc[0][4..7]
        pos += 8;
        rem -= 8;
    }
    while (rem) {
        scalar_update<METRIC>(sum, q[pos], elem_at<CSTRIDE>(p, pos));
        pos++;
        rem--;
    }
    return avx256_reduce(acc, sum);
}

// l2_512 / dot_512 (D/c/l2_avx512_amd64.c:14-178, D/c/dot_avx512_amd64.c),
// the kernels Weaviate dispatches on AMX + AVX-512 hosts (D/l2_amd64.go:19-25,
// D/dot_product_amd64.go:19-25; wvg_set_distance_order).  Below 128 elements
// they equal the AVX2 kernels.  Otherwise: 128 chains a5[j][l] (element
// 128b + 16j + l) over the whole 128-blocks, the tree ((a1+a0) + (a3+a2)) +
// ((a5+a4) + (a7+a6)) per lane, the low then the high 8 lanes added into
// acc[0], and the AVX2 loop continues on the rest with that acc[0].
template <int METRIC, int CSTRIDE>
__device__ __forceinline__ float row_dist_512(const float4 *__restrict__ p, const float4 *__restrict__ q4, int n)
{
    // Manhattan has no SIMD kernel; hamming_512 counts like hamming_256
    if (is_abs_or_neq<METRIC> || n < 128) return row_dot_or_l2_generic<METRIC, CSTRIDE>(p, q4, n);
    const float *q = reinterpret_cast<const float *>(q4);
    float a5[8][16];
#pragma unroll
    for (int j = 0; j < 8; j++)
#pragma unroll
        for (int l = 0; l < 16; l++) a5[j][l] = 0.0f;
    const int nb = n >> 7;
    for (int b = 0; b < nb; b++) {
#pragma unroll
        for (int j = 0; j < 8; j++) {
            float4 xs[4];
#pragma unroll
            for (int c = 0; c < 4; c++) xs[c] = p[(size_t)(b * 32 + j * 4 + c) * CSTRIDE];
#pragma unroll
            for (int c = 0; c < 4; c++) {
                const float4 qq = q4[b * 32 + j * 4 + c];
                acc_update<METRIC>(a5[j][4 * c + 0], qq.x, xs[c].x);
                acc_update<METRIC>(a5[j][4 * c + 1], qq.y, xs[c].y);
                acc_update<METRIC>(a5[j][4 * c + 2], qq.z, xs[c].z);
                acc_update<METRIC>(a5[j][4 * c + 3], qq.w, xs[c].w);
            }
        }
    }
    float acc[4][8];
#pragma unroll
    for (int j = 0; j < 4; j++)
#pragma unroll
        for (int l = 0; l < 8; l++) acc[j][l] = 0.0f;
    float r[16];
#pragma unroll
    for (int l = 0; l < 16; l++) {
        float x0 = a5[1][l] + a5[0][l];
        const float x2 = a5[3][l] + a5[2][l];
        float x4 = a5[5][l] + a5[4][l];
        const float x6 = a5[7][l] + a5[6][l];
        x0 = x2 + x0;
        x4 = x6 + x4;
        r[l] = x4 + x0;
    }
#pragma unroll
    for (int l = 0; l < 8; l++) acc[0][l] = r[l] + acc[0][l];
#pragma unroll
    for (int l = 0; l < 8; l++) acc[0][l] = r[8 + l] + acc[0][l];
    float sum = 0.0f;
    int pos = nb * 128, rem = n - pos;
    while (rem >= 32) {
        float4 xs[8];
#pragma unroll
        for (int cc = 0; cc < 8; cc++) xs[cc] = p[(size_t)((pos >> 2) + cc) * CSTRIDE];
#pragma unroll
        for (int cc = 0; cc < 8; cc++) chunk_update<METRIC>(acc, cc, q4[(pos >> 2) + cc], xs[cc]);
        pos += 32;
        rem -= 32;
    }
    while (rem >= 8) {
        const int c = pos >> 2;
        chunk_update<METRIC>(acc, 0, q4[c], p[(size_t)c * CSTRIDE]);
        chunk_update<METRIC>(acc, 1, q4[c + 1], p[(size_t)(c + 1) * CSTRIDE]);
        pos += 8;
        rem -= 8;
    }
    while (rem) {
        scalar_update<METRIC>(sum, q[pos], elem_at<CSTRIDE>(p, pos));
        pos++;
        rem--;
    }
    return avx256_reduce(acc, sum);
}

// The reduction order of the host's distancer: AVX2 (default, EPYC hosts) or AVX-512.
template <int METRIC, int CSTRIDE>
__device__ __forceinline__ float row_dist(const float4 *__restrict__ p, const float4 *__restrict__ q4, int n, int o512)
{
    return o512 ? row_dist_512<METRIC, CSTRIDE>(p, q4, n) : row_dot_or_l2_generic<METRIC, CSTRIDE>(p, q4, n);
}

// Provider.Wrap of the raw kernel value: L2 identity, dot -x (D/dot_product.go:68-76),
// cosine-dot 1-x (D/cosine_dist.go:38-45), manhattan / hamming identity
// (D/manhattan.go:80-82, D/hamming.go:88-90).
__device__ __forceinline__ float wrap_metric(int metric, float r)
{
    return metric == WVG_M_DOT ? -r : (metric == WVG_M_COSINE ? 1.0f - r : r);
}

}  // namespace wvg
