// wvg_pq.hip -- product quantization on MI355X.
//
// K7 LUT:    DistanceLookUpTable entries lut[i][c] = distance.Step(q_i, C_i[c])
//            (CH/product_quantization.go:85-104; Step is the pure-Go loop,
//            sequential and unfused on amd64: D/l2.go:79-88, D/dot_product.go:87-94).
// K8 ADC:    PQDistancer.Distance (CH/product_quantization.go:352-361):
//            sum += lut[i][code_i] for i = 0..m-1 in order, then Wrap.  The LUT
//            (m*ks*4 bytes, 32 KiB at m=32, ks=256) lives in LDS; codes stream
//            from HBM in the tiled layout (16 codes per 16-byte load per lane).
//            Roofline: HBM, N*m bytes per query (LDS-gather bound when codes
//            are random: see DESIGN.md).
// K9 encode: ProductQuantizer.Encode -> KMeans.Nearest (CH/product_quantization.go:420-426,
//            CH/kmeans.go:103-135): argmin_c l2_256(x_seg, C_s[c]) with the
//            candidate replacing the best unless best < d (ties -> highest c,
//            NaN replaces).
#include "wvg_internal.hpp"
#include "wvg_rowdist.hpp"
#include "wvg_topk.hpp"

namespace wvg {

constexpr int PQ_SCAN_WAVES = 16;  // K8: one workgroup per CU shares the LUT

// Step(a, b) in the pure-Go order: L2 D/l2.go:79-88, dot / cosine
// D/dot_product.go:87-94, manhattan D/manhattan.go:68-78 (sum += |a-b|),
// hamming D/hamming.go:76-86 (sum += 1 where a != b: Go's !=, a NaN counts).
__device__ __forceinline__ float go_step(int metric, const float *a, const float *b, uint32_t n)
{
    float sum = 0.0f;
    if (metric == WVG_M_L2) {
        for (uint32_t i = 0; i < n; i++) {
            float diff = a[i] - b[i];
            float sq = diff * diff;
            sum = sum + sq;
        }
    } else if (metric == WVG_M_MANHATTAN) {
        for (uint32_t i = 0; i < n; i++) sum = sum + __builtin_fabsf(a[i] - b[i]);
    } else if (metric == WVG_M_HAMMING) {
        for (uint32_t i = 0; i < n; i++)
            if (a[i] != b[i]) sum = sum + 1.0f;
    } else {
        for (uint32_t i = 0; i < n; i++) {
            float p = a[i] * b[i];
            sum = sum + p;
        }
    }
    return sum;
}

__global__ void pq_lut_kernel(int metric, const float *q, uint32_t nq, uint32_t qpitch, const float *centers,
                              uint32_t m, uint32_t ks, uint32_t ds, float *lut)
{
    const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t per_q = (uint64_t)m * ks;
    if (g >= per_q * nq) return;
    const uint32_t qi = (uint32_t)(g / per_q);
    const uint32_t r = (uint32_t)(g % per_q);
    const uint32_t seg = r / ks, c = r % ks;
    lut[g] = go_step(metric, q + (size_t)qi * qpitch + (size_t)seg * ds, centers + ((size_t)seg * ks + c) * ds, ds);
}

hipError_t launch_pq_lut(int metric, const float *q, uint32_t nq, uint32_t qpitch, const float *centers, uint32_t m,
                         uint32_t ks, uint32_t ds, float *lut, hipStream_t s)
{
    const uint64_t total = (uint64_t)nq * m * ks;
    if (total == 0) return hipSuccess;
    hipLaunchKernelGGL(pq_lut_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, metric, q, nq, qpitch,
                       centers, m, ks, ds, lut);
    return hipGetLastError();
}

// l2_256 (D/c/l2_avx256_amd64.c:14-107) over element accessors.
template <typename XA, typename CA>
__device__ __forceinline__ float l2_256_acc(XA x, CA c, int n)
{
    float sum = 0.0f;
    if (n < 8) {
        for (int i = 0; i < n; i++) scalar_update<WVG_M_L2>(sum, c(i), x(i));
        return sum;
    }
    float acc[4][8];
#pragma unroll
    for (int j = 0; j < 4; j++)
#pragma unroll
        for (int l = 0; l < 8; l++) acc[j][l] = 0.0f;
    int pos = 0, rem = n;
    while (rem >= 32) {
#pragma unroll
        for (int j = 0; j < 4; j++)
#pragma unroll
            for (int l = 0; l < 8; l++) acc_update<WVG_M_L2>(acc[j][l], x(pos + 8 * j + l), c(pos + 8 * j + l));
        pos += 32;
        rem -= 32;
    }
    while (rem >= 8) {
#pragma unroll
        for (int l = 0; l < 8; l++) acc_update<WVG_M_L2>(acc[0][l], x(pos + l), c(pos + l));
        pos += 8;
        rem -= 8;
    }
    while (rem) {
        scalar_update<WVG_M_L2>(sum, x(pos), c(pos));
        pos++;
        rem--;
    }
    return avx256_reduce(acc, sum);
}

// Encode from the tiled float layout; lane = row.  Output either row-major
// codes [n][m] or, TILED_OUT, the PQ corpus layout (16 codes per 16-byte
// chunk, stored once per chunk).  (diff = point - centroid; l2_256(filteredPoint, c)
// at CH/kmeans.go:120.)
// The centroid reads are wave-uniform: read through the constant address
// space they become s_load_dwordx16 batches whose SGPRs feed the packed
// subtracts directly -- as generic loads every centroid was a vector load
// followed by a full-latency wait.
typedef float f32x2e __attribute__((ext_vector_type(2)));

// pairs (DS == 4, even ks; may be null): the codebook with centroids c and
// c+1 interleaved per coordinate, [m][ks/2][4][2] (pq_pair_layout), so one
// scalar register pair feeds a packed op on two centroids at once.
// Argmin in the pair path.  The reference keeps a centroid when
// !(minD < d) (CH/kmeans.go:126-130): without NaN distances the result is the
// LAST index at the global minimum, so the loop only tracks the running
// minimum (one v_min3_f32 per pair) and the last PAIR that holds it (two
// compares and one select), and the winner inside that pair is decided once
// at the end by recomputing its two distances (the same ops, the same bits):
// 5 VALU per pair for the argmin instead of 8 (two compares, four selects and
// two index moves).  NaN distances need a NaN in the row's segment or in a
// centroid (centroid - row with finite centroids is never NaN: x = +-inf gives
// +inf); `nan_free` says the codebook has none, and a wave whose segment has a
// NaN takes the reference loop.
constexpr int PQ_ENC_GROUP = 4;  // pairs per argmin group (8 centroids: 32 SGPRs of centroids)

// seg_nan (k-means passes): per segment, nonzero when its centroids hold a NaN
// (pq_pairs_kernel writes it with the pair copy); a segment without one takes
// the min3 argmin like a nan_free codebook.  gridDim.y > 1 (row-major codes
// only): workgroup row y encodes segments [y m / G, (y + 1) m / G) of its rows,
// so a small row count (the 100k-row Lloyd assignment) still fills the chip.
template <int DS, bool TILED_OUT>
__global__ void pq_encode_kernel(const float4 *__restrict__ tiled, uint64_t n, uint32_t dim, uint32_t nchunks,
                                 const float *__restrict__ centers, uint32_t m, uint32_t ks, uint32_t ds_rt,
                                 uint8_t *__restrict__ codes, const float *__restrict__ pairs, int nan_free,
                                 const uint32_t *__restrict__ seg_nan, uint64_t half)
{
    // two rows per thread, r and r + half (half: a multiple of 64 >= n / 2): the
    // centroids a wave reads through its scalar loads serve both rows' packed ops
    // (the scalar fetches, not the VALU, held round 3's kernel: SQ_INSTS_VALU at
    // ~50% of the issue slots, 53% of wave cycles waiting; profiles/r04/pmc_enc/)
    const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    const uint64_t rb = r + half;
    const bool hasb = rb < n;
    const uint32_t ds = DS > 0 ? (uint32_t)DS : ds_rt;
    const float4 *rp = tiled + ((r >> 6) * nchunks) * 64 + (r & 63);
    const float4 *rpb = hasb ? tiled + ((rb >> 6) * nchunks) * 64 + (rb & 63) : rp;
    // the nearest centroid of segment s for the row at rpx (nNearest, CH/kmeans.go:103-135)
    auto seg_best = [&](const float4 *rpx, uint32_t s) -> uint32_t {
            const float *cs = centers + (size_t)s * ks * ds;
            uint32_t best = 0;
            float minD = 3.40282346638528859812e+38f;  // math.MaxFloat32
            if constexpr (DS == 4) {
                // segment s is exactly chunk s (dim = 4m): one 16-byte load, scalar unfused path (n < 8)
                const float4 x = rpx[(size_t)s * 64];
                const bool row_nan = !(x.x == x.x && x.y == x.y && x.z == x.z && x.w == x.w);
                if (pairs && (nan_free || (seg_nan && seg_nan[s] == 0u)) && __ballot(row_nan) == 0ull) {  // (see the argmin note above)
                    const f32x2e xx = {x.x, x.x}, xy = {x.y, x.y}, xz = {x.z, x.z}, xw = {x.w, x.w};
                    const __attribute__((address_space(4))) float *cp =
                        (const __attribute__((address_space(4))) float *)(pairs + (size_t)s * ks * 4);
                    auto pair_sum = [&](const float *pp) {  // (c - x)^2 summed in k order for centroids 2p, 2p+1
                        const f32x2e d0 = f32x2e{pp[0], pp[1]} - xx, d1 = f32x2e{pp[2], pp[3]} - xy;
                        const f32x2e d2 = f32x2e{pp[4], pp[5]} - xz, d3 = f32x2e{pp[6], pp[7]} - xw;
                        f32x2e sum = d0 * d0;
                        sum = sum + d1 * d1;
                        sum = sum + d2 * d2;
                        sum = sum + d3 * d3;
                        return sum;
                    };
                    float mn = minD;
                    if ((ks & (2 * PQ_ENC_GROUP - 1)) == 0) {
                        // groups of PQ_ENC_GROUP pairs: the group's minimum by a
                        // v_min3 chain, then ONE compare + select per group for
                        // the last group holding the running minimum (group min
                        // <= the minimum before it, ties included: later wins);
                        // the winner inside it is found once at the end
                        uint32_t bg = 0;
                        for (uint32_t g = 0; g < ks / (2 * PQ_ENC_GROUP); g++) {
                            float gm = 0.0f;
#pragma unroll
                            for (int j = 0; j < PQ_ENC_GROUP; j++) {
                                const __attribute__((address_space(4))) float *pp =
                                    cp + ((size_t)g * PQ_ENC_GROUP + j) * 8;
                                const f32x2e d0 = f32x2e{pp[0], pp[1]} - xx, d1 = f32x2e{pp[2], pp[3]} - xy;
                                const f32x2e d2 = f32x2e{pp[4], pp[5]} - xz, d3 = f32x2e{pp[6], pp[7]} - xw;
                                f32x2e sum = d0 * d0;
                                sum = sum + d1 * d1;
                                sum = sum + d2 * d2;
                                sum = sum + d3 * d3;
                                gm = j == 0 ? __builtin_fminf(sum.x, sum.y)
                                            : __builtin_fminf(__builtin_fminf(gm, sum.x), sum.y);
                            }
                            const bool miss = gm > mn;  // (NaN-free here; ties go to the later group)
                            bg = miss ? bg : g;
                            mn = miss ? mn : gm;
                        }
                        best = 0;  // when nothing reached math.MaxFloat32
#pragma unroll 1
                        for (int j = 0; j < PQ_ENC_GROUP; j++) {  // (per-lane group: vector loads, one pair at a time)
                            const uint32_t p = bg * PQ_ENC_GROUP + j;
                            const f32x2e sb = pair_sum(pairs + ((size_t)s * ks + 2 * p) * 4);
                            if (sb.x == mn) best = 2 * p;
                            if (sb.y == mn) best = 2 * p + 1;
                        }
                    } else {
                        uint32_t bp = 0;
#pragma unroll 4
                        for (uint32_t p = 0; p < ks / 2; p++) {
                            const __attribute__((address_space(4))) float *pp = cp + (size_t)p * 8;
                            const f32x2e d0 = f32x2e{pp[0], pp[1]} - xx, d1 = f32x2e{pp[2], pp[3]} - xy;
                            const f32x2e d2 = f32x2e{pp[4], pp[5]} - xz, d3 = f32x2e{pp[6], pp[7]} - xw;
                            f32x2e sum = d0 * d0;
                            sum = sum + d1 * d1;
                            sum = sum + d2 * d2;
                            sum = sum + d3 * d3;
                            const float m2 = __builtin_fminf(__builtin_fminf(mn, sum.x), sum.y);
                            if ((sum.x == m2) | (sum.y == m2)) bp = p;
                            mn = m2;
                        }
                        const f32x2e sb = pair_sum(pairs + ((size_t)s * ks + 2 * bp) * 4);
                        best = sb.y == mn ? 2 * bp + 1 : 2 * bp;  // 0 when nothing beat math.MaxFloat32
                    }
                    minD = mn;
                } else if (pairs) {
                    // two centroids per packed op: (c_k - x_k)^2 summed in k order,
                    // exactly the scalar path's sub, mul, add sequence per lane
                    const f32x2e xx = {x.x, x.x}, xy = {x.y, x.y}, xz = {x.z, x.z}, xw = {x.w, x.w};
                    const __attribute__((address_space(4))) float *cp =
                        (const __attribute__((address_space(4))) float *)(pairs + (size_t)s * ks * 4);
#pragma unroll 4
                    for (uint32_t p = 0; p < ks / 2; p++) {
                        const __attribute__((address_space(4))) float *pp = cp + (size_t)p * 8;
                        const f32x2e d0 = f32x2e{pp[0], pp[1]} - xx, d1 = f32x2e{pp[2], pp[3]} - xy;
                        const f32x2e d2 = f32x2e{pp[4], pp[5]} - xz, d3 = f32x2e{pp[6], pp[7]} - xw;
                        f32x2e sum = d0 * d0;
                        sum = sum + d1 * d1;
                        sum = sum + d2 * d2;
                        sum = sum + d3 * d3;
                        if (!(minD < sum.x)) {
                            minD = sum.x;
                            best = 2 * p;
                        }
                        if (!(minD < sum.y)) {
                            minD = sum.y;
                            best = 2 * p + 1;
                        }
                    }
                } else {
#pragma unroll 8
                for (uint32_t c = 0; c < ks; c++) {
                    const __attribute__((address_space(4))) float *cc =
                        (const __attribute__((address_space(4))) float *)(cs + (size_t)c * 4);
                    float sum = 0.0f;
                    scalar_update<WVG_M_L2>(sum, cc[0], x.x);
                    scalar_update<WVG_M_L2>(sum, cc[1], x.y);
                    scalar_update<WVG_M_L2>(sum, cc[2], x.z);
                    scalar_update<WVG_M_L2>(sum, cc[3], x.w);
                    if (!(minD < sum)) {
                        minD = sum;
                        best = c;
                    }
                }
                }
            } else {
                const uint32_t base = s * ds;
                auto xa = [&](int i) { return elem_at<64>(rpx, (int)(base + i)); };
                for (uint32_t c = 0; c < ks; c++) {
                    const __attribute__((address_space(4))) float *cv =
                        (const __attribute__((address_space(4))) float *)(cs + (size_t)c * ds);
                    auto ca = [&](int i) { return cv[i]; };
                    const float d = l2_256_acc(xa, ca, (int)ds);
                    if (!(minD < d)) {
                        minD = d;
                        best = c;
                    }
                }
            }
            return best;
    };
    // both rows' codes of segment s: the grouped min3 argmin of the two rows in one pass over the
    // centroids where it applies (the same ops per row as seg_best), else seg_best per row
    auto seg_best2 = [&](uint32_t s, uint32_t &ca, uint32_t &cb) {
        if constexpr (DS == 4) {
            if (pairs && (ks & (2 * PQ_ENC_GROUP - 1)) == 0 && (nan_free || (seg_nan && seg_nan[s] == 0u))) {
                const float4 x = rp[(size_t)s * 64], y = rpb[(size_t)s * 64];
                const bool nan2 = !(x.x == x.x && x.y == x.y && x.z == x.z && x.w == x.w) ||
                                  !(y.x == y.x && y.y == y.y && y.z == y.z && y.w == y.w);
                if (__ballot(nan2) == 0ull) {
                    const f32x2e ax = {x.x, x.x}, ay = {x.y, x.y}, az = {x.z, x.z}, aw = {x.w, x.w};
                    const f32x2e bx = {y.x, y.x}, by = {y.y, y.y}, bz = {y.z, y.z}, bw = {y.w, y.w};
                    auto psum = [](const f32x2e c0, const f32x2e c1, const f32x2e c2, const f32x2e c3, f32x2e px,
                                   f32x2e py, f32x2e pz, f32x2e pw) {
                        const f32x2e d0 = c0 - px, d1 = c1 - py, d2 = c2 - pz, d3 = c3 - pw;
                        f32x2e sum = d0 * d0;
                        sum = sum + d1 * d1;
                        sum = sum + d2 * d2;
                        sum = sum + d3 * d3;
                        return sum;
                    };
                    const __attribute__((address_space(4))) float *cp =
                        (const __attribute__((address_space(4))) float *)(pairs + (size_t)s * ks * 4);
                    float mna = 3.40282346638528859812e+38f, mnb = mna;
                    uint32_t bga = 0, bgb = 0;
                    for (uint32_t g = 0; g < ks / (2 * PQ_ENC_GROUP); g++) {
                        float gma = 0.0f, gmb = 0.0f;
#pragma unroll
                        for (int j = 0; j < PQ_ENC_GROUP; j++) {
                            const __attribute__((address_space(4))) float *pp = cp + ((size_t)g * PQ_ENC_GROUP + j) * 8;
                            const f32x2e c0 = {pp[0], pp[1]}, c1 = {pp[2], pp[3]}, c2 = {pp[4], pp[5]}, c3 = {pp[6], pp[7]};
                            const f32x2e sa = psum(c0, c1, c2, c3, ax, ay, az, aw);
                            const f32x2e sb = psum(c0, c1, c2, c3, bx, by, bz, bw);
                            gma = j == 0 ? __builtin_fminf(sa.x, sa.y) : __builtin_fminf(__builtin_fminf(gma, sa.x), sa.y);
                            gmb = j == 0 ? __builtin_fminf(sb.x, sb.y) : __builtin_fminf(__builtin_fminf(gmb, sb.x), sb.y);
                        }
                        const bool missa = gma > mna, missb = gmb > mnb;  // (ties go to the later group)
                        bga = missa ? bga : g;
                        mna = missa ? mna : gma;
                        bgb = missb ? bgb : g;
                        mnb = missb ? mnb : gmb;
                    }
                    ca = 0;  // when nothing reached math.MaxFloat32
                    cb = 0;
#pragma unroll 1
                    for (int j = 0; j < PQ_ENC_GROUP; j++) {  // the winners inside the last groups at the minimum
                        const uint32_t pa = bga * PQ_ENC_GROUP + j, pb = bgb * PQ_ENC_GROUP + j;
                        const float *qa = pairs + ((size_t)s * ks + 2 * pa) * 4, *qb = pairs + ((size_t)s * ks + 2 * pb) * 4;
                        const f32x2e sa = psum(f32x2e{qa[0], qa[1]}, f32x2e{qa[2], qa[3]}, f32x2e{qa[4], qa[5]},
                                               f32x2e{qa[6], qa[7]}, ax, ay, az, aw);
                        const f32x2e sb = psum(f32x2e{qb[0], qb[1]}, f32x2e{qb[2], qb[3]}, f32x2e{qb[4], qb[5]},
                                               f32x2e{qb[6], qb[7]}, bx, by, bz, bw);
                        if (sa.x == mna) ca = 2 * pa;
                        if (sa.y == mna) ca = 2 * pa + 1;
                        if (sb.x == mnb) cb = 2 * pb;
                        if (sb.y == mnb) cb = 2 * pb + 1;
                    }
                    return;
                }
            }
        }
        ca = seg_best(rp, s);
        cb = hasb ? seg_best(rpb, s) : 0u;
    };
    if constexpr (!TILED_OUT) {
        const uint32_t s0 = (uint32_t)((uint64_t)m * blockIdx.y / gridDim.y);
        const uint32_t s1 = (uint32_t)((uint64_t)m * (blockIdx.y + 1) / gridDim.y);
        for (uint32_t s = s0; s < s1; s++) {
            uint32_t ca, cb;
            seg_best2(s, ca, cb);
            codes[r * m + s] = (uint8_t)ca;
            if (hasb) codes[rb * m + s] = (uint8_t)cb;
        }
        return;
    }
    const uint32_t out_chunks = pq_chunks(m);
    uint32_t w8[8] = {0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u};  // TILED_OUT, m = 32: all codes, rotated before the store
    uint32_t w8b[8] = {0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u};  // (the second row's)
    for (uint32_t oc = 0; oc < out_chunks; oc++) {
        uint32_t w[4] = {0u, 0u, 0u, 0u}, wb[4] = {0u, 0u, 0u, 0u};
        for (uint32_t bsel = 0; bsel < 16; bsel++) {
            const uint32_t s = oc * 16 + bsel;
            if (s >= m) break;
            uint32_t ca, cb;
            seg_best2(s, ca, cb);
            w[bsel >> 2] |= ca << (8 * (bsel & 3));
            wb[bsel >> 2] |= cb << (8 * (bsel & 3));
        }
        if constexpr (TILED_OUT) {
            if (pq_rotated(m)) {
#pragma unroll
                for (int i = 0; i < 4; i++) {
                    if (oc == 0) w8[i] = w[i], w8b[i] = wb[i];
                    else w8[4 + i] = w[i], w8b[4 + i] = wb[i];
                }
            } else {
                reinterpret_cast<uint4 *>(codes)[((r >> 6) * out_chunks + oc) * 64 + (r & 63)] =
                    make_uint4(w[0], w[1], w[2], w[3]);
                if (hasb)
                    reinterpret_cast<uint4 *>(codes)[((rb >> 6) * out_chunks + oc) * 64 + (rb & 63)] =
                        make_uint4(wb[0], wb[1], wb[2], wb[3]);
            }
        }
    }
    if constexpr (TILED_OUT) {
        if (pq_rotated(m)) {
            uint32_t st[8];
            pq32_window(w8, (uint32_t)(r & 31), st);
            uint4 *o = reinterpret_cast<uint4 *>(codes) + ((r >> 6) * 2) * 64 + (r & 63);
            o[0] = make_uint4(st[0], st[1], st[2], st[3]);
            o[64] = make_uint4(st[4], st[5], st[6], st[7]);
            if (hasb) {
                pq32_window(w8b, (uint32_t)(rb & 31), st);
                uint4 *ob = reinterpret_cast<uint4 *>(codes) + ((rb >> 6) * 2) * 64 + (rb & 63);
                ob[0] = make_uint4(st[0], st[1], st[2], st[3]);
                ob[64] = make_uint4(st[4], st[5], st[6], st[7]);
            }
        }
    }
}

hipError_t launch_pq_encode(const float *tiled, uint64_t n, uint32_t dim, const float *centers, uint32_t m,
                            uint32_t ks, uint8_t *codes, hipStream_t s, bool tiled_out, bool nan_free,
                            const uint32_t *seg_nan)
{
    if (n == 0) return hipSuccess;
    const uint32_t ds = dim / m, nchunks = f32_chunks(dim);
    const uint64_t half = (n + 127) / 128 * 64;  // two rows per thread: r and r + half
    const unsigned blocks = (unsigned)((half + 255) / 256);
    // row-major output: segment groups until ~16k workgroups (64k waves) are in flight
    const unsigned groups = tiled_out ? 1u : std::max(1u, std::min<unsigned>(m, 16384u / blocks));
    dim3 grid(blocks, groups), block(256);
    const float4 *t4 = reinterpret_cast<const float4 *>(tiled);
    // codebook buffers (pq_centers_alloc_bytes) carry the pair layout after the table
    const float *pairs = pq_has_pairs(ks, ds) ? centers + (size_t)m * ks * ds : nullptr;
    nan_free = nan_free && tuning().pq_encode_min3 != 0;
    if (tuning().pq_encode_min3 == 0) seg_nan = nullptr;
    if (ds == 4 && dim == 4 * m) {
        if (tiled_out)
            hipLaunchKernelGGL((pq_encode_kernel<4, true>), grid, block, 0, s, t4, n, dim, nchunks, centers, m, ks, ds,
                               codes, pairs, (int)nan_free, seg_nan, half);
        else
            hipLaunchKernelGGL((pq_encode_kernel<4, false>), grid, block, 0, s, t4, n, dim, nchunks, centers, m, ks, ds,
                               codes, pairs, (int)nan_free, seg_nan, half);
    } else {
        if (tiled_out)
            hipLaunchKernelGGL((pq_encode_kernel<0, true>), grid, block, 0, s, t4, n, dim, nchunks, centers, m, ks, ds,
                               codes, nullptr, 0, nullptr, half);
        else
            hipLaunchKernelGGL((pq_encode_kernel<0, false>), grid, block, 0, s, t4, n, dim, nchunks, centers, m, ks, ds,
                               codes, nullptr, 0, nullptr, half);
    }
    return hipGetLastError();
}

__global__ void pq_store_kernel(const uint8_t *codes, const uint64_t *slots, uint64_t n, uint32_t m, uint32_t nchunks,
                                uint4 *tiled)
{
    const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= n * nchunks) return;
    const uint64_t i = g / nchunks;
    const uint32_t c = (uint32_t)(g % nchunks);
    const uint64_t slot = slots ? slots[i] : i;
    uint32_t w[4] = {0u, 0u, 0u, 0u};
    const uint32_t rot = pq_rotated(m) ? (uint32_t)(slot & 31) : 0u;
    for (uint32_t b = 0; b < 16; b++) {
        const uint32_t pos = c * 16 + b;
        const uint32_t seg = rot ? (pos + rot) & 31u : pos;
        if (seg < m) w[b >> 2] |= (uint32_t)codes[i * m + seg] << (8 * (b & 3));
    }
    tiled[((slot >> 6) * nchunks + c) * 64 + (slot & 63)] = make_uint4(w[0], w[1], w[2], w[3]);
}

hipError_t launch_pq_store(const uint8_t *codes, const uint64_t *slots, uint64_t n, uint32_t m, uint32_t nchunks,
                           uint8_t *tiled, hipStream_t s)
{
    const uint64_t total = n * nchunks;
    if (total == 0) return hipSuccess;
    hipLaunchKernelGGL(pq_store_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, codes, slots, n, m,
                       nchunks, reinterpret_cast<uint4 *>(tiled));
    return hipGetLastError();
}

__device__ __forceinline__ uint32_t code_at(const uint4 *cw, int i)
{
    const uint4 v = cw[i >> 4];
    const int w = (i >> 2) & 3;
    const uint32_t word = w == 0 ? v.x : (w == 1 ? v.y : (w == 2 ? v.z : v.w));
    return (word >> (8 * (i & 3))) & 0xFFu;
}

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint4 ld_codes(const uint4 *p)
{
    const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(p));
    return make_uint4(v.x, v.y, v.z, v.w);
}

__device__ __forceinline__ uint64_t pq_tile_mask(const ScanArgs &a, uint64_t t)
{
    uint64_t m = a.valid[t];
    if (a.allow) {
        uint64_t w = t - a.allow_t0;  // allow[0] is tile allow_t0's word
        m &= w < a.allow_words ? a.allow[w] : 0ull;
    }
    return m;
}

// K8: ADC scan.  One workgroup of PQ_SCAN_WAVES waves per CU shares one copy
// of the query's LUT (m x ks fp32) in LDS; lane = row, each lane gathers its
// row's m entries (independent ds_read_b32s) and sums them in segment order
// (CH/product_quantization.go:85-104).  Fixed M: the next live tile's codes are
// loaded (non-temporal) while the current tile is looked up, so the HBM
// latency is covered by 16 waves x 2 tiles in flight per CU.
template <int E, int M, int KS>
__global__ __launch_bounds__(PQ_SCAN_WAVES * 64) void scan_pq_kernel(ScanArgs a, uint64_t *partials)
{
    extern __shared__ __attribute__((aligned(16))) float lut[];
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t qi = blockIdx.y;
    const uint32_t m = M > 0 ? (uint32_t)M : a.pq_m;
    const uint32_t ks = KS > 0 ? (uint32_t)KS : a.pq_ks;
    const float *glut = reinterpret_cast<const float *>(a.queries) + (size_t)qi * a.qpitch;
    for (uint32_t i = threadIdx.x; i < m * ks; i += blockDim.x) lut[i] = glut[i];
    __syncthreads();
    const uint4 *data = reinterpret_cast<const uint4 *>(a.data);
    const uint32_t nch = a.nchunks;
    const uint64_t ntiles = a.tile_end - a.tile_begin;
    const uint64_t total = (uint64_t)gridDim.x * PQ_SCAN_WAVES;
    const uint64_t gw = (uint64_t)blockIdx.x * PQ_SCAN_WAVES + wave;
    const uint64_t t0 = a.tile_begin + ntiles * gw / total, t1 = a.tile_begin + ntiles * (gw + 1) / total;
    WaveTopK<E> tk;
    tk.init((int)a.k);
    if constexpr (M > 0) {
        constexpr int NC = (M + 15) / 16;
        auto next_live = [&](uint64_t t, uint64_t &msk) {
            for (; t < t1; ++t) {
                msk = pq_tile_mask(a, t);
                if (msk) break;
            }
            return t;
        };
        uint64_t m_cur = 0, m_nxt = 0;
        uint64_t t = next_live(t0, m_cur);
        uint4 cur[NC], nxt[NC];
        if (t < t1) {
            const uint4 *rp = data + (size_t)t * NC * 64 + lane;
#pragma unroll
            for (int c = 0; c < NC; c++) cur[c] = ld_codes(rp + (size_t)c * 64);
        }
        while (t < t1) {
            const uint64_t tn = next_live(t + 1, m_nxt);
            if (tn < t1) {
                const uint4 *rp = data + (size_t)tn * NC * 64 + lane;
#pragma unroll
                for (int c = 0; c < NC; c++) nxt[c] = ld_codes(rp + (size_t)c * 64);
            }
            uint4 uc[NC];  // codes in segment order (m = 32 rows are stored rotated)
            if constexpr (M == 32) {
                const uint32_t w[8] = {cur[0].x, cur[0].y, cur[0].z, cur[0].w, cur[1].x, cur[1].y, cur[1].z, cur[1].w};
                uint32_t o[8];
                pq32_window(w, (32u - ((uint32_t)lane & 31u)) & 31u, o);
                uc[0] = make_uint4(o[0], o[1], o[2], o[3]);
                uc[1] = make_uint4(o[4], o[5], o[6], o[7]);
            } else {
#pragma unroll
                for (int c = 0; c < NC; c++) uc[c] = cur[c];
            }
            float v[M];
#pragma unroll
            for (int i = 0; i < M; i++) v[i] = lut[i * ks + code_at(uc, i)];
            float sum = 0.0f;
#pragma unroll
            for (int i = 0; i < M; i++) sum = sum + v[i];
            const float dist = wrap_metric(a.metric, sum);
            tk.offer(((m_cur >> lane) & 1ull) ? wvg_make_key(dist, (uint32_t)(t * 64 + lane)) : WVG_KEY_NONE);
#pragma unroll
            for (int c = 0; c < NC; c++) cur[c] = nxt[c];
            t = tn;
            m_cur = m_nxt;
        }
    } else {
        for (uint64_t t = t0; t < t1; ++t) {
            const uint64_t msk = pq_tile_mask(a, t);
            if (msk == 0ull) continue;
            const uint4 *rp = data + (size_t)t * nch * 64 + lane;
            const float dist = wrap_metric(a.metric, pq_row_sum(rp, nch, m, ks, lut, (uint64_t)lane));
            tk.offer(((msk >> lane) & 1ull) ? wvg_make_key(dist, (uint32_t)(t * 64 + lane)) : WVG_KEY_NONE);
        }
    }
    group_combine_store<E, PQ_SCAN_WAVES>(tk, partials + ((size_t)qi * gridDim.x + blockIdx.x) * a.k);
}

// K8b: ADC scan for m = 32, ks = 256 without LDS bank conflicts.
//
// K8 gathers lut[i][code_i] with every lane of a wave on the same segment i, so
// the 32 lanes of a ds_read_b32 group hit 32 random banks (~4-way conflicts,
// ~8 LDS cycles per read: the scan ran LDS-bound at 57% of HBM).  Here lane l
// (x = l mod 32) reads segment (x + j) mod 32 at step j, so at every step the
// 32 lanes of a group read 32 different segments.
//
// Each row's sum must still run in segment order (CH/product_quantization.go:85-104).
// Lane x therefore works on two rows at once: during the pass over tile p it
// finishes row p (segments x..31, steps 0..31-x) into accumulator A and starts
// row p+1 (segments 0..x-1, steps 32-x..31) into accumulator B.  The LUT image
// in LDS makes that routing free: qword c*64 + s' holds (lut[s'][c], +0.0) for
// s' < 32 and (+0.0, lut[s'-32][c]) for s' >= 32, and step j reads qword
// c*64 + x + j with ds_read_b64 -- the 32 lanes of a group on 32 distinct bank
// pairs (2 LDS cycles) -- then one v_pk_add_f32 adds it to (A, B).  Adding
// +0.0 is exact (a sum that starts at float32(0) never becomes -0.0, and
// inf/NaN sums stay as they are), so A and B are the reference's sequential
// sums bit for bit.  At the end of the pass A is row p's distance, B moves to
// A and B restarts from +0.0.
//
// Rows of m = 32 corpora are stored rotated by slot mod 32 (pq_rotated), so
// lane x's code for step j is stored byte j of row p (j < 32 - x) or of row
// p+1 (j >= 32 - x): one v_bfi per dword with a per-lane byte mask merges the
// two rows, then a byte extract and one v_lshl_or give the LDS address.
// LDS: the 128 KiB image, one workgroup per CU.
typedef float f32x2 __attribute__((ext_vector_type(2)));

// MODE 0: tiles with no live / allowed row are skipped (their codes are never
// loaded; the scan waits on each refill's tile-mask load).  MODE 1 (dense):
// every tile of the range is loaded and its validity word rides in the ring
// as a vector load next to the codes, so no wait sits between refills; used
// without an allow list on mostly-live corpora.  MODE 2: MODE 1's loads with
// no lookups (A/B diagnostic: the access pattern's memory ceiling; results
// are meaningless).
template <int E, int R, bool IL, int NB, int MODE = 0>
__global__ __launch_bounds__(PQ_SCAN_WAVES * 64) void scan_pq32_rot_kernel(ScanArgs a, uint64_t *partials)
{
    extern __shared__ __attribute__((aligned(16))) f32x2 img[];  // [256][64]
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t qi = blockIdx.y;
    const float *glut = reinterpret_cast<const float *>(a.queries) + (size_t)qi * a.qpitch;
    // all of a thread's LUT reads in flight at once (a rolled loop paid one L2
    // round trip per iteration: most of the launch's fixed cost)
    constexpr int FILL = 32 * 256 / (PQ_SCAN_WAVES * 64);
    float fv[FILL];
#pragma unroll
    for (int it = 0; it < FILL; it++) {
        const uint32_t i = (uint32_t)it * (PQ_SCAN_WAVES * 64) + threadIdx.x;
        fv[it] = glut[(i & 31u) * 256u + (i >> 5)];
    }
#pragma unroll
    for (int it = 0; it < FILL; it++) {
        const uint32_t i = (uint32_t)it * (PQ_SCAN_WAVES * 64) + threadIdx.x;
        const uint32_t s = i & 31u, c = i >> 5;
        img[c * 64u + s] = f32x2{fv[it], 0.0f};
        img[c * 64u + 32u + s] = f32x2{0.0f, fv[it]};
    }
    __syncthreads();
    const uint4 *data = reinterpret_cast<const uint4 *>(a.data);
    const uint64_t ntiles = a.tile_end - a.tile_begin;
    // IL: the workgroup owns a contiguous tile range and its waves take every
    // PQ_SCAN_WAVES-th tile of it (the 16 waves stream one 32 KiB block at a
    // time); otherwise every wave owns a contiguous range.
    constexpr uint64_t TS = IL ? PQ_SCAN_WAVES : 1;  // tile stride of a wave
    uint64_t t0, t1;
    if constexpr (IL) {
        t0 = a.tile_begin + ntiles * blockIdx.x / gridDim.x + (uint64_t)wave;
        t1 = a.tile_begin + ntiles * (blockIdx.x + 1) / gridDim.x;
    } else {
        const uint64_t total = (uint64_t)gridDim.x * PQ_SCAN_WAVES;
        const uint64_t gw = (uint64_t)blockIdx.x * PQ_SCAN_WAVES + wave;
        t0 = a.tile_begin + ntiles * gw / total;
        t1 = a.tile_begin + ntiles * (gw + 1) / total;
    }
    WaveTopK<E> tk;
    tk.init((int)a.k);
    if (t0 < t1) {
        const uint32_t x = (uint32_t)lane & 31u;
        const uint32_t x8 = x * 8u;
        // the stored rows are rotated by slot mod 32 = x, so step j's code is
        // stored byte j of row p (j < 32 - x) or of row p+1 (j >= 32 - x)
        uint32_t nmask[8];  // bytes taken from the next row
#pragma unroll
        for (int w = 0; w < 8; w++) {
            uint32_t mk = 0u;
#pragma unroll
            for (int bb = 0; bb < 4; bb++) mk |= (4u * w + bb + x >= 32u) ? (0xFFu << (8 * bb)) : 0u;
            nmask[w] = mk;
        }
        const char *imgb = reinterpret_cast<const char *>(img);

        auto next_live = [&](uint64_t t, uint64_t &msk) {
            if constexpr (MODE != 0) {
                msk = 0;  // dense: the tile's mask comes with its codes (vm)
                return t < t1 ? t : t1;
            }
            for (; t < t1; t += TS) {
                msk = pq_tile_mask(a, t);
                if (msk) break;
            }
            return t;
        };
        // Loads are unconditional (a finished stream re-reads tile t0, whose
        // values are never used) so the waits on the ring stay static.
        auto load = [&](uint64_t t, uint32_t (&w)[8], uint64_t &vm) {
            const uint64_t tt = t < t1 ? t : t0;
            const uint4 *rp = data + (size_t)tt * 2 * 64 + lane;
            const uint4 lo = ld_codes(rp), hi = ld_codes(rp + 64);
            w[0] = lo.x; w[1] = lo.y; w[2] = lo.z; w[3] = lo.w;
            w[4] = hi.x; w[5] = hi.y; w[6] = hi.z; w[7] = hi.w;
            if constexpr (MODE != 0) {  // broadcast vector loads (every lane the same word)
                uint64_t m = t < t1 ? a.valid[tt] : 0ull;
                if (a.allow) {
                    const uint64_t w = tt - a.allow_t0;
                    m &= w < a.allow_words ? a.allow[w] : 0ull;
                }
                vm = m;
            }
        };

        // Ring of R live tiles' codes (R - 2 tiles of HBM latency cover beyond
        // the pass's own two).  Pass i: cur = slot (i-1) mod R = live tile i-1,
        // nxt = slot i mod R = live tile i; afterwards slot (i-1) mod R is
        // refilled with live tile i+R-1.  t1 marks "no tile".
        uint32_t ring[R][8];
        uint64_t rt[R], rm[R], rv[R];  // tile, scalar mask (MODE 0), vector-loaded mask (dense)
        rt[R - 1] = t1;
        rm[R - 1] = 0;
        rv[R - 1] = 0;
        {
            uint64_t t = t0;
#pragma unroll
            for (int s = 0; s < R - 1; s++) {
                uint64_t m = 0;
                t = next_live(t, m);
                rt[s] = t;
                rm[s] = m;
                load(t, ring[s], rv[s]);
                if (t < t1) t += TS;
            }
#pragma unroll
            for (int w = 0; w < 8; w++) ring[R - 1][w] = 0u;
        }
        uint64_t t_fill = rt[R - 2] < t1 ? rt[R - 2] + TS : t1;  // where the next refill searches from
        f32x2 acc = {0.0f, 0.0f};
        // Passes run in groups of R with no per-pass exit, so every load is
        // unconditional and the compiler's waits on the ring stay static; the
        // passes after the last live tile offer nothing (cur slot = t1).
        do {
#pragma unroll
            for (int s = 0; s < R; s++) {
                const int sc = (s + R - 1) % R;  // cur slot
                {
                    uint32_t win[8];
#pragma unroll
                    for (int w = 0; w < 8; w++)
                        asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(win[w]) : "v"(nmask[w]), "v"(ring[s][w]), "v"(ring[sc][w]));
                    if constexpr (MODE == 2) {
                        uint32_t x = 0;
#pragma unroll
                        for (int w = 0; w < 8; w++) x ^= win[w];
                        acc = acc + f32x2{(float)(x & 0xFFu), 0.0f};
                    } else {
                    // batches of NB reads, each all in flight before its adds
#pragma unroll
                    for (int h = 0; h < 32 / NB; h++) {
                        f32x2 v[NB];
#pragma unroll
                        for (int jj = 0; jj < NB; jj++) {
                            const int j = h * NB + jj;
                            // code << 8 by one v_perm (byte j mod 4 into byte 1, zeros elsewhere)
                            const uint32_t c8 = __builtin_amdgcn_perm(0u, win[j >> 2], 0x0C0C000Cu | ((uint32_t)(j & 3) << 8));
                            const uint32_t off = (c8 << 1) + x8;
                            v[jj] = *reinterpret_cast<const f32x2 *>(imgb + off + 8 * j);
                        }
#pragma unroll
                        for (int jj = 0; jj < NB; jj++) acc = acc + v[jj];
                    }
                    }
                    if (rt[sc] < t1) {
                        const uint64_t live = MODE != 0 ? __ballot((rv[sc] >> lane) & 1ull) : rm[sc];
                        tk.offer_dist(wrap_metric(a.metric, acc.x), (uint32_t)(rt[sc] * 64 + lane), live);
                    }
                    acc = f32x2{acc.y, 0.0f};
                    // refill the cur slot with the live tile R-1 passes ahead
                    uint64_t m = 0;
                    const uint64_t t = next_live(t_fill, m);
                    rt[sc] = t;
                    rm[sc] = m;
                    load(t, ring[sc], rv[sc]);
                    t_fill = t < t1 ? t + TS : t1;
                }
            }
        } while (rt[R - 1] < t1);
    }
    group_combine_store<E, PQ_SCAN_WAVES>(tk, partials + ((size_t)qi * gridDim.x + blockIdx.x) * a.k);
}

// K8c: K8b's arithmetic (rotated segments, (A, B) routing in the 128 KiB
// LUT image, rotated row storage) in its dense form, trimmed for issue: the
// counters of K8b show every SIMD issuing ~90 % of the time (VALU ~62 %, LDS
// and SALU the rest) at 73 % of HBM, i.e. the scan is instruction-issue bound,
// so K8c cuts the per-tile overhead around the 32 lookups:
//   - codes come through a per-wave buffer resource: the tile's byte offset
//     is a scalar soffset, the lane's a constant voffset, so a load costs no
//     address VALU, and loads past the wave's range (the ring's tail) return
//     zeros instead of needing a clamp;
//   - tile validity arrives 64 tiles per vector load (lane i = word of tile
//     i of the block, the allow window ANDed in) and two v_readlane per tile
//     turn it into the scalar live mask;
//   - top-k rejection compares the float distance with the K-th distance
//     (offer_dist_fast) instead of building ordered keys first;
//   - the metric's Wrap is a template parameter.
// Every tile of the wave's range is loaded (no skipping of dead tiles): the
// host runs K8c without an allow list on mostly-live corpora and K8b
// otherwise.  The A/B sums are K8b's, so results are bit-identical.
// W (LDS wait pattern): 0 = the compiler's (one s_waitcnt per lookup, so
// each add starts as soon as its value lands: 34 waits per tile, 18 % of the
// tile's instructions); 1 = one wait per batch of NB lookups; 2 = one wait
// per batch with the next batch's lookups already issued (software pipeline).
// W = 7: one-instruction lookup addresses (PQ32_IMG7_BYTES image, below).
//
// The one-v_perm address (W = 7).  K8c's address of step j is
// (code << 9) + 8x + 8j: a v_perm for code << 8 and a v_lshl_add.  Here the
// image is split by form instead of interleaved: region A holds (lut[s][c],
// +0.0) at byte c*256 + 8s, region B holds (+0.0, lut[s][c]) at byte
// PQ32_IMG7_B + c*256 + 8s.  Lane x's address of step j is then
//   8x | code << 8 | (x + j >= 32) << 16,   plus the immediate 8j:
// an A step (x + j < 32) lands on (code, s = x + j) in region A; a B step
// lands on 65536 + code*256 + 8(x + j) = PQ32_IMG7_B + code*256 + 8(x+j-32).
// The three bytes come from ONE v_perm of the merged code word and a per-lane
// constant F[j / 3] = 8x | flag(3k) << 8 | flag(3k+1) << 16 | flag(3k+2) << 24.
// Banks (ds_read_b64, (a/4) mod 64 per 32-lane group): 2(x+j) for A lanes,
// 2(x+j-32) for B lanes -- distinct, as in K8b.  Same sums, same results.
constexpr uint32_t PQ32_IMG7_B = 65536u + 256u;
constexpr uint32_t PQ32_IMG7_BYTES = PQ32_IMG7_B + 65536u;
// LDS address of the dynamic image: the kernel's only static LDS is the
// workgroup top-k buffer (group_combine_store: 16 waves x 64E keys x 8 B)
template <int E>
constexpr uint32_t PQ32_IMG7_BASE = (uint32_t)PQ_SCAN_WAVES * 64u * E * 8u;

#ifdef WVG_TOOLS
// K8c is a tools-build kernel: K8e (below) replaced it as the dense path, and
// K8b serves the product wherever K8e's LDS layout check fails.
// ACT < 16 (diagnostic): only the first ACT waves of the workgroup scan (the
// occupancy the scan needs: ACT / 4 waves per SIMD).
template <int E, int R, int NB, int METRIC, int W = 0, int ACT = PQ_SCAN_WAVES>
__global__ __launch_bounds__(PQ_SCAN_WAVES * 64) void scan_pq32_dense_kernel(ScanArgs a, uint64_t *partials)
{
    static_assert(64 % R == 0, "the ring length divides the 64-tile mask block");
    extern __shared__ __attribute__((aligned(16))) f32x2 img[];  // [256][64] (W = 7: regions A and B)
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t qi = blockIdx.y;
    const float *glut = reinterpret_cast<const float *>(a.queries) + (size_t)qi * a.qpitch;
    constexpr int FILL = 32 * 256 / (PQ_SCAN_WAVES * 64);
    float fv[FILL];
#pragma unroll
    for (int it = 0; it < FILL; it++) {
        const uint32_t i = (uint32_t)it * (PQ_SCAN_WAVES * 64) + threadIdx.x;
        fv[it] = glut[(i & 31u) * 256u + (i >> 5)];
    }
#pragma unroll
    for (int it = 0; it < FILL; it++) {
        const uint32_t i = (uint32_t)it * (PQ_SCAN_WAVES * 64) + threadIdx.x;
        const uint32_t s = i & 31u, c = i >> 5;
        if constexpr (W == 7) {
            img[c * 32u + s] = f32x2{fv[it], 0.0f};
            img[PQ32_IMG7_B / 8u + c * 32u + s] = f32x2{0.0f, fv[it]};
        } else {
            img[c * 64u + s] = f32x2{fv[it], 0.0f};
            img[c * 64u + 32u + s] = f32x2{0.0f, fv[it]};
        }
    }
    __syncthreads();
    const uint64_t ntiles = a.tile_end - a.tile_begin;
    const uint64_t total = (uint64_t)gridDim.x * ACT;
    const uint64_t gw = (uint64_t)blockIdx.x * ACT + (wave < ACT ? wave : 0);
    uint64_t t0 = a.tile_begin + ntiles * gw / total, t1 = a.tile_begin + ntiles * (gw + 1) / total;
    if (wave >= ACT) t1 = t0;
    WaveTopK<E> tk;
    tk.init((int)a.k);
    tk.init_fast();
    if (t0 < t1) {
        const uint32_t n = (uint32_t)(t1 - t0);  // tiles of this wave (2 KiB each)
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<char *>(reinterpret_cast<const char *>(a.data)) + t0 * 2048u, (short)0, (int)(n * 2048u),
            0x00020000);
        const uint32_t voff = (uint32_t)lane * 16u;
        const uint32_t x = (uint32_t)lane & 31u, x8 = x * 8u;
        uint32_t nmask[8];  // bytes of step j taken from the next row (see K8b)
#pragma unroll
        for (int w = 0; w < 8; w++) {
            uint32_t mk = 0u;
#pragma unroll
            for (int bb = 0; bb < 4; bb++) mk |= (4u * w + bb + x >= 32u) ? (0xFFu << (8 * bb)) : 0u;
            nmask[w] = mk;
        }
        uint32_t F[W == 7 ? 11 : 1];  // W = 7: 8x and the B flags of steps 3k..3k+2
#pragma unroll
        for (int k = 0; k < (W == 7 ? 11 : 1); k++) {
            uint32_t f = x8;
#pragma unroll
            for (int b = 0; b < 3; b++) {
                const uint32_t j = 3u * k + b;
                f |= (j < 32u && x + j >= 32u) ? (1u << (8 * (b + 1))) : 0u;
            }
            F[k] = f;
        }
        const char *imgb = reinterpret_cast<const char *>(img);
        // pass order: tiles t0 + i, or t1 - 1 - i when scanning downwards (rev)
        const bool rev = a.reverse & 1u;
        auto tile_of = [&](uint32_t i) -> uint32_t { return rev ? n - 1u - i : i; };
        auto load = [&](uint32_t i, uint32_t (&w)[8]) {  // the i-th tile of the pass order (zeros past it)
            const uint32_t so = i < n ? tile_of(i) * 2048u : n * 2048u;
            const u32x4 lo = __builtin_amdgcn_raw_buffer_load_b128(rs, voff, so, 2);
            const u32x4 hi = __builtin_amdgcn_raw_buffer_load_b128(rs, voff + 1024u, so, 2);
            w[0] = lo.x; w[1] = lo.y; w[2] = lo.z; w[3] = lo.w;
            w[4] = hi.x; w[5] = hi.y; w[6] = hi.z; w[7] = hi.w;
        };
        auto load_masks = [&](uint32_t b) -> uint64_t {  // lane i: live mask of the (64 b + i)-th tile
            const uint32_t ii = b * 64u + (uint32_t)lane;
            const uint64_t t = t0 + (ii < n ? tile_of(ii) : 0u);
            uint64_t m = 0ull;
            if (ii < n) {
                m = a.valid[t];
                if (a.allow) {
                    const uint64_t wi = t - a.allow_t0;
                    m &= wi < a.allow_words ? a.allow[wi] : 0ull;
                }
            }
            return m;
        };
        uint64_t mcur = load_masks(0), mnxt = load_masks(1);
        uint32_t ring[R][8];
#pragma unroll
        for (int s = 0; s < R - 1; s++) load((uint32_t)s, ring[s]);
#pragma unroll
        for (int w = 0; w < 8; w++) ring[R - 1][w] = 0u;
        f32x2 acc = {0.0f, 0.0f};
        uint32_t dummy = __builtin_amdgcn_readfirstlane(wave);  // W == 5 diagnostic (a scalar register)
        // pass i finishes tile i-1 (slot (i-1) mod R) and starts tile i (slot
        // i mod R); n + 1 passes, in groups of R so the ring slots are static
        for (uint32_t base = 0; base <= n; base += R) {
#pragma unroll
            for (int s = 0; s < R; s++) {
                const int sc = (s + R - 1) % R;
                const uint32_t i = base + (uint32_t)s;
                uint32_t win[8];
#pragma unroll
                for (int w = 0; w < 8; w++)
                    asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(win[w]) : "v"(nmask[w]), "v"(ring[s][w]), "v"(ring[sc][w]));
                auto lookup = [&](int j) {
                    if constexpr (W == 7) {  // byte0 = 8x (F), byte1 = code, byte2 = B flag of step j (F)
                        const uint32_t sel =
                            0x0C000004u | ((5u + (uint32_t)(j % 3)) << 16) | ((uint32_t)(j & 3) << 8);
                        const uint32_t off = __builtin_amdgcn_perm(F[j / 3], win[j >> 2], sel);
                        // the image's LDS address is a compile-time constant (after the static
                        // top-k buffer, PQ32_IMG7_BASE; the host checks it), so base + 8j is the
                        // instruction's immediate and the address costs the v_perm only
                        typedef const f32x2 __attribute__((address_space(3))) lds_f32x2;
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Wint-to-pointer-cast"  // LDS pointers are 32-bit
                        return *(lds_f32x2 *)(off + (PQ32_IMG7_BASE<E> + 8u * (uint32_t)j));
#pragma clang diagnostic pop
                    }
                    const uint32_t c8 = __builtin_amdgcn_perm(0u, win[j >> 2], 0x0C0C000Cu | ((uint32_t)(j & 3) << 8));
                    const uint32_t off = (c8 << 1) + x8;
                    return *reinterpret_cast<const f32x2 *>(imgb + off + 8 * j);
                };
                if constexpr (W == 2) {  // batch h+1's lookups in flight while batch h is added
                    static_assert(NB <= 15, "lgkmcnt holds at most 15 outstanding LDS reads");
                    constexpr int NH = 32 / NB;
                    f32x2 v[2][NB];
#pragma unroll
                    for (int jj = 0; jj < NB; jj++) v[0][jj] = lookup(jj);
#pragma unroll
                    for (int h = 0; h < NH; h++) {
                        if (h + 1 < NH) {
#pragma unroll
                            for (int jj = 0; jj < NB; jj++) v[(h + 1) & 1][jj] = lookup((h + 1) * NB + jj);
                        }
                        __builtin_amdgcn_sched_barrier(0);
                        if (h + 1 < NH)
                            __builtin_amdgcn_s_waitcnt(0xC07F | (NB << 8));  // lgkmcnt(NB): batch h landed
                        else
                            __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
                        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                        for (int jj = 0; jj < NB; jj++) acc = acc + v[h & 1][jj];
                    }
                } else if constexpr (W == 6) {  // diagnostic: K8c's loads, masks and offers, no lookups
#pragma unroll
                    for (int w = 0; w < 8; w++) acc.x = acc.x + __uint_as_float(win[w] & 0x3F800000u);
                } else if constexpr (W == 4 || W == 5) {  // diagnostics: K8c + 32 extra VALU (4) / SALU (5) per tile
#pragma unroll
                    for (int h = 0; h < 32 / NB; h++) {
                        f32x2 v[NB];
#pragma unroll
                        for (int jj = 0; jj < NB; jj++) v[jj] = lookup(h * NB + jj);
#pragma unroll
                        for (int jj = 0; jj < NB; jj++) {
                            acc = acc + v[jj];
                            if constexpr (W == 4)
                                asm volatile("v_nop");
                            else
                                asm volatile("s_add_u32 %0, %0, 1" : "+s"(dummy));
                        }
                    }
                } else if constexpr (W == 3) {  // A and B as two scalar add chains instead of one packed chain
                    float ax = acc.x, ay = acc.y;
#pragma unroll
                    for (int h = 0; h < 32 / NB; h++) {
                        f32x2 v[NB];
#pragma unroll
                        for (int jj = 0; jj < NB; jj++) v[jj] = lookup(h * NB + jj);
#pragma unroll
                        for (int jj = 0; jj < NB; jj++) {
                            asm("v_add_f32 %0, %1, %2" : "=v"(ax) : "v"(ax), "v"(v[jj].x));
                            asm("v_add_f32 %0, %1, %2" : "=v"(ay) : "v"(ay), "v"(v[jj].y));
                        }
                    }
                    acc = f32x2{ax, ay};
                } else {
#pragma unroll
                    for (int h = 0; h < 32 / NB; h++) {
                        f32x2 v[NB];
#pragma unroll
                        for (int jj = 0; jj < NB; jj++) v[jj] = lookup(h * NB + jj);
                        if constexpr (W == 1) {  // one wait for the whole batch
                            __builtin_amdgcn_sched_barrier(0);
                            __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
                            __builtin_amdgcn_sched_barrier(0);
                        }
#pragma unroll
                        for (int jj = 0; jj < NB; jj++) acc = acc + v[jj];
                    }
                }
                if (i >= 1 && i <= n) {  // offer tile i-1
                    const uint32_t tl = i - 1u;
                    if (s == 1 && (tl & 63u) == 0u && tl != 0u) {  // (R | 64: block starts land on s == 1)
                        mcur = mnxt;
                        mnxt = load_masks((tl >> 6) + 1u);
                    }
                    const uint64_t live = readlane64(mcur, (int)(tl & 63u));
                    const float dist = METRIC == WVG_M_L2 ? acc.x : (METRIC == WVG_M_DOT ? -acc.x : 1.0f - acc.x);
                    tk.offer_dist_fast(dist, (uint32_t)((t0 + tile_of(tl)) * 64u) + (uint32_t)lane, live);
                }
                acc = f32x2{acc.y, 0.0f};
                load(i + (uint32_t)R - 1u, ring[sc]);  // refill: tile i + R - 1
            }
        }
    }
    group_combine_store<E, PQ_SCAN_WAVES>(tk, partials + ((size_t)qi * gridDim.x + blockIdx.x) * a.k);
}
#endif  // WVG_TOOLS

// K8e: K8c's sums and the one-v_perm image (W = 7) with fewer, wider waves.
// A/B on MI355X (profiles/r02/pq_adc/k8e_*.jsonl): letting only 8 or 12 of
// K8c's 16 waves scan made it FASTER (0.526 -> 0.506-0.516 ms per 100M-row
// scan) while the loads-only skeleton did not change with the wave count --
// 16 streams per CU contend, occupancy is not what is missing.  So a
// workgroup here has WV waves (WV = 8: two per SIMD, up to 256 VGPRs each) and
// each wave runs TP independent tile streams (contiguous halves of its range):
// every pass does the lookups of TP tiles in one basic block, so the adds of
// one stream's chain fill the LDS latency of the other's.  Per stream: its own
// buffer resource (loads past its range return zeros), ring of R tiles and
// 64-tile mask blocks; one register top-k per wave.
template <int E, int WV>
constexpr uint32_t PQ32_WIDE_BASE = (uint32_t)WV * 64u * E * 8u;  // LDS address of the image (after sh[WV][64E])

// MB (round 4): the 64-tile live masks come through buffer loads with no
// branch (a lane past its stream reads 0 from the resource bound; no allow
// list: an empty resource) and stay raw until their block starts.  Before,
// the branchy global loads were waited on at once (s_waitcnt vmcnt(0) every
// 64 tiles, draining the wave's code prefetch).
template <int E, int WV, int R, int NB, int TP, int METRIC, bool IL = false, bool COS = false, bool MB = true>
__global__ __launch_bounds__(WV * 64) void scan_pq32_wide_kernel(ScanArgs a, uint64_t *partials)
{
    static_assert(64 % R == 0, "the ring length divides the 64-tile mask block");
    static_assert(32 % NB == 0, "LDS batches divide the 32 steps");
    extern __shared__ __attribute__((aligned(16))) f32x2 img[];  // regions A and B (PQ32_IMG7_*)
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    // COS (co-scheduled PQ batch, a.cosched): a 1D grid of G ranges x nq queries.  Workgroup id ->
    // (range, query) so that the nq queries of one range are consecutive ids on one XCD (ids
    // with equal id % 8): they are resident together and read the same rows side by side, so all
    // but the first read of a line hit the XCD's L2 (the loads keep the default policy).
    uint32_t qi = blockIdx.y, rng = blockIdx.x, G = gridDim.x;
    if constexpr (COS) {
        G = gridDim.x / a.nq;
        const uint32_t kk = blockIdx.x >> 3;
        rng = (kk / a.nq) * 8u + (blockIdx.x & 7u);
        qi = kk % a.nq;
    }
    const float *glut = reinterpret_cast<const float *>(a.queries) + (size_t)qi * a.qpitch;
    constexpr int FILL = 32 * 256 / (WV * 64);
    float fv[FILL];
#pragma unroll
    for (int it = 0; it < FILL; it++) {
        const uint32_t i = (uint32_t)it * (WV * 64) + threadIdx.x;
        fv[it] = glut[(i & 31u) * 256u + (i >> 5)];
    }
    const uint64_t ntiles = a.tile_end - a.tile_begin;
    // IL (A/B, TP = 1): the workgroup owns one contiguous range and its waves
    // take every WV-th tile of it (the CU streams one 16 KiB block at a time)
    static_assert(!IL || TP == 1, "interleaved waves run one stream");
    constexpr uint32_t STRIDE = IL ? WV : 1;  // tiles between a stream's consecutive tiles
    uint64_t s0[TP];
    uint32_t n[TP];
    uint32_t nmax = 0;
    if constexpr (IL) {
        const uint64_t w0 = a.tile_begin + ntiles * rng / G;
        const uint64_t w1 = a.tile_begin + ntiles * (rng + 1) / G;
        s0[0] = w0 + wave;
        n[0] = s0[0] < w1 ? (uint32_t)((w1 - s0[0] + WV - 1) / WV) : 0u;
        nmax = n[0];
    } else {
        const uint64_t total = (uint64_t)G * WV * TP;  // streams of one query
        const uint64_t g0 = ((uint64_t)rng * WV + wave) * TP;
#pragma unroll
        for (int p = 0; p < TP; p++) {
            s0[p] = a.tile_begin + ntiles * (g0 + p) / total;
            n[p] = (uint32_t)(a.tile_begin + ntiles * (g0 + p + 1) / total - s0[p]);
            nmax = n[p] > nmax ? n[p] : nmax;
        }
    }
    auto span = [&](int p) -> uint32_t { return n[p] ? ((n[p] - 1u) * STRIDE + 1u) * 2048u : 0u; };  // bytes
    WaveTopK<E> tk;
    tk.init((int)a.k);
    tk.init_fast();
    {  // (every wave sets up and issues its first loads, so they overlap the image fill)
        __amdgpu_buffer_rsrc_t rs[TP];
#pragma unroll
        for (int p = 0; p < TP; p++)
            rs[p] = __builtin_amdgcn_make_buffer_rsrc(
                const_cast<char *>(reinterpret_cast<const char *>(a.data)) + s0[p] * 2048u, (short)0,
                (int)span(p), 0x00020000);
        const uint32_t voff = (uint32_t)lane * 16u;
        const uint32_t x = (uint32_t)lane & 31u, x8 = x * 8u;
        uint32_t nmask[8];  // bytes of step j taken from the next row (see K8b)
#pragma unroll
        for (int w = 0; w < 8; w++) {
            uint32_t mk = 0u;
#pragma unroll
            for (int bb = 0; bb < 4; bb++) mk |= (4u * w + bb + x >= 32u) ? (0xFFu << (8 * bb)) : 0u;
            nmask[w] = mk;
        }
        uint32_t F[11];  // 8x and the B flags of steps 3k..3k+2 (see PQ32_IMG7_B)
#pragma unroll
        for (int k = 0; k < 11; k++) {
            uint32_t f = x8;
#pragma unroll
            for (int b = 0; b < 3; b++) {
                const uint32_t j = 3u * k + b;
                f |= (j < 32u && x + j >= 32u) ? (1u << (8 * (b + 1))) : 0u;
            }
            F[k] = f;
        }
        const bool rev = a.reverse & 1u;  // pass order: tiles s0 + i, or the stream's last - i
        auto tile_of = [&](int p, uint32_t i) -> uint32_t { return rev ? n[p] - 1u - i : i; };
        auto load = [&](int p, uint32_t i, uint32_t (&w)[8]) {  // the i-th tile of stream p (zeros past it)
            const uint32_t so = i < n[p] ? tile_of(p, i) * (STRIDE * 2048u) : span(p);
            constexpr int POL = COS ? 0 : 2;  // co-scheduled: keep the lines in L2 for the other queries
            const u32x4 lo = __builtin_amdgcn_raw_buffer_load_b128(rs[p], voff, so, POL);
            const u32x4 hi = __builtin_amdgcn_raw_buffer_load_b128(rs[p], voff + 1024u, so, POL);
            w[0] = lo.x; w[1] = lo.y; w[2] = lo.z; w[3] = lo.w;
            w[4] = hi.x; w[5] = hi.y; w[6] = hi.z; w[7] = hi.w;
        };
        auto load_masks = [&](int p, uint32_t b) -> uint64_t {  // lane i: live mask of stream p's (64 b + i)-th tile
            const uint32_t ii = b * 64u + (uint32_t)lane;
            const uint64_t t = s0[p] + (uint64_t)(ii < n[p] ? tile_of(p, ii) : 0u) * STRIDE;
            uint64_t m = 0ull;
            if (ii < n[p]) {
                m = a.valid[t];
                if (a.allow) {
                    const uint64_t wi = t - a.allow_t0;
                    m &= wi < a.allow_words ? a.allow[wi] : 0ull;
                }
            }
            return m;
        };
        // MB: stream p's valid words from a.valid + s0[p], its allow words from a.allow (word t - allow_t0)
        __amdgpu_buffer_rsrc_t vrs[TP], ars[TP];
        const bool has_allow = a.allow != nullptr;
#pragma unroll
        for (int p = 0; p < TP; p++) {
            vrs[p] = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint64_t *>(a.valid + s0[p]), (short)0,
                                                       (int)(span(p) / 256u), 0x00020000);  // span(p) / 2048 * 8
            ars[p] = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint64_t *>(a.allow), (short)0,
                                                       has_allow ? (int)(a.allow_words * 8u) : 0, 0x00020000);
        }
        // raw words of stream p's (64 b + lane)-th tile: valid (.x) and allow (.y, 0 past the list)
        auto load_raw = [&](int p, uint32_t b, uint64_t &v, uint64_t &al) {
            const uint32_t ii = b * 64u + (uint32_t)lane;
            const uint32_t tt = ii < n[p] ? tile_of(p, ii) * STRIDE : 0u;
            const uint32_t vo = ii < n[p] ? tt * 8u : span(p) / 256u;  // past the bound: reads 0
            const uint64_t wi = s0[p] + tt - a.allow_t0;
            const uint32_t ao = (ii < n[p] && wi < a.allow_words) ? (uint32_t)wi * 8u : 0xFFFFFFF0u;
            const u32x2 x = __builtin_amdgcn_raw_buffer_load_b64(vrs[p], vo, 0, 0);
            const u32x2 y = __builtin_amdgcn_raw_buffer_load_b64(ars[p], ao, 0, 0);
            v = ((uint64_t)x.y << 32) | x.x;
            al = ((uint64_t)y.y << 32) | y.x;
        };
        auto live_of = [&](uint64_t v, uint64_t al) -> uint64_t { return has_allow ? v & al : v; };
        uint64_t mcur[TP], mnxt[TP], mnv[TP], mna[TP];
        uint32_t ring[TP][R][8];
        f32x2 acc[TP];
#pragma unroll
        for (int p = 0; p < TP; p++) {
            if constexpr (MB) {
                uint64_t v0, a0;
                load_raw(p, 0, v0, a0);
                mcur[p] = live_of(v0, a0);
                load_raw(p, 1, mnv[p], mna[p]);
                mnxt[p] = 0ull;
            } else {
                mcur[p] = load_masks(p, 0);
                mnxt[p] = load_masks(p, 1);
                mnv[p] = mna[p] = 0ull;
            }
#pragma unroll
            for (int s = 0; s < R - 1; s++) load(p, (uint32_t)s, ring[p][s]);
#pragma unroll
            for (int w = 0; w < 8; w++) ring[p][R - 1][w] = 0u;
            acc[p] = f32x2{0.0f, 0.0f};
        }
#pragma unroll
        for (int it = 0; it < FILL; it++) {
            const uint32_t i = (uint32_t)it * (WV * 64) + threadIdx.x;
            const uint32_t s = i & 31u, c = i >> 5;
            img[c * 32u + s] = f32x2{fv[it], 0.0f};
            img[PQ32_IMG7_B / 8u + c * 32u + s] = f32x2{0.0f, fv[it]};
        }
        __syncthreads();
        typedef const f32x2 __attribute__((address_space(3))) lds_f32x2;
        // pass i finishes tile i-1 and starts tile i of every stream; nmax + 1 passes in groups of R
        if (nmax > 0)
        for (uint32_t base = 0; base <= nmax; base += R) {
#pragma unroll
            for (int s = 0; s < R; s++) {
                const int sc = (s + R - 1) % R;
                const uint32_t i = base + (uint32_t)s;
                uint32_t win[TP][8];
#pragma unroll
                for (int p = 0; p < TP; p++)
#pragma unroll
                    for (int w = 0; w < 8; w++)
                        asm("v_bfi_b32 %0, %1, %2, %3"
                            : "=v"(win[p][w])
                            : "v"(nmask[w]), "v"(ring[p][s][w]), "v"(ring[p][sc][w]));
#pragma unroll
                for (int h = 0; h < 32 / NB; h++) {
                    f32x2 v[TP][NB];
#pragma unroll
                    for (int jj = 0; jj < NB; jj++) {
                        const int j = h * NB + jj;
                        const uint32_t sel =
                            0x0C000004u | ((5u + (uint32_t)(j % 3)) << 16) | ((uint32_t)(j & 3) << 8);
#pragma unroll
                        for (int p = 0; p < TP; p++) {
                            const uint32_t off = __builtin_amdgcn_perm(F[j / 3], win[p][j >> 2], sel);
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Wint-to-pointer-cast"  // LDS pointers are 32-bit
                            v[p][jj] = *(lds_f32x2 *)(off + (PQ32_WIDE_BASE<E, WV> + 8u * (uint32_t)j));
#pragma clang diagnostic pop
                        }
                    }
#pragma unroll
                    for (int jj = 0; jj < NB; jj++)
#pragma unroll
                        for (int p = 0; p < TP; p++) acc[p] = acc[p] + v[p][jj];
                }
                if (i >= 1 && i <= nmax) {  // offer tile i-1 of every stream that has it
                    const uint32_t tl = i - 1u;
                    if (s == 1 && (tl & 63u) == 0u && tl != 0u) {  // (R | 64: block starts land on s == 1)
#pragma unroll
                        for (int p = 0; p < TP; p++) {
                            if constexpr (MB) {
                                mcur[p] = live_of(mnv[p], mna[p]);
                                // (the raw words die before the loads that replace them are issued, so
                                // the loads land in the loop-carried registers: no copy, no wait here)
                                asm volatile("" : "+v"(mcur[p]));
                                load_raw(p, (tl >> 6) + 1u, mnv[p], mna[p]);
                            } else {
                                mcur[p] = mnxt[p];
                                mnxt[p] = load_masks(p, (tl >> 6) + 1u);
                            }
                        }
                    }
#pragma unroll
                    for (int p = 0; p < TP; p++) {
                        if (tl < n[p]) {
                            const uint64_t live = readlane64(mcur[p], (int)(tl & 63u));
                            const float dist = METRIC == WVG_M_L2 ? acc[p].x
                                               : (METRIC == WVG_M_DOT ? -acc[p].x : 1.0f - acc[p].x);
                            tk.offer_dist_fast(
                                dist, (uint32_t)((s0[p] + (uint64_t)tile_of(p, tl) * STRIDE) * 64u) + (uint32_t)lane,
                                live);
                        }
                    }
                }
#pragma unroll
                for (int p = 0; p < TP; p++) {
                    acc[p] = f32x2{acc[p].y, 0.0f};
                    load(p, i + (uint32_t)R - 1u, ring[p][sc]);  // refill: tile i + R - 1
                }
            }
        }
    }
    group_combine_store<E, WV>(tk, partials + ((size_t)qi * G + rng) * a.k);
}

#ifdef WVG_TOOLS
// K8d (tools build): K8c with the R passes of a ring cycle in ONE basic block.  K8c's
// per-tile offer is a branch, so the compiler schedules every pass on its
// own and the tail of a pass (its last adds waiting on LDS) cannot overlap
// the head of the next (its byte merges and first LDS reads).  Here a pass
// only records its distance and the cheap float filter's verdict (a scalar
// OR); the exact offers of the cycle's R tiles run after the cycle when any
// lane passed, in tile order (a stale, larger tau_f only lets more lanes
// through to the exact test).  Tile masks come R per vector load, one cycle
// ahead (lane l = the l-th tile offered in the cycle).  GL: codes through
// global loads with a scalar tile base (saddr) instead of buffer loads.
template <int E, int R, int NB, int METRIC, bool GL>
__global__ __launch_bounds__(PQ_SCAN_WAVES * 64) void scan_pq32_cycle_kernel(ScanArgs a, uint64_t *partials)
{
    extern __shared__ __attribute__((aligned(16))) f32x2 img[];  // [256][64]
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t qi = blockIdx.y;
    const float *glut = reinterpret_cast<const float *>(a.queries) + (size_t)qi * a.qpitch;
    constexpr int FILL = 32 * 256 / (PQ_SCAN_WAVES * 64);
    float fv[FILL];
#pragma unroll
    for (int it = 0; it < FILL; it++) {
        const uint32_t i = (uint32_t)it * (PQ_SCAN_WAVES * 64) + threadIdx.x;
        fv[it] = glut[(i & 31u) * 256u + (i >> 5)];
    }
#pragma unroll
    for (int it = 0; it < FILL; it++) {
        const uint32_t i = (uint32_t)it * (PQ_SCAN_WAVES * 64) + threadIdx.x;
        const uint32_t s = i & 31u, c = i >> 5;
        img[c * 64u + s] = f32x2{fv[it], 0.0f};
        img[c * 64u + 32u + s] = f32x2{0.0f, fv[it]};
    }
    __syncthreads();
    const uint64_t ntiles = a.tile_end - a.tile_begin;
    const uint64_t total = (uint64_t)gridDim.x * PQ_SCAN_WAVES;
    const uint64_t gw = (uint64_t)blockIdx.x * PQ_SCAN_WAVES + wave;
    const uint64_t t0 = a.tile_begin + ntiles * gw / total, t1 = a.tile_begin + ntiles * (gw + 1) / total;
    WaveTopK<E> tk;
    tk.init((int)a.k);
    tk.init_fast();
    if (t0 < t1) {
        const uint32_t n = (uint32_t)(t1 - t0);
        const char *wbase = reinterpret_cast<const char *>(a.data) + t0 * 2048u;
        const __amdgpu_buffer_rsrc_t rs =
            __builtin_amdgcn_make_buffer_rsrc(const_cast<char *>(wbase), (short)0, (int)(n * 2048u), 0x00020000);
        const uint32_t voff = (uint32_t)lane * 16u;
        const uint32_t x = (uint32_t)lane & 31u, x8 = x * 8u;
        uint32_t nmask[8];
#pragma unroll
        for (int w = 0; w < 8; w++) {
            uint32_t mk = 0u;
#pragma unroll
            for (int bb = 0; bb < 4; bb++) mk |= (4u * w + bb + x >= 32u) ? (0xFFu << (8 * bb)) : 0u;
            nmask[w] = mk;
        }
        const char *imgb = reinterpret_cast<const char *>(img);
        const bool rev = a.reverse & 1u;
        auto tile_of = [&](uint32_t i) -> uint32_t { return rev ? n - 1u - i : i; };
        auto load = [&](uint32_t i, uint32_t (&w)[8]) {
            u32x4 lo, hi;
            if constexpr (GL) {
                const char *tb = wbase + (size_t)tile_of(i < n ? i : 0u) * 2048u;  // past the range: re-read
                lo = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(tb + voff));
                hi = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(tb + voff + 1024u));
            } else {
                const uint32_t so = i < n ? tile_of(i) * 2048u : n * 2048u;  // past the range: zeros
                lo = __builtin_amdgcn_raw_buffer_load_b128(rs, voff, so, 2);
                hi = __builtin_amdgcn_raw_buffer_load_b128(rs, voff + 1024u, so, 2);
            }
            w[0] = lo.x; w[1] = lo.y; w[2] = lo.z; w[3] = lo.w;
            w[4] = hi.x; w[5] = hi.y; w[6] = hi.z; w[7] = hi.w;
        };
        // lane l < R: live mask of the tile offered by pass l of the cycle at
        // `base` (pass order index base - 1 + l; none for index -1 or >= n)
        auto cycle_masks = [&](uint32_t base) -> uint64_t {
            const uint32_t ii = base + (uint32_t)lane - 1u;
            uint64_t m = 0ull;
            if (lane < R && base + (uint32_t)lane >= 1u && ii < n) {
                const uint64_t t = t0 + tile_of(ii);
                m = a.valid[t];
                if (a.allow) {
                    const uint64_t wi = t - a.allow_t0;
                    m &= wi < a.allow_words ? a.allow[wi] : 0ull;
                }
            }
            return m;
        };
        uint64_t mg = cycle_masks(0), mgn = cycle_masks(R);
        uint32_t ring[R][8];
#pragma unroll
        for (int s = 0; s < R - 1; s++) load((uint32_t)s, ring[s]);
#pragma unroll
        for (int w = 0; w < 8; w++) ring[R - 1][w] = 0u;
        f32x2 acc = {0.0f, 0.0f};
        for (uint32_t base = 0; base <= n; base += R) {
            float dist[R];
            uint64_t pending = 0ull;
            const uint64_t open = tk.tau_open ? ~0ull : 0ull;  // list not full yet: every live lane (no branch)
            const float tf = tk.tau_f;
#pragma unroll
            for (int s = 0; s < R; s++) {
                const int sc = (s + R - 1) % R;
                const uint32_t i = base + (uint32_t)s;
                uint32_t win[8];
#pragma unroll
                for (int w = 0; w < 8; w++)
                    asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(win[w]) : "v"(nmask[w]), "v"(ring[s][w]), "v"(ring[sc][w]));
#pragma unroll
                for (int h = 0; h < 32 / NB; h++) {
                    f32x2 v[NB];
#pragma unroll
                    for (int jj = 0; jj < NB; jj++) {
                        const int j = h * NB + jj;
                        const uint32_t c8 = __builtin_amdgcn_perm(0u, win[j >> 2], 0x0C0C000Cu | ((uint32_t)(j & 3) << 8));
                        const uint32_t off = (c8 << 1) + x8;
                        v[jj] = *reinterpret_cast<const f32x2 *>(imgb + off + 8 * j);
                    }
#pragma unroll
                    for (int jj = 0; jj < NB; jj++) acc = acc + v[jj];
                }
                dist[s] = METRIC == WVG_M_L2 ? acc.x : (METRIC == WVG_M_DOT ? -acc.x : 1.0f - acc.x);
                const uint64_t live = readlane64(mg, s);
                pending |= (__ballot(dist[s] <= tf) | open) & live;
                acc = f32x2{acc.y, 0.0f};
                load(i + (uint32_t)R - 1u, ring[sc]);
            }
            if (pending) {  // exact offers of this cycle's tiles, in order
#pragma unroll
                for (int s = 0; s < R; s++) {
                    const uint64_t live = readlane64(mg, s);
                    if (live) {
                        const uint32_t tl = base + (uint32_t)s - 1u;
                        tk.offer_dist_fast(dist[s], (uint32_t)((t0 + tile_of(tl)) * 64u) + (uint32_t)lane, live);
                    }
                }
            }
            mg = mgn;
            mgn = cycle_masks(base + 2u * R);
        }
    }
    group_combine_store<E, PQ_SCAN_WAVES>(tk, partials + ((size_t)qi * gridDim.x + blockIdx.x) * a.k);
}

template <int E, int R, int NB, bool GL>
static void launch_pq_cycle(const ScanArgs &a, uint64_t *partials, dim3 grid, dim3 block, size_t lds, hipStream_t s)
{
    if (a.metric == WVG_M_L2 || a.metric == WVG_M_MANHATTAN || a.metric == WVG_M_HAMMING)  // Wrap = identity
        launch_timed((scan_pq32_cycle_kernel<E, R, NB, WVG_M_L2, GL>), grid, block, lds, s, a, partials);
    else if (a.metric == WVG_M_DOT)
        launch_timed((scan_pq32_cycle_kernel<E, R, NB, WVG_M_DOT, GL>), grid, block, lds, s, a, partials);
    else
        launch_timed((scan_pq32_cycle_kernel<E, R, NB, WVG_M_COSINE, GL>), grid, block, lds, s, a, partials);
}

template <int E, int R, int NB, int W = 0, int ACT = PQ_SCAN_WAVES>
static void launch_pq_dense(const ScanArgs &a, uint64_t *partials, dim3 grid, dim3 block, size_t lds, hipStream_t s)
{
    if (a.metric == WVG_M_L2 || a.metric == WVG_M_MANHATTAN || a.metric == WVG_M_HAMMING)  // Wrap = identity
        launch_timed((scan_pq32_dense_kernel<E, R, NB, WVG_M_L2, W, ACT>), grid, block, lds, s, a, partials);
    else if (a.metric == WVG_M_DOT)
        launch_timed((scan_pq32_dense_kernel<E, R, NB, WVG_M_DOT, W, ACT>), grid, block, lds, s, a, partials);
    else
        launch_timed((scan_pq32_dense_kernel<E, R, NB, WVG_M_COSINE, W, ACT>), grid, block, lds, s, a, partials);
}

// W = 7 reads its image at the compile-time LDS address PQ32_IMG7_BASE<E>: use
// it only where the static LDS really ends there and image + top-k buffer fit
// the CU's 160 KiB (not for E = 4); otherwise variants 29-31 fall through to K8b
template <int E>
static bool img7_ok()
{
    static const bool ok = [] {
        if (PQ32_IMG7_BASE<E> + PQ32_IMG7_BYTES > 160u * 1024u) return false;
        hipFuncAttributes fa{};
        if (hipFuncGetAttributes(&fa, reinterpret_cast<const void *>(&scan_pq32_dense_kernel<E, 8, 16, WVG_M_L2, 7>)) !=
            hipSuccess)
            return false;
        return fa.sharedSizeBytes == PQ32_IMG7_BASE<E>;
    }();
    return ok;
}
#endif  // WVG_TOOLS

// K8e reads its image at the compile-time LDS address PQ32_WIDE_BASE: the
// host launches an instantiation only where the static LDS really ends there
template <int E, int WV, int R, int NB, int TP, bool IL = false, bool COS = false, bool MB = true>
static bool wide_ok()
{
    static const bool ok = [] {
        if (PQ32_WIDE_BASE<E, WV> + PQ32_IMG7_BYTES > 160u * 1024u) return false;
        hipFuncAttributes fa{};
        if (hipFuncGetAttributes(&fa, reinterpret_cast<const void *>(
                                          &scan_pq32_wide_kernel<E, WV, R, NB, TP, WVG_M_L2, IL, COS, MB>)) != hipSuccess)
            return false;
        return fa.sharedSizeBytes == PQ32_WIDE_BASE<E, WV>;
    }();
    return ok;
}

template <int E, int WV, int R, int NB, int TP, bool IL = false, bool COS = false, bool MB = true>
static bool launch_pq_wide(const ScanArgs &a, uint64_t *partials, int groups, hipStream_t s)
{
    if (!wide_ok<E, WV, R, NB, TP, IL, COS, MB>()) return false;
    const dim3 grid = COS ? dim3((unsigned)groups * a.nq) : dim3(groups, a.nq), block(WV * 64);
    const uint32_t lds = PQ32_IMG7_BYTES;
    if (a.metric == WVG_M_L2 || a.metric == WVG_M_MANHATTAN || a.metric == WVG_M_HAMMING)  // Wrap = identity
        launch_timed((scan_pq32_wide_kernel<E, WV, R, NB, TP, WVG_M_L2, IL, COS, MB>), grid, block, lds, s, a, partials);
    else if (a.metric == WVG_M_DOT)
        launch_timed((scan_pq32_wide_kernel<E, WV, R, NB, TP, WVG_M_DOT, IL, COS, MB>), grid, block, lds, s, a, partials);
    else
        launch_timed((scan_pq32_wide_kernel<E, WV, R, NB, TP, WVG_M_COSINE, IL, COS, MB>), grid, block, lds, s, a, partials);
    return true;
}

template <int E>
static hipError_t launch_pq_e(const ScanArgs &a, uint64_t *partials, int groups, hipStream_t s);

#ifdef WVG_TOOLS
// Tools build: every A/B and diagnostic variant (tuning key 7; variants 24-28
// and 34 are diagnostics whose results are NOT distances).
template <int E>
static hipError_t launch_pq_e_variant(const ScanArgs &a, uint64_t *partials, int groups, hipStream_t s)
{
    dim3 grid(groups, a.nq), block(PQ_SCAN_WAVES * 64);
    const size_t lds = (size_t)a.pq_m * a.pq_ks * 4;
    const int v = tuning().pq_variant;
    const bool m32 = a.pq_ks == 256 && a.pq_m == 32 && a.nchunks == 2;
    if (m32 && v >= 14 && v <= 17) {
        // K8d (one basic block per ring cycle): 14 = ring 8 / LDS batches of 8, 15 = ring 4 / 16,
        // 16 = ring 8 / 8 with global loads, 17 = ring 4 / 16 with global loads
        if (v == 14) launch_pq_cycle<E, 8, 8, false>(a, partials, grid, block, 4 * lds, s);
        else if (v == 15) launch_pq_cycle<E, 4, 16, false>(a, partials, grid, block, 4 * lds, s);
        else if (v == 16) launch_pq_cycle<E, 8, 8, true>(a, partials, grid, block, 4 * lds, s);
        else launch_pq_cycle<E, 4, 16, true>(a, partials, grid, block, 4 * lds, s);
        return hipGetLastError();
    }
    if (m32 && v >= 18 && v <= 28) {
        // K8c LDS wait patterns: 18 = one wait per batch of 16, 19 = per batch of 32,
        // 20 = pipelined batches of 8, 21 = one wait per batch of 8;
        // 22 / 23 = scalar A and B add chains, batches of 16 / 8; 24 / 25 = diagnostics (+32 VALU / SALU per
        // tile); 26 / 27 / 28 = diagnostic: loads, masks and offers only (results are not distances), ring 8 / 4 / 2
        if (v == 18) launch_pq_dense<E, 8, 16, 1>(a, partials, grid, block, 4 * lds, s);
        else if (v == 19) launch_pq_dense<E, 8, 32, 1>(a, partials, grid, block, 4 * lds, s);
        else if (v == 20) launch_pq_dense<E, 8, 8, 2>(a, partials, grid, block, 4 * lds, s);
        else if (v == 21) launch_pq_dense<E, 8, 8, 1>(a, partials, grid, block, 4 * lds, s);
        else if (v == 22) launch_pq_dense<E, 8, 16, 3>(a, partials, grid, block, 4 * lds, s);
        else if (v == 23) launch_pq_dense<E, 8, 8, 3>(a, partials, grid, block, 4 * lds, s);
        else if (v == 24) launch_pq_dense<E, 8, 16, 4>(a, partials, grid, block, 4 * lds, s);
        else if (v == 25) launch_pq_dense<E, 8, 16, 5>(a, partials, grid, block, 4 * lds, s);
        else if (v == 26) launch_pq_dense<E, 8, 16, 6>(a, partials, grid, block, 4 * lds, s);
        else if (v == 27) launch_pq_dense<E, 4, 16, 6>(a, partials, grid, block, 4 * lds, s);
        else launch_pq_dense<E, 2, 16, 6>(a, partials, grid, block, 4 * lds, s);
        return hipGetLastError();
    }
    if (m32 && v >= 50 && v <= 56) {
        // K8e mask-load A/B (round 4): 50 = the round-3 product (8 waves, ring 4 / 16, branchy mask
        // loads waited at once); MB (buffered raw masks): 51 = ring 4, 52 = ring 8, 53 = ring 16,
        // 54 = 4 waves, ring 16; round 5: 55 = 16 waves, ring 4; 56 = 16 waves, ring 2
        bool ok;
        if (v == 50) ok = launch_pq_wide<E, 8, 4, 16, 1, false, false, false>(a, partials, groups, s);
        else if (v == 51) ok = launch_pq_wide<E, 8, 4, 16, 1>(a, partials, groups, s);
        else if (v == 52) ok = launch_pq_wide<E, 8, 8, 16, 1>(a, partials, groups, s);
        else if (v == 53) ok = launch_pq_wide<E, 8, 16, 16, 1>(a, partials, groups, s);
        else if (v == 55) ok = launch_pq_wide<E, 16, 4, 16, 1>(a, partials, groups, s);
        else if (v == 56) ok = launch_pq_wide<E, 16, 2, 16, 1>(a, partials, groups, s);
        else ok = launch_pq_wide<E, 4, 16, 16, 1>(a, partials, groups, s);
        if (ok) return hipGetLastError();
    }
    if (m32 && (v == 46 || v == 47)) {  // K8e with interleaved waves (IL): 46 = 8 waves, ring 4 / 16; 47 = ring 8 / 16
        if (v == 46 ? launch_pq_wide<E, 8, 4, 16, 1, true>(a, partials, groups, s)
                    : launch_pq_wide<E, 8, 8, 16, 1, true>(a, partials, groups, s))
            return hipGetLastError();
    }
    if (m32 && (v == 44 || v == 45)) {  // K8e 8 waves, 1 stream, ring 4, LDS batches of 8 / 32
        if (v == 44 ? launch_pq_wide<E, 8, 4, 8, 1>(a, partials, groups, s)
                    : launch_pq_wide<E, 8, 4, 32, 1>(a, partials, groups, s))
            return hipGetLastError();
    }
    if (m32 && v >= 40 && v <= 43) {
        // K8e: 40 = 8 waves, 1 stream, ring 4 / 16; 41 = 8 waves, 1 stream, ring 2 / 16;
        // 42 = 8 waves, 2 streams, ring 2 / 16; 43 = 8 waves, 2 streams, ring 2 / 8
        bool ok;
        if (v == 40) ok = launch_pq_wide<E, 8, 4, 16, 1>(a, partials, groups, s);
        else if (v == 41) ok = launch_pq_wide<E, 8, 2, 16, 1>(a, partials, groups, s);
        else if (v == 42) ok = launch_pq_wide<E, 8, 2, 16, 2>(a, partials, groups, s);
        else ok = launch_pq_wide<E, 8, 2, 8, 2>(a, partials, groups, s);
        if (ok) return hipGetLastError();
    }
    if (m32 && v >= 35 && v <= 39) {
        // K8e (WV waves, TP streams per wave): 35 = 8 waves, 1 stream, ring 8 / LDS batches of 16;
        // 36 = 8 waves, 2 streams, ring 4 / 8; 37 = 8 waves, 2 streams, ring 4 / 16;
        // 38 = 4 waves, 2 streams, ring 8 / 16; 39 = 8 waves, 1 stream, ring 16 / 16
        bool ok;
        if (v == 35) ok = launch_pq_wide<E, 8, 8, 16, 1>(a, partials, groups, s);
        else if (v == 36) ok = launch_pq_wide<E, 8, 4, 8, 2>(a, partials, groups, s);
        else if (v == 37) ok = launch_pq_wide<E, 8, 4, 16, 2>(a, partials, groups, s);
        else if (v == 38) ok = launch_pq_wide<E, 4, 8, 16, 2>(a, partials, groups, s);
        else ok = launch_pq_wide<E, 8, 16, 16, 1>(a, partials, groups, s);
        if (ok) return hipGetLastError();
    }
    if (m32 && v == 34) {  // diagnostic: the K8c skeleton (variant 26) with 8 of the 16 waves scanning
        launch_pq_dense<E, 8, 16, 6, 8>(a, partials, grid, block, 4 * lds, s);
        return hipGetLastError();
    }
    if (m32 && v >= 29 && v <= 33 && img7_ok<E>()) {
        // K8c with one-v_perm lookup addresses (W = 7): 29 = ring 8 / LDS batches of 16, 30 = 8 / 8, 31 = 4 / 16;
        // 32 / 33 = 31 with 8 / 12 of the 16 waves scanning (diagnostic: 2 / 3 waves per SIMD)
        if (v == 29) launch_pq_dense<E, 8, 16, 7>(a, partials, grid, block, PQ32_IMG7_BYTES, s);
        else if (v == 30) launch_pq_dense<E, 8, 8, 7>(a, partials, grid, block, PQ32_IMG7_BYTES, s);
        else if (v == 32) launch_pq_dense<E, 4, 16, 7, 8>(a, partials, grid, block, PQ32_IMG7_BYTES, s);
        else if (v == 33) launch_pq_dense<E, 4, 16, 7, 12>(a, partials, grid, block, PQ32_IMG7_BYTES, s);
        else launch_pq_dense<E, 4, 16, 7>(a, partials, grid, block, PQ32_IMG7_BYTES, s);
        return hipGetLastError();
    }
    // the default for m = 32, ks = 256 on mostly-live corpora without an allow list: K8e (8 waves, ring 4);
    // batches (a.cosched, groups % 8 == 0): co-scheduled over one range per XCD, 16 waves per CU
    // (0.338 ms per query of a 16-query batch at 100M codes vs 0.375 with 8 waves; 8 when the 16-wave
    // top-k buffer and the image exceed the LDS, E = 4)
    if (m32 && v == 0 && a.dense && a.cosched && groups % 8 == 0 &&
        (launch_pq_wide<E, 16, 4, 16, 1, false, true>(a, partials, groups, s) ||
         launch_pq_wide<E, 8, 4, 16, 1, false, true>(a, partials, groups, s)))
        return hipGetLastError();
    if (m32 && v == 0 && a.dense && launch_pq_wide<E, 8, 4, 16, 1>(a, partials, groups, s)) return hipGetLastError();
    if (m32 && (v == 48 || v == 49) && a.dense && a.cosched && groups % 8 == 0) {
        // A/B: co-scheduled batches with 16 waves per CU (the L2 serves most reads, so the
        // 16-wave contention of K8c may no longer bind): 48 = ring 4, 49 = ring 8
        if (v == 48 ? launch_pq_wide<E, 16, 4, 16, 1, false, true>(a, partials, groups, s)
                    : launch_pq_wide<E, 16, 8, 16, 1, false, true>(a, partials, groups, s))
            return hipGetLastError();
    }
    if (m32 && (v == 10 || v == 11 || v == 12 || (v == 0 && a.dense))) {
        // K8c (dense, issue-trimmed): 0 (auto) / 12 = ring 8 / LDS batches of 16, 10 = ring 8 / 8, 11 = ring 4 / 16
        if (v == 11)
            launch_pq_dense<E, 4, 16>(a, partials, grid, block, 4 * lds, s);
        else if (v == 10)
            launch_pq_dense<E, 8, 8>(a, partials, grid, block, 4 * lds, s);
        else
            launch_pq_dense<E, 8, 16>(a, partials, grid, block, 4 * lds, s);
        return hipGetLastError();
    }
    if (m32 && v != 1) {  // K8b: skips dead / disallowed tiles (0 = auto without K8c's conditions, 13 = forced)
        // 128 KiB LUT image; variant 0 = ring 6, per-wave ranges, LDS reads in batches of 16
        // (A/B: 2 = ring 4, 3 = ring 4 interleaved, 4 = batches of 32, 5 = batches of 8)
        switch (tuning().pq_variant) {
        case 6: launch_timed((scan_pq32_rot_kernel<E, 6, false, 16, 1>), grid, block, 4 * lds, s, a, partials); break;
        case 7: launch_timed((scan_pq32_rot_kernel<E, 6, false, 16, 2>), grid, block, 4 * lds, s, a, partials); break;
        case 8: launch_timed((scan_pq32_rot_kernel<E, 4, false, 16, 1>), grid, block, 4 * lds, s, a, partials); break;
        case 9: launch_timed((scan_pq32_rot_kernel<E, 8, false, 16, 1>), grid, block, 4 * lds, s, a, partials); break;
        case 2: launch_timed((scan_pq32_rot_kernel<E, 4, false, 16>), grid, block, 4 * lds, s, a, partials); break;
        case 3: launch_timed((scan_pq32_rot_kernel<E, 4, true, 16>), grid, block, 4 * lds, s, a, partials); break;
        case 4: launch_timed((scan_pq32_rot_kernel<E, 6, false, 32>), grid, block, 4 * lds, s, a, partials); break;
        case 5: launch_timed((scan_pq32_rot_kernel<E, 6, false, 8>), grid, block, 4 * lds, s, a, partials); break;
        default: launch_timed((scan_pq32_rot_kernel<E, 6, false, 16>), grid, block, 4 * lds, s, a, partials); break;
        }
        return hipGetLastError();
    }
    if (a.pq_ks == 256) {
        switch (a.pq_m) {
        case 8: launch_timed((scan_pq_kernel<E, 8, 256>), grid, block, lds, s, a, partials); return hipGetLastError();
        case 16: launch_timed((scan_pq_kernel<E, 16, 256>), grid, block, lds, s, a, partials); return hipGetLastError();
        case 32: launch_timed((scan_pq_kernel<E, 32, 256>), grid, block, lds, s, a, partials); return hipGetLastError();
        case 64: launch_timed((scan_pq_kernel<E, 64, 256>), grid, block, lds, s, a, partials); return hipGetLastError();
        default: break;
        }
    }
    launch_timed((scan_pq_kernel<E, 0, 0>), grid, block, lds, s, a, partials);
    return hipGetLastError();
}
#endif  // WVG_TOOLS

// The product's ADC scan choice.  m = 32, ks = 256 (the rotated layout):
//   - a co-scheduled batch (a.cosched: nq > 1, dense, no allow list): K8e COS,
//     16 waves per CU (8 when the image and the E = 4 top-k buffer exceed the LDS);
//   - a dense corpus (>= 3/4 of the slots live, no allow list): K8e, 8 waves;
//   - otherwise (allow lists, many deletes -- dead tiles are skipped), and
//     wherever K8e's compile-time LDS layout check fails: K8b;
// any other (m, ks): K8, the LUT in LDS in segment order.
template <int E>
static hipError_t launch_pq_e(const ScanArgs &a, uint64_t *partials, int groups, hipStream_t s)
{
#ifdef WVG_TOOLS
    if (tuning().pq_variant != 0) return launch_pq_e_variant<E>(a, partials, groups, s);
#endif
    dim3 grid(groups, a.nq), block(PQ_SCAN_WAVES * 64);
    const size_t lds = (size_t)a.pq_m * a.pq_ks * 4;
    const bool m32 = a.pq_ks == 256 && a.pq_m == 32 && a.nchunks == 2;
    if (m32 && a.dense && a.cosched && groups % 8 == 0 &&
        (launch_pq_wide<E, 16, 4, 16, 1, false, true>(a, partials, groups, s) ||
         launch_pq_wide<E, 8, 4, 16, 1, false, true>(a, partials, groups, s)))
        return hipGetLastError();
    if (m32 && a.dense && launch_pq_wide<E, 8, 4, 16, 1>(a, partials, groups, s)) return hipGetLastError();
    if (m32) {
        launch_timed((scan_pq32_rot_kernel<E, 6, false, 16>), grid, block, 4 * lds, s, a, partials);
        return hipGetLastError();
    }
    if (a.pq_ks == 256) {
        switch (a.pq_m) {
        case 8: launch_timed((scan_pq_kernel<E, 8, 256>), grid, block, lds, s, a, partials); return hipGetLastError();
        case 16: launch_timed((scan_pq_kernel<E, 16, 256>), grid, block, lds, s, a, partials); return hipGetLastError();
        case 32: launch_timed((scan_pq_kernel<E, 32, 256>), grid, block, lds, s, a, partials); return hipGetLastError();
        case 64: launch_timed((scan_pq_kernel<E, 64, 256>), grid, block, lds, s, a, partials); return hipGetLastError();
        default: break;
        }
    }
    launch_timed((scan_pq_kernel<E, 0, 0>), grid, block, lds, s, a, partials);
    return hipGetLastError();
}

hipError_t launch_scan_pq(const ScanArgs &a, uint64_t *partials, int groups, hipStream_t s)
{
    if ((size_t)a.pq_m * a.pq_ks * 4 > 160 * 1024) return hipErrorInvalidValue;
    if (a.k <= 64) return launch_pq_e<1>(a, partials, groups, s);
    if (a.k <= 128) return launch_pq_e<2>(a, partials, groups, s);
    return launch_pq_e<4>(a, partials, groups, s);
}

__global__ void pq_adc_rows_kernel(int metric, const float *lut, uint32_t m, uint32_t ks, const uint8_t *codes,
                                   uint64_t n, float *out)
{
    const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    const uint8_t *c = codes + r * m;
    float sum = 0.0f;
    for (uint32_t i = 0; i < m; i++) sum = sum + lut[(size_t)i * ks + c[i]];
    out[r] = wrap_metric(metric, sum);
}

hipError_t launch_pq_adc_rows(int metric, const float *lut, uint32_t m, uint32_t ks, const uint8_t *codes, uint64_t n,
                              float *out, hipStream_t s)
{
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(pq_adc_rows_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, metric, lut, m, ks,
                       codes, n, out);
    return hipGetLastError();
}

}  // namespace wvg

// ---------------------------------------------------------------------------
// K10: k-means training (KMeans.Fit, CH/kmeans.go:220-250) -- every segment's
// Lloyd loop of ProductQuantizer.Fit (CH/product_quantization.go:372-418) in
// one set of launches per iteration; the host runs the loop control and the
// rare empty-cluster reseed (kmeans.go:177-198).
// ---------------------------------------------------------------------------
namespace wvg {

// One Lloyd pass:
//   assignment = K9 (pq_encode_kernel: nNearest, kmeans.go:103-135, the same
//                rule as the encoder, over a tiled copy of the training rows),
//   kmeans_count_kernel   (changes per segment, cluster sizes, points updated),
//   kmeans_members_kernel (per segment, a stable counting sort of the rows by
//                          cluster: member lists in ascending row order),
//   kmeans_sum_kernel     (one thread per (segment, cluster, dim): the
//                          reference's sequential fp32 sum over the members).
// Points are kept segment-major [m][n].  (Round 2's assign kernel -- one
// thread per (row, segment), centroids from global memory, a global atomic per
// row -- sat 96 % of its wave cycles parked: 8.45 ms per pass at 100k x 128;
// its recalc scanned all n rows per output: 5.56 ms.)

// The pair-interleaved copy of a [m][ks][4] codebook that K9's ds = 4 path
// reads right after the table (pq_pair_layout on the device).
__global__ __launch_bounds__(256) void pq_pairs_kernel(const float *centers, uint32_t m, uint32_t ks, float *out,
                                                       uint32_t *seg_nan)
{
    // workgroup = segment blockIdx.x; element i = (p, k, h) of its ks * 4
    const uint32_t sg = blockIdx.x;
    bool nan = false;
    for (uint32_t i = threadIdx.x; i < ks * 4u; i += 256u) {
        const uint32_t h = i & 1u, k = (i >> 1) & 3u, pr = i >> 3;
        const float v = centers[((size_t)sg * ks + 2 * pr + h) * 4 + k];
        out[(size_t)sg * ks * 4 + i] = v;
        nan |= v != v;
    }
    const int any = __syncthreads_or(nan);
    if (seg_nan && threadIdx.x == 0) seg_nan[sg] = any ? 1u : 0u;
}

hipError_t launch_pq_pairs(const float *centers, uint32_t m, uint32_t ks, float *out, hipStream_t s, uint32_t *seg_nan)
{
    hipLaunchKernelGGL(pq_pairs_kernel, dim3(m), dim3(256), 0, s, centers, m, ks, out, seg_nan);
    return hipGetLastError();
}

// Row blocks of the count / member kernels: at least 4096 rows, at most
// KM_BLOCKS per segment (the member kernel sums the block histograms before
// its own serially).
constexpr uint32_t KM_BLOCKS = 64;
uint64_t kmeans_rows_per(uint64_t n)
{
    const uint64_t r = (n + KM_BLOCKS - 1) / KM_BLOCKS;
    return std::max<uint64_t>(4096, (r + 255) / 256 * 256);
}
uint32_t kmeans_blocks(uint64_t n) { return (uint32_t)((n + kmeans_rows_per(n) - 1) / kmeans_rows_per(n)); }

// Block (s, b): rows [b * rows_per, (b + 1) * rows_per) of an active segment s;
// its cluster histogram also goes to bhist[s][b] (the member kernel's bases).
__global__ __launch_bounds__(256) void kmeans_count_kernel(const uint8_t *codes, uint64_t n, uint32_t m, uint32_t ks,
                                                           const uint8_t *active, uint8_t *points, uint32_t *changes,
                                                           uint32_t *counts, uint64_t rows_per, uint32_t *bhist)
{
    __shared__ uint32_t hist[256];
    __shared__ uint32_t chg;
    const uint32_t sg = blockIdx.x;
    if (!active[sg]) return;
    hist[threadIdx.x] = 0;
    if (threadIdx.x == 0) chg = 0;
    __syncthreads();
    const uint64_t p0 = (uint64_t)blockIdx.y * rows_per, p1 = min(n, p0 + rows_per);
    uint32_t mine = 0;
    for (uint64_t p = p0 + threadIdx.x; p < p1; p += 256) {
        const uint8_t c = codes[p * m + sg];
        uint8_t *pp = points + (size_t)sg * n + p;
        if (*pp != c) {
            *pp = c;
            mine++;
        }
        atomicAdd(&hist[c], 1u);
    }
    atomicAdd(&chg, mine);
    __syncthreads();
    for (uint32_t c = threadIdx.x; c < ks; c += 256) {
        if (hist[c]) atomicAdd(&counts[(size_t)sg * ks + c], hist[c]);
        bhist[((size_t)sg * gridDim.y + blockIdx.y) * ks + c] = hist[c];
    }
    if (threadIdx.x == 0 && chg) atomicAdd(&changes[sg], chg);
}

hipError_t launch_kmeans_count(const uint8_t *codes, uint64_t n, uint32_t m, uint32_t ks, const uint8_t *active,
                               uint8_t *points, uint32_t *changes, uint32_t *counts, uint32_t *bhist, hipStream_t s)
{
    hipLaunchKernelGGL(kmeans_count_kernel, dim3(m, kmeans_blocks(n)), dim3(256), 0, s, codes, n, m, ks, active,
                       points, changes, counts, kmeans_rows_per(n), bhist);
    return hipGetLastError();
}

// Block (s, b) per recalculated segment s and row block b (the count
// kernel's): a cluster's base = its offset (exclusive prefix of the cluster
// sizes, an LDS scan) + its rows in the earlier blocks (bhist); then the
// block's rows in 256-row chunks: a row's place = its cluster's running base +
// the same-cluster rows of earlier waves of the chunk + those of lower lanes
// of its own wave (an 8-ballot match), so every member list is in ascending
// row order.  (Round 3 first had one block per segment walking all n rows
// with a serial prefix: 324 us per pass at 100k rows.)
__global__ __launch_bounds__(256) void kmeans_members_kernel(const uint8_t *points, uint64_t n, uint32_t ks,
                                                             const uint32_t *counts, const uint32_t *bhist,
                                                             uint64_t rows_per, const uint8_t *recalc,
                                                             uint32_t *members, uint32_t *offsets)
{
    __shared__ uint32_t base[256];
    __shared__ uint32_t wcnt[4][256];
    const uint32_t sg = blockIdx.x, b = blockIdx.y;
    if (!recalc[sg]) return;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const uint32_t own = (uint32_t)tid < ks ? counts[(size_t)sg * ks + tid] : 0u;
    uint32_t earlier = 0;
    if ((uint32_t)tid < ks)
        for (uint32_t bb = 0; bb < b; bb++) earlier += bhist[((size_t)sg * gridDim.y + bb) * ks + tid];
    // inclusive scan of `own` over the 256 threads (Hillis-Steele in LDS)
    base[tid] = own;
    __syncthreads();
    for (int d = 1; d < 256; d <<= 1) {
        const uint32_t v = tid >= d ? base[tid - d] : 0u;
        __syncthreads();
        base[tid] += v;
        __syncthreads();
    }
    const uint32_t off = base[tid] - own;
    __syncthreads();
    if ((uint32_t)tid < ks) {
        if (b == 0) offsets[(size_t)sg * ks + tid] = off;
        base[tid] = off + earlier;
    }
    for (int i = tid; i < 4 * 256; i += 256) (&wcnt[0][0])[i] = 0;
    __syncthreads();
    const uint8_t *pts = points + (size_t)sg * n;
    uint32_t *mem = members + (size_t)sg * n;
    const uint64_t r0 = (uint64_t)b * rows_per, r1 = min(n, r0 + rows_per);
    for (uint64_t p0 = r0; p0 < r1; p0 += 256) {
        const uint64_t p = p0 + (uint64_t)tid;
        const bool live = p < r1;
        const uint32_t c = live ? pts[p] : 0u;
        uint64_t same = __ballot(live);
#pragma unroll
        for (int bit = 0; bit < 8; bit++) {
            const uint64_t bb = __ballot(live && ((c >> bit) & 1u));
            same &= ((c >> bit) & 1u) ? bb : ~bb;
        }
        const uint32_t below = (uint32_t)__popcll(same & ((1ull << lane) - 1ull));
        if (live && below == 0) wcnt[w][c] = (uint32_t)__popcll(same);  // the lowest lane of each value
        __syncthreads();
        if (live) {
            uint32_t o = base[c] + below;
            for (int v = 0; v < w; v++) o += wcnt[v][c];
            mem[o] = (uint32_t)p;
        }
        __syncthreads();
        for (uint32_t cc = (uint32_t)tid; cc < ks; cc += 256) {
            base[cc] += wcnt[0][cc] + wcnt[1][cc] + wcnt[2][cc] + wcnt[3][cc];
            wcnt[0][cc] = wcnt[1][cc] = wcnt[2][cc] = wcnt[3][cc] = 0;
        }
        __syncthreads();
    }
}

// recalcCenters (kmeans.go:200-218) from the member lists: centers[s][c][j] =
// (0 + x[m0][j] + x[m1][j] + ...) / float32(size), members ascending; the
// loads of eight members are issued before their adds.  Clusters flagged in
// `skip` (reseeded on the host) are left untouched.
__global__ __launch_bounds__(256) void kmeans_sum_kernel(const float *X, uint64_t n, uint32_t dim, uint32_t m,
                                                         uint32_t ks, uint32_t ds, const uint32_t *members,
                                                         const uint32_t *offsets, const uint32_t *counts,
                                                         const uint8_t *recalc, const uint8_t *skip, float *centers)
{
    const uint64_t g = (uint64_t)blockIdx.x * 256 + threadIdx.x;  // (s, c, j)
    if (g >= (uint64_t)m * ks * ds) return;
    const uint32_t j = (uint32_t)(g % ds), c = (uint32_t)((g / ds) % ks), sg = (uint32_t)(g / ((uint64_t)ds * ks));
    if (!recalc[sg] || skip[(size_t)sg * ks + c]) return;
    const uint32_t cnt = counts[(size_t)sg * ks + c];
    const uint32_t *mem = members + (size_t)sg * n + offsets[(size_t)sg * ks + c];
    const float *xs = X + (size_t)sg * ds + j;
    float sum = 0.0f;
    uint32_t i = 0;
    for (; i + 8 <= cnt; i += 8) {
        float v[8];
#pragma unroll
        for (int u = 0; u < 8; u++) v[u] = xs[(size_t)mem[i + u] * dim];
#pragma unroll
        for (int u = 0; u < 8; u++) sum = sum + v[u];
    }
    for (; i < cnt; i++) sum = sum + xs[(size_t)mem[i] * dim];
    centers[((size_t)sg * ks + c) * ds + j] = sum / (float)cnt;
}

hipError_t launch_kmeans_recalc2(const float *X, uint64_t n, uint32_t dim, const uint8_t *points, uint32_t m,
                                 uint32_t ks, uint32_t ds, const uint8_t *recalc, const uint32_t *counts,
                                 const uint32_t *bhist, const uint8_t *skip, uint32_t *members, uint32_t *offsets,
                                 float *centers, hipStream_t s)
{
    hipLaunchKernelGGL(kmeans_members_kernel, dim3(m, kmeans_blocks(n)), dim3(256), 0, s, points, n, ks, counts, bhist,
                       kmeans_rows_per(n), recalc, members, offsets);
    const uint64_t total = (uint64_t)m * ks * ds;
    hipLaunchKernelGGL(kmeans_sum_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, X, n, dim, m, ks, ds,
                       members, offsets, counts, recalc, skip, centers);
    return hipGetLastError();
}

// buildGlobalDistances (CH/product_quantization.go:236-251): table[s][i][j] =
// Step(C_s[i], C_s[j]) for j <= i, mirrored.
__global__ void pq_sdc_table_kernel(int metric, const float *centers, uint32_t m, uint32_t ks, uint32_t ds,
                                    float *table)
{
    const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= (uint64_t)m * ks * ks) return;
    const uint32_t s = (uint32_t)(g / ((uint64_t)ks * ks));
    const uint32_t r = (uint32_t)(g % ((uint64_t)ks * ks));
    const uint32_t i = r / ks, j = r % ks;
    const uint32_t hi = i > j ? i : j, lo = i > j ? j : i;
    const float *cs = centers + (size_t)s * ks * ds;
    table[g] = go_step(metric, cs + (size_t)hi * ds, cs + (size_t)lo * ds, ds);
}

hipError_t launch_pq_sdc_table(int metric, const float *centers, uint32_t m, uint32_t ks, uint32_t ds, float *table,
                               hipStream_t s)
{
    const uint64_t total = (uint64_t)m * ks * ks;
    if (total == 0) return hipSuccess;
    hipLaunchKernelGGL(pq_sdc_table_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, metric, centers,
                       m, ks, ds, table);
    return hipGetLastError();
}

// DistanceBetweenCompressedVectors (CH/product_quantization.go:297-311):
// sequential sum of table[i][x_i][y_i], then Wrap.
__global__ void pq_sdc_rows_kernel(int metric, const float *table, uint32_t m, uint32_t ks, const uint8_t *x,
                                   const uint8_t *codes, uint64_t n, float *out)
{
    const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    const uint8_t *y = codes + r * m;
    float dist = 0.0f;
    for (uint32_t i = 0; i < m; i++) dist = dist + table[((size_t)i * ks + x[i]) * ks + y[i]];
    out[r] = wrap_metric(metric, dist);
}

hipError_t launch_pq_sdc_rows(int metric, const float *table, uint32_t m, uint32_t ks, const uint8_t *x,
                              const uint8_t *codes, uint64_t n, float *out, hipStream_t s)
{
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(pq_sdc_rows_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, metric, table, m, ks,
                       x, codes, n, out);
    return hipGetLastError();
}

}  // namespace wvg
