// wvg_topk.hpp -- wavefront-level top-k selection in registers.
//
// Replaces the reference's bounded max-heap (V/flat/index.go:497-520 over
// adapters/repos/db/priorityqueue/queue.go) with a register-resident sorted
// list of N = 64*E keys per wave (element i = e*64 + lane lives in register e
// of lane `lane`).  Keys are (ordered dist << 32 | slot), so the unsigned
// order is the lexicographic (dist, id) order: among equal distances the
// smaller id wins.  (The reference keeps whichever tie its heap structure
// happens to keep; results agree except inside exact ties.)
//
// A wave offers 64 candidate keys at a time (one per lane).  Only when some
// lane beats the wave-uniform threshold tau (= key of list element K-1) is the
// batch bitonic-sorted across lanes and bitonic-merged into the list; in the
// steady state of a scan almost every batch is rejected by one v_cmp + ballot.
#pragma once

#include "wvg_common.hpp"

namespace wvg {

// Lane exchange partner = lane ^ M, on the VALU (DPP / gfx950 permlane swaps)
// instead of the LDS crossbar (ds_bpermute): a bitonic stage becomes a few
// VALU moves instead of a ~100-cycle LDS round trip.
//   M = 1, 2, 3 : quad_perm;  4, 8 : row_shl/row_shr by M, selected by lane bit;
//   16 / 32 : v_permlane16_swap / v_permlane32_swap;  63 : reverse (row_mirror
//   then the 16- and 32-lane swaps).
template <int M>
__device__ __forceinline__ uint32_t xor_lane32(uint32_t v)
{
    const int lane = __lane_id();
    if constexpr (M == 1) {
        return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);  // [1,0,3,2]
    } else if constexpr (M == 2) {
        return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, false);  // [2,3,0,1]
    } else if constexpr (M == 4 || M == 8) {
        const uint32_t up = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x100 | M, 0xF, 0xF, false);  // row_shl:M
        const uint32_t dn = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x110 | M, 0xF, 0xF, false);  // row_shr:M
        return (lane & M) ? dn : up;
    } else if constexpr (M == 16) {
        auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
        return (lane & 16) ? r[0] : r[1];
    } else if constexpr (M == 32) {
        auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
        return (lane & 32) ? r[0] : r[1];
    } else {
        static_assert(M == 63, "unsupported lane xor");
        const uint32_t m15 = (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x140, 0xF, 0xF, false);  // row_mirror
        return xor_lane32<32>(xor_lane32<16>(m15));
    }
}

template <int M>
__device__ __forceinline__ uint64_t xor_lane64(uint64_t v)
{
    const uint32_t lo = xor_lane32<M>((uint32_t)v), hi = xor_lane32<M>((uint32_t)(v >> 32));
    return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ uint64_t shfl_xor64(uint64_t v, int m)
{
    switch (m) {  // m is a compile-time constant at every (unrolled) call site
    case 1: return xor_lane64<1>(v);
    case 2: return xor_lane64<2>(v);
    case 4: return xor_lane64<4>(v);
    case 8: return xor_lane64<8>(v);
    case 16: return xor_lane64<16>(v);
    case 32: return xor_lane64<32>(v);
    case 63: return xor_lane64<63>(v);
    default: return __shfl_xor(v, m, 64);
    }
}

// lane i receives lane i-1 (lane 0 receives 0): DPP wave_shr:1.
__device__ __forceinline__ uint64_t shr1_lane64(uint64_t v)
{
    const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)v, 0x138, 0xF, 0xF, false);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(v >> 32), 0x138, 0xF, 0xF, false);
    return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ uint64_t readlane64(uint64_t v, int lane)
{
    uint32_t lo = __builtin_amdgcn_readlane((int)(uint32_t)v, lane);
    uint32_t hi = __builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), lane);
    return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ void cas_lane(uint64_t &k, int stride, bool take_min)
{
    uint64_t o = shfl_xor64(k, stride);
    uint64_t mn = o < k ? o : k;
    uint64_t mx = o < k ? k : o;
    k = take_min ? mn : mx;
}

// Ascending bitonic sort of 64 keys, one per lane.
__device__ __forceinline__ void sort64(uint64_t &k)
{
    const int lane = __lane_id();
#pragma unroll
    for (int size = 2; size <= 64; size <<= 1) {
#pragma unroll
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            bool asc = (lane & size) == 0;
            bool lower = (lane & stride) == 0;
            cas_lane(k, stride, lower == asc);
        }
    }
}

// Bitonic merge (ascending) of a bitonic sequence of N = 64*E keys.
template <int E>
__device__ __forceinline__ void bitonic_merge(uint64_t (&k)[E])
{
    const int lane = __lane_id();
#pragma unroll
    for (int es = E >> 1; es > 0; es >>= 1) {
#pragma unroll
        for (int e = 0; e < E; e++) {
            if ((e & es) == 0) {
                uint64_t a = k[e], b = k[e | es];
                k[e] = a < b ? a : b;
                k[e | es] = a < b ? b : a;
            }
        }
    }
#pragma unroll
    for (int stride = 32; stride > 0; stride >>= 1) {
        bool lower = (lane & stride) == 0;
#pragma unroll
        for (int e = 0; e < E; e++) cas_lane(k[e], stride, lower);
    }
}

// list <- N smallest of (list U sorted64 c), list stays sorted ascending.
template <int E>
__device__ __forceinline__ void merge_sorted64(uint64_t (&l)[E], uint64_t c)
{
    uint64_t r = shfl_xor64(c, 63);  // c reversed: c[63 - lane]
    l[E - 1] = r < l[E - 1] ? r : l[E - 1];
    bitonic_merge<E>(l);
}

// list <- N smallest of (list U other), both sorted ascending, same layout.
template <int E>
__device__ __forceinline__ void merge_lists(uint64_t (&l)[E], const uint64_t (&o)[E])
{
#pragma unroll
    for (int e = 0; e < E; e++) {
        uint64_t r = shfl_xor64(o[E - 1 - e], 63);
        l[e] = r < l[e] ? r : l[e];
    }
    bitonic_merge<E>(l);
}

// list <- list with key x inserted in order (elements shift up by one; the
// last element falls off).  x must be smaller than the list's last element.
template <int E>
__device__ __forceinline__ void insert_one(uint64_t (&l)[E], uint64_t x)
{
    const int lane = __lane_id();
    uint64_t prev[E];
#pragma unroll
    for (int e = 0; e < E; e++) {
        uint64_t p = shr1_lane64(l[e]);
        if (lane == 0) p = e == 0 ? 0ull : readlane64(l[e - 1], 63);  // 0 sorts below every key
        prev[e] = p;
    }
#pragma unroll
    for (int e = 0; e < E; e++) l[e] = l[e] < x ? l[e] : (prev[e] < x ? x : prev[e]);
}

// Batches with at most this many keys below the threshold are inserted one by
// one; larger batches are bitonic-sorted and merged.
constexpr int TOPK_INSERT_MAX = 12;

template <int E>
struct WaveTopK {
    uint64_t l[E];
    uint64_t tau;  // wave-uniform: key of element K-1 (KEY_NONE while not full)
    int k;

    __device__ __forceinline__ void init(int k_)
    {
        k = k_;
#pragma unroll
        for (int e = 0; e < E; e++) l[e] = WVG_KEY_NONE;
        tau = WVG_KEY_NONE;
    }

    __device__ __forceinline__ void refresh_tau()
    {
        // read lane (k-1)&63 of every register, select by (k-1)>>6 on the
        // scalar side: a select on the vector side is turned into a dynamic
        // index through scratch, whose vmcnt(0) wait drains in-flight loads.
        const int idx = k - 1, hi = idx >> 6, lo = idx & 63;
        uint64_t t = readlane64(l[0], lo);
#pragma unroll
        for (int e = 1; e < E; e++) {
            const uint64_t te = readlane64(l[e], lo);
            t = hi == e ? te : t;
        }
        tau = t;
    }

    // Offer (dist, slot) for the lanes set in the wave-uniform `live` mask.  A
    // batch whose ordered distances all lie above the threshold's is rejected
    // with one 32-bit compare and a scalar AND, before any 64-bit key is built.
    __device__ __forceinline__ void offer_dist(float dist, uint32_t slot, uint64_t live)
    {
        const uint32_t o = wvg_ord_f32(dist);
        if ((__ballot(o <= (uint32_t)(tau >> 32)) & live) == 0ull) return;
        const int lane = threadIdx.x & 63;
        offer(((live >> lane) & 1ull) ? (((uint64_t)o << 32) | slot) : WVG_KEY_NONE);
    }

    // offer_dist with the rejection on the float distance itself: while the
    // list is full and its K-th distance tau_f is not NaN, a key below tau
    // needs dist <= tau_f (ord(-0) < ord(+0) where -0 <= +0 holds; NaN never
    // passes and never sorts below a non-NaN tau), so the compare is a
    // superset test; the survivors take the exact path.  tau_f / tau_open
    // must start from init_fast() and are refreshed after each exact offer.
    float tau_f;
    bool tau_open;
    __device__ __forceinline__ void init_fast()
    {
        tau_f = __builtin_inff();
        tau_open = true;
    }
    __device__ __forceinline__ void offer_dist_fast(float dist, uint32_t slot, uint64_t live)
    {
        const uint64_t cand = tau_open ? live : (__ballot(dist <= tau_f) & live);
        if (cand == 0ull) return;
        const int lane = threadIdx.x & 63;
        offer(((live >> lane) & 1ull) ? wvg_make_key(dist, slot) : WVG_KEY_NONE);
        tau_f = wvg_unord_f32((uint32_t)(tau >> 32));
        tau_open = tau == WVG_KEY_NONE || tau_f != tau_f;
    }

    // offer_dist_fast that also records the rows the reference's sequential
    // heap could insert (the heap replay, wvg_replay.hip).  The reference
    // (V/flat/index.go:497-506) inserts row i iff fewer than k rows precede it
    // or d_i < Top().Dist, the k-th smallest distance of ALL rows before i;
    // this wave's k-th smallest over its own rows before this batch of 64 is
    // never below that, nor is `seed` (the k-th smallest before the wave's
    // range), so d_i < min(both) keeps a superset of the inserted rows: the
    // rows it drops are no-ops of insertToHeap.  Distances must not be NaN
    // (Hamming).  Kept keys go to buf[cnt ...] in lane (= docID) order; cnt
    // counts past cap so the host can tell an overflow.  buf is LDS in the
    // scan's fast mode: a global store inside the scan loop would make every
    // load of the loop "maybe clobbered" for the compiler, turning the
    // wave-uniform query words and tile masks into vector loads whose vmcnt(0)
    // waits drain the prefetched tile (K5 3.43 vs 2.81 ms per 100M x 1536).
    __device__ __forceinline__ void offer_dist_emit(float dist, uint32_t slot, uint64_t live, float seed, uint64_t *buf,
                                                    uint32_t &cnt, uint32_t cap)
    {
        const uint64_t cand = tau_open ? live : (__ballot(dist <= tau_f) & live);
        if (cand == 0ull) return;
        const int lane = threadIdx.x & 63;
        const float et = fminf(tau_open ? __builtin_inff() : tau_f, seed);
        const uint64_t em = __ballot(dist < et) & live;
        const uint64_t key = ((live >> lane) & 1ull) ? wvg_make_key(dist, slot) : WVG_KEY_NONE;
        if (em) {
            const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(em >> 32),
                                                             __builtin_amdgcn_mbcnt_lo((uint32_t)em, 0u));
            const uint32_t pos = cnt + below;
            if (((em >> lane) & 1ull) && pos < cap) buf[pos] = key;
            cnt += (uint32_t)__popcll(em);
        }
        offer(key);
        tau_f = wvg_unord_f32((uint32_t)(tau >> 32));
        tau_open = tau == WVG_KEY_NONE || tau_f != tau_f;
    }

    // Offer one key per lane (KEY_NONE for an empty lane).
    __device__ __forceinline__ void offer(uint64_t key)
    {
        uint64_t mask = __ballot(key < tau);  // wave-uniform
        if (mask == 0ull) return;
        if (__popcll(mask) > TOPK_INSERT_MAX) {
            sort64(key);
            merge_sorted64<E>(l, key);
            refresh_tau();
            return;
        }
        while (mask) {
            const int c = __builtin_ctzll(mask);
            mask &= mask - 1;
            const uint64_t x = readlane64(key, c);
            if (x < tau) {
                insert_one<E>(l, x);
                refresh_tau();
            }
        }
    }
};

// Workgroup combine: WAVES wave lists -> one sorted list in wave 0, which
// writes its first K keys to `out` (dense per-workgroup partials: no atomics,
// so the workgroups that all finish together never contend).  A pairwise tree
// (log2 WAVES levels of parallel merges) instead of wave 0 merging the other
// lists one after another: with 16 waves and one workgroup per CU the serial
// chain of 15 merges was the scan's largest fixed cost.  Keys are unique
// (slot in the low bits), so the result does not depend on the merge order.
template <int E, int WAVES>
__device__ __forceinline__ void group_combine_store(WaveTopK<E> &tk, uint64_t *out)
{
    static_assert((WAVES & (WAVES - 1)) == 0, "WAVES must be a power of two");
    __shared__ uint64_t sh[WAVES][64 * E];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (WAVES > 1) {
#pragma unroll
        for (int e = 0; e < E; e++) sh[wave][e * 64 + lane] = tk.l[e];
        __syncthreads();
#pragma unroll
        for (int half = WAVES / 2; half >= 1; half /= 2) {
            if (wave < half) {
                uint64_t o[E];
#pragma unroll
                for (int e = 0; e < E; e++) o[e] = sh[wave + half][e * 64 + lane];
                merge_lists<E>(tk.l, o);
                if (half > 1) {
#pragma unroll
                    for (int e = 0; e < E; e++) sh[wave][e * 64 + lane] = tk.l[e];
                }
            }
            if (half > 1) __syncthreads();
        }
    }
    if (wave != 0) return;
#pragma unroll
    for (int e = 0; e < E; e++) {
        const int i = e * 64 + lane;
        if (i < tk.k) out[i] = tk.l[e];
    }
}

}  // namespace wvg
