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

__device__ __forceinline__ uint64_t shfl_xor64(uint64_t v, int m)
{
    return __shfl_xor(v, m, 64);
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
        const int idx = k - 1;
        uint64_t v = l[0];
#pragma unroll
        for (int e = 1; e < E; e++)
            if ((idx >> 6) == e) v = l[e];
        tau = readlane64(v, idx & 63);
    }

    // Offer one key per lane (KEY_NONE for an empty lane).
    __device__ __forceinline__ void offer(uint64_t key)
    {
        if (__ballot(key < tau) == 0ull) return;  // wave-uniform
        sort64(key);
        merge_sorted64<E>(l, key);
        refresh_tau();
    }
};

// Workgroup combine: WAVES wave lists -> one sorted list in wave 0, which
// writes its first K keys to `out` (dense per-workgroup partials: no atomics,
// so the workgroups that all finish together never contend).
template <int E, int WAVES>
__device__ __forceinline__ void group_combine_store(WaveTopK<E> &tk, uint64_t *out)
{
    __shared__ uint64_t sh[WAVES][64 * E];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (WAVES > 1) {
#pragma unroll
        for (int e = 0; e < E; e++) sh[wave][e * 64 + lane] = tk.l[e];
        __syncthreads();
    }
    if (wave != 0) return;
    for (int w = 1; w < WAVES; w++) {
        uint64_t o[E];
#pragma unroll
        for (int e = 0; e < E; e++) o[e] = sh[w][e * 64 + lane];
        merge_lists<E>(tk.l, o);
    }
#pragma unroll
    for (int e = 0; e < E; e++) {
        const int i = e * 64 + lane;
        if (i < tk.k) out[i] = tk.l[e];
    }
}

}  // namespace wvg
