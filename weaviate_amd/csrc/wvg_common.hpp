// wvg_common.hpp -- shared device/host helpers for the MI355X scoring path.
//
// Device data layout ("row tiles"): the corpus is stored in tiles of 64 rows,
// one row per lane of a wave64.  Inside a tile the 16-byte chunks are
// chunk-major: chunk c of row (64*t + lane) lives at float4 index
//     (t * nchunks + c) * 64 + lane
// so one wave-instruction `global_load_dwordx4` reads 1 KiB contiguous bytes
// (chunk c of all 64 rows), every lane owns a whole row, and the per-row
// reduction needs no cross-lane traffic.  The query is wave-uniform (scalar
// loads).  The validity bitmap has exactly one 64-bit word per tile.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#define WVG_TILE 64

// ---------------------------------------------------------------------------
// Sort keys: (distance, slot) packed into a u64 whose unsigned order is the
// lexicographic (dist, slot) order.  Distances are mapped to an order-
// preserving u32 (NaN canonicalised to +NaN, which sorts after +Inf).
// ---------------------------------------------------------------------------
__host__ __device__ inline uint32_t wvg_ord_f32(float f)
{
    uint32_t u;
    __builtin_memcpy(&u, &f, 4);
    if ((u & 0x7F800000u) == 0x7F800000u && (u & 0x007FFFFFu)) u = 0x7FC00000u;
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__host__ __device__ inline float wvg_unord_f32(uint32_t o)
{
    uint32_t u = (o & 0x80000000u) ? (o & 0x7FFFFFFFu) : ~o;
    float f;
    __builtin_memcpy(&f, &u, 4);
    return f;
}
__host__ __device__ inline uint64_t wvg_make_key(float dist, uint32_t slot)
{
    return ((uint64_t)wvg_ord_f32(dist) << 32) | slot;
}
#define WVG_KEY_NONE 0xFFFFFFFFFFFFFFFFull

// ---------------------------------------------------------------------------
// Synthetic rows: counter-based generator keyed by (seed, row, col).  The CPU
// twin used by the tests is oracle/wv_oracle.c orc_synth_value.
// dist 0: uniform [-1,1) on a 2^-23 grid (V/testinghelpers/helpers.go:125-133
//         draws uniform [-1,1)); dist 1: integers 0..255 (SIFT-like).
// ---------------------------------------------------------------------------
__host__ __device__ inline uint64_t wvg_mix64(uint64_t z)
{
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
__host__ __device__ inline float wvg_synth_value(uint64_t seed_mixed, uint64_t row, uint64_t col, int dist)
{
    uint64_t h = wvg_mix64(seed_mixed ^ ((row << 20) | (col & 0xFFFFF)));
    uint32_t u24 = (uint32_t)(h >> 40);
    if (dist == 1) return (float)(u24 >> 16);
    return (float)u24 * (1.0f / 8388608.0f) - 1.0f;
}

// ---------------------------------------------------------------------------
// Metrics (entities/vectorindex/common/config.go:22-31 names them
// "l2-squared", "dot", "cosine", "manhattan", "hamming"; the provider type of
// cosine is "cosine-dot").  Kernels templated on a metric instantiate L2, DOT
// (raw dot product; cosine is DOT with the 1-x Wrap), MANHATTAN and HAMMING.
// ---------------------------------------------------------------------------
enum { WVG_M_L2 = 0, WVG_M_DOT = 1, WVG_M_COSINE = 2, WVG_M_MANHATTAN = 3, WVG_M_HAMMING = 4 };

__device__ __forceinline__ int wvg_lane() { return __lane_id(); }
