// mall_reuse.hip -- does a scan that starts where the previous one ended
// (alternating direction, "serpentine") find those rows in the 256 MiB
// Infinity Cache?  Tooling only (not product).
//
// Access pattern of the K1 / K8c scans: every wave owns one contiguous range
// and reads it 8 KiB at a time (8 x 1 KiB wave-loads in flight).  Launches are
// back to back over one buffer; per load policy (buffer-load aux bits) and
// buffer size, always-forward vs alternating direction.
// Build: hipcc --offload-arch=gfx950 -O3 tools/mall_reuse.hip -o tools/mall_reuse
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                             \
    do {                                                                                     \
        hipError_t e = (x);                                                                  \
        if (e != hipSuccess) {                                                               \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
            exit(1);                                                                         \
        }                                                                                    \
    } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <int AUX>
__global__ __launch_bounds__(256) void scan_kernel(const char *p, size_t bytes, int rev, unsigned *out)
{
    const int lane = threadIdx.x & 63;
    const size_t waves = (size_t)gridDim.x * 4, w = (size_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const size_t blk = 8192;  // bytes per wave step
    const size_t nblk = bytes / blk;
    const size_t b0 = nblk * w / waves, b1 = nblk * (w + 1) / waves;
    const size_t n = b1 - b0;
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<char *>(p) + b0 * blk, (short)0, (int)(n * blk), 0x00020000);
    unsigned acc = 0;
    for (size_t i = 0; i < n; i++) {
        const unsigned so = (unsigned)((rev ? n - 1 - i : i) * blk);
        u32x4 v[8];
#pragma unroll
        for (int c = 0; c < 8; c++) v[c] = __builtin_amdgcn_raw_buffer_load_b128(rs, lane * 16 + c * 1024, so, AUX);
#pragma unroll
        for (int c = 0; c < 8; c++) acc ^= v[c].x ^ v[c].y ^ v[c].z ^ v[c].w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

// Pattern of the PQ scans: WAVES waves per workgroup (one workgroup per CU),
// 2 KiB tiles, DEPTH tiles loaded per batch per wave; IL: the waves of a
// workgroup take interleaved tiles of one contiguous workgroup range.
template <int WAVES, int DEPTH, bool IL>
__global__ __launch_bounds__(WAVES * 64) void tiles_kernel(const char *p, size_t bytes, unsigned *out)
{
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const size_t ntile = bytes / 2048;
    size_t t0, t1, ts;
    if (IL) {
        t0 = ntile * blockIdx.x / gridDim.x + wv;
        t1 = ntile * (blockIdx.x + 1) / gridDim.x;
        ts = WAVES;
    } else {
        const size_t waves = (size_t)gridDim.x * WAVES, w = (size_t)blockIdx.x * WAVES + wv;
        t0 = ntile * w / waves;
        t1 = ntile * (w + 1) / waves;
        ts = 1;
    }
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<char *>(p), (short)0, (int)0x7FFFFFFF, 0x00020000);
    unsigned acc = 0;
    for (size_t t = t0; t < t1; t += DEPTH * ts) {
        u32x4 v[DEPTH][2];
#pragma unroll
        for (int d = 0; d < DEPTH; d++) {
            const size_t tt = t + d * ts < t1 ? t + d * ts : t0;
            const unsigned so = (unsigned)((tt * 2048) & 0x7FFFFFFFull);  // (wraps above 2 GB: a timing probe only)
            v[d][0] = __builtin_amdgcn_raw_buffer_load_b128(rs, lane * 16, so, 2);
            v[d][1] = __builtin_amdgcn_raw_buffer_load_b128(rs, lane * 16 + 1024, so, 2);
        }
#pragma unroll
        for (int d = 0; d < DEPTH; d++) acc ^= v[d][0].x ^ v[d][1].w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

template <int WAVES, int DEPTH, bool IL>
static void run_tiles(const char *p, size_t bytes, unsigned *out, const char *name)
{
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    for (int i = 0; i < 3; i++)
        hipLaunchKernelGGL((tiles_kernel<WAVES, DEPTH, IL>), dim3(256), dim3(WAVES * 64), 0, 0, p, bytes, out);
    const int iters = 10;
    CHECK(hipEventRecord(a));
    for (int i = 0; i < iters; i++)
        hipLaunchKernelGGL((tiles_kernel<WAVES, DEPTH, IL>), dim3(256), dim3(WAVES * 64), 0, 0, p, bytes, out);
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, a, b));
    const double s = ms / 1e3 / iters;
    printf("{\"bytes\": %zu, \"pattern\": \"%s\", \"us\": %.2f, \"GBps\": %.1f}\n", bytes, name, s * 1e6,
           bytes / s / 1e9);
}

template <int AUX>
static void run(const char *p, size_t bytes, unsigned *out, bool serp, const char *pol)
{
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    const int blocks = 256;  // one 4-wave workgroup per CU, as K1 at d = 128
    for (int i = 0; i < 4; i++)
        hipLaunchKernelGGL((scan_kernel<AUX>), dim3(blocks), dim3(256), 0, 0, p, bytes, serp ? (i & 1) : 0, out);
    const int iters = 20;
    CHECK(hipEventRecord(a));
    for (int i = 0; i < iters; i++)
        hipLaunchKernelGGL((scan_kernel<AUX>), dim3(blocks), dim3(256), 0, 0, p, bytes, serp ? (i & 1) : 0, out);
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, a, b));
    const double s = ms / 1e3 / iters;
    printf("{\"bytes\": %zu, \"policy\": \"%s\", \"serpentine\": %d, \"us\": %.2f, \"GBps\": %.1f}\n", bytes, pol,
           serp ? 1 : 0, s * 1e6, bytes / s / 1e9);
}

int main()
{
    const size_t big = 3200ull * 1000 * 1000;
    char *p;
    unsigned *out;
    CHECK(hipMalloc(&p, big));
    CHECK(hipMalloc(&out, 64));
    CHECK(hipMemset(p, 1, big));
    {
        const size_t bytes = 2000ull * 1000 * 1000;  // below the 2 GB buffer-offset wrap
        run_tiles<16, 4, false>(p, bytes, out, "16 waves, 4 x 2 KiB per wave, own ranges");
        run_tiles<16, 8, false>(p, bytes, out, "16 waves, 8 x 2 KiB per wave, own ranges");
        run_tiles<16, 4, true>(p, bytes, out, "16 waves, 4 x 2 KiB per wave, interleaved in the WG range");
        run_tiles<16, 8, true>(p, bytes, out, "16 waves, 8 x 2 KiB per wave, interleaved in the WG range");
        run_tiles<8, 8, false>(p, bytes, out, "8 waves, 8 x 2 KiB per wave, own ranges");
        run_tiles<4, 8, false>(p, bytes, out, "4 waves, 8 x 2 KiB per wave, own ranges");
        run_tiles<4, 16, false>(p, bytes, out, "4 waves, 16 x 2 KiB per wave, own ranges");
        run_tiles<16, 2, false>(p, bytes, out, "16 waves, 2 x 2 KiB per wave, own ranges");
    }
    for (size_t bytes : {512ull * 1000 * 1000, 3200ull * 1000 * 1000}) {
        for (int serp = 0; serp < 2; serp++) {
            run<0>(p, bytes, out, serp, "default");
            run<2>(p, bytes, out, serp, "nt");
            run<1>(p, bytes, out, serp, "sc0");
            run<3>(p, bytes, out, serp, "sc0_nt");
        }
    }
    return 0;
}
