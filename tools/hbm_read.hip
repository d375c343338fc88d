// hbm_read.hip -- measures the achievable HBM *read* bandwidth on this
// MI355X for a 512 MB streaming read (the 1M x 128 fp32 corpus size), to
// calibrate the roofline of the scan kernel.  Tooling only (not product).
// Build: hipcc --offload-arch=gfx950 -O3 tools/hbm_read.hip -o tools/hbm_read
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                             \
    do {                                                                                     \
        hipError_t e = (x);                                                                  \
        if (e != hipSuccess) {                                                               \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
            exit(1);                                                                         \
        }                                                                                    \
    } while (0)

typedef float f4v __attribute__((ext_vector_type(4)));

template <int UNROLL, bool NT>
__global__ __launch_bounds__(256) void read_kernel(const float4 *__restrict__ p, size_t n4, float *out)
{
    const size_t tid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    float acc = 0.f;
    size_t i = tid;
    for (; i + (UNROLL - 1) * stride < n4; i += UNROLL * stride) {
        f4v v[UNROLL];
        const f4v *q = reinterpret_cast<const f4v *>(p);
#pragma unroll
        for (int u = 0; u < UNROLL; u++) v[u] = NT ? __builtin_nontemporal_load(q + i + u * stride) : q[i + u * stride];
#pragma unroll
        for (int u = 0; u < UNROLL; u++) acc += v[u].x + v[u].y + v[u].z + v[u].w;
    }
    for (; i < n4; i += stride) {
        float4 v = p[i];
        acc += v.x + v.y + v.z + v.w;
    }
    if (acc == 12345.678f) out[0] = acc;  // keep the loads live
}

template <int UNROLL, bool NT>
static void run(const float4 *p, size_t n4, float *out, int blocks, const char *name)
{
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    for (int w = 0; w < 3; w++) hipLaunchKernelGGL((read_kernel<UNROLL, NT>), dim3(blocks), dim3(256), 0, 0, p, n4, out);
    const int iters = 20;
    CHECK(hipEventRecord(a));
    for (int it = 0; it < iters; it++)
        hipLaunchKernelGGL((read_kernel<UNROLL, NT>), dim3(blocks), dim3(256), 0, 0, p, n4, out);
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, a, b));
    const double s = ms / 1e3 / iters;
    printf("{\"variant\": \"%s\", \"blocks\": %d, \"us\": %.2f, \"GBps\": %.1f}\n", name, blocks, s * 1e6,
           n4 * 16.0 / s / 1e9);
}

int main()
{
    const size_t bytes = 512ull * 1000 * 1000;
    const size_t n4 = bytes / 16;
    float4 *p;
    float *out;
    CHECK(hipMalloc(&p, bytes));
    CHECK(hipMalloc(&out, 64));
    CHECK(hipMemset(p, 0, bytes));
    for (int blocks : {1024, 2048, 4096, 8192}) {
        run<4, false>(p, n4, out, blocks, "u4");
        run<8, false>(p, n4, out, blocks, "u8");
        run<8, true>(p, n4, out, blocks, "u8_nt");
    }
    return 0;
}
