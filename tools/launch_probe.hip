// launch_probe.hip -- CPU cost of one hipLaunchKernelGGL call by kernel-argument
// size (tooling only): empty kernels taking 64 B, 512 B, 1344 B (the query-stream
// kernel's ScanArgs + StreamJob with its inline query) of arguments; per size the
// mean wall time of the launch call over 20000 launches (a stream sync every 64).
// Build: hipcc --offload-arch=gfx950 -O2 tools/launch_probe.hip -o tools/launch_probe
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>

template <int N>
struct Blob {
    unsigned char b[N];
};

template <int N>
__global__ void empty_kernel(Blob<N> x, int *out)
{
    if (x.b[N - 1] == 0x5A && threadIdx.x == 1000) out[0] = 1;
}

template <int N>
static void probe(int *out, hipStream_t s, int grid)
{
    Blob<N> x{};
    for (int i = 0; i < 200; i++) hipLaunchKernelGGL(empty_kernel<N>, dim3(grid), dim3(256), 0, s, x, out);
    (void)hipStreamSynchronize(s);
    double sum = 0.0;
    const int n = 20000;
    for (int i = 0; i < n; i++) {
        const auto t0 = std::chrono::steady_clock::now();
        hipLaunchKernelGGL(empty_kernel<N>, dim3(grid), dim3(256), 0, s, x, out);
        sum += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
        if ((i & 63) == 63) (void)hipStreamSynchronize(s);
    }
    (void)hipStreamSynchronize(s);
    printf("{\"arg_bytes\": %d, \"grid\": %d, \"launch_call_us\": %.3f}\n", N, grid, sum / n);
}

int main()
{
    int *out = nullptr;
    hipStream_t s;
    if (hipMalloc(&out, 4) != hipSuccess || hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return 1;
    for (int grid : {257, 513}) {
        probe<64>(out, s, grid);
        probe<512>(out, s, grid);
        probe<1344>(out, s, grid);
        probe<2048>(out, s, grid);
    }
    (void)hipFree(out);
    return 0;
}
