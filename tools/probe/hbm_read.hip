// HBM streaming-rate probe (tools, not product): pure read (16-B nontemporal loads, xor-reduced to
// one word per thread), pure write (16-B stores) and copy, each over a buffer far larger than the
// 256 MiB Infinity Cache, timed with HIP events. Prints one JSON line of GB/s.
//   hipcc --offload-arch=gfx950 -O3 -o hbm_read hbm_read.hip && ./hbm_read [GiB]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef unsigned int u4 __attribute__((ext_vector_type(4)));

__global__ void __launch_bounds__(256) rd(const u4* __restrict__ p, size_t n, unsigned* out) {
    u4 acc = {0u, 0u, 0u, 0u};
    const size_t stride = size_t(gridDim.x) * blockDim.x;
    size_t i = size_t(blockIdx.x) * blockDim.x + threadIdx.x;
    for (; i + 3 * stride < n; i += 4 * stride) {  // four loads in flight per thread
        const u4 a = __builtin_nontemporal_load(p + i), b = __builtin_nontemporal_load(p + i + stride);
        const u4 c = __builtin_nontemporal_load(p + i + 2 * stride), d = __builtin_nontemporal_load(p + i + 3 * stride);
        acc ^= a ^ b ^ c ^ d;
    }
    for (; i < n; i += stride) acc ^= __builtin_nontemporal_load(p + i);
    out[size_t(blockIdx.x) * blockDim.x + threadIdx.x] = acc.x ^ acc.y ^ acc.z ^ acc.w;
}

__global__ void __launch_bounds__(256) wr(u4* __restrict__ p, size_t n) {
    const size_t stride = size_t(gridDim.x) * blockDim.x;
    for (size_t i = size_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride)
        __builtin_nontemporal_store(u4{unsigned(i), 1u, 2u, 3u}, p + i);
}

__global__ void __launch_bounds__(256) cp(const u4* __restrict__ s, u4* __restrict__ d, size_t n) {
    const size_t stride = size_t(gridDim.x) * blockDim.x;
    for (size_t i = size_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride)
        __builtin_nontemporal_store(__builtin_nontemporal_load(s + i), d + i);
}

int main(int argc, char** argv) {
    const double gib = argc > 1 ? atof(argv[1]) : 16.0;
    const size_t bytes = size_t(gib * (1ull << 30)) / 16 * 16, n = bytes / 16;
    u4 *a = nullptr, *b = nullptr;
    unsigned* out = nullptr;
    const int grid = 256 * 32;  // 32 workgroups of 256 threads per CU
    if (hipMalloc(&a, bytes) != hipSuccess || hipMalloc(&b, bytes) != hipSuccess ||
        hipMalloc(&out, size_t(grid) * 256 * 4) != hipSuccess) {
        printf("{\"error\": \"alloc\"}\n");
        return 1;
    }
    hipMemset(a, 1, bytes);
    hipMemset(b, 0, bytes);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    auto timed = [&](auto launch) {
        launch();
        hipDeviceSynchronize();
        float best = 1e30f;
        for (int r = 0; r < 5; ++r) {
            hipEventRecord(e0);
            launch();
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms = 0.f;
            hipEventElapsedTime(&ms, e0, e1);
            best = ms < best ? ms : best;
        }
        return best;
    };
    const float t_rd = timed([&] { hipLaunchKernelGGL(rd, dim3(grid), dim3(256), 0, 0, a, n, out); });
    const float t_wr = timed([&] { hipLaunchKernelGGL(wr, dim3(grid), dim3(256), 0, 0, b, n); });
    const float t_cp = timed([&] { hipLaunchKernelGGL(cp, dim3(grid), dim3(256), 0, 0, a, b, n); });
    printf("{\"bytes\": %zu, \"read_GBps\": %.1f, \"write_GBps\": %.1f, \"copy_GBps_total\": %.1f}\n", bytes,
           bytes / (t_rd * 1e6), bytes / (t_wr * 1e6), 2.0 * bytes / (t_cp * 1e6));
    return 0;
}
