// Standalone GPU check of the device FFT primitives against a double-precision DFT (tools/, not
// part of the library). Build: hipcc --offload-arch=gfx950 -O3 -I dect-nr-plus-sdr_amd/csrc/kernels
#include <hip/hip_runtime.h>

#include <cmath>
#include <complex>
#include <cstdio>
#include <vector>

#include "device_common.hpp"

using namespace dnrp::dev;

template <int SIGN>
__global__ void k_wave(const float2* in, float2* out, const float2* twg) {
    __shared__ float2 xb[4][WFFT_XB];
    __shared__ float2 tw[1024];
    for (int i = threadIdx.x; i < 1024; i += blockDim.x) tw[i] = twg[i];
    __syncthreads();
    const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const float2* x = in + (blockIdx.x * 4 + w) * 1024;
    float2 v[16];
    for (int m = 0; m < 16; ++m) v[m] = x[lane + 64 * m];
    wave_fft1024<SIGN>(v, xb[w], tw, lane);
    for (int m = 0; m < 16; ++m) out[(blockIdx.x * 4 + w) * 1024 + lane + 64 * m] = v[m];
}

int main() {
    const int N = 1024, B = 8;
    std::vector<float2> h(N * B), tw(N), o(N * B);
    srand(1);
    for (auto& z : h) z = make_float2(rand() / (float)RAND_MAX - 0.5f, rand() / (float)RAND_MAX - 0.5f);
    for (int j = 0; j < N; ++j) tw[j] = make_float2((float)std::cos(-2 * M_PI * j / N), (float)std::sin(-2 * M_PI * j / N));
    float2 *di, *dout, *dtw;
    hipMalloc(&di, N * B * 8);
    hipMalloc(&dout, N * B * 8);
    hipMalloc(&dtw, N * 8);
    hipMemcpy(di, h.data(), N * B * 8, hipMemcpyHostToDevice);
    hipMemcpy(dtw, tw.data(), N * 8, hipMemcpyHostToDevice);
    for (int sign : {-1, 1}) {
        if (sign < 0) hipLaunchKernelGGL(k_wave<-1>, dim3(B / 4), dim3(256), 0, 0, di, dout, dtw);
        else hipLaunchKernelGGL(k_wave<1>, dim3(B / 4), dim3(256), 0, 0, di, dout, dtw);
        hipMemcpy(o.data(), dout, N * B * 8, hipMemcpyDeviceToHost);
        double emax = 0, rmax = 0;
        for (int b = 0; b < B; ++b)
            for (int k = 0; k < N; ++k) {
                std::complex<double> acc = 0;
                for (int n = 0; n < N; ++n)
                    acc += std::complex<double>(h[b * N + n].x, h[b * N + n].y) *
                           std::polar(1.0, sign * 2 * M_PI * double(n) * k / N);
                const std::complex<double> g(o[b * N + k].x, o[b * N + k].y);
                emax = std::max(emax, std::abs(g - acc));
                rmax = std::max(rmax, std::abs(acc));
            }
        std::printf("wave_fft1024 sign %+d: max abs err %.3e (max |X| %.2f)\n", sign, emax, rmax);
    }
    return 0;
}
