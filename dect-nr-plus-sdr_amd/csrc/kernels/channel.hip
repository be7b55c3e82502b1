// Simulated wireless channel on the GPU (lib/src/simulation/wireless: channel_awgn.cpp, channel_flat.cpp,
// channel_doubly.cpp + link.cpp, hardware/noise.cpp): n TX windows (dnrp_tx_batch output) through
// N_TX x N_RX links into RX windows. One thread per RX output sample:
//   y_r[n] = noise_r[n] + g * sum_tx h_{r,tx}(x_tx, n - off)
//   awgn:   h = x[n]                                        (channel_awgn_t::superimpose)
//   flat:   h = c_{r,tx} x[n]                               (channel_flat_t, Rayleigh coefficient)
//   doubly: h = sum_i sqrt(p_i / N_sin) x[n - d_i] sum_j exp(j (2 pi ((t mod |P_ij|) / P_ij) + phi_ij))
//           t = t0 + n (global hw time), tapped delay line with N_sin sinusoids per tap
//           (link_t::pass_through_link, link.cpp:246-288; the rotator's per-block restart folded
//           into the per-sample phase)
// Noise: complex Gaussian, standard deviation sigma per component (srsRAN ch_awgn as noise.cpp
// configures it), from a counter-based generator (seed, window, antenna, sample): reproducible and
// independent of the launch geometry.
#include "kernels.hpp"

namespace dnrp::dev {

constexpr uint32_t CH_THREADS = 256;

__device__ __forceinline__ uint64_t ch_mix(uint64_t z) {  // splitmix64 finaliser
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// two independent standard normals for counter c (Box-Muller on two 24-bit uniforms)
__device__ __forceinline__ float2 ch_gauss(uint64_t seed, uint64_t c) {
    const uint64_t h = ch_mix(seed ^ ch_mix(c));
    const float u1 = (static_cast<float>(h >> 40) + 1.0f) * (1.0f / 16777216.0f);  // (0, 1]
    const float u2 = static_cast<float>((h >> 16) & 0xFFFFFFull) * (1.0f / 16777216.0f);
    const float r = sqrtf(-2.0f * __logf(u1));
    float s, co;
    __sincosf(6.28318530717958647692f * u2, &s, &co);
    return make_float2(r * co, r * s);
}

__global__ void __launch_bounds__(CH_THREADS) channel_kernel(channel_args A) {
    const uint32_t row = blockIdx.y, w = row / A.N_RX, r = row % A.N_RX;
    const uint32_t n = blockIdx.x * CH_THREADS + threadIdx.x;
    if (n >= A.S_rx) return;
    const int64_t off = A.offset[w];
    const int64_t t = A.t0[w] + n;
    float2 acc = make_float2(0.f, 0.f);
    for (uint32_t tx = 0; tx < A.N_TX; ++tx) {
        const float2* x = A.tx + (size_t(w) * A.N_TX + tx) * A.S_tx;
        const uint32_t link = r * A.N_TX + tx;
        if (A.kind == CH_DOUBLY) {
            const channel_tap* taps = A.taps + (size_t(w) * A.N_RX * A.N_TX + link) * A.n_taps;
            for (uint32_t i = 0; i < A.n_taps; ++i) {
                const int64_t q = static_cast<int64_t>(n) - off - taps[i].delay;
                if (q < 0 || q >= static_cast<int64_t>(A.S_tx)) continue;
                const float2 xv = x[q];
                float2 g = make_float2(0.f, 0.f);
                const channel_sin* sn = A.sins + ((size_t(w) * A.N_RX * A.N_TX + link) * A.n_taps + i) * A.n_sin;
                for (uint32_t j = 0; j < A.n_sin; ++j) {
                    const int64_t P = sn[j].period;
                    const int64_t aP = P < 0 ? -P : P;
                    const double rev = static_cast<double>(t % aP) / static_cast<double>(P) + sn[j].phase_rev;
                    g = cadd(g, phasor(6.28318530717958647692 * rev));
                }
                acc = cadd(acc, cscale(cmul(xv, g), taps[i].amp));
            }
        } else {
            const int64_t q = static_cast<int64_t>(n) - off;
            if (q < 0 || q >= static_cast<int64_t>(A.S_tx)) continue;
            float2 v = x[q];
            if (A.kind == CH_FLAT) v = cmul(v, A.coef[size_t(w) * A.N_RX * A.N_TX + link]);
            acc = cadd(acc, v);
        }
    }
    acc = cscale(acc, A.large_scale);
    if (A.sigma > 0.f) {
        const float2 z = ch_gauss(A.seed, (uint64_t(row) << 32) | n);
        acc = make_float2(fmaf(A.sigma, z.x, acc.x), fmaf(A.sigma, z.y, acc.y));
    }
    A.rx[size_t(row) * A.S_rx + n] = acc;
}

hipError_t launch_channel(const channel_args& a, uint32_t n, hipStream_t st) {
    const uint64_t rows = uint64_t(n) * a.N_RX;
    if (rows == 0 || a.S_rx == 0) return hipSuccess;
    if (rows > 65535u) return hipErrorInvalidValue;
    hipLaunchKernelGGL(channel_kernel, dim3((a.S_rx + CH_THREADS - 1) / CH_THREADS, static_cast<uint32_t>(rows)),
                       dim3(CH_THREADS), 0, st, a);
    return hipGetLastError();
}

}  // namespace dnrp::dev
