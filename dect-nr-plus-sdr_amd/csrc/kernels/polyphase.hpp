// Register-blocked rational polyphase resampler (resampler_t, lib/src/phy/resample/resampler.cpp:330-454).
//
// Output m of an L/M resampler with group delay D reads inputs p(m) - d, d = 0..HL, weighted by
// h[ph(m) + d*L], where t = D + m*M, p = t / L, ph = t % L. For an "aligned" output m_b with
// ph(m_b) = 0 the L outputs m_b .. m_b+L-1 have the compile-time phases (k*M) % L and newest inputs
// p(m_b) + (k*M) / L. One thread therefore computes a whole block of L outputs from
// W = HL + 1 + ((L-1)*M)/L inputs held in registers, with every tap index a compile-time constant:
// the taps are uniform across the wavefront and are read once per block through the scalar
// (constant) cache instead of per output through LDS. Aligned outputs are m_b = m_star + L*q,
// whose newest input is p_star + M*q (no integer division on the device).
#pragma once

#include "device_common.hpp"

namespace dnrp::dev {

typedef const __attribute__((address_space(4))) float* const_taps_t;

__device__ __forceinline__ const_taps_t as_const_taps(const float* p) {
    return (const_taps_t)(p);
}

template <int L, int M, int HL>
struct pp_block {
    static constexpr int W = HL + 1 + ((L - 1) * M) / L;  // inputs per block

    // x[i] = input p_b - HL + i; y[k] = output m_b + k (unmixed)
    __device__ static __forceinline__ void run(const float2 (&x)[W], const_taps_t h, float2 (&y)[L]) {
#pragma unroll
        for (int k = 0; k < L; ++k) {
            const int ph = (k * M) % L, o = (k * M) / L;
            float ar = 0.f, ai = 0.f;
#pragma unroll
            for (int d = 0; d <= HL; ++d) {
                const float t = h[ph + d * L];
                ar = fmaf(x[HL + o - d].x, t, ar);
                ai = fmaf(x[HL + o - d].y, t, ai);
            }
            y[k] = make_float2(ar, ai);
        }
    }
};

}  // namespace dnrp::dev
