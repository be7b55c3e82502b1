// Ring-buffer window gather (rx_pacer_t::resample_single_unit / resample_until_nto wrap copy,
// lib/src/phy/rx/rx_pacer.cpp:106-143, over radio::buffer_rx_t's per-antenna ring,
// lib/include/dectnrp/radio/buffer_rx.hpp:46-141): window w, antenna a, sample i <- ring sample
// (start[w] + i) mod ring_len of antenna a. HBM-bound copy: 16-B loads and stores where the window
// start and the ring length keep sample pairs contiguous and aligned, 8-B otherwise. A window never
// reads more than ring_len samples (host-checked), so one wrap at most.
#include "kernels.hpp"

namespace dnrp::dev {

constexpr uint32_t RING_THREADS = 256;

__global__ void __launch_bounds__(RING_THREADS) ring_gather_kernel(ring_args A) {
    // grid: x = sample pairs of one (window, antenna) row in RING_THREADS * RING_PAIRS blocks, y = row
    const uint32_t row = blockIdx.y, w = row / A.n_ant, a = row % A.n_ant;
    const int64_t start = A.start[w];
    const uint64_t s0 = static_cast<uint64_t>(start) % A.ring_len;
    const float2* src = A.ring + size_t(a) * A.ant_stride;
    float2* dst = A.out + size_t(row) * A.S_win;
    const bool pairs = ((s0 | A.ring_len | A.S_win) & 1u) == 0 &&
                       ((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst)) & 15u) == 0;
    const uint32_t first = (blockIdx.x * RING_THREADS) * RING_PAIRS + threadIdx.x;
    if (pairs) {
        const float4* s4 = reinterpret_cast<const float4*>(src);
        float4* d4 = reinterpret_cast<float4*>(dst);
        const uint64_t r2 = A.ring_len / 2, p0 = s0 / 2;
        float4 v[RING_PAIRS];
#pragma unroll
        for (int j = 0; j < RING_PAIRS; ++j) {
            const uint32_t i = first + j * RING_THREADS;
            if (i < A.S_win / 2) {
                uint64_t q = p0 + i;
                if (q >= r2) q -= r2;
                v[j] = s4[q];
            }
        }
#pragma unroll
        for (int j = 0; j < RING_PAIRS; ++j) {
            const uint32_t i = first + j * RING_THREADS;
            if (i < A.S_win / 2) d4[i] = v[j];
        }
    } else {
        // one sample per lane, twice the pairs' rows of work per block
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            float2 v[RING_PAIRS];
#pragma unroll
            for (int j = 0; j < RING_PAIRS; ++j) {
                const uint64_t i = 2ull * (blockIdx.x * RING_THREADS) * RING_PAIRS + (2 * j + h) * RING_THREADS + threadIdx.x;
                if (i < A.S_win) {
                    uint64_t q = s0 + i;
                    if (q >= A.ring_len) q -= A.ring_len;
                    v[j] = src[q];
                }
            }
#pragma unroll
            for (int j = 0; j < RING_PAIRS; ++j) {
                const uint64_t i = 2ull * (blockIdx.x * RING_THREADS) * RING_PAIRS + (2 * j + h) * RING_THREADS + threadIdx.x;
                if (i < A.S_win) dst[i] = v[j];
            }
        }
    }
}

hipError_t launch_ring_gather(const ring_args& a, uint32_t n, hipStream_t st) {
    const uint32_t per_block = RING_THREADS * RING_PAIRS;  // sample pairs
    const uint32_t bx = (a.S_win / 2 + 1 + per_block - 1) / per_block;
    const uint64_t rows = uint64_t(n) * a.n_ant;
    if (rows == 0 || bx == 0) return hipSuccess;
    if (rows > 65535u) return hipErrorInvalidValue;
    hipLaunchKernelGGL(ring_gather_kernel, dim3(bx, static_cast<uint32_t>(rows)), dim3(RING_THREADS), 0, st, a);
    return hipGetLastError();
}

}  // namespace dnrp::dev
