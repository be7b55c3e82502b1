// Synchronisation kernels: sync_chunk_t::search() (lib/src/phy/rx/sync/sync_chunk.cpp:143-279)
// for a batch of windows, each window one chunk whose sync resampler starts with zero history.
//
//  sync_steps_kernel   one WG per (window, antenna, tile of 64 detection steps): sync resampler
//                      (M/L polyphase, register blocks) into LDS, then per step the power
//                      sum |x|^2 and the pattern-lag correlation sum x[n-P] conj(x[n]) over the
//                      step's samples (autocorrelator_detection.cpp:107-128, 152-178). These are the
//                      only per-sample passes over the window; everything after reads them.
//  sync_detect_kernel  one WG per window, the detection / coarse-peak state machine:
//                      detection conditions on moving sums of the step values (RMS limits,
//                      front/back RMS, coarse metric band, streak; autocorrelator_detection.cpp:
//                      186-280, movsum_uw.cpp:55-74), then for every detection the per-sample
//                      coarse-peak search over one STF with the smoothed metric
//                      (autocorrelator_peak.cpp:145-264), validity, metric-weighted coarse peak
//                      time, RMS and fractional CFO at the peak (:311-394), skip after the peak.
//                      Windowed sums are exact prefix differences in double (the reference keeps
//                      float running sums with periodic re-summation).
//  sync_fine_kernel    one WG per report: CFO pre-rotation of the strongest antenna's hw-rate
//                      samples around the coarse peak and cross-correlation with every STF
//                      template (crosscorrelator.cpp:80-251) as one forward FFT plus one inverse
//                      FFT per template, argmax over the search range, N_eff_TX, fine peak.
#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "device_common.hpp"
#include "experiments.hpp"
#include "kernels.hpp"
#include "polyphase.hpp"
#include "taps_gen.hpp"

namespace dnrp::dev {

constexpr uint32_t SYNC_THREADS = 256;
constexpr uint32_t SYNC_TILE_STEPS = 64;
constexpr uint32_t SYNC_PAD_PEAK = 32;  // samples before the coarse-peak region (weighted peak can sit left of it)

__device__ __forceinline__ int64_t floordiv(int64_t a, int64_t b) { return a >= 0 ? a / b : -((-a + b - 1) / b); }

// lb[y] for y in [y0, y0 + cnt) of one antenna (input x[i] valid for i in [0, S_win), zero history)
// into dst[y - y0]. taps: LDS block taps (pp path) or the global natural taps (generic path).
// Whole block participates; ends with a barrier.
template <int LR, int MR, int HLR>
__device__ void sync_resample(const sync_args& A, const float2* __restrict__ x, int64_t y0, uint32_t cnt,
                              float2* stage, float2* dst, const float* taps, uint32_t stage_cap = 0xFFFFFFFFu) {
    const int64_t S = A.S_win;
    if constexpr (LR == 1) {
            stage_span<8>(dst, x, y0, cnt, S, threadIdx.x, blockDim.x);
        __syncthreads();
    } else if constexpr (LR == 0) {  // generic L/M (os_min 4/8): direct FIR per output
        for (uint32_t i = threadIdx.x; i < cnt; i += blockDim.x) {
            const int64_t y = y0 + i;
            float2 acc = make_float2(0.f, 0.f);
            if (y >= 0) {
                const uint64_t t = A.delay + static_cast<uint64_t>(y) * A.M;
                const int64_t p = static_cast<int64_t>(t / A.L);
                const uint32_t ph = static_cast<uint32_t>(t % A.L);
                for (uint32_t d = 0; d <= A.hl; ++d) {
                    const int64_t q = p - d;
                    if (q < 0 || q >= S) continue;
                    const float h = A.taps[ph + d * A.L];
                    acc.x = fmaf(x[q].x, h, acc.x);
                    acc.y = fmaf(x[q].y, h, acc.y);
                }
            }
            dst[i] = acc;
        }
        __syncthreads();
    } else {
        using PB = pp_block<LR, MR, HLR>;
        const int64_t ms = A.m_star;
        const int64_t q0 = floordiv(y0 - ms, LR), q1 = floordiv(y0 + cnt - ms + LR - 1, LR);
        // pieces of nbp blocks whose input span fits the stage (stage_cap float2)
        const int64_t nbp = stage_cap >= static_cast<uint32_t>(PB::W) + MR ? (stage_cap - PB::W) / MR + 1 : 1;
        for (int64_t qa = q0; qa < q1; qa += nbp) {
            const int64_t qe = min(qa + nbp, q1);
            const int64_t in0 = static_cast<int64_t>(A.p_star) + MR * qa - HLR;
            const uint32_t n_in = static_cast<uint32_t>(MR * (qe - 1 - qa) + PB::W);
            stage_span<8>(stage, x, in0, n_in, S, threadIdx.x, blockDim.x);
            __syncthreads();
            for (int64_t q = qa + threadIdx.x; q < qe; q += blockDim.x) {
                float2 yv[LR];
                PB::run(stage + MR * (q - qa), taps, yv);
                const int64_t mb = ms + LR * q;
#pragma unroll
                for (int k = 0; k < LR; ++k) {
                    const int64_t idx = mb + k - y0;
                    if (idx >= 0 && idx < static_cast<int64_t>(cnt)) dst[idx] = (mb + k >= 0) ? yv[k] : make_float2(0.f, 0.f);
                }
            }
            __syncthreads();
        }
    }
}

__host__ __device__ inline uint32_t sync_stage_cap(uint32_t L, uint32_t M, uint32_t hl, uint32_t cnt) {
    if (L <= 1) return 0;
    const uint32_t W = hl + 1 + ((L - 1) * M) / L;
    return M * (cnt / L + 2) + W + M;
}

// ===================================================================== per-step sums
template <int LR, int MR, int HLR>
__global__ void __launch_bounds__(SYNC_THREADS) sync_steps_kernel(sync_args A) {
    extern __shared__ __attribute__((aligned(16))) float2 smem[];
    const uint32_t ntile = (A.n_steps + SYNC_TILE_STEPS - 1) / SYNC_TILE_STEPS;
    const uint32_t tile = blockIdx.x % ntile;
    const uint32_t a = (blockIdx.x / ntile) % A.n_ant;
    const uint32_t w = blockIdx.x / (ntile * A.n_ant);
    float* taps = reinterpret_cast<float*>(smem);
    const uint32_t tap_f2 = (A.npp + 3) / 4 * 2;
    float2* lb = smem + tap_f2;
    const uint32_t s0 = tile * SYNC_TILE_STEPS;
    const uint32_t s1 = min(s0 + SYNC_TILE_STEPS, A.n_steps);
    const int64_t y0 = static_cast<int64_t>(s0) * A.step - A.pattern;
    const uint32_t cnt = (s1 - s0) * A.step + A.pattern;
    float2* stage = lb + (cnt + 1) / 2 * 2;
    if (LR > 1)
        stage_copy<4>(taps, A.taps_pp, A.npp, threadIdx.x, blockDim.x);
    const float2* x = A.iq + w * A.win_stride + a * A.ant_stride;
    sync_resample<LR, MR, HLR>(A, x, y0, cnt, stage, lb, taps);
    // step s = s0 + tid/4, quarter tid%4 of its samples; reduce over the 4 lanes
    const uint32_t sl = threadIdx.x >> 2, part = threadIdx.x & 3u;
    const uint32_t s = s0 + sl, seg = A.step >> 2;
    float pw = 0.f;
    float2 c = make_float2(0.f, 0.f);
    if (s < s1) {
        const uint32_t i0 = (s - s0) * A.step + A.pattern + part * seg;  // index of y = s*step + part*seg
        for (uint32_t j = 0; j < seg; ++j) {
            const float2 v = lb[i0 + j];
            pw = fmaf(v.x, v.x, fmaf(v.y, v.y, pw));
            if (s >= 4) {
                const float2 u = lb[i0 + j - A.pattern];  // A = x[n - P], B = x[n]: A conj(B)
                c.x = fmaf(u.x, v.x, fmaf(u.y, v.y, c.x));
                c.y = fmaf(u.y, v.x, fmaf(-u.x, v.y, c.y));
            }
        }
    }
#pragma unroll
    for (int o = 1; o < 4; o <<= 1) {
        pw += __shfl_xor(pw, o);
        c.x += __shfl_xor(c.x, o);
        c.y += __shfl_xor(c.y, o);
    }
    if (s < s1 && part == 0) {
        const size_t o = (static_cast<size_t>(w) * A.n_ant + a) * A.n_steps + s;
        A.P[o] = pw;
        A.Cs[o] = c;
    }
}

// ---- pp resampler path: one wavefront per range of SYNC_WB_STEPS-ish steps, no workgroup barrier
// after the table load. The wave stages its hw-rate input span in its own LDS region, resamples it
// with B polyphase blocks per lane (pp_block::run_multi: one tap-row read serves B blocks, which
// keeps the LDS traffic per FMA under the 128 B/clk/CU the VALU needs), writes the outputs back into
// the region and sums the steps from there.
#ifndef SYNC_WB_DEF
#define SYNC_WB_DEF 4
#endif
#ifndef SYNC_WPG_DEF
#define SYNC_WPG_DEF 2
#endif
constexpr int SYNC_WB = SYNC_WB_DEF;  // blocks per lane

__host__ __device__ inline uint32_t sync_wave_steps(uint32_t L, uint32_t step, uint32_t pattern) {
    return (64u * SYNC_WB * L - pattern - 2 * L) / step;  // steps whose span (+ lookback) fits 64 B blocks
}
__host__ __device__ inline uint32_t sync_wave_region(uint32_t L, uint32_t M, uint32_t hl) {  // float2 per wave
    const uint32_t W = hl + 1 + ((L - 1) * M) / L;
    return (M * (64 * SYNC_WB - 1) + W + 1) / 2 * 2;
}

template <int LR, int MR, int HLR, int WPG>
__global__ void __launch_bounds__(64 * WPG) sync_steps_wave_kernel(sync_args A) {
    extern __shared__ __attribute__((aligned(16))) float2 smem[];
    using PB = pp_block<LR, MR, HLR>;
    float* taps = reinterpret_cast<float*>(smem);
    const uint32_t tap_f2 = (A.npp + 3) / 4 * 2;
    const uint32_t region = sync_wave_region(LR, MR, HLR);
    const uint32_t wv = threadIdx.x >> 6, lane = threadIdx.x & 63u;
    float2* R = smem + tap_f2 + wv * region;
    const uint32_t sw = sync_wave_steps(LR, A.step, A.pattern);
    const uint32_t parts = (A.n_steps + sw - 1) / sw;
    const uint32_t gw = blockIdx.x * WPG + wv;
    const uint32_t part = gw % parts;
    const uint32_t a = (gw / parts) % A.n_ant;
    const uint32_t w = gw / (parts * A.n_ant);
    const uint32_t s0 = part * sw, s1 = min(s0 + sw, A.n_steps);
    const int64_t y0 = static_cast<int64_t>(s0) * A.step - A.pattern;
    const uint32_t cnt = (s1 - s0) * A.step + A.pattern;
    const int64_t ms = A.m_star;
    const int64_t q0 = floordiv(y0 - ms, LR), q1 = floordiv(y0 + cnt - ms + LR - 1, LR);
    const int64_t in0 = static_cast<int64_t>(A.p_star) + MR * q0 - HLR;
    const uint32_t n_in = static_cast<uint32_t>(MR * (q1 - 1 - q0) + PB::W);
    const bool live = w < A.n_win;
    if (live) {
        const float2* x = A.iq + w * A.win_stride + a * A.ant_stride;
        const int64_t S = A.S_win;
        stage_span<24>(R, x, in0, n_in, S, lane, 64);
    }
    stage_copy<4>(taps, A.taps_pp, A.npp, threadIdx.x, blockDim.x);
    __syncthreads();
    if (!live) return;
    float2 y[SYNC_WB][LR];
    const float2* xw[SYNC_WB];
#pragma unroll
    for (int b = 0; b < SYNC_WB; ++b) xw[b] = R + MR * (lane + 64 * b);
    PB::template run_multi<SYNC_WB>(xw, taps, y);
    __builtin_amdgcn_wave_barrier();
    const int64_t nblk = q1 - q0;
#pragma unroll
    for (int b = 0; b < SYNC_WB; ++b) {
        const int64_t j = lane + 64 * b;
        if (j < nblk) {
            const int64_t mb = ms + LR * (q0 + j);
#pragma unroll
            for (int k = 0; k < LR; ++k) {
                const int64_t idx = mb + k - y0;
                if (idx >= 0 && idx < static_cast<int64_t>(cnt)) R[idx] = (mb + k >= 0) ? y[b][k] : make_float2(0.f, 0.f);
            }
        }
    }
    __builtin_amdgcn_wave_barrier();
    // steps: 32 per round, half of each step's samples per lane (reduced over the lane pair). Each
    // lane walks its half starting at its own rotation (j + lane) mod half, so the 32 lanes of a
    // ds_read_b64 half-wave hit 32 different bank pairs (step starts are 0 mod 64 banks).
    const uint32_t half = A.step >> 1, h = lane & 1u, rot = lane % half;
    for (uint32_t sb = s0; sb < s1; sb += 32) {
        const uint32_t s = sb + (lane >> 1);
        float pw = 0.f;
        float2 c = make_float2(0.f, 0.f);
        if (s < s1) {
            const uint32_t i0 = (s - s0) * A.step + A.pattern + h * half;
            for (uint32_t j = 0; j < half; ++j) {
                uint32_t jj = j + rot;
                if (jj >= half) jj -= half;
                const float2 v = R[i0 + jj];
                pw = fmaf(v.x, v.x, fmaf(v.y, v.y, pw));
                if (s >= 4) {
                    const float2 u = R[i0 + jj - A.pattern];
                    c.x = fmaf(u.x, v.x, fmaf(u.y, v.y, c.x));
                    c.y = fmaf(u.y, v.x, fmaf(-u.x, v.y, c.y));
                }
            }
        }
        pw += __shfl_xor(pw, 1);
        c.x += __shfl_xor(c.x, 1);
        c.y += __shfl_xor(c.y, 1);
        if (s < s1 && h == 0) {
            const size_t o = (static_cast<size_t>(w) * A.n_ant + a) * A.n_steps + s;
            A.P[o] = pw;
            A.Cs[o] = c;
        }
    }
}

// ---- streaming path (pp resampler, ring fits): one wavefront walks a segment of steps in chunks
// of 64 polyphase blocks (64 L outputs), software-pipelined: the next chunk's M * 64 new inputs are
// loaded into registers (coalesced, 8 B per lane and instruction) while the current chunk is
// resampled, so every wave keeps its own loads in flight instead of waiting on a staging pass.
// Per wave LDS: the chunk's input window (carry W - M + M * 64) and a 1024-sample output ring
// holding the pattern lookback; no workgroup barrier anywhere.
#ifndef DNRP_SS_SUMG
#define DNRP_SS_SUMG 8  // step-sum samples per group of LDS reads in flight (two halves of 8)
#endif
#ifndef DNRP_SS_LAZY
#define DNRP_SS_LAZY 0  // 1: the FIR window read from LDS as consumed (pp_const::run_lds), not all at once
#endif
#ifndef DNRP_SS_IMAJ
#define DNRP_SS_IMAJ 1  // the FIR window input-major from LDS (pp_const::run_imaj): 131 VGPRs against 159, sync_steps
                        // 13.80 -> 13.31 ms per C4 chunk at the same 11 waves per CU (0: window loaded whole)
#endif
#ifndef DNRP_SS_LOOK
#define DNRP_SS_LOOK 2  // FIR window inputs loaded this many delay rows ahead (pp_const::run_lds)
#endif
#ifndef DNRP_SS_WPE
#define DNRP_SS_WPE 1  // waves per SIMD the register budget must allow (1: the compiler's choice)
#endif
#ifndef DNRP_SS_RING
#define DNRP_SS_RING 1024  // power of two >= 64 * 9 + step + pattern + 9 (host-checked)
#endif
constexpr uint32_t SS_RING = DNRP_SS_RING;
// the pipelined kernel's ring (sync_steps_pipe_kernel). Measured alternative (DESIGN.md
// §6.2): 912 slots (a multiple of 16, so a 16-slot step-sum read never wraps; holds the C4 lookback of
// 64 * 9 + step + pattern + 9 = 905) with the FIR window read lazily (DNRP_SS_LAZY=1) and 4-sample
// step-sum groups (DNRP_SS_SUMG=4): 126 VGPRs and 12.3 KiB, 12 waves per CU instead of 11 -- sync_steps
// 14.17 -> 15.07 ms per 16384-slot chunk (the mod-912 indices and shorter read groups cost more than
// the wave gains); 1024 / lazy / 4: 14.33 ms. Kept: 1024, one load group, two halves of 8.
#ifndef DNRP_SS_PRING
#define DNRP_SS_PRING 1024
#endif
constexpr uint32_t SS_PRING = DNRP_SS_PRING;
static_assert(SS_PRING % 16 == 0, "16-slot step-sum reads stay inside the ring");
__device__ __forceinline__ uint32_t pring(int64_t m) {  // m mod SS_PRING for -2^20 <= m < 2^31 - 2^21
    if constexpr ((SS_PRING & (SS_PRING - 1)) == 0) return static_cast<uint32_t>(m) & (SS_PRING - 1);
    // 32-bit: a constant-divisor modulo is a multiply-high and a few adds, the 64-bit one an emulation
    constexpr uint32_t OFF = ((1u << 20) + SS_PRING - 1) / SS_PRING * SS_PRING;
    return (static_cast<uint32_t>(static_cast<int32_t>(m)) + OFF) % SS_PRING;
}
constexpr uint32_t SS_WPG = 4;

template <int LR, int MR, int HLR>
__host__ __device__ constexpr uint32_t ss_inbuf() {  // float2 per wave, 16-B multiple
    return ((HLR + 1 + ((LR - 1) * MR) / LR - MR) + 64 * MR + 1) / 2 * 2;
}

template <int LR, int MR, int HLR, int SQ, int WPG = SS_WPG>
__global__ void __launch_bounds__(64 * SS_WPG) sync_steps_stream_kernel(sync_args A, uint32_t seg_steps, uint32_t n_seg) {
    using PD = pp_direct<LR, MR, HLR>;
    constexpr int W = PD::W, CARRY = W - MR, NEW = 64 * MR;
    constexpr uint32_t INB = ss_inbuf<LR, MR, HLR>();
    extern __shared__ __attribute__((aligned(16))) float2 smem[];
    const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63u;  // uniform
    float2* inb = smem + wv * (INB + SS_RING);
    float2* ring = inb + INB;
    const uint32_t gw = blockIdx.x * WPG + wv;
    const uint32_t seg = gw % n_seg, a = (gw / n_seg) % A.n_ant, w = gw / (n_seg * A.n_ant);
    if (w >= A.n_win) return;  // no barriers below: a retired wave stalls nobody
    const uint32_t s_a = seg * seg_steps, s_b = min(s_a + seg_steps, A.n_steps);
    if (s_a >= s_b) return;
    const int64_t step = A.step, P = A.pattern;
    const int64_t m_lo = max<int64_t>(0, s_a * step - P), m_hi = s_b * step;
    const int64_t ms = A.m_star;
    const int64_t qa = floordiv(m_lo - ms, LR), qb = floordiv(m_hi - 1 - ms, LR);
    const uint32_t nch = static_cast<uint32_t>((qb - qa + 64) / 64);
    const float2* __restrict__ x = A.iq + w * A.win_stride + a * A.ant_stride;
    const int64_t S = A.S_win;
    const float* taps_g = A.taps;
    auto ld = [&](int64_t q) { return (q >= 0 && q < S) ? x[q] : make_float2(0.f, 0.f); };
    // chunk c: blocks qa + 64 c + lane, window inputs [ib_c, ib_c + CARRY + NEW), ib_c = p_star + M qc - HL
    const int64_t ib0 = static_cast<int64_t>(A.p_star) + MR * qa - HLR;
    float2 pre[MR];
#pragma unroll
    for (int j = 0; j < MR; ++j) pre[j] = ld(ib0 + CARRY + j * 64 + lane);
    if (lane < CARRY) inb[lane] = ld(ib0 + lane);
    uint32_t s_next = s_a;
    const uint32_t sq = A.step >> 2;  // samples per lane quarter of a step
    for (uint32_t c = 0; c < nch; ++c) {
#pragma unroll
        for (int j = 0; j < MR; ++j) inb[CARRY + j * 64 + lane] = pre[j];
        if (c + 1 < nch) {
            const int64_t ibn = ib0 + static_cast<int64_t>(c + 1) * NEW;
#pragma unroll
            for (int j = 0; j < MR; ++j) pre[j] = ld(ibn + CARRY + j * 64 + lane);
        }
        __builtin_amdgcn_wave_barrier();
        float2 xv[W];
        if constexpr ((MR & 1) == 0) PD::template load<true>(inb + MR * lane, xv);
        else PD::template load<false>(inb + MR * lane, xv);
        float2 y[LR];
        {
            // opaque per chunk: the taps are re-read (scalar loads, K$ hits) instead of being hoisted
            // into more SGPRs than a wave has
            const float* tp = taps_g;
            asm volatile("" : "+s"(tp));
            PD::run(xv, (ctap_ptr)(tp), y);
        }
        const int64_t mb = ms + LR * (qa + 64 * static_cast<int64_t>(c) + lane);
        // unconditional: outputs m < 0 (first block only) land in slots that outputs 1024 - L..1023
        // overwrite before any step reads them, and keeping the stores unconditional keeps the
        // compiler from sinking the FMAs into per-output branches
#pragma unroll
        for (int k = 0; k < LR; ++k) ring[static_cast<uint32_t>(mb + k) & (SS_RING - 1)] = y[k];
        // carry: the last W - M inputs of this window start the next one (disjoint from the reads)
        if (lane < CARRY) inb[lane] = inb[NEW + lane];
        __builtin_amdgcn_wave_barrier();
        // steps complete in the ring: 4 lanes per step, a quarter each, bank-rotated walk
        const int64_t m_end = ms + LR * (qa + 64 * static_cast<int64_t>(c) + 64);
        const uint32_t s_end = static_cast<uint32_t>(min<int64_t>(s_b, m_end >= 0 ? m_end / step : 0));
        for (uint32_t sb = s_next; sb < s_end; sb += 16) {
            const uint32_t s = sb + (lane >> 2), part = lane & 3u;
            const uint32_t rot = (2u * ((lane >> 2) & 7u) + ((part >> 1) & 1u) + (lane >> 5)) % sq;
            float pw = 0.f;
            float2 cc = make_float2(0.f, 0.f);
            if (s < s_end) {
                const uint32_t n0 = s * A.step + part * sq;
                const bool corr = static_cast<int64_t>(s) * step >= P;
                if (SQ > 0) {
                    // quarter of 16 samples: n0 and the pattern lag are multiples of 16, so the
                    // quarter never wraps the ring; all 32 reads issue back to back
                    const float2* rv = ring + (n0 & (SS_RING - 1));
                    const float2* ru = ring + ((n0 - A.pattern) & (SS_RING - 1));
                    float2 v[SQ > 0 ? SQ : 1], u[SQ > 0 ? SQ : 1];
#pragma unroll
                    for (int j = 0; j < SQ; ++j) {
                        const uint32_t jj = (j + rot) & (SQ - 1);
                        v[j] = rv[jj];
                        u[j] = corr ? ru[jj] : make_float2(0.f, 0.f);
                    }
#pragma unroll
                    for (int j = 0; j < SQ; ++j) {
                        pw = fmaf(v[j].x, v[j].x, fmaf(v[j].y, v[j].y, pw));
                        cc.x = fmaf(u[j].x, v[j].x, fmaf(u[j].y, v[j].y, cc.x));
                        cc.y = fmaf(u[j].y, v[j].x, fmaf(-u[j].x, v[j].y, cc.y));
                    }
                } else {
                    for (uint32_t j = 0; j < sq; ++j) {
                        uint32_t jj = j + rot;
                        if (jj >= sq) jj -= sq;
                        const uint32_t n = n0 + jj;
                        const float2 v = ring[n & (SS_RING - 1)];
                        pw = fmaf(v.x, v.x, fmaf(v.y, v.y, pw));
                        if (corr) {
                            const float2 u = ring[(n - A.pattern) & (SS_RING - 1)];
                            cc.x = fmaf(u.x, v.x, fmaf(u.y, v.y, cc.x));
                            cc.y = fmaf(u.y, v.x, fmaf(-u.x, v.y, cc.y));
                        }
                    }
                }
            }
#pragma unroll
            for (int o = 1; o < 4; o <<= 1) {
                pw += __shfl_xor(pw, o);
                cc.x += __shfl_xor(cc.x, o);
                cc.y += __shfl_xor(cc.y, o);
            }
            if (s < s_end && part == 0) {
                const size_t o = (static_cast<size_t>(w) * A.n_ant + a) * A.n_steps + s;
                A.P[o] = pw;
                A.Cs[o] = cc;
            }
        }
        s_next = max(s_next, s_end);
        __builtin_amdgcn_wave_barrier();
    }
}

// ---- the streaming path for 64-sample steps with two chunks of loads in flight per wave
// (sync_steps_stream_kernel<.., 16, 1> restated): the window is read through a range-checked buffer
// descriptor (samples outside [0, S_win) read as zeros, no branches), the P / C step values are
// stored the same way, and a chunk completes at most 10 steps (576 outputs), so every chunk issues
// a fixed number of memory instructions. The waits for a chunk's loads are then counted vmcnt(n)
// with the next chunk's loads still in flight, instead of draining the queue.
template <int LR, int MR, int HLR, bool CT>
__device__ __forceinline__ void ss_pipe_chunk(const sync_args& A, float2* inb, float2* ring, float2 (&pre)[MR],
                                              __amdgpu_buffer_rsrc_t xr, __amdgpu_buffer_rsrc_t pr,
                                              __amdgpu_buffer_rsrc_t cr, int64_t ib0, int64_t qa, uint32_t c,
                                              uint32_t s_b, uint32_t& s_next, uint32_t lane) {
    using PD = pp_direct<LR, MR, HLR>;
    constexpr int W = PD::W, CARRY = W - MR, NEW = 64 * MR;
    const int64_t step = A.step, ms = A.m_star;
#pragma unroll
    for (int j = 0; j < MR; ++j) inb[CARRY + j * 64 + lane] = pre[j];
    {  // the chunk after next (past the segment: harmless reads, range-checked)
        const int64_t ibn = ib0 + static_cast<int64_t>(c + 2) * NEW + CARRY + lane;
#pragma unroll
        for (int j = 0; j < MR; ++j) {
            typedef uint32_t u2 __attribute__((ext_vector_type(2)));
            // cache policy nt: the window row is streamed once by this wave
            const u2 v = __builtin_amdgcn_raw_buffer_load_b64(xr, static_cast<uint32_t>((ibn + j * 64) * 8), 0, 2);
            pre[j] = make_float2(__uint_as_float(v.x), __uint_as_float(v.y));
        }
    }
    __builtin_amdgcn_wave_barrier();
    float2 y[LR];
    if constexpr (CT) {
#if DNRP_SS_IMAJ
        pp_const<taps_sync_9_10>::run_imaj(inb + MR * lane, y);  // inb 16-B aligned, MR even
#elif DNRP_SS_LAZY
        pp_const<taps_sync_9_10>::run_lds<DNRP_SS_LOOK>(inb + MR * lane, y);
#else
        float2 xv[W];
        if constexpr ((MR & 1) == 0) PD::template load<true>(inb + MR * lane, xv);
        else PD::template load<false>(inb + MR * lane, xv);
        pp_const<taps_sync_9_10>::run(xv, y);
#endif
    } else {
        float2 xv[W];
        if constexpr ((MR & 1) == 0) PD::template load<true>(inb + MR * lane, xv);
        else PD::template load<false>(inb + MR * lane, xv);
        const float* tp = A.taps;
        asm volatile("" : "+s"(tp));
        PD::run(xv, (ctap_ptr)(tp), y);
    }
    const int64_t mb = ms + LR * (qa + 64 * static_cast<int64_t>(c) + lane);
    if constexpr ((SS_PRING & (SS_PRING - 1)) == 0) {
#pragma unroll
        for (int k = 0; k < LR; ++k) ring[static_cast<uint32_t>(mb + k) & (SS_PRING - 1)] = y[k];
    } else {
        const uint32_t rb = pring(mb);  // the block's 9 outputs: at most one wrap
#pragma unroll
        for (int k = 0; k < LR; ++k) ring[rb + k >= SS_PRING ? rb + k - SS_PRING : rb + k] = y[k];
    }
    if (lane < CARRY) inb[lane] = inb[NEW + lane];
    __builtin_amdgcn_wave_barrier();
    const int64_t m_end = ms + LR * (qa + 64 * static_cast<int64_t>(c) + 64);
    const uint32_t s_end = static_cast<uint32_t>(min<int64_t>(s_b, m_end >= 0 ? m_end / step : 0));
    // one pass of 16 steps covers the chunk's (<= 10) completed steps: 4 lanes per step, a quarter each
    const uint32_t s = s_next + (lane >> 2), part = lane & 3u;
    const uint32_t rot = (2u * ((lane >> 2) & 7u) + ((part >> 1) & 1u) + (lane >> 5)) % 16u;
    const bool live = s < s_end;
    const uint32_t n0 = (live ? s : s_next) * 64u + part * 16u;
    const bool corr = live && static_cast<int64_t>(s) * step >= A.pattern;
    const float2* rv = ring + pring(n0);
    const float2* ru = ring + pring(static_cast<int64_t>(n0) - A.pattern);
    float pw = 0.f;
    float2 cc = make_float2(0.f, 0.f);
    constexpr int SG = DNRP_SS_SUMG;  // samples per group of reads in flight (same summation order)
#pragma unroll
    for (int h = 0; h < 16 / SG; ++h) {
        float2 v[SG], u[SG];
#pragma unroll
        for (int j = 0; j < SG; ++j) {
            const uint32_t jj = (SG * h + j + rot) & 15u;
            v[j] = rv[jj];
            u[j] = ru[jj];
        }
#pragma unroll
        for (int j = 0; j < SG; ++j) {
            pw = fmaf(v[j].x, v[j].x, fmaf(v[j].y, v[j].y, pw));
            cc.x = fmaf(u[j].x, v[j].x, fmaf(u[j].y, v[j].y, cc.x));
            cc.y = fmaf(u[j].y, v[j].x, fmaf(-u[j].x, v[j].y, cc.y));
        }
    }
    // a step before the first full lag has no correlation term: dropped once here, not per sample
    // (the sums of zero products were +0, as the select gives)
    if (!corr) cc = make_float2(0.f, 0.f);
    if (!live) {
        pw = 0.f;
        cc = make_float2(0.f, 0.f);
    }
#pragma unroll
    for (int o = 1; o < 4; o <<= 1) {
        pw += __shfl_xor(pw, o);
        cc.x += __shfl_xor(cc.x, o);
        cc.y += __shfl_xor(cc.y, o);
    }
    const bool st = live && part == 0;
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(pw), pr, st ? s * 4u : 0x80000000u, 0, 0);
    typedef uint32_t u2 __attribute__((ext_vector_type(2)));
    const u2 cv = {__float_as_uint(cc.x), __float_as_uint(cc.y)};
    __builtin_amdgcn_raw_buffer_store_b64(cv, cr, st ? s * 8u : 0x80000000u, 0, 0);
    s_next = max(s_next, s_end);
    __builtin_amdgcn_wave_barrier();
}

template <int LR, int MR, int HLR, bool CT>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(DNRP_SS_WPE))) sync_steps_pipe_kernel(sync_args A, uint32_t seg_steps, uint32_t n_seg) {
    using PD = pp_direct<LR, MR, HLR>;
    constexpr int W = PD::W, CARRY = W - MR, NEW = 64 * MR;
    constexpr uint32_t INB = ss_inbuf<LR, MR, HLR>();
    extern __shared__ __attribute__((aligned(16))) float2 smem[];
    const uint32_t lane = threadIdx.x & 63u;
    float2* inb = smem;
    float2* ring = inb + INB;
    const uint32_t gw = blockIdx.x;
    const uint32_t seg = gw % n_seg, a = (gw / n_seg) % A.n_ant, w = gw / (n_seg * A.n_ant);
    if (w >= A.n_win) return;
    const uint32_t s_a = seg * seg_steps, s_b = min(s_a + seg_steps, A.n_steps);
    if (s_a >= s_b) return;
    const int64_t step = A.step, P = A.pattern;
    const int64_t m_lo = max<int64_t>(0, s_a * step - P), m_hi = s_b * step;
    const int64_t ms = A.m_star;
    const int64_t qa = floordiv(m_lo - ms, LR), qb = floordiv(m_hi - 1 - ms, LR);
    const uint32_t nch = static_cast<uint32_t>((qb - qa + 64) / 64);
    // range-checked rows: the window row (zeros outside [0, S_win)) and the step-value rows. The
    // window row's range ends at the segment's last input: the prefetches past the segment (the two
    // chunks after its last) return zeros without a memory request (they were 6 % of the bytes)
    const float2* x = A.iq + w * A.win_stride + a * A.ant_stride;
    const size_t orow = (static_cast<size_t>(w) * A.n_ant + a) * A.n_steps;
    const int64_t ib0 = static_cast<int64_t>(A.p_star) + MR * qa - HLR;
    const int64_t in_end = experiment(XS_SYNC_NOCLAMP) ? int64_t(A.S_win)
                                                       : min<int64_t>(A.S_win, max<int64_t>(0, ib0 + int64_t(NEW) * nch + CARRY));
    const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(const_cast<float2*>(x), 0, static_cast<int>(in_end * 8), 0x00020000);
    const __amdgpu_buffer_rsrc_t pr = __builtin_amdgcn_make_buffer_rsrc(A.P + orow, 0, static_cast<int>(A.n_steps * 4u), 0x00020000);
    const __amdgpu_buffer_rsrc_t cr = __builtin_amdgcn_make_buffer_rsrc(A.Cs + orow, 0, static_cast<int>(A.n_steps * 8u), 0x00020000);
    typedef uint32_t u2 __attribute__((ext_vector_type(2)));
    auto ldb = [&](int64_t q) {
        const u2 v = __builtin_amdgcn_raw_buffer_load_b64(xr, static_cast<uint32_t>(q * 8), 0, 0);
        return make_float2(__uint_as_float(v.x), __uint_as_float(v.y));
    };
    float2 pa[MR], pb[MR];
#pragma unroll
    for (int j = 0; j < MR; ++j) pa[j] = ldb(ib0 + CARRY + j * 64 + lane);
#pragma unroll
    for (int j = 0; j < MR; ++j) pb[j] = ldb(ib0 + NEW + CARRY + j * 64 + lane);
    if (lane < CARRY) inb[lane] = ldb(ib0 + lane);
    uint32_t s_next = s_a;
    for (uint32_t c = 0; c < nch; c += 2) {  // chunk c + 1 >= nch: harmless work, no stores
        ss_pipe_chunk<LR, MR, HLR, CT>(A, inb, ring, pa, xr, pr, cr, ib0, qa, c, s_b, s_next, lane);
        ss_pipe_chunk<LR, MR, HLR, CT>(A, inb, ring, pb, xr, pr, cr, ib0, qa, c + 1, s_b, s_next, lane);
    }
}

// ===================================================================== detection + coarse peak
struct det_eval {
    float rms, metric;
};

// autocorrelator_detection.cpp:186-280 at the step whose B block starts at s*step (movsums after
// the push: power over the last 4*n_pattern step values, correlation over the last 4*(n_pattern-1)
// with the cover pairwise products per group of 4; front = newest + oldest register, back = the
// two after the oldest: movsum.hpp get_sum_front/get_sum_back with ptr at the oldest element)
// P[i], Cs[i]: step values of step index i (global, or LDS copies addressed through offset pointers)
__device__ __forceinline__ bool detect_eval(const sync_args& A, const float* __restrict__ P, const float2* __restrict__ Cs,
                                            uint32_t s, det_eval& out) {
    const uint32_t np = 4 * A.n_pattern, nc = 4 * A.n_uw;
    // unrolled so each batch of loads is in flight together; the sums keep the reference's order
    double pw = 0.0;
#pragma unroll 8
    for (uint32_t i = 0; i < np; ++i) pw += P[s - (np - 1) + i];
    const double rms = sqrt(pw / static_cast<double>(A.stf_len));
    static_assert(prm::SYNC_RMS_FRONT_STEPS == 2 && prm::SYNC_RMS_BACK_STEPS == 2, "front/back register pairs");
    if (rms < static_cast<double>(A.rms_min) || static_cast<double>(prm::SYNC_RMS_MAX) < rms) return false;
    const double back = static_cast<double>(P[s - (np - 2)]) + P[s - (np - 3)];
    const double front = static_cast<double>(P[s - (np - 1)]) + P[s];
    if (sqrt(back) * prm::SYNC_RMS_FRONT_TO_BACK_RATIO >= sqrt(front)) return false;
    double cr = 0.0, ci = 0.0;
#pragma unroll 4
    for (uint32_t g = 0; g < A.n_uw; ++g) {
        double gr = 0.0, gi = 0.0;
        for (uint32_t j = 0; j < 4; ++j) {
            const float2 v = Cs[s - (nc - 1) + 4 * g + j];
            gr += v.x;
            gi += v.y;
        }
        cr += A.uw[g] * gr;
        ci += A.uw[g] * gi;
    }
    const double q = static_cast<double>(A.prefactor) * sqrt(cr * cr + ci * ci) / pw;
    const double metric = q * q;
    static_assert(prm::SYNC_METRIC_STREAK == 1 && prm::SYNC_METRIC_STREAK_GAIN == 0.0f, "single-step streak");
    if (metric < static_cast<double>(prm::SYNC_METRIC_MIN) || static_cast<double>(prm::SYNC_METRIC_MAX) < metric)
        return false;
    if (!(static_cast<double>(prm::SYNC_METRIC_MIN) < metric)) return false;  // streak_t(0.18, 0, 1)::check
    out.rms = static_cast<float>(rms);
    out.metric = static_cast<float>(metric);
    return true;
}

// exclusive prefix of n double2 values in v[] (in place), one wavefront; v[n] = total
__device__ void wave_scan_d2(double2* v, uint32_t n, uint32_t lane) {
    const uint32_t per = (n + 63) / 64;
    const uint32_t b = lane * per, e = min(b + per, n);
    double sx = 0.0, sy = 0.0;
    for (uint32_t i = b; i < e; ++i) {
        sx += v[i].x;
        sy += v[i].y;
    }
    double ix = sx, iy = sy;  // inclusive scan over lanes
    for (int o = 1; o < 64; o <<= 1) {
        const double tx = __shfl_up(ix, o), ty = __shfl_up(iy, o);
        if (static_cast<int>(lane) >= o) {
            ix += tx;
            iy += ty;
        }
    }
    double rx = ix - sx, ry = iy - sy;
    for (uint32_t i = b; i < e; ++i) {
        const double2 t = v[i];
        v[i] = make_double2(rx, ry);
        rx += t.x;
        ry += t.y;
    }
    if (lane == 63) v[n] = make_double2(ix, iy);
}

#ifdef DNRP_SYNC_PROFILE
#define SYNC_STAMP(i) \
    if (threadIdx.x == 0 && A.prof) A.prof[size_t(w) * 32 + (i)] = wall_clock64()
#else
#define SYNC_STAMP(i)
#endif

struct peak_lds {
    double2* ckc;  // correlation prefix at every 16th product
    double* ckp;   // power prefix at every 16th sample
    float* met;    // metric per position of the peak search (float, as the reference's movsum stages)
};

// autocorrelator_peak.cpp:145-264 for one antenna: per-sample metric over [r0, r0 + D), smoothed
// by the (2 bos + 1)-long moving mean (zero-initialised), last maximum wins (update on >=).
// lbuf[i] = lb[yb + i], yb = r0 - stf_len - SYNC_PAD_PEAK.
__device__ void peak_search(const sync_args& A, const float2* lbuf, uint32_t region, const peak_lds& L, uint32_t r0,
                            double* red, float& pk_metric, uint32_t& pk_idx) {
    const uint32_t P = A.pattern, yoff = A.stf_len + SYNC_PAD_PEAK;  // lbuf index of r0
    const uint32_t nprod = region - P, nsc = (nprod + 15) / 16, nsp = (region + 15) / 16;
    // segment sums: products prod(y) = lb[y-P] conj(lb[y]) indexed from lbuf index P; powers from 0
    // (each thread starts its 16-sample segment at its own rotation: segment starts are 32 banks
    // apart, so an unrotated walk would put a half-wave on two bank pairs)
    for (uint32_t g = threadIdx.x; g < nsc + nsp; g += blockDim.x) {
        if (g < nsc) {
            double sx = 0.0, sy = 0.0;
            for (uint32_t t = 0; t < 16; ++t) {
                const uint32_t j = 16 * g + ((t + g) & 15u);
                if (j >= nprod) continue;
                const float2 c = cmulc(lbuf[j], lbuf[j + P]);
                sx += c.x;
                sy += c.y;
            }
            L.ckc[g] = make_double2(sx, sy);
        } else {
            const uint32_t h = g - nsc;
            double sp = 0.0;
            for (uint32_t t = 0; t < 16; ++t) {
                const uint32_t j = 16 * h + ((t + h) & 15u);
                if (j < region) sp += cnorm(lbuf[j]);
            }
            L.ckp[h] = sp;
        }
    }
    __syncthreads();
#ifdef DNRP_SYNC_PROFILE
    const uint32_t w = blockIdx.x;
#endif
    SYNC_STAMP(12);
    const uint32_t wv = threadIdx.x >> 6, lane = threadIdx.x & 63u;
    if (wv == 0) wave_scan_d2(L.ckc, nsc, lane);
    if (wv == 1) {  // power prefix: scan as double2 with zero imaginary parts via a temporary view
        const uint32_t per = (nsp + 63) / 64;
        const uint32_t b = lane * per, e = min(b + per, nsp);
        double s = 0.0;
        for (uint32_t i = b; i < e; ++i) s += L.ckp[i];
        double inc = s;
        for (int o = 1; o < 64; o <<= 1) {
            const double t = __shfl_up(inc, o);
            if (static_cast<int>(lane) >= o) inc += t;
        }
        double r = inc - s;
        for (uint32_t i = b; i < e; ++i) {
            const double t = L.ckp[i];
            L.ckp[i] = r;
            r += t;
        }
        if (lane == 63) L.ckp[nsp] = inc;
    }
    __syncthreads();
    SYNC_STAMP(13);
    // prefix helpers: PC(z) = sum of prod with product index < z; PP(z) = sum of power index < z
    auto PC = [&](uint32_t z, double& rx, double& ry) {
        const uint32_t g = z >> 4;
        double2 c = L.ckc[g];
        for (uint32_t j = 16 * g; j < z; ++j) {
            const float2 v = cmulc(lbuf[j], lbuf[j + P]);
            c.x += v.x;
            c.y += v.y;
        }
        rx = c.x;
        ry = c.y;
    };
    auto PP = [&](uint32_t z) {
        const uint32_t g = z >> 4;
        double p = L.ckp[g];
        for (uint32_t j = 16 * g; j < z; ++j) p += cnorm(lbuf[j]);
        return p;
    };
    const uint32_t D = A.D, per = (D + blockDim.x - 1) / blockDim.x;
    const uint32_t xb = threadIdx.x * per, xe = min(xb + per, D);
    const uint32_t Lw = P * A.n_uw;  // correlation window (products)
    // metric(x), x = r0 + i: corr over products y in [x - Lw + 1, x]; product index of y = (y - yb) - P
    if (xb < xe) {
        const uint32_t pi_end = yoff + xb - P + 1;  // product index just past y = x
        double cr = 0.0, ci = 0.0;
        for (uint32_t k = 0; k <= A.n_uw; ++k) {
            const float ck = (k > 0 ? A.uw[k - 1] : 0.f) - (k < A.n_uw ? A.uw[k] : 0.f);
            if (ck == 0.f) continue;
            double rx, ry;
            PC(pi_end - Lw + P * k, rx, ry);
            cr += ck * rx;
            ci += ck * ry;
        }
        double pw = PP(yoff + xb + 1) - PP(yoff + xb + 1 - A.stf_len);
        for (uint32_t i = xb; i < xe; ++i) {
            if (i > xb) {  // slide by one sample: every prefix point advances by one product / sample
                const uint32_t pe = yoff + i - P;  // product index entering (y = x)
                for (uint32_t k = 0; k <= A.n_uw; ++k) {
                    const float ck = (k > 0 ? A.uw[k - 1] : 0.f) - (k < A.n_uw ? A.uw[k] : 0.f);
                    if (ck == 0.f) continue;
                    const float2 v = cmulc(lbuf[pe - Lw + P * k], lbuf[pe - Lw + P * k + P]);
                    cr += ck * static_cast<double>(v.x);
                    ci += ck * static_cast<double>(v.y);
                }
                pw += static_cast<double>(cnorm(lbuf[yoff + i])) - static_cast<double>(cnorm(lbuf[yoff + i - A.stf_len]));
            }
            // (prefactor |c| / pw)^2 without the square root (equal to double rounding, stored as float)
            const double pf = static_cast<double>(A.prefactor);
            L.met[i] = static_cast<float>(pf * pf * (cr * cr + ci * ci) / (pw * pw));
        }
    }
    __syncthreads();
    SYNC_STAMP(14);
    // smoother (length 2 bos + 1, zero history) and last-maximum argmax
    const uint32_t ns = (prm::SYNC_PEAK_SMOOTH_LEFT + prm::SYNC_PEAK_SMOOTH_RIGHT) * A.bos + 1;
    double best = -1.0;
    uint32_t bidx = 0;
    if (xb < xe) {
        double sm = 0.0;
        for (uint32_t j = 0; j < ns; ++j)
            if (xb >= j) sm += L.met[xb - j];
        for (uint32_t i = xb; i < xe; ++i) {
            if (i > xb) {
                sm += L.met[i];
                if (i >= ns) sm -= L.met[i - ns];
            }
            const double mean = sm / static_cast<double>(ns);
            if (mean >= best) {
                best = mean;
                bidx = i;
            }
        }
    }
    // block argmax: largest value, latest index among equal values
    for (int o = 32; o > 0; o >>= 1) {
        const double ob = __shfl_xor(best, o);
        const uint32_t oi = __shfl_xor(bidx, o);
        if (ob > best || (ob == best && oi > bidx)) {
            best = ob;
            bidx = oi;
        }
    }
    __syncthreads();
    if (lane == 0) {
        red[2 * wv] = best;
        reinterpret_cast<uint32_t*>(red + 16)[wv] = bidx;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (uint32_t v = 1; v < (blockDim.x >> 6); ++v) {
            const double ob = red[2 * v];
            const uint32_t oi = reinterpret_cast<uint32_t*>(red + 16)[v];
            if (ob > best || (ob == best && oi > bidx)) {
                best = ob;
                bidx = oi;
            }
        }
        pk_metric = static_cast<float>(best);
        pk_idx = r0 + bidx - prm::SYNC_PEAK_SMOOTH_RIGHT * A.bos;  // metric_smoother_bos_offset_to_center_samples
    }
    __syncthreads();
}


// three waves per SIMD (<= 168 VGPRs, a few spills in the post-processing): with three workgroups'
// LDS per CU this beats the 2-wave default in the pipelined bench (A/B on MI355X: 181.4k vs 184.9k
// slot-pairs/s)
#ifndef SYNC_DETECT_ATTR
#define SYNC_DETECT_ATTR __attribute__((amdgpu_waves_per_eu(SPLIT ? DNRP_DET_SPLIT_WPE : 3)))
#endif
// the split form (detection conditions only, no resampling, small LDS): its own register budget
#ifndef DNRP_DET_SPLIT_WPE
#define DNRP_DET_SPLIT_WPE 6  // 69 VGPRs, 7 waves per SIMD (3: the non-split budget, 129 VGPRs)
#endif

struct sync_shared {  // block scalars, at the start of the dynamic LDS (no static __shared__)
    double red[24];
    int s_min;
    float s_rms, s_metric;
    uint32_t s_ant;
    float s_pk_metric[8];
    uint32_t s_pk_idx[8];
};
constexpr uint32_t SYNC_SHARED_F2 = (sizeof(sync_shared) + 15) / 16 * 2;  // float2 slots, 16-B multiple

// The detection / coarse-peak state machine of one window. Two forms of the same loop:
//  SPLIT = false  (sync_detect_kernel): the whole loop in the workgroup, the per-antenna coarse-peak
//                 search inline (resampled STF region in LDS, 3 workgroups per CU);
//  SPLIT = true   (the split rounds): the workgroup runs the detection conditions only and leaves at
//                 the first detection with its state saved (pend = 1); sync_peak_kernel then runs the
//                 coarse-peak search of that detection with one workgroup per (window, antenna), and
//                 the next split launch resumes from the saved state with the peak results. Small
//                 LDS (detection staging only), so many workgroups per CU; the inline form finishes
//                 whatever the split rounds left (several detections or false alarms in one window).
// The split form's coarse-peak search (sync_peak_kernel) evaluates the same metric expression with its
// double sums grouped differently (prefixes on an 8-sample grid): the coarse peaks of the two forms
// agree to double rounding; both are held to the oracle by the same GPU tests (DNRP_SYNC_ROUNDS).
template <int LR, int MR, int HLR, bool SPLIT>
__global__ void __launch_bounds__(SYNC_THREADS) SYNC_DETECT_ATTR sync_detect_kernel(sync_args A) {
    extern __shared__ __attribute__((aligned(16))) float2 smem[];
    sync_shared& sh = *reinterpret_cast<sync_shared*>(smem);
    double* red = sh.red;
    int& s_min = sh.s_min;
    float& s_rms = sh.s_rms;
    float& s_metric = sh.s_metric;
    uint32_t& s_ant = sh.s_ant;
    float* s_pk_metric = sh.s_pk_metric;
    uint32_t* s_pk_idx = sh.s_pk_idx;
    const uint32_t w = blockIdx.x;
    float* taps = reinterpret_cast<float*>(smem + SYNC_SHARED_F2);
    const uint32_t tap_f2 = SPLIT ? 0u : (A.npp + 3) / 4 * 2;
    const uint32_t region = A.stf_len + A.D + SYNC_PAD_PEAK;
    float2* lbuf = smem + SYNC_SHARED_F2 + tap_f2;
    float2* stage = SPLIT ? lbuf : lbuf + (region + 1) / 2 * 2;
    peak_lds pl;  // aliases the staging area (dead once the resampler has run)
    pl.ckc = reinterpret_cast<double2*>(stage);
    pl.ckp = reinterpret_cast<double*>(pl.ckc + (region + 15) / 16 + 2);
    pl.met = reinterpret_cast<float*>(pl.ckp + (region + 15) / 16 + 2);
    // loop registers: the initial state, or the state a split launch saved
    sync_state S0{4u, A.stf_len + A.pattern, 0u, 0u, 0u, 0u, 0.f, 0.f};
    if (!A.first) S0 = A.state[w];
    if (S0.pend == 2) return;  // uniform: finished in an earlier launch
    if (!SPLIT && LR > 1) stage_copy<4>(taps, A.taps_pp, A.npp, threadIdx.x, blockDim.x);
    __syncthreads();
    const float* Pw = A.P + static_cast<size_t>(w) * A.n_ant * A.n_steps;
    const float2* Cw = A.Cs + static_cast<size_t>(w) * A.n_ant * A.n_steps;
    sync_res* out = A.res + static_cast<size_t>(w) * A.max_reports;
    // detection staging (aliases the resampler stage, dead during detection): per antenna det_p
    // powers and det_c correlations
    const uint32_t np = 4 * A.n_pattern, nc = 4 * A.n_uw;
    const uint32_t det_p = (SYNC_THREADS + np + 3) / 4 * 4, det_c = SYNC_THREADS + nc;
    float2* dc = stage;
    float* dp = reinterpret_cast<float*>(dc + A.n_ant * det_c);
    uint32_t nrep = S0.nrep, s_cur = S0.s_cur, ignore = S0.ignore;
    bool resume = S0.pend == 1;  // a saved detection whose coarse peaks sync_peak_kernel has searched
    SYNC_STAMP(0);
    while (nrep < A.max_reports) {
        int sd;
        if (resume) {
            sd = static_cast<int>(S0.sd);
            if (threadIdx.x == 0) {
                s_ant = S0.s_ant;
                s_rms = S0.s_rms;
                s_metric = S0.s_metric;
            }
            if (threadIdx.x < A.n_ant) {
                const float2 r = A.pk[size_t(w) * 8 + threadIdx.x];
                s_pk_metric[threadIdx.x] = r.x;
                s_pk_idx[threadIdx.x] = __float_as_uint(r.y);
            }
            __syncthreads();
        } else {
            // ---------------- detection: first step at or after s_cur meeting the conditions
            if (threadIdx.x == 0) s_min = 0x7FFFFFFF;
            __syncthreads();
            for (uint32_t base = s_cur; base < A.n_steps; base += blockDim.x) {
                // the batch's step values of every antenna in LDS (one coalesced round trip); steps a
                // detection can evaluate have s - (np - 1) >= 0 (ignore >= stf_len + pattern)
                const uint32_t nb = min(blockDim.x, A.n_steps - base);
                const uint32_t lo_p = base >= np - 1 ? base - (np - 1) : 0u, lo_c = base >= nc - 1 ? base - (nc - 1) : 0u;
                const uint32_t len_p = base + nb - lo_p, len_c = base + nb - lo_c;
                for (uint32_t a = 0; a < A.n_ant; ++a) {
                    for (uint32_t i = threadIdx.x; i < len_p; i += blockDim.x) dp[a * det_p + i] = Pw[a * A.n_steps + lo_p + i];
                    for (uint32_t i = threadIdx.x; i < len_c; i += blockDim.x) dc[a * det_c + i] = Cw[a * A.n_steps + lo_c + i];
                }
                __syncthreads();
                const uint32_t s = base + threadIdx.x;
                if (s < A.n_steps && (s + 1) * A.step >= ignore) {
                    for (uint32_t a = 0; a < A.n_ant; ++a) {
                        det_eval e;
                        if (detect_eval(A, dp + a * det_p - lo_p, dc + a * det_c - lo_c, s, e)) {
                            atomicMin(&s_min, static_cast<int>(s));
                            break;
                        }
                    }
                }
                __syncthreads();
                const int found = s_min;
                __syncthreads();
                if (found != 0x7FFFFFFF) break;
            }
            sd = s_min;
            __syncthreads();
            if (sd == 0x7FFFFFFF) break;
            if (threadIdx.x == 0) {
                for (uint32_t a = 0; a < A.n_ant; ++a) {
                    det_eval e;
                    if (detect_eval(A, Pw + a * A.n_steps, Cw + a * A.n_steps, static_cast<uint32_t>(sd), e)) {
                        s_ant = a;
                        s_rms = e.rms;
                        s_metric = e.metric;
                        break;
                    }
                }
            }
            __syncthreads();
            if constexpr (SPLIT) {  // leave with the detection pending: sync_peak_kernel searches its peaks
                if (threadIdx.x == 0)
                    A.state[w] = sync_state{s_cur, ignore, nrep, 1u, static_cast<uint32_t>(sd), s_ant, s_rms, s_metric};
                return;
            }
        }
        SYNC_STAMP(1);
        s_cur = static_cast<uint32_t>(sd) + 1;
        const uint32_t det_time = s_cur * A.step, r0 = det_time - prm::SYNC_JUMP_BACK_PATTERNS * A.pattern;
        const float det_metric = s_metric;
        if (!SPLIT && !resume) {
            // ---------------- coarse peak search over one STF on every antenna
            const int64_t yb = static_cast<int64_t>(r0) - A.stf_len - SYNC_PAD_PEAK;
            for (uint32_t a = 0; a < A.n_ant; ++a) {
                const float2* x = A.iq + w * A.win_stride + a * A.ant_stride;
                sync_resample<LR, MR, HLR>(A, x, yb, region, stage, lbuf, taps, A.det_stage);
                SYNC_STAMP(2 + 2 * min(a, 3u));
                peak_search(A, lbuf, region, pl, r0, red, s_pk_metric[a], s_pk_idx[a]);
                SYNC_STAMP(3 + 2 * min(a, 3u));
            }
        }
        resume = false;
        // post_processing_validity (autocorrelator_peak.cpp:311-364), float as in the reference
        float cm[8];
        float wsum = 0.f, msum = 0.f;
        uint32_t nvalid = 0;
        for (uint32_t a = 0; a < A.n_ant; ++a) {
            cm[a] = 0.f;
            const float m = s_pk_metric[a];
            if (det_metric + prm::SYNC_PEAK_ABOVE_DETECTION >= m) continue;
            if (static_cast<int64_t>(det_time) +
                    static_cast<int64_t>(prm::SYNC_PEAK_DETECTION2PEAK_STFS * static_cast<double>(A.stf_len)) >=
                static_cast<int64_t>(s_pk_idx[a]))
                continue;
            cm[a] = m;
            wsum += m * static_cast<float>(s_pk_idx[a]);
            ++nvalid;
        }
        for (uint32_t a = 0; a < A.n_ant; ++a) msum += cm[a];
        __syncthreads();  // every thread has read the peak results before the next detection overwrites them
        if (nvalid == 0) continue;  // false alarm: detection resumes after this step
        const uint32_t wpk = static_cast<uint32_t>(roundf(wsum / msum));
        if (wpk < A.stf_len - 1) continue;  // STF would start before the chunk (asserted in the reference)
        const uint32_t cpl = wpk - (A.stf_len - 1);
        // post_processing_at_coarse_peak (:366-394, RMS and fractional CFO over the STF at the peak)
        // runs per (report, antenna) in sync_post_kernel, the CFO's antenna sum in sync_fine_kernel:
        // nothing in the detection loop depends on them
        SYNC_STAMP(10);
        if (threadIdx.x == 0) {
            sync_res r{};
            r.found = 1;
            r.det_ant = s_ant;
            r.det_rms = s_rms;
            r.det_metric = det_metric;
            r.det_time = det_time;
            r.det_time_jb = r0;
            r.coarse_local = cpl;
            double g = static_cast<double>(cpl);  // rx_pacer.cpp:306-313
            g *= static_cast<double>(A.M);
            g /= static_cast<double>(A.L);
            r.coarse_64 = static_cast<int64_t>(static_cast<uint32_t>(round(g)));
            for (uint32_t a = 0; a < 8; ++a) {
                r.coarse_metric[a] = a < A.n_ant ? cm[a] : 0.f;
                r.rms[a] = 0.f;  // sync_post_kernel
            }
            r.cfo_frac = 0.f;  // sync_fine_kernel (antenna sum of sync_post_kernel's terms)
            r.cfo_int = 0.f;  // coarse_peak_f_domain.cpp:195-199
            r.u = A.u;
            r.b = A.b;  // coarse_peak_f_domain.cpp:75-120: b of the radio device class
            out[nrep] = r;
        }
        ignore = cpl + static_cast<uint32_t>(prm::SYNC_SKIP_AFTER_PEAK_STFS * static_cast<double>(A.stf_len));  // skip_after_peak
        ++nrep;
        __syncthreads();
    }
    SYNC_STAMP(11);
    if (threadIdx.x == 0) {
        A.n_found[w] = nrep;
        for (uint32_t k = nrep; k < A.max_reports; ++k) out[k].found = 0;
        if (A.state) A.state[w].pend = 2u;
    }
}

// lb[y] for y in [y0, y0 + cnt) of one antenna straight from the window (no LDS staging): each thread
// one polyphase block of L outputs from its W inputs by range-checked buffer loads (zeros outside
// [0, S_win)), put(i, lb[y0 + i]). sync_resample's outputs bit for bit (pp_direct / pp_const sum in
// pp_block's order). CT: the compile-time 9/10 sync taps. No barrier.
template <int LR, int MR, int HLR, bool CT, class PUT>
__device__ __forceinline__ void resample_direct(const sync_args& A, const float2* x, int64_t y0, uint32_t cnt, PUT put) {
    const uint32_t tid = threadIdx.x, T = blockDim.x;
    if constexpr (LR > 1) {
        using PD = pp_direct<LR, MR, HLR>;
        constexpr int W = PD::W;
        const int64_t ms = A.m_star;
        const int64_t q0 = floordiv(y0 - ms, LR), q1 = floordiv(y0 + cnt - ms + LR - 1, LR);
        const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(const_cast<float2*>(x), 0, static_cast<int>(A.S_win * 8u), 0x00020000);
        for (int64_t q = q0 + tid; q < q1; q += T) {
            const int64_t in0 = static_cast<int64_t>(A.p_star) + MR * q - HLR;
            float2 xv[W];
#pragma unroll
            for (int i = 0; i < W; ++i) {  // outside [0, S_win): the range check returns zeros
                typedef uint32_t u2 __attribute__((ext_vector_type(2)));
                const u2 v = __builtin_amdgcn_raw_buffer_load_b64(xr, static_cast<uint32_t>((in0 + i) * 8), 0, 0);
                xv[i] = make_float2(__uint_as_float(v.x), __uint_as_float(v.y));
            }
            float2 y[LR];
            if constexpr (CT) {
                static_assert(taps_sync_9_10::L == LR && taps_sync_9_10::M == MR && taps_sync_9_10::HL == HLR, "taps");
                pp_const<taps_sync_9_10>::run(xv, y);
            } else {
                const float* tp = A.taps;
                asm volatile("" : "+s"(tp));
                PD::run(xv, (ctap_ptr)(tp), y);
            }
            const int64_t mb = ms + LR * q;
#pragma unroll
            for (int k = 0; k < LR; ++k) {
                const int64_t idx = mb + k - y0;
                if (idx >= 0 && idx < static_cast<int64_t>(cnt))
                    put(static_cast<uint32_t>(idx), (mb + k >= 0) ? y[k] : make_float2(0.f, 0.f));
            }
        }
    } else {
        for (uint32_t i = tid; i < cnt; i += T) {
            const int64_t yy = y0 + i;
            float2 acc = make_float2(0.f, 0.f);
            if constexpr (LR == 1) {
                if (yy >= 0 && yy < static_cast<int64_t>(A.S_win)) acc = x[yy];
            } else if (yy >= 0) {  // generic L/M: sync_resample's direct FIR
                const uint64_t t = A.delay + static_cast<uint64_t>(yy) * A.M;
                const int64_t p = static_cast<int64_t>(t / A.L);
                const uint32_t ph = static_cast<uint32_t>(t % A.L);
                for (uint32_t d = 0; d <= A.hl; ++d) {
                    const int64_t q = p - d;
                    if (q < 0 || q >= static_cast<int64_t>(A.S_win)) continue;
                    const float h = A.taps[ph + d * A.L];
                    acc.x = fmaf(x[q].x, h, acc.x);
                    acc.y = fmaf(x[q].y, h, acc.y);
                }
            }
            put(i, acc);
        }
    }
}

// resample_direct for one workgroup with the window span staged in LDS first: the span's inputs
// [ib0, ib0 + n_in) are read by all threads together (coalesced, range-checked: zeros outside
// [0, S_win)) into stage[], then every thread takes the FIR windows of at most two blocks from LDS
// (its own and one tail block -- 9 region outputs per block, so a region of stf_len + D + pad =
// 4640 outputs is 517 blocks for 512 threads), computes them into registers, and after a barrier
// (every window read: stage[] may alias the outputs' slots) hands the outputs to put. One global
// load latency instead of two (the tail blocks' second round), the same sums as resample_direct.
// Preconditions (host, sync_peak_ok): blocks <= 2 T, n_in <= the stage's capacity.
#ifndef DNRP_STAGE_G
#define DNRP_STAGE_G 11  // span loads in flight per thread: sync_peak's 5200-input span by 512 threads and
                         // sync_post's 2600 by 256 in one round trip (6: two)
#endif
template <int LR, int MR, int HLR, bool IMAJ = false, class PUT>
__device__ __forceinline__ void resample_staged(const sync_args& A, const float2* x, int64_t y0, uint32_t cnt,
                                                float2* stage, PUT put) {
    using PD = pp_direct<LR, MR, HLR>;
    constexpr int W = PD::W;
    const uint32_t tid = threadIdx.x, T = blockDim.x;
    const int64_t ms = A.m_star;
    const int64_t q0 = floordiv(y0 - ms, LR), q1 = floordiv(y0 + cnt - ms + LR - 1, LR);
    const uint32_t nb = static_cast<uint32_t>(q1 - q0);
    const int64_t ib0 = static_cast<int64_t>(A.p_star) + MR * q0 - HLR;
    const uint32_t n_in = MR * (nb - 1) + W;
    const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(const_cast<float2*>(x), 0, static_cast<int>(A.S_win * 8u), 0x00020000);
    typedef uint32_t u2 __attribute__((ext_vector_type(2)));
    // indices past the stream end read a range-checked zero; a negative start wraps into the
    // descriptor's "outside" range as well (offsets are unsigned)
    constexpr uint32_t G = DNRP_STAGE_G;  // loads in flight per thread and group
    for (uint32_t i0 = 0; i0 < n_in; i0 += G * T) {
        float2 v[G];
#pragma unroll
        for (uint32_t g = 0; g < G; ++g) {
            const int64_t q = ib0 + i0 + g * T + tid;
            const u2 r = __builtin_amdgcn_raw_buffer_load_b64(xr, q >= 0 ? static_cast<uint32_t>(q * 8) : 0x80000000u, 0, 0);
            v[g] = make_float2(__uint_as_float(r.x), __uint_as_float(r.y));
        }
#pragma unroll
        for (uint32_t g = 0; g < G; ++g)
            if (i0 + g * T + tid < n_in) stage[i0 + g * T + tid] = v[g];
    }
    __syncthreads();
    float2 y[LR], y2[LR];
    const uint32_t b2 = tid + T;
    if constexpr (IMAJ) {  // windows input-major from LDS (stage 16-B aligned, MR even)
        if (tid < nb) pp_const<taps_sync_9_10>::run_imaj(stage + MR * tid, y);
        if (b2 < nb) pp_const<taps_sync_9_10>::run_imaj(stage + MR * b2, y2);
    } else {
        if (tid < nb) {
            float2 xv[W];
            PD::template load<false>(stage + MR * tid, xv);
            pp_const<taps_sync_9_10>::run(xv, y);
        }
        if (b2 < nb) {
            float2 xv[W];
            PD::template load<false>(stage + MR * b2, xv);
            pp_const<taps_sync_9_10>::run(xv, y2);
        }
    }
    __syncthreads();  // every window read before the outputs overwrite the stage
    auto emit = [&](uint32_t b, const float2 (&yy)[LR]) {
        const int64_t mb = ms + LR * (q0 + b);
#pragma unroll
        for (int k = 0; k < LR; ++k) {
            const int64_t idx = mb + k - y0;
            if (idx >= 0 && idx < static_cast<int64_t>(cnt))
                put(static_cast<uint32_t>(idx), (mb + k >= 0) ? yy[k] : make_float2(0.f, 0.f));
        }
    };
    if (tid < nb) emit(tid, y);
    if (b2 < nb) emit(b2, y2);
}

// ---- coarse-peak search of the split rounds (sync_peak_kernel)
// autocorrelator_peak.cpp:145-264 for the pending detection of one (window, antenna), one workgroup
// each. The per-sample metric is the same expression as peak_search's (exact prefix differences in
// double, sliding by one sample), laid out for parallel latency:
//  - the STF region is resampled straight from the window (pp_direct: each thread one polyphase block
//    of L outputs from its W inputs by range-checked buffer loads; no staging round trips);
//  - thread v owns the 8 positions [8v, 8v + 8): every prefix its first position needs sits on the
//    grid z = 8g + 1 (P, the window Lw = P n_uw and stf_len are multiples of 16), so its initial sums
//    are single LDS reads of the inclusive prefixes Q (products) and R (powers) at grid points;
//  - the region buffer is padded by one slot per 32 samples (pidx) and the metric row by one per 8
//    (midx), so the stride-8 accesses of a wave hit distinct banks;
//  - the smoother's initial window sums whole 8-position blocks (blk) instead of 2 bos + 1 samples.
// Double sums in a different order than peak_search: the metric and the smoothed maxima agree to
// double rounding, the argmax to the same tie rules.
__device__ __forceinline__ uint32_t pidx(uint32_t j) { return j + (j >> 5); }
__device__ __forceinline__ uint32_t midx(uint32_t i) { return i + (i >> 3); }

__host__ __device__ inline uint32_t peak8_lbuf(uint32_t region) { return (region + region / 32 + 2) / 2 * 2; }
__host__ __device__ inline uint32_t peak8_nq(uint32_t region, uint32_t P) { return (region - P) / 8 + 2; }
__host__ __device__ inline uint32_t peak8_nr(uint32_t region) { return region / 8 + 2; }
__host__ __device__ inline size_t peak8_alias(uint32_t region, uint32_t P, uint32_t D) {
    const size_t qr = size_t(peak8_nq(region, P)) * 16 + size_t(peak8_nr(region)) * 8;
    const size_t mb = (size_t(D) + D / 8 + 2) / 2 * 2 * 4 + size_t(D / 8) * 8;
    return qr > mb ? qr : mb;
}

// CT: the 9/10 sync resampler's taps compiled in (pp_const<taps_sync_9_10>, host-checked bit for
// bit): immediates next to their FMAs instead of 225 run-time taps held in SGPRs (which spill)
#ifndef DNRP_PEAK_STAGED
#define DNRP_PEAK_STAGED 1  // 1: the STF region's input span staged in LDS first (resample_staged): at 4 waves
                            // per SIMD neutral (2.75 vs 2.72 ms per chunk); what lets the window loads leave
                            // the registers for 6 waves per SIMD below
#endif
#ifndef DNRP_PEAK_IMAJ
#define DNRP_PEAK_IMAJ 1  // the staged windows input-major (pp_const::run_imaj)
#endif
#ifndef DNRP_PEAK_WPE
#define DNRP_PEAK_WPE 6  // 6 waves per SIMD = 3 workgroups per CU (80 VGPRs; the metric's double divisions
                         // spill ~100 B per lane at NUW 8):
                         // 2.76 -> 2.31-2.36 ms per C4 chunk against 4 (104 VGPRs, 2 workgroups per CU)
#endif
template <int LR, int MR, int HLR, bool CT, int NUW>
__global__ void __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(DNRP_PEAK_WPE))) sync_peak_kernel(sync_args A) {
    extern __shared__ __attribute__((aligned(16))) float2 smem[];
    sync_shared& sh = *reinterpret_cast<sync_shared*>(smem);
    double* red = sh.red;
    const uint32_t w = blockIdx.x / A.n_ant, a = blockIdx.x % A.n_ant;
    const sync_state S0 = A.state[w];
    if (S0.pend != 1) return;  // uniform: no detection pending in this window
#ifdef DNRP_SYNC_PROFILE
#define PEAK_STAMP(i) \
    if (threadIdx.x == 0 && a == 0 && A.prof) A.prof[size_t(w) * 32 + 16 + (i)] = wall_clock64()
#else
#define PEAK_STAMP(i)
#endif
    PEAK_STAMP(0);
    const uint32_t P = A.pattern, D = A.D, yoff = A.stf_len + SYNC_PAD_PEAK;
    const uint32_t region = A.stf_len + D + SYNC_PAD_PEAK, nprod = region - P;
    float2* lbuf = smem + SYNC_SHARED_F2;
    double2* Q = reinterpret_cast<double2*>(lbuf + peak8_lbuf(region));
    double* R = reinterpret_cast<double*>(Q + peak8_nq(region, P));
    float* met = reinterpret_cast<float*>(Q);  // after the metric pass (Q, R dead)
    double* blk = reinterpret_cast<double*>(met + (D + D / 8 + 2) / 2 * 2);
    const uint32_t tid = threadIdx.x, T = blockDim.x;
    const uint32_t det_time = (S0.sd + 1) * A.step, r0 = det_time - prm::SYNC_JUMP_BACK_PATTERNS * A.pattern;
    const int64_t yb = static_cast<int64_t>(r0) - A.stf_len - SYNC_PAD_PEAK;
    const float2* x = A.iq + w * A.win_stride + a * A.ant_stride;
    // ---- resampled region lb[yb + i] -> lbuf[pidx(i)] (sync_resample's outputs, bit for bit)
    if constexpr (CT && LR == 9 && DNRP_PEAK_STAGED)
        resample_staged<LR, MR, HLR, DNRP_PEAK_IMAJ>(A, x, yb, region, lbuf, [&](uint32_t i, float2 v) { lbuf[pidx(i)] = v; });
    else
        resample_direct<LR, MR, HLR, CT>(A, x, yb, region, [&](uint32_t i, float2 v) { lbuf[pidx(i)] = v; });
    __syncthreads();
    PEAK_STAMP(1);
    // ---- 8-sample segment sums: products prod[j] = lb[j] conj(lb[j + P]), powers |lb[j]|^2; segment
    // g >= 1 holds j in [8g - 7, 8g], segment 0 j = 0, so the inclusive scan at g is the prefix < 8g + 1
    const uint32_t nq = peak8_nq(region, P) - 1, nr = peak8_nr(region) - 1;
    // all 8 loads of a segment issued together (out-of-range terms read a valid slot and are masked)
    for (uint32_t h = tid; h < nq; h += T) {
        const uint32_t j0 = h == 0 ? 0u : 8 * h - 7, cnt = h == 0 ? 1u : 8u;
        float2 c[8];
#pragma unroll
        for (uint32_t t = 0; t < 8; ++t) {
            const uint32_t j = min(j0 + t, nprod - 1);
            c[t] = cmulc(lbuf[pidx(j)], lbuf[pidx(j + P)]);
        }
        double sx = 0.0, sy = 0.0;
#pragma unroll
        for (uint32_t t = 0; t < 8; ++t)
            if (t < cnt && j0 + t < nprod) {
                sx += c[t].x;
                sy += c[t].y;
            }
        Q[h] = make_double2(sx, sy);
    }
    for (uint32_t h = tid; h < nr; h += T) {
        const uint32_t j0 = h == 0 ? 0u : 8 * h - 7, cnt = h == 0 ? 1u : 8u;
        float p[8];
#pragma unroll
        for (uint32_t t = 0; t < 8; ++t) p[t] = cnorm(lbuf[pidx(min(j0 + t, region - 1))]);
        double sp = 0.0;
#pragma unroll
        for (uint32_t t = 0; t < 8; ++t)
            if (t < cnt && j0 + t < region) sp += p[t];
        R[h] = sp;
    }
    __syncthreads();
    PEAK_STAMP(2);
    const uint32_t wv = tid >> 6, lane = tid & 63u;
    if (wv == 0) wave_scan_d2(Q, nq, lane);  // exclusive: Q[g + 1] = prefix < 8g + 1
    if (wv == 1) {
        const uint32_t per = (nr + 63) / 64;
        const uint32_t b = lane * per, e = min(b + per, nr);
        double sp = 0.0;
        for (uint32_t i = b; i < e; ++i) sp += R[i];
        double inc = sp;
        for (int o = 1; o < 64; o <<= 1) {
            const double t = __shfl_up(inc, o);
            if (static_cast<int>(lane) >= o) inc += t;
        }
        double rr = inc - sp;
        for (uint32_t i = b; i < e; ++i) {
            const double t = R[i];
            R[i] = rr;
            rr += t;
        }
        if (lane == 63) R[nr] = inc;
    }
    __syncthreads();
    PEAK_STAMP(3);
    // ---- metric of the thread's 8 positions (registers)
    const uint32_t Lw = P * A.n_uw, nv = D / 8;
    const double pf = static_cast<double>(A.prefactor);
    float m8[8];
    if (tid < nv) {
        // cover weights ck of the NUW + 1 prefix points (uniform); a zero weight adds an exact zero
        float ck[NUW + 1];
#pragma unroll
        for (int k = 0; k <= NUW; ++k) ck[k] = (k > 0 ? A.uw[k - 1] : 0.f) - (k < NUW ? A.uw[k] : 0.f);
        const uint32_t xb = 8 * tid;
        const uint32_t zb = yoff + xb - P + 1 - Lw;  // = 8g + 1
        double cr = 0.0, ci = 0.0;
        double2 q[NUW + 1];
#pragma unroll
        for (int k = 0; k <= NUW; ++k) q[k] = Q[(zb + P * k - 1) / 8 + 1];
#pragma unroll
        for (int k = 0; k <= NUW; ++k) {
            cr += ck[k] * q[k].x;
            ci += ck[k] * q[k].y;
        }
        double pw = R[(yoff + xb) / 8 + 1] - R[(yoff + xb - A.stf_len) / 8 + 1];
        m8[0] = static_cast<float>(pf * pf * (cr * cr + ci * ci) / (pw * pw));
#pragma unroll
        for (uint32_t ii = 1; ii < 8; ++ii) {
            const uint32_t i = xb + ii;
            const uint32_t pe = yoff + i - P - Lw;  // product index entering (y = x) for k = 0
            float2 u[NUW + 2];
#pragma unroll
            for (int k = 0; k <= NUW + 1; ++k) u[k] = lbuf[pidx(pe + P * k)];
            const float2 s1 = lbuf[pidx(yoff + i)], s0 = lbuf[pidx(yoff + i - A.stf_len)];
#pragma unroll
            for (int k = 0; k <= NUW; ++k) {
                const float2 v = cmulc(u[k], u[k + 1]);
                cr += ck[k] * static_cast<double>(v.x);
                ci += ck[k] * static_cast<double>(v.y);
            }
            pw += static_cast<double>(cnorm(s1)) - static_cast<double>(cnorm(s0));
            m8[ii] = static_cast<float>(pf * pf * (cr * cr + ci * ci) / (pw * pw));
            if (ii & 1) asm volatile("" ::: "memory");  // two slides' loads in flight, not seven (VGPRs)
        }
    }
    __syncthreads();  // Q, R read by every thread: the metric row may overwrite them
    PEAK_STAMP(4);
    if (tid < nv) {
        double bs = 0.0;
#pragma unroll
        for (uint32_t ii = 0; ii < 8; ++ii) {
            met[midx(8 * tid + ii)] = m8[ii];
            bs += m8[ii];
        }
        blk[tid] = bs;
    }
    __syncthreads();
    PEAK_STAMP(5);
    // ---- smoother (length ns = 2 bos + 1, zero history) and last-maximum argmax
    const uint32_t ns = (prm::SYNC_PEAK_SMOOTH_LEFT + prm::SYNC_PEAK_SMOOTH_RIGHT) * A.bos + 1;
    double best = -1.0;
    uint32_t bidx = 0;
    if (tid < nv) {
        const uint32_t xb = 8 * tid, F = (ns - 1) / 8;
        double sm = m8[0];
        for (uint32_t u = 1; u <= F && u <= tid; ++u) sm += blk[tid - u];
        for (uint32_t j = 8 * F + 1; j < ns && j <= xb; ++j) sm += met[midx(xb - j)];
#pragma unroll
        for (uint32_t ii = 0; ii < 8; ++ii) {
            const uint32_t i = xb + ii;
            if (ii > 0) {
                sm += m8[ii];
                if (i >= ns) sm -= met[midx(i - ns)];
            }
            const double mean = sm / static_cast<double>(ns);
            if (mean >= best) {
                best = mean;
                bidx = i;
            }
        }
    }
    for (int o = 32; o > 0; o >>= 1) {
        const double ob = __shfl_xor(best, o);
        const uint32_t oi = __shfl_xor(bidx, o);
        if (ob > best || (ob == best && oi > bidx)) {
            best = ob;
            bidx = oi;
        }
    }
    if (lane == 0) {
        red[wv] = best;  // up to 16 waves: best in red[0, 16), indices in red[16, 24)
        reinterpret_cast<uint32_t*>(red + 16)[wv] = bidx;
    }
    __syncthreads();
    if (tid == 0) {
        for (uint32_t v = 1; v < (T >> 6); ++v) {
            const double ob = red[v];
            const uint32_t oi = reinterpret_cast<uint32_t*>(red + 16)[v];
            if (ob > best || (ob == best && oi > bidx)) {
                best = ob;
                bidx = oi;
            }
        }
        const uint32_t pk_idx = r0 + bidx - prm::SYNC_PEAK_SMOOTH_RIGHT * A.bos;  // metric_smoother_bos_offset_to_center_samples
        A.pk[size_t(w) * 8 + a] = make_float2(static_cast<float>(best), __uint_as_float(pk_idx));
    }
    PEAK_STAMP(6);
}

// ===================================================================== coarse-peak post-processing
// autocorrelator_peak.cpp:366-394 for one (report, antenna): the STF at the coarse peak resampled
// again, its power and cover-weighted pattern correlation (the same loops and block reduction the
// detection kernel ran, so the same doubles) -> rms[a] into the report and the antenna's CFO term
// m_a atan2(c_a) / P into A.post; sync_fine_kernel sums the terms in antenna order. One workgroup
// per (report, antenna) instead of four serial passes inside the detection workgroup.
#ifndef DNRP_POST_STAGED
#define DNRP_POST_STAGED 1
#endif
template <int LR, int MR, int HLR, bool CT>
__global__ void __launch_bounds__(SYNC_THREADS) __attribute__((amdgpu_waves_per_eu(CT && DNRP_POST_STAGED ? 8 : 1))) sync_post_kernel(sync_args A) {
    extern __shared__ __attribute__((aligned(16))) float2 smem[];
    double* red = reinterpret_cast<double*>(smem);  // [24]
    float2* lbuf = smem + 12;  // 16-B aligned (resample_staged's stage)
    const uint32_t rep = blockIdx.x / A.n_ant, a = blockIdx.x % A.n_ant, w = rep / A.max_reports;
    sync_res* rp = A.res + rep;
    const float m = rp->coarse_metric[a];
    if (!rp->found || !(m > 0.f)) return;  // uniform: the whole workgroup leaves
    const float2* x = A.iq + w * A.win_stride + a * A.ant_stride;
    // the STF at the coarse peak (sync_resample's values): compiled-in 9/10 taps -> the span staged in
    // LDS and the FIR input-major from it (DNRP_POST_STAGED, 8 waves per SIMD), else straight from the window
    if constexpr (CT && LR == 9 && DNRP_POST_STAGED)
        resample_staged<LR, MR, HLR, true>(A, x, rp->coarse_local, A.stf_len, lbuf, [&](uint32_t i, float2 v) { lbuf[i] = v; });
    else
        resample_direct<LR, MR, HLR, CT>(A, x, rp->coarse_local, A.stf_len, [&](uint32_t i, float2 v) { lbuf[i] = v; });
    __syncthreads();
    double cr = 0.0, ci = 0.0, pw = 0.0;
    const uint32_t Lw = A.pattern * A.n_uw;
    for (uint32_t i = threadIdx.x; i < A.stf_len; i += blockDim.x) {
        pw += cnorm(lbuf[i]);
        if (i < Lw) {
            const float2 c = cmulc(lbuf[i], lbuf[i + A.pattern]);
            const float u = A.uw[i / A.pattern];
            cr += u * static_cast<double>(c.x);
            ci += u * static_cast<double>(c.y);
        }
    }
    block_sum3(pw, cr, ci, red);
    if (threadIdx.x == 0) {
        rp->rms[a] = sqrtf(static_cast<float>(pw) / static_cast<float>(A.stf_len));
        A.post[size_t(rep) * 8 + a] = m * atan2f(static_cast<float>(ci), static_cast<float>(cr)) / static_cast<float>(A.pattern);
    }
}

// ===================================================================== fine peak
constexpr uint32_t SYNC_FINE_THREADS = 512;  // 8 waves: the FFT passes' butterflies 2 per thread
#ifndef DNRP_FINE_WPE
#define DNRP_FINE_WPE 1  // waves per SIMD the register budget must allow (1: the compiler's choice; radix 8
                         // at 8: 64 VGPRs + 160 B of spills, 1.55-1.57 ms per C4 chunk against 1.50-1.51
                         // at the compiler's 113 VGPRs)
#endif
#ifndef DNRP_FINE_R8
#define DNRP_FINE_R8 1  // 4096-point transforms by fft_r8_4096 (four radix-8 passes; 0: six radix-4 passes):
                        // sync_fine 1.63-1.65 -> 1.50-1.51 ms per C4 chunk (same box)
#endif
#ifndef DNRP_FINE_BATCH
#define DNRP_FINE_BATCH 8  // spectrum x template loads in flight per thread (1: one per loop iteration)
#endif

__global__ void __launch_bounds__(SYNC_FINE_THREADS) __attribute__((amdgpu_waves_per_eu(DNRP_FINE_WPE))) sync_fine_kernel(sync_args A) {
    extern __shared__ __attribute__((aligned(16))) float2 smem[];
    float* s_val = reinterpret_cast<float*>(smem);  // [16]
    uint32_t* s_idx = reinterpret_cast<uint32_t*>(smem + 8);  // [16]
    sync_res* rp = A.res + blockIdx.x;
    if (!rp->found) return;
    const uint32_t w = blockIdx.x / A.max_reports;
    {  // fractional CFO: metric-weighted antenna mean of sync_post_kernel's terms, in antenna order
        float cfo_w = 0.f, msum = 0.f;
        for (uint32_t a = 0; a < A.n_ant; ++a) {
            const float m = rp->coarse_metric[a];
            if (!(m > 0.f)) continue;
            msum += m;
            cfo_w += A.post[size_t(blockIdx.x) * 8 + a];
        }
        __syncthreads();  // every thread has read the report before thread 0 updates it
        if (threadIdx.x == 0) rp->cfo_frac = cfo_w / msum;
        __syncthreads();
    }
    const uint32_t nf = 1u << A.log2_fft;
    // power-of-4 sizes (4096 for C3 / C4): in-place radix-4 DIT on one LDS buffer, the inputs stored
    // at their base-4 digit-reversed positions (ip); otherwise the two-buffer Stockham passes
    const bool ip = (A.log2_fft & 1u) == 0;
    const bool r8 = DNRP_FINE_R8 && A.log2_fft == 12;  // C3 / C4: radix 8, four passes
    // in place: bank-padded slots (r4pad / r8pad), inputs written at their digit-reversed slots
    auto ix = [&](uint32_t i) { return r8 ? r8pad(rev8(i)) : ip ? r4pad(rev4(i, A.log2_fft)) : i; };
    auto ox = [&](uint32_t i) { return r8 ? r8pad(i) : ip ? r4pad(i) : i; };
    auto fft = [&](auto sign, float2* a, float2* b) -> const float2* {
        constexpr int SG = decltype(sign)::value;
        if (r8) {
            fft_r8_4096<SG>(a, A.tw_fft);
            return a;
        }
        if (ip) {
            if (A.log2_fft == 12)  // C3 / C4
                fft_r4_inplace_ct<SG, 12>(a, A.tw_fft);
            else
                fft_r4_inplace<SG, true>(a, A.tw_fft, A.log2_fft);
            return a;
        }
        return fft_pow2<SG>(a, b, A.tw_fft, A.log2_fft);
    };
    const uint32_t nbuf = r8 ? R8_SLOTS : ip ? nf + nf / 32 : nf;  // (the host sizes the LDS the same way)
    float2* xb = smem + 16;
    float2* yb = xb + nbuf;
    // the forward spectrum is read once per template: kept in a global scratch row (L2-resident
    // while the workgroup runs) instead of a third LDS buffer, for two workgroups per CU
    float2* Sb = A.spec + static_cast<size_t>(blockIdx.x) * nf;
    // strongest antenna: first maximum of coarse_peak_array (ant.cpp:104-108)
    uint32_t best = 0;
    for (uint32_t a = 1; a < A.n_ant; ++a)
        if (rp->coarse_metric[a] > rp->coarse_metric[best]) best = a;
    const float cfo_hw = (rp->cfo_frac + rp->cfo_int) * static_cast<float>(A.Mtx) / static_cast<float>(A.Ltx);
    const int64_t base = rp->coarse_64 - static_cast<int64_t>(A.xc_l);
    const uint32_t stage_len = A.xc_len - 1 + A.tmpl_len;
    const float2* x = A.iq + w * A.win_stride + best * A.ant_stride;
    for (uint32_t i0 = 0; i0 < nf; i0 += 8 * blockDim.x) {  // 8 loads in flight per thread
        float2 v[8];
#pragma unroll
        for (uint32_t u = 0; u < 8; ++u) {
            const uint32_t i = i0 + u * blockDim.x + threadIdx.x;
            const int64_t q = base + i;
            v[u] = (i < stage_len && q >= 0 && q < static_cast<int64_t>(A.S_win)) ? x[q] : make_float2(0.f, 0.f);
        }
#pragma unroll
        for (uint32_t u = 0; u < 8; ++u) {
            const uint32_t i = i0 + u * blockDim.x + threadIdx.x;
            if (i < nf) xb[ix(i)] = i < stage_len ? cmul(v[u], phasor(static_cast<double>(cfo_hw) * static_cast<double>(i))) : v[u];
        }
    }
    __syncthreads();
    const float2* S = fft(std::integral_constant<int, -1>{}, xb, yb);
    for (uint32_t i = threadIdx.x; i < nf; i += blockDim.x) Sb[i] = S[ox(i)];
    __syncthreads();  // S's buffer is overwritten below; each thread re-reads only its own Sb[i]
    // per template: its peak metric and index in the header's upper half (s_val / s_idx 8 + k; the
    // wave maxima use 0..7), written by thread 0, the only reader: no registers held across the FFTs
    for (uint32_t k = 0; k < A.n_templates; ++k) {
        const float2* T = A.tmpl_f + static_cast<size_t>(k) * nf;
        if constexpr (DNRP_FINE_BATCH > 1) {
            // the spectrum row and the template read DNRP_FINE_BATCH per thread at a time (one L2
            // round trip per batch instead of one per element), then the products stored
            constexpr uint32_t U = DNRP_FINE_BATCH;
            for (uint32_t i0 = 0; i0 < nf; i0 += U * blockDim.x) {
                float2 sv[U], tv[U];
#pragma unroll
                for (uint32_t u = 0; u < U; ++u) {
                    const uint32_t i = min(i0 + u * blockDim.x + threadIdx.x, nf - 1);
                    sv[u] = Sb[i];
                    tv[u] = T[i];
                }
#pragma unroll
                for (uint32_t u = 0; u < U; ++u) {
                    const uint32_t i = i0 + u * blockDim.x + threadIdx.x;
                    if (i < nf) xb[ix(i)] = cmul(sv[u], tv[u]);
                }
            }
        } else {
            for (uint32_t i = threadIdx.x; i < nf; i += blockDim.x) xb[ix(i)] = cmul(Sb[i], T[i]);
        }
        __syncthreads();
        const float2* R = fft(std::integral_constant<int, 1>{}, xb, yb);
        float bv = -1.f;
        uint32_t bi = 0xFFFFFFFFu;
        for (uint32_t j = threadIdx.x; j < A.xc_len; j += blockDim.x) {
            const float m = cnorm(R[ox(j)]);
            if (m > bv) {  // first maximum (volk_32fc_index_max_32u)
                bv = m;
                bi = j;
            }
        }
        for (int o = 32; o > 0; o >>= 1) {
            const float ov = __shfl_xor(bv, o);
            const uint32_t oi = __shfl_xor(bi, o);
            if (ov > bv || (ov == bv && oi < bi)) {
                bv = ov;
                bi = oi;
            }
        }
        if ((threadIdx.x & 63u) == 0) {
            s_val[threadIdx.x >> 6] = bv;
            s_idx[threadIdx.x >> 6] = bi;
        }
        __syncthreads();
        for (uint32_t v = 0; v < blockDim.x / 64; ++v)
            if (s_val[v] > bv || (s_val[v] == bv && s_idx[v] < bi)) {
                bv = s_val[v];
                bi = s_idx[v];
            }
        if (threadIdx.x == 0) {
            s_val[8 + k] = sqrtf(bv);
            s_idx[8 + k] = bi;
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        const float* xm = s_val + 8;
        const uint32_t* xi = s_idx + 8;
        uint32_t kbest = 0;
        float msum_max = 0.f;
        for (uint32_t k = 0; k < A.n_templates; ++k)
            if (msum_max < xm[k]) {  // strictly larger (crosscorrelator.cpp:214-226)
                msum_max = xm[k];
                kbest = k;
            }
        for (uint32_t k = 0; k < 4; ++k) {
            rp->xc_metric[k] = k < A.n_templates ? xm[k] : 0.f;
            rp->xc_idx[k] = k < A.n_templates ? xi[k] : 0u;
        }
        rp->N_eff_TX = 1u << kbest;
        const float wi = xm[kbest] * static_cast<float>(xi[kbest]);
        rp->fine_local = static_cast<uint32_t>(roundf(wi / msum_max));
        rp->fine_64 = base + rp->fine_local;
    }
}

// ===================================================================== launchers
// float2 slots of sync_detect's stage area: the peak-search arrays and the detection staging alias
// it, and the resampler runs in pieces whose input span fits it (at least 64 blocks per piece)
uint32_t sync_detect_stage(const sync_args& a) {
    const uint32_t region = a.stf_len + a.D + SYNC_PAD_PEAK;
    const size_t alias = ((region + 15) / 16 + 2) * (sizeof(double2) + sizeof(double)) + a.D * sizeof(float);
    const size_t det = a.n_ant * ((SYNC_THREADS + 4 * a.n_uw) * sizeof(float2) +
                                  (SYNC_THREADS + 4 * a.n_pattern + 3) / 4 * 4 * sizeof(float));
    const size_t full = sync_stage_cap(a.L, a.M, a.hl, region);
    const size_t piece = a.L > 1 ? a.hl + 1 + ((a.L - 1) * a.M) / a.L + 64 * a.M : 0;
    const size_t need = std::max((std::max(alias, det) + sizeof(float2) - 1) / sizeof(float2), piece);
    return static_cast<uint32_t>((std::min(full, need) + 1) / 2 * 2);
}

size_t sync_detect_lds(const sync_args& a) {
    const uint32_t region = a.stf_len + a.D + SYNC_PAD_PEAK;
    const size_t taps = (a.npp + 3) / 4 * 2 * sizeof(float2);
    const size_t lb = (region + 1) / 2 * 2 * sizeof(float2);
    const size_t alias = ((region + 15) / 16 + 2) * (sizeof(double2) + sizeof(double)) + a.D * sizeof(float);
    const size_t det = a.n_ant * ((SYNC_THREADS + 4 * a.n_uw) * sizeof(float2) +
                                  (SYNC_THREADS + 4 * a.n_pattern + 3) / 4 * 4 * sizeof(float));
    const size_t stage = size_t(sync_detect_stage(a)) * sizeof(float2);
    return SYNC_SHARED_F2 * sizeof(float2) + taps + lb + std::max(stage, std::max(alias, det));
}

#define SYNC_DISPATCH(KERNEL, GRID, LDS)                                                   \
    do {                                                                                   \
        if (a.L == 9 && a.M == 10 && a.hl == 24)                                           \
            hipLaunchKernelGGL((KERNEL<9, 10, 24>), GRID, dim3(SYNC_THREADS), LDS, st, a); \
        else if (a.L == 9 && a.M == 10 && a.hl == 4)                                       \
            hipLaunchKernelGGL((KERNEL<9, 10, 4>), GRID, dim3(SYNC_THREADS), LDS, st, a);  \
        else if (a.L == 1 && a.M == 1)                                                     \
            hipLaunchKernelGGL((KERNEL<1, 1, 0>), GRID, dim3(SYNC_THREADS), LDS, st, a);   \
        else                                                                               \
            hipLaunchKernelGGL((KERNEL<0, 0, 0>), GRID, dim3(SYNC_THREADS), LDS, st, a);   \
    } while (0)

constexpr int SYNC_WPG = SYNC_WPG_DEF;  // waves per workgroup of the wave kernel
#ifndef DNRP_SS_SEG_CHUNKS
#define DNRP_SS_SEG_CHUNKS 96u  // at most this many chunks of 64 polyphase blocks per sync_steps segment (each
                                // segment re-resamples its lag history first). C4 (1440 steps per window):
                                // 32 -> 5 x 288 steps 12.95 / 12.79 ms, 64 -> 3 x 480 12.71 / 12.74, 96 -> 2 x 720
                                // 12.55 / 12.65, 160 -> 1 x 1440 12.61 / 12.65 (same box)
#endif

hipError_t launch_sync_steps(const sync_args& a, uint32_t n, hipStream_t st) {
    // DNRP_SYNC_STREAM=0 selects the wave kernel below (read per call: tests switch it at run time)
    const char* ss_e = std::getenv("DNRP_SYNC_STREAM");
    const int ss_env = ss_e ? std::atoi(ss_e) : 1;
    if (ss_env && a.L == 9 && a.M == 10 && a.hl == 24 && a.step % 4 == 0 && a.step >= 4 &&
        64u * 9u + a.step + a.pattern + 9u <= SS_RING) {
        // segments of ~32 chunks per (window, antenna): enough waves to fill the chip, little warm-up
        // segments of at most DNRP_SS_SEG_CHUNKS chunks, balanced: ceil(n_steps / max) segments of
        // equal length (a short last segment leaves its waves idle at the tail)
        const uint32_t seg_max = std::max(1u, (DNRP_SS_SEG_CHUNKS * 64u * 9u) / a.step);
        const uint32_t n_seg0 = (a.n_steps + seg_max - 1) / seg_max;
        const uint32_t seg_steps = std::max(1u, (a.n_steps + n_seg0 - 1) / n_seg0);
        const uint32_t n_seg = (a.n_steps + seg_steps - 1) / seg_steps;
        const uint64_t waves = uint64_t(n) * a.n_ant * n_seg;
        const size_t lds = SS_WPG * size_t(ss_inbuf<9, 10, 24>() + SS_RING) * sizeof(float2);
        const dim3 g(static_cast<uint32_t>((waves + SS_WPG - 1) / SS_WPG)), b(64 * SS_WPG);
        // one wave per workgroup: a retired segment frees its LDS at once (A/B on MI355X: sync_steps
        // 4.32 -> 3.81 ms, 176.4k -> 186.0k slot-pairs/s against four); DNRP_SYNC_PIPE=0: the
        // single-chunk-prefetch form (read per call: tests switch it at run time). Compile-time sync
        // taps where the run-time taps are the generated ones (neutral, 3.48 ms both; docs/DESIGN_LOG.md §6)
        const char* pp_e = std::getenv("DNRP_SYNC_PIPE");
        const bool pipe = !pp_e || std::atoi(pp_e);
        if (a.step == 64 && pipe && a.pattern % 16 == 0 && 64u * 9u + a.step + a.pattern + 9u <= SS_PRING) {
            const size_t plds = size_t(ss_inbuf<9, 10, 24>() + SS_PRING) * sizeof(float2);
            if (a.ct_taps)
                hipLaunchKernelGGL((sync_steps_pipe_kernel<9, 10, 24, true>), dim3(static_cast<uint32_t>(waves)), dim3(64),
                                   plds, st, a, seg_steps, n_seg);
            else
                hipLaunchKernelGGL((sync_steps_pipe_kernel<9, 10, 24, false>), dim3(static_cast<uint32_t>(waves)), dim3(64),
                                   plds, st, a, seg_steps, n_seg);
        } else if (a.step == 64)
            hipLaunchKernelGGL((sync_steps_stream_kernel<9, 10, 24, 16, 1>), dim3(static_cast<uint32_t>(waves)), dim3(64),
                               lds / SS_WPG, st, a, seg_steps, n_seg);
        else
            hipLaunchKernelGGL((sync_steps_stream_kernel<9, 10, 24, 0>), g, b, lds, st, a, seg_steps, n_seg);
        return hipGetLastError();
    }
    if (a.L == 9 && a.M == 10 && a.hl == 24) {
        const uint32_t sw = sync_wave_steps(9, a.step, a.pattern);
        const uint32_t waves = n * a.n_ant * ((a.n_steps + sw - 1) / sw);
        const size_t lds = (a.npp + 3) / 4 * 2 * sizeof(float2) + SYNC_WPG * size_t(sync_wave_region(9, 10, 24)) * sizeof(float2);
        hipLaunchKernelGGL((sync_steps_wave_kernel<9, 10, 24, SYNC_WPG>), dim3((waves + SYNC_WPG - 1) / SYNC_WPG),
                           dim3(64 * SYNC_WPG), lds, st, a);
        return hipGetLastError();
    }
    const uint32_t ntile = (a.n_steps + SYNC_TILE_STEPS - 1) / SYNC_TILE_STEPS;
    const uint32_t cnt = SYNC_TILE_STEPS * a.step + a.pattern;
    const size_t lds = (a.npp + 3) / 4 * 2 * sizeof(float2) + (cnt + 1) / 2 * 2 * sizeof(float2) +
                       sync_stage_cap(a.L, a.M, a.hl, cnt) * sizeof(float2);
    const dim3 g(n * a.n_ant * ntile);
    SYNC_DISPATCH(sync_steps_kernel, g, lds);
    return hipGetLastError();
}

#define SYNC_DETECT_INLINE(LR, MR, HLR) sync_detect_kernel<LR, MR, HLR, false>
#define SYNC_DETECT_SPLIT(LR, MR, HLR) sync_detect_kernel<LR, MR, HLR, true>
#define SYNC_DISPATCH2(KERNEL, GRID, LDS)                                                  \
    do {                                                                                   \
        if (a.L == 9 && a.M == 10 && a.hl == 24)                                           \
            hipLaunchKernelGGL((KERNEL(9, 10, 24)), GRID, dim3(SYNC_THREADS), LDS, st, a); \
        else if (a.L == 9 && a.M == 10 && a.hl == 4)                                       \
            hipLaunchKernelGGL((KERNEL(9, 10, 4)), GRID, dim3(SYNC_THREADS), LDS, st, a);  \
        else if (a.L == 1 && a.M == 1)                                                     \
            hipLaunchKernelGGL((KERNEL(1, 1, 0)), GRID, dim3(SYNC_THREADS), LDS, st, a);   \
        else                                                                               \
            hipLaunchKernelGGL((KERNEL(0, 0, 0)), GRID, dim3(SYNC_THREADS), LDS, st, a);   \
    } while (0)

hipError_t launch_sync_detect(const sync_args& a, uint32_t n, hipStream_t st) {
    const dim3 g(n);
    SYNC_DISPATCH2(SYNC_DETECT_INLINE, g, sync_detect_lds(a));
    return hipGetLastError();
}

// split round: detection conditions only (LDS: the block scalars and the detection staging)
hipError_t launch_sync_detect_split(const sync_args& a, uint32_t n, hipStream_t st) {
    const size_t det = a.n_ant * ((SYNC_THREADS + 4 * a.n_uw) * sizeof(float2) +
                                  (SYNC_THREADS + 4 * a.n_pattern + 3) / 4 * 4 * sizeof(float));
    SYNC_DISPATCH2(SYNC_DETECT_SPLIT, dim3(n), SYNC_SHARED_F2 * sizeof(float2) + det);
    return hipGetLastError();
}

// split round: coarse-peak search of the pending detections, one workgroup per (window, antenna)
// one thread per 8 metric positions and, up to 512 threads, one per polyphase block of the region
// (the resampling is one load round trip per block: thread-count sweep on MI355X, C4 per 4096
// windows: 320 threads 0.98 ms, 384 0.93, 512 0.85, 576 1.20)
uint32_t sync_peak_threads(const sync_args& a) {
    const uint32_t region = a.stf_len + a.D + SYNC_PAD_PEAK, nblk = a.L > 1 ? region / a.L + 2 : 0u;
    return std::max({128u, (a.D / 8 + 63) / 64 * 64, std::min(512u, (nblk + 63) / 64 * 64)});
}

size_t sync_peak_lds(const sync_args& a) {
    const uint32_t region = a.stf_len + a.D + SYNC_PAD_PEAK;
    return SYNC_SHARED_F2 * sizeof(float2) + size_t(peak8_lbuf(region)) * sizeof(float2) + peak8_alias(region, a.pattern, a.D);
}

bool sync_taps_match(const float* h, size_t n) {  // run-time sync taps == compiled-in taps, bitwise
    if (n != static_cast<size_t>(taps_sync_9_10::N)) return false;
    for (size_t i = 0; i < n; ++i)
        if (__builtin_bit_cast(uint32_t, h[i]) != __builtin_bit_cast(uint32_t, taps_sync_9_10::h[i])) return false;
    return true;
}

bool sync_peak_ok(const sync_args& a) {  // the grid layout's preconditions (every DECT geometry meets them)
    const uint32_t region = a.stf_len + a.D + SYNC_PAD_PEAK;
    // resample_staged (9/10): at most 2 blocks per thread, the span inside lbuf + the alias area
    const uint32_t nb = region / 9 + 2, n_in = 10 * nb + pp_direct<9, 10, 24>::W;
    const bool staged_ok = !(a.L == 9 && a.M == 10 && a.hl == 24) ||
                           (nb <= 2 * 512 && size_t(n_in) * sizeof(float2) <= size_t(peak8_lbuf(region)) * sizeof(float2) +
                                                                               peak8_alias(region, a.pattern, a.D));
    return a.D % 8 == 0 && a.pattern % 8 == 0 && (a.stf_len + SYNC_PAD_PEAK) % 8 == 0 && a.D / 8 <= 512 &&
           (a.n_uw == 6 || a.n_uw == 8) && sync_peak_lds(a) <= 160 * 1024 && staged_ok;
}

hipError_t launch_sync_peak(const sync_args& a, uint32_t n, hipStream_t st) {
    const dim3 g(n * a.n_ant), b(sync_peak_threads(a));
    const size_t lds = sync_peak_lds(a);
    auto go = [&](auto nuw) {
        constexpr int U = decltype(nuw)::value;
        if (a.L == 9 && a.M == 10 && a.hl == 24 && a.ct_taps)
            hipLaunchKernelGGL((sync_peak_kernel<9, 10, 24, true, U>), g, b, lds, st, a);
        else if (a.L == 9 && a.M == 10 && a.hl == 24)
            hipLaunchKernelGGL((sync_peak_kernel<9, 10, 24, false, U>), g, b, lds, st, a);
        else if (a.L == 9 && a.M == 10 && a.hl == 4)
            hipLaunchKernelGGL((sync_peak_kernel<9, 10, 4, false, U>), g, b, lds, st, a);
        else if (a.L == 1 && a.M == 1)
            hipLaunchKernelGGL((sync_peak_kernel<1, 1, 0, false, U>), g, b, lds, st, a);
        else
            hipLaunchKernelGGL((sync_peak_kernel<0, 0, 0, false, U>), g, b, lds, st, a);
    };
    if (a.n_uw == 6)  // n_pattern 7 (u = 1)
        go(std::integral_constant<int, 6>{});
    else  // n_pattern 9
        go(std::integral_constant<int, 8>{});
    return hipGetLastError();
}

// the staged form (sync_post_kernel<9, 10, 24, true>): compiled-in taps and at most 2 blocks per thread;
// otherwise the run-time-tap form reads the windows straight from the stream (the same sums)
static bool sync_post_staged(const sync_args& a) {
    return DNRP_POST_STAGED && a.L == 9 && a.M == 10 && a.hl == 24 && a.ct_taps && (a.stf_len + 8) / 9 + 2 <= 2 * SYNC_THREADS;
}
size_t sync_post_lds(const sync_args& a) {  // the staged form's input span (n_in inputs) or the STF
    const uint32_t nb = (a.stf_len + 8) / 9 + 2, n_in = 10 * nb + pp_direct<9, 10, 24>::W;
    return (12 + (std::max(a.stf_len, sync_post_staged(a) ? n_in : 0u) + 1) / 2 * 2) * sizeof(float2);
}

hipError_t launch_sync_post(const sync_args& a, uint32_t n, hipStream_t st) {
    const dim3 g(n * a.max_reports * a.n_ant);
    const size_t lds = sync_post_lds(a);
    if (lds > 160 * 1024) return hipErrorInvalidValue;
    if (sync_post_staged(a) || (!DNRP_POST_STAGED && a.L == 9 && a.M == 10 && a.hl == 24 && a.ct_taps))
        hipLaunchKernelGGL((sync_post_kernel<9, 10, 24, true>), g, dim3(SYNC_THREADS), lds, st, a);
    else if (a.L == 9 && a.M == 10 && a.hl == 24)
        hipLaunchKernelGGL((sync_post_kernel<9, 10, 24, false>), g, dim3(SYNC_THREADS), lds, st, a);
    else if (a.L == 9 && a.M == 10 && a.hl == 4)
        hipLaunchKernelGGL((sync_post_kernel<9, 10, 4, false>), g, dim3(SYNC_THREADS), lds, st, a);
    else if (a.L == 1 && a.M == 1)
        hipLaunchKernelGGL((sync_post_kernel<1, 1, 0, false>), g, dim3(SYNC_THREADS), lds, st, a);
    else
        hipLaunchKernelGGL((sync_post_kernel<0, 0, 0, false>), g, dim3(SYNC_THREADS), lds, st, a);
    return hipGetLastError();
}

hipError_t launch_sync_fine(const sync_args& a, uint32_t n, hipStream_t st) {
    const size_t nbuf = size_t(1) << a.log2_fft;
    // in place: one padded buffer (radix 8 at 4096 points: R8_SLOTS)
    const size_t lds = (16 + (DNRP_FINE_R8 && a.log2_fft == 12 ? R8_SLOTS : (a.log2_fft & 1u) == 0 ? nbuf + nbuf / 32 : 2 * nbuf)) * sizeof(float2);
    hipLaunchKernelGGL(sync_fine_kernel, dim3(n * a.max_reports), dim3(SYNC_FINE_THREADS), lds, st, a);
    return hipGetLastError();
}

}  // namespace dnrp::dev
