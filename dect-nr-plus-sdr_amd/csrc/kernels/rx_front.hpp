// One-wavefront RX front end for N_b_DFT_os = 1024 with the compile-time 9/10 resampler taps
// (rx_synced.cpp:711-771: run_mix_resample + run_cp_fft_scale) of rx_fft_wave_kernel (rx.hip). The
// bins go to a caller-given store functor (Y in HBM).
//
// Symbol l (1-based data symbol) yields the DECT-rate outputs m0 .. m0+1023 (the CP outputs are
// skipped); the polyphase blocks q in [qb0, qb1) cover them, reading hw-rate inputs in0 .. in0+n_in
// relative to the fine peak. A wave stages that span in its LDS region R, resamples it there with
// pp_const (output-major, no zero taps), applies the phase-continuous mixer, runs wave_fft1024 and
// hands every occupied bin, amplitude-scaled and STO-derotated, to a store functor.
#pragma once

#include "experiments.hpp"
#include "kernels.hpp"
#include "polyphase.hpp"
#include "taps_gen.hpp"

namespace dnrp::dev {

// float2 slots of one wave's LDS region: the symbol's input span, the FFT's exchange buffer, the bins
__host__ __device__ inline uint32_t rxw_region(uint32_t L, uint32_t M, uint32_t W) {
    const uint32_t n_in = ((1024 + 2 * L) * M) / L + W + M;  // one symbol's input span, upper bound
    const uint32_t r = n_in > WFFT_XB ? n_in : WFFT_XB;
    return (r + 15) / 16 * 16;
}

struct rx_span_t {
    int m0, qb0, qb1;
    int64_t in0;
    uint32_t n_in;
};

template <int LR, int MR, int HLR>
__device__ __forceinline__ rx_span_t rx_span(const rx_front_args& A, uint32_t l) {
    constexpr int W = pp_direct<LR, MR, HLR>::W;
    rx_span_t s;
    const uint32_t n_stf = A.STF_CP + 1024;
    s.m0 = static_cast<int>(n_stf + (l - 1) * (A.CP + 1024) + A.CP);  // first output of symbol l
    s.qb0 = (s.m0 - static_cast<int>(A.m_star)) / LR;                  // m0 >= m_star
    s.qb1 = (s.m0 + 1024 - static_cast<int>(A.m_star) + LR - 1) / LR;
    s.in0 = static_cast<int64_t>(A.p_star) + int64_t(MR) * s.qb0 - HLR;
    s.n_in = static_cast<uint32_t>(MR * (s.qb1 - 1 - s.qb0) + W);
    return s;
}

#ifndef DNRP_FE_IMAJ
#define DNRP_FE_IMAJ 0  // 1: the polyphase windows input-major from LDS (pp_const::run_imaj): rx_epoch 26.84 /
                        // 26.78 vs 26.62 / 26.69 ms (the kernel's VGPR peak is elsewhere), off
#endif
// R[i] = input in0 + i (staged), i < n_in  ->  R[j] = mixed output m0 + j, j < 1024
template <int LR, int MR, int HLR>
__device__ __forceinline__ void rx_resample_ct(const rx_front_args& A, const rx_pkt_in& in, const rx_pkt_state& S,
                                               const rx_span_t& sp, float2* R, uint32_t lane) {
    using PD = pp_direct<LR, MR, HLR>;
    static_assert(taps_rx_9_10::L == LR && taps_rx_9_10::M == MR && taps_rx_9_10::HL == HLR, "generated taps");
    constexpr int BR = (1024 + 2 * LR) / LR / 64 + 1;  // block rounds per lane
    // the outputs of round rd land below every input a later round reads (block q writes
    // R[< LR (q + 1)] and later blocks read from R[MR q'] with q' >= q + 64), so each round stores
    // its outputs before the next round loads its windows
    static_assert(LR * (64 + 1) <= MR * 64, "round outputs stay below the next round's windows");
    const int n_stf = static_cast<int>(A.STF_CP + 1024);
    const double phi_stf = static_cast<double>(n_stf) * in.inc0;  // mixer phase at the first data sample
    const float2 step1 = phasor(S.inc1);
#pragma unroll
    for (int rd = 0; rd < BR; ++rd) {
        const int qr = static_cast<int>(lane) + 64 * rd;
        const int q = sp.qb0 + qr;
        float2 y[LR];
        if constexpr (DNRP_FE_IMAJ && (MR % 2) == 0) {  // window input-major from LDS (R 16-B aligned)
            pp_const<taps_rx_9_10>::run_imaj<true>(R + MR * min(qr, sp.qb1 - 1 - sp.qb0), y);
        } else {
            float2 xv[PD::W];
            PD::template load<(MR % 2) == 0>(R + MR * min(qr, sp.qb1 - 1 - sp.qb0), xv);
            pp_const<taps_rx_9_10>::run(xv, y);
        }
        __builtin_amdgcn_wave_barrier();
        if (q < sp.qb1) {
            const int mb = static_cast<int>(A.m_star) + LR * q;
            float2 r = phasor(phi_stf + static_cast<double>(mb - n_stf) * S.inc1);
#pragma unroll
            for (int k = 0; k < LR; ++k) {
                const uint32_t idx = static_cast<uint32_t>(mb + k - sp.m0);
                if (idx < 1024) R[idx] = cmul(y[k], r);
                r = cmul(r, step1);
            }
        }
        __builtin_amdgcn_wave_barrier();
    }
}

// wave FFT of R[0..1024) (R also serves as the exchange buffer, >= WFFT_XB float2) and the occupied
// bins: FFT bin n -> subcarrier index k (n <= N/2: k = n + N/2; upper half: k = n - off_lower),
// amplitude sqrt(N_b_OCC)/N_b_DFT_os, STO derotation exp(j sto_inc (k - N/2)) by two running
// phasors stepped by 64 bins (the amplitude folded into them). put(k, value) for every k in [0, N_b_OCC]; R is free again when
// put is called (all exchange reads have completed).
// RT: wave_fft1024_rt with the lane's two twiddles w1 = W^(4 (lane & 15)), wl = W^lane loaded by the
// caller (e.g. before its input staging) instead of 27 twiddle loads inside the passes
template <bool RT = false, class Put>
__device__ __forceinline__ void rx_fft_bins(const rx_front_args& A, const rx_pkt_state& S, float2* R, uint32_t lane,
                                            Put&& put, float2 w1 = float2{}, float2 wl = float2{}) {
    float2 v[16];
#pragma unroll
    for (int m = 0; m < 16; ++m) v[m] = R[lane + 64 * m];
    __builtin_amdgcn_wave_barrier();
    if constexpr (experiment(XS_FE_SKIP_FFT))
        ;
    else if constexpr (RT)
        wave_fft1024_rt<-1>(v, R, w1, wl, lane);
    else
        wave_fft1024<-1>(v, R, A.tw, lane);  // twiddles through the L1 (8 KB, every wave)
    __builtin_amdgcn_wave_barrier();
    const uint32_t N = A.N_occ;
    const float2 s64 = phasor(64.0 * S.sto_inc);
    // the amplitude folded into the two derotation phasors: one complex product per bin (A/B per
    // 16384-slot PDC launch: 19.05 / 18.97 -> 18.82 / 18.55 ms)
    float2 pa = cscale(phasor(S.sto_inc * static_cast<double>(lane)), A.amp_scale);
    float2 pb = cscale(phasor(S.sto_inc * (static_cast<double>(lane) - static_cast<double>(A.off_lower) -
                                           static_cast<double>(N / 2))), A.amp_scale);
    if (N == 896 && A.off_lower == 576) {  // beta = 16 at N_b_DFT_os = 1024 (C3 / C4): the bin map is static
        // rows m <= 6 lower half (k = n + 448), row 7 only n = 448 (k = 896), row 8 empty, rows >= 9
        // upper half (k = n - 576): no per-bin range tests or phasor selects, and pa stepped only
        // while it is used; pb still stepped from row 0, so every product is the generic path's
#pragma unroll
        for (int m = 0; m < 16; ++m) {
            const uint32_t n = lane + 64 * m;
            if (m <= 6) put(n + 448, cmul(v[m], pa));
            else if (m == 7 && lane == 0) put(896u, cmul(v[m], pa));
            else if (m >= 9) put(n - 576, cmul(v[m], pb));
            if (m < 7) pa = cmul(pa, s64);
            if (m < 15) pb = cmul(pb, s64);
        }
        return;
    }
#pragma unroll
    for (int m = 0; m < 16; ++m) {
        const uint32_t n = lane + 64 * m;
        uint32_t k = 0xFFFFFFFFu;
        float2 rot = pa;
        if (n <= N / 2) {
            k = n + N / 2;
        } else if (n >= A.off_lower && n < A.off_lower + N / 2) {
            k = n - A.off_lower;
            rot = pb;
        }
        if (k != 0xFFFFFFFFu) put(k, cmul(v[m], rot));
        pa = cmul(pa, s64);
        pb = cmul(pb, s64);
    }
}

// DRS SNR terms of one (antenna, DRS symbol) while its bins sit in the wave's region R (R[k] = bin
// of subcarrier k): for every DRS op of symbol l and each of its transmit streams t, the sums over
// the stream's DRS cells i of |w_i y_i|^2 and |w_i y_i - w_i+1 y_i+1|^2 (rx_snr_kernel's terms: float
// products, summed per lane in float -- at most 4 cells per stream and lane, nd <= 256 -- and across
// lanes in double, where the Y-gather path sums every term in double: the two paths may differ in the
// last float bits, the reference's own volk sums are float) -> A.snr_part; with A.zd also the zero-forced cells
// w_i y_i themselves (the pilot values of channel_antenna.hpp:38-63). The op list is uniform (scalar loads).
__device__ __forceinline__ void rx_drs_partials(const rx_front_args& A, uint32_t slot, uint32_t a, uint32_t l,
                                                uint32_t d0, const float2* R, uint32_t lane) {
    const uint32_t nd = A.n_drs, half = 2 * nd;  // N_b_OCC / 2
    // subcarrier index and value of DRS cell i of stream t with parity p
    auto cell = [&](uint32_t t, uint32_t p, uint32_t i) {
        const uint32_t x = 4 * i + ((t + 2 * p) & 3u);
        const float s = (((A.drs_neg >> ((4 * i + (t & 3u)) % 56)) & 1ull) ? -1.f : 1.f) * (t < 4 ? 1.f : -1.f);
        return cscale(R[x + (x >= half ? 1u : 0u)], s);
    };
    // the op table by scalar loads (uniform symbol and op index): a vector load here would wait
    // (vmcnt retires in order) for the symbol's Y stores just issued. d0: the symbol's first op.
    typedef const __attribute__((address_space(4))) uint32_t* cu32;
    const cu32 dl = reinterpret_cast<cu32>(reinterpret_cast<uintptr_t>(A.dl));
    const cu32 dm = reinterpret_cast<cu32>(reinterpret_cast<uintptr_t>(A.dmeta));
    l = __builtin_amdgcn_readfirstlane(l);
    for (uint32_t d = __builtin_amdgcn_readfirstlane(d0); d < A.n_dops; ++d) {  // ops of a symbol: consecutive
        if (dl[d] != l) break;
        const uint32_t meta = dm[d];
        const uint32_t tf = meta & 0xFFu, tl = (meta >> 8) & 0xFFu, par = (meta >> 16) & 0xFFu;
        // per lane at most 4 (nd <= 256) terms per stream: float sums, double across the lanes; the
        // right neighbour of cell i comes from the next lane (lane 63: the next round's first cell)
        float f1 = 0.f, f2 = 0.f;
        float2* zrow = A.zd ? A.zd + ((size_t(slot) * A.zd_dops + d) * A.N_RX + a) * 4 * A.zd_row : nullptr;
        for (uint32_t t = tf; t <= tl; ++t)
            for (uint32_t i0 = 0; i0 < nd; i0 += 64) {
                const uint32_t i = i0 + lane;
                const float2 v = cell(t, par, min(i, nd - 1));
                if (zrow && i < nd) zrow[t * A.zd_row + i] = v;  // the zero-forced pilot (build_pilots' value)
                float2 vn = make_float2(__shfl_down(v.x, 1), __shfl_down(v.y, 1));
                if (lane == 63) vn = cell(t, par, min(i + 1, nd - 1));
                if (i < nd) f1 += cnorm(v);
                if (i + 1 < nd) f2 += cnorm(csub(v, vn));
            }
        double s1 = f1, s2 = f2;
        for (int o = 32; o > 0; o >>= 1) {
            s1 += __shfl_xor(s1, o);
            s2 += __shfl_xor(s2, o);
        }
        if (lane == 0) A.snr_part[((size_t(slot) * A.n_sym_total + l) * A.N_RX + a) * 8 + tf] = make_double2(s1, s2);
    }
}

}  // namespace dnrp::dev
