// RX kernels for the synchronised receiver (rx_synced_t, lib/src/phy/rx/rx_synced/rx_synced.cpp).
//
//  rx_stf_kernel   one WG per packet: polyphase M/L resampling + CFO mixer of the STF on all RX
//                  antennas, RMS, cover-sequence revert, fractional CFO re-estimate
//                  (rx_synced.cpp:503-661), STF FFT + zero-forcing, fractional STO
//                  (estimator_sto.cpp:47-170), STF SNR (estimator_snr.cpp:48-66).
//  rx_fft_kernel   one WG per (packet, antenna, symbol block): resampling + phase-continuous mixer
//                  + CP removal + FFT + bin extraction + amplitude scaling + STO derotation
//                  (rx_synced.cpp:711-771) into the frequency-domain grid Y in HBM.
//  rx_back_kernel  one WG per packet: interprets the host-built schedule of DRS zero-forcing,
//                  SNR-driven Wiener LUT choice, interpolation events and PCC/PDC cell
//                  combining (MRC / SFBC), int16 soft demapping and descrambling
//                  (rx_synced.cpp:773-1392, pcc_enc.cpp:297, pdc_enc.cpp:339-344).
#include "device_common.hpp"
#include "kernels.hpp"
#include "polyphase.hpp"

namespace dnrp::dev {

__constant__ float k_cover_rx[9] = {1, -1, 1, 1, -1, -1, -1, -1, -1};  // stf.hpp:146-151

// resample outputs m in [m0, m0+cnt) of one antenna stream into dst and mix with
// exp(j*(phi_m0 + (m - m0) * inc)). inbuf must hold cnt*M/L + hl + 4 samples; taps in LDS.
template <int HL>
__device__ void resample_block(const rx_front_args& A, const float2* __restrict__ x, int64_t fine_peak, uint64_t m0,
                               uint32_t cnt, float2* inbuf, float2* dst, const float* taps, double phi_m0,
                               double inc) {
    const uint64_t t0 = A.delay + m0 * A.M;
    const int64_t p0 = static_cast<int64_t>(t0 / A.L);
    const uint64_t t1 = A.delay + (m0 + cnt - 1) * A.M;
    const int64_t p1 = static_cast<int64_t>(t1 / A.L);
    const int64_t q0 = p0 - static_cast<int64_t>(A.hl);
    const uint32_t n_in = static_cast<uint32_t>(p1 - q0 + 1);
    for (uint32_t i = threadIdx.x; i < n_in; i += blockDim.x) {
        const int64_t q = q0 + i;  // input index relative to the fine peak
        const int64_t g = fine_peak + q;
        float2 v = make_float2(0.f, 0.f);
        if (q >= 0 && g >= 0 && g < static_cast<int64_t>(A.S_in)) v = x[g];
        inbuf[i] = v;
    }
    __syncthreads();
    const uint32_t dT = blockDim.x * A.M, dp = dT / A.L, dph = dT % A.L;
    if (threadIdx.x < cnt) {
        const uint64_t t = A.delay + (m0 + threadIdx.x) * A.M;
        uint32_t p = static_cast<uint32_t>(static_cast<int64_t>(t / A.L) - q0);
        uint32_t ph = static_cast<uint32_t>(t % A.L);
        float2 rot = phasor(phi_m0 + static_cast<double>(threadIdx.x) * inc);
        const float2 rstep = phasor(static_cast<double>(blockDim.x) * inc);
        for (uint32_t i = threadIdx.x; i < cnt; i += blockDim.x) {
            float ar = 0.f, ai = 0.f;
            const uint32_t hl = HL >= 0 ? static_cast<uint32_t>(HL) : A.hl;
#pragma unroll
            for (uint32_t d = 0; d <= hl; ++d) {
                const float h = taps[ph + d * A.L];
                const float2 v = inbuf[p - d];
                ar = fmaf(v.x, h, ar);
                ai = fmaf(v.y, h, ai);
            }
            dst[i] = cmul(make_float2(ar, ai), rot);
            rot = cmul(rot, rstep);
            p += dp;
            ph += dph;
            if (ph >= A.L) {
                ph -= A.L;
                ++p;
            }
        }
    }
    __syncthreads();
}

__device__ __forceinline__ void extract_bins(const rx_front_args& A, const float2* F, float2* dst, uint32_t k) {
    const uint32_t N = A.N_occ;
    const float2 v = (k >= N / 2) ? F[k - N / 2] : F[A.off_lower + k];
    *dst = cscale(v, A.amp_scale);
}

// ===================================================================== STF
template <int HL>
__global__ void __launch_bounds__(256) rx_stf_kernel(rx_front_args A) {
    extern __shared__ __attribute__((aligned(16))) float2 smem[];
    __shared__ double red[16];
    const uint32_t pkt = blockIdx.x;
    const uint32_t Nd = A.plan.N, N = A.N_occ, Nf = N + 1;
    const uint32_t n_stf = A.STF_CP + Nd;
    const uint32_t n_in_max = (n_stf * A.M) / A.L + A.hl + 4;
    float2* sbuf = smem;                 // n_stf
    float2* inbuf = sbuf + n_stf;        // n_in_max
    float2* fa = inbuf + n_in_max;       // Nd
    float2* fb = fa + Nd;                // Nd
    float2* twl = fb + Nd;               // Nd
    float2* Ys = twl + Nd;               // [N_RX][Nf]
    float* taps = reinterpret_cast<float*>(Ys + A.N_RX * Nf);
    for (uint32_t i = threadIdx.x; i < Nd; i += blockDim.x) twl[i] = A.tw[i];
    for (uint32_t i = threadIdx.x; i < (A.hl + 1) * A.L; i += blockDim.x) taps[i] = A.taps[i];
    const rx_pkt_in in = A.pin[pkt];
    const uint32_t P = n_stf / A.n_pattern;
    double cs_re = 0.0, cs_im = 0.0;
    rx_pkt_state S;

    for (uint32_t a = 0; a < A.N_RX; ++a) {
        const float2* x = A.iq + (size_t(pkt) * A.N_RX + a) * A.S_in;
        resample_block<HL>(A, x, in.fine_peak, 0, n_stf, inbuf, sbuf, taps, 0.0, in.inc0);
        double e = 0.0, pr = 0.0, pi = 0.0;
        for (uint32_t i = threadIdx.x; i < n_stf; i += blockDim.x) e += cnorm(sbuf[i]);
        e = block_sum(e, red);
        if (a < 8) S.rms[a] = sqrtf(static_cast<float>(e / n_stf));
        for (uint32_t i = threadIdx.x; i < n_stf; i += blockDim.x)
            sbuf[i] = cscale(sbuf[i], k_cover_rx[min(i / A.pattern_len, 8u)]);
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < (A.n_pattern - 1) * P; i += blockDim.x) {
            const float2 c = cmulc(sbuf[i], sbuf[i + P]);
            pr += c.x;
            pi += c.y;
        }
        cs_re += block_sum(pr, red);
        cs_im += block_sum(pi, red);
        for (uint32_t i = threadIdx.x; i < Nd; i += blockDim.x) fa[i] = sbuf[A.STF_CP + i];
        __syncthreads();
        const float2* F = fft_any<-1>(fa, fb, twl, A.plan);
        for (uint32_t k = threadIdx.x; k < Nf; k += blockDim.x) extract_bins(A, F, &Ys[a * Nf + k], k);
        __syncthreads();
    }
    for (uint32_t a = A.N_RX; a < 8; ++a) S.rms[a] = 0.f;
    // fractional CFO re-estimate (rx_synced.cpp:523-558) and mixer adjustment (mixer.cpp:35-39)
    const float delta = atan2f(static_cast<float>(cs_im), static_cast<float>(cs_re)) / static_cast<float>(P);
    {
        float s0, c0, s1, c1;
        sincosf(in.cfo_rad, &s0, &c0);
        sincosf(delta, &s1, &c1);
        const float2 m = cmul(make_float2(c0, s0), make_float2(c1, s1));
        S.inc1 = atan2(static_cast<double>(m.y), static_cast<double>(m.x));
    }
    S.cfo_fine = in.cfo_rad + delta;
    // STF zero-forcing and fractional STO (rx_synced.cpp:663-709, estimator_sto.cpp:124-146)
    const uint32_t n = A.b * 14;
    auto rstf = [&](uint32_t w) { return w < n / 2 ? 4 * w : 4 * w + 4; };
    auto zf = [&](uint32_t a, uint32_t w, double inc) {
        const uint32_t r = rstf(w);
        float2 y = Ys[a * Nf + r];
        if (inc != 0.0) y = cmul(y, phasor(-inc * static_cast<double>(N / 2) + inc * static_cast<double>(r)));
        const float2 s = A.stf[r];
        return make_float2((y.x * s.x + y.y * s.y) / cnorm(s), (y.y * s.x - y.x * s.y) / cnorm(s));
    };
    double inc = 0.0;
    for (uint32_t a = 0; a < A.N_RX; ++a) {
        double br = 0.0, bi = 0.0;
        for (uint32_t i = threadIdx.x; i + 1 < n; i += blockDim.x) {
            float2 p = cmulc(zf(a, i, 0.0), zf(a, i + 1, 0.0));
            if (i == n / 2 - 1) {  // center pair spans 8 subcarriers: rotate back by half its angle
                const float ang = atan2f(p.y, p.x);
                float s, c;
                sincosf(-ang / 2.0f, &s, &c);
                p = cmul(p, make_float2(c, s));
            }
            br += p.x;
            bi += p.y;
        }
        br = block_sum(br, red);
        bi = block_sum(bi, red);
        inc += static_cast<double>(atan2f(static_cast<float>(bi), static_cast<float>(br)) / 4.0f);
    }
    inc /= static_cast<double>(A.N_RX);
    S.sto_inc = inc;
    S.sto_frac = static_cast<float>(atan2(sin(inc), cos(inc)) / 2.0 / 3.14159265358979323846 * Nd);
    // STF SNR on the derotated symbol (estimator_snr.cpp:48-66,104-146)
    double sn = 0.0, nn = 0.0;
    for (uint32_t a = 0; a < A.N_RX; ++a)
        for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
            const float2 z = zf(a, i, inc);
            sn += cnorm(z);
            if (i + 1 < n) nn += cnorm(csub(z, zf(a, i + 1, inc)));
        }
    sn = block_sum(sn, red);
    nn = block_sum(nn, red) / 2.0;
    S.snr_SN = (sn - nn) / 4.0 + nn;
    S.snr_N = nn;
    S.snr_SN_cnt = A.N_RX * n;
    S.snr_N_cnt = A.N_RX * (n - 1);
    S.snr_pcc = S.snr_pdc = 0.f;
    if (threadIdx.x == 0) A.st[pkt] = S;
}

// ===================================================================== data-symbol FFTs
// One WG per (packet, antenna, run of sym_per_block symbols); the symbols are processed in pairs
// (RX_SYM_PASS): resampling of both into LDS, one batched FFT, bin extraction + STO derotation.
// Register-blocked path (LR > 0): thread (s, j) computes the L outputs of aligned block j of symbol s
// straight from HBM (its W-sample window, 16-B loads), taps on the scalar path (polyphase.hpp).
constexpr uint32_t RX_THREADS = 256;

// xv[i] = src[i] with 16-B loads; OFF = 1 when src is 8 mod 16 (then src[-1] is read too)
template <int W, int OFF>
__device__ __forceinline__ void load_window(const float2* src, float2 (&xv)[W]) {
    const float4* v4 = reinterpret_cast<const float4*>(src - OFF);
    float4 t4[(W + OFF + 1) / 2];
#pragma unroll
    for (int i = 0; i < (W + OFF + 1) / 2; ++i) t4[i] = v4[i];
#pragma unroll
    for (int i = 0; i < W; ++i) {
        const int e = i + OFF;
        xv[i] = (e & 1) ? make_float2(t4[e >> 1].z, t4[e >> 1].w) : make_float2(t4[e >> 1].x, t4[e >> 1].y);
    }
}
constexpr uint32_t RX_SYM_PASS = 2;

template <int LR, int MR, int HLR>
__global__ void __launch_bounds__(RX_THREADS) rx_fft_kernel(rx_front_args A) {
    extern __shared__ __attribute__((aligned(16))) float2 smem[];
    const uint32_t Nd = A.plan.N, N = A.N_occ, Nf = N + 1;
    const uint32_t nblk = (A.sym_count + A.sym_per_block - 1) / A.sym_per_block;
    const uint32_t blk = blockIdx.x % nblk;
    const uint32_t a = (blockIdx.x / nblk) % A.N_RX;
    const uint32_t pkt = blockIdx.x / (nblk * A.N_RX);
    float2* fa = smem;                         // [RX_SYM_PASS][Nd]
    float2* fb = fa + RX_SYM_PASS * Nd;        // [RX_SYM_PASS][Nd]
    float2* twl = fb + RX_SYM_PASS * Nd;       // Nd
    float2* rot = twl + Nd;                    // Nf: STO derotation per subcarrier
    float2* inbuf = rot + Nf;                  // generic path only
    float* taps = reinterpret_cast<float*>(inbuf + (LR > 0 ? 0u : (Nd * A.M) / A.L + A.hl + 4));
    for (uint32_t i = threadIdx.x; i < Nd; i += RX_THREADS) twl[i] = A.tw[i];
    if (LR == 0)
        for (uint32_t i = threadIdx.x; i < (A.hl + 1) * A.L; i += RX_THREADS) taps[i] = A.taps[i];
    const rx_pkt_in in = A.pin[pkt];
    const rx_pkt_state S = A.st[pkt];
    const uint32_t n_stf = A.STF_CP + Nd;
    for (uint32_t k = threadIdx.x; k < Nf; k += RX_THREADS)
        rot[k] = phasor(-S.sto_inc * static_cast<double>(N / 2) + S.sto_inc * static_cast<double>(k));
    const float2* x = A.iq + (size_t(pkt) * A.N_RX + a) * A.S_in;
    const double phi_stf = static_cast<double>(n_stf) * in.inc0;  // mixer phase at the first data sample
    const float2 step1 = phasor(S.inc1);
    const uint32_t l0 = A.sym_first + blk * A.sym_per_block;
    const uint32_t l1 = min(A.sym_first + A.sym_count, l0 + A.sym_per_block);
    // valid input window relative to the fine peak: history is zero before it (rx_synced.cpp:711-740)
    const int64_t q_lo = 0, q_hi = static_cast<int64_t>(A.S_in) - in.fine_peak;
    for (uint32_t lp = l0; lp < l1; lp += RX_SYM_PASS) {
        const uint32_t ns = min(RX_SYM_PASS, l1 - lp);
        if constexpr (LR > 0) {
            using PB = pp_block<LR, MR, HLR>;
            const const_taps_t h = as_const_taps(A.taps);
            constexpr uint32_t TPS = RX_THREADS / RX_SYM_PASS;  // threads per symbol
            const uint32_t s = threadIdx.x / TPS;
            if (s < ns) {
                const uint32_t l = lp + s;
                const int m0 = static_cast<int>(n_stf + (l - 1) * (A.CP + Nd) + A.CP);  // first output of symbol l
                const int qb0 = (m0 - static_cast<int>(A.m_star)) / LR;                 // m0 >= m_star
                const int qb1 = (m0 + static_cast<int>(Nd) - static_cast<int>(A.m_star) + LR - 1) / LR;
                for (int q = qb0 + static_cast<int>(threadIdx.x % TPS); q < qb1; q += TPS) {
                    const int mb = static_cast<int>(A.m_star) + LR * q;
                    const int64_t qs = static_cast<int64_t>(A.p_star) + int64_t(MR) * q - HLR;  // first input
                    float2 xv[PB::W];
                    const float2* src = x + in.fine_peak + qs;
                    if (qs - 1 >= q_lo && qs + PB::W + 1 <= q_hi) {
                        if (reinterpret_cast<uintptr_t>(src) & 15u)
                            load_window<PB::W, 1>(src, xv);
                        else
                            load_window<PB::W, 0>(src, xv);
                    } else {
#pragma unroll
                        for (int i = 0; i < PB::W; ++i) {
                            const int64_t qi = qs + i;
                            xv[i] = (qi >= q_lo && qi < q_hi) ? src[i] : make_float2(0.f, 0.f);
                        }
                    }
                    float2 y[LR];
                    const_taps_t hq = h;
                    asm volatile("" : "+s"(hq));  // keep the tap loads inside the loop (SGPR budget)
                    PB::run(xv, hq, y);
                    float2 r = phasor(phi_stf + static_cast<double>(mb - static_cast<int>(n_stf)) * S.inc1);
                    float2* dst = fa + s * Nd;
#pragma unroll
                    for (int k = 0; k < LR; ++k) {
                        const uint32_t idx = static_cast<uint32_t>(mb + k - m0);
                        if (idx < Nd) dst[idx] = cmul(y[k], r);
                        r = cmul(r, step1);
                    }
                }
            }
            __syncthreads();
        } else {
            for (uint32_t s = 0; s < ns; ++s) {
                const uint32_t l = lp + s;
                const uint64_t m0 = n_stf + uint64_t(l - 1) * (A.CP + Nd) + A.CP;
                resample_block<-1>(A, x, in.fine_peak, m0, Nd, inbuf, fa + s * Nd, taps,
                                   phi_stf + static_cast<double>(m0 - n_stf) * S.inc1, S.inc1);
            }
        }
        const float2* F = fft_any<-1>(fa, fb, twl, A.plan, ns);
        for (uint32_t i = threadIdx.x; i < ns * Nf; i += RX_THREADS) {
            const uint32_t s = i / Nf, k = i - s * Nf;
            float2 v;
            extract_bins(A, F + s * Nd, &v, k);
            A.Y[((size_t(pkt) * A.N_RX + a) * A.n_sym_total + lp + s) * A.Nf_pad + k] = cmul(v, rot[k]);
        }
        __syncthreads();
    }
}

#define DNRP_HL_DISPATCH(KERNEL, G, B, LDS, ST, ARGS)                          \
    switch ((ARGS).hl) {                                                       \
        case 24: hipLaunchKernelGGL(KERNEL<24>, G, B, LDS, ST, ARGS); break;  \
        case 4: hipLaunchKernelGGL(KERNEL<4>, G, B, LDS, ST, ARGS); break;    \
        case 0: hipLaunchKernelGGL(KERNEL<0>, G, B, LDS, ST, ARGS); break;    \
        default: hipLaunchKernelGGL(KERNEL<-1>, G, B, LDS, ST, ARGS); break;  \
    }

hipError_t launch_rx_stf(const rx_front_args& a, uint32_t n, hipStream_t st) {
    const uint32_t Nd = a.plan.N, n_stf = a.STF_CP + Nd;
    const size_t lds = (n_stf + (n_stf * a.M) / a.L + a.hl + 4 + 3 * size_t(Nd) + size_t(a.N_RX) * (a.N_occ + 1)) *
                           sizeof(float2) + (a.hl + 1) * a.L * sizeof(float);
    DNRP_HL_DISPATCH(rx_stf_kernel, dim3(n), dim3(256), lds, st, a);
    return hipGetLastError();
}

hipError_t launch_rx_fft(const rx_front_args& a, uint32_t n, hipStream_t st) {
    const uint32_t Nd = a.plan.N;
    const uint32_t nblk = (a.sym_count + a.sym_per_block - 1) / a.sym_per_block;
    const dim3 g(n * a.N_RX * nblk), b(RX_THREADS);
    const bool fast9 = a.L == 9 && a.M == 10 && (a.hl == 24 || a.hl == 4);
    const size_t lds = ((2 * RX_SYM_PASS + 1) * size_t(Nd) + a.N_occ + 1) * sizeof(float2) +
                       (fast9 ? 0 : ((Nd * a.M) / a.L + a.hl + 4) * sizeof(float2) + (a.hl + 1) * a.L * sizeof(float));
    if (a.L == 9 && a.M == 10 && a.hl == 24)  // os_min 1 (225 taps)
        hipLaunchKernelGGL((rx_fft_kernel<9, 10, 24>), g, b, lds, st, a);
    else if (a.L == 9 && a.M == 10 && a.hl == 4)  // os_min 2
        hipLaunchKernelGGL((rx_fft_kernel<9, 10, 4>), g, b, lds, st, a);
    else
        hipLaunchKernelGGL((rx_fft_kernel<0, 0, 0>), g, b, lds, st, a);
    return hipGetLastError();
}

// ===================================================================== back end
__device__ __forceinline__ int16_t q16(float v) {
    const float r = rintf(v);
    return static_cast<int16_t>(fminf(32767.f, fmaxf(-32768.f, r)));
}

// srsRAN demod_soft restatement: LTE max-log per axis with int16 scale constants
__device__ __forceinline__ void demap(float2 y, uint32_t N_bps, float* L) {
    switch (N_bps) {
        case 1:
            L[0] = -100.f * (y.x + y.y);
            break;
        case 2:
            L[0] = -100.f * y.x;
            L[1] = -100.f * y.y;
            break;
        case 4: {
            const float S = 400.f, yr = S * y.x, yi = S * y.y, o = 2.f * S * 0.31622776601683794f;
            L[0] = -yr;
            L[1] = -yi;
            L[2] = fabsf(yr) - o;
            L[3] = fabsf(yi) - o;
            break;
        }
        case 6: {
            const float S = 700.f, yr = S * y.x, yi = S * y.y, q = S * 0.15430334996209191f;
            L[0] = -yr;
            L[1] = -yi;
            L[2] = fabsf(yr) - 4.f * q;
            L[3] = fabsf(yi) - 4.f * q;
            L[4] = fabsf(L[2]) - 2.f * q;
            L[5] = fabsf(L[3]) - 2.f * q;
            break;
        }
        default: {
            const float S = 1000.f, yr = S * y.x, yi = S * y.y, q = S * 0.07669649888473704f;
            L[0] = -yr;
            L[1] = -yi;
            L[2] = fabsf(yr) - 8.f * q;
            L[3] = fabsf(yi) - 8.f * q;
            L[4] = fabsf(L[2]) - 4.f * q;
            L[5] = fabsf(L[3]) - 4.f * q;
            L[6] = fabsf(L[4]) - 2.f * q;
            L[7] = fabsf(L[5]) - 2.f * q;
            break;
        }
    }
}

__device__ __forceinline__ uint32_t seq_bit(const uint8_t* __restrict__ s, uint32_t i) {
    return (s[i >> 3] >> (7u - (i & 7u))) & 1u;
}

__global__ void __launch_bounds__(256) rx_back_kernel(rx_back_args A) {
    extern __shared__ __attribute__((aligned(16))) float2 smem[];
    __shared__ double red[16];
    const uint32_t pkt = blockIdx.x;
    const uint32_t N = A.N_occ, Nf = N + 1, nd = A.n_drs;
    const uint32_t NT = A.N_eff_TX;  // <= 4
    // Interlaced pilot buffer [N_RX][4][2 nd] (channel_antenna.hpp:38-63). The non-interlaced
    // per-DRS-symbol estimates of the reference are the entries at each stream's write offset.
    float2* zfi = smem;
    rx_pkt_state S = A.st[pkt];
    double sn = S.snr_SN, nn = S.snr_N;
    uint32_t sn_cnt = S.snr_SN_cnt, nn_cnt = S.snr_N_cnt;
    uint32_t lut_pick = 0;
    uint32_t ev_mode = 0, ev_rel = 0, ev_swap = 0, ev_lut = 0;
    uint32_t drs_off = 0, ev_off = 0;  // bit t: write offset of stream t in the latest DRS symbol
    const float2* Yp = A.Y + size_t(pkt) * A.N_RX * A.n_sym_total * A.Nf_pad;
    const uint8_t* pdc_seq = A.is_pdc ? A.pdc_seq[pkt] : nullptr;
    int16_t* llr = A.llr + size_t(pkt) * A.llr_stride;
    auto Yat = [&](uint32_t a, uint32_t l, uint32_t k) { return Yp[(size_t(a) * A.n_sym_total + l) * A.Nf_pad + k]; };
    auto snr_db = [&]() -> float {
        if (sn <= 0.0 || nn <= 0.0) return 0.f;
        const float Sa = static_cast<float>((sn - nn) / sn_cnt), Na = static_cast<float>(nn / nn_cnt);
        return 10.f * log10f(Sa / Na);
    };
    // on-the-fly Wiener interpolation at subcarrier k (rx_synced.cpp:932-946)
    auto chest = [&](uint32_t a, uint32_t t, uint32_t k) {
        const uint32_t tl = (t & 3u) ^ ev_swap;
        const uint32_t pw = A.lut_pw[ev_mode][ev_lut][(size_t(ev_rel) * 4 + tl) * Nf + k];
        const uint32_t nI = A.lut_n[ev_mode][ev_lut];
        const float* __restrict__ w = A.lut_w[ev_mode][ev_lut] + size_t(pw >> 16) * nI;
        const float2* z = zfi + (size_t(a) * 4 + t) * 2 * nd;
        uint32_t pos = pw & 0xFFFFu, step = 1;
        if (!ev_mode) {  // non-interlaced pilots of the latest DRS symbol
            pos = 2 * pos + ((ev_off >> t) & 1u);
            step = 2;
        }
        float ar = 0.f, ai = 0.f;
        for (uint32_t i = 0; i < nI; ++i) {
            const float2 v = z[pos + i * step];
            ar = fmaf(v.x, w[i], ar);
            ai = fmaf(v.y, w[i], ai);
        }
        return make_float2(ar, ai);
    };
    // combining + demapping + descrambling of cells [j0, j1); sym(j) gives the OFDM symbol
    auto cells = [&](const uint32_t* kk, uint32_t j0, uint32_t j1, uint32_t N_bps, const uint8_t* seq, auto sym) {
        const uint32_t cnt = j1 - j0;
        const uint32_t units = NT == 1 ? cnt : cnt / 2;
        for (uint32_t u = threadIdx.x; u < units; u += blockDim.x) {
            float2 x0, x1 = make_float2(0.f, 0.f);
            const uint32_t jj = j0 + (NT == 1 ? u : 2 * u);
            const uint32_t l = sym(jj);
            if (NT == 1) {  // MRC (rx_synced.cpp:1204-1306)
                const uint32_t k = kk[jj];
                float2 num = make_float2(0.f, 0.f);
                float den = 0.f;
                for (uint32_t a = 0; a < A.N_RX; ++a) {
                    const float2 h = chest(a, 0, k);
                    num = cadd(num, cmulc(Yat(a, l, k), h));
                    den += cnorm(h);
                }
                x0 = cscale(num, 1.0f / den);
            } else {  // SFBC pair (rx_synced.cpp:1335-1392)
                const uint32_t k0 = kk[jj], k1 = kk[jj + 1];
                const uint32_t pr = A.pair[(jj >> 1) % A.mod];
                const uint32_t tA = pr & 0xFu, tB = pr >> 4;
                float2 n0 = make_float2(0.f, 0.f), n1 = make_float2(0.f, 0.f);
                float den = 0.f;
                for (uint32_t a = 0; a < A.N_RX; ++a) {
                    const float2 h0 = cscale(cadd(chest(a, tA, k0), chest(a, tA, k1)), 0.5f);
                    const float2 h1 = cscale(cadd(chest(a, tB, k0), chest(a, tB, k1)), 0.5f);
                    const float2 r0 = Yat(a, l, k0), r1 = Yat(a, l, k1);
                    n0 = cadd(n0, cadd(cmul(cconj(h0), r0), cmul(h1, cconj(r1))));
                    n1 = cadd(n1, cadd(cmul(make_float2(-h1.x, -h1.y), cconj(r0)), cmul(cconj(h0), r1)));
                    den += cnorm(h0) + cnorm(h1);
                }
                x0 = cscale(n0, 1.0f / den);
                x1 = cscale(n1, 1.0f / den);
            }
            for (uint32_t q = 0; q < (NT == 1 ? 1u : 2u); ++q) {
                float L[8];
                demap(q ? x1 : x0, N_bps, L);
                const uint32_t base = (jj + q) * N_bps;
                for (uint32_t b = 0; b < N_bps; ++b) {
                    const float v = seq_bit(seq, base + b) ? -L[b] : L[b];
                    llr[base + b] = q16(v);
                }
            }
        }
    };

    for (uint32_t o = 0; o < A.n_ops; ++o) {
        const rx_op op = A.ops[o];
        if (op.kind == 1) {  // OP_DRS: zero-forcing (rx_synced.cpp:773-861)
            const uint32_t meta = A.drs_meta[op.b];
            const uint32_t tf = meta & 0xFFu, tlst = (meta >> 8) & 0xFFu, par = (meta >> 16) & 0xFFu;
            const uint32_t l = op.a, rel = op.c, ps = op.d;
            const uint32_t nts = tlst - tf + 1;
            drs_off = 0;
            for (uint32_t t = tf; t <= tlst; ++t) {  // channel_antenna.hpp:38-63 write offsets
                const bool lhs = rel <= 1, hi = (t & 3u) >= 2;
                const uint32_t off = (ps % 2 == 0) ? (lhs ? hi : !hi) : (lhs ? !hi : hi);
                drs_off |= off << t;
            }
            for (uint32_t e = threadIdx.x; e < A.N_RX * nts * nd; e += blockDim.x) {
                const uint32_t i = e % nd, t = tf + (e / nd) % nts, a = e / (nd * nts);
                const uint32_t k = A.drs_k[((par * 4) + (t & 3u)) * nd + i];
                const float2 v = cscale(Yat(a, l, k), A.drs_v[t * nd + i]);
                zfi[(a * 4 + t) * 2 * nd + 2 * i + ((drs_off >> t) & 1u)] = v;
            }
            __syncthreads();
            double s1 = 0.0, s2 = 0.0;  // estimator_snr.cpp:104-146
            for (uint32_t e = threadIdx.x; e < A.N_RX * nts * nd; e += blockDim.x) {
                const uint32_t i = e % nd, t = tf + (e / nd) % nts, a = e / (nd * nts);
                const float2* z = zfi + (a * 4 + t) * 2 * nd + ((drs_off >> t) & 1u);
                const float2 v = z[2 * i];
                s1 += cnorm(v);
                if (i + 1 < nd) s2 += cnorm(csub(v, z[2 * i + 2]));
            }
            sn += block_sum(s1, red);
            nn += block_sum(s2, red) / 2.0;
            sn_cnt += A.N_RX * nts * nd;
            nn_cnt += A.N_RX * nts * (nd - 1);
            // LUT pick: nearest profile SNR, ties to the later profile (rx_synced.cpp:863-891)
            const float s = snr_db();
            float best = fabsf(s - A.prof_snr[0]);
            lut_pick = 0;
            for (uint32_t i = 1; i < 3; ++i) {
                const float d = fabsf(s - A.prof_snr[i]);
                if (d <= best) {
                    best = d;
                    lut_pick = i;
                }
            }
        } else if (op.kind == 2) {  // OP_EVENT
            ev_mode = op.a;
            ev_rel = op.b;
            ev_swap = (op.c & 1u) ? 2u : 0u;
            ev_lut = lut_pick;
            ev_off = drs_off;
        } else if (op.kind == 3) {  // OP_PCC
            const uint32_t l = op.a;
            cells(A.pcc_k, A.pcc_off[op.b], A.pcc_off[op.b + 1], 2, A.pcc_seq, [&](uint32_t) { return l; });
        } else if (op.kind == 4) {  // OP_PDC: merge the run of PDC symbols sharing the current estimate
            uint32_t o2 = o;
            while (o2 + 1 < A.n_ops && A.ops[o2 + 1].kind == 4) ++o2;
            const uint32_t l0 = op.a, l1 = A.ops[o2].a;
            cells(A.pdc_k, A.pdc_off[l0], A.pdc_off[l1 + 1], A.N_bps, pdc_seq,
                  [&](uint32_t j) { return static_cast<uint32_t>(A.pdc_sym[j]); });
            o = o2;
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        if (A.is_pdc)
            A.st[pkt].snr_pdc = snr_db();
        else
            A.st[pkt].snr_pcc = snr_db();
    }
}

hipError_t launch_rx_back(const rx_back_args& a, uint32_t n, hipStream_t st) {
    const size_t lds = size_t(a.N_RX) * 4 * a.n_drs * 2 * sizeof(float2);
    hipLaunchKernelGGL(rx_back_kernel, dim3(n), dim3(256), lds, st, a);
    return hipGetLastError();
}

}  // namespace dnrp::dev
