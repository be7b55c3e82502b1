// RX kernels for the synchronised receiver (rx_synced_t, lib/src/phy/rx/rx_synced/rx_synced.cpp).
//
//  rx_stf_kernel   one WG per packet: polyphase M/L resampling + CFO mixer of the STF on all RX
//                  antennas, RMS, cover-sequence revert, fractional CFO re-estimate
//                  (rx_synced.cpp:503-661), STF FFT + zero-forcing, fractional STO
//                  (estimator_sto.cpp:47-170), STF SNR (estimator_snr.cpp:48-66).
//  rx_fft_kernel   one WG per (packet, antenna, symbol block): resampling + phase-continuous mixer
//                  + CP removal + FFT + bin extraction + amplitude scaling + STO derotation
//                  (rx_synced.cpp:711-771) into the frequency-domain grid Y in HBM.
// The back end (channel estimation, equalisation, demapping) is in rx_back.hip.
#include "device_common.hpp"
#include "experiments.hpp"
#include "kernels.hpp"
#include "polyphase.hpp"
#include "rx_front.hpp"
#include "taps_gen.hpp"

namespace dnrp::dev {

__constant__ float k_cover_rx[9] = DNRP_STF_COVER_SEQUENCE;  // stf.hpp:146-151 (params.hpp)

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
    // input index q relative to the fine peak, zero history before it: valid for q in
    // [max(0, -fine_peak), S_in - fine_peak)
    stage_span_lo<8>(inbuf, x + fine_peak, q0, n_in, fine_peak < 0 ? -fine_peak : 0,
                     static_cast<int64_t>(A.S_in) - fine_peak, threadIdx.x, blockDim.x);
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
// float2 slots of rx_stf_kernel's input staging, which also holds the FFT's two Nd buffers
__host__ __device__ inline uint32_t rx_stf_in(uint32_t n_stf, uint32_t Nd, uint32_t M, uint32_t L, uint32_t hl) {
    const uint32_t n_in = (n_stf * M) / L + hl + 4;
    return n_in > 2 * Nd ? n_in : 2 * Nd;
}

// One workgroup per (packet, antenna): resampling + mixer of the antenna's STF, its RMS, the cover
// revert, its pattern correlation sum and its STF cells (FFT + extraction) -> A.stf_cs / stf_rms /
// stf_ys. The antennas of a packet run in parallel instead of in series inside one workgroup; the
// arithmetic of each antenna is the one the single-workgroup form ran (same 256-thread loops and
// block sums), so rx_stf_kernel's results are unchanged.
__device__ __forceinline__ int64_t floordiv_rx(int64_t a, int64_t b) { return a >= 0 ? a / b : -((-a + b - 1) / b); }
// float2 offset of the tap table in rx_stf_ant_kernel's chunked layout: behind sbuf + the span of one
// chunk of outputs, and behind the two FFT buffers laid over sbuf
__host__ __device__ inline uint32_t rx_stf_chunk_taps(uint32_t n_stf, uint32_t Nd, uint32_t C, uint32_t M, uint32_t L,
                                                      uint32_t hl) {
    const uint32_t a = n_stf + (C * M) / L + hl + 4 + M, b = 2 * Nd;
    return a > b ? a : b;
}
// float2 slots of rx_stf_ant_kernel's compact area: the 9/10 input span of n_stf outputs (upper bound)
__host__ __device__ inline uint32_t rx_stf_area(uint32_t n_stf) { return ((n_stf + 18) * 10) / 9 + 33 + 10 + 2; }

#ifndef DNRP_STF_STAGE_U
#define DNRP_STF_STAGE_U 10  // span loads in flight per thread (C4's ~2400-input STF span by 256 threads: one
                             // round trip; 8: two -- measured neutral, 1.04 ms either way)
#endif
#ifndef DNRP_STF_IMAJ
#define DNRP_STF_IMAJ 1  // compiled-in taps: the FIR input-major from LDS (0: the whole window in registers)
#endif
#ifndef DNRP_STF_WPE
#define DNRP_STF_WPE 8  // waves per SIMD the register budget must allow (256-thread workgroups: = per CU)
#endif
template <int HL, bool CT = false, bool CHUNK = false>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(CT ? DNRP_STF_WPE : 1))) rx_stf_ant_kernel(rx_front_args A) {
    extern __shared__ __attribute__((aligned(16))) float2 smem[];
    __shared__ double red[16];
    const uint32_t pkt = rx_slot_of(A.sel, blockIdx.x / A.N_RX), a = blockIdx.x % A.N_RX;
    const uint32_t Nd = A.plan.N;
    const uint32_t n_stf = A.STF_CP + Nd, n = A.b * 14;  // n: STF cells per antenna
    // compact layout (compiled-in taps, N a power of 4): one area holds the input span at its top and
    // the resampled STF from its bottom (a block's outputs stay below every window: 9 outputs per 10
    // inputs), and the FFT runs in place on its first N slots; otherwise sbuf | inbuf (FFT buffers) | taps
    // chunked layout (A.stf_chunk > 0: N_b_DFT_os = 8192, where sbuf + the whole span exceed the LDS):
    // the STF resampled in chunks of stf_chunk outputs through a small input buffer, the FFT buffers
    // over sbuf once its samples are consumed
    const uint32_t lgN = 31u - __clz(Nd);
    const uint32_t C = CHUNK ? A.stf_chunk : 0u;  // a separate instantiation: its register-staged FFT
                                                   // input would cost the other layouts occupancy
    const bool compact = CT && C == 0 && (lgN & 1u) == 0 && A.STF_CP >= Nd + Nd / 32;  // the host sizes the LDS by the same test
    float2* sbuf = smem;                                    // n_stf
    float2* inbuf = sbuf + n_stf;                           // rx_stf_in(...) / the chunk's span
    float2* fa = C ? smem : inbuf;                          // Nd
    float2* fb = fa + Nd;                                   // Nd
    float* taps = reinterpret_cast<float*>(smem + (C ? rx_stf_chunk_taps(n_stf, Nd, C, A.M, A.L, A.hl)
                                                     : n_stf + rx_stf_in(n_stf, Nd, A.M, A.L, A.hl)));
    if (!CT || C) stage_copy<4>(taps, A.taps, (A.hl + 1) * A.L, threadIdx.x, blockDim.x);
    const rx_pkt_in in = A.pin[pkt];
    const uint32_t P = n_stf / A.n_pattern;
    const float2* x = A.iq + (size_t(in.win) * A.N_RX + a) * A.S_in;
    if (C) {
        __syncthreads();  // taps
        for (uint32_t m0 = 0; m0 < n_stf; m0 += C)
            resample_block<HL>(A, x, in.fine_peak, m0, min(C, n_stf - m0), inbuf, sbuf + m0, taps,
                               static_cast<double>(m0) * in.inc0, in.inc0);
    } else if (CT) {
        // compile-time 9/10 taps: the span staged once, then thread q one polyphase block of 9 outputs
        // from its 33-input window in registers (each tap an immediate, summed newest input first as
        // resample_block does), mixed with a phasor at the block start stepped by the increment
        using PD = pp_direct<9, 10, 24>;
        constexpr int W = PD::W;
        const int64_t ms = A.m_star;
        const int64_t q0 = floordiv_rx(0 - ms, 9), q1 = floordiv_rx(static_cast<int64_t>(n_stf) - ms + 8, 9);
        const int64_t in0 = static_cast<int64_t>(A.p_star) + 10 * q0 - 24;  // relative to the fine peak
        const uint32_t n_in = static_cast<uint32_t>(10 * (q1 - 1 - q0) + W);
        float2* span = compact ? smem + ((rx_stf_area(n_stf) - n_in) & ~1u) : inbuf;
        stage_span_lo<DNRP_STF_STAGE_U>(span, x + in.fine_peak, in0, n_in, in.fine_peak < 0 ? -in.fine_peak : 0,
                         static_cast<int64_t>(A.S_in) - in.fine_peak, threadIdx.x, blockDim.x);
        __syncthreads();
        const float2 step1 = phasor(in.inc0);
        // rounds of blockDim blocks, the same count for every thread: each round's windows are read
        // by every wave before any wave writes that round's outputs (a wave one round ahead would
        // otherwise overwrite windows a slower wave has still to read: with Nd = 4096 a round's
        // outputs reach into the previous round's windows), and a round's outputs stay below every
        // later round's windows
        const uint32_t rounds = static_cast<uint32_t>((q1 - q0 + blockDim.x - 1) / blockDim.x);
        for (uint32_t rd = 0; rd < rounds; ++rd) {
            const int64_t q = q0 + threadIdx.x + int64_t(rd) * blockDim.x;
            float2 y[9];
            const float2* xw = span + 10 * min<int64_t>(q - q0, q1 - 1 - q0);
            if constexpr (DNRP_STF_IMAJ) {
                // input-major, newest input first: window input i (i = W-1 .. 0) updates every output
                // k whose span holds it (d = 24 + o_k - i), so each output sums d = 0 .. 24 in the
                // output-major order below, bit for bit; live state is the 9 sums and one input pair,
                // not the 33-input window (VGPRs: occupancy of this latency-bound kernel)
#pragma unroll
                for (int k = 0; k < 9; ++k) y[k] = make_float2(0.f, 0.f);
                const float4* x4 = reinterpret_cast<const float4*>(xw);  // xw even: 16-B pairs
                float4 nxt = x4[W / 2 - (W % 2 ? 0 : 1)];
#pragma unroll
                for (int j = (W - 1) / 2; j >= 0; --j) {  // pair (2j, 2j + 1), the odd input first
                    const float4 cur = nxt;
                    if (j > 0) nxt = x4[j - 1];
                    asm volatile("" ::: "memory");  // one pair ahead, not the whole window
#pragma unroll
                    for (int e = 1; e >= 0; --e) {
                        const int i = 2 * j + e;
                        if (i >= W) continue;
                        const float2 xi = e ? make_float2(cur.z, cur.w) : make_float2(cur.x, cur.y);
#pragma unroll
                        for (int k = 0; k < 9; ++k) {
                            const int o = (k * 10) / 9, ph = (k * 10) % 9, d = 24 + o - i;
                            if (d < 0 || d > 24) continue;
                            const float h = taps_rx_9_10::h[ph + d * 9];
                            y[k].x = fmaf(xi.x, h, y[k].x);
                            y[k].y = fmaf(xi.y, h, y[k].y);
                        }
                    }
                    // the sums pinned here: the compiler would otherwise sink every FMA behind the
                    // barrier into its output's store branch with the whole window live again
                    asm volatile("" : "+v"(y[0]), "+v"(y[1]), "+v"(y[2]), "+v"(y[3]), "+v"(y[4]), "+v"(y[5]), "+v"(y[6]),
                                 "+v"(y[7]), "+v"(y[8]));
                }
            } else {
                float2 xv[W];
                PD::template load<true>(xw, xv);
#pragma unroll
                for (int k = 0; k < 9; ++k) {
                    const int o = (k * 10) / 9, ph = (k * 10) % 9;
                    float ar = 0.f, ai = 0.f;
#pragma unroll
                    for (int d = 0; d <= 24; ++d) {
                        const float h = taps_rx_9_10::h[ph + d * 9];
                        ar = fmaf(xv[24 + o - d].x, h, ar);
                        ai = fmaf(xv[24 + o - d].y, h, ai);
                    }
                    y[k] = make_float2(ar, ai);
                }
            }
            __syncthreads();  // every window of the round read before its outputs overwrite the span
            if (q >= q1) continue;
            const int64_t mb = ms + 9 * q;
            float2 r = phasor(static_cast<double>(mb) * in.inc0);
#pragma unroll
            for (int k = 0; k < 9; ++k) {
                const int64_t m = mb + k;
                if (m >= 0 && m < static_cast<int64_t>(n_stf)) sbuf[m] = cmul(y[k], r);
                r = cmul(r, step1);
            }
        }
        __syncthreads();
    } else {
        resample_block<HL>(A, x, in.fine_peak, 0, n_stf, inbuf, sbuf, taps, 0.0, in.inc0);
    }
    double e = 0.0, pr = 0.0, pi = 0.0;
    for (uint32_t i = threadIdx.x; i < n_stf; i += blockDim.x) e += cnorm(sbuf[i]);
    e = block_sum(e, red);
    for (uint32_t i = threadIdx.x; i < n_stf; i += blockDim.x)
        sbuf[i] = cscale(sbuf[i], k_cover_rx[min(i / A.pattern_len, 8u)]);
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < (A.n_pattern - 1) * P; i += blockDim.x) {
        const float2 c = cmulc(sbuf[i], sbuf[i + P]);
        pr += c.x;
        pi += c.y;
    }
    pr = block_sum(pr, red);
    pi = block_sum(pi, red);
    const float2* F;
    if (compact) {  // in place on sbuf[0, N + N/32) (bank-padded slots, below STF_CP >= N + N/32): the
                    // inputs sbuf[STF_CP + i] at digit-reversed slots
        for (uint32_t i = threadIdx.x; i < Nd; i += blockDim.x) sbuf[r4pad(rev4(i, lgN))] = sbuf[A.STF_CP + i];
        __syncthreads();
        fft_r4_inplace<-1, true>(sbuf, A.tw, lgN);
        const uint32_t N = A.N_occ;
        float2* ys = A.stf_ys + (size_t(pkt) * 8 + a) * A.stf_ys_stride;
        for (uint32_t w = threadIdx.x; w < n; w += blockDim.x) {  // extract_bins on the padded slots
            const uint32_t k = w < n / 2 ? 4 * w : 4 * w + 4;
            ys[w] = cscale(k >= N / 2 ? sbuf[r4pad(k - N / 2)] : sbuf[r4pad(A.off_lower + k)], A.amp_scale);
        }
        F = nullptr;
    } else if (CHUNK) {  // fa overlaps the STF samples it is filled from: through registers
        constexpr uint32_t MAXR = 8192 / 256;
        float2 v[MAXR];
#pragma unroll
        for (uint32_t j = 0; j < MAXR; ++j) {
            const uint32_t i = threadIdx.x + j * blockDim.x;
            if (i < Nd) v[j] = sbuf[A.STF_CP + i];
        }
        __syncthreads();
#pragma unroll
        for (uint32_t j = 0; j < MAXR; ++j) {
            const uint32_t i = threadIdx.x + j * blockDim.x;
            if (i < Nd) fa[i] = v[j];
        }
        __syncthreads();
        F = fft_any<-1>(fa, fb, A.tw, A.plan);
    } else {
        for (uint32_t i = threadIdx.x; i < Nd; i += blockDim.x) fa[i] = sbuf[A.STF_CP + i];
        __syncthreads();
        F = fft_any<-1>(fa, fb, A.tw, A.plan);
    }
    float2* ys = A.stf_ys + (size_t(pkt) * 8 + a) * A.stf_ys_stride;
    if (!compact)
        for (uint32_t w = threadIdx.x; w < n; w += blockDim.x) extract_bins(A, F, &ys[w], w < n / 2 ? 4 * w : 4 * w + 4);
    if (threadIdx.x == 0) {
        A.stf_rms[size_t(pkt) * 8 + a] = sqrtf(static_cast<float>(e / n_stf));
        A.stf_cs[size_t(pkt) * 8 + a] = make_double2(pr, pi);
    }
}

// One workgroup per packet: the antennas' STF results combined (rx_synced.cpp:503-709): fractional
// CFO re-estimate, STF zero-forcing, fractional STO, STF SNR -> the packet state.
__global__ void __launch_bounds__(256) rx_stf_kernel(rx_front_args A) {
    extern __shared__ __attribute__((aligned(16))) float2 smem[];
    __shared__ double red[16];
    const uint32_t pkt = rx_slot_of(A.sel, blockIdx.x);
    const uint32_t Nd = A.plan.N, N = A.N_occ;
    const uint32_t n_stf = A.STF_CP + Nd, n = A.b * 14;
    float2* Ys = smem;          // [N_RX][n]
    float2* St = Ys + A.N_RX * n;  // [n]: the STF value of cell w (subcarrier rstf(w))
    auto rstf = [&](uint32_t w) { return w < n / 2 ? 4 * w : 4 * w + 4; };
    for (uint32_t w0 = 0; w0 < n; w0 += blockDim.x) {  // every antenna's cells in flight together
        const uint32_t w = w0 + threadIdx.x;
        float2 yv[8], sv = make_float2(0.f, 0.f);
        if (w < n) sv = A.stf[rstf(w)];
#pragma unroll
        for (uint32_t a = 0; a < 8; ++a)
            if (a < A.N_RX && w < n) yv[a] = A.stf_ys[(size_t(pkt) * 8 + a) * A.stf_ys_stride + w];
#pragma unroll
        for (uint32_t a = 0; a < 8; ++a)
            if (a < A.N_RX && w < n) Ys[a * n + w] = yv[a];
        if (w < n) St[w] = sv;
    }
    const rx_pkt_in in = A.pin[pkt];
    const uint32_t P = n_stf / A.n_pattern;
    double cs_re = 0.0, cs_im = 0.0;
    rx_pkt_state S;
    for (uint32_t a = 0; a < A.N_RX; ++a) {  // antenna order, as the single-workgroup form summed
        const double2 c = A.stf_cs[size_t(pkt) * 8 + a];
        cs_re += c.x;
        cs_im += c.y;
    }
#pragma unroll
    for (uint32_t a = 0; a < 8; ++a)  // compile-time slots: S stays in registers, not a scratch struct
        S.rms[a] = a < A.N_RX ? A.stf_rms[size_t(pkt) * 8 + a] : 0.f;
    __syncthreads();
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
    auto zf = [&](uint32_t a, uint32_t w, double inc) {
        const uint32_t r = rstf(w);
        float2 y = Ys[a * n + w];
        if (inc != 0.0) y = cmul(y, phasor(-inc * static_cast<double>(N / 2) + inc * static_cast<double>(r)));
        const float2 s = St[w];
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
// One WG per (packet, antenna, run of sym_per_block symbols); the symbols are processed in passes of
// A.fft_pass (2, or 1 where two do not fit the LDS: N_b_DFT_os >= 4096): resampling into LDS, one
// batched FFT, bin extraction + STO derotation. Register-blocked path (LR > 0): the hw-rate input span
// of the pass is staged in LDS with coalesced loads, then thread j computes the L outputs of aligned
// block j (polyphase.hpp). LDS: fa [pass][Nd] | fb [pass][Nd], aliased by the input span (free once the
// pass is resampled; the next pass stages after the extraction's barrier) | rot [Nf] | twiddles [Nd]
// (A.fft_tw_lds; else read through the L1) | taps.
constexpr uint32_t RX_THREADS = 256;
constexpr uint32_t RX_SYM_PASS = 2;

// LDS samples for one pass's input span (host and device agree on this bound)
__host__ __device__ inline uint32_t rx_in_cap(uint32_t Nd, uint32_t CP, uint32_t L, uint32_t M, uint32_t W,
                                              uint32_t pass = RX_SYM_PASS) {
    return ((pass * (Nd + CP)) * M + L - 1) / L + W + 2 * M + 2 * L;
}

template <int LR, int MR, int HLR>
__global__ void __launch_bounds__(RX_THREADS) rx_fft_kernel(rx_front_args A) {
    extern __shared__ __attribute__((aligned(16))) float2 smem[];
    const uint32_t Nd = A.plan.N, N = A.N_occ, Nf = N + 1;
    const uint32_t nblk = (A.sym_count + A.sym_per_block - 1) / A.sym_per_block;
    const uint32_t blk = blockIdx.x % nblk;
    const uint32_t a = (blockIdx.x / nblk) % A.N_RX;
    const uint32_t pkt = rx_slot_of(A.sel, blockIdx.x / (nblk * A.N_RX));
    using PB = pp_block<(LR > 0 ? LR : 1), (LR > 0 ? MR : 1), (LR > 0 ? HLR : 0)>;
    const uint32_t SP = A.fft_pass;
    const uint32_t in_cap = LR > 0 ? rx_in_cap(Nd, A.CP, LR, MR, PB::W, SP) : (Nd * A.M) / A.L + A.hl + 4;
    float2* fa = smem;                                    // [SP][Nd]
    float2* fb = fa + SP * Nd;                            // [SP][Nd]
    float2* inbuf = fb;                                   // input span of a pass
    float2* rot = fb + max(SP * Nd, in_cap);              // Nf: STO derotation per subcarrier
    float2* twl = rot + Nf;                               // Nd (fft_tw_lds)
    const float2* tw = A.fft_tw_lds ? twl : A.tw;
    float* taps = reinterpret_cast<float*>(twl + (A.fft_tw_lds ? Nd : 0u));
    if (A.fft_tw_lds) stage_copy<4>(twl, A.tw, Nd, threadIdx.x, RX_THREADS);
    if (LR == 0)
        for (uint32_t i = threadIdx.x; i < (A.hl + 1) * A.L; i += RX_THREADS) taps[i] = A.taps[i];
    else
        stage_copy<4>(taps, A.taps_pp, A.npp, threadIdx.x, RX_THREADS);
    const rx_pkt_in in = A.pin[pkt];
    const rx_pkt_state S = A.st[pkt];
    const uint32_t n_stf = A.STF_CP + Nd;
    for (uint32_t k = threadIdx.x; k < Nf; k += RX_THREADS)
        rot[k] = phasor(-S.sto_inc * static_cast<double>(N / 2) + S.sto_inc * static_cast<double>(k));
    const float2* x = A.iq + (size_t(in.win) * A.N_RX + a) * A.S_in;
    const double phi_stf = static_cast<double>(n_stf) * in.inc0;  // mixer phase at the first data sample
    const float2 step1 = phasor(S.inc1);
    const uint32_t l0 = A.sym_first + blk * A.sym_per_block;
    const uint32_t l1 = min(A.sym_first + A.sym_count, l0 + A.sym_per_block);
    // valid input window relative to the fine peak: history is zero before it (rx_synced.cpp:711-740)
    const int64_t q_hi = static_cast<int64_t>(A.S_in) - in.fine_peak, q_lo = in.fine_peak < 0 ? -in.fine_peak : 0;
    auto m_first = [&](uint32_t l) { return static_cast<int>(n_stf + (l - 1) * (A.CP + Nd) + A.CP); };
    for (uint32_t lp = l0; lp < l1; lp += SP) {
        const uint32_t ns = min(SP, l1 - lp);
        if constexpr (LR > 0) {
            const int m_a = m_first(lp), m_b = m_first(lp + ns - 1) + static_cast<int>(Nd);
            const int qb0 = (m_a - static_cast<int>(A.m_star)) / LR;  // m_a >= m_star
            const int qb1 = (m_b - static_cast<int>(A.m_star) + LR - 1) / LR;
            const int64_t in0 = static_cast<int64_t>(A.p_star) + int64_t(MR) * qb0 - HLR;
            const uint32_t n_in = static_cast<uint32_t>(MR * (qb1 - 1 - qb0) + PB::W);
            const float2* src = x + in.fine_peak + in0;
            stage_span_lo<8>(inbuf, src - in0, in0, n_in, q_lo, q_hi, threadIdx.x, RX_THREADS);
            __syncthreads();
            for (int q = qb0 + static_cast<int>(threadIdx.x); q < qb1; q += RX_THREADS) {
                const int mb = static_cast<int>(A.m_star) + LR * q;
                // the symbol this block feeds (blocks in the CP gap feed none)
                const uint32_t s = (ns > 1 && mb + LR > m_first(lp + 1)) ? 1u : 0u;
                const int m0 = m_first(lp + s);
                if (mb + LR <= m0 || mb >= m0 + static_cast<int>(Nd)) continue;
                float2 y[LR];
                PB::run(inbuf + MR * (q - qb0), taps, y);
                float2 r = phasor(phi_stf + static_cast<double>(mb - static_cast<int>(n_stf)) * S.inc1);
                float2* dst = fa + s * Nd;
#pragma unroll
                for (int k = 0; k < LR; ++k) {
                    const uint32_t idx = static_cast<uint32_t>(mb + k - m0);
                    if (idx < Nd) dst[idx] = cmul(y[k], r);
                    r = cmul(r, step1);
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
        const float2* F = fft_any<-1>(fa, fb, tw, A.plan, ns);
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

static bool rx_fft_layout(rx_front_args& a);

// LDS bytes of rx_stf_ant_kernel's launch (compact: the compiled-in taps' in-place layout; sets
// a.stf_chunk where only the chunked layout fits)
static size_t rx_stf_lds(rx_front_args& a) {
    const uint32_t Nd = a.plan.N, n_stf = a.STF_CP + Nd;
    const size_t taps = size_t(a.hl + 1) * a.L * sizeof(float);
    uint32_t lgN = 0;
    while ((1u << lgN) < Nd) ++lgN;
    a.stf_chunk = 0;
    const bool ct = a.stream && a.L == 9 && a.M == 10 && a.hl == 24;
    if (ct && lgN % 2 == 0 && a.STF_CP >= Nd + Nd / 32) return size_t(std::max(rx_stf_area(n_stf), n_stf)) * sizeof(float2);
    const size_t whole = (n_stf + rx_stf_in(n_stf, Nd, a.M, a.L, a.hl)) * sizeof(float2) + taps;
    if (whole <= 160 * 1024 || Nd > 8192) return whole;
    a.stf_chunk = 2048;
    return rx_stf_chunk_taps(n_stf, Nd, a.stf_chunk, a.M, a.L, a.hl) * sizeof(float2) + taps;
}

bool rx_front_fits(const rx_front_args& a_in) {  // every RX front-end launch of the geometry fits the LDS
    rx_front_args a = a_in;
    return rx_stf_lds(a) <= 160 * 1024 && (rx_fft_wave_path(a) || rx_fft_layout(a));
}

hipError_t launch_rx_stf(const rx_front_args& a_in, uint32_t n, hipStream_t st) {
    rx_front_args a = a_in;
    const size_t lds = rx_stf_lds(a);
    if (lds > 160 * 1024) return hipErrorInvalidValue;
    if (a.stf_chunk)  // N_b_DFT_os = 8192: the chunked layout, run-time taps
        hipLaunchKernelGGL((rx_stf_ant_kernel<-1, false, true>), dim3(n * a.N_RX), dim3(256), lds, st, a);
    else if (a.stream && a.L == 9 && a.M == 10 && a.hl == 24)  // compiled-in taps (table taps: 0.50 vs 0.38 ms, docs/DESIGN_LOG.md §6)
        hipLaunchKernelGGL((rx_stf_ant_kernel<24, true>), dim3(n * a.N_RX), dim3(256), lds, st, a);
    else
        DNRP_HL_DISPATCH(rx_stf_ant_kernel, dim3(n * a.N_RX), dim3(256), lds, st, a);
    hipLaunchKernelGGL(rx_stf_kernel, dim3(n), dim3(256), size_t(a.N_RX + 1) * a.b * 14 * sizeof(float2), st, a);
    return hipGetLastError();
}

// ---- N_b_DFT_os = 1024: one wavefront per symbol, no workgroup barrier after the table load.
// The wave stages its symbol's hw-rate input span in its own LDS region, resamples it with the
// register-blocked polyphase blocks (outputs kept in registers), writes the 1024 outputs back into
// the same region as FFT input, runs wave_fft1024 there, and stores the occupied bins, amplitude
// scaled and STO-derotated, straight to Y.
constexpr uint32_t RXW_SYMS = 4;  // symbols (= wavefronts) per workgroup

// WPG symbols (= wavefronts) per workgroup: the compile-time-tap path shares nothing between its
// waves, so it can run one wave per workgroup and free each wave's LDS region when that wave retires
template <int LR, int MR, int HLR, bool CT, int WPG = RXW_SYMS, bool RT = false>
__global__ void __launch_bounds__(RX_THREADS) __attribute__((amdgpu_waves_per_eu(4))) rx_fft_wave_kernel(rx_front_args A) {
    extern __shared__ __attribute__((aligned(16))) float2 smem[];
    using PB = pp_block<LR, MR, HLR>;
    constexpr uint32_t Nd = 1024;
    static_assert(CT || WPG == RXW_SYMS, "the table path shares its tables among RXW_SYMS waves");
    const uint32_t nblk = (A.sym_count + WPG - 1) / WPG;
    const uint32_t blk = blockIdx.x % nblk;
    const uint32_t a = (blockIdx.x / nblk) % A.N_RX;
    const uint32_t pkt = rx_slot_of(A.sel, blockIdx.x / (nblk * A.N_RX));
    const uint32_t region = rxw_region(LR, MR, PB::W);
    // CT (compile-time taps, pp_const): no tap table, twiddles through the L1, only the wave
    // regions live in LDS (4 workgroups per CU instead of 3); otherwise LDS twiddles + tap table
    float2* twl = smem;                                              // Nd (table path)
    float* taps = reinterpret_cast<float*>(twl + Nd);                // npp (table path)
    float2* reg0 = CT ? smem : twl + Nd + (A.npp + 1) / 2;           // RXW_SYMS regions
    if constexpr (!CT) {
        stage_copy<4>(twl, A.tw, Nd, threadIdx.x, RX_THREADS);
        stage_copy<4>(taps, A.taps_pp, A.npp, threadIdx.x, RX_THREADS);
    }
    const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63u;
    const uint32_t li = blk * WPG + w;  // launch symbol
    const bool active = li < A.sym_count;
    const uint32_t l = A.sym_list ? A.sym_list[min(li, A.sym_count - 1)] : A.sym_first + li;
    const rx_pkt_in in = A.pin[pkt];
    const rx_pkt_state S = A.st[pkt];
    const rx_span_t sp = rx_span<LR, MR, HLR>(A, l);
    float2* R = reg0 + w * region;
    // valid input window relative to the fine peak: history is zero before it (rx_synced.cpp:711-740)
    const int64_t q_hi = static_cast<int64_t>(A.S_in) - in.fine_peak, q_lo = in.fine_peak < 0 ? -in.fine_peak : 0;
    const float2* src = A.iq + (size_t(in.win) * A.N_RX + a) * A.S_in + in.fine_peak;
    // a DRS symbol's bins also stay in R for the SNR partial sums: its op-table entry by a scalar load
    // issued ahead of the staging (a vector load here would add a memory round trip to every wave)
    uint32_t so = 0xFFFFu;
    if (A.snr_part && l < A.n_sym_op) {
        const auto* sop = reinterpret_cast<const __attribute__((address_space(4))) uint32_t*>(reinterpret_cast<uintptr_t>(A.sym_op));
        so = (sop[l >> 1] >> (16 * (l & 1u))) & 0xFFFFu;
    }
    float2 w1 = make_float2(1.f, 0.f), wl = w1;
    if constexpr (RT) {  // the FFT's two lane twiddles, in flight with the staging loads
        w1 = wfft_tw<-1>(A.tw, 4 * (lane & 15u));
        wl = wfft_tw<-1>(A.tw, lane);
    }
    if (active) stage_span_lo<20>(R, src, sp.in0, sp.n_in, q_lo, q_hi, lane, 64);
    if constexpr (CT)
        __builtin_amdgcn_wave_barrier();  // only the wave's own staging
    else
        __syncthreads();  // twiddles / taps (and this wave's own staging)
    if (!active) return;
    float2* Yrow = A.Y + ((size_t(pkt) * A.N_RX + a) * A.n_sym_total + l) * A.Nf_pad;
    const bool drs = so != 0xFFFFu;
    if constexpr (CT) {
        rx_resample_ct<LR, MR, HLR>(A, in, S, sp, R, lane);
        // one instantiation of the (large, unrolled) FFT for both kinds of symbol: instruction cache
        const bool to_y = !A.no_y;
        rx_fft_bins<RT>(A, S, R, lane, [&](uint32_t k, float2 v) {
            if (to_y) Yrow[k] = v;
            if (drs) R[k] = v;
        }, w1, wl);
        if (drs) {
            __builtin_amdgcn_wave_barrier();
            rx_drs_partials(A, pkt, a, l, so, R, lane);
        }
        return;
    } else {
        constexpr int BR = (Nd + 2 * LR) / LR / 64 + 1;  // block rounds per lane
        const int n_stf = static_cast<int>(A.STF_CP + Nd);
        const double phi_stf = static_cast<double>(n_stf) * in.inc0;  // mixer phase at the first data sample
        const float2 step1 = phasor(S.inc1);
        float2 ys[BR][LR];
        // all rounds of the lane in one pass over the tap rows (pp_block::run_multi); rounds past
        // the symbol's last block read a valid window and are discarded
        const float2* xw[BR];
#pragma unroll
        for (int rd = 0; rd < BR; ++rd) xw[rd] = R + MR * min(static_cast<int>(lane) + 64 * rd, sp.qb1 - 1 - sp.qb0);
        PB::template run_multi<BR>(xw, taps, ys);
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int rd = 0; rd < BR; ++rd) {
            const int q = sp.qb0 + static_cast<int>(lane) + 64 * rd;
            if (q < sp.qb1) {
                const int mb = static_cast<int>(A.m_star) + LR * q;
                float2 r = phasor(phi_stf + static_cast<double>(mb - n_stf) * S.inc1);
#pragma unroll
                for (int k = 0; k < LR; ++k) {
                    const uint32_t idx = static_cast<uint32_t>(mb + k - sp.m0);
                    if (idx < Nd) R[idx] = cmul(ys[rd][k], r);
                    r = cmul(r, step1);
                }
            }
        }
        __builtin_amdgcn_wave_barrier();
        // table path: twiddles from LDS (rx_fft_bins reads them through A.tw)
        rx_front_args B = A;
        B.tw = twl;
        rx_fft_bins(B, S, R, lane, [&](uint32_t k, float2 v) {
            Yrow[k] = v;
            if (drs) R[k] = v;
        });
        if (drs) {
            __builtin_amdgcn_wave_barrier();
            rx_drs_partials(A, pkt, a, l, so, R, lane);
        }
    }
}

// The compile-time-tap path with SPW consecutive symbols of one (packet, antenna) per wave, one after
// the other in the same LDS region: the per-wave start (packet tables, sync state, lane twiddles)
// is paid once per SPW symbols
#ifndef DNRP_RX_SPW
#define DNRP_RX_SPW 2
#endif
template <int SPW, bool YNT = true>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(4))) rx_fft_wave_ct_kernel(rx_front_args A) {
    extern __shared__ __attribute__((aligned(16))) float2 smem[];
    constexpr int LR = 9, MR = 10, HLR = 24;
    const uint32_t nblk = (A.sym_count + SPW - 1) / SPW;
    const uint32_t blk = blockIdx.x % nblk;
    const uint32_t a = (blockIdx.x / nblk) % A.N_RX;
    const uint32_t pkt = rx_slot_of(A.sel, blockIdx.x / (nblk * A.N_RX));
    const uint32_t lane0 = threadIdx.x & 63u;
    float2* R = smem;
    const rx_pkt_in in = A.pin[pkt];
    const rx_pkt_state S = A.st[pkt];
    const int64_t q_hi = static_cast<int64_t>(A.S_in) - in.fine_peak, q_lo = in.fine_peak < 0 ? -in.fine_peak : 0;
    const float2* src = A.iq + (size_t(in.win) * A.N_RX + a) * A.S_in + in.fine_peak;
    const float2 w1_ = wfft_tw<-1>(A.tw, 4 * (lane0 & 15u)), wl_ = wfft_tw<-1>(A.tw, lane0);
    const bool to_y = !experiment(XS_FE_SKIP_STORE) && !A.no_y;
#pragma unroll 1
    for (int i = 0; i < SPW; ++i) {
        const uint32_t li = blk * SPW + i;
        if (li >= A.sym_count) break;
        // lane index and twiddles opaque per symbol: lane-derived addresses are recomputed in the loop
        // instead of being hoisted out of it (loop-invariant code motion would spill them)
        uint32_t lane = threadIdx.x & 63u;
        float2 w1 = w1_, wl = wl_;
        asm volatile("" : "+v"(lane), "+v"(w1.x), "+v"(w1.y), "+v"(wl.x), "+v"(wl.y));
        const uint32_t l = A.sym_list ? A.sym_list[li] : A.sym_first + li;
        uint32_t so = 0xFFFFu;
        if (A.snr_part && l < A.n_sym_op) {
            const auto* sop = reinterpret_cast<const __attribute__((address_space(4))) uint32_t*>(reinterpret_cast<uintptr_t>(A.sym_op));
            so = (sop[l >> 1] >> (16 * (l & 1u))) & 0xFFFFu;
        }
        const rx_span_t sp = rx_span<LR, MR, HLR>(A, l);
        if (i) __builtin_amdgcn_wave_barrier();  // the previous symbol's reads of R are done
        if constexpr (!experiment(XS_FE_SKIP_LOAD)) {
            if (sp.in0 >= q_lo && sp.in0 + sp.n_in < q_hi)  // the span and one sample past it inside the window
                stage_span_x2<10>(R, src, sp.in0, sp.n_in, lane);
            else
                stage_span_lo<20>(R, src, sp.in0, sp.n_in, q_lo, q_hi, lane, 64);
        }
        __builtin_amdgcn_wave_barrier();
        // the next symbol's span into the caches while this one is computed: one dword per 128-B line
        // (two lines per lane), issued after this span's loads have landed and consumed at the end of
        // the symbol, so no wait of this symbol is on them; the next symbol's span loads then hit L2 /
        // the Infinity Cache instead of HBM
        float pf0 = 0.f, pf1 = 0.f;
        if (experiment(XS_FE_PREFETCH) && i + 1 < SPW && li + 1 < A.sym_count) {
            const rx_span_t sn = rx_span<LR, MR, HLR>(A, A.sym_list ? A.sym_list[li + 1] : l + 1);
            const int64_t lo = max<int64_t>(sn.in0, q_lo), hi = min<int64_t>(sn.in0 + sn.n_in, q_hi) - 1;
            if (hi >= lo) {
                const float* f = reinterpret_cast<const float*>(src);
                pf0 = f[2 * min<int64_t>(lo + 16 * lane, hi)];
                pf1 = f[2 * min<int64_t>(lo + 16 * (lane + 64), hi)];
            }
        }
        float2* Yrow = A.Y + ((size_t(pkt) * A.N_RX + a) * A.n_sym_total + l) * A.Nf_pad;
        const bool drs = so != 0xFFFFu;
        if constexpr (!experiment(XS_FE_SKIP_FIR)) rx_resample_ct<LR, MR, HLR>(A, in, S, sp, R, lane);
        rx_fft_bins<true>(A, S, R, lane, [&](uint32_t k, float2 v) {
            // Y is written once and read by the next launch: nontemporal stores when that launch
            // comes after the whole batch, plain ones when it follows within a cache-sized group
            typedef float f2v __attribute__((ext_vector_type(2)));
            if constexpr (YNT) {
                if (to_y) __builtin_nontemporal_store(f2v{v.x, v.y}, reinterpret_cast<f2v*>(Yrow + k));
            } else {
                if (to_y) Yrow[k] = v;
            }
            if (drs) R[k] = v;
        }, w1, wl);
        if (drs) {
            __builtin_amdgcn_wave_barrier();
            rx_drs_partials(A, pkt, a, l, so, R, lane);
        }
        asm volatile("" ::"v"(pf0), "v"(pf1));  // the prefetch's only consumer
    }
}

bool rx_stream_taps_match(const float* h, size_t n) {  // run-time RX taps == compiled-in taps, bitwise
    if (n != static_cast<size_t>(taps_rx_9_10::N)) return false;
    for (size_t i = 0; i < n; ++i)
        if (__builtin_bit_cast(uint32_t, h[i]) != __builtin_bit_cast(uint32_t, taps_rx_9_10::h[i])) return false;
    return true;
}

bool rx_fft_wave_path(const rx_front_args& a) {
    return a.plan.N == 1024 && a.L == 9 && a.M == 10 && a.hl == 24 && a.sym_per_block == RXW_SYMS;
}

// LDS bytes of rx_fft_kernel for a pass size and twiddle placement
static size_t rx_fft_lds(const rx_front_args& a, uint32_t pass, bool tw_lds) {
    const uint32_t Nd = a.plan.N, Nf = a.N_occ + 1;
    const bool blocked = a.L == 9 && a.M == 10 && (a.hl == 24 || a.hl == 4);
    const uint32_t in_cap = blocked ? rx_in_cap(Nd, a.CP, a.L, a.M, a.hl == 24 ? pp_block<9, 10, 24>::W : pp_block<9, 10, 4>::W, pass)
                                    : (Nd * a.M) / a.L + a.hl + 4;
    const size_t taps = blocked ? size_t(a.npp) * sizeof(float) : size_t(a.hl + 1) * a.L * sizeof(float);
    return (size_t(pass) * Nd + std::max(pass * Nd, in_cap) + Nf + (tw_lds ? Nd : 0u)) * sizeof(float2) + taps;
}

// the generic front end's layout: two symbols per pass with LDS twiddles where they fit, else one
// symbol and / or twiddles through the L1; false: no layout fits the 160 KiB
static bool rx_fft_layout(rx_front_args& a) {
    for (uint32_t pass = RX_SYM_PASS; pass >= 1; --pass)
        for (int tw = 1; tw >= 0; --tw)
            if (rx_fft_lds(a, pass, tw) <= 160 * 1024) {
                a.fft_pass = pass;
                a.fft_tw_lds = static_cast<uint32_t>(tw);
                return true;
            }
    return false;
}

hipError_t launch_rx_fft(const rx_front_args& a_in, uint32_t n, hipStream_t st) {
    rx_front_args a = a_in;
    const uint32_t Nd = a.plan.N;
    const uint32_t nblk = (a.sym_count + a.sym_per_block - 1) / a.sym_per_block;
    const dim3 g(n * a.N_RX * nblk), b(RX_THREADS);
    const bool generic = !rx_fft_wave_path(a);
    if (generic && !rx_fft_layout(a)) return hipErrorInvalidValue;
    auto fast = [&](auto kern) { hipLaunchKernelGGL(kern, g, b, rx_fft_lds(a, a.fft_pass, a.fft_tw_lds), st, a); };
    if (rx_fft_wave_path(a)) {  // os_min 1
        const uint32_t W = pp_block<9, 10, 24>::W;
        if (a.stream) {  // host: run-time taps == compiled-in taps bit for bit
            // one wave per workgroup: each wave's LDS region is freed when it retires instead of with
            // its slowest sibling (A/B on MI355X: 179.4k vs 176.4k slot-pairs/s for 4 waves per
            // workgroup); the FFT with two lane twiddles loaded with the staging (wave_fft1024_rt)
            // instead of 27 inside its passes: 92 instead of 99 VGPRs (17 waves per CU, the LDS limit,
            // not 16) and no twiddle-load latency in the passes (PDC launch 5.44 -> 5.30 ms per C4
            // chunk, same box)
            const size_t lds1 = size_t(rxw_region(9, 10, W)) * sizeof(float2);
            const dim3 gs(n * a.N_RX * ((a.sym_count + DNRP_RX_SPW - 1) / DNRP_RX_SPW));
            if (DNRP_RX_SPW > 1 && a.y_plain)
                hipLaunchKernelGGL((rx_fft_wave_ct_kernel<DNRP_RX_SPW, false>), gs, dim3(64), lds1, st, a);
            else if (DNRP_RX_SPW > 1)
                hipLaunchKernelGGL((rx_fft_wave_ct_kernel<DNRP_RX_SPW>), gs, dim3(64), lds1, st, a);
            else
                hipLaunchKernelGGL((rx_fft_wave_kernel<9, 10, 24, true, 1, true>), dim3(n * a.N_RX * a.sym_count), dim3(64),
                                   lds1, st, a);
        } else {
            const size_t lds = (Nd + (a.npp + 1) / 2 + RXW_SYMS * size_t(rxw_region(9, 10, W))) * sizeof(float2);
            hipLaunchKernelGGL((rx_fft_wave_kernel<9, 10, 24, false>), g, b, lds, st, a);
        }
    } else if (a.L == 9 && a.M == 10 && a.hl == 24)  // os_min 1 (225 taps)
        fast(rx_fft_kernel<9, 10, 24>);
    else if (a.L == 9 && a.M == 10 && a.hl == 4)  // os_min 2
        fast(rx_fft_kernel<9, 10, 4>);
    else
        fast(rx_fft_kernel<0, 0, 0>);
    return hipGetLastError();
}

}  // namespace dnrp::dev
