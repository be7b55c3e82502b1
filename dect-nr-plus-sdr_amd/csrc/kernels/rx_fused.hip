// Fused PDC receiver for N_b_DFT_os = 1024 with the compiled-in 9/10 resampler (the bench geometries
// C3/C4): rx_synced_t::demoddecod_rx_pdc's per-symbol work (rx_synced.cpp:711-771 front end,
// 893-949 Wiener interpolation, 1204-1306 MRC, 1335-1392 SFBC, pdc_enc.cpp:339-344 demap +
// descramble) in one launch without the frequency-domain grid Y in HBM.
//
// Before it, the DRS symbols of the phase go through the front end (rx_fft_wave_kernel on a symbol
// list), which leaves the zero-forced DRS pilots in zd and the SNR partial sums; rx_snr_kernel picks
// the Wiener LUT profiles. Then one workgroup per (packet, PDC symbol), one wavefront per RX antenna:
//   * wave a stages its antenna's hw-rate span, resamples + mixes it, runs wave_fft1024 and keeps the
//     amplitude-scaled, STO-derotated bins in its LDS region (symbols whose bins a preceding launch
//     already holds in Y -- the PCC phase's symbols, DRS symbols carrying PDC cells -- are loaded);
//   * the workgroup then takes the symbol's work units (cells for MRC, SFBC pairs for transmit
//     diversity): the received cells of every antenna from LDS, the Wiener channel from the epoch's
//     pilots in zd (read through the XCD's L2: all symbols of a packet run on one XCD), combining,
//     int16 demapping, descrambling and the LLR stores -- eq_compute's arithmetic (rx_eq.hpp) with the
//     pilot buffer addressed in place instead of staged.
#include "device_common.hpp"
#include "experiments.hpp"
#include "kernels.hpp"
#include "polyphase.hpp"
#include "rx_eq.hpp"
#include "rx_front.hpp"
#include "taps_gen.hpp"

namespace dnrp::dev {

namespace {
constexpr int FL = 9, FM = 10, FHL = 24;  // compiled-in RX resampler (taps_rx_9_10)

__host__ __device__ inline uint32_t fused_region() { return rxw_region(FL, FM, pp_block<FL, FM, FHL>::W); }

// Pilot access of one transmit stream of a unit: the interlaced pilot p (channel_antenna.hpp:38-63
// layout: DRS cell p >> 1 of the op in interlace slot p & 1) of antenna a is
// zp[a * ast + row[p & 1] + min(p >> 1, nd - 1)]; an op-less slot points at the zero op.
struct pilot_rows {
    uint32_t r0, r1;  // selected per tap, never indexed (a runtime index puts the pair in scratch)
};
}  // namespace

// a work unit's tables: the cell index, its subcarriers and SFBC streams (recomputed: cheap), the LUT
// pilot | weight words of its streams at those subcarriers and its scrambling bits (loaded; for the
// first units of a thread before the front end, so that they arrive during it)
template <int NT>
struct fused_unit {
    uint32_t jj, k0, k1, tab;
};
// the loaded part of a unit: scrambling bits, and either its LUT words (pw, the general path) or, for
// an SFBC pair of a full symbol with a 4-tap union window (rx_lut::pair_w), per stream the window's
// first pilot (v[0..1]; its mean weights are loaded with the pilots)
template <int NT>
struct fused_pre {
    static constexpr int NV = NT == 1 ? 1 : 4;
    uint32_t bits, v[NV];
};

// FIR taps of the Wiener interpolation handled per chunk: every pilot and weight load of a chunk is
// issued before its FMAs (one memory round trip per chunk; nI + shift <= 4 at the high-SNR profile)
constexpr uint32_t FUSED_TAPS = 2;

template <int NRX, int NT>
__global__ void __launch_bounds__(64 * NRX) __attribute__((amdgpu_waves_per_eu(NRX <= 4 ? 4 : 2))) rx_fused_kernel(rx_fused_args A) {
    extern __shared__ __attribute__((aligned(16))) float2 smem[];
    const rx_front_args& F = A.F;
    // XCD-aware: workgroup b runs on XCD b % 8; the symbols of one packet are consecutive
    // workgroups of one XCD (b / 8 = packet-of-XCD * n_fsym + symbol), so its pilots stay in that L2
    const uint32_t xs = blockIdx.x >> 3;
    const uint32_t pl = (xs / A.n_fsym) * 8 + (blockIdx.x & 7u), fs = xs % A.n_fsym;
    if (pl >= A.n_pkt) return;
    const uint32_t pkt = rx_slot_of(F.sel, pl), row = rx_row_of(F.sel, pl);
    const uint32_t a = threadIdx.x >> 6, lane = threadIdx.x & 63u, tid = threadIdx.x;
    constexpr uint32_t NTH = 64 * NRX;
    constexpr uint32_t per_unit = NT == 1 ? 1u : 2u;
    // units per thread whose tables are prefetched: C4 (4 antennas, 448 SFBC pairs per symbol) 2
    constexpr int UPT = NT == 1 ? (NRX >= 4 ? 4 : 2) : 2;
    const uint32_t region = fused_region(), Nf = F.N_occ + 1;
    const rx_fsym* fsp = A.fsym + fs;
    const uint32_t l = fsp->l, j0 = fsp->j0, j1 = fsp->j1, info = fsp->info;
    const uint32_t mode = info & 1u, swap = (info >> 1) & 3u, off = (info >> 4) & 0xFFu;
    const uint32_t units = (j1 - j0) / per_unit;
    const uint32_t prof = A.lut_d[size_t(pkt) * RX_MAX_DOPS + fsp->drs_cnt - 1];
    const rx_lut LT = A.luts[mode * 3 + prof];
    const uint32_t* __restrict__ pwr = LT.pw + size_t(fsp->rel) * 4 * Nf;
    const uint8_t* __restrict__ seq = A.pdc_seq[row];
    const uint32_t N_bps = A.N_bps, half = F.N_occ / 2;
    // ---- unit tables: indices recomputed, LUT words and scrambling bits loaded
    auto unit_index = [&](uint32_t u, fused_unit<NT>& q) {
        q.jj = j0 + per_unit * u;
        if ((info >> 13) & 1u) {  // every occupied subcarrier but DC, in order (host-checked)
            const uint32_t c = q.jj - j0;
            q.k0 = c + (c >= half ? 1u : 0u);
            q.k1 = c + 1 + (c + 1 >= half ? 1u : 0u);
        } else {
            q.k0 = A.kk[q.jj];
            q.k1 = per_unit == 2 ? A.kk[q.jj + 1] : q.k0;
        }
        if constexpr (NT == 1) {
            q.tab = 0;
        } else {
            // the SFBC pair table packed 8 bits per entry (a runtime index into the kernel-argument array
            // would copy it to scratch)
            q.tab = static_cast<uint32_t>(A.pair_bits >> (8 * ((q.jj >> 1) % A.mod))) & 0xFFu;
        }
    };
    // SFBC pairs of a full symbol from the precomputed union windows (host: every window <= 4 taps)
    const bool pairtab = NT > 1 && ((info >> 13) & 1u) && LT.pair_w != nullptr;
    const size_t prow = size_t(fsp->rel) * 4 * half;
    auto unit_load = [&](const fused_unit<NT>& q, fused_pre<NT>& p) {
        const uint32_t b0 = (q.jj * N_bps) >> 3, bl = ((q.jj + per_unit) * N_bps - 1) >> 3;
        p.bits = seq[b0] | (b0 + 1 <= bl ? uint32_t(seq[b0 + 1]) << 8 : 0u) | (b0 + 2 <= bl ? uint32_t(seq[b0 + 2]) << 16 : 0u);
        if constexpr (NT == 1) {
            p.v[0] = pwr[swap * Nf + q.k0];
        } else {
            const uint32_t tA = q.tab & 0xFu, tB = q.tab >> 4;
            if (pairtab) {
                const uint32_t u = (q.jj - j0) >> 1;
#pragma unroll
                for (int st = 0; st < 2; ++st)
                    p.v[st] = LT.pair_p[prow + size_t(((st == 0 ? tA : tB) & 3u) ^ swap) * half + u];
            } else {
                p.v[0] = pwr[((tA & 3u) ^ swap) * Nf + q.k0];
                p.v[1] = pwr[((tA & 3u) ^ swap) * Nf + q.k1];
                p.v[2] = pwr[((tB & 3u) ^ swap) * Nf + q.k0];
                p.v[3] = pwr[((tB & 3u) ^ swap) * Nf + q.k1];
            }
        }
    };
    fused_pre<NT> P[UPT];  // the first UPT units of this thread, in flight during the front end
#pragma unroll
    for (int g = 0; g < UPT; ++g) {
        fused_unit<NT> q;
        unit_index(min(tid + g * NTH, units - 1), q);
        unit_load(q, P[g]);
    }
    // ---- front end: this wave's antenna into its LDS region
    float2* R = smem + a * region;
    if (experiment(XS_FUSED_SKIP_FE)) {
        for (uint32_t k = lane; k < Nf; k += 64) R[k] = make_float2(1.f, 0.f);
    } else if ((info >> 12) & 1u) {  // bins already in Y (PCC-phase symbol, or a DRS symbol of this phase)
        const float2* Yrow = F.Y + ((size_t(pkt) * NRX + a) * F.n_sym_total + l) * F.Nf_pad;
        stage_copy<8>(R, Yrow, Nf, lane, 64);
    } else {
        const rx_pkt_in in = F.pin[pkt];
        const rx_pkt_state S = F.st[pkt];
        const rx_span_t sp = rx_span<FL, FM, FHL>(F, l);
        // valid input window relative to the fine peak: history is zero before it (rx_synced.cpp:711-740)
        const int64_t q_hi = static_cast<int64_t>(F.S_in) - in.fine_peak, q_lo = in.fine_peak < 0 ? -in.fine_peak : 0;
        const float2* src = F.iq + (size_t(in.win) * NRX + a) * F.S_in + in.fine_peak;
        const float2 w1 = wfft_tw<-1>(F.tw, 4 * (lane & 15u)), wl = wfft_tw<-1>(F.tw, lane);
        stage_span_lo<20>(R, src, sp.in0, sp.n_in, q_lo, q_hi, lane, 64);
        __builtin_amdgcn_wave_barrier();
        rx_resample_ct<FL, FM, FHL>(F, in, S, sp, R, lane);
        rx_fft_bins<true>(F, S, R, lane, [&](uint32_t k, float2 v) { R[k] = v; }, w1, wl);
    }
    __syncthreads();

    // ---- equalisation of the symbol's units (workgroup-uniform event: LUT mode / row / profile)
    const float* __restrict__ wt = LT.w;
    const uint32_t nI = LT.n, step = mode ? 1u : 2u, nd = F.n_drs, np2 = 2 * nd;
    const size_t ast = size_t(4) * F.zd_row;  // antenna stride in zd
    const float2* __restrict__ zp = F.zd + size_t(pkt) * F.zd_dops * NRX * ast;
    // epoch pilot sources packed 8 bits per stream (uniform; op zd_dops - 1 is the zero op): per lane
    // the rows come from shifts -- a runtime index into a small array (or a select chain the compiler
    // folds into one) would put it in scratch and reload it per tap
    uint64_t dpk[2] = {0, 0};
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int o = 0; o < 2; ++o) {
            const uint32_t d = fsp->src[t][o];
            dpk[o] |= uint64_t(d == 0xFFFFu ? F.zd_dops - 1 : d) << (8 * t);
        }
    auto rows_of = [&](uint32_t t) {
        pilot_rows pr;
        pr.r0 = ((static_cast<uint32_t>(dpk[0] >> (8 * t)) & 0xFFu) * NRX * 4 + t) * F.zd_row;
        pr.r1 = ((static_cast<uint32_t>(dpk[1] >> (8 * t)) & 0xFFu) * NRX * 4 + t) * F.zd_row;
        return pr;
    };
    auto pilot = [&](const pilot_rows& pr, uint32_t p, int ant) {
        const uint32_t r = pr.r0 + ((0u - (p & 1u)) & (pr.r1 - pr.r0));  // slot p & 1, arithmetically
        return zp[ant * ast + r + min(p >> 1, nd - 1)];
    };
    int16_t* __restrict__ llr = A.llr + size_t(row) * A.llr_stride;
    // SFBC pair combining (rx_synced.cpp:1373-1391) of the pair's channels g[rx][stream], demap, store
    auto sfbc_emit = [&](const fused_unit<NT>& q, const fused_pre<NT>& pre, const float2 (&g)[NRX][2]) {
        float2 n0 = make_float2(0.f, 0.f), n1 = make_float2(0.f, 0.f);
        float den = 0.f;
#pragma unroll
        for (int r = 0; r < NRX; ++r) {
            const float2 h0 = g[r][0], h1 = g[r][1];
            const float2 r0 = smem[r * region + q.k0], r1 = smem[r * region + q.k1];
            n0 = cadd(n0, cadd(cmul(cconj(h0), r0), cmul(h1, cconj(r1))));
            n1 = cadd(n1, cadd(cmul(make_float2(-h1.x, -h1.y), cconj(r0)), cmul(cconj(h0), r1)));
            den += cnorm(h0) + cnorm(h1);
        }
        emit_cell(cscale(n0, 1.0f / den), q.jj, q.jj, N_bps, pre.bits, llr);
        emit_cell(cscale(n1, 1.0f / den), q.jj + 1, q.jj, N_bps, pre.bits, llr);
    };
    auto equalise = [&](const fused_unit<NT>& q, const fused_pre<NT>& pre) {
        if constexpr (NT == 1) {
            uint32_t p = pre.v[0] & 0xFFFFu;
            if (!mode) p = 2 * p + (off & 1u);  // non-interlaced: latest DRS symbol only
            const uint32_t wo = (pre.v[0] >> 16) * nI;
            const pilot_rows pr = rows_of(0);
            float2 h[NRX];
#pragma unroll
            for (int r = 0; r < NRX; ++r) h[r] = make_float2(0.f, 0.f);
            for (uint32_t i0 = 0; i0 < nI; i0 += FUSED_TAPS) {
                float wv[FUSED_TAPS];
                float2 z[FUSED_TAPS][NRX];
#pragma unroll
                for (uint32_t c = 0; c < FUSED_TAPS; ++c) {
                    const uint32_t i = i0 + c, pi = p + i * step;
                    wv[c] = i < nI && pi < np2 ? wt[wo + min(i, nI - 1)] : 0.f;
#pragma unroll
                    for (int r = 0; r < NRX; ++r) z[c][r] = pilot(pr, pi, r);
                }
#pragma unroll
                for (uint32_t c = 0; c < FUSED_TAPS; ++c)
#pragma unroll
                    for (int r = 0; r < NRX; ++r) {
                        h[r].x = fmaf(z[c][r].x, wv[c], h[r].x);
                        h[r].y = fmaf(z[c][r].y, wv[c], h[r].y);
                    }
            }
            float2 num = make_float2(0.f, 0.f);
            float den = 0.f;
#pragma unroll
            for (int r = 0; r < NRX; ++r) {  // MRC (rx_synced.cpp:1204-1306)
                const float2 r0 = smem[r * region + q.k0];
                num = cadd(num, cmulc(r0, h[r]));
                den += cnorm(h[r]);
            }
            emit_cell(cscale(num, 1.0f / den), q.jj, q.jj, N_bps, pre.bits, llr);
        } else if (pairtab) {
            // the pair's union windows precomputed: 4 taps per stream, one pass (eq_compute's sums)
            const uint32_t tA = q.tab & 0xFu, tB = q.tab >> 4;
            uint32_t base[2];
            pilot_rows pr[2];
            float4 w4[2];
            const uint32_t u = (q.jj - j0) >> 1;
#pragma unroll
            for (int st = 0; st < 2; ++st) {
                const uint32_t t = st == 0 ? tA : tB;
                base[st] = mode ? pre.v[st] : 2 * pre.v[st] + ((off >> t) & 1u);
                pr[st] = rows_of(t);
                w4[st] = LT.pair_w[prow + size_t((t & 3u) ^ swap) * half + u];
            }
            float2 g[NRX][2];
            float2 z[4][2][NRX];
#pragma unroll
            for (uint32_t c = 0; c < 4; ++c)
#pragma unroll
                for (int st = 0; st < 2; ++st)
#pragma unroll
                    for (int r = 0; r < NRX; ++r) z[c][st][r] = pilot(pr[st], base[st] + c * step, r);
#pragma unroll
            for (int r = 0; r < NRX; ++r) g[r][0] = g[r][1] = make_float2(0.f, 0.f);
#pragma unroll
            for (uint32_t c = 0; c < 4; ++c)
#pragma unroll
                for (int st = 0; st < 2; ++st) {
                    const uint32_t p = base[st] + c * step;
                    // past the pilot row: weight 0 (eq_compute's zero pad)
                    const float wc = c == 0 ? w4[st].x : c == 1 ? w4[st].y : c == 2 ? w4[st].z : w4[st].w;
                    const float wv = p < np2 ? wc : 0.f;
#pragma unroll
                    for (int r = 0; r < NRX; ++r) {
                        g[r][st].x = fmaf(z[c][st][r].x, wv, g[r][st].x);
                        g[r][st].y = fmaf(z[c][st][r].y, wv, g[r][st].y);
                    }
                }
            sfbc_emit(q, pre, g);
        } else {
            const uint32_t tA = q.tab & 0xFu, tB = q.tab >> 4;
            uint32_t pos[4], wo[4];
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                const uint32_t t = c < 2 ? tA : tB;
                uint32_t p = pre.v[c] & 0xFFFFu;
                if (!mode) p = 2 * p + ((off >> t) & 1u);
                pos[c] = p;
                wo[c] = (pre.v[c] >> 16) * nI;
            }
            // SFBC: a stream's pair channel is the mean of its interpolations at k0 and k1
            // (rx_synced.cpp:1365-1371), one pass over the union window with the mean weights (eq_compute)
            uint32_t base[2], sh[2], wlo[2], whi[2];
            pilot_rows pr[2];
#pragma unroll
            for (int s = 0; s < 2; ++s) {
                const bool up = pos[2 * s + 1] >= pos[2 * s];
                base[s] = up ? pos[2 * s] : pos[2 * s + 1];
                sh[s] = (up ? pos[2 * s + 1] - pos[2 * s] : pos[2 * s] - pos[2 * s + 1]) / step;
                wlo[s] = up ? wo[2 * s] : wo[2 * s + 1];
                whi[s] = up ? wo[2 * s + 1] : wo[2 * s];
                pr[s] = rows_of(s == 0 ? tA : tB);
            }
            const uint32_t ntap = nI + max(sh[0], sh[1]);
            float2 g[NRX][2];
#pragma unroll
            for (int r = 0; r < NRX; ++r) g[r][0] = g[r][1] = make_float2(0.f, 0.f);
            for (uint32_t i0 = 0; i0 < ntap; i0 += FUSED_TAPS) {
                float wv[FUSED_TAPS][2];
                float2 z[FUSED_TAPS][2][NRX];
#pragma unroll
                for (uint32_t c = 0; c < FUSED_TAPS; ++c)
#pragma unroll
                    for (int s = 0; s < 2; ++s) {
                        const uint32_t i = i0 + c;
                        const bool il = i < nI, ih = i >= sh[s] && i - sh[s] < nI;
                        const float lo = il ? wt[wlo[s] + i] : 0.f;
                        const float hi = ih ? wt[whi[s] + i - sh[s]] : 0.f;
                        const uint32_t p = base[s] + min(i, nI + sh[s]) * step;
                        // past the stream's union window, or past the pilot row (eq_compute's zero pad)
                        wv[c][s] = p < np2 ? 0.5f * (lo + hi) : 0.f;
#pragma unroll
                        for (int r = 0; r < NRX; ++r) z[c][s][r] = pilot(pr[s], p, r);
                    }
#pragma unroll
                for (uint32_t c = 0; c < FUSED_TAPS; ++c)
#pragma unroll
                    for (int s = 0; s < 2; ++s)
#pragma unroll
                        for (int r = 0; r < NRX; ++r) {
                            g[r][s].x = fmaf(z[c][s][r].x, wv[c][s], g[r][s].x);
                            g[r][s].y = fmaf(z[c][s][r].y, wv[c][s], g[r][s].y);
                        }
            }
            sfbc_emit(q, pre, g);
        }
    };
    if constexpr (experiment(XS_FUSED_SKIP_EQ)) {
#pragma unroll
        for (int g = 0; g < UPT; ++g)
            if (tid + g * NTH < units) llr[(j0 + per_unit * (tid + g * NTH)) * N_bps] = static_cast<int16_t>(P[g].bits + smem[tid].x);
        return;
    }
#pragma unroll
    for (int g = 0; g < UPT; ++g)
        if (tid + g * NTH < units) {
            fused_unit<NT> q;
            unit_index(tid + g * NTH, q);
            equalise(q, P[g]);
        }
    // units past the prefetched ones (narrow workgroups, long symbols): tables loaded here
    for (uint32_t u = tid + UPT * NTH; u < units; u += NTH) {
        fused_unit<NT> q;
        unit_index(u, q);
        fused_pre<NT> p;
        unit_load(q, p);
        equalise(q, p);
    }
}

bool rx_fused_supported(uint32_t N_RX, uint32_t NT) {
    return (N_RX == 1 || N_RX == 2 || N_RX == 4 || N_RX == 8) && (NT == 1 || NT == 2 || NT == 4) && NT <= N_RX;
}

hipError_t launch_rx_fused(const rx_fused_args& a, hipStream_t st) {
    if (!rx_fused_supported(a.F.N_RX, a.NT) || !rx_fft_wave_path(a.F) || !a.F.stream || !a.F.zd || a.n_fsym == 0)
        return hipErrorInvalidValue;
    const dim3 g((a.n_pkt + 7) / 8 * 8 * a.n_fsym), b(64 * a.F.N_RX);
    const size_t lds = size_t(a.F.N_RX) * fused_region() * sizeof(float2);
#define DNRP_FUSED(R, T)                                                   \
    if (a.F.N_RX == R && a.NT == T) {                                      \
        hipLaunchKernelGGL((rx_fused_kernel<R, T>), g, b, lds, st, a);     \
        return hipGetLastError();                                          \
    }
    DNRP_FUSED(1, 1)
    DNRP_FUSED(2, 1)
    DNRP_FUSED(4, 1)
    DNRP_FUSED(8, 1)
    DNRP_FUSED(2, 2)
    DNRP_FUSED(4, 2)
    DNRP_FUSED(8, 2)
    DNRP_FUSED(4, 4)
    DNRP_FUSED(8, 4)
#undef DNRP_FUSED
    return hipErrorInvalidValue;
}

}  // namespace dnrp::dev
