// Per-cell back end of the synchronised receiver (rx_cells_kernel, rx_back.hip): Wiener interpolation
// of the channel from the interlaced pilot buffer (rx_synced.cpp:893-949), MRC (1204-1306) or SFBC
// combining (1335-1392), srsRAN-style int16 soft demapping and descrambling (pcc_enc.cpp:297,
// pdc_enc.cpp:339-344).
#pragma once

#include "device_common.hpp"
#include "experiments.hpp"
#include "kernels.hpp"

namespace dnrp::dev {

#ifndef DNRP_CELLS_CH
#define DNRP_CELLS_CH 3  // SFBC interpolation taps per chunk (eq_compute): 3 keeps rx_cells<4, 4> at 121 VGPRs (4: 131, one workgroup per CU)
#endif

// the pilot-buffer layout of rx_cells_kernel<NRX, NT, SM>: antenna pairs interleaved for the MMSE
// path and for SFBC with an even antenna count (build_pilots)
__host__ __device__ constexpr bool cells_ai(int NRX, int NT) { return NT > 1 && NRX % 2 == 0; }

__device__ __forceinline__ int16_t q16(float v) {
    const float r = rintf(v);
    return static_cast<int16_t>(fminf(32767.f, fmaxf(-32768.f, r)));
}

// two LLRs, each sign-flipped by the top bit of its scrambling word (a sign XOR before the int16
// rounding: q16 clamps asymmetrically, so it must see the flipped value), as one int16 pair: the
// saturating v_cvt_pk_i16_i32 packs them (no-op saturation, the values are clamped already)
__device__ __forceinline__ uint32_t q16_pair(float a, uint32_t fa, float b, uint32_t fb) {
    auto q = [](float v, uint32_t f) {
        const float x = __uint_as_float(__float_as_uint(v) ^ (f & 0x80000000u));
        return static_cast<int>(fminf(32767.f, fmaxf(-32768.f, rintf(x))));
    };
    const auto pk = __builtin_amdgcn_cvt_pk_i16(q(a, fa), q(b, fb));
    return static_cast<uint16_t>(pk[0]) | static_cast<uint32_t>(static_cast<uint16_t>(pk[1])) << 16;
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

// Unit pipeline (one unit: cell jj for MRC, NT == 1, or the SFBC pair jj, jj+1): stage A resolves the
// segment (LDS) and loads the subcarrier indices and symbol; stage B loads the LUT pilot | weight
// words, the received cells of every RX antenna and the unit's scrambling bits; eq_compute works from
// registers and LDS only. The kernel keeps stage A two units ahead and stage B one unit ahead.
struct unit_a {
    uint32_t si, jj, k0, k1, l;
};
template <int NRX, int NT>
struct unit_b {
    static constexpr int NC = NT == 1 ? 1 : 4;  // interpolated channels per unit
    uint32_t si, jj, tab;                       // tab: tA | tB << 4
    uint32_t pw[NC];
    uint32_t sb[3];                             // scrambling bytes from bit (jj N_bps) & ~7 (raw loads)
    float2 r0[NRX], r1[NT == 1 ? 1 : NRX];
};

__device__ __forceinline__ void unit_stage_a(const rx_cells_args& A, const cell_seg* sg, uint32_t nseg, uint32_t& si,
                                             uint32_t u, uint32_t per_unit, unit_a& a) {
    while (si + 1 < nseg && u >= sg[si + 1].u0) ++si;
    a.si = si;
    a.jj = sg[si].j0 + per_unit * (u - sg[si].u0);
    a.k0 = A.kk[a.jj];
    a.k1 = per_unit == 2 ? A.kk[a.jj + 1] : a.k0;
    a.l = A.cell_sym[a.jj];
}

// a pointer that came through LDS or a pointer table as a global one: the loads become global_load
// instead of flat_load (a flat load also counts in lgkmcnt, so every LDS wait would wait for it)
template <class T>
__device__ __forceinline__ const __attribute__((address_space(1))) T* as_global(const T* p) {
    return reinterpret_cast<const __attribute__((address_space(1))) T*>(reinterpret_cast<uintptr_t>(p));
}

template <int NRX, int NT>
__device__ __forceinline__ void unit_stage_b(const rx_cells_args& A, const cell_seg* sg, const uint32_t* pairs,
                                             const float2* __restrict__ Yp, const uint8_t* __restrict__ seq,
                                             const unit_a& a, unit_b<NRX, NT>& b) {
    const uint32_t Nf = A.N_occ + 1;
    const cell_seg& S = sg[a.si];
    const uint32_t swap = (S.info >> 1) & 3u;
    const auto spw = as_global(S.pw);
    const auto sq = as_global(seq);
    b.si = a.si;
    b.jj = a.jj;
    if constexpr (NT == 1) {
        b.tab = 0;
        b.pw[0] = spw[swap * Nf + a.k0];
    } else {
        const uint32_t pr = pairs[(a.jj >> 1) % A.mod];
        const uint32_t tA = pr & 0xFu, tB = pr >> 4;
        b.tab = tA | tB << 4;
        b.pw[0] = spw[((tA & 3u) ^ swap) * Nf + a.k0];
        b.pw[1] = spw[((tA & 3u) ^ swap) * Nf + a.k1];
        b.pw[2] = spw[((tB & 3u) ^ swap) * Nf + a.k0];
        b.pw[3] = spw[((tB & 3u) ^ swap) * Nf + a.k1];
    }
    const size_t ast = size_t(A.n_sym_total) * A.Nf_pad;
    const uint32_t yoff = a.l * A.Nf_pad;
    if constexpr (NT > 1) {
        // the pair's two cells are neighbours except across DC: one 16-B load per antenna (8-B
        // aligned: unaligned dwordx4, k0 + 1 <= N_b_OCC < Nf_pad stays in the row), the DC pair's
        // second cell reloaded. Nontemporal, so that it stays one dwordx4: a plain load with the DC
        // reload behind it is sunk into an 8-B load plus two 4-B loads from a selected address (the
        // cells are read once; nt loads bypass only the L1)
        typedef float f4u __attribute__((ext_vector_type(4), aligned(8)));
        const bool dc = a.k1 != a.k0 + 1;
#pragma unroll
        for (int r = 0; r < NRX; ++r) {
            const f4u v = __builtin_nontemporal_load(reinterpret_cast<const f4u*>(Yp + r * ast + yoff + a.k0));
            b.r0[r] = make_float2(v.x, v.y);
            b.r1[r] = make_float2(v.z, v.w);
        }
        if (dc) {
#pragma unroll
            for (int r = 0; r < NRX; ++r) b.r1[r] = Yp[r * ast + yoff + a.k1];
        }
    } else {
#pragma unroll
        for (int r = 0; r < NRX; ++r) b.r0[r] = Yp[r * ast + yoff + a.k0];
    }
    // the unit's scrambling bits [jj N_bps, (jj + cells) N_bps) lie in at most 3 bytes
    // (loads clamped to the last byte and kept raw: nothing here waits on the loads in flight)
    const uint32_t b0 = (a.jj * A.N_bps) >> 3, bl = ((a.jj + (NT == 1 ? 1u : 2u)) * A.N_bps - 1) >> 3;
    b.sb[0] = sq[b0];
    b.sb[1] = sq[min(b0 + 1, bl)];
    b.sb[2] = sq[min(b0 + 2, bl)];
}

// demap + descramble + int16 of cell j (LLRs j*N_bps .. j*N_bps+N_bps-1); bits: the scrambling bytes
// from bit (j0 N_bps) & ~7 of the unit's first cell j0
__device__ __forceinline__ void emit_cell(float2 x, uint32_t j, uint32_t j0, uint32_t N_bps, uint32_t bits,
                                          int16_t* __restrict__ llr) {
    float L[8];
    demap(x, N_bps, L);
    const uint32_t base = j * N_bps, r0 = base - ((j0 * N_bps) & ~7u);  // bit offset in `bits`
    auto sbit = [&](uint32_t i) { const uint32_t r = r0 + i; return (bits >> (8 * (r >> 3) + 7 - (r & 7u))) & 1u; };
    if (N_bps == 8) {  // one 16-B store; the cell's scrambling byte is byte r0 / 8 of `bits`
        const uint32_t sw = (bits >> r0) << 24;  // LLR b's bit at 31 - b
        uint32_t w[4];
#pragma unroll
        for (int b = 0; b < 8; b += 2) w[b / 2] = q16_pair(L[b], sw << b, L[b + 1], sw << (b + 1));
        int16_t* dst = llr + base;
        if ((reinterpret_cast<uintptr_t>(dst) & 15u) == 0) {
            *reinterpret_cast<uint4*>(dst) = make_uint4(w[0], w[1], w[2], w[3]);
        } else {
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                dst[2 * b] = static_cast<int16_t>(w[b] & 0xFFFFu);
                dst[2 * b + 1] = static_cast<int16_t>(w[b] >> 16);
            }
        }
        return;
    }
#pragma unroll
    for (uint32_t b = 0; b < 8; ++b)
        if (b < N_bps) llr[base + b] = q16(sbit(b) ? -L[b] : L[b]);
}

// Wiener interpolation (rx_synced.cpp:893-949), MRC (1204-1306) or SFBC combining (1335-1392),
// demapping and the LLR store of one unit. zfi: the epoch's pilot rows [NRX][NT][zst]; wtab: the
// weight-table slots.
// NBPS: bits per cell fixed at compile time (8: 256-QAM, the bench's C3 / C4), 0: A.N_bps at run time
template <int NRX, int NT, int NBPS = 0>
__device__ __forceinline__ void eq_compute(const rx_cells_args& A, const cell_seg* sg, const float2* zfi,
                                           const float* wtab, uint32_t zst, const unit_b<NRX, NT>& b,
                                           int16_t* __restrict__ llr) {
    constexpr int NC = unit_b<NRX, NT>::NC;
    const uint32_t N_bps = NBPS ? static_cast<uint32_t>(NBPS) : A.N_bps;
    const uint32_t b0 = (b.jj * N_bps) >> 3, bl = ((b.jj + (NT == 1 ? 1u : 2u)) * N_bps - 1) >> 3;
    const uint32_t bits = b.sb[0] | (b0 + 1 <= bl ? b.sb[1] << 8 : 0u) | (b0 + 2 <= bl ? b.sb[2] << 16 : 0u);
    const uint32_t info = sg[b.si].info, wbase = sg[b.si].wbase;
    const uint32_t mode = info & 1u, off = (info >> 4) & 0xFFu, nI = info >> 12;
    const uint32_t step = mode ? 1u : 2u;
    // SFBC with an even antenna count reads the antenna-pair-interleaved pilot buffer (AI, see
    // build_pilots): positions in float2 of the stream's first pair row, pilot steps of 2 float2
    constexpr bool AI = cells_ai(NRX, NT);
    constexpr uint32_t PS = AI ? 2u : 1u;
    uint32_t pos[NC], wo[NC];  // pilot start (LDS float2 index) and weight offset (LDS float index)
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        const uint32_t t = c < 2 ? (b.tab & 0xFu) : (b.tab >> 4);
        uint32_t p = b.pw[c] & 0xFFFFu;
        if (!mode) p = 2 * p + ((off >> t) & 1u);  // non-interlaced: latest DRS symbol only
        if (experiment(XS_CELLS_ONE_PILOT)) p = 0;
        pos[c] = AI ? ((experiment(XS_CELLS_ONE_ROW) ? 0u : t * (NRX / 2) * zst) + p) * 2
                    : p + (experiment(XS_CELLS_ONE_ROW) ? 0u : t * zst);
        wo[c] = wbase + (experiment(XS_CELLS_ONE_WROW) ? 0u : (b.pw[c] >> 16) * nI);
    }
    if constexpr (NT == 1) {
        float2 h[NRX];
#pragma unroll
        for (int a = 0; a < NRX; ++a) h[a] = make_float2(0.f, 0.f);
        // taps in chunks of CH, the chunk's reads issued before its FMAs; taps past nI read the last
        // one with weight 0 (exact zeros: the tap-ordered sums of the one-tap loop, bit for bit)
        constexpr uint32_t CH = 4;
        for (uint32_t i0 = 0; i0 < nI; i0 += CH) {
            float wv[CH];
            float2 z[CH][NRX];
#pragma unroll
            for (uint32_t j = 0; j < CH; ++j) {
                const uint32_t i = min(i0 + j, nI - 1);
                const float w = wtab[wo[0] + i];
                wv[j] = i0 + j < nI ? w : 0.f;
#pragma unroll
                for (int a = 0; a < NRX; ++a) z[j][a] = zfi[a * NT * zst + pos[0] + i * step];
            }
#pragma unroll
            for (uint32_t j = 0; j < CH; ++j)
#pragma unroll
                for (int a = 0; a < NRX; ++a) {
                    h[a].x = fmaf(z[j][a].x, wv[j], h[a].x);
                    h[a].y = fmaf(z[j][a].y, wv[j], h[a].y);
                }
        }
        float2 num = make_float2(0.f, 0.f);
        float den = 0.f;
#pragma unroll
        for (int a = 0; a < NRX; ++a) {  // MRC (rx_synced.cpp:1204-1306)
            num = cadd(num, cmulc(b.r0[a], h[a]));
            den += cnorm(h[a]);
        }
        emit_cell(cscale(num, 1.0f / den), b.jj, b.jj, N_bps, bits, llr);
    } else {
        // SFBC: a stream's pair channel is the mean of its interpolations at k0 and k1
        // (rx_synced.cpp:1365-1371). Both read the stream's pilot row with windows sh pilots apart
        // (0 or 1 almost everywhere): one pass over the union window of nI + sh taps with the mean
        // weights gives the mean with about half the pilot reads and FMAs of two passes.
        uint32_t base[2], sh[2], wl[2], wh[2];
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            const bool up = pos[2 * s + 1] >= pos[2 * s];
            base[s] = up ? pos[2 * s] : pos[2 * s + 1];
            sh[s] = (up ? pos[2 * s + 1] - pos[2 * s] : pos[2 * s] - pos[2 * s + 1]) / (PS * step);
            wl[s] = up ? wo[2 * s] : wo[2 * s + 1];
            wh[s] = up ? wo[2 * s + 1] : wo[2 * s];
        }
        const uint32_t ntap = nI + max(sh[0], sh[1]);
        const uint32_t psh = (AI ? 1u : 0u) + (mode ? 0u : 1u);  // log2(PS * step): a shift, not v_mul_lo
        float2 g[NRX][2];
#pragma unroll
        for (int a = 0; a < NRX; ++a) g[a][0] = g[a][1] = make_float2(0.f, 0.f);
        // taps in chunks of CH, per stream every LDS read of a chunk (weights at clamped indices,
        // pilots) issued before its FMAs: one LDS latency per chunk and stream instead of per tap,
        // no exec-mask branches. Taps past a stream's union window carry weight 0 (their read stays
        // in the row + ZFI_PAD) and add exact zeros, so the per-(antenna, stream) sums are the
        // tap-ordered sums of the one-tap loop, bit for bit.
        constexpr uint32_t CH = DNRP_CELLS_CH;
        for (uint32_t i0 = 0; i0 < ntap; i0 += CH) {
#pragma unroll
            for (int s = 0; s < 2; ++s) {
                __builtin_amdgcn_sched_barrier(0);  // one stream's chunk live at a time
                float wv[CH];
                float2 z[CH][NRX];
#pragma unroll
                for (uint32_t j = 0; j < CH; ++j) {
                    const uint32_t i = i0 + j, ih = i - sh[s];  // ih wraps for i < sh
                    const float lo = wtab[wl[s] + min(i, nI - 1)], hi = wtab[wh[s] + min(ih, nI - 1)];
                    wv[j] = 0.5f * ((i < nI ? lo : 0.f) + (ih < nI ? hi : 0.f));
                    const uint32_t p = base[s] + (min(i, nI + sh[s]) << psh);
                    if constexpr (AI) {
                        typedef float f4 __attribute__((ext_vector_type(4)));
#pragma unroll
                        for (int q = 0; q < NRX / 2; ++q) {
                            const f4 v = *reinterpret_cast<const f4*>(zfi + p + q * zst * 2);
                            z[j][2 * q] = make_float2(v.x, v.y);
                            z[j][2 * q + 1] = make_float2(v.z, v.w);
                        }
                    } else {
#pragma unroll
                        for (int a = 0; a < NRX; ++a) z[j][a] = zfi[a * NT * zst + p];
                    }
                }
#pragma unroll
                for (uint32_t j = 0; j < CH; ++j)
#pragma unroll
                    for (int a = 0; a < NRX; ++a) {
                        g[a][s].x = fmaf(z[j][a].x, wv[j], g[a][s].x);
                        g[a][s].y = fmaf(z[j][a].y, wv[j], g[a][s].y);
                    }
            }
        }
        float2 n0 = make_float2(0.f, 0.f), n1 = make_float2(0.f, 0.f);
        float den = 0.f;
#pragma unroll
        for (int a = 0; a < NRX; ++a) {  // SFBC pair combining (rx_synced.cpp:1373-1391)
            const float2 h0 = g[a][0], h1 = g[a][1];
            n0 = cadd(n0, cadd(cmul(cconj(h0), b.r0[a]), cmul(h1, cconj(b.r1[a]))));
            n1 = cadd(n1, cadd(cmul(make_float2(-h1.x, -h1.y), cconj(b.r0[a])), cmul(cconj(h0), b.r1[a])));
            den += cnorm(h0) + cnorm(h1);
        }
        emit_cell(cscale(n0, 1.0f / den), b.jj, b.jj, N_bps, bits, llr);
        emit_cell(cscale(n1, 1.0f / den), b.jj + 1, b.jj, N_bps, bits, llr);
    }
}

// ===================================================================== spatial multiplexing (MMSE)
// N_SS = NT > 1 spatial streams on the NT transmit streams (tx.cpp:1051-1067: symbol s of cell j is
// spatial-stream symbol j NT + s). Not in the reference receiver (run_pdc_mode_AxA_MIMO,
// rx_synced.cpp:1331-1333, \todo): opt-in (dnrp_ctx_set_rx_mode). Per cell the Wiener-interpolated
// channel H[rx][ss] of every stream, linear MMSE x = (H^H H + nv I)^-1 H^H y with nv the SNR
// estimator's noise variance at the epoch's LUT pick, unbiased per stream by
// beta_s = 1 - nv [(H^H H + nv I)^-1]_ss, then the same demapper and descrambling as MRC / SFBC.
// The NT x NT Hermitian solve runs per lane in registers (Cholesky, L^-1): per cell it is ~NRX NT^2
// complex MACs for the Gram matrix and ~NT^3 for the solve -- a lane-per-subcarrier batch of tiny
// independent systems, which the lane layout keeps off the matrix cores (measured: the Gram matrix
// on v_mfma_f32_4x4x1_16b_f32, XS_MMSE_MFMA below, is 1.7x slower; docs/DESIGN_LOG.md §6).
template <int NRX, int NT>
struct unit_sm {
    uint32_t si, jj;
    uint32_t pw[NT];  // LUT pilot | weight words of every stream at the cell's subcarrier
    uint32_t sb[5];   // scrambling bytes from bit (jj NT N_bps) & ~7: NT N_bps <= 32 bits
    float2 r0[NRX];
};

template <int NRX, int NT>
__device__ __forceinline__ void unit_stage_b_sm(const rx_cells_args& A, const cell_seg* sg,
                                                const float2* __restrict__ Yp, const uint8_t* __restrict__ seq,
                                                const unit_a& a, unit_sm<NRX, NT>& b) {
    const uint32_t Nf = A.N_occ + 1;
    const cell_seg& S = sg[a.si];
    const uint32_t swap = (S.info >> 1) & 3u;
    b.si = a.si;
    b.jj = a.jj;
#pragma unroll
    for (int t = 0; t < NT; ++t) b.pw[t] = as_global(S.pw)[((static_cast<uint32_t>(t) & 3u) ^ swap) * Nf + a.k0];
    const size_t ast = size_t(A.n_sym_total) * A.Nf_pad;
    const uint32_t yoff = a.l * A.Nf_pad;
#pragma unroll
    for (int r = 0; r < NRX; ++r) b.r0[r] = Yp[r * ast + yoff + a.k0];
    const uint32_t b0 = (a.jj * NT * A.N_bps) >> 3, bl = ((a.jj + 1) * NT * A.N_bps - 1) >> 3;
#pragma unroll
    for (int i = 0; i < 5; ++i) b.sb[i] = as_global(seq)[min(b0 + i, bl)];
}

// demap + descramble + int16 of one symbol: LLRs base .. base + N_bps - 1; sw: the symbol's
// scrambling bits from the top (LLR k's bit at 31 - k)
__device__ __forceinline__ void emit_symw(float2 x, uint32_t base, uint32_t N_bps, uint32_t sw,
                                          int16_t* __restrict__ llr) {
    float L[8];
    demap(x, N_bps, L);
    uint32_t w[4];  // the symbol's LLRs as int16 pairs
#pragma unroll
    for (uint32_t k = 0; k < 8; k += 2) w[k / 2] = k < N_bps ? q16_pair(L[k], sw << k, L[k + 1], sw << (k + 1)) : 0u;
    // one store per symbol where the width allows (N_bps LLRs = 2 N_bps bytes at their natural
    // alignment), else per LLR
    int16_t* dst = llr + base;
    const uintptr_t ad = reinterpret_cast<uintptr_t>(dst);
    if (N_bps == 8 && (ad & 15u) == 0) {
        *reinterpret_cast<uint4*>(dst) = make_uint4(w[0], w[1], w[2], w[3]);
    } else if (N_bps == 4 && (ad & 7u) == 0) {
        *reinterpret_cast<uint2*>(dst) = make_uint2(w[0], w[1]);
    } else if ((N_bps == 6 || N_bps == 2) && (ad & 3u) == 0) {
        uint32_t* d32 = reinterpret_cast<uint32_t*>(dst);
        d32[0] = w[0];
        if (N_bps == 6) {
            d32[1] = w[1];
            d32[2] = w[2];
        }
    } else {
#pragma unroll
        for (uint32_t k = 0; k < 8; ++k)
            if (k < N_bps) dst[k] = static_cast<int16_t>(k & 1u ? w[k / 2] >> 16 : w[k / 2] & 0xFFFFu);
    }
}

// Experiment (XS_MMSE_MFMA): the 4x4 Gram H^H H of the wave's 64 cells on the matrix pipe. The
// 16-block 4x4x1 MFMA takes lane 4b+i's A/B value as row/column i of block b and returns G_b[i][j]
// in lane 4b+j, component i. Per group of 16 cells: the group's H goes through the wave's LDS
// scratch [NRX][4] rows of 16 cells so lane 4b+i holds H[a][i] of cell b, 4*NRX MFMAs (re: hr hr^T
// + hi hi^T, im: hr hi^T - hi hr^T), G back through [4][4] rows of 16 cells to the cell's lane. A row
// stride of 24 float2 puts the four rows one half-wave reads on disjoint bank quarters. Needs the
// whole wave.
template <int NRX>
__device__ __forceinline__ void gram_mfma(const float2 (&h)[NRX][4], float2* scr, float nv, float (&gd)[4],
                                          float2 (&go)[4][4]) {
    typedef float v4f __attribute__((ext_vector_type(4)));
    const uint32_t lane = threadIdx.x & 63u, c = lane & 15u, blk = lane >> 2, col = lane & 3u;
    auto wsync = [] {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    };
#pragma unroll
    for (uint32_t g = 0; g < 4; ++g) {
        if ((lane >> 4) == g) {
#pragma unroll
            for (int a = 0; a < NRX; ++a)
#pragma unroll
                for (int t = 0; t < 4; ++t) scr[(a * 4 + t) * 24 + c] = h[a][t];
        }
        wsync();
        float2 hv[NRX];
#pragma unroll
        for (int a = 0; a < NRX; ++a) hv[a] = scr[(a * 4 + col) * 24 + blk];
        wsync();
        v4f gr = {0.f, 0.f, 0.f, 0.f}, gi = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int a = 0; a < NRX; ++a) {
            gr = __builtin_amdgcn_mfma_f32_4x4x1f32(hv[a].x, hv[a].x, gr, 0, 0, 0);
            gr = __builtin_amdgcn_mfma_f32_4x4x1f32(hv[a].y, hv[a].y, gr, 0, 0, 0);
            gi = __builtin_amdgcn_mfma_f32_4x4x1f32(hv[a].x, hv[a].y, gi, 0, 0, 0);
            gi = __builtin_amdgcn_mfma_f32_4x4x1f32(-hv[a].y, hv[a].x, gi, 0, 0, 0);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) scr[(i * 4 + col) * 24 + blk] = make_float2(gr[i], gi[i]);
        wsync();
        const bool mine = (lane >> 4) == g;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const float2 d = scr[(i * 4 + i) * 24 + c];
            if (mine) gd[i] = nv + d.x;
#pragma unroll
            for (int j = 0; j < i; ++j) {
                const float2 v = scr[(i * 4 + j) * 24 + c];
                if (mine) go[i][j] = v;
            }
        }
        wsync();
    }
}

template <int NRX, int NT, int NBPS = 0>
__device__ __forceinline__ void eq_mmse(const rx_cells_args& A, const cell_seg* sg, const float2* zfi, const float* wtab,
                                        uint32_t zst, float nv, const unit_sm<NRX, NT>& b, int16_t* __restrict__ llr,
                                        float2* scr = nullptr, bool act = true) {
    const uint32_t N_bps = NBPS ? NBPS : A.N_bps;
    const uint32_t info = sg[b.si].info, wbase = sg[b.si].wbase;
    const uint32_t mode = info & 1u, off = (info >> 4) & 0xFFu, nI = info >> 12;
    const uint32_t sh = mode ? 0u : 1u;  // pilot step 1 (mode lr) or 2 (mode l, interlaced)
    // Wiener interpolation of every (rx, stream) at the cell (rx_synced.cpp:932-946); the pilot
    // buffer holds antenna pairs interleaved here (build_pilots<., ., true>): one 16-B read per pair
    // and tap, the pairs zst * 2 cells apart
    static_assert(NRX % 2 == 0, "MMSE: antenna pairs");
    typedef float f4 __attribute__((ext_vector_type(4)));
    float2 h[NRX][NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
        uint32_t p = b.pw[t] & 0xFFFFu;
        if (!mode) p = 2 * p + ((off >> t) & 1u);
        const float2* zr = zfi + (t * (NRX / 2) * zst + p) * 2;
        const float* wb = wtab + wbase + (b.pw[t] >> 16) * nI;
        const uint32_t zs = 2u << sh;
#pragma unroll
        for (int a = 0; a < NRX; ++a) h[a][t] = make_float2(0.f, 0.f);
#pragma unroll 4
        for (uint32_t i = 0; i < nI; ++i, zr += zs) {
            const float w = wb[i];
#pragma unroll
            for (int q = 0; q < NRX / 2; ++q) {
                const f4 z = *reinterpret_cast<const f4*>(zr + q * zst * 2);
                h[2 * q][t].x = fmaf(z.x, w, h[2 * q][t].x);
                h[2 * q][t].y = fmaf(z.y, w, h[2 * q][t].y);
                h[2 * q + 1][t].x = fmaf(z.z, w, h[2 * q + 1][t].x);
                h[2 * q + 1][t].y = fmaf(z.w, w, h[2 * q + 1][t].y);
            }
        }
    }
    // G = H^H H + nv I (diagonal gd, strictly lower go[i][j] = sum_a conj(h_ai) h_aj), z = H^H y
    float gd[NT];
    float2 go[NT][NT], zz[NT];
    constexpr bool mf = experiment(XS_MMSE_MFMA) && NT == 4;
    if constexpr (mf) gram_mfma<NRX>(h, scr, nv, gd, go);
#pragma unroll
    for (int i = 0; i < NT; ++i) {
        zz[i] = make_float2(0.f, 0.f);
#pragma unroll
        for (int a = 0; a < NRX; ++a) zz[i] = cadd(zz[i], cmulc(b.r0[a], h[a][i]));
        if constexpr (mf) continue;
        gd[i] = nv;
#pragma unroll
        for (int a = 0; a < NRX; ++a) gd[i] += cnorm(h[a][i]);
#pragma unroll
        for (int j = 0; j < i; ++j) {
            go[i][j] = make_float2(0.f, 0.f);
#pragma unroll
            for (int a = 0; a < NRX; ++a) go[i][j] = cadd(go[i][j], cmulc(h[a][j], h[a][i]));
        }
    }
    // Cholesky G = L L^H (real diagonal ld, reciprocal il), then Mi = L^-1
    float il[NT];
    float2 Lm[NT][NT], Mi[NT][NT];
#pragma unroll
    for (int j = 0; j < NT; ++j) {
        float d = gd[j];
#pragma unroll
        for (int m = 0; m < j; ++m) d -= cnorm(Lm[j][m]);
        il[j] = rsqrtf(fmaxf(d, 1e-30f));
#pragma unroll
        for (int i = j + 1; i < NT; ++i) {
            float2 v = go[i][j];
#pragma unroll
            for (int m = 0; m < j; ++m) v = csub(v, cmulc(Lm[i][m], Lm[j][m]));
            Lm[i][j] = cscale(v, il[j]);
        }
    }
#pragma unroll
    for (int j = 0; j < NT; ++j) {
        Mi[j][j] = make_float2(il[j], 0.f);
#pragma unroll
        for (int i = j + 1; i < NT; ++i) {
            float2 v = make_float2(0.f, 0.f);
#pragma unroll
            for (int m = j; m < i; ++m) v = cadd(v, cmul(Lm[i][m], Mi[m][j]));
            Mi[i][j] = cscale(v, -il[i]);
        }
    }
    // w = L^-1 z; x = L^-H w; [G^-1]_ss = sum_m |Mi[m][s]|^2
    float2 w[NT];
#pragma unroll
    for (int m = 0; m < NT; ++m) {
        w[m] = make_float2(0.f, 0.f);
#pragma unroll
        for (int q = 0; q <= m; ++q) w[m] = cadd(w[m], cmul(Mi[m][q], zz[q]));
    }
    // the cell's scrambling bits big-endian from bit (b_first & ~7): bit r at 63 - r
    const uint32_t b_first = b.jj * NT * N_bps;
    const uint64_t be = static_cast<uint64_t>((b.sb[0] & 0xFFu) << 24 | (b.sb[1] & 0xFFu) << 16 | (b.sb[2] & 0xFFu) << 8 |
                                              (b.sb[3] & 0xFFu))
                            << 32 |
                        static_cast<uint64_t>(b.sb[4] & 0xFFu) << 24;
#pragma unroll
    for (int s = 0; s < NT; ++s) {
        float2 x = make_float2(0.f, 0.f);
        float ginv = 0.f;
#pragma unroll
        for (int m = s; m < NT; ++m) {
            x = cadd(x, cmulc(w[m], Mi[m][s]));
            ginv += cnorm(Mi[m][s]);
        }
        const float beta = 1.f - nv * ginv;
        const uint32_t sw = static_cast<uint32_t>((be << ((b_first & 7u) + s * N_bps)) >> 32);
        if (act) emit_symw(cscale(x, 1.0f / beta), b_first + s * N_bps, N_bps, sw, llr);
    }
}

// The epoch's pilot buffer: zero-forced DRS cells of every (rx, ts) at their interlace slots
// (channel_antenna.hpp:38-63), read from the DRS symbols in Y. Whole workgroup, no barrier. The
// source DRS op of every (ts, interlace slot), its parity and symbol are workgroup-uniform (scalar
// loads); a thread loads the subcarrier indices of one pilot index for every (ts, slot) at once, then
// the cells of every (rx, ts, slot): two memory round trips. Slots without a source read a valid
// cell and store zero. Layout [NRX][NT][zst], or for the MMSE path (AI) antenna pairs interleaved,
// [NT][NRX / 2][zst][2]: one 16-B read per antenna pair and tap. (All NRX antennas of a pilot
// contiguous, [NT][zst][NRX], puts the lanes' pilots 32 B apart and reads 8-16 B of each: 9
// conflict cycles per LDS instruction, measured; padded to NRX + 1 cells per pilot it is conflict-
// free but 25 % larger, one workgroup per CU instead of two: slower still.)
template <int NRX, int NT, bool AI = false>
__device__ __forceinline__ void build_pilots(const rx_cells_args& A, const rx_epoch* E, const float2* Yp, float2* zfi,
                                             uint32_t tid, uint32_t nthreads) {
    const uint32_t nd = A.n_drs, zst = zfi_stride(nd);
    const size_t ast = size_t(A.n_sym_total) * A.Nf_pad;
    auto zi = [&](uint32_t a, uint32_t t, uint32_t idx) {
        return AI ? ((t * (NRX / 2) + a / 2) * zst + idx) * 2 + (a & 1u) : (a * NT + t) * zst + idx;
    };
    for (uint32_t e = tid; e < NRX * NT * ZFI_PAD; e += nthreads)
        zfi[zi(e / ZFI_PAD / NT, e / ZFI_PAD % NT, 2 * nd + e % ZFI_PAD)] = make_float2(0.f, 0.f);
    // sources of all (ts, slot) first, then their DRS ops (two scalar round trips); a slot without a
    // source reads op 0 and is stored as zero
    uint32_t src[NT][2], kb[NT][2], yo[NT][2];
    bool ok[NT][2];
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int o = 0; o < 2; ++o) src[t][o] = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(E->src[t][o]));
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int o = 0; o < 2; ++o) {
            ok[t][o] = src[t][o] != 0xFFFFu;
            const uint32_t op = ok[t][o] ? src[t][o] : 0u;
            const uint32_t par = A.n_dops ? (A.dmeta[op] >> 16) & 0xFFu : 0u, l = A.n_dops ? A.dl[op] : 0u;
            kb[t][o] = ok[t][o] ? par * 4 + (t & 3u) : (t & 3u);
            yo[t][o] = ok[t][o] ? l * A.Nf_pad : 0u;
        }
    for (uint32_t i = tid; i < nd; i += nthreads) {
        uint32_t k[NT][2];
        float dv[NT];
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            dv[t] = A.drs_v[t * nd + i];
#pragma unroll
            for (int o = 0; o < 2; ++o) k[t][o] = A.drs_k[kb[t][o] * nd + i];
        }
        float2 v[NT][2][NRX];
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
            for (int o = 0; o < 2; ++o)
#pragma unroll
                for (int a = 0; a < NRX; ++a) v[t][o][a] = Yp[a * ast + yo[t][o] + k[t][o]];
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
            for (int o = 0; o < 2; ++o)
#pragma unroll
                for (int a = 0; a < NRX; ++a)
                    zfi[zi(a, t, 2 * i + o)] = ok[t][o] ? cscale(v[t][o][a], dv[t]) : make_float2(0.f, 0.f);
    }
}

// build_pilots in two halves for one thread per (pilot index pi, interlace slot po) -- the fast form
// where 2 n_drs <= threads: pilot_offsets issues the dependent source loads (the epoch's DRS ops ->
// their parity and symbol -> the pilot's subcarrier and DRS value) and returns each stream's cell
// offset in the packet's Y rows; pilot_cells loads the cells and stores the zero-forced pilots (plus
// the row padding). Same loads and values as build_pilots.
template <int NT>
__device__ __forceinline__ void pilot_offsets(const rx_cells_args& A, const rx_epoch* E, uint32_t tid, uint32_t (&pyk)[NT],
                                              float (&pdv)[NT], uint32_t& pok) {
    const uint32_t nd = A.n_drs, pi = tid >> 1, po = tid & 1u;
    pok = 0;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
        const uint32_t s0 = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(E->src[t][0])),
                       s1 = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(E->src[t][1]));
        const uint32_t src = po ? s1 : s0;
        const bool ok = src != 0xFFFFu;
        const uint32_t op = ok ? src : 0u;
        const uint32_t par = A.n_dops ? (A.dmeta[op] >> 16) & 0xFFu : 0u, l = A.n_dops ? A.dl[op] : 0u;
        const uint32_t kb = ok ? par * 4 + (t & 3u) : (t & 3u), yo = ok ? l * A.Nf_pad : 0u;
        pok |= ok ? 1u << t : 0u;
        pdv[t] = A.drs_v[t * nd + pi];
        pyk[t] = yo + A.drs_k[kb * nd + pi];
    }
}

template <int NRX, int NT>
__device__ __forceinline__ void pilot_cells(const rx_cells_args& A, const float2* Yp, float2* zfi, uint32_t tid,
                                            uint32_t nthreads, bool act, const uint32_t (&pyk)[NT], const float (&pdv)[NT],
                                            uint32_t pok) {
    constexpr bool AI = cells_ai(NRX, NT);
    const uint32_t nd = A.n_drs, zst = zfi_stride(nd), pi = tid >> 1, po = tid & 1u;
    const size_t ast = size_t(A.n_sym_total) * A.Nf_pad;
    auto zi = [&](uint32_t a, uint32_t t, uint32_t idx) {
        return AI ? ((t * (NRX / 2) + a / 2) * zst + idx) * 2 + (a & 1u) : (a * NT + t) * zst + idx;
    };
    for (uint32_t e = tid; e < NRX * NT * ZFI_PAD; e += nthreads)
        zfi[zi(e / ZFI_PAD / NT, e / ZFI_PAD % NT, 2 * nd + e % ZFI_PAD)] = make_float2(0.f, 0.f);
    if (act) {
        float2 pv[NT][NRX];
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
            for (int a = 0; a < NRX; ++a) pv[t][a] = Yp[a * ast + pyk[t]];
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
            for (int a = 0; a < NRX; ++a)
                zfi[zi(a, t, 2 * pi + po)] = ((pok >> t) & 1u) ? cscale(pv[t][a], pdv[t]) : make_float2(0.f, 0.f);
    }
}

}  // namespace dnrp::dev
