// Per-cell back end of the synchronised receiver (rx_cells_kernel, rx_back.hip): Wiener interpolation
// of the channel from the interlaced pilot buffer (rx_synced.cpp:893-949), MRC (1204-1306) or SFBC
// combining (1335-1392), srsRAN-style int16 soft demapping and descrambling (pcc_enc.cpp:297,
// pdc_enc.cpp:339-344).
#pragma once

#include "device_common.hpp"
#include "kernels.hpp"

namespace dnrp::dev {

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

// demap + descramble + int16 of cell j (LLRs j*N_bps .. j*N_bps+N_bps-1)
__device__ __forceinline__ void emit_cell(float2 x, uint32_t j, uint32_t N_bps, const uint8_t* __restrict__ seq,
                                          int16_t* __restrict__ llr) {
    float L[8];
    demap(x, N_bps, L);
    const uint32_t base = j * N_bps;
    if (N_bps == 8) {  // one scrambling byte, one 16-B store
        const uint32_t sb = seq[j];
        uint32_t w[4];
#pragma unroll
        for (int b = 0; b < 8; b += 2) {
            const float v0 = ((sb >> (7 - b)) & 1u) ? -L[b] : L[b];
            const float v1 = ((sb >> (6 - b)) & 1u) ? -L[b + 1] : L[b + 1];
            w[b / 2] = static_cast<uint16_t>(q16(v0)) | (static_cast<uint32_t>(static_cast<uint16_t>(q16(v1))) << 16);
        }
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
    for (uint32_t b = 0; b < 8; ++b) {
        if (b < N_bps) {
            const uint32_t i = base + b;
            const uint32_t sbit = (seq[i >> 3] >> (7u - (i & 7u))) & 1u;
            llr[i] = q16(sbit ? -L[b] : L[b]);
        }
    }
}

#ifndef CELL_WCHUNK_DEF
#define CELL_WCHUNK_DEF 4
#endif
constexpr uint32_t CELL_WCHUNK = CELL_WCHUNK_DEF;  // interpolation taps per weight-load batch

// One work unit: cell jj (MRC, NT == 1) or the SFBC pair jj, jj+1 (NT > 1) under segment S's
// interpolation event, in two steps so a caller can take the dependent index loads of one unit off
// the critical path of another: eq_gather resolves the unit's segment, subcarrier indices and LUT
// pilot | weight indices (kk -> pw), eq_finish loads the received cells of every RX antenna together
// with the interpolation weights, reads the epoch's pilot buffer zfi [NRX][NT][2 nd], interpolates,
// combines, demaps and stores. lut: the Wiener LUT profile picked after the segment's last DRS.
template <int NT>
struct eq_work {
    static constexpr int NC = NT == 1 ? 1 : 4;  // interpolated channels per unit
    uint32_t jj, k0, k1, yoff;
    uint32_t meta;  // mode | tA << 1 | tB << 5 | off << 9 | nI << 17
    const float* wt;
    uint32_t pw[NC];
};

__device__ __forceinline__ uint32_t eq_meta_mode(uint32_t m) { return m & 1u; }
__device__ __forceinline__ uint32_t eq_meta_tA(uint32_t m) { return (m >> 1) & 0xFu; }
__device__ __forceinline__ uint32_t eq_meta_tB(uint32_t m) { return (m >> 5) & 0xFu; }
__device__ __forceinline__ uint32_t eq_meta_off(uint32_t m) { return (m >> 9) & 0xFFu; }
__device__ __forceinline__ uint32_t eq_meta_nI(uint32_t m) { return m >> 17; }

// yoff: offset of the unit's symbol row in the packet's Y block (antenna 0)
template <int NT>
__device__ __forceinline__ void eq_gather(const rx_cells_args& A, const rx_seg& S, uint32_t lut, uint32_t jj, uint32_t yoff,
                                          eq_work<NT>& w) {
    const uint32_t Nf = A.N_occ + 1;
    const rx_lut LT = A.luts[S.mode * 3 + lut];
    const uint32_t* __restrict__ pwt = LT.pw + size_t(S.rel) * 4 * Nf;
    w.jj = jj;
    w.yoff = yoff;
    w.wt = LT.w;
    uint32_t tA = 0, tB = 0;
    if constexpr (NT == 1) {
        w.k0 = w.k1 = A.kk[jj];
        w.pw[0] = pwt[(0u ^ S.swap) * Nf + w.k0];
    } else {
        w.k0 = A.kk[jj];
        w.k1 = A.kk[jj + 1];
        const uint32_t pr = A.pair[(jj >> 1) % A.mod];
        tA = pr & 0xFu;
        tB = pr >> 4;
        w.pw[0] = pwt[((tA & 3u) ^ S.swap) * Nf + w.k0];
        w.pw[1] = pwt[((tA & 3u) ^ S.swap) * Nf + w.k1];
        w.pw[2] = pwt[((tB & 3u) ^ S.swap) * Nf + w.k0];
        w.pw[3] = pwt[((tB & 3u) ^ S.swap) * Nf + w.k1];
    }
    w.meta = (S.mode & 1u) | tA << 1 | tB << 5 | (S.off & 0xFFu) << 9 | LT.n << 17;
}

// Y: the packet's received cells [NRX][n_sym_total][Nf_pad]
template <int NRX, int NT>
__device__ __forceinline__ void eq_finish(const rx_cells_args& A, const eq_work<NT>& W, const float2* __restrict__ Y,
                                          const float2* zfi, uint32_t nd2, const uint8_t* __restrict__ seq,
                                          int16_t* __restrict__ llr) {
    constexpr int NC = eq_work<NT>::NC;
    const size_t ast = size_t(A.n_sym_total) * A.Nf_pad;
    float2 r0[NRX], r1[NT == 1 ? 1 : NRX];
#pragma unroll
    for (int a = 0; a < NRX; ++a) {
        r0[a] = Y[a * ast + W.yoff + W.k0];
        if constexpr (NT > 1) r1[a] = Y[a * ast + W.yoff + W.k1];
    }
    const uint32_t mode = eq_meta_mode(W.meta), off = eq_meta_off(W.meta), nI = eq_meta_nI(W.meta);
    const uint32_t step = mode ? 1u : 2u;
    // interpolation weights and pilot start of channel c (stream tA / tB at k0 / k1)
    const float* w[NC];
    uint32_t pos[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        const uint32_t t = c < 2 ? eq_meta_tA(W.meta) : eq_meta_tB(W.meta);
        w[c] = W.wt + size_t(W.pw[c] >> 16) * nI;
        uint32_t p = W.pw[c] & 0xFFFFu;
        if (!mode) p = 2 * p + ((off >> t) & 1u);  // non-interlaced: latest DRS symbol only
        pos[c] = p + t * nd2;
    }
    float2 h[NRX][NC];
#pragma unroll
    for (int a = 0; a < NRX; ++a)
#pragma unroll
        for (int c = 0; c < NC; ++c) h[a][c] = make_float2(0.f, 0.f);
    // weights in chunks of CELL_WCHUNK taps: all of a chunk's (global / L1) weight loads are in
    // flight together instead of one dependent load per tap
    for (uint32_t i0 = 0; i0 < nI; i0 += CELL_WCHUNK) {
        float wc[NC][CELL_WCHUNK];
#pragma unroll
        for (int c = 0; c < NC; ++c)
#pragma unroll
            for (uint32_t ii = 0; ii < CELL_WCHUNK; ++ii) wc[c][ii] = i0 + ii < nI ? w[c][i0 + ii] : 0.f;
#pragma unroll
        for (uint32_t ii = 0; ii < CELL_WCHUNK; ++ii) {
            if (i0 + ii >= nI) break;
#pragma unroll
            for (int c = 0; c < NC; ++c) {
                const uint32_t p = pos[c] + (i0 + ii) * step;
#pragma unroll
                for (int a = 0; a < NRX; ++a) {
                    const float2 z = zfi[a * NT * nd2 + p];
                    h[a][c].x = fmaf(z.x, wc[c][ii], h[a][c].x);
                    h[a][c].y = fmaf(z.y, wc[c][ii], h[a][c].y);
                }
            }
        }
    }
    if constexpr (NT == 1) {
        float2 num = make_float2(0.f, 0.f);
        float den = 0.f;
#pragma unroll
        for (int a = 0; a < NRX; ++a) {  // MRC (rx_synced.cpp:1204-1306)
            num = cadd(num, cmulc(r0[a], h[a][0]));
            den += cnorm(h[a][0]);
        }
        emit_cell(cscale(num, 1.0f / den), W.jj, A.N_bps, seq, llr);
    } else {
        float2 n0 = make_float2(0.f, 0.f), n1 = make_float2(0.f, 0.f);
        float den = 0.f;
#pragma unroll
        for (int a = 0; a < NRX; ++a) {  // SFBC pair (rx_synced.cpp:1335-1392)
            const float2 h0 = cscale(cadd(h[a][0], h[a][1]), 0.5f);
            const float2 h1 = cscale(cadd(h[a][2], h[a][3]), 0.5f);
            n0 = cadd(n0, cadd(cmul(cconj(h0), r0[a]), cmul(h1, cconj(r1[a]))));
            n1 = cadd(n1, cadd(cmul(make_float2(-h1.x, -h1.y), cconj(r0[a])), cmul(cconj(h0), r1[a])));
            den += cnorm(h0) + cnorm(h1);
        }
        emit_cell(cscale(n0, 1.0f / den), W.jj, A.N_bps, seq, llr);
        emit_cell(cscale(n1, 1.0f / den), W.jj + 1, A.N_bps, seq, llr);
    }
}

// The epoch's pilot buffer: zero-forced DRS cells of every (rx, ts) at their interlace slots
// (channel_antenna.hpp:38-63), read from the DRS symbols in Y. Whole workgroup, no barrier. The
// source DRS op of every (ts, interlace slot), its parity and symbol are workgroup-uniform (scalar
// loads); a thread then has the DRS cells of one pilot index i for every (rx, ts, slot) in flight
// together: two dependent loads (drs_k -> Y) instead of a four-load chain per element.
template <int NRX, int NT>
__device__ __forceinline__ void build_pilots(const rx_cells_args& A, const rx_epoch* E, const float2* Yp, float2* zfi,
                                             uint32_t tid, uint32_t nthreads) {
    const uint32_t nd = A.n_drs, nd2 = 2 * nd;
    const size_t ast = size_t(A.n_sym_total) * A.Nf_pad;
    uint32_t kb[NT][2], yo[NT][2];  // drs_k row base (~0: no source) and Y row offset
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int o = 0; o < 2; ++o) {
            const uint32_t src = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(E->src[t][o]));
            kb[t][o] = 0xFFFFFFFFu;
            yo[t][o] = 0;
            if (src != 0xFFFFu) {
                const uint32_t par = (A.dmeta[src] >> 16) & 0xFFu;
                kb[t][o] = (par * 4 + (t & 3u)) * nd;
                yo[t][o] = A.dl[src] * A.Nf_pad;
            }
        }
    for (uint32_t i = tid; i < nd; i += nthreads) {
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            const float dv = A.drs_v[t * nd + i];
#pragma unroll
            for (int o = 0; o < 2; ++o) {
                float2 v[NRX];
#pragma unroll
                for (int a = 0; a < NRX; ++a) v[a] = make_float2(0.f, 0.f);
                if (kb[t][o] != 0xFFFFFFFFu) {
                    const uint32_t k = A.drs_k[kb[t][o] + i];
#pragma unroll
                    for (int a = 0; a < NRX; ++a) v[a] = cscale(Yp[a * ast + yo[t][o] + k], dv);
                }
#pragma unroll
                for (int a = 0; a < NRX; ++a) zfi[(a * NT + t) * nd2 + 2 * i + o] = v[a];
            }
        }
    }
}

}  // namespace dnrp::dev
