// Fused TX kernel, symbol-parallel: one workgroup = one (packet, antenna, run of K OFDM symbols).
//
// A WG synthesises the K symbols of its run plus the symbol before them, whose tail is the
// resampler history, so runs are independent and the whole slot is in flight at once:
//   staged d-bits (descrambled)  ->  scramble/modulate (PCC QPSK, PDC BPSK..256QAM), transmit
//   diversity flip, DRS/STF cells, beamforming row W[a,:], FFT-bin mirror and scaling
//   ->  IFFT whose last pass writes the cyclic-prefixed (and STF-covered) time-domain symbol
//   straight into a linear LDS buffer
//   ->  register-blocked polyphase L/M resampler (polyphase.hpp) + phase-continuous mixer -> HBM.
// Two IFFT engines: for N_b_DFT_os = 1024 (the u=8, b=16 benchmark size) every wavefront owns one
// symbol end to end (bins built in registers, wave_fft1024, no workgroup barrier until the
// resampler); other sizes use the workgroup-wide batched Stockham FFT.
// Restates tx_t::generate_tx_packet (lib/src/phy/tx/tx.cpp:165-314) and its callees
// run_pcc/run_drs/run_pdc (936-1116), run_beamforming (729-860), run_ifft_cp_scale (862-911),
// stf_t::apply_cover_sequence (sections_part3/stf.cpp:104-138), resampler_t (resampler.cpp:330-454)
// and mixer_t::mix_phase_continuous (mixer.cpp:41-65). Only the packed d-bits are read and only
// the final hw-rate IQ is written: HBM traffic = ceil(G/8) + 25 bytes in, N_TX * S * 8 bytes out.
#include "device_common.hpp"
#include "experiments.hpp"
#include "kernels.hpp"
#include "polyphase.hpp"
#include "taps_gen.hpp"

namespace dnrp::dev {

__constant__ float k_cover[9] = DNRP_STF_COVER_SEQUENCE;  // stf.hpp:146-151 (params.hpp)
// the same sequence as a sign mask (bit q: entry q is -1), for the streaming kernel: no vector load
constexpr uint32_t cover_neg_mask() {
    constexpr float cv[9] = DNRP_STF_COVER_SEQUENCE;
    uint32_t mk = 0;
    for (int q = 0; q < 9; ++q) mk |= (cv[q] < 0.f ? 1u : 0u) << q;
    return mk;
}
constexpr bool cover_is_sign() {
    constexpr float cv[9] = DNRP_STF_COVER_SEQUENCE;
    for (int q = 0; q < 9; ++q)
        if (cv[q] != 1.f && cv[q] != -1.f) return false;
    return true;
}
static_assert(cover_is_sign(), "cover sequence entries are +-1");
__device__ __forceinline__ float cover_sign(uint32_t q) { return ((cover_neg_mask() >> q) & 1u) ? -1.f : 1.f; }

// streaming TX, 256-QAM: constellation from the separable 16-level table (two conflict-free reads
// and the index bit gathers) instead of the 256-entry table (one read, ~3 conflict cycles). A/B on
// MI355X: TX 19.25-19.48 vs 18.83-18.98 ms per 16384-slot chunk -- the gathers' VALU (+5 % per
// wave) cost more than the conflicts; off by default

constexpr uint32_t TX_THREADS = 256;     // block-FFT path workgroup
constexpr uint32_t TX_WAVE_MAX = 512;    // wave path: one wavefront per symbol slot, 64 (K + 1) threads
constexpr uint32_t TX_MAX_SLOTS = 8;     // K + 1 (wave path)
constexpr uint32_t TX_BLOCK_SLOTS = 4;   // K + 1 (block-FFT path)
constexpr uint32_t TX_BIN_REG = 4;    // FFT bins per thread per symbol, block path (N_b_DFT_os <= 1024)

__device__ __forceinline__ uint32_t bits_of(uint32_t b0, uint32_t b1, uint32_t bitoff, uint32_t nbits) {
    const uint32_t w = (b0 << 8) | b1;
    return (w >> (16u - (bitoff & 7u) - nbits)) & ((1u << nbits) - 1u);
}

__device__ __forceinline__ bool nz(float2 w) { return w.x != 0.f || w.y != 0.f; }

__device__ __forceinline__ int floor_div(int a, int b) { return a >= 0 ? a / b : -((-a + b - 1) / b); }

// per-WG view of one (packet, antenna, run)
struct tx_wg {
    const tx_args* A;
    tx_pkt P;
    uint32_t pkt, ant, Nd, N, Nf, hl, len0, lenD;
    uint32_t l_first, l_last, s0, nsl, base_q, sbyte0, pdc_bytes;
    bool last_run;
    float2 *lin, *twl, *qtab, *pccs, *wrow;
    float* hpl;
    uint8_t* sb;
    const uint8_t *dpdc, *cpdc;

    __device__ uint32_t bsym(uint32_t l) const { return l == 0 ? 0u : len0 + (l - 1) * lenD; }
    __device__ float2* slot(uint32_t l) const { return lin + A->HP + bsym(l) - base_q; }

    __device__ float2 pdc_sym(uint32_t s) const {  // complex PDC symbol s of the packet
        if (A->N_bps == 8 && A->stage_bytes) return qtab[sb[s - sbyte0]];  // 256-QAM: one byte per symbol
        const uint32_t bit = s * A->N_bps;
        if (A->stage_bytes) {
            const uint32_t lb = bit - (sbyte0 << 3), bo = lb >> 3;
            return qtab[bits_of(sb[bo], sb[bo + 1], lb, A->N_bps)];
        }
        const uint32_t bo = bit >> 3;
        const uint32_t b1 = bo + 1 < pdc_bytes ? uint32_t(dpdc[bo + 1] ^ cpdc[bo + 1]) : 0u;
        return qtab[bits_of(dpdc[bo] ^ cpdc[bo], b1, bit, A->N_bps)];
    }

    // value of FFT bin n (its cell code c) of symbol l, scaled (tx.cpp:936-1116, 729-860, 862-871)
    __device__ float2 bin(uint32_t c, uint32_t n, uint32_t l) const {
        auto flip = [](float2 nb, uint32_t j) {  // pairwise swap + (-re,+im) / (+re,-im) pattern
            return (j & 1u) ? make_float2(nb.x, -nb.y) : make_float2(-nb.x, nb.y);
        };
        const uint32_t ty = c & CODE_MASK, j = c & CODE_J_MASK;
        const uint32_t pr = (c >> CODE_PAIR_SHIFT) & 0xFFu;  // TS pair A | B << 4 (host-precomputed)
        float2 v = make_float2(0.f, 0.f);
        if (ty == CODE_STF) {
            const uint32_t k = n <= N / 2 ? N / 2 + n : n - A->off_lower;
            v = cmul(wrow[0], A->stf[k]);
        } else if (ty == CODE_DRS) {
            v = cscale(wrow[j & 7u], (j & 8u) ? -1.f : 1.f);
        } else if (ty == CODE_PCC) {
            if (A->N_TS == 1) {
                v = cmul(wrow[0], pccs[j]);
            } else {
                v = cadd(cmul(wrow[pr & 0xFu], pccs[j]), cmul(wrow[pr >> 4], flip(pccs[j ^ 1u], j)));
            }
        } else if (ty == CODE_PDC) {
            if (A->txdiv) {
                const float2 wa = wrow[pr & 0xFu], wb = wrow[pr >> 4];
                if (nz(wa)) v = cmul(wa, pdc_sym(j));
                if (nz(wb)) v = cadd(v, cmul(wb, flip(pdc_sym(j ^ 1u), j)));
            } else {
                for (uint32_t ss = 0; ss < A->N_SS; ++ss)
                    if (nz(wrow[ss])) v = cadd(v, cmul(wrow[ss], pdc_sym(j * A->N_SS + ss)));
            }
        }
        return cscale(v, l == 0 ? P.scale_stf : P.scale_df);
    }

    // cell code of FFT bin n in symbol l (0 for guard / DC-free bins outside the occupied band)
    __device__ uint32_t code(uint32_t l, uint32_t n) const {
        uint32_t k = 0xFFFFFFFFu;
        if (n <= N / 2)
            k = N / 2 + n;
        else if (n >= A->off_lower && n < A->off_lower + N / 2)
            k = n - A->off_lower;
        return (n < Nd && k != 0xFFFFFFFFu) ? A->code[size_t(l) * Nf + k] : 0u;
    }

    // wave path (N_b_DFT_os = 1024): the wave's whole symbol v[m] = x[lane + 64 m] into its CP
    // layout: 16 plain stores, then the cyclic prefix copied from the symbol's tail and, for the
    // STF, the cover sequence (ofdm.cpp:62-79, stf.cpp:104-138) in short rolled loops
    __device__ void put_symbol(uint32_t l, const float2 (&v)[16], uint32_t lane) const {
        float2* dst = slot(l);
        const uint32_t cp = l == 0 ? A->STF_CP : A->CP;
#pragma unroll
        for (int m = 0; m < 16; ++m) dst[cp + lane + 64 * m] = v[m];
        __builtin_amdgcn_wave_barrier();  // a wave's LDS accesses complete in order
        for (uint32_t i = lane; i < cp; i += 64) dst[i] = dst[cp + ((i + 2048u - cp) & 1023u)];
        if (l == 0) {
            __builtin_amdgcn_wave_barrier();
            for (uint32_t i = lane; i < cp + 1024; i += 64) dst[i] = cscale(dst[i], k_cover[min(i / A->pattern_len, 8u)]);
        }
    }

    // time-domain sample n of symbol l into its CP layout (ofdm.cpp:62-79, stf.cpp:104-138)
    __device__ void put(uint32_t l, uint32_t n, float2 v) const {
        float2* dst = slot(l);
        if (l == 0) {
            for (uint32_t i = A->STF_CP + n;; i -= Nd) {  // the STF CP may exceed one FFT length
                dst[i] = cscale(v, k_cover[min(i / A->pattern_len, 8u)]);
                if (i < Nd) break;
            }
        } else {
            dst[A->CP + n] = v;
            if (n >= Nd - A->CP) dst[A->CP + n - Nd] = v;
        }
    }
};

template <bool WAVE>
__device__ __forceinline__ tx_wg tx_setup(const tx_args& A, float2* smem, uint32_t (*rc)[16] = nullptr) {
    tx_wg w;
    w.A = &A;
    const uint32_t run = blockIdx.x % A.n_runs, pa = blockIdx.x / A.n_runs;
    w.pkt = pa / A.N_TX;
    w.ant = pa % A.N_TX;
    w.P = A.pk[w.pkt];
    w.Nd = A.plan.N;
    w.N = A.N_occ;
    w.Nf = w.N + 1;
    w.hl = A.hl;
    w.len0 = A.STF_CP + w.Nd;
    w.lenD = A.CP + w.Nd;
    w.l_first = run * A.K;
    w.l_last = min(w.l_first + A.K, A.N_DF + 1) - 1;
    w.s0 = w.l_first > 0 ? w.l_first - 1 : 0u;
    w.nsl = w.l_last - w.s0 + 1;
    w.last_run = (run + 1 == A.n_runs);
    w.base_q = w.bsym(w.s0);
    w.lin = smem;  // [lin_len] head pad | symbols s0..l_last | tail pad
    float2* p = w.lin + A.lin_len;
    if (!WAVE) p += A.bufB_len;  // block FFT ping-pong partner / output staging
    // wave path: the FFT reads the (L2/L1-resident) global twiddle table, no LDS copy
    w.twl = WAVE ? const_cast<float2*>(A.tw) : p;
    w.qtab = WAVE ? p : w.twl + w.Nd;
    w.pccs = w.qtab + 256;
    w.wrow = w.pccs + 98;
    w.hpl = reinterpret_cast<float*>(w.wrow + 8);
    w.sb = reinterpret_cast<uint8_t*>(w.hpl + A.npp);
    w.dpdc = A.pdc_d + size_t(w.pkt) * A.pdc_stride;
    w.cpdc = w.P.pdc_seq;
    w.pdc_bytes = (A.G + 7) / 8;
    w.sbyte0 = (A.pdc_off[max(w.s0, 1u)] * A.N_SS * A.N_bps) >> 3;

    // ---- staging: tables, PCC symbols, beamforming row, taps, descrambled PDC bytes
    const uint8_t* dpcc = A.pcc_d + size_t(w.pkt) * 25;
    if constexpr (WAVE) {
        // wave path (N_b_DFT_os = 1024): every global load of the staging phase, the symbol's
        // cell codes included, is issued before the first LDS store -> one memory round trip
        const uint32_t t = threadIdx.x;
        const uint32_t b = t >> 6, lane = t & 63u, l = w.s0 + b;
        if (rc)
#pragma unroll
            for (int m = 0; m < 16; ++m) (*rc)[m] = b < w.nsl ? w.code(l, lane + 64 * m) : 0u;
        const uint32_t nq = 1u << A.N_bps;
        const float2 r_q = t < nq ? A.qam[t] : make_float2(0.f, 0.f);
        uint32_t r_pcc = 0;
        if (t < 98) r_pcc = uint32_t(dpcc[(2 * t) >> 3] ^ A.pcc_seq[(2 * t) >> 3]);
        const float2 r_w = t < A.N_TS ? A.W[(w.P.codebook * A.N_TX + w.ant) * A.N_TS + t] : make_float2(0.f, 0.f);
        float r_h[2];
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const uint32_t i = t + blockDim.x * j;
            r_h[j] = i < A.npp ? A.taps_pp[i] : 0.f;
        }
        uint32_t r_sb[12];
#pragma unroll
        for (int j = 0; j < 12; ++j) {
            const uint32_t i = t + blockDim.x * j, g = w.sbyte0 + i;
            r_sb[j] = (i < A.stage_bytes && g < w.pdc_bytes) ? uint32_t(w.dpdc[g] ^ w.cpdc[g]) : 0u;
        }
        if (t < nq) w.qtab[t] = r_q;
        if (t < 98) {  // QPSK (TS 36.211 7.1.2): (1 - 2 b0, 1 - 2 b1) / sqrt(2)
            const uint32_t q = bits_of(r_pcc, 0u, 2 * t, 2);
            w.pccs[t] = make_float2((q & 2u) ? -0.70710678f : 0.70710678f, (q & 1u) ? -0.70710678f : 0.70710678f);
        }
        if (t < A.N_TS) w.wrow[t] = r_w;
#pragma unroll
        for (int j = 0; j < 2; ++j)
            if (t + blockDim.x * j < A.npp) w.hpl[t + blockDim.x * j] = r_h[j];
#pragma unroll
        for (int j = 0; j < 12; ++j)
            if (t + blockDim.x * j < A.stage_bytes) w.sb[t + blockDim.x * j] = static_cast<uint8_t>(r_sb[j]);
        // tails beyond the register batch (not reached by the shipped configurations)
        for (uint32_t i = t + 2 * blockDim.x; i < A.npp; i += blockDim.x) w.hpl[i] = A.taps_pp[i];
        for (uint32_t i = t + 12 * blockDim.x; i < A.stage_bytes; i += blockDim.x) {
            const uint32_t g = w.sbyte0 + i;
            w.sb[i] = g < w.pdc_bytes ? static_cast<uint8_t>(w.dpdc[g] ^ w.cpdc[g]) : 0u;
        }
        return w;
    }
    // every copy keeps several loads in flight per thread (stage_gen): a plain strided loop waits
    // for each load before issuing the next
    stage_copy<4>(w.twl, A.tw, w.Nd, threadIdx.x, blockDim.x);
    stage_copy<1>(w.qtab, A.qam, 1u << A.N_bps, threadIdx.x, blockDim.x);
    for (uint32_t j = threadIdx.x; j < 98; j += blockDim.x) {
        const uint32_t bo = (2 * j) >> 3;
        w.pccs[j] = A.qpsk[bits_of(dpcc[bo] ^ A.pcc_seq[bo], 0u, 2 * j, 2)];
    }
    for (uint32_t i = threadIdx.x; i < A.N_TS; i += blockDim.x)
        w.wrow[i] = A.W[(w.P.codebook * A.N_TX + w.ant) * A.N_TS + i];
    stage_copy<2>(w.hpl, A.taps_pp, A.npp, threadIdx.x, blockDim.x);
    const uint8_t* __restrict__ dp = w.dpdc;
    const uint8_t* __restrict__ cp = w.cpdc;
    const uint32_t sb0 = w.sbyte0, nb = w.pdc_bytes;
    stage_gen<8>(w.sb, A.stage_bytes, threadIdx.x, blockDim.x, [&](uint32_t i) {
        const uint32_t g = sb0 + i;
        return g < nb ? static_cast<uint8_t>(dp[g] ^ cp[g]) : static_cast<uint8_t>(0u);
    });
    return w;
}

// zero pads around the run's symbols: history before the packet, flush samples after it
__device__ __forceinline__ void tx_zero_pads(const tx_wg& w) {
    const uint32_t data_end = w.A->HP + w.bsym(w.l_last + 1) - w.base_q;
    for (uint32_t i = threadIdx.x; i < w.A->HP; i += blockDim.x) w.lin[i] = make_float2(0.f, 0.f);
    for (uint32_t i = data_end + threadIdx.x; i < w.A->lin_len; i += blockDim.x) w.lin[i] = make_float2(0.f, 0.f);
}

// resample + mix every output whose newest input lies in the run (the last run adds the flush
// samples) and store it; GI / slot tail zeros on the last run (tx.cpp:679-714)
template <int LR, int MR, int HLR>
__device__ __forceinline__ void tx_resample(const tx_wg& w) {
    const tx_args& A = *w.A;
    const tx_pkt& P = w.P;
    const uint32_t B_lo = w.bsym(w.l_first), B_hi = w.last_run ? w.bsym(A.N_DF + 1) + w.hl : w.bsym(w.l_last + 1);
    auto n_out = [&](uint32_t B) {  // outputs m with delay + m*M < B*L (B*L < 2^32: host-checked)
        const uint32_t t = B * A.L;
        return t > A.delay ? min((t - A.delay + A.M - 1) / A.M, A.n_keep) : 0u;
    };
    const uint32_t m_lo = n_out(B_lo), m_hi = n_out(B_hi);
    float2* out = reinterpret_cast<float2*>(A.out) + size_t(w.pkt * A.N_TX + w.ant) * A.S;
    const int lin_off = static_cast<int>(A.HP) - static_cast<int>(w.base_q);
    if constexpr (LR > 0) {
        using PB = pp_block<LR, MR, HLR>;
        const float2 step1 = P.do_mix ? phasor(P.inc) : make_float2(1.f, 0.f);
        const int q_lo = floor_div(static_cast<int>(m_lo) - static_cast<int>(A.m_star), LR);
        const int q_hi = floor_div(static_cast<int>(m_hi) - static_cast<int>(A.m_star) + LR - 1, LR);
        const int idx_max = static_cast<int>(A.lin_len) - PB::W;
        if (q_hi - q_lo <= 2 * static_cast<int>(blockDim.x) && m_hi - m_lo <= A.lin_len) {
            // coalesced stores: the blocks' outputs go through LDS (over the consumed input buffer)
            // and leave as contiguous 16-B lane stores; a direct store from the block layout would
            // spread every store instruction over ~40 cache lines (lanes 10 outputs apart)
            float2 y[2][LR];
            int mbs[2];
            {
                // both blocks of the thread in one pass over the tap rows (pp_block::run_multi);
                // clamped window starts only occur for outputs that are not stored
                const float2* xw[2];
#pragma unroll
                for (int r = 0; r < 2; ++r) {
                    const int q = q_lo + static_cast<int>(threadIdx.x) + r * static_cast<int>(blockDim.x);
                    const int pb = static_cast<int>(A.p_star) + MR * q;
                    xw[r] = w.lin + min(max(pb - HLR + lin_off, 0), idx_max);
                }
                PB::template run_multi<2>(xw, w.hpl, y);
            }
#pragma unroll
            for (int r = 0; r < 2; ++r) {
                const int q = q_lo + static_cast<int>(threadIdx.x) + r * static_cast<int>(blockDim.x);
                mbs[r] = static_cast<int>(A.m_star) + LR * q;
                if (q < q_hi) {
                    if (P.do_mix) {
                        float2 rot = phasor(P.ph0 + static_cast<double>(mbs[r]) * P.inc);
#pragma unroll
                        for (int k = 0; k < LR; ++k) {
                            y[r][k] = cmul(y[r][k], rot);
                            rot = cmul(rot, step1);
                        }
                    }
                }
            }
            __syncthreads();  // every lane's reads of lin are done
            float2* ob = w.lin;
#pragma unroll
            for (int r = 0; r < 2; ++r) {
                const int q = q_lo + static_cast<int>(threadIdx.x) + r * static_cast<int>(blockDim.x);
                if (q < q_hi) {
#pragma unroll
                    for (int k = 0; k < LR; ++k) {
                        const uint32_t m = static_cast<uint32_t>(mbs[r] + k);
                        if (m - m_lo < m_hi - m_lo) ob[m - m_lo] = y[r][k];
                    }
                }
            }
            __syncthreads();
            const uint32_t n = m_hi - m_lo;
            const uint32_t head = min(n, (reinterpret_cast<uintptr_t>(out + m_lo) & 15u) ? 1u : 0u);
            if (threadIdx.x < head) out[m_lo] = ob[0];
            const uint32_t npair = (n - head) / 2;
            float4* o4 = reinterpret_cast<float4*>(out + m_lo + head);
            for (uint32_t i = threadIdx.x; i < npair; i += blockDim.x) {
                const float2 a = ob[head + 2 * i], b = ob[head + 2 * i + 1];
                o4[i] = make_float4(a.x, a.y, b.x, b.y);
            }
            if (threadIdx.x == 0 && ((n - head) & 1u)) out[m_hi - 1] = ob[n - 1];
        } else
        for (int q = q_lo + static_cast<int>(threadIdx.x); q < q_hi; q += blockDim.x) {
            const int mb = static_cast<int>(A.m_star) + LR * q;
            const int pb = static_cast<int>(A.p_star) + MR * q;        // newest input of output mb
            const int idx = min(max(pb - HLR + lin_off, 0), idx_max);  // clamp: only unstored outputs clip
            float2 y[LR];
            PB::run(w.lin + idx, w.hpl, y);
            float2 rot = P.do_mix ? phasor(P.ph0 + static_cast<double>(mb) * P.inc) : make_float2(1.f, 0.f);
#pragma unroll
            for (int k = 0; k < LR; ++k) {
                const uint32_t m = static_cast<uint32_t>(mb + k);
                if (P.do_mix) {
                    y[k] = cmul(y[k], rot);
                    rot = cmul(rot, step1);
                }
                if (m - m_lo < m_hi - m_lo) out[m] = y[k];
            }
        }
    } else {
        for (uint32_t m = m_lo + threadIdx.x; m < m_hi; m += blockDim.x) {
            const uint64_t t = A.delay + uint64_t(m) * A.M;
            const int p = static_cast<int>(t / A.L);
            const uint32_t ph = static_cast<uint32_t>(t % A.L);
            float ar = 0.f, ai = 0.f;
            for (uint32_t d = 0; d <= w.hl; ++d) {
                const float hv = A.taps[ph + d * A.L];
                const float2 x = w.lin[p - static_cast<int>(d) + lin_off];
                ar = fmaf(x.x, hv, ar);
                ai = fmaf(x.y, hv, ai);
            }
            float2 y = make_float2(ar, ai);
            if (P.do_mix) y = cmul(y, phasor(P.ph0 + static_cast<double>(m) * P.inc));
            out[m] = y;
        }
    }
    if (w.last_run)
        for (uint32_t m = m_hi + threadIdx.x; m < A.S; m += blockDim.x) out[m] = make_float2(0.f, 0.f);
}

// ---- N_b_DFT_os = 1024: wavefront b owns slot b (symbol s0 + b)
template <int LR, int MR, int HLR>
__global__ void __launch_bounds__(TX_WAVE_MAX) tx_kernel_wave(tx_args A) {
    extern __shared__ __attribute__((aligned(16))) float2 smem[];
    uint32_t rc[16];  // cell codes of the wave's 16 bins per lane, loaded with the staging
    const tx_wg w = tx_setup<true>(A, smem, &rc);
    tx_zero_pads(w);
    const uint32_t b = threadIdx.x >> 6, lane = threadIdx.x & 63u;
    const uint32_t l = w.s0 + b;
    __syncthreads();
    if (b < w.nsl) {
        float2 v[16];
#pragma unroll
        for (int m = 0; m < 16; ++m) v[m] = w.bin(rc[m], lane + 64 * m, l);
        float2* xb = w.slot(l);  // the symbol's own slot (>= 1152 samples) is the exchange buffer
        wave_fft1024<+1>(v, xb, w.twl, lane);
        __builtin_amdgcn_wave_barrier();
        w.put_symbol(l, v, lane);
    }
    __syncthreads();
    tx_resample<LR, MR, HLR>(w);
}

// ---- streaming TX: N_b_DFT_os = 1024, L/M = 10/9 (os_min 1), CP 128, STF CP 1280.
// One wavefront walks one (packet, antenna, segment) through 1152-sample input pieces: the STF is
// pieces 0 and 1, DF symbol l is piece l + 1, later pieces are the zero flush. Per piece: cell
// mapping into registers -> wave_fft1024 -> the piece's cyclic-prefixed (STF: covered) samples into
// the wave's LDS buffer behind the 30-sample resampler carry -> 128 polyphase blocks (two per lane,
// output-major pp_direct, taps in SGPRs) + phase-continuous mixer -> outputs staged through the
// same buffer and stored as contiguous 16-B lane stores. The next symbol's PDC bytes (and their
// Gold sequence) are in flight while a piece is resampled. No workgroup barrier after the
// constellation load; the carry makes every symbol's history free (no extra FFT per run).
constexpr uint32_t TXS_WPG = 4;
constexpr uint32_t TXS_PIECE = 1152;                  // input samples per piece = 128 blocks of 9
constexpr uint32_t TXS_CARRY = 30;                    // inputs before the piece its first window reads
// float2 per wave: carry + piece + 2 pad slots (zero; the matrix-core blocks read 32 window inputs,
// the last block one slot past the piece, with a zero tap)
constexpr uint32_t TXS_BUF = TXS_CARRY + TXS_PIECE + 2;
constexpr uint32_t TXS_XB = 32;                       // FFT exchange / PDC byte staging offset
constexpr uint32_t TXS_WROW = 12;                     // beamforming row (8) + descrambled PCC bytes (32 B)
static_assert(TXS_XB + WFFT_XB <= TXS_CARRY + TXS_PIECE, "FFT exchange buffer must fit behind the carry");

// TXS_TXDIV1: transmit diversity where every antenna's W row holds one nonzero entry (TM5 codebook 0:
// W = I / 2): the antenna sends one stream of each SFBC pair, so a bin needs one PDC symbol and one
// complex product, not two (the other product is an exact zero in TXS_TXDIV)
// TXS_SM1: spatial multiplexing with one nonzero W entry per antenna row (TM6 codebook 0): the antenna
// sends one of the N_SS symbols of a cell, not a sum over all of them
enum { TXS_SISO = 0, TXS_TXDIV = 1, TXS_SM = 2, TXS_TXDIV1 = 3, TXS_SM1 = 4 };
// spatial multiplexing: N_SS streams of N_bps bits per cell put up to ~3 KB of PDC bytes into a symbol
// (4 streams of 64-QAM: 2.6 KB); its staging window is 4 KiB, the first KiB prefetched with the other
// modes' window, the rest loaded when the symbol starts (A.sb_chunks 1 KiB chunks, host-checked)
constexpr uint32_t TXS_SBW_SM = 4096;
static_assert(TXS_XB * 8 + TXS_SBW_SM <= (TXS_CARRY + TXS_PIECE) * 8, "staging window behind the carry");

__device__ __forceinline__ uint32_t txs_sym(uint32_t r, uint32_t N_DF) {  // symbol of piece r (N_DF+1: none)
    return r <= 1 ? 0u : (r - 1 <= N_DF ? r - 1 : N_DF + 1);
}

// MF: the polyphase blocks' form -- 0 VALU (pp_const), 1 matrix cores in split fp16 (three passes of
// v_mfma_f32_16x16x32_f16), 2 matrix cores in f32 (v_mfma_f32_16x16x4_f32, exact f32 products)
template <int MF>
__device__ __forceinline__ float2 txs_slot(float2 v) {  // buffer slot of a piece sample (MF 1: split fp16 words)
    if constexpr (MF == 1) return __builtin_bit_cast(float2, mf_split(v));
    else return v;
}

struct txs_wave {
    const tx_args* A;
    tx_pkt P;
    uint32_t pkt, ant, lane;
    float2 *buf, *wrow, *qtab;
    float* qlev;  // 256-QAM: level of the 4-bit index ((v >> 1) & 5) | ((v >> 4) & 10), the I part of qtab
    float2 w0;  // unscaled W[ant][0]: the STF bins carry scale_stf alone (tx.cpp:864-871)
    float2 wsel;  // TXS_TXDIV1: the antenna's one nonzero W entry, scale_df applied
    uint32_t tsel;  // TXS_TXDIV1: its stream
    const uint8_t *dpdc, *cpdc;
    uint32_t pdc_bytes;

    // first staged byte of symbol l (16-B aligned), PDC cells from pdc_off[l] & ~1 (SFBC partners)
    __device__ uint32_t stage_base(uint32_t l) const {
        // l is wave-uniform: a scalar load (constant address space), no vector-memory wait
        const uint32_t j0 = reinterpret_cast<const __attribute__((address_space(4))) uint32_t*>(reinterpret_cast<uintptr_t>(A->pdc_off))[l] & ~1u;
        return ((j0 * A->N_SS * A->N_bps) >> 3) & ~15u;
    }
    // 16-B chunk of the descrambled PDC bytes at byte g (zero beyond the packet) as the d-bit and
    // Gold-sequence words, XORed where they are used: the loads are a prefetch, not waited for here
    __device__ void chunk(uint32_t g, uint4& d, uint4& c) const {
        if (g + 16 <= pdc_bytes) {
            // the d-bit rows need not be 16-B aligned (byte stride): one unaligned dwordx4 load
            __builtin_memcpy(&d, dpdc + g, 16);
            // the Gold row is 16-B aligned device memory: a global (not flat) load, so it retires in the
            // vector-memory counter alone
            typedef uint32_t u4v __attribute__((ext_vector_type(4)));
            const u4v cv = *reinterpret_cast<const __attribute__((address_space(1))) u4v*>(reinterpret_cast<uintptr_t>(cpdc + g));
            c = make_uint4(cv.x, cv.y, cv.z, cv.w);
            return;
        }
        uint32_t w[4] = {0u, 0u, 0u, 0u};
        for (uint32_t i = 0; i < 16; ++i)
            if (g + i < pdc_bytes) w[i >> 2] |= uint32_t(dpdc[g + i] ^ cpdc[g + i]) << (8 * (i & 3));
        d = make_uint4(w[0], w[1], w[2], w[3]);
        c = make_uint4(0u, 0u, 0u, 0u);
    }
    // branch-free cell values: every source is read unconditionally at an in-bounds (masked)
    // index and the code type selects the result, so 16 bins per lane cost no divergent control
    // flow and no exec-mask SGPRs
    __device__ float2 pcc_sym(const uint8_t* pcb, uint32_t j) const {  // QPSK (TS 36.211 7.1.2) of PCC bits 2j, 2j+1
        const uint32_t bo = ((2 * j) >> 3) & 31u;
        const uint32_t q = (uint32_t(pcb[bo]) >> (6u - ((2 * j) & 7u))) & 3u;
        return make_float2((q & 2u) ? -0.70710678f : 0.70710678f, (q & 1u) ? -0.70710678f : 0.70710678f);
    }
    // SBW: bytes of the staging window (1 KiB; spatial multiplexing TXS_SM up to 4 KiB)
    template <bool Q8, uint32_t SBW = 1024>
    __device__ float2 pdc_sym(const uint8_t* sb, uint32_t ab, uint32_t s) const {
        if (Q8) {
            const uint32_t v = sb[(s - ab) & (SBW - 1)];
            if constexpr (experiment(XS_TX_NO_QTAB)) return make_float2(static_cast<float>(v), -static_cast<float>(v));
            if constexpr (experiment(XS_TX_QLEV)) {
                // 256-QAM is separable (36.211 7.1.5: I from bits 0, 2, 4, 6, Q from bits 1, 3, 5, 7, the
                // same level function): two reads of the 16-level table, conflict-free (16 words on 16
                // banks), instead of one 8-B read of the 256-entry table at a data-random index
                const uint32_t iI = ((v >> 1) & 5u) | ((v >> 4) & 10u), iQ = (v & 5u) | ((v >> 3) & 10u);
                return make_float2(qlev[iI], qlev[iQ]);
            }
            return qtab[v];
        }
        // byte bo of the window and its successor (the host keeps both inside it; the masks only bound
        // the LDS index)
        const uint32_t lb = s * A->N_bps - 8 * ab, bo = (lb >> 3) & (SBW - 1);
        return qtab[bits_of(sb[bo], sb[(bo + 1) & (SBW - 1)], lb, A->N_bps)];
    }
    // value of FFT bin n with cell code c in DF symbol l >= 1, scaled (tx.cpp:944-1116, 729-860, 862-871)
    // MODE: TXS_SISO (N_TS = 1), TXS_TXDIV (transmit diversity), TXS_SM (N_SS streams, PCC paired)
    template <int MODE, bool Q8, bool PCC>
    __device__ float2 bin_df(uint32_t c, const uint8_t* sb, uint32_t ab, const uint8_t* pcb) const {
        if constexpr (experiment(XS_TX_TRIVIAL_BINS)) return make_float2(__uint_as_float(c), 0.f);
        const uint32_t ty = c & CODE_MASK, j = c & CODE_J_MASK, pr = (c >> CODE_PAIR_SHIFT) & 0xFFu;
        if constexpr (MODE == TXS_TXDIV1 || MODE == TXS_SM1) {
            // the pair (tA, tB) of this cell: the antenna's stream is tA (x0 = symbol j) or tB (the
            // flipped partner, symbol j ^ 1) or neither; DRS cells carry their stream in tA. Sign flips
            // and the choice of result as bit masks: no control flow (the compiler turns value selects
            // around the table reads into exec-mask branches, which serialise the 16 bins' LDS reads).
            // TXS_SM1: a PDC cell carries the antenna's stream symbol j N_SS + tsel, unflipped (the PCC
            // stays transmit-diversity paired)
            constexpr bool SM1 = MODE == TXS_SM1;
            const bool ua = (pr & 0xFu) == tsel, ub = (pr >> 4) == tsel;
            const bool pdc = ty == CODE_PDC;
            const uint32_t jp = j ^ (ua ? 0u : 1u);
            const uint32_t js = SM1 && pdc ? j * A->N_SS + tsel : jp;
            float2 x = pdc_sym<Q8, SM1 ? TXS_SBW_SM : 1024u>(sb, ab, js);
            if constexpr (PCC) {
                const float2 px = pcc_sym(pcb, jp);
                x = ty == CODE_PCC ? px : x;
            }
            const uint32_t nf = (ua || (SM1 && pdc)) ? 0u : 0x80000000u;  // the partner's flip (-re, +im) / (+re, -im)
            const uint32_t fx = (j & 1u) ? 0u : nf, fy = (j & 1u) ? nf : 0u;
            x = make_float2(__uint_as_float(__float_as_uint(x.x) ^ fx), __uint_as_float(__float_as_uint(x.y) ^ fy));
            const float2 v = cmul(wsel, x);
            const uint32_t ds = (j & 8u) ? 0x80000000u : 0u;  // DRS value +-1 times the W entry
            const float2 d = make_float2(__uint_as_float(__float_as_uint(wsel.x) ^ ds), __uint_as_float(__float_as_uint(wsel.y) ^ ds));
            const bool kv = (pdc && (SM1 || ua || ub)) || (PCC && ty == CODE_PCC && (ua || ub)), kd = ty == CODE_DRS && ua;
            const uint32_t mv = 0u - static_cast<uint32_t>(kv), md = 0u - static_cast<uint32_t>(kd);
            return make_float2(__uint_as_float((__float_as_uint(v.x) & mv) | (__float_as_uint(d.x) & md)),
                               __uint_as_float((__float_as_uint(v.y) & mv) | (__float_as_uint(d.y) & md)));
        }
        float2 x0 = pdc_sym<Q8>(sb, ab, j);
        float2 v, wa_drs = make_float2(0.f, 0.f);
        if (MODE == TXS_SISO) {  // SISO (N_SS = 1): PCC and PDC alike
            if (PCC && ty == CODE_PCC) x0 = pcc_sym(pcb, j);
            v = cmul(wrow[0], x0);
        } else if (MODE == TXS_TXDIV || (PCC && ty == CODE_PCC)) {
            // transmit diversity pair (transmit_diversity_precoding.cpp:37-75): the PCC always,
            // the PDC in the transmit-diversity modes
            float2 x1 = pdc_sym<Q8>(sb, ab, j ^ 1u);
            if (PCC && ty == CODE_PCC) {
                x0 = pcc_sym(pcb, j);
                x1 = pcc_sym(pcb, j ^ 1u);
            }
            x1 = (j & 1u) ? make_float2(x1.x, -x1.y) : make_float2(-x1.x, x1.y);
            v = cadd(cmul(wrow[pr & 0xFu], x0), cmul(wrow[pr >> 4], x1));
            if (MODE == TXS_TXDIV) wa_drs = wrow[pr & 0xFu];
        } else {
            v = make_float2(0.f, 0.f);
            for (uint32_t ss = 0; ss < A->N_SS; ++ss) v = cadd(v, cmul(wrow[ss], pdc_sym<Q8, TXS_SBW_SM>(sb, ab, j * A->N_SS + ss)));
        }
        // DRS codes carry their stream in the pair field: in transmit diversity the pair's first W
        // entry above is the DRS weight (no second read)
        const float2 d = cscale(MODE == TXS_TXDIV ? wa_drs : wrow[j & 7u], (j & 8u) ? -1.f : 1.f);
        v = ty == CODE_DRS ? d : v;
        v = (ty == CODE_PDC || ty == CODE_DRS || (PCC && ty == CODE_PCC)) ? v : make_float2(0.f, 0.f);
        return v;  // wrow carries scale_df (one multiply per W entry instead of two per bin)
    }
    // TXS_TXDIV1 / TXS_SM1 from the antenna stream's own code table (ctx.cpp, kernels.hpp OH_*):
    // the pair tests, the partner index and its flips were resolved on the host, so a bin is one
    // table read, the flips as sign XORs and one complex product -- a DRS cell as the point (+-1, 0)
    // (its sign an OH_FX flip), an empty cell as a zero W entry (bin_df's TXS_TXDIV1 branch, equal
    // up to the sign of zero). Against the pair-testing form: TX 17.07 -> 16.66 ms per 16384 slots
    template <bool Q8, bool PCC, uint32_t SBW>
    __device__ float2 bin_oh(uint32_t c, const uint8_t* sb, uint32_t ab, const uint8_t* pcb) const {
        if constexpr (experiment(XS_TX_TRIVIAL_BINS)) return make_float2(__uint_as_float(c), 0.f);
        const uint32_t ty = c & CODE_MASK, js = c & CODE_J_MASK;
        float2 x = pdc_sym<Q8, SBW>(sb, ab, js);
        if constexpr (PCC) {
            const float2 px = pcc_sym(pcb, js);
            x = ty == CODE_PCC ? px : x;
        }
        const bool kd = ty == CODE_DRS, kz = ty == 0u;
        x = make_float2(kd ? 1.f : x.x, kd ? 0.f : x.y);
        x = make_float2(__uint_as_float(__float_as_uint(x.x) ^ ((c << 11) & 0x80000000u)),
                        __uint_as_float(__float_as_uint(x.y) ^ ((c << 10) & 0x80000000u)));
        return cmul(make_float2(kz ? 0.f : wsel.x, kz ? 0.f : wsel.y), x);
    }
    // STF bin n (stf.cpp:185-285 values, STF scaling)
    __device__ float2 bin_stf(uint32_t c, uint32_t n) const {
        const uint32_t N = A->N_occ;
        const uint32_t k = n <= N / 2 ? N / 2 + n : n - A->off_lower;
        const float2 v = cscale(cmul(w0, A->stf[min(k, N)]), P.scale_stf);
        return (c & CODE_MASK) == CODE_STF ? v : make_float2(0.f, 0.f);
    }
};

// Outputs m0 .. m0 + N - 1, staged in buf[0, N), to the wave's output row as contiguous 16-B lane
// stores of the output pairs (m, m + 1), m even (so no pair straddles 0 or S, both even); with an
// odd m0 the first and last output go alone. Branch-free: lanes out of [0, S) store past the
// descriptor's range (dropped by the hardware) and outputs >= n_keep are zero, so every call issues
// the same stores -- the next piece's input waits stay counted (vmcnt(n)), not a drain of them.
// inner (uniform): [m0, m0 + N) inside [0, n_keep), no per-element range work.
// SHIFT: output i staged at buf[i + head], so that every pair sits on a 16-B boundary (one b128 read,
// conflict-free, instead of two b64 reads at a 16-B lane stride: 2-way conflicts)
template <int N, bool SHIFT = false>
__device__ __forceinline__ void txs_emit(const float2* buf, __amdgpu_buffer_rsrc_t orsrc, uint32_t head, uint32_t lid,
                                         int m0, int S, int n_keep) {
    constexpr int K = (N / 2 + 63) / 64;
    const bool inner = m0 >= 0 && m0 + N <= n_keep;
    const uint32_t sh = SHIFT ? head : 0u;
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const uint32_t e = head + 2 * (lid + 64 * k);  // local output pair (e, e + 1)
        // clamped to the last pair of e's parity (N even), so that SHIFT keeps ec + sh even
        const uint32_t ec = min(e, static_cast<uint32_t>(N - 2) - (SHIFT ? head : 0u));
        float2 a, b;
        if constexpr (SHIFT) {
            const float4 p = *reinterpret_cast<const float4*>(buf + ec + sh);
            a = make_float2(p.x, p.y);
            b = make_float2(p.z, p.w);
        } else {
            a = buf[ec];
            b = buf[ec + 1];
        }
        const int m = m0 + static_cast<int>(e);
        mf_u4 v = {__float_as_uint(a.x), __float_as_uint(a.y), __float_as_uint(b.x), __float_as_uint(b.y)};
        uint32_t off = static_cast<uint32_t>(m) * 8u;
        if ((k + 1) * 128 >= N || !inner) {  // the last store (partly filled with an odd m0), or a packet edge
            const bool ok = e <= static_cast<uint32_t>(N - 2) && m >= 0 && m < S;
            const bool ka = m < n_keep, kb = m + 1 < n_keep;
            v = mf_u4{ka ? v.x : 0u, ka ? v.y : 0u, kb ? v.z : 0u, kb ? v.w : 0u};
            off = ok ? off : 0x80000000u;
        }
        // nontemporal (cache policy nt): the samples are written once and read by a later launch
        __builtin_amdgcn_raw_buffer_store_b128(v, orsrc, off, 0, 2);
    }
    {  // odd m0: the first and last output alone (lanes 0, 1)
        const uint32_t e = lid == 0 ? 0u : static_cast<uint32_t>(N - 1);
        const float2 a = buf[e + sh];
        const int m = m0 + static_cast<int>(e);
        const bool ok = head && lid < 2 && m >= 0 && m < S;
        const float2 ov = m < n_keep ? a : make_float2(0.f, 0.f);
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(mf_u2, ov), orsrc, ok ? static_cast<uint32_t>(m) * 8u : 0x80000000u, 0, 0);
    }
}

template <int LR, int MR, int HLR, int MODE, bool Q8, int MF>
#ifndef DNRP_TX_IMAJ
#define DNRP_TX_IMAJ 0  // 1: the polyphase windows input-major from LDS (pp_const::run_imaj; 96 VGPRs against
                        // 120 at the same LDS-bound 16 waves per CU): TX 17.13 / 17.07 vs 16.99 / 16.99 ms, off
#endif
#ifndef DNRP_TX_WPE
#define DNRP_TX_WPE 4  // waves per SIMD (5: 96 VGPRs + 120 B/lane of spills)
#endif
__global__ void __launch_bounds__(64 * TXS_WPG) __attribute__((amdgpu_waves_per_eu(DNRP_TX_WPE))) tx_stream_kernel(tx_args A, uint32_t n) {
    using PD = pp_direct<LR, MR, HLR>;
    static_assert(PD::W == TXS_CARRY + 1, "carry = window - 1");
    static_assert(taps_tx_10_9::L == LR && taps_tx_10_9::M == MR && taps_tx_10_9::HL == HLR, "generated taps");
    extern __shared__ __attribute__((aligned(16))) float2 smem[];
    float2* qtab = smem;  // [256] per workgroup (256-QAM: the 16 levels in its first 8 slots)
    // wave index made provably uniform: everything derived from it (packet, segment, loop bounds,
    // pointers) stays in SGPRs and the piece loop is not divergent control flow
    const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63u;
    if constexpr (Q8 && experiment(XS_TX_QLEV)) {
        // level i = re of the table entry whose I bits (0, 2, 4, 6) give index i and Q bits are 0
        if (threadIdx.x < 16) {
            const uint32_t i = threadIdx.x;
            const uint32_t v = ((i & 8u) << 4) | ((i & 2u) << 4) | ((i & 4u) << 1) | ((i & 1u) << 1);
            reinterpret_cast<float*>(qtab)[i] = A.qam[v].x;
        }
    } else {
        const uint32_t nq = 1u << A.N_bps;
        for (uint32_t i = threadIdx.x; i < nq; i += blockDim.x) qtab[i] = A.qam[i];
    }
    txs_wave T;
    T.A = &A;
    T.lane = lane;
    T.qtab = qtab;
    T.qlev = reinterpret_cast<float*>(qtab);
    T.buf = smem + 256 + wv * (TXS_BUF + TXS_WROW);
    T.wrow = T.buf + TXS_BUF;
    const uint32_t gw = blockIdx.x * TXS_WPG + wv;
    T.ant = gw % A.N_TX;
    const uint32_t seg = (gw / A.N_TX) % A.n_seg;
    T.pkt = gw / (A.N_TX * A.n_seg);
    const bool live = T.pkt < n;
    uint8_t* pcb = reinterpret_cast<uint8_t*>(T.wrow + 8);
    if (live) {
        T.P = A.pk[T.pkt];
        // the W row pre-scaled by the data-field scaling (tx.cpp:582-594, 864-871)
        if (lane < A.N_TS) T.wrow[lane] = cscale(A.W[(T.P.codebook * A.N_TX + T.ant) * A.N_TS + lane], T.P.scale_df);
        T.w0 = A.W[(T.P.codebook * A.N_TX + T.ant) * A.N_TS];
        if constexpr (MODE == TXS_TXDIV1 || MODE == TXS_SM1) {  // the row's nonzero entry (host-checked: exactly one)
            T.tsel = 0;
            for (uint32_t t = 0; t < A.N_TS; ++t)
                if (nz(A.W[(T.P.codebook * A.N_TX + T.ant) * A.N_TS + t])) T.tsel = t;
            T.wsel = cscale(A.W[(T.P.codebook * A.N_TX + T.ant) * A.N_TS + T.tsel], T.P.scale_df);
        }
        if (lane < 32) pcb[lane] = lane < 25 ? static_cast<uint8_t>(A.pcc_d[size_t(T.pkt) * 25 + lane] ^ A.pcc_seq[lane]) : 0u;
    }
    __syncthreads();  // the only workgroup barrier: qtab / wrow visible
    if (!live) return;
    const uint32_t r_a = seg * A.piece_per_seg, r_b = min(r_a + A.piece_per_seg, A.n_pieces);
    if (r_a >= r_b) return;
    T.dpdc = A.pdc_d + size_t(T.pkt) * A.pdc_stride;
    T.cpdc = T.P.pdc_seq;
    T.pdc_bytes = (A.G + 7) / 8;
    float2* buf = T.buf;
    float2* out = reinterpret_cast<float2*>(A.out) + size_t(T.pkt * A.N_TX + T.ant) * A.S;
    uint8_t* sb = reinterpret_cast<uint8_t*>(buf + TXS_XB);
    // block grid: piece r holds blocks q = q0 + 128 r + (lane + 64 b), window at buf[base0 + 9 (lane + 64 b)]
    const int qlo0 = -static_cast<int>((A.p_star + 8) / MR);  // ceil((0 - p_star - 8) / 9)
    const uint32_t base0 = static_cast<uint32_t>(static_cast<int>(A.p_star) + MR * qlo0 + 8);
    const int mfirst0 = static_cast<int>(A.m_star) + LR * qlo0;  // first output of piece 0
    const float2 step1 = T.P.do_mix ? phasor(T.P.inc) : make_float2(1.f, 0.f);
    // the FFT's two lane twiddles, loaded once (wave_fft1024_rt)
    const float2 tw1 = wfft_tw<+1>(A.tw, 4 * (lane & 15u)), twl = wfft_tw<+1>(A.tw, lane);
    // MF: the lane's block taps for the matrix cores (polyphase.hpp mf_blocks), split fp16 hi / lo:
    // B[i = 8 (lane >> 4) + j][c = lane & 15] = h[ph_c + (HL + o_c - i) L] inside output c's span
    mf_h8 gh, gl;
    float g32[8];  // MF 2: B[k = 4 s + (lane >> 4)][c = lane & 15] of k-step s, f32
    float2 step10 = make_float2(1.f, 0.f), step160 = step10;
    if constexpr (MF != 0) {
        const uint32_t c = lane & 15u, hq = lane >> 4;
        const int o = static_cast<int>(MR * c) / LR, ph = static_cast<int>(MR * c) % LR;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            if constexpr (MF == 1) {
                const int d = HLR + o - static_cast<int>(8 * hq) - j;
                const float t = (c < LR && d >= 0 && d <= HLR) ? A.taps[ph + d * LR] : 0.f;
                const mf_h2 hv = __builtin_amdgcn_cvt_pkrtz(t, 0.f);
                gh[j] = hv.x;
                gl[j] = __builtin_amdgcn_cvt_pkrtz(t - static_cast<float>(hv.x), 0.f).x;
            } else {
                const int d = HLR + o - static_cast<int>(4 * j + hq);
                g32[j] = (c < LR && d >= 0 && d <= HLR) ? A.taps[ph + d * LR] : 0.f;
            }
        }
        if (T.P.do_mix) {
            step10 = phasor(10.0 * T.P.inc);
            step160 = phasor(160.0 * T.P.inc);
        }
        if (lane < 2) buf[TXS_CARRY + TXS_PIECE + lane] = make_float2(0.f, 0.f);
    }
    if (seg == 0)  // outputs before piece 0's first block see only zero input
        for (int m = lane; m < mfirst0; m += 64) out[m] = make_float2(0.f, 0.f);
    const uint32_t r_start = r_a > 0 ? r_a - 1 : 0;
    // the wave's output row as a buffer: out-of-range offsets are dropped by the range check
    const __amdgpu_buffer_rsrc_t orsrc = __builtin_amdgcn_make_buffer_rsrc(out, 0, static_cast<int>(A.S * 8u), 0x00020000);
    if (r_a == 0 && lane < TXS_CARRY) buf[lane] = make_float2(0.f, 0.f);
    // PDC bytes of the first symbol
    const uint32_t l_cur = txs_sym(r_start, A.N_DF);
    uint4 pre = make_uint4(0u, 0u, 0u, 0u), prc = pre;
    if (l_cur >= 1 && l_cur <= A.N_DF) T.chunk(T.stage_base(l_cur) + 16 * lane, pre, prc);
    // cell codes of the piece's 16 bins per lane, loaded one piece ahead: issued before the piece's
    // output stores, so waiting for them never waits for those stores (vmcnt retires in order)
    uint32_t cd[16];
    // one-hot W rows: the antenna stream's own code table (bin_oh)
    constexpr bool OH = MODE == TXS_TXDIV1 || MODE == TXS_SM1;
    const uint32_t* ctab = OH ? A.code_oh + size_t(T.tsel) * (A.N_DF + 1) * 1024 : A.code_bin;
    auto load_codes = [&](uint32_t rr, uint32_t ln) {
        const uint32_t ls = txs_sym(rr, A.N_DF);
        const uint4* crow = reinterpret_cast<const uint4*>(ctab + size_t(min(ls, A.N_DF)) * 1024);
#pragma unroll
        for (int j = 0; j < 4; ++j) {  // the codes of bins ln + 64 m, m = 4 j .. 4 j + 3, in one load
            const uint4 c = crow[64 * j + ln];
            cd[4 * j] = c.x;
            cd[4 * j + 1] = c.y;
            cd[4 * j + 2] = c.z;
            cd[4 * j + 3] = c.w;
        }
    };
    load_codes(r_start, lane);
    // the next piece's inputs (cell codes, PDC bytes of its symbol), issued once the FFT is done:
    // pre / prc / cd are redefined on every path here, so none of them is live across the FFT
    auto prefetch_next = [&](uint32_t r, uint32_t lid) {
        load_codes(r + 1, lid);
        const uint32_t l = txs_sym(r, A.N_DF), ln = txs_sym(r + 1, A.N_DF);
        if (r + 1 < r_b && ln != l && ln >= 1 && ln <= A.N_DF) {
            T.chunk(T.stage_base(ln) + 16 * lid, pre, prc);
        } else {
            pre = make_uint4(0u, 0u, 0u, 0u);
            prc = pre;
        }
    };
    // drain the prologue's loads: the loop header then sees only the back edge's pending loads and
    // stores, and the code-row wait stays counted (the in-loop loads precede the piece's stores)
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
    for (uint32_t r = r_start; r < r_b; ++r) {
        // lid index opaque per piece: lid-dependent addresses are recomputed in the loop instead of
        // being hoisted out of it as dozens of 64-bit VGPR pairs (loop-invariant code motion)
        uint32_t lid = lane;
        asm volatile("" : "+v"(lid));
        const uint32_t l = txs_sym(r, A.N_DF);
        float2 v[16];
        const bool real = l <= A.N_DF;
        if (real) {
            // stage this symbol's bytes, prefetch the next symbol's
            const uint32_t ab = (l >= 1) ? T.stage_base(l) : 0u;
            if (l >= 1) reinterpret_cast<uint4*>(sb)[lid] = make_uint4(pre.x ^ prc.x, pre.y ^ prc.y, pre.z ^ prc.z, pre.w ^ prc.w);
            if constexpr (MODE == TXS_SM || MODE == TXS_SM1) {
                if (l >= 1)
                    for (uint32_t c = 1; c < A.sb_chunks; ++c) {  // the window's other KiBs, not prefetched
                        uint4 d, e;
                        T.chunk(ab + 1024 * c + 16 * lid, d, e);
                        reinterpret_cast<uint4*>(sb)[64 * c + lid] = make_uint4(d.x ^ e.x, d.y ^ e.y, d.z ^ e.z, d.w ^ e.w);
                    }
            }
            __builtin_amdgcn_wave_barrier();
            if (l == 0) {
#pragma unroll
                for (int m = 0; m < 16; ++m) v[m] = T.bin_stf(cd[m], lid + 64 * m);
            } else if ((l < 32) && ((A.pcc_syms >> l) & 1u)) {
#pragma unroll
                for (int m = 0; m < 16; ++m) {
                    if constexpr (OH) v[m] = T.template bin_oh<Q8, true, MODE == TXS_SM1 ? TXS_SBW_SM : 1024u>(cd[m], sb, ab, pcb);
                    else v[m] = T.template bin_df<MODE, Q8, true>(cd[m], sb, ab, pcb);
                }
            } else {
#pragma unroll
                for (int m = 0; m < 16; ++m) {
                    // two groups of 8 bins: the table reads of 8 bins in flight at a time (all 16 spill)
                    if (OH && m == 8) __builtin_amdgcn_sched_barrier(0);
                    if constexpr (OH) v[m] = T.template bin_oh<Q8, false, MODE == TXS_SM1 ? TXS_SBW_SM : 1024u>(cd[m], sb, ab, pcb);
                    else v[m] = T.template bin_df<MODE, Q8, false>(cd[m], sb, ab, pcb);
                }
            }
            __builtin_amdgcn_wave_barrier();
            {
                // two lane twiddles held over the loop (27 hoisted ones would cost 54 VGPRs)
                // laundered: keeps LICM from hoisting the twiddle powers derived from them
                float2 w1 = tw1, wl = twl;
                asm volatile("" : "+v"(w1.x), "+v"(w1.y), "+v"(wl.x), "+v"(wl.y));
                wave_fft1024_rt<+1>(v, buf + TXS_XB, w1, wl, lid);
            }
            __builtin_amdgcn_wave_barrier();
            // piece samples: sample i of the symbol is X[(i - cp) mod 1024] (STF: times the cover)
            if (l >= 1) {  // DF symbol (CP 128): sample nn + 128, CP copies of the last 128 (m >= 14)
#pragma unroll
                for (int m = 0; m < 16; ++m) {
                    const float2 sv = txs_slot<MF>(v[m]);
                    buf[TXS_CARRY + 128 + lid + 64 * m] = sv;
                    if (m >= 14) buf[TXS_CARRY + lid + 64 * (m - 14)] = sv;
                }
            } else {  // STF (CP 1280, covered): piece r holds samples [1152 r, 1152 r + 1152)
                const uint32_t cp = A.STF_CP, len = cp + 1024, i0 = r == 1 ? TXS_PIECE : 0u;
#pragma unroll
                for (int m = 0; m < 16; ++m) {
                    const uint32_t nn = lid + 64 * m;
                    for (uint32_t i = (nn + cp) & 1023u; i < len; i += 1024)
                        if (i - i0 < TXS_PIECE) buf[TXS_CARRY + i - i0] = txs_slot<MF>(cscale(v[m], cover_sign(min(i / A.pattern_len, 8u))));
                }
            }
        } else {
            for (uint32_t i = lid; i < TXS_PIECE; i += 64) buf[TXS_CARRY + i] = make_float2(0.f, 0.f);
        }
        __builtin_amdgcn_wave_barrier();
        float2 creg = make_float2(0.f, 0.f);
        if (MF != 0 && r >= r_a) {
            // 8 groups of 16 blocks on the matrix cores (lane: output phase c = lid & 15 of blocks
            // 16 g + 4 (lid >> 4) + q, phases >= 10 idle), each group's 160 outputs transposed through
            // LDS slots [0, 160) -- dead once the windows of group 1 are read (they start at slot
            // base0 + 144) -- into contiguous 16-B lane stores: group 0 is staged after group 1 is computed
            const uint32_t c = lid & 15u, hq = lid >> 4;
            const uint2* slots = reinterpret_cast<const uint2*>(buf) + base0 + MR * c + 8 * hq;
            const int mrow = mfirst0 + static_cast<int>(1280 * r);
            const int mb = mrow + static_cast<int>(40 * hq + c);
            const uint32_t head = static_cast<uint32_t>(mfirst0) & 1u;  // pairs start at even outputs
            float2 rot = make_float2(1.f, 0.f);
            if (T.P.do_mix) rot = phasor(T.P.ph0 + static_cast<double>(mb) * T.P.inc);
            prefetch_next(r, lid);
            auto group = [&](int g, float2 (&y)[4]) {
                mf_f4 cr, ci;
                if constexpr (MF == 1) {
                    uint2 w[8];
#pragma unroll
                    for (int j = 0; j < 8; ++j) w[j] = slots[MR * 16 * g + j];
                    mf_blocks(w, gh, gl, cr, ci);
                } else {
                    // A[block c][input k = 4 s + hq] of k-step s: one float2 slot per lane and step
                    const float2* wb = buf + base0 + MR * (16 * g + c) + hq;
                    cr = mf_f4{0.f, 0.f, 0.f, 0.f};
                    ci = cr;
#pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        const float2 xv = wb[4 * j];
                        cr = __builtin_amdgcn_mfma_f32_16x16x4f32(xv.x, g32[j], cr, 0, 0, 0);
                        ci = __builtin_amdgcn_mfma_f32_16x16x4f32(xv.y, g32[j], ci, 0, 0, 0);
                    }
                }
                float2 rr = rot;
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    y[q] = make_float2(cr[q], ci[q]);
                    if (T.P.do_mix) {
                        y[q] = cmul(y[q], rr);
                        rr = cmul(rr, step10);
                    }
                }
                if (T.P.do_mix) rot = cmul(rot, step160);
            };
            // branch-free stores: out-of-range lanes get an offset past the descriptor's range, which
            // the hardware drops -- a fixed store count per piece, so the next piece's input waits are
            // counted ones (vmcnt(n)), not a drain of this piece's stores
            auto stage = [&](int g, const float2 (&y)[4]) {
                if (c < LR) {
#pragma unroll
                    for (int q = 0; q < 4; ++q) buf[10 * (4 * hq + q) + c] = y[q];
                }
                __builtin_amdgcn_wave_barrier();
                txs_emit<160>(buf, orsrc, head, lid, mrow + 160 * g, static_cast<int>(A.S), static_cast<int>(A.n_keep));
                __builtin_amdgcn_wave_barrier();
            };
            // one group ahead: group g + 1's matrix work is in flight while group g is staged (and
            // group 0 waits for group 1's windows to be read before its slots are reused)
            float2 y0[4], y1[4];
            group(0, y0);
#pragma unroll
            for (int g = 0; g < 8; g += 2) {
                group(g + 1, y1);
                stage(g, y0);
                if (g + 2 < 8) group(g + 2, y0);
                stage(g + 1, y1);
            }
            if (lid < TXS_CARRY) creg = buf[TXS_PIECE + lid];
        } else if (r >= r_a) {
            float2 y[2][LR];
#pragma unroll
            for (int b = 0; b < 2; ++b) {
                __builtin_amdgcn_sched_barrier(0);  // one window live at a time
                if constexpr (DNRP_TX_IMAJ) {  // window input-major from LDS (8-B reads: MR odd)
                    pp_const<taps_tx_10_9>::run_imaj<false>(buf + base0 + MR * (lid + 64 * b), y[b]);
                } else {
                    float2 xv[PD::W];
                    PD::template load<false>(buf + base0 + MR * (lid + 64 * b), xv);
                    pp_const<taps_tx_10_9>::run(xv, y[b]);
                }
                if (T.P.do_mix) {
                    const int mb = mfirst0 + static_cast<int>(1280 * r) + LR * static_cast<int>(lid + 64 * b);
                    float2 rot = phasor(T.P.ph0 + static_cast<double>(mb) * T.P.inc);
#pragma unroll
                    for (int k = 0; k < LR; ++k) {
                        y[b][k] = cmul(y[b][k], rot);
                        rot = cmul(rot, step1);
                    }
                }
            }
            prefetch_next(r, lid);
            __builtin_amdgcn_wave_barrier();
            if (lid < TXS_CARRY) creg = buf[TXS_PIECE + lid];
            __builtin_amdgcn_wave_barrier();
            const uint32_t head = static_cast<uint32_t>(mfirst0) & 1u;  // packet-uniform
#pragma unroll
            for (int b = 0; b < 2; ++b) {
                // the block's outputs as 16-B pairs at even slots (a lane's 10 outputs: 8 dwords x 10
                // apart, conflict-free in every 8-lane group; 8-B stores at a 10-slot stride are 2-way)
                static_assert(LR % 2 == 0, "pairs of outputs");
                float2* dst = buf + head + LR * lid;
                auto st4 = [&](int k) { *reinterpret_cast<float4*>(dst + k) = make_float4(y[b][k].x, y[b][k].y, y[b][k + 1].x, y[b][k + 1].y); };
                if (head == 0) {
#pragma unroll
                    for (int k = 0; k < LR; k += 2) st4(k);
                } else {
                    dst[0] = y[b][0];
#pragma unroll
                    for (int k = 1; k + 1 < LR; k += 2) st4(k);
                    dst[LR - 1] = y[b][LR - 1];
                }
                __builtin_amdgcn_wave_barrier();
                txs_emit<640, true>(buf, orsrc, static_cast<uint32_t>(mfirst0) & 1u, lid, mfirst0 + static_cast<int>(1280 * r) + 640 * b,
                              static_cast<int>(A.S), static_cast<int>(A.n_keep));
                __builtin_amdgcn_wave_barrier();
            }
        } else {  // the history piece ahead of the segment: nothing to store
            prefetch_next(r, lid);
            // drained here so the loop header's merge keeps the storing path's counted wait
            __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
            if (lid < TXS_CARRY) creg = buf[TXS_PIECE + lid];
        }
        __builtin_amdgcn_wave_barrier();
        if (lid < TXS_CARRY) buf[lid] = creg;
        __builtin_amdgcn_wave_barrier();
    }
    if (r_b == A.n_pieces) {  // slot tail (GI and beyond): zeros
        const int m_end = mfirst0 + static_cast<int>(1280 * A.n_pieces);
        for (int m = max(m_end, 0) + static_cast<int>(lane); m < static_cast<int>(A.S); m += 64) out[m] = make_float2(0.f, 0.f);
    }
}

bool tx_stream_taps_match(const float* h, size_t n) {  // run-time taps == compiled-in taps, bitwise
    if (n != static_cast<size_t>(taps_tx_10_9::N)) return false;
    for (size_t i = 0; i < n; ++i)
        if (__builtin_bit_cast(uint32_t, h[i]) != __builtin_bit_cast(uint32_t, taps_tx_10_9::h[i])) return false;
    return true;
}

size_t tx_stream_lds() { return (256 + TXS_WPG * (TXS_BUF + TXS_WROW)) * sizeof(float2); }

// ---- other FFT sizes: workgroup-wide batched Stockham FFT
template <int LR, int MR, int HLR>
__global__ void __launch_bounds__(TX_THREADS) tx_kernel(tx_args A) {
    extern __shared__ __attribute__((aligned(16))) float2 smem[];
    const tx_wg w = tx_setup<false>(A, smem);
    float2* bufB = w.lin + A.lin_len;
    const uint32_t Nd = w.Nd;
    // the last IFFT pass must read bufB (it writes lin): place the grid accordingly
    const uint32_t npass = fft_num_passes(A.plan);
    float2* gin = ((npass - 1) % 2 == 0) ? bufB : w.lin;
    float2* gout = (gin == w.lin) ? bufB : w.lin;
    uint32_t rc[TX_BLOCK_SLOTS][TX_BIN_REG];
#pragma unroll
    for (uint32_t b = 0; b < TX_BLOCK_SLOTS; ++b)
#pragma unroll
        for (uint32_t r = 0; r < TX_BIN_REG; ++r)
            rc[b][r] = b < w.nsl ? w.code(w.s0 + b, threadIdx.x + r * TX_THREADS) : 0u;
    __syncthreads();
#pragma unroll
    for (uint32_t b = 0; b < TX_BLOCK_SLOTS; ++b) {
        if (b >= w.nsl) break;
#pragma unroll
        for (uint32_t r = 0; r < TX_BIN_REG; ++r) {
            const uint32_t n = threadIdx.x + r * TX_THREADS;
            if (n >= Nd) break;
            gin[b * Nd + n] = w.bin(rc[b][r], n, w.s0 + b);
        }
    }
    __syncthreads();
    fft_store<+1>(gin, gout, w.twl, A.plan, w.nsl, [&](uint32_t b, uint32_t n, float2 v) { w.put(w.s0 + b, n, v); });
    // the IFFT used the whole of lin as scratch: pads are zeroed after it
    tx_zero_pads(w);
    __syncthreads();
    tx_resample<LR, MR, HLR>(w);
}

// ---- N_b_DFT_os > 1024: symbol-parallel through a DECT-rate scratch in HBM. An 8192-point
// symbol's ping-pong buffers alone take 128 KiB of LDS, so the block path's runs (K symbols plus the
// history symbol, resampled in LDS) do not fit; here workgroup (packet, antenna, symbol l) builds the
// bins, runs the IFFT (twiddles from the L2) and stores the cyclic-prefixed, STF-covered symbol
// into A.big, then one thread per hw-rate output runs the FIR over the scratch (tx_resample's run-time
// tap form: inputs before the packet and past its flush samples are the zero history), the mixer and
// the GI / slot-tail zeros (tx.cpp:679-714).
constexpr uint32_t TX_BIG_THREADS = 512;

__global__ void __launch_bounds__(TX_BIG_THREADS) tx_big_sym_kernel(tx_args A) {
    extern __shared__ __attribute__((aligned(16))) float2 smem[];
    const uint32_t l = blockIdx.x % (A.N_DF + 1), pa = blockIdx.x / (A.N_DF + 1);
    tx_wg w{};
    w.A = &A;
    w.pkt = pa / A.N_TX;
    w.ant = pa % A.N_TX;
    w.P = A.pk[w.pkt];
    w.Nd = A.plan.N;
    w.N = A.N_occ;
    w.Nf = w.N + 1;
    w.hl = A.hl;
    w.len0 = A.STF_CP + w.Nd;
    w.lenD = A.CP + w.Nd;
    float2* fa = smem;
    float2* fb = smem + w.Nd;
    w.qtab = fb + w.Nd;
    w.pccs = w.qtab + 256;
    w.wrow = w.pccs + 98;
    w.dpdc = A.pdc_d + size_t(w.pkt) * A.pdc_stride;
    w.cpdc = w.P.pdc_seq;
    w.pdc_bytes = (A.G + 7) / 8;  // A.stage_bytes = 0: PDC bytes straight from HBM
    const uint8_t* dpcc = A.pcc_d + size_t(w.pkt) * 25;
    for (uint32_t i = threadIdx.x; i < (1u << A.N_bps); i += blockDim.x) w.qtab[i] = A.qam[i];
    for (uint32_t j = threadIdx.x; j < 98; j += blockDim.x) {
        const uint32_t bo = (2 * j) >> 3;
        w.pccs[j] = A.qpsk[bits_of(dpcc[bo] ^ A.pcc_seq[bo], 0u, 2 * j, 2)];
    }
    for (uint32_t i = threadIdx.x; i < A.N_TS; i += blockDim.x) w.wrow[i] = A.W[(w.P.codebook * A.N_TX + w.ant) * A.N_TS + i];
    __syncthreads();
    for (uint32_t n = threadIdx.x; n < w.Nd; n += blockDim.x) fa[n] = w.bin(w.code(l, n), n, l);
    __syncthreads();
    float2* dst = A.big + size_t(pa) * A.big_len + w.bsym(l);
    const uint32_t Nd = w.Nd;
    fft_store<+1>(fa, fb, A.tw, A.plan, 1, [&](uint32_t, uint32_t n, float2 v) {
        if (l == 0) {
            for (uint32_t i = A.STF_CP + n;; i -= Nd) {  // the STF CP may exceed one FFT length
                dst[i] = cscale(v, k_cover[min(i / A.pattern_len, 8u)]);
                if (i < Nd) break;
            }
        } else {
            dst[A.CP + n] = v;
            if (n >= Nd - A.CP) dst[A.CP + n - Nd] = v;
        }
    });
}

// grid: (packet, antenna) x output blocks folded into x (gridDim.y is capped at 65536 rows)
__global__ void __launch_bounds__(256) tx_big_resample_kernel(tx_args A, uint32_t total) {
    const uint32_t nb = (A.S + 255) / 256;
    const uint32_t pa = blockIdx.x / nb, m = (blockIdx.x % nb) * 256 + threadIdx.x;
    if (m >= A.S) return;
    float2* out = reinterpret_cast<float2*>(A.out) + size_t(pa) * A.S;
    // outputs m with delay + m M < (total + hl) L: the packet and its flush samples
    const uint64_t tb = uint64_t(total + A.hl) * A.L;
    const uint32_t m_hi = tb > A.delay ? static_cast<uint32_t>(min<uint64_t>((tb - A.delay + A.M - 1) / A.M, A.n_keep)) : 0u;
    if (m >= m_hi) {
        out[m] = make_float2(0.f, 0.f);
        return;
    }
    const tx_pkt& P = A.pk[pa / A.N_TX];
    const float2* x = A.big + size_t(pa) * A.big_len;
    const uint64_t t = A.delay + uint64_t(m) * A.M;
    const int64_t p = static_cast<int64_t>(t / A.L);
    const uint32_t ph = static_cast<uint32_t>(t % A.L);
    float ar = 0.f, ai = 0.f;
    for (uint32_t d = 0; d <= A.hl; ++d) {
        const int64_t j = p - d;
        if (j < 0 || j >= int64_t(total)) continue;  // zero history / flush: fma(0, h, a) == a
        const float hv = A.taps[ph + d * A.L];
        const float2 xv = x[j];
        ar = fmaf(xv.x, hv, ar);
        ai = fmaf(xv.y, hv, ai);
    }
    float2 y = make_float2(ar, ai);
    if (P.do_mix) y = cmul(y, phasor(P.ph0 + static_cast<double>(m) * P.inc));
    out[m] = y;
}

size_t tx_lds_bytes(const tx_args& a) {
    const bool wave = a.plan.N == 1024;
    return (size_t(a.lin_len) + (wave ? 0 : a.bufB_len + a.plan.N) + 256 + 98 + 8) * sizeof(float2) +
           a.npp * sizeof(float) + ((a.stage_bytes + 2 + 15) & ~15u);
}

hipError_t launch_tx(const tx_args& a, uint32_t n, hipStream_t st) {
    if (a.stream) {
        const uint64_t waves = uint64_t(n) * a.N_TX * a.n_seg;
        const dim3 g(static_cast<uint32_t>((waves + TXS_WPG - 1) / TXS_WPG)), b(64 * TXS_WPG);
        const int mode = a.N_TS == 1 ? TXS_SISO : a.txdiv ? (a.onehot ? TXS_TXDIV1 : TXS_TXDIV) : (a.onehot ? TXS_SM1 : TXS_SM);
#define DNRP_TXS(MODE, Q8)                                                                                       \
    do {                                                                                                         \
        if (a.mfma == 2) hipLaunchKernelGGL((tx_stream_kernel<10, 9, 22, MODE, Q8, 2>), g, b, tx_stream_lds(), st, a, n); \
        else if (a.mfma) hipLaunchKernelGGL((tx_stream_kernel<10, 9, 22, MODE, Q8, 1>), g, b, tx_stream_lds(), st, a, n); \
        else hipLaunchKernelGGL((tx_stream_kernel<10, 9, 22, MODE, Q8, 0>), g, b, tx_stream_lds(), st, a, n);      \
    } while (0)
        if (a.N_bps == 8) {
            if (mode == TXS_SISO) DNRP_TXS(TXS_SISO, true);
            else if (mode == TXS_TXDIV) DNRP_TXS(TXS_TXDIV, true);
            else if (mode == TXS_TXDIV1) DNRP_TXS(TXS_TXDIV1, true);
            else if (mode == TXS_SM1) DNRP_TXS(TXS_SM1, true);
            else DNRP_TXS(TXS_SM, true);
        } else {
            if (mode == TXS_SISO) DNRP_TXS(TXS_SISO, false);
            else if (mode == TXS_TXDIV) DNRP_TXS(TXS_TXDIV, false);
            else if (mode == TXS_TXDIV1) DNRP_TXS(TXS_TXDIV1, false);
            else if (mode == TXS_SM1) DNRP_TXS(TXS_SM1, false);
            else DNRP_TXS(TXS_SM, false);
        }
#undef DNRP_TXS
        return hipGetLastError();
    }
    if (a.big) {
        if (a.N_bps > 8 || a.stage_bytes || a.N_TS > 8) return hipErrorInvalidValue;
        const uint32_t total = a.STF_CP + a.N_DF * a.CP + (a.N_DF + 1) * a.plan.N;
        if (total > a.big_len) return hipErrorInvalidValue;
        const size_t lds = (2 * size_t(a.plan.N) + 256 + 98 + 8) * sizeof(float2);
        if (lds > 160 * 1024 || a.big_batch == 0) return hipErrorInvalidValue;
        // passes of big_batch packets through the scratch (the host caps its size), each pass with
        // the packet-indexed arguments offset to its first packet; the largest pass's grids checked
        // before the first launch, so a call either runs every pass or none
        const uint64_t np_max = min(a.big_batch, n);
        if (uint64_t((a.S + 255) / 256) * np_max * a.N_TX > 0x7FFFFFFFull ||
            np_max * a.N_TX * (a.N_DF + 1) > 0x7FFFFFFFull)
            return hipErrorInvalidValue;
        for (uint32_t p0 = 0; p0 < n; p0 += a.big_batch) {
            const uint32_t np = min(a.big_batch, n - p0);
            tx_args b = a;
            b.pk = a.pk + p0;
            b.pcc_d = a.pcc_d + size_t(p0) * 25;
            b.pdc_d = a.pdc_d + size_t(p0) * a.pdc_stride;
            b.out = a.out + size_t(p0) * a.N_TX * a.S * 2;
            const uint64_t gx = uint64_t((a.S + 255) / 256) * np * a.N_TX;
            hipLaunchKernelGGL(tx_big_sym_kernel, dim3(np * a.N_TX * (a.N_DF + 1)), dim3(TX_BIG_THREADS), lds, st, b);
            hipLaunchKernelGGL(tx_big_resample_kernel, dim3(static_cast<uint32_t>(gx)), dim3(256), 0, st, b, total);
        }
        return hipGetLastError();
    }
    const bool wave = a.plan.N == 1024;
    if (a.K + 1 > TX_MAX_SLOTS || a.N_bps > 8) return hipErrorInvalidValue;
    if (!wave && (a.K + 1 > TX_BLOCK_SLOTS || a.plan.N > TX_BIN_REG * TX_THREADS)) return hipErrorInvalidValue;
    const size_t lds = tx_lds_bytes(a);
    const dim3 g(n * a.N_TX * a.n_runs), b(wave ? 64 * (a.K + 1) : TX_THREADS);
#define DNRP_TX_LAUNCH(LR, MR, HLR)                                                      \
    do {                                                                                 \
        if (wave)                                                                        \
            hipLaunchKernelGGL((tx_kernel_wave<LR, MR, HLR>), g, b, lds, st, a);         \
        else                                                                             \
            hipLaunchKernelGGL((tx_kernel<LR, MR, HLR>), g, b, lds, st, a);              \
    } while (0)
    if (a.L == 10 && a.M == 9 && a.hl == 22)  // os_min 1 (223 taps)
        DNRP_TX_LAUNCH(10, 9, 22);
    else if (a.L == 10 && a.M == 9 && a.hl == 4)  // os_min 2 (45 taps)
        DNRP_TX_LAUNCH(10, 9, 4);
    else if (a.L == 1 && a.M == 1)
        DNRP_TX_LAUNCH(1, 1, 0);
    else
        DNRP_TX_LAUNCH(0, 0, 0);
#undef DNRP_TX_LAUNCH
    return hipGetLastError();
}

}  // namespace dnrp::dev
