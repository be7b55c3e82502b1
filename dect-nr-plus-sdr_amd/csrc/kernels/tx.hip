// Fused TX kernel, symbol-parallel: one workgroup = one (packet, antenna, run of K OFDM symbols).
//
// A WG synthesises the K symbols of its run plus the symbol before them, whose tail is the
// resampler history, so runs are independent and the whole slot is in flight at once:
//   staged d-bits (descrambled)  ->  scramble/modulate (PCC QPSK, PDC BPSK..256QAM), transmit
//   diversity flip, DRS/STF cells, beamforming row W[a,:], FFT-bin mirror and scaling
//   ->  batched Stockham IFFT whose last pass writes the cyclic-prefixed (and STF-covered)
//   time-domain symbols straight into a linear LDS buffer
//   ->  register-blocked polyphase L/M resampler (polyphase.hpp) + phase-continuous mixer -> HBM.
// Restates tx_t::generate_tx_packet (lib/src/phy/tx/tx.cpp:165-314) and its callees
// run_pcc/run_drs/run_pdc (936-1116), run_beamforming (729-860), run_ifft_cp_scale (862-911),
// stf_t::apply_cover_sequence (sections_part3/stf.cpp:104-138), resampler_t (resampler.cpp:330-454)
// and mixer_t::mix_phase_continuous (mixer.cpp:41-65). Only the packed d-bits are read and only
// the final hw-rate IQ is written: HBM traffic = ceil(G/8) + 25 bytes in, N_TX * S * 8 bytes out.
#include "device_common.hpp"
#include "kernels.hpp"
#include "polyphase.hpp"

namespace dnrp::dev {

__constant__ float k_cover[9] = {1, -1, 1, 1, -1, -1, -1, -1, -1};  // stf.hpp:146-151

constexpr uint32_t TX_THREADS = 256;
constexpr uint32_t TX_MAX_SLOTS = 4;  // K + 1
constexpr uint32_t TX_BIN_REG = 4;    // FFT bins per thread per symbol (N_b_DFT_os <= 1024)

__device__ __forceinline__ uint32_t bits_of(uint32_t b0, uint32_t b1, uint32_t bitoff, uint32_t nbits) {
    const uint32_t w = (b0 << 8) | b1;
    return (w >> (16u - (bitoff & 7u) - nbits)) & ((1u << nbits) - 1u);
}

__device__ __forceinline__ bool nz(float2 w) { return w.x != 0.f || w.y != 0.f; }

__device__ __forceinline__ int floor_div(int a, int b) { return a >= 0 ? a / b : -((-a + b - 1) / b); }

// LR > 0: compile-time L/M/HL (register-blocked resampler); LR == 0: runtime L/M (generic path)
template <int LR, int MR, int HLR>
__global__ void __launch_bounds__(TX_THREADS) tx_kernel(tx_args A) {
    extern __shared__ __attribute__((aligned(16))) float2 smem[];
    const uint32_t run = blockIdx.x % A.n_runs, pa = blockIdx.x / A.n_runs;
    const uint32_t pkt = pa / A.N_TX, ant = pa % A.N_TX;
    const tx_pkt P = A.pk[pkt];
    const uint32_t Nd = A.plan.N, N = A.N_occ, Nf = N + 1;
    const uint32_t hl = LR > 0 ? static_cast<uint32_t>(HLR) : A.hl;
    const uint32_t len0 = A.STF_CP + Nd, lenD = A.CP + Nd;
    auto bsym = [&](uint32_t l) { return l == 0 ? 0u : len0 + (l - 1) * lenD; };  // first input of symbol l
    const uint32_t l_first = run * A.K, l_last = min(l_first + A.K, A.N_DF + 1) - 1;
    const uint32_t s0 = l_first > 0 ? l_first - 1 : 0u;  // first synthesised symbol
    const uint32_t nsl = l_last - s0 + 1;
    const bool last_run = (run + 1 == A.n_runs);
    const uint32_t base_q = bsym(s0);  // input index held at lin[HP]

    float2* lin = smem;                    // [lin_len] head pad | symbols s0..l_last | tail pad
    float2* bufB = lin + A.lin_len;       // [nsl][Nd] FFT ping-pong partner, then output staging
    float2* twl = bufB + A.bufB_len;
    float2* qtab = twl + Nd;               // constellation, 1 << N_bps
    float2* pccs = qtab + 256;             // 98 PCC QPSK symbols
    float2* wrow = pccs + 98;              // W[ant][0..N_TS)
    float* hpl = reinterpret_cast<float*>(wrow + 8);      // block taps [W][LP] (polyphase.hpp)
    uint8_t* sb = reinterpret_cast<uint8_t*>(hpl + A.npp);  // staged PDC bytes of the run

    const uint8_t* __restrict__ dpcc = A.pcc_d + size_t(pkt) * 25;
    const uint8_t* __restrict__ dpdc = A.pdc_d + size_t(pkt) * A.pdc_stride;
    const uint8_t* __restrict__ cpdc = P.pdc_seq;
    const uint32_t pdc_bytes = (A.G + 7) / 8;
    const uint32_t bpc = A.N_SS * A.N_bps;  // bits per PDC cell
    const uint32_t sbyte0 = (A.pdc_off[max(s0, 1u)] * bpc) >> 3;

    // ---- staging: tables, PCC symbols, beamforming row, descrambled PDC bytes, zero pads
    for (uint32_t i = threadIdx.x; i < Nd; i += TX_THREADS) twl[i] = A.tw[i];
    for (uint32_t i = threadIdx.x; i < A.npp; i += TX_THREADS) hpl[i] = A.taps_pp[i];
    for (uint32_t i = threadIdx.x; i < (1u << A.N_bps); i += TX_THREADS) qtab[i] = A.qam[i];
    for (uint32_t j = threadIdx.x; j < 98; j += TX_THREADS) {
        const uint32_t bo = (2 * j) >> 3;
        pccs[j] = A.qpsk[bits_of(dpcc[bo] ^ A.pcc_seq[bo], 0u, 2 * j, 2)];
    }
    for (uint32_t i = threadIdx.x; i < A.N_TS; i += TX_THREADS) wrow[i] = A.W[(P.codebook * A.N_TX + ant) * A.N_TS + i];
    for (uint32_t i = threadIdx.x; i < A.stage_bytes; i += TX_THREADS) {
        const uint32_t g = sbyte0 + i;
        sb[i] = g < pdc_bytes ? static_cast<uint8_t>(dpdc[g] ^ cpdc[g]) : 0u;
    }
    // the last IFFT pass must read bufB (it writes lin): place the grid accordingly
    const uint32_t npass = fft_num_passes(A.plan);
    float2* gin = ((npass - 1) % 2 == 0) ? bufB : lin;
    float2* gout = (gin == lin) ? bufB : lin;

    // ---- code rows of the run into registers (independent loads, one round trip)
    uint32_t rc[TX_MAX_SLOTS][TX_BIN_REG];
#pragma unroll
    for (uint32_t b = 0; b < TX_MAX_SLOTS; ++b)
#pragma unroll
        for (uint32_t r = 0; r < TX_BIN_REG; ++r) {
            const uint32_t n = threadIdx.x + r * TX_THREADS;
            uint32_t k = 0xFFFFFFFFu;
            if (n <= N / 2)
                k = N / 2 + n;
            else if (n >= A.off_lower && n < A.off_lower + N / 2)
                k = n - A.off_lower;
            rc[b][r] = (b < nsl && n < Nd && k != 0xFFFFFFFFu) ? A.code[size_t(s0 + b) * Nf + k] : 0u;
        }
    __syncthreads();

    auto flip = [&](float2 nb, uint32_t j) {  // pairwise swap + (-re,+im) / (+re,-im) pattern
        return (j & 1u) ? make_float2(nb.x, -nb.y) : make_float2(-nb.x, nb.y);
    };
    auto pdc_sym = [&](uint32_t s) {  // complex PDC symbol s of the packet
        const uint32_t bit = s * A.N_bps;
        if (A.stage_bytes) {
            const uint32_t lb = bit - (sbyte0 << 3), bo = lb >> 3;
            return qtab[bits_of(sb[bo], sb[bo + 1], lb, A.N_bps)];
        }
        const uint32_t bo = bit >> 3;
        const uint32_t b1 = bo + 1 < pdc_bytes ? uint32_t(dpdc[bo + 1] ^ cpdc[bo + 1]) : 0u;
        return qtab[bits_of(dpdc[bo] ^ cpdc[bo], b1, bit, A.N_bps)];
    };

    // ---- frequency-domain cells onto FFT bins (tx.cpp:936-1116, 729-860, 862-871)
#pragma unroll
    for (uint32_t b = 0; b < TX_MAX_SLOTS; ++b) {
        if (b >= nsl || (A.dbg & 1)) break;
        const uint32_t l = s0 + b;
        const float sc = (l == 0) ? P.scale_stf : P.scale_df;
#pragma unroll
        for (uint32_t r = 0; r < TX_BIN_REG; ++r) {
            const uint32_t n = threadIdx.x + r * TX_THREADS;
            if (n >= Nd) break;
            const uint32_t c = rc[b][r];
            const uint32_t ty = c & CODE_MASK, j = c & ~CODE_MASK;
            float2 v = make_float2(0.f, 0.f);
            if (ty == CODE_STF) {
                const uint32_t k = n <= N / 2 ? N / 2 + n : n - A.off_lower;
                v = cmul(wrow[0], A.stf[k]);
            } else if (ty == CODE_DRS) {
                v = cscale(wrow[j & 7u], (j & 8u) ? -1.f : 1.f);
            } else if (ty == CODE_PCC) {
                if (A.N_TS == 1) {
                    v = cmul(wrow[0], pccs[j]);
                } else {
                    const uint32_t pr = A.pair[(j >> 1) % A.mod];
                    v = cadd(cmul(wrow[pr & 0xFu], pccs[j]), cmul(wrow[pr >> 4], flip(pccs[j ^ 1u], j)));
                }
            } else if (ty == CODE_PDC) {
                if (A.txdiv) {
                    const uint32_t pr = A.pair[(j >> 1) % A.mod];
                    const float2 wa = wrow[pr & 0xFu], wb = wrow[pr >> 4];
                    if (nz(wa)) v = cmul(wa, pdc_sym(j));
                    if (nz(wb)) v = cadd(v, cmul(wb, flip(pdc_sym(j ^ 1u), j)));
                } else {
                    for (uint32_t ss = 0; ss < A.N_SS; ++ss)
                        if (nz(wrow[ss])) v = cadd(v, cmul(wrow[ss], pdc_sym(j * A.N_SS + ss)));
                }
            }
            gin[b * Nd + n] = cscale(v, sc);
        }
    }
    __syncthreads();

    // ---- IFFT; last pass = CP insertion (ofdm.cpp:62-79) + STF cover sequence into lin
    if (!(A.dbg & 2)) fft_store<+1>(gin, gout, twl, A.plan, nsl, [&](uint32_t b, uint32_t n, float2 v) {
        const uint32_t l = s0 + b;
        const uint32_t cp = l == 0 ? A.STF_CP : A.CP;
        float2* dst = lin + A.HP + bsym(l) - base_q;
        if (l == 0) {
            for (uint32_t i = cp + n;; i -= Nd) {  // the STF CP may exceed one FFT length
                dst[i] = cscale(v, k_cover[min(i / A.pattern_len, 8u)]);
                if (i < Nd) break;
            }
        } else {
            dst[cp + n] = v;
            if (n >= Nd - cp) dst[cp + n - Nd] = v;
        }
    });

    // zero pads around the symbols (history before the packet, flush after it); the IFFT used
    // the whole buffer as scratch, so this comes after it
    const uint32_t data_end = A.HP + bsym(l_last + 1) - base_q;
    for (uint32_t i = threadIdx.x; i < A.HP; i += TX_THREADS) lin[i] = make_float2(0.f, 0.f);
    for (uint32_t i = data_end + threadIdx.x; i < A.lin_len; i += TX_THREADS) lin[i] = make_float2(0.f, 0.f);
    __syncthreads();

    // ---- outputs whose newest input lies in this run (the last run adds the flush samples)
    const uint32_t B_lo = bsym(l_first), B_hi = last_run ? bsym(A.N_DF + 1) + hl : bsym(l_last + 1);
    auto n_out = [&](uint32_t B) {  // outputs m with delay + m*M < B*L
        const uint64_t t = uint64_t(B) * A.L;
        return t > A.delay ? min(static_cast<uint32_t>((t - A.delay + A.M - 1) / A.M), A.n_keep) : 0u;
    };
    const uint32_t m_lo = n_out(B_lo), m_hi = n_out(B_hi);
    float2* out = reinterpret_cast<float2*>(A.out) + size_t(pkt * A.N_TX + ant) * A.S;
    const int lin_off = static_cast<int>(A.HP) - static_cast<int>(base_q);
    if constexpr (LR > 0) {
        using PB = pp_block<LR, MR, HLR>;
        const float2 step1 = P.do_mix ? phasor(P.inc) : make_float2(1.f, 0.f);
        const int q_lo = floor_div(static_cast<int>(m_lo) - static_cast<int>(A.m_star), LR);
        const int q_hi = floor_div(static_cast<int>(m_hi) - static_cast<int>(A.m_star) + LR - 1, LR);
        const int idx_max = static_cast<int>(A.lin_len) - PB::W;
        float2* ostage = bufB;  // [bufB_len + Nd + 256] >= outputs of any run (host-checked)
        for (int q = q_lo + static_cast<int>(threadIdx.x); q < q_hi && !(A.dbg & 4); q += TX_THREADS) {
            const int mb = static_cast<int>(A.m_star) + LR * q;
            const int pb = static_cast<int>(A.p_star) + MR * q;  // newest input of output mb
            const int idx = min(max(pb - HLR + lin_off, 0), idx_max);  // clamp: only unstored outputs clip
            float2 y[LR];
            PB::run(lin + idx, hpl, y);
            float2 rot = P.do_mix ? phasor(P.ph0 + static_cast<double>(mb) * P.inc) : make_float2(1.f, 0.f);
#pragma unroll
            for (int k = 0; k < LR; ++k) {
                const uint32_t m = static_cast<uint32_t>(mb + k);
                if (P.do_mix) {
                    y[k] = cmul(y[k], rot);
                    rot = cmul(rot, step1);
                }
                if (m - m_lo < m_hi - m_lo) ostage[m - m_lo] = y[k];
            }
        }
        __syncthreads();
        // coalesced write-out of the run's outputs (bufB + twiddles + constellation are free now)
        const uint32_t cnt = m_hi - m_lo;
        float2* o = out + m_lo;
        uint32_t i0 = 0;
        if ((m_lo & 1u) && cnt) {
            if (threadIdx.x == 0) o[0] = ostage[0];
            i0 = 1;
        }
        const uint32_t npair = (cnt - i0) / 2;
        for (uint32_t i = threadIdx.x; i < npair; i += TX_THREADS) {
            const float2 a = ostage[i0 + 2 * i], b = ostage[i0 + 2 * i + 1];
            *reinterpret_cast<float4*>(o + i0 + 2 * i) = make_float4(a.x, a.y, b.x, b.y);
        }
        if ((cnt - i0) & 1u)
            if (threadIdx.x == 0) o[cnt - 1] = ostage[cnt - 1];
    } else {
        for (uint32_t m = m_lo + threadIdx.x; m < m_hi; m += TX_THREADS) {
            const uint64_t t = A.delay + uint64_t(m) * A.M;
            const int p = static_cast<int>(t / A.L);
            const uint32_t ph = static_cast<uint32_t>(t % A.L);
            float ar = 0.f, ai = 0.f;
            for (uint32_t d = 0; d <= hl; ++d) {
                const float hv = A.taps[ph + d * A.L];
                const float2 x = lin[p - static_cast<int>(d) + lin_off];
                ar = fmaf(x.x, hv, ar);
                ai = fmaf(x.y, hv, ai);
            }
            float2 y = make_float2(ar, ai);
            if (P.do_mix) y = cmul(y, phasor(P.ph0 + static_cast<double>(m) * P.inc));
            out[m] = y;
        }
    }
    // ---- GI and slot tail (tx.cpp:679-714)
    if (last_run)
        for (uint32_t m = m_hi + threadIdx.x; m < A.S; m += TX_THREADS) out[m] = make_float2(0.f, 0.f);
}

size_t tx_lds_bytes(const tx_args& a) {
    return (size_t(a.lin_len) + a.bufB_len + a.plan.N + 256 + 98 + 8) * sizeof(float2) +
           a.npp * sizeof(float) + ((a.stage_bytes + 2 + 15) & ~15u);
}

hipError_t launch_tx(const tx_args& a, uint32_t n, hipStream_t st) {
    if (a.K + 1 > TX_MAX_SLOTS || a.plan.N > TX_BIN_REG * TX_THREADS || a.N_bps > 8) return hipErrorInvalidValue;
    const size_t lds = tx_lds_bytes(a);
    const dim3 g(n * a.N_TX * a.n_runs), b(TX_THREADS);
    if (a.L == 10 && a.M == 9 && a.hl == 22)  // os_min 1 (223 taps)
        hipLaunchKernelGGL((tx_kernel<10, 9, 22>), g, b, lds, st, a);
    else if (a.L == 10 && a.M == 9 && a.hl == 4)  // os_min 2 (45 taps)
        hipLaunchKernelGGL((tx_kernel<10, 9, 4>), g, b, lds, st, a);
    else if (a.L == 1 && a.M == 1)
        hipLaunchKernelGGL((tx_kernel<1, 1, 0>), g, b, lds, st, a);
    else
        hipLaunchKernelGGL((tx_kernel<0, 0, 0>), g, b, lds, st, a);
    return hipGetLastError();
}

}  // namespace dnrp::dev
