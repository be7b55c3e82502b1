// Fused TX kernel: one workgroup = one (packet, antenna) slot stream.
//
// Per OFDM symbol (STF + N_DF data symbols), fully in LDS:
//   scramble + modulate (PCC QPSK / PDC BPSK..256QAM) + transmit-diversity flip + DRS/STF cells
//   -> beamforming row W[a,:] -> FFT-bin mirror + scaling -> Stockham IFFT -> CP (+ STF cover)
//   -> rational polyphase resampler L/M over a circular input ring -> phase-continuous mixer -> HBM.
// The cell codes and the (descrambled) PDC source bytes of symbol l+1 are fetched into registers
// while symbol l runs through the IFFT and parked in a double-buffered LDS stage, so the symbol
// loop never waits on global memory. The resampler is register-blocked (polyphase.hpp): one thread
// computes L consecutive outputs from registers with the taps on the scalar path.
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

constexpr uint32_t TX_THREADS = 512;
constexpr uint32_t TX_CODE_REG = 2;   // code words per thread per symbol (Nf <= 1024)
constexpr uint32_t TX_BYTE_REG = 4;   // staged PDC bytes per thread per symbol (<= 2048)

__device__ __forceinline__ uint32_t bits_of(uint32_t b0, uint32_t b1, uint32_t bitoff, uint32_t nbits) {
    const uint32_t w = (b0 << 8) | b1;
    return (w >> (16u - (bitoff & 7u) - nbits)) & ((1u << nbits) - 1u);
}

__device__ __forceinline__ bool nz(float2 w) { return w.x != 0.f || w.y != 0.f; }

__device__ __forceinline__ int floor_div(int a, int b) { return a >= 0 ? a / b : -((-a + b - 1) / b); }

// LR > 0: compile-time L/M/HL (register-blocked resampler); LR == 0: runtime L/M (generic path)
template <int LR, int MR, int HLR>
__global__ void __launch_bounds__(TX_THREADS) __attribute__((amdgpu_waves_per_eu(4, 8))) tx_kernel(tx_args A) {
    extern __shared__ __attribute__((aligned(16))) float2 smem[];
    const uint32_t pkt = blockIdx.x / A.N_TX, ant = blockIdx.x % A.N_TX;
    const tx_pkt P = A.pk[pkt];
    const uint32_t Nd = A.plan.N, N = A.N_occ, Nf = N + 1;
    const uint32_t R = A.ring;
    const uint32_t hl = LR > 0 ? static_cast<uint32_t>(HLR) : A.hl;
    float2* bufA = smem;
    float2* bufB = bufA + Nd;
    float2* twl = bufB + Nd;                          // twiddles
    float2* ring = twl + Nd;                          // resampler input ring, input q at (q + hl) % R
    float2* pccs = ring + R;                          // 98 PCC QPSK symbols
    float2* wrow = pccs + 98;                         // W[ant][0..N_TS)
    uint32_t* code_st = reinterpret_cast<uint32_t*>(wrow + 8);  // [2][Nf]
    uint8_t* byte_st = reinterpret_cast<uint8_t*>(code_st + 2 * Nf);  // [2][stage_bytes]
    float* taps = reinterpret_cast<float*>(byte_st + ((2 * A.stage_bytes + 15) & ~15u));  // generic path

    const uint8_t* __restrict__ dpcc = A.pcc_d + size_t(pkt) * 25;
    const uint8_t* __restrict__ dpdc = A.pdc_d + size_t(pkt) * A.pdc_stride;
    const uint8_t* __restrict__ cpdc = P.pdc_seq;
    const uint32_t pdc_bytes = (A.G + 7) / 8;
    const uint32_t bits_per_cell = A.N_SS * A.N_bps;

    for (uint32_t j = threadIdx.x; j < 98; j += TX_THREADS) {
        const uint32_t bo = (2 * j) >> 3;
        pccs[j] = A.qpsk[bits_of(dpcc[bo] ^ A.pcc_seq[bo], 0u, 2 * j, 2)];
    }
    for (uint32_t i = threadIdx.x; i < A.N_TS; i += TX_THREADS) wrow[i] = A.W[(P.codebook * A.N_TX + ant) * A.N_TS + i];
    for (uint32_t i = threadIdx.x; i < hl; i += TX_THREADS) ring[i] = make_float2(0.f, 0.f);  // zero history
    for (uint32_t i = threadIdx.x; i < Nd; i += TX_THREADS) twl[i] = A.tw[i];
    if (LR == 0)
        for (uint32_t i = threadIdx.x; i < (A.hl + 1) * A.L; i += TX_THREADS) taps[i] = A.taps[i];

    // ---- per-symbol source prefetch (registers) and parking (LDS stage)
    uint32_t rc[TX_CODE_REG];
    uint32_t rb[TX_BYTE_REG];
    auto stage_byte0 = [&](uint32_t l) { return (A.pdc_off[l] * bits_per_cell) >> 3; };
    auto fetch = [&](uint32_t l) {
#pragma unroll
        for (uint32_t r = 0; r < TX_CODE_REG; ++r) {
            const uint32_t k = threadIdx.x + r * TX_THREADS;
            rc[r] = k < Nf ? A.code[size_t(l) * Nf + k] : 0u;
        }
        if (A.stage_bytes) {
            const uint32_t b0 = l >= 1 ? stage_byte0(l) : 0u;
#pragma unroll
            for (uint32_t r = 0; r < TX_BYTE_REG; ++r) {
                const uint32_t i = threadIdx.x + r * TX_THREADS, g = b0 + i;
                rb[r] = (l >= 1 && i < A.stage_bytes && g < pdc_bytes) ? uint32_t(dpdc[g] ^ cpdc[g]) : 0u;
            }
        }
    };
    auto park = [&](uint32_t buf) {
#pragma unroll
        for (uint32_t r = 0; r < TX_CODE_REG; ++r) {
            const uint32_t k = threadIdx.x + r * TX_THREADS;
            if (k < Nf) code_st[buf * Nf + k] = rc[r];
        }
        if (A.stage_bytes) {
#pragma unroll
            for (uint32_t r = 0; r < TX_BYTE_REG; ++r) {
                const uint32_t i = threadIdx.x + r * TX_THREADS;
                if (i < A.stage_bytes) byte_st[buf * A.stage_bytes + i] = static_cast<uint8_t>(rb[r]);
            }
        }
    };
    fetch(0);
    park(0);
    __syncthreads();

    auto flip = [&](float2 nb, uint32_t j) {  // pairwise swap + (-re,+im) / (+re,-im) pattern
        return (j & 1u) ? make_float2(nb.x, -nb.y) : make_float2(-nb.x, nb.y);
    };

    float2* out = reinterpret_cast<float2*>(A.out) + size_t(pkt * A.N_TX + ant) * A.S;
    const float2 step1 = P.do_mix ? phasor(P.inc) : make_float2(1.f, 0.f);
    uint32_t base_in = 0;  // input index of the current symbol's first sample
    uint32_t m_next = 0;   // next output sample index

    for (uint32_t l = 0; l <= A.N_DF + 1; ++l) {
        const bool flush = (l == A.N_DF + 1);
        const uint32_t cur = l & 1u;
        uint32_t len;
        const uint32_t r0 = (base_in + hl) % R;  // ring slot of the symbol's first sample
        if (!flush) {
            const float sc = (l == 0) ? P.scale_stf : P.scale_df;
            const uint32_t* code = code_st + cur * Nf;
            const uint8_t* sb = byte_st + cur * A.stage_bytes;
            const uint32_t sbit0 = l >= 1 ? (stage_byte0(l) << 3) : 0u;
            auto pdc_sym = [&](uint32_t s) {  // complex symbol s of the packet, from the stage
                const uint32_t bit = s * A.N_bps;
                if (A.stage_bytes) {
                    const uint32_t lb = bit - sbit0, bo = lb >> 3;
                    return A.qam[bits_of(sb[bo], sb[bo + 1], lb, A.N_bps)];
                }
                const uint32_t bo = bit >> 3;
                const uint32_t b1 = bo + 1 < pdc_bytes ? uint32_t(dpdc[bo + 1] ^ cpdc[bo + 1]) : 0u;
                return A.qam[bits_of(dpdc[bo] ^ cpdc[bo], b1, bit, A.N_bps)];
            };
            // ---- frequency-domain cells onto FFT bins (tx.cpp:936-1116, 729-860, 862-871)
            for (uint32_t n = threadIdx.x; n < Nd; n += TX_THREADS) {
                uint32_t k = 0xFFFFFFFFu;
                if (n <= N / 2)
                    k = N / 2 + n;
                else if (n >= A.off_lower && n < A.off_lower + N / 2)
                    k = n - A.off_lower;
                float2 v = make_float2(0.f, 0.f);
                if (k != 0xFFFFFFFFu) {
                    const uint32_t c = code[k];
                    const uint32_t ty = c & CODE_MASK, j = c & ~CODE_MASK;
                    if (ty == CODE_STF) {
                        v = cmul(wrow[0], A.stf[k]);
                    } else if (ty == CODE_DRS) {
                        const float s = (j & 8u) ? -1.f : 1.f;
                        v = cscale(wrow[j & 7u], s);
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
                    v = cscale(v, sc);
                }
                bufA[n] = v;
            }
            if (l + 1 <= A.N_DF) fetch(l + 1);  // in flight during the IFFT
            __syncthreads();
            float2* td = fft_any<+1>(bufA, bufB, twl, A.plan);
            if (l + 1 <= A.N_DF) park(cur ^ 1u);
            // ---- CP insertion (ofdm.cpp:62-79) + STF cover sequence into the input ring
            const uint32_t CP = (l == 0) ? A.STF_CP : A.CP;
            const uint32_t cpm = CP % Nd;
            len = CP + Nd;
            for (uint32_t i = threadIdx.x; i < len; i += TX_THREADS) {
                uint32_t src = i + Nd - cpm;
                src = src >= Nd ? src - Nd : src;
                src = src >= Nd ? src - Nd : src;
                float2 s = td[src];
                if (l == 0) s = cscale(s, k_cover[min(i / A.pattern_len, 8u)]);
                uint32_t r = r0 + i;
                r = r >= R ? r - R : r;
                ring[r] = s;
            }
        } else {
            len = hl;  // resample_final_samples(): history followed by zeros
            for (uint32_t i = threadIdx.x; i < len; i += TX_THREADS) {
                uint32_t r = r0 + i;
                r = r >= R ? r - R : r;
                ring[r] = make_float2(0.f, 0.f);
            }
        }
        __syncthreads();
        // ---- polyphase resampling of every output whose window ends in this symbol
        const uint32_t p_end = base_in + len;
        const uint64_t t_end = uint64_t(p_end) * A.L;  // outputs need delay + m*M < t_end
        uint32_t m_end = t_end > A.delay ? static_cast<uint32_t>((t_end - A.delay + A.M - 1) / A.M) : 0u;
        m_end = min(m_end, A.n_keep);
        if constexpr (LR > 0) {
            using PB = pp_block<LR, MR, HLR>;
            const const_taps_t h = as_const_taps(A.taps);
            const int q_lo = floor_div(static_cast<int>(m_next) - static_cast<int>(A.m_star), LR);
            const int q_hi = floor_div(static_cast<int>(m_end) - static_cast<int>(A.m_star) + LR - 1, LR);
            for (int q = q_lo + static_cast<int>(threadIdx.x); q < q_hi; q += TX_THREADS) {
                const int mb = static_cast<int>(A.m_star) + LR * q;
                const int pb = static_cast<int>(A.p_star) + MR * q;  // newest input of output mb
                uint32_t r = static_cast<uint32_t>(pb + static_cast<int>(R)) % R;  // slot of input pb - HL
                float2 x[PB::W];
#pragma unroll
                for (int i = 0; i < PB::W; ++i) {
                    x[i] = ring[r];
                    r = (r + 1 == R) ? 0u : r + 1;
                }
                float2 y[LR];
                const_taps_t hq = h;
                asm volatile("" : "+s"(hq));  // keep the tap loads inside the loop (SGPR budget)
                PB::run(x, hq, y);
                float2 rot = P.do_mix ? phasor(P.ph0 + static_cast<double>(mb) * P.inc) : make_float2(1.f, 0.f);
#pragma unroll
                for (int k = 0; k < LR; ++k) {
                    const uint32_t m = static_cast<uint32_t>(mb + k);
                    if (P.do_mix) {
                        y[k] = cmul(y[k], rot);
                        rot = cmul(rot, step1);
                    }
                    if (m - m_next < m_end - m_next) out[m] = y[k];
                }
            }
        } else {
            const uint32_t m0 = m_next + threadIdx.x;
            const uint32_t dT = TX_THREADS * A.M, dp = dT / A.L, dph = dT % A.L;
            const float2 rstep = P.do_mix ? phasor(static_cast<double>(TX_THREADS) * P.inc) : make_float2(1.f, 0.f);
            if (m0 < m_end) {
                const uint64_t t = A.delay + uint64_t(m0) * A.M;
                uint32_t p = static_cast<uint32_t>(t / A.L) + hl;  // input index + hl of the newest input
                uint32_t ph = static_cast<uint32_t>(t % A.L);
                float2 rot = P.do_mix ? phasor(P.ph0 + static_cast<double>(m0) * P.inc) : make_float2(1.f, 0.f);
                for (uint32_t m = m0; m < m_end; m += TX_THREADS) {
                    float ar = 0.f, ai = 0.f;
                    for (uint32_t d = 0; d <= hl; ++d) {
                        const float hv = taps[ph + d * A.L];
                        const float2 x = ring[(p - d) % R];
                        ar = fmaf(x.x, hv, ar);
                        ai = fmaf(x.y, hv, ai);
                    }
                    float2 y = make_float2(ar, ai);
                    if (P.do_mix) {
                        y = cmul(y, rot);
                        rot = cmul(rot, rstep);
                    }
                    out[m] = y;
                    p += dp;
                    ph += dph;
                    if (ph >= A.L) {
                        ph -= A.L;
                        ++p;
                    }
                }
            }
        }
        m_next = max(m_next, m_end);
        base_in = p_end;
        // no barrier: the next symbol writes ring slots this FIR window does not read
    }
    // ---- GI and slot tail (tx.cpp:679-714)
    for (uint32_t m = m_next + threadIdx.x; m < A.S; m += TX_THREADS) out[m] = make_float2(0.f, 0.f);
}

hipError_t launch_tx(const tx_args& a, uint32_t n, hipStream_t st) {
    const uint32_t Nf = a.N_occ + 1;
    const size_t lds = (3 * size_t(a.plan.N) + a.ring + 98 + 8) * sizeof(float2) + 2 * Nf * sizeof(uint32_t) +
                       ((2 * a.stage_bytes + 15) & ~15u) + (a.hl + 1) * a.L * sizeof(float);
    const dim3 g(n * a.N_TX), b(TX_THREADS);
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
