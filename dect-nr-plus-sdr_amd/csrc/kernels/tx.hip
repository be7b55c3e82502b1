// Fused TX kernel: one workgroup = one (packet, antenna) slot stream.
//
// Per OFDM symbol (STF + N_DF data symbols), fully in LDS:
//   scramble + modulate (PCC QPSK / PDC BPSK..256QAM) + transmit-diversity flip + DRS/STF cells
//   -> beamforming row W[a,:] -> FFT-bin mirror + scaling -> Stockham IFFT -> CP (+ STF cover)
//   -> rational polyphase resampler L/M with carried history -> phase-continuous mixer -> HBM.
// Restates tx_t::generate_tx_packet (lib/src/phy/tx/tx.cpp:165-314) and its callees
// run_pcc/run_drs/run_pdc (936-1116), run_beamforming (729-860), run_ifft_cp_scale (862-911),
// stf_t::apply_cover_sequence (sections_part3/stf.cpp:104-138), resampler_t (resampler.cpp:330-454)
// and mixer_t::mix_phase_continuous (mixer.cpp:41-65). Only the packed d-bits are read and only
// the final hw-rate IQ is written: HBM traffic = ceil(G/8) + 25 bytes in, N_TX * S * 8 bytes out.
#include "device_common.hpp"
#include "kernels.hpp"

namespace dnrp::dev {

__constant__ float k_cover[9] = {1, -1, 1, 1, -1, -1, -1, -1, -1};  // stf.hpp:146-151

__device__ __forceinline__ uint32_t bits_at(const uint8_t* __restrict__ d, const uint8_t* __restrict__ c,
                                            uint32_t bitoff, uint32_t nbits, uint32_t nbytes) {
    const uint32_t bo = bitoff >> 3;
    const uint32_t b0 = d[bo] ^ c[bo];
    const uint32_t b1 = (bo + 1 < nbytes) ? (d[bo + 1] ^ c[bo + 1]) : 0u;
    const uint32_t w = (b0 << 8) | b1;
    return (w >> (16u - (bitoff & 7u) - nbits)) & ((1u << nbits) - 1u);
}

__global__ void __launch_bounds__(256) tx_kernel(tx_args A) {
    extern __shared__ __attribute__((aligned(16))) float2 smem[];
    const uint32_t pkt = blockIdx.x / A.N_TX, ant = blockIdx.x % A.N_TX;
    const tx_pkt P = A.pk[pkt];
    const uint32_t Nd = A.plan.N, N = A.N_occ, Nf = N + 1;
    float2* bufA = smem;
    float2* bufB = bufA + Nd;
    float2* xbuf = bufB + Nd;               // [hl history | current symbol (<= STF_CP + Nd)]
    float2* pccs = xbuf + A.xbuf_len;        // 98 PCC QPSK symbols
    float2* wrow = pccs + 98;                // W[ant][0..N_TS)
    __shared__ float2 red_dummy;
    (void)red_dummy;

    const uint8_t* __restrict__ dpcc = A.pcc_d + size_t(pkt) * 25;
    const uint8_t* __restrict__ dpdc = A.pdc_d + size_t(pkt) * A.pdc_stride;
    const uint32_t pdc_bytes = (A.G + 7) / 8;

    for (uint32_t j = threadIdx.x; j < 98; j += blockDim.x) pccs[j] = A.qpsk[bits_at(dpcc, A.pcc_seq, 2 * j, 2, 25)];
    for (uint32_t i = threadIdx.x; i < A.N_TS; i += blockDim.x) wrow[i] = A.W[(P.codebook * A.N_TX + ant) * A.N_TS + i];
    for (uint32_t i = threadIdx.x; i < A.hl; i += blockDim.x) xbuf[i] = make_float2(0.f, 0.f);
    __syncthreads();

    auto pdc_sym = [&](uint32_t s) { return A.qam[bits_at(dpdc, P.pdc_seq, s * A.N_bps, A.N_bps, pdc_bytes)]; };
    auto flip = [&](float2 nb, uint32_t j) {  // pairwise swap + (-re,+im) / (+re,-im) pattern
        return (j & 1u) ? make_float2(nb.x, -nb.y) : make_float2(-nb.x, nb.y);
    };

    float2* out = reinterpret_cast<float2*>(A.out) + size_t(pkt * A.N_TX + ant) * A.S;
    uint64_t base_in = 0;  // inputs consumed before the current symbol
    uint32_t m_next = 0;   // next output sample index

    for (uint32_t l = 0; l <= A.N_DF + 1; ++l) {
        const bool flush = (l == A.N_DF + 1);
        uint32_t len;
        if (!flush) {
            const float sc = (l == 0) ? P.scale_stf : P.scale_df;
            const uint32_t* __restrict__ code = A.code + size_t(l) * Nf;
            // ---- frequency-domain cells onto FFT bins (tx.cpp:936-1116, 729-860, 862-871)
            for (uint32_t n = threadIdx.x; n < Nd; n += blockDim.x) {
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
                            v = cadd(cmul(wrow[pr & 0xFu], pdc_sym(j)), cmul(wrow[pr >> 4], flip(pdc_sym(j ^ 1u), j)));
                        } else {
                            for (uint32_t ss = 0; ss < A.N_SS; ++ss) v = cadd(v, cmul(wrow[ss], pdc_sym(j * A.N_SS + ss)));
                        }
                    }
                    v = cscale(v, sc);
                }
                bufA[n] = v;
            }
            __syncthreads();
            float2* td = fft_lds<+1>(bufA, bufB, A.tw, A.plan);
            // ---- CP insertion (ofdm.cpp:62-79) + STF cover sequence, appended after the history
            const uint32_t CP = (l == 0) ? A.STF_CP : A.CP;
            len = CP + Nd;
            for (uint32_t i = threadIdx.x; i < len; i += blockDim.x) {
                float2 s = td[(i + Nd - (CP % Nd)) % Nd];
                if (l == 0) s = cscale(s, k_cover[min(i / A.pattern_len, 8u)]);
                xbuf[A.hl + i] = s;
            }
        } else {
            len = A.hl;  // resample_final_samples(): history followed by zeros
            for (uint32_t i = threadIdx.x; i < len; i += blockDim.x) xbuf[A.hl + i] = make_float2(0.f, 0.f);
        }
        __syncthreads();
        // ---- polyphase resampling of every output whose window ends in this symbol
        const uint64_t p_end = base_in + len;
        const uint64_t t_end = p_end * A.L;  // outputs need delay + m*M < t_end
        uint32_t m_end = t_end > A.delay ? static_cast<uint32_t>((t_end - A.delay + A.M - 1) / A.M) : 0u;
        m_end = min(m_end, A.n_keep);
        for (uint32_t m = m_next + threadIdx.x; m < m_end; m += blockDim.x) {
            const uint64_t t = A.delay + uint64_t(m) * A.M;
            const uint32_t p = static_cast<uint32_t>(t / A.L - base_in) + A.hl;  // index into xbuf
            const uint32_t ph = static_cast<uint32_t>(t % A.L);
            float ar = 0.f, ai = 0.f;
            for (uint32_t d = 0; d <= A.hl; ++d) {
                const float h = A.taps[ph + d * A.L];
                const float2 x = xbuf[p - d];
                ar = fmaf(x.x, h, ar);
                ai = fmaf(x.y, h, ai);
            }
            float2 y = make_float2(ar, ai);
            if (P.do_mix) y = cmul(y, phasor(P.ph0 + static_cast<double>(m) * P.inc));
            out[m] = y;
        }
        m_next = max(m_next, m_end);
        base_in = p_end;
        __syncthreads();
        // ---- keep the last hl inputs as history
        if (!flush) {
            for (uint32_t i = threadIdx.x; i < A.hl; i += blockDim.x) bufA[i] = xbuf[len + i];
            __syncthreads();
            for (uint32_t i = threadIdx.x; i < A.hl; i += blockDim.x) xbuf[i] = bufA[i];
            __syncthreads();
        }
    }
    // ---- GI and slot tail (tx.cpp:679-714)
    for (uint32_t m = m_next + threadIdx.x; m < A.S; m += blockDim.x) out[m] = make_float2(0.f, 0.f);
}

hipError_t launch_tx(const tx_args& a, uint32_t n, hipStream_t st) {
    const size_t lds = (2 * size_t(a.plan.N) + a.xbuf_len + 98 + 8) * sizeof(float2);
    hipLaunchKernelGGL(tx_kernel, dim3(n * a.N_TX), dim3(256), lds, st, a);
    return hipGetLastError();
}

}  // namespace dnrp::dev
