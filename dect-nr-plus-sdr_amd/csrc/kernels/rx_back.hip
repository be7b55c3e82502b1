// RX back end of the synchronised receiver: channel estimation, equalisation, soft demapping.
//
//  rx_snr_kernel    one WG per packet: zero-forcing of every DRS symbol of the phase, SNR
//                   accumulation (estimator_snr.cpp:104-146) and the SNR-driven Wiener LUT profile
//                   pick after each DRS symbol (rx_synced.cpp:863-891). One wavefront per DRS
//                   symbol; the accumulation itself is a short serial prefix.
//  rx_cells_kernel  one WG per (packet, epoch): an epoch is a run of cell work over which the
//                   interlaced pilot buffer (channel_antenna.hpp:38-63) does not change. The WG
//                   rebuilds that buffer in LDS from the zero-forced DRS cells of Y, then every
//                   thread takes whole work units (a cell for MRC, an SFBC pair for transmit
//                   diversity): Wiener interpolation of the channel at the unit's subcarriers
//                   (rx_synced.cpp:932-946), MRC (1204-1306) or SFBC combining (1335-1392),
//                   srsRAN-style int16 soft demapping and descrambling (pcc_enc.cpp:297,
//                   pdc_enc.cpp:339-344).
// Y layout: [packet][N_RX][n_sym_total][Nf_pad] float2 (rx_fft_kernel).
#include "device_common.hpp"
#include "experiments.hpp"
#include "kernels.hpp"
#include "rx_eq.hpp"

namespace dnrp::dev {

// ===================================================================== SNR chain
constexpr uint32_t SNR_THREADS = 256, MAX_DOPS = RX_MAX_DOPS;
constexpr int SNR_ROUNDS = 4;  // DRS cells per (symbol, stream) <= 256 (b <= 16: 224)

template <int NRX>
__global__ void __launch_bounds__(SNR_THREADS) rx_snr_kernel(rx_snr_args A) {
    __shared__ double s1s[MAX_DOPS], s2s[MAX_DOPS];
    const uint32_t pkt = rx_slot_of(A.sel, blockIdx.x), nd = A.n_drs;
    const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63u, nw = SNR_THREADS / 64;
    const size_t ast = size_t(A.n_sym_total) * A.Nf_pad;
    const float2* Yp = A.Y + size_t(pkt) * NRX * ast;
    if (A.snr_part) {  // the front end's partial sums of every RX antenna (one lane each)
        for (uint32_t d = wave; d < A.n_dops; d += nw) {
            const uint32_t meta = __builtin_amdgcn_readfirstlane(A.dmeta[d]);
            const uint32_t l = __builtin_amdgcn_readfirstlane(A.dl[d]);
            const uint32_t tf = meta & 0xFFu;
            double s1 = 0.0, s2 = 0.0;
            if (lane < NRX) {
                const double2 p = A.snr_part[((size_t(pkt) * A.n_sym_total + l) * NRX + lane) * 8 + tf];
                s1 = p.x;
                s2 = p.y;
            }
            for (int o = 32; o > 0; o >>= 1) {
                s1 += __shfl_xor(s1, o);
                s2 += __shfl_xor(s2, o);
            }
            if (lane == 0) {
                s1s[d] = s1;
                s2s[d] = s2;
            }
        }
    }
    for (uint32_t d = A.snr_part ? A.n_dops : wave; d < A.n_dops; d += nw) {
        const uint32_t meta = __builtin_amdgcn_readfirstlane(A.dmeta[d]);
        const uint32_t l = __builtin_amdgcn_readfirstlane(A.dl[d]);
        const uint32_t tf = meta & 0xFFu, tl = (meta >> 8) & 0xFFu, par = (meta >> 16) & 0xFFu;
        const float2* rows = Yp + size_t(l) * A.Nf_pad;
        double s1 = 0.0, s2 = 0.0;
        // lanes take 64 consecutive DRS cells of one transmit stream for every RX antenna at once
        // (the subcarrier index and DRS value are shared by the antennas); the right neighbour of
        // the noise difference comes from the next lane, lane 63 fetches its own
        for (uint32_t t = tf; t <= tl; ++t) {
            const uint32_t* __restrict__ kb = A.drs_k + (par * 4 + (t & 3u)) * nd;
            const float* __restrict__ vv = A.drs_v + t * nd;
            // all SNR_ROUNDS rounds' index loads, then all their cells, in flight together
            uint32_t k[SNR_ROUNDS], k1[SNR_ROUNDS];
            float w[SNR_ROUNDS], w1[SNR_ROUNDS];
#pragma unroll
            for (int r = 0; r < SNR_ROUNDS; ++r) {
                const uint32_t i = 64 * r + lane;
                const bool in = i < nd, nx = lane == 63 && i + 1 < nd;
                k[r] = in ? kb[i] : 0u;
                k1[r] = nx ? kb[i + 1] : 0u;
                w[r] = in ? vv[i] : 0.f;
                w1[r] = nx ? vv[i + 1] : 0.f;
            }
            float2 y[SNR_ROUNDS][NRX], y1[SNR_ROUNDS][NRX];
#pragma unroll
            for (int r = 0; r < SNR_ROUNDS; ++r)
#pragma unroll
                for (int a = 0; a < NRX; ++a) {
                    y[r][a] = rows[a * ast + k[r]];
                    y1[r][a] = rows[a * ast + k1[r]];
                }
#pragma unroll
            for (int r = 0; r < SNR_ROUNDS; ++r) {
                const uint32_t i = 64 * r + lane;
                if (64 * r >= nd) break;
                const bool in = i < nd;
#pragma unroll
                for (int a = 0; a < NRX; ++a) {
                    const float2 v = cscale(y[r][a], w[r]);
                    float2 vn = make_float2(__shfl_down(v.x, 1), __shfl_down(v.y, 1));
                    if (lane == 63) vn = cscale(y1[r][a], w1[r]);
                    if (in) s1 += cnorm(v);
                    if (i + 1 < nd) s2 += cnorm(csub(v, vn));
                }
            }
        }
        for (int o = 32; o > 0; o >>= 1) {
            s1 += __shfl_xor(s1, o);
            s2 += __shfl_xor(s2, o);
        }
        if (lane == 0) {
            s1s[d] = s1;
            s2s[d] = s2;
        }
    }
    __syncthreads();
    if (threadIdx.x != 0) return;
    rx_pkt_state* st = A.st + pkt;
    double sn = st->snr_SN, nn = st->snr_N;
    uint32_t sn_cnt = st->snr_SN_cnt, nn_cnt = st->snr_N_cnt;
    auto snr_db = [&]() -> float {
        if (sn <= 0.0 || nn <= 0.0) return 0.f;
        const float Sa = static_cast<float>((sn - nn) / sn_cnt), Na = static_cast<float>(nn / nn_cnt);
        return 10.f * log10f(Sa / Na);
    };
    for (uint32_t d = 0; d < A.n_dops; ++d) {
        const uint32_t meta = A.dmeta[d];
        const uint32_t nts = ((meta >> 8) & 0xFFu) - (meta & 0xFFu) + 1;
        sn += s1s[d];
        nn += s2s[d] / 2.0;
        sn_cnt += A.N_RX * nts * nd;
        nn_cnt += A.N_RX * nts * (nd - 1);
        // nearest profile SNR, ties to the later profile (rx_synced.cpp:863-891)
        const float s = snr_db();
        float best = fabsf(s - A.prof_snr[0]);
        uint32_t pick = 0;
        for (uint32_t i = 1; i < 3; ++i) {
            const float dd = fabsf(s - A.prof_snr[i]);
            if (dd <= best) {
                best = dd;
                pick = i;
            }
        }
        A.lut_d[size_t(pkt) * MAX_DOPS + d] = static_cast<uint8_t>(pick);
        // noise variance per RX cell behind the pick (MMSE regularisation of spatial multiplexing)
        A.nv_d[size_t(pkt) * MAX_DOPS + d] = nn > 0.0 ? static_cast<float>(nn / nn_cnt) : 0.f;
    }
    if (A.is_pdc)
        st->snr_pdc = snr_db();
    else
        st->snr_pcc = snr_db();
}

hipError_t launch_rx_snr(const rx_snr_args& a, uint32_t n, hipStream_t st) {
    if (a.n_dops > MAX_DOPS || a.n_drs > 64 * SNR_ROUNDS || (a.snr_part && a.N_RX > 64)) return hipErrorInvalidValue;
    switch (a.N_RX) {
        case 1: hipLaunchKernelGGL(rx_snr_kernel<1>, dim3(n), dim3(SNR_THREADS), 0, st, a); break;
        case 2: hipLaunchKernelGGL(rx_snr_kernel<2>, dim3(n), dim3(SNR_THREADS), 0, st, a); break;
        case 4: hipLaunchKernelGGL(rx_snr_kernel<4>, dim3(n), dim3(SNR_THREADS), 0, st, a); break;
        case 8: hipLaunchKernelGGL(rx_snr_kernel<8>, dim3(n), dim3(SNR_THREADS), 0, st, a); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// ===================================================================== cells
constexpr uint32_t CELL_THREADS = 512;
#ifndef DNRP_CELLS_PILOT_PRE
#define DNRP_CELLS_PILOT_PRE 0  // 1: pilot sources issued before the weight-table staging: neutral (rx_pcc 0.347 /
                                // 0.349 vs 0.345 / 0.349 ms, C4SM rx_pdc 17.58 / 17.66 vs 17.58 / 17.67), off
#endif

template <int NRX, int NT, bool SM = false, int NBPS = 0>
__global__ void __launch_bounds__(CELL_THREADS) rx_cells_kernel(rx_cells_args A) {
    extern __shared__ __attribute__((aligned(16))) float2 smem[];
    const uint32_t zst = zfi_stride(A.n_drs);
    float2* zfi = smem;                                                       // [NRX][NT][zst]
    float* wtab = reinterpret_cast<float*>(zfi + NRX * NT * zst);            // slots: mode l, mode lr
    cell_seg* sg = reinterpret_cast<cell_seg*>(wtab + A.wcap[0] + A.wcap[1]);  // CELL_MAX_SEGS
    uint32_t* pairs = reinterpret_cast<uint32_t*>(sg + CELL_MAX_SEGS);       // 12
    // XCD-aware: workgroups are dealt round-robin over the 8 XCDs, so workgroup b runs on XCD b % 8;
    // the epochs of one packet are consecutive on one XCD (b / 8 = packet-of-XCD * n_epochs + epoch)
    // and re-read the packet's DRS cells from that XCD's L2 instead of HBM
    const uint32_t xs = blockIdx.x >> 3;
    const uint32_t pl = (xs / A.n_epochs) * 8 + (blockIdx.x & 7u), ep = xs % A.n_epochs;
    if (pl >= A.n_pkt) return;
    const uint32_t pkt = rx_slot_of(A.sel, pl), row = rx_row_of(A.sel, pl);
    const rx_epoch* E = A.epochs + ep;
    const uint32_t units = E->units, seg0 = E->seg0, nseg = E->seg1 - E->seg0;
    const float2* Yp = A.Y + size_t(pkt) * NRX * A.n_sym_total * A.Nf_pad;
    const uint32_t tid = threadIdx.x;
    // the epoch's segments share one DRS count (host-checked), so one LUT profile: weight table
    // slot m holds the profile's table of mode m (l / lr)
    const uint8_t* lutp = A.lut_d + size_t(pkt) * RX_MAX_DOPS;
    const uint32_t dc = nseg ? A.segs[seg0].drs_cnt : 0u;
    const uint32_t prof = dc ? lutp[dc - 1] : 0u;
    // the pilot buffer's dependent source loads first (pilot_offsets, where 2 n_drs <= threads), so
    // they overlap the weight-table staging instead of following it
    const bool ppre = DNRP_CELLS_PILOT_PRE && 2 * A.n_drs <= CELL_THREADS;  // uniform
    const bool pact = ppre && tid < 2 * A.n_drs;
    uint32_t pyk[NT] = {}, pok = 0;
    float pdv[NT] = {};
    if (pact) pilot_offsets<NT>(A, E, tid, pyk, pdv, pok);
    if (units) {
#pragma unroll
        for (uint32_t m = 0; m < 2; ++m) {
            const rx_lut LT = A.luts[m * 3 + prof];
            for (uint32_t i = tid; i < LT.nw; i += CELL_THREADS) wtab[m * A.wcap[0] + i] = LT.w[i];
        }
        if (tid < nseg) {
            const rx_seg S = A.segs[seg0 + tid];
            const rx_lut LT = A.luts[S.mode * 3 + prof];
            cell_seg c;
            c.u0 = S.u0;
            c.j0 = S.j0;
            c.l = S.l;
            c.info = (S.mode & 1u) | (S.swap & 3u) << 1 | (S.off & 0xFFu) << 4 | LT.n << 12;
            c.pw = LT.pw + size_t(S.rel) * 4 * (A.N_occ + 1);
            c.wbase = (S.mode & 1u) * A.wcap[0];
            c.pad = 0;
            sg[tid] = c;
        }
        if (tid < 12) pairs[tid] = A.pair[tid];
    }
    if constexpr (!experiment(XS_CELLS_SKIP_PRO)) {
        if (ppre)
            pilot_cells<NRX, NT>(A, Yp, zfi, tid, CELL_THREADS, pact, pyk, pdv, pok);
        else
            build_pilots<NRX, NT, cells_ai(NRX, NT)>(A, E, Yp, zfi, tid, CELL_THREADS);
    }
    __syncthreads();
    if constexpr (experiment(XS_CELLS_SKIP_MAIN)) {
        if (tid < units) A.llr[size_t(row) * A.llr_stride + tid] = static_cast<int16_t>(zfi[tid].x);
        return;
    }
    constexpr bool wave_mf = SM && experiment(XS_MMSE_MFMA) && NT == 4;
    if (!wave_mf && tid >= units) return;
    const uint8_t* __restrict__ seq = A.is_pdc ? A.pdc_seq[row] : A.pcc_seq;
    int16_t* __restrict__ llr = A.llr + size_t(row) * A.llr_stride;
    if constexpr (wave_mf) {
        // experiment: MFMA Gram (rx_eq.hpp gram_mfma) needs every lane of the wave, so the wave runs
        // a uniform trip count over clamped units and stores only its real ones
        const float nv = dc ? A.nv_d[size_t(pkt) * RX_MAX_DOPS + dc - 1] : 0.f;
        const uint32_t wf = tid & ~63u;
        if (wf >= units) return;
        const uint32_t nit = (units - wf + CELL_THREADS - 1) / CELL_THREADS;
        float2* scr = reinterpret_cast<float2*>(reinterpret_cast<char*>(smem) +
                                                (cell_lds_bytes(NRX, NT, A.n_drs, A.wcap[0], A.wcap[1]) + 15) / 16 * 16) +
                      (tid >> 6) * NRX * 4 * 24;
        auto cl = [&](uint32_t x) { return min(x, units - 1); };
        uint32_t si = 0;
        unit_a na;
        unit_sm<NRX, NT> cur;
        uint32_t u = tid;
        unit_stage_a(A, sg, nseg, si, cl(u), 1u, na);
        unit_stage_b_sm<NRX, NT>(A, sg, Yp, seq, na, cur);
        if (nit > 1) unit_stage_a(A, sg, nseg, si, cl(u + CELL_THREADS), 1u, na);
        for (uint32_t it = 0; it < nit; ++it, u += CELL_THREADS) {
            unit_sm<NRX, NT> nb;
            const bool m1 = it + 1 < nit, m2 = it + 2 < nit;
            if (m1) unit_stage_b_sm<NRX, NT>(A, sg, Yp, seq, na, nb);
            if (m2) unit_stage_a(A, sg, nseg, si, cl(u + 2 * CELL_THREADS), 1u, na);
            eq_mmse<NRX, NT, NBPS>(A, sg, zfi, wtab, zst, nv, cur, llr, scr, u < units);
            if (m1) cur = nb;
        }
        return;
    }
    if constexpr (SM) {  // spatial multiplexing: unit = one cell carrying NT symbols, MMSE (rx_eq.hpp)
        const float nv = dc ? A.nv_d[size_t(pkt) * RX_MAX_DOPS + dc - 1] : 0.f;
        uint32_t si = 0;
        unit_a na;
        unit_sm<NRX, NT> cur;
        uint32_t u = tid;
        unit_stage_a(A, sg, nseg, si, u, 1u, na);
        unit_stage_b_sm<NRX, NT>(A, sg, Yp, seq, na, cur);
        if (u + CELL_THREADS < units) unit_stage_a(A, sg, nseg, si, u + CELL_THREADS, 1u, na);
        for (; u < units; u += CELL_THREADS) {
            unit_sm<NRX, NT> nb;
            const bool m1 = u + CELL_THREADS < units, m2 = u + 2 * CELL_THREADS < units;
            if (m1) unit_stage_b_sm<NRX, NT>(A, sg, Yp, seq, na, nb);
            if (m2) unit_stage_a(A, sg, nseg, si, u + 2 * CELL_THREADS, 1u, na);
            eq_mmse<NRX, NT, NBPS>(A, sg, zfi, wtab, zst, nv, cur, llr);
            if (m1) cur = nb;
        }
        return;
    }
    constexpr uint32_t per_unit = NT == 1 ? 1u : 2u;
    // stage A two units ahead, stage B one unit ahead of eq_compute (rx_eq.hpp)
    uint32_t si = 0;
    unit_a na;
    unit_b<NRX, NT> cur;
    uint32_t u = tid;
    unit_stage_a(A, sg, nseg, si, u, per_unit, na);
    unit_stage_b<NRX, NT>(A, sg, pairs, Yp, seq, na, cur);
    if (u + CELL_THREADS < units) unit_stage_a(A, sg, nseg, si, u + CELL_THREADS, per_unit, na);
    for (; u < units; u += CELL_THREADS) {
        unit_b<NRX, NT> nb;
        const bool m1 = u + CELL_THREADS < units, m2 = u + 2 * CELL_THREADS < units;
        if (m1) unit_stage_b<NRX, NT>(A, sg, pairs, Yp, seq, na, nb);
        if (m2) unit_stage_a(A, sg, nseg, si, u + 2 * CELL_THREADS, per_unit, na);
        eq_compute<NRX, NT, NBPS>(A, sg, zfi, wtab, zst, cur, llr);
        if (m1) cur = nb;
    }
}

hipError_t launch_rx_cells(const rx_cells_args& a, uint32_t n, hipStream_t st) {
    const size_t lds = cell_lds_bytes(a.N_RX, a.NT, a.n_drs, a.wcap[0], a.wcap[1]);
    if (lds > 160 * 1024 || a.n_pkt != n) return hipErrorInvalidValue;
    const dim3 g((n + 7) / 8 * 8 * a.n_epochs), b(CELL_THREADS);
    // 256-QAM (N_bps = 8, the bench's C3 / C4) with the demapper width compiled in
#define DNRP_CELLS(R, T)                                                                 \
    if (a.N_RX == R && a.NT == T) {                                                      \
        if (a.N_bps == 8)                                                                \
            hipLaunchKernelGGL((rx_cells_kernel<R, T, false, 8>), g, b, lds, st, a);     \
        else                                                                             \
            hipLaunchKernelGGL((rx_cells_kernel<R, T>), g, b, lds, st, a);               \
        return hipGetLastError();                                                        \
    }
    DNRP_CELLS(1, 1)
    DNRP_CELLS(2, 1)
    DNRP_CELLS(4, 1)
    DNRP_CELLS(8, 1)
    DNRP_CELLS(2, 2)
    DNRP_CELLS(4, 2)
    DNRP_CELLS(8, 2)
    DNRP_CELLS(4, 4)
    DNRP_CELLS(8, 4)
#undef DNRP_CELLS
    return hipErrorInvalidValue;
}

hipError_t launch_rx_cells_sm(const rx_cells_args& a, uint32_t n, hipStream_t st) {
    size_t lds = cell_lds_bytes(a.N_RX, a.NT, a.n_drs, a.wcap[0], a.wcap[1]);
    if (experiment(XS_MMSE_MFMA) && a.NT == 4) lds = (lds + 15) / 16 * 16 + CELL_THREADS / 64 * a.N_RX * 4 * 24 * sizeof(float2);
    if (lds > 160 * 1024 || a.n_pkt != n) return hipErrorInvalidValue;
    const dim3 g((n + 7) / 8 * 8 * a.n_epochs), b(CELL_THREADS);
    // the demapper width compiled in for 64- and 256-QAM
#define DNRP_CELLS_SM(R, T)                                                              \
    if (a.N_RX == R && a.NT == T) {                                                      \
        if (a.N_bps == 6)                                                                \
            hipLaunchKernelGGL((rx_cells_kernel<R, T, true, 6>), g, b, lds, st, a);      \
        else if (a.N_bps == 8)                                                           \
            hipLaunchKernelGGL((rx_cells_kernel<R, T, true, 8>), g, b, lds, st, a);      \
        else                                                                             \
            hipLaunchKernelGGL((rx_cells_kernel<R, T, true>), g, b, lds, st, a);         \
        return hipGetLastError();                                                        \
    }
    DNRP_CELLS_SM(2, 2)
    DNRP_CELLS_SM(4, 2)
    DNRP_CELLS_SM(8, 2)
    DNRP_CELLS_SM(4, 4)
    DNRP_CELLS_SM(8, 4)
#undef DNRP_CELLS_SM
    return hipErrorInvalidValue;
}

// ===================================================================== MIMO report
// estimator_mimo.cpp:80-222 (mode_single_spatial_stream_3_7, metric HIGHEST_MIN_RX_POWER): lane wm
// scores codebook entry wm (min over the receive side of |sum_tx sum_c H w|, times the entry's
// scaling), the first maximum wins. H: the latest zero-forced DRS value of each (rx, ts) at the 4
// wideband cells (RX_SYNCED_PARAM_MIMO_N_WIDEBAND_CELLS), float sums in the reference's order.
__device__ uint32_t mimo_pick(const float2* H, uint32_t N_TX_virt, uint32_t N_RX_virt, bool transposed, uint32_t N_TS,
                              const float2* W, const float* sc, uint32_t A0, uint32_t ncb, uint32_t lane) {
    float best = -1.0e6f;
    uint32_t bidx = 0xFFFFFFFFu;
    for (uint32_t wm = A0 + lane; wm < ncb; wm += 64) {
        float power_inner = 1.0e6f;
        for (uint32_t rx = 0; rx < N_RX_virt; ++rx) {
            float2 sum = make_float2(0.f, 0.f);
            for (uint32_t tx = 0; tx < N_TX_virt; ++tx) {
                const float2 w = W[wm * N_TX_virt + tx];
                const uint32_t hrx = transposed ? tx : rx, hts = transposed ? rx : tx;
                float2 part = make_float2(0.f, 0.f);
                for (uint32_t c = 0; c < 4; ++c) part = cadd(part, cmul(H[(hrx * N_TS + hts) * 4 + c], w));
                sum = cadd(sum, part);
            }
            const float p = hypotf(sum.x, sum.y);
            if (p < power_inner) power_inner = p;
        }
        power_inner *= sc[wm];
        if (best < power_inner) {
            best = power_inner;
            bidx = wm;
        }
    }
    for (int o = 32; o > 0; o >>= 1) {
        const float ob = __shfl_xor(best, o);
        const uint32_t oi = __shfl_xor(bidx, o);
        if (ob > best || (ob == best && oi < bidx)) {
            best = ob;
            bidx = oi;
        }
    }
    return bidx;
}

__global__ void __launch_bounds__(64) rx_mimo_kernel(rx_mimo_args A) {
    __shared__ float2 H[8 * 8 * 4];
    const uint32_t pkt = rx_slot_of(A.sel, blockIdx.x), row = rx_row_of(A.sel, blockIdx.x), lane = threadIdx.x;
    const float2* Yp = A.Y + size_t(pkt) * A.N_RX * A.n_sym_total * A.Nf_pad;
    for (uint32_t e = lane; e < A.N_RX * A.N_TS * 4; e += 64) {
        const uint32_t rx = e / (A.N_TS * 4), tc = e % (A.N_TS * 4);
        if (A.zd) {  // the zero-forced pilots of the fused receiver: the same values, sign applied
            const uint32_t zc = A.zcells[tc];
            H[e] = A.zd[(((size_t(pkt) * A.zd_dops + (zc >> 16)) * A.N_RX + rx) * 4 + tc / 4) * A.zd_row + (zc & 0xFFFFu)];
            continue;
        }
        const uint32_t cell = A.cells[tc];
        H[e] = cscale(Yp[(size_t(rx) * A.n_sym_total + (cell >> 16)) * A.Nf_pad + (cell & 0xFFFFu)], A.signs[tc]);
    }
    __syncthreads();
    const uint32_t idx = A.N_TS == 1 ? 0u : mimo_pick(H, A.N_TS, A.N_RX, false, A.N_TS, A.Wtx, A.stx, A.A_tx, A.ncb_tx, lane);
    const uint32_t idr = A.N_RX == 1 ? 0u : mimo_pick(H, A.N_RX, A.N_TS, true, A.N_TS, A.Wrx, A.srx, A.A_rx, A.ncb_rx, lane);
    if (lane == 0) {
        A.out[3 * row] = A.N_TS;
        A.out[3 * row + 1] = idx;
        A.out[3 * row + 2] = idr;
    }
}

hipError_t launch_rx_mimo(const rx_mimo_args& a, uint32_t n, hipStream_t st) {
    if (a.N_RX > 8 || a.N_TS > 8) return hipErrorInvalidValue;
    hipLaunchKernelGGL(rx_mimo_kernel, dim3(n), dim3(64), 0, st, a);
    return hipGetLastError();
}

}  // namespace dnrp::dev
