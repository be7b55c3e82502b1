// PDC phase per (packet, epoch) workgroup: front end and equaliser in one launch.
//
// The Y path runs the front end over every PDC symbol of the batch (rx_fft_wave_ct_kernel), stores the
// occupied bins to Y in HBM and reads them back in rx_cells_kernel one launch later: 35 GB written and
// read again per 16384-slot C4 chunk. Here one workgroup owns a (packet, epoch) -- an epoch is the run
// of cell work over one interlaced pilot buffer (rx_back.hip) -- and
//   1. its 8 wavefronts run the front end of the epoch's symbols for every RX antenna (the wave
//      front end of rx.hip: span staged in the wave's LDS region, 9/10 polyphase with compile-time
//      taps + mixer, wave_fft1024, amplitude and STO derotation), the bins stored to the packet's Y
//      rows with plain stores;
//   2. after a workgroup barrier the same workgroup equalises the epoch (rx_cells_kernel's body:
//      pilot buffer and Wiener tables in LDS aliased over the front end's wave regions, Wiener
//      interpolation, MRC / SFBC combining, int16 demap, descramble) from those rows, which it wrote
//      microseconds earlier: the reads are served by the L2 / Infinity Cache instead of HBM.
// Symbols of the phase read by no epoch's cells, and the DRS symbols (their pilots and SNR sums feed
// the SNR chain's LUT picks of every later epoch, rx_synced.cpp:863-891), run before in the DRS pass
// (rx_fft_wave_ct_kernel on the symbol list, then rx_snr_kernel). Every front-end symbol belongs to
// exactly one epoch (host-checked), so no workgroup reads a row another one writes.
// Reference: rx_synced.cpp:711-771 (front end), 893-949 + 1028-1163 + 1335-1392 (equalisation).
#include "device_common.hpp"
#include "experiments.hpp"
#include "kernels.hpp"
#include "rx_eq.hpp"
#include "rx_front.hpp"

namespace dnrp::dev {

constexpr uint32_t EP_THREADS = 512, EP_WAVES = EP_THREADS / 64;
#ifndef DNRP_EP_YNT
#define DNRP_EP_YNT 0  // 1: nontemporal Y stores (A/B; plain stores keep the rows for the equaliser)
#endif
#ifndef DNRP_EP_AMAJOR
#define DNRP_EP_AMAJOR 0  // 1: tasks antenna-major (a wave's tasks are consecutive symbols of one antenna)
#endif

__host__ __device__ inline size_t ep_front_lds() { return size_t(EP_WAVES) * rxw_region(9, 10, pp_block<9, 10, 24>::W) * sizeof(float2); }

#ifndef DNRP_EP_PREFETCH
#define DNRP_EP_PREFETCH 1  // the pilot buffer's source loads issued before the phase barrier
#endif

template <int NRX, int NT, int NBPS>
__global__ void __launch_bounds__(EP_THREADS) __attribute__((amdgpu_waves_per_eu(4))) rx_epoch_kernel(rx_epoch_args X) {
    extern __shared__ __attribute__((aligned(16))) float2 smem[];
    constexpr int LR = 9, MR = 10, HLR = 24;
    const rx_front_args& F = X.F;
    const rx_cells_args& A = X.C;
    // XCD-aware as rx_cells_kernel: workgroup b runs on XCD b % 8, the epochs of one packet
    // consecutive on one XCD
    const uint32_t xs = blockIdx.x >> 3;
    const uint32_t pl = (xs / A.n_epochs) * 8 + (blockIdx.x & 7u), ep = xs % A.n_epochs;
    if (pl >= A.n_pkt) return;  // uniform per workgroup
    const uint32_t pkt = rx_slot_of(A.sel, pl), row = rx_row_of(A.sel, pl);
    const uint32_t tid = threadIdx.x, w = tid >> 6;

    // ---- 1. front end of the epoch's symbols, task = (symbol, antenna), wave w takes w, w + 8, ...
    {
        const uint32_t region = rxw_region(LR, MR, pp_block<LR, MR, HLR>::W);
        float2* R = smem + w * region;
        const uint32_t s0 = X.ep_off[ep], ntask = experiment(XS_EP_SKIP_FE) ? 0u : (X.ep_off[ep + 1] - s0) * NRX;
        const uint32_t lane0 = tid & 63u;
        const rx_pkt_in in = F.pin[pkt];
        const rx_pkt_state S = F.st[pkt];
        const int64_t q_hi = static_cast<int64_t>(F.S_in) - in.fine_peak, q_lo = in.fine_peak < 0 ? -in.fine_peak : 0;
        const float2 w1_ = wfft_tw<-1>(F.tw, 4 * (lane0 & 15u)), wl_ = wfft_tw<-1>(F.tw, lane0);
#pragma unroll 1
        for (uint32_t t = w; t < ntask; t += EP_WAVES) {
            // lane-derived values opaque per task (as rx_fft_wave_ct_kernel: no hoisting that spills)
            uint32_t lane = tid & 63u;
            float2 w1 = w1_, wl = wl_;
            asm volatile("" : "+v"(lane), "+v"(w1.x), "+v"(w1.y), "+v"(wl.x), "+v"(wl.y));
            const uint32_t ns = X.ep_off[ep + 1] - s0;
            const uint32_t l = DNRP_EP_AMAJOR ? X.ep_sym[s0 + t % ns] : X.ep_sym[s0 + t / NRX];
            const uint32_t a = DNRP_EP_AMAJOR ? t / ns : t % NRX;
            const float2* src = F.iq + (size_t(in.win) * NRX + a) * F.S_in + in.fine_peak;
            const rx_span_t sp = rx_span<LR, MR, HLR>(F, l);
            if (t != w) __builtin_amdgcn_wave_barrier();  // the previous task's reads of R are done
            if (sp.in0 >= q_lo && sp.in0 + sp.n_in < q_hi)
                stage_span_x2<10>(R, src, sp.in0, sp.n_in, lane);
            else
                stage_span_lo<20>(R, src, sp.in0, sp.n_in, q_lo, q_hi, lane, 64);
            __builtin_amdgcn_wave_barrier();
            rx_resample_ct<LR, MR, HLR>(F, in, S, sp, R, lane);
            const size_t yimg = experiment(XS_EP_SLOTY) ? blockIdx.x % (64u * A.n_epochs) : pkt;
            float2* Yrow = F.Y + ((yimg * NRX + a) * F.n_sym_total + l) * F.Nf_pad;
            rx_fft_bins<true>(F, S, R, lane, [&](uint32_t k, float2 v) {
                if constexpr (DNRP_EP_YNT) {
                    typedef float f2v __attribute__((ext_vector_type(2)));
                    __builtin_nontemporal_store(f2v{v.x, v.y}, reinterpret_cast<f2v*>(Yrow + k));
                } else {
                    Yrow[k] = v;
                }
            }, w1, wl);
        }
    }
    // The pilot buffer's global loads (build_pilots' sources and cells: three dependent round trips)
    // issued by every wave right after its last front-end task, while the workgroup waits at the phase
    // barrier for the waves still transforming; stored to LDS after it (the LDS is the front end's
    // until then). One thread per (pilot index pi, interlace slot po), NT x NRX cells each; the same
    // loads and values as build_pilots. pre = the geometry fits (2 n_drs <= threads).
    const rx_epoch* E = A.epochs + ep;
    const float2* Yp = A.Y + size_t(pkt) * NRX * A.n_sym_total * A.Nf_pad;
    const uint8_t* lutp = A.lut_d + size_t(pkt) * RX_MAX_DOPS;
    const uint32_t nd = A.n_drs;
    const bool pre = DNRP_EP_PREFETCH && 2 * nd <= EP_THREADS;  // uniform
    const bool pact = pre && tid < 2 * nd;
    uint32_t pyk[NT] = {}, pok = 0;
    float pdv[NT] = {};
    if (pact) pilot_offsets<NT>(A, E, tid, pyk, pdv, pok);
    // the weight tables' sources (LUT profile pick -> table -> rows: uniform) and the segment
    // descriptors, also before the barrier
    const uint32_t units = E->units, seg0 = E->seg0, nseg = E->seg1 - E->seg0;
    const uint32_t dc = nseg ? A.segs[seg0].drs_cnt : 0u;
    const uint32_t prof = dc ? lutp[dc - 1] : 0u;
    const rx_lut LW0 = A.luts[prof], LW1 = A.luts[3 + prof];  // the two modes' weight tables (uniform)
    cell_seg pc{};
    const bool has_c = units && tid < nseg;
    if (DNRP_EP_PREFETCH && has_c) {
        const rx_seg Sg = A.segs[seg0 + tid];
        const rx_lut LT = A.luts[Sg.mode * 3 + prof];
        pc.u0 = Sg.u0;
        pc.j0 = Sg.j0;
        pc.l = Sg.l;
        pc.info = (Sg.mode & 1u) | (Sg.swap & 3u) << 1 | (Sg.off & 0xFFu) << 4 | LT.n << 12;
        pc.pw = LT.pw + size_t(Sg.rel) * 4 * (A.N_occ + 1);
        pc.wbase = (Sg.mode & 1u) * A.wcap[0];
        pc.pad = 0;
    }
    __syncthreads();  // the epoch's rows written (workgroup-scope release / acquire), LDS free again
    if constexpr (experiment(XS_EP_SKIP_EQ)) return;

    // ---- 2. equalisation of the epoch (rx_cells_kernel, MRC / SFBC)
    const uint32_t zst = zfi_stride(A.n_drs);
    float2* zfi = smem;                                                       // [NRX][NT][zst]
    float* wtab = reinterpret_cast<float*>(zfi + NRX * NT * zst);            // slots: mode l, mode lr
    cell_seg* sg = reinterpret_cast<cell_seg*>(wtab + A.wcap[0] + A.wcap[1]);  // CELL_MAX_SEGS
    uint32_t* pairs = reinterpret_cast<uint32_t*>(sg + CELL_MAX_SEGS);       // 12
    if (units) {
#pragma unroll
        for (uint32_t m = 0; m < 2; ++m) {
            const rx_lut LT = m ? LW1 : LW0;
            for (uint32_t i = tid; i < LT.nw; i += EP_THREADS) wtab[m * A.wcap[0] + i] = LT.w[i];
        }
        if (DNRP_EP_PREFETCH && has_c) {
            sg[tid] = pc;
        } else if (tid < nseg) {
            const rx_seg Sg = A.segs[seg0 + tid];
            const rx_lut LT = A.luts[Sg.mode * 3 + prof];
            cell_seg c;
            c.u0 = Sg.u0;
            c.j0 = Sg.j0;
            c.l = Sg.l;
            c.info = (Sg.mode & 1u) | (Sg.swap & 3u) << 1 | (Sg.off & 0xFFu) << 4 | LT.n << 12;
            c.pw = LT.pw + size_t(Sg.rel) * 4 * (A.N_occ + 1);
            c.wbase = (Sg.mode & 1u) * A.wcap[0];
            c.pad = 0;
            sg[tid] = c;
        }
        if (tid < 12) pairs[tid] = A.pair[tid];
    }
    if (pre) {
        pilot_cells<NRX, NT>(A, Yp, zfi, tid, EP_THREADS, pact, pyk, pdv, pok);
    } else {
        build_pilots<NRX, NT, cells_ai(NRX, NT)>(A, E, Yp, zfi, tid, EP_THREADS);
    }
    if constexpr (experiment(XS_EP_SLOTY)) Yp = A.Y + size_t(blockIdx.x % (64u * A.n_epochs)) * NRX * A.n_sym_total * A.Nf_pad;
    __syncthreads();
    if (tid >= units) return;
    const uint8_t* __restrict__ seq = A.pdc_seq[row];
    int16_t* __restrict__ llr = A.llr + size_t(row) * A.llr_stride;
    constexpr uint32_t per_unit = NT == 1 ? 1u : 2u;
    // stage A two units ahead, stage B one unit ahead of eq_compute (rx_eq.hpp)
    uint32_t si = 0;
    unit_a na;
    unit_b<NRX, NT> cur;
    uint32_t u = tid;
    unit_stage_a(A, sg, nseg, si, u, per_unit, na);
    unit_stage_b<NRX, NT>(A, sg, pairs, Yp, seq, na, cur);
    if (u + EP_THREADS < units) unit_stage_a(A, sg, nseg, si, u + EP_THREADS, per_unit, na);
    for (; u < units; u += EP_THREADS) {
        unit_b<NRX, NT> nb;
        const bool m1 = u + EP_THREADS < units, m2 = u + 2 * EP_THREADS < units;
        if (m1) unit_stage_b<NRX, NT>(A, sg, pairs, Yp, seq, na, nb);
        if (m2) unit_stage_a(A, sg, nseg, si, u + 2 * EP_THREADS, per_unit, na);
        eq_compute<NRX, NT, NBPS>(A, sg, zfi, wtab, zst, cur, llr);
        if (m1) cur = nb;
    }
}

bool rx_epoch_supported(uint32_t N_RX, uint32_t NT) {
    return (NT == 1 && (N_RX == 1 || N_RX == 2 || N_RX == 4)) || (NT == 2 && (N_RX == 2 || N_RX == 4)) || (NT == 4 && N_RX == 4);
}

size_t rx_epoch_lds(const rx_cells_args& a) {
    return std::max(ep_front_lds(), cell_lds_bytes(a.N_RX, a.NT, a.n_drs, a.wcap[0], a.wcap[1]));
}

hipError_t launch_rx_epoch(const rx_epoch_args& x, uint32_t n, hipStream_t st) {
    const rx_cells_args& a = x.C;
    const size_t lds = rx_epoch_lds(a);
    if (lds > 160 * 1024 || a.n_pkt != n || x.F.plan.N != 1024 || !rx_epoch_supported(a.N_RX, a.NT)) return hipErrorInvalidValue;
    const dim3 g((n + 7) / 8 * 8 * a.n_epochs), b(EP_THREADS);
#define DNRP_EP(R, T)                                                                   \
    if (a.N_RX == R && a.NT == T) {                                                     \
        if (a.N_bps == 8)                                                               \
            hipLaunchKernelGGL((rx_epoch_kernel<R, T, 8>), g, b, lds, st, x);           \
        else                                                                            \
            hipLaunchKernelGGL((rx_epoch_kernel<R, T, 0>), g, b, lds, st, x);           \
        return hipGetLastError();                                                       \
    }
    DNRP_EP(1, 1)
    DNRP_EP(2, 1)
    DNRP_EP(4, 1)
    DNRP_EP(2, 2)
    DNRP_EP(4, 2)
    DNRP_EP(4, 4)
#undef DNRP_EP
    return hipErrorInvalidValue;
}

}  // namespace dnrp::dev
