// Internal state of the C-ABI context shared by the host translation units (ctx.cpp: TX / RX
// phases, sync.cpp: synchronisation). Not part of the public interface.
#pragma once

#include <hip/hip_runtime.h>

#include <cmath>
#include <cstring>
#include <map>
#include <memory>
#include <string>
#include <tuple>
#include <vector>

#include "../kernels/kernels.hpp"
#include "dnrp.h"
#include "geometry.hpp"


#define HIPCHK(x)                                  \
    do {                                           \
        if ((x) != hipSuccess) return DNRP_EDEVICE; \
    } while (0)


namespace dnrp::host {

// device buffer owning wrapper
struct dbuf {
    void* p = nullptr;
    size_t n = 0;
    hipEvent_t busy = nullptr;  // per-call argument buffers: recorded after the last kernel reading it
    dbuf() = default;
    dbuf(const dbuf&) = delete;
    dbuf& operator=(const dbuf&) = delete;
    ~dbuf() {
        if (p) (void)hipFree(p);
        if (busy) (void)hipEventDestroy(busy);
    }
    // before refilling a per-call argument buffer on stream st: the kernels of an earlier call
    // (possibly on another stream) that read it must have finished
    hipError_t wait_idle(hipStream_t st) {
        if (!busy) return hipEventCreateWithFlags(&busy, hipEventDisableTiming);
        return hipStreamWaitEvent(st, busy, 0);
    }
    // after the launches reading it on stream st
    hipError_t mark_busy(hipStream_t st) {
        if (!busy && hipEventCreateWithFlags(&busy, hipEventDisableTiming) != hipSuccess) return hipErrorUnknown;
        return hipEventRecord(busy, st);
    }
    bool ensure(size_t bytes) {
        if (bytes <= n) return true;
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
        if (hipMalloc(&p, bytes) != hipSuccess) return false;
        n = bytes;
        return true;
    }
    template <typename T>
    bool upload(const std::vector<T>& v) {
        if (!ensure(std::max<size_t>(v.size() * sizeof(T), 16))) return false;
        return hipMemcpy(p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice) == hipSuccess;
    }
    template <typename T>
    T* as() const {
        return static_cast<T*>(p);
    }
};

struct pinned {
    void* p = nullptr;
    size_t n = 0;
    hipEvent_t ev = nullptr;
    ~pinned() {
        if (p) (void)hipHostFree(p);
        if (ev) (void)hipEventDestroy(ev);
    }
    void* get(size_t bytes) {
        if (!ev) (void)hipEventCreateWithFlags(&ev, hipEventDisableTiming);
        (void)hipEventSynchronize(ev);  // previous async copy out of this buffer is done
        if (bytes > n) {
            if (p) (void)hipHostFree(p);
            p = nullptr;
            n = 0;
            if (hipHostMalloc(&p, bytes, hipHostMallocDefault) != hipSuccess) return nullptr;
            n = bytes;
        }
        return p;
    }
};

dev::fft_plan make_plan(uint32_t N);
std::vector<float2> twiddles(uint32_t N);                   // forward, exp(-2 pi i j / N)
std::vector<float2> constellation(uint32_t N_bps);
std::vector<float> taps_polyphase(const geo::resampler_t& rs, uint32_t* count);
double phasor_arg(double rad);
void fill_pairs(uint32_t N_TS, uint32_t* pair, uint32_t& mod);

struct tx_tables {
    dnrp_packet_sizes q{};
    geo::tm_t tm{};
    geo::dims_t dm{};
    dev::fft_plan plan{};
    geo::resampler_t rs;
    dbuf code, stf, W, taps, taps_pp, tw, qam, qpsk, pdc_off;
    dbuf code_bin;  // [N_DF+1][1024] code per FFT bin, bin lane + 64 m at [m / 4][lane][m % 4] (streaming TX kernel, N_b_DFT_os = 1024)
    dbuf code_oh;   // [N_TS][N_DF+1][1024] one-hot W codes per antenna stream (kernels.hpp OH_*; empty: not built)
    uint32_t pcc_syms = 0;  // bit l: symbol l carries PCC cells
    uint32_t npp = 0;  // floats in taps_pp
    std::vector<float> wscale, wscale_opt;  // per codebook: standard / optimal_scaling_DAC
    std::vector<uint8_t> w_onehot;           // per codebook: one nonzero entry in every antenna row
    std::vector<uint32_t> pdc_off_h;  // host copy of maps.pdc_sym_off
};

// device copy of a geo::rx_plan_t
struct rx_plan_dev {
    uint32_t n_dops = 0, n_epochs = 0;
    bool cells_ok = true;  // every epoch fits rx_cells_kernel: <= CELL_MAX_SEGS segments, one DRS count
    dbuf dl, dmeta, segs, epochs;
    dbuf sym_op;  // [n_sym] first DRS op at symbol l, 0xFFFF: none (the front end's DRS test)
    uint32_t n_sym_op = 0;
    bool upload(const geo::rx_plan_t& p) {
        static_assert(sizeof(geo::rx_seg_t) == sizeof(dev::rx_seg), "rx_seg layout");
        static_assert(sizeof(geo::rx_epoch_t) == sizeof(dev::rx_epoch), "rx_epoch layout");
        n_dops = static_cast<uint32_t>(p.dl.size());
        n_epochs = static_cast<uint32_t>(p.epochs.size());
        for (const auto& e : p.epochs) {
            cells_ok = cells_ok && e.seg1 - e.seg0 <= dev::CELL_MAX_SEGS;
            for (uint32_t i = e.seg0; i < e.seg1; ++i) cells_ok = cells_ok && p.segs[i].drs_cnt == p.segs[e.seg0].drs_cnt;
        }
        uint32_t lmax = 0;
        for (uint32_t l : p.dl) lmax = std::max(lmax, l);
        std::vector<uint16_t> so((lmax + 2) & ~1u, 0xFFFFu);  // whole dwords (scalar loads)
        for (uint32_t d = n_dops; d-- > 0;) so[p.dl[d]] = static_cast<uint16_t>(d);
        n_sym_op = lmax + 1;
        return dl.upload(p.dl) && dmeta.upload(p.dmeta) && segs.upload(p.segs) && epochs.upload(p.epochs) && sym_op.upload(so);
    }
};

struct rx1_tables {  // per (u, b, N_eff_TX): STF/PCC phase
    uint32_t u, b, N_eff_TX, Nd, N_occ, off_lower, CP, STF_CP, n_pattern, pattern_len;
    dev::fft_plan plan{};
    geo::resampler_t rs;
    geo::maps_t maps;
    uint32_t pcc_max = 0;
    bool drs_arith = false;  // DRS tables match rx_drs_partials' arithmetic (front-end SNR sums)
    dbuf stf, tw, taps, taps_pp, drs_k, drs_v, pcc_k, pcc_sym;
    uint32_t npp = 0;  // floats in taps_pp
    rx_plan_dev bplan;  // PCC phase back end
    dbuf lut_pw[2][3], lut_w[2][3], luts;
    dbuf lut_pair_w[2][3], lut_pair_p[2][3];  // SFBC pair union windows of full symbols (rx_lut::pair_w)
    uint32_t lut_n[2][3] = {}, lut_nw[2][3] = {}, lut_T[2] = {};
    uint32_t wcap[2] = {};  // largest weight table of mode l / lr (rx_cells_kernel LDS slots)
};

struct rx2_tables {  // per (psdef): PDC phase
    dnrp_packet_sizes q{};
    geo::maps_t maps;
    dbuf pdc_k, pdc_sym;
    rx_plan_dev bplan;  // PDC phase back end
    bool sm = false;    // spatial multiplexing (N_SS > 1): MMSE cells kernel
    // MIMO report (estimator_mimo_t): wideband DRS cells, single-stream codebooks
    uint32_t N_TS = 1, ncb_tx = 0, A_tx = 0, ncb_rx = 0, A_rx = 0;
    dbuf mimo_cells, mimo_signs, Wtx, stx, Wrx, srx;
    // fused PDC receiver (kernels/rx_fused.hip): its symbol table, the phase's DRS symbols the front
    // end runs first (after the PCC phase's), whether those carry PDC cells (their bins then go to Y),
    // and the MIMO report's wideband cells in the zero-forced pilots (op << 16 | DRS cell)
    bool fused_ok = false, drs_y = false;
    uint32_t n_fsym = 0, n_drs_syms = 0;
    dbuf fsym, drs_syms, mimo_zcells;
    // epoch receiver (kernels/rx_epoch.hip): per plan epoch the front-end symbols it owns (PDC-bearing,
    // after the PCC phase, not DRS: each in exactly one epoch), and the phase's DRS symbols for the
    // DRS pass ahead of it
    bool ep_ok = false;
    uint32_t n_ep_drs = 0;
    dbuf ep_off, ep_sym, ep_drs;
};

struct netid_seq {
    uint32_t nbits = 0;
    dbuf t1, t2;
};


struct sync_tables {  // per (u, b) of the searched STF: sync_chunk_t / crosscorrelator_t constructors
    uint32_t u = 0, b = 0, n_pattern = 0, stf_len = 0, pattern = 0, step = 0, D = 0, bos = 0;
    uint32_t xc_l = 0, xc_len = 0, tmpl_len = 0, n_templates = 0, log2_fft = 0;
    float rms_min = 0.f;
    geo::resampler_t rs;  // sync resampler (RX direction)
    uint32_t m_star = 0, p_star = 0, npp = 0;
    dbuf taps, taps_pp, tmpl_f, tw_fft;
};

}  // namespace dnrp::host

struct dnrp_ctx {
    using tx_tables = dnrp::host::tx_tables;
    using rx1_tables = dnrp::host::rx1_tables;
    using rx2_tables = dnrp::host::rx2_tables;
    using netid_seq = dnrp::host::netid_seq;
    using dbuf = dnrp::host::dbuf;
    using pinned = dnrp::host::pinned;
    dnrp_cfg cfg{};
    std::map<std::tuple<uint32_t, uint32_t, uint32_t, uint32_t, uint32_t, uint32_t, uint32_t>, std::unique_ptr<tx_tables>> txt;
    std::map<std::tuple<uint32_t, uint32_t, uint32_t>, std::unique_ptr<rx1_tables>> rx1t;
    std::map<std::tuple<uint32_t, uint32_t, uint32_t, uint32_t, uint32_t, uint32_t, uint32_t>, std::unique_ptr<rx2_tables>> rx2t;
    std::map<uint32_t, std::unique_ptr<netid_seq>> netid;
    dbuf pcc_seq;
    // batch scratch
    dbuf tx_pk, rx_in, rx_st, Y, pdc_seq_ptrs, lut_d, nv_d, mimo_out;
    dbuf tx_big;  // N_b_DFT_os > 1024: DECT-rate symbols [n][N_TX][big_len] (tx.hip tx_big_sym_kernel)
    dbuf stf_part;  // [max_batch][8] double2 cs | [max_batch][8] float rms | [max_batch][8][14 b_max] float2 cells
    dbuf snr_part;  // [slot][n_sym_total][N_RX][8] double2: front-end DRS SNR partial sums
    // zero-forced DRS pilots [slot][zd_dops][N_RX][4][zd_row] (rx_front_args::zd); op zd_dops - 1 of
    // every slot stays zero (the fused receiver's op-less interlace slots), zd_key: layout it was zeroed for
    dbuf zd;
    uint32_t zd_dops = 0, zd_row = 0;
    std::tuple<void*, size_t, uint32_t, uint32_t, uint32_t> zd_key{};
    // per PCC call: the DRS SNR sums (and pilots) come from the front end (DNRP_RX_SNR_FRONT, read
    // once per PCC call so that its PDC call agrees), and the PDC phase may take the fused receiver
    bool rx_snr_front = true, rx_fused = true;
    // PDC phase in packet groups (DNRP_RX_GROUP packets, 0: one launch set): the front end of group g+1
    // on the caller's stream beside the back end of group g on rx_aux, Y of a group re-read from the
    // caches; fork / join through rx_fork / rx_join
    uint32_t rx_group = 0;
    // PDC phase through the epoch receiver (kernels/rx_epoch.hip, DNRP_RX_EPOCH): 0 off, 1 where it
    // applies and pays (N_RX >= 4), 2 wherever it applies (tests)
    uint32_t rx_epoch = 1;
    hipStream_t rx_aux = nullptr;
    hipEvent_t rx_fork = nullptr, rx_join = nullptr;
    uint32_t rx_mode = 0;  // DNRP_RX_MODE_* (dnrp_ctx_set_rx_mode)
    pinned st_tx, st_rxin, st_seq, st_rep;
    // retained RX phase-1 state: per PCC-batch slot its (u, b, N_eff_TX) tables and symbol
    // capacity; Y is laid out with the batch-wide maxima rx_nsym_cap / rx_Nf_pad
    bool rx_valid = false;
    uint32_t rx_n = 0, rx_S_in = 0, rx_nsym_cap = 0, rx_Nf_pad = 0, rx_n_windows = 0;
    const float* rx_iq = nullptr;  // the PCC call's windows: the PDC call must read the same ones
    std::vector<rx1_tables*> rx_slot_t;
    std::vector<uint32_t> rx_slot_cap;
    dbuf rx_sel, rx_sel2;  // [max_batch][2] launch packet -> slot / output row (PCC / PDC call), one slice per group
    pinned st_sel, st_sel2;
    // synchronisation: per (u, b) tables, step sums and reports
    std::map<std::pair<uint32_t, uint32_t>, std::unique_ptr<dnrp::host::sync_tables>> synct;
    dbuf sy_P, sy_C, sy_res, sy_cnt, sy_spec, sy_post, sy_state, sy_pk;
    // ring-buffer gather / continuous-stream synchronisation (stream.cpp)
    dbuf ring_start, ring_win;
    pinned st_ring, st_stream;
    // simulated channel (channel.cpp): per-call link realisations
    dbuf chan_tab;
    pinned st_chan;
    // timing: HIP events recorded on the caller's stream around every launch (DNRP_TIMING=1)
    bool timing = false;
    struct ev_pool {
        std::vector<std::pair<hipEvent_t, hipEvent_t>> ev;
        size_t used = 0;
    };
    std::map<std::string, ev_pool> ev;
    // device turbo decoding (fec.cpp dnrp_pdc_decode_batch, kernels/fec.hip): per-size tables
    // (circular-buffer lists) built at the first call, plan and work buffers
    dbuf fec_tab, fec_cbs, fec_waves, fec_work16, fec_tail, fec_bits, fec_ck, fec_cbout, fec_tbarg;
    dbuf fec_cbs2, fec_waves2, fec_map2, fec_work16b, fec_tailb, fec_cbout2;  // continuation of undecided blocks
    std::vector<uint32_t> fec_valid_off, fec_start;  // per K index ([idx][rv] for start)
    ~dnrp_ctx() {
        if (rx_aux) (void)hipStreamDestroy(rx_aux);
        if (rx_fork) (void)hipEventDestroy(rx_fork);
        if (rx_join) (void)hipEventDestroy(rx_join);
        for (auto& e : ev)
            for (auto& p : e.second.ev) {
                (void)hipEventDestroy(p.first);
                (void)hipEventDestroy(p.second);
            }
    }
    void tic(const char* name, hipStream_t s) {
        if (!timing) return;
        auto& pool = ev[name];
        if (pool.used == pool.ev.size()) {
            std::pair<hipEvent_t, hipEvent_t> p{};
            (void)hipEventCreate(&p.first);
            (void)hipEventCreate(&p.second);
            pool.ev.push_back(p);
        }
        (void)hipEventRecord(pool.ev[pool.used].first, s);
    }
    void toc(const char* name, hipStream_t s) {
        if (!timing) return;
        auto& pool = ev[name];
        (void)hipEventRecord(pool.ev[pool.used].second, s);
        ++pool.used;
    }
};
