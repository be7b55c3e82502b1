// ORACLE — TEST INFRASTRUCTURE ONLY (see oracle.hpp header).
#pragma once

#include <complex>
#include <cstdint>
#include <vector>

#include "oracle.hpp"

namespace orc {

// mimo_report_t index where the reference defines no result (estimator_mimo.cpp:180 asserts)
constexpr uint32_t MIMO_REF_UNDEFINED = 0xFFFFFFFEu;

struct cfg_t {  // worker_pool_config_t subset: radio device class maxima + resampling
    uint32_t u_max = 8, b_max = 16, os_min = 1, L = 10, M = 9;
    bool chestim_mode_lr = true;  // phy.json chestim_mode_lr_default
    uint32_t stride = 2;          // phy.json chestim_mode_lr_t_stride_default
};

struct tx_desc_t {  // tx_descriptor_t + tx_meta_t subset (tx_descriptor.hpp, tx_meta.hpp)
    uint32_t codebook_index = 0, network_id = 0, plcf_type = 1, GI_percentage = 5;
    float DAC_scale = 1.0f;
    bool optimal_scaling_DAC = false;
    double iq_phase_rad = 0.0, iq_phase_increment_rad = 0.0;
};

struct rx_in_t {  // sync_report_t subset + HARQ scrambling parameters
    const float* iq;  // [N_RX][S_in] interleaved cf32
    uint32_t N_RX, S_in;
    int64_t fine_peak;  // sync_report_t::fine_peak_time_64 relative to iq[0]
    double cfo_rad;     // cfo_fractional_rad + cfo_integer_rad
    uint32_t network_id, plcf_type;
    const float* sync_rms = nullptr;  // sync_report_t::rms_array[8] (nullable)
    bool sm_mmse = false;             // demodulate N_SS > 1 by MMSE (not in the reference, rx_synced.cpp:1331)
};

struct rx_out_t {
    std::vector<int16_t> pcc_llr, pdc_llr;   // descrambled
    std::vector<float> pcc_llr_f, pdc_llr_f; // pre-quantisation values, descrambled
    std::vector<float> rms;
    float cfo_fine_rad = 0, sto_fractional = 0, snr_pcc_db = 0, snr_pdc_db = 0;
    uint32_t mimo_N_TS_other = 0, mimo_idx = 0, mimo_idx_reciprocal = 0;  // mimo_report_t (MIMO_REF_UNDEFINED: none)
};

struct dims_t {
    uint32_t N_b_DFT_os, N_b_DFT, N_b_OCC, off_lower, CP_os, STF_CP_os;
    uint32_t N_no_GI_os, N_no_GI_os_rs, N_packet_os_rs, n_pattern, pattern_len;
    void init(const cfg_t& cfg, const packet_sizes_t& ps);
    uint32_t transmit_len(uint32_t gi_percentage) const;
};

uint32_t pdc_c_init(uint32_t network_id, uint32_t plcf_type);
void demap_float(const cd& y, uint32_t N_bps, double* L);
int16_t llr_to_i16(double v);

template <typename R>
void tx_packet(const cfg_t& cfg, const packet_sizes_t& ps, const tx_desc_t& d, const uint8_t* pcc_d,
               const uint8_t* pdc_d, std::vector<std::vector<std::complex<R>>>& out, uint32_t S_slot);

template <typename R>
void rx_packet(const cfg_t& cfg, const packet_sizes_t& ps, const rx_in_t& in, rx_out_t& out);


// ---------------------------------------------------------------- synchronisation (oracle_sync.cpp)
struct sync_cfg_t {  // radio device class minima u/b (sync_chunk.cpp:54-57), resampler L/M (TX values)
    uint32_t u = 8, b = 16, os_min = 1, L = 10, M = 9;
    uint32_t N_ant = 1, N_ant_limited = 1;  // physical antennas (templates), antennas searched
    uint32_t chunk_len = 0;                 // hw samples of the chunk (search covers A + B)
};
struct sync_geom_t {
    uint32_t n_pattern, bos, stf_len, pattern, step, A, B, C, D, search_len, lb_len;
    uint32_t xc_l, xc_len, tmpl_len, n_templates;
    float rms_min;
};
struct sync_out_t {  // sync_report_t (sync_report.hpp:29-98)
    uint32_t found, det_ant;
    float det_rms, det_metric;
    uint32_t det_time, det_time_jb, coarse_local;
    int64_t coarse_64;
    float coarse_metric[8], rms[8];
    float cfo_frac;
    uint32_t u, b, N_eff_TX, fine_local;
    int64_t fine_64;
    float xc_metric[4];
    uint32_t xc_idx[4];
};
sync_geom_t sync_geometry(const sync_cfg_t& c);
std::vector<cd> stf_template(const sync_cfg_t& c, uint32_t N_eff_TX);
template <typename R>
std::vector<sync_out_t> sync_search(const sync_cfg_t& c, const float* iq, uint32_t S_win, uint32_t max_reports);

}  // namespace orc
