// ORACLE — TEST INFRASTRUCTURE ONLY.
//
// CPU restatement of the reference DECT NR+ lower-PHY path (maxpenner/DECT-NR-Plus-SDR,
// lib/src/phy + lib/src/sections_part3) used as the parity checker for the HIP path and as the
// CPU baseline ("port") in bench.py. Only tests/, __graft_entry__.smoke() and bench.py's
// cpu_baseline leg may load it. The product library (dect-nr-plus-sdr_amd/) never links it.
//
// Pinning status:
//   * pinned against the reference's own compiled sources (oracle/_ref, built by
//     oracle/Makefile from /root/reference): numerologies, tm_mode, mcs, transport block size,
//     packet structure lengths, Kaiser resampler taps, Bessel/sinc channel statistics.
//   * pinned against SURVEY.md §8 numbers produced from the reference sources:
//     N_PDC_subc / G / N_TB for the benchmark configurations.
//   * parity unpinned (srsRAN semantics absent from the image, restated from 3GPP TS 36.211 /
//     srsRAN release_23_11 behaviour): LTE constellation tables, int16 soft demapper scale and
//     rounding, Gold sequence; the STF/DRS/PCC/PDC cell maps are restated from the reference's
//     sections_part3 code (which cannot be compiled here without srsRAN headers).
#pragma once

#include <complex>
#include <cstdint>
#include <vector>

namespace orc {

using cd = std::complex<double>;
using cf = std::complex<float>;

// ---------------------------------------------------------------- configuration types
struct psdef_t {  // sections_part3/derivative/packet_sizes_def.hpp
    uint32_t u, b, PacketLengthType, PacketLength, tm_mode_index, mcs_index, Z;
};

struct numerology_t {  // sections_part3/numerologies.cpp:27-70
    uint32_t u, b, delta_u_f, N_SLOT_u_symb, N_SLOT_u_subslot, N_b_DFT, N_b_CP, N_b_OCC;
    uint32_t N_guards_top, N_guards_bottom;
    double T_u_symb;
};

struct tm_mode_t {  // sections_part3/tm_mode.cpp:27-137
    uint32_t index, N_eff_TX, N_SS, N_TS, N_TX;
    bool cl;
};

struct mcs_t {  // sections_part3/mcs.cpp:27-105
    uint32_t index, N_bps, R_num, R_den;
};

struct packet_sizes_t {  // sections_part3/derivative/packet_sizes.cpp:99-236
    psdef_t psdef;
    numerology_t num;
    tm_mode_t tm;
    mcs_t mcs;
    uint32_t N_PACKET_symb, N_DF_symb, N_PDC_subc, N_DRS_subc, G, N_PDC_bits, N_TB_bits, C;
    uint32_t N_samples_STF, N_samples_STF_CP_only, N_samples_DF, N_samples_GI;
    uint32_t N_samples_packet_no_GI, N_samples_packet;
};

numerology_t get_numerology(uint32_t u, uint32_t b);
tm_mode_t get_tm_mode(uint32_t index);
mcs_t get_mcs(uint32_t index);
uint32_t get_N_TB_bits(uint32_t N_SS, uint32_t N_PDC_subc, uint32_t N_bps, uint32_t Rn,
                       uint32_t Rd, uint32_t Z);
bool get_packet_sizes(const psdef_t& d, packet_sizes_t& q);
void special_values(float z, float* out5);

// ---------------------------------------------------------------- geometry tables
// Transmit-stream vector index i in [0, N_b_OCC] maps to subcarrier k = i - N_b_OCC/2.
std::vector<int> k_b_OCC(uint32_t b);
// STF values (length N_b_OCC+1) with DC, scale 1.0 (tx_rx.cpp:71, stf.cpp:27-88,185-285)
std::vector<cd> stf_values(uint32_t b, uint32_t N_eff_TX, double scale = 1.0);
// DRS cell indices (drs.cpp:196-212): parity n%2, transmit stream t (0..3) -> N_b_OCC/4 indices
std::vector<uint32_t> drs_k_i(uint32_t b, uint32_t t, uint32_t n_parity);
// DRS values (drs.cpp:214-254) for transmit stream t (0..7)
std::vector<double> drs_y(uint32_t b, uint32_t t);
// PCC linear indices (pcc.cpp:132-259) -> per-symbol lists (l, k_i)
void pcc_cells(uint32_t b, uint32_t N_TS, std::vector<uint32_t>& l_sym,
               std::vector<std::vector<uint32_t>>& k_per_sym);
// PDC per-symbol cell lists for an actual packet (pdc.cpp:31-205 incl. repetition semantics)
std::vector<std::vector<uint32_t>> pdc_cells_packet(uint32_t b, uint32_t N_TS, uint32_t N_DF);
// DRS symbol schedule for a packet (drs.cpp:90-127): per DF symbol l: ts_first, ts_last, parity
struct drs_sym_t {
    uint32_t l, ts_first, ts_last, k_parity, y_hi;  // y_hi: 1 if values for TS 4..7
};
std::vector<drs_sym_t> drs_schedule(uint32_t N_TS, uint32_t N_DF);

// Transmit diversity (transmit_diversity_precoding.cpp:28-95)
uint32_t txdiv_modulo(uint32_t N_TS);
void txdiv_pair(uint32_t N_TS, uint32_t i_mod, uint32_t& A, uint32_t& B);
// Beamforming matrices (beamforming_and_antenna_port_mapping.cpp:27-320): row-major [N_TX][N_TS]
std::vector<cd> W_matrix(uint32_t N_TS, uint32_t N_TX, uint32_t codebook);
double W_scaling(uint32_t N_TS, uint32_t N_TX, uint32_t codebook);
double W_scaling_optimal_DAC(uint32_t N_TS, uint32_t N_TX, uint32_t codebook);  // beamforming_...mapping.cpp:146-186
extern const float STF_COVER_SEQ[9];  // stf.hpp:146-151 (cover sequence active)
uint32_t W_codebook_max(uint32_t N_TS, uint32_t N_TX);

// LTE Gold sequence (3GPP TS 36.211 §7.2), bits 0/1
std::vector<uint8_t> gold_sequence(uint32_t c_init, uint32_t len);

// LTE constellations (3GPP TS 36.211 §7.1), index = N_bps bits MSB first
std::vector<cd> constellation(uint32_t N_bps);

// Kaiser low-pass design, float arithmetic as in phy/filter/kaiser.cpp:35-122
std::vector<float> kaiser(float f_pass, float f_stop, float ripple_dB, float att_dB, float fs,
                          bool force_odd);

// Rational polyphase resampler (resampler.cpp:56-298) as a closed-form stream operator.
struct resampler_t {
    uint32_t L = 1, M = 1, filter_length = 0, delay = 0, hl = 0;  // hl = history length
    std::vector<float> h;                                      // taps * L, zero padded
    void design(uint32_t L, uint32_t M, uint32_t os_min);
    // number of outputs for N inputs incl. final flush (get_N_samples_after_resampling + flush)
    uint64_t n_out_no_flush(uint64_t N) const;
};

// ---------------------------------------------------------------- channel estimation LUTs
struct chest_lut_t {  // channel_lut.cpp:168-350 for one (lut kind, b)
    uint32_t ps_t_length = 0, nof_interp = 0, N_f = 0;
    std::vector<uint32_t> idx_pilot;    // [t][ts(4)][f]
    std::vector<uint32_t> idx_weight;   // [t][ts(4)][f]
    std::vector<float> weights;         // [n_vec][nof_interp]
    uint32_t pilot(uint32_t t, uint32_t ts, uint32_t f) const {
        return idx_pilot[(t * 4 + ts) * N_f + f];
    }
    uint32_t weight(uint32_t t, uint32_t ts, uint32_t f) const {
        return idx_weight[(t * 4 + ts) * N_f + f];
    }
};
struct chest_stats_t {
    double delta_u_f, T_u_symb, nu_max_hz, tau_rms_sec, snr_db, sigma;
    uint32_t n_lr, n_l;
};
// Three SNR profiles of rx_synced_param.hpp:216-232 for numerology u_max
std::vector<chest_stats_t> chest_profiles(uint32_t u_max);
// N_step_virtual in {0,5,10}; b_max decides weight-vector dedupe order
chest_lut_t build_chest_lut(uint32_t N_step_virtual, uint32_t b, uint32_t b_max,
                            const chest_stats_t& st);

}  // namespace orc
