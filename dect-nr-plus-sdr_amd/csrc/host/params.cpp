// Host-only queries of the reference parameters the library is built on (include/dnrp.h
// dnrp_query_param / dnrp_param_name) and of the radio device classes (dnrp_get_radio_device_class).
// Every value comes from csrc/params.hpp, the constants the host code and kernels actually use;
// the names are the reference's own macro / field names so tests/test_oracle_pins.py can compare
// them one by one with the values the reference headers compile to.
#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "../params.hpp"
#include "dnrp.h"
#include "geometry.hpp"
#include "kernels.hpp"

namespace {

using namespace dnrp::prm;

struct entry {
    std::string name;
    double value;
};

std::vector<entry> build_table() {
    std::vector<entry> t;
    auto add = [&](const char* n, double v) { t.push_back({n, v}); };
    add("SECTIONS_PART_3_STF_COVER_SEQUENCE_ACTIVE", STF_COVER_SEQUENCE_ACTIVE);
    // sync_param.hpp
    add("RX_SYNC_PARAM_MAX_NOF_BUFFERABLE_SYNC_BEFORE_ACQUIRING_BATON", SYNC_MAX_BUFFERABLE);
    add("RX_SYNC_PARAM_AUTOCORRELATOR_ANTENNA_LIMIT", SYNC_ANTENNA_LIMIT);
    add("RX_SYNC_PARAM_SYNC_TIME_UNIQUE_LIMIT_IN_STF_PATTERNS_DP", SYNC_TIME_UNIQUE_LIMIT_PATTERNS);
    add("RX_SYNC_PARAM_AUTOCORRELATOR_DETECTION_OVERLAP_LENGTH_IN_STFS_DP", SYNC_OVERLAP_STFS);
    add("RX_SYNC_PARAM_AUTOCORRELATOR_DETECTION_STEP_DIVIDER", SYNC_STEP_DIVIDER);
    add("RX_SYNC_PARAM_AUTOCORRELATOR_DETECTION_RMS_THRESHOLD_MIN_REFERENCE_SAMPLE_RATE_DP", SYNC_RMS_MIN_REF_RATE);
    add("RX_SYNC_PARAM_AUTOCORRELATOR_DETECTION_RMS_THRESHOLD_MIN_SP", SYNC_RMS_MIN);
    add("RX_SYNC_PARAM_AUTOCORRELATOR_DETECTION_RMS_THRESHOLD_MAX_SP", SYNC_RMS_MAX);
    add("RX_SYNC_PARAM_AUTOCORRELATOR_DETECTION_RMS_FRONT_STEPS", SYNC_RMS_FRONT_STEPS);
    add("RX_SYNC_PARAM_AUTOCORRELATOR_DETECTION_RMS_BACK_STEPS", SYNC_RMS_BACK_STEPS);
    add("RX_SYNC_PARAM_AUTOCORRELATOR_DETECTION_RMS_FRONT_TO_BACK_RATIO", SYNC_RMS_FRONT_TO_BACK_RATIO);
    add("RX_SYNC_PARAM_AUTOCORRELATOR_DETECTION_METRIC_THRESHOLD_MIN_SP", SYNC_METRIC_MIN);
    add("RX_SYNC_PARAM_AUTOCORRELATOR_DETECTION_METRIC_THRESHOLD_MAX_SP", SYNC_METRIC_MAX);
    add("RX_SYNC_PARAM_AUTOCORRELATOR_DETECTION_METRIC_STREAK_RELATIVE_GAIN_SP", SYNC_METRIC_STREAK_GAIN);
    add("RX_SYNC_PARAM_AUTOCORRELATOR_DETECTION_METRIC_STREAK", SYNC_METRIC_STREAK);
    add("RX_SYNC_PARAM_AUTOCORRELATOR_DETECTION_JUMP_BACK_IN_PATTERNS", SYNC_JUMP_BACK_PATTERNS);
    add("RX_SYNC_PARAM_AUTOCORRELATOR_DETECTION_SKIP_AFTER_PEAK_IN_STFS_DP", SYNC_SKIP_AFTER_PEAK_STFS);
    add("RX_SYNC_PARAM_AUTOCORRELATOR_PEAK_SAMPLES_REQUEST_IN_PATTERNS", SYNC_PEAK_REQUEST_PATTERNS);
    add("RX_SYNC_PARAM_AUTOCORRELATOR_PEAK_MAX_SEARCH_LENGTH_IN_STFS_DP", SYNC_PEAK_MAX_SEARCH_STFS);
    add("RX_SYNC_PARAM_AUTOCORRELATOR_PEAK_MOVMEAN_SMOOTH_LEFT", SYNC_PEAK_SMOOTH_LEFT);
    add("RX_SYNC_PARAM_AUTOCORRELATOR_PEAK_MOVMEAN_SMOOTH_RIGHT", SYNC_PEAK_SMOOTH_RIGHT);
    add("RX_SYNC_PARAM_AUTOCORRELATOR_PEAK_METRIC_ABOVE_DETECTION_THRESHOLD_SP", SYNC_PEAK_ABOVE_DETECTION);
    add("RX_SYNC_PARAM_AUTOCORRELATOR_PEAK_DETECTION2PEAK_IN_STFS_DP", SYNC_PEAK_DETECTION2PEAK_STFS);
    add("RX_SYNC_PARAM_CROSSCORRELATOR_CFO_PRECORRECTION", SYNC_XC_CFO_PRECORRECTION);
    add("RX_SYNC_PARAM_CROSSCORRELATOR_STF_LENGTH_EFFECTIVE_DP", SYNC_XC_STF_LENGTH_EFFECTIVE);
    add("RX_SYNC_PARAM_CROSSCORRELATOR_SEARCH_LEFT_SAMPLES", SYNC_XC_SEARCH_LEFT);
    add("RX_SYNC_PARAM_CROSSCORRELATOR_SEARCH_RIGHT_SAMPLES", SYNC_XC_SEARCH_RIGHT);
    // rx_synced_param.hpp
    add("RX_SYNCED_PARAM_STO_INTEGER_MOVE_INTO_CP_IN_PERCENTAGE_OF_STF", RX_STO_INTO_CP_PERCENT);
    add("RX_SYNCED_PARAM_RMS_FILL_COMPLETELY_OR_KEEP_WHAT_SYNCHRONIZATION_PROVIDED", RX_RMS_FILL_OR_KEEP);
    add("RX_SYNCED_PARAM_RMS_PERCENTAGE_OF_STF_USED_FOR_RMS_ESTIMATION", RX_RMS_STF_PERCENT);
    add("RX_SYNCED_PARAM_RMS_KEEP_VALUES_PROVIDED_BY_SYNC", RX_RMS_KEEP_SYNC);
    add("RX_SYNCED_PARAM_CFO_CORRECTION", RX_CFO_CORRECTION);
    add("RX_SYNCED_PARAM_CFO_FRACTIONAL_ADJUST", RX_CFO_FRACTIONAL_ADJUST);
    add("RX_SYNCED_PARAM_AMPLITUDE_SCALING", RX_AMPLITUDE_SCALING);
    add("RX_SYNCED_PARAM_STO_FRACTIONAL_BASED_ON_STF", RX_STO_FRACTIONAL_STF);
    add("RX_SYNCED_PARAM_STO_RESIDUAL_BASED_ON_DRS", RX_STO_RESIDUAL_DRS);
    add("RX_SYNCED_PARAM_CFO_RESIDUAL_BASED_ON_DRS", RX_CFO_RESIDUAL_DRS);
    add("RX_SYNCED_PARAM_WEIGHTS_TYPE_CHOICE", RX_WEIGHTS_TYPE_CHOICE);
    for (int i = 0; i < 3; ++i) {
        const std::string k = "[" + std::to_string(i) + "]";
        t.push_back({"RX_SYNCED_PARAM_NU_MAX_HZ_VEC" + k, RX_NU_MAX_HZ[i]});
        t.push_back({"RX_SYNCED_PARAM_TAU_RMS_SEC_VEC" + k, RX_TAU_RMS_SEC[i]});
        t.push_back({"RX_SYNCED_PARAM_SNR_DB_VEC" + k, RX_SNR_DB[i]});
        t.push_back({"RX_SYNCED_PARAM_NOF_DRS_INTERP_LR_VEC" + k, static_cast<double>(RX_N_INTERP_LR[i])});
        t.push_back({"RX_SYNCED_PARAM_NOF_DRS_INTERP_L_VEC" + k, static_cast<double>(RX_N_INTERP_L[i])});
    }
    add("RX_SYNCED_PARAM_CHANNEL_LUT_OPT_INDEX_PREVIOUS", RX_LUT_OPT_INDEX_PREVIOUS);
    add("RX_SYNCED_PARAM_CHANNEL_LUT_SEARCH_ABORT_THRESHOLD", RX_LUT_SEARCH_ABORT);
    add("RX_SYNCED_PARAM_CHANNEL_LUT_LOOKUP_AFTER_EVERY_DRS_SYMBOL_OR_ONCE", RX_LUT_LOOKUP_EVERY_DRS);
    add("RX_SYNCED_PARAM_SNR_BASED_ON_STF", RX_SNR_STF);
    add("RX_SYNCED_PARAM_SNR_BASED_ON_DRS", RX_SNR_DRS);
    add("RX_SYNCED_PARAM_SNR_BASED_ON_DRS_N_TS_MAX", RX_SNR_DRS_N_TS_MAX);
    add("RX_SYNCED_PARAM_MIMO_BASED_ON_STF_AND_DRS_AT_PACKET_END", RX_MIMO_AT_PACKET_END);
    add("RX_SYNCED_PARAM_MIMO_N_WIDEBAND_CELLS", RX_MIMO_WIDEBAND_CELLS);
    add("RX_SYNCED_PARAM_MODE_3_7_METRIC", RX_MODE_3_7_METRIC);
    add("RX_SYNCED_PARAM_BLOCK_N_SS_TX_LARGER_1_AT_PCC", RX_BLOCK_N_SS_GT_1_AT_PCC);
    add("RX_SYNCED_PARAM_BLOCK_N_EFF_TX_LARGER_1_AT_PDC", RX_BLOCK_N_EFF_TX_GT_1_AT_PDC);
    // resampler_param.hpp: arrays indexed [user][os]
    const uint32_t osv[4] = {1, 2, 4, 8};
    for (uint32_t u = 0; u < 3; ++u)
        for (uint32_t o = 0; o < 4; ++o) {
            const std::string k = "[" + std::to_string(u) + "][" + std::to_string(osv[o]) + "]";
            t.push_back({"resampler_param_t::f_pass_norm" + k, RS_F_PASS[u][o]});
            t.push_back({"resampler_param_t::f_stop_norm" + k, RS_F_STOP[u][o]});
            t.push_back({"resampler_param_t::f_stop_att_dB" + k, RS_ATT_DB[u][o]});
        }
    add("resampler_param_t::PASSBAND_RIPPLE_DONT_CARE", RS_RIPPLE_DONT_CARE);
    // constants.hpp
    add("constants::N_b_DFT_min_u_b", N_B_DFT_MIN_U_B);
    add("constants::N_b_CP_min_u_b", N_B_CP_MIN_U_B);
    add("constants::samp_rate_min_u_b", SAMP_RATE_MIN_U_B);
    add("constants::subcarrier_spacing_min_u_b", SUBCARRIER_SPACING_MIN_U_B);
    add("constants::N_stf_pattern_u1", N_STF_PATTERN_U1);
    add("constants::N_stf_pattern_u248", N_STF_PATTERN_U248);
    add("constants::N_samples_stf_pattern", N_SAMPLES_STF_PATTERN);
    add("constants::N_STF_cells_b_1", N_STF_CELLS_B_1);
    add("constants::N_STF_cells_spacing", N_STF_CELLS_SPACING);
    add("constants::N_STF_cells_spacing_center", N_STF_CELLS_SPACING_CENTER);
    add("constants::N_TS_max", N_TS_MAX);
    add("constants::pcc_bits", PCC_BITS);
    add("constants::pcc_cells", PCC_CELLS);
    return t;
}

const std::vector<entry>& table() {
    static const std::vector<entry> t = build_table();
    return t;
}

// sections_part3/radio_device_class.cpp:26-150 (the classes the reference lists)
struct rdc_row {
    const char* name;
    dnrp_radio_device_class c;
};
const rdc_row RDC[] = {
    {"1.1.1.A", {1, 1, 1, 7, 8, 2, 25344, 2048, 4}},    {"1.1.1.B", {1, 1, 1, 7, 8, 2, 25344, 6144, 4}},
    {"8.1.1.A", {8, 1, 1, 7, 8, 2, 25344, 6144, 4}},    {"1.8.1.A", {1, 8, 1, 7, 8, 2, 25344, 6144, 4}},
    {"2.8.2.A", {2, 8, 2, 7, 8, 2, 25344, 6144, 4}},    {"2.12.4.A", {2, 12, 4, 7, 8, 2, 25344, 2048, 4}},
    {"2.12.4.B", {2, 12, 4, 7, 8, 2, 25344, 6144, 4}},  {"8.12.8.A", {8, 12, 8, 9, 8, 2, 225344, 6144, 16}},
    {"8.16.8.A", {8, 16, 8, 9, 8, 2, 225344, 6144, 16}},
};

}  // namespace

extern "C" {

int dnrp_query_param(const char* name, double* value) {
    if (!name || !value) return DNRP_EINVAL;
    for (const auto& e : table())
        if (e.name == name) {
            *value = e.value;
            return DNRP_OK;
        }
    return DNRP_EINVAL;
}

const char* dnrp_param_name(uint32_t index) {
    const auto& t = table();
    return index < t.size() ? t[index].name.c_str() : nullptr;
}

int dnrp_get_radio_device_class(const char* name, dnrp_radio_device_class* out) {
    if (!name || !out) return DNRP_EINVAL;
    for (const auto& r : RDC)
        if (std::strcmp(r.name, name) == 0) {
            *out = r.c;
            return DNRP_OK;
        }
    return DNRP_ECONFIG;  // the reference asserts on an unknown class string
}

int dnrp_query_table(const char* name, const uint32_t* arg, uint32_t n_arg, float* out, uint32_t cap) {
    using namespace dnrp;
    if (!name || (n_arg && !arg)) return DNRP_EINVAL;
    std::vector<float> v;
    const std::string n(name);
    auto a = [&](uint32_t i) { return i < n_arg ? arg[i] : 0u; };
    try {
        if (n == "W" || n == "W_scaling" || n == "W_scaling_optimal_DAC") {  // (N_TS, N_TX, codebook)
            if (n_arg != 3) return DNRP_EINVAL;
            if (a(2) >= geo::W_codebooks(a(0), a(1))) return DNRP_EINVAL;
            float sc = 1.0f;
            const auto w = geo::W_matrix(a(0), a(1), a(2), &sc);
            if (n == "W") {
                for (const auto& c : w) {
                    v.push_back(c.real());
                    v.push_back(c.imag());
                }
            } else {
                v.push_back(n == "W_scaling" ? sc : geo::W_scaling_optimal_DAC(a(0), a(1), a(2)));
            }
        } else if (n == "W_codebooks") {  // (N_TS, N_TX)
            if (n_arg != 2) return DNRP_EINVAL;
            v.push_back(static_cast<float>(geo::W_codebooks(a(0), a(1))));
        } else if (n == "cells_lds_bytes") {  // (u_max, b_max, b, N_RX, N_eff_TX): rx_cells_kernel's LDS
            // staging for the geometry (ctx.cpp launch_back: above 160 KiB -> DNRP_EUNSUPPORTED); the
            // weight-table slots as get_rx1 sizes them from the Wiener LUTs of both modes
            if (n_arg != 5 || a(2) == 0 || a(2) > a(1) || a(4) == 0 || a(4) > 8) return DNRP_EINVAL;
            const uint32_t Nsv = a(4) <= 2 ? 5 : 10;
            uint32_t wcap[2] = {};
            for (uint32_t mode = 0; mode < 2; ++mode)
                for (uint32_t p = 0; p < 3; ++p) {
                    const auto L = geo::build_lut(mode ? Nsv : 0, a(2), a(1), a(0), p);
                    wcap[mode] = std::max(wcap[mode], (static_cast<uint32_t>(L.weights.size()) + 3u) & ~3u);
                }
            v.push_back(static_cast<float>(dnrp::dev::cell_lds_bytes(a(3), a(4), 56 * a(2) / 4, wcap[0], wcap[1])));
        } else if (n == "stf") {  // (b, N_eff_TX): transmit-stream vector [N_b_OCC + 1] re/im, scale 1
            if (n_arg != 2 || !(a(0) == 1 || a(0) == 2 || a(0) == 4 || a(0) == 8 || a(0) == 12 || a(0) == 16) ||
                !(a(1) == 1 || a(1) == 2 || a(1) == 4 || a(1) == 8))
                return DNRP_EINVAL;
            for (const auto& c : geo::stf_values(a(0), a(1))) {
                v.push_back(c.real());
                v.push_back(c.imag());
            }
        } else if (n == "drs_values") {  // (b, t): the N_b_OCC/4 DRS values of transmit stream t
            if (n_arg != 2 || a(0) == 0 || a(0) > 16 || a(1) > 7) return DNRP_EINVAL;
            const auto m = geo::build_maps(a(0), 1, 1, 1);
            const uint32_t nd = static_cast<uint32_t>(m.drs_v.size() / 8);
            v.assign(m.drs_v.begin() + size_t(a(1)) * nd, m.drs_v.begin() + size_t(a(1) + 1) * nd);
        } else if (n == "txdiv_pairs") {  // (N_TS): the SFBC stream pairs of one cycle, A0 B0 A1 B1 ...
            if (n_arg != 1 || !(a(0) == 2 || a(0) == 4 || a(0) == 8)) return DNRP_EINVAL;
            for (uint32_t i = 0; i < geo::txdiv_modulo(a(0)); ++i) {
                uint32_t A, B;
                geo::txdiv_pair(a(0), i, A, B);
                v.push_back(static_cast<float>(A));
                v.push_back(static_cast<float>(B));
            }
        } else if (n == "stf_cover_sequence") {
            v.assign(prm::STF_COVER, prm::STF_COVER + 9);
        } else if (n == "symbol_cells") {  // (b, N_TS, N_eff_TX, N_DF): per symbol l = 0..N_DF: PCC, PDC, DRS cells
            if (n_arg != 4 || a(0) == 0 || a(0) > 16 || a(1) == 0 || a(1) > 8 || a(2) == 0 || a(2) > 8 || a(3) > 1024)
                return DNRP_EINVAL;
            const auto m = geo::build_maps(a(0), a(1), a(2), a(3));
            for (uint32_t l = 0; l <= a(3); ++l) {
                uint32_t pcc = 0, drs = 0;
                for (uint32_t s = 0; s < m.pcc_l.size(); ++s)
                    if (m.pcc_l[s] == l) pcc = m.pcc_sym_off[s + 1] - m.pcc_sym_off[s];
                for (const auto& d : m.drs)
                    if (d.l == l) drs += (d.ts_last - d.ts_first + 1) * static_cast<uint32_t>(m.drs_v.size() / 8);
                v.push_back(static_cast<float>(pcc));
                v.push_back(static_cast<float>(m.pdc_sym_off[l + 1] - m.pdc_sym_off[l]));
                v.push_back(static_cast<float>(drs));
            }
        } else {
            return DNRP_EINVAL;
        }
    } catch (...) {
        return DNRP_EINVAL;
    }
    if (out) {
        if (cap < v.size()) return DNRP_EINVAL;
        std::memcpy(out, v.data(), v.size() * sizeof(float));
    }
    return static_cast<int>(v.size());
}

}  // extern "C"
