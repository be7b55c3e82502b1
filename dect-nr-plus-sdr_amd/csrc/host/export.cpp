// Host-only JSON export in the reference's formats (include/dnrp.h dnrp_tx_packet_json,
// dnrp_rx_packet_json): tx_t::write_all_data_to_json (tx.cpp:316-427) and the PHY part of
// worker_tx_rx_t::collect_and_write_json (worker_tx_rx.cpp:354-410), so packets generated or
// received on the GPU can be read by the reference's analysis scripts. Plus the TX length a radio
// buffer publishes (tx_t::run_meta_dependencies, tx.cpp:555-566).
#include <cmath>
#include <cstdio>
#include <string>
#include <vector>

#include "dnrp.h"
#include "geometry.hpp"

using namespace dnrp;

namespace {

struct json_out {  // minimal ordered JSON writer (objects, arrays of numbers)
    std::string s;
    std::vector<bool> first{true};
    void sep() {
        if (!first.back()) s += ',';
        first.back() = false;
    }
    void key(const char* k) {
        sep();
        s += '"';
        s += k;
        s += "\":";
    }
    void open(const char* k) {
        if (k) key(k); else sep();
        s += '{';
        first.push_back(true);
    }
    void close() {
        s += '}';
        first.pop_back();
    }
    template <class T>
    void num(const char* k, T v) {
        key(k);
        s += fmt(v);
    }
    static std::string fmt(double v) {
        if (!std::isfinite(v)) return "null";
        char b[40];
        std::snprintf(b, sizeof b, "%.9g", v);
        return b;
    }
    static std::string fmt(float v) { return fmt(static_cast<double>(v)); }
    static std::string fmt(uint32_t v) { return std::to_string(v); }
    static std::string fmt(uint64_t v) { return std::to_string(v); }
    static std::string fmt(int64_t v) { return std::to_string(v); }
    template <class F>
    void arr(const char* k, size_t n, F&& at) {
        key(k);
        s += '[';
        for (size_t i = 0; i < n; ++i) {
            if (i) s += ',';
            s += fmt(at(i));
        }
        s += ']';
    }
};

bool write_file(const std::string& s, const char* path) {
    FILE* f = std::fopen(path, "wb");
    if (!f) return false;
    const bool ok = std::fwrite(s.data(), 1, s.size(), f) == s.size();
    return std::fclose(f) == 0 && ok;
}

std::vector<uint32_t> unpack(const uint8_t* p, uint32_t n) {  // MSB first (srsran_bit_unpack_vector)
    std::vector<uint32_t> v(n);
    for (uint32_t i = 0; i < n; ++i) v[i] = (p[i >> 3] >> (7 - (i & 7))) & 1u;
    return v;
}

uint32_t transmit_len(const geo::dims_t& dm, uint32_t gi_percent) {  // tx.cpp:555-566
    return dm.N_no_GI_rs + (dm.N_packet_rs - dm.N_no_GI_rs) * gi_percent / 100;
}

}  // namespace

extern "C" {

int dnrp_tx_transmit_length(const dnrp_cfg* cfg, const dnrp_psdef* psdef, uint32_t GI_percentage, uint32_t* len) {
    if (!cfg || !psdef || !len || GI_percentage > 100 || cfg->L == 0 || cfg->M == 0 || cfg->os_min == 0) return DNRP_EINVAL;
    dnrp_packet_sizes q;
    if (!geo::packet_sizes(*psdef, q)) return DNRP_ECONFIG;
    if (psdef->u > cfg->u_max || psdef->b > cfg->b_max) return DNRP_EUNSUPPORTED;
    *len = transmit_len(geo::make_dims(*cfg, *psdef, q), GI_percentage);
    return DNRP_OK;
}

int dnrp_tx_packet_json(const dnrp_cfg* cfg, const dnrp_psdef* psdef, const dnrp_tx_desc* desc, uint32_t rv,
                        uint64_t tx_order_id, int64_t tx_time_64, const uint8_t* pcc_d, const uint8_t* pdc_d,
                        const float* iq, uint32_t S, const char* path) {
    if (!cfg || !psdef || !desc || !pcc_d || !pdc_d || !iq || !path || desc->GI_percentage > 100) return DNRP_EINVAL;
    dnrp_packet_sizes q;
    geo::tm_t tm;
    if (!geo::packet_sizes(*psdef, q, &tm)) return DNRP_ECONFIG;
    if (psdef->u > cfg->u_max || psdef->b > cfg->b_max) return DNRP_EUNSUPPORTED;
    const auto dm = geo::make_dims(*cfg, *psdef, q);
    const uint32_t n_tr = transmit_len(dm, desc->GI_percentage);
    if (S < n_tr) return DNRP_EINVAL;
    const uint32_t os = prm::rs_os_index(cfg->os_min);
    json_out j;
    j.open(nullptr);
    j.num("u", psdef->u);
    j.num("b", psdef->b);
    j.num("PacketLengthType", psdef->PacketLengthType);
    j.num("PacketLength", psdef->PacketLength);
    j.num("tm_mode", psdef->tm_mode_index);
    j.num("mcs_index", psdef->mcs_index);
    j.num("Z", psdef->Z);
    j.num("oversampling", static_cast<double>(dm.Nd) / static_cast<double>(q.N_b_DFT));
    j.num("codebook_index", desc->codebook_index);
    j.num("PLCF_type", desc->plcf_type);
    j.num("rv", rv);
    j.num("network_id", desc->network_id);
    j.num("N_samples_packet_no_GI_os_rs", dm.N_no_GI_rs);
    j.num("N_samples_transmit_os_rs", n_tr);
    j.open("tx_descriptor");
    j.num("tx_order_id", tx_order_id);
    j.num("tx_time_64", tx_time_64);
    j.close();
    j.open("tx_meta");
    j.num("iq_phase_rad", desc->iq_phase_rad);
    j.num("iq_phase_increment_s2s_post_resampling_rad", desc->iq_phase_increment_s2s_post_resampling_rad);
    j.num("GI_percentage", desc->GI_percentage);
    j.close();
    j.open("data");
    j.open("binary");
    // PLCF and TB (before channel coding) exist only above the FEC, outside this library: empty
    j.arr("PLCF", 0, [](size_t) { return 0u; });
    const auto pcc = unpack(pcc_d, prm::PCC_BITS), pdc = unpack(pdc_d, q.G);
    j.arr("PCC", pcc.size(), [&](size_t i) { return pcc[i]; });
    j.arr("TB", 0, [](size_t) { return 0u; });
    j.arr("PDC", pdc.size(), [&](size_t i) { return pdc[i]; });
    j.close();
    // antenna streams concatenated: all real parts of antenna 0, then antenna 1, ... (tx.cpp:393-421)
    j.open("IQ");
    j.arr("real", size_t(n_tr) * tm.N_TX, [&](size_t i) { return iq[2 * ((i / n_tr) * size_t(S) + i % n_tr)]; });
    j.arr("imag", size_t(n_tr) * tm.N_TX, [&](size_t i) { return iq[2 * ((i / n_tr) * size_t(S) + i % n_tr) + 1]; });
    j.close();
    j.close();
    j.open("resampling");
    const uint64_t rate = uint64_t(cfg->u_max) * cfg->b_max * prm::SAMP_RATE_MIN_U_B * cfg->os_min * cfg->L / cfg->M;
    j.num("samp_rate", rate);
    j.num("L", cfg->L);
    j.num("M", cfg->M);
    j.num("f_pass_norm", prm::RS_F_PASS[prm::RS_TX][os]);
    j.num("f_stop_norm", prm::RS_F_STOP[prm::RS_TX][os]);
    j.num("passband_ripple_dB", prm::RS_RIPPLE_DONT_CARE);
    j.num("stopband_attenuation_dB", prm::RS_ATT_DB[prm::RS_TX][os]);
    j.num("oversampling_minimum", cfg->os_min);
    j.close();
    j.close();
    return write_file(j.s, path) ? DNRP_OK : DNRP_EINVAL;
}

int dnrp_rx_packet_json(const dnrp_cfg* cfg, uint32_t worker_id, const dnrp_sync_result* sr, uint32_t mcs_index,
                        const dnrp_pcc_report* pcc, const dnrp_pdc_report* pdc, const char* path) {
    if (!cfg || !sr || !path || cfg->M == 0) return DNRP_EINVAL;
    const uint32_t n_ant = std::min(cfg->N_TX_max, 8u);
    json_out j;
    j.open(nullptr);
    j.num("worker_id", worker_id);
    j.open("RADIO");
    j.num("samp_rate", uint64_t(cfg->u_max) * cfg->b_max * prm::SAMP_RATE_MIN_U_B * cfg->os_min * cfg->L / cfg->M);
    j.num("N_TX_min", cfg->N_TX_max);
    j.close();
    j.open("PHY");
    j.open("worker_pool_config");
    j.num("L", cfg->L);
    j.num("M", cfg->M);
    j.num("dect_samp_rate_max_oversampled", uint64_t(cfg->u_max) * cfg->b_max * prm::SAMP_RATE_MIN_U_B * cfg->os_min);
    j.close();
    j.open("sync_report");  // worker_tx_rx.cpp:380-396
    j.num("detection_ant_idx", sr->detection_ant_idx);
    j.num("detection_rms", sr->detection_rms);
    j.num("detection_metric", sr->detection_metric);
    j.num("u", sr->u);
    j.arr("coarse_peak_array", n_ant, [&](size_t i) { return sr->coarse_peak_array[i]; });
    j.arr("rms_array", n_ant, [&](size_t i) { return sr->rms_array[i]; });
    j.num("cfo_f", sr->cfo_fractional_rad);
    j.num("b", sr->b);
    j.num("cfo_i", sr->cfo_integer_rad);
    j.num("coarse_peak_time", sr->coarse_peak_time);
    j.num("N_eff_TX", sr->N_eff_TX);
    j.num("fine_peak_time", sr->fine_peak_time);
    if (pcc) j.num("sto_fractional", pcc->sto_fractional);
    j.close();
    j.open("rx_synced");  // rx_synced.cpp:444-449 (the channel estimates are not exported)
    const float snr = pdc ? pdc->snr_dB : pcc ? pcc->snr_dB : 0.0f;
    j.num("snr", snr);
    j.num("mcs", mcs_index);
    j.close();
    j.close();
    j.close();
    return write_file(j.s, path) ? DNRP_OK : DNRP_EINVAL;
}

}  // extern "C"
