// ORACLE — TEST INFRASTRUCTURE ONLY (see oracle.hpp header).
// extern "C" surface of the oracle for ctypes (tests/, bench.py cpu_baseline, smoke()).
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <random>
#include <string>
#include <thread>

#include "oracle.hpp"
#include "oracle_dsp.hpp"
#include "oracle_params.hpp"

using namespace orc;

static psdef_t to_psdef(const uint32_t* p) { return psdef_t{p[0], p[1], p[2], p[3], p[4], p[5], p[6]}; }
static cfg_t to_cfg(const uint32_t* c) {
    cfg_t g;
    g.u_max = c[0];
    g.b_max = c[1];
    g.os_min = c[2];
    g.L = c[3];
    g.M = c[4];
    g.chestim_mode_lr = c[5] != 0;
    g.stride = c[6];
    return g;
}

extern "C" {

// ---- the reference parameters the restatement uses, by the reference's names (oracle_params.hpp);
// compared with the reference-compiled values in tests/test_oracle_pins.py. -1: unknown name.
int oracle_query_param(const char* name, double* v) {
    using namespace orc::prm;
    const std::string n(name);
    struct kv {
        const char* k;
        double v;
    };
    static const kv T[] = {
        {"RX_SYNC_PARAM_AUTOCORRELATOR_ANTENNA_LIMIT", ANTENNA_LIMIT},
        {"RX_SYNC_PARAM_AUTOCORRELATOR_DETECTION_OVERLAP_LENGTH_IN_STFS_DP", OVERLAP_STFS},
        {"RX_SYNC_PARAM_AUTOCORRELATOR_DETECTION_STEP_DIVIDER", STEP_DIVIDER},
        {"RX_SYNC_PARAM_AUTOCORRELATOR_DETECTION_RESUM_PERIODICITY_IN_STEPS", DET_RESUM},
        {"RX_SYNC_PARAM_AUTOCORRELATOR_DETECTION_RMS_THRESHOLD_MIN_REFERENCE_SAMPLE_RATE_DP", RMS_MIN_REF_RATE},
        {"RX_SYNC_PARAM_AUTOCORRELATOR_DETECTION_RMS_THRESHOLD_MIN_SP", RMS_MIN},
        {"RX_SYNC_PARAM_AUTOCORRELATOR_DETECTION_RMS_THRESHOLD_MAX_SP", RMS_MAX},
        {"RX_SYNC_PARAM_AUTOCORRELATOR_DETECTION_RMS_FRONT_STEPS", RMS_FRONT_STEPS},
        {"RX_SYNC_PARAM_AUTOCORRELATOR_DETECTION_RMS_BACK_STEPS", RMS_BACK_STEPS},
        {"RX_SYNC_PARAM_AUTOCORRELATOR_DETECTION_RMS_FRONT_TO_BACK_RATIO", RMS_FRONT_TO_BACK},
        {"RX_SYNC_PARAM_AUTOCORRELATOR_DETECTION_METRIC_THRESHOLD_MIN_SP", METRIC_MIN},
        {"RX_SYNC_PARAM_AUTOCORRELATOR_DETECTION_METRIC_THRESHOLD_MAX_SP", METRIC_MAX},
        {"RX_SYNC_PARAM_AUTOCORRELATOR_DETECTION_METRIC_STREAK_RELATIVE_GAIN_SP", STREAK_GAIN},
        {"RX_SYNC_PARAM_AUTOCORRELATOR_DETECTION_METRIC_STREAK", STREAK},
        {"RX_SYNC_PARAM_AUTOCORRELATOR_DETECTION_JUMP_BACK_IN_PATTERNS", JUMP_BACK_PATTERNS},
        {"RX_SYNC_PARAM_AUTOCORRELATOR_DETECTION_SKIP_AFTER_PEAK_IN_STFS_DP", SKIP_AFTER_PEAK_STFS},
        {"RX_SYNC_PARAM_AUTOCORRELATOR_PEAK_SAMPLES_REQUEST_IN_PATTERNS", PEAK_REQUEST_PATTERNS},
        {"RX_SYNC_PARAM_AUTOCORRELATOR_PEAK_RESUM_PERIODICITY_IN_STEPS", PEAK_RESUM},
        {"RX_SYNC_PARAM_AUTOCORRELATOR_PEAK_MAX_SEARCH_LENGTH_IN_STFS_DP", PEAK_MAX_SEARCH_STFS},
        {"RX_SYNC_PARAM_AUTOCORRELATOR_PEAK_MOVMEAN_SMOOTH_LEFT", SMOOTH_LEFT},
        {"RX_SYNC_PARAM_AUTOCORRELATOR_PEAK_MOVMEAN_SMOOTH_RIGHT", SMOOTH_RIGHT},
        {"RX_SYNC_PARAM_AUTOCORRELATOR_PEAK_METRIC_ABOVE_DETECTION_THRESHOLD_SP", PEAK_ABOVE_DETECTION},
        {"RX_SYNC_PARAM_AUTOCORRELATOR_PEAK_DETECTION2PEAK_IN_STFS_DP", DETECTION2PEAK_STFS},
        {"RX_SYNC_PARAM_CROSSCORRELATOR_SEARCH_LEFT_SAMPLES", XC_SEARCH_LEFT},
        {"RX_SYNC_PARAM_CROSSCORRELATOR_SEARCH_RIGHT_SAMPLES", XC_SEARCH_RIGHT},
        {"RX_SYNCED_PARAM_CHANNEL_LUT_SEARCH_ABORT_THRESHOLD", LUT_SEARCH_ABORT},
        {"RX_SYNCED_PARAM_MIMO_N_WIDEBAND_CELLS", MIMO_WIDEBAND_CELLS},
        {"RX_SYNCED_PARAM_RMS_PERCENTAGE_OF_STF_USED_FOR_RMS_ESTIMATION", RMS_STF_PERCENT},
        {"RX_SYNCED_PARAM_RMS_KEEP_VALUES_PROVIDED_BY_SYNC", RMS_KEEP_SYNC},
        {"resampler_param_t::PASSBAND_RIPPLE_DONT_CARE", RS_RIPPLE},
    };
    for (const auto& e : T)
        if (n == e.k) {
            *v = e.v;
            return 0;
        }
    const char* vec[5] = {"RX_SYNCED_PARAM_NU_MAX_HZ_VEC[", "RX_SYNCED_PARAM_TAU_RMS_SEC_VEC[", "RX_SYNCED_PARAM_SNR_DB_VEC[",
                          "RX_SYNCED_PARAM_NOF_DRS_INTERP_LR_VEC[", "RX_SYNCED_PARAM_NOF_DRS_INTERP_L_VEC["};
    for (int k = 0; k < 5; ++k)
        for (int i = 0; i < 3; ++i)
            if (n == std::string(vec[k]) + std::to_string(i) + "]") {
                const double vals[5] = {NU_MAX_HZ[i], TAU_RMS_SEC[i], SNR_DB[i], double(N_INTERP_LR[i]),
                                        double(N_INTERP_L[i])};
                *v = vals[k];
                return 0;
            }
    const int osv[4] = {1, 2, 4, 8};
    for (int u = 0; u < 3; ++u)
        for (int o = 0; o < 4; ++o) {
            const std::string k = "[" + std::to_string(u) + "][" + std::to_string(osv[o]) + "]";
            if (n == "resampler_param_t::f_pass_norm" + k) return *v = RS_F_PASS[o], 0;
            if (n == "resampler_param_t::f_stop_norm" + k) return *v = RS_F_STOP[o], 0;
            if (n == "resampler_param_t::f_stop_att_dB" + k) return *v = RS_ATT_DB[o], 0;
        }
    return -1;
}

// out: N_PACKET_symb, N_DF_symb, N_PDC_subc, N_DRS_subc, G, N_PDC_bits, N_TB_bits, C,
//      N_samples_STF, N_samples_STF_CP_only, N_samples_DF, N_samples_GI, N_samples_packet_no_GI,
//      N_samples_packet, N_bps, N_eff_TX, N_SS, N_TS, N_TX, N_b_DFT, N_b_OCC
int oracle_packet_sizes(const uint32_t* psdef, uint32_t* out) {
    try {
        packet_sizes_t q;
        if (!get_packet_sizes(to_psdef(psdef), q)) return -1;
        const uint32_t v[] = {q.N_PACKET_symb, q.N_DF_symb, q.N_PDC_subc, q.N_DRS_subc, q.G, q.N_PDC_bits,
                              q.N_TB_bits, q.C, q.N_samples_STF, q.N_samples_STF_CP_only, q.N_samples_DF,
                              q.N_samples_GI, q.N_samples_packet_no_GI, q.N_samples_packet, q.mcs.N_bps,
                              q.tm.N_eff_TX, q.tm.N_SS, q.tm.N_TS, q.tm.N_TX, q.num.N_b_DFT, q.num.N_b_OCC};
        std::memcpy(out, v, sizeof(v));
        return 0;
    } catch (...) {
        return -2;
    }
}

// ---- table pins against tests/golden/ref_tables.json (reference-compiled fixture)
// out: u, b, delta_u_f, N_SLOT_u_symb, N_SLOT_u_subslot, N_b_DFT, N_b_CP, N_b_OCC, N_guards_top,
//      N_guards_bottom; T_u_symb in *T
int oracle_numerology(uint32_t u, uint32_t b, uint32_t* out, double* T) {
    try {
        const auto q = get_numerology(u, b);
        const uint32_t v[] = {q.u, q.b, q.delta_u_f, q.N_SLOT_u_symb, q.N_SLOT_u_subslot, q.N_b_DFT, q.N_b_CP,
                              q.N_b_OCC, q.N_guards_top, q.N_guards_bottom};
        std::memcpy(out, v, sizeof(v));
        *T = q.T_u_symb;
        return 0;
    } catch (...) {
        return -2;
    }
}

// out: index, N_eff_TX, N_SS, cl, N_TS, N_TX
int oracle_tm_mode(uint32_t index, uint32_t* out) {
    try {
        const auto t = get_tm_mode(index);
        const uint32_t v[] = {t.index, t.N_eff_TX, t.N_SS, t.cl ? 1u : 0u, t.N_TS, t.N_TX};
        std::memcpy(out, v, sizeof(v));
        return 0;
    } catch (...) {
        return -2;
    }
}

// out: index, N_bps, R_numerator, R_denominator
int oracle_mcs(uint32_t index, uint32_t* out) {
    try {
        const auto m = get_mcs(index);
        const uint32_t v[] = {m.index, m.N_bps, m.R_num, m.R_den};
        std::memcpy(out, v, sizeof(v));
        return 0;
    } catch (...) {
        return -2;
    }
}

uint32_t oracle_tbs(uint32_t N_SS, uint32_t N_PDC_subc, uint32_t mcs, uint32_t Z) {
    const auto m = get_mcs(mcs);
    return get_N_TB_bits(N_SS, N_PDC_subc, m.N_bps, m.R_num, m.R_den, Z);
}

int oracle_k_b_occ(uint32_t b, int32_t* out, uint32_t cap) {
    const auto k = k_b_OCC(b);
    if (k.size() > cap) return -1;
    for (size_t i = 0; i < k.size(); ++i) out[i] = k[i];
    return static_cast<int>(k.size());
}

void oracle_special(float z, float* out5) { special_values(z, out5); }

// out: N_b_DFT_os, off_lower, CP_os, STF_CP_os, N_no_GI_os, N_no_GI_os_rs, N_packet_os_rs
int oracle_dims(const uint32_t* cfg, const uint32_t* psdef, uint32_t* out) {
    try {
        packet_sizes_t q;
        if (!get_packet_sizes(to_psdef(psdef), q)) return -1;
        dims_t d;
        d.init(to_cfg(cfg), q);
        const uint32_t v[] = {d.N_b_DFT_os, d.off_lower, d.CP_os, d.STF_CP_os, d.N_no_GI_os, d.N_no_GI_os_rs,
                              d.N_packet_os_rs};
        std::memcpy(out, v, sizeof(v));
        return 0;
    } catch (...) {
        return -2;
    }
}

int oracle_kaiser(float fp, float fs_, float ripple, float att, uint32_t max_n, float* out) {
    const auto k = kaiser(fp, fs_, ripple, att, 1.0f, true);
    if (k.size() > max_n) return -1;
    std::memcpy(out, k.data(), k.size() * sizeof(float));
    return static_cast<int>(k.size());
}

int oracle_gold(uint32_t c_init, uint32_t len, uint8_t* out) {
    const auto c = gold_sequence(c_init, len);
    std::memcpy(out, c.data(), len);
    return 0;
}

int oracle_stf(uint32_t b, uint32_t N_eff_TX, double* out_re_im) {
    const auto v = stf_values(b, N_eff_TX);
    for (size_t i = 0; i < v.size(); ++i) {
        out_re_im[2 * i] = v[i].real();
        out_re_im[2 * i + 1] = v[i].imag();
    }
    return static_cast<int>(v.size());
}

// flattened per-symbol PDC lists: out_cnt[l] for l in [0,N_DF], out_k concatenated
int oracle_pdc_cells(uint32_t b, uint32_t N_TS, uint32_t N_DF, uint32_t* out_cnt, uint32_t* out_k) {
    const auto v = pdc_cells_packet(b, N_TS, N_DF);
    uint32_t o = 0;
    for (uint32_t l = 0; l <= N_DF; ++l) {
        out_cnt[l] = static_cast<uint32_t>(v[l].size());
        for (uint32_t k : v[l]) out_k[o++] = k;
    }
    return static_cast<int>(o);
}

int oracle_pcc_cells(uint32_t b, uint32_t N_TS, uint32_t* out_l, uint32_t* out_k) {
    std::vector<uint32_t> l;
    std::vector<std::vector<uint32_t>> k;
    pcc_cells(b, N_TS, l, k);
    uint32_t o = 0;
    for (size_t s = 0; s < l.size(); ++s)
        for (uint32_t kk : k[s]) {
            out_l[o] = l[s];
            out_k[o++] = kk;
        }
    return static_cast<int>(o);
}

// LUT export: returns number of weight vectors; idx arrays sized T*4*(56b+1)
int oracle_chest_lut(uint32_t Nsv, uint32_t b, uint32_t b_max, uint32_t u_max, uint32_t profile,
                     uint32_t* idx_pilot, uint32_t* idx_weight, float* weights, uint32_t max_w) {
    try {
        const auto prof = chest_profiles(u_max);
        const auto L = build_chest_lut(Nsv, b, b_max, prof.at(profile));
        std::memcpy(idx_pilot, L.idx_pilot.data(), L.idx_pilot.size() * 4);
        std::memcpy(idx_weight, L.idx_weight.data(), L.idx_weight.size() * 4);
        if (L.weights.size() > max_w) return -1;
        std::memcpy(weights, L.weights.data(), L.weights.size() * 4);
        return static_cast<int>(L.weights.size() / L.nof_interp);
    } catch (...) {
        return -2;
    }
}

// literal tables (pinned against tests/golden/ref_literals.json)
int oracle_W(uint32_t N_TS, uint32_t N_TX, uint32_t codebook, double* out_re_im, double* scaling) {
    try {
        const auto w = W_matrix(N_TS, N_TX, codebook);
        for (size_t i = 0; i < w.size(); ++i) {
            out_re_im[2 * i] = w[i].real();
            out_re_im[2 * i + 1] = w[i].imag();
        }
        scaling[0] = W_scaling(N_TS, N_TX, codebook);
        scaling[1] = W_scaling_optimal_DAC(N_TS, N_TX, codebook);
        return static_cast<int>(w.size());
    } catch (...) {
        return -1;
    }
}
int oracle_W_codebooks(uint32_t N_TS, uint32_t N_TX) {
    try {
        return static_cast<int>(W_codebook_max(N_TS, N_TX)) + 1;
    } catch (...) {
        return -1;
    }
}
int oracle_drs_values(uint32_t b, uint32_t t, double* out) {
    const auto v = drs_y(b, t);
    std::memcpy(out, v.data(), v.size() * sizeof(double));
    return static_cast<int>(v.size());
}
int oracle_txdiv_pairs(uint32_t N_TS, uint32_t* out) {
    const uint32_t m = txdiv_modulo(N_TS);
    for (uint32_t i = 0; i < m; ++i) txdiv_pair(N_TS, i, out[2 * i], out[2 * i + 1]);
    return static_cast<int>(m);
}
void oracle_cover_sequence(float* out9) { std::memcpy(out9, STF_COVER_SEQ, 9 * sizeof(float)); }

// desc_u: codebook, network_id, plcf_type, GI_percentage, optimal_scaling_DAC ; desc_f: DAC_scale, phase, phase_inc
int oracle_tx(const uint32_t* cfg, const uint32_t* psdef, const uint32_t* desc_u, const double* desc_f,
              const uint8_t* pcc_d, const uint8_t* pdc_d, float* out, uint32_t S_slot, int use_float) {
    try {
        packet_sizes_t q;
        if (!get_packet_sizes(to_psdef(psdef), q)) return -1;
        tx_desc_t d;
        d.codebook_index = desc_u[0];
        d.network_id = desc_u[1];
        d.plcf_type = desc_u[2];
        d.GI_percentage = desc_u[3];
        d.optimal_scaling_DAC = desc_u[4] != 0;
        d.DAC_scale = static_cast<float>(desc_f[0]);
        d.iq_phase_rad = desc_f[1];
        d.iq_phase_increment_rad = desc_f[2];
        const cfg_t c = to_cfg(cfg);
        auto store = [&](const auto& v) {
            for (size_t a = 0; a < v.size(); ++a)
                for (uint32_t m = 0; m < S_slot; ++m) {
                    out[(a * S_slot + m) * 2] = static_cast<float>(v[a][m].real());
                    out[(a * S_slot + m) * 2 + 1] = static_cast<float>(v[a][m].imag());
                }
        };
        if (use_float) {
            std::vector<std::vector<std::complex<float>>> v;
            tx_packet<float>(c, q, d, pcc_d, pdc_d, v, S_slot);
            store(v);
        } else {
            std::vector<std::vector<std::complex<double>>> v;
            tx_packet<double>(c, q, d, pcc_d, pdc_d, v, S_slot);
            store(v);
        }
        dims_t dm;
        dm.init(c, q);
        return static_cast<int>(dm.transmit_len(d.GI_percentage));
    } catch (const std::exception& e) {
        std::fprintf(stderr, "oracle_tx: %s\n", e.what());
        return -2;
    }
}

// meta out: [0..7] rms, 8 cfo_fine_rad, 9 sto_fractional, 10 snr_pcc_db, 11 snr_pdc_db,
//           12 mimo N_TS_other, 13 tm_3_7_beamforming_idx, 14 tm_3_7_beamforming_reciprocal_idx
int oracle_rx(const uint32_t* cfg, const uint32_t* psdef, uint32_t N_RX, const float* iq, uint32_t S_in,
              int64_t fine_peak, double cfo_rad, uint32_t network_id, uint32_t plcf_type, int16_t* pcc_llr,
              int16_t* pdc_llr, float* pcc_llr_f, float* pdc_llr_f, float* meta, int use_float, const float* sync_rms,
              int sm_mmse) {
    try {
        packet_sizes_t q;
        if (!get_packet_sizes(to_psdef(psdef), q)) return -1;
        rx_in_t in{iq, N_RX, S_in, fine_peak, cfo_rad, network_id, plcf_type, sync_rms, sm_mmse != 0};
        rx_out_t o;
        if (use_float)
            rx_packet<float>(to_cfg(cfg), q, in, o);
        else
            rx_packet<double>(to_cfg(cfg), q, in, o);
        std::memcpy(pcc_llr, o.pcc_llr.data(), 196 * 2);
        std::memcpy(pdc_llr, o.pdc_llr.data(), q.G * 2);
        if (pcc_llr_f) std::memcpy(pcc_llr_f, o.pcc_llr_f.data(), 196 * 4);
        if (pdc_llr_f) std::memcpy(pdc_llr_f, o.pdc_llr_f.data(), q.G * 4);
        for (uint32_t a = 0; a < 8; ++a) meta[a] = a < o.rms.size() ? o.rms[a] : 0.0f;
        meta[8] = o.cfo_fine_rad;
        meta[9] = o.sto_fractional;
        meta[10] = o.snr_pcc_db;
        meta[11] = o.snr_pdc_db;
        meta[12] = static_cast<float>(o.mimo_N_TS_other);
        // 0xFFFFFFFF (no recommendation) as -1: exact in a float
        // MIMO_REF_UNDEFINED (the reference asserts / throws) -> -2
        meta[13] = o.mimo_idx == MIMO_REF_UNDEFINED ? -2.f : static_cast<float>(o.mimo_idx);
        meta[14] = o.mimo_idx_reciprocal == MIMO_REF_UNDEFINED ? -2.f : static_cast<float>(o.mimo_idx_reciprocal);
        return 0;
    } catch (const std::exception& e) {
        std::fprintf(stderr, "oracle_rx: %s\n", e.what());
        return -2;
    }
}

// CPU baseline: n_packets TX+RX loopback slot-pairs (float path), one packet per thread at a time
// (worker_tx_rx_t model). With sync_chunk > 0 each RX window holds the packet after sync_pre
// hw samples and is synchronised first (sync_chunk_t::search, float path), RX starting at the
// found fine peak. Returns wall seconds, or negative on error.
double oracle_loopback_timed2(const uint32_t* cfg, const uint32_t* psdef, uint32_t n_packets, uint32_t n_threads,
                              uint64_t seed, uint32_t sync_pre, uint32_t sync_chunk, double* phase_s) {
    try {
        packet_sizes_t q;
        if (!get_packet_sizes(to_psdef(psdef), q)) return -1.0;
        const cfg_t c = to_cfg(cfg);
        dims_t dm;
        dm.init(c, q);
        const uint32_t S = dm.N_packet_os_rs;
        std::atomic<uint32_t> next{0};
        std::atomic<int> err{0};
        std::vector<double> t_tx(n_threads, 0.0), t_rx(n_threads, 0.0);  // thread seconds per phase
        auto worker = [&](uint32_t tid) {
            using clk = std::chrono::steady_clock;
            std::mt19937_64 rng(seed + tid);
            std::vector<uint8_t> pcc(25), pdc((q.G + 7) / 8);
            std::vector<float> iq(2ull * q.tm.N_TX * S);
            while (true) {
                const uint32_t i = next.fetch_add(1);
                if (i >= n_packets) break;
                for (auto& b : pcc) b = static_cast<uint8_t>(rng());
                for (auto& b : pdc) b = static_cast<uint8_t>(rng());
                tx_desc_t d;
                d.network_id = 100 + i % 6;
                d.plcf_type = 1 + i % 2;
                std::vector<std::vector<std::complex<float>>> v;
                const auto c0 = clk::now();
                tx_packet<float>(c, q, d, pcc.data(), pdc.data(), v, S);
                const auto c1 = clk::now();
                t_tx[tid] += std::chrono::duration<double>(c1 - c0).count();
                int64_t fine = 0;
                if (sync_chunk) {
                    std::fill(iq.begin(), iq.end(), 0.0f);
                    for (size_t a = 0; a < v.size(); ++a)
                        std::memcpy(&iq[2ull * (a * S + sync_pre)], v[a].data(), (S - sync_pre) * 8);
                    sync_cfg_t sc;
                    sc.u = q.psdef.u;
                    sc.b = q.psdef.b;
                    sc.os_min = c.os_min;
                    sc.L = c.L;
                    sc.M = c.M;
                    sc.N_ant = sc.N_ant_limited = q.tm.N_TX;
                    sc.chunk_len = sync_chunk;
                    const auto r = sync_search<float>(sc, iq.data(), S, 1);
                    if (r.empty()) {
                        err = 2;
                        continue;
                    }
                    fine = r[0].fine_64;
                } else {
                    for (size_t a = 0; a < v.size(); ++a)
                        std::memcpy(&iq[2ull * a * S], v[a].data(), S * 8);
                }
                rx_in_t in{iq.data(), q.tm.N_TX, S, fine, 0.0, d.network_id, d.plcf_type};
                rx_out_t o;
                rx_packet<float>(c, q, in, o);
                t_rx[tid] += std::chrono::duration<double>(clk::now() - c1).count();  // sync + RX
                if (o.pdc_llr.size() != q.G) err = 1;
            }
        };
        const auto t0 = std::chrono::steady_clock::now();
        std::vector<std::thread> th;
        for (uint32_t t = 0; t < n_threads; ++t) th.emplace_back(worker, t);
        for (auto& t : th) t.join();
        const auto t1 = std::chrono::steady_clock::now();
        if (err) return -3.0 - err;
        if (phase_s) {
            phase_s[0] = phase_s[1] = 0.0;
            for (uint32_t t = 0; t < n_threads; ++t) {
                phase_s[0] += t_tx[t];
                phase_s[1] += t_rx[t];
            }
        }
        return std::chrono::duration<double>(t1 - t0).count();
    } catch (...) {
        return -2.0;
    }
}

double oracle_loopback_timed(const uint32_t* cfg, const uint32_t* psdef, uint32_t n_packets, uint32_t n_threads,
                             uint64_t seed, uint32_t sync_pre, uint32_t sync_chunk) {
    return oracle_loopback_timed2(cfg, psdef, n_packets, n_threads, seed, sync_pre, sync_chunk, nullptr);
}

// Synchronisation of one window (= one chunk starting at iq[0]); reports in search order.
// scfg: u, b, os_min, L, M, N_ant, N_ant_limited, chunk_len ; iq [N_ant_limited][S_win] cf32
// out [max_reports][SYNC_NF] doubles: found, det_ant, det_rms, det_metric, det_time, det_time_jb,
//   coarse_local, coarse_64, cfo_frac, u, b, N_eff_TX, fine_local, fine_64, coarse_metric[8],
//   rms[8], xc_metric[4], xc_idx[4]
static constexpr int SYNC_NF = 38;
int oracle_sync(const uint32_t* scfg, const float* iq, uint32_t S_win, uint32_t max_reports, int use_float,
                double* out) {
    try {
        sync_cfg_t c;
        c.u = scfg[0];
        c.b = scfg[1];
        c.os_min = scfg[2];
        c.L = scfg[3];
        c.M = scfg[4];
        c.N_ant = scfg[5];
        c.N_ant_limited = scfg[6];
        c.chunk_len = scfg[7];
        const auto r = use_float ? sync_search<float>(c, iq, S_win, max_reports)
                                 : sync_search<double>(c, iq, S_win, max_reports);
        for (size_t i = 0; i < r.size(); ++i) {
            const auto& o = r[i];
            double* d = out + i * SYNC_NF;
            const double v[14] = {double(o.found), double(o.det_ant), o.det_rms, o.det_metric, double(o.det_time),
                                  double(o.det_time_jb), double(o.coarse_local), double(o.coarse_64), o.cfo_frac,
                                  double(o.u), double(o.b), double(o.N_eff_TX), double(o.fine_local),
                                  double(o.fine_64)};
            for (int k = 0; k < 14; ++k) d[k] = v[k];
            for (int k = 0; k < 8; ++k) d[14 + k] = o.coarse_metric[k];
            for (int k = 0; k < 8; ++k) d[22 + k] = o.rms[k];
            for (int k = 0; k < 4; ++k) d[30 + k] = o.xc_metric[k];
            for (int k = 0; k < 4; ++k) d[34 + k] = o.xc_idx[k];
        }
        return static_cast<int>(r.size());
    } catch (const std::exception& e) {
        std::fprintf(stderr, "oracle_sync: %s\n", e.what());
        return -2;
    }
}

// out: geometry n_pattern, bos, stf_len, pattern, step, A, B, C, D, search_len, lb_len, xc_l,
//      xc_len, tmpl_len, n_templates ; *rms_min
int oracle_sync_geometry(const uint32_t* scfg, uint32_t* out, float* rms_min) {
    sync_cfg_t c;
    c.u = scfg[0];
    c.b = scfg[1];
    c.os_min = scfg[2];
    c.L = scfg[3];
    c.M = scfg[4];
    c.N_ant = scfg[5];
    c.N_ant_limited = scfg[6];
    c.chunk_len = scfg[7];
    const auto g = sync_geometry(c);
    const uint32_t v[] = {g.n_pattern, g.bos, g.stf_len, g.pattern, g.step, g.A, g.B, g.C, g.D, g.search_len,
                          g.lb_len, g.xc_l, g.xc_len, g.tmpl_len, g.n_templates};
    std::memcpy(out, v, sizeof(v));
    *rms_min = g.rms_min;
    return 0;
}

// STF template (cf32 interleaved, tmpl_len samples)
int oracle_stf_template(const uint32_t* scfg, uint32_t N_eff_TX, float* out) {
    try {
        sync_cfg_t c;
        c.u = scfg[0];
        c.b = scfg[1];
        c.os_min = scfg[2];
        c.L = scfg[3];
        c.M = scfg[4];
        const auto t = stf_template(c, N_eff_TX);
        for (size_t i = 0; i < t.size(); ++i) {
            out[2 * i] = static_cast<float>(t[i].real());
            out[2 * i + 1] = static_cast<float>(t[i].imag());
        }
        return static_cast<int>(t.size());
    } catch (...) {
        return -2;
    }
}

}  // extern "C"
