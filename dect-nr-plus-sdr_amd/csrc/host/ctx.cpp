// C-ABI implementation (include/dnrp.h): context, per-configuration device tables, network-ID
// scrambling sequences, batched TX / RX phase launches.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <tuple>
#include <vector>

#include "ctx_internal.hpp"

using namespace dnrp;
using namespace dnrp::host;

namespace dnrp::host {


dev::fft_plan make_plan(uint32_t N) {
    dev::fft_plan p{};
    p.N = N;
    uint32_t r = N;
    while (r % 4 == 0 && r > 1) {
        p.radix[p.nr++] = 4;
        r /= 4;
    }
    while (r % 2 == 0) {
        p.radix[p.nr++] = 2;
        r /= 2;
    }
    while (r % 3 == 0) {
        p.radix[p.nr++] = 3;
        r /= 3;
    }
    return p;  // r must be 1 (sizes 64..16384 of tx_rx.hpp:67-69)
}

std::vector<float2> twiddles(uint32_t N) {
    std::vector<float2> t(N);
    for (uint32_t j = 0; j < N; ++j) {
        const double a = -2.0 * M_PI * static_cast<double>(j) / static_cast<double>(N);
        t[j] = make_float2(static_cast<float>(std::cos(a)), static_cast<float>(std::sin(a)));
    }
    return t;
}

std::vector<float2> constellation(uint32_t N_bps) {  // 3GPP TS 36.211 §7.1, index bits MSB first
    const uint32_t n = 1u << N_bps;
    std::vector<float2> t(n);
    auto bit = [&](uint32_t i, uint32_t k) { return static_cast<int>((i >> (N_bps - 1 - k)) & 1u); };
    for (uint32_t i = 0; i < n; ++i) {
        double re = 0, im = 0, nrm = 1;
        switch (N_bps) {
            case 1:
                re = im = 1 - 2 * bit(i, 0);
                nrm = std::sqrt(2.0);
                break;
            case 2:
                re = 1 - 2 * bit(i, 0);
                im = 1 - 2 * bit(i, 1);
                nrm = std::sqrt(2.0);
                break;
            case 4:
                re = (1 - 2 * bit(i, 0)) * (2 - (1 - 2 * bit(i, 2)));
                im = (1 - 2 * bit(i, 1)) * (2 - (1 - 2 * bit(i, 3)));
                nrm = std::sqrt(10.0);
                break;
            case 6:
                re = (1 - 2 * bit(i, 0)) * (4 - (1 - 2 * bit(i, 2)) * (2 - (1 - 2 * bit(i, 4))));
                im = (1 - 2 * bit(i, 1)) * (4 - (1 - 2 * bit(i, 3)) * (2 - (1 - 2 * bit(i, 5))));
                nrm = std::sqrt(42.0);
                break;
            default:
                re = (1 - 2 * bit(i, 0)) * (8 - (1 - 2 * bit(i, 2)) * (4 - (1 - 2 * bit(i, 4)) * (2 - (1 - 2 * bit(i, 6)))));
                im = (1 - 2 * bit(i, 1)) * (8 - (1 - 2 * bit(i, 3)) * (4 - (1 - 2 * bit(i, 5)) * (2 - (1 - 2 * bit(i, 7)))));
                nrm = std::sqrt(170.0);
                break;
        }
        t[i] = make_float2(static_cast<float>(re / nrm), static_cast<float>(im / nrm));
    }
    return t;
}

// input-major block taps for the register-blocked resampler (polyphase.hpp): rows i = 0..W-1 of
// LP = 4*ceil(L/4) floats, g[i][k] = h[ph_k + (hl + o_k - i) * L] inside output k's FIR span
std::vector<float> taps_polyphase(const geo::resampler_t& rs, uint32_t* count) {
    const uint32_t L = rs.L, M = rs.M, hl = rs.hl;
    const uint32_t W = hl + 1 + ((L - 1) * M) / L, lp = (L + 3) / 4 * 4;
    std::vector<float> g(size_t(W) * lp, 0.0f);
    for (uint32_t i = 0; i < W; ++i)
        for (uint32_t k = 0; k < L; ++k) {
            const int d = static_cast<int>(hl + (k * M) / L) - static_cast<int>(i);
            if (d >= 0 && d <= static_cast<int>(hl)) g[i * lp + k] = rs.h[(k * M) % L + d * L];
        }
    *count = static_cast<uint32_t>(g.size());
    return g;
}

double phasor_arg(double rad) {  // mixer_t::set_phase* builds float phasors (mixer.cpp:27-33)
    const float c = std::cos(static_cast<float>(rad)), s = std::sin(static_cast<float>(rad));
    return std::atan2(static_cast<double>(s), static_cast<double>(c));
}

void fill_pairs(uint32_t N_TS, uint32_t* pair, uint32_t& mod) {  // transmit_diversity_precoding.cpp:48-75
    std::memset(pair, 0, 12 * sizeof(uint32_t));
    mod = 1;
    if (N_TS <= 1) return;
    mod = geo::txdiv_modulo(N_TS);
    for (uint32_t i = 0; i < mod; ++i) {
        uint32_t A, B;
        geo::txdiv_pair(N_TS, i, A, B);
        pair[i] = A | (B << 4);
    }
}


}  // namespace dnrp::host

namespace {

uint32_t G_cap_default(const dnrp_cfg& c) {
    // scrambling sequences cover at least one PacketLength=2 slot packet of the device class
    dnrp_psdef d{c.u_max, c.b_max, 1, 2, 0, 9, 6144};
    dnrp_packet_sizes q;
    if (geo::packet_sizes(d, q)) return q.G;
    return 1u << 20;
}

int ensure_seq(dnrp_ctx* ctx, netid_seq& s, uint32_t nid, uint32_t nbits) {
    if (s.nbits >= nbits) return DNRP_OK;
    const uint32_t len = std::max(nbits, G_cap_default(ctx->cfg));
    // scrambling_pdc.cpp:41-48: type 1 c_init = id & 0xFF, type 2 c_init = id >> 8
    if (!s.t1.upload(geo::gold_bits_packed(nid & 0xFFu, len))) return DNRP_ENOMEM;
    if (!s.t2.upload(geo::gold_bits_packed(nid >> 8, len))) return DNRP_ENOMEM;
    s.nbits = len;
    return DNRP_OK;
}

tx_tables* get_tx(dnrp_ctx* ctx, const dnrp_psdef& d, int* err) {
    const auto key = std::make_tuple(d.u, d.b, d.PacketLengthType, d.PacketLength, d.tm_mode_index, d.mcs_index, d.Z);
    auto it = ctx->txt.find(key);
    if (it != ctx->txt.end()) return it->second.get();
    auto t = std::make_unique<tx_tables>();
    if (!geo::packet_sizes(d, t->q, &t->tm)) {
        *err = DNRP_ECONFIG;
        return nullptr;
    }
    const auto& c = ctx->cfg;
    if (d.u > c.u_max || d.b > c.b_max || t->q.N_TX > c.N_TX_max || t->q.N_bps > 8) {
        *err = DNRP_EUNSUPPORTED;
        return nullptr;
    }
    t->dm = geo::make_dims(c, d, t->q);
    t->plan = make_plan(t->dm.Nd);
    t->rs = geo::make_resampler(c.L, c.M, c.os_min, prm::RS_TX);
    const auto m = geo::build_maps(d.b, t->tm.N_TS, t->tm.N_eff_TX, t->q.N_DF_symb);
    std::vector<float2> stf(m.Nf);
    for (uint32_t k = 0; k < m.Nf; ++k) stf[k] = make_float2(m.stf[k].real(), m.stf[k].imag());
    std::vector<float2> W;
    const uint32_t ncb = geo::W_codebooks(t->tm.N_TS, t->tm.N_TX);
    for (uint32_t cb = 0; cb < ncb; ++cb) {
        float s = 1.0f;
        for (const auto& w : geo::W_matrix(t->tm.N_TS, t->tm.N_TX, cb, &s)) W.push_back(make_float2(w.real(), w.imag()));
        t->wscale.push_back(s);
        t->wscale_opt.push_back(geo::W_scaling_optimal_DAC(t->tm.N_TS, t->tm.N_TX, cb));
        // one nonzero entry in every antenna row (tx.hip TXS_TXDIV1)
        bool oh = true;
        for (uint32_t a = 0; a < t->tm.N_TX; ++a) {
            uint32_t nzc = 0;
            for (uint32_t ts = 0; ts < t->tm.N_TS; ++ts) {
                const float2 w = W[(size_t(cb) * t->tm.N_TX + a) * t->tm.N_TS + ts];
                nzc += (w.x != 0.f || w.y != 0.f) ? 1u : 0u;
            }
            oh = oh && nzc == 1;
        }
        t->w_onehot.push_back(oh ? 1 : 0);
    }
    t->pdc_off_h = m.pdc_sym_off;
    // transmit diversity TS pair (A | B << 4) per PCC/PDC cell into the code words (kernels.hpp CODE_*)
    std::vector<uint32_t> code = m.code;
    {
        uint32_t pair[12], mod = 1;
        fill_pairs(t->tm.N_TS, pair, mod);
        for (auto& c : code) {
            const uint32_t ty = c & dev::CODE_MASK;
            if (ty == dev::CODE_DRS) {  // DRS: the stream in the pair field too (one W-row read per bin)
                c |= (c & 7u) << dev::CODE_PAIR_SHIFT;
                continue;
            }
            if (ty != dev::CODE_PCC && ty != dev::CODE_PDC) continue;
            const uint32_t j = c & ~dev::CODE_MASK;
            if (j > dev::CODE_J_MASK) {
                *err = DNRP_EUNSUPPORTED;
                return nullptr;
            }
            c = ty | j | (pair[(j >> 1) % mod] << dev::CODE_PAIR_SHIFT);
        }
    }
    if (uint64_t(t->dm.N_packet_rs + 2 * t->rs.hl) * t->rs.L >= (1ull << 32)) {  // 32-bit output indexing
        *err = DNRP_EUNSUPPORTED;
        return nullptr;
    }
    {
        // streaming TX kernel: cell code per FFT bin (tx.hip tx_wg::code layout, 0 for empty bins)
        const uint32_t N = t->q.N_b_OCC, Nf = N + 1, Nd = t->dm.Nd;
        if (Nd == 1024) {
            std::vector<uint32_t> cb(size_t(t->q.N_DF_symb + 1) * 1024, 0u);
            for (uint32_t l = 0; l <= t->q.N_DF_symb; ++l)
                for (uint32_t nn = 0; nn < 1024; ++nn) {
                    uint32_t k = 0xFFFFFFFFu;
                    if (nn <= N / 2) k = N / 2 + nn;
                    else if (nn >= t->dm.off_lower && nn < t->dm.off_lower + N / 2) k = nn - t->dm.off_lower;
                    // bin nn = lane + 64 m of the kernel's layout at [m / 4][lane][m % 4]: one 16-B load
                    // per lane fetches the codes of four of its bins
                    const uint32_t ln = nn & 63u, m = nn >> 6;
                    if (k != 0xFFFFFFFFu) cb[size_t(l) * 1024 + ((m >> 2) * 64 + ln) * 4 + (m & 3u)] = code[size_t(l) * Nf + k];
                }
            for (uint32_t l = 0; l <= t->q.N_DF_symb; ++l)
                for (uint32_t k = 0; k < Nf; ++k)
                    if ((code[size_t(l) * Nf + k] & dev::CODE_MASK) == dev::CODE_PCC) {
                        if (l >= 32) {
                            *err = DNRP_EUNSUPPORTED;
                            return nullptr;
                        }
                        t->pcc_syms |= 1u << l;
                    }
            if (!t->code_bin.upload(cb)) {
                *err = DNRP_ENOMEM;
                return nullptr;
            }
            // one-hot W rows: every bin's code resolved per antenna stream ts (tx.hip bin_oh), so the
            // kernel maps a bin without the pair tests (tx.hip bin_df TXS_TXDIV1 / TXS_SM1 restated)
            const uint32_t NTS = t->tm.N_TS;
            bool oh_ok = NTS > 1;
            std::vector<uint32_t> oh(oh_ok ? size_t(NTS) * cb.size() : 0u, 0u);
            for (uint32_t ts = 0; ts < NTS && oh_ok; ++ts)
                for (size_t i = 0; i < cb.size(); ++i) {
                    const uint32_t c = cb[i], ty = c & dev::CODE_MASK, j = c & dev::CODE_J_MASK;
                    const uint32_t pr = (c >> dev::CODE_PAIR_SHIFT) & 0xFFu;
                    const bool ua = (pr & 0xFu) == ts, ub = (pr >> 4) == ts;
                    uint32_t o = 0;
                    if (ty == dev::CODE_DRS) {
                        if (ua) o = dev::CODE_DRS | ((j & 8u) ? dev::OH_FX : 0u);
                    } else if (ty == dev::CODE_PDC && !t->tm.txdiv) {  // spatial multiplexing: the stream's symbol
                        const uint64_t js = uint64_t(j) * t->tm.N_SS + ts;
                        if (js > dev::CODE_J_MASK) oh_ok = false;
                        o = dev::CODE_PDC | static_cast<uint32_t>(js & dev::CODE_J_MASK);
                    } else if ((ty == dev::CODE_PDC || ty == dev::CODE_PCC) && (ua || ub)) {
                        // SFBC: stream A maps symbol j, stream B the partner j ^ 1 with (-re, +im) for
                        // even j, (+re, -im) for odd j (transmit_diversity_precoding.cpp:37-75)
                        const uint32_t flip = ua ? 0u : ((j & 1u) ? dev::OH_FY : dev::OH_FX);
                        o = ty | (j ^ (ua ? 0u : 1u)) | flip;
                    } else if (ty == dev::CODE_STF) {
                        o = c;
                    }
                    oh[size_t(ts) * cb.size() + i] = o;
                }
            if (oh_ok && !t->code_oh.upload(oh)) {
                *err = DNRP_ENOMEM;
                return nullptr;
            }
        }
    }
    if (!t->code.upload(code) || !t->stf.upload(stf) || !t->pdc_off.upload(m.pdc_sym_off) || !t->W.upload(W) || !t->taps.upload(t->rs.h) || !t->taps_pp.upload(taps_polyphase(t->rs, &t->npp)) ||
        !t->tw.upload(twiddles(t->dm.Nd)) || !t->qam.upload(constellation(t->q.N_bps)) ||
        !t->qpsk.upload(constellation(2))) {
        *err = DNRP_ENOMEM;
        return nullptr;
    }
    auto* r = t.get();
    ctx->txt[key] = std::move(t);
    return r;
}

// OFDM symbol of every PCC cell (rx_cells_kernel reads the symbol per cell in both phases)
std::vector<uint16_t> pcc_cell_symbols(const geo::maps_t& m) {
    std::vector<uint16_t> sym(m.pcc_k.size());
    for (size_t s = 0; s + 1 < m.pcc_sym_off.size(); ++s)
        for (uint32_t j = m.pcc_sym_off[s]; j < m.pcc_sym_off[s + 1]; ++j) sym[j] = static_cast<uint16_t>(m.pcc_l[s]);
    return sym;
}

dev::rx_front_args front_args(dnrp_ctx* ctx, rx1_tables* t, const float* iq, const uint32_t* sel,
                              const rx_plan_dev* plan = nullptr);

// SFBC pair union windows of full symbols (rx_lut::pair_w, the fused receiver): per LUT row, stream
// class and pair u on subcarriers 2u, 2u + 1 (DC skipped) eq_compute's mean weights 0.5f (lo + hi) per
// tap of the union window, in the same float arithmetic. Left empty (false is only an upload failure)
// when some union window has more than 4 taps (the low-SNR profiles).
bool pair_windows(const geo::lut_t& L, uint32_t N_occ, dbuf& pair_w, dbuf& pair_p) {
    const uint32_t Nf = N_occ + 1, half = N_occ / 2, np = half, n = L.n;
    std::vector<float4> pw4(size_t(L.T) * 4 * np);
    std::vector<uint32_t> pb(size_t(L.T) * 4 * np);
    for (uint32_t r = 0; r < L.T; ++r)
        for (uint32_t cl = 0; cl < 4; ++cl)
            for (uint32_t u = 0; u < np; ++u) {
                const uint32_t k0 = 2 * u + (2 * u >= half ? 1u : 0u), k1 = 2 * u + 1 + (2 * u + 1 >= half ? 1u : 0u);
                const uint32_t w0 = L.pilot_weight[(size_t(r) * 4 + cl) * Nf + k0];
                const uint32_t w1 = L.pilot_weight[(size_t(r) * 4 + cl) * Nf + k1];
                const uint32_t p0 = w0 & 0xFFFFu, p1 = w1 & 0xFFFFu;
                const bool up = p1 >= p0;
                const uint32_t sh = up ? p1 - p0 : p0 - p1;
                const uint32_t wl = (up ? w0 : w1) >> 16, wh = (up ? w1 : w0) >> 16;
                if (n + sh > 4) return true;
                float wv[4];
                for (uint32_t i = 0; i < 4; ++i) {
                    const float lo = i < n ? L.weights[size_t(wl) * n + i] : 0.f;
                    const float hi = i >= sh && i - sh < n ? L.weights[size_t(wh) * n + i - sh] : 0.f;
                    wv[i] = 0.5f * (lo + hi);
                }
                pw4[(size_t(r) * 4 + cl) * np + u] = make_float4(wv[0], wv[1], wv[2], wv[3]);
                pb[(size_t(r) * 4 + cl) * np + u] = up ? p0 : p1;
            }
    return pair_w.upload(pw4) && pair_p.upload(pb);
}

rx1_tables* get_rx1(dnrp_ctx* ctx, uint32_t u, uint32_t b, uint32_t N_eff_TX, int* err) {
    const auto key = std::make_tuple(u, b, N_eff_TX);
    auto it = ctx->rx1t.find(key);
    if (it != ctx->rx1t.end()) return it->second.get();
    const auto& c = ctx->cfg;
    if (!(N_eff_TX == 1 || N_eff_TX == 2 || N_eff_TX == 4)) {  // N_eff_TX = 8 PCC ps LUT, see DESIGN.md
        *err = DNRP_EUNSUPPORTED;
        return nullptr;
    }
    if (u > c.u_max || b > c.b_max || N_eff_TX > c.N_TX_max) {
        *err = DNRP_EUNSUPPORTED;
        return nullptr;
    }
    auto t = std::make_unique<rx1_tables>();
    t->u = u;
    t->b = b;
    t->N_eff_TX = N_eff_TX;
    const uint64_t rate = uint64_t(c.u_max) * c.b_max * 1728000ull * c.os_min;
    t->Nd = static_cast<uint32_t>(rate / (uint64_t(u) * 27000ull));
    t->N_occ = 56 * b;
    t->off_lower = 32 * b + (t->Nd - 64 * b) + 4 * b;
    t->CP = 8 * b * t->Nd / (64 * b);
    const uint32_t stf = u == 1 ? 112 * b : 144 * b;
    t->STF_CP = (stf - 64 * b) * t->Nd / (64 * b);
    t->n_pattern = u == 1 ? 7 : 9;
    t->pattern_len = 16 * b * t->Nd / (64 * b);
    t->plan = make_plan(t->Nd);
    t->rs = geo::make_resampler(c.M, c.L, c.os_min, prm::RS_RX_SYNCED);  // RX swaps L and M (rx_synced.cpp:65-73)
    t->maps = geo::build_maps(b, N_eff_TX, N_eff_TX, 20);
    std::vector<geo::op_t> pcc_ops, dummy;
    geo::build_rx_ops(t->maps, N_eff_TX, 20, c.chestim_mode_lr != 0, std::max(1u, c.chestim_lr_stride), pcc_ops, dummy,
                      t->pcc_max);
    std::vector<float2> stfv(t->maps.Nf);
    for (uint32_t k = 0; k < t->maps.Nf; ++k) stfv[k] = make_float2(t->maps.stf[k].real(), t->maps.stf[k].imag());
    const auto plan = geo::build_rx_plan(t->maps, pcc_ops, N_eff_TX);
    t->drs_arith = geo::drs_tables_arithmetic(t->maps);
    bool ok = t->stf.upload(stfv) && t->tw.upload(twiddles(t->Nd)) && t->taps.upload(t->rs.h) && t->taps_pp.upload(taps_polyphase(t->rs, &t->npp)) &&
              t->drs_k.upload(t->maps.drs_k) && t->drs_v.upload(t->maps.drs_v) && t->pcc_k.upload(t->maps.pcc_k) &&
              t->pcc_sym.upload(pcc_cell_symbols(t->maps)) &&
              t->bplan.upload(plan);
    const uint32_t Nsv = N_eff_TX <= 2 ? 5 : 10;
    for (uint32_t mode = 0; mode < 2 && ok; ++mode)
        for (uint32_t p = 0; p < 3 && ok; ++p) {
            const auto L = geo::build_lut(mode ? Nsv : 0, b, c.b_max, c.u_max, p);
            ok = t->lut_pw[mode][p].upload(L.pilot_weight) && t->lut_w[mode][p].upload(L.weights) &&
                 (N_eff_TX < 2 || pair_windows(L, t->N_occ, t->lut_pair_w[mode][p], t->lut_pair_p[mode][p]));
            t->lut_n[mode][p] = L.n;
            t->lut_nw[mode][p] = static_cast<uint32_t>(L.weights.size());
            // 16-B slots: the segment table behind both weight tables stays 16-B aligned in LDS
            t->wcap[mode] = std::max(t->wcap[mode], (t->lut_nw[mode][p] + 3u) & ~3u);
            ok = ok && L.n < (1u << 15);  // eq_work packs the tap count into 15 bits
            t->lut_T[mode] = L.T;
        }
    std::vector<dev::rx_lut> luts(6);
    for (uint32_t mode = 0; mode < 2; ++mode)
        for (uint32_t p = 0; p < 3; ++p)
            luts[mode * 3 + p] = {t->lut_pw[mode][p].as<uint32_t>(), t->lut_w[mode][p].as<float>(), t->lut_n[mode][p],
                                  t->lut_nw[mode][p], t->lut_pair_w[mode][p].as<float4>(), t->lut_pair_p[mode][p].as<uint32_t>()};
    if (!ok || !t->luts.upload(luts)) {
        *err = DNRP_ENOMEM;
        return nullptr;
    }
    // a geometry is rejected only when neither the chunked STF layout (rx.hip rx_stf_lds, used from
    // N_b_DFT_os = 8192) nor any rx_fft layout fits one CU's 160 KiB of LDS
    if (!dev::rx_front_fits(front_args(ctx, t.get(), nullptr, nullptr))) {
        *err = DNRP_EUNSUPPORTED;
        return nullptr;
    }
    auto* r = t.get();
    ctx->rx1t[key] = std::move(t);
    return r;
}

rx2_tables* get_rx2(dnrp_ctx* ctx, const dnrp_psdef& d, int* err) {
    const auto key = std::make_tuple(d.u, d.b, d.PacketLengthType, d.PacketLength, d.tm_mode_index, d.mcs_index, d.Z);
    auto it = ctx->rx2t.find(key);
    if (it != ctx->rx2t.end()) return it->second.get();
    auto t = std::make_unique<rx2_tables>();
    geo::tm_t tm;
    if (!geo::packet_sizes(d, t->q, &tm)) {
        *err = DNRP_ECONFIG;
        return nullptr;
    }
    // rx_synced.cpp:1331-1333: spatial multiplexing (AxA MIMO) is a \todo in the reference receiver;
    // demodulated here by MMSE only when the context opted in (DNRP_RX_MODE_SM_MMSE)
    const bool sm = tm.N_SS > 1;
    if ((sm && !(ctx->rx_mode & DNRP_RX_MODE_SM_MMSE)) || (sm && (tm.N_SS != tm.N_eff_TX || tm.N_SS > 4 ||
                                                                 ctx->cfg.N_TX_max < tm.N_SS)) ||
        tm.N_eff_TX > 4 || t->q.N_bps > 8) {
        *err = DNRP_EUNSUPPORTED;
        return nullptr;
    }
    t->sm = sm;
    t->maps = geo::build_maps(d.b, tm.N_TS, tm.N_eff_TX, t->q.N_DF_symb);
    std::vector<geo::op_t> pcc_ops, pdc_ops;
    uint32_t pm;
    geo::build_rx_ops(t->maps, tm.N_eff_TX, t->q.N_DF_symb, ctx->cfg.chestim_mode_lr != 0,
                      std::max(1u, ctx->cfg.chestim_lr_stride), pcc_ops, pdc_ops, pm);
    const auto plan = geo::build_rx_plan(t->maps, pdc_ops, tm.N_eff_TX, !sm);
    std::vector<uint16_t> csym(t->maps.pdc_k.size());
    for (uint32_t l = 0; l <= t->q.N_DF_symb; ++l)
        for (uint32_t j = t->maps.pdc_sym_off[l]; j < t->maps.pdc_sym_off[l + 1]; ++j) csym[j] = static_cast<uint16_t>(l);
    if (!t->pdc_k.upload(t->maps.pdc_k) || !t->pdc_sym.upload(csym) || !t->bplan.upload(plan)) {
        *err = DNRP_ENOMEM;
        return nullptr;
    }
    // MIMO report tables (estimator_mimo.cpp:80-160): per TS the latest DRS symbol carrying it, its
    // cells at offset step/2 + c*step (step = N_DRS_cells_b / 4) and their DRS values
    {
        const uint32_t NTS = tm.N_eff_TX, nd = t->maps.drs_v.size() / 8, step = nd / prm::RX_MIMO_WIDEBAND_CELLS,
                       off = step / 2;
        constexpr uint32_t NW = prm::RX_MIMO_WIDEBAND_CELLS;
        static_assert(NW == 4, "rx_mimo_kernel sums 4 wideband cells");
        std::vector<uint32_t> cells(NTS * NW, 0);
        std::vector<float> signs(NTS * NW, 1.f);
        for (uint32_t ts = 0; ts < NTS; ++ts) {
            const geo::drs_sym_t* last = nullptr;
            for (const auto& d : t->maps.drs)
                if (d.ts_first <= ts && ts <= d.ts_last) last = &d;
            if (!last) continue;
            for (uint32_t c = 0; c < NW; ++c) {
                const uint32_t i = off + c * step;
                cells[ts * NW + c] = (last->l << 16) | t->maps.drs_k[(last->parity * 4 + ts % 4) * nd + i];
                signs[ts * NW + c] = t->maps.drs_v[ts * nd + i];
            }
        }
        static const uint32_t A_nonzero[9] = {0, 0, 2, 0, 12, 0, 0, 0, 0};  // beamforming_...mapping.hpp:110-119, N_TS = 1
        auto book = [&](uint32_t N, dbuf& W, dbuf& sc, uint32_t& ncb, uint32_t& A0) {
            if (N < 2) return true;
            if (N != 2 && N != 4) {
                // no single-stream codebook for 8 antennas (W_t::get_W(1, 8) is the SISO entry, and
                // the reference's W_mat_single.at(tx) throws, estimator_mimo.cpp:160-200): no
                // candidates, so rx_mimo_kernel reports 0xFFFFFFFF ("no recommendation")
                ncb = 0;
                A0 = 0;
                return W.upload(std::vector<float2>{make_float2(0.f, 0.f)}) && sc.upload(std::vector<float>{0.f});
            }
            ncb = geo::W_codebooks(1, N);
            A0 = A_nonzero[N];
            std::vector<float2> w;
            std::vector<float> s;
            for (uint32_t cb = 0; cb < ncb; ++cb) {
                float f = 1.f;
                for (const auto& v : geo::W_matrix(1, N, cb, &f)) w.push_back(make_float2(v.real(), v.imag()));
                s.push_back(f);
            }
            return W.upload(w) && sc.upload(s);
        };
        t->N_TS = NTS;
        if (!t->mimo_cells.upload(cells) || !t->mimo_signs.upload(signs) || !book(NTS, t->Wtx, t->stx, t->ncb_tx, t->A_tx) ||
            !book(ctx->cfg.N_TX_max, t->Wrx, t->srx, t->ncb_rx, t->A_rx)) {
            *err = DNRP_ENOMEM;
            return nullptr;
        }
        // the same cells in the fused receiver's zero-forced pilots: DRS op of the phase plan, cell index
        std::vector<uint32_t> zc(NTS * NW, 0);
        for (uint32_t ts = 0; ts < NTS; ++ts) {
            const geo::drs_sym_t* last = nullptr;
            for (const auto& d : t->maps.drs)
                if (d.ts_first <= ts && ts <= d.ts_last) last = &d;
            uint32_t dop = 0;
            while (last && dop < plan.dl.size() && plan.dl[dop] != last->l) ++dop;
            for (uint32_t c = 0; c < NW; ++c) zc[ts * NW + c] = (dop << 16) | (off + c * step);
        }
        if (!t->mimo_zcells.upload(zc)) {
            *err = DNRP_ENOMEM;
            return nullptr;
        }
    }
    // fused PDC receiver (kernels/rx_fused.hip): one entry per PDC-bearing symbol with the event of
    // its plan segment and the pilot sources of its epoch. Holds where every segment is a run of whole
    // symbols and, for transmit diversity, every symbol has an even cell count (SFBC pairs do not
    // straddle symbols); otherwise the Y path runs.
    {
        const auto& m = t->maps;
        auto is_drs = [&](uint32_t l) {
            for (const auto& d : m.drs)
                if (d.l == l) return true;
            return false;
        };
        const bool pairs = tm.N_eff_TX > 1;
        bool ok = !sm && (tm.N_eff_TX == 1 || tm.N_eff_TX == 2 || tm.N_eff_TX == 4) && plan.dl.size() <= dev::RX_MAX_DOPS;
        std::vector<dev::rx_fsym> fs;
        for (const auto& e : plan.epochs)
            for (uint32_t s = e.seg0; s < e.seg1 && ok; ++s) {
                const auto& g = plan.segs[s];
                ok = g.kind == geo::OP_PDC && g.drs_cnt > 0;
                uint32_t j = g.j0;
                for (uint32_t l = 0; l <= t->q.N_DF_symb && j < g.j1 && ok; ++l) {
                    const uint32_t c0 = m.pdc_sym_off[l], c1 = m.pdc_sym_off[l + 1];
                    if (c1 <= j || c0 == c1) continue;
                    if (c0 != j || c1 > g.j1 || (pairs && ((c0 | c1) & 1u))) {
                        ok = false;
                        break;
                    }
                    dev::rx_fsym f{};
                    f.l = l;
                    f.j0 = c0;
                    f.j1 = c1;
                    const bool from_y = l <= pm || is_drs(l);
                    // every occupied subcarrier but DC in order: the kernel computes the subcarriers
                    const uint32_t N = 56 * d.b;
                    bool full = c1 - c0 == N;
                    for (uint32_t c = 0; c < N && full; ++c) full = m.pdc_k[c0 + c] == c + (c >= N / 2 ? 1u : 0u);
                    f.info = (g.mode & 1u) | (g.swap & 3u) << 1 | (g.off & 0xFFu) << 4 | (from_y ? 1u : 0u) << 12 |
                             (full ? 1u : 0u) << 13;
                    f.rel = g.rel;
                    f.drs_cnt = g.drs_cnt;
                    std::memcpy(f.src, e.src, sizeof(f.src));
                    fs.push_back(f);
                    j = c1;
                }
                ok = ok && j == g.j1;
            }
        std::vector<uint16_t> dsy;
        for (const auto& d : m.drs)
            if (d.l > pm && d.l <= t->q.N_DF_symb) {
                dsy.push_back(static_cast<uint16_t>(d.l));
                if (m.pdc_sym_off[d.l + 1] > m.pdc_sym_off[d.l]) t->drs_y = true;
            }
        if (dsy.empty()) dsy.push_back(0);  // keeps the upload non-empty; n_drs_syms stays 0
        t->n_drs_syms = static_cast<uint32_t>(dsy.size()) - (dsy[0] == 0 ? 1u : 0u);
        t->n_fsym = static_cast<uint32_t>(fs.size());
        t->fused_ok = ok && !fs.empty();
        if (t->fused_ok && (!t->fsym.upload(fs) || !t->drs_syms.upload(dsy))) {
            *err = DNRP_ENOMEM;
            return nullptr;
        }
    }
    // epoch receiver (kernels/rx_epoch.hip): the symbols whose bins each epoch's cells read, minus the
    // PCC phase's (in Y from the PCC call) and the DRS symbols (the DRS pass); a symbol claimed by two
    // epochs (or an epoch list past 16 bits) leaves the Y path in charge
    {
        const auto& m = t->maps;
        auto is_drs = [&](uint32_t l) {
            for (const auto& d : m.drs)
                if (d.l == l) return true;
            return false;
        };
        bool ok = !sm && plan.dl.size() <= dev::RX_MAX_DOPS;
        std::vector<uint16_t> off{0}, syms, dsy;
        std::vector<int> owner(t->q.N_DF_symb + 2, -1);
        for (size_t e = 0; e < plan.epochs.size() && ok; ++e) {
            std::vector<uint32_t> ls;
            for (uint32_t s = plan.epochs[e].seg0; s < plan.epochs[e].seg1; ++s) {
                const auto& g = plan.segs[s];
                if (g.kind != geo::OP_PDC) {
                    ok = false;
                    break;
                }
                for (uint32_t l = 1; l <= t->q.N_DF_symb; ++l)
                    if (m.pdc_sym_off[l] < g.j1 && m.pdc_sym_off[l + 1] > g.j0 && l > pm && !is_drs(l)) ls.push_back(l);
            }
            std::sort(ls.begin(), ls.end());
            ls.erase(std::unique(ls.begin(), ls.end()), ls.end());
            for (uint32_t l : ls) {
                if (owner[l] >= 0) ok = false;
                owner[l] = static_cast<int>(e);
                syms.push_back(static_cast<uint16_t>(l));
            }
            off.push_back(static_cast<uint16_t>(syms.size()));
        }
        for (const auto& d : m.drs)
            if (d.l > pm && d.l <= t->q.N_DF_symb) dsy.push_back(static_cast<uint16_t>(d.l));
        t->n_ep_drs = static_cast<uint32_t>(dsy.size());
        if (syms.empty()) syms.push_back(0);  // non-empty uploads
        if (dsy.empty()) dsy.push_back(0);
        t->ep_ok = ok && plan.epochs.size() > 0;
        if (t->ep_ok && (!t->ep_off.upload(off) || !t->ep_sym.upload(syms) || !t->ep_drs.upload(dsy))) {
            *err = DNRP_ENOMEM;
            return nullptr;
        }
    }
    auto* r = t.get();
    ctx->rx2t[key] = std::move(t);
    return r;
}

// the DRS SNR sums of a phase come from the front end (rx_fft_wave_kernel) where it runs; both phases
// of a packet use the same PCC-phase geometry t, so the PCC and PDC launches agree
bool snr_from_front(dnrp_ctx* ctx, rx1_tables* t);

dev::rx_front_args front_args(dnrp_ctx* ctx, rx1_tables* t, const float* iq, const uint32_t* sel,
                              const rx_plan_dev* plan) {
    dev::rx_front_args a{};
    a.plan = t->plan;
    a.N_occ = t->N_occ;
    a.off_lower = t->off_lower;
    a.CP = t->CP;
    a.STF_CP = t->STF_CP;
    a.N_RX = ctx->cfg.N_TX_max;
    a.S_in = ctx->rx_S_in;
    a.n_pattern = t->n_pattern;
    a.pattern_len = t->pattern_len;
    a.b = t->b;
    a.L = t->rs.L;
    a.M = t->rs.M;
    a.delay = t->rs.delay;
    a.hl = t->rs.hl;
    a.m_star = 0;
    while ((t->rs.delay + a.m_star * t->rs.M) % t->rs.L) ++a.m_star;
    a.p_star = (t->rs.delay + a.m_star * t->rs.M) / t->rs.L;
    a.sym_per_block = 4;
    a.Nf_pad = ctx->rx_Nf_pad;
    a.n_sym_total = ctx->rx_nsym_cap + 1;
    a.amp_scale = std::sqrt(static_cast<float>(t->N_occ)) / static_cast<float>(t->Nd);
    a.taps = t->taps.as<float>();
    a.taps_pp = t->taps_pp.as<float>();
    a.npp = t->npp;
    a.tw = t->tw.as<float2>();
    a.stf = t->stf.as<float2>();
    a.iq = reinterpret_cast<const float2*>(iq);
    a.sel = sel;
    a.pin = ctx->rx_in.as<dev::rx_pkt_in>();
    a.st = ctx->rx_st.as<dev::rx_pkt_state>();
    a.Y = ctx->Y.as<float2>();
    {  // STF per (packet, antenna) scratch (dnrp_rx_pcc_batch sizes it): cs | rms | cells
        const size_t mb = ctx->cfg.max_batch;
        a.stf_cs = ctx->stf_part.as<double2>();
        a.stf_rms = reinterpret_cast<float*>(a.stf_cs + mb * 8);
        a.stf_ys = reinterpret_cast<float2*>(a.stf_rms + mb * 8);
        a.stf_ys_stride = 14 * ctx->cfg.b_max;
    }
    // compile-time-tap front end (rx.hip rx_fft_wave_kernel<.., true>) where the run-time taps are
    // the generated ones bit for bit (the tap-table variant measured slower, docs/DESIGN_LOG.md §6)
    a.stream = dev::rx_stream_taps_match(t->rs.h.data(), t->rs.h.size()) ? 1u : 0u;
    if (plan && dev::rx_fft_wave_path(a)) {
        a.snr_part = ctx->snr_part.as<double2>();
        a.dl = plan->dl.as<uint32_t>();
        a.dmeta = plan->dmeta.as<uint32_t>();
        a.n_dops = plan->n_dops;
        a.n_drs = t->N_occ / 4;
        a.drs_neg = geo::drs_neg_mask();
        a.sym_op = plan->sym_op.as<uint16_t>();
        a.n_sym_op = plan->n_sym_op;
        // the zero-forced pilots next to the SNR sums (the fused PDC receiver's source), where the
        // plan's ops fit below the zero op
        if (ctx->rx_fused && ctx->zd.p && plan->n_dops + 1 <= ctx->zd_dops) {
            a.zd = ctx->zd.as<float2>();
            a.zd_dops = ctx->zd_dops;
            a.zd_row = ctx->zd_row;
        }
    }
    a.n_drs = t->N_occ / 4;
    return a;
}

bool snr_from_front(dnrp_ctx* ctx, rx1_tables* t) {
    return ctx->rx_snr_front && t->drs_arith && dev::rx_fft_wave_path(front_args(ctx, t, nullptr, nullptr));
}

dev::rx_cells_args cells_args(dnrp_ctx* ctx, rx1_tables* t, const rx_plan_dev& plan, uint32_t n, const uint32_t* sel,
                              bool pdc, uint32_t N_bps, const uint32_t* kk, const uint16_t* cell_sym, int16_t* llr,
                              uint32_t llr_stride, bool sm);

// back-end launches of one phase: SNR chain, then cells (rx_back.hip); cells = false: the SNR chain
// only (the fused PDC receiver and the epoch receiver equalise)
int launch_back(dnrp_ctx* ctx, rx1_tables* t, const rx_plan_dev& plan, uint32_t n, const uint32_t* sel, bool pdc,
                uint32_t N_bps, const uint32_t* kk, const uint16_t* cell_sym, int16_t* llr, uint32_t llr_stride,
                hipStream_t st, bool sm = false, bool cells = true) {
    const char* name = pdc ? "rx_pdc" : "rx_pcc";
    if (plan.n_dops > dev::RX_MAX_DOPS || (cells && !plan.cells_ok)) return DNRP_EUNSUPPORTED;
    if (cells) {  // the cells kernels' LDS staging (rx_back.hip): a geometry beyond one CU is unsupported
        const uint32_t R = ctx->cfg.N_TX_max, T = t->N_eff_TX;
        if (dev::cell_lds_bytes(R, T, t->N_occ / 4, t->wcap[0], t->wcap[1]) > 160 * 1024) return DNRP_EUNSUPPORTED;
        // the MMSE cells kernel's instantiations
        if (sm && !((R == 2 || R == 4 || R == 8) && (T == 2 || T == 4) && T <= R)) return DNRP_EUNSUPPORTED;
    }
    if (!ctx->lut_d.ensure(size_t(ctx->cfg.max_batch) * dev::RX_MAX_DOPS) ||
        !ctx->nv_d.ensure(size_t(ctx->cfg.max_batch) * dev::RX_MAX_DOPS * sizeof(float)))
        return DNRP_ENOMEM;
    dev::rx_snr_args s{};
    s.N_RX = ctx->cfg.N_TX_max;
    s.Nf_pad = ctx->rx_Nf_pad;
    s.n_sym_total = ctx->rx_nsym_cap + 1;
    s.n_drs = t->N_occ / 4;
    s.n_dops = plan.n_dops;
    s.is_pdc = pdc;
    s.dl = plan.dl.as<uint32_t>();
    s.dmeta = plan.dmeta.as<uint32_t>();
    s.drs_k = t->drs_k.as<uint32_t>();
    s.drs_v = t->drs_v.as<float>();
    for (int p = 0; p < 3; ++p) s.prof_snr[p] = geo::lut_profile_snr_db(p);
    s.Y = ctx->Y.as<float2>();
    s.st = ctx->rx_st.as<dev::rx_pkt_state>();
    s.lut_d = ctx->lut_d.as<uint8_t>();
    s.nv_d = ctx->nv_d.as<float>();
    s.sel = sel;
    s.snr_part = snr_from_front(ctx, t) ? ctx->snr_part.as<double2>() : nullptr;
    dev::rx_cells_args c = cells_args(ctx, t, plan, n, sel, pdc, N_bps, kk, cell_sym, llr, llr_stride, sm);
    ctx->tic(name, st);
    if (dev::launch_rx_snr(s, n, st) != hipSuccess) return DNRP_EDEVICE;
    if (cells && plan.n_epochs &&
        (sm ? dev::launch_rx_cells_sm(c, n, st) : dev::launch_rx_cells(c, n, st)) != hipSuccess)
        return DNRP_EDEVICE;
    ctx->toc(name, st);
    return DNRP_OK;
}

// the cells kernels' arguments of one phase (rx_cells_kernel, rx_epoch_kernel)
dev::rx_cells_args cells_args(dnrp_ctx* ctx, rx1_tables* t, const rx_plan_dev& plan, uint32_t n, const uint32_t* sel,
                              bool pdc, uint32_t N_bps, const uint32_t* kk, const uint16_t* cell_sym, int16_t* llr,
                              uint32_t llr_stride, bool sm) {
    dev::rx_cells_args c{};
    c.N_occ = t->N_occ;
    c.N_RX = ctx->cfg.N_TX_max;
    c.NT = t->N_eff_TX;
    c.Nf_pad = ctx->rx_Nf_pad;
    c.n_sym_total = ctx->rx_nsym_cap + 1;
    c.n_drs = t->N_occ / 4;
    c.n_dops = plan.n_dops;
    c.n_epochs = plan.n_epochs;
    c.n_pkt = n;
    c.N_bps = N_bps;
    c.wcap[0] = t->wcap[0];
    c.wcap[1] = t->wcap[1];
    fill_pairs(t->N_eff_TX, c.pair, c.mod);
    c.is_pdc = pdc;
    c.sm = sm ? 1u : 0u;
    c.nv_d = ctx->nv_d.as<float>();
    c.epochs = plan.epochs.as<dev::rx_epoch>();
    c.segs = plan.segs.as<dev::rx_seg>();
    c.dl = plan.dl.as<uint32_t>();
    c.dmeta = plan.dmeta.as<uint32_t>();
    c.drs_k = t->drs_k.as<uint32_t>();
    c.drs_v = t->drs_v.as<float>();
    c.kk = kk;
    c.cell_sym = cell_sym;
    c.luts = t->luts.as<dev::rx_lut>();
    c.Y = ctx->Y.as<float2>();
    c.lut_d = ctx->lut_d.as<uint8_t>();
    c.pcc_seq = ctx->pcc_seq.as<uint8_t>();
    c.pdc_seq = static_cast<const uint8_t* const*>(ctx->pdc_seq_ptrs.p);
    c.llr = llr;
    c.llr_stride = llr_stride;
    c.sel = sel;
    return c;
}

}  // namespace

extern "C" {

const char* dnrp_strerror(int code) {
    switch (code) {
        case DNRP_OK: return "ok";
        case DNRP_EINVAL: return "invalid argument";
        case DNRP_ECONFIG: return "invalid packet configuration";
        case DNRP_EUNSUPPORTED: return "configuration not supported by the reference receiver";
        case DNRP_ENOMEM: return "device memory allocation failed or batch too large";
        case DNRP_EDEVICE: return "HIP runtime error";
        case DNRP_ENETID: return "network ID not registered";
        case DNRP_ESTATE: return "no preceding dnrp_rx_pcc_batch";
        default: return "unknown error";
    }
}

int dnrp_ctx_create(const dnrp_cfg* cfg, dnrp_ctx** out) {
    if (!cfg || !out) return DNRP_EINVAL;
    *out = nullptr;
    const auto& c = *cfg;
    const bool uok = c.u_max == 1 || c.u_max == 2 || c.u_max == 4 || c.u_max == 8;
    const bool bok = c.b_max == 1 || c.b_max == 2 || c.b_max == 4 || c.b_max == 8 || c.b_max == 12 || c.b_max == 16;
    const bool nok = c.N_TX_max == 1 || c.N_TX_max == 2 || c.N_TX_max == 4 || c.N_TX_max == 8;
    const bool ook = c.os_min == 1 || c.os_min == 2 || c.os_min == 4 || c.os_min == 8;
    if (!uok || !bok || !nok || !ook || c.L == 0 || c.M == 0 || c.max_batch == 0) return DNRP_EINVAL;
    if (!((c.L == 1 && c.M == 1) || c.L > c.M)) return DNRP_EINVAL;  // TX up-samples (rx_pacer.cpp:50-52)
    if (hipSetDevice(c.device) != hipSuccess) return DNRP_EDEVICE;
    auto ctx = std::make_unique<dnrp_ctx>();
    ctx->cfg = c;
    if (ctx->cfg.chestim_lr_stride == 0) ctx->cfg.chestim_lr_stride = 1;
    const char* tm = std::getenv("DNRP_TIMING");
    ctx->timing = tm && tm[0] == '1';
    if (!ctx->pcc_seq.upload(geo::gold_bits_packed(0x44454354u, 200))) return DNRP_ENOMEM;  // pcc_enc.cpp:46,104
    *out = ctx.release();
    return DNRP_OK;
}

int dnrp_ctx_destroy(dnrp_ctx* ctx) {
    if (!ctx) return DNRP_EINVAL;
    (void)hipSetDevice(ctx->cfg.device);
    (void)hipDeviceSynchronize();
    delete ctx;
    return DNRP_OK;
}

int dnrp_add_network_id(dnrp_ctx* ctx, uint32_t network_id) {
    if (!ctx) return DNRP_EINVAL;
    auto& s = ctx->netid[network_id];
    if (!s) s = std::make_unique<netid_seq>();
    return ensure_seq(ctx, *s, network_id, G_cap_default(ctx->cfg));
}

int dnrp_get_packet_sizes(const dnrp_ctx* ctx, const dnrp_psdef* d, dnrp_packet_sizes* out) {
    if (!ctx || !d || !out) return DNRP_EINVAL;
    dnrp_packet_sizes q;
    if (!geo::packet_sizes(*d, q)) return DNRP_ECONFIG;
    if (d->u > ctx->cfg.u_max || d->b > ctx->cfg.b_max) return DNRP_EUNSUPPORTED;
    const auto dm = geo::make_dims(ctx->cfg, *d, q);
    q.N_b_DFT_os = dm.Nd;
    q.N_samples_packet_no_GI_os_rs = dm.N_no_GI_rs;
    q.N_samples_packet_os_rs = dm.N_packet_rs;
    *out = q;
    return DNRP_OK;
}

int dnrp_compute_packet_sizes(const dnrp_cfg* cfg, const dnrp_psdef* d, dnrp_packet_sizes* out) {
    if (!d || !out) return DNRP_EINVAL;
    dnrp_packet_sizes q;
    if (!geo::packet_sizes(*d, q)) return DNRP_ECONFIG;
    q.N_b_DFT_os = q.N_samples_packet_no_GI_os_rs = q.N_samples_packet_os_rs = 0;
    if (cfg) {
        if (cfg->L == 0 || cfg->M == 0 || cfg->os_min == 0 || d->u > cfg->u_max || d->b > cfg->b_max)
            return DNRP_EINVAL;
        const auto dm = geo::make_dims(*cfg, *d, q);
        q.N_b_DFT_os = dm.Nd;
        q.N_samples_packet_no_GI_os_rs = dm.N_no_GI_rs;
        q.N_samples_packet_os_rs = dm.N_packet_rs;
    }
    *out = q;
    return DNRP_OK;
}

int dnrp_tx_batch(dnrp_ctx* ctx, const dnrp_psdef* psdef, uint32_t n, const dnrp_tx_desc* desc, const uint8_t* pcc_d,
                  const uint8_t* pdc_d, uint32_t pdc_stride, float* iq_out, uint32_t S, void* stream) {
    if (!ctx || !psdef || (n > 0 && (!desc || !pcc_d || !pdc_d || !iq_out))) return DNRP_EINVAL;
    if (n == 0) return DNRP_OK;
    if (n > ctx->cfg.max_batch) return DNRP_ENOMEM;
    (void)hipSetDevice(ctx->cfg.device);
    int err = DNRP_OK;
    tx_tables* t = get_tx(ctx, *psdef, &err);
    if (!t) return err;
    if (S < t->dm.N_packet_rs || pdc_stride < (t->q.G + 7) / 8) return DNRP_EINVAL;
    if (t->q.N_b_OCC + 1 > 1024) return DNRP_EUNSUPPORTED;
    auto* pk = static_cast<dev::tx_pkt*>(ctx->st_tx.get(sizeof(dev::tx_pkt) * n));
    if (!pk) return DNRP_ENOMEM;
    for (uint32_t i = 0; i < n; ++i) {
        const auto& d = desc[i];
        if ((d.plcf_type != 1 && d.plcf_type != 2) || d.GI_percentage > 100) return DNRP_EINVAL;
        if (d.codebook_index >= t->wscale.size()) return DNRP_EINVAL;
        auto it = ctx->netid.find(d.network_id);
        if (it == ctx->netid.end()) return DNRP_ENETID;
        if ((err = ensure_seq(ctx, *it->second, d.network_id, t->q.G)) != DNRP_OK) return err;
        pk[i].pdc_seq = (d.plcf_type == 1 ? it->second->t1 : it->second->t2).as<uint8_t>();
        pk[i].codebook = d.codebook_index;
        // tx.cpp:582-594: standard W scaling, or the dynamic-range optimised one
        const float sc = d.DAC_scale * (d.optimal_scaling_DAC ? t->wscale_opt[d.codebook_index] : t->wscale[d.codebook_index]);
        pk[i].scale_stf = 1.0f / std::sqrt(static_cast<float>(t->q.N_b_OCC / 4)) * sc;
        pk[i].scale_df = 1.0f / std::sqrt(static_cast<float>(t->q.N_b_OCC)) * sc;
        pk[i].ph0 = phasor_arg(d.iq_phase_rad);
        pk[i].inc = phasor_arg(d.iq_phase_increment_s2s_post_resampling_rad);
        pk[i].do_mix = (pk[i].ph0 != 0.0 || pk[i].inc != 0.0) ? 1u : 0u;
    }
    hipStream_t st = static_cast<hipStream_t>(stream);
    if (!ctx->tx_pk.ensure(sizeof(dev::tx_pkt) * ctx->cfg.max_batch)) return DNRP_ENOMEM;
    HIPCHK(ctx->tx_pk.wait_idle(st));
    HIPCHK(hipMemcpyAsync(ctx->tx_pk.p, pk, sizeof(dev::tx_pkt) * n, hipMemcpyHostToDevice, st));
    HIPCHK(hipEventRecord(ctx->st_tx.ev, st));
    dev::tx_args a{};
    a.plan = t->plan;
    a.N_occ = t->q.N_b_OCC;
    a.off_lower = t->dm.off_lower;
    a.CP = t->dm.CP;
    a.STF_CP = t->dm.STF_CP;
    a.N_DF = t->q.N_DF_symb;
    a.N_TS = t->tm.N_TS;
    a.N_TX = t->tm.N_TX;
    a.N_SS = t->tm.N_SS;
    a.N_bps = t->q.N_bps;
    a.txdiv = t->tm.txdiv;
    fill_pairs(t->tm.N_TS, a.pair, a.mod);
    a.pattern_len = t->dm.pattern_len;
    a.L = t->rs.L;
    a.M = t->rs.M;
    a.delay = t->rs.delay;
    a.hl = t->rs.hl;
    a.n_keep = std::min(t->dm.N_no_GI_rs, S);
    a.S = S;
    a.pdc_stride = pdc_stride;
    a.G = t->q.G;
    // symbol runs (tx.hip): K symbols per WG plus the preceding symbol as resampler history
    // wave path (one wavefront per symbol slot): K = 6 symbols + history per 7-wave workgroup
    // (C4, 4096 slots per launch: K=3 12.3 ms, K=4 16.6, K=5 15.2, K=6 11.4, K=7 15.9 — LDS sets
    // 4 / 2 / 2 / 2 / 1 workgroups per CU); block path K = 3.
    const bool wave = t->dm.Nd == 1024;
    const uint32_t K = wave ? 6u : 3u;
    a.K = K;
    a.n_runs = (t->q.N_DF_symb + 1 + K - 1) / K;
    a.m_star = 0;
    while ((t->rs.delay + a.m_star * t->rs.M) % t->rs.L) ++a.m_star;
    a.p_star = (t->rs.delay + a.m_star * t->rs.M) / t->rs.L;
    a.HP = 2 * (t->rs.hl + t->rs.M + 1);
    {
        const uint32_t len0 = t->dm.STF_CP + t->dm.Nd, lenD = t->dm.CP + t->dm.Nd;
        auto bsym = [&](uint32_t l) { return l == 0 ? 0u : len0 + (l - 1) * lenD; };
        const uint32_t bpc = t->tm.N_SS * t->q.N_bps;
        uint32_t mx = 0, span = 0;
        for (uint32_t r = 0; r < a.n_runs; ++r) {
            const uint32_t lf = r * K, ll = std::min(lf + K, t->q.N_DF_symb + 1) - 1, s0 = std::max(lf, 1u) - 1;
            span = std::max(span, bsym(ll + 1) - bsym(s0));
            const uint64_t b0 = (uint64_t(t->pdc_off_h[std::max(s0, 1u)]) * bpc) >> 3;
            const uint64_t b1 = ((uint64_t(t->pdc_off_h[ll + 1]) * bpc + 7) >> 3) + 1;
            if (b1 > b0) mx = std::max<uint32_t>(mx, static_cast<uint32_t>(b1 - b0));
        }
        a.stage_bytes = mx <= 8192 ? (mx + 3) / 4 * 4 : 0;
        a.lin_len = std::max(2 * a.HP + span, (K + 1) * t->dm.Nd);
        // output staging reuses bufB + twiddles + constellation: size bufB for the longest run
        const uint32_t max_out = static_cast<uint32_t>((uint64_t(span + t->rs.hl) * t->rs.L + t->rs.M - 1) / t->rs.M) + t->rs.L;
        a.bufB_len = std::max((K + 1) * t->dm.Nd, max_out > t->dm.Nd + 256 ? max_out - t->dm.Nd - 256 : 0u);
    }
    if (t->dm.Nd > 1024) {
        // beyond the block path's registers (tx_kernel stages <= 4 bins per thread): the symbols go
        // through a DECT-rate scratch (tx.hip tx_big_sym_kernel), e.g. u < u_max at b_max = 16
        const uint64_t total = uint64_t(t->dm.STF_CP) + uint64_t(t->q.N_DF_symb) * t->dm.CP + uint64_t(t->q.N_DF_symb + 1) * t->dm.Nd;
        a.big_len = static_cast<uint32_t>((total + 3) / 4 * 4);
        // the scratch is capped at 4 GiB: larger batches run in passes of big_batch packets (tx.hip);
        // DNRP_TX_BIG_CAP (bytes, read per call) lowers the cap so a test can force several passes
        const uint64_t row_bytes = sizeof(float) * 2 * uint64_t(a.big_len) * t->tm.N_TX;
        uint64_t cap = uint64_t(4) << 30;
        if (const char* e = std::getenv("DNRP_TX_BIG_CAP")) cap = std::min<uint64_t>(cap, std::strtoull(e, nullptr, 10));
        a.big_batch = static_cast<uint32_t>(std::max<uint64_t>(1, std::min<uint64_t>(n, cap / row_bytes)));
        if (!ctx->tx_big.ensure(row_bytes * a.big_batch)) return DNRP_ENOMEM;
        HIPCHK(ctx->tx_big.wait_idle(st));
        a.big = ctx->tx_big.as<float2>();
        a.stage_bytes = 0;
    }
    a.code = t->code.as<uint32_t>();
    a.pdc_off = t->pdc_off.as<uint32_t>();
    a.stf = t->stf.as<float2>();
    a.W = t->W.as<float2>();
    a.taps = t->taps.as<float>();
    a.taps_pp = t->taps_pp.as<float>();
    a.npp = t->npp;
    a.tw = t->tw.as<float2>();
    a.qam = t->qam.as<float2>();
    a.qpsk = t->qpsk.as<float2>();
    a.pcc_seq = ctx->pcc_seq.as<uint8_t>();
    a.pcc_d = pcc_d;
    a.pdc_d = pdc_d;
    a.out = iq_out;
    a.pk = ctx->tx_pk.as<dev::tx_pkt>();
    // streaming kernel (tx.hip tx_stream_kernel) where its geometry holds
    a.stream = 0;
    if (wave && t->code_bin.p && dev::tx_stream_taps_match(t->rs.h.data(), t->rs.h.size()) && a.L == 10 && a.M == 9 && a.hl == 22 && a.CP == 128 && a.STF_CP == 1280 &&
        a.pattern_len * 9 == a.STF_CP + 1024 && S % 2 == 0 && (reinterpret_cast<uintptr_t>(iq_out) & 15u) == 0) {
        // every symbol's PDC bytes (SFBC partners included) within its staging window: 1 KiB, spatial
        // multiplexing 4 KiB (tx.hip TXS_SBW_SM: its first KiB prefetched, the rest loaded per symbol)
        const uint32_t bpc = t->tm.N_SS * t->q.N_bps;
        const bool sm = t->tm.N_TS > 1 && !t->tm.txdiv;
        uint64_t span = 0;
        for (uint32_t l = 1; l <= t->q.N_DF_symb; ++l) {
            const uint64_t j0 = t->pdc_off_h[l] & ~1u, j1 = (uint64_t(t->pdc_off_h[l + 1]) + 1) & ~1ull;
            const uint64_t ab = ((j0 * bpc) >> 3) & ~15ull, hi = ((j1 * bpc + 7) >> 3) + 1;
            span = std::max(span, hi - ab);
        }
        const bool fits = span <= (sm ? 4096u : 1024u);
        a.sb_chunks = static_cast<uint32_t>((span + 1023) / 1024);
        const int qlo0 = -static_cast<int>((a.p_star + 8) / 9);
        const int64_t mfirst0 = int64_t(a.m_star) + 10 * qlo0;
        if (fits) {
            a.stream = 1;
            // polyphase blocks on the matrix cores (tx.hip, polyphase.hpp mf_blocks): opt-in A/B,
            // DNRP_TX_MFMA=1 (read per call); the VALU blocks measured faster (docs/DESIGN_LOG.md)
            const char* mf_env = std::getenv("DNRP_TX_MFMA");
            a.mfma = mf_env ? static_cast<uint32_t>(std::min(2, std::max(0, std::atoi(mf_env)))) : 0u;  // 2: f32 MFMA
            a.code_bin = t->code_bin.as<uint32_t>();
            a.onehot = t->tm.N_TS > 1 && t->code_oh.p ? 1u : 0u;  // transmit diversity or spatial multiplexing
            for (uint32_t i = 0; i < n && a.onehot; ++i)
                a.onehot = t->w_onehot[desc[i].codebook_index] ? 1u : 0u;
            a.code_oh = t->code_oh.as<uint32_t>();
            a.pcc_syms = t->pcc_syms;
            a.n_pieces = static_cast<uint32_t>((int64_t(a.n_keep) - mfirst0 + 1279) / 1280);
            // enough wavefronts for ~8 rounds of 16 per CU; each extra segment costs one history FFT
            const uint64_t per = uint64_t(n) * a.N_TX;
            uint32_t ns = static_cast<uint32_t>(std::min<uint64_t>((32768 + per - 1) / per, std::max(1u, a.n_pieces / 8)));
            a.n_seg = std::max(1u, ns);
            a.piece_per_seg = (a.n_pieces + a.n_seg - 1) / a.n_seg;
            a.n_seg = (a.n_pieces + a.piece_per_seg - 1) / a.piece_per_seg;
        }
    }
    ctx->tic("tx", st);
    if (dev::launch_tx(a, n, st) != hipSuccess) return DNRP_EDEVICE;
    ctx->toc("tx", st);
    HIPCHK(ctx->tx_pk.mark_busy(st));
    if (a.big) HIPCHK(ctx->tx_big.mark_busy(st));
    return DNRP_OK;
}

int dnrp_rx_pcc_batch(dnrp_ctx* ctx, uint32_t n, const dnrp_sync_report* sr, const float* iq_in, uint32_t n_windows,
                      uint32_t S_in, int16_t* pcc_llr, dnrp_pcc_report* rep, void* stream) {
    if (!ctx || (n > 0 && (!sr || !iq_in || !pcc_llr))) return DNRP_EINVAL;
    ctx->rx_valid = false;
    if (n == 0) return DNRP_OK;
    if (n > ctx->cfg.max_batch) return DNRP_ENOMEM;
    (void)hipSetDevice(ctx->cfg.device);
    // packets grouped by (u, b, N_eff_TX) of their sync report: one launch set per group, each
    // packet processed exactly as an independent demoddecod_rx_pcc call (rx_synced.cpp:186-323)
    std::map<std::tuple<uint32_t, uint32_t, uint32_t>, std::vector<uint32_t>> groups;
    for (uint32_t i = 0; i < n; ++i) {
        if (sr[i].fine_peak_time >= static_cast<int64_t>(S_in) || sr[i].fine_peak_time <= -static_cast<int64_t>(S_in))
            return DNRP_EINVAL;
        if (sr[i].window >= n_windows) return DNRP_EINVAL;  // the kernels read iq_in + window * N_RX * S_in
        groups[std::make_tuple(sr[i].u, sr[i].b, sr[i].N_eff_TX)].push_back(i);
    }
    int err = DNRP_OK;
    const uint64_t dect = uint64_t(S_in) * ctx->cfg.M / ctx->cfg.L;  // DECT-rate samples in the window
    std::vector<std::pair<rx1_tables*, const std::vector<uint32_t>*>> gl;
    uint32_t cap_max = 0, nf_max = 0;
    ctx->rx_slot_t.assign(n, nullptr);
    ctx->rx_slot_cap.assign(n, 0);
    for (const auto& g : groups) {
        rx1_tables* t = get_rx1(ctx, std::get<0>(g.first), std::get<1>(g.first), std::get<2>(g.first), &err);
        if (!t) return err;
        // symbols that fit into the window: (S_in * M/L - STF) / symbol
        const uint64_t n_stf = t->STF_CP + t->Nd;
        if (dect < n_stf + t->CP + t->Nd) return DNRP_EINVAL;
        const uint32_t cap = static_cast<uint32_t>((dect - n_stf) / (t->CP + t->Nd));
        if (cap < t->pcc_max) return DNRP_EINVAL;
        cap_max = std::max(cap_max, cap);
        nf_max = std::max(nf_max, (t->N_occ + 1 + 63) / 64 * 64);
        for (uint32_t i : g.second) {
            ctx->rx_slot_t[i] = t;
            ctx->rx_slot_cap[i] = cap;
        }
        gl.emplace_back(t, &g.second);
    }
    hipStream_t st = static_cast<hipStream_t>(stream);
    ctx->rx_nsym_cap = cap_max;
    ctx->rx_Nf_pad = nf_max;
    ctx->rx_S_in = S_in;
    ctx->rx_n = n;
    ctx->rx_iq = iq_in;
    ctx->rx_n_windows = n_windows;
    const size_t ybytes = size_t(n) * ctx->cfg.N_TX_max * (ctx->rx_nsym_cap + 1) * ctx->rx_Nf_pad * sizeof(float2);
    const size_t pbytes = size_t(n) * (ctx->rx_nsym_cap + 1) * ctx->cfg.N_TX_max * 8 * sizeof(double2);
    if (!ctx->Y.ensure(ybytes) || !ctx->snr_part.ensure(pbytes) || !ctx->rx_in.ensure(sizeof(dev::rx_pkt_in) * ctx->cfg.max_batch) ||
        !ctx->rx_st.ensure(sizeof(dev::rx_pkt_state) * ctx->cfg.max_batch) ||
        !ctx->rx_sel.ensure(2 * sizeof(uint32_t) * ctx->cfg.max_batch) ||
        !ctx->stf_part.ensure(size_t(ctx->cfg.max_batch) * 8 * (sizeof(double2) + sizeof(float) + 14 * ctx->cfg.b_max * sizeof(float2))))
        return DNRP_ENOMEM;
    {
        // A/B switches, read once per PCC call so that its PDC call agrees with it:
        // DNRP_RX_SNR_FRONT=0 -> rx_snr gathers the DRS cells from Y (no front-end sums, no pilots,
        // so no fused receiver); DNRP_RX_FUSED=1 -> the PDC phase through the fused receiver
        // (rx_fused.hip) instead of Y and rx_cells: parity-tested, slower on MI355X (docs/DESIGN_LOG.md §6)
        const char* e = std::getenv("DNRP_RX_SNR_FRONT");
        ctx->rx_snr_front = !e || std::atoi(e);
        const char* f = std::getenv("DNRP_RX_FUSED");
        ctx->rx_fused = ctx->rx_snr_front && f && std::atoi(f);
        // DNRP_RX_EPOCH: the PDC phase through the epoch receiver (rx_epoch.hip) -- 1 (default) with 4 or
        // more RX antennas, where it measured faster (C4: 1.2 ms per 16384-slot chunk; SISO C3 loses,
        // 7.2 vs 5.5 ms per 8192: one symbol task per wave and epoch), 2 for every geometry it supports,
        // 0 never (Y + rx_cells); DESIGN.md §6
        const char* ep = std::getenv("DNRP_RX_EPOCH");
        ctx->rx_epoch = ep ? static_cast<uint32_t>(std::atoi(ep)) : 1u;
        const char* gr = std::getenv("DNRP_RX_GROUP");
        ctx->rx_group = gr ? static_cast<uint32_t>(std::atoi(gr)) : 0u;
        // zero-forced DRS pilots of every slot (the fused receiver's only): at most one DRS symbol per
        // 5 symbols (N_eff_TX <= 4) plus the zero op
        ctx->zd_row = 14 * ctx->cfg.b_max;
        ctx->zd_dops = std::min<uint32_t>(dev::RX_MAX_DOPS, (cap_max + 4) / 5 + 2) + 1;
        const size_t zbytes = size_t(n) * ctx->zd_dops * ctx->cfg.N_TX_max * 4 * ctx->zd_row * sizeof(float2);
        if (ctx->rx_fused) {
            if (!ctx->zd.ensure(zbytes)) return DNRP_ENOMEM;
            // the size is part of the key: a reallocation can return the same base address
            const auto key = std::make_tuple(ctx->zd.p, ctx->zd.n, ctx->zd_dops, ctx->zd_row, ctx->cfg.N_TX_max);
            if (key != ctx->zd_key) {  // a new layout: the zero op of every slot (and all else) zeroed once
                HIPCHK(hipMemsetAsync(ctx->zd.p, 0, ctx->zd.n, st));
                ctx->zd_key = key;
            }
        }
    }
    auto* pin = static_cast<dev::rx_pkt_in*>(ctx->st_rxin.get(sizeof(dev::rx_pkt_in) * n));
    auto* sel = static_cast<uint32_t*>(ctx->st_sel.get(2 * sizeof(uint32_t) * n));
    if (!pin || !sel) return DNRP_ENOMEM;
    for (uint32_t i = 0; i < n; ++i) {
        pin[i].fine_peak = sr[i].fine_peak_time;
        pin[i].cfo_rad = sr[i].cfo_fractional_rad + sr[i].cfo_integer_rad;
        pin[i].inc0 = phasor_arg(pin[i].cfo_rad);
        pin[i].win = sr[i].window;
    }
    {
        uint32_t o = 0;
        for (const auto& g : gl)
            for (uint32_t i : *g.second) {
                sel[2 * o] = i;
                sel[2 * o + 1] = i;  // PCC LLR row = slot
                ++o;
            }
    }
    HIPCHK(hipMemcpyAsync(ctx->rx_in.p, pin, sizeof(dev::rx_pkt_in) * n, hipMemcpyHostToDevice, st));
    HIPCHK(hipEventRecord(ctx->st_rxin.ev, st));
    HIPCHK(hipMemcpyAsync(ctx->rx_sel.p, sel, 2 * sizeof(uint32_t) * n, hipMemcpyHostToDevice, st));
    HIPCHK(hipEventRecord(ctx->st_sel.ev, st));
    uint32_t off = 0;
    for (const auto& g : gl) {
        rx1_tables* t = g.first;
        const uint32_t ng = static_cast<uint32_t>(g.second->size());
        const uint32_t* gsel = ctx->rx_sel.as<uint32_t>() + 2 * off;
        off += ng;
        auto fa = front_args(ctx, t, iq_in, gsel, snr_from_front(ctx, t) ? &t->bplan : nullptr);
        ctx->tic("rx_stf", st);
        if (dev::launch_rx_stf(fa, ng, st) != hipSuccess) return DNRP_EDEVICE;
        ctx->toc("rx_stf", st);
        fa.sym_first = 1;
        fa.sym_count = t->pcc_max;
        ctx->tic("rx_fft_pcc", st);
        if (dev::launch_rx_fft(fa, ng, st) != hipSuccess) return DNRP_EDEVICE;
        ctx->toc("rx_fft_pcc", st);
        if ((err = launch_back(ctx, t, t->bplan, ng, gsel, false, 2, t->pcc_k.as<uint32_t>(), t->pcc_sym.as<uint16_t>(), pcc_llr, 196,
                               st)) != DNRP_OK)
            return err;
    }
    ctx->rx_valid = true;
    if (rep) {
        std::vector<dev::rx_pkt_state> S(n);
        HIPCHK(hipMemcpyAsync(S.data(), ctx->rx_st.p, sizeof(dev::rx_pkt_state) * n, hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
        for (uint32_t i = 0; i < n; ++i) {
            rep[i].snr_dB = S[i].snr_pcc;
            rep[i].cfo_fractional_rad = sr[i].cfo_fractional_rad + (S[i].cfo_fine - pin[i].cfo_rad);
            rep[i].sto_fractional = S[i].sto_frac;
            // run_stf_rms_estimation (rx_synced.cpp:620-655): sync's RMS kept where it is > 0
            for (int a = 0; a < 8; ++a)
                rep[i].rms[a] = (prm::RX_RMS_KEEP_SYNC && sr[i].rms[a] > 0.0f) ? sr[i].rms[a] : S[i].rms[a];
        }
    }
    return DNRP_OK;
}

int dnrp_rx_pdc_batch(dnrp_ctx* ctx, uint32_t m, const dnrp_pdc_req* req, const float* iq_in, uint32_t n_windows,
                      uint32_t S_in, int16_t* pdc_llr, uint32_t llr_stride, dnrp_pdc_report* rep, void* stream) {
    if (!ctx || (m > 0 && (!req || !iq_in || !pdc_llr))) return DNRP_EINVAL;
    // no packet continues with its PDC: nothing to enqueue, whatever the PCC call before (an empty
    // chunk enqueues no job either, worker_sync.cpp:170-190)
    if (m == 0) return DNRP_OK;
    if (!ctx->rx_valid) return DNRP_ESTATE;
    // the PDC symbols are read from the PCC call's windows (the state it kept points into them)
    if (iq_in != ctx->rx_iq || n_windows != ctx->rx_n_windows) return DNRP_ESTATE;
    if (m > ctx->rx_n || S_in != ctx->rx_S_in) return DNRP_EINVAL;
    (void)hipSetDevice(ctx->cfg.device);
    int err = DNRP_OK;
    // requests grouped by (PCC-phase tables, PLCF-announced psdef) (rx_synced.cpp:325-436 per packet)
    using key_t = std::tuple<rx1_tables*, uint32_t, uint32_t, uint32_t, uint32_t, uint32_t, uint32_t, uint32_t>;
    std::map<key_t, std::vector<uint32_t>> groups;
    std::vector<uint8_t> seen(ctx->rx_n, 0);
    for (uint32_t r = 0; r < m; ++r) {
        const auto& q = req[r];
        if (q.pcc_index >= ctx->rx_n || seen[q.pcc_index]) return DNRP_EINVAL;
        seen[q.pcc_index] = 1;
        if (q.plcf_type != 1 && q.plcf_type != 2) return DNRP_EINVAL;
        const auto& d = q.psdef;
        groups[key_t(ctx->rx_slot_t[q.pcc_index], d.u, d.b, d.PacketLengthType, d.PacketLength, d.tm_mode_index,
                     d.mcs_index, d.Z)]
            .push_back(r);
    }
    hipStream_t st = static_cast<hipStream_t>(stream);
    if (!ctx->pdc_seq_ptrs.ensure(sizeof(void*) * ctx->cfg.max_batch) ||
        !ctx->rx_sel2.ensure(2 * sizeof(uint32_t) * ctx->cfg.max_batch))
        return DNRP_ENOMEM;
    auto** seqp = static_cast<const uint8_t**>(ctx->st_seq.get(sizeof(void*) * m));
    auto* sel = static_cast<uint32_t*>(ctx->st_sel2.get(2 * sizeof(uint32_t) * m));
    if (!seqp || !sel) return DNRP_ENOMEM;
    std::vector<std::pair<rx2_tables*, const std::vector<uint32_t>*>> gl;
    uint32_t o = 0;
    for (const auto& g : groups) {
        rx1_tables* t = std::get<0>(g.first);
        const dnrp_psdef& d = req[g.second.front()].psdef;
        rx2_tables* t2 = get_rx2(ctx, d, &err);
        if (!t2) return err;
        if (d.u != t->u || d.b != t->b || t2->q.N_eff_TX != t->N_eff_TX) return DNRP_EINVAL;
        if (llr_stride < t2->q.G) return DNRP_EINVAL;
        for (uint32_t r : g.second) {
            if (t2->q.N_DF_symb > ctx->rx_slot_cap[req[r].pcc_index]) return DNRP_EINVAL;
            auto it = ctx->netid.find(req[r].network_id);
            if (it == ctx->netid.end()) return DNRP_ENETID;
            if ((err = ensure_seq(ctx, *it->second, req[r].network_id, t2->q.G)) != DNRP_OK) return err;
            seqp[r] = (req[r].plcf_type == 1 ? it->second->t1 : it->second->t2).as<uint8_t>();
            sel[2 * o] = req[r].pcc_index;
            sel[2 * o + 1] = r;
            ++o;
        }
        gl.emplace_back(t2, &g.second);
    }
    HIPCHK(hipMemcpyAsync(ctx->pdc_seq_ptrs.p, seqp, sizeof(void*) * m, hipMemcpyHostToDevice, st));
    HIPCHK(hipEventRecord(ctx->st_seq.ev, st));
    HIPCHK(hipMemcpyAsync(ctx->rx_sel2.p, sel, 2 * sizeof(uint32_t) * m, hipMemcpyHostToDevice, st));
    HIPCHK(hipEventRecord(ctx->st_sel2.ev, st));
    if (rep && !ctx->mimo_out.ensure(size_t(ctx->cfg.max_batch) * 3 * sizeof(uint32_t))) return DNRP_ENOMEM;
    uint32_t off = 0;
    size_t gi = 0;
    for (const auto& g : groups) {
        rx1_tables* t = std::get<0>(g.first);
        rx2_tables* t2 = gl[gi++].first;
        const uint32_t ng = static_cast<uint32_t>(g.second.size());
        const uint32_t* gsel = ctx->rx_sel2.as<uint32_t>() + 2 * off;
        off += ng;
        auto fa = front_args(ctx, t, iq_in, gsel, snr_from_front(ctx, t) ? &t2->bplan : nullptr);
        // fused receiver (kernels/rx_fused.hip): the front end's pilots in zd, the compile-time-tap
        // wave front end, an instantiated (N_RX, N_eff_TX) pair
        const bool fused = ctx->rx_fused && t2->fused_ok && fa.zd && fa.stream && dev::rx_fft_wave_path(fa) &&
                           dev::rx_fused_supported(fa.N_RX, t->N_eff_TX);
        if (fused) {
            // the phase's DRS symbols first (pilots, SNR sums; their bins to Y only where they carry
            // PDC cells), then the SNR chain / LUT picks, then one fused launch for every PDC symbol
            fa.sym_first = 0;
            fa.sym_list = t2->drs_syms.as<uint16_t>();
            fa.sym_count = t2->n_drs_syms;
            fa.no_y = t2->drs_y ? 0u : 1u;
            if (fa.sym_count) {
                ctx->tic("rx_fft_pdc", st);
                if (dev::launch_rx_fft(fa, ng, st) != hipSuccess) return DNRP_EDEVICE;
                ctx->toc("rx_fft_pdc", st);
            }
            if ((err = launch_back(ctx, t, t2->bplan, ng, gsel, true, t2->q.N_bps, nullptr, nullptr, pdc_llr,
                                   llr_stride, st, false, false)) != DNRP_OK)
                return err;
            dev::rx_fused_args x{};
            x.F = fa;
            x.F.sym_list = nullptr;
            x.n_pkt = ng;
            x.n_fsym = t2->n_fsym;
            x.NT = t->N_eff_TX;
            x.N_bps = t2->q.N_bps;
            {
                uint32_t pr[12];
                fill_pairs(t->N_eff_TX, pr, x.mod);
                for (uint32_t i = 0; i < x.mod && i < 8; ++i) x.pair_bits |= uint64_t(pr[i] & 0xFFu) << (8 * i);
            }
            x.fsym = t2->fsym.as<dev::rx_fsym>();
            x.kk = t2->pdc_k.as<uint32_t>();
            x.luts = t->luts.as<dev::rx_lut>();
            x.lut_d = ctx->lut_d.as<uint8_t>();
            x.pdc_seq = static_cast<const uint8_t* const*>(ctx->pdc_seq_ptrs.p);
            x.llr = pdc_llr;
            x.llr_stride = llr_stride;
            ctx->tic("rx_fused", st);
            if (dev::launch_rx_fused(x, st) != hipSuccess) return DNRP_EDEVICE;
            ctx->toc("rx_fused", st);
        } else {
            fa.zd = nullptr;  // no reader
            fa.sym_first = t->pcc_max + 1;
            const uint32_t G = ctx->rx_group;
            dev::rx_cells_args ec{};
            const bool epoch = (ctx->rx_epoch >= 2 || (ctx->rx_epoch == 1 && fa.N_RX >= 4)) && t2->ep_ok && !t2->sm &&
                               fa.stream && dev::rx_fft_wave_path(fa) &&
                               t2->bplan.cells_ok && t2->bplan.n_epochs &&
                               dev::rx_epoch_supported(fa.N_RX, t->N_eff_TX) &&
                               dev::rx_epoch_lds(ec = cells_args(ctx, t, t2->bplan, ng, gsel, true, t2->q.N_bps,
                                                                 t2->pdc_k.as<uint32_t>(), t2->pdc_sym.as<uint16_t>(),
                                                                 pdc_llr, llr_stride, false)) <= 160 * 1024;
            if (epoch) {
                // DRS pass (the phase's DRS symbols: pilots in Y, SNR sums), the SNR chain's LUT picks,
                // then one workgroup per (packet, epoch): front end of the epoch's symbols + equaliser
                if (t2->n_ep_drs) {
                    auto fd = fa;
                    fd.sym_first = 0;
                    fd.sym_list = t2->ep_drs.as<uint16_t>();
                    fd.sym_count = t2->n_ep_drs;
                    ctx->tic("rx_fft_pdc", st);
                    if (dev::launch_rx_fft(fd, ng, st) != hipSuccess) return DNRP_EDEVICE;
                    ctx->toc("rx_fft_pdc", st);
                }
                if ((err = launch_back(ctx, t, t2->bplan, ng, gsel, true, t2->q.N_bps, nullptr, nullptr, pdc_llr,
                                       llr_stride, st, false, false)) != DNRP_OK)
                    return err;
                dev::rx_epoch_args x{};
                x.F = fa;
                x.C = ec;
                x.ep_off = t2->ep_off.as<uint16_t>();
                x.ep_sym = t2->ep_sym.as<uint16_t>();
                ctx->tic("rx_epoch", st);
                if (dev::launch_rx_epoch(x, ng, st) != hipSuccess) return DNRP_EDEVICE;
                ctx->toc("rx_epoch", st);
            } else if (G && ng > G && t2->q.N_DF_symb > t->pcc_max && fa.stream && dev::rx_fft_wave_path(fa)) {
                // packet groups: front end of group g on st, back end of group g on rx_aux once that
                // front end is done, so group g+1's front end runs beside group g's back end and the
                // back end reads Y (plain stores) while it is still in the L2 / Infinity Cache
                if (!ctx->rx_aux) {
                    HIPCHK(hipStreamCreateWithFlags(&ctx->rx_aux, hipStreamNonBlocking));
                    HIPCHK(hipEventCreateWithFlags(&ctx->rx_fork, hipEventDisableTiming));
                    HIPCHK(hipEventCreateWithFlags(&ctx->rx_join, hipEventDisableTiming));
                }
                fa.sym_count = t2->q.N_DF_symb - t->pcc_max;
                fa.y_plain = 1;
                ctx->tic("rx_pdc_phase", st);  // both streams' launches of the phase, fork to join
                for (uint32_t g0 = 0; g0 < ng; g0 += G) {
                    const uint32_t gn = std::min(G, ng - g0);
                    auto fg = fa;
                    fg.sel = gsel + 2 * g0;
                    ctx->tic("rx_fft_pdc", st);
                    if (dev::launch_rx_fft(fg, gn, st) != hipSuccess) return DNRP_EDEVICE;
                    ctx->toc("rx_fft_pdc", st);
                    HIPCHK(hipEventRecord(ctx->rx_fork, st));
                    HIPCHK(hipStreamWaitEvent(ctx->rx_aux, ctx->rx_fork, 0));
                    if ((err = launch_back(ctx, t, t2->bplan, gn, gsel + 2 * g0, true, t2->q.N_bps, t2->pdc_k.as<uint32_t>(),
                                           t2->pdc_sym.as<uint16_t>(), pdc_llr, llr_stride, ctx->rx_aux, t2->sm)) != DNRP_OK)
                        return err;
                }
                HIPCHK(hipEventRecord(ctx->rx_join, ctx->rx_aux));
                HIPCHK(hipStreamWaitEvent(st, ctx->rx_join, 0));
                ctx->toc("rx_pdc_phase", st);
            } else {
                if (t2->q.N_DF_symb > t->pcc_max) {
                    fa.sym_count = t2->q.N_DF_symb - t->pcc_max;
                    ctx->tic("rx_fft_pdc", st);
                    if (dev::launch_rx_fft(fa, ng, st) != hipSuccess) return DNRP_EDEVICE;
                    ctx->toc("rx_fft_pdc", st);
                }
                if ((err = launch_back(ctx, t, t2->bplan, ng, gsel, true, t2->q.N_bps, t2->pdc_k.as<uint32_t>(),
                                       t2->pdc_sym.as<uint16_t>(), pdc_llr, llr_stride, st, t2->sm)) != DNRP_OK)
                    return err;
            }
        }
        if (rep) {
            // MIMO report at the packet end (rx_synced.cpp:417-436; the reference runs it after a
            // successful CRC, which is the caller's decision here)
            dev::rx_mimo_args ma{};
            ma.N_RX = ctx->cfg.N_TX_max;
            ma.N_TS = t2->N_TS;
            ma.Nf_pad = ctx->rx_Nf_pad;
            ma.n_sym_total = ctx->rx_nsym_cap + 1;
            ma.ncb_tx = t2->ncb_tx;
            ma.A_tx = t2->A_tx;
            ma.ncb_rx = t2->ncb_rx;
            ma.A_rx = t2->A_rx;
            ma.cells = t2->mimo_cells.as<uint32_t>();
            ma.signs = t2->mimo_signs.as<float>();
            ma.Wtx = t2->Wtx.as<float2>();
            ma.stx = t2->stx.as<float>();
            ma.Wrx = t2->Wrx.as<float2>();
            ma.srx = t2->srx.as<float>();
            ma.Y = ctx->Y.as<float2>();
            ma.out = ctx->mimo_out.as<uint32_t>();
            ma.sel = gsel;
            if (fused) {  // the DRS bins of this phase are not in Y: the pilots hold the same values
                ma.zd = fa.zd;
                ma.zcells = t2->mimo_zcells.as<uint32_t>();
                ma.zd_dops = fa.zd_dops;
                ma.zd_row = fa.zd_row;
            }
            if (dev::launch_rx_mimo(ma, ng, st) != hipSuccess) return DNRP_EDEVICE;
        }
    }
    if (rep) {
        std::vector<dev::rx_pkt_state> S(ctx->rx_n);
        std::vector<uint32_t> mo(3 * size_t(m));
        HIPCHK(hipMemcpyAsync(S.data(), ctx->rx_st.p, sizeof(dev::rx_pkt_state) * ctx->rx_n, hipMemcpyDeviceToHost, st));
        HIPCHK(hipMemcpyAsync(mo.data(), ctx->mimo_out.p, mo.size() * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
        for (uint32_t r = 0; r < m; ++r) {
            rep[r].snr_dB = S[req[r].pcc_index].snr_pdc;
            rep[r].mimo_N_RX = ctx->cfg.N_TX_max;
            rep[r].mimo_N_TS_other = mo[3 * r];
            rep[r].tm_3_7_beamforming_idx = mo[3 * r + 1];
            rep[r].tm_3_7_beamforming_reciprocal_idx = mo[3 * r + 2];
        }
    }
    return DNRP_OK;
}

int dnrp_ctx_set_rx_mode(dnrp_ctx* ctx, uint32_t flags) {
    if (!ctx || (flags & ~uint32_t(DNRP_RX_MODE_SM_MMSE))) return DNRP_EINVAL;
    if (flags != ctx->rx_mode) ctx->rx2t.clear();  // PDC tables depend on the mode
    ctx->rx_mode = flags;
    ctx->rx_valid = false;
    return DNRP_OK;
}

int dnrp_sync(dnrp_ctx* ctx, void* stream) {
    if (!ctx) return DNRP_EINVAL;
    return hipStreamSynchronize(static_cast<hipStream_t>(stream)) == hipSuccess ? DNRP_OK : DNRP_EDEVICE;
}

int dnrp_last_kernel_ms(const dnrp_ctx* ctx, const char* name, float* ms) {
    if (!ctx || !name || !ms) return DNRP_EINVAL;
    auto it = ctx->ev.find(name);
    if (it == ctx->ev.end() || it->second.used == 0) return DNRP_EINVAL;
    const auto& p = it->second.ev[it->second.used - 1];
    if (hipEventSynchronize(p.second) != hipSuccess) return DNRP_EDEVICE;
    return hipEventElapsedTime(ms, p.first, p.second) == hipSuccess ? DNRP_OK : DNRP_EDEVICE;
}

int dnrp_kernel_time_total(dnrp_ctx* ctx, const char* name, float* total_ms, uint32_t* count, int reset) {
    if (!ctx || !name || !total_ms || !count) return DNRP_EINVAL;
    *total_ms = 0.0f;
    *count = 0;
    auto it = ctx->ev.find(name);
    if (it == ctx->ev.end()) return DNRP_OK;
    auto& pool = it->second;
    for (size_t i = 0; i < pool.used; ++i) {
        float ms = 0.0f;
        if (hipEventSynchronize(pool.ev[i].second) != hipSuccess) return DNRP_EDEVICE;
        if (hipEventElapsedTime(&ms, pool.ev[i].first, pool.ev[i].second) != hipSuccess) return DNRP_EDEVICE;
        *total_ms += ms;
    }
    *count = static_cast<uint32_t>(pool.used);
    if (reset) pool.used = 0;
    return DNRP_OK;
}

}  // extern "C"
