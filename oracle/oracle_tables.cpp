// ORACLE — TEST INFRASTRUCTURE ONLY (see oracle.hpp header).
// Restatement of the reference's sections_part3 geometry, filter design and channel-estimation
// LUT generation. Each function cites the reference file it follows.
#include <algorithm>
#include <cassert>
#include <cmath>
#include <cstdio>
#include <stdexcept>

#include "oracle.hpp"
#include "oracle_params.hpp"

namespace orc {

// ---------------------------------------------------------------- numerologies.cpp:27-70
numerology_t get_numerology(uint32_t u, uint32_t b) {
    numerology_t q{};
    q.u = u;
    q.b = b;
    q.delta_u_f = u * 27000;
    q.T_u_symb = (64.0 + 8.0) / 64.0 / static_cast<double>(q.delta_u_f);
    q.N_SLOT_u_symb = u * 10;
    q.N_SLOT_u_subslot = u * 2;
    q.N_b_DFT = b * 64;
    q.N_b_CP = b * 8;
    q.N_b_OCC = b * 56;
    q.N_guards_top = (q.N_b_DFT - q.N_b_OCC) / 2 - 1;
    q.N_guards_bottom = q.N_guards_top + 1;
    return q;
}

// ---------------------------------------------------------------- tm_mode.cpp:27-137
tm_mode_t get_tm_mode(uint32_t index) {
    // {N_eff_TX, N_SS, cl, N_TS, N_TX} per Table 7.2-1 of ETSI TS 103 636-3
    static const uint32_t T[12][5] = {{1, 1, 0, 1, 1}, {2, 1, 0, 2, 2}, {2, 2, 0, 2, 2},
                                      {1, 1, 1, 1, 2}, {2, 2, 1, 2, 2}, {4, 1, 0, 4, 4},
                                      {4, 4, 0, 4, 4}, {1, 1, 1, 1, 4}, {2, 2, 1, 2, 4},
                                      {4, 4, 1, 4, 4}, {8, 1, 0, 8, 8}, {8, 8, 0, 8, 8}};
    if (index > 11) throw std::runtime_error("tm_mode undefined");
    tm_mode_t q{};
    q.index = index;
    q.N_eff_TX = T[index][0];
    q.N_SS = T[index][1];
    q.cl = T[index][2] != 0;
    q.N_TS = T[index][3];
    q.N_TX = T[index][4];
    return q;
}

// ---------------------------------------------------------------- mcs.cpp:27-105
mcs_t get_mcs(uint32_t index) {
    static const uint32_t T[12][3] = {{1, 1, 2}, {2, 1, 2}, {2, 3, 4}, {4, 1, 2},
                                      {4, 3, 4}, {6, 2, 3}, {6, 3, 4}, {6, 5, 6},
                                      {8, 3, 4}, {8, 5, 6}, {10, 3, 4}, {10, 5, 6}};
    if (index > 11) throw std::runtime_error("mcs undefined");
    return mcs_t{index, T[index][0], T[index][1], T[index][2]};
}

// ---------------------------------------------------------------- transport_block_size.cpp
uint32_t get_N_TB_bits(uint32_t N_SS, uint32_t N_PDC_subc, uint32_t N_bps, uint32_t Rn,
                       uint32_t Rd, uint32_t Z) {
    const uint32_t G = N_SS * N_PDC_subc * N_bps;
    const uint32_t N_PDC_bits = (G * Rn) / Rd;
    const uint32_t L = 24;
    const uint32_t M = N_PDC_bits <= 512 ? 8 : N_PDC_bits <= 1024 ? 16 : N_PDC_bits <= 2048 ? 32 : 64;
    const uint32_t N_M = (N_PDC_bits / M) * M;
    if (N_M == 0 || N_M <= L) return 0;
    if (N_M <= Z) return N_M - L;
    const uint32_t C = (N_M - L + Z - 1) / Z;
    return N_M - (C + 1) * L;
}

// turbo code internal interleaver sizes, 3GPP TS 36.212 Table 5.1.3-3 (188 entries)
static std::vector<uint32_t> tc_cb_sizes() {
    std::vector<uint32_t> s;
    for (uint32_t k = 40; k <= 512; k += 8) s.push_back(k);
    for (uint32_t k = 528; k <= 1024; k += 16) s.push_back(k);
    for (uint32_t k = 1056; k <= 2048; k += 32) s.push_back(k);
    for (uint32_t k = 2112; k <= 6144; k += 64) s.push_back(k);
    return s;
}

// fix/cbsegm.cpp:56-118 — returns false on error, sets C and filler bits F
static bool cbsegm(uint32_t tbs, uint32_t Z, uint32_t& C, uint32_t& F) {
    static const std::vector<uint32_t> sz = tc_cb_sizes();
    if (tbs == 0) {
        C = 0;
        F = 0;
        return true;
    }
    const uint32_t B = tbs + 24;
    uint32_t Bp;
    if (B <= Z) {
        C = 1;
        Bp = B;
    } else {
        C = (B + (Z - 24) - 1) / (Z - 24);
        Bp = B + 24 * C;
    }
    const uint32_t long_cb = (Bp - 1) / C + 1;
    uint32_t j = 0;
    while (j < sz.size() && sz[j] < long_cb) ++j;
    if (j == sz.size()) return false;
    const uint32_t K1 = sz[j];
    uint32_t K2 = 0, C1, C2;
    if (C == 1) {
        C1 = 1;
        C2 = 0;
    } else {
        if (j == 0) return false;
        K2 = sz[j - 1];
        C2 = (C * K1 - Bp) / (K1 - K2);
        C1 = C - C2;
    }
    F = C1 * K1 + C2 * K2 - Bp;
    return true;
}

static uint32_t get_N_DF_symb(uint32_t u, uint32_t N_PACKET_symb) {  // pdc.cpp:156-166
    return u == 1 ? N_PACKET_symb - 2 : (u == 2 || u == 4) ? N_PACKET_symb - 3 : N_PACKET_symb - 4;
}

static uint32_t nof_drs_symbols_per_ts(uint32_t N_PACKET_symb, uint32_t N_eff_TX) {  // pdc.cpp:168-192
    const uint32_t N_step = N_eff_TX <= 2 ? 5 : 10;
    uint32_t n = N_PACKET_symb / N_step;
    if (N_step == 10 && N_PACKET_symb % 10 != 0) ++n;
    return n;
}

static uint32_t get_N_PDC_subc(uint32_t N_PACKET_symb, uint32_t u, uint32_t N_eff_TX,
                               uint32_t N_b_OCC) {  // pdc.cpp:194-215
    const uint32_t N_DF = get_N_DF_symb(u, N_PACKET_symb);
    const uint32_t N_DRS = N_eff_TX * N_b_OCC / 4 * nof_drs_symbols_per_ts(N_PACKET_symb, N_eff_TX);
    if (N_DF * N_b_OCC <= N_DRS + 98) return 0;
    return N_DF * N_b_OCC - N_DRS - 98;
}

// ---------------------------------------------------------------- packet_sizes.cpp:99-236
bool get_packet_sizes(const psdef_t& d, packet_sizes_t& q) {
    const uint32_t u = d.u, b = d.b;
    const bool u_ok = (u == 1 || u == 2 || u == 4 || u == 8);
    const bool b_ok = (b == 1 || b == 2 || b == 4 || b == 8 || b == 12 || b == 16);
    if (!u_ok || !b_ok || d.PacketLengthType > 1 || d.PacketLength == 0 || d.PacketLength > 16 ||
        d.tm_mode_index > 11 || d.mcs_index > 11 || (d.Z != 2048 && d.Z != 6144))
        return false;
    q = packet_sizes_t{};
    q.psdef = d;
    q.num = get_numerology(u, b);
    q.N_PACKET_symb = d.PacketLengthType == 0
                          ? d.PacketLength * q.num.N_SLOT_u_symb / q.num.N_SLOT_u_subslot
                          : d.PacketLength * q.num.N_SLOT_u_symb;
    if (q.N_PACKET_symb < 5 || q.N_PACKET_symb > 1280 || q.N_PACKET_symb % 5 != 0) return false;
    q.tm = get_tm_mode(d.tm_mode_index);
    if (q.tm.N_eff_TX == 4 && q.N_PACKET_symb < 15) return false;
    if (u == 8 && q.tm.N_eff_TX == 8 && (q.N_PACKET_symb < 20 || q.N_PACKET_symb % 10 != 0))
        return false;
    q.N_PDC_subc = get_N_PDC_subc(q.N_PACKET_symb, u, q.tm.N_eff_TX, q.num.N_b_OCC);
    if (q.N_PDC_subc == 0) return false;
    q.mcs = get_mcs(d.mcs_index);
    q.N_TB_bits = get_N_TB_bits(q.tm.N_SS, q.N_PDC_subc, q.mcs.N_bps, q.mcs.R_num, q.mcs.R_den, d.Z);
    if (q.N_TB_bits == 0) return false;
    q.G = q.tm.N_SS * q.N_PDC_subc * q.mcs.N_bps;
    q.N_PDC_bits = (q.G * q.mcs.R_num) / q.mcs.R_den;
    uint32_t C, F;
    if (!cbsegm(q.N_TB_bits, d.Z, C, F) || F > 0) return false;
    q.C = C;
    q.N_DF_symb = get_N_DF_symb(u, q.N_PACKET_symb);
    q.N_DRS_subc = q.tm.N_eff_TX * q.num.N_b_OCC / 4 *
                   nof_drs_symbols_per_ts(q.N_PACKET_symb, q.tm.N_eff_TX);
    const uint32_t sym = 72 * b;  // transmission_packet_structure.cpp:39-93
    q.N_samples_STF = u == 1 ? sym * 14 / 9 : sym * 2;
    q.N_samples_STF_CP_only = q.N_samples_STF - 64 * b;
    q.N_samples_DF = sym * q.N_DF_symb;
    q.N_samples_GI = u == 1 ? sym * 4 / 9 : (u == 2 || u == 4) ? sym : sym * 2;
    q.N_samples_packet_no_GI = q.N_samples_STF + q.N_samples_DF;
    q.N_samples_packet = q.N_samples_packet_no_GI + q.N_samples_GI;
    return true;
}

// ---------------------------------------------------------------- physical_resources.cpp
std::vector<int> k_b_OCC(uint32_t b) {
    const int N = static_cast<int>(56 * b);
    std::vector<int> k;
    for (int i = -N / 2; i <= -1; ++i) k.push_back(i);
    for (int i = 1; i <= N / 2; ++i) k.push_back(i);
    return k;
}

// ---------------------------------------------------------------- stf.cpp:27-88,185-285
static const int STF_Y_B1[14] = {1, -1, 1, 1, -1, 1, 1, -1, 1, 1, 1, -1, -1, -1};
static const int STF_Y_B2[28] = {-1, 1,  -1, 1, 1,  -1, 1,  1, -1, 1, 1,  1,  -1, 1,
                                 -1, -1, -1, 1, -1, -1, -1, 1, 1,  1, -1, -1, -1, -1};
static const int STF_Y_B4[56] = {-1, -1, -1, 1,  -1, 1,  -1, -1, 1,  1,  1,  1,  -1, 1,
                                 -1, -1, -1, 1,  -1, 1,  1,  -1, -1, -1, -1, -1, 1,  -1,
                                 1,  1,  1,  -1, 1,  -1, 1,  1,  -1, -1, -1, -1, 1,  -1,
                                 -1, -1, -1, 1,  -1, 1,  1,  -1, -1, -1, -1, -1, 1,  -1};

static std::vector<int> flip_pm(const std::vector<int>& in) {  // fliplr then (-1)^k
    std::vector<int> out(in.size());
    for (size_t i = 0; i < in.size(); ++i) out[i] = in[in.size() - 1 - i] * ((i % 2 == 0) ? 1 : -1);
    return out;
}

static std::vector<int> stf_polarity(uint32_t b) {
    std::vector<int> y4(STF_Y_B4, STF_Y_B4 + 56);
    if (b == 1) return std::vector<int>(STF_Y_B1, STF_Y_B1 + 14);
    if (b == 2) return std::vector<int>(STF_Y_B2, STF_Y_B2 + 28);
    if (b == 4) return y4;
    std::vector<int> y8 = y4;
    const auto r4 = flip_pm(y4);
    y8.insert(y8.end(), r4.begin(), r4.end());
    if (b == 8) return y8;
    std::vector<int> y16 = y8;
    const auto r8 = flip_pm(y8);
    y16.insert(y16.end(), r8.begin(), r8.end());
    if (b == 16) return y16;
    // b == 12: 168 values starting at offset 2*14
    return std::vector<int>(y16.begin() + 28, y16.begin() + 28 + 168);
}

std::vector<cd> stf_values(uint32_t b, uint32_t N_eff_TX, double scale) {
    const uint32_t N = 56 * b;
    const auto k = k_b_OCC(b);
    const auto pol = stf_polarity(b);
    uint32_t lg = 0;
    while ((1u << lg) < N_eff_TX) ++lg;
    // stf.cpp computes fac in float: scale * (cos(pi/4), sin(pi/4)) as floats
    const cf fac = cf{static_cast<float>(scale), 0.0f} *
                   cf{static_cast<float>(std::cos(M_PI / 4.0)), static_cast<float>(std::sin(M_PI / 4.0))};
    std::vector<cd> out(N + 1, cd{0.0, 0.0});
    for (uint32_t i = 0; i < N / 4; ++i) {
        const int ki = (i < N / 8) ? k[i * 4] : k[N / 2 + 3 + (i - N / 8) * 4];
        const cf v = cf{static_cast<float>(pol[(i + 2 * lg) % (N / 4)]), 0.0f} * fac;
        out[ki + static_cast<int>(N / 2)] = cd{v.real(), v.imag()};
    }
    return out;
}

// ---------------------------------------------------------------- drs.cpp
static const int DRS_Y_B1[56] = {1,  1,  1,  1,  -1, 1,  1,  -1, -1, 1,  1,  1,  1,  -1,
                                 1,  -1, 1,  1,  -1, 1,  -1, 1,  -1, 1,  1,  1,  1,  1,
                                 -1, 1,  -1, -1, 1,  1,  -1, -1, -1, -1, 1,  -1, -1, -1,
                                 -1, -1, 1,  1,  1,  -1, 1,  1,  -1, -1, 1,  -1, -1, -1};

std::vector<uint32_t> drs_k_i(uint32_t b, uint32_t t, uint32_t n_parity) {
    const uint32_t N = 56 * b;
    const auto k = k_b_OCC(b);
    std::vector<uint32_t> out(N / 4);
    for (uint32_t i = 0; i < N / 4; ++i)
        out[i] = static_cast<uint32_t>(k[i * 4 + (t + (n_parity % 2) * 2) % 4] + static_cast<int>(N / 2));
    return out;
}

std::vector<double> drs_y(uint32_t b, uint32_t t) {
    const uint32_t N = 56 * b;
    std::vector<double> out(N / 4);
    for (uint32_t i = 0; i < N / 4; ++i) {
        const double v = DRS_Y_B1[(4 * i + t % 4) % 56];
        out[i] = t < 4 ? v : -v;
    }
    return out;
}

std::vector<drs_sym_t> drs_schedule(uint32_t N_TS, uint32_t N_DF) {
    std::vector<drs_sym_t> out;
    uint32_t l_next = 1, ts_first = 0, parity = 0, y_hi = 0;
    while (l_next <= N_DF) {
        drs_sym_t s{};
        s.l = l_next;
        s.ts_first = ts_first;
        s.ts_last = ts_first == 0 ? std::min(N_TS - 1, 3u) : 7u;
        s.k_parity = parity;
        s.y_hi = y_hi;
        out.push_back(s);
        if (N_TS <= 2) {
            l_next += 5;
            parity ^= 1;
        } else if (N_TS == 4) {
            l_next += 10;
            parity ^= 1;
        } else {
            if (l_next % 2 == 1) {
                l_next += 1;
            } else {
                l_next += 9;
                parity ^= 1;
            }
            y_hi ^= 1;
            ts_first = ts_first == 0 ? 4 : 0;
        }
    }
    return out;
}

// drs.cpp:129-180 linear DRS indices for a virtual frame (u=8)
static std::vector<std::vector<uint32_t>> drs_linear(uint32_t b, uint32_t N_PACKET_symb, uint32_t N_TS) {
    const uint32_t N_b_DFT = 64 * b, N = 56 * b;
    const auto k = k_b_OCC(b);
    const uint32_t N_step = N_TS <= 2 ? 5 : 10;
    const uint32_t n_symb = nof_drs_symbols_per_ts(N_PACKET_symb, N_TS);
    std::vector<std::vector<uint32_t>> out(N_TS);
    for (uint32_t t = 0; t < N_TS; ++t) {
        for (uint32_t n = 0; n < n_symb; ++n) {
            const uint32_t l = 1 + t / 4 + n * N_step;
            const int off = static_cast<int>(N_b_DFT / 2 + N_b_DFT * l);
            for (uint32_t i = 0; i < N / 4; ++i)
                out[t].push_back(static_cast<uint32_t>(k[i * 4 + (t + (n % 2) * 2) % 4] + off));
        }
    }
    return out;
}

static void mark_virtual_frame(std::vector<int>& vf, uint32_t b, uint32_t n_symb) {
    const uint32_t N_b_DFT = 64 * b, gt = 4 * b - 1, gb = 4 * b;
    for (uint32_t l = 0; l < n_symb; ++l)
        for (uint32_t i = 0; i < N_b_DFT; ++i) vf[l * N_b_DFT + i] = static_cast<int>(l * N_b_DFT + i);
    for (uint32_t l = 0; l < n_symb; ++l) {
        vf[l * N_b_DFT + N_b_DFT / 2] = -1;
        for (uint32_t i = 0; i < gb; ++i) vf[l * N_b_DFT + i] = -2;
        for (uint32_t i = N_b_DFT - gt; i < N_b_DFT; ++i) vf[l * N_b_DFT + i] = -2;
    }
}

// pcc.cpp:132-259
static std::vector<uint32_t> pcc_linear(uint32_t b, uint32_t N_TS) {
    const uint32_t N_b_DFT = 64 * b, NP = 20;
    std::vector<int> vf(NP * N_b_DFT);
    mark_virtual_frame(vf, b, NP);
    for (const auto& v : drs_linear(b, NP, N_TS))
        for (uint32_t i : v) vf[i] = -3;
    std::vector<uint32_t> kp;
    uint32_t l = 1, unalloc = 98;
    while (true) {
        std::vector<uint32_t> avail;
        for (uint32_t i = 0; i < N_b_DFT; ++i)
            if (vf[l * N_b_DFT + i] >= 0) avail.push_back(static_cast<uint32_t>(vf[l * N_b_DFT + i]));
        const uint32_t U = static_cast<uint32_t>(avail.size());
        if (U < unalloc) {
            kp.insert(kp.end(), avail.begin(), avail.end());
            ++l;
            unalloc -= U;
            continue;
        }
        const uint32_t R = 7, C = U / R;
        if (U % R != 0) throw std::runtime_error("PCC: U not a multiple of 7");
        bool done = false;
        for (uint32_t c = 0; c < C && !done; ++c)
            for (uint32_t r = 0; r < R; ++r) {
                kp.push_back(avail[r * C + c]);
                if (--unalloc == 0) {
                    done = true;
                    break;
                }
            }
        std::sort(kp.begin(), kp.end());
        break;
    }
    return kp;
}

void pcc_cells(uint32_t b, uint32_t N_TS, std::vector<uint32_t>& l_sym,
               std::vector<std::vector<uint32_t>>& k_per_sym) {
    const uint32_t N_b_DFT = 64 * b, gb = 4 * b;
    l_sym.clear();
    k_per_sym.clear();
    for (uint32_t lin : pcc_linear(b, N_TS)) {
        const uint32_t l = lin / N_b_DFT;
        if (l_sym.empty() || l_sym.back() != l) {
            l_sym.push_back(l);
            k_per_sym.emplace_back();
        }
        k_per_sym.back().push_back(lin - l * N_b_DFT - gb);
    }
}

// pdc.cpp:31-110, 131-153, 217-300
std::vector<std::vector<uint32_t>> pdc_cells_packet(uint32_t b, uint32_t N_TS, uint32_t N_DF) {
    const uint32_t N_b_DFT = 64 * b, N = 56 * b, gb = 4 * b, NP = 30;
    std::vector<int> vf(NP * N_b_DFT);
    mark_virtual_frame(vf, b, NP);
    for (const auto& v : drs_linear(b, NP, N_TS))
        for (uint32_t i : v) vf[i] = -3;
    for (uint32_t i : pcc_linear(b, N_TS)) vf[i] = -4;
    const uint32_t N_DF_v = NP - 4;  // u = 8
    std::vector<std::vector<uint32_t>> rep(N_DF_v + 1);
    for (uint32_t l = 1; l < 1 + N_DF_v; ++l)
        for (uint32_t i = 0; i < N_b_DFT; ++i)
            if (vf[l * N_b_DFT + i] >= 0) rep[l].push_back(i - gb);
    rep.resize(21);
    for (uint32_t i = 0; i < rep.size(); ++i)
        if (i != 10 && rep[i].size() == N) rep[i].resize(1);
    const uint32_t l_limit = N_TS <= 2 ? 6 : 11, l_repeat = 10;
    std::vector<std::vector<uint32_t>> out(N_DF + 1);
    for (uint32_t l = 1; l <= N_DF; ++l) {
        uint32_t le = l <= l_limit ? l : l - ((l - l_limit) / l_repeat) * l_repeat;
        if (rep.at(le).size() == 1) le = 10;
        out[l] = rep.at(le);
    }
    return out;
}

// ---------------------------------------------------------------- transmit_diversity_precoding.cpp
uint32_t txdiv_modulo(uint32_t N_TS) { return N_TS == 2 ? 1 : N_TS == 4 ? 6 : 12; }

void txdiv_pair(uint32_t N_TS, uint32_t i_mod, uint32_t& A, uint32_t& B) {
    static const uint32_t P4[6][2] = {{0, 1}, {2, 3}, {0, 2}, {1, 3}, {0, 3}, {1, 2}};
    static const uint32_t P8[12][2] = {{0, 1}, {2, 3}, {4, 5}, {6, 7}, {0, 4}, {1, 5},
                                       {2, 6}, {3, 7}, {0, 2}, {1, 3}, {4, 6}, {5, 7}};
    if (N_TS == 2) {
        A = 0;
        B = 1;
    } else if (N_TS == 4) {
        A = P4[i_mod][0];
        B = P4[i_mod][1];
    } else {
        A = P8[i_mod][0];
        B = P8[i_mod][1];
    }
}

// ---------------------------------------------------------------- beamforming (Tables 6.3.4-1..6)
// entries: 0, 1, -1, 2 (=j), -2 (=-j)
static const std::vector<std::vector<int>>& W_table(uint32_t N_TS, uint32_t N_TX) {
    static const std::vector<std::vector<int>> W0 = {{1}};
    static const std::vector<std::vector<int>> W1 = {{1, 0}, {0, 1}, {1, 1}, {1, -1}, {1, 2}, {1, -2}};
    static const std::vector<std::vector<int>> W2 = {
        {1, 0, 0, 0},   {0, 1, 0, 0},  {0, 0, 1, 0},   {0, 0, 0, 1},   {1, 0, 1, 0},   {1, 0, -1, 0},
        {1, 0, 2, 0},   {1, 0, -2, 0}, {0, 1, 0, 1},   {0, 1, 0, -1},  {0, 1, 0, 2},   {0, 1, 0, -2},
        {1, 1, 1, 1},   {1, 1, 2, 2},  {1, 1, -1, -1}, {1, 1, -2, -2}, {1, 2, 1, 2},   {1, 2, 2, -1},
        {1, 2, -1, -2}, {1, 2, -2, 1}, {1, -1, 1, -1}, {1, -1, 2, -2}, {1, -1, -1, 1}, {1, -1, -2, 2},
        {1, -2, 1, -2}, {1, -2, 2, 1}, {1, -2, -1, 2}, {1, -2, -2, -1}};
    static const std::vector<std::vector<int>> W3 = {{1, 0, 0, 1}, {1, 1, 1, -1}, {1, 1, 2, -2}};
    static const std::vector<std::vector<int>> W4 = {
        {1, 0, 0, 1, 0, 0, 0, 0},     {1, 0, 0, 0, 0, 1, 0, 0},     {1, 0, 0, 0, 0, 0, 0, 1},
        {0, 0, 1, 0, 0, 1, 0, 0},     {0, 0, 1, 0, 0, 0, 0, 1},     {0, 0, 0, 0, 1, 0, 0, 1},
        {1, 0, 0, 1, 1, 0, 0, -2},    {1, 0, 0, 1, 1, 0, 0, 2},     {1, 0, 0, 1, -2, 0, 0, 1},
        {1, 0, 0, 1, -2, 0, 0, -1},   {1, 0, 0, 1, -1, 0, 0, -2},   {1, 0, 0, 1, -1, 0, 0, 2},
        {1, 0, 0, 1, 2, 0, 0, 1},     {1, 0, 0, 1, 2, 0, 0, -1},    {1, 1, 1, 1, 1, -1, 1, -1},
        {1, 1, 1, 1, 2, -2, 2, -2},   {1, 1, 2, 2, 1, -1, 2, -2},   {1, 1, 2, 2, 2, -2, -1, 1},
        {1, 1, -1, -1, 1, -1, -1, 1}, {1, 1, -1, -1, 2, -2, -2, 2}, {1, 1, -2, -2, 1, -1, -2, 2},
        {1, 1, -2, -2, 2, -2, 1, -1}};
    static const std::vector<std::vector<int>> W5 = {
        {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1},
        {1, 1, 0, 0, 0, 0, 1, 1, 1, -1, 0, 0, 0, 0, 1, -1},
        {1, 1, 0, 0, 0, 0, 1, 1, 2, -2, 0, 0, 0, 0, 2, -2},
        {1, 1, 1, 1, 1, -1, 1, -1, 1, 1, -1, -1, 1, -1, -1, 1},
        {1, 1, 1, 1, 1, -1, 1, -1, 2, 2, -2, -2, 2, -2, -2, 2}};
    static const std::vector<std::vector<int>> W6 = [] {
        std::vector<int> m(64, 0);
        for (int i = 0; i < 8; ++i) m[i * 8 + i] = 1;
        return std::vector<std::vector<int>>{m};
    }();
    if (N_TS == 1 && N_TX == 1) return W0;
    if (N_TS == 1 && N_TX == 2) return W1;
    if (N_TS == 1 && N_TX == 4) return W2;
    if (N_TS == 2 && N_TX == 2) return W3;
    if (N_TS == 2 && N_TX == 4) return W4;
    if (N_TS == 4 && N_TX == 4) return W5;
    if (N_TS == 8 && N_TX == 8) return W6;
    throw std::runtime_error("W undefined for N_TS/N_TX");
}

uint32_t W_codebook_max(uint32_t N_TS, uint32_t N_TX) {
    return static_cast<uint32_t>(W_table(N_TS, N_TX).size() - 1);
}

std::vector<cd> W_matrix(uint32_t N_TS, uint32_t N_TX, uint32_t codebook) {
    const auto& e = W_table(N_TS, N_TX).at(codebook);
    std::vector<cd> w(e.size());
    for (size_t i = 0; i < e.size(); ++i) {
        const int v = e[i];
        w[i] = v == 2 ? cd{0, 1} : v == -2 ? cd{0, -1} : cd{static_cast<double>(v), 0};
    }
    return w;
}

double W_scaling(uint32_t N_TS, uint32_t N_TX, uint32_t codebook) {
    const auto& e = W_table(N_TS, N_TX).at(codebook);
    float cnt = 0.0f;
    for (int v : e)
        if (v != 0) cnt += 1.0f;
    return static_cast<double>(1.0f / std::sqrt(cnt));
}

// W_t::scaling_factor_optimal_DAC, one list per matrix family in the constructor's order
double W_scaling_optimal_DAC(uint32_t N_TS, uint32_t N_TX, uint32_t codebook) {
    (void)W_table(N_TS, N_TX).at(codebook);
    const float h = 1.0f / std::sqrt(2.0f), q = 1.0f / std::sqrt(4.0f);
    float v = 1.0f;
    if (N_TS == 2 && N_TX == 2) v = codebook == 0 ? 1.0f : h;
    if (N_TS == 2 && N_TX == 4) v = codebook < 14 ? 1.0f : h;
    if (N_TS == 4 && N_TX == 4) {
        static const float t[5] = {1.0f, h, h, q, q};
        v = t[codebook];
    }
    return static_cast<double>(v);
}

const float STF_COVER_SEQ[9] = {1, -1, 1, 1, -1, -1, -1, -1, -1};

// ---------------------------------------------------------------- 3GPP TS 36.211 §7.2
std::vector<uint8_t> gold_sequence(uint32_t c_init, uint32_t len) {
    const uint32_t Nc = 1600;
    std::vector<uint8_t> x1(Nc + len + 31, 0), x2(Nc + len + 31, 0), c(len);
    x1[0] = 1;
    for (uint32_t i = 0; i < 31; ++i) x2[i] = (c_init >> i) & 1u;
    for (uint32_t n = 0; n < Nc + len; ++n) {
        x1[n + 31] = (x1[n + 3] + x1[n]) & 1u;
        x2[n + 31] = (x2[n + 3] + x2[n + 2] + x2[n + 1] + x2[n]) & 1u;
    }
    for (uint32_t n = 0; n < len; ++n) c[n] = (x1[n + Nc] + x2[n + Nc]) & 1u;
    return c;
}

// ---------------------------------------------------------------- 3GPP TS 36.211 §7.1
std::vector<cd> constellation(uint32_t N_bps) {
    const uint32_t n = 1u << N_bps;
    std::vector<cd> t(n);
    auto bit = [&](uint32_t idx, uint32_t k) { return static_cast<int>((idx >> (N_bps - 1 - k)) & 1u); };
    for (uint32_t idx = 0; idx < n; ++idx) {
        double re = 0, im = 0;
        switch (N_bps) {
            case 1:
                re = im = (1 - 2 * bit(idx, 0)) / std::sqrt(2.0);
                break;
            case 2:
                re = (1 - 2 * bit(idx, 0)) / std::sqrt(2.0);
                im = (1 - 2 * bit(idx, 1)) / std::sqrt(2.0);
                break;
            case 4:
                re = (1 - 2 * bit(idx, 0)) * (2 - (1 - 2 * bit(idx, 2))) / std::sqrt(10.0);
                im = (1 - 2 * bit(idx, 1)) * (2 - (1 - 2 * bit(idx, 3))) / std::sqrt(10.0);
                break;
            case 6:
                re = (1 - 2 * bit(idx, 0)) * (4 - (1 - 2 * bit(idx, 2)) * (2 - (1 - 2 * bit(idx, 4)))) /
                     std::sqrt(42.0);
                im = (1 - 2 * bit(idx, 1)) * (4 - (1 - 2 * bit(idx, 3)) * (2 - (1 - 2 * bit(idx, 5)))) /
                     std::sqrt(42.0);
                break;
            case 8:
                re = (1 - 2 * bit(idx, 0)) *
                     (8 - (1 - 2 * bit(idx, 2)) * (4 - (1 - 2 * bit(idx, 4)) * (2 - (1 - 2 * bit(idx, 6))))) /
                     std::sqrt(170.0);
                im = (1 - 2 * bit(idx, 1)) *
                     (8 - (1 - 2 * bit(idx, 3)) * (4 - (1 - 2 * bit(idx, 5)) * (2 - (1 - 2 * bit(idx, 7))))) /
                     std::sqrt(170.0);
                break;
            default:
                throw std::runtime_error("unsupported N_bps");
        }
        t[idx] = cd{re, im};
    }
    return t;
}

// ---------------------------------------------------------------- phy/filter/{kaiser,bessel,rectangular}.cpp
static double bessel_series(double z, bool modified) {  // bessel.cpp:27-55, 8 terms
    double r = 0.0;
    uint64_t fac = 1;
    for (uint32_t k = 0; k <= 8; ++k) {
        if (k > 0) fac *= k;
        const double num = modified ? std::pow(0.25 * z * z, static_cast<double>(k))
                                    : std::pow(-0.25 * z * z, static_cast<double>(k));
        const double f = static_cast<double>(fac);
        r += num / (f * f);
    }
    return r;
}
static float bessel_J0(float z) { return static_cast<float>(bessel_series(z, false)); }
static float bessel_I0(float z) { return static_cast<float>(bessel_series(z, true)); }
static float sinc_f(float n) {
    return (n == 0.0f) ? 1.0f : static_cast<float>(std::sin(M_PI * n) / (M_PI * n));
}

// J0(z), I0(z), sinc(z - 2), r_f_uni(1 us, z * 27 kHz), r_t_jakes(500 Hz, z * 5.2083 us): the sample
// points of tests/golden/ref_tables.json "special" (channel_statistics.cpp:27-33 in float)
void special_values(float z, float* out) {
    out[0] = bessel_J0(z);
    out[1] = bessel_I0(z);
    out[2] = sinc_f(z - 2.0f);
    out[3] = sinc_f(static_cast<float>(M_PI) * 1.0e-6f * (z * 27000.0f));
    out[4] = bessel_J0(2.0f * static_cast<float>(M_PI) * 500.0f * (z * 5.2083e-6f));
}

std::vector<float> kaiser(float f_pass, float f_stop, float ripple_dB, float att_dB, float fs,
                          bool force_odd) {
    const float d0 = std::pow(10.0f, -att_dB / 20.0f);
    const float d1 = std::pow(10.0f, ripple_dB / 20.0f) - 1.0f;
    const float delta = std::min(d0, d1);
    const float A = -20.0f * std::log10(delta);
    float beta = 0.0f;
    if (A > 50.0f)
        beta = 0.1102f * (A - 8.7f);
    else if (21.0f <= A && A <= 50.0f)
        beta = static_cast<float>(0.5842f * std::pow((A - 21.0f), 0.4f) + 0.07886 * (A - 21.0f));
    const float fpn = f_pass / fs, fsn = f_stop / fs;
    const float bw = fsn - fpn;
    const float order = static_cast<float>((A - 7.95f) / (2.285f * 2.0f * M_PI * bw));
    uint32_t N = static_cast<uint32_t>(std::ceil(order + 1.0f));
    if (force_odd && N % 2 == 0) N += 1;
    std::vector<float> w(N), rect(N), out(N);
    for (uint32_t n = 0; n < N; ++n) {
        const float Nf = static_cast<float>(N), nf = static_cast<float>(n);
        const float arg = beta * std::sqrt(1.0f - std::pow(2.0f * nf / (Nf - 1.0f) - 1.0f, 2.0f));
        w[n] = bessel_I0(arg) / bessel_I0(beta);
    }
    const float fc = fpn + bw / 2.0f;
    for (uint32_t n = 0; n < N; ++n) {
        const float Nf = static_cast<float>(N), nf = static_cast<float>(n);
        rect[n] = 2.0f * fc * sinc_f(2.0f * fc * (nf - (Nf - 1.0f) / 2.0f));
    }
    float norm = 0.0f;
    for (uint32_t n = 0; n < N; ++n) {
        w[n] = w[n] * rect[n];
        norm += w[n];
    }
    for (uint32_t n = 0; n < N; ++n) out[n] = w[n] / norm;
    return out;
}

// resampler.cpp:56-160 + resampler_param.hpp:77-88 (TX/SYNC/RX_SYNCED share the values)
void resampler_t::design(uint32_t L_, uint32_t M_, uint32_t os_min) {
    L = L_;
    M = M_;
    h.clear();
    if (L == 1 && M == 1) {
        filter_length = 1;
        delay = 0;
        hl = 0;
        h = {1.0f};
        return;
    }
    int oi = -1;
    switch (os_min) {
        case 1: oi = 0; break;
        case 2: oi = 1; break;
        case 4: oi = 2; break;
        case 8: oi = 3; break;
        default: throw std::runtime_error("os_min undefined");
    }
    const float LM = std::max(static_cast<float>(L), static_cast<float>(M));
    auto taps = kaiser(prm::RS_F_PASS[oi] / LM, prm::RS_F_STOP[oi] / LM, prm::RS_RIPPLE, prm::RS_ATT_DB[oi], 1.0f, true);
    filter_length = static_cast<uint32_t>(taps.size());
    delay = (filter_length - 1) / 2;
    for (auto& t : taps) t *= static_cast<float>(L);
    const uint32_t padded = ((filter_length + L - 1) / L) * L;
    taps.resize(padded, 0.0f);
    hl = padded / L - 1;
    h = taps;
}

uint64_t resampler_t::n_out_no_flush(uint64_t N) const {
    if (L == 1 && M == 1) return N;
    const uint64_t NL = N * L;
    if (NL <= delay) return 0;
    return (NL - delay + M - 1) / M;
}

// ---------------------------------------------------------------- channel_lut.cpp / wiener.hpp
std::vector<chest_stats_t> chest_profiles(uint32_t u_max) {
    const auto nm = get_numerology(u_max, 1);
    const double* nu = prm::NU_MAX_HZ;
    const double* tau = prm::TAU_RMS_SEC;
    const double* snr = prm::SNR_DB;
    const uint32_t *nlr = prm::N_INTERP_LR, *nl = prm::N_INTERP_L;
    std::vector<chest_stats_t> v;
    for (int i = 0; i < 3; ++i) {
        chest_stats_t s{};
        s.delta_u_f = nm.delta_u_f;
        s.T_u_symb = nm.T_u_symb;
        s.nu_max_hz = nu[i];
        s.tau_rms_sec = tau[i];
        s.snr_db = snr[i];
        s.sigma = 1.0 / std::pow(10.0, snr[i] / 10.0);
        s.n_lr = nlr[i];
        s.n_l = nl[i];
        v.push_back(s);
    }
    return v;
}

namespace {
struct coord {
    double f, t;
};
double corr_tf(const coord& A, const coord& B, const chest_stats_t& st) {
    const double df = A.f - B.f, dt = A.t - B.t;
    // channel_statistics.cpp:27-33 with float parameters
    const float tau = static_cast<float>(st.tau_rms_sec), fdf = static_cast<float>(df * st.delta_u_f);
    const float rf = sinc_f(static_cast<float>(M_PI) * tau * fdf);
    const float nu = static_cast<float>(st.nu_max_hz), fdt = static_cast<float>(dt * st.T_u_symb);
    const float rt = bessel_J0(2.0f * static_cast<float>(M_PI) * nu * fdt);
    return static_cast<double>(rf) * static_cast<double>(rt);
}
// Gaussian elimination with partial pivoting (Rpp is symmetric positive definite, full rank,
// so the least-norm solution of the reference's CompleteOrthogonalDecomposition coincides).
std::vector<double> solve(std::vector<double> A, std::vector<double> b, uint32_t n) {
    for (uint32_t c = 0; c < n; ++c) {
        uint32_t p = c;
        for (uint32_t r = c + 1; r < n; ++r)
            if (std::fabs(A[r * n + c]) > std::fabs(A[p * n + c])) p = r;
        if (p != c) {
            for (uint32_t k = 0; k < n; ++k) std::swap(A[c * n + k], A[p * n + k]);
            std::swap(b[c], b[p]);
        }
        for (uint32_t r = c + 1; r < n; ++r) {
            const double f = A[r * n + c] / A[c * n + c];
            for (uint32_t k = c; k < n; ++k) A[r * n + k] -= f * A[c * n + k];
            b[r] -= f * b[c];
        }
    }
    std::vector<double> x(n);
    for (int r = static_cast<int>(n) - 1; r >= 0; --r) {
        double s = b[r];
        for (uint32_t k = r + 1; k < n; ++k) s -= A[r * n + k] * x[k];
        x[r] = s / A[r * n + r];
    }
    return x;
}

void fill_lut(uint32_t Nsv, uint32_t b, const chest_stats_t& st, chest_lut_t& lut,
              std::vector<std::vector<float>>& vecs) {
    const uint32_t N_f = 56 * b + 1, T = Nsv + 1, n = Nsv > 0 ? st.n_lr : st.n_l;
    lut.ps_t_length = T;
    lut.nof_interp = n;
    lut.N_f = N_f;
    lut.idx_pilot.assign(T * 4 * N_f, 0);
    lut.idx_weight.assign(T * 4 * N_f, 0);
    for (uint32_t ts = 0; ts < 4; ++ts) {
        const auto kl = drs_k_i(b, ts, 0), kr = drs_k_i(b, ts, 1);
        std::vector<coord> cv;
        const double t0 = 1.0, t1 = 1.0 + Nsv;
        for (size_t p = 0; p < kl.size(); ++p) {
            if (Nsv > 0) {
                if (ts <= 1) {
                    cv.push_back({static_cast<double>(kl[p]), t0});
                    cv.push_back({static_cast<double>(kr[p]), t1});
                } else {
                    cv.push_back({static_cast<double>(kr[p]), t1});
                    cv.push_back({static_cast<double>(kl[p]), t0});
                }
            } else {
                cv.push_back({static_cast<double>(kl[p]), t0});
            }
        }
        for (uint32_t t = 1; t <= T; ++t) {
            uint32_t prev = 0;
            std::vector<double> Rpp(n * n);
            for (uint32_t f = 0; f < N_f; ++f) {
                const coord D{static_cast<double>(f), static_cast<double>(t)};
                double best = 1e9;
                uint32_t opt = 0;
                for (uint32_t i = prev; i <= cv.size() - n; ++i) {
                    double s = 0;
                    for (uint32_t j = i; j < i + n; ++j)
                        s += std::sqrt(std::pow(D.f - cv[j].f, 2.0) + std::pow(D.t - cv[j].t, 2.0));
                    if (s < best) {
                        best = s;
                        opt = i;
                    }
                    if (s > best * prm::LUT_SEARCH_ABORT) break;
                }
                if (f == 0 || opt != prev)  // channel_lut.cpp:399-437 refresh rule
                    for (uint32_t r = 0; r < n; ++r)
                        for (uint32_t c = 0; c < n; ++c)
                            Rpp[r * n + c] = corr_tf(cv[opt + r], cv[opt + c], st) + (r == c ? st.sigma : 0.0);
                std::vector<double> rdp(n);
                for (uint32_t r = 0; r < n; ++r) rdp[r] = corr_tf(D, cv[opt + r], st);
                const auto w = solve(Rpp, rdp, n);
                double sum = 0;
                for (double x : w) sum += x;
                std::vector<float> wf(n);
                for (uint32_t r = 0; r < n; ++r) wf[r] = static_cast<float>(w[r] / sum);
                // channel_lut.cpp:563-620 dedupe with 1e-4 threshold
                int known = -1;
                for (size_t v = 0; v < vecs.size() && known < 0; ++v) {
                    float mx = 0.0f, dv = 0.0f;
                    for (uint32_t r = 0; r < n; ++r) {
                        const float d = wf[r] - vecs[v][r];
                        if (std::fabs(d) > mx) {
                            mx = std::fabs(d);
                            dv = d;
                        }
                    }
                    if (std::fabs(static_cast<double>(dv)) < 1e-4) known = static_cast<int>(v);
                }
                if (known < 0) {
                    vecs.push_back(wf);
                    known = static_cast<int>(vecs.size() - 1);
                }
                const size_t o = ((t - 1) * 4 + ts) * N_f + f;
                lut.idx_pilot[o] = opt;
                lut.idx_weight[o] = static_cast<uint32_t>(known);
                prev = opt;
            }
        }
    }
}
}  // namespace

chest_lut_t build_chest_lut(uint32_t Nsv, uint32_t b, uint32_t b_max, const chest_stats_t& st) {
    std::vector<std::vector<float>> vecs;
    chest_lut_t lut;
    if (b != b_max) {
        chest_lut_t tmp;
        fill_lut(Nsv, b_max, st, tmp, vecs);  // b_max vectors first (channel_lut.cpp:238-262)
    }
    fill_lut(Nsv, b, st, lut, vecs);
    const uint32_t n = Nsv > 0 ? st.n_lr : st.n_l;
    lut.weights.resize(vecs.size() * n);
    for (size_t v = 0; v < vecs.size(); ++v)
        for (uint32_t r = 0; r < n; ++r) lut.weights[v * n + r] = vecs[v][r];
    return lut;
}

}  // namespace orc
