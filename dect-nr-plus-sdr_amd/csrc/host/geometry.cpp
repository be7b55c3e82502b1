// Host-side DECT NR+ geometry for the GPU path. See geometry.hpp. Each block cites the reference
// file it restates (paths relative to maxpenner/DECT-NR-Plus-SDR).
#include "geometry.hpp"

#include <cstring>

#include <algorithm>
#include <cmath>
#include <stdexcept>

namespace dnrp::geo {

// ------------------------------------------------------------ sections_part3 scalar tables
static const uint8_t TM[12][5] = {  // {N_eff_TX, N_SS, cl, N_TS, N_TX}, tm_mode.cpp:27-137
    {1, 1, 0, 1, 1}, {2, 1, 0, 2, 2}, {2, 2, 0, 2, 2}, {1, 1, 1, 1, 2}, {2, 2, 1, 2, 2}, {4, 1, 0, 4, 4},
    {4, 4, 0, 4, 4}, {1, 1, 1, 1, 4}, {2, 2, 1, 2, 4}, {4, 4, 1, 4, 4}, {8, 1, 0, 8, 8}, {8, 8, 0, 8, 8}};
static const uint8_t MCS[12][3] = {  // {N_bps, R_num, R_den}, mcs.cpp:27-105
    {1, 1, 2}, {2, 1, 2}, {2, 3, 4}, {4, 1, 2}, {4, 3, 4}, {6, 2, 3},
    {6, 3, 4}, {6, 5, 6}, {8, 3, 4}, {8, 5, 6}, {10, 3, 4}, {10, 5, 6}};

static uint32_t n_drs_symbols(uint32_t N_PACKET, uint32_t N_eff_TX) {  // pdc.cpp:168-192
    const uint32_t step = N_eff_TX <= 2 ? 5 : 10;
    return N_PACKET / step + ((step == 10 && N_PACKET % 10) ? 1 : 0);
}

static bool cb_segmentation(uint32_t tbs, uint32_t Z, uint32_t& C, uint32_t& F) {  // fix/cbsegm.cpp:56-118
    // TS 36.212 Table 5.1.3-3 interleaver sizes: 40..512/8, 528..1024/16, 1056..2048/32, 2112..6144/64
    auto kidx = [](uint32_t K) -> int {
        static std::vector<uint32_t> s;
        if (s.empty()) {
            for (uint32_t k = 40; k <= 512; k += 8) s.push_back(k);
            for (uint32_t k = 528; k <= 1024; k += 16) s.push_back(k);
            for (uint32_t k = 1056; k <= 2048; k += 32) s.push_back(k);
            for (uint32_t k = 2112; k <= 6144; k += 64) s.push_back(k);
        }
        const auto it = std::lower_bound(s.begin(), s.end(), K);
        return it == s.end() ? -1 : static_cast<int>(it - s.begin());
    };
    auto ksize = [](int j) -> uint32_t {
        if (j < 60) return 40 + 8 * j;
        if (j < 92) return 528 + 16 * (j - 60);
        if (j < 124) return 1056 + 32 * (j - 92);
        return 2112 + 64 * (j - 124);
    };
    if (tbs == 0) {
        C = F = 0;
        return true;
    }
    const uint32_t B = tbs + 24;
    uint32_t Bp = B;
    C = 1;
    if (B > Z) {
        C = (B + Z - 24 - 1) / (Z - 24);
        Bp = B + 24 * C;
    }
    const int j = kidx((Bp - 1) / C + 1);
    if (j < 0) return false;
    const uint32_t K1 = ksize(j);
    uint32_t K2 = 0, C1 = 1, C2 = 0;
    if (C > 1) {
        if (j == 0) return false;
        K2 = ksize(j - 1);
        C2 = (C * K1 - Bp) / (K1 - K2);
        C1 = C - C2;
    }
    F = C1 * K1 + C2 * K2 - Bp;
    return true;
}

bool packet_sizes(const dnrp_psdef& d, dnrp_packet_sizes& q, tm_t* tm_out) {  // packet_sizes.cpp:99-236
    const uint32_t u = d.u, b = d.b;
    if (!(u == 1 || u == 2 || u == 4 || u == 8)) return false;
    if (!(b == 1 || b == 2 || b == 4 || b == 8 || b == 12 || b == 16)) return false;
    if (d.PacketLengthType > 1 || d.PacketLength < 1 || d.PacketLength > 16) return false;
    if (d.tm_mode_index > 11 || d.mcs_index > 11 || (d.Z != 2048 && d.Z != 6144)) return false;
    q = dnrp_packet_sizes{};
    const uint32_t N_P = d.PacketLengthType == 0 ? d.PacketLength * 5 : d.PacketLength * 10 * u;
    if (N_P < 5 || N_P > 1280 || N_P % 5) return false;
    tm_t tm{d.tm_mode_index, TM[d.tm_mode_index][0], TM[d.tm_mode_index][1], TM[d.tm_mode_index][3],
            TM[d.tm_mode_index][4], TM[d.tm_mode_index][2] != 0,
            d.tm_mode_index == 1 || d.tm_mode_index == 5 || d.tm_mode_index == 10};
    if (tm.N_eff_TX == 4 && N_P < 15) return false;
    if (u == 8 && tm.N_eff_TX == 8 && (N_P < 20 || N_P % 10)) return false;
    const uint32_t N_occ = 56 * b;
    const uint32_t N_DF = u == 1 ? N_P - 2 : (u <= 4 ? N_P - 3 : N_P - 4);
    const uint32_t N_DRS = tm.N_eff_TX * N_occ / 4 * n_drs_symbols(N_P, tm.N_eff_TX);
    if (N_DF * N_occ <= N_DRS + 98) return false;
    const uint32_t N_PDC = N_DF * N_occ - N_DRS - 98;
    const uint32_t N_bps = MCS[d.mcs_index][0], Rn = MCS[d.mcs_index][1], Rd = MCS[d.mcs_index][2];
    const uint32_t G = tm.N_SS * N_PDC * N_bps;
    const uint32_t N_PDC_bits = G * Rn / Rd;  // transport_block_size.cpp:24-66
    const uint32_t Mq = N_PDC_bits <= 512 ? 8 : N_PDC_bits <= 1024 ? 16 : N_PDC_bits <= 2048 ? 32 : 64;
    const uint32_t N_M = N_PDC_bits / Mq * Mq;
    if (N_M <= 24) return false;
    const uint32_t N_TB = N_M <= d.Z ? N_M - 24 : N_M - ((N_M - 24 + d.Z - 1) / d.Z + 1) * 24;
    uint32_t C, F;
    if (!cb_segmentation(N_TB, d.Z, C, F) || F > 0) return false;
    q.N_PACKET_symb = N_P;
    q.N_DF_symb = N_DF;
    q.N_PDC_subc = N_PDC;
    q.N_DRS_subc = N_DRS;
    q.G = G;
    q.N_PDC_bits = N_PDC_bits;
    q.N_TB_bits = N_TB;
    q.N_TB_byte = (N_TB + 7) / 8;
    q.C = C;
    const uint32_t sym = 72 * b;  // transmission_packet_structure.cpp
    q.N_samples_STF = u == 1 ? sym * 14 / 9 : sym * 2;
    q.N_samples_STF_CP_only = q.N_samples_STF - 64 * b;
    q.N_samples_DF = sym * N_DF;
    q.N_samples_GI = u == 1 ? sym * 4 / 9 : (u <= 4 ? sym : 2 * sym);
    q.N_samples_packet_no_GI = q.N_samples_STF + q.N_samples_DF;
    q.N_samples_packet = q.N_samples_packet_no_GI + q.N_samples_GI;
    q.N_bps = N_bps;
    q.N_eff_TX = tm.N_eff_TX;
    q.N_SS = tm.N_SS;
    q.N_TS = tm.N_TS;
    q.N_TX = tm.N_TX;
    q.N_b_DFT = 64 * b;
    q.N_b_OCC = N_occ;
    if (tm_out) *tm_out = tm;
    return true;
}

dims_t make_dims(const dnrp_cfg& cfg, const dnrp_psdef& d, const dnrp_packet_sizes& q) {
    dims_t m{};
    const uint64_t rate = uint64_t(cfg.u_max) * cfg.b_max * 1728000ull * cfg.os_min;
    m.Nd = static_cast<uint32_t>(rate / (uint64_t(d.u) * 27000ull));
    m.N_occ = q.N_b_OCC;
    m.Nf = q.N_b_OCC + 1;
    m.off_lower = q.N_b_DFT / 2 + (m.Nd - q.N_b_DFT) + 4 * d.b;  // tx_rx.cpp:197-240
    m.CP = 8 * d.b * m.Nd / q.N_b_DFT;
    m.STF_CP = q.N_samples_STF_CP_only * m.Nd / q.N_b_DFT;
    m.N_no_GI = q.N_samples_packet_no_GI * m.Nd / q.N_b_DFT;
    m.N_no_GI_rs = static_cast<uint32_t>((uint64_t(m.N_no_GI) * cfg.L + cfg.M - 1) / cfg.M);
    m.N_packet_rs = q.N_samples_packet * m.Nd / q.N_b_DFT / cfg.M * cfg.L;
    m.n_pattern = d.u == 1 ? 7 : 9;
    m.pattern_len = 16 * d.b * m.Nd / q.N_b_DFT;
    return m;
}

// ------------------------------------------------------------ cell maps
// subcarrier value k (-N/2..-1, 1..N/2) of occupied index i (physical_resources.cpp:24-35)
static int kocc(uint32_t N, uint32_t i) {
    return i < N / 2 ? static_cast<int>(i) - static_cast<int>(N / 2) : static_cast<int>(i) - static_cast<int>(N / 2) + 1;
}

static const int8_t DRS_Y[56] = {1,  1,  1,  1,  -1, 1,  1,  -1, -1, 1,  1,  1,  1,  -1, 1,  -1, 1,  1,  -1,
                                 1,  -1, 1,  -1, 1,  1,  1,  1,  1,  -1, 1,  -1, -1, 1,  1,  -1, -1, -1, -1,
                                 1,  -1, -1, -1, -1, -1, 1,  1,  1,  -1, 1,  1,  -1, -1, 1,  -1, -1, -1};
static const int8_t STF_B1[14] = {1, -1, 1, 1, -1, 1, 1, -1, 1, 1, 1, -1, -1, -1};
static const int8_t STF_B2[28] = {-1, 1, -1, 1, 1, -1, 1, 1, -1, 1, 1, 1, -1, 1,
                                  -1, -1, -1, 1, -1, -1, -1, 1, 1, 1, -1, -1, -1, -1};
static const int8_t STF_B4[56] = {-1, -1, -1, 1, -1, 1, -1, -1, 1, 1, 1, 1, -1, 1, -1, -1, -1, 1, -1,
                                  1,  1,  -1, -1, -1, -1, -1, 1, -1, 1, 1, 1, -1, 1, -1, 1, 1, -1, -1,
                                  -1, -1, 1, -1, -1, -1, -1, 1, -1, 1, 1, -1, -1, -1, -1, -1, 1, -1};

static std::vector<int> stf_polarity(uint32_t b) {  // stf.cpp:207-250
    auto ext = [](std::vector<int> v) {            // v ++ fliplr(v) .* (-1)^k
        const size_t n = v.size();
        for (size_t i = 0; i < n; ++i) v.push_back(v[n - 1 - i] * ((i & 1) ? -1 : 1));
        return v;
    };
    if (b == 1) return std::vector<int>(STF_B1, STF_B1 + 14);
    if (b == 2) return std::vector<int>(STF_B2, STF_B2 + 28);
    std::vector<int> v(STF_B4, STF_B4 + 56);
    if (b == 4) return v;
    v = ext(v);
    if (b == 8) return v;
    v = ext(v);
    if (b == 16) return v;
    return std::vector<int>(v.begin() + 28, v.begin() + 28 + 168);  // b = 12
}

static std::vector<drs_sym_t> drs_schedule(uint32_t N_TS, uint32_t N_DF) {  // drs.cpp:90-127
    std::vector<drs_sym_t> v;
    uint32_t l = 1, first = 0, par = 0;
    while (l <= N_DF) {
        v.push_back({l, first, first == 0 ? std::min(N_TS - 1, 3u) : 7u, par});
        if (N_TS <= 2) {
            l += 5;
            par ^= 1;
        } else if (N_TS == 4) {
            l += 10;
            par ^= 1;
        } else {
            if (l & 1) {
                l += 1;
            } else {
                l += 9;
                par ^= 1;
            }
            first = first == 0 ? 4 : 0;
        }
    }
    return v;
}

// virtual frame of n_symb symbols x N_b_DFT, -1 = occupied (DC, guards, DRS[, PCC])
static std::vector<int8_t> virtual_frame(uint32_t b, uint32_t N_TS, uint32_t n_symb) {
    const uint32_t Nb = 64 * b, N = 56 * b;
    std::vector<int8_t> free_(n_symb * Nb, 1);
    for (uint32_t l = 0; l < n_symb; ++l) {
        free_[l * Nb + Nb / 2] = 0;
        for (uint32_t i = 0; i < 4 * b; ++i) free_[l * Nb + i] = 0;
        for (uint32_t i = Nb - (4 * b - 1); i < Nb; ++i) free_[l * Nb + i] = 0;
    }
    const uint32_t step = N_TS <= 2 ? 5 : 10;
    const uint32_t nd = n_drs_symbols(n_symb, N_TS);  // drs.cpp:129-180 with u = 8
    for (uint32_t t = 0; t < N_TS; ++t)
        for (uint32_t n = 0; n < nd; ++n) {
            const uint32_t l = 1 + t / 4 + n * step;
            for (uint32_t i = 0; i < N / 4; ++i)
                free_[l * Nb + Nb / 2 + kocc(N, i * 4 + (t + (n % 2) * 2) % 4)] = 0;
        }
    return free_;
}

static std::vector<uint32_t> pcc_linear(uint32_t b, uint32_t N_TS) {  // pcc.cpp:132-259
    const uint32_t Nb = 64 * b;
    auto vf = virtual_frame(b, N_TS, 20);
    std::vector<uint32_t> out;
    uint32_t need = 98;
    for (uint32_t l = 1; need > 0; ++l) {
        std::vector<uint32_t> U;
        for (uint32_t i = 0; i < Nb; ++i)
            if (vf[l * Nb + i]) U.push_back(l * Nb + i);
        if (U.size() < need) {
            out.insert(out.end(), U.begin(), U.end());
            need -= static_cast<uint32_t>(U.size());
            continue;
        }
        const uint32_t C = static_cast<uint32_t>(U.size()) / 7;  // R_PCC = 7 rows, read column-wise
        for (uint32_t c = 0; c < C && need; ++c)
            for (uint32_t r = 0; r < 7 && need; ++r, --need) out.push_back(U[r * C + c]);
    }
    std::sort(out.begin(), out.end());
    return out;
}

std::vector<cf32> stf_values(uint32_t b, uint32_t N_eff_TX) {  // stf.cpp:171-183, 185-285
    const uint32_t N = 56 * b;
    const auto pol = stf_polarity(b);
    uint32_t lg = 0;
    while ((1u << lg) < N_eff_TX) ++lg;
    const cf32 fac = cf32(1.0f, 0.0f) * cf32(static_cast<float>(std::cos(M_PI / 4.0)), static_cast<float>(std::sin(M_PI / 4.0)));
    std::vector<cf32> v(N + 1, cf32(0, 0));
    for (uint32_t i = 0; i < N / 4; ++i) {
        const uint32_t occ = i < N / 8 ? 4 * i : N / 2 + 3 + 4 * (i - N / 8);
        const uint32_t k = static_cast<uint32_t>(kocc(N, occ) + static_cast<int>(N / 2));
        v[k] = cf32(static_cast<float>(pol[(i + 2 * lg) % (N / 4)]), 0.0f) * fac;
    }
    return v;
}

float drs_value(uint32_t t, uint32_t i) { return static_cast<float>(DRS_Y[(4 * i + t % 4) % 56] * (t < 4 ? 1 : -1)); }

uint64_t drs_neg_mask() {
    uint64_t m = 0;
    for (uint32_t j = 0; j < 56; ++j) m |= uint64_t(DRS_Y[j] < 0) << j;
    return m;
}

// the front end's arithmetic DRS cells (rx_front.hpp rx_drs_partials) against the tables
bool drs_tables_arithmetic(const maps_t& m) {
    const uint32_t N = m.Nf - 1, nd = N / 4;
    const uint64_t neg = drs_neg_mask();
    for (uint32_t p = 0; p < 2; ++p)
        for (uint32_t t = 0; t < 8; ++t)
            for (uint32_t i = 0; i < nd; ++i) {
                const uint32_t x = 4 * i + ((t + 2 * p) & 3u), k = x + (x >= N / 2 ? 1u : 0u);
                const float s = (((neg >> ((4 * i + (t & 3u)) % 56)) & 1ull) ? -1.f : 1.f) * (t < 4 ? 1.f : -1.f);
                if (m.drs_k[(p * 4 + t % 4) * nd + i] != k || m.drs_v[t * nd + i] != s) return false;
            }
    return true;
}

maps_t build_maps(uint32_t b, uint32_t N_TS, uint32_t N_eff_TX, uint32_t N_DF) {
    maps_t m;
    const uint32_t Nb = 64 * b, N = 56 * b, Nf = N + 1, gb = 4 * b;
    m.b = b;
    m.N_TS = N_TS;
    m.N_DF = N_DF;
    m.Nf = Nf;
    m.code.assign((N_DF + 1) * Nf, CODE_NONE);
    // STF (stf.cpp:171-183, 185-285), scale 1.0 as built in tx_rx.cpp:71
    m.stf = stf_values(b, N_eff_TX);
    for (uint32_t k = 0; k < Nf; ++k)
        if (m.stf[k] != cf32(0, 0)) m.code[k] = CODE_STF;
    // DRS tables (drs.cpp:196-254)
    m.drs_k.resize(2 * 4 * (N / 4));
    m.drs_v.resize(8 * (N / 4));
    for (uint32_t par = 0; par < 2; ++par)
        for (uint32_t t = 0; t < 4; ++t)
            for (uint32_t i = 0; i < N / 4; ++i)
                m.drs_k[(par * 4 + t) * (N / 4) + i] =
                    static_cast<uint32_t>(kocc(N, 4 * i + (t + 2 * par) % 4) + static_cast<int>(N / 2));
    for (uint32_t t = 0; t < 8; ++t)
        for (uint32_t i = 0; i < N / 4; ++i)
            m.drs_v[t * (N / 4) + i] = drs_value(t, i);
    m.drs = drs_schedule(N_TS, N_DF);
    for (const auto& d : m.drs)
        for (uint32_t t = d.ts_first; t <= d.ts_last; ++t)
            for (uint32_t i = 0; i < N / 4; ++i) {
                const uint32_t k = m.drs_k[(d.parity * 4 + t % 4) * (N / 4) + i];
                const bool neg = m.drs_v[t * (N / 4) + i] < 0;
                m.code[d.l * Nf + k] = CODE_DRS | t | (neg ? 8u : 0u);
            }
    // PCC (pcc.cpp)
    const auto pl = pcc_linear(b, N_TS);
    for (uint32_t j = 0; j < pl.size(); ++j) {
        const uint32_t l = pl[j] / Nb, k = pl[j] % Nb - gb;
        if (m.pcc_l.empty() || m.pcc_l.back() != l) {
            m.pcc_l.push_back(l);
            m.pcc_sym_off.push_back(j);
        }
        m.pcc_k.push_back(k);
        if (l <= N_DF) m.code[l * Nf + k] = CODE_PCC | j;
    }
    m.pcc_sym_off.push_back(static_cast<uint32_t>(pl.size()));
    // PDC (pdc.cpp:31-153, 217-300): repetition pattern of a 30-symbol u=8 virtual packet
    auto vf = virtual_frame(b, N_TS, 30);
    for (uint32_t x : pl) vf[x] = 0;
    std::vector<std::vector<uint32_t>> rep(21);
    for (uint32_t l = 1; l <= 20; ++l)
        for (uint32_t i = 0; i < Nb; ++i)
            if (vf[l * Nb + i]) rep[l].push_back(i - gb);
    for (uint32_t l = 0; l < rep.size(); ++l)
        if (l != 10 && rep[l].size() == N) rep[l].resize(1);
    const uint32_t l_limit = N_TS <= 2 ? 6 : 11;
    m.pdc_sym_off.assign(N_DF + 2, 0);
    uint32_t j = 0;
    for (uint32_t l = 0; l <= N_DF; ++l) {
        m.pdc_sym_off[l] = j;
        if (l == 0) continue;
        uint32_t le = l <= l_limit ? l : l - ((l - l_limit) / 10) * 10;
        if (rep[le].size() == 1) le = 10;
        for (uint32_t k : rep[le]) {
            m.pdc_k.push_back(k);
            m.code[l * Nf + k] = CODE_PDC | j;
            ++j;
        }
    }
    m.pdc_sym_off[N_DF + 1] = j;
    return m;
}

// ------------------------------------------------------------ beamforming (Tables 6.3.4-1..6)
static const std::vector<std::vector<int8_t>>& Wtab(uint32_t N_TS, uint32_t N_TX) {
    // 2 = j, -2 = -j; row-major [antenna][transmit stream]
    static const std::vector<std::vector<int8_t>> w11 = {{1}};
    static const std::vector<std::vector<int8_t>> w12 = {{1, 0}, {0, 1}, {1, 1}, {1, -1}, {1, 2}, {1, -2}};
    static const std::vector<std::vector<int8_t>> w14 = [] {
        std::vector<std::vector<int8_t>> v = {{1, 0, 0, 0}, {0, 1, 0, 0}, {0, 0, 1, 0}, {0, 0, 0, 1},
                                              {1, 0, 1, 0}, {1, 0, -1, 0}, {1, 0, 2, 0}, {1, 0, -2, 0},
                                              {0, 1, 0, 1}, {0, 1, 0, -1}, {0, 1, 0, 2}, {0, 1, 0, -2}};
        const int8_t ph[4] = {1, 2, -1, -2};  // {1, j, -1, -j}
        auto mul = [](int8_t a, int8_t b) -> int8_t {  // product in {1, j, -1, -j} encoded
            auto idx = [](int8_t x) { return x == 1 ? 0 : x == 2 ? 1 : x == -1 ? 2 : 3; };
            static const int8_t r[4] = {1, 2, -1, -2};
            return r[(idx(a) + idx(b)) % 4];
        };
        for (int p1 = 0; p1 < 4; ++p1)
            for (int p2 = 0; p2 < 4; ++p2) v.push_back({1, ph[p1], ph[p2], mul(ph[p1], ph[p2])});
        return v;
    }();
    static const std::vector<std::vector<int8_t>> w22 = {{1, 0, 0, 1}, {1, 1, 1, -1}, {1, 1, 2, -2}};
    static const std::vector<std::vector<int8_t>> w24 = {
        {1, 0, 0, 1, 0, 0, 0, 0},     {1, 0, 0, 0, 0, 1, 0, 0},     {1, 0, 0, 0, 0, 0, 0, 1},
        {0, 0, 1, 0, 0, 1, 0, 0},     {0, 0, 1, 0, 0, 0, 0, 1},     {0, 0, 0, 0, 1, 0, 0, 1},
        {1, 0, 0, 1, 1, 0, 0, -2},    {1, 0, 0, 1, 1, 0, 0, 2},     {1, 0, 0, 1, -2, 0, 0, 1},
        {1, 0, 0, 1, -2, 0, 0, -1},   {1, 0, 0, 1, -1, 0, 0, -2},   {1, 0, 0, 1, -1, 0, 0, 2},
        {1, 0, 0, 1, 2, 0, 0, 1},     {1, 0, 0, 1, 2, 0, 0, -1},    {1, 1, 1, 1, 1, -1, 1, -1},
        {1, 1, 1, 1, 2, -2, 2, -2},   {1, 1, 2, 2, 1, -1, 2, -2},   {1, 1, 2, 2, 2, -2, -1, 1},
        {1, 1, -1, -1, 1, -1, -1, 1}, {1, 1, -1, -1, 2, -2, -2, 2}, {1, 1, -2, -2, 1, -1, -2, 2},
        {1, 1, -2, -2, 2, -2, 1, -1}};
    static const std::vector<std::vector<int8_t>> w44 = {
        {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1},      {1, 1, 0, 0, 0, 0, 1, 1, 1, -1, 0, 0, 0, 0, 1, -1},
        {1, 1, 0, 0, 0, 0, 1, 1, 2, -2, 0, 0, 0, 0, 2, -2},    {1, 1, 1, 1, 1, -1, 1, -1, 1, 1, -1, -1, 1, -1, -1, 1},
        {1, 1, 1, 1, 1, -1, 1, -1, 2, 2, -2, -2, 2, -2, -2, 2}};
    static const std::vector<std::vector<int8_t>> w88 = [] {
        std::vector<int8_t> e(64, 0);
        for (int i = 0; i < 8; ++i) e[9 * i] = 1;
        return std::vector<std::vector<int8_t>>{e};
    }();
    if (N_TS == 1 && N_TX == 1) return w11;
    if (N_TS == 1 && N_TX == 2) return w12;
    if (N_TS == 1 && N_TX == 4) return w14;
    if (N_TS == 2 && N_TX == 2) return w22;
    if (N_TS == 2 && N_TX == 4) return w24;
    if (N_TS == 4 && N_TX == 4) return w44;
    if (N_TS == 8 && N_TX == 8) return w88;
    throw std::runtime_error("no beamforming matrix for N_TS/N_TX");
}

uint32_t W_codebooks(uint32_t N_TS, uint32_t N_TX) { return static_cast<uint32_t>(Wtab(N_TS, N_TX).size()); }

std::vector<cf32> W_matrix(uint32_t N_TS, uint32_t N_TX, uint32_t cb, float* scaling) {
    const auto& e = Wtab(N_TS, N_TX).at(cb);
    std::vector<cf32> w(e.size());
    float nz = 0.0f;
    for (size_t i = 0; i < e.size(); ++i) {
        w[i] = e[i] == 2 ? cf32(0, 1) : e[i] == -2 ? cf32(0, -1) : cf32(static_cast<float>(e[i]), 0);
        if (e[i] != 0) nz += 1.0f;
    }
    if (scaling) *scaling = 1.0f / std::sqrt(nz);  // beamforming_and_antenna_port_mapping.cpp:307-320
    return w;
}

float W_scaling_optimal_DAC(uint32_t N_TS, uint32_t N_TX, uint32_t cb) {
    (void)Wtab(N_TS, N_TX).at(cb);  // throws for an undefined matrix
    const float r2 = 1.0f / std::sqrt(2.0f), r4 = 1.0f / std::sqrt(4.0f);
    if (N_TS == 2 && N_TX == 2) return cb == 0 ? 1.0f : r2;   // {1, 1/sqrt2, 1/sqrt2}
    if (N_TS == 2 && N_TX == 4) return cb < 14 ? 1.0f : r2;   // 14 x 1, 8 x 1/sqrt2
    if (N_TS == 4 && N_TX == 4) return cb == 0 ? 1.0f : cb < 3 ? r2 : r4;  // {1, r2, r2, r4, r4}
    return 1.0f;  // SISO, N_TS = 1 (N_TX 2 / 4), N_TS = 8
}

uint32_t txdiv_modulo(uint32_t N_TS) { return N_TS <= 2 ? 1u : N_TS == 4 ? 6u : 12u; }

void txdiv_pair(uint32_t N_TS, uint32_t i, uint32_t& A, uint32_t& B) {
    static const uint8_t P4[6][2] = {{0, 1}, {2, 3}, {0, 2}, {1, 3}, {0, 3}, {1, 2}};
    static const uint8_t P8[12][2] = {{0, 1}, {2, 3}, {4, 5}, {6, 7}, {0, 4}, {1, 5},
                                      {2, 6}, {3, 7}, {0, 2}, {1, 3}, {4, 6}, {5, 7}};
    i %= txdiv_modulo(N_TS);
    A = N_TS <= 2 ? 0u : N_TS == 4 ? P4[i][0] : P8[i][0];
    B = N_TS <= 2 ? 1u : N_TS == 4 ? P4[i][1] : P8[i][1];
}

// ------------------------------------------------------------ Gold sequence (TS 36.211 §7.2)
std::vector<uint8_t> gold_bits_packed(uint32_t c_init, uint32_t nbits) {
    std::vector<uint8_t> out((nbits + 7) / 8, 0);
    uint32_t x1 = 1, x2 = c_init & 0x7FFFFFFFu;  // 31-bit LFSR states, bit i = x(n+i)
    for (uint32_t n = 0; n < 1600 + nbits; ++n) {
        if (n >= 1600) {
            const uint32_t i = n - 1600;
            if ((x1 ^ x2) & 1u) out[i / 8] |= static_cast<uint8_t>(0x80u >> (i % 8));
        }
        const uint32_t f1 = ((x1 >> 3) ^ x1) & 1u;
        const uint32_t f2 = ((x2 >> 3) ^ (x2 >> 2) ^ (x2 >> 1) ^ x2) & 1u;
        x1 = (x1 >> 1) | (f1 << 30);
        x2 = (x2 >> 1) | (f2 << 30);
    }
    return out;
}

// ------------------------------------------------------------ filters (phy/filter/*.cpp)
static double bessel8(double z, bool modified) {  // bessel.cpp:27-55 (8-term series)
    double r = 0.0, fac = 1.0;
    for (int k = 0; k <= 8; ++k) {
        if (k) fac *= k;
        r += std::pow(modified ? 0.25 * z * z : -0.25 * z * z, static_cast<double>(k)) / (fac * fac);
    }
    return r;
}
static float sincf_ref(float n) {  // rectangular.cpp:26
    return n == 0.0f ? 1.0f : static_cast<float>(std::sin(M_PI * n) / (M_PI * n));
}

static std::vector<float> kaiser_lpf(float fp, float fs, float ripple_dB, float att_dB) {  // kaiser.cpp:35-122
    const float delta = std::min(std::pow(10.0f, -att_dB / 20.0f), std::pow(10.0f, ripple_dB / 20.0f) - 1.0f);
    const float A = -20.0f * std::log10(delta);
    float beta = 0.0f;
    if (A > 50.0f)
        beta = 0.1102f * (A - 8.7f);
    else if (A >= 21.0f)
        beta = static_cast<float>(0.5842f * std::pow(A - 21.0f, 0.4f) + 0.07886 * (A - 21.0f));
    const float tb = fs - fp;
    const float order = static_cast<float>((A - 7.95f) / (2.285f * 2.0f * M_PI * tb));
    uint32_t N = static_cast<uint32_t>(std::ceil(order + 1.0f));
    if (N % 2 == 0) ++N;
    const float fc = fp + tb / 2.0f;
    const float i0b = static_cast<float>(bessel8(beta, true));
    std::vector<float> h(N);
    float norm = 0.0f;
    for (uint32_t n = 0; n < N; ++n) {
        const float Nf = static_cast<float>(N), nf = static_cast<float>(n);
        const float w = static_cast<float>(bessel8(beta * std::sqrt(1.0f - std::pow(2.0f * nf / (Nf - 1.0f) - 1.0f, 2.0f)), true)) / i0b;
        h[n] = w * (2.0f * fc * sincf_ref(2.0f * fc * (nf - (Nf - 1.0f) / 2.0f)));
        norm += h[n];
    }
    for (auto& x : h) x /= norm;
    return h;
}

resampler_t make_resampler(uint32_t L, uint32_t M, uint32_t os_min, uint32_t user) {  // resampler.cpp:56-160
    resampler_t r;
    r.L = L;
    r.M = M;
    if (L == 1 && M == 1) {
        r.h = {1.0f};
        return r;
    }
    // resampler_param.hpp:77-88 filter of this user and oversampling (resampler.cpp:74-95)
    const uint32_t o = prm::rs_os_index(os_min);
    const float LM = static_cast<float>(std::max(L, M));
    auto h = kaiser_lpf(prm::RS_F_PASS[user][o] / LM, prm::RS_F_STOP[user][o] / LM, prm::RS_RIPPLE_DONT_CARE,
                        prm::RS_ATT_DB[user][o]);
    r.delay = static_cast<uint32_t>((h.size() - 1) / 2);
    for (auto& x : h) x *= static_cast<float>(L);
    const uint32_t padded = static_cast<uint32_t>((h.size() + L - 1) / L * L);
    h.resize(padded, 0.0f);
    r.taps = padded / L;
    r.hl = r.taps - 1;
    r.h = h;
    return r;
}

// ------------------------------------------------------------ Wiener LUTs (channel_lut.cpp, wiener.hpp)
float lut_profile_snr_db(uint32_t p) {
    return static_cast<float>(prm::RX_SNR_DB[p]);  // RX_SYNCED_PARAM_SNR_DB_VEC (rx_synced_param.hpp:216-232)
}

namespace {
struct pt {
    double f, t;
};
struct stats_t {
    double duf, Ts, nu, tau, sigma;
};
double corr(const pt& a, const pt& b, const stats_t& s) {  // channel_statistics.cpp:27-33
    const float rf = sincf_ref(static_cast<float>(M_PI) * static_cast<float>(s.tau) * static_cast<float>((a.f - b.f) * s.duf));
    const float rt = static_cast<float>(bessel8(2.0f * static_cast<float>(M_PI) * static_cast<float>(s.nu) *
                                                    static_cast<float>((a.t - b.t) * s.Ts), false));
    return static_cast<double>(rf) * static_cast<double>(rt);
}
// Cholesky solve of the SPD Wiener-Hopf system (equals the reference's least-norm COD solution
// for these full-rank matrices)
std::vector<double> chol_solve(std::vector<double> A, std::vector<double> y, uint32_t n) {
    for (uint32_t j = 0; j < n; ++j) {
        double d = A[j * n + j];
        for (uint32_t k = 0; k < j; ++k) d -= A[j * n + k] * A[j * n + k];
        d = std::sqrt(d);
        A[j * n + j] = d;
        for (uint32_t i = j + 1; i < n; ++i) {
            double s = A[i * n + j];
            for (uint32_t k = 0; k < j; ++k) s -= A[i * n + k] * A[j * n + k];
            A[i * n + j] = s / d;
        }
    }
    for (uint32_t i = 0; i < n; ++i) {
        double s = y[i];
        for (uint32_t k = 0; k < i; ++k) s -= A[i * n + k] * y[k];
        y[i] = s / A[i * n + i];
    }
    for (int i = static_cast<int>(n) - 1; i >= 0; --i) {
        double s = y[i];
        for (uint32_t k = i + 1; k < n; ++k) s -= A[k * n + i] * y[k];
        y[i] = s / A[i * n + i];
    }
    return y;
}

void lut_fill(uint32_t Nsv, uint32_t b, const stats_t& st, uint32_t n, lut_t* out,
              std::vector<std::vector<float>>& vecs) {
    const uint32_t N = 56 * b, Nf = N + 1, T = Nsv + 1;
    if (out) {
        out->T = T;
        out->n = n;
        out->Nf = Nf;
        out->pilot_weight.assign(T * 4 * Nf, 0);
    }
    auto kdrs = [&](uint32_t t, uint32_t par, uint32_t i) {
        return static_cast<double>(kocc(N, 4 * i + (t + 2 * par) % 4) + static_cast<int>(N / 2));
    };
    for (uint32_t ts = 0; ts < 4; ++ts) {
        std::vector<pt> cv;  // s0_calc_drs_pilot_vec
        for (uint32_t i = 0; i < N / 4; ++i) {
            if (Nsv == 0) {
                cv.push_back({kdrs(ts, 0, i), 1.0});
            } else if (ts <= 1) {
                cv.push_back({kdrs(ts, 0, i), 1.0});
                cv.push_back({kdrs(ts, 1, i), 1.0 + Nsv});
            } else {
                cv.push_back({kdrs(ts, 1, i), 1.0 + Nsv});
                cv.push_back({kdrs(ts, 0, i), 1.0});
            }
        }
        for (uint32_t t = 1; t <= T; ++t) {
            uint32_t prev = 0;
            std::vector<double> R(n * n);
            for (uint32_t f = 0; f < Nf; ++f) {
                const pt D{static_cast<double>(f), static_cast<double>(t)};
                double best = 1e9;
                uint32_t opt = 0;
                for (uint32_t i = prev; i + n <= cv.size(); ++i) {  // s1_find_opt_idx_pilot
                    double s = 0.0;
                    for (uint32_t j = i; j < i + n; ++j)
                        s += std::sqrt(std::pow(D.f - cv[j].f, 2.0) + std::pow(D.t - cv[j].t, 2.0));
                    if (s < best) {
                        best = s;
                        opt = i;
                    }
                    if (s > best * prm::RX_LUT_SEARCH_ABORT) break;
                }
                if (f == 0 || opt != prev)
                    for (uint32_t r = 0; r < n; ++r)
                        for (uint32_t c = 0; c < n; ++c)
                            R[r * n + c] = corr(cv[opt + r], cv[opt + c], st) + (r == c ? st.sigma : 0.0);
                std::vector<double> rdp(n);
                for (uint32_t r = 0; r < n; ++r) rdp[r] = corr(D, cv[opt + r], st);
                const auto w = chol_solve(R, rdp, n);
                double sum = 0.0;
                for (double x : w) sum += x;
                std::vector<float> wf(n);
                for (uint32_t r = 0; r < n; ++r) wf[r] = static_cast<float>(w[r] / sum);
                int known = -1;  // s3_find_weight_vec_index: first vector within 1e-4
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
                    known = static_cast<int>(vecs.size()) - 1;
                }
                if (out) out->pilot_weight[((t - 1) * 4 + ts) * Nf + f] = opt | (static_cast<uint32_t>(known) << 16);
                prev = opt;
            }
        }
    }
}
}  // namespace

lut_t build_lut(uint32_t Nsv, uint32_t b, uint32_t b_max, uint32_t u_max, uint32_t profile) {
    stats_t st{27000.0 * u_max, 72.0 / 64.0 / (27000.0 * u_max), prm::RX_NU_MAX_HZ[profile], prm::RX_TAU_RMS_SEC[profile],
               1.0 / std::pow(10.0, static_cast<double>(lut_profile_snr_db(profile)) / 10.0)};
    const uint32_t n = Nsv > 0 ? prm::RX_N_INTERP_LR[profile] : prm::RX_N_INTERP_L[profile];
    std::vector<std::vector<float>> vecs;
    if (b != b_max) lut_fill(Nsv, b_max, st, n, nullptr, vecs);
    lut_t L;
    lut_fill(Nsv, b, st, n, &L, vecs);
    L.weights.reserve(vecs.size() * n);
    for (const auto& v : vecs) L.weights.insert(L.weights.end(), v.begin(), v.end());
    return L;
}

// ------------------------------------------------------------ RX schedules
void build_rx_ops(const maps_t& m, uint32_t N_eff_TX, uint32_t N_DF, bool mode_lr, uint32_t stride,
                  std::vector<op_t>& pcc_ops, std::vector<op_t>& pdc_ops, uint32_t& pcc_max) {
    pcc_ops.clear();
    pdc_ops.clear();
    const uint32_t N_step = N_eff_TX <= 2 ? 5 : 10, ps_len = N_eff_TX <= 2 ? 6 : 11;
    uint32_t drs_i = 0;
    auto is_drs = [&](uint32_t l) { return drs_i < m.drs.size() && m.drs[drs_i].l == l; };
    auto has_pdc = [&](uint32_t l) { return m.pdc_sym_off[l + 1] > m.pdc_sym_off[l]; };
    pcc_max = m.pcc_l.back();
    // phase 1 (rx_synced.cpp:283-302): mode l, ps 0
    uint32_t rel = 0, l = 1, pcc_sym = 0, ps_idx = 0;
    std::vector<op_t> replay;  // DRS/event ops phase 2 must replay to rebuild its state
    for (; l <= pcc_max; ++l) {
        if (is_drs(l)) {
            const op_t d{OP_DRS, l, drs_i, rel, 0}, e{OP_EVENT, 0, rel, 0, m.drs[drs_i].ts_first};
            pcc_ops.push_back(d);
            pcc_ops.push_back(e);
            replay.push_back(d);
            replay.push_back(e);
            ++drs_i;
        }
        if (pcc_sym < m.pcc_l.size() && m.pcc_l[pcc_sym] == l) {
            pcc_ops.push_back({OP_PCC, l, pcc_sym, 0, 0});
            ++pcc_sym;
        }
        ++rel;
    }
    pdc_ops = replay;
    // phase 2, mode lr (rx_synced.cpp:1028-1110)
    const uint32_t nof_full_ps = (N_DF - (ps_len - N_step)) / N_step;
    if (mode_lr && nof_full_ps > 0) {
        while (ps_idx < nof_full_ps) {
            const uint32_t first = 1 + ps_idx * N_step, last = ps_len + ps_idx * N_step;
            if (ps_idx > 0) rel = 1;
            for (; l <= last; ++l) {
                if (is_drs(l)) pdc_ops.push_back({OP_DRS, l, drs_i++, rel, ps_idx});
                ++rel;
            }
            const uint32_t start = ps_idx == 0 ? 0 : 1;
            for (rel = start; rel <= N_step; ++rel) {
                if ((rel - start) % stride == 0) pdc_ops.push_back({OP_EVENT, 1, rel, ps_idx, 0});
                if (has_pdc(first + rel)) pdc_ops.push_back({OP_PDC, first + rel, 0, 0, 0});
            }
            ++ps_idx;
            rel = 0;
        }
    }
    // phase 2, mode l (rx_synced.cpp:1112-1163)
    if (ps_idx == 0) {
        for (uint32_t i = 1; i < l; ++i)
            if (has_pdc(i)) pdc_ops.push_back({OP_PDC, i, 0, 0, 0});
        rel = l - 1;
    }
    for (; l <= N_DF; ++l) {
        if (is_drs(l)) {
            pdc_ops.push_back({OP_DRS, l, drs_i, rel, ps_idx});
            pdc_ops.push_back({OP_EVENT, 0, rel, ps_idx, m.drs[drs_i].ts_first});
            ++drs_i;
        }
        if (has_pdc(l)) pdc_ops.push_back({OP_PDC, l, 0, 0, 0});
        ++rel;
        if (rel == N_step) {
            ++ps_idx;
            rel = 0;
        }
    }
}

rx_plan_t build_rx_plan(const maps_t& m, const std::vector<op_t>& ops, uint32_t NT, bool pair_units) {
    rx_plan_t p;
    uint16_t src[4][2];
    for (auto& r : src) r[0] = r[1] = RX_SRC_NONE;
    uint32_t drs_off = 0, drs_cnt = 0;
    bool dirty = true;
    rx_seg_t ev{};
    const bool pairs = NT > 1 && pair_units;
    auto units = [&](const rx_seg_t& s) { return pairs ? (s.j1 - s.j0) / 2 : s.j1 - s.j0; };
    auto add = [&](rx_seg_t s) {
        if (s.j1 <= s.j0) return;
        if (dirty || p.epochs.empty()) {
            rx_epoch_t e{};
            std::memcpy(e.src, src, sizeof(src));
            e.seg0 = e.seg1 = static_cast<uint32_t>(p.segs.size());
            p.epochs.push_back(e);
            dirty = false;
        }
        auto& e = p.epochs.back();
        if (s.kind == OP_PDC && e.seg1 > e.seg0) {  // extend a run of PDC symbols on the same event
            auto& b = p.segs.back();
            if (b.kind == OP_PDC && b.j1 == s.j0 && b.mode == s.mode && b.rel == s.rel && b.swap == s.swap &&
                b.off == s.off && b.drs_cnt == s.drs_cnt) {
                e.units -= units(b);
                b.j1 = s.j1;
                e.units += units(b);
                return;
            }
        }
        s.u0 = e.units;
        e.units += units(s);
        p.segs.push_back(s);
        e.seg1 = static_cast<uint32_t>(p.segs.size());
    };
    for (const auto& op : ops) {
        if (op.kind == OP_DRS) {
            const auto& d = m.drs[op.b];
            const uint32_t dop = static_cast<uint32_t>(p.dl.size());
            p.dl.push_back(d.l);
            p.dmeta.push_back(d.ts_first | (d.ts_last << 8) | (d.parity << 16));
            drs_off = 0;
            for (uint32_t t = d.ts_first; t <= d.ts_last; ++t) {  // channel_antenna.hpp:38-63 write offsets
                const uint32_t rel = op.c, ps = op.d;
                const bool lhs = rel <= 1, hi = (t & 3u) >= 2;
                const uint32_t off = (ps % 2 == 0) ? (lhs ? hi : !hi) : (lhs ? !hi : hi);
                drs_off |= off << t;
                src[t][off] = static_cast<uint16_t>(dop);
            }
            ++drs_cnt;
            dirty = true;
        } else if (op.kind == OP_EVENT) {
            ev.mode = op.a;
            ev.rel = op.b;
            ev.swap = (op.c & 1u) ? 2u : 0u;
            ev.off = drs_off;
            ev.drs_cnt = drs_cnt;
        } else if (op.kind == OP_PCC) {
            rx_seg_t s = ev;
            s.kind = OP_PCC;
            s.l = op.a;
            s.j0 = m.pcc_sym_off[op.b];
            s.j1 = m.pcc_sym_off[op.b + 1];
            add(s);
        } else if (op.kind == OP_PDC) {
            rx_seg_t s = ev;
            s.kind = OP_PDC;
            s.l = op.a;
            s.j0 = m.pdc_sym_off[op.a];
            s.j1 = m.pdc_sym_off[op.a + 1];
            add(s);
        }
    }
    return p;
}

}  // namespace dnrp::geo
