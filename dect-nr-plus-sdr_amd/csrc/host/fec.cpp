// fec.cpp — DECT NR+ channel coding on the host (see fec.hpp), behind the C-ABI in dnrp.h:
//   dnrp_fec_cbsegm    <- sp3::fix::srsran_cbsegm_FIX        (sections_part3/fix/cbsegm.cpp:65-123)
//   dnrp_pcc_encode    <- pcc_enc_encode up to scrambling     (phy/fec/pcc_enc.cpp:145-208)
//   dnrp_pcc_decode    <- pcc_enc_decode after descrambling   (phy/fec/pcc_enc.cpp:215-364)
//   dnrp_pdc_encode    <- pdc_encode_codeblocks w/o scrambling(phy/fec/pdc_enc.cpp:127-229)
//   dnrp_pdc_decode    <- pdc_decode_codeblocks w/o descramb. (phy/fec/pdc_enc.cpp:291-492)
//   dnrp_harq_rx_*     <- harq::buffer_rx_t softbuffer (cb softbits, cb CRC flags, cb data)
// Scrambling is not repeated here: dnrp_tx_batch scrambles the d-bits and dnrp_rx_pcc/pdc_batch
// descramble the LLRs (the library's boundary, pcc_enc.cpp:212,297 / pdc_enc.cpp:220,339-344).
#include "fec.hpp"

#include <algorithm>
#include <array>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>

#include "ctx_internal.hpp"
#include "dnrp.h"
#include "fec_dev.hpp"

namespace dnrp::fec {

// TS 36.212 Table 5.1.3-3: (f1, f2) of the QPP interleaver for each code-block size K. The K column
// itself follows from the table's steps (8 up to 512, 16 up to 1024, 32 up to 2048, 64 up to 6144)
// and is pinned against the reference's tc_cb_sizes (cbsegm.cpp:34-46, tests/golden/ref_fec.json);
// every (f1, f2) row is checked to be a permutation (tests/test_fec_host.py).
static const uint16_t kQpp[kNofCbSizes][2] = {
    {3, 10},    {7, 12},    {19, 42},   {7, 16},    {7, 18},    {11, 20},   {5, 22},    {11, 24},
    {7, 26},    {41, 84},   {103, 90},  {15, 32},   {9, 34},    {17, 108},  {9, 38},    {21, 120},
    {101, 84},  {21, 44},   {57, 46},   {23, 48},   {13, 50},   {27, 52},   {11, 36},   {27, 56},
    {85, 58},   {29, 60},   {33, 62},   {15, 32},   {17, 198},  {33, 68},   {103, 210}, {19, 36},
    {19, 74},   {37, 76},   {19, 78},   {21, 120},  {21, 82},   {115, 84},  {193, 86},  {21, 44},
    {133, 90},  {81, 46},   {45, 94},   {23, 48},   {243, 98},  {151, 40},  {155, 102}, {25, 52},
    {51, 106},  {47, 72},   {91, 110},  {29, 168},  {29, 114},  {247, 58},  {29, 118},  {89, 180},
    {91, 122},  {157, 62},  {55, 84},   {31, 64},   {17, 66},   {35, 68},   {227, 420}, {65, 96},
    {19, 74},   {37, 76},   {41, 234},  {39, 80},   {185, 82},  {43, 252},  {21, 86},   {155, 44},
    {79, 120},  {139, 92},  {23, 94},   {217, 48},  {25, 98},   {17, 80},   {127, 102}, {25, 52},
    {239, 106}, {17, 48},   {137, 110}, {215, 112}, {29, 114},  {15, 58},   {147, 118}, {29, 60},
    {59, 122},  {65, 124},  {55, 84},   {31, 64},   {17, 66},   {171, 204}, {67, 140},  {35, 72},
    {19, 74},   {39, 76},   {19, 78},   {199, 240}, {21, 82},   {211, 252}, {21, 86},   {43, 88},
    {149, 60},  {45, 92},   {49, 846},  {71, 48},   {13, 28},   {17, 80},   {25, 102},  {183, 104},
    {55, 954},  {127, 96},  {27, 110},  {29, 112},  {29, 114},  {57, 116},  {45, 354},  {31, 120},
    {59, 610},  {185, 124}, {113, 420}, {31, 64},   {17, 66},   {171, 136}, {209, 420}, {253, 216},
    {367, 444}, {265, 456}, {181, 468}, {39, 80},   {27, 164},  {127, 504}, {143, 172}, {43, 88},
    {29, 300},  {45, 92},   {157, 188}, {47, 96},   {13, 28},   {111, 240}, {443, 204}, {51, 104},
    {51, 212},  {451, 192}, {257, 220}, {57, 336},  {313, 228}, {271, 232}, {179, 236}, {331, 120},
    {363, 244}, {375, 248}, {127, 168}, {31, 64},   {33, 130},  {43, 264},  {33, 134},  {477, 408},
    {35, 138},  {233, 280}, {357, 142}, {337, 480}, {37, 146},  {71, 444},  {71, 120},  {37, 152},
    {39, 462},  {127, 234}, {39, 158},  {39, 80},   {31, 96},   {113, 902}, {41, 166},  {251, 336},
    {43, 170},  {21, 86},   {43, 174},  {45, 176},  {45, 178},  {161, 120}, {89, 182},  {323, 184},
    {47, 186},  {23, 94},   {47, 190},  {263, 480}};

uint32_t cb_size(uint32_t idx) {
    if (idx < 60) return 40 + 8 * idx;
    if (idx < 92) return 528 + 16 * (idx - 60);
    if (idx < 124) return 1056 + 32 * (idx - 92);
    if (idx < kNofCbSizes) return 2112 + 64 * (idx - 124);
    return 0;
}

int cb_index(uint32_t long_cb) {
    for (uint32_t j = 0; j < kNofCbSizes; ++j)
        if (cb_size(j) >= long_cb) return (int)j;
    return -1;
}

void qpp_params(uint32_t idx, uint32_t* f1, uint32_t* f2) {
    *f1 = idx < kNofCbSizes ? kQpp[idx][0] : 0;
    *f2 = idx < kNofCbSizes ? kQpp[idx][1] : 0;
}

// Per code-block size: QPP permutation and the rate-matching circular-buffer map. Built once.
struct SizeTables {
    std::vector<uint32_t> pi;    // QPP interleaver
    std::vector<int32_t> wmap;   // circular buffer position -> stream * (K + 4) + index, -1 = dummy bit
    uint32_t R = 0, Kpi = 0;
};
static std::array<SizeTables, kNofCbSizes> g_tab;
static std::array<std::once_flag, kNofCbSizes> g_once;

// TS 36.212 §5.1.4.1.1 inter-column permutation of the 32-column sub-block interleaver
static const uint8_t kPerm[32] = {0, 16, 8,  24, 4, 20, 12, 28, 2, 18, 10, 26, 6, 22, 14, 30,
                                  1, 17, 9,  25, 5, 21, 13, 29, 3, 19, 11, 27, 7, 23, 15, 31};

static const SizeTables& tables(uint32_t idx) {
    std::call_once(g_once[idx], [idx] {
        SizeTables& t = g_tab[idx];
        const uint32_t K = cb_size(idx);
        t.pi.resize(K);
        const uint64_t f1 = kQpp[idx][0], f2 = kQpp[idx][1];
        for (uint64_t i = 0; i < K; ++i) t.pi[i] = (uint32_t)((f1 * i + f2 * i * i) % K);
        const uint32_t D = K + 4;
        t.R = (D + 31) / 32;
        t.Kpi = 32 * t.R;
        const uint32_t ND = t.Kpi - D;
        t.wmap.assign(3 * t.Kpi, -1);
        for (uint32_t k = 0; k < t.Kpi; ++k) {
            const uint32_t y01 = kPerm[k / t.R] + 32 * (k % t.R);             // streams 0 and 1
            const uint32_t y2 = (kPerm[k / t.R] + 32 * (k % t.R) + 1) % t.Kpi;  // stream 2
            if (y01 >= ND) {
                t.wmap[k] = (int32_t)(y01 - ND);
                t.wmap[t.Kpi + 2 * k] = (int32_t)(D + y01 - ND);
            }
            if (y2 >= ND) t.wmap[t.Kpi + 2 * k + 1] = (int32_t)(2 * D + y2 - ND);
        }
    });
    return g_tab[idx];
}

const std::vector<uint32_t>& qpp(uint32_t idx) { return tables(idx).pi; }

static uint32_t rm_k0(const SizeTables& t, uint32_t rv);

// circular-buffer list of a size (non-dummy positions in buffer order: stream << 16 | index) and
// the list index where soft bit 0 of redundancy version rv lands
static std::vector<uint32_t> valid_list(uint32_t idx) {
    const SizeTables& t = tables(idx);
    const uint32_t D = cb_size(idx) + 4;
    std::vector<uint32_t> v;
    v.reserve(3 * D);
    for (int32_t m : t.wmap)
        if (m >= 0) v.push_back(((uint32_t)m / D) << 16 | ((uint32_t)m % D));
    return v;
}
static uint32_t valid_start(uint32_t idx, uint32_t rv) {
    const SizeTables& t = tables(idx);
    const uint32_t k0 = rm_k0(t, rv) % (3 * t.Kpi);
    uint32_t n = 0;
    for (uint32_t pos = 0; pos < k0; ++pos) n += t.wmap[pos] >= 0;
    return n;
}

int cbsegm(uint32_t tbs, uint32_t Z, Segm* s) {
    std::memset(s, 0, sizeof(*s));
    s->Z = Z;
    if (tbs == 0) return 0;
    const uint32_t B = tbs + 24;
    s->tbs = tbs;
    uint32_t Bp;
    if (B <= Z) {
        s->C = 1;
        Bp = B;
    } else {
        if (Z <= 24) return -1;
        s->C = (B + (Z - 24) - 1) / (Z - 24);
        Bp = B + 24 * s->C;
    }
    const int i1 = cb_index((Bp - 1) / s->C + 1);
    if (i1 < 0) return -1;
    s->K1 = cb_size((uint32_t)i1);
    s->K1_idx = (uint32_t)i1;
    if (s->C == 1) {
        s->C1 = 1;
    } else {
        if (i1 == 0) return -1;
        s->K2 = cb_size((uint32_t)i1 - 1);
        s->K2_idx = (uint32_t)i1 - 1;
        s->C2 = (s->C * s->K1 - Bp) / (s->K1 - s->K2);
        s->C1 = s->C - s->C2;
    }
    s->F = s->C1 * s->K1 + s->C2 * s->K2 - Bp;
    return 0;
}

uint32_t crc_bits(const uint8_t* data, uint32_t nbits, uint32_t poly, uint32_t len) {
    const uint32_t mask = (len == 32) ? 0xFFFFFFFFu : ((1u << len) - 1);
    uint32_t reg = 0;
    uint32_t i = 0;
    if (len >= 8) {
        // byte-wise (MSB first) over the whole bytes
        static thread_local uint32_t tab[256], tab_poly = 0, tab_len = 0;
        if (tab_poly != poly || tab_len != len) {
            for (uint32_t b = 0; b < 256; ++b) {
                uint32_t r = b << (len - 8);
                for (int k = 0; k < 8; ++k) r = (r & (1u << (len - 1))) ? ((r << 1) ^ poly) & mask : (r << 1) & mask;
                tab[b] = r;
            }
            tab_poly = poly;
            tab_len = len;
        }
        for (; i + 8 <= nbits; i += 8) reg = ((reg << 8) & mask) ^ tab[((reg >> (len - 8)) ^ data[i / 8]) & 0xFF];
    }
    for (; i < nbits; ++i) {
        const uint32_t bit = (data[i / 8] >> (7 - i % 8)) & 1;
        const uint32_t top = (reg >> (len - 1)) & 1;
        reg = (reg << 1) & mask;
        if (top ^ bit) reg ^= poly;
    }
    return reg;
}

// ---- turbo encoder (TS 36.212 §5.1.3.2): g0 = 1 + D^2 + D^3 feedback, g1 = 1 + D + D^3 ----------
static void rsc(const uint8_t* in, const uint32_t* pi, uint32_t K, uint8_t* z, uint8_t tx[3], uint8_t tz[3]) {
    uint32_t s1 = 0, s2 = 0, s3 = 0;
    for (uint32_t k = 0; k < K; ++k) {
        const uint32_t c = pi ? in[pi[k]] : in[k];
        const uint32_t a = c ^ s2 ^ s3;
        z[k] = (uint8_t)(a ^ s1 ^ s3);
        s3 = s2;
        s2 = s1;
        s1 = a;
    }
    for (int t = 0; t < 3; ++t) {  // trellis termination: input = feedback, register fills with 0
        tx[t] = (uint8_t)(s2 ^ s3);
        tz[t] = (uint8_t)(s1 ^ s3);
        s3 = s2;
        s2 = s1;
        s1 = 0;
    }
}

void turbo_encode(const uint8_t* c, uint32_t idx, uint8_t* d0, uint8_t* d1, uint8_t* d2) {
    const uint32_t K = cb_size(idx);
    const auto& pi = tables(idx).pi;
    uint8_t x1[3], z1[3], x2[3], z2[3];
    std::memcpy(d0, c, K);
    rsc(c, nullptr, K, d1, x1, z1);
    rsc(c, pi.data(), K, d2, x2, z2);
    d0[K] = x1[0], d0[K + 1] = z1[1], d0[K + 2] = x2[0], d0[K + 3] = z2[1];
    d1[K] = z1[0], d1[K + 1] = x1[2], d1[K + 2] = z2[0], d1[K + 3] = x2[2];
    d2[K] = x1[1], d2[K + 1] = z1[2], d2[K + 2] = x2[1], d2[K + 3] = z2[2];
}

// ---- rate matching (TS 36.212 §5.1.4.1) -----------------------------------------------------------
uint32_t rm_kw(uint32_t idx) { return 3 * tables(idx).Kpi; }

static uint32_t rm_k0(const SizeTables& t, uint32_t rv) {
    const uint32_t Ncb = 3 * t.Kpi;  // no soft-buffer limitation (srsran_rm_turbo_tx_lut)
    return t.R * (2 * ((Ncb + 8 * t.R - 1) / (8 * t.R)) * rv + 2);
}

void rm_tx(const uint8_t* d0, const uint8_t* d1, const uint8_t* d2, uint32_t idx, uint32_t E, uint32_t rv,
           uint8_t* e) {
    const SizeTables& t = tables(idx);
    const uint32_t D = cb_size(idx) + 4, Ncb = 3 * t.Kpi;
    uint32_t pos = rm_k0(t, rv) % Ncb;
    for (uint32_t k = 0; k < E;) {
        const int32_t m = t.wmap[pos];
        if (m >= 0) {
            const uint32_t s = (uint32_t)m / D, i = (uint32_t)m % D;
            e[k++] = s == 0 ? d0[i] : (s == 1 ? d1[i] : d2[i]);
        }
        if (++pos == Ncb) pos = 0;
    }
}

void rm_rx(const int16_t* e, uint32_t idx, uint32_t E, uint32_t rv, int16_t* w) {
    const SizeTables& t = tables(idx);
    const uint32_t Ncb = 3 * t.Kpi;
    uint32_t pos = rm_k0(t, rv) % Ncb;
    for (uint32_t k = 0; k < E;) {
        if (t.wmap[pos] >= 0) {
            const int32_t v = (int32_t)w[pos] + e[k++];
            w[pos] = (int16_t)std::min(32767, std::max(-32768, v));
        }
        if (++pos == Ncb) pos = 0;
    }
}

void rm_deinterleave(const int16_t* w, uint32_t idx, int32_t* d0, int32_t* d1, int32_t* d2) {
    const SizeTables& t = tables(idx);
    const uint32_t D = cb_size(idx) + 4;
    for (uint32_t pos = 0; pos < 3 * t.Kpi; ++pos) {
        const int32_t m = t.wmap[pos];
        if (m < 0) continue;
        const uint32_t s = (uint32_t)m / D, i = (uint32_t)m % D;
        (s == 0 ? d0 : (s == 1 ? d1 : d2))[i] = w[pos];
    }
}

// ---- max-log-MAP decoder --------------------------------------------------------------------------
// State s = 4 s1 + 2 s2 + s3 (s1 = newest register bit). LLRs: positive = bit 1. Branch metric of
// input u / parity p: u (L_sys + L_apriori) + p L_par (the max-log metric up to a per-step constant).
// Integer arithmetic throughout, so the device decoder reproduces it bit for bit.
static constexpr int32_t kNeg = -(1 << 28);
static inline void trans(uint32_t s, uint32_t u, uint32_t* next, uint32_t* p) {
    const uint32_t s1 = (s >> 2) & 1, s2 = (s >> 1) & 1, s3 = s & 1;
    const uint32_t a = u ^ s2 ^ s3;
    *p = a ^ s1 ^ s3;
    *next = (a << 2) | (s1 << 1) | s2;
}

// One constituent decoder over K steps + 3 tail steps. A[k] = systematic + a priori, B[k] = parity,
// tx/tz = tail systematic / parity. Writes the full LLR into llr and the extrinsic into le.
static void map_decode(uint32_t K, const int32_t* A, const int32_t* B, const int32_t* tx, const int32_t* tz,
                       int32_t* alpha, int32_t* llr, int32_t* le) {
    int32_t* al = alpha;
    for (int s = 0; s < 8; ++s) al[s] = s == 0 ? 0 : kNeg;
    for (uint32_t k = 0; k < K; ++k) {
        const int32_t* a0 = al + 8 * k;
        int32_t* a1 = al + 8 * (k + 1);
        for (int s = 0; s < 8; ++s) a1[s] = kNeg;
        for (uint32_t s = 0; s < 8; ++s)
            for (uint32_t u = 0; u < 2; ++u) {
                uint32_t nx, p;
                trans(s, u, &nx, &p);
                const int32_t v = a0[s] + (u ? A[k] : 0) + (p ? B[k] : 0);
                a1[nx] = std::max(a1[nx], v);
            }
        int32_t mx = a1[0];
        for (int s = 1; s < 8; ++s) mx = std::max(mx, a1[s]);
        for (int s = 0; s < 8; ++s) a1[s] = std::max(a1[s] - mx, kNeg);
    }
    // backward through the termination (input forced to the feedback value, register fills with 0)
    int32_t be[8], bn[8];
    for (int s = 0; s < 8; ++s) be[s] = s == 0 ? 0 : kNeg;
    for (int t = 2; t >= 0; --t) {
        for (uint32_t s = 0; s < 8; ++s) {
            const uint32_t u = ((s >> 1) ^ s) & 1;  // s2 ^ s3
            uint32_t nx, p;
            trans(s, u, &nx, &p);
            bn[s] = be[nx] + (u ? tx[t] : 0) + (p ? tz[t] : 0);
        }
        int32_t mx = bn[0];
        for (int s = 1; s < 8; ++s) mx = std::max(mx, bn[s]);
        for (int s = 0; s < 8; ++s) be[s] = std::max(bn[s] - mx, kNeg);
    }
    for (int64_t k = (int64_t)K - 1; k >= 0; --k) {
        const int32_t* a0 = al + 8 * k;
        int32_t m1 = INT32_MIN, m0 = INT32_MIN;
        for (uint32_t s = 0; s < 8; ++s) {
            int32_t b = INT32_MIN;
            for (uint32_t u = 0; u < 2; ++u) {
                uint32_t nx, p;
                trans(s, u, &nx, &p);
                const int32_t g = (u ? A[k] : 0) + (p ? B[k] : 0);
                const int32_t v = a0[s] + g + be[nx];
                if (u) m1 = std::max(m1, v); else m0 = std::max(m0, v);
                b = std::max(b, g + be[nx]);
            }
            bn[s] = b;
        }
        llr[k] = m1 - m0;
        const int32_t e = llr[k] - A[k];
        le[k] = std::min(32767, std::max(-32767, (e * 3) >> 2));  // extrinsic x3/4, int16 range
        int32_t mx = bn[0];
        for (int s = 1; s < 8; ++s) mx = std::max(mx, bn[s]);
        for (int s = 0; s < 8; ++s) be[s] = std::max(bn[s] - mx, kNeg);
    }
}

void Tdec::load(const int16_t* w, uint32_t idx_) {
    idx = idx_;
    K = cb_size(idx);
    std::vector<int32_t> d0(K + 4), d1(K + 4), d2(K + 4);
    rm_deinterleave(w, idx, d0.data(), d1.data(), d2.data());
    sys.assign(d0.begin(), d0.begin() + K);
    p1.assign(d1.begin(), d1.begin() + K);
    p2.assign(d2.begin(), d2.begin() + K);
    // tails: encoder 1 (x, z) x3 then encoder 2 (x', z') x3 (TS 36.212 §5.1.3.2.2)
    tail = {d0[K], d2[K], d1[K + 1], d1[K], d0[K + 1], d2[K + 1],
            d0[K + 2], d2[K + 2], d1[K + 3], d1[K + 2], d0[K + 3], d2[K + 3]};
    le1.assign(K, 0);
    le2.assign(K, 0);
    llr.assign(K, 0);
    alpha.resize(8 * (K + 1));
}

void Tdec::iterate(uint8_t* bits) {
    const auto& pi = tables(idx).pi;
    std::vector<int32_t> A(K), Ai(K), tmp(K);
    // decoder 1: a priori = deinterleaved extrinsic of decoder 2
    for (uint32_t i = 0; i < K; ++i) tmp[pi[i]] = le2[i];
    for (uint32_t k = 0; k < K; ++k) A[k] = sys[k] + tmp[k];
    map_decode(K, A.data(), p1.data(), &tail[0], &tail[3], alpha.data(), llr.data(), le1.data());
    // decoder 2 on the interleaved sequence
    for (uint32_t i = 0; i < K; ++i) Ai[i] = sys[pi[i]] + le1[pi[i]];
    map_decode(K, Ai.data(), p2.data(), &tail[6], &tail[9], alpha.data(), llr.data(), le2.data());
    for (uint32_t i = 0; i < K; ++i) bits[pi[i]] = llr[i] > 0;
}

}  // namespace dnrp::fec

// ==== C-ABI =========================================================================================
using namespace dnrp::fec;

static void pack_bits(const uint8_t* u, uint32_t n, uint8_t* out, uint32_t bit_off) {
    for (uint32_t i = 0; i < n; ++i) {
        const uint32_t b = bit_off + i;
        if (u[i]) out[b / 8] |= (uint8_t)(0x80 >> (b % 8));
        else out[b / 8] &= (uint8_t)~(0x80 >> (b % 8));
    }
}
static void unpack_bits(const uint8_t* p, uint32_t bit_off, uint32_t n, uint8_t* u) {
    for (uint32_t i = 0; i < n; ++i) u[i] = (p[(bit_off + i) / 8] >> (7 - (bit_off + i) % 8)) & 1;
}

struct dnrp_harq_rx {
    uint32_t C_max, Kw_max, K_max;
    std::vector<int16_t> w;      // [C_max][Kw_max] accumulated softbits (softbuffer->buffer_f)
    std::vector<uint8_t> crc;    // [C_max] code-block CRC ok (softbuffer->cb_crc)
    std::vector<uint8_t> data;   // [C_max][K_max/8] decoded code blocks kept for retransmissions
};

static int segm_of(const dnrp_fec_cfg* cfg, Segm* s) {
    if (!cfg || cfg->N_bps == 0 || cfg->N_TB_bits == 0 || cfg->N_TB_bits % 8 || cfg->rv > 3) return DNRP_EINVAL;
    if (cbsegm(cfg->N_TB_bits, cfg->Z, s) != 0) return DNRP_ECONFIG;
    if (s->F != 0) return DNRP_ECONFIG;  // filler bits not supported (pdc_enc.cpp:144)
    return DNRP_OK;
}

// E of code block r (pdc_enc.cpp:148-175)
static uint32_t cb_E(const Segm& s, uint32_t r, uint32_t Qm, uint32_t G) {
    const uint32_t Gp = G / Qm, gamma = Gp % s.C;
    return r <= s.C - gamma - 1 ? Qm * (Gp / s.C) : Qm * ((Gp + s.C - 1) / s.C);
}

extern "C" {

int dnrp_fec_cbsegm(uint32_t N_TB_bits, uint32_t Z, dnrp_cbsegm* out) {
    if (!out) return DNRP_EINVAL;
    Segm s;
    if (cbsegm(N_TB_bits, Z, &s) != 0) return DNRP_ECONFIG;
    *out = {s.tbs, s.Z, s.C, s.C1, s.C2, s.K1, s.K2, s.K1_idx, s.K2_idx, s.F};
    return DNRP_OK;
}

int dnrp_fec_cb_size(uint32_t idx, uint32_t* K, uint32_t* f1, uint32_t* f2) {
    if (idx >= kNofCbSizes || !K) return DNRP_EINVAL;
    *K = cb_size(idx);
    uint32_t a, b;
    qpp_params(idx, &a, &b);
    if (f1) *f1 = a;
    if (f2) *f2 = b;
    return DNRP_OK;
}

int dnrp_crc(const uint8_t* data, uint32_t nbits, uint32_t kind, uint32_t* crc) {
    if (!data || !crc) return DNRP_EINVAL;
    switch (kind) {
        case DNRP_CRC16: *crc = crc_bits(data, nbits, kCrc16, 16); break;
        case DNRP_CRC24A: *crc = crc_bits(data, nbits, kCrc24A, 24); break;
        case DNRP_CRC24B: *crc = crc_bits(data, nbits, kCrc24B, 24); break;
        default: return DNRP_EINVAL;
    }
    return DNRP_OK;
}

int dnrp_pcc_encode(const uint8_t* plcf, uint32_t plcf_type, uint32_t closed_loop, uint32_t beamforming,
                    uint8_t* d) {
    if (!plcf || !d || (plcf_type != 1 && plcf_type != 2)) return DNRP_EINVAL;
    const uint32_t nb = plcf_type == 1 ? kPlcfType1Bits : kPlcfType2Bits;
    uint8_t c_packed[12] = {0};
    std::memcpy(c_packed, plcf, nb / 8);
    const uint16_t mask = closed_loop ? (beamforming ? kMaskClBf : kMaskCl) : (beamforming ? kMaskBf : kMaskNone);
    const uint32_t crc = crc_bits(c_packed, nb, kCrc16, 16) ^ mask;
    c_packed[nb / 8] = (uint8_t)(crc >> 8);
    c_packed[nb / 8 + 1] = (uint8_t)crc;
    const uint32_t idx = (uint32_t)cb_index(nb + 16);  // K = 56 / 96: no filler bits
    const uint32_t K = cb_size(idx);
    std::vector<uint8_t> c(K), d0(K + 4), d1(K + 4), d2(K + 4), e(kPccBits);
    unpack_bits(c_packed, 0, K, c.data());
    turbo_encode(c.data(), idx, d0.data(), d1.data(), d2.data());
    rm_tx(d0.data(), d1.data(), d2.data(), idx, kPccBits, 0, e.data());  // rv 0 (TS 103 636-3 §7.5.3)
    std::memset(d, 0, 25);
    pack_bits(e.data(), kPccBits, d, 0);
    return DNRP_OK;
}

int dnrp_pcc_decode(const int16_t* llr, uint32_t plcf_type_test, uint8_t* plcf, uint32_t* closed_loop,
                    uint32_t* beamforming, uint32_t* iterations) {
    if (!llr || !plcf || (plcf_type_test != 1 && plcf_type_test != 2)) return DNRP_EINVAL;
    const uint32_t nb = plcf_type_test == 1 ? kPlcfType1Bits : kPlcfType2Bits;
    const uint32_t idx = (uint32_t)cb_index(nb + 16);
    const uint32_t K = cb_size(idx);
    std::vector<int16_t> w(rm_kw(idx), 0);
    rm_rx(llr, idx, kPccBits, 0, w.data());
    Tdec dec;
    dec.load(w.data(), idx);
    std::vector<uint8_t> bits(K);
    uint8_t packed[12];
    for (uint32_t it = 1; it <= kPccMaxIter; ++it) {
        dec.iterate(bits.data());
        std::memset(packed, 0, sizeof(packed));
        pack_bits(bits.data(), K, packed, 0);
        const uint32_t rx = ((uint32_t)packed[nb / 8] << 8) | packed[nb / 8 + 1];
        const uint32_t re = crc_bits(packed, nb, kCrc16, 16);
        const uint16_t masks[4] = {kMaskNone, kMaskCl, kMaskBf, kMaskClBf};  // pcc_enc.cpp:329-349
        for (int m = 0; m < 4; ++m)
            if ((rx ^ masks[m]) == re) {
                std::memcpy(plcf, packed, nb / 8);
                if (closed_loop) *closed_loop = (m & 1) != 0;
                if (beamforming) *beamforming = (m & 2) != 0;
                if (iterations) *iterations = it;
                return 1;
            }
    }
    if (iterations) *iterations = kPccMaxIter;
    return 0;
}

int dnrp_pdc_encode(const dnrp_fec_cfg* cfg, const uint8_t* tb, uint8_t* d) {
    Segm s;
    int rc = segm_of(cfg, &s);
    if (rc) return rc;
    if (!tb || !d) return DNRP_EINVAL;
    const uint32_t tbs = cfg->N_TB_bits, Qm = cfg->N_bps, G = cfg->G;
    // b = a || CRC24A (TS 36.212 §5.1.1), segmented K- blocks first (pdc_enc.cpp:159-165)
    std::vector<uint8_t> b(tbs + 24);
    unpack_bits(tb, 0, tbs, b.data());
    const uint32_t tcrc = crc_bits(tb, tbs, kCrc24A, 24);
    for (int i = 0; i < 24; ++i) b[tbs + i] = (tcrc >> (23 - i)) & 1;
    std::memset(d, 0, (G + 7) / 8);
    std::vector<uint8_t> c, d0, d1, d2, e, cpk;
    uint32_t rp = 0, wp = 0;
    for (uint32_t r = 0; r < s.C; ++r) {
        const uint32_t K = r < s.C2 ? s.K2 : s.K1, idx = r < s.C2 ? s.K2_idx : s.K1_idx;
        const uint32_t rlen = s.C > 1 ? K - 24 : K;
        c.assign(b.begin() + rp, b.begin() + rp + rlen);
        if (s.C > 1) {  // code-block CRC24B
            cpk.assign((rlen + 7) / 8, 0);
            pack_bits(c.data(), rlen, cpk.data(), 0);
            const uint32_t cc = crc_bits(cpk.data(), rlen, kCrc24B, 24);
            for (int i = 0; i < 24; ++i) c.push_back((cc >> (23 - i)) & 1);
        }
        d0.resize(K + 4), d1.resize(K + 4), d2.resize(K + 4);
        turbo_encode(c.data(), idx, d0.data(), d1.data(), d2.data());
        const uint32_t E = cb_E(s, r, Qm, G);
        e.resize(E);
        rm_tx(d0.data(), d1.data(), d2.data(), idx, E, cfg->rv, e.data());
        pack_bits(e.data(), E, d, wp);
        rp += rlen;
        wp += E;
    }
    return DNRP_OK;
}

int dnrp_harq_rx_create(uint32_t N_TB_bits_max, uint32_t Z, dnrp_harq_rx** out) {
    if (!out) return DNRP_EINVAL;
    Segm s;
    if (cbsegm(N_TB_bits_max, Z, &s) != 0 || s.C == 0) return DNRP_ECONFIG;
    // C of any smaller TB <= C of the largest; size the blocks for the largest code block of Z
    const int imax = cb_index(std::min<uint32_t>(Z, 6144));
    if (imax < 0) return DNRP_ECONFIG;
    auto* h = new dnrp_harq_rx;
    h->C_max = s.C;
    h->Kw_max = rm_kw((uint32_t)imax);
    h->K_max = cb_size((uint32_t)imax);
    h->w.assign((size_t)h->C_max * h->Kw_max, 0);
    h->crc.assign(h->C_max, 0);
    h->data.assign((size_t)h->C_max * (h->K_max / 8), 0);
    *out = h;
    return DNRP_OK;
}

int dnrp_harq_rx_reset(dnrp_harq_rx* h) {
    if (!h) return DNRP_EINVAL;
    std::fill(h->w.begin(), h->w.end(), 0);
    std::fill(h->crc.begin(), h->crc.end(), 0);
    return DNRP_OK;
}

int dnrp_harq_rx_destroy(dnrp_harq_rx* h) {
    delete h;
    return DNRP_OK;
}

int dnrp_pdc_decode(dnrp_harq_rx* hb, const dnrp_fec_cfg* cfg, const int16_t* llr, uint32_t n_llr, uint8_t* tb,
                    uint32_t* iterations) {
    Segm s;
    int rc = segm_of(cfg, &s);
    if (rc) return rc;
    if (!llr || !tb || n_llr > cfg->G) return DNRP_EINVAL;
    std::unique_ptr<dnrp_harq_rx, int (*)(dnrp_harq_rx*)> own(nullptr, dnrp_harq_rx_destroy);
    if (!hb) {  // one-shot decode: a fresh softbuffer
        dnrp_harq_rx* h = nullptr;
        if ((rc = dnrp_harq_rx_create(cfg->N_TB_bits, cfg->Z, &h))) return rc;
        own.reset(h);
        hb = h;
    }
    if (s.C > hb->C_max || rm_kw(s.K1_idx) > hb->Kw_max) return DNRP_EINVAL;
    const uint32_t tbs = cfg->N_TB_bits, Qm = cfg->N_bps, G = cfg->G;
    std::vector<uint8_t> data((tbs + 48 + 7) / 8 + 8, 0), bits;
    Tdec dec;
    uint32_t it_total = 0, wp = 0, r = 0;
    for (; r < s.C; ++r) {
        const uint32_t K = r < s.C2 ? s.K2 : s.K1, idx = r < s.C2 ? s.K2_idx : s.K1_idx;
        const uint32_t rlen = s.C == 1 ? K : K - 24;
        // read positions as srsRAN's decode_tb_cb (pdc_enc.cpp:322-332): the block at index
        // C - gamma is read with the shorter length although it was written with Qm more bits
        const uint32_t Gp = G / Qm, gamma = Gp % s.C, n_e = Qm * (Gp / s.C);
        uint32_t rpos = r * n_e, n_e2 = n_e;
        if (r > s.C - gamma) {
            n_e2 = n_e + Qm;
            rpos = (s.C - gamma) * n_e + (r - (s.C - gamma)) * n_e2;
        }
        if (rpos + n_e2 > n_llr) break;  // not enough soft bits yet (pdc_enc.cpp:334-337)
        int16_t* w = &hb->w[(size_t)r * hb->Kw_max];
        uint8_t* keep = &hb->data[(size_t)r * (hb->K_max / 8)];
        if (!hb->crc[r]) {
            rm_rx(llr + rpos, idx, n_e2, cfg->rv, w);
            dec.load(w, idx);
            bits.resize(K);
            std::vector<uint8_t> pk((K + 7) / 8);
            for (uint32_t it = 1; it <= kPdcMaxIter; ++it) {
                dec.iterate(bits.data());
                ++it_total;
                std::fill(pk.begin(), pk.end(), 0);
                pack_bits(bits.data(), K, pk.data(), 0);
                const bool ok = s.C > 1 ? crc_bits(pk.data(), K, kCrc24B, 24) == 0
                                        : crc_bits(pk.data(), tbs + 24, kCrc24A, 24) == 0;
                if (ok && it >= kPdcMinIter) {
                    hb->crc[r] = 1;
                    break;
                }
            }
            pack_bits(bits.data(), K, data.data(), wp);
            if (hb->crc[r]) std::memcpy(keep, pk.data(), rlen / 8);
        } else {
            std::vector<uint8_t> kb(rlen);
            unpack_bits(keep, 0, rlen, kb.data());
            pack_bits(kb.data(), rlen, data.data(), wp);
        }
        wp += rlen;
    }
    if (iterations) *iterations = it_total;
    std::memcpy(tb, data.data(), tbs / 8);
    if (r < s.C) return 0;
    for (uint32_t i = 0; i < s.C; ++i)
        if (!hb->crc[i]) return 0;
    if (s.C == 1) return 1;
    // all code blocks passed: check the transport-block CRC (pdc_enc.cpp:478-488)
    const uint32_t tcrc = crc_bits(data.data(), tbs, kCrc24A, 24);
    uint32_t rx = 0;
    for (int i = 0; i < 24; ++i) rx = (rx << 1) | ((data[(tbs + i) / 8] >> (7 - (tbs + i) % 8)) & 1);
    if (tcrc == rx) return 1;
    std::fill(hb->crc.begin(), hb->crc.begin() + s.C, 0);  // false alarm: reset the CB CRC flags
    return 0;
}

}  // extern "C"

// ---- device turbo decoding -----------------------------------------------------------------------
// PDC decoding runs the first 3 iterations for every code block, then continues the undecided ones in
// dense waves (run_tdec; same-box A/B at 5 dB: a split after 2 / 3 / 4 iterations 156 / 145 / 161 ms
// per 4096 C4 TBs, one pass 0.95 s, docs/DESIGN_LOG.md §5a)
static uint32_t pdc_split() { return 3u; }

static int fec_tables(dnrp_ctx* ctx) {
    if (!ctx->fec_valid_off.empty()) return DNRP_OK;
    std::vector<uint32_t> tab, voff(kNofCbSizes), st(kNofCbSizes * 4);
    for (uint32_t idx = 0; idx < kNofCbSizes; ++idx) {
        const auto v = valid_list(idx);
        voff[idx] = (uint32_t)tab.size();
        tab.insert(tab.end(), v.begin(), v.end());
        for (uint32_t rv = 0; rv < 4; ++rv) st[idx * 4 + rv] = valid_start(idx, rv);
    }
    if (!ctx->fec_tab.upload(tab)) return DNRP_ENOMEM;
    ctx->fec_valid_off = voff, ctx->fec_start = st;
    return DNRP_OK;
}

// Groups code blocks of equal size into waves (up to ~3 GB of scratch per launch group) and runs
// de-matching + turbo iterations; cb_pkt receives the packet of each code block in launch order
// (the order of ctx->fec_cbout).
static int run_tdec(dnrp_ctx* ctx, const std::vector<std::vector<dnrp::dev::FecCb>>& by_idx,
                    const std::vector<std::vector<uint32_t>>& pkt_of, const int16_t* llr, uint8_t* tb,
                    uint32_t max_iter, uint32_t min_iter, uint32_t split, hipStream_t s, std::vector<uint32_t>& cb_pkt,
                    std::vector<uint32_t>& cb_out, int16_t* sb = nullptr, uint8_t* flags = nullptr) {
    using namespace dnrp::dev;
    std::vector<FecCb> cbs;
    std::vector<FecWave> waves;
    std::vector<uint32_t> grp_first_wave{0}, grp_first_cb{0};
    uint64_t data = 0, ck = 0;
    // one launch should hold every wave (the kernel is latency-bound: waves resident together
    // overlap): scratch per launch group up to half the free device memory, at most 32 GiB
    size_t mem_free = 0, mem_total = 0;
    (void)hipMemGetInfo(&mem_free, &mem_total);
    const uint64_t kMaxGroupBytes = std::min<uint64_t>(32ull << 30, std::max<uint64_t>(1ull << 30, mem_free / 2));
    for (uint32_t idx = 0; idx < kNofCbSizes; ++idx) {
        const auto& v = by_idx[idx];
        const uint32_t K = cb_size(idx);
        const uint64_t wave_bytes = (uint64_t)K * 64 * 11 + (uint64_t)(K / FEC_WIN) * 8 * 64 * 4;
        for (size_t c0 = 0; c0 < v.size(); c0 += 64) {
            if (data * 11 / 5 + ck * 4 + wave_bytes > kMaxGroupBytes) {  // new group (work16 + bits + ck)
                grp_first_wave.push_back((uint32_t)waves.size());
                grp_first_cb.push_back((uint32_t)cbs.size());
                data = ck = 0;
            }
            FecWave w{};
            w.data_off = data, w.ck_off = ck, w.K = K;
            w.n = (uint32_t)std::min<size_t>(64, v.size() - c0);
            w.valid_off = ctx->fec_valid_off[idx];
            qpp_params(idx, &w.f1, &w.f2);
            w.first_cb = (uint32_t)cbs.size() - grp_first_cb.back();
            const uint32_t wrel = (uint32_t)waves.size() - grp_first_wave.back();
            for (uint32_t l = 0; l < w.n; ++l) {
                FecCb cb = v[c0 + l];
                cb.wave = wrel, cb.lane = l;
                cbs.push_back(cb);
                cb_pkt.push_back(pkt_of[idx][c0 + l]);
            }
            waves.push_back(w);
            data += (uint64_t)5 * K * 64;
            ck += (uint64_t)(K / FEC_WIN) * 8 * 64;
        }
    }
    grp_first_wave.push_back((uint32_t)waves.size());
    grp_first_cb.push_back((uint32_t)cbs.size());
    // per-group scratch sized for the largest group
    uint64_t max_data = 0, max_ck = 0;
    for (size_t g = 0; g + 1 < grp_first_wave.size(); ++g) {
        const uint32_t w1 = grp_first_wave[g + 1] - 1;
        if (grp_first_wave[g + 1] == grp_first_wave[g]) continue;
        max_data = std::max<uint64_t>(max_data, waves[w1].data_off + (uint64_t)5 * waves[w1].K * 64);
        max_ck = std::max<uint64_t>(max_ck, waves[w1].ck_off + (uint64_t)(waves[w1].K / FEC_WIN) * 8 * 64);
    }
    const uint32_t n_grp_waves_max = [&] {
        uint32_t mx = 0;
        for (size_t g = 0; g + 1 < grp_first_wave.size(); ++g) mx = std::max(mx, grp_first_wave[g + 1] - grp_first_wave[g]);
        return mx;
    }();
    if (!ctx->fec_cbs.upload(cbs) || !ctx->fec_waves.upload(waves) || !ctx->fec_work16.ensure(max_data * 2) ||
        !ctx->fec_bits.ensure(max_data / 5 + 16) || !ctx->fec_ck.ensure(max_ck * 4 + 16) ||
        !ctx->fec_tail.ensure((size_t)n_grp_waves_max * 12 * 64 * 4 + 16) || !ctx->fec_cbout.ensure(cbs.size() * 4 + 16))
        return DNRP_ENOMEM;
    // Every launch group runs the first `split` iterations for all its code blocks, then the blocks
    // still undecided are gathered densely into new waves and continue from their state (a wave
    // otherwise runs until its slowest lane stops: at marginal SNR one failing block in 64 held
    // the other 63 to the maximum). Same iterations, same results as one pass.
    cb_out.assign(cbs.size(), 0);
    for (size_t g = 0; g + 1 < grp_first_wave.size(); ++g) {
        FecArgs A{};
        A.llr = llr, A.tb = tb, A.tab = ctx->fec_tab.as<uint32_t>();
        A.cbs = ctx->fec_cbs.as<FecCb>() + grp_first_cb[g];
        A.waves = ctx->fec_waves.as<FecWave>() + grp_first_wave[g];
        A.work16 = ctx->fec_work16.as<int16_t>(), A.tail = ctx->fec_tail.as<int32_t>();
        A.bits = ctx->fec_bits.as<uint8_t>(), A.ck = ctx->fec_ck.as<int32_t>();
        A.cb_out = ctx->fec_cbout.as<uint32_t>() + grp_first_cb[g];
        A.n_cb = grp_first_cb[g + 1] - grp_first_cb[g];
        A.n_waves = grp_first_wave[g + 1] - grp_first_wave[g];
        const bool two = split > 0 && split < max_iter;
        A.max_iter = two ? split : max_iter, A.min_iter = min_iter, A.it_first = 1, A.final_pass = two ? 0 : 1;
        A.sb = sb, A.flags = flags;
        ctx->tic("fec_dematch", s);
        if (launch_fec_dematch(A, s)) return DNRP_EDEVICE;
        ctx->toc("fec_dematch", s);
        ctx->tic("fec_tdec", s);
        if (launch_fec_tdec(A, A.n_waves, s)) return DNRP_EDEVICE;
        ctx->toc("fec_tdec", s);
        uint32_t* out = cb_out.data() + grp_first_cb[g];
        HIPCHK(hipMemcpyAsync(out, A.cb_out, (size_t)A.n_cb * 4, hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
        if (!two) continue;
        // undecided blocks of the group -> dense waves per size (the group's waves are size-ordered)
        std::vector<FecCb> cbs2;
        std::vector<FecWave> waves2;
        std::vector<uint32_t> src_of, slot;
        uint64_t d2 = 0, c2 = 0;
        for (uint32_t wi = 0; wi < A.n_waves; ++wi) {
            const FecWave& ow = waves[grp_first_wave[g] + wi];
            for (uint32_t l = 0; l < ow.n; ++l) {
                const uint32_t c = ow.first_cb + l;  // group-relative
                if (!(out[c] & 8u)) continue;
                if (waves2.empty() || waves2.back().K != ow.K || waves2.back().n == 64) {
                    FecWave nw = ow;
                    nw.data_off = d2, nw.ck_off = c2, nw.n = 0, nw.first_cb = (uint32_t)cbs2.size();
                    waves2.push_back(nw);
                    d2 += (uint64_t)5 * ow.K * 64;
                    c2 += (uint64_t)(ow.K / FEC_WIN) * 8 * 64;
                }
                FecCb cb = cbs[grp_first_cb[g] + c];
                cb.wave = (uint32_t)waves2.size() - 1, cb.lane = waves2.back().n++;
                cbs2.push_back(cb);
                src_of.push_back(wi << 6 | l);
                slot.push_back(c);
            }
        }
        if (cbs2.empty()) continue;
        if (!ctx->fec_cbs2.upload(cbs2) || !ctx->fec_waves2.upload(waves2) || !ctx->fec_map2.upload(src_of) ||
            !ctx->fec_work16b.ensure(d2 * 2 + 16) || !ctx->fec_tailb.ensure(waves2.size() * 12 * 64 * 4 + 16) ||
            !ctx->fec_cbout2.ensure(cbs2.size() * 4 + 16))
            return DNRP_ENOMEM;
        FecCompactArgs Cp{};
        Cp.src16 = A.work16, Cp.src_tail = A.tail, Cp.src_waves = A.waves;
        Cp.dst16 = ctx->fec_work16b.as<int16_t>(), Cp.dst_tail = ctx->fec_tailb.as<int32_t>();
        Cp.dst_waves = ctx->fec_waves2.as<FecWave>(), Cp.src_of = ctx->fec_map2.as<uint32_t>();
        if (launch_fec_compact(Cp, (uint32_t)waves2.size(), s)) return DNRP_EDEVICE;
        FecArgs B = A;
        B.cbs = ctx->fec_cbs2.as<FecCb>(), B.waves = ctx->fec_waves2.as<FecWave>();
        B.work16 = ctx->fec_work16b.as<int16_t>(), B.tail = ctx->fec_tailb.as<int32_t>();
        B.cb_out = ctx->fec_cbout2.as<uint32_t>();
        B.n_cb = (uint32_t)cbs2.size(), B.n_waves = (uint32_t)waves2.size();
        B.max_iter = max_iter, B.it_first = split + 1, B.final_pass = 1;
        ctx->tic("fec_tdec", s);
        if (launch_fec_tdec(B, B.n_waves, s)) return DNRP_EDEVICE;
        ctx->toc("fec_tdec", s);
        std::vector<uint32_t> o2(cbs2.size());
        HIPCHK(hipMemcpyAsync(o2.data(), B.cb_out, o2.size() * 4, hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
        for (size_t j = 0; j < o2.size(); ++j) out[slot[j]] = o2[j];
    }
    return DNRP_OK;
}

static int pdc_decode_batch(dnrp_ctx* ctx, uint32_t m, const dnrp_fec_cfg* cfg, const int16_t* llr, uint32_t llr_stride,
                            uint8_t* tb, uint32_t tb_stride, uint8_t* crc_ok, uint32_t* iterations, void* stream,
                            int16_t* sb, uint64_t sb_stride, uint8_t* flags, uint32_t flag_stride) {
    using namespace dnrp::dev;
    if (!ctx || (m && (!cfg || !llr || !tb || !crc_ok))) return DNRP_EINVAL;
    if (m == 0) return DNRP_OK;
    (void)hipSetDevice(ctx->cfg.device);
    hipStream_t s = static_cast<hipStream_t>(stream);
    int rc = fec_tables(ctx);
    if (rc) return rc;
    // plan: code blocks of every packet (pdc_enc.cpp:316-332), grouped by size
    std::vector<Segm> sg(m);
    std::vector<std::vector<FecCb>> by_idx(kNofCbSizes);
    std::vector<std::vector<uint32_t>> pkt_of(kNofCbSizes);
    for (uint32_t i = 0; i < m; ++i) {
        if ((rc = segm_of(&cfg[i], &sg[i]))) return rc;
        const Segm& g = sg[i];
        const uint32_t tbs = cfg[i].N_TB_bits, Qm = cfg[i].N_bps, G = cfg[i].G;
        if (llr_stride < G || tb_stride < tbs / 8 + 3) return DNRP_EINVAL;
        if (sb && (sb_stride < (uint64_t)g.C * 3 * (g.K1 + 4) || flag_stride < g.C)) return DNRP_EINVAL;
        const uint32_t Gp = G / Qm, gamma = Gp % g.C, n_e = Qm * (Gp / g.C);
        uint32_t wp = 0;
        for (uint32_t r = 0; r < g.C; ++r) {
            const uint32_t K = r < g.C2 ? g.K2 : g.K1, idx = r < g.C2 ? g.K2_idx : g.K1_idx;
            uint32_t rpos = r * n_e, n_e2 = n_e;
            if (r > g.C - gamma) {
                n_e2 = n_e + Qm;
                rpos = (g.C - gamma) * n_e + (r - (g.C - gamma)) * n_e2;
            }
            FecCb cb{};
            cb.llr_off = (uint64_t)i * llr_stride + rpos;
            cb.tb_off = (uint64_t)i * tb_stride + wp / 8;
            cb.E = n_e2;
            cb.start = ctx->fec_start[idx * 4 + cfg[i].rv];
            cb.poly = g.C > 1 ? kCrc24B : kCrc24A;
            cb.out_bytes = g.C > 1 ? (K - 24) / 8 : K / 8;
            cb.sb_off = (uint64_t)i * sb_stride + (uint64_t)r * 3 * (g.K1 + 4);
            cb.flag_off = (uint64_t)i * flag_stride + r;
            by_idx[idx].push_back(cb);
            pkt_of[idx].push_back(i);
            wp += g.C > 1 ? K - 24 : K;
        }
    }
    std::vector<uint32_t> cb_pkt, cb_out;
    if ((rc = run_tdec(ctx, by_idx, pkt_of, llr, tb, kPdcMaxIter, kPdcMinIter, pdc_split(), s, cb_pkt, cb_out, sb, flags)))
        return rc;
    // transport-block CRC of the packets with several code blocks
    std::vector<uint64_t> tb_off;
    std::vector<uint32_t> nbytes, multi;
    for (uint32_t i = 0; i < m; ++i)
        if (sg[i].C > 1) tb_off.push_back((uint64_t)i * tb_stride), nbytes.push_back(cfg[i].N_TB_bits / 8), multi.push_back(i);
    const size_t nm = multi.size();
    std::vector<uint8_t> argbuf(nm * 12 + nm * 4 + 16);
    if (nm) {
        std::memcpy(argbuf.data(), tb_off.data(), nm * 8);
        std::memcpy(argbuf.data() + nm * 8, nbytes.data(), nm * 4);
        if (!ctx->fec_tbarg.upload(argbuf)) return DNRP_ENOMEM;
        FecTbArgs T{};
        T.tb = tb, T.tb_off = ctx->fec_tbarg.as<uint64_t>();
        T.nbytes = reinterpret_cast<const uint32_t*>(ctx->fec_tbarg.as<uint8_t>() + nm * 8);
        T.ok = reinterpret_cast<uint32_t*>(ctx->fec_tbarg.as<uint8_t>() + nm * 12);
        T.n = (uint32_t)nm;
        if (launch_fec_tbcrc(T, s)) return DNRP_EDEVICE;
    }
    std::vector<uint32_t> tb_ok(nm);
    if (nm) HIPCHK(hipMemcpyAsync(tb_ok.data(), ctx->fec_tbarg.as<uint8_t>() + nm * 12, nm * 4, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    std::vector<uint32_t> it(m, 0);
    for (uint32_t i = 0; i < m; ++i) crc_ok[i] = 1;
    for (size_t c = 0; c < cb_out.size(); ++c) {
        it[cb_pkt[c]] += cb_out[c] >> 4;
        if (!(cb_out[c] & 1)) crc_ok[cb_pkt[c]] = 0;
    }
    for (size_t j = 0; j < nm; ++j)
        if (!tb_ok[j]) {
            // every code block passed but the transport block did not: a false alarm, the HARQ flags
            // of the packet are reset (pdc_enc.cpp:484-488)
            if (flags && crc_ok[multi[j]]) HIPCHK(hipMemsetAsync(flags + (size_t)multi[j] * flag_stride, 0, sg[multi[j]].C, s));
            crc_ok[multi[j]] = 0;
        }
    HIPCHK(hipStreamSynchronize(s));
    if (iterations)
        for (uint32_t i = 0; i < m; ++i) iterations[i] = it[i];
    return DNRP_OK;
}

extern "C" int dnrp_pdc_decode_batch(dnrp_ctx* ctx, uint32_t m, const dnrp_fec_cfg* cfg, const int16_t* llr,
                                     uint32_t llr_stride, uint8_t* tb, uint32_t tb_stride, uint8_t* crc_ok,
                                     uint32_t* iterations, void* stream) {
    return pdc_decode_batch(ctx, m, cfg, llr, llr_stride, tb, tb_stride, crc_ok, iterations, stream, nullptr, 0,
                            nullptr, 0);
}

extern "C" int dnrp_pdc_decode_batch_harq(dnrp_ctx* ctx, uint32_t m, const dnrp_fec_cfg* cfg, const int16_t* llr,
                                          uint32_t llr_stride, int16_t* softbuf, uint64_t sb_stride, uint8_t* cb_crc,
                                          uint32_t crc_stride, uint8_t* tb, uint32_t tb_stride, uint8_t* crc_ok,
                                          uint32_t* iterations, void* stream) {
    if (!softbuf || !cb_crc) return DNRP_EINVAL;
    return pdc_decode_batch(ctx, m, cfg, llr, llr_stride, tb, tb_stride, crc_ok, iterations, stream, softbuf,
                            sb_stride, cb_crc, crc_stride);
}

extern "C" int dnrp_pdc_softbuffer_size(uint32_t N_TB_bits, uint32_t Z, uint64_t* entries, uint32_t* n_cb) {
    Segm g;
    if (!entries || cbsegm(N_TB_bits, Z, &g) != 0) return DNRP_EINVAL;
    *entries = (uint64_t)g.C * 3 * (g.K1 + 4);
    if (n_cb) *n_cb = g.C;
    return DNRP_OK;
}

// device encoder planning shared by the PDC and PLCF batches: code blocks in packet order, each at a
// 64-bit aligned offset of the packed scratch; per packet its first block, per block its first bit in
// the packet's d row (kernels/fec.hip fec_encode_kernel, fec_pack_kernel)
struct enc_plan {
    std::vector<dnrp::dev::FecEncCb> cbs;
    std::vector<uint32_t> first, pstart, G;
    std::vector<uint64_t> oo;
    uint64_t bits = 0;
    uint32_t max_bytes = 0;
    bool bytes = true;  // every block starts on a byte of its row and has whole bytes: direct mode
    void add(dnrp::dev::FecEncCb cb, uint32_t ps) {
        // the RSC state map over one lane's chunk (zero input): s = s1 | s2 << 1 | s3 << 2 -> (s2 ^ s3, s1, s2)
        const uint32_t Lc = dnrp::dev::fec_enc_chunk(cb.K);
        cb.mA = 0;
        for (uint32_t b = 0; b < 3; ++b) {
            uint32_t st = 1u << b;
            for (uint32_t i = 0; i < Lc; ++i) st = (((st >> 1) ^ (st >> 2)) & 1u) | ((st & 1u) << 1) | (((st >> 1) & 1u) << 2);
            cb.mA |= st << (3 * b);
        }
        cb.oo = bits;
        cb.pstart = ps;
        bytes = bytes && ps % 8 == 0 && cb.E % 8 == 0;
        bits += (cb.E + 63ull) / 64 * 64;
        oo.push_back(cb.oo);
        pstart.push_back(ps);
        cbs.push_back(cb);
    }
};

// upload the plan and run encoder + pack (tbcrc: per-packet TB CRCs already enqueued, or null)
static int run_encode(dnrp_ctx* ctx, enc_plan& P, const uint8_t* tb, const uint32_t* tbcrc, uint8_t* d, uint32_t d_stride,
                      hipStream_t s) {
    using namespace dnrp::dev;
    const size_t n = P.G.size(), nc = P.cbs.size();
    P.first.push_back(static_cast<uint32_t>(nc));
    std::vector<uint8_t> args((n + 1) * 4 + nc * 4 + nc * 8 + n * 4 + 64);
    uint8_t* ap = args.data();
    const size_t o_first = 0, o_ps = (n + 1) * 4, o_oo = (o_ps + nc * 4 + 7) / 8 * 8, o_G = o_oo + nc * 8;
    std::memcpy(ap + o_first, P.first.data(), (n + 1) * 4);
    std::memcpy(ap + o_ps, P.pstart.data(), nc * 4);
    std::memcpy(ap + o_oo, P.oo.data(), nc * 8);
    std::memcpy(ap + o_G, P.G.data(), n * 4);
    if (!ctx->fec_cbs.upload(P.cbs) || !ctx->fec_bits.ensure(P.bits / 8 + 64) || !ctx->fec_waves.upload(args))
        return DNRP_ENOMEM;
    FecEncArgs E{};
    E.tb = tb, E.tab = ctx->fec_tab.as<uint32_t>(), E.cbs = ctx->fec_cbs.as<FecEncCb>();
    E.tbcrc = tbcrc, E.ebits = ctx->fec_bits.as<uint8_t>();
    if (P.bytes) E.d = d, E.d_stride = d_stride;  // no scratch, no pack
    ctx->tic("fec_encode", s);
    if (launch_fec_encode(E, static_cast<uint32_t>(nc), s)) return DNRP_EDEVICE;
    ctx->toc("fec_encode", s);
    if (P.bytes) {
        HIPCHK(hipStreamSynchronize(s));
        return DNRP_OK;
    }
    const uint8_t* dargs = ctx->fec_waves.as<uint8_t>();
    FecPackArgs K{};
    K.ebits = E.ebits;
    K.cb_first = reinterpret_cast<const uint32_t*>(dargs + o_first);
    K.pstart = reinterpret_cast<const uint32_t*>(dargs + o_ps);
    K.oo = reinterpret_cast<const uint64_t*>(dargs + o_oo);
    K.G = reinterpret_cast<const uint32_t*>(dargs + o_G);
    K.d = d, K.d_stride = d_stride, K.n = static_cast<uint32_t>(n), K.max_bytes = P.max_bytes;
    ctx->tic("fec_pack", s);
    if (launch_fec_pack(K, s)) return DNRP_EDEVICE;
    ctx->toc("fec_pack", s);
    HIPCHK(hipStreamSynchronize(s));
    return DNRP_OK;
}

extern "C" int dnrp_pdc_encode_batch(dnrp_ctx* ctx, uint32_t m, const dnrp_fec_cfg* cfg, const uint8_t* tb,
                                     uint32_t tb_stride, uint8_t* d, uint32_t d_stride, void* stream) {
    using namespace dnrp::dev;
    if (!ctx || (m && (!cfg || !tb || !d))) return DNRP_EINVAL;
    if (m == 0) return DNRP_OK;
    (void)hipSetDevice(ctx->cfg.device);
    hipStream_t s = static_cast<hipStream_t>(stream);
    int rc = fec_tables(ctx);
    if (rc) return rc;
    enc_plan P;
    std::vector<uint64_t> tb_off_all(m);
    std::vector<uint32_t> nbytes(m);
    for (uint32_t i = 0; i < m; ++i) {
        Segm g;
        if ((rc = segm_of(&cfg[i], &g))) return rc;
        const uint32_t tbs = cfg[i].N_TB_bits, Qm = cfg[i].N_bps, G = cfg[i].G;
        if (tb_stride < tbs / 8 || d_stride < (G + 7) / 8) return DNRP_EINVAL;
        nbytes[i] = tbs / 8, tb_off_all[i] = (uint64_t)i * tb_stride;
        P.G.push_back(G);
        P.first.push_back(static_cast<uint32_t>(P.cbs.size()));
        P.max_bytes = std::max(P.max_bytes, (G + 7) / 8);
        uint32_t rp = 0, wp = 0;
        for (uint32_t r = 0; r < g.C; ++r) {
            const uint32_t K = r < g.C2 ? g.K2 : g.K1, idx = r < g.C2 ? g.K2_idx : g.K1_idx;
            FecEncCb cb{};
            cb.tb_off = (uint64_t)i * tb_stride, cb.pkt = i, cb.tbs = tbs;
            cb.rp = rp, cb.rlen = g.C > 1 ? K - 24 : K, cb.E = cb_E(g, r, Qm, G);
            cb.start = ctx->fec_start[idx * 4 + cfg[i].rv], cb.crc24b = g.C > 1;
            cb.K = K, cb.valid_off = ctx->fec_valid_off[idx];
            qpp_params(idx, &cb.f1, &cb.f2);
            P.add(cb, wp);
            rp += cb.rlen;
            wp += cb.E;
        }
    }
    // per-packet TB CRC24A first (fec_tbcrc_kernel), then the encoder and the pack
    std::vector<uint8_t> args(m * (8 + 4 + 4) + 64);
    std::memcpy(args.data(), tb_off_all.data(), m * 8);
    std::memcpy(args.data() + m * 8, nbytes.data(), m * 4);
    if (!ctx->fec_tbarg.upload(args)) return DNRP_ENOMEM;
    uint8_t* dargs = ctx->fec_tbarg.as<uint8_t>();
    uint32_t* tbcrc = reinterpret_cast<uint32_t*>(dargs + m * 12);
    FecTbArgs T{};
    T.tb = tb, T.tb_off = reinterpret_cast<const uint64_t*>(dargs), T.nbytes = reinterpret_cast<const uint32_t*>(dargs + m * 8);
    T.crc_out = tbcrc, T.n = m;
    ctx->tic("fec_tbcrc", s);
    if (launch_fec_tbcrc(T, s)) return DNRP_EDEVICE;
    ctx->toc("fec_tbcrc", s);
    return run_encode(ctx, P, tb, tbcrc, d, d_stride, s);
}

extern "C" int dnrp_pcc_decode_batch(dnrp_ctx* ctx, uint32_t n, const uint32_t* plcf_type_test, const int16_t* llr,
                                     uint32_t llr_stride, uint8_t* plcf, uint32_t plcf_stride, uint8_t* result,
                                     uint32_t* iterations, void* stream) {
    using namespace dnrp::dev;
    if (!ctx || (n && (!plcf_type_test || !llr || !plcf || !result))) return DNRP_EINVAL;
    if (n == 0) return DNRP_OK;
    if (llr_stride < kPccBits || plcf_stride < kPlcfType2Bits / 8) return DNRP_EINVAL;
    (void)hipSetDevice(ctx->cfg.device);
    hipStream_t s = static_cast<hipStream_t>(stream);
    int rc = fec_tables(ctx);
    if (rc) return rc;
    std::vector<std::vector<FecCb>> by_idx(kNofCbSizes);
    std::vector<std::vector<uint32_t>> pkt_of(kNofCbSizes);
    for (uint32_t i = 0; i < n; ++i) {
        const uint32_t t = plcf_type_test[i];
        if (t != 1 && t != 2) return DNRP_EINVAL;
        const uint32_t nb = t == 1 ? kPlcfType1Bits : kPlcfType2Bits, idx = (uint32_t)cb_index(nb + 16);
        FecCb cb{};
        cb.llr_off = (uint64_t)i * llr_stride;
        cb.tb_off = (uint64_t)i * plcf_stride;
        cb.E = kPccBits;
        cb.start = ctx->fec_start[idx * 4];  // rv 0 (TS 103 636-3 §7.5.3)
        cb.poly = kCrc16;                    // CRC16 under the four masks (pcc_enc.cpp:329-349)
        cb.out_bytes = nb / 8;
        by_idx[idx].push_back(cb);
        pkt_of[idx].push_back(i);
    }
    std::vector<uint32_t> cb_pkt, cb_out;
    if ((rc = run_tdec(ctx, by_idx, pkt_of, llr, plcf, kPccMaxIter, 1, 0, s, cb_pkt, cb_out))) return rc;
    for (size_t c = 0; c < cb_out.size(); ++c) {
        const uint32_t i = cb_pkt[c];
        result[i] = (cb_out[c] & 1) ? (uint8_t)(1 + ((cb_out[c] >> 1) & 3)) : 0;
        if (iterations) iterations[i] = cb_out[c] >> 4;
    }
    return DNRP_OK;
}

extern "C" int dnrp_pcc_encode_batch(dnrp_ctx* ctx, uint32_t n, const uint32_t* plcf_type, const uint32_t* closed_loop,
                                     const uint32_t* beamforming, const uint8_t* plcf, uint32_t plcf_stride, uint8_t* d,
                                     uint32_t d_stride, void* stream) {
    using namespace dnrp::dev;
    if (!ctx || (n && (!plcf_type || !plcf || !d))) return DNRP_EINVAL;
    if (n == 0) return DNRP_OK;
    if (d_stride < 25) return DNRP_EINVAL;
    (void)hipSetDevice(ctx->cfg.device);
    hipStream_t s = static_cast<hipStream_t>(stream);
    int rc = fec_tables(ctx);
    if (rc) return rc;
    enc_plan P;
    P.max_bytes = (kPccBits + 7) / 8;
    for (uint32_t i = 0; i < n; ++i) {
        const uint32_t t = plcf_type[i];
        if (t != 1 && t != 2) return DNRP_EINVAL;
        const uint32_t nb = t == 1 ? kPlcfType1Bits : kPlcfType2Bits, idx = (uint32_t)cb_index(nb + 16);
        if (plcf_stride < nb / 8) return DNRP_EINVAL;
        const bool cl = closed_loop && closed_loop[i], bf = beamforming && beamforming[i];
        FecEncCb cb{};
        cb.tb_off = (uint64_t)i * plcf_stride, cb.pkt = i, cb.tbs = nb;
        cb.rp = 0, cb.rlen = nb + 16, cb.E = kPccBits, cb.start = ctx->fec_start[idx * 4];  // rv 0
        cb.crc16 = 1, cb.mask = cl ? (bf ? kMaskClBf : kMaskCl) : (bf ? kMaskBf : kMaskNone);
        cb.K = cb_size(idx), cb.valid_off = ctx->fec_valid_off[idx];
        qpp_params(idx, &cb.f1, &cb.f2);
        P.G.push_back(kPccBits);
        P.first.push_back(static_cast<uint32_t>(P.cbs.size()));
        P.add(cb, 0);
    }
    return run_encode(ctx, P, plcf, nullptr, d, d_stride, s);
}
