// ORACLE — TEST INFRASTRUCTURE ONLY (see oracle.hpp header).
// Scalar restatement of the reference synchronisation of one chunk, sync_chunk_t::search()
// (lib/src/phy/rx/sync/sync_chunk.cpp:143-279), repeated until the chunk is exhausted:
//   sync resampler            rx_pacer.cpp:106-143, sync_chunk.cpp:40-48 (L/M swapped, reset per chunk)
//   autocorrelator_detection  autocorrelator_detection.cpp:107-285, movsum_uw.cpp:55-74, movsum.hpp
//   autocorrelator_peak       autocorrelator_peak.cpp:109-385 (coarse_peak_f_domain disabled:
//                             b = b of the radio device class, integer CFO 0, coarse_peak_f_domain.cpp:51-203)
//   crosscorrelator           crosscorrelator.cpp:80-251, stf_template.cpp:81-206
// The moving sums keep the reference's running-sum/resum schedule in the sample type R (double:
// checker; float: CPU baseline).
#include <algorithm>
#include <cmath>
#include <stdexcept>

#include "oracle.hpp"
#include "oracle_dsp.hpp"
#include "oracle_params.hpp"

namespace orc {

namespace {

const float* const COVER_SEQ = STF_COVER_SEQ;  // stf.hpp:146-151 (cover active)

// movsum.hpp:28-120
template <typename T>
struct movsum_t {
    std::vector<T> reg;
    uint32_t len = 0, ptr = 0;
    T sum{};
    void init(uint32_t n) {
        len = n;
        reg.assign(n, T{});
        ptr = 0;
        sum = T{};
    }
    void pop_push(T v) {
        sum -= reg[ptr];
        sum += v;
        reg[ptr] = v;
        ptr = (ptr + 1) % len;
    }
    void resum() {
        sum = T{};
        for (auto& x : reg) sum += x;
    }
    uint32_t front_idx(uint32_t nbw) const {
        nbw %= len;
        return nbw > ptr ? len - (nbw - ptr) : ptr - nbw;
    }
    T sum_front(uint32_t n) const {
        T r{};
        for (uint32_t i = 0; i < n; ++i) r += reg[front_idx(i)];
        return r;
    }
    T sum_back(uint32_t n) const {
        T r{};
        for (uint32_t i = 0; i < n; ++i) r += reg[(ptr + 1 + i) % len];
        return r;
    }
};

// movsum_uw.cpp:27-123: moving sum with +-1 weights per group of n_rep positions
template <typename C>
struct movsum_uw_t : movsum_t<C> {
    std::vector<float> uw;
    uint32_t n_rep = 1;
    std::vector<uint32_t> pos_neg, neg_pos;
    void init_uw(const std::vector<float>& w, uint32_t rep) {
        uw = w;
        n_rep = rep;
        this->init(static_cast<uint32_t>(w.size()) * rep);
        pos_neg.clear();
        neg_pos.clear();
        const uint32_t n = this->len;
        for (uint32_t i = 1; i < w.size(); ++i) {
            if (w[i - 1] == -1.0f && w[i] == 1.0f) pos_neg.push_back(n - i * rep);
            if (w[i - 1] == 1.0f && w[i] == -1.0f) neg_pos.push_back(n - i * rep);
        }
    }
    void pop_push(C v) {
        auto& reg = this->reg;
        auto& ptr = this->ptr;
        this->sum -= static_cast<typename C::value_type>(uw.front()) * reg[ptr];
        reg[ptr] = v;  // prefactor_push = uw.back() = 1
        this->sum += reg[ptr];
        for (auto nb : pos_neg) this->sum -= static_cast<typename C::value_type>(2) * reg[this->front_idx(nb)];
        for (auto nb : neg_pos) this->sum += static_cast<typename C::value_type>(2) * reg[this->front_idx(nb)];
        ptr = (ptr + 1) % this->len;
    }
    void resum() {
        this->sum = C{};
        for (uint32_t i = 0; i < uw.size(); ++i) {
            const uint32_t B = this->front_idx(this->len - i * n_rep);
            C part{};
            for (uint32_t j = 0; j < n_rep; ++j) part += this->reg[(B + j) % this->len];
            this->sum += static_cast<typename C::value_type>(uw[i]) * part;
        }
    }
};

std::vector<float> cover_pairwise(uint32_t n_pattern) {  // stf.cpp:140-159
    std::vector<float> r(n_pattern - 1);
    for (uint32_t i = 0; i + 1 < n_pattern; ++i) r[i] = COVER_SEQ[i] * COVER_SEQ[i + 1];
    return r;
}

}  // namespace

sync_geom_t sync_geometry(const sync_cfg_t& c) {
    sync_geom_t g;
    g.n_pattern = c.u == 1 ? 7 : 9;
    g.bos = c.b * c.os_min;
    g.stf_len = 16 * g.n_pattern * g.bos;
    g.pattern = g.stf_len / g.n_pattern;
    g.step = g.pattern / prm::STEP_DIVIDER;                          // autocorrelator_detection.cpp:49
    g.A = c.chunk_len / c.L * c.M;                                    // sync_chunk.cpp:63-64
    g.B = static_cast<uint32_t>(prm::OVERLAP_STFS * g.stf_len);      // sync_chunk.cpp:63-66
    g.C = prm::PEAK_REQUEST_PATTERNS * g.pattern;
    g.D = static_cast<uint32_t>(prm::PEAK_MAX_SEARCH_STFS * g.stf_len);  // sync_chunk.cpp:68
    g.search_len = g.A + g.B;
    g.lb_len = g.A + g.B + g.C + g.D;
    g.xc_l = prm::XC_SEARCH_LEFT * c.b * c.os_min * c.L / c.M;        // crosscorrelator.cpp:53-56
    g.xc_len = g.xc_l + prm::XC_SEARCH_RIGHT * c.b * c.os_min * c.L / c.M + 1;
    g.tmpl_len = g.stf_len * c.L / c.M;                                // stf_template.cpp:33
    g.n_templates = c.N_ant >= 8 ? 4 : c.N_ant >= 4 ? 3 : c.N_ant >= 2 ? 2 : 1;
    g.rms_min = static_cast<float>(prm::RMS_MIN * std::sqrt(static_cast<double>(c.u) * c.b * 1728000.0 / prm::RMS_MIN_REF_RATE));
    return g;
}

// stf_template.cpp:81-206: STF of b for N_eff_TX, IFFT + CP, 1/sqrt(N_occ/4), cover, TX resampler
// incl. the final flush, truncated to stf_len * L / M
std::vector<cd> stf_template(const sync_cfg_t& c, uint32_t N_eff_TX) {
    const auto nm = get_numerology(c.u, c.b);
    const uint32_t Nd = 64 * c.b * c.os_min, N = nm.N_b_OCC;
    const uint32_t cp = (Nd / 4) * (c.u == 1 ? 3 : 5), len = cp + Nd;
    const uint32_t guard_os = (Nd - nm.N_b_DFT) / 2;
    const uint32_t off_lower = nm.N_b_DFT / 2 + 2 * guard_os + nm.N_guards_bottom;
    const auto stf = stf_values(c.b, N_eff_TX);
    std::vector<cd> bins(Nd, cd{0, 0});
    const double scale = 1.0 / std::sqrt(static_cast<double>(static_cast<float>(N / 4)));
    for (uint32_t k = 0; k <= N; ++k) bins[(k >= N / 2) ? (k - N / 2) : (off_lower + k)] = stf[k] * scale;
    std::vector<cd> td(Nd);
    for (uint32_t n = 0; n < Nd; ++n) {  // unnormalised inverse DFT (FFTW backward)
        cd acc{0, 0};
        for (uint32_t k = 0; k < Nd; ++k) {
            if (bins[k] == cd{0, 0}) continue;
            const double a = 2.0 * M_PI * static_cast<double>((static_cast<uint64_t>(k) * n) % Nd) / Nd;
            acc += bins[k] * cd{std::cos(a), std::sin(a)};
        }
        td[n] = acc;
    }
    const uint32_t pat = 16 * c.b * c.os_min, n_pat = c.u == 1 ? 7 : 9;
    std::vector<cd> x(len);
    for (uint32_t i = 0; i < len; ++i) {
        x[i] = td[(i + Nd - (cp % Nd)) % Nd];
        const uint32_t p = i / pat;
        if (p < n_pat) x[i] *= static_cast<double>(COVER_SEQ[p]);
    }
    resampler_t rs;
    rs.design(c.L, c.M, c.os_min);
    const uint32_t out_len = len * c.L / c.M;
    std::vector<cd> y(out_len, cd{0, 0});
    const int64_t Nx = len;
    for (uint32_t m = 0; m < out_len; ++m) {
        if (c.L == 1 && c.M == 1) {
            y[m] = x[m];
            continue;
        }
        const uint64_t t = rs.delay + static_cast<uint64_t>(m) * rs.M;
        const int64_t p = static_cast<int64_t>(t / rs.L);
        const uint32_t ph = static_cast<uint32_t>(t % rs.L);
        const uint32_t dmax = static_cast<uint32_t>(std::min<int64_t>(rs.hl, p));
        const uint32_t dmin = p >= Nx ? static_cast<uint32_t>(p - Nx + 1) : 0u;
        cd acc{0, 0};
        for (uint32_t dd = dmin; dd <= dmax; ++dd) acc += x[p - dd] * static_cast<double>(rs.h[ph + dd * rs.L]);
        y[m] = acc;
    }
    return y;
}

template <typename R>
std::vector<sync_out_t> sync_search(const sync_cfg_t& c, const float* iq, uint32_t S_win, uint32_t max_reports) {
    using C = std::complex<R>;
    const sync_geom_t g = sync_geometry(c);
    const uint32_t NA = c.N_ant_limited;
    std::vector<sync_out_t> res;

    // ---- sync resampler output for the whole chunk (zero history at the chunk start)
    resampler_t rs;
    rs.design(c.M, c.L, c.os_min);
    std::vector<std::vector<C>> lb(NA, std::vector<C>(g.lb_len));
    for (uint32_t a = 0; a < NA; ++a) {
        const float* s = iq + 2ull * a * S_win;
        for (uint32_t m = 0; m < g.lb_len; ++m) {
            C acc{0, 0};
            if (rs.L == 1 && rs.M == 1) {
                if (m < S_win) acc = C(s[2 * m], s[2 * m + 1]);
            } else {
                const uint64_t t = rs.delay + static_cast<uint64_t>(m) * rs.M;
                const int64_t p = static_cast<int64_t>(t / rs.L);
                const uint32_t ph = static_cast<uint32_t>(t % rs.L);
                const uint32_t dmax = static_cast<uint32_t>(std::min<int64_t>(rs.hl, p));
                for (uint32_t dd = 0; dd <= dmax; ++dd) {
                    const int64_t q = p - dd;
                    if (q >= static_cast<int64_t>(S_win)) continue;
                    acc += C(s[2 * q], s[2 * q + 1]) * static_cast<R>(rs.h[ph + dd * rs.L]);
                }
            }
            lb[a][m] = acc;
        }
    }

    // ---- detection state (autocorrelator_detection.cpp:34-105)
    const auto uw = cover_pairwise(g.n_pattern);
    std::vector<movsum_uw_t<C>> dcorr(NA);
    std::vector<movsum_t<R>> dpow(NA);
    for (uint32_t a = 0; a < NA; ++a) {
        dcorr[a].init_uw(uw, 4);
        dpow[a].init(g.n_pattern * 4);
    }
    const R prefactor = static_cast<R>(static_cast<float>(g.n_pattern) / static_cast<float>(g.n_pattern - 1));
    uint32_t resum_cnt = 0, ignore_before = g.stf_len + g.pattern;
    // set_power_of_first_stf_pattern
    for (uint32_t a = 0; a < NA; ++a)
        for (uint32_t i = 0; i < 4; ++i) {
            R p = 0;
            for (uint32_t j = 0; j < g.step; ++j) p += std::norm(lb[a][i * g.step + j]);
            dpow[a].pop_push(p);
        }
    uint32_t r = g.pattern;

    // ---- peak search state (autocorrelator_peak.cpp:37-81)
    std::vector<movsum_uw_t<C>> pcorr(NA);
    std::vector<movsum_t<R>> ppow(NA), smooth(NA);
    const uint32_t smooth_right = prm::SMOOTH_RIGHT * g.bos;
    for (uint32_t a = 0; a < NA; ++a) {
        pcorr[a].init_uw(uw, g.pattern);
        ppow[a].init(g.stf_len);
        smooth[a].init(prm::SMOOTH_LEFT * g.bos + 1 + smooth_right);
    }
    auto set_initial_movsums = [&](uint32_t start) {  // autocorrelator_peak.cpp:266-309
        for (uint32_t a = 0; a < NA; ++a) {
            for (uint32_t i = 0; i < pcorr[a].len; ++i) pcorr[a].reg[i] = lb[a][start + i] * std::conj(lb[a][start + g.pattern + i]);
            pcorr[a].ptr = 0;
            pcorr[a].resum();
            smooth[a].init(smooth[a].len);
            for (uint32_t i = 0; i < g.stf_len; ++i) ppow[a].reg[i] = std::norm(lb[a][start + i]);
            ppow[a].ptr = 0;
            ppow[a].resum();
        }
    };

    const std::vector<std::vector<cd>> tmpl = [&] {
        std::vector<std::vector<cd>> t;
        for (uint32_t k = 0, n = 1; k < g.n_templates; ++k, n *= 2) t.push_back(stf_template(c, n));
        return t;
    }();

    while (r < g.search_len && res.size() < max_reports) {
        // ================= detection: one step (autocorrelator_detection.cpp:152-284)
        for (uint32_t a = 0; a < NA; ++a) {
            C cs{0, 0};
            R ps = 0;
            for (uint32_t j = 0; j < g.step; ++j) {
                cs += lb[a][r - g.pattern + j] * std::conj(lb[a][r + j]);
                ps += std::norm(lb[a][r + j]);
            }
            dcorr[a].pop_push(cs);
            dpow[a].pop_push(ps);
        }
        if (resum_cnt++ == prm::DET_RESUM) {
            for (uint32_t a = 0; a < NA; ++a) {
                dcorr[a].resum();
                dpow[a].resum();
            }
            resum_cnt = 0;
        }
        r += g.step;
        if (ignore_before > r) continue;
        int det = -1;
        R det_rms = 0, det_metric = 0;
        for (uint32_t a = 0; a < NA && det < 0; ++a) {
            const R power = dpow[a].sum;
            const R rms = std::sqrt(power / static_cast<R>(g.stf_len));
            if (rms < static_cast<R>(g.rms_min) || static_cast<R>(prm::RMS_MAX) < rms) continue;
            const R rms_back = std::sqrt(dpow[a].sum_back(prm::RMS_BACK_STEPS));
            const R rms_front = std::sqrt(dpow[a].sum_front(prm::RMS_FRONT_STEPS));
            if (rms_back * static_cast<R>(prm::RMS_FRONT_TO_BACK) >= rms_front) continue;
            const R q = prefactor * std::abs(dcorr[a].sum) / power;
            const R metric = q * q;
            static_assert(prm::STREAK == 1 && prm::STREAK_GAIN == 0.0f, "single-step streak");
            if (metric < static_cast<R>(prm::METRIC_MIN) || static_cast<R>(prm::METRIC_MAX) < metric) continue;  // streak reset
            if (!(static_cast<R>(prm::METRIC_MIN) < metric)) continue;  // streak_t(0.18, 0, 1)::check
            det = static_cast<int>(a);
            det_rms = rms;
            det_metric = metric;
        }
        if (det < 0) continue;

        // ================= coarse peak (autocorrelator_peak.cpp:109-264)
        sync_out_t o{};
        o.det_ant = static_cast<uint32_t>(det);
        o.det_rms = static_cast<float>(det_rms);
        o.det_metric = static_cast<float>(det_metric);
        o.det_time = r;
        o.det_time_jb = r - prm::JUMP_BACK_PATTERNS * g.pattern;
        o.u = c.u;
        const uint32_t r0 = o.det_time_jb, r_max = r0 + g.D;
        set_initial_movsums(r0 - g.stf_len);
        std::vector<R> pk_metric(NA, 0);
        std::vector<uint32_t> pk_idx(NA, 0);
        uint32_t presum = 0;
        for (uint32_t rr = r0; rr < r_max; rr += g.pattern) {  // calls of one pattern each
            const uint32_t cons = std::min(g.pattern, r_max - rr);
            for (uint32_t a = 0; a < NA; ++a) {
                for (uint32_t k = 0; k < cons; ++k) {
                    const uint32_t x = rr + k;
                    pcorr[a].pop_push(lb[a][x - g.pattern] * std::conj(lb[a][x]));
                    ppow[a].pop_push(std::norm(lb[a][x]));
                    const R q = prefactor * std::abs(pcorr[a].sum) / ppow[a].sum;
                    smooth[a].pop_push(q * q);
                    const R sm = smooth[a].sum / static_cast<R>(smooth[a].len);
                    if (sm >= pk_metric[a]) {
                        pk_metric[a] = sm;
                        pk_idx[a] = x - smooth_right;
                    }
                    if (presum++ == prm::PEAK_RESUM) {
                        for (uint32_t b2 = 0; b2 < NA; ++b2) {
                            pcorr[b2].resum();
                            ppow[b2].resum();
                            smooth[b2].resum();
                        }
                        presum = 0;
                    }
                }
            }
        }
        // post_processing_validity (autocorrelator_peak.cpp:311-364)
        // (the report fields and these sums are float in the reference: sync_report.hpp, :316)
        float wsum = 0.f;
        uint32_t nvalid = 0;
        for (uint32_t a = 0; a < NA; ++a) {
            const float m = static_cast<float>(pk_metric[a]);
            if (o.det_metric + prm::PEAK_ABOVE_DETECTION >= m) continue;
            if (static_cast<int64_t>(o.det_time) + static_cast<int64_t>(prm::DETECTION2PEAK_STFS * g.stf_len) >=
                static_cast<int64_t>(pk_idx[a]))
                continue;
            o.coarse_metric[a] = m;
            wsum += m * static_cast<float>(pk_idx[a]);
            ++nvalid;
        }
        if (nvalid == 0) continue;  // false alarm: detection continues after this step
        float msum = 0.f;  // coarse_peak_array.get_sum()
        for (uint32_t a = 0; a < NA; ++a) msum += o.coarse_metric[a];
        const uint32_t wpk = static_cast<uint32_t>(std::round(wsum / msum));
        if (wpk < g.stf_len - 1) continue;  // STF before the chunk start (asserted in the reference)
        const uint32_t cpl = wpk - (g.stf_len - 1);
        o.coarse_local = cpl;
        // post_processing_at_coarse_peak (autocorrelator_peak.cpp:366-394)
        set_initial_movsums(cpl);
        float cfo_w = 0.f, msum2 = 0.f;
        for (uint32_t a = 0; a < NA; ++a) {
            if (!(o.coarse_metric[a] > 0.0f)) continue;
            const float m = static_cast<float>(pk_metric[a]);
            msum2 += m;
            const float pw = static_cast<float>(ppow[a].sum);
            o.rms[a] = std::sqrt(pw / static_cast<float>(g.stf_len));
            const std::complex<float> cs(static_cast<float>(pcorr[a].sum.real()), static_cast<float>(pcorr[a].sum.imag()));
            cfo_w += m * std::arg(cs) / static_cast<float>(g.pattern);
        }
        o.cfo_frac = cfo_w / msum2;
        o.b = c.b;  // coarse_peak_f_domain: b of the radio device class, integer CFO 0
        // skip_after_peak (autocorrelator_detection.cpp:130-138)
        ignore_before = cpl + static_cast<uint32_t>(prm::SKIP_AFTER_PEAK_STFS * g.stf_len);
        // coarse peak to hw time (rx_pacer.cpp:306-313, sync resampler L=M_tx, M=L_tx)
        double gt = static_cast<double>(cpl);
        gt *= static_cast<double>(c.L);
        gt /= static_cast<double>(c.M);
        o.coarse_64 = static_cast<int64_t>(static_cast<uint32_t>(std::round(gt)));

        // ================= fine peak (crosscorrelator.cpp:80-251), hw rate, strongest antenna
        uint32_t best = 0;
        for (uint32_t a = 1; a < NA; ++a)
            if (o.coarse_metric[a] > o.coarse_metric[best]) best = a;
        const double cfo_hw = static_cast<double>((o.cfo_frac + 0.0f) * static_cast<float>(c.M) / static_cast<float>(c.L));
        const int64_t base = o.coarse_64 - g.xc_l;
        const uint32_t stage_len = g.xc_len - 1 + g.tmpl_len;
        std::vector<cd> stage(stage_len);
        const float* s = iq + 2ull * best * S_win;
        for (uint32_t i = 0; i < stage_len; ++i) {
            const int64_t q = base + i;
            const cd v = (q >= 0 && q < static_cast<int64_t>(S_win)) ? cd(s[2 * q], s[2 * q + 1]) : cd(0, 0);
            const double ph = cfo_hw * static_cast<double>(i);
            stage[i] = v * cd(std::cos(ph), std::sin(ph));
        }
        float msum_best = 0.f;
        uint32_t nbest = 0;
        for (uint32_t k = 0; k < g.n_templates; ++k) {
            double mx = -1;
            uint32_t idx = 0;
            for (uint32_t j = 0; j < g.xc_len; ++j) {
                cd acc{0, 0};
                for (uint32_t i = 0; i < g.tmpl_len; ++i) acc += stage[j + i] * std::conj(tmpl[k][i]);
                const double m2 = std::norm(acc);
                if (m2 > mx) {
                    mx = m2;
                    idx = j;
                }
            }
            o.xc_metric[k] = static_cast<float>(std::sqrt(mx));
            o.xc_idx[k] = idx;
            if (msum_best < o.xc_metric[k]) {  // strictly larger (crosscorrelator.cpp:214-226)
                msum_best = o.xc_metric[k];
                nbest = k;
            }
        }
        o.N_eff_TX = 1u << nbest;
        o.fine_local = static_cast<uint32_t>(std::round(o.xc_metric[nbest] * static_cast<float>(o.xc_idx[nbest]) / msum_best));
        o.fine_64 = base + o.fine_local;
        o.found = 1;
        res.push_back(o);
    }
    return res;
}

template std::vector<sync_out_t> sync_search<double>(const sync_cfg_t&, const float*, uint32_t, uint32_t);
template std::vector<sync_out_t> sync_search<float>(const sync_cfg_t&, const float*, uint32_t, uint32_t);

}  // namespace orc
