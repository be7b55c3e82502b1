// C-ABI synchronisation entry point (include/dnrp.h dnrp_rx_sync_batch): per-(u, b) tables built
// as the sync_chunk_t / crosscorrelator_t / stf_template_t constructors do
// (sync_chunk.cpp:32-123, crosscorrelator.cpp:22-59, stf_template.cpp:22-206), then three launches
// (kernels/sync.hip).
#include <hip/hip_runtime.h>

#include <cmath>
#include <complex>
#include <cstring>
#include <memory>
#include <vector>

#include <cstdio>
#include <cstdlib>

#include "ctx_internal.hpp"

using namespace dnrp;
using namespace dnrp::host;

namespace {

using cd = std::complex<double>;

const float* const COVER = prm::STF_COVER;  // stf.hpp:146-151 (cover sequence active)

// unnormalised DFT of any length: the STF IFFT is 64 b os points (768 / 1536 / 3072 for b = 12),
// the template spectra are powers of two. Init-time only.
void dft_direct(std::vector<cd>& x, int sign) {
    const size_t n = x.size();
    std::vector<cd> y(n, cd(0, 0));
    for (size_t k = 0; k < n; ++k) {
        cd acc(0, 0);
        for (size_t i = 0; i < n; ++i) {
            const double a = sign * 2.0 * M_PI * static_cast<double>((k * i) % n) / static_cast<double>(n);
            acc += x[i] * cd(std::cos(a), std::sin(a));
        }
        y[k] = acc;
    }
    x.swap(y);
}

void fft_host(std::vector<cd>& x, int sign) {  // iterative radix-2 for powers of two, unnormalised
    const size_t n = x.size();
    if (n == 0 || (n & (n - 1))) return dft_direct(x, sign);
    for (size_t i = 1, j = 0; i < n; ++i) {
        size_t bit = n >> 1;
        for (; j & bit; bit >>= 1) j ^= bit;
        j ^= bit;
        if (i < j) std::swap(x[i], x[j]);
    }
    for (size_t len = 2; len <= n; len <<= 1) {
        const double a = sign * 2.0 * M_PI / static_cast<double>(len);
        for (size_t i = 0; i < n; i += len)
            for (size_t k = 0; k < len / 2; ++k) {
                const cd w(std::cos(a * k), std::sin(a * k));
                const cd u = x[i + k], v = x[i + k + len / 2] * w;
                x[i + k] = u + v;
                x[i + k + len / 2] = u - v;
            }
    }
}

// stf_template_t::generate_stf_time_domain (stf_template.cpp:81-206): the STF of (b, N_eff_TX) at
// N_b_DFT_os = 64 b os, IFFT + CP, 1/sqrt(N_b_OCC/4), cover sequence, TX resampler L/M with the
// final flush, truncated to stf_len * L / M hw samples
std::vector<cd> stf_template(uint32_t u, uint32_t b, uint32_t os, const geo::resampler_t& rs_tx, uint32_t N_eff_TX) {
    const uint32_t N = 56 * b, Nb = 64 * b, Nd = Nb * os;
    const uint32_t off_lower = Nb / 2 + (Nd - Nb) + 4 * b;  // insert offset + mirror (tx_rx.cpp:197-240)
    const uint32_t cp = (Nd / 4) * (u == 1 ? 3 : 5), len = cp + Nd;
    const auto stf = geo::stf_values(b, N_eff_TX);
    const double scale = 1.0 / std::sqrt(static_cast<double>(static_cast<float>(N / 4)));
    std::vector<cd> bins(Nd, cd(0, 0));
    for (uint32_t k = 0; k <= N; ++k)
        bins[(k >= N / 2) ? (k - N / 2) : (off_lower + k)] = cd(stf[k].real(), stf[k].imag()) * scale;
    fft_host(bins, +1);  // FFTW backward = unnormalised inverse
    const uint32_t pat = 16 * b * os, n_pat = u == 1 ? 7 : 9;
    std::vector<cd> x(len);
    for (uint32_t i = 0; i < len; ++i) {
        x[i] = bins[(i + Nd - (cp % Nd)) % Nd];
        if (i / pat < n_pat) x[i] *= static_cast<double>(COVER[i / pat]);
    }
    const uint32_t L = rs_tx.L, M = rs_tx.M, out_len = len * L / M;
    std::vector<cd> y(out_len, cd(0, 0));
    for (uint32_t m = 0; m < out_len; ++m) {
        if (L == 1 && M == 1) {
            y[m] = x[m];
            continue;
        }
        const uint64_t t = rs_tx.delay + static_cast<uint64_t>(m) * M;
        const int64_t p = static_cast<int64_t>(t / L);
        const uint32_t ph = static_cast<uint32_t>(t % L);
        cd acc(0, 0);
        for (uint32_t d = 0; d <= rs_tx.hl; ++d) {
            const int64_t q = p - d;
            if (q < 0 || q >= static_cast<int64_t>(len)) continue;
            acc += x[q] * static_cast<double>(rs_tx.h[ph + d * L]);
        }
        y[m] = acc;
    }
    return y;
}

sync_tables* get_sync(dnrp_ctx* ctx, uint32_t u, uint32_t b, int* err) {
    auto& slot = ctx->synct[{u, b}];
    if (slot) return slot.get();
    const auto& c = ctx->cfg;
    auto t = std::make_unique<sync_tables>();
    t->u = u;
    t->b = b;
    t->n_pattern = u == 1 ? prm::N_STF_PATTERN_U1 : prm::N_STF_PATTERN_U248;  // stf.hpp:91-97
    t->bos = b * c.os_min;
    t->stf_len = prm::N_SAMPLES_STF_PATTERN * t->n_pattern * t->bos;
    t->pattern = prm::N_SAMPLES_STF_PATTERN * t->bos;
    t->step = t->pattern / prm::SYNC_STEP_DIVIDER;  // autocorrelator_detection.cpp:49
    t->D = static_cast<uint32_t>(prm::SYNC_PEAK_MAX_SEARCH_STFS * t->stf_len);  // sync_chunk.cpp:68
    t->rms_min = static_cast<float>(prm::SYNC_RMS_MIN * std::sqrt(static_cast<double>(u) * b * prm::SAMP_RATE_MIN_U_B /
                                                                  prm::SYNC_RMS_MIN_REF_RATE));
    t->xc_l = prm::SYNC_XC_SEARCH_LEFT * b * c.os_min * c.L / c.M;  // crosscorrelator.cpp:53-56
    t->xc_len = t->xc_l + prm::SYNC_XC_SEARCH_RIGHT * b * c.os_min * c.L / c.M + 1;
    t->tmpl_len = t->stf_len * c.L / c.M;
    t->n_templates = c.N_TX_max >= 8 ? 4 : c.N_TX_max >= 4 ? 3 : c.N_TX_max >= 2 ? 2 : 1;  // physical_resources.hpp:44
    uint32_t lg = 0;
    while ((1u << lg) < t->xc_len - 1 + t->tmpl_len) ++lg;
    t->log2_fft = lg;
    const uint32_t nf = 1u << lg;
    // sync resampler: RX direction, L and M swapped (sync_chunk.cpp:40-48)
    t->rs = geo::make_resampler(c.M, c.L, c.os_min, prm::RS_SYNC);
    if (!(c.L == 1 && c.M == 1)) {
        while ((t->rs.delay + t->m_star * t->rs.M) % t->rs.L) ++t->m_star;
        t->p_star = (t->rs.delay + t->m_star * t->rs.M) / t->rs.L;
    }
    const auto rs_tx = geo::make_resampler(c.L, c.M, c.os_min, prm::RS_TX);  // stf_template.cpp: TX filter
    std::vector<float2> tf(size_t(t->n_templates) * nf);
    for (uint32_t k = 0; k < t->n_templates; ++k) {
        auto tm = stf_template(u, b, c.os_min, rs_tx, 1u << k);
        tm.resize(nf, cd(0, 0));
        fft_host(tm, -1);
        for (uint32_t i = 0; i < nf; ++i) {
            const cd v = std::conj(tm[i]) / static_cast<double>(nf);
            tf[size_t(k) * nf + i] = make_float2(static_cast<float>(v.real()), static_cast<float>(v.imag()));
        }
    }
    std::vector<float> pp = (c.L == 1 && c.M == 1) ? std::vector<float>{0.f} : taps_polyphase(t->rs, &t->npp);
    if (c.L == 1 && c.M == 1) t->npp = 0;
    if (!t->taps.upload(t->rs.h) || !t->taps_pp.upload(pp) || !t->tmpl_f.upload(tf) || !t->tw_fft.upload(twiddles(nf))) {
        *err = DNRP_ENOMEM;
        return nullptr;
    }
    slot = std::move(t);
    return slot.get();
}

}  // namespace

extern "C" int dnrp_rx_sync_batch(dnrp_ctx* ctx, const dnrp_sync_cfg* sc, uint32_t n, const float* iq,
                                  uint64_t win_stride, uint64_t ant_stride, uint32_t S_win, dnrp_sync_result* res,
                                  uint32_t* n_found, void* stream) {
    static_assert(sizeof(dnrp_sync_result) == sizeof(dev::sync_res), "dnrp_sync_result layout");
    if (!ctx || !sc || (n > 0 && (!iq || !res))) return DNRP_EINVAL;
    if (n == 0) return DNRP_OK;
    if (n > ctx->cfg.max_batch) return DNRP_ENOMEM;
    const bool uok = sc->u == 1 || sc->u == 2 || sc->u == 4 || sc->u == 8;
    const bool bok = sc->b == 1 || sc->b == 2 || sc->b == 4 || sc->b == 8 || sc->b == 12 || sc->b == 16;
    if (!uok || !bok || sc->u > ctx->cfg.u_max || sc->b > ctx->cfg.b_max) return DNRP_EINVAL;
    if (sc->N_ant_limited == 0 || sc->N_ant_limited > ctx->cfg.N_TX_max || sc->N_ant_limited > prm::SYNC_ANTENNA_LIMIT)
        return DNRP_EINVAL;
    if (sc->max_reports == 0 || S_win == 0 || sc->chunk_len < ctx->cfg.L) return DNRP_EINVAL;
    (void)hipSetDevice(ctx->cfg.device);
    int err = DNRP_OK;
    sync_tables* t = get_sync(ctx, sc->u, sc->b, &err);
    if (!t) return err;
    const auto& c = ctx->cfg;
    dev::sync_args a{};
    a.n_ant = sc->N_ant_limited;
    a.n_pattern = t->n_pattern;
    a.stf_len = t->stf_len;
    a.pattern = t->pattern;
    a.step = t->step;
    const uint64_t A_len = uint64_t(sc->chunk_len) / c.L * c.M;  // sync_chunk.cpp:63-64
    const uint64_t search = A_len + static_cast<uint32_t>(prm::SYNC_OVERLAP_STFS * t->stf_len);
    if (search > (1u << 30)) return DNRP_EINVAL;
    a.search_len = static_cast<uint32_t>(search);
    a.D = t->D;
    a.bos = t->bos;
    a.n_steps = (a.search_len + a.step - 1) / a.step;
    a.L = t->rs.L;
    a.M = t->rs.M;
    a.delay = t->rs.delay;
    a.hl = t->rs.hl;
    a.ct_taps = dev::sync_taps_match(t->rs.h.data(), t->rs.h.size()) ? 1u : 0u;
    a.m_star = t->m_star;
    a.p_star = t->p_star;
    a.npp = t->npp;
    a.taps = t->taps.as<float>();
    a.taps_pp = t->taps_pp.as<float>();
    a.rms_min = t->rms_min;
    a.prefactor = static_cast<float>(t->n_pattern) / static_cast<float>(t->n_pattern - 1);
    a.n_uw = t->n_pattern - 1;
    for (uint32_t i = 0; i < a.n_uw; ++i) a.uw[i] = COVER[i] * COVER[i + 1];  // stf.cpp:140-159
    a.iq = reinterpret_cast<const float2*>(iq);
    a.win_stride = win_stride;
    a.ant_stride = ant_stride;
    a.S_win = S_win;
    a.n_win = n;
    a.max_reports = sc->max_reports;
    a.Ltx = c.L;
    a.Mtx = c.M;
    a.xc_l = t->xc_l;
    a.xc_len = t->xc_len;
    a.tmpl_len = t->tmpl_len;
    a.n_templates = t->n_templates;
    a.log2_fft = t->log2_fft;
    a.tmpl_f = t->tmpl_f.as<float2>();
    a.tw_fft = t->tw_fft.as<float2>();
    a.u = sc->u;
    a.b = sc->b;
    a.det_stage = dev::sync_detect_stage(a);
    if (dev::sync_detect_lds(a) > 160 * 1024 || (16 + 2 * (size_t(1) << a.log2_fft)) * sizeof(float2) > 160 * 1024)
        return DNRP_EUNSUPPORTED;
    const size_t nsa = size_t(n) * a.n_ant * a.n_steps;
    if (!ctx->sy_P.ensure(nsa * sizeof(float)) || !ctx->sy_C.ensure(nsa * sizeof(float2)) ||
        !ctx->sy_res.ensure(size_t(n) * a.max_reports * sizeof(dev::sync_res)) || !ctx->sy_cnt.ensure(size_t(n) * 4) ||
        !ctx->sy_spec.ensure(size_t(n) * a.max_reports * (size_t(1) << a.log2_fft) * sizeof(float2)) ||
        !ctx->sy_post.ensure(size_t(n) * a.max_reports * 8 * sizeof(float)) ||
        !ctx->sy_state.ensure(size_t(n) * sizeof(dev::sync_state)) || !ctx->sy_pk.ensure(size_t(n) * 8 * sizeof(float2)))
        return DNRP_ENOMEM;
    a.state = ctx->sy_state.as<dev::sync_state>();
    a.pk = ctx->sy_pk.as<float2>();
    a.spec = ctx->sy_spec.as<float2>();
    a.post = ctx->sy_post.as<float>();
    a.P = ctx->sy_P.as<float>();
    a.Cs = ctx->sy_C.as<float2>();
    a.res = ctx->sy_res.as<dev::sync_res>();
    a.n_found = ctx->sy_cnt.as<uint32_t>();
    hipStream_t st = static_cast<hipStream_t>(stream);
    ctx->tic("sync_steps", st);
    if (dev::launch_sync_steps(a, n, st) != hipSuccess) return DNRP_EDEVICE;
    ctx->toc("sync_steps", st);
#ifdef DNRP_SYNC_PROFILE
    // phase clocks of sync_detect per window (tools/sync_profile.py): averages to stderr
    static dbuf prof;
    const bool do_prof = std::getenv("DNRP_SYNC_PROFILE") && prof.ensure(size_t(n) * 32 * 8);
    a.prof = do_prof ? prof.as<unsigned long long>() : nullptr;
    if (do_prof) HIPCHK(hipMemsetAsync(prof.p, 0, size_t(n) * 32 * 8, st));
#endif
    // detection + coarse peak: `rounds` split rounds (detection-only workgroups, then one coarse-peak
    // workgroup per (window, antenna) of every pending detection), then the inline form finishes what
    // is left (windows with more detections than rounds); DNRP_SYNC_ROUNDS=0: the inline form alone.
    // Default: split with several antennas (their peak searches run in parallel instead of in series:
    // C4 4 antennas 199k -> 205k slot-pairs/s), inline with one (no series to break up, and the extra
    // dependent launches lengthen the sync chain the host waits on: C3 654k inline vs 573k split,
    // C2 equal; same-box A/B on MI355X). Read per call (tests switch it at run time).
    const char* rd_e = std::getenv("DNRP_SYNC_ROUNDS");
    const int rounds = !dev::sync_peak_ok(a) ? 0 : rd_e ? std::max(0, std::atoi(rd_e)) : (a.n_ant > 1 ? 2 : 0);
    a.first = 1;
    for (int r = 0; r < rounds; ++r) {
        ctx->tic("sync_detect", st);
        if (dev::launch_sync_detect_split(a, n, st) != hipSuccess) return DNRP_EDEVICE;
        ctx->toc("sync_detect", st);
        a.first = 0;
        ctx->tic("sync_peak", st);
        if (dev::launch_sync_peak(a, n, st) != hipSuccess) return DNRP_EDEVICE;
        ctx->toc("sync_peak", st);
    }
    ctx->tic("sync_detect", st);
    if (dev::launch_sync_detect(a, n, st) != hipSuccess) return DNRP_EDEVICE;
    ctx->toc("sync_detect", st);
#ifdef DNRP_SYNC_PROFILE
    if (do_prof) {
        std::vector<unsigned long long> h(size_t(n) * 32);
        HIPCHK(hipMemcpyAsync(h.data(), prof.p, h.size() * 8, hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
        double acc[16] = {};
        uint32_t cnt = 0;
        for (uint32_t i = 0; i < n; ++i) {
            const unsigned long long* r = &h[size_t(i) * 32];
            if (!r[0] || !r[11]) continue;
            ++cnt;
            unsigned long long prev = r[0];
            for (int k = 1; k < 12; ++k)
                if (r[k]) {
                    acc[k] += double(r[k] - prev);
                    prev = r[k];
                }
        }
        std::fprintf(stderr, "sync_detect phases (wall_clock64 ticks, mean over %u windows):", cnt);
        for (int k = 1; k < 12; ++k) std::fprintf(stderr, " p%d=%.0f", k, cnt ? acc[k] / cnt : 0.0);
        double q[4] = {};
        for (uint32_t i = 0; i < n; ++i) {
            const unsigned long long* r = &h[size_t(i) * 32];
            if (!r[8] || !r[12] || !r[13] || !r[14]) continue;
            q[0] += double(r[12] - r[8]);
            q[1] += double(r[13] - r[12]);
            q[2] += double(r[14] - r[13]);
            q[3] += double(r[9] - r[14]);
        }
        std::fprintf(stderr, " | last peak search: sums %.0f scans %.0f metric %.0f smooth+argmax %.0f\n",
                     cnt ? q[0] / cnt : 0.0, cnt ? q[1] / cnt : 0.0, cnt ? q[2] / cnt : 0.0, cnt ? q[3] / cnt : 0.0);
        double pq[6] = {};
        uint32_t pc = 0;
        for (uint32_t i = 0; i < n; ++i) {  // sync_peak_kernel of antenna 0 (split rounds)
            const unsigned long long* r = &h[size_t(i) * 32 + 16];
            if (!r[0] || !r[6]) continue;
            ++pc;
            for (int k = 0; k < 6; ++k) pq[k] += double(r[k + 1] - r[k]);
        }
        std::fprintf(stderr, "sync_peak phases (%u windows): resample %.0f sums %.0f scans %.0f metric %.0f met %.0f smooth+argmax %.0f\n",
                     pc, pc ? pq[0] / pc : 0.0, pc ? pq[1] / pc : 0.0, pc ? pq[2] / pc : 0.0, pc ? pq[3] / pc : 0.0,
                     pc ? pq[4] / pc : 0.0, pc ? pq[5] / pc : 0.0);
    }
#endif
    ctx->tic("sync_post", st);
    if (dev::launch_sync_post(a, n, st) != hipSuccess) return DNRP_EDEVICE;
    ctx->toc("sync_post", st);
    ctx->tic("sync_fine", st);
    if (dev::launch_sync_fine(a, n, st) != hipSuccess) return DNRP_EDEVICE;
    ctx->toc("sync_fine", st);
    HIPCHK(hipMemcpyAsync(res, a.res, size_t(n) * a.max_reports * sizeof(dev::sync_res), hipMemcpyDeviceToHost, st));
    if (n_found) HIPCHK(hipMemcpyAsync(n_found, a.n_found, size_t(n) * 4, hipMemcpyDeviceToHost, st));
    return DNRP_OK;
}
