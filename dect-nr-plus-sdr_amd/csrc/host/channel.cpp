// C-ABI of the simulated wireless channel (include/dnrp.h dnrp_channel_*), the GPU counterpart of the
// reference's virtual space links (lib/src/simulation/wireless/channel_{awgn,flat,doubly}.cpp,
// link.cpp, lib/src/simulation/hardware/noise.cpp): per-window link realisations drawn on the host
// from a seed (link_t::randomize, channel_flat_t::randomize_small_scale), applied by
// kernels/channel.hip.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstring>
#include <random>
#include <vector>

#include "ctx_internal.hpp"

using namespace dnrp;
using namespace dnrp::host;

namespace {

// generic power delay profiles (link.hpp:88-108 = 3GPP TS 36.104 Annex B EPA / EVA / ETU, via
// srsRAN fading.c): delays in ns, powers in dB; NAN ends a profile
constexpr uint32_t PDP_N = 3, PDP_TAPS = 9, N_SIN = 40;  // WIRELESS_CHANNEL_DOUBLY_NOF_{PROFILE,TAPS,SINUSOIDS}
constexpr double PDP_DELAY_NS[PDP_N][PDP_TAPS] = {{0, 30, 70, 90, 110, 190, 410, NAN, NAN},
                                                  {0, 30, 150, 310, 370, 710, 1090, 1730, 2510},
                                                  {0, 50, 120, 200, 230, 500, 1600, 2300, 5000}};
constexpr double PDP_POWER_DB[PDP_N][PDP_TAPS] = {{+0.0f, -1.0f, -2.0f, -3.0f, -8.0f, -17.2f, -20.8f, NAN, NAN},
                                                  {+0.0f, -1.5f, -1.4f, -3.6f, -0.6f, -9.1f, -7.0f, -12.0f, -16.9f},
                                                  {-1.0f, -1.0f, -1.0f, +0.0f, +0.0f, +0.0f, -3.0f, -5.0f, -7.0f}};
constexpr double DOPPLER_DEADBAND_HZ = 0.01f;  // link.hpp:123
constexpr float TAU_RMS_NS_MAX = 2000, FD_HZ_MAX = 2000;

double tau_rms_ns(const double* d, const double* p_db, uint32_t n) {  // link.cpp:288-322
    std::vector<double> p(n);
    double sum = 0.0;
    for (uint32_t i = 0; i < n; ++i) sum += (p[i] = std::pow(10.0, p_db[i] / 10.0));
    double mean = 0.0;
    for (uint32_t i = 0; i < n; ++i) mean += d[i] * (p[i] /= sum);
    double v = 0.0;
    for (uint32_t i = 0; i < n; ++i) v += (d[i] - mean) * (d[i] - mean) * p[i];
    return std::sqrt(v);
}

// link_t::set_pdp (link.cpp:66-120): profile delays scaled to tau_rms, quantised to samples (floor),
// equal delays merged, powers normalised to 1; amplitude per tap as link.cpp:280-283
void set_pdp(const dnrp_channel_cfg& c, std::vector<dev::channel_tap>& taps) {
    uint32_t nf = 0;
    while (nf < PDP_TAPS && std::isfinite(PDP_DELAY_NS[c.pdp_idx][nf])) ++nf;
    const double scale = c.tau_rms_ns / tau_rms_ns(PDP_DELAY_NS[c.pdp_idx], PDP_POWER_DB[c.pdp_idx], nf);
    const double Ts = 1.0 / static_cast<double>(c.samp_rate);
    std::vector<uint32_t> dl;
    std::vector<double> pw;
    for (uint32_t i = 0; i < nf; ++i) {
        const uint32_t a = static_cast<uint32_t>(std::floor(PDP_DELAY_NS[c.pdp_idx][i] * 1.0e-9 * scale / Ts));
        const double b = std::pow(10.0, PDP_POWER_DB[c.pdp_idx][i] / 10.0);
        size_t j = 0;
        while (j < dl.size() && dl[j] != a) ++j;
        if (j == dl.size()) {
            dl.push_back(a);
            pw.push_back(b);
        } else {
            pw[j] += b;
        }
    }
    double sum = 0.0;
    for (double v : pw) sum += v;
    taps.clear();
    for (size_t i = 0; i < dl.size(); ++i) {
        float s = 1.0f / std::sqrt(static_cast<float>(N_SIN));
        s *= std::sqrt(pw[i] / sum);
        taps.push_back({static_cast<int32_t>(dl[i]), s});
    }
}

uint64_t mix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

bool cfg_ok(const dnrp_channel_cfg* c) {
    if (!c || c->kind > DNRP_CH_DOUBLY) return false;
    if (c->kind == DNRP_CH_DOUBLY && (c->pdp_idx >= PDP_N || c->samp_rate == 0 || !(c->tau_rms_ns >= 0.0f) ||
                                      c->tau_rms_ns > TAU_RMS_NS_MAX || !(c->fD_Hz >= 0.0f) || c->fD_Hz > FD_HZ_MAX))
        return false;
    return true;
}

// realisation of window w: flat coefficients [N_RX][N_TX] or per link the taps and N_SIN sinusoids per
// tap (link_t::randomize, link.cpp:144-200: Jakes' model, uniform angles of arrival and phases)
void realise(const dnrp_channel_cfg& c, uint32_t w, uint32_t N_TX, uint32_t N_RX, const std::vector<dev::channel_tap>& pdp,
             float2* coef, dev::channel_tap* taps, dev::channel_sin* sins) {
    std::mt19937_64 g(mix64(c.seed ^ mix64(w + 1)));
    std::uniform_real_distribution<double> um1p1(-1.0, 1.0);
    std::normal_distribution<float> randn(0.0f, 1.0f);
    const uint32_t nl = N_RX * N_TX, nt = static_cast<uint32_t>(pdp.size());
    for (uint32_t l = 0; l < nl; ++l) {
        if (c.kind == DNRP_CH_FLAT) {  // channel_flat.cpp:80-89
            const float re = randn(g) * float(M_SQRT1_2), im = randn(g) * float(M_SQRT1_2);
            coef[l] = make_float2(re, im);
        } else if (c.kind == DNRP_CH_DOUBLY) {
            for (uint32_t i = 0; i < nt; ++i) {
                taps[l * nt + i] = pdp[i];
                for (uint32_t j = 0; j < N_SIN; ++j) {
                    const double ang = um1p1(g) * 2.0 * M_PI;
                    const double fd = c.fD_Hz * std::cos(ang);
                    auto& s = sins[(size_t(l) * nt + i) * N_SIN + j];
                    s.period = (-DOPPLER_DEADBAND_HZ < fd && fd < DOPPLER_DEADBAND_HZ)
                                   ? INT64_MAX
                                   : static_cast<int64_t>(static_cast<double>(c.samp_rate) / fd);
                    const float ph = static_cast<float>(um1p1(g)) * 2.0f * static_cast<float>(M_PI);
                    s.phase_rev = static_cast<double>(ph) / (2.0 * M_PI);
                }
            }
        }
    }
}

float noise_sigma(const dnrp_channel_cfg& c) {  // noise.cpp:30-42 -> srsRAN ch_awgn set_n0
    if (!(c.snr_db < DNRP_CH_NOISELESS_DB) || !(c.net_bw_norm > 0.0f)) return 0.0f;
    const float n0_db = -10.0f * std::log10(c.net_bw_norm) - c.snr_db;
    return std::pow(10.0f, n0_db / 20.0f) * static_cast<float>(M_SQRT1_2);
}

}  // namespace

extern "C" {

int dnrp_channel_realization(const dnrp_channel_cfg* cfg, uint32_t window, uint32_t N_TX, uint32_t N_RX, uint32_t* n_taps,
                             int32_t* delay, float* amp, int64_t* period, double* phase_rev, float* coef) {
    if (!cfg_ok(cfg) || !n_taps || N_TX == 0 || N_RX == 0 || N_TX > 8 || N_RX > 8) return DNRP_EINVAL;
    std::vector<dev::channel_tap> pdp;
    if (cfg->kind == DNRP_CH_DOUBLY) set_pdp(*cfg, pdp);
    const uint32_t nl = N_RX * N_TX, nt = static_cast<uint32_t>(pdp.size());
    std::vector<float2> cf(nl);
    std::vector<dev::channel_tap> tp(size_t(nl) * std::max(nt, 1u));
    std::vector<dev::channel_sin> sn(size_t(nl) * std::max(nt, 1u) * N_SIN);
    realise(*cfg, window, N_TX, N_RX, pdp, cf.data(), tp.data(), sn.data());
    *n_taps = nt;
    for (uint32_t l = 0; l < nl; ++l) {
        if (coef) {
            coef[2 * l] = cf[l].x;
            coef[2 * l + 1] = cf[l].y;
        }
        for (uint32_t i = 0; i < nt; ++i) {
            if (delay) delay[l * nt + i] = tp[l * nt + i].delay;
            if (amp) amp[l * nt + i] = tp[l * nt + i].amp;
            for (uint32_t j = 0; j < N_SIN; ++j) {
                const size_t k = (size_t(l) * nt + i) * N_SIN + j;
                if (period) period[k] = sn[k].period;
                if (phase_rev) phase_rev[k] = sn[k].phase_rev;
            }
        }
    }
    return DNRP_OK;
}

int dnrp_channel_batch(dnrp_ctx* ctx, const dnrp_channel_cfg* cfg, uint32_t n, uint32_t N_TX, const float* tx,
                       uint32_t S_tx, uint32_t N_RX, const int64_t* offset, const int64_t* t0, float* rx, uint32_t S_rx,
                       void* stream) {
    if (!ctx || !cfg_ok(cfg) || (n > 0 && (!tx || !rx || !offset || !t0))) return DNRP_EINVAL;
    if (n == 0) return DNRP_OK;
    if (N_TX == 0 || N_RX == 0 || N_TX > 8 || N_RX > 8 || S_tx == 0 || S_rx == 0) return DNRP_EINVAL;
    if (uint64_t(n) * N_RX > 65535u) return DNRP_ENOMEM;
    (void)hipSetDevice(ctx->cfg.device);
    hipStream_t st = static_cast<hipStream_t>(stream);
    std::vector<dev::channel_tap> pdp;
    if (cfg->kind == DNRP_CH_DOUBLY) set_pdp(*cfg, pdp);
    const uint32_t nl = N_RX * N_TX, nt = static_cast<uint32_t>(pdp.size());
    const size_t b_meta = sizeof(int64_t) * 2 * n, b_coef = sizeof(float2) * nl * n,
                 b_taps = sizeof(dev::channel_tap) * nl * nt * n, b_sins = sizeof(dev::channel_sin) * nl * nt * N_SIN * n;
    const size_t bytes = b_meta + b_coef + b_taps + b_sins;
    auto* h = static_cast<char*>(ctx->st_chan.get(bytes));
    if (!h || !ctx->chan_tab.ensure(bytes)) return DNRP_ENOMEM;
    std::memcpy(h, offset, sizeof(int64_t) * n);
    std::memcpy(h + sizeof(int64_t) * n, t0, sizeof(int64_t) * n);
    auto* coef = reinterpret_cast<float2*>(h + b_meta);
    auto* taps = reinterpret_cast<dev::channel_tap*>(h + b_meta + b_coef);
    auto* sins = reinterpret_cast<dev::channel_sin*>(h + b_meta + b_coef + b_taps);
    for (uint32_t w = 0; w < n; ++w)
        realise(*cfg, w, N_TX, N_RX, pdp, coef + size_t(w) * nl, taps + size_t(w) * nl * nt,
                sins + size_t(w) * nl * nt * N_SIN);
    HIPCHK(ctx->chan_tab.wait_idle(st));
    HIPCHK(hipMemcpyAsync(ctx->chan_tab.p, h, bytes, hipMemcpyHostToDevice, st));
    HIPCHK(hipEventRecord(ctx->st_chan.ev, st));
    char* d = static_cast<char*>(ctx->chan_tab.p);
    dev::channel_args a{};
    a.kind = cfg->kind;
    a.N_TX = N_TX;
    a.N_RX = N_RX;
    a.S_tx = S_tx;
    a.S_rx = S_rx;
    a.n_taps = nt;
    a.n_sin = N_SIN;
    a.tx = reinterpret_cast<const float2*>(tx);
    a.rx = reinterpret_cast<float2*>(rx);
    a.offset = reinterpret_cast<const int64_t*>(d);
    a.t0 = reinterpret_cast<const int64_t*>(d + sizeof(int64_t) * n);
    a.coef = reinterpret_cast<const float2*>(d + b_meta);
    a.taps = reinterpret_cast<const dev::channel_tap*>(d + b_meta + b_coef);
    a.sins = reinterpret_cast<const dev::channel_sin*>(d + b_meta + b_coef + b_taps);
    a.large_scale = cfg->large_scale;
    a.sigma = noise_sigma(*cfg);
    a.seed = mix64(cfg->seed ^ 0x6E6F697365ull);  // "noise": independent of the link draws
    if (dev::launch_channel(a, n, st) != hipSuccess) return DNRP_EDEVICE;
    return ctx->chan_tab.mark_busy(st) == hipSuccess ? DNRP_OK : DNRP_EDEVICE;
}

}  // extern "C"
