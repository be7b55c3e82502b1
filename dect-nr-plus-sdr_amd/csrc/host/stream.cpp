// C-ABI entry points over a buffer_rx_t-style ring (include/dnrp.h): the wrap-copy window gather
// of rx_pacer_t (rx_pacer.cpp:106-143) and the continuous-stream synchronisation of the sync worker
// pool: consecutive chunks searched by sync_chunk_t::search() (sync_chunk.cpp:125-279), reports
// converted to global time (sync_chunk.cpp:213-245) and filtered by the baton's uniqueness test in
// chunk order (worker_sync.cpp:110-221,320-330, baton.cpp:157-169, worker_pool.cpp:299-321).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <vector>

#include "ctx_internal.hpp"

using namespace dnrp;
using namespace dnrp::host;

namespace {

int gather(dnrp_ctx* ctx, const float* ring, uint64_t ring_len, uint64_t ant_stride, uint32_t N_ant, uint32_t n,
           const int64_t* start, uint32_t S_win, float* out, hipStream_t st) {
    if (!ring || !start || !out || ring_len == 0 || N_ant == 0 || S_win == 0) return DNRP_EINVAL;
    if (S_win > ring_len) return DNRP_EINVAL;  // a window is at most one ring turn
    if (N_ant > 1 && ant_stride < ring_len) return DNRP_EINVAL;
    if (uint64_t(n) * N_ant > 65535u) return DNRP_ENOMEM;
    for (uint32_t w = 0; w < n; ++w)
        if (start[w] < 0) return DNRP_EINVAL;
    auto* hs = static_cast<int64_t*>(ctx->st_ring.get(sizeof(int64_t) * n));
    if (!hs || !ctx->ring_start.ensure(sizeof(int64_t) * n)) return DNRP_ENOMEM;
    std::memcpy(hs, start, sizeof(int64_t) * n);
    HIPCHK(ctx->ring_start.wait_idle(st));
    HIPCHK(hipMemcpyAsync(ctx->ring_start.p, hs, sizeof(int64_t) * n, hipMemcpyHostToDevice, st));
    HIPCHK(hipEventRecord(ctx->st_ring.ev, st));
    dev::ring_args a{};
    a.ring = reinterpret_cast<const float2*>(ring);
    a.ring_len = ring_len;
    a.ant_stride = ant_stride;
    a.start = ctx->ring_start.as<int64_t>();
    a.out = reinterpret_cast<float2*>(out);
    a.n_ant = N_ant;
    a.S_win = S_win;
    if (dev::launch_ring_gather(a, n, st) != hipSuccess) return DNRP_EDEVICE;
    return ctx->ring_start.mark_busy(st) == hipSuccess ? DNRP_OK : DNRP_EDEVICE;
}

}  // namespace

extern "C" {

int dnrp_ring_gather(dnrp_ctx* ctx, const float* ring, uint64_t ring_len, uint64_t ant_stride, uint32_t N_ant,
                     uint32_t n, const int64_t* start, uint32_t S_win, float* out, void* stream) {
    if (!ctx) return DNRP_EINVAL;
    if (n == 0) return DNRP_OK;
    (void)hipSetDevice(ctx->cfg.device);
    return gather(ctx, ring, ring_len, ant_stride, N_ant, n, start, S_win, out, static_cast<hipStream_t>(stream));
}

int dnrp_sync_stream_init(const dnrp_ctx* ctx, const dnrp_sync_cfg* sc, dnrp_sync_stream_state* state) {
    if (!ctx || !sc || !state) return DNRP_EINVAL;
    // worker_pool_t::get_sync_time_unique_limit (worker_pool.cpp:299-321): one STF pattern of the
    // radio device class' shortest STF at b_min * os_min
    const uint32_t pattern = prm::N_SAMPLES_STF_PATTERN * sc->b * ctx->cfg.os_min;
    state->sync_time_unique_limit = static_cast<int64_t>(static_cast<double>(pattern) * prm::SYNC_TIME_UNIQUE_LIMIT_PATTERNS);
    state->sync_time_last = prm::UNDEFINED_EARLY_64;  // baton.cpp:47-52
    state->packets = state->not_unique = 0;
    return DNRP_OK;
}

uint32_t dnrp_sync_stream_window(const dnrp_ctx* ctx, const dnrp_sync_cfg* sc) {
    if (!ctx || !sc || sc->b == 0) return 0;
    // a chunk's search reads its A + B + C + D DECT samples (sync_chunk.cpp:63-69: B = the overlap
    // into the next chunk, C one pattern, D the coarse-peak search) plus the cross-correlation span
    // after the coarse peak (left/right search + one STF, crosscorrelator.cpp:53-57) at the hw rate,
    // and the resampler's filter span: chunk_len + that tail, rounded up to an even sample count
    const auto& c = ctx->cfg;
    const uint32_t n_pat = sc->u == 1 ? prm::N_STF_PATTERN_U1 : prm::N_STF_PATTERN_U248;
    const uint32_t bos = sc->b * c.os_min, stf = prm::N_SAMPLES_STF_PATTERN * n_pat * bos;
    const double dect_tail = prm::SYNC_OVERLAP_STFS * stf + stf / n_pat + prm::SYNC_PEAK_MAX_SEARCH_STFS * stf +
                             (prm::SYNC_XC_SEARCH_LEFT + prm::SYNC_XC_SEARCH_RIGHT) * bos + 2.0 * stf;
    const uint64_t tail = static_cast<uint64_t>(dect_tail * c.L / c.M) + 512;
    return static_cast<uint32_t>((uint64_t(sc->chunk_len) + tail + 1) & ~1ull);
}

int dnrp_rx_sync_stream(dnrp_ctx* ctx, const dnrp_sync_cfg* sc, const float* ring, uint64_t ring_len,
                        uint64_t ant_stride, int64_t t0, uint32_t n_chunks, dnrp_sync_stream_state* state,
                        dnrp_sync_result* out, uint32_t* n_out, uint32_t* chunk_of, void* stream) {
    if (!ctx || !sc || !state || !out || !n_out || !ring || t0 < 0) return DNRP_EINVAL;
    *n_out = 0;
    if (n_chunks == 0) return DNRP_OK;
    if (n_chunks > ctx->cfg.max_batch) return DNRP_ENOMEM;
    (void)hipSetDevice(ctx->cfg.device);
    hipStream_t st = static_cast<hipStream_t>(stream);
    const uint32_t S_win = dnrp_sync_stream_window(ctx, sc);
    const uint32_t N_ant = sc->N_ant_limited;
    if (S_win == 0 || S_win > ring_len) return DNRP_EINVAL;
    // chunk k = global samples [t0 + k chunk_len, ...) (worker_sync.cpp:42-54: consecutive chunks of
    // the interleaved sync workers), each window gathered from the ring with the wrap copy
    std::vector<int64_t> starts(n_chunks);
    for (uint32_t k = 0; k < n_chunks; ++k) starts[k] = t0 + int64_t(k) * sc->chunk_len;
    const size_t wbytes = size_t(n_chunks) * N_ant * S_win * sizeof(float2);
    if (!ctx->ring_win.ensure(wbytes)) return DNRP_ENOMEM;
    int err = gather(ctx, ring, ring_len, ant_stride, N_ant, n_chunks, starts.data(), S_win, ctx->ring_win.as<float>(), st);
    if (err != DNRP_OK) return err;
    const size_t rbytes = size_t(n_chunks) * sc->max_reports * sizeof(dnrp_sync_result);
    auto* res = static_cast<dnrp_sync_result*>(ctx->st_stream.get(rbytes + sizeof(uint32_t) * n_chunks));
    if (!res) return DNRP_ENOMEM;
    auto* cnt = reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(res) + rbytes);
    err = dnrp_rx_sync_batch(ctx, sc, n_chunks, ctx->ring_win.as<float>(), uint64_t(N_ant) * S_win, S_win, S_win, res, cnt,
                             stream);
    if (err != DNRP_OK) return err;
    HIPCHK(hipEventRecord(ctx->st_stream.ev, st));
    HIPCHK(hipStreamSynchronize(st));
    // baton: chunks in order, reports of a chunk in search order; local -> global time
    // (sync_chunk.cpp:213-245), then is_sync_time_unique (baton.cpp:157-169)
    uint32_t m = 0;
    for (uint32_t k = 0; k < n_chunks; ++k)
        for (uint32_t r = 0; r < std::min(cnt[k], sc->max_reports); ++r) {
            dnrp_sync_result s = res[size_t(k) * sc->max_reports + r];
            if (!s.found) continue;
            s.coarse_peak_time += starts[k];
            s.fine_peak_time += starts[k];
            if (s.fine_peak_time - state->sync_time_last > state->sync_time_unique_limit) {
                state->sync_time_last = s.fine_peak_time;
                ++state->packets;
                out[m] = s;
                if (chunk_of) chunk_of[m] = k;
                ++m;
            } else {
                ++state->not_unique;  // worker_sync_t stats.job_packet_not_unique
            }
        }
    *n_out = m;
    return DNRP_OK;
}

}  // extern "C"
