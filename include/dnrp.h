/*
 * dnrp.h — C-ABI of the MI355X-native DECT NR+ lower PHY (libdnrp.so).
 *
 * Drop-in boundary for the OFDM TX/RX hot path of maxpenner/DECT-NR-Plus-SDR. The reference has
 * no FFI; its path is three C++ classes owned per worker thread. Each entry point below replaces
 * one of them, batched over many independent packets (slots):
 *
 *   dnrp_ctx_create        <- tx_rx_t / tx_t / rx_synced_t constructors
 *                             (lib/src/phy/tx_rx.cpp:38-129, tx/tx.cpp:48-141,
 *                              rx/rx_synced/rx_synced.cpp:55-174)
 *   dnrp_add_network_id    <- tx_rx_t::add_new_network_id (lib/include/dectnrp/phy/tx_rx.hpp:52,
 *                             sections_part3/scrambling_pdc.cpp:36-57)
 *   dnrp_get_packet_sizes  <- sp3::get_packet_sizes (sections_part3/derivative/packet_sizes.cpp:99)
 *   dnrp_compute_packet_sizes  (same, context-free and host-only)
 *   dnrp_tx_batch          <- tx_t::generate_tx_packet (lib/include/dectnrp/phy/tx/tx.hpp:80-81,
 *                             lib/src/phy/tx/tx.cpp:165-314), FEC boundary between rate matching
 *                             and scrambling (pcc_enc.cpp:212, pdc_enc.cpp:218-221)
 *   dnrp_rx_sync_batch     <- sync_chunk_t::search() per window (lib/include/dectnrp/phy/rx/sync/
 *                             sync_chunk.hpp:72, lib/src/phy/rx/sync/sync_chunk.cpp:143-279)
 *   dnrp_rx_pcc_batch      <- rx_synced_t::demoddecod_rx_pcc up to the descrambled PCC d-bits
 *                             (lib/include/dectnrp/phy/rx/rx_synced/rx_synced.hpp:93,
 *                              rx_synced.cpp:186-302, pcc_enc.cpp:297)
 *   dnrp_rx_pdc_batch      <- rx_synced_t::demoddecod_rx_pdc up to the descrambled PDC d-bits
 *                             (rx_synced.hpp:103, rx_synced.cpp:325-436, pdc_enc.cpp:339-344)
 *   dnrp_ctx_destroy       <- destructors
 *
 * Conventions (all functions):
 *   - return 0 on success, a negative DNRP_E* code on argument/configuration error; never abort.
 *   - bulk buffers (bits, IQ, LLRs) are DEVICE pointers on the context's HIP device; descriptor
 *     and report arrays are HOST pointers. IQ is interleaved cf32, one contiguous stream per
 *     antenna (radio/complex.hpp:28, buffer_tx.hpp, buffer_rx.hpp).
 *   - work is stream-ordered on the caller's hipStream_t (passed as void*, NULL = default
 *     stream); host report arrays are valid after dnrp_sync() or a stream synchronisation.
 *   - one context per submitting host thread; contexts are not thread-safe (like the reference's
 *     per-worker tx_t/rx_synced_t objects).
 *   - LLRs are int16, positive means bit 1 (phy_config.hpp:39-41, fec/test/tb2pdc.cpp:173-176).
 */
#ifndef DNRP_H
#define DNRP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DNRP_OK 0
#define DNRP_EINVAL (-1)      /* bad argument / null pointer */
#define DNRP_ECONFIG (-2)     /* packet configuration not valid (get_packet_sizes -> nullopt) */
#define DNRP_EUNSUPPORTED (-3)/* valid DECT NR+ configuration the reference RX cannot demodulate */
#define DNRP_ENOMEM (-4)      /* device allocation failed / batch larger than max_batch */
#define DNRP_EDEVICE (-5)     /* HIP runtime error */
#define DNRP_ENETID (-6)      /* network ID not registered with dnrp_add_network_id */
#define DNRP_ESTATE (-7)      /* dnrp_rx_pdc_batch without a preceding dnrp_rx_pcc_batch */

typedef struct dnrp_ctx dnrp_ctx;

/* worker_pool_config_t subset (phy/worker_pool_config.hpp) */
typedef struct {
    uint32_t u_max, b_max;      /* radio device class maxima (sections_part3/radio_device_class.cpp) */
    uint32_t N_TX_max;          /* physical antennas; RX uses N_RX = N_TX_max (rx_synced.hpp:120-126) */
    uint32_t os_min;            /* minimum oversampling (phy.json os_min) */
    uint32_t L, M;              /* hw/DECT resampling ratio L/M for TX, M/L for RX (phy_config.cpp:28-94) */
    uint32_t chestim_mode_lr;   /* phy.json chestim_mode_lr_default */
    uint32_t chestim_lr_stride; /* phy.json chestim_mode_lr_t_stride_default */
    uint32_t max_batch;         /* packets per batch call */
    int32_t device;             /* HIP device ordinal */
} dnrp_cfg;

/* sp3::packet_sizes_def_t */
typedef struct {
    uint32_t u, b, PacketLengthType, PacketLength, tm_mode_index, mcs_index, Z;
} dnrp_psdef;

/* sp3::packet_sizes_t + context-dependent hw-rate sizes */
typedef struct {
    uint32_t N_PACKET_symb, N_DF_symb, N_PDC_subc, N_DRS_subc, G, N_PDC_bits, N_TB_bits, N_TB_byte, C;
    uint32_t N_samples_STF, N_samples_STF_CP_only, N_samples_DF, N_samples_GI;
    uint32_t N_samples_packet_no_GI, N_samples_packet;
    uint32_t N_bps, N_eff_TX, N_SS, N_TS, N_TX, N_b_DFT, N_b_OCC;
    uint32_t N_b_DFT_os;                  /* FFT size used (tx.cpp:439) */
    uint32_t N_samples_packet_no_GI_os_rs;/* hw samples carrying the packet (tx.cpp:527-529) */
    uint32_t N_samples_packet_os_rs;      /* hw samples of the slot window incl. full GI */
} dnrp_packet_sizes;

/* tx_descriptor_t + tx_meta_t subset (phy/tx/tx_descriptor.hpp, phy/tx/tx_meta.hpp) */
typedef struct {
    uint32_t codebook_index;
    uint32_t network_id;      /* must have been registered */
    uint32_t plcf_type;       /* 1 or 2: selects the PDC scrambling sequence */
    uint32_t GI_percentage;   /* share of the GI actually transmitted (zeros) */
    float DAC_scale;
    float iq_phase_rad;
    float iq_phase_increment_s2s_post_resampling_rad;
    uint32_t optimal_scaling_DAC; /* 0: standard W scaling, 1: W_t::scaling_factor_optimal_DAC (tx.cpp:582-592) */
} dnrp_tx_desc;

/* sync_report_t fields consumed by rx_synced_t (phy/rx/sync/sync_report.hpp) */
typedef struct {
    int64_t fine_peak_time;   /* hw-rate sample index of the packet start inside its window */
    float cfo_fractional_rad; /* per DECT-rate sample */
    float cfo_integer_rad;
    uint32_t u, b, N_eff_TX;
    uint32_t window;          /* window of iq_in holding the packet (the sync window it was found in:
                                 several packets of one window share it) */
    float rms[8];             /* sync_report_t::rms_array (dnrp_sync_result::rms_array): the RX keeps
                                 the values > 0 and estimates the others over the STF
                                 (RX_SYNCED_PARAM_RMS_KEEP_VALUES_PROVIDED_BY_SYNC, rx_synced.cpp:620-655) */
} dnrp_sync_report;

/* Synchronisation of one batch of windows (sync_chunk_t, worker_pool_config_t subset) */
typedef struct {
    uint32_t u, b;          /* radio device class u_min / b_min: the STF searched for (sync_chunk.cpp:54-57) */
    uint32_t N_ant_limited; /* antennas searched, <= cfg.N_TX_max (RX_SYNC_PARAM_AUTOCORRELATOR_ANTENNA_LIMIT) */
    uint32_t chunk_len;     /* hw samples per chunk; the search covers chunk_len/L*M + 4 STFs at the
                               DECT rate (sync_chunk.cpp:63-66), the window must hold the peak and
                               cross-correlation samples after it (zeros are read past S_win) */
    uint32_t max_reports;   /* packets reported per window (successive search() calls on one chunk) */
} dnrp_sync_cfg;

/* sync_report_t (phy/rx/sync/sync_report.hpp:29-98) of one synchronised packet. "local" times are
 * DECT-rate sample indices of the chunk's resampled buffer, the others hw sample indices relative
 * to the window start. fine_peak_time / cfo_fractional_rad / cfo_integer_rad / u / b / N_eff_TX are
 * what dnrp_rx_pcc_batch consumes (as a dnrp_sync_report). */
typedef struct {
    uint32_t found;                   /* 1: packet synchronised; 0: slot unused */
    uint32_t detection_ant_idx;
    float detection_rms, detection_metric;
    uint32_t detection_time_local, detection_time_with_jump_back_local;
    uint32_t coarse_peak_time_local, fine_peak_time_local;
    int64_t coarse_peak_time;
    int64_t fine_peak_time;
    float coarse_peak_array[8];       /* > 0: antenna had a valid coarse peak (its smoothed metric) */
    float rms_array[8];
    float cfo_fractional_rad, cfo_integer_rad;
    uint32_t u, b, N_eff_TX, reserved;
    float fine_peak_metric[4];        /* |xcorr| maximum per STF template N_eff_TX = 1, 2, 4, 8 */
    uint32_t fine_peak_index[4];
} dnrp_sync_result;

/* PHY part of pcc_report_t plus the sync_report_t values rx_synced_t refines (rx_synced.cpp:530-580) */
typedef struct {
    float snr_dB;             /* estimator_snr after STF + DRS of the PCC symbols */
    float cfo_fractional_rad; /* sync value + STF re-estimate */
    float sto_fractional;     /* samples, estimator_sto on the STF */
    float rms[8];             /* per RX antenna: the sync report's value where > 0, else the STF estimate */
} dnrp_pcc_report;

/* PHY part of pdc_report_t (rx_synced.cpp:432-435) with its mimo_report_t
 * (phy/rx/rx_synced/mimo/mimo_report.hpp; estimator_mimo.cpp:80-222) */
typedef struct {
    float snr_dB;
    uint32_t mimo_N_RX;                          /* own physical antennas */
    uint32_t mimo_N_TS_other;                    /* transmit streams received (N_eff_TX) */
    uint32_t tm_3_7_beamforming_idx;             /* codebook index recommended to the other side */
    uint32_t tm_3_7_beamforming_reciprocal_idx;  /* codebook index for this side if reciprocal */
} dnrp_pdc_report;

/* Per-packet PDC request = what maclow_phy_t carries once the MAC has decided from the decoded PLCF
 * to continue with the PDC (phy/interfaces/maclow_phy.hpp: continue_with_pdc, hp_rx): the HARQ
 * process' packet configuration (harq::process_rx_t::get_packet_sizes -> psdef), network ID and
 * PLCF type (rx_synced.cpp:325-350), plus the packet's slot in the preceding dnrp_rx_pcc_batch
 * (the rx_synced_t state the reference keeps between demoddecod_rx_pcc and demoddecod_rx_pdc).
 * Packets the MAC rejected (continue_with_pdc = false) are simply not requested. */
typedef struct {
    dnrp_psdef psdef;     /* u, b and N_eff_TX (tm_mode_index) must match the PCC slot's sync report */
    uint32_t pcc_index;   /* slot index i of sr[i] in the preceding dnrp_rx_pcc_batch, each at most once */
    uint32_t network_id;
    uint32_t plcf_type;   /* 1 or 2: selects the PDC descrambling sequence (scrambling_pdc.cpp:41-48) */
} dnrp_pdc_req;

int dnrp_ctx_create(const dnrp_cfg* cfg, dnrp_ctx** out);
int dnrp_ctx_destroy(dnrp_ctx* ctx);
int dnrp_add_network_id(dnrp_ctx* ctx, uint32_t network_id);
int dnrp_get_packet_sizes(const dnrp_ctx* ctx, const dnrp_psdef* psdef, dnrp_packet_sizes* out);
/* Same as dnrp_get_packet_sizes without a context or device: the reference's static
 * sp3::get_packet_sizes (sections_part3/derivative/packet_sizes.cpp:99-236). The oversampled /
 * resampled fields (N_b_DFT_os, N_samples_packet_*_os_rs) are filled from cfg when cfg is not
 * NULL (tx.cpp:429-600 geometry), else 0. Host-only: safe on machines without a GPU. */
int dnrp_compute_packet_sizes(const dnrp_cfg* cfg, const dnrp_psdef* psdef, dnrp_packet_sizes* out);

/*
 * TX: n packets of one configuration.
 *   pcc_d   device [n][25] bytes: 196 rate-matched PCC bits, unscrambled, MSB first
 *   pdc_d   device [n][pdc_stride] bytes: G rate-matched PDC bits, unscrambled, MSB first
 *   iq_out  device [n][N_TX][S] cf32; samples [0, N_samples_packet_no_GI_os_rs) carry the packet,
 *           the rest (GI and slot tail) are written as zeros. S >= N_samples_packet_os_rs.
 */
int dnrp_tx_batch(dnrp_ctx* ctx, const dnrp_psdef* psdef, uint32_t n, const dnrp_tx_desc* desc,
                  const uint8_t* pcc_d, const uint8_t* pdc_d, uint32_t pdc_stride, float* iq_out,
                  uint32_t S, void* stream);

/*
 * Synchronisation: sync_chunk_t::search() on n windows, each window one chunk whose sync resampler
 * starts with zero history at sample 0 (reset_localbuffer, sync_chunk.cpp:300-311). Detection,
 * coarse peak and fine peak as in the reference; up to max_reports packets per window in search
 * order (the reference returns them from successive search() calls).
 *   iq       device cf32; window w, antenna a, sample i at iq[2*(w*win_stride + a*ant_stride + i)]
 *            (strides in samples: [n][N_RX][S] windows or per-antenna continuous streams)
 *   res      host [n][max_reports]; n_found host [n] (optional). Valid after dnrp_sync().
 */
int dnrp_rx_sync_batch(dnrp_ctx* ctx, const dnrp_sync_cfg* sc, uint32_t n, const float* iq, uint64_t win_stride,
                       uint64_t ant_stride, uint32_t S_win, dnrp_sync_result* res, uint32_t* n_found, void* stream);

/*
 * RX phase 1: synchronised PCC demodulation of n packets. Each packet is processed with the
 * (u, b, N_eff_TX) of its own sync report (packets are grouped internally, like independent
 * demoddecod_rx_pcc calls).
 *   sr       host [n]; packet i lies in window sr[i].window of iq_in at sr[i].fine_peak_time (may
 *            be negative: zero history before the window start)
 *   iq_in    device [n_windows][N_RX][S_in] cf32, N_RX = cfg.N_TX_max; DNRP_EINVAL if any
 *            sr[i].window >= n_windows (the kernels read window sr[i].window of iq_in)
 *   pcc_llr  device [n][196] int16, descrambled
 *   rep      host [n] (optional)
 * Device state for phase 2 (STF estimates, PCC-phase channel estimates) is kept in the context
 * until the next dnrp_rx_pcc_batch.
 */
int dnrp_rx_pcc_batch(dnrp_ctx* ctx, uint32_t n, const dnrp_sync_report* sr, const float* iq_in,
                      uint32_t n_windows, uint32_t S_in, int16_t* pcc_llr, dnrp_pcc_report* rep, void* stream);

/*
 * RX phase 2: PDC demodulation of any subset of the packets of the preceding dnrp_rx_pcc_batch,
 * each with its own PLCF-announced configuration (mixed MCS / PacketLength / network IDs are
 * grouped internally).
 *   req      host [m], m <= n of the PCC batch, distinct pcc_index values
 *   iq_in    the PCC call's iq_in, n_windows and S_in: the PDC symbols are read from these windows,
 *            so they must stay valid and unchanged until this call's work has completed
 *   pdc_llr  device [m][llr_stride] int16: row r = the G descrambled LLRs of req[r]
 *   rep      host [m] (optional)
 * Returns DNRP_ESTATE without a preceding PCC batch or for an iq_in / n_windows other than the
 * PCC call's, DNRP_EINVAL for a pcc_index out of range or repeated, a psdef whose u/b/N_eff_TX
 * differ from the slot's sync report, S_in different from the PCC call, or llr_stride < G.
 */
int dnrp_rx_pdc_batch(dnrp_ctx* ctx, uint32_t m, const dnrp_pdc_req* req, const float* iq_in, uint32_t n_windows,
                      uint32_t S_in, int16_t* pdc_llr, uint32_t llr_stride, dnrp_pdc_report* rep, void* stream);

int dnrp_sync(dnrp_ctx* ctx, void* stream);

/*
 * Receiver options beyond the reference (default 0: exactly the reference's receiver).
 *   DNRP_RX_MODE_SM_MMSE  dnrp_rx_pdc_batch demodulates spatial multiplexing (N_SS = N_eff_TX in
 *                         {2, 4}: TM 2/4/6/8/9, N_RX >= N_SS) by linear MMSE per cell, x = (H^H H +
 *                         nv I)^-1 H^H y with the Wiener-interpolated channel of every transmit stream
 *                         and the SNR estimator's noise variance nv, unbiased per stream, then the same
 *                         soft demapper. The reference leaves run_pdc_mode_AxA_MIMO empty
 *                         (rx_synced.cpp:1331-1333) and returns DNRP_EUNSUPPORTED without this flag.
 * Takes effect for the next dnrp_rx_pcc_batch (a preceding PCC batch's state is dropped).
 */
#define DNRP_RX_MODE_SM_MMSE 1u
int dnrp_ctx_set_rx_mode(dnrp_ctx* ctx, uint32_t flags);

/*
 * Ring-buffer window gather <- rx_pacer_t's wrap copy (rx_pacer.cpp:106-143) over the per-antenna
 * ring of radio::buffer_rx_t (radio/buffer_rx.hpp:46-141; sample of global time t at index
 * t % ring_len). Copies window w = global samples [start[w], start[w] + S_win) of antennas
 * 0..N_ant-1 into out [n][N_ant][S_win] cf32 (device), ready for dnrp_rx_sync_batch or the RX.
 *   ring   device cf32, antenna a at ring + 2*a*ant_stride floats (ant_stride >= ring_len)
 *   start  host [n], >= 0; S_win <= ring_len (one wrap at most); n * N_ant <= 65535
 */
int dnrp_ring_gather(dnrp_ctx* ctx, const float* ring, uint64_t ring_len, uint64_t ant_stride, uint32_t N_ant,
                     uint32_t n, const int64_t* start, uint32_t S_win, float* out, void* stream);

/* Continuous-stream synchronisation state = baton_t's uniqueness state (baton.cpp:37-52,157-169):
 * the latest unique fine peak time and the minimum distance to it (worker_pool.cpp:299-321) */
typedef struct {
    int64_t sync_time_last;          /* global hw time of the latest unique packet */
    int64_t sync_time_unique_limit;  /* one STF pattern at b * os_min (..._UNIQUE_LIMIT_IN_STF_PATTERNS_DP) */
    uint64_t packets, not_unique;    /* worker_sync_t stats: job_packet, job_packet_not_unique */
} dnrp_sync_stream_state;

int dnrp_sync_stream_init(const dnrp_ctx* ctx, const dnrp_sync_cfg* sc, dnrp_sync_stream_state* state);

/* hw samples one chunk's search reads from the ring: chunk_len plus the detection overlap into the
 * next chunk, the coarse-peak and cross-correlation spans and the resampler filter (sync_chunk.cpp:
 * 32-123); 0 on a bad argument. Must be <= the ring length. */
uint32_t dnrp_sync_stream_window(const dnrp_ctx* ctx, const dnrp_sync_cfg* sc);

/*
 * Continuous-stream synchronisation <- the sync worker pool (worker_sync_t::work,
 * worker_sync.cpp:57-221) over n_chunks consecutive chunks of sc->chunk_len hw samples starting at
 * global time t0: every chunk's window is gathered from the ring, searched with
 * sync_chunk_t::search() (up to sc->max_reports packets per chunk), its reports converted to global
 * time (coarse_peak_time / fine_peak_time, sync_chunk.cpp:213-245) and passed through the baton's
 * double-detection filter in chunk order (baton.cpp:157-169: unique iff fine_peak_time - last >
 * limit). out (host, n_chunks * max_reports) receives the unique reports in time order, n_out their
 * count, chunk_of (host, optional) the chunk each was found in. Blocking: returns after the stream's
 * work has completed. Call again with t0 advanced by n_chunks * chunk_len to continue the stream.
 */
int dnrp_rx_sync_stream(dnrp_ctx* ctx, const dnrp_sync_cfg* sc, const float* ring, uint64_t ring_len,
                        uint64_t ant_stride, int64_t t0, uint32_t n_chunks, dnrp_sync_stream_state* state,
                        dnrp_sync_result* out, uint32_t* n_out, uint32_t* chunk_of, void* stream);

/*
 * Simulated wireless channel <- the virtual space links of the reference's simulator
 * (lib/src/simulation/wireless/channel_awgn.cpp, channel_flat.cpp, channel_doubly.cpp + link.cpp;
 * noise: lib/src/simulation/hardware/noise.cpp). Applies N_TX x N_RX links to n TX windows:
 *   awgn    every TX antenna superimposed onto every RX antenna (large-scale factor only)
 *   flat    one Rayleigh coefficient per link and window
 *   doubly  tapped delay line per link: a 3GPP power delay profile (link.hpp:88-108, pdp_idx 0..2 =
 *           EPA / EVA / ETU) scaled to tau_rms_ns, 40 Doppler sinusoids per tap (Jakes, fD_Hz)
 * then complex AWGN with n0 = -10 log10(net_bw_norm) - snr_db dB (per unit signal power in the net
 * bandwidth; snr_db >= DNRP_CH_NOISELESS_DB: none). Link realisations are drawn per window from the
 * seed (window index within the call); dnrp_channel_realization returns them (host only).
 *   tx      device [n][N_TX][S_tx] cf32; rx device [n][N_RX][S_rx] cf32 (every sample written)
 *   offset  host [n]: TX sample 0 lands at RX sample offset[w] (zero input outside [0, S_tx))
 *   t0      host [n]: global hw time of RX sample 0 (phases of the Doppler sinusoids)
 */
#define DNRP_CH_AWGN 0
#define DNRP_CH_FLAT 1
#define DNRP_CH_DOUBLY 2
#define DNRP_CH_NOISELESS_DB 1000.0f
typedef struct {
    uint32_t kind;          /* DNRP_CH_* */
    uint32_t pdp_idx;       /* doubly: power delay profile 0..2 */
    float tau_rms_ns;       /* doubly: delay spread, <= 2000 */
    float fD_Hz;            /* doubly: maximum Doppler, <= 2000 */
    uint32_t samp_rate;     /* hw sample rate in S/s (tap delays, Doppler periods) */
    float large_scale;      /* amplitude factor of every link (path loss / RX sensitivity) */
    float snr_db;           /* noise level, see above */
    float net_bw_norm;      /* N_b_OCC / N_b_DFT_os scaled to the hw rate (noise.cpp net_bandwidth_norm) */
    uint64_t seed;
} dnrp_channel_cfg;

int dnrp_channel_batch(dnrp_ctx* ctx, const dnrp_channel_cfg* cfg, uint32_t n, uint32_t N_TX, const float* tx,
                       uint32_t S_tx, uint32_t N_RX, const int64_t* offset, const int64_t* t0, float* rx, uint32_t S_rx,
                       void* stream);
/* Host only: window w's realisation. n_taps receives the taps per link (doubly); arrays (optional)
 * are [N_RX][N_TX][n_taps] delay (samples) / amp, [N_RX][N_TX][n_taps][40] period / phase_rev
 * (initial phase in revolutions), [N_RX][N_TX][2] coef (flat). */
int dnrp_channel_realization(const dnrp_channel_cfg* cfg, uint32_t window, uint32_t N_TX, uint32_t N_RX, uint32_t* n_taps,
                             int32_t* delay, float* amp, int64_t* period, double* phase_rev, float* coef);

/* Host only. N_samples_transmit_os_rs: the samples a radio buffer holds once the packet is complete
 * (packet without GI + GI_percentage % of the GI, tx.cpp:555-566) = the final value of the
 * reference's progressive buffer_tx_t::set_tx_length_samples_cnt (tx.cpp:241,277,292). dnrp_tx_batch
 * completes every buffer before its stream work completes; samples past this length are zero. */
int dnrp_tx_transmit_length(const dnrp_cfg* cfg, const dnrp_psdef* psdef, uint32_t GI_percentage, uint32_t* len);

/* Host only: JSON export in the reference's formats.
 *   dnrp_tx_packet_json <- tx_t::write_all_data_to_json (tx.cpp:316-427): packet definition, TX
 *     meta, d-bits of PCC and PDC (PLCF / TB fields empty: they sit above the FEC), the antenna
 *     streams (host copy of dnrp_tx_batch's iq_out row, [N_TX][S] cf32) up to the transmit length,
 *     resampler parameters.
 *   dnrp_rx_packet_json <- worker_tx_rx_t::collect_and_write_json's RADIO/PHY part
 *     (worker_tx_rx.cpp:354-396; rx_synced's channel estimates are not exported). */
int dnrp_tx_packet_json(const dnrp_cfg* cfg, const dnrp_psdef* psdef, const dnrp_tx_desc* desc, uint32_t rv,
                        uint64_t tx_order_id, int64_t tx_time_64, const uint8_t* pcc_d, const uint8_t* pdc_d,
                        const float* iq, uint32_t S, const char* path);
int dnrp_rx_packet_json(const dnrp_cfg* cfg, uint32_t worker_id, const dnrp_sync_result* sr, uint32_t mcs_index,
                        const dnrp_pcc_report* pcc, const dnrp_pdc_report* pdc, const char* path);

/* sp3::radio_device_class_t (sections_part3/radio_device_class.hpp): the capabilities of a device
 * class string such as "8.16.8.A"; a worker pool sizes itself from them (dnrp_cfg.u_max = u_min,
 * b_max = b_min, N_TX_max = N_TX_min, as worker_pool_config_t does). Host only. DNRP_ECONFIG for a
 * class the reference does not list (radio_device_class.cpp:26-150). */
typedef struct {
    uint32_t u_min, b_min, N_TX_min, mcs_index_min, M_DL_HARQ_min, M_connection_DL_HARQ_min, N_soft_min, Z_min;
    uint32_t PacketLength_min;
} dnrp_radio_device_class;
int dnrp_get_radio_device_class(const char* name, dnrp_radio_device_class* out);

/* The reference parameters the library is built with, by the reference's own names (sync_param.hpp
 * RX_SYNC_PARAM_*, rx_synced_param.hpp RX_SYNCED_PARAM_* incl. "NAME[i]" vector entries, flags as
 * 1 = defined / 0 = not defined, resampler_param_t::f_pass_norm[user][os] etc., constants::*).
 * Host only: DNRP_EINVAL for an unknown name. dnrp_param_name(i) enumerates them (NULL past the end). */
int dnrp_query_param(const char* name, double* value);
const char* dnrp_param_name(uint32_t index);
/* The literal tables of sections_part3 the library builds its device tables from (host only), for
 * pinning against the reference's own text (tests/golden/ref_literals.json). Returns the number of
 * floats (out may be NULL to ask for it; cap = floats available), DNRP_EINVAL for an unknown name or
 * bad arguments. Names (arguments):
 *   "W" (N_TS, N_TX, codebook)   W_t matrix [N_TX][N_TS] re/im (Tables 6.3.4-1..6)
 *   "W_scaling" / "W_scaling_optimal_DAC" (N_TS, N_TX, codebook)   its scaling factor (tx.cpp:582-592)
 *   "W_codebooks" (N_TS, N_TX)   number of codebook entries
 *   "stf" (b, N_eff_TX)          stf_t transmit-stream vector [N_b_OCC + 1] re/im, scale 1 (stf.cpp:185-285)
 *   "drs_values" (b, t)          the N_b_OCC/4 DRS values of transmit stream t (drs.cpp:227-254)
 *   "txdiv_pairs" (N_TS)         Y_i_t::index_N_TS_x rows A0 B0 A1 B1 ... (transmit_diversity_precoding.cpp:48-75)
 *   "stf_cover_sequence" ()      stf_t::cover_sequence (stf.hpp:146-151)
 *   "cells_lds_bytes" (u_max, b_max, b, N_RX, N_eff_TX)   LDS bytes of the PDC equaliser's staging for
 *                                the geometry; above 160 KiB dnrp_rx_*_batch return DNRP_EUNSUPPORTED */
int dnrp_query_table(const char* name, const uint32_t* arg, uint32_t n_arg, float* out, uint32_t cap);

/* Kernel timing (only when the environment has DNRP_TIMING=1 at dnrp_ctx_create): HIP events
 * recorded on the caller's stream around each launch. Names: "tx", "sync_steps", "sync_detect",
 * "sync_post", "sync_fine", "rx_stf", "rx_fft_pcc", "rx_pcc", "rx_fft_pdc", "rx_pdc". */
int dnrp_last_kernel_ms(const dnrp_ctx* ctx, const char* name, float* ms);
int dnrp_kernel_time_total(dnrp_ctx* ctx, const char* name, float* total_ms, uint32_t* count, int reset);

/*
 * Channel coding (host only) <- phy/fec/fec.cpp (fec_t), pcc_enc.cpp, pdc_enc.cpp and
 * sections_part3/fix/cbsegm.cpp: CRC attachment, code-block segmentation, LTE turbo code (TS 36.212
 * §5.1.3, QPP interleaver), turbo rate matching (§5.1.4.1) and a max-log-MAP turbo decoder with
 * CRC early stopping. The split with the GPU path is the reference's scrambler: the encoders output
 * the rate-matched d-bits dnrp_tx_batch takes (pcc_d / pdc_d: unscrambled, MSB first) and the
 * decoders take the descrambled int16 LLRs dnrp_rx_pcc_batch / dnrp_rx_pdc_batch return.
 */
#define DNRP_CRC16 0   /* PLCF CRC, g = 0x1021 (pcc_enc.cpp:88-91) */
#define DNRP_CRC24A 1  /* transport-block CRC, g = 0x864CFB (pdc_enc.cpp:60-63) */
#define DNRP_CRC24B 2  /* code-block CRC, g = 0x800063 (pdc_enc.cpp:56-59) */

/* srsran_cbsegm_t as filled by srsran_cbsegm_FIX (cbsegm.cpp:65-123): C2 blocks of K2 first */
typedef struct {
    uint32_t tbs, Z, C, C1, C2, K1, K2, K1_idx, K2_idx, F;
} dnrp_cbsegm;

/* sp3::fec_cfg_t (sections_part3/derivative/fec_cfg.hpp). PLCF_type and network_id select the
 * scrambling sequence, which the GPU path applies: they are carried for the mirror only. */
typedef struct {
    uint32_t PLCF_type, closed_loop, beamforming, N_TB_bits, N_bps, rv, G, network_id, Z;
} dnrp_fec_cfg;

/* HARQ RX softbuffer (harq::buffer_rx_t): accumulated code-block softbits, code-block CRC flags
 * and the code blocks already decoded, kept across redundancy versions of one transport block. */
typedef struct dnrp_harq_rx dnrp_harq_rx;

int dnrp_crc(const uint8_t* data, uint32_t nbits, uint32_t kind, uint32_t* crc);
int dnrp_fec_cbsegm(uint32_t N_TB_bits, uint32_t Z, dnrp_cbsegm* out);
/* row idx (0..187) of TS 36.212 Table 5.1.3-3: K and the QPP coefficients f1, f2 (optional) */
int dnrp_fec_cb_size(uint32_t idx, uint32_t* K, uint32_t* f1, uint32_t* f2);

/* fec_t::encode_plcf without the scrambling: plcf (5 or 10 bytes) -> d [25] bytes (196 bits).
 * closed_loop / beamforming select the CRC mask (pcc_enc.cpp:170-183). */
int dnrp_pcc_encode(const uint8_t* plcf, uint32_t plcf_type, uint32_t closed_loop, uint32_t beamforming, uint8_t* d);
/* fec_t::decode_plcf_test after the descrambling: llr [196] -> 1 if a PLCF of plcf_type_test passed
 * its CRC under one of the four masks (plcf [5 or 10], closed_loop, beamforming set), 0 if not.
 * Up to 5 turbo iterations, stopping at the first CRC match (pcc_enc.cpp:309-351). */
int dnrp_pcc_decode(const int16_t* llr, uint32_t plcf_type_test, uint8_t* plcf, uint32_t* closed_loop,
                    uint32_t* beamforming, uint32_t* iterations);

/* fec_t::encode_tb without the scrambling: tb [N_TB_bits/8] -> d [ceil(G/8)] (redundancy version
 * cfg->rv). DNRP_ECONFIG for a segmentation with filler bits (pdc_enc.cpp:144). */
int dnrp_pdc_encode(const dnrp_fec_cfg* cfg, const uint8_t* tb, uint8_t* d);
/* fec_t::decode_tb after the descrambling: the first n_llr <= G LLRs of the packet (code blocks
 * whose soft bits are not all present yet are left for a later call, pdc_enc.cpp:334-337) ->
 * tb [N_TB_bits/8]. Returns 1 if the transport block passed its CRC(s), 0 if not. hb: the HARQ
 * softbuffer to combine into (reset it for a new transport block), or NULL for a one-shot decode.
 * Up to 10 iterations per code block, CRC early stop after at least 2. */
int dnrp_pdc_decode(dnrp_harq_rx* hb, const dnrp_fec_cfg* cfg, const int16_t* llr, uint32_t n_llr, uint8_t* tb,
                    uint32_t* iterations);
/*
 * Device turbo decoding of m transport blocks <- fec_t::decode_tb for many packets at once (one-shot:
 * a fresh softbuffer, all G soft bits present), with the host decoder's arithmetic: each code block
 * decodes to the same bits after the same number of iterations as dnrp_pdc_decode.
 *   cfg         host [m]: N_TB_bits, N_bps, rv, G, Z of each packet
 *   llr         device, row i at llr + i*llr_stride (>= G_i): descrambled LLRs (dnrp_rx_pdc_batch output)
 *   tb          device, row i at tb + i*tb_stride (>= N_TB_bits_i/8 + 3): decoded transport block
 *               followed by its received CRC24A
 *   crc_ok      host [m]: 1 if every code block and the transport block passed their CRCs
 *   iterations  host [m] (optional): turbo iterations summed over the packet's code blocks
 * Blocking: returns after the work on the stream has completed.
 */
int dnrp_pdc_decode_batch(dnrp_ctx* ctx, uint32_t m, const dnrp_fec_cfg* cfg, const int16_t* llr, uint32_t llr_stride,
                          uint8_t* tb, uint32_t tb_stride, uint8_t* crc_ok, uint32_t* iterations, void* stream);
/* The same with HARQ soft combining (harq::buffer_rx_t on the device): per packet a softbuffer row
 * (softbuf + i*sb_stride int16, >= dnrp_pdc_softbuffer_size entries) and code-block CRC flags
 * (cb_crc + i*crc_stride, >= C bytes), both zeroed by the caller for a new transport block and kept
 * across its redundancy versions, like the host dnrp_pdc_decode with a dnrp_harq_rx: blocks that
 * passed earlier are neither combined nor decoded again (their bytes stay in the tb row, so pass the
 * same tb rows for every redundancy version), the others add the new soft bits; a transport-block
 * CRC failure after all block CRCs passed resets the packet's flags. Same results as the host path. */
int dnrp_pdc_decode_batch_harq(dnrp_ctx* ctx, uint32_t m, const dnrp_fec_cfg* cfg, const int16_t* llr,
                               uint32_t llr_stride, int16_t* softbuf, uint64_t sb_stride, uint8_t* cb_crc,
                               uint32_t crc_stride, uint8_t* tb, uint32_t tb_stride, uint8_t* crc_ok, uint32_t* iterations,
                               void* stream);
/* softbuffer entries (C * 3 * (K+ + 4)) and code blocks of a transport block (host only) */
int dnrp_pdc_softbuffer_size(uint32_t N_TB_bits, uint32_t Z, uint64_t* entries, uint32_t* n_cb);
/*
 * Device channel encoding of m transport blocks <- fec_t::encode_tb for many packets at once
 * (without the scrambling): bit-exact with dnrp_pdc_encode.
 *   tb  device, row i at tb + i*tb_stride (>= N_TB_bits_i/8)
 *   d   device, row i at d + i*d_stride (>= ceil(G_i/8)): the pdc_d rows dnrp_tx_batch takes
 * Blocking: returns after the work on the stream has completed.
 */
int dnrp_pdc_encode_batch(dnrp_ctx* ctx, uint32_t m, const dnrp_fec_cfg* cfg, const uint8_t* tb, uint32_t tb_stride,
                          uint8_t* d, uint32_t d_stride, void* stream);
/*
 * Device PLCF decoding of n PCCs <- fec_t::decode_plcf_test for many packets at once (after the
 * descrambling): turbo decoding (K = 56 / 96, up to 5 iterations, stop at the first CRC match) and
 * the CRC16 check under the four masks, with the host decoder's arithmetic (same bits, iterations).
 *   plcf_type_test  host [n]: 1 or 2 per packet
 *   llr             device, row i at llr + i*llr_stride (>= 196): dnrp_rx_pcc_batch's pcc_llr
 *   plcf            device, row i at plcf + i*plcf_stride (>= 10): the decoded PLCF (5 or 10 bytes)
 *   result          host [n]: 0 = no PLCF of that type; 1 + m for a CRC match under mask m
 *                   (0 none, 1 closed loop, 2 beamforming, 3 both: pcc_enc.cpp:170-183)
 *   iterations      host [n] (optional)
 * Blocking: returns after the work on the stream has completed.
 */
int dnrp_pcc_decode_batch(dnrp_ctx* ctx, uint32_t n, const uint32_t* plcf_type_test, const int16_t* llr,
                          uint32_t llr_stride, uint8_t* plcf, uint32_t plcf_stride, uint8_t* result, uint32_t* iterations,
                          void* stream);
/* Device PLCF encoding of n packets <- fec_t::encode_plcf for many packets at once (without the
 * scrambling): bit-exact with dnrp_pcc_encode.
 *   plcf_type host [n] (1 / 2); closed_loop, beamforming host [n] (optional, CRC mask selection)
 *   plcf      device, row i at plcf + i*plcf_stride (5 or 10 bytes)
 *   d         device, row i at d + i*d_stride (>= 25): dnrp_tx_batch's pcc_d rows
 * Blocking: returns after the work on the stream has completed. */
int dnrp_pcc_encode_batch(dnrp_ctx* ctx, uint32_t n, const uint32_t* plcf_type, const uint32_t* closed_loop,
                          const uint32_t* beamforming, const uint8_t* plcf, uint32_t plcf_stride, uint8_t* d,
                          uint32_t d_stride, void* stream);
int dnrp_harq_rx_create(uint32_t N_TB_bits_max, uint32_t Z, dnrp_harq_rx** out);
int dnrp_harq_rx_reset(dnrp_harq_rx* hb);
int dnrp_harq_rx_destroy(dnrp_harq_rx* hb);

const char* dnrp_strerror(int code);

#ifdef __cplusplus
}
#endif

#endif /* DNRP_H */
