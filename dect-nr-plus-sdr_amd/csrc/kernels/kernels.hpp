// Kernel argument blocks and launchers shared by the host context (host/ctx.cpp) and the HIP
// kernels (kernels/*.hip). Plain structs, passed by value as kernel arguments.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "device_common.hpp"
#include "../params.hpp"

namespace dnrp::dev {

// TX cell codes: type in bits 29-31; PCC/PDC: cell index j in bits 0-19 and the transmit
// diversity TS pair A | B << 4 of cell j (pair table entry (j >> 1) % mod) in bits 20-27
// (host-precomputed); DRS: stream | sign << 3
enum : uint32_t {
    CODE_J_MASK = 0xFFFFFu,
    CODE_PAIR_SHIFT = 20,
    CODE_PCC = 1u << 29,
    CODE_PDC = 2u << 29,
    CODE_DRS = 3u << 29,
    CODE_STF = 4u << 29,
    CODE_MASK = 7u << 29,
    // one-hot W rows (tx.hip TXS_TXDIV1 / TXS_SM1): the code of a bin as seen by the antenna whose
    // nonzero W entry is stream ts (host-built per ts, ctx.cpp). Type PCC / PDC / DRS only where that
    // stream carries the cell (else 0); bits 0..19: the symbol index to map (SFBC partner or spatial
    // stream resolved), OH_FX / OH_FY: sign of its re / im part flipped (DRS: the point (1, 0), OH_FX
    // for the value -1)
    OH_FX = 1u << 20,
    OH_FY = 1u << 21,
};

// ---------------------------------------------------------------- TX
struct tx_pkt {
    const uint8_t* pdc_seq;  // packed Gold sequence for (network_id, plcf_type)
    uint32_t codebook, do_mix;
    float scale_stf, scale_df;
    double ph0, inc;  // effective mixer phase and per-sample increment (float phasor emulated)
};

struct tx_args {
    fft_plan plan;  // IFFT size N_b_DFT_os
    uint32_t N_occ, off_lower, CP, STF_CP, N_DF, N_TS, N_TX, N_SS, N_bps, txdiv, mod, pattern_len;
    uint32_t L, M, delay, hl, n_keep, S, pdc_stride, G;
    uint32_t m_star, p_star;  // first phase-0 output (delay + m_star*M = p_star*L), polyphase.hpp
    // symbol runs: WG (packet, antenna, run) synthesises symbols [run*K, run*K+K) plus the symbol
    // before them (resampler history) into a linear cyclic-prefixed buffer of lin_len samples
    uint32_t K, n_runs, HP, lin_len, bufB_len;
    uint32_t stage_bytes;  // PDC source bytes of one run staged in LDS (0: read HBM directly)
    uint32_t mfma;         // streaming kernel: polyphase blocks on the matrix cores (split fp16)
    uint32_t pair[12];     // transmit diversity TS pairs, A | B << 4
    const uint32_t* code;
    const uint32_t* pdc_off;  // [N_DF+2] first PDC cell of each symbol
    const float2* stf;
    const float2* W;     // [codebooks][N_TX][N_TS]
    const float* taps;     // [(hl+1)*L]
    const float* taps_pp;  // input-major block taps [W][LP] (polyphase.hpp)
    uint32_t npp;          // floats in taps_pp
    const float2* tw;      // forward twiddles exp(-2 pi i j / N)
    const float2* qam;     // constellation for N_bps
    const float2* qpsk;  // QPSK table for the PCC
    const uint8_t* pcc_seq;
    const uint8_t* pcc_d;
    const uint8_t* pdc_d;
    float* out;
    const tx_pkt* pk;
    // streaming kernel (tx_stream_kernel, N_b_DFT_os = 1024, L/M = 10/9, CP 128 / STF CP 1280):
    // one wavefront per (packet, antenna, segment of 1152-sample input pieces)
    const uint32_t* code_bin;  // [N_DF+1][1024] cell code of every FFT bin (0: empty), bin lane + 64 m at [m / 4][lane][m % 4]
    uint32_t n_pieces, n_seg, piece_per_seg, stream;
    uint32_t pcc_syms;         // bit l: symbol l (< 32) carries PCC cells
    uint32_t onehot;           // transmit diversity with one nonzero W entry per antenna row (every packet)
    const uint32_t* code_oh;   // onehot: [N_TS][N_DF+1][1024] per-stream codes (code_bin layout), see OH_*
    uint32_t sb_chunks;        // spatial multiplexing: 1 KiB chunks of a symbol's PDC staging window (<= 4)
    // N_b_DFT_os > 1024 (beyond the block path's registers): every symbol's cyclic-prefixed DECT-rate
    // samples through a scratch [packet][antenna][big_len] (tx_big_sym_kernel, tx_big_resample_kernel)
    float2* big;
    uint32_t big_len;
    uint32_t big_batch;  // packets per scratch pass (the scratch holds big_batch x N_TX rows)
};
hipError_t launch_tx(const tx_args& a, uint32_t n, hipStream_t st);
bool tx_stream_taps_match(const float* h, size_t n);  // compiled-in 10/9 taps == run-time taps

// ---------------------------------------------------------------- RX
struct rx_pkt_in {          // from sync_report_t
    int64_t fine_peak;
    double inc0;            // effective CFO phasor increment (float phasor emulated)
    float cfo_rad;          // sync CFO (fractional + integer)
    uint32_t win;           // window of iq_in holding the packet (dnrp_sync_report::window)
};

struct rx_pkt_state {       // written by rx_stf_kernel, read by the later RX kernels
    double inc1;            // mixer increment after the STF fine CFO adjustment
    double sto_inc;         // STO phase increment per subcarrier
    double snr_SN, snr_N;   // SNR accumulators after the STF
    uint32_t snr_SN_cnt, snr_N_cnt;
    float cfo_fine, sto_frac;
    float rms[8];
    float snr_pcc, snr_pdc;
};

struct rx_front_args {
    fft_plan plan;
    uint32_t N_occ, off_lower, CP, STF_CP, N_RX, S_in, n_pattern, pattern_len, b;
    uint32_t L, M, delay, hl;  // RX resampler (L and M already swapped)
    uint32_t m_star, p_star;   // first phase-0 output (delay + m_star*M = p_star*L), polyphase.hpp
    uint32_t sym_first, sym_count, sym_per_block, Nf_pad, n_sym_total;
    float amp_scale;           // sqrt(N_b_OCC) / N_b_DFT_os
    const float* taps;
    const float* taps_pp;      // input-major block taps [W][LP] (polyphase.hpp)
    uint32_t npp;              // floats in taps_pp
    const float2* tw;
    const float2* stf;         // STF values for (b, N_eff_TX)
    const float2* iq;          // [windows][N_RX][S_in]
    const rx_pkt_in* pin;
    rx_pkt_state* st;
    float2* Y;                 // [n][N_RX][n_sym_total][Nf_pad]
    uint32_t stream;           // compile-time-tap front end allowed (host: compiled-in taps match)
    const uint32_t* sel;       // [launch packets][2]: PCC-batch slot, output row (rx_slot_of / rx_row_of)
    // DRS SNR partial sums taken while a DRS symbol's bins are in the wave (rx_fft_wave_kernel):
    // snr_part[((slot n_sym_total + l) N_RX + rx) 8 + ts_first] = (sum |w y|^2, sum |w y_i - w y_i+1|^2)
    // over the DRS cells of every stream of the op at symbol l (estimator_snr.cpp:104-146 terms);
    // null: rx_snr gathers them from Y. The DRS cells are computed, not loaded: stream t, parity p,
    // cell i at occupied index 4 i + (t + 2 p) % 4 (DC skipped), value -+1 from drs_neg bit
    // (4 i + t % 4) % 56, negated for t >= 4 (drs.cpp:196-254; host-checked against drs_k / drs_v)
    double2* snr_part;
    const uint32_t* dl;        // the phase plan's DRS ops (rx_snr_args)
    const uint32_t* dmeta;
    uint64_t drs_neg;          // bit j: y_b_1[j] = -1 (drs.hpp)
    const uint16_t* sym_op;    // [n_sym_op]: first DRS op of symbol l, 0xFFFF: none
    uint32_t n_dops, n_drs, n_sym_op;
    // STF front end per (packet, antenna) (rx_stf_ant_kernel -> rx_stf_kernel): per slot and antenna
    // the cover-reverted pattern correlation sum, the RMS and the b*14 STF cells
    double2* stf_cs;           // [slot][8]
    float* stf_rms;            // [slot][8]
    float2* stf_ys;            // [slot][8][stf_ys_stride]
    uint32_t stf_ys_stride;
    // symbol list of the launch (rx_fft_wave_kernel): launch symbol i is sym_list[i] instead of
    // sym_first + i (the PDC phase's DRS symbols ahead of the fused receiver, rx_fused.hip)
    const uint16_t* sym_list;
    uint32_t no_y;             // 1: the bins are not stored to Y (nothing reads them there)
    // zero-forced DRS pilots taken with the SNR partial sums (rx_drs_partials), the fused PDC
    // receiver's pilot source: zd[((slot zd_dops + d) N_RX + rx) 4 + t][zd_row] (DRS op d of the phase
    // plan; the PCC plan's ops are the prefix of the PDC plan's), null: not written
    float2* zd;
    uint32_t zd_dops, zd_row;
    uint32_t fft_pass, fft_tw_lds;  // rx_fft_kernel layout (launch_rx_fft: symbols per pass, LDS twiddles)
    uint32_t stf_chunk;             // rx_stf_ant_kernel: 0, or outputs per resampling chunk (launch_rx_stf)
    uint32_t y_plain;               // 1: Y stored with plain (cache-allocating) stores, re-read from the
                                    // caches by the next packet group's back end; 0: nontemporal stores
};
bool rx_fft_wave_path(const rx_front_args& a);  // launch_rx_fft takes rx_fft_wave_kernel (snr_part supported)
hipError_t launch_rx_stf(const rx_front_args& a, uint32_t n, hipStream_t st);
bool rx_front_fits(const rx_front_args& a);  // the STF and FFT front-end launches fit the 160 KiB LDS
bool rx_stream_taps_match(const float* h, size_t n);  // compiled-in 9/10 taps == run-time taps
hipError_t launch_rx_fft(const rx_front_args& a, uint32_t n, hipStream_t st);

// Packet selection of one RX launch: launch-local packet i works on PCC-batch slot sel[2i] (its
// window, state and Y rows) and writes output row sel[2i+1] (LLRs, reports). The host groups the
// packets of a batch call by configuration and launches each group with its own sel slice.
__device__ __forceinline__ uint32_t rx_slot_of(const uint32_t* sel, uint32_t i) { return sel[2 * i]; }
__device__ __forceinline__ uint32_t rx_row_of(const uint32_t* sel, uint32_t i) { return sel[2 * i + 1]; }
constexpr uint32_t RX_MAX_DOPS = 64;  // DRS ops per phase; lut_d holds RX_MAX_DOPS bytes per slot

// back end, see geometry.hpp rx_plan_t (identical layouts)
struct rx_seg {
    uint32_t kind, l, j0, j1, mode, rel, swap, off, drs_cnt, u0;
};
struct rx_epoch {
    uint16_t src[4][2];
    uint32_t seg0, seg1, units;
};

struct rx_snr_args {        // DRS zero-forcing SNR chain + LUT profile picks, one WG per packet
    uint32_t N_RX, Nf_pad, n_sym_total, n_drs, n_dops, is_pdc;
    const uint32_t* dl;     // per DRS op: symbol
    const uint32_t* dmeta;  // per DRS op: ts_first | ts_last << 8 | parity << 16
    const uint32_t* drs_k;  // [2][4][n_drs]
    const float* drs_v;     // [8][n_drs]
    float prof_snr[3];
    const float2* Y;
    rx_pkt_state* st;
    uint8_t* lut_d;         // [slot][RX_MAX_DOPS]: profile picked after each DRS op
    float* nv_d;            // [slot][RX_MAX_DOPS]: noise variance per RX cell after each DRS op
    const uint32_t* sel;    // launch packet -> slot / output row
    const double2* snr_part;  // front-end partial sums (rx_front_args::snr_part) or null: gather from Y
};
hipError_t launch_rx_snr(const rx_snr_args& a, uint32_t n, hipStream_t st);

struct rx_lut {             // one Wiener LUT: [T][4][Nf] pilot | weight << 16, weights [n_vec][n]
    const uint32_t* pw;
    const float* w;
    uint32_t n, nw;         // taps per weight vector, floats in w (n_vec n)
    // SFBC pairs of a full PDC symbol (pair u on subcarriers 2u, 2u + 1, DC skipped) per LUT row and
    // stream class c = (t & 3) ^ swap: the union window's first pilot (LUT units) and its 4 mean
    // weights 0.5 (w_k0 + w_k1) (eq_compute's, zero-padded); null where a union window exceeds 4 taps
    const float4* pair_w;   // [T][4][N_occ / 2]
    const uint32_t* pair_p; // [T][4][N_occ / 2]
};

struct rx_cells_args {      // equalisation + demapping, one WG per (packet, epoch)
    uint32_t N_occ, N_RX, NT, Nf_pad, n_sym_total, n_drs, n_dops, n_epochs, N_bps, mod, is_pdc;
    uint32_t n_pkt;  // launch packets (the grid is padded to whole XCD rounds, rx_cells_kernel)
    uint32_t sm;               // 1: spatial multiplexing, NT = N_SS streams per cell, MMSE (unit = cell)
    uint32_t wcap[2];          // floats of the LDS weight-table slot of mode l / lr (largest such table)
    uint32_t pair[12];
    const rx_epoch* epochs;
    const rx_seg* segs;
    const uint32_t* dl;
    const uint32_t* dmeta;
    const uint32_t* drs_k;
    const float* drs_v;
    const uint32_t* kk;        // pcc_k (PCC phase) or pdc_k (PDC phase)
    const uint16_t* cell_sym;  // per PCC (PCC phase) / PDC cell: OFDM symbol
    const rx_lut* luts;        // [mode l / lr][profile] (device table: no dynamic kernel-argument indexing)
    const float2* Y;
    const uint8_t* lut_d;
    const float* nv_d;         // [slot][RX_MAX_DOPS] noise variance after each DRS op (MMSE)
    const uint8_t* pcc_seq;
    const uint8_t* const* pdc_seq;  // per output row (PDC phase)
    int16_t* llr;                   // PCC: [n][196], PDC: [m][llr_stride] (output rows)
    uint32_t llr_stride;
    const uint32_t* sel;            // launch packet -> slot / output row
};
hipError_t launch_rx_cells(const rx_cells_args& a, uint32_t n, hipStream_t st);

// PDC phase per (packet, epoch) workgroup (rx_epoch.hip): the front end of the epoch's symbols
// (ep_sym[ep_off[e] .. ep_off[e + 1]), each symbol in exactly one epoch) into Y, then the epoch's
// equalisation from those rows. N_b_DFT_os = 1024 with the compile-time 9/10 taps; MRC / SFBC.
struct rx_epoch_args {
    rx_front_args F;
    rx_cells_args C;
    const uint16_t* ep_off;  // [n_epochs + 1]
    const uint16_t* ep_sym;
};
bool rx_epoch_supported(uint32_t N_RX, uint32_t NT);
size_t rx_epoch_lds(const rx_cells_args& a);
hipError_t launch_rx_epoch(const rx_epoch_args& x, uint32_t n, hipStream_t st);
// spatial multiplexing (a.sm): N_RX x N_SS in {2, 4, 8} x {2, 4} with N_RX >= N_SS
hipError_t launch_rx_cells_sm(const rx_cells_args& a, uint32_t n, hipStream_t st);

// rx_cells_kernel's per-workgroup LDS staging (rx_back.hip, rx_eq.hpp).
// The epoch's pilot buffer zfi: one row per (rx, ts) of 2 nd interlaced pilots plus ZFI_PAD zeros (a
// union window may run past a row's last pilot). Rows start on the same bank (stride a multiple of 32
// float2 = 64 dwords): a wave's lanes take consecutive SFBC pairs, whose streams alternate between
// rows while their pilot positions advance by one per lane, so one read instruction of the wave hits
// bank 2 p_lane + const whatever row each lane is in -- 32 distinct even banks per half-wave. (With
// rows 2 nd + 8 slots apart, 912 dwords for b = 16, lanes 8 apart in different rows collided.)
constexpr uint32_t ZFI_PAD = 8;
constexpr uint32_t CELL_MAX_SEGS = 64;  // segments per epoch (host-checked, rx_plan_dev)
__host__ __device__ constexpr uint32_t zfi_stride(uint32_t n_drs) { return (2 * n_drs + ZFI_PAD + 31) / 32 * 32; }

// An epoch segment with the packet's Wiener LUT resolved: the LUT row block of the segment's
// processing-stage symbol and its weight table's slot in LDS
struct cell_seg {
    uint32_t u0, j0, l;
    uint32_t info;       // mode | swap << 1 | off << 4 | nI << 12
    const uint32_t* pw;  // LT.pw + rel * 4 * Nf
    uint32_t wbase, pad;
};

// LDS bytes of one rx_cells workgroup: pilot buffer, the weight-table slots of mode l and lr,
// segments, SFBC pairs
__host__ __device__ constexpr size_t cell_lds_bytes(uint32_t N_RX, uint32_t NT, uint32_t n_drs, uint32_t wcap_l,
                                                    uint32_t wcap_lr) {
    return size_t(N_RX) * NT * zfi_stride(n_drs) * 8 + size_t(wcap_l + wcap_lr) * 4 + CELL_MAX_SEGS * sizeof(cell_seg) +
           16 * 4;
}


// ---- fused PDC receiver (rx_fused.hip): one workgroup per (packet, PDC symbol), one wavefront per RX
// antenna resamples, mixes and transforms its antenna's symbol into LDS (or loads the bins a
// preceding launch left in Y), then the workgroup equalises the symbol's cells from LDS with the
// Wiener-interpolated channel of the zero-forced DRS pilots (zd) and writes the LLRs: no Y round trip.
struct rx_fsym {                // one PDC-bearing symbol of the phase plan
    uint32_t l, j0, j1;         // OFDM symbol, its PDC cells [j0, j1)
    uint32_t info;              // mode | swap << 1 | off << 4 | from_y << 12 (bins from Y: PCC-phase or DRS symbol)
    uint32_t rel, drs_cnt;      // LUT row, DRS ops before the event (LUT profile pick)
    uint16_t src[4][2];         // epoch pilot sources: DRS op of (stream, interlace slot), 0xFFFF none
};
struct rx_fused_args {
    rx_front_args F;            // front end (F.sym_* unused), Y, zd
    uint32_t n_pkt, n_fsym, NT, N_bps, mod, pad0;
    uint64_t pair_bits;         // SFBC pair i (A | B << 4) in bits 8i..8i+7 (mod <= 6 for N_eff_TX <= 4)
    const rx_fsym* fsym;
    const uint32_t* kk;         // pdc_k
    const rx_lut* luts;         // [mode][profile]
    const uint8_t* lut_d;       // [slot][RX_MAX_DOPS] profile after each DRS op (rx_snr_kernel)
    const uint8_t* const* pdc_seq;  // per output row
    int16_t* llr;
    uint32_t llr_stride;
};
hipError_t launch_rx_fused(const rx_fused_args& a, hipStream_t st);
bool rx_fused_supported(uint32_t N_RX, uint32_t NT);  // instantiated (N_RX, N_eff_TX) pairs

struct rx_mimo_args {  // estimator_mimo_t::process_drs at the packet end, one wavefront per packet
    uint32_t N_RX, N_TS, Nf_pad, n_sym_total;
    uint32_t ncb_tx, A_tx, ncb_rx, A_rx;  // single-stream codebooks (1, N_TS) and (1, N_RX): size, first used
    const uint32_t* cells;  // [N_TS][4]: symbol << 16 | subcarrier index of the wideband DRS cells
    const float* signs;     // [N_TS][4]: DRS value (+-1)
    const float2* Wtx;      // [ncb_tx][N_TS]
    const float* stx;       // [ncb_tx] scaling factors
    const float2* Wrx;      // [ncb_rx][N_RX]
    const float* srx;
    const float2* Y;
    uint32_t* out;          // [row][3]: N_TS_other, tm_3_7_beamforming_idx, tm_3_7_beamforming_reciprocal_idx
    const uint32_t* sel;    // launch packet -> slot / output row
    // fused PDC receiver: the cells from the zero-forced pilots zd (rx_front_args::zd) instead of Y;
    // zcells[N_TS][4] = DRS op << 16 | DRS cell index
    const float2* zd;
    const uint32_t* zcells;
    uint32_t zd_dops, zd_row;
};
hipError_t launch_rx_mimo(const rx_mimo_args& a, uint32_t n, hipStream_t st);


// ---- ring-buffer window gather (ring.hip): buffer_rx_t ring -> linear windows (rx_pacer.cpp:106-143)
constexpr int RING_PAIRS = 4;  // sample pairs per thread
struct ring_args {
    const float2* ring;     // antenna a at ring + a * ant_stride, ring_len samples each
    uint64_t ring_len, ant_stride;
    const int64_t* start;   // [n] global start time of each window (>= 0), device
    float2* out;            // [n][n_ant][S_win]
    uint32_t n_ant, S_win;
};
hipError_t launch_ring_gather(const ring_args& a, uint32_t n, hipStream_t st);

// ---- simulated wireless channel (channel.hip): simulation/wireless channel_{awgn,flat,doubly}
enum : uint32_t { CH_AWGN = 0, CH_FLAT = 1, CH_DOUBLY = 2 };
struct channel_tap {
    int32_t delay;  // samples (link_t::set_pdp)
    float amp;      // sqrt(p_i) / sqrt(N_sin), as link.cpp:280-283 scales
};
struct channel_sin {
    int64_t period;     // samples per Doppler cycle, signed (INT64_MAX inside the dead band)
    double phase_rev;   // initial phase / 2 pi
};
struct channel_args {
    uint32_t kind, N_TX, N_RX, S_tx, S_rx, n_taps, n_sin;
    const float2* tx;        // [n][N_TX][S_tx]
    float2* rx;              // [n][N_RX][S_rx]
    const int64_t* offset;   // [n] TX sample 0 lands at RX sample offset
    const int64_t* t0;       // [n] global time of RX sample 0 (Doppler phases)
    const float2* coef;      // flat: [n][N_RX][N_TX]
    const channel_tap* taps; // doubly: [n][N_RX][N_TX][n_taps]
    const channel_sin* sins; // doubly: [n][N_RX][N_TX][n_taps][n_sin]
    float large_scale, sigma;
    uint64_t seed;
};
hipError_t launch_channel(const channel_args& a, uint32_t n, hipStream_t st);

// ---- synchronisation (sync.hip): sync_chunk_t::search() per window, reports in search order
struct sync_res {  // layout of dnrp_sync_result (include/dnrp.h)
    uint32_t found, det_ant;
    float det_rms, det_metric;
    uint32_t det_time, det_time_jb, coarse_local, fine_local;
    int64_t coarse_64, fine_64;
    float coarse_metric[8], rms[8];
    float cfo_frac, cfo_int;
    uint32_t u, b, N_eff_TX, pad;
    float xc_metric[4];
    uint32_t xc_idx[4];
};
struct sync_args {
    uint32_t n_ant, n_pattern, stf_len, pattern, step, search_len, D, bos, n_steps;
    uint32_t L, M, delay, hl, m_star, p_star;  // sync resampler (RX direction, L/M swapped)
    uint32_t npp;                              // floats in taps_pp
    const float* taps;                         // h[(hl+1)*L]
    const float* taps_pp;                      // input-major block taps (polyphase.hpp)
    float rms_min, prefactor;
    float uw[8];                               // cover-sequence pairwise products
    uint32_t n_uw;
    const float2* iq;                          // window w, antenna a: iq + w*win_stride + a*ant_stride
    uint64_t win_stride, ant_stride;
    uint32_t S_win, n_win;
    float* P;                                  // [n][n_ant][n_steps] step powers
    float2* Cs;                                // [n][n_ant][n_steps] step correlations
    uint32_t max_reports;
    uint32_t det_stage;                        // sync_detect: float2 slots of the resampler stage (sync_detect_lds)
    unsigned long long* prof;                  // DNRP_SYNC_PROFILE builds: per-window phase clocks [n][16]
    sync_res* res;                             // [n][max_reports]
    uint32_t* n_found;                         // [n]
    // fine search (crosscorrelator.cpp): hw rate, FFT correlation against the STF templates
    uint32_t Ltx, Mtx, xc_l, xc_len, tmpl_len, n_templates, log2_fft;
    const float2* tmpl_f;                      // [n_templates][n_fft] conj(DFT(template)) / n_fft
    const float2* tw_fft;                      // forward twiddles of n_fft
    float2* spec;                              // sync_fine scratch: forward spectrum per report [n * max_reports][n_fft]
    float* post;                               // [n * max_reports][8]: per antenna m_a atan2(c_a) / P (sync_post_kernel)
    uint32_t u, b;
    // split detection (sync_detect_split / sync_peak_kernel rounds): per window the detection state
    // machine's registers between launches, and the per-antenna coarse-peak results of the pending
    // detection
    struct sync_state* state;                  // [n]
    float2* pk;                                // [n][8]: (metric, index bits) per antenna
    uint32_t first;                            // 1: the launch starts every window from the initial state
    uint32_t ct_taps;                          // host: the sync taps equal taps_sync_9_10 (compile-time-tap kernels)
};
struct sync_state {  // sync_detect_kernel's loop registers (autocorrelator_detection / _peak state)
    uint32_t s_cur, ignore, nrep, pend;  // pend: 0 searching, 1 coarse peak pending, 2 finished
    uint32_t sd, s_ant;
    float s_rms, s_metric;
};
hipError_t launch_sync_steps(const sync_args& a, uint32_t n, hipStream_t st);
hipError_t launch_sync_detect(const sync_args& a, uint32_t n, hipStream_t st);
hipError_t launch_sync_detect_split(const sync_args& a, uint32_t n, hipStream_t st);
hipError_t launch_sync_peak(const sync_args& a, uint32_t n, hipStream_t st);
bool sync_peak_ok(const sync_args& a);
bool sync_taps_match(const float* h, size_t n);  // compiled-in 9/10 sync taps == run-time taps
hipError_t launch_sync_post(const sync_args& a, uint32_t n, hipStream_t st);
hipError_t launch_sync_fine(const sync_args& a, uint32_t n, hipStream_t st);
uint32_t sync_detect_stage(const sync_args& a);
size_t sync_detect_lds(const sync_args& a);

}  // namespace dnrp::dev
