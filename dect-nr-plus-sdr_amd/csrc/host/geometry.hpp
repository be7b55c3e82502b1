// Host-side DECT NR+ geometry for the GPU path: packet sizes, per-symbol cell-code maps, DRS/STF
// tables, beamforming matrices, resampler taps, Gold sequences, Wiener channel-estimation LUTs and
// the RX operation schedules. Everything here runs once per configuration at context init (the
// reference builds the same objects in its constructors: tx_rx.cpp:38-129, rx_synced.cpp:55-174)
// and is uploaded to HBM as flat tables shared by every packet of a batch.
#pragma once

#include <complex>
#include <cstdint>
#include <vector>

#include "dnrp.h"
#include "../params.hpp"

namespace dnrp::geo {

using cf32 = std::complex<float>;

// cell codes, one u32 per (symbol l, transmit-stream index k in [0, N_b_OCC])
enum : uint32_t {
    CODE_NONE = 0u << 29,
    CODE_PCC = 1u << 29,  // bits 0..28: PCC cell index (0..97)
    CODE_PDC = 2u << 29,  // bits 0..28: PDC cell index
    CODE_DRS = 3u << 29,  // bits 0..2: transmit stream, bit 3: value is -1
    CODE_STF = 4u << 29,  // value from the STF table at k
    CODE_MASK = 7u << 29,
};

struct tm_t {
    uint32_t index, N_eff_TX, N_SS, N_TS, N_TX;
    bool cl, txdiv;
};

bool packet_sizes(const dnrp_psdef& d, dnrp_packet_sizes& q, tm_t* tm = nullptr);

// FFT size and hw-rate lengths for a context (tx.cpp:429-600)
struct dims_t {
    uint32_t Nd, N_occ, Nf, off_lower, CP, STF_CP, N_no_GI, N_no_GI_rs, N_packet_rs;
    uint32_t n_pattern, pattern_len;
};
dims_t make_dims(const dnrp_cfg& cfg, const dnrp_psdef& d, const dnrp_packet_sizes& q);

struct drs_sym_t {
    uint32_t l, ts_first, ts_last, parity;
};

// per-configuration maps (geometry of one (b, N_TS, N_DF) packet)
struct maps_t {
    uint32_t b, N_TS, N_DF, Nf;
    std::vector<uint32_t> code;        // [(N_DF+1) * Nf]
    std::vector<uint32_t> pcc_l;       // symbols carrying PCC (ascending)
    std::vector<uint32_t> pcc_k;       // [98] cell index k, in PCC order
    std::vector<uint32_t> pcc_sym_off; // [pcc_l.size()+1] offsets into pcc_k
    std::vector<uint32_t> pdc_k;       // all PDC cells in order
    std::vector<uint32_t> pdc_sym_off; // [N_DF+2] offsets into pdc_k per symbol (l = 0..N_DF)
    std::vector<drs_sym_t> drs;
    std::vector<cf32> stf;             // [Nf]
    std::vector<uint32_t> drs_k;       // [2 parity][4 ts][N_occ/4]
    std::vector<float> drs_v;          // [8 ts][N_occ/4], +-1
};
maps_t build_maps(uint32_t b, uint32_t N_TS, uint32_t N_eff_TX, uint32_t N_DF);
// STF values with DC (length N_b_OCC+1) for N_eff_TX, scale 1.0
std::vector<cf32> stf_values(uint32_t b, uint32_t N_eff_TX);

std::vector<cf32> W_matrix(uint32_t N_TS, uint32_t N_TX, uint32_t codebook, float* scaling);
uint32_t W_codebooks(uint32_t N_TS, uint32_t N_TX);
// W_t::scaling_factor_optimal_DAC (beamforming_and_antenna_port_mapping.cpp:146-186): the scaling
// tx_meta_t::optimal_scaling_DAC selects instead of 1/sqrt(non-zero entries) (tx.cpp:582-592)
float W_scaling_optimal_DAC(uint32_t N_TS, uint32_t N_TX, uint32_t codebook);
// Y_i_t::index_N_TS_x (transmit_diversity_precoding.cpp:48-75): transmit-stream pair i of the SFBC
// cycle and the cycle length (get_modulo: 1 / 6 / 12 for N_TS = 2 / 4 / 8)
uint32_t txdiv_modulo(uint32_t N_TS);
void txdiv_pair(uint32_t N_TS, uint32_t i, uint32_t& A, uint32_t& B);
// DRS value of transmit stream t at DRS cell i (drs.cpp:227-254): +-y_b_1[(4 i + t % 4) % 56]
float drs_value(uint32_t t, uint32_t i);
uint64_t drs_neg_mask();                     // bit j: DRS y_b_1[j] = -1 (drs.hpp)
bool drs_tables_arithmetic(const maps_t& m);  // drs_k / drs_v == the front end's arithmetic DRS cells

std::vector<uint8_t> gold_bits_packed(uint32_t c_init, uint32_t nbits);  // MSB-first bytes

// polyphase resampler taps (resampler.cpp:56-160): h[(hl+1)*L], delay, history length
struct resampler_t {
    uint32_t L = 1, M = 1, delay = 0, hl = 0, taps = 1;
    std::vector<float> h;
};
resampler_t make_resampler(uint32_t L, uint32_t M, uint32_t os_min, uint32_t user);  // user: prm::rs_user

// Wiener LUT for one (N_step_virtual, b, SNR profile) — channel_lut.cpp:168-620
struct lut_t {
    uint32_t T = 0, n = 0, Nf = 0;
    std::vector<uint32_t> pilot_weight;  // [T][4][Nf] packed: pilot index | weight index << 16
    std::vector<float> weights;          // [n_vec][n]
};
lut_t build_lut(uint32_t N_step_virtual, uint32_t b, uint32_t b_max, uint32_t u_max, uint32_t profile);
float lut_profile_snr_db(uint32_t profile);

// RX schedules: a WG-uniform op list interpreted by the RX kernels (rx_synced.cpp:283-302,
// 1028-1163 restated as data instead of control flow)
enum : uint32_t {
    OP_DRS = 1,    // a = symbol l, b = index in maps.drs, c = rel (stage-relative index), d = ps_idx
    OP_EVENT = 2,  // a = mode (0: l / 1: lr), b = rel (LUT t index), c = ps_idx, d = ts_first
    OP_PCC = 3,    // a = symbol l, b = index into pcc_l
    OP_PDC = 4,    // a = symbol l
};
struct op_t {
    uint32_t kind, a, b, c, d;
};
void build_rx_ops(const maps_t& m, uint32_t N_eff_TX, uint32_t N_DF, bool mode_lr, uint32_t stride,
                  std::vector<op_t>& pcc_ops, std::vector<op_t>& pdc_ops, uint32_t& pcc_max_symbol);

// RX back-end plan derived from one op list. The DRS symbols in processing order feed the
// sequential SNR / LUT-pick chain (one WG per packet); the cell work is grouped into epochs of
// constant pilot-buffer content, each a list of segments sharing one interpolation event (one WG
// per packet x epoch). src[t][o]: DRS op whose zero-forced pilots sit at interlace offset o of
// stream t in the epoch's pilot buffer (channel_antenna.hpp:38-63), RX_SRC_NONE if never written.
constexpr uint16_t RX_SRC_NONE = 0xFFFF;
struct rx_seg_t {
    uint32_t kind;     // OP_PCC / OP_PDC
    uint32_t l;        // PCC: OFDM symbol
    uint32_t j0, j1;   // cell range (pcc_k / pdc_k indices)
    uint32_t mode, rel, swap, off;  // event: LUT mode, row, TS swap (0/2), write offsets of the latest DRS
    uint32_t drs_cnt;  // DRS ops processed before the event (selects the LUT profile pick)
    uint32_t u0;       // first work unit (cell or SFBC pair) of the segment within its epoch
};
struct rx_epoch_t {
    uint16_t src[4][2];
    uint32_t seg0, seg1, units;
};
struct rx_plan_t {
    std::vector<uint32_t> dl, dmeta;  // per DRS op: symbol; ts_first | ts_last << 8 | parity << 16
    std::vector<rx_seg_t> segs;
    std::vector<rx_epoch_t> epochs;
};
// pair_units: a work unit is an SFBC pair of cells when N_eff_TX > 1 (transmit diversity); false for
// spatial multiplexing, whose unit is one cell carrying N_SS symbols
rx_plan_t build_rx_plan(const maps_t& m, const std::vector<op_t>& ops, uint32_t N_eff_TX, bool pair_units = true);

}  // namespace dnrp::geo
