// Reference parameters the lower PHY is defined by: one constexpr per compile-time switch or value
// of the reference's parameter headers, named after the reference macro / field it restates. Host
// code and kernels use these names instead of literals; dnrp_query_param() exports them by the
// reference's own names, and tests/test_oracle_pins.py compares every one with the value the
// reference headers compile to (oracle/_ref harness -> tests/golden/ref_tables.json "params").
//
//   sync_param.hpp        lib/include/dectnrp/phy/rx/sync/sync_param.hpp (cover-sequence branches,
//                         SECTIONS_PART_3_STF_COVER_SEQUENCE_ACTIVE: stf_param.hpp:23)
//   rx_synced_param.hpp   lib/include/dectnrp/phy/rx/rx_synced/rx_synced_param.hpp
//   resampler_param.hpp   lib/include/dectnrp/phy/resample/resampler_param.hpp:77-88
//   constants.hpp         lib/include/dectnrp/constants.hpp
#pragma once

#include <stdint.h>

namespace dnrp::prm {

// ------------------------------------------------------------------ stf_param.hpp
constexpr bool STF_COVER_SEQUENCE_ACTIVE = true;
// stf_t::cover_sequence (stf.hpp:146-151), the SECTIONS_PART_3_STF_COVER_SEQUENCE_ACTIVE branch:
// +-1 per STF pattern (9 patterns for u >= 2, the first 7 for u = 1)
#define DNRP_STF_COVER_SEQUENCE {1.0f, -1.0f, 1.0f, 1.0f, -1.0f, -1.0f, -1.0f, -1.0f, -1.0f}
constexpr float STF_COVER[9] = DNRP_STF_COVER_SEQUENCE;

// ------------------------------------------------------------------ sync_param.hpp
constexpr uint32_t SYNC_MAX_BUFFERABLE = 10;             // RX_SYNC_PARAM_MAX_NOF_BUFFERABLE_SYNC_BEFORE_ACQUIRING_BATON
constexpr uint32_t SYNC_ANTENNA_LIMIT = 8;               // RX_SYNC_PARAM_AUTOCORRELATOR_ANTENNA_LIMIT
constexpr double SYNC_TIME_UNIQUE_LIMIT_PATTERNS = 1.0;  // RX_SYNC_PARAM_SYNC_TIME_UNIQUE_LIMIT_IN_STF_PATTERNS_DP
constexpr double SYNC_OVERLAP_STFS = 4.0;                // ..._DETECTION_OVERLAP_LENGTH_IN_STFS_DP
constexpr uint32_t SYNC_STEP_DIVIDER = 4;                // ..._DETECTION_STEP_DIVIDER
constexpr double SYNC_RMS_MIN_REF_RATE = 30.72e6;        // ..._DETECTION_RMS_THRESHOLD_MIN_REFERENCE_SAMPLE_RATE_DP
constexpr float SYNC_RMS_MIN = 0.005f;                   // ..._DETECTION_RMS_THRESHOLD_MIN_SP
constexpr float SYNC_RMS_MAX = 2.0f;                     // ..._DETECTION_RMS_THRESHOLD_MAX_SP
constexpr uint32_t SYNC_RMS_FRONT_STEPS = 2;             // ..._DETECTION_RMS_FRONT_STEPS
constexpr uint32_t SYNC_RMS_BACK_STEPS = 2;              // ..._DETECTION_RMS_BACK_STEPS
constexpr double SYNC_RMS_FRONT_TO_BACK_RATIO = 0.5;     // ..._DETECTION_RMS_FRONT_TO_BACK_RATIO
constexpr float SYNC_METRIC_MIN = 0.18f;                 // ..._DETECTION_METRIC_THRESHOLD_MIN_SP
constexpr float SYNC_METRIC_MAX = 1.50f;                 // ..._DETECTION_METRIC_THRESHOLD_MAX_SP
constexpr float SYNC_METRIC_STREAK_GAIN = 0.0f;          // ..._DETECTION_METRIC_STREAK_RELATIVE_GAIN_SP
constexpr uint32_t SYNC_METRIC_STREAK = 1;               // ..._DETECTION_METRIC_STREAK
constexpr uint32_t SYNC_JUMP_BACK_PATTERNS = 1;          // ..._DETECTION_JUMP_BACK_IN_PATTERNS
constexpr double SYNC_SKIP_AFTER_PEAK_STFS = 2.0;        // ..._DETECTION_SKIP_AFTER_PEAK_IN_STFS_DP
constexpr uint32_t SYNC_PEAK_REQUEST_PATTERNS = 1;       // ..._PEAK_SAMPLES_REQUEST_IN_PATTERNS
constexpr double SYNC_PEAK_MAX_SEARCH_STFS = 1.0;        // ..._PEAK_MAX_SEARCH_LENGTH_IN_STFS_DP
constexpr uint32_t SYNC_PEAK_SMOOTH_LEFT = 1;            // ..._PEAK_MOVMEAN_SMOOTH_LEFT
constexpr uint32_t SYNC_PEAK_SMOOTH_RIGHT = 1;           // ..._PEAK_MOVMEAN_SMOOTH_RIGHT
constexpr float SYNC_PEAK_ABOVE_DETECTION = -0.25f;      // ..._PEAK_METRIC_ABOVE_DETECTION_THRESHOLD_SP
constexpr double SYNC_PEAK_DETECTION2PEAK_STFS = -0.3;   // ..._PEAK_DETECTION2PEAK_IN_STFS_DP
constexpr bool SYNC_XC_CFO_PRECORRECTION = true;         // RX_SYNC_PARAM_CROSSCORRELATOR_CFO_PRECORRECTION
constexpr double SYNC_XC_STF_LENGTH_EFFECTIVE = 1.0;     // ..._CROSSCORRELATOR_STF_LENGTH_EFFECTIVE_DP
constexpr uint32_t SYNC_XC_SEARCH_LEFT = 16;             // ..._CROSSCORRELATOR_SEARCH_LEFT_SAMPLES
constexpr uint32_t SYNC_XC_SEARCH_RIGHT = 16;            // ..._CROSSCORRELATOR_SEARCH_RIGHT_SAMPLES

// ------------------------------------------------------------------ rx_synced_param.hpp
constexpr uint32_t RX_STO_INTO_CP_PERCENT = 0;           // RX_SYNCED_PARAM_STO_INTEGER_MOVE_INTO_CP_IN_PERCENTAGE_OF_STF
constexpr bool RX_RMS_FILL_OR_KEEP = true;               // RX_SYNCED_PARAM_RMS_FILL_COMPLETELY_OR_KEEP_WHAT_SYNCHRONIZATION_PROVIDED
constexpr uint32_t RX_RMS_STF_PERCENT = 100;             // RX_SYNCED_PARAM_RMS_PERCENTAGE_OF_STF_USED_FOR_RMS_ESTIMATION
constexpr bool RX_RMS_KEEP_SYNC = true;                  // RX_SYNCED_PARAM_RMS_KEEP_VALUES_PROVIDED_BY_SYNC
constexpr bool RX_CFO_CORRECTION = true;                 // RX_SYNCED_PARAM_CFO_CORRECTION
constexpr bool RX_CFO_FRACTIONAL_ADJUST = true;          // RX_SYNCED_PARAM_CFO_FRACTIONAL_ADJUST
constexpr bool RX_AMPLITUDE_SCALING = true;              // RX_SYNCED_PARAM_AMPLITUDE_SCALING
constexpr bool RX_STO_FRACTIONAL_STF = true;             // RX_SYNCED_PARAM_STO_FRACTIONAL_BASED_ON_STF
constexpr bool RX_STO_RESIDUAL_DRS = false;              // RX_SYNCED_PARAM_STO_RESIDUAL_BASED_ON_DRS (not defined)
constexpr bool RX_CFO_RESIDUAL_DRS = false;              // RX_SYNCED_PARAM_CFO_RESIDUAL_BASED_ON_DRS (not defined)
constexpr uint32_t RX_WEIGHTS_TYPE_CHOICE = 0;           // RX_SYNCED_PARAM_WEIGHTS_TYPE_CHOICE (real weights)
constexpr double RX_NU_MAX_HZ[3] = {100.0, 100.0, 500.0};     // RX_SYNCED_PARAM_NU_MAX_HZ_VEC
constexpr double RX_TAU_RMS_SEC[3] = {0.1e-6, 0.1e-6, 1.0e-6}; // RX_SYNCED_PARAM_TAU_RMS_SEC_VEC
constexpr double RX_SNR_DB[3] = {-5.0, 15.0, 35.0};           // RX_SYNCED_PARAM_SNR_DB_VEC
constexpr uint32_t RX_N_INTERP_LR[3] = {14, 8, 3};            // RX_SYNCED_PARAM_NOF_DRS_INTERP_LR_VEC
constexpr uint32_t RX_N_INTERP_L[3] = {7, 4, 2};              // RX_SYNCED_PARAM_NOF_DRS_INTERP_L_VEC
constexpr bool RX_LUT_OPT_INDEX_PREVIOUS = true;         // RX_SYNCED_PARAM_CHANNEL_LUT_OPT_INDEX_PREVIOUS
constexpr double RX_LUT_SEARCH_ABORT = 1.1;              // RX_SYNCED_PARAM_CHANNEL_LUT_SEARCH_ABORT_THRESHOLD
constexpr bool RX_LUT_LOOKUP_EVERY_DRS = true;           // RX_SYNCED_PARAM_CHANNEL_LUT_LOOKUP_AFTER_EVERY_DRS_SYMBOL_OR_ONCE
constexpr bool RX_SNR_STF = true;                        // RX_SYNCED_PARAM_SNR_BASED_ON_STF
constexpr bool RX_SNR_DRS = true;                        // RX_SYNCED_PARAM_SNR_BASED_ON_DRS
constexpr uint32_t RX_SNR_DRS_N_TS_MAX = 8;              // RX_SYNCED_PARAM_SNR_BASED_ON_DRS_N_TS_MAX
constexpr bool RX_MIMO_AT_PACKET_END = true;             // RX_SYNCED_PARAM_MIMO_BASED_ON_STF_AND_DRS_AT_PACKET_END
constexpr uint32_t RX_MIMO_WIDEBAND_CELLS = 4;           // RX_SYNCED_PARAM_MIMO_N_WIDEBAND_CELLS
constexpr uint32_t RX_MODE_3_7_METRIC = 0;               // RX_SYNCED_PARAM_MODE_3_7_METRIC (HIGHEST_MIN_RX_POWER)
constexpr bool RX_BLOCK_N_SS_GT_1_AT_PCC = true;         // RX_SYNCED_PARAM_BLOCK_N_SS_TX_LARGER_1_AT_PCC
constexpr bool RX_BLOCK_N_EFF_TX_GT_1_AT_PDC = false;    // RX_SYNCED_PARAM_BLOCK_N_EFF_TX_LARGER_1_AT_PDC (not defined)

// ------------------------------------------------------------------ resampler_param.hpp:77-88
// [user TX / SYNC / RX_SYNCED][os_min 1, 2, 4, 8]
constexpr float RS_F_PASS[3][4] = {{0.48f, 0.30f, 0.20f, 0.15f}, {0.48f, 0.30f, 0.20f, 0.15f}, {0.48f, 0.30f, 0.20f, 0.15f}};
constexpr float RS_F_STOP[3][4] = {{0.499f, 0.499f, 0.499f, 0.499f}, {0.499f, 0.499f, 0.499f, 0.499f}, {0.499f, 0.499f, 0.499f, 0.499f}};
constexpr float RS_ATT_DB[3][4] = {{14.0f, 20.0f, 20.0f, 20.0f}, {14.0f, 20.0f, 20.0f, 20.0f}, {14.0f, 20.0f, 20.0f, 20.0f}};
constexpr float RS_RIPPLE_DONT_CARE = 100.0f;            // resampler_param_t::PASSBAND_RIPPLE_DONT_CARE
enum rs_user : uint32_t { RS_TX = 0, RS_SYNC = 1, RS_RX_SYNCED = 2 };
__host__ __device__ constexpr uint32_t rs_os_index(uint32_t os) { return os == 1 ? 0 : os == 2 ? 1 : os == 4 ? 2 : 3; }

// ------------------------------------------------------------------ common/adt/miscellaneous.hpp:71
constexpr int64_t UNDEFINED_EARLY_64 = INT64_MIN / 8;    // common::adt::UNDEFINED_EARLY_64

// ------------------------------------------------------------------ constants.hpp
constexpr uint32_t N_B_DFT_MIN_U_B = 64;                 // constants::N_b_DFT_min_u_b
constexpr uint32_t N_B_CP_MIN_U_B = 8;                   // constants::N_b_CP_min_u_b
constexpr uint32_t SAMP_RATE_MIN_U_B = 1728000;          // constants::samp_rate_min_u_b
constexpr uint32_t SUBCARRIER_SPACING_MIN_U_B = 27000;   // constants::subcarrier_spacing_min_u_b
constexpr uint32_t N_STF_PATTERN_U1 = 7;                 // constants::N_stf_pattern_u1
constexpr uint32_t N_STF_PATTERN_U248 = 9;               // constants::N_stf_pattern_u248
constexpr uint32_t N_SAMPLES_STF_PATTERN = 16;           // constants::N_samples_stf_pattern
constexpr uint32_t N_STF_CELLS_B_1 = 14;                 // constants::N_STF_cells_b_1
constexpr uint32_t N_STF_CELLS_SPACING = 4;              // constants::N_STF_cells_spacing
constexpr uint32_t N_STF_CELLS_SPACING_CENTER = 8;       // constants::N_STF_cells_spacing_center
constexpr uint32_t N_TS_MAX = 8;                         // constants::N_TS_max
constexpr uint32_t PCC_BITS = 196;                       // constants::pcc_bits
constexpr uint32_t PCC_CELLS = 98;                       // constants::pcc_cells

}  // namespace dnrp::prm
