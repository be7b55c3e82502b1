// ORACLE — TEST INFRASTRUCTURE ONLY (see oracle.hpp header).
// The reference parameters the oracle restatement is built with, one constexpr per reference macro
// / field (names in the comments). Kept separate from the product's csrc/params.hpp on purpose: the
// checker does not share code with the thing it checks. oracle_query_param() exports them by the
// reference's names; tests/test_oracle_pins.py compares them with the reference-compiled values.
#pragma once

#include <cstdint>

namespace orc::prm {

// sync_param.hpp (cover-sequence branches)
constexpr uint32_t ANTENNA_LIMIT = 8;                 // RX_SYNC_PARAM_AUTOCORRELATOR_ANTENNA_LIMIT
constexpr double OVERLAP_STFS = 4.0;                  // ..._DETECTION_OVERLAP_LENGTH_IN_STFS_DP
constexpr uint32_t STEP_DIVIDER = 4;                  // ..._DETECTION_STEP_DIVIDER
constexpr uint32_t DET_RESUM = 16;                    // ..._DETECTION_RESUM_PERIODICITY_IN_STEPS
constexpr double RMS_MIN_REF_RATE = 30.72e6;          // ..._DETECTION_RMS_THRESHOLD_MIN_REFERENCE_SAMPLE_RATE_DP
constexpr float RMS_MIN = 0.005f;                     // ..._DETECTION_RMS_THRESHOLD_MIN_SP
constexpr float RMS_MAX = 2.0f;                       // ..._DETECTION_RMS_THRESHOLD_MAX_SP
constexpr uint32_t RMS_FRONT_STEPS = 2;               // ..._DETECTION_RMS_FRONT_STEPS
constexpr uint32_t RMS_BACK_STEPS = 2;                // ..._DETECTION_RMS_BACK_STEPS
constexpr double RMS_FRONT_TO_BACK = 0.5;             // ..._DETECTION_RMS_FRONT_TO_BACK_RATIO
constexpr float METRIC_MIN = 0.18f;                   // ..._DETECTION_METRIC_THRESHOLD_MIN_SP
constexpr float METRIC_MAX = 1.50f;                   // ..._DETECTION_METRIC_THRESHOLD_MAX_SP
constexpr float STREAK_GAIN = 0.0f;                   // ..._DETECTION_METRIC_STREAK_RELATIVE_GAIN_SP
constexpr uint32_t STREAK = 1;                        // ..._DETECTION_METRIC_STREAK
constexpr uint32_t JUMP_BACK_PATTERNS = 1;            // ..._DETECTION_JUMP_BACK_IN_PATTERNS
constexpr double SKIP_AFTER_PEAK_STFS = 2.0;          // ..._DETECTION_SKIP_AFTER_PEAK_IN_STFS_DP
constexpr uint32_t PEAK_REQUEST_PATTERNS = 1;         // ..._PEAK_SAMPLES_REQUEST_IN_PATTERNS
constexpr uint32_t PEAK_RESUM = 64;                   // ..._PEAK_RESUM_PERIODICITY_IN_STEPS
constexpr double PEAK_MAX_SEARCH_STFS = 1.0;          // ..._PEAK_MAX_SEARCH_LENGTH_IN_STFS_DP
constexpr uint32_t SMOOTH_LEFT = 1;                   // ..._PEAK_MOVMEAN_SMOOTH_LEFT
constexpr uint32_t SMOOTH_RIGHT = 1;                  // ..._PEAK_MOVMEAN_SMOOTH_RIGHT
constexpr float PEAK_ABOVE_DETECTION = -0.25f;        // ..._PEAK_METRIC_ABOVE_DETECTION_THRESHOLD_SP
constexpr double DETECTION2PEAK_STFS = -0.3;          // ..._PEAK_DETECTION2PEAK_IN_STFS_DP
constexpr uint32_t XC_SEARCH_LEFT = 16;               // ..._CROSSCORRELATOR_SEARCH_LEFT_SAMPLES
constexpr uint32_t XC_SEARCH_RIGHT = 16;              // ..._CROSSCORRELATOR_SEARCH_RIGHT_SAMPLES

// rx_synced_param.hpp
constexpr double NU_MAX_HZ[3] = {100.0, 100.0, 500.0f};      // RX_SYNCED_PARAM_NU_MAX_HZ_VEC
constexpr double TAU_RMS_SEC[3] = {0.1e-6, 0.1e-6, 1.0e-6};  // RX_SYNCED_PARAM_TAU_RMS_SEC_VEC
constexpr double SNR_DB[3] = {-5.0, 15.0, 35.0};             // RX_SYNCED_PARAM_SNR_DB_VEC
constexpr uint32_t N_INTERP_LR[3] = {14, 8, 3};              // RX_SYNCED_PARAM_NOF_DRS_INTERP_LR_VEC
constexpr uint32_t N_INTERP_L[3] = {7, 4, 2};                // RX_SYNCED_PARAM_NOF_DRS_INTERP_L_VEC
constexpr double LUT_SEARCH_ABORT = 1.1;                     // RX_SYNCED_PARAM_CHANNEL_LUT_SEARCH_ABORT_THRESHOLD
constexpr uint32_t MIMO_WIDEBAND_CELLS = 4;                  // RX_SYNCED_PARAM_MIMO_N_WIDEBAND_CELLS
constexpr uint32_t RMS_STF_PERCENT = 100;                    // RX_SYNCED_PARAM_RMS_PERCENTAGE_OF_STF_USED_FOR_RMS_ESTIMATION
constexpr bool RMS_KEEP_SYNC = true;                         // RX_SYNCED_PARAM_RMS_KEEP_VALUES_PROVIDED_BY_SYNC

// resampler_param.hpp:77-88, index [os 1/2/4/8] (identical for the TX / SYNC / RX_SYNCED users)
constexpr float RS_F_PASS[4] = {0.48f, 0.30f, 0.20f, 0.15f};
constexpr float RS_F_STOP[4] = {0.499f, 0.499f, 0.499f, 0.499f};
constexpr float RS_ATT_DB[4] = {14.0f, 20.0f, 20.0f, 20.0f};
constexpr float RS_RIPPLE = 100.0f;                          // resampler_param_t::PASSBAND_RIPPLE_DONT_CARE

}  // namespace orc::prm
