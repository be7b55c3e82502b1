// fec.hpp — channel coding of DECT NR+ (ETSI TS 103 636-3 §6.1 / §7.5-7.6 = the LTE turbo chain of
// 3GPP TS 36.212 §5.1): CRC attachment, code-block segmentation, the 8-state PCCC turbo code with
// its QPP interleaver, turbo rate matching and a max-log-MAP turbo decoder.
//
// The reference calls srsRAN_4G release_23_11 for all of this (phy/fec/pcc_enc.cpp:145-364,
// pdc_enc.cpp:127-492, fec.cpp:82-150, sections_part3/fix/cbsegm.cpp:55-144); srsRAN is not part of
// /root/reference, so the arithmetic here is restated from TS 36.212 and the reference's call sites.
// Host code: the reference runs FEC on the CPU in the worker threads (worker_tx_rx.cpp:166-201).
#pragma once
#include <cstdint>
#include <vector>

namespace dnrp::fec {

constexpr uint32_t kNofCbSizes = 188;       // TS 36.212 Table 5.1.3-3 rows (SRSRAN_NOF_TC_CB_SIZES)
constexpr uint32_t kCrc16 = 0x1021;         // g_CRC16  (TS 36.212 §5.1.1), PLCF CRC (TS 103 636-3 §7.5.2.1)
constexpr uint32_t kCrc24A = 0x864CFB;      // g_CRC24A, transport-block CRC (§7.6.2)
constexpr uint32_t kCrc24B = 0x800063;      // g_CRC24B, code-block CRC
constexpr uint32_t kPlcfType1Bits = 40, kPlcfType2Bits = 80, kPccBits = 196;
constexpr uint32_t kPccMaxIter = 5;         // pcc_enc.cpp:39
constexpr uint32_t kPdcMaxIter = 10;        // pdc_enc.cpp:36
constexpr uint32_t kPdcMinIter = 2;         // SRSRAN_PDSCH_MIN_TDEC_ITERS (pdc_enc.cpp:275)
// PLCF CRC masks (pcc_enc.cpp:41-44, TS 103 636-3 §7.5.2.2-3)
constexpr uint16_t kMaskNone = 0x0000, kMaskCl = 0x5555, kMaskBf = 0xAAAA, kMaskClBf = 0xFFFF;

uint32_t cb_size(uint32_t idx);             // K of row idx (0 on a bad index)
int cb_index(uint32_t long_cb);             // first row with K >= long_cb, -1 if none (cbsegm.cpp:125-136)
void qpp_params(uint32_t idx, uint32_t* f1, uint32_t* f2);
const std::vector<uint32_t>& qpp(uint32_t idx);  // pi(i) = (f1 i + f2 i^2) mod K, cached

struct Segm { uint32_t tbs, Z, C, C1, C2, K1, K2, K1_idx, K2_idx, F; };
int cbsegm(uint32_t tbs, uint32_t Z, Segm* s);   // srsran_cbsegm_FIX (cbsegm.cpp:65-123)

// CRC over nbits of MSB-first packed bytes (init 0, no reflection, no final xor)
uint32_t crc_bits(const uint8_t* data, uint32_t nbits, uint32_t poly, uint32_t len);

// Turbo code of one code block of K bits (unpacked 0/1): d0, d1, d2 of K + 4 bits each
void turbo_encode(const uint8_t* c, uint32_t idx, uint8_t* d0, uint8_t* d1, uint8_t* d2);

// Turbo rate matching of one code block: E output bits starting at redundancy version rv
void rm_tx(const uint8_t* d0, const uint8_t* d1, const uint8_t* d2, uint32_t idx, uint32_t E, uint32_t rv,
           uint8_t* e);
// Inverse: accumulate E soft bits into the circular-buffer softbuffer w (Kw = 3 Kpi entries,
// saturating int16), the srsran_rm_turbo_rx_lut_ (..., enable_input_tdec = false) role.
void rm_rx(const int16_t* e, uint32_t idx, uint32_t E, uint32_t rv, int16_t* w);
uint32_t rm_kw(uint32_t idx);               // 3 * Kpi
// Softbuffer -> decoder streams d0/d1/d2 (K + 4 each, dummy bits dropped)
void rm_deinterleave(const int16_t* w, uint32_t idx, int32_t* d0, int32_t* d1, int32_t* d2);

// Max-log-MAP turbo decoder state of one code block (int32 metrics, extrinsic scaled by 3/4)
struct Tdec {
    uint32_t idx = 0, K = 0;
    std::vector<int32_t> sys, p1, p2, tail, le1, le2, llr;
    std::vector<int32_t> alpha;
    void load(const int16_t* w, uint32_t idx_);  // new code block from its softbuffer
    void iterate(uint8_t* bits);                 // one iteration (both constituent decoders), hard bits out
};

}  // namespace dnrp::fec
