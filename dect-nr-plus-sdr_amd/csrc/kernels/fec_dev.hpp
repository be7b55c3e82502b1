// fec_dev.hpp — device-side turbo decoding of PDC transport blocks (dnrp_pdc_decode_batch):
// the batched form of fec_t::decode_tb (phy/fec/pdc_enc.cpp:291-492) with the arithmetic of the
// host decoder in csrc/host/fec.cpp (integer max-log-MAP, extrinsic x3/4, CRC early stop), so a code
// block decodes to the same bits after the same number of iterations on both.
//
// Layout: code blocks of equal size K are grouped 64 to a wavefront, one code block per lane; the
// wave's soft streams are stored [k][lane] (int16), so the QPP-interleaved accesses of a wave — the
// interleaver depends only on K — are coalesced 128-B rows. Forward state metrics are kept only at
// every 8th step (checkpoints [k/8][state][lane]); the backward pass recomputes each 8-step window's
// metrics in registers. The interleaver addresses are computed by the QPP recurrence on the scalar
// unit (no index loads in the dependency chain); decoder 2 writes its extrinsic back in natural order.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace dnrp::dev {

constexpr uint32_t FEC_WIN = 8;      // backward-pass window (steps); every K is a multiple of 8
constexpr int32_t FEC_NEG = -(1 << 28);

struct FecCb {           // one code block
    uint64_t llr_off;    // element offset of its first soft bit in the LLR input
    uint64_t tb_off;     // byte offset of its decoded data in the TB output
    uint32_t E;          // soft bits read (n_e2, pdc_enc.cpp:322-332)
    uint32_t start;      // index into the size's circular-buffer list where soft bit 0 lands (rv)
    uint32_t wave, lane;
    uint32_t poly;       // CRC over the K decoded bits: CRC24B (C > 1), CRC24A (C == 1), CRC16 (PLCF)
    uint32_t out_bytes;  // decoded bytes written (K/8 for C == 1, (K-24)/8 otherwise)
    uint64_t sb_off;     // HARQ: element offset of its softbuffer (3 streams x (K + 4), stream-major)
    uint64_t flag_off;   // HARQ: its code-block CRC flag
};

struct FecWave {
    uint64_t data_off;   // element offset of the wave's [k][64] arrays in the work buffer
    uint64_t ck_off;     // element offset of its checkpoints
    uint32_t K, n;       // code-block size, lanes in use
    uint32_t valid_off;  // offset of the size's circular-buffer list (3 (K + 4) entries: stream << 16 | index)
    uint32_t f1, f2;     // QPP coefficients: pi(i) = (f1 i + f2 i^2) mod K, stepped with scalar ops
    uint32_t first_cb;   // FecCb index of lane 0 (lanes are consecutive)
};

struct FecArgs {
    const int16_t* llr;
    uint8_t* tb;
    const uint32_t* tab;
    const FecCb* cbs;
    const FecWave* waves;
    int16_t* work16;     // sys, p1, p2, le1, le2: 5 x K x 64 per wave (data_off)
    int32_t* tail;       // [wave][12][64]
    uint8_t* bits;       // [wave][K][64] hard decisions (at data_off / 5)
    int32_t* ck;         // checkpoints (ck_off)
    uint32_t* cb_out;    // per code block: iterations << 4 | pending << 3 | CRC16 mask << 1 | crc ok
    int16_t* sb;         // HARQ softbuffers (nullptr: one-shot decoding)
    uint8_t* flags;      // HARQ code-block CRC flags (softbuffer->cb_crc)
    uint32_t n_cb, n_waves, max_iter, min_iter;
    uint32_t it_first;   // first iteration number of this launch (1, or the split + 1 of a continuation)
    uint32_t final_pass; // 0: blocks still undecided after max_iter keep their state and report pending
};

struct FecCompactArgs {  // continuation: undecided blocks gathered densely into new waves
    const int16_t* src16;
    const int32_t* src_tail;
    const FecWave* src_waves;
    int16_t* dst16;
    int32_t* dst_tail;
    const FecWave* dst_waves;
    const uint32_t* src_of;  // per new code block: source wave << 6 | source lane
};

struct FecTbArgs {       // transport-block CRC24A of packets with C > 1
    const uint8_t* tb;
    const uint64_t* tb_off;
    const uint32_t* nbytes;  // N_TB_bits / 8 (the CRC follows)
    uint32_t* ok;            // decoder: 1 if the CRC after the TB matches
    uint32_t* crc_out;       // encoder (non-null): the computed CRC instead
    uint32_t n;
};

struct FecEncCb {        // one code block of dnrp_pdc_encode_batch / dnrp_pcc_encode_batch
    uint64_t tb_off;     // byte offset of the packet's transport block
    uint64_t oo;         // bit offset of its rate-matched bits in the packed scratch (multiple of 64)
    uint32_t pkt;        // packet index (TB CRC)
    uint32_t tbs;        // N_TB_bits of the packet
    uint32_t rp;         // first bit of b = a || CRC24A the block takes
    uint32_t rlen;       // bits taken (K - 24 with a CRC24B, K otherwise)
    uint32_t E, start;   // rate-matched bits, circular-buffer list start of the redundancy version
    uint32_t crc24b;     // 1: append a code-block CRC
    uint32_t crc16;      // 1: PLCF: b = a || CRC16 ^ mask computed here (pcc_enc.cpp:166-183)
    uint32_t mask;       // PLCF CRC mask
    uint32_t K, f1, f2;  // block size, QPP coefficients
    uint32_t valid_off;  // the size's circular-buffer list in the table
    uint32_t pstart;     // first bit of its rate-matched bits in the packet's d row
    uint32_t mA;         // RSC state map A^Lc (Lc = fec_enc_chunk(K)) as three 3-bit columns
};

// bits per lane of a K-bit code block in fec_encode_kernel (a multiple of 32, at most 96)
__host__ __device__ constexpr uint32_t fec_enc_chunk(uint32_t K) {
    return ((K + 63) / 64 + 31) / 32 * 32 > 32 ? ((K + 63) / 64 + 31) / 32 * 32 : 32;
}

struct FecEncArgs {
    const uint8_t* tb;
    const uint32_t* tab;
    const FecEncCb* cbs;      // packet order
    const uint32_t* tbcrc;    // per packet
    uint8_t* ebits;           // packed rate-matched bits (FecEncCb::oo)
    uint8_t* d;               // non-null: direct mode, every block's bits whole bytes of its d row
    uint32_t d_stride;
};

struct FecPackArgs {          // packed scratch -> MSB-first d rows
    const uint8_t* ebits;
    const uint32_t* cb_first; // per packet its first code block, [n + 1]
    const uint32_t* pstart;   // per code block: first bit in its packet's row
    const uint64_t* oo;       // per code block: bit offset in the scratch
    const uint32_t* G;
    uint8_t* d;
    uint32_t d_stride, n, max_bytes;
};

int launch_fec_dematch(const FecArgs& a, hipStream_t s);
int launch_fec_tdec(const FecArgs& a, uint32_t n_waves, hipStream_t s);
int launch_fec_compact(const FecCompactArgs& a, uint32_t n_waves, hipStream_t s);
int launch_fec_tbcrc(const FecTbArgs& a, hipStream_t s);
int launch_fec_encode(const FecEncArgs& a, uint32_t n_cb, hipStream_t s);
int launch_fec_pack(const FecPackArgs& a, hipStream_t s);

}  // namespace dnrp::dev
