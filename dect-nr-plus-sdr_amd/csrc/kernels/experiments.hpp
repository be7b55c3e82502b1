// Compile-time experiment switches: phase-skip and attribution builds of the hot kernels
// (tools/build_variant.sh NAME "-DDNRP_EXPERIMENTS=<bits>" ...). Their results are meaningless, only
// their timings and counters are read. The shipped build defines no bit, so every
// switch below is a constant false and the guarded code is the product's.
#pragma once

#ifndef DNRP_EXPERIMENTS
#define DNRP_EXPERIMENTS 0u
#endif

namespace dnrp::dev {

enum xs_bit : unsigned {
    // RX front end (rx_fft_wave_ct_kernel): no span loads / FIR / FFT / Y stores
    XS_FE_SKIP_LOAD = 1u << 0,
    XS_FE_SKIP_FIR = 1u << 1,
    XS_FE_SKIP_FFT = 1u << 2,
    XS_FE_SKIP_STORE = 1u << 3,
    // rx_cells_kernel: no pilot buffer / prologue only
    XS_CELLS_SKIP_PRO = 1u << 4,
    XS_CELLS_SKIP_MAIN = 1u << 5,
    // rx_fused_kernel: no front end / no equalisation
    XS_FUSED_SKIP_FE = 1u << 6,
    XS_FUSED_SKIP_EQ = 1u << 7,
    // sync_steps_pipe_kernel: the whole window row in range (no clamp to the segment)
    XS_SYNC_NOCLAMP = 1u << 8,
    // attribution of LDS bank conflicts: rx_cells pilot reads all from stream row 0 / weight reads
    // from one row; tx_stream_kernel constellation from the byte itself (no table read)
    XS_CELLS_ONE_ROW = 1u << 9,
    XS_CELLS_ONE_WROW = 1u << 10,
    XS_TX_NO_QTAB = 1u << 11,
    XS_TX_TRIVIAL_BINS = 1u << 12,
    XS_CELLS_ONE_PILOT = 1u << 13,  // rx_cells: every unit reads its windows from pilot 0 (conflict attribution)  // TX: a DF bin's value is its code (no mapping; timing / ISA only)
};

__host__ __device__ constexpr bool experiment(unsigned bit) { return (DNRP_EXPERIMENTS & bit) != 0u; }

}  // namespace dnrp::dev
