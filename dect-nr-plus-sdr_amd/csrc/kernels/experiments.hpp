// Compile-time experiment switches (tools/build_variant.sh NAME "-DDNRP_EXPERIMENTS=<bits>" ...).
// Two kinds: phase-skip and attribution builds of the hot kernels, whose results are meaningless
// and only their timings and counters are read; and measured alternatives that compute the same
// results but lost their A/B (docs/DESIGN_LOG.md §6), kept buildable for re-measurement. The shipped build
// defines no bit, so every switch below is a constant false and the guarded code is the product's.
#pragma once

#ifndef DNRP_EXPERIMENTS
#define DNRP_EXPERIMENTS 0u
#endif

namespace dnrp::dev {

enum xs_bit : unsigned {
    // ---- phase skips (output meaningless)
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
    // ---- attribution (output meaningless)
    // LDS bank conflicts: rx_cells pilot reads all from stream row 0 / weight reads from one row /
    // every unit's windows from pilot 0; tx_stream_kernel constellation from the byte itself
    XS_CELLS_ONE_ROW = 1u << 9,
    XS_CELLS_ONE_WROW = 1u << 10,
    XS_TX_NO_QTAB = 1u << 11,
    XS_CELLS_ONE_PILOT = 1u << 13,
    // TX: a DF bin's value is its code (the bin mapping's share of the kernel)
    XS_TX_TRIVIAL_BINS = 1u << 12,
    // ---- measured alternatives (same results, slower)
    // wave FFT exchange slots XOR-swizzled instead of padded (conflict-free, +1-2 % TX)
    XS_WFFT_SWZ = 1u << 14,
    // 256-QAM TX constellation from a separable 16-level table (two conflict-free reads, +3 % TX)
    XS_TX_QLEV = 1u << 15,
    // RX front end: the next symbol's span touched into L2 while this one is computed (+1.5 %)
    XS_FE_PREFETCH = 1u << 16,
    // MMSE Gram matrix of 16 cells per v_mfma_f32_4x4x1_16b_f32 (x1.7 rx_pdc in C4SM)
    XS_MMSE_MFMA = 1u << 17,
    // rx_epoch_kernel phase skips (output meaningless): no front-end tasks / no equalisation
    XS_EP_SKIP_FE = 1u << 18,
    XS_EP_SKIP_EQ = 1u << 19,
    // rx_epoch_kernel: Y rows of the epoch in one of 64 x 8 x n_epochs packet images picked by
    // blockIdx (racy, output meaningless): the timing with the rows kept on-die
    XS_EP_SLOTY = 1u << 20,
};

__host__ __device__ constexpr bool experiment(unsigned bit) { return (DNRP_EXPERIMENTS & bit) != 0u; }

}  // namespace dnrp::dev
