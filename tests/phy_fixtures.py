"""Synthetic packet/channel generation shared by the tests and bench.py (TEST/BENCH INFRASTRUCTURE).

BASELINE.md §3 synthetic inputs: uniform d-bits, network IDs 100..105, PLCF type alternating,
CFO within +-1.75 subcarriers at the DECT rate, GI 5 %, AWGN, packet start at a seeded offset in
[0, 32) hw samples of a slot window of N_samples_packet_os_rs samples.
"""
import numpy as np

CONFIGS = {
    # name: (psdef tuple (u,b,PLT,PL,tm,mcs), cfg tuple (u_max,b_max,N_TX_max,os_min,L,M))
    "C2": ((1, 1, 1, 1, 0, 1), (1, 1, 1, 1, 10, 9)),
    "C3": ((8, 16, 1, 1, 0, 8), (8, 16, 1, 1, 10, 9)),
    "C4": ((8, 16, 1, 1, 5, 8), (8, 16, 4, 1, 10, 9)),
}

# GPU parity configurations (tests/test_gpu_parity.py; the oracle loopback runs all of them on the
# CPU in tests/test_oracle_loopback.py). The bench configurations C2/C3/C4 plus every mode the
# reference RX supports that the bench does not exercise.
# name: psdef (u, b, PLT, PL, tm, mcs), ctx (u_max, b_max, N_TX_max, os_min, L, M), chestim lr,
#       per-packet SNRs (dB), TX codebook
PARITY_CASES = {
    "C2": ((1, 1, 1, 1, 0, 1), (1, 1, 1, 1, 10, 9), 1, (10.0, 10.0, 10.0), 0),
    "C3": ((8, 16, 1, 1, 0, 8), (8, 16, 1, 1, 10, 9), 1, (30.0, 30.0, 30.0), 0),
    "C4": ((8, 16, 1, 1, 5, 8), (8, 16, 4, 1, 10, 9), 1, (30.0, 30.0, 30.0), 0),
    **{f"C1_mcs{m}": ((1, 1, 1, 1, 0, m), (1, 1, 1, 1, 10, 9), 1, (-2.0, 5.0, 20.0), 0) for m in (0, 2, 3, 4, 5, 6, 7)},
    "mrc2_64qam": ((1, 2, 1, 2, 0, 6), (1, 2, 2, 1, 10, 9), 1, (12.0, 25.0), 0),
    "mrc4_16qam": ((2, 4, 1, 1, 0, 4), (2, 4, 4, 1, 10, 9), 1, (8.0, 20.0), 0),
    "tm1_txdiv2": ((4, 8, 1, 1, 1, 5), (4, 8, 2, 1, 10, 9), 1, (15.0, 28.0), 0),
    "tm5_u2b4": ((2, 4, 1, 2, 5, 6), (2, 4, 4, 1, 10, 9), 1, (18.0, 30.0), 0),
    "tm3_codebook3": ((2, 2, 1, 2, 3, 6), (2, 2, 2, 1, 10, 9), 1, (20.0, 30.0), 3),
    "tm7_codebook9": ((1, 4, 1, 1, 7, 3), (1, 4, 4, 1, 10, 9), 1, (10.0, 20.0), 9),
    "lmode_siso": ((1, 1, 1, 2, 0, 3), (1, 1, 1, 1, 10, 9), 0, (6.0, 15.0), 0),
    "lmode_C4": ((8, 16, 1, 1, 5, 8), (8, 16, 4, 1, 10, 9), 0, (30.0, 30.0), 0),
    "lmode_txdiv2": ((2, 2, 1, 3, 1, 4), (2, 2, 2, 1, 10, 9), 0, (12.0, 25.0), 0),
    "lm40_27_b12": ((1, 12, 1, 1, 0, 4), (1, 12, 1, 1, 40, 27), 1, (15.0, 25.0), 0),
    "lm40_27_u8b12_tm5": ((8, 12, 1, 1, 5, 6), (8, 12, 4, 1, 40, 27), 1, (25.0, 30.0), 0),
    "lm1_1_tm1": ((2, 2, 1, 1, 1, 3), (2, 2, 2, 1, 1, 1), 1, (10.0, 25.0), 0),
    "lm1_1_u8b16": ((8, 16, 1, 1, 0, 8), (8, 16, 1, 1, 1, 1), 1, (30.0, 30.0), 0),
    "os2": ((1, 1, 1, 1, 0, 2), (1, 1, 1, 2, 10, 9), 1, (5.0, 20.0), 0),
    "os2_u2b2_tm1": ((2, 2, 1, 1, 1, 4), (2, 2, 2, 2, 10, 9), 1, (15.0, 25.0), 0),
    "subslot_tm5": ((1, 2, 0, 3, 5, 7), (1, 2, 4, 1, 10, 9), 1, (22.0, 30.0), 0),
    # a u = 2 packet in a u_max = 8 / b_max = 16 context: N_b_DFT_os = 4096, the STF front end's
    # compact in-place layout over several rounds of polyphase blocks (rx_stf_ant_kernel)
    "u2_in_u8b16": ((2, 4, 1, 1, 0, 4), (8, 16, 1, 1, 10, 9), 1, (20.0, 30.0), 0),
    # u = 1 at the same rate: N_b_DFT_os = 8192, the STF front end's chunked layout (rx_stf_ant_kernel)
    # and the generic FFT front end with one symbol per pass, twiddles through the L1 (rx_fft_kernel)
    "u1_in_u8b16": ((1, 16, 1, 1, 0, 4), (8, 16, 1, 1, 10, 9), 1, (20.0,), 0),
    # C4's packet at os_min = 2: N_b_DFT_os = 2048, 45-tap resamplers, TX through the DECT-rate scratch
    # (tx_big_sym_kernel) and the RX generic FFT front end
    "os2_C4": ((8, 16, 1, 1, 5, 8), (8, 16, 4, 2, 10, 9), 1, (30.0,), 0),
}


# TX-only parity configurations: transmission modes the reference RX cannot demodulate (spatial
# multiplexing, N_SS > 1: rx_synced.cpp:1331-1333) or that the RX here declines (N_eff_TX = 8,
# DESIGN.md §7) -- their TX (tx.cpp:1004-1116 N_SS streams, transmit_diversity_precoding.cpp modulo
# 12 pairs, beamforming_and_antenna_port_mapping.cpp 8-antenna W) still has a parity gate.
TX_ONLY_CASES = {
    "tm2_sm2": ((2, 2, 1, 2, 2, 4), (2, 2, 2, 1, 10, 9), 1, (), 0),
    "tm6_sm4": ((1, 4, 1, 2, 6, 3), (1, 4, 4, 1, 10, 9), 1, (), 0),
    "tm9_sm4_cb": ((1, 2, 1, 2, 9, 2), (1, 2, 4, 1, 10, 9), 1, (), 1),
    "tm10_txdiv8": ((1, 2, 1, 2, 10, 4), (1, 2, 8, 1, 10, 9), 1, (), 0),
    "tm10_u8b16": ((8, 16, 1, 1, 10, 8), (8, 16, 8, 1, 10, 9), 1, (), 0),
    "tm11_sm8": ((1, 4, 1, 1, 11, 2), (1, 4, 8, 1, 10, 9), 1, (), 0),
    # 4 spatial streams at mu8 b16 on the streaming TX kernel: 2.6 / 3.5 KB of PDC bytes per symbol,
    # the 4 KiB staging window (tx.hip TXS_SBW_SM)
    "tm6_u8b16_64qam": ((8, 16, 1, 1, 6, 6), (8, 16, 4, 1, 10, 9), 1, (), 0),
    "tm6_u8b16_256qam": ((8, 16, 1, 1, 6, 8), (8, 16, 4, 1, 10, 9), 1, (), 0),
    # the streaming kernel's multi-bit byte path (N_bps < 8: symbols straddle bytes), SISO and TM5
    "u8b16_64qam": ((8, 16, 1, 1, 0, 6), (8, 16, 1, 1, 10, 9), 1, (), 0),
    "tm5_u8b16_16qam": ((8, 16, 1, 1, 5, 4), (8, 16, 4, 1, 10, 9), 1, (), 0),
}


def case(name):
    """(psdef tuple, cfg tuple) of a configuration name of CONFIGS, PARITY_CASES or TX_ONLY_CASES."""
    if name in CONFIGS:
        return CONFIGS[name]
    c = PARITY_CASES.get(name) or TX_ONLY_CASES[name]
    return c[0], c[1]


def random_bits(rng, n_bits):
    return rng.integers(0, 2, n_bits, dtype=np.uint8)


def mixing_matrix(rng, n_rx, n_tx):
    if n_rx == 1 and n_tx == 1:
        return np.ones((1, 1), dtype=np.complex64)
    H = (rng.standard_normal((n_rx, n_tx)) + 1j * rng.standard_normal((n_rx, n_tx))) / np.sqrt(2 * n_tx)
    return H.astype(np.complex64)


def channel(rng, iq_tx, n_rx, S_in, offset, cfo_hw_rad, snr_db, H=None):
    """iq_tx complex64 [N_TX, S] -> rx window complex64 [n_rx, S_in]."""
    n_tx, S = iq_tx.shape
    if H is None:
        H = mixing_matrix(rng, n_rx, n_tx)
    y = H @ iq_tx
    out = np.zeros((n_rx, S_in), dtype=np.complex128)
    n = min(S, S_in - offset)
    out[:, offset:offset + n] = y[:, :n]
    out *= np.exp(1j * cfo_hw_rad * np.arange(S_in))[None, :]
    if snr_db is not None:
        p = np.mean(np.abs(y[:, : S // 2]) ** 2)
        sigma = np.sqrt(p / 10 ** (snr_db / 10) / 2)
        out += sigma * (rng.standard_normal(out.shape) + 1j * rng.standard_normal(out.shape))
    return out.astype(np.complex64)


def sync_window(rng, O, name, S_win, starts, cfo_dect_rad, snr_db=30.0, n_rx=None, seed_bits=None):
    """One sync window (complex64 [n_rx, S_win]) holding oracle-TX packets of configuration `name`
    starting at the hw-sample offsets `starts` (each with its own random N_RX x N_TX mixing), CFO
    cfo_dect_rad per DECT-rate sample (the TX mixer applies it at the hw rate), AWGN at snr_db
    relative to the packet power. Returns (window, [(pcc_d, pdc_d, network_id, plcf_type)])."""
    psd, cfgt = case(name)
    cf = O.cfg(cfgt[0], cfgt[1], os_min=cfgt[3], L=cfgt[4], M=cfgt[5])
    ps = O.psdef(*psd)
    sz = O.packet_sizes(ps)
    n_rx = n_rx or cfgt[2]
    S_slot = O.dims(cf, ps)["N_packet_os_rs"]
    win = np.zeros((n_rx, S_win), np.complex128)
    meta, p_sig = [], []
    for i, st in enumerate(starts):
        pcc = rng.integers(0, 256, 25, dtype=np.uint8)
        pdc = rng.integers(0, 256, (sz["G"] + 7) // 8, dtype=np.uint8)
        nid, pt = 100 + i % 6, 1 + i % 2
        x, _ = O.tx(cf, ps, pcc, pdc, S_slot, network_id=nid, plcf_type=pt,
                    phase_inc=cfo_dect_rad * cfgt[5] / cfgt[4])
        H = mixing_matrix(rng, n_rx, x.shape[0])
        y = H @ x
        n = min(S_slot, S_win - st)
        win[:, st:st + n] += y[:, :n]
        p_sig.append(np.mean(np.abs(y[:, : S_slot // 2]) ** 2))
        meta.append((pcc, pdc, nid, pt))
    if snr_db is not None:
        p = np.mean(p_sig) if p_sig else 0.05
        sigma = np.sqrt(p / 10 ** (snr_db / 10) / 2)
        win += sigma * (rng.standard_normal(win.shape) + 1j * rng.standard_normal(win.shape))
    return win.astype(np.complex64), meta
