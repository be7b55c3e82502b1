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
