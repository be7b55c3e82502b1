"""Oracle self-consistency on CPU (TEST INFRASTRUCTURE check): the oracle's TX restatement feeds its
RX restatement through a seeded channel (random N_RX x N_TX mixing, integer offset, CFO, AWGN) and
must recover every PCC/PDC bit at high SNR, report the SNR it was given, and its float path (the
reference's float arithmetic, used as the CPU baseline) must agree with the double path."""
import numpy as np
import pytest

import oracle_py as O
import phy_fixtures as F


def _loop(name, snr_db, seed, use_float=False, n_rx=None):
    rng = np.random.default_rng(seed)
    ps_t, cf_t = F.CONFIGS[name]
    u_max, b_max, ntx_max, os_min, L, M = cf_t
    ps, cf = O.psdef(*ps_t), O.cfg(u_max, b_max, os_min, L, M)
    sz = O.packet_sizes(ps)
    S = O.dims(cf, ps)["N_packet_os_rs"]
    pcc_bits = F.random_bits(rng, 196)
    pdc_bits = F.random_bits(rng, sz["G"])
    iq_tx, _ = O.tx(cf, ps, O.pack_bits(pcc_bits), O.pack_bits(pdc_bits), S, network_id=101, plcf_type=2,
                    use_float=use_float)
    off = int(rng.integers(0, 32))
    cfo_dect = rng.uniform(-1.75, 1.75) * 2 * np.pi / O.dims(cf, ps)["N_b_DFT_os"]
    win = F.channel(rng, iq_tx, n_rx or ntx_max, S, off, cfo_dect * M / L, snr_db)
    r = O.rx(cf, ps, win, off, -cfo_dect, network_id=101, plcf_type=2, use_float=use_float)
    return pcc_bits, pdc_bits, r


@pytest.mark.parametrize("name,snr", [("C2", 25.0), ("C3", 40.0), ("C4", 40.0)])
def test_loopback_recovers_bits(name, snr):
    pcc_bits, pdc_bits, r = _loop(name, snr, seed=5)
    assert np.array_equal((r["pcc_llr"] > 0).astype(np.uint8), pcc_bits)
    # 256-QAM sits ~36 dB above the resampler / interpolation error floor: allow 1e-4 BER there
    n_err = int(np.sum((r["pdc_llr"] > 0).astype(np.uint8) != pdc_bits))
    assert n_err <= (0 if name == "C2" else 1e-4 * pdc_bits.size), n_err
    # estimator_snr.cpp measures on the DRS cells; the channel defines SNR on time samples, and the
    # resampler / interpolation error floor caps the estimate near 36.6 dB (noise-free input)
    assert abs(r["snr_pdc"] - min(snr, 36.6)) < 3.0, r["snr_pdc"]


def test_float_path_matches_double_path():
    _, _, rd = _loop("C2", 20.0, seed=9)
    _, _, rf = _loop("C2", 20.0, seed=9, use_float=True)
    d = np.abs(rd["pdc_llr"].astype(np.int32) - rf["pdc_llr"].astype(np.int32))
    assert d.max() <= 2, d.max()
    assert abs(rd["snr_pdc"] - rf["snr_pdc"]) < 0.01


def test_llr_sign_convention_and_scale():
    # positive LLR = bit 1 (phy_config.hpp:39-41); QPSK PCC magnitudes ~100/sqrt(2) per unit amplitude
    pcc_bits, _, r = _loop("C2", 60.0, seed=3)
    mag = np.abs(r["pcc_llr"].astype(np.float64))
    assert 50 < np.median(mag) < 100
    assert np.array_equal(np.sign(r["pcc_llr"]) > 0, pcc_bits.astype(bool))


def test_gold_sequence_properties():
    # 3GPP TS 36.211 §7.2 Gold sequence (Nc = 1600): balanced, and c_init selects the sequence
    a, b = O.gold(0x44454354, 4096), O.gold(0x44454355, 4096)
    assert abs(int(a.sum()) - 2048) < 150
    assert np.mean(a != b) > 0.4
    assert np.array_equal(O.gold(0x44454354, 100), a[:100])


def test_mimo_report_codebook_search():
    """estimator_mimo_t (A29): for a rank-one channel H = g w^T, the recommended single-stream
    codebook entry (both directions) is the one matching w (maximises min RX power)."""
    import phy_fixtures as F
    psd, cfgt = F.CONFIGS["C4"]
    cf = O.cfg(cfgt[0], cfgt[1])
    ps = O.psdef(*psd)
    sz = O.packet_sizes(ps)
    rng = np.random.default_rng(12)
    S = O.dims(cf, ps)["N_packet_os_rs"]
    x, _ = O.tx(cf, ps, rng.integers(0, 256, 25, dtype=np.uint8),
                rng.integers(0, 256, (sz["G"] + 7) // 8, dtype=np.uint8), S)
    # W_2 codebook entry 17 = (1, j, j, -1) / 2 for 4 antennas (beamforming_and_antenna_port_mapping.cpp:252-257);
    # the receiver sees TS streams through H[rx][ts]; a rank-one H = g (x) conj(w) aligns best with entry 17
    w = np.array([1, 1j, 1j, -1]) / 2
    g = np.array([1.0, 0.9, 1.1, 0.95])
    H = np.outer(g, np.conj(w)).astype(np.complex64)
    r = O.rx(cf, ps, (H @ x).astype(np.complex64))
    assert r["mimo_N_TS_other"] == 4
    assert r["mimo_idx"] == 17


@pytest.mark.parametrize("name", sorted(F.PARITY_CASES))
def test_loopback_parity_cases(name):
    """Every GPU parity configuration (phy_fixtures.PARITY_CASES) round-trips through the oracle on
    the CPU at 30 dB: the checker itself supports the mode before the HIP path is compared with it."""
    psd, cf_t, lr, _, cb = F.PARITY_CASES[name]
    u_max, b_max, n_ant, os_min, L, M = cf_t
    cf, ps = O.cfg(u_max, b_max, os_min, L, M, lr=lr), O.psdef(*psd)
    sz = O.packet_sizes(ps)
    S = O.dims(cf, ps)["N_packet_os_rs"]
    rng = np.random.default_rng(1)
    pcc_bits, pdc_bits = F.random_bits(rng, 196), F.random_bits(rng, sz["G"])
    x, _ = O.tx(cf, ps, O.pack_bits(pcc_bits), O.pack_bits(pdc_bits), S, codebook=cb)
    assert x.shape[0] == sz["N_TX"]
    win = F.channel(rng, x, n_ant, S, 5, 0.0, 30.0)
    r = O.rx(cf, ps, win, 5, 0.0, 100, 1)
    assert np.array_equal((r["pcc_llr"] > 0).astype(np.uint8), pcc_bits)
    assert np.mean((r["pdc_llr"] > 0).astype(np.uint8) != pdc_bits) < 5e-3
