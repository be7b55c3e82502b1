"""Simulated wireless channel on the GPU (dnrp_channel_batch, kernels/channel.hip) against a numpy
restatement of channel_awgn_t / channel_flat_t / channel_doubly_t + link_t::pass_through_link
(simulation/wireless/*.cpp) fed with the same link realisation (dnrp_channel_realization).

Noiseless outputs within 2e-5 relative L2 per (window, antenna) (float vs double sinusoid sums);
noise by its statistics (variance from noise.cpp's n0 within 3 %, zero mean, uncorrelated I/Q,
independent antennas); and the loopback GPU TX -> doubly-selective channel -> GPU sync -> GPU RX
recovering the bits (a functional check, parity unpinned: the reference draws its channel from a
time-seeded generator).
"""
import numpy as np
import pytest

import oracle_py as O
import phy_fixtures as F

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu


def _np_channel(cfg, tx, offsets, t0s, S_rx, n_rx):
    import dnrp
    n, n_tx, S_tx = tx.shape
    out = np.zeros((n, n_rx, S_rx), np.complex128)
    for w in range(n):
        r = dnrp.channel_realization(cfg, w, n_tx, n_rx)
        nn = np.arange(S_rx)
        t = t0s[w] + nn
        for rx in range(n_rx):
            for k in range(n_tx):
                if cfg.kind == dnrp.CH_DOUBLY:
                    for i, (d, a) in enumerate(zip(r["delay"][rx, k], r["amp"][rx, k])):
                        q = nn - offsets[w] - d
                        ok = (q >= 0) & (q < S_tx)
                        x = np.where(ok, tx[w, k, np.clip(q, 0, S_tx - 1)], 0)
                        g = np.zeros(S_rx, np.complex128)
                        for P, ph in zip(r["period"][rx, k, i], r["phase_rev"][rx, k, i]):
                            g += np.exp(2j * np.pi * ((t % abs(int(P))) / float(P) + ph))
                        out[w, rx] += float(a) * x * g
                else:
                    q = nn - offsets[w]
                    ok = (q >= 0) & (q < S_tx)
                    x = np.where(ok, tx[w, k, np.clip(q, 0, S_tx - 1)], 0)
                    out[w, rx] += x * (r["coef"][rx, k] if cfg.kind == dnrp.CH_FLAT else 1.0)
    return out * cfg.large_scale


def _dev(a):
    return torch.from_numpy(np.ascontiguousarray(a.astype(np.complex64)).view(np.float32).reshape(*a.shape, 2)).to("cuda:0")


@pytest.mark.parametrize("kind", [0, 1, 2])
def test_channel_noiseless(kind):
    import dnrp
    rng = np.random.default_rng(51 + kind)
    phy = dnrp.Phy(1, 2, 4, 1, 10, 9, max_batch=8)
    n, n_tx, n_rx, S_tx, S_rx = 3, 2, 3, 700, 1000
    tx = (rng.standard_normal((n, n_tx, S_tx)) + 1j * rng.standard_normal((n, n_tx, S_tx))).astype(np.complex64)
    offsets = [5, 120, 400]
    t0s = [0, 987654321, 2 ** 40 + 17]
    cfg = dnrp.ChannelCfg(kind, 1, 800.0, 900.0, 7680000, 0.7, dnrp.CH_NOISELESS_DB, 1.0, 99)
    rx = torch.zeros((n, n_rx, S_rx, 2), dtype=torch.float32, device="cuda:0")
    phy.channel_batch(cfg, _dev(tx), offsets, t0s, rx)
    phy.sync()
    got = rx.cpu().numpy().view(np.complex64)[..., 0]
    ref = _np_channel(cfg, tx, offsets, t0s, S_rx, n_rx)
    for w in range(n):
        for r in range(n_rx):
            err = np.linalg.norm(got[w, r] - ref[w, r]) / np.linalg.norm(ref[w, r])
            assert err < 2e-5, (kind, w, r, err)
    assert np.all(got[:, :, :5] == 0)  # before the first TX sample: nothing


def test_channel_noise_statistics():
    import dnrp
    phy = dnrp.Phy(1, 2, 4, 1, 10, 9, max_batch=8)
    n, S = 4, 200000
    tx = torch.zeros((n, 1, 16, 2), dtype=torch.float32, device="cuda:0")
    cfg = dnrp.ChannelCfg(dnrp.CH_AWGN, 0, 0.0, 0.0, 1, 1.0, 10.0, 0.8, 123)
    rx = torch.zeros((n, 2, S, 2), dtype=torch.float32, device="cuda:0")
    phy.channel_batch(cfg, tx, [0] * n, [0] * n, rx)
    phy.sync()
    z = rx.cpu().numpy().view(np.complex64)[..., 0].astype(np.complex128)
    n0 = 10 ** ((-10 * np.log10(0.8) - 10.0) / 10)  # noise.cpp -> ch_awgn set_n0
    assert abs(np.mean(np.abs(z) ** 2) / n0 - 1) < 0.03
    assert abs(np.mean(z.real)) < 0.01 * np.sqrt(n0) and abs(np.mean(z.real * z.imag)) < 0.01 * n0
    c = np.mean(z[:, 0] * np.conj(z[:, 1]))
    assert abs(c) < 0.01 * n0  # antennas independent
    k = np.mean(z[:, 0, 1:] * np.conj(z[:, 0, :-1]))
    assert abs(k) < 0.01 * n0  # white


def test_loopback_doubly_selective():
    """GPU TX -> EVA doubly-selective 4x4 channel with AWGN -> GPU sync -> GPU PCC/PDC demodulation."""
    import dnrp
    rng = np.random.default_rng(61)
    name = "C4"
    psd, cfgt = F.CONFIGS[name]
    phy = dnrp.Phy(*cfgt, max_batch=8)
    for nid in range(100, 106):
        phy.add_network_id(nid)
    ps = dnrp.psdef(*psd)
    sz = phy.packet_sizes(ps)
    S, G, n = sz["N_samples_packet_os_rs"], sz["G"], 4
    pcc = torch.from_numpy(rng.integers(0, 256, (n, 25), dtype=np.uint8)).cuda()
    pdc = torch.from_numpy(rng.integers(0, 256, (n, (G + 7) // 8), dtype=np.uint8)).cuda()
    descs = [dnrp.TxDesc(0, 100 + i, 1 + i % 2, 5, 1.0, 0.0, 0.0, 0) for i in range(n)]
    tx = torch.empty((n, 4, S, 2), dtype=torch.float32, device="cuda:0")
    phy.tx_batch(ps, descs, pcc, pdc, tx)
    pre, S_rx = 2400, S + 2400
    rate = 8 * 16 * 1728000 * 10 // 9
    cfg = dnrp.ChannelCfg(dnrp.CH_DOUBLY, 1, 50.0, 20.0, rate, 1.0, 30.0, 896 / 1024 * 9 / 10, 7)
    rx = torch.empty((n, 4, S_rx, 2), dtype=torch.float32, device="cuda:0")
    offs = [pre + int(o) for o in rng.integers(0, 32, n)]
    phy.channel_batch(cfg, tx, offs, [int(10 ** 9 * i) for i in range(n)], rx)
    sc = dnrp.SyncCfg(psd[0], psd[1], 4, 89280, 1)
    res, cnt = phy.rx_sync_batch(sc, rx, n, S_rx, 4 * S_rx, S_rx)
    phy.sync()
    assert list(cnt) == [1] * n
    reps = dnrp.sync_reports(res[:, 0])
    assert np.all(np.abs(reps["fine_peak_time"] - np.array(offs)) <= 8)  # delay spread shifts the peak
    pcc_llr = torch.zeros((n, 196), dtype=torch.int16, device="cuda:0")
    pdc_llr = torch.zeros((n, G), dtype=torch.int16, device="cuda:0")
    phy.rx_pcc_batch(reps, rx, pcc_llr)
    phy.rx_pdc_batch([dnrp.PdcReq(ps, i, 100 + i, 1 + i % 2) for i in range(n)], rx, pdc_llr)
    phy.sync()
    bits = np.unpackbits(pdc.cpu().numpy(), axis=1)[:, :G]
    ber = np.mean(bits != (pdc_llr.cpu().numpy() > 0))
    pcc_ber = np.mean(np.unpackbits(pcc.cpu().numpy(), axis=1)[:, :196] != (pcc_llr.cpu().numpy() > 0))
    assert pcc_ber < 0.02 and ber < 0.05, (pcc_ber, ber)
