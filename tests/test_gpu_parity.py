"""GPU parity tests: libdnrp.so (HIP, gfx950) against the CPU oracle on identical inputs.

Tolerances:
  * TX IQ: relative L2 error per packet and antenna <= 1e-4 (float IQ), GI/tail exactly zero.
  * RX: int16 LLRs |delta| <= 1 LSB against the double-precision oracle (pre-quantisation float
    values agree to ~1e-5 relative; the +-1 covers rounding-boundary flips), SNR reports within
    0.05 dB, hard decisions identical.
"""
import numpy as np
import pytest

import oracle_py as O
import phy_fixtures as F

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu


def _ctx(name, max_batch=8):
    import dnrp
    ps, cf = F.CONFIGS[name]
    u_max, b_max, ntx, os_min, L, M = cf
    phy = dnrp.Phy(u_max, b_max, ntx, os_min, L, M, max_batch=max_batch)
    for nid in range(100, 106):
        phy.add_network_id(nid)
    return phy, dnrp.psdef(*ps), O.psdef(*ps), O.cfg(u_max, b_max, os_min, L, M)


def _tx_inputs(rng, n, sz):
    pcc_bits = [F.random_bits(rng, 196) for _ in range(n)]
    pdc_bits = [F.random_bits(rng, sz["G"]) for _ in range(n)]
    pcc = np.stack([np.concatenate([O.pack_bits(b), np.zeros(0, np.uint8)]) for b in pcc_bits])
    stride = (sz["G"] + 7) // 8
    pdc = np.stack([O.pack_bits(b) for b in pdc_bits])
    assert pcc.shape == (n, 25) and pdc.shape == (n, stride)
    return pcc_bits, pdc_bits, pcc, pdc


def _gpu_tx(phy, ps, descs, pcc, pdc, S):
    dev = torch.device("cuda:0")
    n = len(descs)
    sz = phy.packet_sizes(ps)
    out = torch.empty((n, sz["N_TX"], S, 2), dtype=torch.float32, device=dev)
    out.fill_(7.0)  # poison: every sample must be written
    phy.tx_batch(ps, descs, torch.from_numpy(pcc).to(dev), torch.from_numpy(pdc).to(dev), out)
    phy.sync()
    return out.cpu().numpy().view(np.complex64)[..., 0]


@pytest.mark.parametrize("name", ["C2", "C3", "C4"])
def test_tx_parity(name):
    import dnrp
    rng = np.random.default_rng(0xDEC7)
    phy, ps, ops, ocf = _ctx(name)
    sz = phy.packet_sizes(ps)
    S = sz["N_samples_packet_os_rs"]
    n = 3
    _, _, pcc, pdc = _tx_inputs(rng, n, sz)
    descs = []
    for i in range(n):
        cfo = (rng.uniform(-1.75, 1.75) * 2 * np.pi / sz["N_b_DFT_os"]) if i > 0 else 0.0
        descs.append(dnrp.TxDesc(0, 100 + i, 1 + i % 2, 5, 1.0, float(rng.uniform(-3, 3)) if i == 2 else 0.0,
                                 cfo, 0))
    iq = _gpu_tx(phy, ps, descs, pcc, pdc, S)
    for i, d in enumerate(descs):
        ref, n_tx = O.tx(ocf, ops, pcc[i], pdc[i], S, codebook=0, network_id=d.network_id,
                         plcf_type=d.plcf_type, gi=5, dac=1.0, phase=float(np.float32(d.iq_phase_rad)),
                         phase_inc=float(np.float32(d.iq_phase_increment_s2s_post_resampling_rad)))
        keep = sz["N_samples_packet_no_GI_os_rs"]
        for a in range(sz["N_TX"]):
            e = np.linalg.norm(iq[i, a, :keep] - ref[a, :keep]) / np.linalg.norm(ref[a, :keep])
            assert e <= 1e-4, (name, i, a, e)
            assert np.all(iq[i, a, keep:] == 0), (name, i, a)
        assert n_tx == keep + (S - keep) * 5 // 100


def _rx_case(name, snr_db, n=3, seed=11):
    import dnrp
    rng = np.random.default_rng(seed)
    phy, ps, ops, ocf = _ctx(name)
    sz = phy.packet_sizes(ps)
    S = sz["N_samples_packet_os_rs"]
    n_rx = phy.cfg.N_TX_max
    _, _, pcc, pdc = _tx_inputs(rng, n, sz)
    windows, reports, nids, types = [], [], [], []
    L, M = int(phy.cfg.L), int(phy.cfg.M)
    for i in range(n):
        nid, pt = 100 + (i % 6), 1 + i % 2
        iq_tx, _ = O.tx(ocf, ops, pcc[i], pdc[i], S, network_id=nid, plcf_type=pt)
        off = int(rng.integers(0, 32))
        cfo_dect = rng.uniform(-1.75, 1.75) * 2 * np.pi / sz["N_b_DFT_os"]  # rad per DECT sample
        cfo_hw = cfo_dect * M / L
        win = F.channel(rng, iq_tx, n_rx, S, off, cfo_hw, snr_db)
        windows.append(win)
        # sync estimate with a small residual error the STF re-estimate has to remove
        est = -cfo_dect + rng.uniform(-0.02, 0.02) * 2 * np.pi / sz["N_b_DFT_os"]
        reports.append(dnrp.SyncReport(off, float(est), 0.0, ops[0], ops[1], sz["N_eff_TX"]))
        nids.append(nid)
        types.append(pt)
    dev = torch.device("cuda:0")
    iq = torch.from_numpy(np.stack(windows).view(np.float32).reshape(n, n_rx, S, 2)).to(dev)
    pcc_llr = torch.zeros((n, 196), dtype=torch.int16, device=dev)
    pdc_llr = torch.zeros((n, sz["G"]), dtype=torch.int16, device=dev)
    rep1 = phy.rx_pcc_batch(reports, iq, pcc_llr, want_report=True)
    rep2 = phy.rx_pdc_batch(ps, [dnrp.PdcReq(nids[i], types[i]) for i in range(n)], pdc_llr, want_report=True)
    phy.sync()
    g_pcc, g_pdc = pcc_llr.cpu().numpy(), pdc_llr.cpu().numpy()
    res = []
    for i in range(n):
        r = O.rx(ocf, ops, windows[i], reports[i].fine_peak_time,
                 float(np.float32(reports[i].cfo_fractional_rad)), nids[i], types[i])
        res.append((g_pcc[i], g_pdc[i], rep1[i], rep2[i], r))
    return res


@pytest.mark.parametrize("name,snr", [("C2", 10.0), ("C3", 30.0), ("C4", 30.0)])
def test_rx_parity(name, snr):
    for g_pcc, g_pdc, r1, r2, r in _rx_case(name, snr):
        d_pcc = np.abs(g_pcc.astype(np.int32) - r["pcc_llr"].astype(np.int32))
        d_pdc = np.abs(g_pdc.astype(np.int32) - r["pdc_llr"].astype(np.int32))
        assert d_pcc.max() <= 1, (name, d_pcc.max(), np.argmax(d_pcc))
        assert d_pdc.max() <= 1, (name, d_pdc.max(), np.argmax(d_pdc), np.mean(d_pdc))
        assert abs(r1.snr_dB - r["snr_pcc"]) < 0.05, (r1.snr_dB, r["snr_pcc"])
        assert abs(r2.snr_dB - r["snr_pdc"]) < 0.05, (r2.snr_dB, r["snr_pdc"])
        # mimo_report_t (estimator_mimo.cpp): codebook recommendations exact
        assert (r2.mimo_N_TS_other, r2.tm_3_7_beamforming_idx, r2.tm_3_7_beamforming_reciprocal_idx) == \
            (r["mimo_N_TS_other"], r["mimo_idx"], r["mimo_idx_reciprocal"])
        assert abs(r1.sto_fractional - r["sto"]) < 1e-3
        for a in range(len(r["rms"])):
            assert abs(r1.rms[a] - r["rms"][a]) <= 1e-4 * max(1.0, r["rms"][a])
