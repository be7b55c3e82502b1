"""GPU synchronisation parity: dnrp_rx_sync_batch (kernels/sync.hip) against the oracle restatement
of sync_chunk_t::search() (oracle/oracle_sync.cpp) on identical windows.

Tolerances: found flags, report count, detection antenna and time, N_eff_TX and the fine peak time
exact; coarse peak time within 1 DECT sample (smoothed-metric plateau: float vs double sums can
move the last maximum by one position); fractional CFO within 2e-6 rad per DECT sample; RMS and
metrics within 1e-3 relative. Then the synchronised chain: GPU sync -> GPU PCC/PDC demodulation
against the oracle RX started from the same (GPU) sync report (int16 LLRs within 1 LSB), after the
oracle's own search has found the same fine peak.

Geometries: the bench configurations C2/C3/C4 (L/M 10/9, hl 24 stream kernel) plus every other sync
kernel instantiation dispatched at kernels/sync.hip SYNC_DISPATCH / launch_sync_steps: L = M = 1
(<1,1,0>), 40/27 (<0,0,0>, generic taps), os_min 2 (<9,10,4>), two transmit streams, and eight
antennas with the fourth STF template (N_eff_TX = 8, crosscorrelator.cpp:122-251,
physical_resources.hpp:44); the wave-kernel fallback of the step sums (DNRP_SYNC_STREAM=0).
"""
import numpy as np
import pytest

import llr_gate
import oracle_py as O
import phy_fixtures as F

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu


def _phy(name, max_batch=8):
    import dnrp
    ps, cf = F.case(name)
    u_max, b_max, ntx, os_min, L, M = cf
    lr = F.PARITY_CASES[name][2] if name in F.PARITY_CASES else 1
    phy = dnrp.Phy(u_max, b_max, ntx, os_min, L, M, chestim_mode_lr=bool(lr), max_batch=max_batch)
    for nid in range(100, 106):
        phy.add_network_id(nid)
    return phy


def _compare(g, o, where):
    assert int(g["found"]) == o["found"] == 1, where
    assert int(g["detection_ant_idx"]) == o["det_ant"], where
    assert int(g["detection_time_local"]) == o["det_time"], (where, int(g["detection_time_local"]), o["det_time"])
    assert abs(int(g["coarse_peak_time_local"]) - o["coarse_local"]) <= 1, (where, int(g["coarse_peak_time_local"]),
                                                                            o["coarse_local"])
    assert int(g["N_eff_TX"]) == o["N_eff_TX"], where
    assert int(g["fine_peak_time"]) == o["fine_64"], (where, int(g["fine_peak_time"]), o["fine_64"])
    assert abs(float(g["cfo_fractional_rad"]) - o["cfo_frac"]) < 2e-6, (where, float(g["cfo_fractional_rad"]),
                                                                         o["cfo_frac"])
    np.testing.assert_allclose(g["detection_metric"], o["det_metric"], rtol=1e-3)
    np.testing.assert_allclose(g["coarse_peak_array"], o["coarse_metric"], rtol=1e-3, atol=1e-6)
    np.testing.assert_allclose(g["rms_array"], o["rms"], rtol=1e-3, atol=1e-7)
    nt = int(np.count_nonzero(o["xc_metric"]))
    np.testing.assert_allclose(g["fine_peak_metric"][:nt], o["xc_metric"][:nt], rtol=1e-3)


def _run(phy, sc, windows, max_reports, stream_layout=False):
    """windows: list of complex64 [n_ant, S]. Returns the GPU results [n, max_reports]."""
    dev = torch.device("cuda:0")
    n = len(windows)
    n_ant, S = windows[0].shape
    if stream_layout:  # per-antenna continuous streams, window w at w*S
        streams = np.concatenate(windows, axis=1)  # [n_ant, n*S]
        t = torch.from_numpy(np.ascontiguousarray(streams).view(np.float32).reshape(n_ant, n * S, 2)).to(dev)
        res, cnt = phy.rx_sync_batch(sc, t, n, S, S, n * S)
    else:
        t = torch.from_numpy(np.stack(windows).view(np.float32).reshape(n, n_ant, S, 2)).to(dev)
        res, cnt = phy.rx_sync_batch(sc, t, n, S, n_ant * S, S)
    phy.sync()
    return res, cnt


SYNC_GEOMETRIES = [
    ("C4", 20480, 4096, False), ("C3", 20480, 4096, True), ("C2", 1500, 400, False),
    ("lm1_1_u8b16", 20480, 4096, False),        # L = M = 1: sync kernels <1, 1, 0>
    ("lm40_27_u8b12_tm5", 20480, 4096, True),   # 40/27: generic-tap kernels <0, 0, 0>
    ("os2_u2b2_tm1", 6000, 1200, False),        # os_min 2: 9/10 with 45 taps <9, 10, 4>
    ("tm1_txdiv2", 12800, 2560, False),         # 2 antennas, N_eff_TX = 2 template
    ("tm10_u8b16", 20480, 4096, False),         # 8 antennas, 4th STF template (N_eff_TX = 8)
]


@pytest.mark.parametrize("name,S_win,chunk,stream_layout", SYNC_GEOMETRIES)
def test_sync_parity(name, S_win, chunk, stream_layout):
    _sync_parity(name, S_win, chunk, stream_layout)


@pytest.mark.parametrize("name", ["C4", "C3"])
def test_sync_parity_wave_kernel(name, monkeypatch):
    """The step-sum wave kernel (sync_steps_wave_kernel, used when the stream kernel's geometry does
    not hold) against the oracle: DNRP_SYNC_STREAM=0 forces it."""
    monkeypatch.setenv("DNRP_SYNC_STREAM", "0")
    _sync_parity(name, 20480, 4096, False)


@pytest.mark.parametrize("name,stream_layout", [("C4", False), ("C3", True)])
def test_sync_parity_single_prefetch(name, stream_layout, monkeypatch):
    """The one-chunk-prefetch stream kernel (sync_steps_stream_kernel<.., 16, 1>) that the pipelined
    kernel (sync_steps_pipe_kernel, default for 64-sample steps) replaced: DNRP_SYNC_PIPE=0."""
    monkeypatch.setenv("DNRP_SYNC_PIPE", "0")
    _sync_parity(name, 20480, 4096, stream_layout)


def _sync_parity(name, S_win, chunk, stream_layout):
    import dnrp
    rng = np.random.default_rng(21)
    psd, cfgt = F.case(name)
    n_ant = cfgt[2]
    phy = _phy(name)
    windows, truth = [], []
    for i in range(5):
        start = int(rng.integers(0.15 * S_win, 0.3 * S_win))
        cfo = rng.uniform(-1.75, 1.75) * 2 * np.pi / (64 * psd[1] * cfgt[3])  # +-1.75 subcarriers
        win, _ = F.sync_window(rng, O, name, S_win, [start], cfo)
        windows.append(win)
        truth.append((start, cfo))
    noise, _ = F.sync_window(rng, O, name, S_win, [], 0.0)
    windows.append(noise)
    sc = dnrp.SyncCfg(psd[0], psd[1], n_ant, chunk, 2)
    res, cnt = _run(phy, sc, windows, 2, stream_layout)
    osc = O.sync_cfg(psd[0], psd[1], os_min=cfgt[3], L=cfgt[4], M=cfgt[5], n_ant=n_ant, chunk_len=chunk)
    for w, win in enumerate(windows):
        ref = O.sync(osc, win, max_reports=2)
        assert int(cnt[w]) == len(ref), (w, int(cnt[w]), len(ref))
        for k, o in enumerate(ref):
            _compare(res[w, k], o, (name, w, k))
        for k in range(len(ref), 2):
            assert int(res[w, k]["found"]) == 0
        if w < len(truth):
            assert int(res[w, 0]["fine_peak_time"]) == truth[w][0]
            assert int(res[w, 0]["N_eff_TX"]) == O.packet_sizes(O.psdef(*psd))["N_eff_TX"]


@pytest.mark.parametrize("name,rounds", [("C4", "0"), ("C4", "1"), ("tm10_u8b16", "1"), ("C3", "3")])
def test_sync_parity_detect_rounds(name, rounds, monkeypatch):
    """Detection + coarse peak with DNRP_SYNC_ROUNDS split rounds (detection-only workgroups, then one
    coarse-peak workgroup per window and antenna) before the inline kernel finishes: 0 = the inline
    kernel alone, 1 = every window's first report resolved by the inline kernel's resume path."""
    monkeypatch.setenv("DNRP_SYNC_ROUNDS", rounds)
    _sync_parity(name, 20480, 4096, False)


@pytest.mark.parametrize("rounds", ["0", "1", "2", "4"])
def test_sync_two_packets_per_window(rounds, monkeypatch):
    """Two packets per window: with 1 or 2 split rounds the second (or the empty tail search) is left
    to the inline kernel, with 4 the split rounds finish every window."""
    monkeypatch.setenv("DNRP_SYNC_ROUNDS", rounds)
    import dnrp
    rng = np.random.default_rng(23)
    phy = _phy("C2")
    made = [F.sync_window(rng, O, "C2", 3000, [300 + 7 * i, 1650 - 5 * i], 0.4 * (i - 1) * 2 * np.pi / 64)
            for i in range(3)]
    windows = [m[0] for m in made]
    sc = dnrp.SyncCfg(1, 1, 1, 3000, 4)
    res, cnt = _run(phy, sc, windows, 4)
    osc = O.sync_cfg(1, 1, n_ant=1, chunk_len=3000)
    for w, win in enumerate(windows):
        ref = O.sync(osc, win, max_reports=4)
        assert len(ref) == 2 and int(cnt[w]) == 2
        for k, o in enumerate(ref):
            _compare(res[w, k], o, (w, k))
    # both packets of every window demodulated from the shared window (dnrp_sync_report::window)
    reps = dnrp.found_reports(res, cnt)
    assert list(reps["window"]) == [0, 0, 1, 1, 2, 2]
    dev = torch.device("cuda:0")
    iq = torch.from_numpy(np.stack(windows).view(np.float32).reshape(3, 1, 3000, 2)).to(dev)
    ps = dnrp.psdef(*F.CONFIGS["C2"][0])
    G = phy.packet_sizes(ps)["G"]
    pcc_llr = torch.zeros((6, 196), dtype=torch.int16, device=dev)
    pdc_llr = torch.zeros((6, G), dtype=torch.int16, device=dev)
    phy.rx_pcc_batch(reps, iq, pcc_llr)
    meta = [m for _, ms in made for m in ms]
    phy.rx_pdc_batch([dnrp.PdcReq(ps, i, meta[i][2], meta[i][3]) for i in range(6)], iq, pdc_llr)
    phy.sync()
    ocf, ops = O.cfg(1, 1), O.psdef(*F.CONFIGS["C2"][0])
    for i in range(6):
        r = O.rx(ocf, ops, windows[int(reps["window"][i])], int(reps["fine_peak_time"][i]),
                 float(reps["cfo_fractional_rad"][i]), meta[i][2], meta[i][3])
        llr_gate.check(("two_per_window", i, "pcc"), pcc_llr[i].cpu().numpy(), r["pcc_llr"])
        llr_gate.check(("two_per_window", i, "pdc"), pdc_llr[i].cpu().numpy(), r["pdc_llr"])
        assert np.array_equal(np.unpackbits(meta[i][1])[:G], (r["pdc_llr"] > 0).astype(np.uint8)), i


@pytest.mark.parametrize("name", ["C4", "lm1_1_u8b16", "lm40_27_u8b12_tm5", "os2_u2b2_tm1", "tm1_txdiv2"])
def test_sync_then_demodulate(name):
    """GPU sync -> GPU RX on the synchronised windows vs the oracle RX fed the same (GPU) sync report,
    int16 LLRs within the +-1 gate; the oracle's own search must find the same fine peak and CFO."""
    import dnrp
    rng = np.random.default_rng(25)
    psd, cfgt = F.case(name)
    lr = F.PARITY_CASES[name][2] if name in F.PARITY_CASES else 1
    n_ant = cfgt[2]
    phy = _phy(name)
    ps = dnrp.psdef(*psd)
    sz = phy.packet_sizes(ps)
    S = sz["N_samples_packet_os_rs"]
    pre = sz["N_samples_STF"] * cfgt[3] * cfgt[4] // cfgt[5]  # one STF of lead-in at the hw rate
    S_win = S + pre + 32
    chunk = S_win * 7 // 8
    windows, metas = [], []
    for i in range(2):
        cfo = rng.uniform(-1.75, 1.75) * 2 * np.pi / sz["N_b_DFT_os"]
        win, meta = F.sync_window(rng, O, name, S_win, [pre + int(rng.integers(0, 32))], cfo)
        windows.append(win)
        metas.append(meta[0])
    sc = dnrp.SyncCfg(psd[0], psd[1], n_ant, chunk, 1)
    res, cnt = _run(phy, sc, windows, 1)
    assert list(cnt) == [1, 1]
    dev = torch.device("cuda:0")
    iq = torch.from_numpy(np.stack(windows).view(np.float32).reshape(2, n_ant, S_win, 2)).to(dev)
    reps = dnrp.sync_reports(res[:, 0])
    pcc_llr = torch.zeros((2, 196), dtype=torch.int16, device=dev)
    pdc_llr = torch.zeros((2, sz["G"]), dtype=torch.int16, device=dev)
    phy.rx_pcc_batch(reps, iq, pcc_llr)
    phy.rx_pdc_batch([dnrp.PdcReq(ps, i, m[2], m[3]) for i, m in enumerate(metas)], iq, pdc_llr)
    phy.sync()
    g_pcc, g_pdc = pcc_llr.cpu().numpy(), pdc_llr.cpu().numpy()
    ocf = O.cfg(cfgt[0], cfgt[1], os_min=cfgt[3], L=cfgt[4], M=cfgt[5], lr=lr)
    osc = O.sync_cfg(psd[0], psd[1], os_min=cfgt[3], L=cfgt[4], M=cfgt[5], n_ant=n_ant, chunk_len=chunk)
    for i, win in enumerate(windows):
        o = O.sync(osc, win, max_reports=1)[0]
        fine, cfo_g = int(res[i, 0]["fine_peak_time"]), float(res[i, 0]["cfo_fractional_rad"])
        assert o["fine_64"] == fine and abs(o["cfo_frac"] - cfo_g) < 2e-6, (name, i, o["fine_64"], fine)
        r = O.rx(ocf, O.psdef(*psd), win, fine, cfo_g, metas[i][2], metas[i][3])
        llr_gate.check((name, i, "pcc"), g_pcc[i], r["pcc_llr"])
        llr_gate.check((name, i, "pdc"), g_pdc[i], r["pdc_llr"])
        bits = np.unpackbits(metas[i][1])[: sz["G"]]
        assert np.mean((g_pdc[i] > 0).astype(np.uint8) != bits) < 2e-2, name
