"""Oracle synchronisation (oracle/oracle_sync.cpp) — restatement of sync_chunk_t::search()
(lib/src/phy/rx/sync/sync_chunk.cpp:143-279): detection, coarse peak, fine peak. Parity unpinned
(VOLK/srsRAN float accumulation order is absent from the image): checked here against the
configuration geometry the reference constructors compute, against the oracle TX (pinned by the
loopback tests) for the STF templates, and by recovering known packet positions, CFOs and N_eff_TX.
"""
import numpy as np
import pytest

import oracle_py as O
import phy_fixtures as F


def test_geometry_c4_c2():
    g = O.sync_geometry(O.sync_cfg(8, 16, n_ant=4, chunk_len=102400))
    # sync_chunk.cpp:54-69, crosscorrelator.cpp:53-57, stf_template.cpp:33, physical_resources.hpp:44
    assert (g["stf_len"], g["pattern"], g["step"], g["n_pattern"]) == (2304, 256, 64, 9)
    assert (g["A"], g["B"], g["C"], g["D"]) == (92160, 9216, 256, 2304)
    assert (g["xc_l"], g["xc_len"], g["tmpl_len"], g["n_templates"]) == (284, 569, 2560, 3)
    assert abs(g["rms_min"] - 0.005 * np.sqrt(221.184e6 / 30.72e6)) < 1e-7
    g = O.sync_geometry(O.sync_cfg(1, 1, n_ant=1, chunk_len=800))
    assert (g["stf_len"], g["pattern"], g["step"], g["n_pattern"]) == (112, 16, 4, 7)
    assert (g["xc_l"], g["xc_len"], g["tmpl_len"], g["n_templates"]) == (17, 35, 124, 1)


@pytest.mark.parametrize("name,n_eff", [("C3", 1), ("C2", 1)])
def test_template_is_the_tx_stf(name, n_eff):
    """stf_template_t builds the STF the TX sends (SISO, W = 1, DAC scale 1): first samples equal."""
    psd, cfgt = F.CONFIGS[name]
    cf = O.cfg(cfgt[0], cfgt[1], L=cfgt[4], M=cfgt[5])
    ps = O.psdef(*psd)
    sz = O.packet_sizes(ps)
    rng = np.random.default_rng(3)
    x, _ = O.tx(cf, ps, rng.integers(0, 256, 25, dtype=np.uint8),
                rng.integers(0, 256, (sz["G"] + 7) // 8, dtype=np.uint8), O.dims(cf, ps)["N_packet_os_rs"])
    t = O.stf_template(O.sync_cfg(psd[0], psd[1], L=cfgt[4], M=cfgt[5], n_ant=1), n_eff)
    n = len(t) - 40  # the TX resampler tail of the first data symbol reaches back ~hl samples
    np.testing.assert_allclose(t[:n], x[0, :n], rtol=0, atol=1e-5 * np.abs(t).max())


def _check_found(rep, start, cfo, n_eff):
    assert rep["found"] == 1
    assert rep["fine_64"] == start
    assert rep["N_eff_TX"] == n_eff
    assert abs(rep["cfo_frac"] + cfo) < 2e-4  # estimate is the correction (negative of the CFO)


@pytest.mark.parametrize("name,n_eff,S_win,start,chunk", [
    ("C4", 4, 20480, 3007, 4096), ("C3", 1, 20480, 2811, 4096), ("C2", 1, 1500, 333, 400)])
def test_single_packet(name, n_eff, S_win, start, chunk):
    rng = np.random.default_rng(7)
    psd, cfgt = F.CONFIGS[name]
    cfo = 0.9 * 2 * np.pi / (64 * psd[1])  # 0.9 subcarriers per DECT sample
    win, _ = F.sync_window(rng, O, name, S_win, [start], cfo)
    sc = O.sync_cfg(psd[0], psd[1], L=cfgt[4], M=cfgt[5], n_ant=cfgt[2], chunk_len=chunk)
    r = O.sync(sc, win)
    assert len(r) == 1
    _check_found(r[0], start, cfo, n_eff)
    rf = O.sync(sc, win, use_float=True)  # CPU-baseline (float) path takes the same decisions
    assert [(d["fine_64"], d["N_eff_TX"], d["coarse_local"]) for d in rf] == [(r[0]["fine_64"], n_eff, r[0]["coarse_local"])]


def test_two_packets_in_one_chunk_and_noise():
    rng = np.random.default_rng(9)
    cfo = -0.6 * 2 * np.pi / 64
    win, _ = F.sync_window(rng, O, "C2", 3000, [300, 1650], cfo)
    sc = O.sync_cfg(1, 1, n_ant=1, chunk_len=3000)
    r = O.sync(sc, win, max_reports=4)
    assert [d["fine_64"] for d in r] == [300, 1650]
    for d in r:
        _check_found(d, d["fine_64"], cfo, 1)
    assert r[1]["det_time"] >= r[0]["coarse_local"] + 2 * 112  # skip_after_peak
    noise, _ = F.sync_window(rng, O, "C2", 3000, [], 0.0)
    assert O.sync(sc, noise, max_reports=4) == []


def test_identity_resampler():
    """L = M = 1 (radio at the DECT rate): no resampling, search range +-16 b os."""
    rng = np.random.default_rng(5)
    cfo = 0.3 * 2 * np.pi / 64
    psd = F.CONFIGS["C2"][0]
    cf = O.cfg(1, 1, L=1, M=1)
    ps = O.psdef(*psd)
    sz = O.packet_sizes(ps)
    x, _ = O.tx(cf, ps, rng.integers(0, 256, 25, dtype=np.uint8),
                rng.integers(0, 256, (sz["G"] + 7) // 8, dtype=np.uint8), 720, phase_inc=cfo)
    win = np.zeros((1, 1400), np.complex64)
    win[0, 250:250 + 720] = x[0]
    win += 0.003 * (rng.standard_normal(win.shape) + 1j * rng.standard_normal(win.shape))
    sc = O.sync_cfg(1, 1, L=1, M=1, n_ant=1, chunk_len=1000)
    assert O.sync_geometry(sc)["xc_l"] == 16
    r = O.sync(sc, win)
    assert len(r) == 1
    _check_found(r[0], 250, cfo, 1)
