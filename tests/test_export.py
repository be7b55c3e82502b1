"""Host-only JSON export and TX length (dnrp_tx_transmit_length, dnrp_tx_packet_json,
dnrp_rx_packet_json) in the reference's formats (tx.cpp:316-427, worker_tx_rx.cpp:354-396,
tx.cpp:555-566). No GPU: the IQ written is the oracle TX's."""
import json
import os
import sys

import numpy as np

import oracle_py as O
import phy_fixtures as F

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "dect-nr-plus-sdr_amd"))


def test_transmit_length_c3():
    import dnrp
    ps = dnrp.psdef(8, 16, 1, 1, 0, 8)
    # SURVEY.md §8(a) A1 (compiled reference geometry): no-GI 99840 + 5 % of the 2560-sample GI
    assert dnrp.tx_transmit_length(ps, 5, 8, 16) == 99968
    assert dnrp.tx_transmit_length(ps, 0, 8, 16) == 99840
    assert dnrp.tx_transmit_length(ps, 100, 8, 16) == 102400


def test_tx_packet_json(tmp_path):
    import dnrp
    psd, cft = F.CONFIGS["C2"]
    cf, ops = O.cfg(*cft[:2], os_min=cft[3], L=cft[4], M=cft[5]), O.psdef(*psd)
    sz = O.packet_sizes(ops)
    rng = np.random.default_rng(3)
    pcc = rng.integers(0, 256, 25, dtype=np.uint8)
    pdc = rng.integers(0, 256, (sz["G"] + 7) // 8, dtype=np.uint8)
    S = O.dims(cf, ops)["N_packet_os_rs"]
    x, _ = O.tx(cf, ops, pcc, pdc, S, network_id=101, plcf_type=2)
    desc = dnrp.TxDesc(0, 101, 2, 5, 1.0, 0.25, 0.001, 0)
    path = tmp_path / "tx_packet_0000000000"
    dnrp.tx_packet_json(path, dnrp.psdef(*psd), desc, pcc, pdc, x.astype(np.complex64), *cft[:3], os_min=cft[3],
                        L=cft[4], M=cft[5], tx_order_id=7, tx_time_64=123456789)
    j = json.loads(path.read_text())
    n_tr = dnrp.tx_transmit_length(dnrp.psdef(*psd), 5, *cft[:2])
    assert (j["u"], j["b"], j["PacketLengthType"], j["PacketLength"], j["tm_mode"], j["mcs_index"]) == tuple(psd)
    assert j["Z"] == 6144 and j["PLCF_type"] == 2 and j["network_id"] == 101 and j["oversampling"] == 1
    assert j["N_samples_transmit_os_rs"] == n_tr and j["N_samples_packet_no_GI_os_rs"] <= n_tr
    assert j["tx_descriptor"] == {"tx_order_id": 7, "tx_time_64": 123456789}
    assert j["tx_meta"]["GI_percentage"] == 5 and abs(j["tx_meta"]["iq_phase_rad"] - 0.25) < 1e-7
    assert j["data"]["binary"]["PCC"] == list(np.unpackbits(pcc)[:196])
    assert j["data"]["binary"]["PDC"] == list(np.unpackbits(pdc)[: sz["G"]])
    re = np.array(j["data"]["IQ"]["real"], np.float32)
    im = np.array(j["data"]["IQ"]["imag"], np.float32)
    xs = x.astype(np.complex64)[:, :n_tr].reshape(-1)  # antenna streams concatenated
    assert np.array_equal(re, xs.real) and np.array_equal(im, xs.imag)
    r = j["resampling"]
    assert (r["L"], r["M"], r["oversampling_minimum"]) == (10, 9, 1) and r["samp_rate"] == 1920000
    assert abs(r["f_pass_norm"] - 0.48) < 1e-7 and r["stopband_attenuation_dB"] == 14


def test_rx_packet_json(tmp_path):
    import dnrp
    res = np.zeros(1, dnrp.SYNC_RESULT_DTYPE)
    res["found"], res["u"], res["b"], res["N_eff_TX"] = 1, 8, 16, 4
    res["fine_peak_time"], res["coarse_peak_time"] = 10 ** 12 + 5, 10 ** 12
    res["rms_array"][0, :4] = [0.1, 0.2, 0.3, 0.4]
    res["cfo_fractional_rad"] = -0.0125
    pcc = dnrp.PccReport(21.5, -0.0124, 0.3)
    pdc = dnrp.PdcReport(22.25, 4, 4, 3, 1)
    path = tmp_path / "rx.json"
    dnrp.rx_packet_json(path, res[0], 8, 16, 4, 8, pcc, pdc, worker_id=2)
    j = json.loads(path.read_text())
    s = j["PHY"]["sync_report"]
    assert j["worker_id"] == 2 and j["RADIO"]["samp_rate"] == 245760000 and j["RADIO"]["N_TX_min"] == 4
    assert s["fine_peak_time"] == 10 ** 12 + 5 and s["coarse_peak_time"] == 10 ** 12 and s["N_eff_TX"] == 4
    # %.9g: every float round-trips exactly through the text
    assert np.array_equal(np.array(s["rms_array"], np.float32), np.array([0.1, 0.2, 0.3, 0.4], np.float32))
    assert abs(s["cfo_f"] + 0.0125) < 1e-9 and abs(s["sto_fractional"] - 0.3) < 1e-7
    assert j["PHY"]["rx_synced"] == {"snr": 22.25, "mcs": 8}
