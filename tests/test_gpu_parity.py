"""GPU parity tests: libdnrp.so (HIP, gfx950) against the CPU oracle on identical inputs.

Tolerances:
  * TX IQ: relative L2 error per packet and antenna <= 1e-4 (float IQ), GI/tail exactly zero.
  * RX: int16 LLRs |delta| <= 1 LSB against the double-precision oracle (pre-quantisation float
    values agree to ~1e-5 relative; the +-1 covers rounding-boundary flips), with |mean delta| <= 0.01
    LSB and at most 1 % of the LLRs of a packet differing (tests/llr_gate.py), SNR reports within
    0.05 dB, STO within 1e-3 samples, RMS within 1e-4 relative, MIMO report exact.

Configurations (CASES): the bench configurations C2/C3/C4 plus every mode the reference RX
supports that the bench does not exercise — the loopback_simulator device class 1.1.1.A at every
MCS 0..7 (BPSK / QPSK / 16-QAM / 64-QAM map and demap, fix/mod.cpp:32-135) over SNR -2..20 dB,
MRC with 2 and 4 RX antennas (rx_synced.cpp:1204-1306), transmit diversity with 2 and 4 streams
(TM1 / TM5), closed-loop beamforming codebooks (TM3 / TM7), the chestim l-mode
(chestim_mode_lr = 0, rx_synced.cpp:1112-1163), the resampling ratios 40/27 and 1/1 and
os_min = 2 (phy_config.cpp:28-58, resampler.cpp:456-562), beta = 12 (768-point radix-3 FFT),
subslot packets (PacketLengthType 0).
"""
import numpy as np
import pytest

import llr_gate
import oracle_py as O
import phy_fixtures as F

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

CASES = F.PARITY_CASES
TX_CASES = {**F.PARITY_CASES, **F.TX_ONLY_CASES}


def _ctx(name, max_batch=8, stride=2):
    import dnrp
    ps, cf, lr, _, _ = TX_CASES[name]
    u_max, b_max, ntx, os_min, L, M = cf
    phy = dnrp.Phy(u_max, b_max, ntx, os_min, L, M, chestim_mode_lr=bool(lr), stride=stride, max_batch=max_batch)
    for nid in range(100, 106):
        phy.add_network_id(nid)
    return phy, dnrp.psdef(*ps), O.psdef(*ps), O.cfg(u_max, b_max, os_min, L, M, lr=lr, stride=stride)


def _tx_inputs(rng, n, sz):
    pcc = np.stack([O.pack_bits(F.random_bits(rng, 196)) for _ in range(n)])
    pdc = np.stack([O.pack_bits(F.random_bits(rng, sz["G"])) for _ in range(n)])
    assert pcc.shape == (n, 25) and pdc.shape == (n, (sz["G"] + 7) // 8)
    return pcc, pdc


def _gpu_tx(phy, ps, descs, pcc, pdc, S):
    dev = torch.device("cuda:0")
    n = len(descs)
    sz = phy.packet_sizes(ps)
    out = torch.empty((n, sz["N_TX"], S, 2), dtype=torch.float32, device=dev)
    out.fill_(7.0)  # poison: every sample must be written
    phy.tx_batch(ps, descs, torch.from_numpy(pcc).to(dev), torch.from_numpy(pdc).to(dev), out)
    phy.sync()
    return out.cpu().numpy().view(np.complex64)[..., 0]


def _check_tx(iq_gpu, ref, sz, S, n_tx_ref, tag):
    keep = sz["N_samples_packet_no_GI_os_rs"]
    scale = max(np.linalg.norm(ref[a, :keep]) for a in range(sz["N_TX"]))
    for a in range(sz["N_TX"]):
        nr = np.linalg.norm(ref[a, :keep])
        # antennas a codebook leaves silent (zero W row) are compared against the loudest antenna
        e = np.linalg.norm(iq_gpu[a, :keep] - ref[a, :keep]) / (nr if nr > 0 else scale)
        assert e <= 1e-4, (tag, a, e)
        assert np.all(iq_gpu[a, keep:] == 0), (tag, a)
    assert n_tx_ref == keep + (S - keep) * 5 // 100


@pytest.mark.parametrize("name", sorted(TX_CASES))
def test_tx_parity(name):
    import dnrp
    rng = np.random.default_rng(0xDEC7)
    phy, ps, ops, ocf = _ctx(name)
    cb = TX_CASES[name][4]
    sz = phy.packet_sizes(ps)
    S = sz["N_samples_packet_os_rs"]
    n = 3
    pcc, pdc = _tx_inputs(rng, n, sz)
    descs = []
    for i in range(n):
        cfo = (rng.uniform(-1.75, 1.75) * 2 * np.pi / sz["N_b_DFT_os"]) if i > 0 else 0.0
        descs.append(dnrp.TxDesc(cb, 100 + i, 1 + i % 2, 5, 1.0 if i != 1 else 0.7,
                                 float(rng.uniform(-3, 3)) if i == 2 else 0.0, cfo, 0))
    iq = _gpu_tx(phy, ps, descs, pcc, pdc, S)
    for i, d in enumerate(descs):
        ref, n_tx = O.tx(ocf, ops, pcc[i], pdc[i], S, codebook=cb, network_id=d.network_id,
                         plcf_type=d.plcf_type, gi=5, dac=float(np.float32(d.DAC_scale)),
                         phase=float(np.float32(d.iq_phase_rad)),
                         phase_inc=float(np.float32(d.iq_phase_increment_s2s_post_resampling_rad)))
        _check_tx(iq[i], ref, sz, S, n_tx, (name, i))


@pytest.mark.parametrize("name", sorted(TX_CASES))
@pytest.mark.parametrize("form", ["1", "2"])
def test_tx_parity_matrix_blocks(name, form, monkeypatch):
    """The streaming TX kernel's opt-in matrix-core polyphase blocks (DNRP_TX_MFMA=1: split-fp16
    v_mfma_f32_16x16x32_f16, polyphase.hpp mf_blocks; DNRP_TX_MFMA=2: f32 v_mfma_f32_16x16x4_f32) against
    the same oracle and tolerance; configurations outside the streaming kernel's geometry ignore the
    switch."""
    monkeypatch.setenv("DNRP_TX_MFMA", form)
    test_tx_parity(name)


@pytest.mark.parametrize("name", ["os2_C4", "u2_in_u8b16", "u1_in_u8b16"])
def test_tx_big_passes(name, monkeypatch):
    """N_b_DFT_os > 1024 (tx_big_sym_kernel + tx_big_resample_kernel through the DECT-rate scratch):
    DNRP_TX_BIG_CAP=1 shrinks the scratch cap so every packet runs in a pass of its own (big_batch = 1
    < n), with the packet-indexed arguments offset per pass -- first, middle and last packet at
    parity with the oracle."""
    monkeypatch.setenv("DNRP_TX_BIG_CAP", "1")
    test_tx_parity(name)


@pytest.mark.parametrize("name,cb", [("tm5_u2b4", 3), ("tm2_sm2", 1), ("C4", 0)])
def test_tx_optimal_scaling_dac(name, cb):
    """tx_meta_t::optimal_scaling_DAC (tx.cpp:582-592): W_t::scaling_factor_optimal_DAC instead of
    1/sqrt(non-zero W entries) -- 0.5 instead of 0.25 for N_TS = N_TX = 4 codebook 3, 1/sqrt2 instead
    of 1/2 for N_TS = N_TX = 2 codebook 1 (tests/golden/ref_literals.json)."""
    import dnrp
    rng = np.random.default_rng(0xDAC)
    phy, ps, ops, ocf = _ctx(name)
    sz = phy.packet_sizes(ps)
    S = sz["N_samples_packet_os_rs"]
    pcc, pdc = _tx_inputs(rng, 2, sz)
    descs = [dnrp.TxDesc(cb, 100 + i, 1 + i, 5, 1.0, 0.0, 0.0, i) for i in range(2)]  # std, optimal
    iq = _gpu_tx(phy, ps, descs, pcc, pdc, S)
    for i, d in enumerate(descs):
        ref, n_tx = O.tx(ocf, ops, pcc[i], pdc[i], S, codebook=cb, network_id=d.network_id, plcf_type=d.plcf_type,
                         optimal_dac=bool(i))
        _check_tx(iq[i], ref, sz, S, n_tx, (name, cb, i))
    ratio = np.linalg.norm(iq[1]) / np.linalg.norm(iq[0])  # different payloads, same power per packet
    want = dnrp.query_table("W_scaling_optimal_DAC", sz["N_TS"], sz["N_TX"], cb)[0] / \
        dnrp.query_table("W_scaling", sz["N_TS"], sz["N_TX"], cb)[0]
    assert abs(ratio / want - 1) < 0.05, (name, ratio, want)


def _rx_windows(rng, name, phy, ps, ops, ocf, snrs, cb=0):
    """Oracle-TX packets through a random N_RX x N_TX mixing, CFO and AWGN at per-packet SNRs.
    Returns the windows, sync reports (with a small residual CFO error), network IDs, PLCF types
    and the transmitted packed bits."""
    import dnrp
    sz = phy.packet_sizes(ps)
    S = sz["N_samples_packet_os_rs"]
    n_rx = phy.cfg.N_TX_max
    n = len(snrs)
    pcc, pdc = _tx_inputs(rng, n, sz)
    windows, reports, nids, types = [], [], [], []
    L, M = int(phy.cfg.L), int(phy.cfg.M)
    for i in range(n):
        nid, pt = 100 + (i % 6), 1 + i % 2
        iq_tx, _ = O.tx(ocf, ops, pcc[i], pdc[i], S, codebook=cb, network_id=nid, plcf_type=pt)
        off = int(rng.integers(0, 32))
        cfo_dect = rng.uniform(-1.75, 1.75) * 2 * np.pi / sz["N_b_DFT_os"]  # rad per DECT sample
        win = F.channel(rng, iq_tx, n_rx, S, off, cfo_dect * M / L, snrs[i])
        windows.append(win)
        est = -cfo_dect + rng.uniform(-0.02, 0.02) * 2 * np.pi / sz["N_b_DFT_os"]
        reports.append(dnrp.SyncReport(off, float(est), 0.0, ops[0], ops[1], sz["N_eff_TX"]))
        nids.append(nid)
        types.append(pt)
    return windows, reports, nids, types, pcc, pdc


def _oracle_rx(ocf, ops, win, rep, nid, pt):
    return O.rx(ocf, ops, win, rep.fine_peak_time, float(np.float32(rep.cfo_fractional_rad)), nid, pt)


def _check_rx(name, g_pcc, g_pdc, r1, r2, r):
    # max |delta| <= 1, |mean delta| and the fraction of nonzero deltas bounded (tests/llr_gate.py)
    llr_gate.check((name, "pcc"), g_pcc, r["pcc_llr"])
    llr_gate.check((name, "pdc"), g_pdc[: len(r["pdc_llr"])], r["pdc_llr"])
    if r1 is not None:
        assert abs(r1.snr_dB - r["snr_pcc"]) < 0.05, (name, r1.snr_dB, r["snr_pcc"])
        assert abs(r1.sto_fractional - r["sto"]) < 1e-3, (name, r1.sto_fractional, r["sto"])
        for a in range(len(r["rms"])):
            assert abs(r1.rms[a] - r["rms"][a]) <= 1e-4 * max(1.0, r["rms"][a]), (name, a)
    if r2 is not None:
        assert abs(r2.snr_dB - r["snr_pdc"]) < 0.05, (name, r2.snr_dB, r["snr_pdc"])
        # mimo_report_t (estimator_mimo.cpp): codebook recommendations exact; where the reference has
        # no result (8 antennas: estimator_mimo.cpp:180 asserts, the oracle flags MIMO_REF_UNDEFINED)
        # the product's defined "no recommendation" 0xFFFFFFFF is checked as a documented divergence
        assert r2.mimo_N_TS_other == r["mimo_N_TS_other"], name
        for g, o in ((r2.tm_3_7_beamforming_idx, r["mimo_idx"]),
                     (r2.tm_3_7_beamforming_reciprocal_idx, r["mimo_idx_reciprocal"])):
            assert g == (0xFFFFFFFF if o == O.MIMO_REF_UNDEFINED else o), (name, g, o)


@pytest.mark.parametrize("name", sorted(CASES))
def test_rx_parity(name, stride=2):
    _rx_parity(name, stride)


def _rx_parity(name, stride=2):
    """Runs one RX parity case; returns the context (its kernel timers, with DNRP_TIMING=1)."""
    import dnrp
    rng = np.random.default_rng(11)
    phy, ps, ops, ocf = _ctx(name, stride=stride)
    snrs, cb = CASES[name][3], CASES[name][4]
    sz = phy.packet_sizes(ps)
    S = sz["N_samples_packet_os_rs"]
    windows, reports, nids, types, _, pdc = _rx_windows(rng, name, phy, ps, ops, ocf, snrs, cb)
    n, n_rx = len(windows), phy.cfg.N_TX_max
    # packet 0's sync report carries an RMS for antenna 0 only: kept, the others estimated
    # (RX_SYNCED_PARAM_RMS_KEEP_VALUES_PROVIDED_BY_SYNC, rx_synced.cpp:620-655)
    reports[0].rms[0] = 0.123
    sync_rms = [[0.123] + [0.0] * 7] + [None] * (n - 1)
    dev = torch.device("cuda:0")
    iq = torch.from_numpy(np.stack(windows).view(np.float32).reshape(n, n_rx, S, 2)).to(dev)
    pcc_llr = torch.zeros((n, 196), dtype=torch.int16, device=dev)
    pdc_llr = torch.zeros((n, sz["G"]), dtype=torch.int16, device=dev)
    rep1 = phy.rx_pcc_batch(reports, iq, pcc_llr, want_report=True)
    rep2 = phy.rx_pdc_batch([dnrp.PdcReq(ps, i, nids[i], types[i]) for i in range(n)], iq, pdc_llr,
                            want_report=True)
    phy.sync()
    g_pcc, g_pdc = pcc_llr.cpu().numpy(), pdc_llr.cpu().numpy()
    for i in range(n):
        r = O.rx(ocf, ops, windows[i], reports[i].fine_peak_time, float(np.float32(reports[i].cfo_fractional_rad)),
                 nids[i], types[i], sync_rms=sync_rms[i])
        _check_rx((name, i), g_pcc[i], g_pdc[i], rep1[i], rep2[i], r)
        if i == 0:
            assert rep1[0].rms[0] == np.float32(0.123) and r["rms"][0] == np.float32(0.123)
        if snrs[i] >= 20.0:  # uncoded hard decisions well above the demapping noise floor
            bits = np.unpackbits(pdc[i])[: sz["G"]]
            assert np.mean(bits != (g_pdc[i] > 0)) < 2e-2, (name, i)
    return phy


@pytest.mark.parametrize("name,stride", [("tm5_u2b4", 1), ("tm5_u2b4", 3), ("C4", 1), ("C4", 3), ("mrc2_64qam", 3),
                                         ("C3", 1), ("tm1_txdiv2", 4)])
def test_rx_parity_stride(name, stride):
    """chestim_mode_lr_t_stride_default other than 2 (rx_synced.cpp:85,1097: the lr-mode interpolation
    event every `stride` symbols of a processing stage) against the oracle run with the same stride."""
    test_rx_parity(name, stride)


@pytest.mark.parametrize("name", ["C4", "C3", "tm5_u2b4", "mrc2_64qam", "mrc4_16qam", "lmode_C4", "lmode_txdiv2",
                                  "tm1_txdiv2", "tm3_codebook3", "subslot_tm5", "u2_in_u8b16"])
def test_rx_parity_fused(name, monkeypatch):
    """DNRP_RX_FUSED=1: the PDC phase through the fused receiver (rx_fused.hip: the DRS symbols' front end
    leaves zero-forced pilots, then one workgroup per (packet, symbol) transforms every antenna into LDS
    and equalises from there, no Y round trip) instead of Y + rx_cells -- same oracle and gates.
    Geometries outside the fused kernel (N_b_DFT_os != 1024) run the Y path either way."""
    _rx_parity_fused(name, 2, monkeypatch)


def _rx_parity_fused(name, stride, monkeypatch):
    monkeypatch.setenv("DNRP_RX_FUSED", "1")
    monkeypatch.setenv("DNRP_TIMING", "1")  # launch counts: the fused kernel ran exactly where it applies
    phy = _rx_parity(name, stride)
    ps = TX_CASES[name][0]
    import dnrp
    n_fused = phy.kernel_time_total("rx_fused")[1]
    if phy.packet_sizes(dnrp.psdef(*ps))["N_b_DFT_os"] == 1024:
        assert n_fused > 0, name
    else:
        assert n_fused == 0, name


@pytest.mark.parametrize("name,stride", [("C4", 1), ("tm5_u2b4", 3)])
def test_rx_parity_fused_stride(name, stride, monkeypatch):
    _rx_parity_fused(name, stride, monkeypatch)


EPOCH_CASES = ["C4", "C3", "C2", "tm5_u2b4", "mrc2_64qam", "mrc4_16qam", "lmode_C4", "lmode_txdiv2", "lmode_siso",
               "tm1_txdiv2", "tm3_codebook3", "tm7_codebook9", "subslot_tm5", "C1_mcs0", "u2_in_u8b16"]


def _rx_parity_epoch(name, stride, monkeypatch):
    """DNRP_RX_EPOCH=2: the PDC phase through the epoch receiver (rx_epoch.hip: DRS pass, SNR chain, then one
    workgroup per (packet, epoch) running the front end of the epoch's symbols and equalising them) instead
    of the batch-wide front end + rx_cells, for every geometry it supports (the default, 1, takes it with
    4+ RX antennas only) -- same oracle and gates. Geometries outside it (N_b_DFT_os != 1024) run the Y
    path; where it applies, the launch count proves it ran."""
    monkeypatch.setenv("DNRP_RX_EPOCH", "2")
    monkeypatch.setenv("DNRP_TIMING", "1")
    phy = _rx_parity(name, stride)
    import dnrp
    n_ep = phy.kernel_time_total("rx_epoch")[1]
    if phy.packet_sizes(dnrp.psdef(*TX_CASES[name][0]))["N_b_DFT_os"] == 1024:
        assert n_ep > 0, name
    else:
        assert n_ep == 0, name


@pytest.mark.parametrize("name", EPOCH_CASES)
def test_rx_parity_epoch(name, monkeypatch):
    _rx_parity_epoch(name, 2, monkeypatch)


@pytest.mark.parametrize("name,stride", [("C4", 1), ("C4", 3), ("tm5_u2b4", 3), ("C3", 1), ("tm1_txdiv2", 4)])
def test_rx_parity_epoch_stride(name, stride, monkeypatch):
    _rx_parity_epoch(name, stride, monkeypatch)


@pytest.mark.parametrize("name", ["C4", "C3", "C2", "tm5_u2b4", "mrc4_16qam", "lmode_C4", "tm1_txdiv2", "subslot_tm5"])
def test_rx_parity_ypath(name, monkeypatch):
    """DNRP_RX_EPOCH=0: the PDC phase through the batch-wide front end into Y and rx_cells (the path the
    epoch receiver replaced as the default) -- same oracle and gates, and no epoch launch."""
    monkeypatch.setenv("DNRP_RX_EPOCH", "0")
    monkeypatch.setenv("DNRP_TIMING", "1")
    phy = _rx_parity(name)
    assert phy.kernel_time_total("rx_epoch")[1] == 0, name


def test_rx_largest_cells_geometry(monkeypatch):
    """8 RX antennas x 4 transmit streams at b = 16 (TM5 into an N_TX_max = 8 context): the largest
    N_RX / NT / b of the cells kernel's LDS staging (pilot rows of 8 x 4 streams, both weight tables).
    The host states the staging size ("cells_lds_bytes"); the one outcome it implies is asserted:
    parity against the oracle when it fits one CU's 160 KiB, else DNRP_EUNSUPPORTED before any
    launch (never a device error)."""
    import dnrp
    name = "tm5_u8b16_rx8"
    spec = ((8, 16, 1, 1, 5, 8), (8, 16, 8, 1, 10, 9), 1, (30.0,), 0)
    monkeypatch.setitem(CASES, name, spec)
    monkeypatch.setitem(TX_CASES, name, spec)
    lds = int(dnrp.query_table("cells_lds_bytes", 8, 16, 16, 8, 4)[0])
    if lds <= 160 * 1024:
        _rx_parity(name)
    else:
        with pytest.raises(dnrp.DnrpError) as e:
            _rx_parity(name)
        assert e.value.code == -3, str(e.value)  # DNRP_EUNSUPPORTED


def test_rx_fused_growing_batch(monkeypatch):
    """DNRP_RX_FUSED=1 with a small PCC/PDC batch and then a larger one in the same context: the pilot
    buffer zd is reallocated (possibly at the same address) and its op-less interlace slot must be
    zeroed again (ctx.cpp zd_key includes the size) -- both batches at parity."""
    import dnrp
    monkeypatch.setenv("DNRP_RX_FUSED", "1")
    rng = np.random.default_rng(23)
    phy, ps, ops, ocf = _ctx("C4", max_batch=8)
    sz = phy.packet_sizes(ps)
    S, n_rx, dev = sz["N_samples_packet_os_rs"], phy.cfg.N_TX_max, torch.device("cuda:0")
    for n in (2, 8):
        windows, reports, nids, types, _, _ = _rx_windows(rng, "C4", phy, ps, ops, ocf, (30.0,) * n)
        iq = torch.from_numpy(np.stack(windows).view(np.float32).reshape(n, n_rx, S, 2)).to(dev)
        pcc_llr = torch.zeros((n, 196), dtype=torch.int16, device=dev)
        pdc_llr = torch.zeros((n, sz["G"]), dtype=torch.int16, device=dev)
        phy.rx_pcc_batch(reports, iq, pcc_llr)
        phy.rx_pdc_batch([dnrp.PdcReq(ps, i, nids[i], types[i]) for i in range(n)], iq, pdc_llr)
        phy.sync()
        for i in (0, n - 1):
            r = _oracle_rx(ocf, ops, windows[i], reports[i], nids[i], types[i])
            _check_rx(("grow", n, i), pcc_llr[i].cpu().numpy(), pdc_llr[i].cpu().numpy(), None, None, r)


@pytest.mark.parametrize("name", ["C4", "C3", "C2"])
def test_rx_parity_snr_from_y(name, monkeypatch):
    """DNRP_RX_SNR_FRONT=0: the DRS SNR sums gathered by rx_snr_kernel from Y instead of the front end's
    partial sums (rx_front.hpp rx_drs_partials) -- the same oracle and gates on both paths."""
    monkeypatch.setenv("DNRP_RX_SNR_FRONT", "0")
    test_rx_parity(name)


def test_rx_pdc_per_packet_requests():
    """One PCC batch of 8 packets with mixed transmission modes (N_eff_TX 1 / 2 / 4 in one call),
    then a PDC batch in which the MAC dropped 2 packets (continue_with_pdc = false) and the rest
    announce 3 different MCS and 2 PacketLengths, requested out of order
    (worker_tx_rx.cpp:166-201, rx_synced.cpp:325-436)."""
    import dnrp
    u_max, b_max, ntx, os_min, L, M = 2, 4, 4, 1, 10, 9
    phy = dnrp.Phy(u_max, b_max, ntx, os_min, L, M, max_batch=8)
    for nid in range(100, 106):
        phy.add_network_id(nid)
    ocf = O.cfg(u_max, b_max, os_min, L, M)
    # (tm, mcs, PacketLength) per packet
    kinds = [(0, 2, 1), (5, 4, 2), (1, 6, 1), (0, 4, 2), (5, 6, 1), (1, 2, 2), (0, 6, 1), (5, 2, 1)]
    rng = np.random.default_rng(5)
    S = max(phy.packet_sizes(dnrp.psdef(2, 4, 1, k[2], k[0], k[1]))["N_samples_packet_os_rs"] for k in kinds)
    windows, reports, meta = [], [], []
    for i, (tm, mcs, pl) in enumerate(kinds):
        ps = dnrp.psdef(2, 4, 1, pl, tm, mcs)
        ops = O.psdef(2, 4, 1, pl, tm, mcs)
        sz = phy.packet_sizes(ps)
        pcc, pdc = _tx_inputs(rng, 1, sz)
        nid, pt = 100 + i % 6, 1 + i % 2
        x, _ = O.tx(ocf, ops, pcc[0], pdc[0], sz["N_samples_packet_os_rs"], network_id=nid, plcf_type=pt)
        off = int(rng.integers(0, 32))
        cfo_dect = rng.uniform(-1.5, 1.5) * 2 * np.pi / sz["N_b_DFT_os"]
        win = F.channel(rng, x, ntx, S, off, cfo_dect * M / L, 25.0)
        windows.append(win)
        reports.append(dnrp.SyncReport(off, float(-cfo_dect), 0.0, 2, 4, sz["N_eff_TX"]))
        meta.append((ps, ops, nid, pt, sz))
    dev = torch.device("cuda:0")
    iq = torch.from_numpy(np.stack(windows).view(np.float32).reshape(8, ntx, S, 2)).to(dev)
    pcc_llr = torch.zeros((8, 196), dtype=torch.int16, device=dev)
    phy.rx_pcc_batch(reports, iq, pcc_llr)
    order = [6, 1, 3, 0, 7, 4]  # packets 2 and 5 rejected by the MAC
    reqs = [dnrp.PdcReq(meta[i][0], i, meta[i][2], meta[i][3]) for i in order]
    g_max = max(meta[i][4]["G"] for i in order)
    pdc_llr = torch.full((len(order), g_max), 12345, dtype=torch.int16, device=dev)
    rep = phy.rx_pdc_batch(reqs, iq, pdc_llr, want_report=True)
    phy.sync()
    g_pcc, g_pdc = pcc_llr.cpu().numpy(), pdc_llr.cpu().numpy()
    assert len({(meta[i][4]["N_bps"]) for i in order}) == 3
    for r_idx, i in enumerate(order):
        ps, ops, nid, pt, sz = meta[i]
        r = _oracle_rx(ocf, ops, windows[i], reports[i], nid, pt)
        _check_rx(("mixed", i), g_pcc[i], g_pdc[r_idx], None, rep[r_idx], r)
        assert np.all(g_pdc[r_idx, sz["G"]:] == 12345), "LLRs past G untouched"


def test_rx_pdc_request_errors():
    import dnrp
    phy, ps, ops, ocf = _ctx("C2")
    sz = phy.packet_sizes(ps)
    S = sz["N_samples_packet_os_rs"]
    dev = torch.device("cuda:0")
    iq = torch.zeros((2, 1, S, 2), dtype=torch.float32, device=dev)
    pcc_llr = torch.zeros((2, 196), dtype=torch.int16, device=dev)
    pdc_llr = torch.zeros((2, sz["G"]), dtype=torch.int16, device=dev)
    with pytest.raises(dnrp.DnrpError) as e:  # no PCC batch yet
        phy.rx_pdc_batch([dnrp.PdcReq(ps, 0, 100, 1)], iq, pdc_llr)
    assert e.value.code == -7
    phy.rx_pcc_batch([dnrp.SyncReport(0, 0.0, 0.0, 1, 1, 1)] * 2, iq, pcc_llr)
    for reqs in ([dnrp.PdcReq(ps, 2, 100, 1)],                                       # slot out of range
                 [dnrp.PdcReq(ps, 1, 100, 1), dnrp.PdcReq(ps, 1, 100, 1)],          # slot twice
                 [dnrp.PdcReq(dnrp.psdef(1, 1, 1, 1, 1, 1), 0, 100, 1)]):           # N_eff_TX != sync report
        with pytest.raises(dnrp.DnrpError) as e:
            phy.rx_pdc_batch(reqs, iq, pdc_llr)
        assert e.value.code in (-1, -3), e.value.code
    with pytest.raises(dnrp.DnrpError) as e:
        phy.rx_pdc_batch([dnrp.PdcReq(ps, 0, 999, 1)], iq, pdc_llr)
    assert e.value.code == -6
    # the PDC symbols come from the PCC call's windows: another buffer is a state error
    other = iq.clone()
    with pytest.raises(dnrp.DnrpError) as e:
        phy.rx_pdc_batch([dnrp.PdcReq(ps, 0, 100, 1)], other, pdc_llr)
    assert e.value.code == -7


def test_rx_empty_chunk_then_parity():
    """A chunk of noise only: sync finds no packet, the PCC batch is empty (n = 0) and so is the PDC
    batch (m = 0) -- both return OK (no job without a packet, worker_sync.cpp:170-190), also when
    the empty PDC batch follows an empty PCC batch; then a normal batch in the same context is at
    parity."""
    import dnrp
    rng = np.random.default_rng(31)
    phy, ps, ops, ocf = _ctx("C2")
    sz = phy.packet_sizes(ps)
    S = sz["N_samples_packet_os_rs"]
    dev = torch.device("cuda:0")
    noise = (rng.normal(size=(4, 1, S)) + 1j * rng.normal(size=(4, 1, S))).astype(np.complex64) * 0.01
    iq0 = torch.from_numpy(noise.view(np.float32).reshape(4, 1, S, 2)).to(dev)
    sc = dnrp.SyncCfg(1, 1, 1, S * 7 // 8, 1)
    res, cnt = phy.rx_sync_batch(sc, iq0, 4, S, S, S)
    phy.sync()
    assert int(np.asarray(cnt[:4]).sum()) == 0
    reps = dnrp.found_reports(res, cnt[:4])
    assert len(reps) == 0
    pcc_llr = torch.zeros((4, 196), dtype=torch.int16, device=dev)
    pdc_llr = torch.zeros((4, sz["G"]), dtype=torch.int16, device=dev)
    for _ in range(2):
        phy.rx_pcc_batch(reps, iq0, pcc_llr)
        phy.rx_pdc_batch([], iq0, pdc_llr)
    phy.sync()
    windows, reports, nids, types, _, _ = _rx_windows(rng, "C2", phy, ps, ops, ocf, (20.0, 30.0))
    iq = torch.from_numpy(np.stack(windows).view(np.float32).reshape(2, 1, S, 2)).to(dev)
    phy.rx_pcc_batch(reports, iq, pcc_llr)
    phy.rx_pdc_batch([dnrp.PdcReq(ps, i, nids[i], types[i]) for i in range(2)], iq, pdc_llr)
    phy.sync()
    for i in range(2):
        r = _oracle_rx(ocf, ops, windows[i], reports[i], nids[i], types[i])
        _check_rx(("after_empty", i), pcc_llr[i].cpu().numpy(), pdc_llr[i].cpu().numpy(), None, None, r)


def test_rx_window_index_checked_by_c_abi():
    """dnrp_rx_pcc_batch range-checks sync_report.window against n_windows in C (a zeroed or garbage
    report must not make the kernels read past iq_in), bypassing the Python-side check."""
    import ctypes as C
    import dnrp
    phy, ps, ops, ocf = _ctx("C2")
    S = phy.packet_sizes(ps)["N_samples_packet_os_rs"]
    dev = torch.device("cuda:0")
    iq = torch.zeros((2, 1, S, 2), dtype=torch.float32, device=dev)
    pcc_llr = torch.zeros((2, 196), dtype=torch.int16, device=dev)
    for win in (2, 0xFFFFFFFE):
        reps = (dnrp.SyncReport * 2)(dnrp.SyncReport(0, 0.0, 0.0, 1, 1, 1, window=0),
                                     dnrp.SyncReport(0, 0.0, 0.0, 1, 1, 1, window=win))
        rc = dnrp.lib().dnrp_rx_pcc_batch(phy._ctx, 2, C.cast(reps, C.c_void_p), C.c_void_p(iq.data_ptr()), 2, S,
                                          C.c_void_p(pcc_llr.data_ptr()), None, None)
        assert rc == -1, (win, rc)
    reps = (dnrp.SyncReport * 2)(dnrp.SyncReport(0, 0.0, 0.0, 1, 1, 1, window=0),
                                 dnrp.SyncReport(0, 0.0, 0.0, 1, 1, 1, window=1))
    assert dnrp.lib().dnrp_rx_pcc_batch(phy._ctx, 2, C.cast(reps, C.c_void_p), C.c_void_p(iq.data_ptr()), 2, S,
                                        C.c_void_p(pcc_llr.data_ptr()), None, None) == 0
    phy.sync()


# Spatial multiplexing with the MMSE receiver (opt-in DNRP_RX_MODE_SM_MMSE; the reference RX has no
# AxA MIMO, rx_synced.cpp:1331-1333, so the oracle's MMSE restatement is parity-unpinned):
# name: psdef, ctx cfg, SNRs
SM_CASES = {
    "tm6_u2b4_16qam": ((2, 4, 1, 2, 6, 4), (2, 4, 4, 1, 10, 9), (20.0, 30.0)),
    "tm6_u8b16_64qam": ((8, 16, 1, 1, 6, 6), (8, 16, 4, 1, 10, 9), (30.0,)),
    "tm6_u8b16_256qam": ((8, 16, 1, 1, 6, 8), (8, 16, 4, 1, 10, 9), (40.0,)),
    "tm2_sm2_u2b2": ((2, 2, 1, 2, 2, 6), (2, 2, 2, 1, 10, 9), (15.0, 30.0)),
    "tm4_cl_sm2_u1b4": ((1, 4, 1, 2, 4, 3), (1, 4, 2, 1, 10, 9), (25.0,)),
    # 8 RX antennas: rx_cells_kernel<8, 4, true> and <8, 2, true>
    "tm6_u2b4_8rx_16qam": ((2, 4, 1, 2, 6, 4), (2, 4, 8, 1, 10, 9), (25.0,)),
    "tm2_sm2_u2b2_8rx": ((2, 2, 1, 2, 2, 6), (2, 2, 8, 1, 10, 9), (20.0,)),
}


@pytest.mark.parametrize("name", sorted(SM_CASES))
def test_rx_sm_mmse_parity(name):
    """GPU MMSE (rx_cells_kernel<., ., true>) vs the oracle's double-precision MMSE on the same windows:
    int16 LLRs within 1 LSB, SNR report within 0.05 dB; without the opt-in the PDC request is
    DNRP_EUNSUPPORTED, as the reference's receiver declines N_SS > 1."""
    import dnrp
    rng = np.random.default_rng(17)
    ps_t, cf, snrs = SM_CASES[name]
    u_max, b_max, ntx, os_min, L, M = cf
    phy = dnrp.Phy(u_max, b_max, ntx, os_min, L, M, max_batch=4)
    for nid in range(100, 106):
        phy.add_network_id(nid)
    ps, ops, ocf = dnrp.psdef(*ps_t), O.psdef(*ps_t), O.cfg(u_max, b_max, os_min, L, M)
    sz = phy.packet_sizes(ps)
    assert sz["N_SS"] > 1
    S = sz["N_samples_packet_os_rs"]
    windows, reports, nids, types, _, pdc = _rx_windows(rng, name, phy, ps, ops, ocf, snrs)
    n = len(windows)
    dev = torch.device("cuda:0")
    iq = torch.from_numpy(np.stack(windows).view(np.float32).reshape(n, ntx, S, 2)).to(dev)
    pcc_llr = torch.zeros((n, 196), dtype=torch.int16, device=dev)
    pdc_llr = torch.zeros((n, sz["G"]), dtype=torch.int16, device=dev)
    reqs = [dnrp.PdcReq(ps, i, nids[i], types[i]) for i in range(n)]
    phy.rx_pcc_batch(reports, iq, pcc_llr)
    with pytest.raises(dnrp.DnrpError) as e:  # the reference receiver's behaviour by default
        phy.rx_pdc_batch(reqs, iq, pdc_llr)
    assert e.value.code == -3
    phy.set_rx_mode(phy.RX_MODE_SM_MMSE)
    rep1 = phy.rx_pcc_batch(reports, iq, pcc_llr, want_report=True)
    rep2 = phy.rx_pdc_batch(reqs, iq, pdc_llr, want_report=True)
    phy.sync()
    g_pcc, g_pdc = pcc_llr.cpu().numpy(), pdc_llr.cpu().numpy()
    for i in range(n):
        r = O.rx(ocf, ops, windows[i], reports[i].fine_peak_time, float(np.float32(reports[i].cfo_fractional_rad)),
                 nids[i], types[i], sm_mmse=True)
        _check_rx((name, i), g_pcc[i], g_pdc[i], rep1[i], None, r)
        assert abs(rep2[i].snr_dB - r["snr_pdc"]) < 0.05, (name, i)
        if snrs[i] >= 30.0 and sz["N_bps"] <= 4:  # uncoded decisions; random flat H can be ill-conditioned
            bits = np.unpackbits(pdc[i])[: sz["G"]]
            assert np.mean(bits != (g_pdc[i] > 0)) < 5e-2, (name, i, np.mean(bits != (g_pdc[i] > 0)))


def test_rx_tm10_unsupported():
    """N_eff_TX = 8 (device class 8.16.8.A): the reference receiver aborts on its l-mode LUT at the
    TS 4-7 DRS symbol; the boundary returns DNRP_EUNSUPPORTED instead of output."""
    import dnrp
    phy = dnrp.Phy(8, 16, 8, 1, 10, 9, max_batch=2)
    ps = dnrp.psdef(8, 16, 1, 1, 10, 8)
    S = phy.packet_sizes(ps)["N_samples_packet_os_rs"]
    dev = torch.device("cuda:0")
    iq = torch.zeros((1, 8, S, 2), dtype=torch.float32, device=dev)
    pcc_llr = torch.zeros((1, 196), dtype=torch.int16, device=dev)
    with pytest.raises(dnrp.DnrpError) as e:
        phy.rx_pcc_batch([dnrp.SyncReport(0, 0.0, 0.0, 8, 16, 8)], iq, pcc_llr)
    assert e.value.code == -3


def test_rx_negative_fine_peak():
    """A sync report whose packet starts before the window (fine_peak_time < 0): the samples before
    the window read as zero history, never memory before the window row."""
    import dnrp
    rng = np.random.default_rng(3)
    phy, ps, ops, ocf = _ctx("C2")
    sz = phy.packet_sizes(ps)
    S = sz["N_samples_packet_os_rs"]
    pcc, pdc = _tx_inputs(rng, 1, sz)
    x, _ = O.tx(ocf, ops, pcc[0], pdc[0], S, network_id=100, plcf_type=1)
    win = F.channel(rng, x, 1, S, 0, 0.0, 30.0)
    shift = 3
    cut = np.zeros_like(win)
    cut[:, : S - shift] = win[:, shift:]
    dev = torch.device("cuda:0")
    # two windows: a poisoned one in front makes a read before window 1 visible
    both = np.stack([np.full_like(cut, 1e6 + 1e6j), cut])
    iq = torch.from_numpy(both.view(np.float32).reshape(2, 1, S, 2)).to(dev)
    rep = [dnrp.SyncReport(0, 0.0, 0.0, 1, 1, 1), dnrp.SyncReport(-shift, 0.0, 0.0, 1, 1, 1)]
    pcc_llr = torch.zeros((2, 196), dtype=torch.int16, device=dev)
    pdc_llr = torch.zeros((1, sz["G"]), dtype=torch.int16, device=dev)
    phy.rx_pcc_batch(rep, iq, pcc_llr)
    phy.rx_pdc_batch([dnrp.PdcReq(ps, 1, 100, 1)], iq, pdc_llr)
    phy.sync()
    r = O.rx(ocf, ops, cut, -shift, 0.0, 100, 1)
    _check_rx("neg_peak", pcc_llr[1].cpu().numpy(), pdc_llr[0].cpu().numpy(), None, None, r)


@pytest.mark.parametrize("name,n", [("C4", 4096), ("C3", 8192), ("C4", 16384)])
def test_full_chunk_edges(name, n):
    _full_chunk_edges(name, n)


def test_rx_epoch_default_geometries(monkeypatch):
    """The default (DNRP_RX_EPOCH unset) takes the epoch receiver with 4 RX antennas (C4) and the Y path for
    SISO (C3), as measured."""
    monkeypatch.delenv("DNRP_RX_EPOCH", raising=False)
    monkeypatch.setenv("DNRP_TIMING", "1")
    assert _rx_parity("C4").kernel_time_total("rx_epoch")[1] > 0
    assert _rx_parity("C3").kernel_time_total("rx_epoch")[1] == 0


@pytest.mark.parametrize("name,n", [("C4", 16384), ("C3", 8192)])
def test_full_chunk_edges_ypath(name, n, monkeypatch):
    """The bench chunk through the Y path (DNRP_RX_EPOCH=0): grid and Y offsets past 2^32."""
    monkeypatch.setenv("DNRP_RX_EPOCH", "0")
    _full_chunk_edges(name, n)


def _full_chunk_edges(name, n):
    """A full bench chunk (C4: 4096 packets, C3: 8192, and the bench's C4 chunk of 16384 packets, whose
    window and Y offsets pass 2^32 float2 elements; max_batch = chunk): TX and RX of the first, middle
    and last packet compared with the oracle (rx_synced.cpp:325-436), chunk-boundary indexing included."""
    import dnrp
    import math
    phy, ps, ops, ocf = _ctx(name, max_batch=n)
    sz = phy.packet_sizes(ps)
    n_ant = sz["N_TX"]
    S, G = sz["N_samples_packet_os_rs"], sz["G"]
    dev = torch.device("cuda:0")
    gen = torch.Generator(device=dev)
    gen.manual_seed(7)
    pcc_d = torch.randint(0, 256, (n, 25), dtype=torch.uint8, device=dev, generator=gen)
    pdc_d = torch.randint(0, 256, (n, (G + 7) // 8), dtype=torch.uint8, device=dev, generator=gen)
    rng = np.random.default_rng(9)
    cfo_dect = rng.uniform(-1.75, 1.75, n) * 2 * math.pi / sz["N_b_DFT_os"]
    descs = [dnrp.TxDesc(0, 100 + i % 6, 1 + i % 2, 5, 1.0, 0.0, float(cfo_dect[i] * 9 / 10), 0) for i in range(n)]
    tx = torch.empty((n, n_ant, S, 2), dtype=torch.float32, device=dev)
    phy.tx_batch(ps, descs, pcc_d, pdc_d, tx)
    phy.sync()
    probe = [0, n // 2 - 1, n - 1]
    pcc_h, pdc_h = pcc_d.cpu().numpy(), pdc_d.cpu().numpy()
    for i in probe:
        ref, n_tx = O.tx(ocf, ops, pcc_h[i], pdc_h[i], S, network_id=100 + i % 6, plcf_type=1 + i % 2,
                         phase_inc=float(np.float32(descs[i].iq_phase_increment_s2s_post_resampling_rad)))
        _check_tx(tx[i].cpu().numpy().view(np.complex64)[..., 0], ref, sz, S, n_tx, (name, i))
    # channel on the device: per-packet N x N mixing + AWGN, in place into the windows
    rx = torch.empty_like(tx)
    with torch.no_grad():
        for c0 in range(0, n, 256):
            x = torch.view_as_complex(tx[c0:c0 + 256])
            H = torch.complex(torch.randn(x.shape[0], n_ant, n_ant, device=dev, generator=gen),
                              torch.randn(x.shape[0], n_ant, n_ant, device=dev, generator=gen)) / math.sqrt(2 * n_ant)
            y = torch.einsum("brt,bts->brs", H, x)
            y = y + 0.003 * torch.complex(torch.randn(y.shape, device=dev, generator=gen),
                                          torch.randn(y.shape, device=dev, generator=gen))
            rx[c0:c0 + 256] = torch.view_as_real(y)
            del x, y
    del tx
    reps = [dnrp.SyncReport(0, float(-cfo_dect[i]), 0.0, 8, 16, sz["N_eff_TX"]) for i in range(n)]
    pcc_llr = torch.zeros((n, 196), dtype=torch.int16, device=dev)
    pdc_llr = torch.zeros((n, G), dtype=torch.int16, device=dev)
    phy.rx_pcc_batch(reps, rx, pcc_llr)
    phy.rx_pdc_batch([dnrp.PdcReq(ps, i, 100 + i % 6, 1 + i % 2) for i in range(n)], rx, pdc_llr)
    phy.sync()
    for i in probe:
        win = rx[i].cpu().numpy().view(np.complex64)[..., 0]
        r = O.rx(ocf, ops, win, 0, float(np.float32(-cfo_dect[i])), 100 + i % 6, 1 + i % 2)
        _check_rx((name, i), pcc_llr[i].cpu().numpy(), pdc_llr[i].cpu().numpy(), None, None, r)
