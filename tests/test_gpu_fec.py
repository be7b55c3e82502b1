"""End-to-end loopback with channel coding (SURVEY.md §8(f) row 1, C1's purpose): PLCF and transport
blocks are FEC-encoded on the host (dnrp.fec <- fec_t::encode_plcf / encode_tb), transmitted by the
GPU TX (dnrp_tx_batch), passed through a random MIMO channel with CFO and AWGN, demodulated by the
GPU RX (dnrp_rx_pcc_batch / dnrp_rx_pdc_batch) and decoded on the host (fec_t::decode_plcf_test /
decode_tb), as worker_tx_rx_t does per packet (worker_tx_rx.cpp:126-201). Checks: every PLCF and
transport block passes its CRC with the transmitted contents at SNRs well above threshold, the
closed-loop/beamforming CRC mask is recovered, and at an SNR far below threshold every CRC fails
(no false passes) — for the GPU LLRs and for the oracle RX's LLRs of the same windows alike."""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
import oracle_py as O
import phy_fixtures as PF

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

# (psdef u, b, PacketLengthType, PacketLength, tm, mcs), (u_max, b_max, N_TX, os_min, L, M)
LOOPS = {
    "C2_siso_mcs1": ((1, 1, 1, 1, 0, 1), (1, 1, 1, 1, 10, 9)),
    "1.1.1.A_mcs4": ((1, 1, 1, 2, 0, 4), (1, 1, 1, 1, 10, 9)),
    "u2b4_tm5_mcs6": ((2, 4, 1, 1, 5, 6), (2, 4, 4, 1, 10, 9)),
    "u2b4_mrc2_mcs3": ((2, 4, 1, 2, 0, 3), (2, 4, 2, 1, 10, 9)),
    # spatial multiplexing, MMSE receiver (opt-in, DNRP_RX_MODE_SM_MMSE; not in the reference RX)
    "u2b4_tm6_sm4_mcs4": ((2, 4, 1, 2, 6, 4), (2, 4, 4, 1, 10, 9)),
    "u8b16_tm6_sm4_mcs4": ((8, 16, 1, 1, 6, 4), (8, 16, 4, 1, 10, 9)),
    "u2b2_tm2_sm2_mcs6": ((2, 2, 1, 2, 2, 6), (2, 2, 2, 1, 10, 9)),
}
SM_TM = (2, 4, 6, 8, 9)  # transmission modes with N_SS > 1


def _loop(name, snr_db, n=4, seed=1):
    import dnrp
    import dnrp.fec as FE
    ps_t, cf = LOOPS[name]
    u_max, b_max, ntx, os_min, L, M = cf
    phy = dnrp.Phy(u_max, b_max, ntx, os_min, L, M, max_batch=n)
    for nid in range(100, 106):
        phy.add_network_id(nid)
    sm = ps_t[4] in SM_TM
    if sm:
        phy.set_rx_mode(phy.RX_MODE_SM_MMSE)
    ps = dnrp.psdef(*ps_t)
    sz = phy.packet_sizes(ps)
    S = sz["N_samples_packet_os_rs"]
    rng = np.random.default_rng(seed)
    plcf_types = [1 + i % 2 for i in range(n)]
    plcfs = [rng.integers(0, 256, 5 * t, dtype=np.uint8) for t in plcf_types]
    masks = [(i % 2, (i // 2) % 2) for i in range(n)]
    tbs = [rng.integers(0, 256, sz["N_TB_bits"] // 8, dtype=np.uint8) for _ in range(n)]
    fcfg = FE.fec_cfg(sz["N_TB_bits"], sz["N_bps"], sz["G"], Z=6144)
    assert sz["N_TB_bits"] % 8 == 0
    pcc = np.stack([FE.pcc_encode(plcfs[i], plcf_types[i], *masks[i]) for i in range(n)])
    pdc = np.stack([FE.pdc_encode(fcfg, tbs[i]) for i in range(n)])
    dev = torch.device("cuda:0")
    # the GPU encoder produces the same d-bits (dnrp_pdc_encode_batch); TX from its output
    pdc_dev = torch.zeros((n, pdc.shape[1]), dtype=torch.uint8, device=dev)
    FE.pdc_encode_batch(phy, [fcfg] * n, torch.from_numpy(np.stack(tbs)).to(dev), pdc_dev)
    assert (pdc_dev.cpu().numpy() == pdc).all(), name
    descs = [dnrp.TxDesc(0, 100 + i, plcf_types[i], 5, 1.0, 0.0, 0.0, 0) for i in range(n)]
    out = torch.empty((n, sz["N_TX"], S, 2), dtype=torch.float32, device=dev)
    phy.tx_batch(ps, descs, torch.from_numpy(pcc).to(dev), pdc_dev, out)
    phy.sync()
    iq_tx = out.cpu().numpy().view(np.complex64)[..., 0]
    windows, reports = [], []
    for i in range(n):
        off = int(rng.integers(0, 32))
        cfo = rng.uniform(-1.5, 1.5) * 2 * np.pi / sz["N_b_DFT_os"]
        H = None
        if sm:  # spatial multiplexing: a random channel of condition number 2.5 (U diag V^H)
            q = lambda: np.linalg.qr(rng.standard_normal((ntx, ntx)) + 1j * rng.standard_normal((ntx, ntx)))[0]
            H = (q() @ np.diag(np.linspace(1.0, 0.4, ntx)) @ q().conj().T).astype(np.complex64)
        windows.append(PF.channel(rng, iq_tx[i], ntx, S, off, cfo * M / L, snr_db, H=H))
        reports.append(dnrp.SyncReport(off, float(-cfo), 0.0, ps_t[0], ps_t[1], sz["N_eff_TX"]))
    iq = torch.from_numpy(np.stack(windows).view(np.float32).reshape(n, ntx, S, 2)).to(dev)
    pcc_llr = torch.zeros((n, 196), dtype=torch.int16, device=dev)
    pdc_llr = torch.zeros((n, sz["G"]), dtype=torch.int16, device=dev)
    phy.rx_pcc_batch(reports, iq, pcc_llr)
    phy.rx_pdc_batch([dnrp.PdcReq(ps, i, 100 + i, plcf_types[i]) for i in range(n)], iq, pdc_llr)
    phy.sync()
    g_pcc, g_pdc = pcc_llr.cpu().numpy(), pdc_llr.cpu().numpy()
    # GPU turbo decoding of the GPU LLRs (dnrp_pdc_decode_batch)
    tb_dev = torch.zeros((n, sz["N_TB_bits"] // 8 + 3), dtype=torch.uint8, device=dev)
    g_ok, _ = FE.pdc_decode_batch(phy, [fcfg] * n, pdc_llr, tb_dev)
    g_tb = tb_dev.cpu().numpy()
    plcf_dev = torch.zeros((n, 10), dtype=torch.uint8, device=dev)
    g_res, _ = FE.pcc_decode_batch(phy, plcf_types, pcc_llr, plcf_dev)  # dnrp_pcc_decode_batch
    g_plcf = plcf_dev.cpu().numpy()
    ocf = O.cfg(u_max, b_max, os_min, L, M)
    ops = O.psdef(*ps_t)
    res = []
    for i in range(n):
        r = O.rx(ocf, ops, windows[i], reports[i].fine_peak_time, float(np.float32(reports[i].cfo_fractional_rad)),
                 100 + i, plcf_types[i], sm_mmse=sm)
        for src, lp, ld in (("gpu", g_pcc[i], g_pdc[i]), ("oracle", r["pcc_llr"], r["pdc_llr"])):
            ok_c, got_plcf, cl, bf, _ = FE.pcc_decode(lp, plcf_types[i])
            ok_d, got_tb, _ = FE.pdc_decode(fcfg, ld)
            res.append((src, i, ok_c, ok_c and (got_plcf == plcfs[i]).all() and (cl, bf) == tuple(map(bool, masks[i])),
                        ok_d, ok_d and (got_tb == tbs[i]).all()))
        m_exp = 1 + masks[i][0] + 2 * masks[i][1]
        res.append(("gpu-decoder", i, g_res[i] > 0, g_res[i] == m_exp and (g_plcf[i, : 5 * plcf_types[i]] == plcfs[i]).all(),
                    bool(g_ok[i]),
                    bool(g_ok[i]) and (g_tb[i, : sz["N_TB_bits"] // 8] == tbs[i]).all()))
    return res


@pytest.mark.parametrize("name", sorted(LOOPS))
def test_fec_loopback_crc_pass(name):
    for src, i, ok_c, good_c, ok_d, good_d in _loop(name, 30.0):
        assert ok_c and good_c, (name, src, i, "PLCF")
        assert ok_d and good_d, (name, src, i, "TB")


def test_fec_loopback_crc_fail_far_below_threshold():
    for src, i, ok_c, good_c, ok_d, good_d in _loop("u2b4_tm5_mcs6", -8.0, seed=2):
        assert not ok_d, (src, i)           # 64-QAM rate-3/4-class TB at -8 dB: undecodable
        assert ok_c == good_c, (src, i)     # a PLCF CRC pass must carry the transmitted PLCF


# (N_TB_bits, Qm, G, Z, rv, Es/N0 dB of BPSK-equivalent LLRs): C = 1 / C > 1, several sizes per
# call, the C4 transport block (58 + 2 code blocks: waves of 64 same-size blocks, partial waves),
# clean inputs (2 iterations), marginal ones (more iterations, some blocks failing at 10), rv 2 / 3
# (SNR = 1/sigma^2 of the +-1 soft bits)
DEC_CASES = [(296, 2, 644, 6144, 0, 30.0), (363464, 8, 486640, 6144, 0, 30.0), (363464, 8, 486640, 6144, 0, 30.0),
             (14560, 6, 19572, 6144, 0, 4.0), (5000 * 8, 4, 60000, 2048, 0, 3.5), (1000 * 8, 2, 12000, 6144, 3, 3.5),
             (363464, 8, 486640, 6144, 0, 4.5), (296, 2, 644, 6144, 0, -1.0), (40 * 8, 1, 2000, 2048, 0, -6.0),
             (4136, 2, 16000, 6144, 2, 1.0)]


def test_gpu_turbo_decoder_matches_host():
    """dnrp_pdc_decode_batch against the host decoder dnrp_pdc_decode (the reference's per-packet
    decode_tb role): identical CRC status, iteration counts and decoded bytes for every packet."""
    import dnrp
    import dnrp.fec as FE
    import fec_np as ON  # noqa: F401  (oracle/ on sys.path above)
    phy = dnrp.Phy(1, 1, 1, max_batch=1)
    rng = np.random.default_rng(9)
    cfgs, llrs, tbs = [], [], []
    for tbs_bits, Qm, G, Z, rv, snr in DEC_CASES:
        while ON.cbsegm(tbs_bits, Z)[2] != 0:
            tbs_bits += 8
        G -= G % Qm
        cfg = FE.fec_cfg(tbs_bits, Qm, G, Z=Z, rv=rv)
        tb = rng.integers(0, 256, tbs_bits // 8, dtype=np.uint8)
        x = 2.0 * np.unpackbits(FE.pdc_encode(cfg, tb))[:G] - 1
        y = x + rng.normal(0, 10 ** (-snr / 20), G)
        llrs.append(np.round(np.clip(y * 300, -32768, 32767)).astype(np.int16))
        cfgs.append(cfg)
        tbs.append(tb)
    m = len(cfgs)
    g_max = max(c.G for c in cfgs)
    llr = np.zeros((m, g_max + 5), np.int16)
    for i in range(m):
        llr[i, : cfgs[i].G] = llrs[i]
    dev = torch.device("cuda:0")
    tb_dev = torch.full((m, max(c.N_TB_bits for c in cfgs) // 8 + 7), 0xEE, dtype=torch.uint8, device=dev)
    ok, it = FE.pdc_decode_batch(phy, cfgs, torch.from_numpy(llr).to(dev), tb_dev)
    g_tb = tb_dev.cpu().numpy()
    n_fail = 0
    for i in range(m):
        h_ok, h_tb, h_it = FE.pdc_decode(cfgs[i], llrs[i])
        assert (bool(ok[i]), int(it[i])) == (h_ok, h_it), (i, DEC_CASES[i], ok[i], it[i], h_ok, h_it)
        assert (g_tb[i, : cfgs[i].N_TB_bits // 8] == h_tb).all(), (i, DEC_CASES[i])
        if h_ok:
            assert (h_tb == tbs[i]).all()
        n_fail += not h_ok
    assert ok[0] and ok[1] and ok[2] and 1 <= n_fail <= m - 3


def test_gpu_decoders_match_numpy_oracle():
    """dnrp_pdc_decode_batch and dnrp_pcc_decode_batch against oracle/fec_np.py's numpy max-log-MAP
    decoder (independent of the library's code; tests/test_fec_decoder_oracle.py holds the host
    decoder to the same oracle): CRC verdict, iterations and bits, clean / marginal / failing inputs."""
    import dnrp
    import dnrp.fec as FE
    import fec_np as ON
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import test_fec_decoder_oracle as TD
    phy = dnrp.Phy(1, 1, 1, max_batch=8)
    dev = torch.device("cuda:0")
    cfgs, llrs, want = [], [], []
    for tbs, Qm, G, rv, snr in TD.PDC_CASES:
        while not TD._tbs_valid(tbs):
            tbs += 8
        rng = np.random.default_rng(tbs + G)
        tb = rng.integers(0, 256, tbs // 8, dtype=np.uint8)
        cfg = FE.fec_cfg(tbs, Qm, G, rv=rv)
        llr = TD.noisy(np.unpackbits(FE.pdc_encode(cfg, tb))[:G], snr, rng)
        cfgs.append(cfg)
        llrs.append(llr)
        want.append(ON.pdc_decode(llr, tbs, 6144, Qm, G, rv, TD.qpp_of))
    m = len(cfgs)
    buf = np.zeros((m, max(c.G for c in cfgs)), np.int16)
    for i in range(m):
        buf[i, : cfgs[i].G] = llrs[i]
    tb_dev = torch.zeros((m, max(c.N_TB_bits for c in cfgs) // 8 + 3), dtype=torch.uint8, device=dev)
    ok, it = FE.pdc_decode_batch(phy, cfgs, torch.from_numpy(buf).to(dev), tb_dev)
    g_tb = tb_dev.cpu().numpy()
    for i, (ok_o, bits_o, it_o) in enumerate(want):
        assert (bool(ok[i]), int(it[i])) == (bool(ok_o), it_o), (TD.PDC_CASES[i], ok[i], it[i], ok_o, it_o)
        assert np.array_equal(np.unpackbits(g_tb[i, : cfgs[i].N_TB_bits // 8]), bits_o), TD.PDC_CASES[i]
    # PLCF: both types, the four CRC masks, clean / marginal / failing
    rng = np.random.default_rng(77)
    types, llr_p, want_p = [], [], []
    for trial in range(8):
        t = 1 + trial % 2
        plcf = rng.integers(0, 256, 5 * t, dtype=np.uint8)
        d = np.unpackbits(FE.pcc_encode(plcf, t, trial % 2, (trial // 2) % 2))[:196]
        l = TD.noisy(d, (8.0, 0.0, -6.0)[trial % 3], rng)
        types.append(t)
        llr_p.append(l)
        want_p.append(ON.pcc_decode(l, t, TD.qpp_of))
    plcf_dev = torch.zeros((8, 10), dtype=torch.uint8, device=dev)
    res, it = FE.pcc_decode_batch(phy, types, torch.from_numpy(np.stack(llr_p)).to(dev), plcf_dev)
    got = plcf_dev.cpu().numpy()
    for i, (ok_o, bits_o, m_o, it_o) in enumerate(want_p):
        assert (bool(res[i] > 0), int(it[i])) == (bool(ok_o), it_o), (i, res[i], it[i], ok_o, it_o)
        if ok_o:
            assert res[i] == 1 + m_o[0] + 2 * m_o[1]
            assert np.array_equal(np.unpackbits(got[i, : 5 * types[i]]), bits_o)


def test_gpu_encoder_matches_host():
    """dnrp_pdc_encode_batch against dnrp_pdc_encode (itself bit-exact against the numpy oracle):
    mixed sizes, Z, modulation orders and redundancy versions in one call."""
    import dnrp
    import dnrp.fec as FE
    import fec_np as ON  # noqa: F401
    phy = dnrp.Phy(1, 1, 1, max_batch=1)
    rng = np.random.default_rng(4)
    cfgs, tbs = [], []
    for tbs_bits, Qm, G, Z, rv, _ in DEC_CASES + [(2960, 1, 7001, 2048, 1, 0), (6144 * 3, 6, 60000, 2048, 2, 0),
                                                  (48000, 8, 97000, 6144, 3, 0)]:
        while ON.cbsegm(tbs_bits, Z)[2] != 0:
            tbs_bits += 8
        G -= G % Qm
        cfgs.append(FE.fec_cfg(tbs_bits, Qm, G, Z=Z, rv=rv))
        tbs.append(rng.integers(0, 256, tbs_bits // 8, dtype=np.uint8))
    m = len(cfgs)
    dev = torch.device("cuda:0")
    tb = np.zeros((m, max(c.N_TB_bits for c in cfgs) // 8 + 1), np.uint8)
    for i in range(m):
        tb[i, : len(tbs[i])] = tbs[i]
    d = torch.full((m, max((c.G + 7) // 8 for c in cfgs) + 3), 0xAB, dtype=torch.uint8, device=dev)
    FE.pdc_encode_batch(phy, cfgs, torch.from_numpy(tb).to(dev), d)
    g = d.cpu().numpy()
    for i in range(m):
        ref = FE.pdc_encode(cfgs[i], tbs[i])
        assert (g[i, : len(ref)] == ref).all(), (i, cfgs[i].N_TB_bits, cfgs[i].G)


def test_gpu_plcf_decoder_matches_host():
    """dnrp_pcc_decode_batch against dnrp_pcc_decode: both PLCF types, all four CRC masks, blind
    tests of the wrong type, clean to marginal SNRs: same result, iterations and PLCF bytes."""
    import dnrp
    import dnrp.fec as FE
    phy = dnrp.Phy(1, 1, 1, max_batch=1)
    rng = np.random.default_rng(12)
    n = 96
    types, tests, plcfs, llrs = [], [], [], []
    for i in range(n):
        t = 1 + i % 2
        pl = rng.integers(0, 256, 5 * t, dtype=np.uint8)
        d = FE.pcc_encode(pl, t, (i // 2) % 2, (i // 4) % 2)
        snr = [30.0, 4.0, 2.0, 0.0, -3.0][i % 5]
        y = 2.0 * np.unpackbits(d)[:196] - 1 + rng.normal(0, 10 ** (-snr / 20), 196)
        llrs.append(np.round(np.clip(y * 300, -32768, 32767)).astype(np.int16))
        types.append(t)
        tests.append(t if i % 7 else 3 - t)  # every 7th packet tested for the other type
        plcfs.append(pl)
    dev = torch.device("cuda:0")
    llr = torch.from_numpy(np.stack(llrs)).to(dev)
    plcf = torch.full((n, 12), 0xCD, dtype=torch.uint8, device=dev)
    res, it = FE.pcc_decode_batch(phy, tests, llr, plcf)
    g = plcf.cpu().numpy()
    n_ok = 0
    for i in range(n):
        ok, h_pl, cl, bf, h_it = FE.pcc_decode(llrs[i], tests[i])
        assert (res[i] > 0) == ok and it[i] == h_it, (i, res[i], it[i], ok, h_it)
        if ok:
            assert res[i] == 1 + int(cl) + 2 * int(bf)
            assert (g[i, : 5 * tests[i]] == h_pl).all()
            n_ok += 1
    assert 30 <= n_ok < n


def test_gpu_harq_combining_matches_host():
    """dnrp_pdc_decode_batch_harq over redundancy versions 0, 2, 3, 1 of the same transport blocks at
    an SNR where one transmission is not enough, against the host decoder with a dnrp_harq_rx per
    packet (pdc_decode_codeblocks' softbuffer semantics): identical CRC status, iterations and bytes
    after every redundancy version."""
    import dnrp
    import dnrp.fec as FE
    import fec_np as ON  # noqa: F401
    phy = dnrp.Phy(1, 1, 1, max_batch=1)
    rng = np.random.default_rng(21)
    cases = [(4136, 2, 6000, -3.0), (14560, 4, 19572, -1.0), (14560, 4, 19572, 6.0), (45432, 8, 60000, 0.0),
             (296, 2, 644, -4.0), (2960, 1, 7000, -2.0)]
    cfgs, tbs, snrs = [], [], []
    for tbs_bits, Qm, G, snr in cases:
        while ON.cbsegm(tbs_bits, 6144)[2] != 0:
            tbs_bits += 8
        G -= G % Qm
        cfgs.append(FE.fec_cfg(tbs_bits, Qm, G))
        tbs.append(rng.integers(0, 256, tbs_bits // 8, dtype=np.uint8))
        snrs.append(snr)
    m = len(cfgs)
    dev = torch.device("cuda:0")
    ent = max(FE.softbuffer_size(c.N_TB_bits)[0] for c in cfgs)
    ncb = max(FE.softbuffer_size(c.N_TB_bits)[1] for c in cfgs)
    sb = torch.zeros((m, ent), dtype=torch.int16, device=dev)
    flags = torch.zeros((m, ncb), dtype=torch.uint8, device=dev)
    tb_dev = torch.zeros((m, max(c.N_TB_bits for c in cfgs) // 8 + 3), dtype=torch.uint8, device=dev)
    hbs = [FE.HarqRx(c.N_TB_bits) for c in cfgs]
    g_max = max(c.G for c in cfgs)
    n_ok_first = None
    for rv in (0, 2, 3, 1):
        llr = np.zeros((m, g_max), np.int16)
        rows = []
        for i, c in enumerate(cfgs):
            ci = FE.fec_cfg(c.N_TB_bits, c.N_bps, c.G, rv=rv)
            cfgs[i] = ci
            x = 2.0 * np.unpackbits(FE.pdc_encode(ci, tbs[i]))[: c.G] - 1
            y = x + rng.normal(0, 10 ** (-snrs[i] / 20), c.G)
            rows.append(np.round(np.clip(y * 200, -32768, 32767)).astype(np.int16))
            llr[i, : c.G] = rows[-1]
        ok, it = FE.pdc_decode_batch_harq(phy, cfgs, torch.from_numpy(llr).to(dev), sb, flags, tb_dev)
        g_tb = tb_dev.cpu().numpy()
        for i in range(m):
            h_ok, h_tb, h_it = FE.pdc_decode(cfgs[i], rows[i], hbs[i])
            assert (bool(ok[i]), int(it[i])) == (h_ok, h_it), (rv, i, ok[i], it[i], h_ok, h_it)
            assert (g_tb[i, : cfgs[i].N_TB_bits // 8] == h_tb).all(), (rv, i)
            if h_ok:
                assert (h_tb == tbs[i]).all()
        if n_ok_first is None:
            n_ok_first = int(ok.sum())
    assert n_ok_first < m and int(ok.sum()) > n_ok_first


def test_gpu_plcf_encoder_matches_host():
    """dnrp_pcc_encode_batch against dnrp_pcc_encode: both PLCF types, all four CRC masks."""
    import dnrp
    import dnrp.fec as FE
    phy = dnrp.Phy(1, 1, 1, max_batch=1)
    rng = np.random.default_rng(31)
    n = 70
    types = [1 + (i % 3 == 0) for i in range(n)]
    cl = [(i // 2) % 2 for i in range(n)]
    bf = [(i // 5) % 2 for i in range(n)]
    plcf = rng.integers(0, 256, (n, 10), dtype=np.uint8)
    dev = torch.device("cuda:0")
    d = torch.full((n, 27), 0x5A, dtype=torch.uint8, device=dev)
    FE.pcc_encode_batch(phy, types, torch.from_numpy(plcf).to(dev), d, cl, bf)
    g = d.cpu().numpy()
    for i in range(n):
        ref = FE.pcc_encode(plcf[i, : 5 * types[i]], types[i], cl[i], bf[i])
        assert (g[i, :25] == ref).all(), i
