"""GPU ring-buffer gather and continuous-stream synchronisation (include/dnrp.h dnrp_ring_gather,
dnrp_rx_sync_stream) against numpy / the oracle.

- dnrp_ring_gather: bit-exact against a numpy wrap copy (rx_pacer.cpp:106-143) for odd and even
  ring lengths, windows that wrap, start times beyond one ring turn.
- dnrp_rx_sync_stream: a continuous stream of C2 packets in a ring, searched chunk by chunk. The
  checker gathers the same windows in numpy, runs the oracle's sync_chunk_t::search() on each and
  applies the baton's uniqueness test (baton.cpp:157-169) in chunk order; the GPU must report the
  same unique packets (fine peak time exact, found in the same chunk), every true packet exactly
  once, and count the same double detections. Then every unique packet is demodulated from RX
  windows gathered out of the ring at its fine peak and compared with the oracle RX (LLRs within 1).
"""
import numpy as np
import pytest

import llr_gate
import oracle_py as O
import phy_fixtures as F

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu


def _phy(name, max_batch=64):
    import dnrp
    ps, cf = F.CONFIGS[name]
    u_max, b_max, ntx, os_min, L, M = cf
    phy = dnrp.Phy(u_max, b_max, ntx, os_min, L, M, max_batch=max_batch)
    for nid in range(100, 106):
        phy.add_network_id(nid)
    return phy


def _np_gather(ring, starts, S_win):
    R = ring.shape[1]
    return np.stack([ring[:, (np.arange(S_win) + int(s)) % R] for s in starts])


def _to_dev(a):
    return torch.from_numpy(np.ascontiguousarray(a).view(np.float32).reshape(*a.shape, 2)).to("cuda:0")


@pytest.mark.parametrize("n_ant,R,S_win", [(2, 10001, 3000), (4, 20000, 4096), (1, 4096, 4096)])
def test_ring_gather(n_ant, R, S_win):
    rng = np.random.default_rng(31 + R)
    phy = _phy("C4" if n_ant > 1 else "C2")
    ring = (rng.standard_normal((n_ant, R)) + 1j * rng.standard_normal((n_ant, R))).astype(np.complex64)
    starts = [0, 7, R - 1, R - S_win // 3, 3 * R + 5, 2 * R - 2, R // 2 + 1]
    out = torch.zeros((len(starts), n_ant, S_win, 2), dtype=torch.float32, device="cuda:0")
    phy.ring_gather(_to_dev(ring), starts, S_win, out)
    phy.sync()
    got = out.cpu().numpy().view(np.complex64)[..., 0]
    assert np.array_equal(got, _np_gather(ring, starts, S_win))


def _oracle_stream(osc, ring, t0, n_chunks, chunk, S_win, max_reports, limit):
    """numpy gather + oracle search per chunk + baton uniqueness, in chunk order"""
    last, out, dup = O_UNDEFINED_EARLY, [], 0
    for k in range(n_chunks):
        tk = t0 + k * chunk
        win = _np_gather(ring, [tk], S_win)[0]
        for r in O.sync(osc, win, max_reports=max_reports):
            t = tk + r["fine_64"]
            if t - last > limit:
                last = t
                out.append((t, k, r))
            else:
                dup += 1
    return out, dup


O_UNDEFINED_EARLY = np.iinfo(np.int64).min // 8


def test_sync_stream_c2():
    import dnrp
    rng = np.random.default_rng(41)
    name = "C2"
    psd, cfgt = F.CONFIGS[name]
    phy = _phy(name)
    chunk, n_chunks, max_reports = 400, 24, 3
    sc = dnrp.SyncCfg(psd[0], psd[1], 1, chunk, max_reports)
    S_win = phy.sync_stream_window(sc)
    assert S_win >= chunk
    # a stream of packets at irregular spacing (some start close to chunk edges), stored in a ring
    # that the searched range wraps around
    T = n_chunks * chunk + S_win
    times = [150, 1190, 2001, 3395, 4800, 6210, 7604, 8399]
    made = []
    stream = np.zeros((1, T), np.complex64)
    for i, t in enumerate(times):
        cfo = rng.uniform(-1.2, 1.2) * 2 * np.pi / 64
        win, meta = F.sync_window(rng, O, name, 900, [0], cfo, snr_db=None)
        stream[:, t:t + 900] += win
        made.append(meta[0])
    p = np.mean(np.abs(stream[stream != 0]) ** 2)
    sigma = np.sqrt(p / 10 ** 2.5 / 2)
    stream = (stream + sigma * (rng.standard_normal(stream.shape) + 1j * rng.standard_normal(stream.shape))).astype(
        np.complex64)
    R = T
    g0 = 5 * R + R // 3  # global time of stream sample 0: the ring wraps inside the stream
    ring = np.zeros((1, R), np.complex64)
    ring[:, (g0 + np.arange(T)) % R] = stream
    state = phy.sync_stream_init(sc)
    assert state.sync_time_unique_limit == 16  # one STF pattern at b = 1, os_min = 1
    ring_d = _to_dev(ring)
    got, chunk_of = [], []
    for part in range(2):  # two calls continue one stream (the state carries the baton)
        t0 = g0 + part * (n_chunks // 2) * chunk
        res, ck = phy.rx_sync_stream(sc, ring_d, t0, n_chunks // 2, state)
        got += list(res)
        chunk_of += [int(c) + part * (n_chunks // 2) for c in ck]
    osc = O.sync_cfg(psd[0], psd[1], L=cfgt[4], M=cfgt[5], n_ant=1, chunk_len=chunk)
    ref, dup = _oracle_stream(osc, ring, g0, n_chunks, chunk, S_win, max_reports, state.sync_time_unique_limit)
    assert len(got) == len(ref), ([int(g["fine_peak_time"]) for g in got], [r[0] for r in ref])
    for g, k, (t, kr, r) in zip(got, chunk_of, ref):
        assert int(g["fine_peak_time"]) == t and k == kr
        assert int(g["N_eff_TX"]) == r["N_eff_TX"]
        assert abs(float(g["cfo_fractional_rad"]) - r["cfo_frac"]) < 2e-6
    assert int(state.not_unique) == dup and dup > 0  # the chunk overlap detects packets twice
    assert [int(g["fine_peak_time"]) - g0 for g in got] == times  # every packet exactly once

    # demodulate every unique packet from RX windows gathered out of the ring at its fine peak
    ps = dnrp.psdef(*psd)
    sz = phy.packet_sizes(ps)
    pre, S_in = 64, sz["N_samples_packet_os_rs"] + 256
    starts = [int(g["fine_peak_time"]) - pre for g in got]
    win_d = torch.zeros((len(got), 1, S_in, 2), dtype=torch.float32, device="cuda:0")
    phy.ring_gather(ring_d, starts, S_in, win_d)
    reps = dnrp.sync_reports(np.array(got, dtype=dnrp.SYNC_RESULT_DTYPE))
    reps["fine_peak_time"] = pre
    pcc = torch.zeros((len(got), 196), dtype=torch.int16, device="cuda:0")
    pdc = torch.zeros((len(got), sz["G"]), dtype=torch.int16, device="cuda:0")
    phy.rx_pcc_batch(reps, win_d, pcc)
    phy.rx_pdc_batch([dnrp.PdcReq(ps, i, m[2], m[3]) for i, m in enumerate(made)], win_d, pdc)
    phy.sync()
    wins = _np_gather(ring, starts, S_in)
    ocf = O.cfg(cfgt[0], cfgt[1], os_min=cfgt[3], L=cfgt[4], M=cfgt[5])
    for i, m in enumerate(made):
        r = O.rx(ocf, O.psdef(*psd), wins[i], pre, float(got[i]["cfo_fractional_rad"]), m[2], m[3])
        llr_gate.check(("ring", i, "pcc"), pcc[i].cpu().numpy(), r["pcc_llr"])
        llr_gate.check(("ring", i, "pdc"), pdc[i].cpu().numpy(), r["pdc_llr"])
        assert np.array_equal(np.unpackbits(m[1])[: sz["G"]], (pdc[i].cpu().numpy() > 0).astype(np.uint8)), i
