"""Simulated wireless channel, host side (dnrp_channel_realization; no GPU): power delay profiles as
link_t::set_pdp builds them (link.cpp:66-120, restated below from link.hpp:88-108 = 3GPP TS 36.104
Annex B EPA / EVA / ETU), Jakes' Doppler sinusoids (link.cpp:144-200) and Rayleigh flat
coefficients (channel_flat.cpp:80-89) by their distribution."""
import math
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "dect-nr-plus-sdr_amd"))

PDP = [([0, 30, 70, 90, 110, 190, 410], [0.0, -1.0, -2.0, -3.0, -8.0, -17.2, -20.8]),
       ([0, 30, 150, 310, 370, 710, 1090, 1730, 2510], [0.0, -1.5, -1.4, -3.6, -0.6, -9.1, -7.0, -12.0, -16.9]),
       ([0, 50, 120, 200, 230, 500, 1600, 2300, 5000], [-1.0, -1.0, -1.0, 0.0, 0.0, 0.0, -3.0, -5.0, -7.0])]


def _tau_rms(d, p_db):
    p = 10.0 ** (np.asarray(p_db, np.float64) / 10.0)
    p /= p.sum()
    mean = np.sum(np.asarray(d, np.float64) * p)
    return math.sqrt(np.sum((np.asarray(d) - mean) ** 2 * p))


def _set_pdp(idx, tau_rms_ns, samp_rate):
    d, p_db = PDP[idx]
    scale = tau_rms_ns / _tau_rms(d, p_db)
    delays, powers = [], []
    for dn, pdb in zip(d, p_db):
        a = int(math.floor(dn * 1e-9 * scale / (1.0 / samp_rate)))
        b = 10.0 ** (pdb / 10.0)
        if a in delays:
            powers[delays.index(a)] += b
        else:
            delays.append(a)
            powers.append(b)
    s = sum(powers)
    amps = [np.float32(np.float32(1.0) / np.sqrt(np.float32(40.0))) * np.float32(math.sqrt(p / s)) for p in powers]
    return delays, np.array(amps, np.float32)


@pytest.mark.parametrize("idx,tau,rate", [(0, 43.13, 245760000), (1, 356.65, 245760000), (2, 990.93, 30720000),
                                          (1, 100.0, 1728000), (0, 0.0, 245760000)])
def test_pdp_matches_set_pdp(idx, tau, rate):
    import dnrp
    c = dnrp.ChannelCfg(dnrp.CH_DOUBLY, idx, tau, 10.0, rate, 1.0, dnrp.CH_NOISELESS_DB, 1.0, 3)
    r = dnrp.channel_realization(c, 0, 2, 2)
    d, a = _set_pdp(idx, tau, rate)
    for rx in range(2):
        for tx in range(2):
            assert list(r["delay"][rx, tx]) == d
            np.testing.assert_allclose(r["amp"][rx, tx], a, rtol=1e-6)
    assert abs(float(np.sum(r["amp"][0, 0].astype(np.float64) ** 2)) * 40 - 1.0) < 1e-5  # unit power


def test_doppler_jakes():
    import dnrp
    fd, rate = 500.0, 245760000
    c = dnrp.ChannelCfg(dnrp.CH_DOUBLY, 1, 300.0, fd, rate, 1.0, dnrp.CH_NOISELESS_DB, 1.0, 11)
    per, ph = [], []
    for w in range(20):
        r = dnrp.channel_realization(c, w, 2, 2)
        per.append(r["period"].ravel())
        ph.append(r["phase_rev"].ravel())
    per, ph = np.concatenate(per), np.concatenate(ph)
    f = rate / per[per != np.iinfo(np.int64).max].astype(np.float64)
    assert np.all(np.abs(f) <= fd * (1 + 1e-6))  # fD cos(angle)
    # Jakes: cos of a uniform angle -> arcsine law, E[f] = 0, E[f^2] = fD^2 / 2
    assert abs(np.mean(f)) < 0.05 * fd
    assert abs(np.mean(f ** 2) / (fd ** 2 / 2) - 1) < 0.06
    assert np.all(np.abs(ph) <= 1.0 + 1e-9) and abs(np.mean(ph)) < 0.03  # rand_m1p1() * 2 pi
    # realisations differ between windows and repeat for the same (seed, window)
    assert not np.array_equal(dnrp.channel_realization(c, 0, 2, 2)["period"], dnrp.channel_realization(c, 1, 2, 2)["period"])
    assert np.array_equal(dnrp.channel_realization(c, 4, 2, 2)["phase_rev"], dnrp.channel_realization(c, 4, 2, 2)["phase_rev"])


def test_flat_rayleigh():
    import dnrp
    c = dnrp.ChannelCfg(dnrp.CH_FLAT, 0, 0.0, 0.0, 1, 1.0, dnrp.CH_NOISELESS_DB, 1.0, 5)
    z = np.concatenate([dnrp.channel_realization(c, w, 4, 4)["coef"].ravel() for w in range(400)])
    assert abs(np.mean(np.abs(z) ** 2) - 1.0) < 0.05
    assert abs(np.mean(z)) < 0.05 and abs(np.mean(z.real * z.imag)) < 0.03


def test_bad_channel_cfg():
    import dnrp
    with pytest.raises(dnrp.DnrpError):
        dnrp.channel_realization(dnrp.ChannelCfg(7, 0, 0.0, 0.0, 1, 1.0, 0.0, 1.0, 0), 0, 1, 1)
    with pytest.raises(dnrp.DnrpError):  # tau_rms above tau_rms_ns_max (link.hpp:82)
        dnrp.channel_realization(dnrp.ChannelCfg(2, 0, 2500.0, 10.0, 245760000, 1.0, 0.0, 1.0, 0), 0, 1, 1)
