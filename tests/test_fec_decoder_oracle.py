"""Both product turbo decoders against the numpy max-log-MAP decoder of oracle/fec_np.py.

The decoder arithmetic of srsRAN's tdec is absent from /root/reference (parity unpinned,
SURVEY.md §8(c)); oracle/fec_np.py restates the receive chain independently of the library's code
(rate de-matching into a saturating int16 circular buffer, integer max-log-MAP with renormalised
metrics, extrinsic x3/4, the reference's read position and length per code block,
pdc_enc.cpp:322-332, the iteration limits and CRC rules of pcc_enc.cpp:309-351 / pdc_enc.cpp).
Checked: CRC verdict, decoded bits and iteration count equal -- on clean, marginal and failing
inputs, one and several code blocks, two code-block sizes in one transport block, rv 0 and 2.
The GPU decoders (dnrp_pdc_decode_batch / dnrp_pcc_decode_batch) against the same oracle:
tests/test_gpu_fec.py::test_gpu_decoders_match_numpy_oracle."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import fec_np as ON  # noqa: E402

dnrp = pytest.importorskip("dnrp")
import dnrp.fec as F  # noqa: E402


def qpp_of(K):
    _, f1, f2 = F.cb_size(ON.cb_sizes().index(K))
    return f1, f2


def noisy(bits, snr_db, rng, scale=64.0):
    """BPSK-equivalent soft bits (positive = bit 1, tb2pdc.cpp:173-176) at snr_db, int16"""
    x = 2.0 * bits - 1
    y = x + rng.normal(0, 10 ** (-snr_db / 20), len(bits))
    return np.round(np.clip(y * scale, -32767, 32767)).astype(np.int16)


# (tbs, Qm, G, rv, snr_db): C = 1 (4 iterations); C = 3 with two block sizes and gamma != 0 (block
# C - gamma read short); C = 2 at marginal SNR (extra iterations) and below it (blocks failing at 10);
# rv 2; far below threshold
PDC_CASES = [(296, 2, 644, 0, 6.0), (4136, 4, 8800, 0, 1.5), (14000, 2, 30002, 0, 1.0), (7000, 6, 12000, 0, 5.0),
             (7000, 6, 12000, 0, 0.5), (2000, 2, 3000, 2, 3.0), (1024, 2, 2400, 0, -4.0)]


def _tbs_valid(tbs):
    try:
        return F.cbsegm(tbs, 6144)["F"] == 0
    except Exception:
        return False


@pytest.mark.parametrize("case", PDC_CASES, ids=lambda c: "tbs%d_G%d_rv%d_%gdB" % (c[0], c[2], c[3], c[4]))
def test_host_pdc_decoder_matches_numpy(case):
    tbs, Qm, G, rv, snr = case
    while not _tbs_valid(tbs):
        tbs += 8
    rng = np.random.default_rng(tbs + G)
    tb = rng.integers(0, 256, tbs // 8, dtype=np.uint8)
    cfg = F.fec_cfg(tbs, Qm, G, rv=rv)
    d = np.unpackbits(F.pdc_encode(cfg, tb))[:G]
    llr = noisy(d, snr, rng)
    ok_h, tb_h, it_h = F.pdc_decode(cfg, llr)
    ok_o, bits_o, it_o = ON.pdc_decode(llr, tbs, 6144, Qm, G, rv, qpp_of)
    if case[2] == 30002:  # the intended segmentation: C = 3, two sizes, gamma = 1
        sg = F.cbsegm(tbs, 6144)
        assert sg["C"] == 3 and sg["K1"] != sg["K2"] and (G // Qm) % 3 == 1, sg
    assert (ok_h, it_h) == (bool(ok_o), it_o), (case, ok_h, it_h, ok_o, it_o)
    assert np.array_equal(np.unpackbits(tb_h), bits_o), case


@pytest.mark.parametrize("plcf_type", [1, 2])
@pytest.mark.parametrize("snr", [8.0, 0.0, -6.0])
def test_host_pcc_decoder_matches_numpy(plcf_type, snr):
    rng = np.random.default_rng(plcf_type * 10 + int(snr) + 100)
    for trial in range(3):
        plcf = rng.integers(0, 256, 5 * plcf_type, dtype=np.uint8)
        cl, bf = trial % 2, (trial // 2) % 2
        d = np.unpackbits(F.pcc_encode(plcf, plcf_type, cl, bf))[:196]
        llr = noisy(d, snr, rng)
        ok_h, plcf_h, cl_h, bf_h, it_h = F.pcc_decode(llr, plcf_type)
        ok_o, bits_o, m_o, it_o = ON.pcc_decode(llr, plcf_type, qpp_of)
        assert (ok_h, it_h) == (bool(ok_o), it_o), (plcf_type, snr, trial)
        if ok_h:
            assert np.array_equal(np.unpackbits(plcf_h), bits_o) and (cl_h, bf_h) == tuple(map(bool, m_o))
