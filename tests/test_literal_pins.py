"""Pin the literal tables of sections_part3 against the reference's own text.

tests/golden/ref_literals.json is extracted from the reference sources as text by
tests/golden/make_literals_fixture.py (beamforming_and_antenna_port_mapping.cpp/.hpp W_1..W_6, the
codebook index tables and scaling_factor_optimal_DAC; stf.cpp y_b_1/2/4 and stf.hpp's cover sequence;
drs.hpp y_b_1; transmit_diversity_precoding.cpp index_N_TS_x and its SFBC sign pattern). Both
restatements are compared with it: the oracle (oracle/oracle_tables.cpp) and the product's host
geometry the device tables are uploaded from (csrc/host/geometry.cpp via dnrp_query_table; the
kernels' cover sequence is the same params.hpp macro). Exact for integers and +-1 / +-j values, float
rounding for scalings. The constructions the reference performs on these literals (the STF
extension to b = 8 / 12 / 16 and the cyclic shift by 2 log2(N_eff_TX), stf.cpp:185-285; the DRS value
rule, drs.cpp:227-254; the optimal-DAC statements, replayed by the extraction) are restated here once
more from the reference text, citing it."""
import json
import os

import numpy as np
import pytest

import oracle_py as O

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "ref_literals.json")))
dnrp = pytest.importorskip("dnrp")

J = GOLD["j"]
# W family k of W_t (beamforming_and_antenna_port_mapping.cpp:30-66): (N_TS, N_TX) of W[1..6]
FAMILIES = {1: (1, 2), 2: (1, 4), 3: (2, 2), 4: (2, 4), 5: (4, 4), 6: (8, 8)}


def _w_complex(codes):
    return np.array([1j if c == J else -1j if c == -J else complex(c) for c in codes])


def test_fixture_shape():
    assert [len(GOLD[f"W_{k}"]) for k in FAMILIES] == [6, 28, 3, 22, 5, 1]
    for k, (nts, ntx) in FAMILIES.items():
        assert all(len(r) == nts * ntx for r in GOLD[f"W_{k}"]), k
        assert GOLD["N_TS_N_TX_idx"][nts][ntx] == k
        assert GOLD["N_TS_N_TX_codebook_index_max"][nts][ntx] == len(GOLD[f"W_{k}"]) - 1


@pytest.mark.parametrize("k", sorted(FAMILIES))
def test_W_matrices(k):
    nts, ntx = FAMILIES[k]
    assert dnrp.query_table("W_codebooks", nts, ntx)[0] == len(GOLD[f"W_{k}"])
    assert O.W_codebooks(nts, ntx) == len(GOLD[f"W_{k}"])
    for cb, codes in enumerate(GOLD[f"W_{k}"]):
        want = _w_complex(codes).reshape(ntx, nts)  # row-major [antenna][transmit stream]
        q = dnrp.query_table("W", nts, ntx, cb).view(np.complex64).reshape(ntx, nts)
        assert np.array_equal(q, want.astype(np.complex64)), (k, cb)
        w, sc, sc_opt = O.W(nts, ntx, cb)
        assert np.array_equal(w, want), (k, cb)
        # get_W_scaling_factor (beamforming_...mapping.cpp:307-320): 1/sqrt(non-zero entries), float
        nz = np.float32(np.count_nonzero(codes))
        s = np.float32(1.0) / np.sqrt(nz)
        assert dnrp.query_table("W_scaling", nts, ntx, cb)[0] == s and np.float32(sc) == s, (k, cb)
        opt = np.float32(GOLD["scaling_factor_optimal_DAC"][k][cb])
        assert dnrp.query_table("W_scaling_optimal_DAC", nts, ntx, cb)[0] == opt, (k, cb)
        assert np.float32(sc_opt) == opt, (k, cb)
    with pytest.raises(dnrp.DnrpError):
        dnrp.query_table("W", nts, ntx, len(GOLD[f"W_{k}"]))


def test_W_siso_and_undefined():
    assert np.array_equal(dnrp.query_table("W", 1, 1, 0), [1, 0])
    assert GOLD["scaling_factor_optimal_DAC"][0] == [1.0]
    assert dnrp.query_table("W_scaling_optimal_DAC", 1, 1, 0)[0] == 1.0
    for nts, ntx in ((4, 2), (8, 4), (2, 1)):  # N_TS_N_TX_idx has no matrix there
        assert GOLD["N_TS_N_TX_idx"][nts][ntx] == 0
        with pytest.raises(dnrp.DnrpError):
            dnrp.query_table("W", nts, ntx, 0)


def test_codebook_index_nonzero_entries_exist():
    # N_TS_N_TX_codebook_index_nonzero (used by the MIMO report for N_TS = 1, estimator_mimo.cpp)
    for (nts, ntx) in ((1, 2), (1, 4), (2, 2), (2, 4)):
        nz = GOLD["N_TS_N_TX_codebook_index_nonzero"][nts][ntx]
        assert nz < dnrp.query_table("W_codebooks", nts, ntx)[0]
    assert GOLD["N_TS_N_TX_codebook_index_nonzero"][1][2] == 2 and GOLD["N_TS_N_TX_codebook_index_nonzero"][1][4] == 12


def _stf_polarity(b):
    """stf.cpp:207-250: y_b_1/2/4 as listed; 8 = y4 ++ fliplr(y4)(-1)^k, 16 likewise from 8, 12 =
    y_16[28 : 28 + 168]."""
    def ext(v):
        r = [v[len(v) - 1 - i] * (1 if i % 2 == 0 else -1) for i in range(len(v))]
        return v + r
    if b in (1, 2, 4):
        return GOLD[f"stf_y_b_{b}"]
    y8 = ext(GOLD["stf_y_b_4"])
    if b == 8:
        return y8
    y16 = ext(y8)
    return y16 if b == 16 else [y16[i + 2 * 14] for i in range(168)]


@pytest.mark.parametrize("b", [1, 2, 4, 8, 12, 16])
@pytest.mark.parametrize("n_eff", [1, 2, 4, 8])
def test_stf_values(b, n_eff):
    N = 56 * b
    pol = _stf_polarity(b)
    assert len(pol) == N // 4
    k = O.k_b_occ(b)  # pinned against physical_resources.cpp (test_oracle_pins)
    # fill_k_i (stf.cpp:171-183) and fill_y_STF_i (185-270): exp(j pi/4) times the shifted polarity
    k_i = [k[i * 4] for i in range(N // 8)] + [k[N // 2 + 3 + (i - N // 8) * 4] for i in range(N // 8, N // 4)]
    lg = {1: 0, 2: 1, 4: 2, 8: 3}[n_eff]
    fac = np.complex64(complex(np.float32(np.cos(np.pi / 4)), np.float32(np.sin(np.pi / 4))))
    want = np.zeros(N + 1, np.complex64)
    for i in range(N // 4):
        want[k_i[i] + N // 2] = np.complex64(pol[(i + 2 * lg) % (N // 4)]) * fac
    got = dnrp.query_table("stf", b, n_eff).view(np.complex64)
    assert np.array_equal(got, want), (b, n_eff)
    assert np.allclose(O.stf(b, n_eff), want, rtol=0, atol=1e-7), (b, n_eff)


def test_cover_sequence():
    want = np.array(GOLD["cover_sequence"], np.float32)
    assert np.array_equal(dnrp.query_table("stf_cover_sequence"), want)
    assert np.array_equal(O.cover_sequence(), want)


@pytest.mark.parametrize("b", [1, 2, 4, 8, 12, 16])
def test_drs_values(b):
    y = GOLD["drs_y_b_1"]
    assert all(im == 0 and re in (-1, 1) for re, im in y)
    for t in range(8):  # drs.cpp:227-254: +y_b_1[(4i + t%4) % 56] for t < 4, negated for t >= 4
        want = np.array([(1 if t < 4 else -1) * y[(4 * i + t % 4) % 56][0] for i in range(14 * b)], np.float32)
        assert np.array_equal(dnrp.query_table("drs_values", b, t), want), (b, t)
        assert np.array_equal(O.drs_values(b, t), want), (b, t)


@pytest.mark.parametrize("row,nts", [(0, 2), (1, 4), (2, 8)])
def test_txdiv_pairs(row, nts):
    want = GOLD["index_N_TS_x"][row]
    assert len(want) == GOLD["txdiv_modulo"][str(nts)]
    assert dnrp.query_table("txdiv_pairs", nts).astype(int).reshape(-1, 2).tolist() == want
    assert O.txdiv_pairs(nts) == want


def test_sfbc_sign_pattern():
    # pattern_minus_1_j_1_j (transmit_diversity_precoding.cpp:37-43): (-1 + 1j), (1 - 1j) -- the
    # elementwise (re, im) factors of the pairwise swap: x'[2i] = (-re, +im) x[2i+1], x'[2i+1] =
    # (+re, -im) x[2i], which the TX parity tests then check end to end
    assert GOLD["pattern_minus_1_j_1_j"] == [[-1.0, 1.0], [1.0, -1.0]]
