"""The LLR parity gate itself (tests/llr_gate.py) on synthetic rows: it must pass sparse boundary
flips and fail what the old max-only gate let through -- a systematic half-LSB bias and a 30 % flip
rate (VERDICT r05 "What's weak" #1)."""
import numpy as np
import pytest

import llr_gate


def _row(n=200000, seed=1):
    rng = np.random.default_rng(seed)
    return rng.integers(-30000, 30000, n).astype(np.int16)


def test_gate_passes_sparse_flips():
    o = _row()
    g = o.astype(np.int32)
    idx = np.random.default_rng(2).choice(len(o), 500, replace=False)  # 0.25 %, both signs
    g[idx] += np.where(np.arange(500) % 2 == 0, 1, -1)
    mx, mean, frac = llr_gate.check("sparse", g, o)
    assert mx == 1 and frac == pytest.approx(0.0025) and abs(mean) < 1e-4


def test_gate_rejects_bias():
    o = _row()
    g = o.astype(np.int32)
    g[::20] += 1  # 5 % of the values one LSB up: a rounding bias max |d| <= 1 cannot see
    with pytest.raises(AssertionError):
        llr_gate.check("bias", g, o)


def test_gate_rejects_many_flips():
    o = _row()
    g = o.astype(np.int32)
    rng = np.random.default_rng(3)
    idx = rng.choice(len(o), int(0.3 * len(o)), replace=False)
    g[idx] += rng.choice([-1, 1], len(idx))  # unbiased, but 30 % differ
    with pytest.raises(AssertionError):
        llr_gate.check("flips", g, o)


def test_gate_small_rows_allow_two_flips():
    o = _row(196)
    g = o.astype(np.int32)
    g[[5, 100]] += 1
    llr_gate.check("pcc", g, o)
    g[150] += 1
    with pytest.raises(AssertionError):
        llr_gate.check("pcc3", g, o)


def test_gate_rejects_two_lsb():
    o = _row(1000)
    g = o.astype(np.int32)
    g[7] += 2
    with pytest.raises(AssertionError):
        llr_gate.check("two", g, o)
