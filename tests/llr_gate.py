"""The int16 LLR parity gate shared by the GPU RX tests (test infrastructure, no GPU needed to import).

A GPU LLR row passes against the oracle's row of the same packet when
  * max |g - o| <= 1 LSB (the float path against the oracle's double path, rounded once each: a value
    near a rounding boundary may land on either side),
  * |mean(g - o)| <= max(0.01, 2 / n) LSB (no systematic bias: a kernel that rounds half an LSB the
    wrong way on every value, or flips many values the same way, fails here although max <= 1),
  * the fraction of nonzero differences <= max(0.01, 2 / n) (boundary flips are rare; a kernel that
    differs by one on 30 % of the values fails here).
n is the row length; the 2 / n floor lets a 196-LLR PCC row carry two boundary flips.
(VERDICT r05 "What's weak" #1; reference demapper call sites rx_synced.cpp:999,1281-1299.)

With DNRP_PARITY_STATS=<path> every checked row appends one JSON line (tag, n, max, mean, fraction)
so the observed fractions can be quoted.
"""
import json
import os

import numpy as np

MEAN_MAX = 0.01
FRAC_MAX = 0.01


def check(tag, g, o):
    """Assert the gate for one row; returns (max, mean, fraction)."""
    g = np.asarray(g).astype(np.int32).ravel()
    o = np.asarray(o).astype(np.int32).ravel()
    assert g.shape == o.shape, (tag, g.shape, o.shape)
    n = len(o)
    if n == 0:
        return 0, 0.0, 0.0
    d = g - o
    mx = int(np.abs(d).max())
    mean = float(d.mean())
    frac = float(np.count_nonzero(d)) / n
    path = os.environ.get("DNRP_PARITY_STATS")
    if path:
        with open(path, "a") as f:
            f.write(json.dumps({"tag": str(tag), "n": n, "max": mx, "mean": mean, "frac": frac}) + "\n")
    floor = 2.0 / n
    assert mx <= 1, (tag, "max", mx, int(np.argmax(np.abs(d))))
    assert abs(mean) <= max(MEAN_MAX, floor), (tag, "mean", mean)
    assert frac <= max(FRAC_MAX, floor), (tag, "fraction", frac)
    return mx, mean, frac
