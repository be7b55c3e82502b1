"""ORACLE — TEST INFRASTRUCTURE ONLY (imported by tests/, never by the product path).

numpy restatement of the DECT NR+ channel-coding transmit chain the reference delegates to
srsRAN_4G release_23_11 (absent from /root/reference): CRC attachment, code-block segmentation,
turbo encoding and turbo rate matching, written from 3GPP TS 36.212 §5.1 (which ETSI TS 103 636-3
§6.1 adopts) in a matrix formulation independent of csrc/host/fec.cpp's index tables. Call
sites followed:
  pcc_enc_encode        lib/src/phy/fec/pcc_enc.cpp:145-213 (CRC16 + mask, K = 56 / 96, E = 196, rv 0)
  pdc_encode_codeblocks lib/src/phy/fec/pdc_enc.cpp:127-229 (CRC24A, CRC24B per block when C > 1,
                        K- blocks first, E per block from Gp = G / Qm and gamma = Gp mod C)
  srsran_cbsegm_FIX     lib/src/sections_part3/fix/cbsegm.cpp:55-123
Parity status: the K column (cb_sizes) is pinned to the reference's tc_cb_sizes
(tests/golden/ref_fec.json); the QPP coefficients (f1, f2) are TS 36.212 Table 5.1.3-3 constants
taken from the library under test and checked only to be permutations — parity unpinned for them,
as for every srsRAN arithmetic.
"""
import numpy as np

CRC16, CRC24A, CRC24B = (0x11021, 16), (0x1864CFB, 24), (0x1800063, 24)
PERM = [0, 16, 8, 24, 4, 20, 12, 28, 2, 18, 10, 26, 6, 22, 14, 30,
        1, 17, 9, 25, 5, 21, 13, 29, 3, 19, 11, 27, 7, 23, 15, 31]


def cb_sizes():
    return ([40 + 8 * i for i in range(60)] + [528 + 16 * i for i in range(32)] +
            [1056 + 32 * i for i in range(32)] + [2112 + 64 * i for i in range(64)])


def crc(bits, g):
    """polynomial long division of bits(x) * x^L by g(x) (TS 36.212 §5.1.1), remainder as L bits"""
    poly, L = g
    gb = np.array([(poly >> (L - i)) & 1 for i in range(L + 1)], np.uint8)
    r = np.concatenate([np.asarray(bits, np.uint8), np.zeros(L, np.uint8)])
    for i in range(len(bits)):
        if r[i]:
            r[i:i + L + 1] ^= gb
    return r[-L:]


def cbsegm(B_tb, Z):
    """TS 36.212 §5.1.2 with the reference's max code-block size Z -> (C, [K per block])"""
    B = B_tb + 24
    if B <= Z:
        C, Bp = 1, B
    else:
        C = -(-B // (Z - 24))
        Bp = B + 24 * C
    ks = cb_sizes()
    Kp = min(k for k in ks if C * k >= Bp)
    if C == 1:
        return 1, [Kp], Kp - Bp
    Km = max(k for k in ks if k < Kp)
    Cm = (C * Kp - Bp) // (Kp - Km)
    F = (C - Cm) * Kp + Cm * Km - Bp
    return C, [Km] * Cm + [Kp] * (C - Cm), F


def qpp(K, f1, f2):
    i = np.arange(K, dtype=np.int64)
    return ((f1 * i + f2 * i * i) % K).astype(np.int64)


def _rsc(c):
    """8-state constituent encoder, transfer function [1, g1/g0], g0 = 1+D^2+D^3, g1 = 1+D+D^3"""
    reg = [0, 0, 0]  # a_{k-1}, a_{k-2}, a_{k-3}
    z = []
    for ck in c:
        a = int(ck) ^ reg[1] ^ reg[2]
        z.append(a ^ reg[0] ^ reg[2])
        reg = [a, reg[0], reg[1]]
    tail = []
    for _ in range(3):
        x = reg[1] ^ reg[2]
        tail.append((x, reg[0] ^ reg[2]))
        reg = [0, reg[0], reg[1]]
    return np.array(z, np.uint8), tail


def turbo(c, f1, f2):
    """-> d0, d1, d2 (TS 36.212 §5.1.3.2 incl. trellis termination)"""
    K = len(c)
    z1, t1 = _rsc(c)
    z2, t2 = _rsc(np.asarray(c)[qpp(K, f1, f2)])
    x, z = [t[0] for t in t1], [t[1] for t in t1]
    xp, zp = [t[0] for t in t2], [t[1] for t in t2]
    d0 = np.concatenate([c, [x[0], z[1], xp[0], zp[1]]]).astype(np.uint8)
    d1 = np.concatenate([z1, [z[0], x[2], zp[0], xp[2]]]).astype(np.uint8)
    d2 = np.concatenate([z2, [x[1], z[2], xp[1], zp[2]]]).astype(np.uint8)
    return d0, d1, d2


def _subblock(d, third):
    """sub-block interleaver as a matrix: rows of 32 after ND dummy (-1) bits, column permutation"""
    D = len(d)
    R = -(-D // 32)
    y = np.concatenate([-np.ones(32 * R - D, np.int16), d.astype(np.int16)])
    if not third:
        return y.reshape(R, 32)[:, PERM].T.reshape(-1)
    Kpi = 32 * R
    k = np.arange(Kpi)
    return y[(np.array(PERM)[k // R] + 32 * (k % R) + 1) % Kpi]


def rate_match(d0, d1, d2, E, rv):
    v0, v1, v2 = _subblock(d0, False), _subblock(d1, False), _subblock(d2, True)
    Kpi = len(v0)
    R = Kpi // 32
    w = np.concatenate([v0, np.stack([v1, v2], 1).reshape(-1)])
    Ncb = len(w)
    k0 = R * (2 * int(np.ceil(Ncb / (8 * R))) * rv + 2)
    order = np.roll(w, -k0)
    valid = order[order >= 0]
    reps = -(-E // len(valid))
    return np.tile(valid, reps)[:E].astype(np.uint8)


def pcc_encode(plcf_bits, cl, bf, qpp_of):
    mask = {(0, 0): 0x0000, (1, 0): 0x5555, (0, 1): 0xAAAA, (1, 1): 0xFFFF}[(int(cl), int(bf))]
    p = crc(plcf_bits, CRC16) ^ np.array([(mask >> (15 - i)) & 1 for i in range(16)], np.uint8)
    c = np.concatenate([plcf_bits, p]).astype(np.uint8)
    K = len(c)
    assert K in cb_sizes()
    return rate_match(*turbo(c, *qpp_of(K)), 196, 0)


def pdc_encode(tb_bits, Z, Qm, G, rv, qpp_of):
    tbs = len(tb_bits)
    b = np.concatenate([tb_bits, crc(tb_bits, CRC24A)]).astype(np.uint8)
    C, Ks, F = cbsegm(tbs, Z)
    assert F == 0
    Gp = G // Qm
    gamma = Gp % C
    out, rp = [], 0
    for r, K in enumerate(Ks):
        n = K - 24 if C > 1 else K
        c = b[rp:rp + n]
        if C > 1:
            c = np.concatenate([c, crc(c, CRC24B)])
        rp += n
        E = Qm * (Gp // C) if r <= C - gamma - 1 else Qm * (-(-Gp // C))
        out.append(rate_match(*turbo(c, *qpp_of(K)), E, rv))
    return np.concatenate(out)
