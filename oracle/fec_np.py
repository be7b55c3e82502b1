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


# ================================================================================ decoder
# Receive side of the same chain: turbo rate de-matching into a soft circular buffer and an integer
# max-log-MAP turbo decoder, restated for the checker from TS 36.212 §5.1.3-5.1.4 and the call sites
# pcc_enc_decode (pcc_enc.cpp:215-364: E = 196, rv 0, <= 5 iterations, first CRC16 match under the
# four masks) and pdc_decode_codeblocks (pdc_enc.cpp:291-492: the read position rp / length n_e2 of
# code block r -- block C - gamma read with the shorter length although written with Qm more bits --,
# <= 10 iterations with a CRC early stop after >= 2, the transport-block CRC24A after all block CRCs).
# srsRAN's tdec arithmetic is absent from /root/reference (parity unpinned); the conventions of the
# library's decoder are restated here independently of its code: soft bits added into an int16
# circular buffer with saturation in soft-bit order; branch metric u (L_sys + L_apriori) + p L_par;
# forward / backward metrics renormalised by their maximum each step and floored at -2^28; the
# termination trellis closes the backward recursion; extrinsic = (L - L_sys - L_apriori) * 3 >> 2
# saturated to +-32767; hard decision L > 0 on decoder 2's output.
NEG = -(1 << 28)


def _trellis():
    """NEXT[s, u], PAR[s, u] of the 8-state constituent encoder (_rsc), state s = 4 a_{k-1} +
    2 a_{k-2} + a_{k-3}; tail input / parity of each state (register flushed with a = 0)."""
    nxt = np.zeros((8, 2), np.int64)
    par = np.zeros((8, 2), np.int64)
    for s in range(8):
        r0, r1, r2 = (s >> 2) & 1, (s >> 1) & 1, s & 1
        for u in range(2):
            a = u ^ r1 ^ r2
            par[s, u] = a ^ r0 ^ r2
            nxt[s, u] = (a << 2) | (r0 << 1) | r1
    tail_u = np.array([((s >> 1) & 1) ^ (s & 1) for s in range(8)], np.int64)
    return nxt, par, tail_u


_NXT, _PAR, _TU = _trellis()


def _norm(m):
    return np.maximum(m - m.max(axis=1, keepdims=True), NEG)


def map_decode(A, B, tx, tz):
    """A, B: int64 [nb, K] systematic + a priori / parity; tx, tz: [nb, 3] tail LLRs of this
    constituent code. Returns (L [nb, K], extrinsic [nb, K])."""
    nb, K = A.shape
    alpha = np.full((K + 1, nb, 8), NEG, np.int64)
    alpha[0, :, 0] = 0
    for k in range(K):
        a0 = alpha[k]
        a1 = np.full((nb, 8), NEG, np.int64)
        for s in range(8):
            for u in range(2):
                v = a0[:, s] + (A[:, k] if u else 0) + (B[:, k] if _PAR[s, u] else 0)
                n = _NXT[s, u]
                a1[:, n] = np.maximum(a1[:, n], v)
        alpha[k + 1] = _norm(a1)
    be = np.full((nb, 8), NEG, np.int64)
    be[:, 0] = 0
    for t in (2, 1, 0):
        bn = np.empty((nb, 8), np.int64)
        for s in range(8):
            u = _TU[s]
            bn[:, s] = be[:, _NXT[s, u]] + (tx[:, t] if u else 0) + (tz[:, t] if _PAR[s, u] else 0)
        be = _norm(bn)
    L = np.zeros((nb, K), np.int64)
    for k in range(K - 1, -1, -1):
        m = [np.full(nb, np.iinfo(np.int64).min), np.full(nb, np.iinfo(np.int64).min)]
        bn = np.full((nb, 8), np.iinfo(np.int64).min, np.int64)
        for s in range(8):
            for u in range(2):
                g = (A[:, k] if u else 0) + (B[:, k] if _PAR[s, u] else 0) + be[:, _NXT[s, u]]
                m[u] = np.maximum(m[u], alpha[k][:, s] + g)
                bn[:, s] = np.maximum(bn[:, s], g)
        L[:, k] = m[1] - m[0]
        be = _norm(bn)
    ext = np.clip(((L - A) * 3) >> 2, -32767, 32767)
    return L, ext


def _buffer_map(K):
    """circular-buffer position -> (stream, index) of the rate matcher (-1 for dummy bits)"""
    D = K + 4
    idx = np.arange(D)
    v0, v1, v2 = _subblock(idx, False), _subblock(idx, False), _subblock(idx, True)
    st = np.concatenate([np.zeros(len(v0), np.int64), np.tile([1, 2], len(v1))])
    ix = np.concatenate([v0, np.stack([v1, v2], 1).reshape(-1)]).astype(np.int64)
    st[ix < 0] = -1
    return st, ix


def rate_dematch(llr, K, rv, w=None):
    """soft bits llr (E) added into the int16 circular buffer w (3 Kpi, new if None) from k0(rv),
    skipping dummy positions, saturating; returns w"""
    st, ix = _buffer_map(K)
    Ncb = len(st)
    R = Ncb // 96
    k0 = R * (2 * int(np.ceil(Ncb / (8 * R))) * rv + 2)
    w = np.zeros(Ncb, np.int64) if w is None else w.astype(np.int64)
    valid = np.roll(np.arange(Ncb), -k0)
    valid = valid[st[valid] >= 0]
    for j, v in enumerate(np.asarray(llr, np.int64)):
        p = valid[j % len(valid)]
        w[p] = min(32767, max(-32768, w[p] + v))
    return w


def _streams(w, K):
    st, ix = _buffer_map(K)
    d = np.zeros((3, K + 4), np.int64)
    m = st >= 0
    d[st[m], ix[m]] = w[m]
    return d


def turbo_decode(ws, K, f1, f2, max_iter, check, min_iter=1):
    """ws: list of soft circular buffers of one code-block size K. Iterates decoder 1 / decoder 2;
    after iteration it (>= min_iter) a block whose hard decisions pass check(bits) stops.
    Returns [(ok, bits, iterations)]."""
    d = np.stack([_streams(w, K) for w in ws])  # [nb, 3, K+4]
    sys_, p1, p2 = d[:, 0, :K], d[:, 1, :K], d[:, 2, :K]
    # tails (TS 36.212 §5.1.3.2.2): x_K..K+2 / z_K..K+2 of encoder 1, then x' / z' of encoder 2
    tx1 = np.stack([d[:, 0, K], d[:, 2, K], d[:, 1, K + 1]], 1)
    tz1 = np.stack([d[:, 1, K], d[:, 0, K + 1], d[:, 2, K + 1]], 1)
    tx2 = np.stack([d[:, 0, K + 2], d[:, 2, K + 2], d[:, 1, K + 3]], 1)
    tz2 = np.stack([d[:, 1, K + 2], d[:, 0, K + 3], d[:, 2, K + 3]], 1)
    pi = qpp(K, f1, f2)
    nb = len(ws)
    le2 = np.zeros((nb, K), np.int64)
    out = [None] * nb
    live = np.arange(nb)
    for it in range(1, max_iter + 1):
        apr = np.zeros((len(live), K), np.int64)
        apr[:, pi] = le2[live]                     # deinterleaved extrinsic of decoder 2
        _, le1 = map_decode(sys_[live] + apr, p1[live], tx1[live], tz1[live])
        Ai = sys_[live][:, pi] + le1[:, pi]        # decoder 2 on the interleaved sequence
        L2, e2 = map_decode(Ai, p2[live], tx2[live], tz2[live])
        le2[live] = e2
        bits = np.zeros((len(live), K), np.uint8)
        bits[:, pi] = (L2 > 0).astype(np.uint8)
        keep = []
        for j, b in enumerate(live):
            if it >= min_iter and check(bits[j]):
                out[b] = (True, bits[j], it)
            elif it == max_iter:
                out[b] = (False, bits[j], it)
            else:
                keep.append(j)
        live = live[keep]
        if len(live) == 0:
            break
    return out


def pcc_decode(llr, plcf_type, qpp_of):
    """-> (ok, plcf bits, (closed_loop, beamforming), iterations)"""
    nb = 40 if plcf_type == 1 else 80
    K = nb + 16
    w = rate_dematch(llr[:196], K, 0)
    masks = [(0, 0, 0x0000), (1, 0, 0x5555), (0, 1, 0xAAAA), (1, 1, 0xFFFF)]
    hit = {}

    def check(bits):
        r = crc(bits[:nb], CRC16)
        for cl, bf, m in masks:
            if np.array_equal(r ^ np.array([(m >> (15 - i)) & 1 for i in range(16)], np.uint8), bits[nb:K]):
                hit["m"] = (cl, bf)
                return True
        return False

    ok, bits, it = turbo_decode([w], K, *qpp_of(K), 5, check)[0]
    return ok, bits[:nb], hit.get("m") if ok else None, it


def pdc_decode(llr, tbs, Z, Qm, G, rv, qpp_of):
    """one-shot decode of the G descrambled soft bits -> (ok, tb bits, total iterations)"""
    C, Ks, F = cbsegm(tbs, Z)
    assert F == 0
    Gp = G // Qm
    gamma = Gp % C
    n_e = Qm * (Gp // C)
    llr = np.asarray(llr, np.int64)
    blocks = []
    for r, K in enumerate(Ks):
        rp, n_e2 = r * n_e, n_e
        if r > C - gamma:
            n_e2 = n_e + Qm
            rp = (C - gamma) * n_e + (r - (C - gamma)) * n_e2
        blocks.append(rate_dematch(llr[rp:rp + n_e2], K, rv))
    res = [None] * C
    for K in sorted(set(Ks)):
        ids = [r for r in range(C) if Ks[r] == K]
        if C > 1:
            check = lambda b: np.array_equal(crc(b[:-24], CRC24B), b[-24:])
        else:
            check = lambda b: np.array_equal(crc(b[:tbs], CRC24A), b[tbs:tbs + 24])
        for r, o in zip(ids, turbo_decode([blocks[r] for r in ids], K, *qpp_of(K), 10, check, min_iter=2)):
            res[r] = o
    its = sum(o[2] for o in res)
    b = np.concatenate([o[1][: (K - 24 if C > 1 else K)] for o, K in zip(res, Ks)])
    ok = all(o[0] for o in res)
    if ok and C > 1:
        ok = np.array_equal(crc(b[:tbs], CRC24A), b[tbs:tbs + 24])
    return ok, b[:tbs], its
