"""Host channel coding of libdnrp.so (include/dnrp.h, csrc/host/fec.cpp) — the reference's fec_t
(lib/src/phy/fec/fec.cpp:28-148) without the scrambling, which the GPU path applies:

  pcc_encode  <- fec_t::encode_plcf      (pcc_enc.cpp:145-208)
  pcc_decode  <- fec_t::decode_plcf_test (pcc_enc.cpp:215-364)
  pdc_encode  <- fec_t::encode_tb        (pdc_enc.cpp:127-229)
  pdc_decode  <- fec_t::decode_tb        (pdc_enc.cpp:291-492), HarqRx <- harq::buffer_rx_t
  pdc_decode_batch: decode_tb of many packets on the GPU (kernels/fec.hip), same arithmetic
  pdc_encode_batch: encode_tb of many packets on the GPU, bit-exact with pdc_encode
  pcc_decode_batch: decode_plcf_test of many packets on the GPU, same arithmetic as pcc_decode
  cbsegm      <- sp3::fix::srsran_cbsegm_FIX (sections_part3/fix/cbsegm.cpp:65-123)

Bits are numpy uint8 arrays packed MSB first, LLRs numpy int16 (positive = bit 1).
"""
import ctypes as C

import numpy as np

from . import DnrpError, lib as _lib

CRC16, CRC24A, CRC24B = 0, 1, 2
P = C.c_void_p


class CbSegm(C.Structure):
    _fields_ = [(n, C.c_uint32) for n in ("tbs", "Z", "C", "C1", "C2", "K1", "K2", "K1_idx", "K2_idx", "F")]

    def as_dict(self):
        return {n: int(getattr(self, n)) for n, _ in self._fields_}


class FecCfg(C.Structure):
    """sp3::fec_cfg_t (sections_part3/derivative/fec_cfg.hpp)"""
    _fields_ = [(n, C.c_uint32) for n in ("PLCF_type", "closed_loop", "beamforming", "N_TB_bits", "N_bps", "rv", "G",
                                         "network_id", "Z")]


_ready = False


def lib():
    global _ready
    L = _lib()
    if not _ready:
        u32p = C.POINTER(C.c_uint32)
        L.dnrp_crc.argtypes = [P, C.c_uint32, C.c_uint32, u32p]
        L.dnrp_fec_cbsegm.argtypes = [C.c_uint32, C.c_uint32, C.POINTER(CbSegm)]
        L.dnrp_fec_cb_size.argtypes = [C.c_uint32, u32p, u32p, u32p]
        L.dnrp_pcc_encode.argtypes = [P, C.c_uint32, C.c_uint32, C.c_uint32, P]
        L.dnrp_pcc_decode.argtypes = [P, C.c_uint32, P, u32p, u32p, u32p]
        L.dnrp_pdc_encode.argtypes = [C.POINTER(FecCfg), P, P]
        L.dnrp_pdc_decode.argtypes = [P, C.POINTER(FecCfg), P, C.c_uint32, P, u32p]
        L.dnrp_harq_rx_create.argtypes = [C.c_uint32, C.c_uint32, C.POINTER(P)]
        L.dnrp_harq_rx_reset.argtypes = [P]
        L.dnrp_harq_rx_destroy.argtypes = [P]
        L.dnrp_pdc_decode_batch.argtypes = [P, C.c_uint32, P, P, C.c_uint32, P, C.c_uint32, P, P, P]
        L.dnrp_pdc_encode_batch.argtypes = [P, C.c_uint32, P, P, C.c_uint32, P, C.c_uint32, P]
        L.dnrp_pcc_decode_batch.argtypes = [P, C.c_uint32, P, P, C.c_uint32, P, C.c_uint32, P, P, P]
        L.dnrp_pdc_decode_batch_harq.argtypes = [P, C.c_uint32, P, P, C.c_uint32, P, C.c_uint64, P, C.c_uint32, P,
                                                 C.c_uint32, P, P, P]
        L.dnrp_pcc_encode_batch.argtypes = [P, C.c_uint32, P, P, P, P, C.c_uint32, P, C.c_uint32, P]
        L.dnrp_pdc_softbuffer_size.argtypes = [C.c_uint32, C.c_uint32, C.POINTER(C.c_uint64), C.POINTER(C.c_uint32)]
        _ready = True
    return L


def _chk(rc, what):
    if rc < 0:
        raise DnrpError(rc, what)
    return rc


def _ptr(a):
    return a.ctypes.data_as(P)


def crc(data, nbits, kind):
    data = np.ascontiguousarray(data, dtype=np.uint8)
    assert data.size * 8 >= nbits
    out = C.c_uint32()
    _chk(lib().dnrp_crc(_ptr(data), nbits, kind, C.byref(out)), "dnrp_crc")
    return out.value


def cbsegm(N_TB_bits, Z):
    out = CbSegm()
    _chk(lib().dnrp_fec_cbsegm(N_TB_bits, Z, C.byref(out)), "dnrp_fec_cbsegm")
    return out.as_dict()


def cb_size(idx):
    K, f1, f2 = C.c_uint32(), C.c_uint32(), C.c_uint32()
    _chk(lib().dnrp_fec_cb_size(idx, C.byref(K), C.byref(f1), C.byref(f2)), "dnrp_fec_cb_size")
    return K.value, f1.value, f2.value


def pcc_encode(plcf, plcf_type, closed_loop=False, beamforming=False):
    plcf = np.ascontiguousarray(plcf, dtype=np.uint8)
    assert plcf.size == (5 if plcf_type == 1 else 10)
    d = np.zeros(25, np.uint8)
    _chk(lib().dnrp_pcc_encode(_ptr(plcf), plcf_type, int(closed_loop), int(beamforming), _ptr(d)), "dnrp_pcc_encode")
    return d


def pcc_decode(llr, plcf_type_test):
    """-> (ok, plcf bytes, closed_loop, beamforming, iterations)"""
    llr = np.ascontiguousarray(llr, dtype=np.int16)
    assert llr.size == 196
    plcf = np.zeros(10, np.uint8)
    cl, bf, it = C.c_uint32(), C.c_uint32(), C.c_uint32()
    ok = _chk(lib().dnrp_pcc_decode(_ptr(llr), plcf_type_test, _ptr(plcf), C.byref(cl), C.byref(bf), C.byref(it)),
              "dnrp_pcc_decode")
    return bool(ok), plcf[:5 if plcf_type_test == 1 else 10], bool(cl.value), bool(bf.value), it.value


def fec_cfg(N_TB_bits, N_bps, G, Z=6144, rv=0, PLCF_type=1, network_id=0):
    return FecCfg(PLCF_type, 0, 0, N_TB_bits, N_bps, rv, G, network_id, Z)


def pdc_encode(cfg, tb):
    tb = np.ascontiguousarray(tb, dtype=np.uint8)
    assert tb.size == cfg.N_TB_bits // 8
    d = np.zeros((cfg.G + 7) // 8, np.uint8)
    _chk(lib().dnrp_pdc_encode(C.byref(cfg), _ptr(tb), _ptr(d)), "dnrp_pdc_encode")
    return d


class HarqRx:
    """harq::buffer_rx_t: softbuffer kept across redundancy versions of one transport block"""

    def __init__(self, N_TB_bits_max, Z=6144):
        self.h = P()
        _chk(lib().dnrp_harq_rx_create(N_TB_bits_max, Z, C.byref(self.h)), "dnrp_harq_rx_create")

    def reset(self):
        _chk(lib().dnrp_harq_rx_reset(self.h), "dnrp_harq_rx_reset")

    def __del__(self):
        if getattr(self, "h", None):
            lib().dnrp_harq_rx_destroy(self.h)
            self.h = None


def pdc_decode(cfg, llr, hb=None, n_llr=None):
    """-> (crc ok, tb bytes, turbo iterations)"""
    llr = np.ascontiguousarray(llr, dtype=np.int16)
    n_llr = cfg.G if n_llr is None else n_llr
    assert llr.size >= n_llr
    tb = np.zeros(cfg.N_TB_bits // 8, np.uint8)
    it = C.c_uint32()
    ok = _chk(lib().dnrp_pdc_decode(hb.h if hb else None, C.byref(cfg), _ptr(llr), n_llr, _ptr(tb), C.byref(it)),
              "dnrp_pdc_decode")
    return bool(ok), tb, it.value


def pdc_decode_batch(phy, cfgs, llr, tb, stream=None):
    """GPU turbo decoding of len(cfgs) transport blocks (one-shot). llr: int16 device tensor [m][>= G],
    tb: uint8 device tensor [m][>= N_TB_bits/8 + 3] (decoded TB + its CRC24A).
    -> (crc_ok bool array [m], iterations array [m])"""
    import torch
    from . import _stream_ptr
    m = len(cfgs)
    assert llr.dtype == torch.int16 and llr.dim() == 2 and llr.is_contiguous() and llr.shape[0] >= m and llr.is_cuda
    assert tb.dtype == torch.uint8 and tb.dim() == 2 and tb.is_contiguous() and tb.shape[0] >= m and tb.is_cuda
    assert all(c.G <= llr.shape[1] and c.N_TB_bits // 8 + 3 <= tb.shape[1] for c in cfgs)
    arr = (FecCfg * max(m, 1))(*cfgs)
    ok = np.zeros(m, np.uint8)
    it = np.zeros(m, np.uint32)
    _chk(lib().dnrp_pdc_decode_batch(phy._ctx, m, arr, C.c_void_p(llr.data_ptr()), llr.shape[1],
                                     C.c_void_p(tb.data_ptr()), tb.shape[1], _ptr(ok), _ptr(it), _stream_ptr(stream)),
         "dnrp_pdc_decode_batch")
    return ok.astype(bool), it


def pdc_encode_batch(phy, cfgs, tb, d, stream=None):
    """GPU channel encoding of len(cfgs) transport blocks: tb uint8 device tensor [m][>= N_TB_bits/8]
    -> d uint8 device tensor [m][>= ceil(G/8)] (unscrambled d-bits, dnrp_tx_batch's pdc_d rows)."""
    import torch
    from . import _stream_ptr
    m = len(cfgs)
    assert tb.dtype == torch.uint8 and tb.dim() == 2 and tb.is_contiguous() and tb.shape[0] >= m and tb.is_cuda
    assert d.dtype == torch.uint8 and d.dim() == 2 and d.is_contiguous() and d.shape[0] >= m and d.is_cuda
    assert all(c.N_TB_bits // 8 <= tb.shape[1] and (c.G + 7) // 8 <= d.shape[1] for c in cfgs)
    arr = (FecCfg * max(m, 1))(*cfgs)
    _chk(lib().dnrp_pdc_encode_batch(phy._ctx, m, arr, C.c_void_p(tb.data_ptr()), tb.shape[1],
                                     C.c_void_p(d.data_ptr()), d.shape[1], _stream_ptr(stream)), "dnrp_pdc_encode_batch")


def pcc_decode_batch(phy, plcf_types, llr, plcf, stream=None):
    """GPU PLCF decoding: llr int16 device tensor [n][>= 196] (dnrp_rx_pcc_batch's pcc_llr), plcf uint8
    device tensor [n][>= 10]. -> (result uint8 [n]: 0 = no PLCF, 1 + CRC mask index; iterations [n])"""
    import torch
    from . import _stream_ptr
    n = len(plcf_types)
    assert llr.dtype == torch.int16 and llr.dim() == 2 and llr.is_contiguous() and llr.shape[0] >= n and llr.is_cuda
    assert llr.shape[1] >= 196
    assert plcf.dtype == torch.uint8 and plcf.dim() == 2 and plcf.is_contiguous() and plcf.shape[0] >= n and plcf.is_cuda
    assert plcf.shape[1] >= 10
    types = np.ascontiguousarray(plcf_types, dtype=np.uint32)
    res = np.zeros(n, np.uint8)
    it = np.zeros(n, np.uint32)
    _chk(lib().dnrp_pcc_decode_batch(phy._ctx, n, _ptr(types), C.c_void_p(llr.data_ptr()), llr.shape[1],
                                     C.c_void_p(plcf.data_ptr()), plcf.shape[1], _ptr(res), _ptr(it),
                                     _stream_ptr(stream)), "dnrp_pcc_decode_batch")
    return res, it


def softbuffer_size(N_TB_bits, Z=6144):
    """-> (softbuffer entries, code blocks) of one transport block"""
    e, c = C.c_uint64(), C.c_uint32()
    _chk(lib().dnrp_pdc_softbuffer_size(N_TB_bits, Z, C.byref(e), C.byref(c)), "dnrp_pdc_softbuffer_size")
    return e.value, c.value


def pdc_decode_batch_harq(phy, cfgs, llr, softbuf, cb_crc, tb, stream=None):
    """GPU turbo decoding with HARQ soft combining: softbuf int16 [m][>= entries], cb_crc uint8 [m][>= C]
    device tensors zeroed for a new transport block and kept across its redundancy versions; tb as for
    pdc_decode_batch (same rows every redundancy version). -> (crc_ok [m], iterations [m])"""
    import torch
    from . import _stream_ptr
    m = len(cfgs)
    for t, dt in ((llr, torch.int16), (softbuf, torch.int16), (cb_crc, torch.uint8), (tb, torch.uint8)):
        assert t.dtype == dt and t.dim() == 2 and t.is_contiguous() and t.shape[0] >= m and t.is_cuda
    arr = (FecCfg * max(m, 1))(*cfgs)
    ok = np.zeros(m, np.uint8)
    it = np.zeros(m, np.uint32)
    _chk(lib().dnrp_pdc_decode_batch_harq(phy._ctx, m, arr, C.c_void_p(llr.data_ptr()), llr.shape[1],
                                          C.c_void_p(softbuf.data_ptr()), softbuf.shape[1],
                                          C.c_void_p(cb_crc.data_ptr()), cb_crc.shape[1], C.c_void_p(tb.data_ptr()),
                                          tb.shape[1], _ptr(ok), _ptr(it), _stream_ptr(stream)),
         "dnrp_pdc_decode_batch_harq")
    return ok.astype(bool), it


def pcc_encode_batch(phy, plcf_types, plcf, d, closed_loop=None, beamforming=None, stream=None):
    """GPU PLCF encoding: plcf uint8 device tensor [n][>= 5 / 10] -> d uint8 device tensor [n][>= 25]
    (unscrambled PCC d-bits, dnrp_tx_batch's pcc_d rows)."""
    import torch
    from . import _stream_ptr
    n = len(plcf_types)
    assert plcf.dtype == torch.uint8 and plcf.dim() == 2 and plcf.is_contiguous() and plcf.shape[0] >= n and plcf.is_cuda
    assert d.dtype == torch.uint8 and d.dim() == 2 and d.is_contiguous() and d.shape[0] >= n and d.is_cuda
    assert d.shape[1] >= 25 and plcf.shape[1] >= 5 * max(plcf_types, default=1)
    t = np.ascontiguousarray(plcf_types, dtype=np.uint32)
    cl = None if closed_loop is None else np.ascontiguousarray(closed_loop, dtype=np.uint32)
    bf = None if beamforming is None else np.ascontiguousarray(beamforming, dtype=np.uint32)
    _chk(lib().dnrp_pcc_encode_batch(phy._ctx, n, _ptr(t), None if cl is None else _ptr(cl),
                                     None if bf is None else _ptr(bf), C.c_void_p(plcf.data_ptr()), plcf.shape[1],
                                     C.c_void_p(d.data_ptr()), d.shape[1], _stream_ptr(stream)), "dnrp_pcc_encode_batch")
