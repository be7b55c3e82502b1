"""Python host binding of libdnrp.so (include/dnrp.h) — the MI355X DECT NR+ lower PHY.

Mirrors the reference's per-worker PHY objects with batched calls:
  Phy.tx_batch      <- tx_t::generate_tx_packet      (lib/src/phy/tx/tx.cpp:165-314)
  Phy.rx_sync_batch <- sync_chunk_t::search()         (lib/src/phy/rx/sync/sync_chunk.cpp:143-279)
  Phy.rx_pcc_batch  <- rx_synced_t::demoddecod_rx_pcc (rx_synced.cpp:186-323)
  Phy.rx_pdc_batch  <- rx_synced_t::demoddecod_rx_pdc (rx_synced.cpp:325-436)
  Phy.add_network_id <- tx_rx_t::add_new_network_id (tx_rx.hpp:52)
Device buffers are torch tensors on the context's device (torch is plumbing only: allocation
and streams). Errors raise DnrpError carrying the C error code; the library must be present —
there is no fallback path.
"""
import ctypes as C
import os

import numpy as np

# torch ships its own HIP runtime (torch/lib/libamdhip64.so, SONAME libamdhip64.so.7). Loading it
# first lets libdnrp.so bind to the same runtime instead of a second copy from /opt/rocm, so
# device pointers and streams from torch tensors are valid inside the library.
import torch  # noqa: F401

_HERE = os.path.dirname(os.path.abspath(__file__))
# DNRP_LIB: an alternative build of the library (tools/build_variant.sh, A/B experiments)
LIB_PATH = os.environ.get("DNRP_LIB") or os.path.join(os.path.dirname(_HERE), "libdnrp.so")


class DnrpError(RuntimeError):
    def __init__(self, code, what):
        super().__init__(f"{what}: {code} ({strerror(code)})")
        self.code = code


class Cfg(C.Structure):
    _fields_ = [("u_max", C.c_uint32), ("b_max", C.c_uint32), ("N_TX_max", C.c_uint32), ("os_min", C.c_uint32),
                ("L", C.c_uint32), ("M", C.c_uint32), ("chestim_mode_lr", C.c_uint32),
                ("chestim_lr_stride", C.c_uint32), ("max_batch", C.c_uint32), ("device", C.c_int32)]


class PsDef(C.Structure):
    _fields_ = [(n, C.c_uint32) for n in ("u", "b", "PacketLengthType", "PacketLength", "tm_mode_index",
                                         "mcs_index", "Z")]


PS_FIELDS = ["N_PACKET_symb", "N_DF_symb", "N_PDC_subc", "N_DRS_subc", "G", "N_PDC_bits", "N_TB_bits", "N_TB_byte",
             "C", "N_samples_STF", "N_samples_STF_CP_only", "N_samples_DF", "N_samples_GI",
             "N_samples_packet_no_GI", "N_samples_packet", "N_bps", "N_eff_TX", "N_SS", "N_TS", "N_TX", "N_b_DFT",
             "N_b_OCC", "N_b_DFT_os", "N_samples_packet_no_GI_os_rs", "N_samples_packet_os_rs"]


class PacketSizes(C.Structure):
    _fields_ = [(n, C.c_uint32) for n in PS_FIELDS]

    def as_dict(self):
        return {n: int(getattr(self, n)) for n in PS_FIELDS}


class TxDesc(C.Structure):
    _fields_ = [("codebook_index", C.c_uint32), ("network_id", C.c_uint32), ("plcf_type", C.c_uint32),
                ("GI_percentage", C.c_uint32), ("DAC_scale", C.c_float), ("iq_phase_rad", C.c_float),
                ("iq_phase_increment_s2s_post_resampling_rad", C.c_float), ("optimal_scaling_DAC", C.c_uint32)]


class SyncReport(C.Structure):
    _fields_ = [("fine_peak_time", C.c_int64), ("cfo_fractional_rad", C.c_float), ("cfo_integer_rad", C.c_float),
                ("u", C.c_uint32), ("b", C.c_uint32), ("N_eff_TX", C.c_uint32), ("window", C.c_uint32),
                ("rms", C.c_float * 8)]

    AUTO_WINDOW = 0xFFFFFFFF

    def __init__(self, fine_peak_time=0, cfo_fractional_rad=0.0, cfo_integer_rad=0.0, u=0, b=0, N_eff_TX=0,
                 window=None, rms=None):
        # window omitted: the report's own index in the batch (one packet per window, resolved by
        # Phy.rx_pcc_batch); rms omitted: no sync RMS, the RX estimates every antenna's
        super().__init__(fine_peak_time, cfo_fractional_rad, cfo_integer_rad, u, b, N_eff_TX,
                         SyncReport.AUTO_WINDOW if window is None else window,
                         (C.c_float * 8)(*(list(rms or []) + [0.0] * 8)[:8]))


class SyncCfg(C.Structure):
    _fields_ = [("u", C.c_uint32), ("b", C.c_uint32), ("N_ant_limited", C.c_uint32), ("chunk_len", C.c_uint32),
                ("max_reports", C.c_uint32)]


class SyncResult(C.Structure):
    _fields_ = [("found", C.c_uint32), ("detection_ant_idx", C.c_uint32), ("detection_rms", C.c_float),
                ("detection_metric", C.c_float), ("detection_time_local", C.c_uint32),
                ("detection_time_with_jump_back_local", C.c_uint32), ("coarse_peak_time_local", C.c_uint32),
                ("fine_peak_time_local", C.c_uint32), ("coarse_peak_time", C.c_int64), ("fine_peak_time", C.c_int64),
                ("coarse_peak_array", C.c_float * 8), ("rms_array", C.c_float * 8), ("cfo_fractional_rad", C.c_float),
                ("cfo_integer_rad", C.c_float), ("u", C.c_uint32), ("b", C.c_uint32), ("N_eff_TX", C.c_uint32),
                ("reserved", C.c_uint32), ("fine_peak_metric", C.c_float * 4), ("fine_peak_index", C.c_uint32 * 4)]


def _np_dtype(st):
    names, formats, offsets = [], [], []
    for name, ct in st._fields_:
        names.append(name)
        if hasattr(ct, "_length_"):
            formats.append((np.dtype(ct._type_), (ct._length_,)))
        else:
            formats.append(np.dtype(ct))
        offsets.append(getattr(st, name).offset)
    return np.dtype({"names": names, "formats": formats, "offsets": offsets, "itemsize": C.sizeof(st)})


SYNC_RESULT_DTYPE = _np_dtype(SyncResult)
SYNC_REPORT_DTYPE = _np_dtype(SyncReport)


def sync_reports(results, windows=None):
    """dnrp_sync_result rows -> dnrp_sync_report array for rx_pcc_batch (vectorised). windows: the
    sync window of each row (default: row i was found in window i)."""
    r = np.zeros(len(results), SYNC_REPORT_DTYPE)
    for k in ("fine_peak_time", "cfo_fractional_rad", "cfo_integer_rad", "u", "b", "N_eff_TX"):
        r[k] = results[k]
    r["rms"] = results["rms_array"]
    r["window"] = np.arange(len(results)) if windows is None else windows
    return r


def found_reports(res, n_found):
    """All packets a sync batch found: res [n_win, max_reports] + n_found [n_win] -> the
    dnrp_sync_report array of the found packets in window order (window = its sync window)."""
    n_found = np.asarray(n_found).astype(np.int64)
    if len(n_found) and (n_found == 1).all():  # one packet per window: a view, no record gather
        return sync_reports(res[:, 0], np.arange(len(n_found)))
    win = np.repeat(np.arange(len(n_found)), n_found)
    # report index within its window: position minus the window's first position (vectorised)
    k = np.arange(len(win), dtype=np.int64) - np.repeat(np.cumsum(n_found) - n_found, n_found)
    return sync_reports(res[win, k], win)


class PccReport(C.Structure):
    _fields_ = [("snr_dB", C.c_float), ("cfo_fractional_rad", C.c_float), ("sto_fractional", C.c_float),
                ("rms", C.c_float * 8)]


class PdcReport(C.Structure):
    _fields_ = [("snr_dB", C.c_float), ("mimo_N_RX", C.c_uint32), ("mimo_N_TS_other", C.c_uint32),
                ("tm_3_7_beamforming_idx", C.c_uint32), ("tm_3_7_beamforming_reciprocal_idx", C.c_uint32)]


class PdcReq(C.Structure):
    """dnrp_pdc_req: PLCF-announced psdef, slot in the preceding PCC batch, network ID, PLCF type."""
    _fields_ = [("psdef", PsDef), ("pcc_index", C.c_uint32), ("network_id", C.c_uint32), ("plcf_type", C.c_uint32)]


class SyncStreamState(C.Structure):
    """dnrp_sync_stream_state: baton_t's uniqueness state across dnrp_rx_sync_stream calls."""
    _fields_ = [("sync_time_last", C.c_int64), ("sync_time_unique_limit", C.c_int64), ("packets", C.c_uint64),
                ("not_unique", C.c_uint64)]


CH_AWGN, CH_FLAT, CH_DOUBLY = 0, 1, 2
CH_NOISELESS_DB = 1000.0
CH_N_SIN = 40  # WIRELESS_CHANNEL_DOUBLY_NOF_SINUSOIDS (link.hpp:126)


class ChannelCfg(C.Structure):
    """dnrp_channel_cfg: simulated wireless channel (simulation/wireless channel_{awgn,flat,doubly})."""
    _fields_ = [("kind", C.c_uint32), ("pdp_idx", C.c_uint32), ("tau_rms_ns", C.c_float), ("fD_Hz", C.c_float),
                ("samp_rate", C.c_uint32), ("large_scale", C.c_float), ("snr_db", C.c_float),
                ("net_bw_norm", C.c_float), ("seed", C.c_uint64)]


EXPORTS = ["dnrp_ctx_create", "dnrp_ctx_destroy", "dnrp_add_network_id", "dnrp_get_packet_sizes",
           "dnrp_compute_packet_sizes", "dnrp_tx_batch", "dnrp_rx_sync_batch",
           "dnrp_rx_pcc_batch", "dnrp_rx_pdc_batch", "dnrp_sync", "dnrp_last_kernel_ms", "dnrp_kernel_time_total",
           "dnrp_strerror", "dnrp_get_radio_device_class", "dnrp_query_param", "dnrp_param_name",
           "dnrp_ring_gather", "dnrp_sync_stream_init", "dnrp_sync_stream_window", "dnrp_rx_sync_stream",
           "dnrp_channel_batch", "dnrp_channel_realization", "dnrp_tx_transmit_length", "dnrp_tx_packet_json",
           "dnrp_rx_packet_json", "dnrp_crc", "dnrp_fec_cbsegm", "dnrp_fec_cb_size", "dnrp_pcc_encode",
           "dnrp_pcc_decode", "dnrp_pdc_encode", "dnrp_pdc_decode", "dnrp_harq_rx_create", "dnrp_harq_rx_reset",
           "dnrp_harq_rx_destroy", "dnrp_pdc_decode_batch", "dnrp_pdc_encode_batch",
           "dnrp_pcc_decode_batch", "dnrp_pdc_decode_batch_harq", "dnrp_pdc_softbuffer_size",
           "dnrp_pcc_encode_batch", "dnrp_query_table", "dnrp_ctx_set_rx_mode"]

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"libdnrp.so not built at {LIB_PATH} (run __graft_entry__.build())")
        L = C.CDLL(LIB_PATH)
        P = C.c_void_p
        L.dnrp_ctx_create.argtypes = [C.POINTER(Cfg), C.POINTER(P)]
        L.dnrp_ctx_destroy.argtypes = [P]
        L.dnrp_add_network_id.argtypes = [P, C.c_uint32]
        L.dnrp_get_packet_sizes.argtypes = [P, C.POINTER(PsDef), C.POINTER(PacketSizes)]
        L.dnrp_compute_packet_sizes.argtypes = [C.POINTER(Cfg), C.POINTER(PsDef), C.POINTER(PacketSizes)]
        L.dnrp_tx_batch.argtypes = [P, C.POINTER(PsDef), C.c_uint32, C.POINTER(TxDesc), P, P, C.c_uint32, P,
                                    C.c_uint32, P]
        L.dnrp_rx_sync_batch.argtypes = [P, C.POINTER(SyncCfg), C.c_uint32, P, C.c_uint64, C.c_uint64, C.c_uint32,
                                         P, P, P]
        L.dnrp_rx_pcc_batch.argtypes = [P, C.c_uint32, P, P, C.c_uint32, C.c_uint32, P,
                                        C.POINTER(PccReport), P]
        L.dnrp_rx_pdc_batch.argtypes = [P, C.c_uint32, C.POINTER(PdcReq), P, C.c_uint32, C.c_uint32, P, C.c_uint32,
                                        C.POINTER(PdcReport), P]
        L.dnrp_sync.argtypes = [P, P]
        L.dnrp_ctx_set_rx_mode.argtypes = [P, C.c_uint32]
        L.dnrp_ring_gather.argtypes = [P, P, C.c_uint64, C.c_uint64, C.c_uint32, C.c_uint32, P, C.c_uint32, P, P]
        L.dnrp_channel_batch.argtypes = [P, C.POINTER(ChannelCfg), C.c_uint32, C.c_uint32, P, C.c_uint32, C.c_uint32, P, P,
                                         P, C.c_uint32, P]
        L.dnrp_channel_realization.argtypes = [C.POINTER(ChannelCfg), C.c_uint32, C.c_uint32, C.c_uint32,
                                               C.POINTER(C.c_uint32), P, P, P, P, P]
        L.dnrp_tx_transmit_length.argtypes = [C.POINTER(Cfg), C.POINTER(PsDef), C.c_uint32, C.POINTER(C.c_uint32)]
        L.dnrp_tx_packet_json.argtypes = [C.POINTER(Cfg), C.POINTER(PsDef), C.POINTER(TxDesc), C.c_uint32, C.c_uint64,
                                          C.c_int64, P, P, P, C.c_uint32, C.c_char_p]
        L.dnrp_rx_packet_json.argtypes = [C.POINTER(Cfg), C.c_uint32, P, C.c_uint32, C.POINTER(PccReport),
                                          C.POINTER(PdcReport), C.c_char_p]
        L.dnrp_sync_stream_init.argtypes = [P, C.POINTER(SyncCfg), C.POINTER(SyncStreamState)]
        L.dnrp_sync_stream_window.argtypes = [P, C.POINTER(SyncCfg)]
        L.dnrp_sync_stream_window.restype = C.c_uint32
        L.dnrp_rx_sync_stream.argtypes = [P, C.POINTER(SyncCfg), P, C.c_uint64, C.c_uint64, C.c_int64, C.c_uint32,
                                          C.POINTER(SyncStreamState), P, C.POINTER(C.c_uint32), P, P]
        L.dnrp_last_kernel_ms.argtypes = [P, C.c_char_p, C.POINTER(C.c_float)]
        L.dnrp_kernel_time_total.argtypes = [P, C.c_char_p, C.POINTER(C.c_float), C.POINTER(C.c_uint32), C.c_int]
        L.dnrp_query_table.argtypes = [C.c_char_p, P, C.c_uint32, P, C.c_uint32]
        L.dnrp_strerror.argtypes = [C.c_int]
        L.dnrp_strerror.restype = C.c_char_p
        _lib = L
    return _lib


def strerror(code):
    return lib().dnrp_strerror(int(code)).decode()


def _chk(rc, what):
    if rc != 0:
        raise DnrpError(rc, what)


def psdef(u, b, plt, pl, tm, mcs, Z=6144):
    return PsDef(u, b, plt, pl, tm, mcs, Z)


def compute_packet_sizes(ps, u_max=None, b_max=None, os_min=1, L=10, M=9):
    """Context-free packet geometry (host only). With u_max/b_max the oversampled fields are set."""
    out = PacketSizes()
    cfg = Cfg(u_max, b_max, 1, os_min, L, M, 1, 2, 1, 0) if u_max else None
    rc = lib().dnrp_compute_packet_sizes(C.byref(cfg) if cfg else None, C.byref(ps), C.byref(out))
    if rc != 0:
        raise DnrpError(rc, "dnrp_compute_packet_sizes")
    return out.as_dict()


def query_table(name, *args):
    """Host-only: a literal table the library builds its device tables from (dnrp_query_table) as a
    float32 array."""
    a = np.ascontiguousarray(np.asarray(args, dtype=np.uint32))
    ap = C.c_void_p(a.ctypes.data) if len(a) else None
    n = lib().dnrp_query_table(str(name).encode(), ap, len(a), None, 0)
    if n < 0:
        raise DnrpError(n, f"dnrp_query_table({name}, {args})")
    out = np.zeros(max(1, n), np.float32)
    _chk(min(0, lib().dnrp_query_table(str(name).encode(), ap, len(a), C.c_void_p(out.ctypes.data), n)),
         "dnrp_query_table")
    return out[:n]


def channel_realization(cfg, window, n_tx, n_rx):
    """Host-only: window `window`'s link realisation of a ChannelCfg (dnrp_channel_realization):
    dict with delay / amp [n_rx, n_tx, taps], period / phase_rev [n_rx, n_tx, taps, 40], coef [n_rx, n_tx]."""
    nt = C.c_uint32()
    _chk(lib().dnrp_channel_realization(C.byref(cfg), window, n_tx, n_rx, C.byref(nt), None, None, None, None, None),
         "dnrp_channel_realization")
    t = max(1, nt.value)
    delay = np.zeros((n_rx, n_tx, t), np.int32)
    amp = np.zeros((n_rx, n_tx, t), np.float32)
    period = np.zeros((n_rx, n_tx, t, CH_N_SIN), np.int64)
    phase = np.zeros((n_rx, n_tx, t, CH_N_SIN), np.float64)
    coef = np.zeros((n_rx, n_tx, 2), np.float32)
    _chk(lib().dnrp_channel_realization(C.byref(cfg), window, n_tx, n_rx, C.byref(nt), C.c_void_p(delay.ctypes.data),
                                        C.c_void_p(amp.ctypes.data), C.c_void_p(period.ctypes.data),
                                        C.c_void_p(phase.ctypes.data), C.c_void_p(coef.ctypes.data)),
         "dnrp_channel_realization")
    k = nt.value
    return {"delay": delay[..., :k], "amp": amp[..., :k], "period": period[:, :, :k], "phase_rev": phase[:, :, :k],
            "coef": coef[..., 0] + 1j * coef[..., 1]}


def _host_cfg(u_max, b_max, n_ant, os_min=1, L=10, M=9):
    return Cfg(u_max, b_max, n_ant, os_min, L, M, 1, 2, 1, 0)


def tx_transmit_length(ps, GI_percentage, u_max, b_max, os_min=1, L=10, M=9):
    """Host-only: N_samples_transmit_os_rs (tx.cpp:555-566) of a packet configuration."""
    out = C.c_uint32()
    _chk(lib().dnrp_tx_transmit_length(C.byref(_host_cfg(u_max, b_max, 1, os_min, L, M)), C.byref(ps), GI_percentage,
                                       C.byref(out)), "dnrp_tx_transmit_length")
    return int(out.value)


def tx_packet_json(path, ps, desc, pcc_d, pdc_d, iq, u_max, b_max, n_tx, os_min=1, L=10, M=9, rv=0, tx_order_id=0,
                   tx_time_64=0):
    """Host-only: tx_t::write_all_data_to_json of one packet. pcc_d / pdc_d uint8 (packed d-bits),
    iq complex64 [N_TX, S] (a host copy of the dnrp_tx_batch output row)."""
    pcc = np.ascontiguousarray(pcc_d, np.uint8)
    pdc = np.ascontiguousarray(pdc_d, np.uint8)
    x = np.ascontiguousarray(iq, np.complex64)
    _chk(lib().dnrp_tx_packet_json(C.byref(_host_cfg(u_max, b_max, n_tx, os_min, L, M)), C.byref(ps), C.byref(desc), rv,
                                   tx_order_id, tx_time_64, C.c_void_p(pcc.ctypes.data), C.c_void_p(pdc.ctypes.data),
                                   C.c_void_p(x.ctypes.data), x.shape[1], str(path).encode()), "dnrp_tx_packet_json")


def rx_packet_json(path, sync_result, u_max, b_max, n_ant, mcs_index, pcc_report=None, pdc_report=None, os_min=1, L=10,
                   M=9, worker_id=0):
    """Host-only: the RADIO/PHY part of worker_tx_rx_t::collect_and_write_json for one packet."""
    r = np.ascontiguousarray(np.asarray(sync_result, dtype=SYNC_RESULT_DTYPE).reshape(1))
    _chk(lib().dnrp_rx_packet_json(C.byref(_host_cfg(u_max, b_max, n_ant, os_min, L, M)), worker_id,
                                   C.c_void_p(r.ctypes.data), mcs_index, C.byref(pcc_report) if pcc_report else None,
                                   C.byref(pdc_report) if pdc_report else None, str(path).encode()),
         "dnrp_rx_packet_json")


def _check_tensor(t, what, dtype, ndim, device):
    """Shapes, dtype, layout and device of a buffer handed to libdnrp.so (the C side trusts them)."""
    import torch
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{what}: expected a torch tensor")
    if t.dtype != dtype:
        raise TypeError(f"{what}: dtype {t.dtype}, expected {dtype}")
    if t.dim() != ndim:
        raise ValueError(f"{what}: {t.dim()} dimensions, expected {ndim}")
    if not t.is_contiguous():
        raise ValueError(f"{what}: must be contiguous")
    if t.device.type != "cuda" or (t.device.index or 0) != device:
        raise ValueError(f"{what}: must live on cuda:{device}, is on {t.device}")


def _stream_ptr(stream):
    if stream is None:
        return None
    return C.c_void_p(int(stream.cuda_stream) if hasattr(stream, "cuda_stream") else int(stream))


class Phy:
    """One context = one submitting thread (like one worker_tx_rx_t)."""

    def __init__(self, u_max, b_max, N_TX_max, os_min=1, L=10, M=9, chestim_mode_lr=True, stride=2, max_batch=64,
                 device=0):
        self.cfg = Cfg(u_max, b_max, N_TX_max, os_min, L, M, int(chestim_mode_lr), stride, max_batch, device)
        self._ctx = C.c_void_p()
        _chk(lib().dnrp_ctx_create(C.byref(self.cfg), C.byref(self._ctx)), "dnrp_ctx_create")

    def close(self):
        if self._ctx:
            lib().dnrp_ctx_destroy(self._ctx)
            self._ctx = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    RX_MODE_SM_MMSE = 1

    def set_rx_mode(self, flags):
        """dnrp_ctx_set_rx_mode: RX_MODE_SM_MMSE enables the MMSE receiver for spatial multiplexing."""
        _chk(lib().dnrp_ctx_set_rx_mode(self._ctx, int(flags)), "dnrp_ctx_set_rx_mode")

    def add_network_id(self, nid):
        _chk(lib().dnrp_add_network_id(self._ctx, nid), "dnrp_add_network_id")

    def packet_sizes(self, ps):
        out = PacketSizes()
        _chk(lib().dnrp_get_packet_sizes(self._ctx, C.byref(ps), C.byref(out)), "dnrp_get_packet_sizes")
        return out.as_dict()

    def tx_batch(self, ps, descs, pcc_d, pdc_d, iq_out, stream=None):
        """pcc_d uint8 [n,25], pdc_d uint8 [n,stride], iq_out float32 [n,N_TX,S,2] (torch, device)."""
        import torch
        n = len(descs)
        dev = int(self.cfg.device)
        _check_tensor(pcc_d, "pcc_d", torch.uint8, 2, dev)
        _check_tensor(pdc_d, "pdc_d", torch.uint8, 2, dev)
        _check_tensor(iq_out, "iq_out", torch.float32, 4, dev)
        sz = self.packet_sizes(ps)
        if pcc_d.shape[0] < n or pcc_d.shape[1] != 25:
            raise ValueError(f"pcc_d shape {tuple(pcc_d.shape)}, expected [>={n}, 25]")
        if pdc_d.shape[0] < n or pdc_d.shape[1] < (sz["G"] + 7) // 8:
            raise ValueError(f"pdc_d shape {tuple(pdc_d.shape)}, expected [>={n}, >={(sz['G'] + 7) // 8}]")
        if iq_out.shape[0] < n or iq_out.shape[1] != sz["N_TX"] or iq_out.shape[3] != 2:
            raise ValueError(f"iq_out shape {tuple(iq_out.shape)}, expected [>={n}, {sz['N_TX']}, S, 2]")
        arr = descs if isinstance(descs, C.Array) else (TxDesc * n)(*descs)
        _chk(lib().dnrp_tx_batch(self._ctx, C.byref(ps), n, arr, C.c_void_p(pcc_d.data_ptr()),
                                 C.c_void_p(pdc_d.data_ptr()), pdc_d.shape[1], C.c_void_p(iq_out.data_ptr()),
                                 iq_out.shape[2], _stream_ptr(stream)), "dnrp_tx_batch")

    def rx_sync_batch(self, sc, iq, n, S_win, win_stride, ant_stride, res=None, n_found=None, stream=None):
        """sync_chunk_t::search() on n windows of the device cf32 tensor iq (strides in samples).
        res: numpy SYNC_RESULT_DTYPE [n, max_reports] (pinned memory keeps the copy asynchronous);
        valid after sync(). Returns (res, n_found)."""
        import torch
        _check_tensor(iq, "iq", torch.float32, iq.dim(), int(self.cfg.device))
        if iq.shape[-1] != 2:
            raise ValueError("iq: last dimension must be 2 (interleaved cf32)")
        if n > 0:
            last = (n - 1) * win_stride + (sc.N_ant_limited - 1) * ant_stride + S_win
            if last > iq.numel() // 2:
                raise ValueError(f"iq holds {iq.numel() // 2} samples, the windows reach {last}")
        if res is None:
            res = np.zeros((n, sc.max_reports), SYNC_RESULT_DTYPE)
        if n_found is None:
            n_found = np.zeros(n, np.uint32)
        assert res.dtype == SYNC_RESULT_DTYPE and res.size >= n * sc.max_reports and res.flags.c_contiguous
        assert n_found.dtype == np.uint32 and n_found.size >= n
        _chk(lib().dnrp_rx_sync_batch(self._ctx, C.byref(sc), n, C.c_void_p(iq.data_ptr()), win_stride, ant_stride,
                                      S_win, C.c_void_p(res.ctypes.data), C.c_void_p(n_found.ctypes.data),
                                      _stream_ptr(stream)), "dnrp_rx_sync_batch")
        return res, n_found

    def _check_rx_windows(self, iq_in):
        import torch
        _check_tensor(iq_in, "iq_in", torch.float32, 4, int(self.cfg.device))
        if iq_in.shape[1] != self.cfg.N_TX_max or iq_in.shape[3] != 2:
            raise ValueError(f"iq_in shape {tuple(iq_in.shape)}, expected [windows, {self.cfg.N_TX_max}, S_in, 2]")

    def rx_pcc_batch(self, reports, iq_in, pcc_llr, want_report=False, stream=None):
        """reports: list of SyncReport or a numpy SYNC_REPORT_DTYPE array (see sync_reports()).
        iq_in float32 [n, N_RX, S_in, 2]; pcc_llr int16 [n, 196]."""
        import torch
        n = len(reports)
        self._check_rx_windows(iq_in)
        _check_tensor(pcc_llr, "pcc_llr", torch.int16, 2, int(self.cfg.device))
        if pcc_llr.shape[0] < n or pcc_llr.shape[1] != 196:
            raise ValueError(f"pcc_llr shape {tuple(pcc_llr.shape)}, expected [>={n}, 196]")
        if isinstance(reports, np.ndarray):
            assert reports.dtype == SYNC_REPORT_DTYPE and reports.flags.c_contiguous
            wins = reports["window"]
            arr = C.c_void_p(reports.ctypes.data)
        else:
            arr_s = (SyncReport * n)(*reports)
            for i in range(n):  # SyncReport(...) without a window: its own index
                if arr_s[i].window == SyncReport.AUTO_WINDOW:
                    arr_s[i].window = i
            wins = np.array([r.window for r in arr_s], np.int64)
            arr = C.cast(arr_s, C.c_void_p)
        if n and (wins.max() >= iq_in.shape[0] or wins.min() < 0):
            raise ValueError(f"sync report window {int(wins.max())} outside iq_in ({iq_in.shape[0]} windows)")
        rep = (PccReport * n)() if want_report else None
        _chk(lib().dnrp_rx_pcc_batch(self._ctx, n, arr, C.c_void_p(iq_in.data_ptr()), iq_in.shape[0], iq_in.shape[2],
                                     C.c_void_p(pcc_llr.data_ptr()), rep, _stream_ptr(stream)), "dnrp_rx_pcc_batch")
        return rep

    def rx_pdc_batch(self, reqs, iq_in, pdc_llr, want_report=False, stream=None):
        """reqs: PdcReq per packet the MAC continues with (psdef, pcc_index, network_id, plcf_type);
        iq_in: the windows of the preceding rx_pcc_batch; pdc_llr int16 [m, >= max G] (row r = reqs[r])."""
        import torch
        m = len(reqs)
        self._check_rx_windows(iq_in)
        _check_tensor(pdc_llr, "pdc_llr", torch.int16, 2, int(self.cfg.device))
        arr = reqs if isinstance(reqs, C.Array) else (PdcReq * m)(*reqs)
        # distinct psdefs of the requests, vectorised over the array's memory (a Python loop over
        # 16384 ctypes records takes ~50 ms per call)
        nw = C.sizeof(PsDef) // 4  # PsDef: uint32 fields only
        w = np.frombuffer(arr, dtype=np.uint32, count=m * C.sizeof(PdcReq) // 4).reshape(m, -1)[:, :nw] if m else None
        if w is None:
            keys = set()
        elif (w == w[0]).all():
            keys = {tuple(int(x) for x in w[0])}
        else:
            rows = np.unique(np.ascontiguousarray(w).view(np.dtype((np.void, 4 * nw))).ravel())
            keys = {tuple(int(x) for x in np.frombuffer(r.tobytes(), np.uint32)) for r in rows}
        g_max = max((self.packet_sizes(PsDef(*k))["G"] for k in keys), default=0)
        if pdc_llr.shape[0] < m or pdc_llr.shape[1] < g_max:
            raise ValueError(f"pdc_llr shape {tuple(pdc_llr.shape)}, expected [>={m}, >={g_max}]")
        rep = (PdcReport * m)() if want_report else None
        _chk(lib().dnrp_rx_pdc_batch(self._ctx, m, arr, C.c_void_p(iq_in.data_ptr()), iq_in.shape[0], iq_in.shape[2],
                                     C.c_void_p(pdc_llr.data_ptr()), pdc_llr.shape[1], rep, _stream_ptr(stream)),
             "dnrp_rx_pdc_batch")
        return rep

    def sync(self, stream=None):
        _chk(lib().dnrp_sync(self._ctx, _stream_ptr(stream)), "dnrp_sync")

    def _check_ring(self, ring, n_ant):
        import torch
        _check_tensor(ring, "ring", torch.float32, 3, int(self.cfg.device))
        if ring.shape[0] < n_ant or ring.shape[2] != 2:
            raise ValueError(f"ring shape {tuple(ring.shape)}, expected [>= {n_ant}, ring_len, 2]")

    def ring_gather(self, ring, starts, S_win, out, n_ant=None, stream=None):
        """buffer_rx_t ring (float32 [N_ant, ring_len, 2], sample t at t % ring_len) -> windows
        out float32 [n, n_ant, S_win, 2] starting at the global times `starts` (rx_pacer wrap copy)."""
        import torch
        n_ant = n_ant or ring.shape[0]
        self._check_ring(ring, n_ant)
        st = np.ascontiguousarray(np.asarray(starts, dtype=np.int64))
        n = len(st)
        _check_tensor(out, "out", torch.float32, 4, int(self.cfg.device))
        if out.shape[0] < n or out.shape[1] != n_ant or out.shape[2] != S_win or out.shape[3] != 2:
            raise ValueError(f"out shape {tuple(out.shape)}, expected [>={n}, {n_ant}, {S_win}, 2]")
        _chk(lib().dnrp_ring_gather(self._ctx, C.c_void_p(ring.data_ptr()), ring.shape[1], ring.shape[1], n_ant, n,
                                    C.c_void_p(st.ctypes.data), S_win, C.c_void_p(out.data_ptr()), _stream_ptr(stream)),
             "dnrp_ring_gather")

    def channel_batch(self, cfg, tx, offsets, t0s, rx, stream=None):
        """Simulated channel: tx float32 [n, N_TX, S_tx, 2] -> rx float32 [n, N_RX, S_rx, 2] (device);
        offsets / t0s: per window, TX sample 0 at RX sample offset, global time of RX sample 0."""
        import torch
        dev = int(self.cfg.device)
        _check_tensor(tx, "tx", torch.float32, 4, dev)
        _check_tensor(rx, "rx", torch.float32, 4, dev)
        off = np.ascontiguousarray(np.asarray(offsets, dtype=np.int64))
        t0 = np.ascontiguousarray(np.asarray(t0s, dtype=np.int64))
        n = len(off)
        if len(t0) != n or tx.shape[0] < n or rx.shape[0] < n or tx.shape[3] != 2 or rx.shape[3] != 2:
            raise ValueError("channel_batch: window counts / shapes disagree")
        _chk(lib().dnrp_channel_batch(self._ctx, C.byref(cfg), n, tx.shape[1], C.c_void_p(tx.data_ptr()), tx.shape[2],
                                      rx.shape[1], C.c_void_p(off.ctypes.data), C.c_void_p(t0.ctypes.data),
                                      C.c_void_p(rx.data_ptr()), rx.shape[2], _stream_ptr(stream)), "dnrp_channel_batch")

    def sync_stream_init(self, sc):
        state = SyncStreamState()
        _chk(lib().dnrp_sync_stream_init(self._ctx, C.byref(sc), C.byref(state)), "dnrp_sync_stream_init")
        return state

    def sync_stream_window(self, sc):
        return int(lib().dnrp_sync_stream_window(self._ctx, C.byref(sc)))

    def rx_sync_stream(self, sc, ring, t0, n_chunks, state, stream=None):
        """Continuous-stream sync of n_chunks chunks from global time t0 over the ring; returns the
        unique reports (SYNC_RESULT_DTYPE, global times) and the chunk each was found in."""
        self._check_ring(ring, sc.N_ant_limited)
        out = np.zeros(max(1, n_chunks * sc.max_reports), SYNC_RESULT_DTYPE)
        chunk_of = np.zeros(max(1, n_chunks * sc.max_reports), np.uint32)
        n_out = C.c_uint32()
        _chk(lib().dnrp_rx_sync_stream(self._ctx, C.byref(sc), C.c_void_p(ring.data_ptr()), ring.shape[1],
                                       ring.shape[1], int(t0), n_chunks, C.byref(state), C.c_void_p(out.ctypes.data),
                                       C.byref(n_out), C.c_void_p(chunk_of.ctypes.data), _stream_ptr(stream)),
             "dnrp_rx_sync_stream")
        return out[: n_out.value], chunk_of[: n_out.value]

    def kernel_time_total(self, name, reset=True):
        ms, cnt = C.c_float(), C.c_uint32()
        _chk(lib().dnrp_kernel_time_total(self._ctx, name.encode(), C.byref(ms), C.byref(cnt), int(reset)),
             "dnrp_kernel_time_total")
        return float(ms.value), int(cnt.value)

    def last_kernel_ms(self, name):
        ms = C.c_float()
        _chk(lib().dnrp_last_kernel_ms(self._ctx, name.encode(), C.byref(ms)), "dnrp_last_kernel_ms")
        return float(ms.value)
