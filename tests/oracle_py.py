"""ctypes bindings to oracle/liboracle.so — TEST INFRASTRUCTURE ONLY.

Used by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg. The product path
(dect-nr-plus-sdr_amd/) never imports this module.
"""
import ctypes as C
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# ORACLE_LIB: another build of the same sources (bench.py's cpu_baseline builds one -march=native)
# mimo_report_t index where the reference defines no result (oracle_dsp.hpp MIMO_REF_UNDEFINED)
MIMO_REF_UNDEFINED = 0xFFFFFFFE
LIB_PATH = os.environ.get("ORACLE_LIB") or os.path.join(ROOT, "oracle", "liboracle.so")

_lib = None

U32P = np.ctypeslib.ndpointer(dtype=np.uint32, flags="C_CONTIGUOUS")
F32P = np.ctypeslib.ndpointer(dtype=np.float32, flags="C_CONTIGUOUS")
F64P = np.ctypeslib.ndpointer(dtype=np.float64, flags="C_CONTIGUOUS")
U8P = np.ctypeslib.ndpointer(dtype=np.uint8, flags="C_CONTIGUOUS")
I16P = np.ctypeslib.ndpointer(dtype=np.int16, flags="C_CONTIGUOUS")

PS_FIELDS = ["N_PACKET_symb", "N_DF_symb", "N_PDC_subc", "N_DRS_subc", "G", "N_PDC_bits", "N_TB_bits", "C",
             "N_samples_STF", "N_samples_STF_CP_only", "N_samples_DF", "N_samples_GI",
             "N_samples_packet_no_GI", "N_samples_packet", "N_bps", "N_eff_TX", "N_SS", "N_TS", "N_TX",
             "N_b_DFT", "N_b_OCC"]
DIM_FIELDS = ["N_b_DFT_os", "off_lower", "CP_os", "STF_CP_os", "N_no_GI_os", "N_no_GI_os_rs", "N_packet_os_rs"]


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True,
                           stdout=subprocess.DEVNULL)
        L = C.CDLL(LIB_PATH)
        L.oracle_packet_sizes.argtypes = [U32P, U32P]
        L.oracle_dims.argtypes = [U32P, U32P, U32P]
        L.oracle_kaiser.argtypes = [C.c_float, C.c_float, C.c_float, C.c_float, C.c_uint32, F32P]
        L.oracle_gold.argtypes = [C.c_uint32, C.c_uint32, U8P]
        L.oracle_stf.argtypes = [C.c_uint32, C.c_uint32, F64P]
        L.oracle_pdc_cells.argtypes = [C.c_uint32, C.c_uint32, C.c_uint32, U32P, U32P]
        L.oracle_pcc_cells.argtypes = [C.c_uint32, C.c_uint32, U32P, U32P]
        L.oracle_chest_lut.argtypes = [C.c_uint32] * 5 + [U32P, U32P, F32P, C.c_uint32]
        L.oracle_tx.argtypes = [U32P, U32P, U32P, F64P, U8P, U8P, F32P, C.c_uint32, C.c_int]
        L.oracle_rx.argtypes = [U32P, U32P, C.c_uint32, F32P, C.c_uint32, C.c_int64, C.c_double, C.c_uint32,
                                C.c_uint32, I16P, I16P, C.c_void_p, C.c_void_p, F32P, C.c_int, C.c_void_p, C.c_int]
        L.oracle_loopback_timed.argtypes = [U32P, U32P, C.c_uint32, C.c_uint32, C.c_uint64, C.c_uint32, C.c_uint32]
        L.oracle_loopback_timed.restype = C.c_double
        L.oracle_loopback_timed2.argtypes = [U32P, U32P, C.c_uint32, C.c_uint32, C.c_uint64, C.c_uint32, C.c_uint32,
                                             F64P]
        L.oracle_loopback_timed2.restype = C.c_double
        L.oracle_numerology.argtypes = [C.c_uint32, C.c_uint32, U32P, C.POINTER(C.c_double)]
        L.oracle_tm_mode.argtypes = [C.c_uint32, U32P]
        L.oracle_mcs.argtypes = [C.c_uint32, U32P]
        L.oracle_tbs.argtypes = [C.c_uint32] * 4
        L.oracle_tbs.restype = C.c_uint32
        L.oracle_k_b_occ.argtypes = [C.c_uint32, np.ctypeslib.ndpointer(dtype=np.int32, flags="C_CONTIGUOUS"),
                                     C.c_uint32]
        L.oracle_special.argtypes = [C.c_float, F32P]
        L.oracle_sync.argtypes = [U32P, F32P, C.c_uint32, C.c_uint32, C.c_int, F64P]
        L.oracle_sync_geometry.argtypes = [U32P, U32P, C.POINTER(C.c_float)]
        L.oracle_stf_template.argtypes = [U32P, C.c_uint32, F32P]
        L.oracle_query_param.argtypes = [C.c_char_p, C.POINTER(C.c_double)]
        L.oracle_W.argtypes = [C.c_uint32, C.c_uint32, C.c_uint32, F64P, F64P]
        L.oracle_W_codebooks.argtypes = [C.c_uint32, C.c_uint32]
        L.oracle_drs_values.argtypes = [C.c_uint32, C.c_uint32, F64P]
        L.oracle_txdiv_pairs.argtypes = [C.c_uint32, U32P]
        L.oracle_cover_sequence.argtypes = [F32P]
        _lib = L
    return _lib


def psdef(u, b, plt, pl, tm, mcs, Z=6144):
    return np.array([u, b, plt, pl, tm, mcs, Z], dtype=np.uint32)


def cfg(u_max, b_max, os_min=1, L=10, M=9, lr=1, stride=2):
    return np.array([u_max, b_max, os_min, L, M, lr, stride], dtype=np.uint32)


def packet_sizes(ps):
    out = np.zeros(len(PS_FIELDS), dtype=np.uint32)
    if lib().oracle_packet_sizes(np.asarray(ps, dtype=np.uint32), out) != 0:
        return None
    return dict(zip(PS_FIELDS, (int(x) for x in out)))


def dims(cf, ps):
    out = np.zeros(len(DIM_FIELDS), dtype=np.uint32)
    assert lib().oracle_dims(cf, ps, out) == 0
    return dict(zip(DIM_FIELDS, (int(x) for x in out)))


def kaiser(fp, fs, ripple, att):
    out = np.zeros(4096, dtype=np.float32)
    n = lib().oracle_kaiser(fp, fs, ripple, att, 4096, out)
    return out[:n].copy()


def gold(c_init, n):
    out = np.zeros(n, dtype=np.uint8)
    lib().oracle_gold(c_init, n, out)
    return out


def tx(cf, ps, pcc_d, pdc_d, S_slot, codebook=0, network_id=100, plcf_type=1, gi=5, dac=1.0, phase=0.0,
       phase_inc=0.0, use_float=False, optimal_dac=False):
    sz = packet_sizes(ps)
    out = np.zeros((sz["N_TX"], S_slot, 2), dtype=np.float32)
    du = np.array([codebook, network_id, plcf_type, gi, int(optimal_dac)], dtype=np.uint32)
    df = np.array([dac, phase, phase_inc], dtype=np.float64)
    n = lib().oracle_tx(cf, ps, du, df, np.ascontiguousarray(pcc_d, dtype=np.uint8),
                        np.ascontiguousarray(pdc_d, dtype=np.uint8), out, S_slot, int(use_float))
    assert n > 0, n
    return out.view(np.complex64)[..., 0], n


def rx(cf, ps, iq, fine_peak=0, cfo_rad=0.0, network_id=100, plcf_type=1, use_float=False, sync_rms=None,
       sm_mmse=False):
    """iq: complex64 [N_RX, S_in]; sync_rms: the sync report's rms_array (8 floats, optional);
    sm_mmse: demodulate spatial multiplexing (N_SS > 1) by MMSE. Returns dict with int16/float LLRs
    and meta."""
    sz = packet_sizes(ps)
    iq = np.ascontiguousarray(iq, dtype=np.complex64)
    n_rx, s_in = iq.shape
    pcc = np.zeros(196, dtype=np.int16)
    pdc = np.zeros(sz["G"], dtype=np.int16)
    pccf = np.zeros(196, dtype=np.float32)
    pdcf = np.zeros(sz["G"], dtype=np.float32)
    meta = np.zeros(16, dtype=np.float32)
    srms = None if sync_rms is None else np.ascontiguousarray(np.resize(np.asarray(sync_rms, np.float32), 8))
    r = lib().oracle_rx(cf, ps, n_rx, iq.view(np.float32).reshape(-1), s_in, int(fine_peak), float(cfo_rad),
                        network_id, plcf_type, pcc, pdc, pccf.ctypes.data, pdcf.ctypes.data, meta,
                        int(use_float), srms.ctypes.data if srms is not None else None, int(sm_mmse))
    assert r == 0, r
    return dict(pcc_llr=pcc, pdc_llr=pdc, pcc_llr_f=pccf, pdc_llr_f=pdcf, rms=meta[:8].copy(),
                cfo_fine=float(meta[8]), sto=float(meta[9]), snr_pcc=float(meta[10]), snr_pdc=float(meta[11]),
                mimo_N_TS_other=int(meta[12]), mimo_idx=int(meta[13]) & 0xFFFFFFFF, mimo_idx_reciprocal=int(meta[14]) & 0xFFFFFFFF)


def loopback_timed(cf, ps, n_packets, n_threads, seed=0xDEC7, sync_pre=0, sync_chunk=0, phases=False):
    """wall seconds of n_packets TX + (sync +) RX slot-pairs on n_threads; phases=True also returns
    the thread-seconds spent in TX and in sync + RX"""
    if not phases:
        return lib().oracle_loopback_timed(cf, ps, n_packets, n_threads, seed, sync_pre, sync_chunk)
    ph = np.zeros(2)
    t = lib().oracle_loopback_timed2(cf, ps, n_packets, n_threads, seed, sync_pre, sync_chunk, ph)
    return t, float(ph[0]), float(ph[1])


def pack_bits(bits):
    return np.packbits(np.asarray(bits, dtype=np.uint8))


def query_param(name):
    """The oracle's value of a reference parameter (None if the restatement does not use it)."""
    v = C.c_double()
    return v.value if lib().oracle_query_param(name.encode(), C.byref(v)) == 0 else None


# ---- reference-table restatements (pinned by tests/golden/ref_tables.json)
def numerology(u, b):
    out = np.zeros(10, np.uint32)
    T = C.c_double()
    if lib().oracle_numerology(u, b, out, C.byref(T)) != 0:
        raise ValueError((u, b))
    keys = ["u", "b", "delta_u_f", "N_SLOT_u_symb", "N_SLOT_u_subslot", "N_b_DFT", "N_b_CP", "N_b_OCC",
            "N_guards_top", "N_guards_bottom"]
    d = {k: int(v) for k, v in zip(keys, out)}
    d["T_u_symb"] = T.value
    return d


def tm_mode(i):
    out = np.zeros(6, np.uint32)
    if lib().oracle_tm_mode(i, out) != 0:
        raise ValueError(i)
    return dict(zip(["index", "N_eff_TX", "N_SS", "cl", "N_TS", "N_TX"], map(int, out)))


def mcs(i):
    out = np.zeros(4, np.uint32)
    if lib().oracle_mcs(i, out) != 0:
        raise ValueError(i)
    return dict(zip(["index", "N_bps", "R_num", "R_den"], map(int, out)))


def tbs(N_SS, N_PDC, mcs_index, Z):
    return int(lib().oracle_tbs(N_SS, N_PDC, mcs_index, Z))


def k_b_occ(b):
    out = np.zeros(1024, np.int32)
    n = lib().oracle_k_b_occ(b, out, out.size)
    return out[:n].tolist()


def W(N_TS, N_TX, codebook):
    """(W [N_TX][N_TS] complex, standard scaling, optimal-DAC scaling), None if undefined."""
    out, sc = np.zeros(2 * 64), np.zeros(2)
    n = lib().oracle_W(N_TS, N_TX, codebook, out, sc)
    if n < 0:
        return None
    return out[: 2 * n].view(np.complex128).reshape(N_TX, N_TS), float(sc[0]), float(sc[1])


def W_codebooks(N_TS, N_TX):
    return lib().oracle_W_codebooks(N_TS, N_TX)


def stf(b, n_eff_tx):
    out = np.zeros(2 * (56 * b + 1))
    n = lib().oracle_stf(b, n_eff_tx, out)
    return out[: 2 * n].view(np.complex128)


def drs_values(b, t):
    out = np.zeros(14 * b)
    return out[: lib().oracle_drs_values(b, t, out)]


def txdiv_pairs(N_TS):
    out = np.zeros(24, np.uint32)
    return out[: 2 * lib().oracle_txdiv_pairs(N_TS, out)].reshape(-1, 2).tolist()


def cover_sequence():
    out = np.zeros(9, np.float32)
    lib().oracle_cover_sequence(out)
    return out


def special(z):
    out = np.zeros(5, np.float32)
    lib().oracle_special(np.float32(z), out)
    return out


# ---- synchronisation (oracle_sync.cpp)
SYNC_KEYS = ["found", "det_ant", "det_rms", "det_metric", "det_time", "det_time_jb", "coarse_local", "coarse_64",
             "cfo_frac", "u", "b", "N_eff_TX", "fine_local", "fine_64"]
SYNC_GEOM_KEYS = ["n_pattern", "bos", "stf_len", "pattern", "step", "A", "B", "C", "D", "search_len", "lb_len",
                  "xc_l", "xc_len", "tmpl_len", "n_templates"]


def sync_cfg(u, b, os_min=1, L=10, M=9, n_ant=1, n_lim=None, chunk_len=0):
    return np.array([u, b, os_min, L, M, n_ant, n_ant if n_lim is None else n_lim, chunk_len], dtype=np.uint32)


def sync_geometry(scfg):
    out = np.zeros(len(SYNC_GEOM_KEYS), np.uint32)
    r = C.c_float()
    lib().oracle_sync_geometry(np.asarray(scfg, np.uint32), out, C.byref(r))
    g = dict(zip(SYNC_GEOM_KEYS, map(int, out)))
    g["rms_min"] = r.value
    return g


def stf_template(scfg, n_eff_tx):
    g = sync_geometry(scfg)
    out = np.zeros(2 * g["tmpl_len"], np.float32)
    n = lib().oracle_stf_template(np.asarray(scfg, np.uint32), n_eff_tx, out)
    assert n == g["tmpl_len"], n
    return out.view(np.complex64).copy()


def sync(scfg, iq, max_reports=4, use_float=False):
    """iq: complex64 [N_ant_limited, S_win] window (chunk starting at iq[:, 0]). Returns a list of dicts."""
    iq = np.ascontiguousarray(iq, dtype=np.complex64)
    out = np.zeros((max_reports, 38), np.float64)
    n = lib().oracle_sync(np.asarray(scfg, np.uint32), iq.view(np.float32).reshape(-1), iq.shape[1], max_reports,
                          int(use_float), out)
    assert n >= 0, n
    res = []
    for i in range(n):
        d = {k: out[i, j] for j, k in enumerate(SYNC_KEYS)}
        for k in ("found", "det_ant", "det_time", "det_time_jb", "coarse_local", "coarse_64", "u", "b", "N_eff_TX",
                  "fine_local", "fine_64"):
            d[k] = int(d[k])
        d["coarse_metric"] = out[i, 14:22].copy()
        d["rms"] = out[i, 22:30].copy()
        d["xc_metric"] = out[i, 30:34].copy()
        d["xc_idx"] = out[i, 34:38].astype(np.int64)
        res.append(d)
    return res
