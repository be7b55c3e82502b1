"""C-ABI surface of libdnrp.so on a machine without a GPU: the library loads, exports every entry
point include/dnrp.h declares, validates arguments before touching a device, and its host-side
packet geometry (dnrp_compute_packet_sizes) equals the oracle's restatement of
sections_part3/derivative/packet_sizes.cpp for every configuration of the grid."""
import ctypes as C
import os
import re

import numpy as np
import pytest

import oracle_py as O
import phy_fixtures as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "dnrp.h")

dnrp = pytest.importorskip("dnrp")


def declared():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*[A-Za-z_][\w\s\*]*?\b(dnrp_\w+)\s*\(", src, flags=re.M)))


def test_exports_every_declared_symbol():
    names = declared()
    assert len(names) >= 12, names
    lib = dnrp.lib()
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    assert sorted(dnrp.EXPORTS) == names


def test_strerror():
    assert dnrp.strerror(0) == "ok"
    for code in (-1, -2, -3, -4, -5, -6, -7):
        assert dnrp.strerror(code) not in ("", "unknown error")
    assert dnrp.strerror(-99) == "unknown error"


@pytest.mark.parametrize("bad", [
    dict(u_max=3), dict(b_max=5), dict(N_TX_max=3), dict(os_min=3), dict(L=0), dict(M=0), dict(max_batch=0),
    dict(L=9, M=10),  # TX must up-sample (rx_pacer.cpp:50-52)
])
def test_ctx_create_rejects_invalid_config_before_device(bad):
    kw = dict(u_max=8, b_max=16, N_TX_max=4, os_min=1, L=10, M=9, chestim_mode_lr=1, chestim_lr_stride=2,
              max_batch=4, device=0)
    kw.update(bad)
    cfg = dnrp.Cfg(*[kw[f] for f, _ in dnrp.Cfg._fields_])
    ctx = C.c_void_p()
    assert dnrp.lib().dnrp_ctx_create(C.byref(cfg), C.byref(ctx)) == -1
    assert not ctx.value


def test_null_arguments():
    L = dnrp.lib()
    assert L.dnrp_ctx_create(None, None) == -1
    assert L.dnrp_get_packet_sizes(None, None, None) == -1
    assert L.dnrp_compute_packet_sizes(None, None, None) == -1
    assert L.dnrp_tx_batch(None, None, 0, None, None, None, 0, None, 0, None) == -1
    assert L.dnrp_sync(None, None) == -1
    assert L.dnrp_rx_sync_batch(None, None, 0, None, 0, 0, 0, None, None, None) == -1


def _grid():
    for u in (1, 2, 4, 8):
        for b in (1, 2, 4, 8, 12, 16):
            for plt in (0, 1):
                for pl in (1, 2, 5, 16):
                    for tm in (0, 1, 2, 5, 6):
                        for mcs in (0, 1, 4, 8, 9):
                            yield (u, b, plt, pl, tm, mcs)


def test_packet_sizes_match_oracle_on_grid():
    n_ok = n_bad = 0
    for t in _grid():
        ref = O.packet_sizes(O.psdef(*t))
        try:
            got = dnrp.compute_packet_sizes(dnrp.psdef(*t))
        except dnrp.DnrpError as e:
            assert ref is None, (t, e)
            n_bad += 1
            continue
        assert ref is not None, t
        for k, v in ref.items():
            assert got[k] == v, (t, k, got[k], v)
        n_ok += 1
    assert n_ok > 500 and n_bad > 50, (n_ok, n_bad)


@pytest.mark.parametrize("name", sorted(F.CONFIGS))
def test_oversampled_dims_match_oracle(name):
    ps, cf = F.CONFIGS[name]
    u_max, b_max, _, os_min, L, M = cf
    got = dnrp.compute_packet_sizes(dnrp.psdef(*ps), u_max, b_max, os_min, L, M)
    d = O.dims(O.cfg(u_max, b_max, os_min, L, M), O.psdef(*ps))
    assert got["N_b_DFT_os"] == d["N_b_DFT_os"]
    assert got["N_samples_packet_no_GI_os_rs"] == d["N_no_GI_os_rs"]
    assert got["N_samples_packet_os_rs"] == d["N_packet_os_rs"]


def test_benchmark_configurations_match_survey():
    # SURVEY.md §5 / BASELINE.md: G, N_PDC_subc, N_TB_bits of the headline configurations
    want = {"C2": (644, 322, 296), "C3": (515312, 64414, 384896), "C4": (486640, 60830, 363464)}
    for name, (G, npdc, ntb) in want.items():
        q = dnrp.compute_packet_sizes(dnrp.psdef(*F.CONFIGS[name][0]))
        assert (q["G"], q["N_PDC_subc"], q["N_TB_bits"]) == (G, npdc, ntb), name
    c4 = dnrp.compute_packet_sizes(dnrp.psdef(*F.CONFIGS["C4"][0]), 8, 16, 1, 10, 9)
    assert (c4["N_b_DFT_os"], c4["N_samples_packet_os_rs"]) == (1024, 102400)


def test_no_gpu_context_fails_loudly():
    torch = pytest.importorskip("torch")
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(dnrp.DnrpError) as e:
        dnrp.Phy(1, 1, 1)
    assert e.value.code == -5  # DNRP_EDEVICE: no silent CPU fallback


@pytest.mark.parametrize("name", ["C2", "C3", "C4", "tm1_txdiv2", "mrc4_16qam", "subslot_tm5", "lm40_27_b12"])
def test_symbol_cells_table(name):
    """dnrp_query_table("symbol_cells"): per symbol the PCC / PDC / DRS cells of the packet geometry the
    RX plans (and bench.py's byte counts) come from -- every occupied subcarrier of a DF symbol is one
    of them (none in symbol 0, the STF), the PCC holds its 98 cells, the PDC cells carry G bits."""
    psd, cf = F.case(name)
    ps = dnrp.psdef(*psd)
    sz = dnrp.compute_packet_sizes(ps, cf[0], cf[1], cf[3], cf[4], cf[5])
    cells = dnrp.query_table("symbol_cells", psd[1], sz["N_TS"], sz["N_eff_TX"], sz["N_DF_symb"]).reshape(-1, 3)
    assert cells.shape == (sz["N_DF_symb"] + 1, 3)
    assert not cells[0].any()
    assert (cells[1:].sum(1) <= sz["N_b_OCC"]).all()
    assert cells[:, 0].sum() == 98
    assert cells[:, 1].sum() * sz["N_bps"] * sz["N_SS"] == sz["G"]
    assert cells[1, 2] > 0  # the first DF symbol carries DRS
