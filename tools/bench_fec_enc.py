"""GPU channel-encoding time (outside bench.py's headline): dnrp_pdc_encode_batch on
n C4 transport blocks (N_TB = 363464 bits, 60 code blocks of 6144, G = 486640, 256-QAM) and the PLCF
encoder on n PLCFs; per-kernel times from the library's HIP events (fec_tbcrc, fec_encode, fec_pack).
Checks the first, middle and last packet against the host encoder. Prints one JSON line.
Usage: python tools/bench_fec_enc.py [--n 16384] [--reps 3]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dect-nr-plus-sdr_amd"))
os.environ.setdefault("DNRP_TIMING", "1")

import torch  # noqa: E402

import dnrp  # noqa: E402
import dnrp.fec as FE  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=16384)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    phy = dnrp.Phy(8, 16, 4, 1, 10, 9, max_batch=a.n)
    ps = dnrp.psdef(8, 16, 1, 1, 5, 8)
    sz = phy.packet_sizes(ps)
    G, ntb = sz["G"], sz["N_TB_bits"]
    cfg = FE.fec_cfg(ntb, sz["N_bps"], G, Z=ps.Z)
    gen = torch.Generator(device=dev)
    gen.manual_seed(5)
    tb = torch.randint(0, 256, (a.n, ntb // 8 + 3), dtype=torch.uint8, device=dev, generator=gen)
    d = torch.empty((a.n, (G + 7) // 8), dtype=torch.uint8, device=dev)
    FE.pdc_encode_batch(phy, [cfg] * a.n, tb, d)  # warm-up (tables)
    names = ("fec_tbcrc", "fec_encode", "fec_pack")
    for nm in names:
        phy.kernel_time_total(nm, reset=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.reps):
        FE.pdc_encode_batch(phy, [cfg] * a.n, tb, d)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / a.reps
    kt = {nm: phy.kernel_time_total(nm, reset=True)[0] / a.reps for nm in names}
    th, dh = tb.cpu().numpy(), d.cpu().numpy()
    ok = all(np.array_equal(FE.pdc_encode(cfg, th[i, : ntb // 8]), dh[i]) for i in (0, a.n // 2, a.n - 1))
    # PLCF encoder on the device (dnrp_pcc_encode_batch)
    plcf = torch.randint(0, 256, (a.n, 10), dtype=torch.uint8, device=dev, generator=gen)
    pd = torch.empty((a.n, 25), dtype=torch.uint8, device=dev)
    types = [1 + i % 2 for i in range(a.n)]
    FE.pcc_encode_batch(phy, types, plcf, pd)
    for nm in names:
        phy.kernel_time_total(nm, reset=True)
    FE.pcc_encode_batch(phy, types, plcf, pd)
    torch.cuda.synchronize()
    kp = {nm: phy.kernel_time_total(nm, reset=True)[0] for nm in names}
    ph, pdh = plcf.cpu().numpy(), pd.cpu().numpy()
    ok_p = all(np.array_equal(FE.pcc_encode(ph[i, : 5 * types[i]], types[i]), pdh[i]) for i in (0, 1, a.n - 1))
    print(json.dumps({"n": a.n, "tb_bits": ntb, "code_blocks_per_tb": sz["C"], "wall_ms": round(wall * 1e3, 3),
                      "kernel_ms": {k: round(v, 3) for k, v in kt.items()}, "host_equal": bool(ok),
                      "plcf_kernel_ms": {k: round(v, 3) for k, v in kp.items()}, "plcf_host_equal": bool(ok_p)}), flush=True)


if __name__ == "__main__":
    main()
