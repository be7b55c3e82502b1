"""Channel-decoding throughput (not part of bench.py's headline, which
excludes FEC as BASELINE.md does): dnrp_pdc_decode_batch on n C4 transport blocks (N_TB = 363464
bits, 60 code blocks, G = 486640, Z = 6144) against the host decoder dnrp_pdc_decode on one core.

LLRs: one encoded transport block as +-1 soft bits with Gaussian noise per packet at --snr (1/sigma^2
of the soft bits), scaled by 300 to int16, generated on the GPU. Prints one JSON line.
Usage: python tools/bench_fec.py [--n 1024] [--snr 30] [--reps 3]
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
    ap.add_argument("--n", type=int, default=1024)
    ap.add_argument("--snr", type=float, default=30.0)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--host", type=int, default=4, help="transport blocks timed on the host decoder")
    a = ap.parse_args()
    tbs, Qm, G = 363464, 8, 486640
    cfg = FE.fec_cfg(tbs, Qm, G)
    rng = np.random.default_rng(1)
    tb = rng.integers(0, 256, tbs // 8, dtype=np.uint8)
    x = 2.0 * np.unpackbits(FE.pdc_encode(cfg, tb))[:G] - 1
    dev = torch.device("cuda:0")
    phy = dnrp.Phy(1, 1, 1, max_batch=1)
    xg = torch.from_numpy(x.astype(np.float32)).to(dev)
    g = torch.Generator(device=dev).manual_seed(7)
    sigma = 10 ** (-a.snr / 20)
    llr = torch.empty((a.n, G), dtype=torch.int16, device=dev)
    for i in range(a.n):
        y = xg + sigma * torch.randn(G, device=dev, generator=g)
        llr[i] = torch.clamp(torch.round(y * 300), -32768, 32767).to(torch.int16)
    tb_dev = torch.zeros((a.n, tbs // 8 + 3), dtype=torch.uint8, device=dev)
    cfgs = [cfg] * a.n
    FE.pdc_decode_batch(phy, cfgs[:8], llr, tb_dev)  # warm-up (tables, code objects)
    phy.kernel_time_total("fec_dematch"), phy.kernel_time_total("fec_tdec")  # reset the totals
    best = None
    for _ in range(a.reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ok, it = FE.pdc_decode_batch(phy, cfgs, llr, tb_dev)
        dt = time.perf_counter() - t0
        best = dt if best is None else min(best, dt)
    k_dem = phy.kernel_time_total("fec_dematch")[0] / a.reps
    k_dec = phy.kernel_time_total("fec_tdec")[0] / a.reps
    good = int(ok.sum())
    same = bool((tb_dev[:, : tbs // 8].cpu().numpy() == tb[None, :]).all(axis=1)[ok].all()) if good else False
    # GPU encoder (dnrp_pdc_encode_batch) on the same transport blocks
    tb_in = torch.from_numpy(np.tile(tb, (a.n, 1))).to(dev)
    d_out = torch.zeros((a.n, (G + 7) // 8), dtype=torch.uint8, device=dev)
    FE.pdc_encode_batch(phy, cfgs[:8], tb_in, d_out)
    phy.kernel_time_total("fec_encode")
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    FE.pdc_encode_batch(phy, cfgs, tb_in, d_out)
    enc_s = time.perf_counter() - t0
    enc_k = phy.kernel_time_total("fec_encode")[0]
    enc_ok = bool((d_out[-1].cpu().numpy() == FE.pdc_encode(cfg, tb)).all())
    # host decoder, one core
    h_llr = llr[: a.host].cpu().numpy()
    t0 = time.perf_counter()
    h_ok = [FE.pdc_decode(cfg, h_llr[i])[0] for i in range(a.host)]
    h_dt = (time.perf_counter() - t0) / a.host
    print(json.dumps({
        "what": "PDC turbo decoding, C4 transport blocks (363464 bits, 60 code blocks)",
        "n_tb": a.n, "snr_db": a.snr, "gpu_s": round(best, 4), "gpu_tb_per_s": round(a.n / best, 1),
        "gpu_info_mbit_per_s": round(a.n * tbs / best / 1e6, 1),
        "kernel_ms": {"fec_dematch": k_dem, "fec_tdec": k_dec},
        "crc_ok": good, "decoded_equal_tx": same, "iterations_per_cb": float(it.mean() / 60.0),
        "host_1core_s_per_tb": round(h_dt, 4), "host_ok": int(sum(h_ok)),
        "gpu_encode_s": round(enc_s, 4), "gpu_encode_kernel_ms": round(enc_k, 3), "gpu_encode_tb_per_s": round(a.n / enc_s, 1),
        "gpu_encode_equal_host": enc_ok,
        "gpu_vs_1core": round((a.n / best) / (1 / h_dt), 1)}))


if __name__ == "__main__":
    main()
