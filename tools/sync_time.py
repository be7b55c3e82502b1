"""Synchronisation kernels alone on the bench workload's window geometry (noise windows; the
detection then finds nothing, so sync_detect times only its scan): per-kernel ms per chunk.
python tools/sync_time.py [workload] [chunk] [reps]"""
import os
import sys

os.environ.setdefault("DNRP_TIMING", "1")
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "dect-nr-plus-sdr_amd"))
import torch  # noqa: E402

import bench  # noqa: E402
import dnrp  # noqa: E402


def main():
    wl = sys.argv[1] if len(sys.argv) > 1 else "C4"
    chunk = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    psd, cfgt = bench.WORKLOADS[wl][:2]
    u_max, b_max, n_ant, os_min, L, M = cfgt
    phy = dnrp.Phy(*cfgt, max_batch=chunk)
    ps = dnrp.psdef(*psd)
    sz = phy.packet_sizes(ps)
    S = sz["N_samples_packet_os_rs"]
    tl = sz["N_samples_packet_no_GI_os_rs"] + (S - sz["N_samples_packet_no_GI_os_rs"]) * 5 // 100
    pre = bench.sync_pre(psd, L, M, S - tl - 32)
    S_rx = max(S, pre + 32 + tl)
    g = torch.Generator(device="cuda:0")
    g.manual_seed(3)
    iq = torch.randn((chunk, n_ant, S_rx, 2), generator=g, device="cuda:0") * 0.01
    sc = dnrp.SyncCfg(psd[0], psd[1], n_ant, bench.sync_chunk_len(S_rx, psd, L, M), 1)
    phy.rx_sync_batch(sc, iq, chunk, S_rx, n_ant * S_rx, S_rx)
    phy.sync()
    names = ["sync_steps", "sync_detect", "sync_peak", "sync_post", "sync_fine"]
    for nm in names:
        phy.kernel_time_total(nm, reset=True)
    for _ in range(reps):
        phy.rx_sync_batch(sc, iq, chunk, S_rx, n_ant * S_rx, S_rx)
    phy.sync()
    out = {nm: round(phy.kernel_time_total(nm)[0] / reps, 3) for nm in names}
    print(os.environ.get("TAG", ""), wl, out, flush=True)


if __name__ == "__main__":
    main()
