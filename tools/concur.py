"""Concurrency probe: do the pipeline's kernels overlap when enqueued on separate streams?
python tools/concur.py [workload] [chunk] -- per pair of stages (TX, sync, RX) the time of each alone
and of both launched together on two streams (HIP events around the pair, after a device sync).
Same inputs as bench.py (make_inputs). Prints one JSON line."""
import json
import os
import sys
import time

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "dect-nr-plus-sdr_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
import dnrp  # noqa: E402


def main():
    wl = sys.argv[1] if len(sys.argv) > 1 else "C4"
    psd, cfgt, _, chunk0, _ = bench.WORKLOADS[wl]
    chunk = int(sys.argv[2]) if len(sys.argv) > 2 else chunk0
    u_max, b_max, n_ant, os_min, L, M = cfgt
    dev = torch.device("cuda:0")
    phy = dnrp.Phy(u_max, b_max, n_ant, os_min, L, M, max_batch=chunk)
    for nid in range(100, 106):
        phy.add_network_id(nid)
    ps = dnrp.psdef(*psd)
    sz = phy.packet_sizes(ps)
    S = sz["N_samples_packet_os_rs"]
    tl = sz["N_samples_packet_no_GI_os_rs"] + (S - sz["N_samples_packet_no_GI_os_rs"]) * 5 // 100
    pre = bench.sync_pre(psd, L, M, S - tl - 32)
    S_rx = max(S, pre + 32 + tl)
    n_tx, n_rx = sz["N_TX"], n_ant
    pcc_d, pdc_d, descs, tx_out, rx_in, offs, _ = bench.make_inputs(dev, psd, sz, 0, chunk, n_tx, n_rx, S, S_rx, pre, L, M,
                                                                    phy, ps)
    pcc_llr = torch.empty((chunk, 196), dtype=torch.int16, device=dev)
    pdc_llr = torch.empty((chunk, sz["G"]), dtype=torch.int16, device=dev)
    sc = dnrp.SyncCfg(psd[0], psd[1], n_rx, bench.sync_chunk_len(S_rx, psd, L, M), 1)
    # pinned report buffers (asynchronous copies, as bench.py)
    rb = torch.empty(chunk * dnrp.SYNC_RESULT_DTYPE.itemsize, dtype=torch.uint8, pin_memory=True)
    res = rb.numpy().view(dnrp.SYNC_RESULT_DTYPE).reshape(chunk, 1)
    cnt = torch.empty(chunk, dtype=torch.int32, pin_memory=True).numpy().view(np.uint32)
    sA, sB = torch.cuda.Stream(device=dev), torch.cuda.Stream(device=dev)
    phy.rx_sync_batch(sc, rx_in, chunk, S_rx, n_rx * S_rx, S_rx, res=res, n_found=cnt, stream=sA)
    torch.cuda.synchronize()
    reps = dnrp.found_reports(res, cnt)
    reqs = (dnrp.PdcReq * len(reps))(*[dnrp.PdcReq(ps, i, 100 + i % 6, 1 + i % 2) for i in range(len(reps))])

    def tx(s):
        phy.tx_batch(ps, descs, pcc_d, pdc_d, tx_out, stream=s)

    def sync(s):
        phy.rx_sync_batch(sc, rx_in, chunk, S_rx, n_rx * S_rx, S_rx, res=res, n_found=cnt, stream=s)

    def rx(s):
        phy.rx_pcc_batch(reps, rx_in, pcc_llr, stream=s)
        phy.rx_pdc_batch(reqs, rx_in, pdc_llr, stream=s)

    stages = {"tx": tx, "sync": sync, "rx": rx}

    def timed(fns, reps_=3):
        best = 1e30
        for _ in range(reps_):
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            cur = torch.cuda.current_stream(dev)
            e0.record(cur)
            ends = []
            for f, s in zip(fns, (sA, sB)):
                s.wait_event(e0)
                f(s)
                ev = torch.cuda.Event()
                ev.record(s)
                ends.append(ev)
            for ev in ends:
                cur.wait_event(ev)
            e1.record(cur)
            torch.cuda.synchronize()
            best = min(best, e0.elapsed_time(e1))
        return round(best, 3)

    def pipe(n_total, order):
        """bench.py's loop (sync one chunk ahead, TX, wait, RX) over n_total chunks on three streams"""
        s_sync = torch.cuda.Stream(device=dev, priority=-1)
        s_tx, s_rx = sA, sB
        evs = [torch.cuda.Event() for _ in range(3)]
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        sync(s_sync)
        evs[0].record(s_sync)
        for k in range(n_total):
            if k + 1 < n_total:
                sync(s_sync)
                evs[(k + 1) % 3].record(s_sync)
            if order == "rx_first" and k > 0:
                rx(s_rx)
            tx(s_tx)
            evs[k % 3].synchronize()
            if order != "rx_first":
                rx(s_rx)
        if order == "rx_first":
            rx(s_rx)
        torch.cuda.synchronize()
        return round((time.perf_counter() - t0) * 1e3 / n_total, 3)

    out = {"workload": wl, "chunk": chunk, "timing": os.environ.get("DNRP_TIMING", "0")}
    for order in ("bench", "rx_first"):
        pipe(2, order)
        out[f"pipe_{order}_ms_per_chunk"] = pipe(8, order)
    for k, f in stages.items():
        out[k] = timed([f])
    for a, b in (("tx", "sync"), ("tx", "rx"), ("sync", "rx")):
        out[f"{a}+{b}"] = timed([stages[a], stages[b]])
        out[f"{a}+{b}_serial_sum"] = round(out[a] + out[b], 3)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
