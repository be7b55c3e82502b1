"""TX kernel alone: ms per chunk of the bench workload (random d-bits), for kernel experiments.
python tools/tx_time.py [workload] [chunk] [reps] -- prints one line: workload, chunk, ms per chunk."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "dect-nr-plus-sdr_amd"))
import torch  # noqa: E402

import bench  # noqa: E402
import dnrp  # noqa: E402


def main():
    wl = sys.argv[1] if len(sys.argv) > 1 else "C4"
    chunk = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    psd, cfgt = bench.WORKLOADS[wl][:2]
    phy = dnrp.Phy(*cfgt, max_batch=chunk)
    for nid in range(100, 106):
        phy.add_network_id(nid)
    ps = dnrp.psdef(*psd)
    sz = phy.packet_sizes(ps)
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev)
    g.manual_seed(1)
    pcc = torch.randint(0, 256, (chunk, 25), dtype=torch.uint8, device=dev, generator=g)
    pdc = torch.randint(0, 256, (chunk, (sz["G"] + 7) // 8), dtype=torch.uint8, device=dev, generator=g)
    descs = (dnrp.TxDesc * chunk)(*[dnrp.TxDesc(0, 100 + i % 6, 1 + i % 2, 5, 1.0, 0.0, 0.001 * (i % 7), 0) for i in range(chunk)])
    out = torch.empty((chunk, sz["N_TX"], sz["N_samples_packet_os_rs"], 2), dtype=torch.float32, device=dev)
    phy.tx_batch(ps, descs, pcc, pdc, out)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        phy.tx_batch(ps, descs, pcc, pdc, out)
    e1.record()
    torch.cuda.synchronize()
    print(f"{os.environ.get('TAG', '')} {wl} chunk {chunk} tx ms/chunk {e0.elapsed_time(e1) / reps:.3f}", flush=True)




def fill_rate():
    """HBM write ceiling for the same output buffer: torch fill of the TX output (13.4 GB for C4)."""
    wl = sys.argv[1] if len(sys.argv) > 1 else "C4"
    chunk = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
    psd, cfgt = bench.WORKLOADS[wl][:2]
    phy = dnrp.Phy(*cfgt, max_batch=1)
    sz = phy.packet_sizes(dnrp.psdef(*psd))
    out = torch.empty((chunk, sz["N_TX"], sz["N_samples_packet_os_rs"], 2), dtype=torch.float32, device="cuda:0")
    out.zero_()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        out.zero_()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 5
    print(f"fill {out.numel() * 4 / 1e9:.2f} GB {ms:.3f} ms {out.numel() * 4 / ms / 1e6:.0f} GB/s", flush=True)


if __name__ == "__main__":
    fill_rate() if os.environ.get("FILL") else main()
