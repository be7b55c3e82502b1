"""HBM probe: achievable read, write and read+write (copy) rates on this GPU for large buffers
(torch kernels), the ceilings the streaming kernels are compared with (docs/DESIGN_LOG.md §6)."""
import json
import torch

dev = torch.device("cuda:0")
n = 8 << 30  # 8 GiB per buffer
a = torch.empty(n // 4, dtype=torch.float32, device=dev)
b = torch.empty(n // 4, dtype=torch.float32, device=dev)
a.fill_(1.0)
b.fill_(2.0)
out = {}


def t(fn, bytes_moved, reps=5):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    return round(bytes_moved / ms / 1e6, 1)


out["write_GBs"] = t(lambda: a.fill_(3.0), n)
out["read_GBs"] = t(lambda: a.sum(), n)
out["copy_GBs_total"] = t(lambda: b.copy_(a), 2 * n)
# read 2 : write 1 (a + b -> a)
out["add_r2w1_GBs_total"] = t(lambda: a.add_(b), 3 * n)
print(json.dumps(out), flush=True)
