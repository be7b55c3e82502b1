"""Per-(kernel, grid) summary of a rocprofv3 kernel trace CSV: one kernel template runs with several
grids (PCC/PDC front end, the 4096-slot chunks vs the tail), so the --stats average mixes them.
python tools/trace_by_grid.py <run_kernel_trace.csv> [--tail N] [name-substring ...]
--tail N keeps the last N launches of every (kernel, grid): bench.py's closing one-stream step (the
launches the roofline's HIP-event durations come from; the pipelined launches overlap each other)."""
import csv
import statistics
import sys
from collections import defaultdict


def main():
    path = sys.argv[1]
    keys = sys.argv[2:]
    tail = 0
    if keys[:1] == ["--tail"]:
        tail, keys = int(keys[1]), keys[2:]
    rows = defaultdict(list)
    with open(path, newline="") as f:
        for r in csv.DictReader(f):
            name = r["Kernel_Name"]
            if keys and not any(k in name for k in keys):
                continue
            short = name.split("(")[0].replace("void ", "").replace("dnrp::dev::", "")
            grid = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
            rows[(short, grid)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    print(f"{'kernel@grid':64s} {'calls':>6s} {'avg_ms':>8s} {'median':>8s} {'min':>8s} {'max':>8s}")
    if tail:
        rows = {k: v[-tail:] for k, v in rows.items()}
    for (short, grid), d in sorted(rows.items(), key=lambda kv: -sum(kv[1])):
        print(f"{short + '@' + str(grid):64s} {len(d):6d} {statistics.fmean(d):8.3f} "
              f"{statistics.median(d):8.3f} {min(d):8.3f} {max(d):8.3f}")


if __name__ == "__main__":
    main()
