"""Multi-rank path of bench.py on CPU (gloo, world_size 2): one process per device, independent slot
shards, no data-path collective; only the timing reduction (MAX over ranks) crosses ranks, and the
reported value is the whole-job aggregate."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

import bench  # noqa: E402


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rng = np.random.default_rng(bench.slot_seed(bench.slot_range(rank, world, 2048)[0]))
        shard = rng.integers(0, 256, 64, dtype=np.uint8)  # first bytes of this rank's d-bit shard
        dist.barrier()
        t = bench.max_over_ranks(0.5 + rank, dist, "cpu")  # rank 1 is the slow one
        rate = bench.whole_job_rate(1024, 3, world, t)
        q.put((rank, shard.tobytes(), t, rate))
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_two_rank_shards_and_max_timing():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (r0, s0, t0, v0), (r1, s1, t1, v1) = res
    assert s0 != s1                        # independent shards
    assert t0 == t1 == 1.5                 # every rank reports the slowest rank's time
    assert v0 == v1 == pytest.approx(1024 * 3 * 2 / 1.5)


def test_single_rank_is_identity():
    assert bench.max_over_ranks(2.5) == 2.5
    assert bench.whole_job_rate(100, 2, 1, 4.0) == 50.0


def test_slot_ranges_partition():
    for world in (1, 2, 3, 4, 8):
        for total in (8, 1000, 524288):
            r = [bench.slot_range(g, world, total) for g in range(world)]
            assert r[0][0] == 0 and r[-1][1] == total
            assert all(r[g][1] == r[g + 1][0] for g in range(world - 1))
            assert all(lo == g * total // world and hi == (g + 1) * total // world for g, (lo, hi) in enumerate(r))


def test_bench_launcher_two_ranks():
    """bench.py --gpus 2 without a torchrun launcher spawns one child per device (RANK /
    LOCAL_RANK / WORLD_SIZE set before any device call); each owns its contiguous slot shard, draws
    its inputs from the global slot index, and rank 0 reports the whole-job rate over the slowest
    rank's time."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    out = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--dist-check",
                          "--batch", "1000", "--steps", "3"], env=env, capture_output=True, text=True, timeout=180)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout  # rank 0 only
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2
    sh = sorted(d["shards"], key=lambda e: e["rank"])
    assert [e["slots"] for e in sh] == [[0, 1000], [1000, 2000]]
    assert [e["local_rank"] for e in sh] == [0, 1]
    assert sh[0]["pid"] != sh[1]["pid"] and os.getpid() not in (sh[0]["pid"], sh[1]["pid"])
    for e in sh:  # inputs are a function of the global slot index, not of the rank
        exp = np.random.default_rng(bench.slot_seed(e["slots"][0])).integers(0, 256, 64, dtype=np.uint8)[:8]
        assert e["dbits0"] == exp.tolist()
    assert sh[0]["dbits0"] != sh[1]["dbits0"]
    assert d["elapsed"] >= 0.1  # the slowest rank (rank 1 sleeps 0.1 s)
    assert d["value"] == pytest.approx(1000 * 3 * 2 / d["elapsed"])
