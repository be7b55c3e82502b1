"""Multi-rank path of bench.py on CPU (gloo, world_size 2): one process per device, independent slot
shards, no data-path collective; only the timing reduction (MAX over ranks) crosses ranks, and the
reported value is the whole-job aggregate."""
import os
import socket

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
        rng = np.random.default_rng(bench.shard_seed(rank))
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
