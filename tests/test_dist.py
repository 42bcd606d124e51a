"""world_size-2 gloo tests of the multi-GPU plumbing (fishnet_amd/dist.py) on
CPU: net-image broadcast, per-rank shards, max-over-ranks, result gather."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from tests.conftest import ROOT


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    import sys
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist

    import fishnet_amd as F
    from fishnet_amd import dist as D

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        cpu = torch.device("cpu")
        image = F.Net.from_bytes(F.synthesize_net(7, 128, 0)).image() if rank == 0 else None
        buf = D.broadcast_image(image, cpu)
        local_image = F.Net.from_bytes(F.synthesize_net(7, 128, 0)).image()
        same_image = bool(np.array_equal(buf.numpy(), local_image))
        pos = F.random_playouts(D.shard_seed(1, rank), 50, threads=2)
        mx = D.max_over_ranks(float(rank + 1), cpu)
        local = np.arange(rank * 10, rank * 10 + 3 + rank, dtype=np.int32)
        gathered = D.gather_to_rank0(local, cpu)
        q.put((rank, same_image, pos.tobytes(), mx, None if gathered is None else gathered.tolist()))
    finally:
        dist.destroy_process_group()


def test_two_rank_gloo_plumbing():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r = q.get(timeout=120)
        res[r[0]] = r
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[0][1] and res[1][1]                 # every rank holds rank 0's image
    assert res[0][2] != res[1][2]                  # disjoint shards (different seeds)
    assert res[0][3] == res[1][3] == 2.0           # max over ranks
    assert res[0][4] == [0, 1, 2, 10, 11, 12, 13]  # ragged gather, rank order
    assert res[1][4] is None


@pytest.mark.parametrize("total,world", [(10, 3), (1, 2), (1000, 8)])
def test_shard_range_partitions(total, world):
    from fishnet_amd.dist import shard_range
    spans = [shard_range(total, r, world) for r in range(world)]
    assert spans[0][0] == 0 and spans[-1][1] == total
    assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
