"""Multi-process (world_size 2, gloo on CPU) coverage of the sharded path: query sharding, result
gather, and the blob broadcast transport used to replicate the BVH.  The RCCL/GPU variant of the same
functions runs in the driver's multi-GPU bench."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from mesh_amd.distributed import gather_results, shard_range


def test_shard_range_partitions():
    for n in [0, 1, 7, 8, 100, 100_000_003]:
        for world in [1, 2, 3, 8]:
            ranges = [shard_range(n, r, world) for r in range(world)]
            assert ranges[0][0] == 0 and ranges[-1][1] == n
            for (a, b), (c, d) in zip(ranges, ranges[1:]):
                assert b == c and b - a >= d - c >= b - a - 1
    with pytest.raises(ValueError):
        shard_range(10, 2, 2)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        total = 1001
        a, b = shard_range(total, rank, world)
        # each rank "answers" its shard: face = global query index, point = index * (1, 2, 3)
        idx = torch.arange(a, b, dtype=torch.int64)
        face = idx.to(torch.int32)
        pt = idx.to(torch.float64)[:, None] * torch.tensor([1.0, 2.0, 3.0], dtype=torch.float64)
        gf = gather_results(face, total)
        gp = gather_results(pt, total)
        # blob broadcast transport (the BVH replication path, here with a host byte blob)
        blob = torch.arange(4096, dtype=torch.int64).to(torch.uint8) if rank == 0 else torch.empty(4096, dtype=torch.uint8)
        dist.broadcast(blob, 0)
        out_q.put((rank, gf.numpy().copy(), gp.numpy().copy(), int(blob.sum())))
    finally:
        dist.destroy_process_group()


def test_gather_and_broadcast_world2():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want_sum = int(torch.arange(4096).to(torch.uint8).sum())
    for rank, gf, gp, bsum in res:
        assert (gf == np.arange(1001)).all()
        assert (gp == np.arange(1001)[:, None] * np.array([1.0, 2.0, 3.0])).all()
        assert bsum == want_sum
