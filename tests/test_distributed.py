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


# ---- blob replication path end to end (host side) and the C4 / C5 shard + gather index math ----
def _worker_blob_and_shards(rank, world, port, out_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import ctypes
        from mesh_amd import _native
        from mesh_amd.distributed import (blob_info, broadcast_bytes, gather_columns, gather_mesh_slabs,
                                          shard_range)
        res = {}
        # (1) rank 0 lays out a tree blob with the library (header + payload pattern), broadcasts it;
        #     every rank parses and validates the header with msh_blob_header_parse (no device)
        blob = None
        if rank == 0:
            inf = _native.BlobInfo()
            hdr = np.zeros(4096, np.uint8)
            _native.check(_native.lib().msh_blob_header_write(0, 50002, 100000, 100000, hdr.ctypes.data, hdr.size,
                                                              ctypes.byref(inf)))
            payload = np.zeros(int(inf.total), np.uint8)
            payload[:4096] = hdr[:4096]
            payload[int(inf.off_nodes):] = (np.arange(payload.size - int(inf.off_nodes)) % 251).astype(np.uint8)
            blob = torch.from_numpy(payload)
        got = broadcast_bytes(blob, 0)
        full = got.numpy()
        info = blob_info(full.tobytes())
        res["info"] = info
        res["tail_sum"] = int(full[int(info["off_nodes"]):].astype(np.int64).sum())
        # a truncated blob is rejected by the same parser
        try:
            blob_info(full[: int(info["total"]) - 1].tobytes())
            res["truncated_rejected"] = False
        except ValueError:
            res["truncated_rejected"] = True
        # (2) C5 visibility: (C, P) assembled from vertex-range column slabs
        C, P = 3, 1001
        v0, v1 = shard_range(P, rank, world)
        cols = torch.arange(v0, v1, dtype=torch.float64)[None, :] + 10000.0 * torch.arange(C)[:, None]
        res["vis"] = gather_columns(cols, P).numpy()
        # (3) C4: meshes sharded by range, host slabs gathered over the mesh axis (uint32 + float64)
        B, S = 7, 5
        b0, b1 = shard_range(B, rank, world)
        face = (np.arange(b0, b1)[:, None] * 100 + np.arange(S)[None, :]).astype(np.uint32)
        face[:, 0] = 0xFFFFFFFF  # a NO_FACE row survives the int32 transport
        pt = np.arange(b0, b1, dtype=np.float64)[:, None, None] * np.ones((1, S, 3))
        gf, gp = gather_mesh_slabs((face, pt), B)
        res["face"], res["pt"] = gf, gp
        out_q.put((rank, res))
    finally:
        dist.destroy_process_group()


def test_blob_and_shards_world2():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_blob_and_shards, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    infos = [r["info"] for _, r in res]
    assert infos[0] == infos[1]
    info = infos[0]
    assert info["kind"] == 0 and info["n_points"] == 50002 and info["n_faces"] == 100000
    assert info["node_bytes"] == 64 and info["leaf_bytes"] == 80
    assert info["off_nodes"] >= info["off_vertices"] + 50002 * 24
    assert info["off_leaves"] >= info["off_nodes"] + (100000 - 1) * info["node_bytes"]
    assert info["total"] >= info["off_leaves"] + 100000 * 80
    n = info["total"] - info["off_nodes"]
    want = int((np.arange(n) % 251).sum())
    C, P, B, S = 3, 1001, 7, 5
    for _, r in res:
        assert r["tail_sum"] == want and r["truncated_rejected"]
        assert (r["vis"] == np.arange(P)[None, :] + 10000.0 * np.arange(C)[:, None]).all()
        wf = (np.arange(B)[:, None] * 100 + np.arange(S)[None, :]).astype(np.uint32)
        wf[:, 0] = 0xFFFFFFFF
        assert r["face"].dtype == np.uint32 and (r["face"] == wf).all()
        assert (r["pt"] == np.arange(B, dtype=np.float64)[:, None, None]).all()


# ---- the bench's N > 1 step: every batch's results all-gathered, overlapped with the next batch ----
def _worker_ring(rank, world, port, out_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from mesh_amd.distributed import ResultRing, gather_results_into
        n = 257
        slabs = [(torch.empty(n, dtype=torch.int32), torch.empty((n, 3), dtype=torch.float64)) for _ in range(2)]
        gathered = [(torch.empty(world * n, dtype=torch.int32), torch.empty((world * n, 3), dtype=torch.float64))
                    for _ in range(2)]
        ring = ResultRing(slabs, gathered)

        def compute(k):
            def run(slab):
                face, pt = slab
                face.copy_(torch.arange(n, dtype=torch.int32) + 1000 * rank + 100000 * k)
                pt.copy_(face.to(torch.float64)[:, None] * torch.tensor([1.0, -1.0, 0.5], dtype=torch.float64))
            return run

        res = {"batches": []}
        for k in range(5):  # batch k - 1's gather may still run while batch k is computed
            b = ring.step(compute(k))
            if k >= 1:  # the previous batch's answer is intact in its own buffer while batch k runs
                g = ring.result(1 - b)
                res["batches"].append((k - 1, g[0].numpy().copy(), g[1].numpy().copy()))
        ring.drain()
        g = ring.result(b)
        res["batches"].append((4, g[0].numpy().copy(), g[1].numpy().copy()))
        # shape / dtype validation of the equal-shard gather
        try:
            gather_results_into(torch.empty(world * n + 1, dtype=torch.int32), slabs[0][0])
            res["bad_shape_rejected"] = False
        except ValueError:
            res["bad_shape_rejected"] = True
        out_q.put((rank, res))
    finally:
        dist.destroy_process_group()


def test_result_ring_world2():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_ring, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    n = 257
    for _, r in res:
        assert [k for k, _, _ in r["batches"]] == [0, 1, 2, 3, 4]
        for k, face, pt in r["batches"]:
            want = np.concatenate([np.arange(n) + 1000 * q + 100000 * k for q in range(world)]).astype(np.int32)
            assert (face == want).all()
            assert (pt == want[:, None].astype(np.float64) * np.array([1.0, -1.0, 0.5])).all()
        assert r["bad_shape_rejected"]


# ---- the bench's N > 1 workload: one C3 stream, drawn whole on every rank, answered in contiguous shards ----
def _worker_stream(rank, world, port, out_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import workloads as W
        from mesh_amd.distributed import gather_results
        S = 10_007  # not a multiple of the world size: the shards differ by one row
        q = W.c3_stream(S, "cpu")
        mine, (a, b) = W.c3_shard(q, rank, world)
        assert mine.is_contiguous() and mine.data_ptr() == q[a].data_ptr()
        # every rank drew the same stream; the gathered shards reassemble it (and its N = 1 draw)
        whole = gather_results(mine.clone(), S)
        out_q.put((rank, (a, b), whole.numpy().copy(), W.c3_stream(S, "cpu").numpy()))
    finally:
        dist.destroy_process_group()


def test_c3_stream_shards_world2():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_stream, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=180) for _ in range(world)], key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    import workloads as W
    ref = W.c3_stream(10_007, "cpu").numpy()
    assert [r[1] for r in res] == [(0, 5004), (5004, 10_007)]
    for _, _, whole, own in res:
        assert np.array_equal(whole, ref) and np.array_equal(own, ref)
    assert ref.min() >= -1.1 and ref.max() <= 1.1


# ---- the narrow exchange: faces all-gathered in place, the other ranks' rows rebuilt from (row, face) ----
def _worker_narrow(rank, world, port, out_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from mesh_amd.distributed import NarrowRing
        n = 131
        q_all = torch.arange(world * n * 3, dtype=torch.float64).reshape(world * n, 3) / 7.0

        def rule(q, face):  # stands in for the closest-point construction on a given face
            return (face * 3 + 1).to(torch.int32), q * 2.0 + face.to(torch.float64)[:, None]

        def rebuild(q, face, part, pt, stream):
            p, x = rule(q, face)
            part.copy_(p)
            pt.copy_(x)

        gathered = [(torch.full((world * n,), -5, dtype=torch.int32), torch.full((world * n,), -5, dtype=torch.int32),
                     torch.full((world * n, 3), -5.0, dtype=torch.float64)) for _ in range(2)]
        ring = NarrowRing(None, q_all, n, gathered, rebuild=rebuild)
        res = []
        for k in range(4):
            def compute(fc, pa, pt, k=k):
                rows = torch.arange(rank * n, (rank + 1) * n)
                fc.copy_((rows * 5 + k).to(torch.int32))
                p, x = rule(q_all[rank * n:(rank + 1) * n], fc)
                pa.copy_(p)
                pt.copy_(x)
            b = ring.step(compute)
            if k >= 1:
                g = ring.result(1 - b)
                res.append((k - 1, [t.numpy().copy() for t in g]))
        ring.drain()
        res.append((3, [t.numpy().copy() for t in ring.result(b)]))
        out_q.put((rank, res))
    finally:
        dist.destroy_process_group()


def test_narrow_ring_world2():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_narrow, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    n = 131
    q_all = np.arange(world * n * 3, dtype=np.float64).reshape(world * n, 3) / 7.0
    for _, batches in res:
        assert [k for k, _ in batches] == [0, 1, 2, 3]
        for k, (face, part, pt) in batches:
            want_f = (np.arange(world * n) * 5 + k).astype(np.int32)
            assert (face == want_f).all()
            assert (part == want_f * 3 + 1).all()
            assert (pt == q_all * 2.0 + want_f[:, None]).all()


def _worker_ring_inplace(rank, world, port, out_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from mesh_amd.distributed import ResultRing
        n = 97
        gathered = [(torch.full((world * n,), -1, dtype=torch.int32), torch.full((world * n, 3), -1.0, dtype=torch.float64))
                    for _ in range(2)]
        ring = ResultRing(None, gathered)  # in place: the slabs are this rank's rows of the gathered buffers
        res = []
        for k in range(3):
            def run(slab, k=k):
                face, pt = slab
                face.copy_(torch.arange(n, dtype=torch.int32) + 1000 * rank + 100000 * k)
                pt.copy_(face.to(torch.float64)[:, None] * torch.tensor([2.0, 0.5, -1.0], dtype=torch.float64))
            b = ring.step(run)
            g = ring.result(b)
            res.append((k, g[0].numpy().copy(), g[1].numpy().copy()))
        ring.drain()
        out_q.put((rank, res))
    finally:
        dist.destroy_process_group()


def test_result_ring_in_place_world2():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_ring_inplace, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    n = 97
    for _, batches in res:
        for k, face, pt in batches:
            want = np.concatenate([np.arange(n) + 1000 * r + 100000 * k for r in range(world)]).astype(np.int32)
            assert (face == want).all()
            assert (pt == want[:, None].astype(np.float64) * np.array([2.0, 0.5, -1.0])).all()
