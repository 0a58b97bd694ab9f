"""Child process of tests/test_dist_gpu.py (not a test module): the multi-GPU code path on the box's one GPU.

Launched by torch.distributed.run with one rank, so its first GPU work is the nccl (RCCL) process group's
initialisation, exactly as a rank of bench.py's N > 1 run starts.  It then runs every collective path of
mesh_amd/distributed.py at world size 1 and compares each answer bit for bit with the one-process answer of the
same data (no process group involved):
  * replicate_tree: RCCL broadcast of the packed tree blob, unpacked on the source too (the receiver side of the
    transport; the blob is msh_tree_blob_pack's) -> closest points equal to the original handle's;
  * ResultRing: three query batches, each all-gathered (all_gather_into_tensor, async) while the next one runs;
  * NarrowRing (faces all-gathered in place) and the rebuild of points / parts from (row, face) it uses for the other
    ranks' rows (msh_tree_points_from_faces_device, here on every row, MSH_NO_FACE rows included);
  * visibility_sharded / alongnormal_sharded (C5) and batch_nearest_sharded (C4) through their all-gathers.
Writes a JSON report to argv[1].  The reference loops this split parallelises: spatialsearchmodule.cpp:212-217,
visibility.cpp:136-173 (search.py:21-30 for C4's tree per mesh).
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def main(out_path):
    import torch
    import torch.distributed as dist

    local = int(os.environ["LOCAL_RANK"])
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", device_id=dev)  # the first GPU work of this process
    import numpy as np
    import workloads as W
    from mesh_amd import _native, spatialsearch
    from mesh_amd.distributed import (ResultRing, alongnormal_device, alongnormal_sharded, batch_nearest_sharded,
                                      nearest_device, replicate_tree, visibility_device, visibility_sharded)
    from mesh_amd.mesh import Mesh
    from mesh_amd.search import AabbTreeBatch

    _native.set_device(local)
    rep = {"world": dist.get_world_size(), "backend": dist.get_backend()}

    def same(a, b):
        return all(bool(torch.equal(x, y)) for x, y in zip(a, b))

    # (1) tree replication through the RCCL broadcast, unpacked on the source
    v, f = W.geodesic_icosphere(40)  # 32,000 faces: above the entry cut's minimum
    src = spatialsearch.aabbtree_compute(v, f)
    dup = replicate_tree(src, src=0, unpack_on_src=True)
    rep["replica_is_new_handle"] = dup.ptr != src.ptr
    S = 300_000
    q = W.c3_stream(S, dev)

    def answer(tree, qq):
        n = qq.shape[0]
        out = (torch.empty(n, dtype=torch.int32, device=dev), torch.empty(n, dtype=torch.int32, device=dev),
               torch.empty((n, 3), dtype=torch.float64, device=dev))
        nearest_device(tree, qq, out[0], out[1], out[2])
        return out

    want = answer(src, q)
    got = answer(dup, q)
    torch.cuda.synchronize()
    rep["replica_equal"] = same(want, got)
    rep["replica_entry_cut"] = dup.entry_cut_info()["state"]

    # (2) ResultRing: 3 batches, each batch's all-gather overlapping the next batch's traversal
    world = dist.get_world_size()
    n = S // 3
    slabs = [(torch.empty(n, dtype=torch.int32, device=dev), torch.empty(n, dtype=torch.int32, device=dev),
              torch.empty((n, 3), dtype=torch.float64, device=dev)) for _ in range(2)]
    gathered = [(torch.empty(world * n, dtype=torch.int32, device=dev),
                 torch.empty(world * n, dtype=torch.int32, device=dev),
                 torch.empty((world * n, 3), dtype=torch.float64, device=dev)) for _ in range(2)]
    ring = ResultRing(slabs, gathered)
    batches = []

    def check(k, g):
        batches.append(same(g, tuple(x[k * n:(k + 1) * n] for x in want)))

    b = 0
    for k in range(3):
        b = ring.step(lambda sl, k=k: nearest_device(dup, q[k * n:(k + 1) * n], sl[0], sl[1], sl[2]))
        if k >= 1:  # batch k - 1 is intact in its own buffer while batch k runs
            check(k - 1, ring.result(1 - b))
    ring.drain()
    check(2, ring.result(b))
    rep["ring_batches_equal"] = batches

    # (2b) the narrow exchange: NarrowRing (faces all-gathered in place) for 3 steps of one batch, and the rebuild of
    # points and parts from (row, face) -- at world 1 no other rank's rows exist, so it runs on every row here
    from mesh_amd.distributed import NarrowRing, points_from_faces_device
    nbuf = [(torch.empty(world * n, dtype=torch.int32, device=dev), torch.empty(world * n, dtype=torch.int32, device=dev),
             torch.empty((world * n, 3), dtype=torch.float64, device=dev)) for _ in range(2)]
    nring = NarrowRing(dup, q[:world * n], n, nbuf)
    nb = []
    for k in range(3):
        b = nring.step(lambda fc, pa, pt: nearest_device(dup, q[:n], fc, pa, pt))
        if k >= 1:
            nb.append(same(nring.result(1 - b), tuple(x[:n] for x in want)))
    nring.drain()
    nb.append(same(nring.result(b), tuple(x[:n] for x in want)))
    rep["narrow_batches_equal"] = nb
    rpart = torch.empty_like(want[1])
    rpt = torch.empty_like(want[2])
    points_from_faces_device(dup, q, want[0], rpart, rpt)
    nf = want[0].clone()
    nf[::97] = -1  # MSH_NO_FACE rows: NaN points, part 0
    npart = torch.empty_like(want[1])
    npt = torch.empty_like(want[2])
    points_from_faces_device(dup, q, nf, npart, npt)
    torch.cuda.synchronize()
    rep["rebuild_equal"] = bool(torch.equal(rpart, want[1]) and torch.equal(rpt, want[2]))
    rep["rebuild_no_face"] = bool(torch.isnan(npt[::97]).all() and (npart[::97] == 0).all() and
                                  torch.equal(npt[1::97], want[2][1::97]))

    # (3) C5: visibility and nearest_alongnormal through their sharded helpers (all-gathers at world 1)
    v5, f5 = W.geodesic_icosphere(30)
    t5 = replicate_tree(spatialsearch.aabbtree_compute(v5, f5), src=0, unpack_on_src=True)
    vn = torch.from_numpy(Mesh(v=v5, f=f5).estimate_vertex_normals()).to(dev)
    cams = torch.from_numpy(W.fibonacci_cameras(8, 3.0)).to(dev)
    P = v5.shape[0]
    vis1 = torch.empty((8, P), dtype=torch.int32, device=dev)
    ndc1 = torch.empty((8, P), dtype=torch.float64, device=dev)
    visibility_device(t5, cams, vis1, ndc1, vn, None, 1e-3, 0, P)
    vis2, ndc2 = visibility_sharded(t5, cams, vn)
    torch.cuda.synchronize()
    rep["visibility_equal"] = same((vis1, ndc1), (vis2, ndc2))
    rep["visibility_visible_frac"] = float((vis1 != 0).double().mean())
    rng = np.random.default_rng(7)
    p = torch.from_numpy(v5 + rng.normal(0.0, 0.01, v5.shape)).to(dev)
    nn = vn.clone()
    d1 = torch.empty(P, dtype=torch.float64, device=dev)
    fc1 = torch.empty(P, dtype=torch.int32, device=dev)
    pt1 = torch.empty((P, 3), dtype=torch.float64, device=dev)
    alongnormal_device(t5, p, nn, d1, fc1, pt1)
    d2, fc2, pt2 = alongnormal_sharded(t5, p, nn)
    torch.cuda.synchronize()
    # rays without a hit carry NaN points: compare their bit patterns
    rep["alongnormal_equal"] = bool(torch.equal(d1, d2) and torch.equal(fc1, fc2) and
                                    torch.equal(pt1.view(torch.int64), pt2.view(torch.int64)))
    rep["alongnormal_hit_frac"] = float((fc1 != -1).double().mean())

    # (4) C4: meshes sharded by range, the mesh-slab all-gather
    B, S4 = 24, 3000
    v4, f4, q4 = W.c4_batch_range(0, B, B, S4)
    one = AabbTreeBatch(v4, f4).nearest(q4, nearest_part=True)
    sh = batch_nearest_sharded(v4, f4, q4, device=dev)
    rep["c4_equal"] = all(np.array_equal(a, b) for a, b in zip(one, sh))
    rep["c4_dtypes"] = [str(a.dtype) for a in sh]

    with open(out_path, "w") as fh:
        json.dump(rep, fh)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main(sys.argv[1])
