"""Multi-GPU execution of the search path: one process per GPU over torch.distributed (backend "nccl"
is RCCL on ROCm; xGMI between MI355X GPUs).

The path partitions by query: every rank holds the same mesh + BVH and answers a contiguous shard of
the queries.  The BVH is built once (on `src`) and replicated with ONE RCCL broadcast of its packed
blob (mesh vertices + 64-B nodes + 80-B leaves), instead of every rank rebuilding it.  Results stay
sharded in each rank's HBM; `gather_results` concatenates shards where a caller needs them in one
place (one all_gather per output array, padded to the largest shard).
"""
import numpy as np

from . import _native


def shard_range(n, rank, world):
    """Contiguous [start, stop) of `n` items for `rank` of `world` (first n % world ranks get +1)."""
    if world <= 0 or not (0 <= rank < world):
        raise ValueError("bad rank/world %r/%r" % (rank, world))
    base, rem = divmod(int(n), int(world))
    start = rank * base + min(rank, rem)
    return start, start + base + (1 if rank < rem else 0)


def replicate_tree(tree, src=0, device=None, group=None):
    """Broadcast a built tree from rank `src` to every rank (RCCL over xGMI); returns this rank's handle.

    `tree` is the handle on `src` (ignored elsewhere).  The blob is staged in a torch uint8 tensor
    on the rank's current CUDA (HIP) device.
    """
    import torch
    import torch.distributed as dist

    rank = dist.get_rank(group)
    dev = torch.device("cuda", torch.cuda.current_device() if device is None else device)
    nbytes = torch.zeros(1, dtype=torch.int64, device=dev)
    if rank == src:
        nbytes[0] = _native.blob_size(tree)
    dist.broadcast(nbytes, src, group=group)
    n = int(nbytes.item())
    blob = torch.empty(n, dtype=torch.uint8, device=dev)
    if rank == src:
        _native.blob_pack(tree, blob.data_ptr(), None)
    torch.cuda.synchronize(dev)
    dist.broadcast(blob, src, group=group)
    torch.cuda.synchronize(dev)
    if rank == src:
        return tree
    kind = {0: "triangles", 1: "normals", 2: "points"}
    h = _native.blob_unpack(blob.data_ptr(), n, dev.index, None)
    h.kind = kind.get(int(h.info().kind), "triangles")
    return h


def gather_results(local, total, group=None):
    """All-gather a sharded result tensor (first dim = this rank's shard of `total` rows)."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    counts = [shard_range(total, r, world)[1] - shard_range(total, r, world)[0] for r in range(world)]
    mx = max(counts)
    pad = torch.zeros((mx,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    pad[: local.shape[0]] = local
    bufs = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(bufs, pad, group=group)
    return torch.cat([b[:c] for b, c in zip(bufs, counts)], 0)


def nearest_device(tree, q, face, part, pt, stream=None):
    """Device-resident closest-point query on torch tensors (q (S,3) f64, face/part (S,) int32 viewed as
    uint32, pt (S,3) f64), asynchronous on `stream` (default: torch's current stream)."""
    import torch

    if stream is None:
        stream = torch.cuda.current_stream(q.device).cuda_stream
    S = q.shape[0]
    _native.check(_native.lib().msh_tree_nearest_device(
        tree.ptr, q.data_ptr(), S, face.data_ptr(), part.data_ptr() if part is not None else None, pt.data_ptr(),
        stream))


def as_numpy_u32(t):
    return t.cpu().numpy().view(np.uint32)


def _stream(t, stream):
    import torch
    return torch.cuda.current_stream(t.device).cuda_stream if stream is None else stream


def nearest_bary_device(tree, q, face, pt, w, stream=None):
    """Device-resident closest point + barycentric weights (msh_tree_nearest_bary_device): q (S,3) f64,
    face (S,) int32 viewed as uint32, pt (S,3) f64, w (S,3) f64."""
    _native.check(_native.lib().msh_tree_nearest_bary_device(tree.ptr, q.data_ptr(), q.shape[0], face.data_ptr(),
                                                             pt.data_ptr(), w.data_ptr(), _stream(q, stream)))


def alongnormal_device(tree, p, n, dist, face, pt, stream=None):
    """Device-resident nearest_alongnormal (msh_tree_nearest_alongnormal_device) on torch tensors:
    p, n (S,3) f64 -> dist (S,) f64, face (S,) int32 viewed as uint32, pt (S,3) f64."""
    _native.check(_native.lib().msh_tree_nearest_alongnormal_device(
        tree.ptr, p.data_ptr(), n.data_ptr(), p.shape[0], dist.data_ptr(), face.data_ptr(), pt.data_ptr(),
        _stream(p, stream)))


def visibility_device(tree, cams, vis, ndc, normals=None, sensors=None, min_dist=1e-3, v_begin=0, v_count=None,
                      stream=None):
    """Device-resident visibility of main-mesh vertices [v_begin, v_begin + v_count) from every camera
    (msh_visibility_device): cams (C,3) f64, normals (P,3) f64 (global vertex index) or None, sensors
    (C,9) or None -> vis (C, v_count) int32 viewed as uint32, ndc (C, v_count) f64."""
    if v_count is None:
        v_count = int(tree.info().n_points) - v_begin
    _native.check(_native.lib().msh_visibility_device(
        tree.ptr, cams.data_ptr(), cams.shape[0], normals.data_ptr() if normals is not None else None,
        sensors.data_ptr() if sensors is not None else None, float(min_dist), int(v_begin), int(v_count),
        vis.data_ptr(), ndc.data_ptr(), _stream(cams, stream)))


def visibility_sharded(tree, cams, normals=None, sensors=None, min_dist=1e-3, group=None):
    """C5's multi-GPU split of visibility_compute (visibility.cpp:136-173 loops cameras x vertices):
    every rank casts the rays of its contiguous vertex range for all cameras, then the (C, P) result is
    assembled on every rank by one all_gather per output (vertex-range slabs, padded)."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    P = int(tree.info().n_points)
    C = cams.shape[0]
    v0, v1 = shard_range(P, rank, world)
    vis = torch.empty((C, v1 - v0), dtype=torch.int32, device=cams.device)
    ndc = torch.empty((C, v1 - v0), dtype=torch.float64, device=cams.device)
    visibility_device(tree, cams, vis, ndc, normals, sensors, min_dist, v0, v1 - v0)
    if world == 1:
        return vis, ndc
    # gather along the vertex axis: transpose so the sharded axis is first
    vis_all = gather_results(vis.t().contiguous(), P, group).t().contiguous()
    ndc_all = gather_results(ndc.t().contiguous(), P, group).t().contiguous()
    return vis_all, ndc_all
