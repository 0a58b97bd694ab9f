"""Multi-GPU execution of the search path: one process per GPU over torch.distributed (backend "nccl"
is RCCL on ROCm; xGMI between MI355X GPUs).

The path partitions by query: every rank holds the same mesh + BVH and answers a contiguous shard of
the queries.  The BVH is built once (on `src`) and replicated with ONE RCCL broadcast of its packed
blob (mesh vertices + the 64-B nodes + 80-B leaves; the sizes are in blob_info's node_bytes / leaf_bytes),
instead of every rank rebuilding it.  Results stay sharded in each rank's HBM; `gather_results`
concatenates shards where a caller needs them in one place (one all_gather per output array, padded to
the largest shard); `gather_results_into` gathers equal shards straight into a preallocated tensor, and
`ResultRing` overlaps each batch's gather with the next batch's traversal.
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


def broadcast_bytes(blob, src=0, group=None, device=None):
    """Broadcast a uint8 tensor from rank `src` (its size first, then the bytes) and return this rank's
    copy.  `blob` is the tensor on `src` (ignored elsewhere); the copy lives on `device` (default: the
    device of `blob` on src, the current CUDA device elsewhere when the backend is nccl, else the CPU)."""
    import torch
    import torch.distributed as dist

    rank = dist.get_rank(group)
    if device is None:
        if rank == src:
            device = blob.device
        elif dist.get_backend(group) == "nccl":
            device = torch.device("cuda", torch.cuda.current_device())
        else:
            device = torch.device("cpu")
    nbytes = torch.zeros(1, dtype=torch.int64, device=device)
    if rank == src:
        nbytes[0] = blob.numel()
    dist.broadcast(nbytes, src, group=group)
    out = blob if rank == src else torch.empty(int(nbytes.item()), dtype=torch.uint8, device=device)
    dist.broadcast(out, src, group=group)
    return out


def blob_info(header_bytes):
    """Parse + validate a packed tree blob's header (host bytes, at least the header) with the library's
    msh_blob_header_parse (no device needed) -> dict of the layout fields."""
    import ctypes
    buf = np.frombuffer(bytes(header_bytes), dtype=np.uint8).copy()
    inf = _native.BlobInfo()
    _native.check(_native.lib().msh_blob_header_parse(buf.ctypes.data, buf.size, ctypes.byref(inf)))
    return {name: (list(getattr(inf, name)) if name == "origin" else getattr(inf, name)) for name, _ in inf._fields_}


def replicate_tree(tree, src=0, device=None, group=None, unpack_on_src=False):
    """Broadcast a built tree from rank `src` to every rank (RCCL over xGMI); returns this rank's handle.

    `tree` is the handle on `src` (ignored elsewhere).  The blob is packed into a torch uint8 tensor on
    the rank's current CUDA (HIP) device, broadcast once, and unpacked in place on the receivers.  With
    `unpack_on_src` the source also unpacks the broadcast blob and returns that new handle (the receiver side of
    the transport, which then runs even at world size 1; the caller keeps `tree`)."""
    import torch
    import torch.distributed as dist

    rank = dist.get_rank(group)
    dev = torch.device("cuda", torch.cuda.current_device() if device is None else device)
    blob = None
    if rank == src:
        blob = torch.empty(_native.blob_size(tree), dtype=torch.uint8, device=dev)
        _native.blob_pack(tree, blob.data_ptr(), None)
    torch.cuda.synchronize(dev)
    blob = broadcast_bytes(blob, src, group, device=dev)
    torch.cuda.synchronize(dev)
    if rank == src and not unpack_on_src:
        return tree
    kind = {0: "triangles", 1: "normals", 2: "points"}
    h = _native.blob_unpack(blob.data_ptr(), blob.numel(), dev.index, None)
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


def gather_results_into(out, local, group=None, async_op=False):
    """All-gather equal shards into a preallocated tensor: rank r's (n, ...) `local` lands in rows
    [r n, (r + 1) n) of `out` (world n, ...) — one all_gather_into_tensor, no padding, no concatenation.
    With async_op the work handle is returned: on RCCL the gather runs on the process group's stream after
    the work already enqueued on the current stream, and handle.wait() makes the current stream wait for it."""
    import torch.distributed as dist

    world = dist.get_world_size(group)
    if out.shape[0] != world * local.shape[0] or tuple(out.shape[1:]) != tuple(local.shape[1:]):
        raise ValueError("gather_results_into: out %s does not hold %d shards of %s"
                         % (tuple(out.shape), world, tuple(local.shape)))
    if out.dtype != local.dtype or not out.is_contiguous() or not local.is_contiguous():
        raise ValueError("gather_results_into: dtype / contiguity mismatch")
    return dist.all_gather_into_tensor(out, local, group=group, async_op=async_op)


class ResultRing(object):
    """Double-buffered result slabs of a stream of query batches on every rank, each batch's results
    all-gathered into its own gathered buffer (the whole answer on every rank, rank-major rows).  Batch k is
    answered into slab k % 2 and gathered into gathered[k % 2] while the all-gather of batch k - 1 runs on the
    process group's stream (over xGMI on RCCL), so the exchange overlaps the next traversal instead of following
    it; a slab and its gathered buffer are rewritten only after the gather that used them has completed (its
    handle is waited on, on the current stream, first).

    slabs: two tuples of local result tensors (e.g. face, part, point), or None for the in-place form (each slab the
    view of this rank's rows of its gathered buffer); gathered: two tuples of the matching (world n, ...) tensors
    (passing the same tuple twice is allowed when only the timing matters: the two gathers then write one buffer in
    turn).  step(compute) calls compute(slab) to enqueue batch k's work on the
    current stream, starts its gathers and returns k % 2; result(b) waits for batch b's gathers and returns
    gathered[b] — the answer of the newest batch started in that buffer; drain() waits for every gather."""

    def __init__(self, slabs, gathered, group=None):
        import torch.distributed as dist

        if slabs is None:
            # in place: this rank's slab of buffer b is the view of its own rows of gathered[b], and the all-gather
            # runs in place (no copy of the local rows; at world size 1 nothing moves)
            world, rank = dist.get_world_size(group), dist.get_rank(group)
            n = gathered[0][0].shape[0] // world
            slabs = [tuple(x[rank * n:(rank + 1) * n] for x in g) for g in gathered]
        if len(slabs) != 2 or len(gathered) != 2 or any(len(s) != len(gathered[0]) for s in slabs) or \
                len(gathered[1]) != len(gathered[0]):
            raise ValueError("ResultRing: two slabs and two gathered buffers of the same tensors")
        self.slabs, self.gathered, self.group = slabs, gathered, group
        self.pending = [[], []]
        self.k = 0

    def step(self, compute):
        b = self.k & 1
        self._wait(b)
        compute(self.slabs[b])
        self.pending[b] = [gather_results_into(g, x, self.group, async_op=True)
                           for g, x in zip(self.gathered[b], self.slabs[b])]
        self.k += 1
        return b

    def _wait(self, b):
        for w in self.pending[b]:
            w.wait()
        self.pending[b] = []

    def result(self, b):
        self._wait(b)
        return self.gathered[b]

    def drain(self):
        for b in (0, 1):
            self._wait(b)


def points_from_faces_device(tree, q, face, part, pt, stream=None):
    """msh_tree_points_from_faces_device: the closest point (and part) of each row of q (S,3) f64 on the face given
    in face (S,) int32 viewed as uint32 -- the construction the traversal stores for the face it finds, so rows
    answered with that face get their points bit for bit.  part may be None.  Asynchronous on `stream`."""
    _native.check(_native.lib().msh_tree_points_from_faces_device(
        tree.ptr, q.data_ptr(), q.shape[0], face.data_ptr(), part.data_ptr() if part is not None else None,
        pt.data_ptr(), _stream(q, stream)))


class NarrowRing(object):
    """The narrow form of ResultRing's exchange for closest-point batches: only the faces travel (4 B per row instead
    of face + part + point, 32 B), and every rank rebuilds the other ranks' points and parts from (query row, face)
    with msh_tree_points_from_faces_device, bit for bit the points their owners computed.  Every rank holds the
    whole query stream of a batch (q_all, rank-major: rank r's rows are [r n, (r + 1) n)), as bench.py's C3 stream
    and a broadcast query batch do.

    gathered: two tuples (face (world n,) int32, part (world n,) int32, point (world n, 3) f64).  step(compute) calls
    compute(face, part, point) with this rank's rows of buffer k % 2 (views: the answers land in place), starts the
    in-place all-gather of the face array, and finishes batch k - 1 -- its gather waited for and the other ranks'
    rows rebuilt on a side stream, so the rebuild overlaps batch k's traversal; result(b) / drain() wait for it."""

    def __init__(self, tree, q_all, n, gathered, group=None, rebuild=None):
        import torch
        import torch.distributed as dist

        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        if len(gathered) != 2 or any(len(g) != 3 for g in gathered) or q_all.shape[0] != self.world * n:
            raise ValueError("NarrowRing: two (face, part, point) buffers of world x n rows and a q_all of as many")
        for g in gathered:
            if g[0].shape[0] != self.world * n or g[1].shape[0] != self.world * n or tuple(g[2].shape) != (self.world * n, 3):
                raise ValueError("NarrowRing: gathered buffers of %d rows expected" % (self.world * n))
        self.tree, self.q_all, self.n, self.gathered, self.group = tree, q_all, n, gathered, group
        # rebuild(q, face, part, point, stream): the other ranks' rows (default: msh_tree_points_from_faces_device);
        # host tensors (the gloo tests) run it inline, without a side stream
        self.rebuild = rebuild or (lambda q, f, pa, pt, st: points_from_faces_device(tree, q, f, pa, pt, stream=st))
        self.side = torch.cuda.Stream(device=q_all.device) if q_all.is_cuda else None
        self.gwork = [None, None]   # the face all-gather of the batch in buffer b
        self.done = [None, None]    # event: buffer b's rebuild finished (on the side stream)
        self.k = 0

    def _own(self, b):
        a, z = self.rank * self.n, (self.rank + 1) * self.n
        return tuple(x[a:z] for x in self.gathered[b])

    def _finish(self, b):
        """wait for buffer b's face gather on the side stream and rebuild the other ranks' rows there"""
        import contextlib
        import torch
        w = self.gwork[b]
        if w is None:
            return
        self.gwork[b] = None
        face, part, pt = self.gathered[b]
        with (torch.cuda.stream(self.side) if self.side is not None else contextlib.nullcontext()):
            w.wait()  # the side stream waits for the gather (host tensors: the gather completes)
            a, z = self.rank * self.n, (self.rank + 1) * self.n
            for lo, hi in ((0, a), (z, self.world * self.n)):
                if hi > lo:
                    self.rebuild(self.q_all[lo:hi], face[lo:hi], part[lo:hi], pt[lo:hi],
                                 self.side.cuda_stream if self.side is not None else None)
            if self.side is not None:
                ev = torch.cuda.Event()
                ev.record(self.side)
                self.done[b] = ev

    def _ready(self, b):
        """the current stream waits until buffer b's batch is complete (gathered and rebuilt)"""
        import torch
        self._finish(b)
        if self.done[b] is not None:
            torch.cuda.current_stream(self.q_all.device).wait_event(self.done[b])
            self.done[b] = None

    def step(self, compute):
        import torch.distributed as dist

        b = self.k & 1
        self._ready(b)  # batch k - 2's buffer is free again
        face, part, pt = self._own(b)
        compute(face, part, pt)
        self.gwork[b] = dist.all_gather_into_tensor(self.gathered[b][0], face, group=self.group, async_op=True)
        self._finish(1 - b)  # batch k - 1: its rebuild overlaps this batch's traversal
        self.k += 1
        return b

    def result(self, b):
        self._ready(b)
        return self.gathered[b]

    def drain(self):
        for b in (0, 1):
            self._ready(b)


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


def _group(group=None):
    """(world, rank, collective) of the calling process: the sharded helpers below take their collective path (the
    all-gathers) whenever a process group is initialised, world size 1 included, so one GPU runs the same code as
    a multi-GPU node; without a process group they answer everything locally."""
    import torch.distributed as dist

    if not dist.is_initialized():
        return 1, 0, False
    return dist.get_world_size(group), dist.get_rank(group), True


def gather_columns(local, total, group=None):
    """All-gather a 2-D tensor sharded along its LAST axis (this rank holds the columns
    shard_range(total, rank, world)) into the whole (rows, total) tensor on every rank."""
    t = local.t().contiguous()
    return gather_results(t, total, group).t().contiguous()


def visibility_sharded(tree, cams, normals=None, sensors=None, min_dist=1e-3, group=None):
    """C5's multi-GPU split of visibility_compute (visibility.cpp:136-173 loops cameras x vertices):
    every rank casts the rays of its contiguous vertex range for all cameras, then the (C, P) result is
    assembled on every rank by one all_gather per output (vertex-range slabs, padded)."""
    import torch
    import torch.distributed as dist

    world, rank, coll = _group(group)
    P = int(tree.info().n_points)
    C = cams.shape[0]
    v0, v1 = shard_range(P, rank, world)
    vis = torch.empty((C, v1 - v0), dtype=torch.int32, device=cams.device)
    ndc = torch.empty((C, v1 - v0), dtype=torch.float64, device=cams.device)
    visibility_device(tree, cams, vis, ndc, normals, sensors, min_dist, v0, v1 - v0)
    if not coll:
        return vis, ndc
    return gather_columns(vis, P, group), gather_columns(ndc, P, group)


def alongnormal_sharded(tree, p, n, group=None):
    """C5's split of nearest_alongnormal: rank r answers the rays shard_range(S, r, world) of the (S,3)
    device tensors p, n; the (dist, face, point) slabs are all-gathered."""
    import torch
    import torch.distributed as dist

    world, rank, coll = _group(group)
    S = p.shape[0]
    a, b = shard_range(S, rank, world)
    d = torch.empty(b - a, dtype=torch.float64, device=p.device)
    fc = torch.empty(b - a, dtype=torch.int32, device=p.device)
    pt = torch.empty((b - a, 3), dtype=torch.float64, device=p.device)
    alongnormal_device(tree, p[a:b].contiguous(), n[a:b].contiguous(), d, fc, pt)
    if not coll:
        return d, fc, pt
    return gather_results(d, S, group), gather_results(fc, S, group), gather_results(pt, S, group)


def batch_nearest_sharded(v, f, q, group=None, device=None):
    """C4's multi-GPU split (BASELINE configs[3]): the B meshes of one topology are sharded by mesh range
    with no broadcast — rank r builds the batched tree of meshes shard_range(B, r, world) from its own
    host slice and answers their queries (the reference builds one AabbTree per mesh, search.py:21-30).
    v (B,P,3), f (T,3), q (B,S,3) host arrays -> (face (B,S) u32, part (B,S) u32, point (B,S,3) f64) numpy
    arrays on every rank (one all_gather per output over the mesh axis)."""
    import torch
    import torch.distributed as dist
    from .search import AabbTreeBatch

    world, rank, coll = _group(group)
    B, S = q.shape[0], q.shape[1]
    b0, b1 = shard_range(B, rank, world)
    if b1 > b0:
        face, part, pt = AabbTreeBatch(v[b0:b1], f).nearest(q[b0:b1], nearest_part=True)
    else:
        face, part, pt = np.empty((0, S), np.uint32), np.empty((0, S), np.uint32), np.empty((0, S, 3))
    if not coll:
        return face, part, pt
    return gather_mesh_slabs((face, part, pt), B, group, device)


def gather_mesh_slabs(arrays, B, group=None, device=None):
    """All-gather host numpy slabs sharded over the mesh axis (rank r holds meshes shard_range(B, r, world))
    -> the whole (B, ...) arrays on every rank.  uint32 arrays travel as int32 bit patterns."""
    import torch
    import torch.distributed as dist

    if device is None:
        device = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(group) == "nccl" else "cpu"
    out = []
    for a in arrays:
        u32 = a.dtype == np.uint32
        t = torch.from_numpy(np.ascontiguousarray(a.view(np.int32) if u32 else a)).to(device)
        g = gather_results(t, B, group).cpu().numpy()
        out.append(g.view(np.uint32) if u32 else g)
    return tuple(out)
