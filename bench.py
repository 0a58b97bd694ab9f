"""Benchmark: closest-point queries/sec against a 1M-face mesh on MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[2]): class-I geodesic icosphere, frequency 224 = 1,003,520
faces / 501,762 vertices; ONE stream of 100M queries uniform in [-1.1, 1.1]^3 (seed 3) per step, sharded
contiguously over the N GPUs: every rank draws the whole stream in HBM (the same rows on every device) and
answers its shard_range.  One step = one pass of the hot path over the stream: query Morton codes -> LDS radix
sort -> LBVH traversal with fp64 CGAL-construction refinement -> results scattered back to query order (face
u32, part u32, point 3 x f64), and for N > 1 the all-gather of every rank's (face, part, point) slab, so the
whole 100M-row answer is on every rank (SURVEY §8(d)'s primary metric; RCCL over xGMI, each batch's gather
overlapped with the next batch's traversal by a double-buffered ResultRing, every gather finished inside the
timed region).  `value` = 100M x steps / max-over-ranks wall time (strong scaling).  Beside it for N > 1:
`value_without_allgather` (the same steps without the exchange) and `value_weak_100M_per_gpu` (every rank
answers the whole 100M stream and the N x 100M answers are all-gathered: the round-3 weak-scaling line).
The BVH build is setup (reported as build_ms); for N > 1 it is built on rank 0 and replicated with one RCCL
broadcast.  For N > 1 (or --secondary on) two more lines ride along, beside `value` and never as it:
`c5_visibility_sharded` (BASELINE configs[4]: 160M visibility rays per step, vertex ranges sharded) and
`c4_batch_sharded` (configs[3]: 4096 meshes x 10k scan points per step, mesh ranges sharded), see secondary().
For N > 1 `value_narrow_exchange` repeats the steps with the narrow exchange (faces all-gathered, the other ranks'
points rebuilt from (row, face): NarrowRing).  The tree asks for the fine entry cut (it answers many batches); the cut
is built by the first (warm-up) query, its time reported as entry_cut_ms.  `one_shot` (N = 1) times a fresh tree's
build + first batch with the default (coarse) cut.  --dist runs every collective path at N = 1 too (the nccl process
group, the broadcast unpacked on the source, both exchanges, the secondaries), as an 8-GPU node's ranks do.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--queries Q]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...
    python -m torch.distributed.run --nproc-per-node 1 ... bench.py --gpus 1 --dist

Rank 0 prints ONE JSON line.  `roofline` is for the traversal kernel (k_knn) on rank 0's shard: algorithmic
bytes per launch = S_rank * (56 + 64 * nodes/query + 80 * leaves/query) with the per-query
counts from the instrumented traversal of the same queries, divided by that kernel's average duration
measured with HIP events on its launch stream over the timed region.  `cpu_baseline` times the
oracle's CGAL-faithful restatement (1 thread, the reference's effective serial path) on a bounded
sample of the same workload.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "closest-point queries/sec vs 1M-face mesh at 1/2/4/8 MI355X + HBM GB/s"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
L2_PEAK_GBS = 34500.0  # MI355X_MICROARCH.md §L2: ~34.5 TB/s aggregate over the 8 XCDs


def waves_per_simd(isa):
    """Resident waves per SIMD of a 256-thread-block kernel with `vgpr` VGPRs and `lds` bytes of LDS per block
    (gfx950: 512 VGPRs per SIMD lane, 160 KB of LDS per CU, 4 SIMDs per CU; at most 8 waves per SIMD)."""
    vg, lds = int(isa.get("vgpr") or 0), int(isa.get("lds") or 0)
    by_vgpr = 512 // vg if vg else 8
    by_lds = (163840 // lds) * 4 // 4 if lds else 8  # blocks per CU x 4 waves per block / 4 SIMDs
    return min(8, by_vgpr, by_lds)


def issue_frac(tr):
    """VALU-busy fraction of the traversal kernel's SIMDs from the PMC record: each resident wave issues VALU in
    wave_cycles_valu_frac of its cycles, and waves_per_simd waves share a SIMD's VALU."""
    if not tr or tr.get("wave_cycles_valu_frac") is None or "vgpr" not in (tr.get("isa") or {}):
        return None
    return min(1.0, tr["wave_cycles_valu_frac"] * waves_per_simd(tr["isa"]))


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--queries", type=int, default=100_000_000,
                    help="queries per step: one C3 stream, sharded contiguously over the GPUs")
    ap.add_argument("--no-weak", action="store_true", help="N > 1: skip the weak-scaling (100M per GPU) line")
    ap.add_argument("--freq", type=int, default=224, help="icosphere frequency (224 -> 1,003,520 faces)")
    ap.add_argument("--cpu-queries", type=int, default=24000,
                    help="CPU baseline: fixed sample of queries per host thread (1 thread: ~12 s)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-one-shot", action="store_true",
                    help="skip the one-shot line (profiling runs: its fresh tree's traversals would mix into the kernel "
                         "statistics of the timed one)")
    ap.add_argument("--secondary", choices=("auto", "on", "off"), default="auto",
                    help="C5 visibility and C4 batch lines beside value (auto: when the collective path runs, the "
                         "configs north_star shards across GPUs)")
    ap.add_argument("--dist", action="store_true",
                    help="the collective path at any N, N = 1 included: the nccl (RCCL) process group, the tree's "
                         "RCCL broadcast unpacked on every rank (the source too), the ResultRing all-gathers, the "
                         "no-allgather / weak lines and the sharded C4 / C5 secondaries.  Launch under "
                         "torch.distributed.run (a plain launch gets a one-rank rendezvous on 127.0.0.1)")
    return ap.parse_args()


def free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def host_threads():
    """Host threads this process may use (the GPU box exports OMP_NUM_THREADS = its CPU share)."""
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and int(env) > 0:
        return int(env)
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:
        return os.cpu_count() or 1


def cpu_baseline(v, f, per_thread, stream_rows):
    """Oracle CGAL-tree restatement on the bench's own C3 query stream (rank 0), in two modes:
      * 1 thread (the reference's aabbtree_nearest loop is serial: its omp pragma is compiled out,
        spatialsearchmodule.cpp:212-214) -> the reported `cpu_baseline`;
      * all host threads this process may use (OpenMP over queries) -> `cpu_baseline_allcores`.
    Each mode answers a FIXED sample — the first rows of the stream the GPU answers (stream_rows(k): its first k
    rows copied to the host; per_thread x threads queries after 2,000 x threads warm-up rows) — and reports its
    total queries / total time, so the sample's
    content (its few costly queries near the sphere's centre, equidistant from much of the mesh) is identical
    from run to run and only the host's speed varies; 4 sub-chunks give the spread."""
    from oracle import oracle as O
    t0 = time.perf_counter()
    tree = O.CgalTree(v, f, hint=True)
    build_s = time.perf_counter() - t0
    out = {}
    for mode, threads in (("1", 1), ("all", host_threads())):
        n = per_thread * threads
        warm = 2000 * threads
        pool = stream_rows(warm + n)
        tree.nearest(pool[:warm], threads=threads)
        chunk = n // 4
        times = []
        for k in range(4):
            q = np.ascontiguousarray(pool[warm + k * chunk:warm + (k + 1) * chunk])
            t0 = time.perf_counter()
            tree.nearest(q, threads=threads)
            times.append(time.perf_counter() - t0)
        rates = [chunk / t for t in times]
        out[mode] = (4 * chunk / sum(times), 4 * chunk, threads, min(rates), max(rates))

    def obj(mode, label):
        rate, n, threads, lo, hi = out[mode]
        return {"value": rate, "unit": "queries/s", "cores": threads, "kind": "port",
                "sample": "%d uniform C3 queries (rows %d.. of the bench's own stream, the rows the GPU answers, "
                          "copied to the host; the same rows every session), total queries / total time (4 "
                          "sub-chunks: %.0f-%.0f q/s) on the "
                          "1,003,520-face icosphere; CGAL-faithful restatement (median-split AABB tree + KD hint, "
                          "fp64, g++ -O3 -ffp-contract=off), %s; tree build %.2f s excluded"
                          % (n, 2000 * threads, lo, hi, label, build_s)}
    return (obj("1", "1 thread (the reference's aabbtree_nearest loop is serial, spatialsearchmodule.cpp:212-217)"),
            obj("all", "OpenMP over queries on %d host threads" % out["all"][2]))


def secondary(timed, world, rank, dev, steps, coll):
    """BASELINE configs[4] and [3] through their multi-GPU splits (north_star: C5 rays sharded across the GPUs,
    C4 meshes split by range), reported beside `value`, never as it.  Each is timed like the headline (barrier +
    sync around K steps, max over ranks), after one untimed step:
      * C5 visibility: 64 Fibonacci cameras x the 2.5M vertices of the 5M-face bumped icosphere (160M rays); the
        tree is built on rank 0 and replicated by RCCL broadcast; every rank casts its vertex range for all
        cameras (visibility_device), and `with_gather` adds the all-gather that assembles the (C, P) outputs on
        every rank (visibility_sharded; reference loop visibility.cpp:136-173);
      * C4: 4096 meshes of one topology x 10k scan points; every rank generates only its mesh range, builds its
        batched tree and answers (batched build + query through the numpy API, then the mesh-slab all-gather:
        batch_nearest_sharded; the reference builds one AabbTree per mesh, spatialsearchmodule.cpp:272-321)."""
    import torch
    from mesh_amd import spatialsearch
    from mesh_amd.distributed import (batch_nearest_sharded, replicate_tree, shard_range, visibility_device,
                                      visibility_sharded)
    from mesh_amd.mesh import Mesh
    import workloads as W
    out = {}
    v5, f5 = W.c5_mesh()
    t5 = spatialsearch.aabbtree_compute(v5, f5) if rank == 0 else None
    if coll:
        r5 = replicate_tree(t5, src=0, unpack_on_src=world == 1)
        if r5 is not t5 and t5 is not None:
            t5.free()
        t5 = r5
    vn = torch.from_numpy(Mesh(v=v5, f=f5).estimate_vertex_normals()).to(dev)
    cams = torch.from_numpy(W.fibonacci_cameras(64, 3.0)).to(dev)
    P, C = v5.shape[0], 64
    a0, a1 = shard_range(P, rank, world)
    vis = torch.empty((C, a1 - a0), dtype=torch.int32, device=dev)
    ndc = torch.empty((C, a1 - a0), dtype=torch.float64, device=dev)
    local = lambda: visibility_device(t5, cams, vis, ndc, vn, None, 1e-3, a0, a1 - a0)  # noqa: E731
    gathered = lambda: visibility_sharded(t5, cams, vn)  # noqa: E731
    local()
    gathered()
    el_l = timed(local, steps)
    el_g = timed(gathered, steps)
    out["c5_visibility_sharded"] = {
        "workload": "C5: bumped icosphere (5,000,000 faces / 2,500,002 v), visibility of every vertex from 64 "
                    "Fibonacci cameras (160M rays) per step, vertex ranges sharded over the GPUs",
        "rays_per_s": C * P * steps / el_l, "ms_per_step": el_l / steps * 1e3,
        "rays_per_s_with_gather": C * P * steps / el_g, "ms_per_step_with_gather": el_g / steps * 1e3,
        "rays_per_gpu": C * (a1 - a0)}
    del t5, vn, vis, ndc, v5, f5
    torch.cuda.empty_cache()
    B, S = 4096, 10_000
    b0, b1 = shard_range(B, rank, world)
    t0 = time.perf_counter()
    v4, f4, q4 = W.c4_batch_range(b0, b1, B, S)
    gen_s = time.perf_counter() - t0
    step4 = lambda: batch_nearest_sharded(v4, f4, q4, device=dev)  # noqa: E731
    step4()
    el4 = timed(step4, steps)
    out["c4_batch_sharded"] = {
        "workload": "C4: 4096 meshes (5,042 v / 10,080 f, one topology) x 10k scan points per step, mesh ranges "
                    "sharded over the GPUs: batched build + query (numpy API) + mesh-slab all-gather",
        "queries_per_s": B * S * steps / el4, "ms_per_step": el4 / steps * 1e3, "meshes_per_gpu": b1 - b0,
        "input_generation_s": gen_s}
    return out


def load_traffic(workload, S, build_id):
    """profiles/pmc_traffic.json (scripts/pmc_summary.py): PMC HBM bytes per launch of the traversal
    kernels, and the latency-side counters of the same session.  Returned only when it was measured on
    this workload AND on the kernels of the loaded library (its build_id, msh_build_id: a hash of the
    sources) — otherwise (None, reason), so a profile of other code is never paired with this timing."""
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(p) as fh:
            d = json.load(fh)
    except (OSError, ValueError) as e:
        return None, "no PMC profile (%s)" % type(e).__name__
    if d.get("workload") != workload or int(d.get("queries") or 0) != S:
        return None, "PMC profile is of another workload"
    if d.get("build_id") != build_id:
        return None, "PMC profile is of build %s (code %s), not of the loaded build %s" % (
            d.get("build_id"), d.get("code"), build_id)
    return d, None


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        sys.exit("bench.py: --gpus %d but WORLD_SIZE %d (launch N>1 with torch.distributed.run --nproc-per-node N)"
                 % (args.gpus, world))
    # coll: the multi-GPU code path (process group, broadcast, all-gathers); always for N > 1, and at N = 1 with
    # --dist, so one GPU runs exactly what an 8-GPU node runs
    coll = world > 1 or args.dist
    if coll and "MASTER_ADDR" not in os.environ:  # --dist without torch.distributed.run: a one-rank rendezvous
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(free_port()), RANK="0", WORLD_SIZE="1")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if coll:
        dist.init_process_group("nccl", device_id=dev)

    from mesh_amd import _native, spatialsearch
    from mesh_amd.distributed import NarrowRing, ResultRing, nearest_device, points_from_faces_device, replicate_tree
    import workloads as W

    _native.set_device(local)
    v, f = W.geodesic_icosphere(args.freq)
    T = int(f.shape[0])
    S = args.queries
    workload = W.c3_workload_name(args.freq, S)

    # ---- setup: BVH build (rank 0) + RCCL replication ----
    tree = None
    if rank == 0:
        tree = spatialsearch.aabbtree_compute(v, f)
    build_ms = tree.info().build_ms if tree is not None else 0.0
    bcast_ms = 0.0
    if coll:
        torch.cuda.synchronize()
        dist.barrier()
        t0 = time.perf_counter()
        # at N = 1 the source unpacks the broadcast blob too, and the timed steps run on that handle
        replica = replicate_tree(tree, src=0, unpack_on_src=world == 1)
        bcast_ms = (time.perf_counter() - t0) * 1e3
        if replica is not tree:
            if tree is not None:
                tree.free()
            tree = replica

    # ---- inputs resident in HBM: the whole stream on every rank, this rank's contiguous shard ----
    q_all = W.c3_stream(S, dev)
    q, (a0, b0) = W.c3_shard(q_all, rank, world)
    S_loc = b0 - a0
    rows = -(-S // world)  # slab rows: the largest shard (equal shards for the all-gather)
    stream = torch.cuda.current_stream(dev).cuda_stream

    def slab(n):
        return (torch.empty(n, dtype=torch.int32, device=dev), torch.empty(n, dtype=torch.int32, device=dev),
                torch.empty((n, 3), dtype=torch.float64, device=dev))

    slabs = [slab(rows)]  # the steps without an exchange (N = 1, and the no-allgather line)
    ring = None
    if coll:
        # in place: each batch is answered into its own rows of the gathered buffers, which are all-gathered in place
        ring = ResultRing(None, [slab(world * rows) for _ in range(2)])

    def answer(sl):
        nearest_device(tree, q, sl[0][:S_loc], sl[1][:S_loc], sl[2][:S_loc], stream=stream)

    def step():  # one batch: the query pipeline on this rank's shard, and for N > 1 the all-gather of the answer
        if ring is None:
            answer(slabs[0])
        else:
            ring.step(answer)

    def timed(run, steps, rg=None):
        """barrier + sync, `steps` calls of run (every gather drained), sync + barrier; max over ranks"""
        if coll:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            run()
        if rg is not None:
            rg.drain()
        torch.cuda.synchronize()
        if coll:
            dist.barrier()
        el = time.perf_counter() - t0
        if coll:
            t = torch.tensor([el], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t.item())
        return el

    # the tree answers warmup + steps batches of 100M rows: a kept tree, which asks for the fine entry cut (64 cells per
    # face) at its first query instead of the coarse one the automatic policy builds first (api.cpp ensure_entry_cut)
    tree.set_entry_cut(-1)
    for _ in range(args.warmup):  # the first query also builds the tree's entry cut (lazily, once)
        step()
    if ring is not None:
        ring.drain()
    torch.cuda.synchronize()
    cut = tree.entry_cut_info()

    # ---- timed region: K steps (N > 1: each with its result all-gather) ----
    _native.timing_reset()
    _native.timing_enable(True)
    elapsed = timed(step, args.steps, ring)
    _native.timing_enable(False)
    k_ms, k_n = _native.timing_get("nearest")
    p1_ms, p1_n = _native.timing_get("knn_pass1")
    p2_ms, p2_n = _native.timing_get("knn_pass2")
    sl_ms, sl_n = _native.timing_get("knn_lead2")
    ld_ms, ld_n = _native.timing_get("knn_lead")
    fl_ms, fl_n = _native.timing_get("knn_follow")
    s_ms, s_n = _native.timing_get("sort")
    m_ms, m_n = _native.timing_get("morton")
    g_ms, g_n = _native.timing_get("gather")
    u_ms, u_n = _native.timing_get("unpermute")

    # ---- N > 1, reported beside value (never as value): the same steps without the exchange, with the narrow
    # exchange (faces only, the other ranks' points rebuilt locally: NarrowRing), and the weak-scaling line (every
    # rank answers the whole stream; the world x S answers are all-gathered) ----
    elapsed_no_ag = elapsed_weak = elapsed_narrow = None
    probe = None
    errors = {}
    if coll:
        elapsed_no_ag = timed(lambda: answer(slabs[0]), args.steps)
        if S % world == 0:
            try:  # a line beside value: a failure is reported, not fatal to the value line
                nring = NarrowRing(tree, q_all, S // world, [slab(S) for _ in range(2)])

                def narrow_step():
                    nring.step(lambda fc, pa, pt: nearest_device(tree, q, fc, pa, pt, stream=stream))

                narrow_step()
                nring.drain()
                elapsed_narrow = timed(narrow_step, args.steps, nring)
                del nring
            except Exception as e:  # noqa: BLE001
                errors["narrow_exchange"] = "%s: %s" % (type(e).__name__, e)
            torch.cuda.empty_cache()
        # the narrow exchange's rebuild on its own: the points and parts of 7/8 of the stream (what a rank of N = 8
        # rebuilds per step) from (row, face), against this rank's answers of the same rows (N = 1: all of them)
        if world == 1:
            m = S - S // 8
            answer(slabs[0])
            fc, pa, pt = (x[:m] for x in slabs[0])
            rp, rpt = torch.empty_like(pa), torch.empty_like(pt)
            points_from_faces_device(tree, q[:m], fc, rp, rpt, stream=stream)
            torch.cuda.synchronize()
            equal = bool(torch.equal(rp, pa) and torch.equal(rpt.view(torch.int64), pt.view(torch.int64)))
            _native.timing_reset()
            _native.timing_enable(True)
            for _ in range(args.steps):
                points_from_faces_device(tree, q[:m], fc, rp, rpt, stream=stream)
            torch.cuda.synchronize()
            _native.timing_enable(False)
            pms, pn = _native.timing_get("points_from_faces")
            probe = {"rows": m, "ms": pms / max(pn, 1), "bit_equal_to_traversal": equal,
                     "bytes_per_row_model": 24 + 4 + 4 + 80 + 24 + 4,
                     "note": "msh_tree_points_from_faces_device over rows [0, 7/8 S) of the stream (q row + face in, "
                             "face -> leaf map, the 80-B leaf, point + part out), HIP events on its stream"}
            del rp, rpt
            torch.cuda.empty_cache()
        if not args.no_weak:
            del ring
            torch.cuda.empty_cache()
            wg = slab(world * S)  # one gathered buffer written by both batches in turn: only the timing matters
            wring = ResultRing(None, [wg, wg])

            def weak_step():
                wring.step(lambda sl: nearest_device(tree, q_all, sl[0], sl[1], sl[2], stream=stream))

            weak_step()
            wring.drain()
            elapsed_weak = timed(weak_step, args.steps, wring)
            del wring, wg
            torch.cuda.empty_cache()

    # one-shot device caller (untimed for value): a fresh tree from the host mesh, its first 100M-row batch with the
    # automatic entry cut (the coarse grid, built by that call), results in HBM -- build + cut + batch
    one_shot = None
    if world == 1 and not args.no_one_shot:
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        t1 = spatialsearch.aabbtree_compute(v, f)
        nearest_device(t1, q, slabs[0][0][:S_loc], slabs[0][1][:S_loc], slabs[0][2][:S_loc], stream=stream)
        torch.cuda.synchronize()
        el1 = time.perf_counter() - t0
        c1 = t1.entry_cut_info()
        one_shot = {"ms": el1 * 1e3, "queries_per_s": S_loc / el1, "build_ms": t1.info().build_ms,
                    "entry_cut": {"G": c1["G"], "bytes": c1["bytes"], "build_ms": c1["build_ms"]},
                    "note": "wall time of aabbtree_compute (host mesh in) + one %d-row nearest_device call on the fresh "
                            "tree (its automatic entry cut built by that call), inputs and outputs in HBM" % S_loc}
        t1.free()
        del t1

    sec = None
    if args.secondary == "on" or (args.secondary == "auto" and coll):
        try:  # lines beside value: a failure is reported, not fatal to the value line
            sec = secondary(timed, world, rank, dev, args.steps, coll)
        except Exception as e:  # noqa: BLE001
            errors["secondary"] = "%s: %s" % (type(e).__name__, e)
            torch.cuda.empty_cache()

    # ---- instrumented traversal (untimed): algorithmic bytes of this rank's shard ----
    nodes, leaves = _native.ctypes.c_uint64(0), _native.ctypes.c_uint64(0)
    _native.check(_native.lib().msh_tree_nearest_stats(tree.ptr, q.data_ptr(), S_loc, _native.ctypes.byref(nodes),
                                                        _native.ctypes.byref(leaves)))
    n_node = nodes.value / S_loc
    n_leaf = leaves.value / S_loc
    info = tree.info()
    node_b, leaf_b = int(info.node_bytes), int(info.leaf_bytes)
    # bytes the traversal requests per query with this layout (node_b-B nodes, leaf_b-B leaves), and the
    # same counts priced with SURVEY §8(d)'s 64-B node model
    bytes_per_query = 56 + node_b * n_node + leaf_b * n_leaf
    bytes_per_query_s8d = 56 + 64 * n_node + 80 * n_leaf

    if rank != 0:
        if coll:
            dist.barrier()
            dist.destroy_process_group()
        return
    avg_kernel_s = (k_ms / max(k_n, 1)) / 1e3
    achieved = S_loc * bytes_per_query / avg_kernel_s / 1e9
    achieved_s8d = S_loc * bytes_per_query_s8d / avg_kernel_s / 1e9
    build_id = _native.build_id()
    tr, tr_reason = load_traffic(workload, S, build_id) if world == 1 else (None, "PMC profiles are of the N = 1 run")
    traffic = tr.get("bytes_per_launch") if tr else None
    total_q = S * args.steps
    out = {
        "metric": METRIC,
        "value": total_q / elapsed,
        "unit": "queries/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (seeded icosphere mesh + uniform query stream generated in HBM)",
        "config": {"workload": workload, "faces": T, "queries_total": S, "queries_per_gpu": S_loc,
                   "parallelism": "dp%d (one query stream sharded contiguously per GPU, BVH replicated by RCCL "
                                  "broadcast, answers all-gathered)" % world},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "kernel": "k_knn<0,false,true,true> + k_knn_coop<0,false> (pass 1 + pass 2: traversal + fp64 refinement)",
                     "kernel_ms": avg_kernel_s * 1e3, "queries_per_launch": S_loc, "bytes_per_query": bytes_per_query,
                     "node_bytes": node_b, "leaf_bytes": leaf_b,
                     "nodes_per_query": n_node, "leaves_per_query": n_leaf,
                     "s8d_64B_nodes": {"bytes_per_query": bytes_per_query_s8d, "achieved": achieved_s8d,
                                       "frac": achieved_s8d / HBM_PEAK_GBS},
                     "measured": ({"hbm_GBps": tr["bytes_per_launch"] / avg_kernel_s / 1e9,
                                   "l2_hit_rate": tr.get("l2_hit_rate"), "code": tr.get("code"),
                                   "build_id": tr.get("build_id"), "pmc_traversal_ms": tr.get("traversal_ms"),
                                   "isa": tr.get("isa")}
                                  if tr else None),
                     "traffic_note": tr_reason,
                     # the §8(d) byte model prices every node and leaf read as an HBM transfer; L2 and the
                     # Infinity Cache serve most of them (measured.hbm_GBps), so the model's rate can pass the peak
                     "frac_note": ("above 1: the §8(d) model counts cache-served node and leaf re-reads as HBM bytes; "
                                   "the fabric traffic is `measured`, and the kernel is bound by instruction issue "
                                   "and dependent-load latency (`latency`)") if achieved > HBM_PEAK_GBS else None,
                     # latency side: what bounds the kernel (node steps issued per second, live; lane
                     # occupancy and memory waits from the same build's SQ counters)
                     # two more ceilings for the same kernel (the HBM `frac` above prices cache-served re-reads as
                     # HBM bytes): the algorithmic bytes against the aggregate L2 rate (MI355X_MICROARCH.md §L2,
                     # ~34.5 TB/s), and the VALU pipe's busy fraction from the same build's SQ counters
                     # (wave-cycles issuing VALU x resident waves per SIMD)
                     "l2": achieved / L2_PEAK_GBS,
                     "l2_peak": L2_PEAK_GBS,
                     "issue": issue_frac(tr),
                     "issue_note": "SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES of k_knn x resident waves per SIMD (from its "
                                   "VGPR and LDS use; profiles/pmc_traffic.json at the same build id)" if tr else None,
                     "latency": {"node_steps_per_s": S_loc * n_node / avg_kernel_s,
                                 "leaf_tests_per_s": S_loc * n_leaf / avg_kernel_s,
                                 "lanes_active_valu": tr.get("lanes_active_valu") if tr else None,
                                 "wave_cycles_waiting_frac": tr.get("wave_cycles_waiting_frac") if tr else None,
                                 "wave_cycles_valu_frac": tr.get("wave_cycles_valu_frac") if tr else None}},
        "breakdown_ms_per_step": {"traversal": k_ms / max(k_n, 1), "pass1": p1_ms / max(p1_n, 1),
                                  "pass1_superleaders": sl_ms / max(sl_n, 1),
                                  "pass1_leaders": ld_ms / max(ld_n, 1), "pass1_followers": fl_ms / max(fl_n, 1),
                                  "pass2": p2_ms / max(p2_n, 1), "sort": s_ms / max(s_n, 1),
                                  "morton": m_ms / max(m_n, 1), "gather": g_ms / max(g_n, 1),
                                  "unpermute": u_ms / max(u_n, 1)},
        "build_ms": build_ms,
        "entry_cut_ms": cut["build_ms"],
        "entry_cut": {"state": cut["state"], "G": cut["G"], "bytes": cut["bytes"]},
        "build_id": build_id,
        "bvh_broadcast_ms": bcast_ms,
        # the multi-GPU code path ran (process group, RCCL broadcast + unpack, all-gathers): N > 1, or --dist at N = 1
        "collectives": ("nccl (RCCL), world %d%s" % (world, ", the source unpacks the broadcast blob" if world == 1
                                                      else "")) if coll else None,
    }
    if elapsed_no_ag is not None:
        out["value_without_allgather"] = total_q / elapsed_no_ag
        out["ms_per_step_without_allgather"] = elapsed_no_ag / args.steps * 1e3
        out["allgather_bytes_per_step"] = world * rows * 32  # (face u32, part u32, point 3 x f64) of every shard
    if elapsed_narrow is not None:
        out["value_narrow_exchange"] = total_q / elapsed_narrow
        out["ms_per_step_narrow_exchange"] = elapsed_narrow / args.steps * 1e3
        out["narrow_exchange_bytes_per_step"] = S * 4  # the face array, all-gathered in place
    if probe is not None:
        out["narrow_rebuild_probe"] = probe
    if one_shot is not None:
        out["one_shot"] = one_shot
    if errors:
        out["errors"] = errors
    if elapsed_weak is not None:
        out["value_weak_100M_per_gpu"] = world * S * args.steps / elapsed_weak
        out["ms_per_step_weak"] = elapsed_weak / args.steps * 1e3
    if sec:
        out.update(sec)
    if world == 1 and not args.no_cpu:
        out["cpu_baseline"], out["cpu_baseline_allcores"] = cpu_baseline(
            v, f, args.cpu_queries, lambda k: np.ascontiguousarray(q_all[:k].cpu().numpy()))
    print(json.dumps(out), flush=True)
    if coll:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
