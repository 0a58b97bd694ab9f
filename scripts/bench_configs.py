"""Secondary measurements for BASELINE.md configs C1, C2, C4, C5, and C3 through the numpy API (bench.py
measures C3 device-resident, the headline).

One JSON line per config on stdout: the GPU path through the numpy API (the reference's entry points:
host arrays in, host arrays out), the device-resident rate (inputs already in HBM) where it differs, the
kernel time from the library's HIP-event timers, and the oracle's CGAL-faithful CPU restatement on a
sample (1 thread and all host threads).  Inputs are the seeded synthetic workloads of workloads.py.

    python scripts/bench_configs.py [--configs c1,c2,c3np,c4,c5] [--reps 3]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def pmc_of(target, kernel, units):
    """Measured fabric bytes of `kernel` in this config from profiles/pmc_configs.json (scripts/pmc_configs.py),
    only when that profile was taken of the loaded library (same msh_build_id); `units` = rays or queries per
    dispatch, to express them per unit.  None (with the reason) otherwise."""
    from mesh_amd import _native
    try:
        with open(os.path.join(ROOT, "profiles", "pmc_configs.json")) as fh:
            prof = json.load(fh).get(target)
    except (OSError, ValueError):
        prof = None
    if not prof:
        return {"note": "no PMC profile of %s" % target}
    if prof.get("build_id") != _native.build_id():
        return {"note": "PMC profile of %s is of build %s, not of the loaded build %s" % (
            target, prof.get("build_id"), _native.build_id())}
    k = prof["kernels"].get(kernel)
    if not k or not k.get("hbm_bytes_per_dispatch"):
        return {"note": "kernel %s not in the PMC profile" % kernel}
    return {"hbm_bytes_per_unit": k["hbm_bytes_per_dispatch"] / units, "hbm_GBps": k["hbm_GBps"],
            "l2_hit_rate": k["l2_hit_rate"], "pmc_ms_per_dispatch": k["ms_per_dispatch"],
            "build_id": prof["build_id"], "code": prof["code"],
            "note": "bytes leaving L2 (Infinity Cache hits included; DRAM traffic is at most this), "
                    "(2 FETCH_SIZE + WRITE_SIZE) KB per dispatch, gfx950 correction"}


def pmc_traversal(target, S):
    """Measured fabric bytes per query of the closest-point traversal (pass-1 launches + pass 2) in a config's
    PMC profile: every dispatch's bytes over (traversals x S), the profile's traversals = pass-2 dispatches (the
    entry cut's traversal dropped by pmc_configs.py --skip 1)."""
    k1, k2 = "msh::k_knn<0, false, true, true>", "msh::k_knn_coop<0, false>"
    a, b = pmc_of(target, k1, 1), pmc_of(target, k2, 1)
    if "hbm_bytes_per_unit" not in a or "hbm_bytes_per_unit" not in b:
        return a if "hbm_bytes_per_unit" not in a else b
    with open(os.path.join(ROOT, "profiles", "pmc_configs.json")) as fh:
        ks = json.load(fh)[target]["kernels"]
    n_trav = ks[k2]["dispatches"]
    tot = ks[k1]["hbm_bytes_total"] + ks[k2]["hbm_bytes_total"]
    hit = [ks[k]["counters_per_dispatch"] for k in (k1, k2)]
    h = sum(c.get("TCC_HIT_sum", 0.0) * ks[k]["dispatches"] for c, k in zip(hit, (k1, k2)))
    m = sum(c.get("TCC_MISS_sum", 0.0) * ks[k]["dispatches"] for c, k in zip(hit, (k1, k2)))
    return {"hbm_bytes_per_query": tot / (n_trav * S), "traversals": n_trav,
            "l2_hit_rate": h / (h + m) if h + m > 0 else None, "build_id": a["build_id"], "code": a["code"],
            "note": a["note"]}


def timed(fn, reps):
    from mesh_amd import _native
    # warm-up (allocations, code objects): two calls, the second held like the loop's previous result, so
    # the timed calls run in the steady state of a caller that keeps one result while asking for the next
    # (host calls: two pinned result blocks in the pool, reused alternately)
    out = fn()
    out = fn()
    _native.timing_reset()
    _native.timing_enable(True)
    t0 = time.perf_counter()
    for _ in range(reps):
        out = fn()
    wall = (time.perf_counter() - t0) / reps
    _native.timing_enable(False)
    return out, wall


def kernel_ms(name):
    from mesh_amd import _native
    ms, n = _native.timing_get(name)
    return ms / max(n, 1)


def host_threads():
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and int(env) > 0:
        return int(env)
    return len(os.sched_getaffinity(0))


def cpu_rates(v, f, q, budget_s=6.0):
    """Oracle CGAL-tree restatement on a sample of q: (1-thread q/s, all-thread q/s, threads); median of
    5 timed chunks after 2 warm-ups per mode (shortened for the secondary configs)."""
    from oracle import oracle as O
    tree = O.CgalTree(v, f, hint=True)
    out = []
    for threads in (1, host_threads()):
        n = min(q.shape[0], 1000 * threads)
        t0 = time.perf_counter()
        tree.nearest(q[:n], threads=threads)
        rate = n / max(time.perf_counter() - t0, 1e-6)
        chunk = int(min(max(rate * budget_s / 2 / 7, 200), q.shape[0]))
        rates = []
        for k in range(7):
            sel = q[(k * chunk) % max(q.shape[0] - chunk, 1):][:chunk]
            t0 = time.perf_counter()
            tree.nearest(sel, threads=threads)
            if k >= 2:
                rates.append(sel.shape[0] / (time.perf_counter() - t0))
        out.append(float(np.median(rates)))
    return out[0], out[1], host_threads()


def cpu_chunk_rates(run, units_per_item, n_items, budget_s=6.0):
    """run(lo, hi, threads) processes items [lo, hi) on the oracle; returns (1-thread units/s, all-thread
    units/s, threads): median of 5 timed chunks after 2 warm-ups per mode, chunks sized to the budget."""
    out = []
    for threads in (1, host_threads()):
        n = min(n_items, 50 * threads)
        t0 = time.perf_counter()
        run(0, n, threads)
        rate = n / max(time.perf_counter() - t0, 1e-6)
        chunk = int(min(max(rate * budget_s / 2 / 7, 8), n_items))
        rates = []
        for k in range(7):
            lo = (k * chunk) % max(n_items - chunk, 1)
            t0 = time.perf_counter()
            run(lo, lo + chunk, threads)
            if k >= 2:
                rates.append(chunk * units_per_item / (time.perf_counter() - t0))
        out.append(float(np.median(rates)))
    return out[0], out[1], host_threads()


def c1(reps):
    from mesh_amd.search import AabbTree
    from mesh_amd.mesh import Mesh
    import workloads as W
    v, f = W.sphere_fixture()
    q = W.c1_queries()
    tree = AabbTree(Mesh(v=v, f=f))
    _, wall = timed(lambda: tree.nearest(q, nearest_part=True), reps)
    c1t, cmt, th = cpu_rates(v, f, q)
    return {"config": "C1 sphere.obj (840 faces), 100k queries, AabbTree.nearest(nearest_part=True)",
            "queries_per_s_numpy_api": q.shape[0] / wall, "ms_numpy_api": wall * 1e3,
            "ms_traversal_kernel": kernel_ms("nearest"),
            "cpu_ref_1t_qps": c1t, "cpu_ref_omp_qps": cmt, "cpu_threads": th}


def c2(reps):
    import torch
    from mesh_amd import spatialsearch
    from mesh_amd.distributed import nearest_device
    import workloads as W
    v, f = W.c2_mesh()
    q = W.c2_queries()
    t0 = time.perf_counter()
    tree = spatialsearch.aabbtree_compute(v, f)
    build_wall = time.perf_counter() - t0
    _, wall = timed(lambda: spatialsearch.aabbtree_nearest(tree, q), reps)
    S = q.shape[0]
    dq = torch.from_numpy(q).cuda()
    face = torch.empty(S, dtype=torch.int32, device="cuda")
    part = torch.empty(S, dtype=torch.int32, device="cuda")
    pt = torch.empty((S, 3), dtype=torch.float64, device="cuda")
    wall_d = _device_timed(lambda: nearest_device(tree, dq, face, part, pt), reps)
    c1t, cmt, th = cpu_rates(v, f, q) if os.environ.get("MESH_AMD_NO_CPU") != "1" else (None, None, None)
    return {"config": "C2 SMPL-topology stand-in (6,890 v / 13,776 f), 10M near-surface queries",
            "queries_per_s_device": S / wall_d, "ms_traversal_kernel": kernel_ms("nearest"),
            "queries_per_s_numpy_api": S / wall, "ms_numpy_api": wall * 1e3,
            "build_ms_gpu": tree.info().build_ms, "build_ms_wall": build_wall * 1e3,
            "measured": pmc_traversal("c2", S),
            "cpu_ref_1t_qps": c1t, "cpu_ref_omp_qps": cmt, "cpu_threads": th}


def c3np(reps):
    """C3 through the reference's entry point (the secondary metric of SURVEY §8(d)): 100M host queries in,
    host arrays out — H2D + sort + traversal + D2H.  Two host paths of the library, timed on the same call:
    pageable -> pinned staging slabs copied by the library's host workers (the default) and the caller's arrays
    page-locked in place (hipHostRegister, MESH_AMD_HOST_REGISTER=1); both must give identical arrays."""
    from mesh_amd import spatialsearch
    import workloads as W
    v, f = W.c3_mesh()
    q = np.random.default_rng(3).uniform(-1.1, 1.1, (100_000_000, 3))
    tree = spatialsearch.aabbtree_compute(v, f)
    res = {}
    outs = {}
    for mode in ("0", "1"):
        os.environ["MESH_AMD_HOST_REGISTER"] = mode
        outs[mode], wall = timed(lambda: spatialsearch.aabbtree_nearest(tree, q), reps)
        res[mode] = (wall, kernel_ms("nearest"))
    os.environ.pop("MESH_AMD_HOST_REGISTER", None)
    same = all(np.array_equal(a, b) for a, b in zip(outs["1"], outs["0"]))
    return {"config": "C3 icosphere (1,003,520 faces), 100M uniform host queries, aabbtree_nearest (numpy API)",
            "queries_per_s_numpy_api": q.shape[0] / res["0"][0], "ms_numpy_api": res["0"][0] * 1e3,
            "host_path": "results carved from the library's pinned pool (downloaded in place), inputs through pinned "
                         "staging slabs filled by the library's copy workers, an 8M-row chunk then 20M-row chunks (host_plan)",
            "queries_per_s_numpy_api_registered": q.shape[0] / res["1"][0], "ms_numpy_api_registered": res["1"][0] * 1e3,
            "registered_equals_staged": bool(same),
            "ms_traversal_kernel": res["0"][1], "pcie_bytes_per_query": 56}


def c4(reps):
    import torch
    from mesh_amd import _native
    from mesh_amd.search import AabbTreeBatch
    import workloads as W
    t0 = time.perf_counter()
    v, f, q = W.c4_batch()
    gen_s = time.perf_counter() - t0

    def run():
        tree = AabbTreeBatch(v, f)
        return tree, tree.nearest(q, nearest_part=True)

    (tree, _), wall = timed(run, reps)
    n = q.shape[0] * q.shape[1]
    B, S = q.shape[0], q.shape[1]
    dq = torch.from_numpy(q).cuda()
    face = torch.empty((B, S), dtype=torch.int32, device="cuda")
    part = torch.empty((B, S), dtype=torch.int32, device="cuda")
    pt = torch.empty((B, S, 3), dtype=torch.float64, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
    h = tree.cpp_handle
    wall_d = _device_timed(lambda: _native.check(_native.lib().msh_batch_nearest_device(
        h.ptr, dq.data_ptr(), S, face.data_ptr(), part.data_ptr(), pt.data_ptr(), stream)), reps)
    # CPU: one CGAL-restatement tree per mesh (the reference's per-mesh AabbTree), 8 sampled meshes
    r1, rm = [], []
    for b in np.linspace(0, B - 1, 8).astype(int):
        a1, am, th = cpu_rates(v[b], f, q[b], budget_s=2.0)
        r1.append(a1)
        rm.append(am)
    return {"config": "C4 4096 meshes (5,042 v / 10,080 f, shared topology) x 10k scan points: batched build + query",
            "queries_per_s_numpy_api_build_plus_query": n / wall, "ms_build_plus_query_numpy_api": wall * 1e3,
            "queries_per_s_device_query_only": n / wall_d, "ms_device_query": wall_d * 1e3,
            "build_ms_gpu": tree.cpp_handle.info().build_ms, "ms_traversal_kernel": kernel_ms("nearest_batch"),
            "input_generation_s": gen_s, "cpu_ref_1t_qps_query_only": float(np.median(r1)),
            "cpu_ref_omp_qps_query_only": float(np.median(rm)), "cpu_threads": th,
            "cpu_note": "median over 8 sampled meshes of one CGAL-restatement tree each; tree builds excluded"}


def facade(reps):
    """Mesh.closest_faces_and_points end to end (the reference builds one AabbTree per call, mesh.py:454-455):
    build + query through the numpy API, on C2 (10M near-surface queries) and C3 (100M uniform queries).  The
    facade's tree goes without the entry cut (one batch does not pay for it); the same call on a tree that
    builds its cut on the first query is timed beside it."""
    from mesh_amd.mesh import Mesh
    from mesh_amd import search
    import workloads as W
    out = {"config": "Mesh.closest_faces_and_points end to end (tree build + entry cut policy + query, numpy API)"}
    for name, (v, f), q in (("c2", W.c2_mesh(), W.c2_queries()),
                            ("c3", W.c3_mesh(), np.random.default_rng(3).uniform(-1.1, 1.1, (100_000_000, 3)))):
        m = Mesh(v=v, f=f)
        _, wall = timed(lambda: m.closest_faces_and_points(q), reps)

        def with_cut():
            t = search.AabbTree(m)
            r = t.nearest(q)
            return r, t.cpp_handle.entry_cut_info()["build_ms"], t.cpp_handle.info().build_ms
        (_, cut_ms, build_ms), wall_cut = timed(with_cut, reps)
        out[name] = {"queries": q.shape[0], "ms_facade": wall * 1e3, "queries_per_s_facade": q.shape[0] / wall,
                     "ms_with_entry_cut": wall_cut * 1e3, "entry_cut_build_ms": cut_ms, "tree_build_ms_gpu": build_ms}
    return out


def _device_timed(fn, reps):
    import torch
    from mesh_amd import _native
    fn()
    torch.cuda.synchronize()
    _native.timing_reset()
    _native.timing_enable(True)
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / reps
    _native.timing_enable(False)
    return wall


def c5(reps):
    """C5: 10M nearest_alongnormal rays + visibility of 2.5M vertices from 64 cameras on the 5M-face bumped
    icosphere.  Device-resident rays/s (inputs in HBM) with the ray-kernel roofline, plus the numpy-API
    (end-to-end) rate of alongnormal."""
    import torch
    from mesh_amd import _native, spatialsearch
    from mesh_amd.distributed import alongnormal_device, visibility_device
    from mesh_amd.mesh import Mesh
    import workloads as W
    v, f = W.c5_mesh()
    tree = spatialsearch.aabbtree_compute(v, f)
    info = tree.info()
    nb, lb = int(info.node_bytes), int(info.leaf_bytes)
    p, n, _, _ = W.c5_rays(v, f, 10_000_000, seed=5)
    S = p.shape[0]
    _, wall_np = timed(lambda: spatialsearch.aabbtree_nearest_alongnormal(tree, p, n), reps)
    dp, dn = torch.from_numpy(p).cuda(), torch.from_numpy(n).cuda()
    d = torch.empty(S, dtype=torch.float64, device="cuda")
    fc = torch.empty(S, dtype=torch.int32, device="cuda")
    pt = torch.empty((S, 3), dtype=torch.float64, device="cuda")
    wall_r = _device_timed(lambda: alongnormal_device(tree, dp, dn, d, fc, pt), reps)
    k_r = kernel_ms("alongnormal")
    nodes, leaves = _native.ctypes.c_uint64(0), _native.ctypes.c_uint64(0)
    _native.check(_native.lib().msh_tree_nearest_alongnormal_stats(tree.ptr, dp.data_ptr(), dn.data_ptr(), S,
                                                                    _native.ctypes.byref(nodes),
                                                                    _native.ctypes.byref(leaves)))
    nn_r, nl_r = nodes.value / S, leaves.value / S
    b_r = 48 + 36 + nb * nn_r + lb * nl_r  # 48 B in + 36 B out per ray + nodes + leaves
    del d, fc, pt
    # visibility: 64 Fibonacci cameras, vertex normals (GPU), all vertices
    cams = W.fibonacci_cameras(64, 3.0)
    vn = Mesh(v=v, f=f).estimate_vertex_normals()
    dc, dvn = torch.from_numpy(cams).cuda(), torch.from_numpy(vn).cuda()
    P, C = v.shape[0], cams.shape[0]
    vis = torch.empty((C, P), dtype=torch.int32, device="cuda")
    ndc = torch.empty((C, P), dtype=torch.float64, device="cuda")
    wall_v = _device_timed(lambda: visibility_device(tree, dc, vis, ndc, dvn), reps)
    k_v = kernel_ms("visibility")
    # the same call through the numpy entry point (visibility_compute: the (C, P) outputs downloaded camera chunk by
    # camera chunk into pinned pool arrays); its bound is the kernel plus 12 B per ray over the host link
    from mesh_amd import visibility as VIS
    _, wall_vnp = timed(lambda: VIS.visibility_compute(cams=cams, tree=tree, n=vn), reps)
    link_gbs = 57.0  # pinned device-to-host rate of the box (profiles/r04_pcie_probe.json)
    _native.check(_native.lib().msh_visibility_stats(tree.ptr, dc.data_ptr(), C, 1e-3, _native.ctypes.byref(nodes),
                                                      _native.ctypes.byref(leaves)))
    R = C * P
    nn_v, nl_v = nodes.value / R, leaves.value / R
    cpu = c5_cpu(v, f, p, n, cams, vn) if os.environ.get("MESH_AMD_NO_CPU") != "1" else {}
    b_v = 12 + 48.0 / C + nb * nn_v + lb * nl_v  # 12 B out per ray, 48 B in amortised over C cameras
    return {"config": "C5 bumped icosphere (5,000,000 faces / 2,500,002 v): 10M nearest_alongnormal rays; "
                      "visibility 64 Fibonacci cameras x 2.5M vertices (160M rays), vertex normals",
            "alongnormal": {"rays_per_s_device": S / wall_r, "kernel_ms": k_r, "wall_ms_device": wall_r * 1e3,
                            "rays_per_s_numpy_api": S / wall_np, "nodes_per_ray": nn_r, "leaves_per_ray": nl_r,
                            "bytes_per_ray": b_r, "achieved_GBps": S * b_r / (k_r / 1e3) / 1e9,
                            "frac_of_8TBps": S * b_r / (k_r / 1e3) / 8e12,
                            "frac_note": "byte model (SURVEY 8d): every node and leaf request priced at full size, "
                                         "cache-served re-reads included",
                            "measured": pmc_of("c5", "msh::k_rays<0, false>", S)},
            "visibility": {"rays_per_s_device": R / wall_v, "kernel_ms": k_v, "wall_ms_device": wall_v * 1e3,
                           "rays_per_s_numpy_api": R / wall_vnp, "ms_numpy_api": wall_vnp * 1e3,
                           "numpy_bound_ms": k_v + 12.0 * R / link_gbs / 1e6,
                           "numpy_over_bound": wall_vnp * 1e3 / (k_v + 12.0 * R / link_gbs / 1e6),
                           "numpy_bound_note": "kernel + 12 B per ray of outputs at %.0f GB/s (no overlap)" % link_gbs,
                           "nodes_per_ray": nn_v, "leaves_per_ray": nl_v, "bytes_per_ray": b_v,
                           "achieved_GBps": R * b_v / (k_v / 1e3) / 1e9,
                           "frac_of_8TBps": R * b_v / (k_v / 1e3) / 8e12,
                           "frac_note": "byte model (SURVEY 8d): above 1 because L2 and the Infinity Cache serve the "
                                        "node re-reads (cache-served, not HBM); `measured` holds the fabric bytes",
                           "measured": pmc_of("c5", "msh::k_rays<1, false>", R),
                           "visible_fraction": float(vis.double().mean().item())},
            "build_ms_gpu": info.build_ms, **cpu}


def c5_cpu(v, f, p, n, cams, vn):
    """C5 on the oracle's CGAL-tree restatement (median-split tree, no hint; ray/box slab tests, the
    reference's all_intersections of both rays / do_intersect first-hit exit): rays per second on samples
    of the same rays (alongnormal) and of the same vertices seen from all 64 cameras (visibility)."""
    from oracle import oracle as O
    t0 = time.perf_counter()
    tree = O.CgalVisibilityTree(v, f)
    build_s = time.perf_counter() - t0
    rng = np.random.default_rng(55)
    sp = rng.permutation(p.shape[0])[:2_000_000]
    ps, ns = np.ascontiguousarray(p[sp]), np.ascontiguousarray(n[sp])
    a1, am, th = cpu_chunk_rates(lambda lo, hi, t: tree.alongnormal(ps[lo:hi], ns[lo:hi], threads=t), 1,
                                 ps.shape[0])
    sv = rng.permutation(v.shape[0])
    C = cams.shape[0]
    v1, vm, _ = cpu_chunk_rates(lambda lo, hi, t: tree.visibility(cams, n=vn, src_idx=sv[lo:hi], threads=t), C,
                                sv.shape[0])
    return {"cpu_ref_threads": th, "cpu_tree_build_s": build_s,
            "cpu_ref_alongnormal_1t_rays_per_s": a1, "cpu_ref_alongnormal_omp_rays_per_s": am,
            "cpu_ref_visibility_1t_rays_per_s": v1, "cpu_ref_visibility_omp_rays_per_s": vm,
            "cpu_sample": "random subsets of the same 10M alongnormal rays / of the 2.5M vertices x 64 cameras; "
                          "median of 5 timed chunks after 2 warm-ups, ~6 s per mode"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="c1,c2,c3np,c4,c5")
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    from mesh_amd import _native
    _native.set_device(0)
    fns = {"c1": c1, "c2": c2, "c3np": c3np, "c4": c4, "c5": c5, "facade": facade}
    for name in args.configs.split(","):
        r = fns[name](args.reps)
        r["name"] = name
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
