"""Secondary measurements for BASELINE.md configs C1, C2, C4, C5 (bench.py measures C3, the headline).

One JSON line per config on stdout.  Every number comes from the GPU path through the numpy API (the
reference's entry points: host arrays in, host arrays out) with the kernel time from the library's
HIP-event timers beside it.  Inputs are the seeded synthetic workloads of workloads.py.

    python scripts/bench_configs.py [--configs c1,c2,c4,c5] [--reps 3]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def timed(fn, reps):
    from mesh_amd import _native
    fn()  # warm-up (allocations, code objects)
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


def c1(reps):
    from mesh_amd.search import AabbTree
    from mesh_amd.mesh import Mesh
    import workloads as W
    v, f = W.sphere_fixture()
    q = W.c1_queries()
    tree = AabbTree(Mesh(v=v, f=f))
    _, wall = timed(lambda: tree.nearest(q, nearest_part=True), reps)
    return {"config": "C1 sphere.obj (840 faces), 100k queries, AabbTree.nearest(nearest_part=True)",
            "queries_per_s_numpy_api": q.shape[0] / wall, "ms_numpy_api": wall * 1e3,
            "ms_traversal_kernel": kernel_ms("nearest")}


def c2(reps):
    from mesh_amd import spatialsearch
    import workloads as W
    v, f = W.c2_mesh()
    q = W.c2_queries()
    t0 = time.perf_counter()
    tree = spatialsearch.aabbtree_compute(v, f)
    build_wall = time.perf_counter() - t0
    _, wall = timed(lambda: spatialsearch.aabbtree_nearest(tree, q), reps)
    return {"config": "C2 SMPL-topology stand-in (6,890 v / 13,776 f), 10M near-surface queries",
            "queries_per_s_numpy_api": q.shape[0] / wall, "ms_numpy_api": wall * 1e3,
            "ms_traversal_kernel": kernel_ms("nearest"), "build_ms_gpu": tree.info().build_ms,
            "build_ms_wall": build_wall * 1e3}


def c4(reps):
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
    return {"config": "C4 4096 meshes (5,042 v / 10,080 f, shared topology) x 10k scan points: batched build + query",
            "queries_per_s_numpy_api": n / wall, "ms_build_plus_query_numpy_api": wall * 1e3,
            "build_ms_gpu": tree.cpp_handle.info().build_ms, "ms_traversal_kernel": kernel_ms("nearest_batch"),
            "input_generation_s": gen_s}


def c5(reps):
    from mesh_amd import spatialsearch
    from mesh_amd.visibility import visibility_compute
    import workloads as W
    v, f = W.c5_mesh()
    tree = spatialsearch.aabbtree_compute(v, f)
    rng = np.random.default_rng(5)
    p, fi = W.surface_samples(v, f, 10_000_000, seed=5, sigma=0.0)
    tri = v[f[fi].astype(np.int64)]
    nrm = np.cross(tri[:, 1] - tri[:, 0], tri[:, 2] - tri[:, 0])
    nrm /= np.linalg.norm(nrm, axis=1, keepdims=True)
    p = p + nrm * rng.normal(scale=0.01, size=(p.shape[0], 1))
    _, wall_r = timed(lambda: spatialsearch.aabbtree_nearest_alongnormal(tree, p, nrm), reps)
    k_r = kernel_ms("alongnormal")
    # 64 cameras on a Fibonacci sphere of radius 3, vertex normals
    k = np.arange(64) + 0.5
    phi = np.arccos(1 - 2 * k / 64)
    th = np.pi * (1 + 5 ** 0.5) * k
    cams = 3.0 * np.stack([np.cos(th) * np.sin(phi), np.sin(th) * np.sin(phi), np.cos(phi)], axis=1)
    vn = np.zeros_like(v)
    fn = np.cross(v[f[:, 1]] - v[f[:, 0]], v[f[:, 2]] - v[f[:, 0]])
    for c in range(3):
        np.add.at(vn, f[:, c], fn)
    vn /= np.linalg.norm(vn, axis=1, keepdims=True)
    (vis, _), wall_v = timed(lambda: visibility_compute(cams=cams, tree=tree, n=vn), 1)
    return {"config": "C5 bumped icosphere (5,000,000 faces): 10M nearest_alongnormal rays; visibility 64 cams x 2.5M v",
            "rays_per_s_alongnormal_numpy_api": p.shape[0] / wall_r, "ms_alongnormal_kernel": k_r,
            "rays_per_s_visibility_numpy_api": vis.size / wall_v, "ms_visibility_kernel": kernel_ms("visibility"),
            "visible_fraction": float(vis.mean())}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="c1,c2,c4,c5")
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    from mesh_amd import _native
    _native.set_device(0)
    fns = {"c1": c1, "c2": c2, "c4": c4, "c5": c5}
    for name in args.configs.split(","):
        r = fns[name](args.reps)
        r["name"] = name
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
