"""A/B of the C5 ray kernels (BASELINE configs[4]) for one library build (MESH_AMD_LIB selects it): device-resident
nearest_alongnormal over the 10M C5 rays and visibility of the 2.5M vertices from 64 cameras, kernel times from the
library's HIP-event timers, node / leaf counts from the instrumented launches, and a SHA-256 of every output array,
so two builds can be compared bit for bit over all 10M rays and 160M visibility rays (a build already swept against
the oracle's brute force vouches for the other).  One JSON line on stdout.

    MESH_AMD_LIB=build/variants/x.so python scripts/c5_ab.py [--reps 5] [--brute 0]
"""
import argparse
import hashlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def sha(t):
    return hashlib.sha256(t.cpu().numpy().tobytes()).hexdigest()[:16]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--brute", type=int, default=0, help="also check this many rays against the oracle's brute force")
    args = ap.parse_args()
    import torch
    import workloads as W
    from mesh_amd import _native, spatialsearch
    from mesh_amd.distributed import alongnormal_device, visibility_device
    from mesh_amd.mesh import Mesh

    v, f = W.c5_mesh()
    tree = spatialsearch.aabbtree_compute(v, f)
    p, n, _, _ = W.c5_rays(v, f, 10_000_000, seed=5)
    S = p.shape[0]
    dp, dn = torch.from_numpy(p).cuda(), torch.from_numpy(n).cuda()
    d = torch.empty(S, dtype=torch.float64, device="cuda")
    fc = torch.empty(S, dtype=torch.int32, device="cuda")
    pt = torch.empty((S, 3), dtype=torch.float64, device="cuda")
    out = {"lib": os.path.basename(_native.LIB_PATH), "build_id": _native.build_id()}

    import time
    walls = {}

    def run(name, fn):
        fn()
        torch.cuda.synchronize()
        _native.timing_reset()
        _native.timing_enable(True)
        t0 = time.perf_counter()
        for _ in range(args.reps):
            fn()
        torch.cuda.synchronize()
        walls[name] = (time.perf_counter() - t0) / args.reps * 1e3
        _native.timing_enable(False)
        ms, cnt = _native.timing_get(name)
        walls[name + "_parts"] = {k: _native.timing_get(k)[0] / args.reps for k in ("morton", "sort", "gather")}
        return ms / max(cnt, 1)

    k_a = run("alongnormal", lambda: alongnormal_device(tree, dp, dn, d, fc, pt))
    nodes, leaves = _native.ctypes.c_uint64(0), _native.ctypes.c_uint64(0)
    _native.check(_native.lib().msh_tree_nearest_alongnormal_stats(tree.ptr, dp.data_ptr(), dn.data_ptr(), S,
                                                                    _native.ctypes.byref(nodes),
                                                                    _native.ctypes.byref(leaves)))
    out["alongnormal"] = {"kernel_ms": k_a, "rays_per_s_kernel": S / k_a * 1e3, "wall_ms": walls["alongnormal"],
                          "rays_per_s_device": S / walls["alongnormal"] * 1e3,
                          "order_ms": walls["alongnormal_parts"], "nodes_per_ray": nodes.value / S,
                          "leaves_per_ray": leaves.value / S,
                          "sha": [sha(d), sha(fc), sha(pt)]}
    if args.brute:
        from oracle import oracle as O
        idx = np.random.default_rng(11).choice(S, args.brute, replace=False)
        bd, bf, bpt = O.brute_alongnormal(v, f, p[idx], n[idx])
        gd, gf, gp = d.cpu().numpy()[idx], fc.cpu().numpy().view(np.uint32)[idx], pt.cpu().numpy()[idx]
        hit = bf != 0xFFFFFFFF
        bad = int(np.count_nonzero(gd != bd) + np.count_nonzero(gf != bf) +
                  np.count_nonzero(np.any(gp[hit] != bpt[hit], axis=1)))
        out["alongnormal"]["brute_rays"] = int(args.brute)
        out["alongnormal"]["brute_mismatches"] = bad
    del d, fc, pt
    cams = W.fibonacci_cameras(64, 3.0)
    vn = Mesh(v=v, f=f).estimate_vertex_normals()
    dc, dvn = torch.from_numpy(cams).cuda(), torch.from_numpy(vn).cuda()
    P, C = v.shape[0], cams.shape[0]
    vis = torch.empty((C, P), dtype=torch.int32, device="cuda")
    ndc = torch.empty((C, P), dtype=torch.float64, device="cuda")
    k_v = run("visibility", lambda: visibility_device(tree, dc, vis, ndc, dvn))
    _native.check(_native.lib().msh_visibility_stats(tree.ptr, dc.data_ptr(), C, 1e-3, _native.ctypes.byref(nodes),
                                                      _native.ctypes.byref(leaves)))
    out["visibility"] = {"kernel_ms": k_v, "wall_ms": walls["visibility"], "rays_per_s_kernel": C * P / k_v * 1e3, "nodes_per_ray": nodes.value / (C * P),
                         "leaves_per_ray": leaves.value / (C * P), "sha": [sha(vis), sha(ndc)]}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
