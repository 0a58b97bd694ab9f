"""Development measurement: where the C3 traversal time goes, split by query population.

Runs the device-resident closest-point path on the C3 mesh for query sets drawn from the bench's
distribution (uniform in [-1.1, 1.1]^3): all, inside the unit sphere, outside, and radial shells, and
prints per set the traversal time per query and the instrumented node / leaf counts per query (one JSON
line per set).

    python scripts/c3_split.py [--queries 10000000]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--queries", type=int, default=10_000_000)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    import torch
    from mesh_amd import _native, spatialsearch
    from mesh_amd.distributed import nearest_device
    import workloads as W

    _native.set_device(0)
    v, f = W.c3_mesh()
    tree = spatialsearch.aabbtree_compute(v, f)
    S = args.queries
    rng = np.random.default_rng(3)
    pool = rng.uniform(-1.1, 1.1, (int(S * 3.2), 3))
    r = np.linalg.norm(pool, axis=1)
    sets = {
        "all": pool[:S],
        "inside": pool[r < 1.0][:S],
        "outside": pool[r >= 1.0][:S],
        "core_0_0.5": pool[r < 0.5],
        "shell_0.5_0.9": pool[(r >= 0.5) & (r < 0.9)],
        "shell_0.9_1.0": pool[(r >= 0.9) & (r < 1.0)],
        "shell_1.0_1.1": pool[(r >= 1.0) & (r < 1.1)],
        "outer_1.1+": pool[r >= 1.1],
    }
    for name, q in sets.items():
        q = np.ascontiguousarray(q)
        n = q.shape[0]
        dq = torch.from_numpy(q).cuda()
        face = torch.empty(n, dtype=torch.int32, device="cuda")
        part = torch.empty(n, dtype=torch.int32, device="cuda")
        pt = torch.empty((n, 3), dtype=torch.float64, device="cuda")
        nearest_device(tree, dq, face, part, pt)
        torch.cuda.synchronize()
        _native.timing_reset()
        _native.timing_enable(True)
        for _ in range(args.reps):
            nearest_device(tree, dq, face, part, pt)
        torch.cuda.synchronize()
        _native.timing_enable(False)
        res = {"set": name, "queries": n, "fraction_of_uniform": float(n) / pool.shape[0]}
        for k in ("nearest", "knn_pass1", "knn_pass2", "sort", "gather", "unpermute"):
            ms, c = _native.timing_get(k)
            res[k + "_ms"] = ms / max(c, 1)
        res["ns_per_query"] = res["nearest_ms"] * 1e6 / n
        nodes, leaves = _native.ctypes.c_uint64(0), _native.ctypes.c_uint64(0)
        _native.check(_native.lib().msh_tree_nearest_stats(tree.ptr, dq.data_ptr(), n, _native.ctypes.byref(nodes),
                                                            _native.ctypes.byref(leaves)))
        res["nodes_per_query"] = nodes.value / n
        res["leaves_per_query"] = leaves.value / n
        print(json.dumps(res), flush=True)
        del dq, face, part, pt
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
