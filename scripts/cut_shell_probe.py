"""Where does the fine entry cut pay on C3?  Node visits and traversal time per query of the C3 stream, split into bands
of the query's distance to the (unit) icosphere, for entry-cut grids G = 0 (root starts), 200 (the coarse automatic
grid) and 400 (the fine one).  One process, one JSON line per grid.

    python scripts/cut_shell_probe.py [--queries 20000000]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

BANDS = (0.0, 0.01, 0.02, 0.05, 0.1, 0.2, 0.4, 10.0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--queries", type=int, default=20_000_000)
    ap.add_argument("--grids", default="0,200,400")
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    import torch
    import workloads as W
    from mesh_amd import _native, spatialsearch
    from mesh_amd.distributed import nearest_device
    v, f = W.geodesic_icosphere(224)
    q = W.c3_stream(args.queries, "cuda:0")
    r = torch.linalg.norm(q, dim=1)
    d = (r - 1.0).abs()
    subsets = []
    for lo, hi in zip(BANDS[:-1], BANDS[1:]):
        m = (d >= lo) & (d < hi)
        subsets.append(((lo, hi), q[m].contiguous()))
    for G in (int(x) for x in args.grids.split(",")):
        t = spatialsearch.aabbtree_compute(v, f)
        t.set_entry_cut(G)
        rec = {"G": G, "build_id": _native.build_id(), "bands": []}
        for (lo, hi), qs in subsets:
            n = qs.shape[0]
            face = torch.empty(n, dtype=torch.int32, device="cuda:0")
            part = torch.empty_like(face)
            pt = torch.empty((n, 3), dtype=torch.float64, device="cuda:0")
            nearest_device(t, qs, face, part, pt)
            torch.cuda.synchronize()
            _native.timing_reset()
            _native.timing_enable(True)
            for _ in range(args.reps):
                nearest_device(t, qs, face, part, pt)
            torch.cuda.synchronize()
            _native.timing_enable(False)
            ms = sum(_native.timing_get(k)[0] for k in ("knn_pass1", "knn_pass2")) / args.reps
            nodes, leaves = _native.ctypes.c_uint64(0), _native.ctypes.c_uint64(0)
            _native.check(_native.lib().msh_tree_nearest_stats(t.ptr, qs.data_ptr(), n, _native.ctypes.byref(nodes),
                                                                _native.ctypes.byref(leaves)))
            rec["bands"].append({"band": [lo, hi], "frac": n / args.queries, "nodes": nodes.value / max(n, 1),
                                 "leaves": leaves.value / max(n, 1), "ns_per_query": ms * 1e6 / max(n, 1)})
        rec["cut"] = t.entry_cut_info()
        t.free()
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
