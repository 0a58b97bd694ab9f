"""Time the entry cut's build phases on C3 (one process per library build; MESH_AMD_LIB selects it): the cell-centre
walks (sort, pass 1, pass 2), the cut kernel, the grid's node visits per query on the C3 stream.  One JSON line.

    python scripts/cut_build_probe.py [--grid -1|G] [--queries 20000000]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--grid", type=int, default=-1)
    ap.add_argument("--queries", type=int, default=20_000_000)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    import torch
    import workloads as W
    from mesh_amd import _native, spatialsearch
    from mesh_amd.distributed import nearest_device
    v, f = W.geodesic_icosphere(224)
    q = W.c3_stream(args.queries, "cuda:0")
    face = torch.empty(args.queries, dtype=torch.int32, device="cuda:0")
    part = torch.empty_like(face)
    pt = torch.empty((args.queries, 3), dtype=torch.float64, device="cuda:0")
    out = {"lib": os.path.basename(_native.LIB_PATH), "build_id": _native.build_id(), "builds": []}
    for _ in range(args.reps):
        t = spatialsearch.aabbtree_compute(v, f)
        t.set_entry_cut(args.grid)
        torch.cuda.synchronize()
        _native.timing_reset()
        _native.timing_enable(True)
        nearest_device(t, q[:1000], face[:1000], part[:1000], pt[:1000])
        torch.cuda.synchronize()
        _native.timing_enable(False)
        names = ["cut_level", "knn_pass1", "knn_pass2", "sort", "morton", "nearest"]
        rec = {n: _native.timing_get(n) for n in names}
        info = t.entry_cut_info()
        rec["cut"] = info
        # node visits of the C3 stream from this grid
        nodes, leaves = _native.ctypes.c_uint64(0), _native.ctypes.c_uint64(0)
        _native.check(_native.lib().msh_tree_nearest_stats(t.ptr, q.data_ptr(), args.queries, _native.ctypes.byref(nodes),
                                                            _native.ctypes.byref(leaves)))
        rec["nodes_per_query"] = nodes.value / args.queries
        rec["leaves_per_query"] = leaves.value / args.queries
        out["builds"].append(rec)
        t.free()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
