"""Entry-cut grid for the facade's one-shot trees (mesh.py closest_faces_and_points): a fresh tree per call, as the
reference builds one AabbTree per call, timed end to end through the numpy API with each grid (0 = none, -1 = the
automatic 64-cells-per-face grid) on C3 (100M uniform queries) and C2 (10M near-surface queries).  One JSON line
per (config, grid).

    python scripts/facade_cut_ab.py [--reps 3]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    import workloads as W
    from mesh_amd import search, _native
    from mesh_amd.mesh import Mesh
    cases = (("c3", W.c3_mesh(), np.random.default_rng(3).uniform(-1.1, 1.1, (100_000_000, 3)), (0, 100, 126, 160, 200)),
             ("c2", W.c2_mesh(), W.c2_queries(), (0, 24, 48, -1)))
    for name, (v, f), q, grids in cases:
        m = Mesh(v=v, f=f)
        for G in grids:
            def call():
                t = search.AabbTree(m)
                t.cpp_handle.set_entry_cut(G)
                r = t.nearest(q)
                return r, t.cpp_handle.entry_cut_info()
            call()  # warm-up (allocations, pools)
            walls, infos = [], []
            for _ in range(args.reps):
                t0 = time.perf_counter()
                _, info = call()
                walls.append(time.perf_counter() - t0)
                infos.append(info)
            print(json.dumps({"config": name, "G": G, "queries": int(q.shape[0]), "ms": [w * 1e3 for w in walls],
                              "ms_median": float(np.median(walls) * 1e3), "cut_build_ms": infos[-1]["build_ms"],
                              "cut_state": infos[-1]["state"], "cut_G": infos[-1]["G"], "build_id": _native.build_id()}),
                  flush=True)


if __name__ == "__main__":
    main()
