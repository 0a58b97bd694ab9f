"""One-off parity sweeps at full config sizes (not part of the test suite: each takes up to a minute of host
brute force), one JSON line per config:
  c3  bench.py's exact query stream (100M uniform queries generated in HBM, seed 3) through the device entry
      point; K random rows plus the rows nearest the sphere's centre (the deferred pass-2 queries);
  c2  the 10M C2 queries through the numpy entry point (aabbtree_nearest); K random rows;
  c5  the 10M C5 nearest_alongnormal rays through the numpy entry point; --rays random rays;
  c5v visibility_compute (numpy) on the C5 mesh from the 64 Fibonacci cameras with vertex normals: --pairs
      (camera, vertex) pairs (8 cameras x pairs/8 vertices), and --sensor-pairs more with random sensors
      (2 cameras), against oracle.brute_visibility (every one of the 5M triangles).
Every checked row must equal the oracle's exhaustive brute force bit for bit (same tie rule).

    python scripts/parity_sweep.py [--configs c3,c2,c5] [--rows 20000] [--centre 2000]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def sweep_c3(args):
    import torch
    from mesh_amd import _native, spatialsearch
    from mesh_amd.distributed import nearest_device
    from oracle import oracle as O
    import workloads as W
    v, f = W.c3_mesh()
    S = 100_000_000
    g = torch.Generator(device="cuda:0")
    g.manual_seed(3)
    dq = (torch.rand((S, 3), generator=g, dtype=torch.float64, device="cuda:0") * 2.2 - 1.1).contiguous()
    print("c3: stream generated", file=sys.stderr, flush=True)
    t = spatialsearch.aabbtree_compute(v, f)
    df = torch.empty(S, dtype=torch.int32, device="cuda:0")
    dp = torch.empty(S, dtype=torch.int32, device="cuda:0")
    dpt = torch.empty((S, 3), dtype=torch.float64, device="cuda:0")
    nearest_device(t, dq, df, dp, dpt)
    torch.cuda.synchronize()
    q = dq.cpu().numpy()
    del dq
    face = df.cpu().numpy().view(np.uint32)
    part = dp.cpu().numpy().view(np.uint32)
    pt = dpt.cpu().numpy()
    r = np.sqrt(np.einsum("ij,ij->i", q, q))
    idx = np.concatenate([np.random.default_rng(11).choice(S, args.rows, replace=False),
                          np.argpartition(r, args.centre)[:args.centre]])
    t0 = time.perf_counter()
    chunks = []
    for c0 in range(0, idx.size, 2000):  # progress lines: a long silent brute force looks hung on the GPU box
        chunks.append(O.brute_nearest(v, f, q[idx[c0:c0 + 2000]]))
        print("c3 brute force: %d / %d rows" % (min(c0 + 2000, idx.size), idx.size), file=sys.stderr, flush=True)
    bf, bp, bpt = (np.concatenate([c[k] for c in chunks]) for k in range(3))
    bad = np.nonzero((face[idx] != bf) | (part[idx] != bp) | np.any(pt[idx] != bpt, axis=1))[0]
    return dict(workload="C3 headline stream (100M uniform queries, seed 3, device entry point)",
                random_rows=args.rows, centre_rows=args.centre, rows_checked=int(idx.size), mismatches=int(bad.size),
                first_mismatch_rows=idx[bad[:10]].tolist(), brute_force_s=time.perf_counter() - t0,
                check="face, part code and point bit-exact vs oracle.brute_nearest (lexicographic (d2, face))")


def sweep_c2(args):
    from mesh_amd import spatialsearch
    from oracle import oracle as O
    import workloads as W
    v, f = W.c2_mesh()
    q = W.c2_queries()
    face, part, pt = spatialsearch.aabbtree_nearest(spatialsearch.aabbtree_compute(v, f), q)
    idx = np.random.default_rng(12).choice(q.shape[0], 5 * args.rows, replace=False)
    t0 = time.perf_counter()
    chunks = []
    for c0 in range(0, idx.size, 20000):  # progress lines (a silent minute looks hung on the GPU box)
        chunks.append(O.brute_nearest(v, f, q[idx[c0:c0 + 20000]]))
        print("c2 brute force: %d / %d rows" % (min(c0 + 20000, idx.size), idx.size), file=sys.stderr, flush=True)
    bf, bp, bpt = (np.concatenate([c[k] for c in chunks]) for k in range(3))
    bad = np.nonzero((face[0][idx] != bf) | (part[0][idx] != bp) | np.any(pt[idx] != bpt, axis=1))[0]
    return dict(workload="C2 10M near-surface queries (numpy entry point aabbtree_nearest)", rows_checked=int(idx.size),
                mismatches=int(bad.size), first_mismatch_rows=idx[bad[:10]].tolist(), brute_force_s=time.perf_counter() - t0,
                check="face, part code and point bit-exact vs oracle.brute_nearest")


def sweep_c5(args):
    from mesh_amd import spatialsearch
    from oracle import oracle as O
    import workloads as W
    v, f = W.c5_mesh()
    p, n, _, _ = W.c5_rays(v, f)
    d, face, pt = spatialsearch.aabbtree_nearest_alongnormal(spatialsearch.aabbtree_compute(v, f), p, n)
    idx = np.random.default_rng(13).choice(p.shape[0], args.rays, replace=False)
    t0 = time.perf_counter()
    parts = []
    for c0 in range(0, idx.size, 2000):  # progress lines
        parts.append(O.brute_alongnormal(v, f, p[idx[c0:c0 + 2000]], n[idx[c0:c0 + 2000]]))
        print("c5 brute force: %d / %d rays" % (min(c0 + 2000, idx.size), idx.size), file=sys.stderr, flush=True)
    bd, bf, bpt = (np.concatenate([c[k] for c in parts]) for k in range(3))
    hit = bd < 1e100
    same_pt = np.all((pt[idx] == bpt) | ~hit[:, None], axis=1)
    bad = np.nonzero((d[idx] != bd) | (face[idx] != bf) | ~same_pt)[0]
    return dict(workload="C5 10M nearest_alongnormal rays on the 5M-face bumped icosphere (numpy entry point)",
                rows_checked=int(idx.size), mismatches=int(bad.size), first_mismatch_rows=idx[bad[:10]].tolist(),
                misses=int((~hit).sum()), brute_force_s=time.perf_counter() - t0,
                check="dist, face and (for hits) point bit-exact vs oracle.brute_alongnormal")


def sweep_c5v(args):
    from mesh_amd import spatialsearch, visibility
    from mesh_amd.mesh import Mesh
    from oracle import oracle as O
    import workloads as W
    v, f = W.c5_mesh()
    t = spatialsearch.aabbtree_compute(v, f)
    vn = Mesh(v=v, f=f).estimate_vertex_normals()
    cams = W.fibonacci_cameras(64, 3.0)
    P = v.shape[0]
    rng = np.random.default_rng(14)
    vis, ndc = visibility.visibility_compute(cams=cams, tree=t, n=vn)
    ci = np.sort(rng.choice(64, 8, replace=False))
    vi = np.sort(rng.choice(P, args.pairs // 8, replace=False))
    t0 = time.perf_counter()
    bv, bn = [], []
    for c in ci:  # progress lines
        a, b = O.brute_visibility(v, f, cams[c:c + 1], n=vn, src_idx=vi)
        bv.append(a)
        bn.append(b)
        print("c5v brute force: camera %d (%d vertices)" % (c, vi.size), file=sys.stderr, flush=True)
    bv, bn = np.concatenate(bv), np.concatenate(bn)
    bad = int(np.count_nonzero((vis[ci][:, vi] != bv) | (ndc[ci][:, vi] != bn)))
    # sensors (visibility.cpp:79-85,96-111): 2 cameras with random sensor frames
    sc = np.sort(rng.choice(64, 2, replace=False))
    sens = rng.normal(size=(2, 9))
    svis, sndc = visibility.visibility_compute(cams=cams[sc], tree=t, n=vn, sensors=sens)
    si = np.sort(rng.choice(P, args.sensor_pairs // 2, replace=False))
    sv, sn = O.brute_visibility(v, f, cams[sc], n=vn, sensors=sens, src_idx=si)
    sbad = int(np.count_nonzero((svis[:, si] != sv) | (sndc[:, si] != sn)))
    return dict(workload="C5 visibility_compute (numpy entry point) on the 5M-face bumped icosphere, 64 Fibonacci cameras, "
                         "vertex normals; sensor frames on 2 cameras",
                pairs_checked=int(bv.size), sensor_pairs_checked=int(sv.size), rows_checked=int(bv.size + sv.size),
                visible_frac=float(bv.mean()), sensor_visible_frac=float(sv.mean()), mismatches=bad + sbad,
                brute_force_s=time.perf_counter() - t0,
                check="vis and n.dir bit-exact vs oracle.brute_visibility (any hit over all 5M triangles)")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="c3")
    ap.add_argument("--rows", type=int, default=20000)
    ap.add_argument("--centre", type=int, default=2000)
    ap.add_argument("--rays", type=int, default=20000, help="c5: alongnormal rays checked")
    ap.add_argument("--pairs", type=int, default=18000, help="c5v: (camera, vertex) pairs without sensors")
    ap.add_argument("--sensor-pairs", type=int, default=2000, help="c5v: pairs with sensors")
    args = ap.parse_args()
    from mesh_amd import _native
    _native.set_device(0)
    fails = 0
    for c in args.configs.split(","):
        r = {"c3": sweep_c3, "c2": sweep_c2, "c5": sweep_c5, "c5v": sweep_c5v}[c](args)
        r["config"] = c
        r["build_id"] = _native.build_id()
        fails += r["mismatches"]
        print(json.dumps(r), flush=True)
    sys.exit(1 if fails else 0)


if __name__ == "__main__":
    main()
