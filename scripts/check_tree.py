"""Diagnostic: download a built LBVH (via the blob API) and check every node's child bounds against the
primitives below it: AABB containment/tightness and oriented-box (frame n, t, b = n x t) containment,
child-pointer sanity and depth.  Prints one JSON line."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def parse_blob(b):
    hdr = np.frombuffer(b[:256].tobytes(), dtype=np.uint64)
    # BlobHeader: magic, (kind,max_depth) i32x2, P, T, T_main, v_rows, eps, scene f32x6, off_v, off_nodes,
    # off_leaves, total, origin f64x3
    T = int(hdr[3])
    max_depth = int(np.frombuffer(b[8:16].tobytes(), dtype=np.int32)[1])
    off_nodes, off_leaves = int(hdr[11]), int(hdr[12])
    origin = np.frombuffer(b[112:136].tobytes(), dtype=np.float64)
    nodes = np.frombuffer(b[off_nodes:off_nodes + (T - 1) * 128].tobytes(), dtype=np.float32).reshape(T - 1, 32)
    leaves = np.frombuffer(b[off_leaves:off_leaves + T * 80].tobytes(), dtype=np.float64).reshape(T, 10)
    return T, max_depth, origin, nodes, leaves


def check_mesh(v, f):
    import torch
    from mesh_amd import _native, spatialsearch
    t = spatialsearch.aabbtree_compute(np.ascontiguousarray(v, np.float64), np.ascontiguousarray(f, np.uint32))
    n = _native.blob_size(t)
    blob = torch.empty(n, dtype=torch.uint8, device="cuda:0")
    _native.blob_pack(t, blob.data_ptr())
    T, max_depth, origin, nodes, leaves = parse_blob(blob.cpu().numpy())
    child = nodes[:, 6:8].copy().view(np.int32)
    tri = leaves[:, :9].reshape(T, 3, 3) - origin
    llo, lhi = tri.min(1), tri.max(1)
    # leaf ranges by post-order
    rng_lo = np.zeros(T - 1, np.int64)
    rng_hi = np.zeros(T - 1, np.int64)
    order, stack = [], [0]
    while stack:
        x = stack.pop()
        order.append(x)
        stack.extend(int(c) for c in child[x] if c >= 0)
    for x in reversed(order):
        lo_, hi_ = [], []
        for c in child[x]:
            if c >= 0:
                lo_.append(rng_lo[c]); hi_.append(rng_hi[c])
            else:
                lo_.append(~c); hi_.append(~c)
        rng_lo[x], rng_hi[x] = min(lo_), max(hi_)
    aabb_bad = obb_bad = 0
    loose = []
    for x in range(T - 1):
        nf, tf = nodes[x, 0:3].astype(np.float64), nodes[x, 3:6].astype(np.float64)
        b = np.array([nodes[x, 1] * nodes[x, 5] - nodes[x, 2] * nodes[x, 4],
                      nodes[x, 2] * nodes[x, 3] - nodes[x, 0] * nodes[x, 5],
                      nodes[x, 0] * nodes[x, 4] - nodes[x, 1] * nodes[x, 3]], dtype=np.float32).astype(np.float64)
        A = np.stack([nf, tf, b])
        for s in (0, 1):
            c = child[x, s]
            a, e = (rng_lo[c], rng_hi[c]) if c >= 0 else (~c, ~c)
            pts = tri[a:e + 1].reshape(-1, 3)
            ab = nodes[x, 8 + 12 * s: 14 + 12 * s].astype(np.float64)
            ob = nodes[x, 14 + 12 * s: 20 + 12 * s].astype(np.float64)
            if np.any(pts.min(0) < ab[:3]) or np.any(pts.max(0) > ab[3:]):
                aabb_bad += 1
            pr = pts @ A.T
            if np.any(pr.min(0) < ob[:3]) or np.any(pr.max(0) > ob[3:]):
                obb_bad += 1
            if x < 2000:
                ext = max(float((pts.max(0) - pts.min(0)).max()), 1e-12)
                loose.append(float(max((pts.min(0) - ab[:3]).max(), (ab[3:] - pts.max(0)).max()) / ext))
    res = {"T": T, "max_depth": max_depth, "reached_nodes": len(order), "aabb_containment_violations": aabb_bad,
           "obb_containment_violations": obb_bad, "worst_relative_aabb_looseness_first2000": max(loose),
           "origin": origin.tolist()}
    return res


if __name__ == "__main__":
    import workloads as W
    from mesh_amd import _native
    _native.set_device(0)
    print(json.dumps(check_mesh(*W.geodesic_icosphere(int(sys.argv[1]) if len(sys.argv) > 1 else 40))))
