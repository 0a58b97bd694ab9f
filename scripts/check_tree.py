"""Diagnostic: download a built LBVH (via the blob API) and check every node's child bounds against the
primitives below it: containment and tightness of the quantised oriented boxes (frame n, t, b = n x t;
bound = base + u * 2^e decoded in fp32 exactly as the kernels do), child-pointer sanity and depth.
Prints one JSON line."""
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
    nodes = np.frombuffer(b[off_nodes:off_nodes + (T - 1) * 64].tobytes(), dtype=np.uint8).reshape(T - 1, 64)
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
    fl = nodes.copy().view(np.float32)  # (T-1, 16)
    child = fl[:, 6:8].copy().view(np.int32)
    base = fl[:, 8:11]
    u = nodes[:, 44:56].reshape(T - 1, 2, 6).astype(np.float32)
    # bf16 scales (common.h encode_scales): float 14 = S0 << 16 | S2, float 15 = S1 << 16
    w14 = nodes[:, 56:60].copy().view(np.uint32)[:, 0]
    w15 = nodes[:, 60:64].copy().view(np.uint32)[:, 0]
    sb = np.stack([w14 & np.uint32(0xFFFF0000), w15 & np.uint32(0xFFFF0000), (w14 << np.uint32(16))], axis=1)
    scale = np.ascontiguousarray(sb, dtype=np.uint32).view(np.float32)  # (T-1, 3)
    # base + u * s in fp32: the product is exact, the sum rounds once (as fmaf in the kernels)
    dec = (np.tile(base, 2)[:, None, :] + u * np.tile(scale, 2)[:, None, :]).astype(np.float32)  # (T-1, 2, 6)
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
    obb_bad = 0
    loose = []
    for x in range(T - 1):
        n32, t32 = fl[x, 0:6:2], fl[x, 1:6:2]  # frame pairs (n_k, t_k), common.h encode_frame
        nf, tf = n32.astype(np.float64), t32.astype(np.float64)
        b = np.array([n32[1] * t32[2] - n32[2] * t32[1],
                      n32[2] * t32[0] - n32[0] * t32[2],
                      n32[0] * t32[1] - n32[1] * t32[0]], dtype=np.float32).astype(np.float64)
        A = np.stack([nf, tf, b])
        prs = []
        for s in (0, 1):
            c = child[x, s]
            a, e = (rng_lo[c], rng_hi[c]) if c >= 0 else (~c, ~c)
            pts = tri[a:e + 1].reshape(-1, 3)
            prs.append(pts @ A.T)
        union = np.maximum(np.maximum(prs[0].max(0), prs[1].max(0)) - np.minimum(prs[0].min(0), prs[1].min(0)), 1e-12)
        for s in (0, 1):
            ob = dec[x, s].astype(np.float64)
            pr = prs[s]
            if np.any(pr.min(0) < ob[:3]) or np.any(pr.max(0) > ob[3:]):
                obb_bad += 1
            if x < 2000:
                # slack of each bound relative to the node's range along that axis (one code step <= 2/254)
                # (less the fp32 outward rounding of the unquantised bound: 4 ulps of its magnitude)
                ulp = 4.0 * np.spacing(np.abs(ob).astype(np.float32)).astype(np.float64)
                loose.append(float(max(((pr.min(0) - ob[:3] - ulp[:3]) / union).max(),
                                       ((ob[3:] - pr.max(0) - ulp[3:]) / union).max())))
    res = {"T": T, "max_depth": max_depth, "reached_nodes": len(order), "obb_containment_violations": obb_bad,
           "worst_relative_obb_looseness_first2000": max(loose), "origin": origin.tolist()}
    return res


if __name__ == "__main__":
    import workloads as W
    from mesh_amd import _native
    _native.set_device(0)
    print(json.dumps(check_mesh(*W.geodesic_icosphere(int(sys.argv[1]) if len(sys.argv) > 1 else 40))))
