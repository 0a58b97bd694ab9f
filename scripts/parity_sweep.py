"""One-off parity sweep of the C3 headline stream (not part of the test suite: it takes about a minute of
host brute force).  Runs bench.py's exact query stream (100M uniform queries generated in HBM, seed 3)
through the device entry point, then checks K random rows plus the rows nearest the sphere's centre (the
deferred pass-2 queries) bit for bit against the oracle's exhaustive brute force (same tie rule), and
prints one JSON line.

    python scripts/parity_sweep.py [--rows 20000] [--centre 2000]
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
    ap.add_argument("--rows", type=int, default=20000)
    ap.add_argument("--centre", type=int, default=2000)
    args = ap.parse_args()
    import torch
    from mesh_amd import _native, spatialsearch
    from mesh_amd.distributed import nearest_device
    from oracle import oracle as O
    import workloads as W

    _native.set_device(0)
    v, f = W.c3_mesh()
    S = 100_000_000
    g = torch.Generator(device="cuda:0")
    g.manual_seed(3)
    dq = (torch.rand((S, 3), generator=g, dtype=torch.float64, device="cuda:0") * 2.2 - 1.1).contiguous()
    t = spatialsearch.aabbtree_compute(v, f)
    df = torch.empty(S, dtype=torch.int32, device="cuda:0")
    dp = torch.empty(S, dtype=torch.int32, device="cuda:0")
    dpt = torch.empty((S, 3), dtype=torch.float64, device="cuda:0")
    nearest_device(t, dq, df, dp, dpt)
    torch.cuda.synchronize()
    q = dq.cpu().numpy()
    face = df.cpu().numpy().view(np.uint32)
    part = dp.cpu().numpy().view(np.uint32)
    pt = dpt.cpu().numpy()
    r = np.sqrt(np.einsum("ij,ij->i", q, q))
    idx = np.concatenate([np.random.default_rng(11).choice(S, args.rows, replace=False),
                          np.argpartition(r, args.centre)[:args.centre]])
    t0 = time.perf_counter()
    bf, bp, bpt, _ = O.brute_nearest(v, f, q[idx])
    brute_s = time.perf_counter() - t0
    bad = np.nonzero((face[idx] != bf) | (part[idx] != bp) | np.any(pt[idx] != bpt, axis=1))[0]
    print(json.dumps({"workload": "C3 headline stream (100M uniform queries, seed 3, device entry point)",
                      "build_id": _native.build_id(), "rows_checked": int(idx.size),
                      "random_rows": args.rows, "centre_rows": args.centre, "mismatches": int(bad.size),
                      "first_mismatch_rows": idx[bad[:10]].tolist(), "brute_force_s": brute_s,
                      "check": "face, part code and point bit-exact vs oracle.brute_nearest (lexicographic (d2, face))"}),
          flush=True)
    sys.exit(1 if bad.size else 0)


if __name__ == "__main__":
    main()
