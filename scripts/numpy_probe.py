"""Where the numpy entry point's time goes (C3, 100M host queries through msh_tree_nearest).

Times, on the GPU box, each as the median of `--reps` calls:
  * call_fresh     — aabbtree_nearest as a caller uses it (fresh np.empty outputs: first-touch page faults);
  * call_prefault  — the same C entry point into output arrays that were already written once;
  * fault_fill     — np.empty + writing every page of the 3.2 GB of outputs from one thread;
  * copy_1t        — one-thread memcpy of the 2.4 GB query array into a prefaulted array;
  * --sweep        — MESH_AMD_HOST_CHUNK variants of call_prefault, and the registered path
                     (MESH_AMD_COPY_THREADS is read once per process: set it on the command line).
Prints one JSON line per measurement.

    python scripts/numpy_probe.py [--queries 100000000] [--reps 3]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def med(fn, reps):
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--queries", type=int, default=100_000_000)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--sweep", action="store_true")
    args = ap.parse_args()
    from mesh_amd import _native as N, spatialsearch
    import workloads as W
    v, f = W.c3_mesh()
    S = args.queries
    q = np.random.default_rng(3).uniform(-1.1, 1.1, (S, 3))
    tree = spatialsearch.aabbtree_compute(v, f)
    spatialsearch.aabbtree_nearest(tree, q[:1000])

    def emit(name, s, **kw):
        print(json.dumps(dict(name=name, ms=s * 1e3, queries_per_s=S / s, **kw)), flush=True)

    emit("call_fresh", med(lambda: spatialsearch.aabbtree_nearest(tree, q), args.reps))
    face = np.ones((1, S), np.uint32)
    part = np.ones((1, S), np.uint32)
    pt = np.ones((S, 3))

    def pre():
        N.check(N.lib().msh_tree_nearest(tree.ptr, N.dptr(q), S, N.uptr(face), N.uptr(part), N.dptr(pt)))
    emit("call_prefault", med(pre, args.reps))

    def fault_fill():
        a = np.empty((S, 3))
        a.fill(1.0)
        b = np.empty(S, np.uint32)
        b.fill(1)
        c = np.empty(S, np.uint32)
        c.fill(1)
    emit("fault_fill_1t", med(fault_fill, args.reps), bytes=S * 32)
    dst = np.ones_like(q)
    emit("copy_1t", med(lambda: np.copyto(dst, q), args.reps), bytes=S * 24)
    del dst
    if args.sweep:
        for env, vals in (("MESH_AMD_HOST_CHUNK", ("1048576", "2097152", "8388608", "16777216")),):
            for val in vals:
                os.environ[env] = val
                emit("call_prefault", med(pre, args.reps), env={env: val})
                os.environ.pop(env)
        os.environ["MESH_AMD_HOST_REGISTER"] = "1"
        emit("call_prefault_registered", med(pre, args.reps))
        os.environ.pop("MESH_AMD_HOST_REGISTER")


if __name__ == "__main__":
    main()
