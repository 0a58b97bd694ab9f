"""Development tool: traversal cost model (see bvh_model.cpp).  python tools/bvh_model.py"""
import ctypes
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
SO = "/tmp/libbvhmodel.so"


def load():
    if not os.path.exists(SO):
        subprocess.check_call(["g++", "-O3", "-std=c++17", "-fPIC", "-fopenmp", "-shared",
                               os.path.join(ROOT, "tools", "bvh_model.cpp"), "-o", SO])
    return ctypes.CDLL(SO)


def counts(v, f, q, kind=0):
    L = load()
    v = np.ascontiguousarray(v, np.float64)
    f = np.ascontiguousarray(f, np.uint32)
    q = np.ascontiguousarray(q, np.float64)
    S = q.shape[0]
    nn = np.zeros(S, np.uint32)
    nl = np.zeros(S, np.uint32)
    d = ctypes.c_int(0)
    P = ctypes.c_void_p
    L.model_counts(P(v.ctypes.data), P(f.ctypes.data), ctypes.c_int(f.shape[0]), P(q.ctypes.data), ctypes.c_long(S),
                   ctypes.c_int(kind), P(nn.ctypes.data), P(nl.ctypes.data), ctypes.byref(d))
    return nn, nl, d.value


if __name__ == "__main__":
    import workloads as W
    freq = int(sys.argv[1]) if len(sys.argv) > 1 else 224
    v, f = W.geodesic_icosphere(freq)
    q = np.random.default_rng(3).uniform(-1.1, 1.1, (20000, 3))
    for kind in (0, 1):
        nn, nl, d = counts(v, f, q, kind)
        r = np.linalg.norm(q, axis=1)
        print("kind", kind, "depth", d, "nodes avg %.1f p50 %d p99 %d max %d" % (nn.mean(), np.median(nn), np.percentile(nn, 99), nn.max()),
              "leaves avg %.1f" % nl.mean())
        for lo, hi in [(0, 0.2), (0.2, 0.5), (0.5, 0.9), (0.9, 1.1), (1.1, 2)]:
            m = (r >= lo) & (r < hi)
            print("   r in [%.1f,%.1f): n=%d nodes %.0f leaves %.0f" % (lo, hi, m.sum(), nn[m].mean(), nl[m].mean()))
