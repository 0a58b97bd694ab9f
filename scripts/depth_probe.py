import sys, numpy as np
sys.path.insert(0, '.')
import workloads as W
from mesh_amd import _native, spatialsearch
_native.set_device(0)
for name, (v, f) in [("c2", W.c2_mesh()), ("c3", W.c3_mesh()), ("c5", W.c5_mesh()), ("sphere", W.sphere_fixture())]:
    t = spatialsearch.aabbtree_compute(v, f)
    i = t.info()
    print(name, "max_depth", i.max_depth, "build_ms", round(i.build_ms, 2), flush=True)
