"""Drop-in for the ``psbody.mesh.aabb_normals`` extension (mesh/src/aabb_normals.cpp, AABB_n_tree.h).

Closest point under the metric ``||q - p|| + eps * (1 - n_q . n_tri)`` (AABB_n_tree.h:40-84) and the
self-intersection count (aabb_normals.cpp:192-207), on the gfx950 kernels.  Ties resolve to the
lexicographic minimum of (metric, face).  Deliberate differences: query
arrays are coerced to (N,3) float64 (reference: no dtype check, :122-129); a build failure raises
RuntimeError (reference: returns an un-INCREF'd None, :105-108).
"""
import numpy as np

from . import _native as N


def aabbtree_n_compute(v, f, eps):
    """Tree with normal weight ``eps``: aabb_normals.cpp:63-110."""
    if not isinstance(v, np.ndarray) or not isinstance(f, np.ndarray):
        raise TypeError("aabbtree_n_compute() arguments 1-2 must be numpy.ndarray")
    if v.dtype != np.float64 or v.ndim != 2:
        raise ValueError("Vertices must be of type double, and 2 dimensional")
    if f.dtype != np.uint32 or f.ndim != 2:
        raise ValueError("Faces must be of type uint32, and 2 dimensional")
    if v.shape[1] != 3 or f.shape[1] != 3:
        raise ValueError("Input must be Nx3")
    return N.build_ntree(np.ascontiguousarray(v), np.ascontiguousarray(f), float(eps))


def aabbtree_n_nearest(tree, v, n):
    """(face (1,S) uint32, point (S,3) float64): aabb_normals.cpp:112-190."""
    if not isinstance(tree, N.Handle) or tree.kind != "normals" or tree.ptr is None:
        raise TypeError("aabbtree_n_nearest: expected a handle from aabbtree_n_compute")
    if not isinstance(v, np.ndarray):
        raise ValueError("First argument must be a NumPy array")
    if not isinstance(n, np.ndarray):
        raise ValueError("Second argument must be a NumPy array")
    if v.ndim != 2 or v.shape[1] != 3:
        raise ValueError("Input must be Nx3")
    if n.ndim != 2 or n.shape[1] != v.shape[1] or n.shape[0] != v.shape[0]:
        raise ValueError("Normals should have same dimensions as points")
    v = np.ascontiguousarray(v, dtype=np.float64)
    n = np.ascontiguousarray(n, dtype=np.float64)
    S = v.shape[0]
    face, pt = N.empty_results(((1, S), np.uint32), ((S, 3), np.float64))
    N.check(N.lib().msh_ntree_nearest(tree.ptr, N.dptr(v), N.dptr(n), S, N.uptr(face), N.dptr(pt)))
    return face, pt


def aabbtree_n_selfintersects(tree):
    """Number of triangles intersecting a non-adjacent triangle: aabb_normals.cpp:192-207."""
    if not isinstance(tree, N.Handle) or tree.kind != "normals" or tree.ptr is None:
        raise TypeError("aabbtree_n_selfintersects: expected a handle from aabbtree_n_compute")
    c = N.ctypes.c_int64(0)
    N.check(N.lib().msh_ntree_selfintersects(tree.ptr, N.ctypes.byref(c)))
    return int(c.value)
