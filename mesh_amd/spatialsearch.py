"""Drop-in for the ``psbody.mesh.spatialsearch`` extension (mesh/src/spatialsearchmodule.cpp).

Same function names, argument order, return shapes/dtypes and ValueError messages as the reference;
the work runs in libmeshsearch's gfx950 kernels (LBVH build, Morton-sorted traversal, fp64 CGAL
constructions).  Deliberate differences:
  * ``aabbtree_nearest`` coerces the query to (N,3) float64 C order instead of reading raw memory
    (reference: spatialsearchmodule.cpp:175-180 checks only dims[1]).
  * ``aabbtree_nearest_alongnormal`` fills face=0xFFFFFFFF / point=NaN on rows with no hit (reference:
    uninitialised memory, :309-311); dist stays 1e100 as in the reference.
  * ``aabbtree_intersections_indices`` is registered and returns ascending indices (reference: not in
    the method table, :35-40, and racy push_back, :393-402).
"""
import numpy as np

from . import _native as N


class Mesh_IntersectionsError(Exception):
    """Module error object (spatialsearchmodule.cpp:33,60-62)."""


def _check_mesh_arrays(v, f):
    # spatialsearchmodule.cpp:79-97 ("O!O!" + dtype/ndim/Nx3 checks)
    if not isinstance(v, np.ndarray) or not isinstance(f, np.ndarray):
        raise TypeError("aabbtree_compute() arguments must be numpy.ndarray")
    if v.dtype != np.float64 or v.ndim != 2:
        raise ValueError("Vertices must be of type double, and 2 dimensional")
    if f.dtype != np.uint32 or f.ndim != 2:
        raise ValueError("Faces must be of type uint32, and 2 dimensional")
    if v.shape[1] != 3 or f.shape[1] != 3:
        raise ValueError("Input must be Nx3")
    return np.ascontiguousarray(v), np.ascontiguousarray(f)


def aabbtree_compute(v, f):
    """Build the search tree over triangles ``v[f]`` -> opaque handle (capsule in the reference)."""
    v, f = _check_mesh_arrays(v, f)
    return N.build_tree(v, f)


def _tree(tree, fn):
    if not isinstance(tree, N.Handle) or tree.ptr is None:
        raise TypeError("%s: expected a tree handle from aabbtree_compute" % fn)
    if tree.kind == "points":
        raise TypeError("%s: handle is a point tree" % fn)
    return tree


def aabbtree_nearest(tree, q):
    """(face (1,S) uint32, part (1,S) uint32, point (S,3) float64): spatialsearchmodule.cpp:165-220."""
    tree = _tree(tree, "aabbtree_nearest")
    if not isinstance(q, np.ndarray):
        raise TypeError("aabbtree_nearest() argument 2 must be numpy.ndarray")
    if q.ndim != 2 or q.shape[1] != 3:
        raise ValueError("Input must be Nx3")
    q = np.ascontiguousarray(q, dtype=np.float64)
    S = q.shape[0]
    face, part, pt = N.empty_results(((1, S), np.uint32), ((1, S), np.uint32), ((S, 3), np.float64))
    N.check(N.lib().msh_tree_nearest(tree.ptr, N.dptr(q), S, N.uptr(face), N.uptr(part), N.dptr(pt)))
    return face, part, pt


def aabbtree_nearest_barycentric(tree, q):
    """(face (S,) uint32, point (S,3) float64, weights (S,3) float64) of the closest point.

    One launch replaces ``aabbtree_nearest`` followed by ``Mesh.barycentric_coordinates_for_points``
    (mesh.py:218-222; Heidrich's projection, geometry/barycentric_coordinates_of_projection.py:9-49), the
    pair landmarks.py:58-63 calls: the weights are computed in the traversal kernel from the winning
    triangle and refer to its vertices ``f[face]``.
    """
    tree = _tree(tree, "aabbtree_nearest_barycentric")
    if not isinstance(q, np.ndarray):
        raise TypeError("aabbtree_nearest_barycentric() argument 2 must be numpy.ndarray")
    if q.ndim != 2 or q.shape[1] != 3:
        raise ValueError("Input must be Nx3")
    if tree.kind != "triangles":
        raise TypeError("aabbtree_nearest_barycentric: handle is not a triangle tree")
    q = np.ascontiguousarray(q, dtype=np.float64)
    S = q.shape[0]
    face, pt, w = N.empty_results(((S,), np.uint32), ((S, 3), np.float64), ((S, 3), np.float64))
    N.check(N.lib().msh_tree_nearest_bary(tree.ptr, N.dptr(q), S, N.uptr(face), N.dptr(pt), N.dptr(w)))
    return face, pt, w


def aabbtree_nearest_alongnormal(tree, p, n):
    """(dist (S,) float64, face (S,) uint32, point (S,3) float64): spatialsearchmodule.cpp:222-323."""
    tree = _tree(tree, "aabbtree_nearest_alongnormal")
    if not isinstance(p, np.ndarray) or not isinstance(n, np.ndarray):
        raise TypeError("aabbtree_nearest_alongnormal() arguments must be numpy.ndarray")
    if p.ndim != 2 or n.ndim != 2 or p.shape[1] != 3 or n.shape[1] != 3 or p.shape[0] != n.shape[0]:
        raise ValueError("Points and normals must be Nx3")
    p = np.ascontiguousarray(p, dtype=np.float64)
    n = np.ascontiguousarray(n, dtype=np.float64)
    S = p.shape[0]
    dist, face, pt = N.empty_results(((S,), np.float64), ((S,), np.uint32), ((S, 3), np.float64))
    N.check(N.lib().msh_tree_nearest_alongnormal(tree.ptr, N.dptr(p), N.dptr(n), S, N.dptr(dist), N.uptr(face),
                                                  N.dptr(pt)))
    return dist, face, pt


def aabbtree_intersections_indices(tree, qv, qf):
    """Ascending indices of query faces intersecting the mesh: spatialsearchmodule.cpp:326-417."""
    tree = _tree(tree, "aabbtree_intersections_indices")
    if not isinstance(qv, np.ndarray) or not isinstance(qf, np.ndarray):
        raise TypeError("aabbtree_intersections_indices() arguments must be numpy.ndarray")
    if qv.dtype != np.float64 or qv.ndim != 2:
        raise ValueError("Query Vertices must be of type double, and 2 dimensional")
    if qf.dtype != np.uint32 or qf.ndim != 2:
        raise ValueError("Query Faces must be of type uint32, and 2 dimensional")
    if qv.shape[1] != 3 or qf.shape[1] != 3:
        raise ValueError("Input must be Nx3")
    qv = np.ascontiguousarray(qv)
    qf = np.ascontiguousarray(qf)
    out = np.empty(qf.shape[0], dtype=np.uint32)
    K = N._sz(0)
    N.check(N.lib().msh_tree_intersections(tree.ptr, N.dptr(qv), qv.shape[0], N.uptr(qf), qf.shape[0], N.uptr(out),
                                            N.ctypes.byref(K)), Mesh_IntersectionsError)
    return out[:K.value].copy()
