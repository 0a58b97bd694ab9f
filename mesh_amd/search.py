"""Drop-in for ``psbody.mesh.search`` (mesh/search.py): same class names, constructor and method
signatures, and return shapes/dtypes; the bodies are delegations to this package's GPU modules.

``AabbTree`` / ``AabbNormalsTree`` / ``CGALClosestPointTree`` apply the same input coercions as the
reference (search.py:24,29,35-36,76,95).  ``ClosestPointTree`` answers all queries with one GPU launch
over a point LBVH instead of the reference's per-query scipy KDTree loop (search.py:59-61); the nearest
vertex is the lexicographic minimum of (distance, vertex index).
"""
import numpy as np

from . import _native as N

__all__ = ['AabbTree', 'AabbNormalsTree', 'ClosestPointTree', 'CGALClosestPointTree', 'AabbTreeBatch']


def _f64c(a):
    return np.ascontiguousarray(a, dtype=np.float64)


def _u32c(a):
    return np.ascontiguousarray(a, dtype=np.uint32)


class AabbTree(object):
    """Closest-point / ray / intersection search over the triangles of ``m`` (search.py:19-49).

    Built once on the GPU (LBVH); the handle lives in ``cpp_handle`` as in the reference.
    """

    def __init__(self, m):
        from . import spatialsearch
        self.cpp_handle = spatialsearch.aabbtree_compute(_f64c(m.v).copy(), _u32c(m.f).copy())

    def nearest(self, v_samples, nearest_part=False):
        """Closest face (1,S) u32 and point (S,3) f64 for each sample.

        With ``nearest_part=True`` a third array (1,S) u32 is returned between them that classifies
        where the point lies on its triangle (a,b,c): 0 inside, 1/2/3 on edge ab/bc/ca, 4/5/6 at
        vertex a/b/c.
        """
        from . import spatialsearch
        faces, parts, pts = spatialsearch.aabbtree_nearest(self.cpp_handle, _f64c(v_samples))
        if nearest_part:
            return faces, parts, pts
        return faces, pts

    def nearest_alongnormal(self, points, normals):
        """Nearest hit of the lines through ``points`` along +/-``normals``: (dist, face, point)."""
        from . import spatialsearch
        return spatialsearch.aabbtree_nearest_alongnormal(self.cpp_handle, points.astype(np.float64),
                                                          normals.astype(np.float64))

    def nearest_barycentric(self, v_samples):
        """(face (S,) u32, point (S,3) f64, barycentric weights (S,3) f64) of the closest point.

        Fused replacement of ``nearest`` followed by ``Mesh.barycentric_coordinates_for_points``
        (mesh.py:218-222, Heidrich projection, geometry/barycentric_coordinates_of_projection.py:9-49);
        the weights are computed in the traversal kernel from the winning triangle.
        """
        from . import spatialsearch
        return spatialsearch.aabbtree_nearest_barycentric(self.cpp_handle, _f64c(v_samples))

    def intersections_indices(self, q_v, q_f):
        """Indices (ascending, u32) of the query triangles ``q_v[q_f]`` that touch the mesh.

        The reference method cannot run (its module function is unregistered and imported by an
        absolute name, search.py:46); this one is wired to the GPU triangle-triangle kernel.
        """
        from . import spatialsearch
        return spatialsearch.aabbtree_intersections_indices(self.cpp_handle, _f64c(q_v), _u32c(q_f))


class ClosestPointTree(object):
    """Nearest mesh vertex for query points; faces are ignored (search.py:52-65)."""

    def __init__(self, m):
        self.v = m.v
        self._h = N.build_points(_f64c(m.v))

    def _query(self, v_samples):
        q = _f64c(v_samples).reshape(-1, 3)
        S = q.shape[0]
        idx, dist = N.empty_results(((S,), np.uint32), ((S,), np.float64))
        N.check(N.lib().msh_points_nearest(self._h.ptr, N.dptr(q), S, N.uptr(idx), N.dptr(dist)))
        return idx.astype(np.intp), dist

    def nearest(self, v_samples):
        # same container types as the reference's zip(*[...]) over per-sample KDTree queries
        idx, dist = self._query(v_samples)
        return (tuple(idx), tuple(dist))

    def nearest_vertices(self, v_samples):
        # row gather by vertex index (the reference's tuple indexing breaks for >= 3 samples,
        # SURVEY.md Appendix B)
        idx, _ = self._query(v_samples)
        return self.v[idx]


class CGALClosestPointTree(object):
    """Nearest vertex through the triangle tree (search.py:68-86).

    Every vertex becomes a tiny triangle (its three corners displaced by 1e-12 along +x, +y and
    -(x+y)), so the closest face index is the closest vertex index.
    """

    def __init__(self, m):
        from . import spatialsearch
        self.v = m.v
        n = m.v.shape[0]
        ids = np.arange(n)
        tri = np.stack([ids, ids + n, ids + 2 * n], axis=1)
        d = 1e-12
        corners = np.concatenate([m.v + [d, 0.0, 0.0], m.v + [0.0, d, 0.0], m.v - [d, d, 0.0]], axis=0)
        self.cpp_handle = spatialsearch.aabbtree_compute(_f64c(corners).copy(), _u32c(tri).copy())

    def _faces(self, v_samples):
        from . import spatialsearch
        faces, _, _ = spatialsearch.aabbtree_nearest(self.cpp_handle, _f64c(v_samples))
        return faces.flatten()

    def nearest(self, v_samples):
        fi = self._faces(v_samples)
        dist = np.sqrt(np.sum((self.v[fi] - v_samples) ** 2.0, axis=1)).flatten()
        return fi, dist

    def nearest_vertices(self, v_samples):
        return self.v[self._faces(v_samples)]


class AabbNormalsTree(object):
    """Closest face under the distance + normal-agreement metric (search.py:89-100).

    The reference fixes the normal weight eps at 0.1 (search.py:94); so does this class.
    """

    EPS = 0.1

    def __init__(self, m):
        from . import aabb_normals
        self.tree_handle = aabb_normals.aabbtree_n_compute(_f64c(m.v), _u32c(m.f).copy(), self.EPS)

    def nearest(self, v_samples, n_samples):
        from . import aabb_normals
        return aabb_normals.aabbtree_n_nearest(self.tree_handle, v_samples, n_samples)


class AabbTreeBatch(object):
    """Many meshes sharing one topology, searched together (scan-to-mesh registration, BASELINE C4).

    The reference answers this with one ``AabbTree`` per mesh (search.py:21-30); ``AabbTreeBatch(v, f)``
    builds all B trees in one batched GPU build and ``nearest(q)`` answers every mesh's queries in one
    launch.  ``nearest(q)[..., b]`` equals ``AabbTree(mesh_b).nearest(q[b])`` with mesh-local face
    indices; shapes gain a leading mesh axis: face (B,S) uint32, part (B,S) uint32, point (B,S,3).
    """

    def __init__(self, v, f):
        v = _f64c(v)
        f = _u32c(f)
        if v.ndim != 3 or v.shape[2] != 3:
            raise ValueError("Vertices must be BxPx3")
        if f.ndim != 2 or f.shape[1] != 3:
            raise ValueError("Faces must be Tx3")
        self.n_meshes = v.shape[0]
        self.cpp_handle = N.build_batch(v, f)

    def _q(self, v_samples):
        q = _f64c(v_samples)
        if q.ndim != 3 or q.shape[0] != self.n_meshes or q.shape[2] != 3:
            raise ValueError("Queries must be BxSx3 with B = %d" % self.n_meshes)
        return q

    def nearest(self, v_samples, nearest_part=False):
        q = self._q(v_samples)
        B, S = q.shape[0], q.shape[1]
        face, part, pt = N.empty_results(((B, S), np.uint32), ((B, S), np.uint32), ((B, S, 3), np.float64))
        N.check(N.lib().msh_batch_nearest(self.cpp_handle.ptr, N.dptr(q), S, N.uptr(face), N.uptr(part),
                                          N.dptr(pt)))
        return (face, part, pt) if nearest_part else (face, pt)

    def nearest_barycentric(self, v_samples):
        """(face (B,S) u32, point (B,S,3) f64, barycentric weights (B,S,3) f64) per mesh."""
        q = self._q(v_samples)
        B, S = q.shape[0], q.shape[1]
        face, pt, bary = N.empty_results(((B, S), np.uint32), ((B, S, 3), np.float64), ((B, S, 3), np.float64))
        N.check(N.lib().msh_batch_nearest_bary(self.cpp_handle.ptr, N.dptr(q), S, N.uptr(face), N.dptr(pt),
                                               N.dptr(bary)))
        return face, pt, bary
