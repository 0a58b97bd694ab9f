"""Drop-in for ``psbody.mesh.search`` (mesh/search.py): same classes, signatures and return types.

``AabbTree`` / ``AabbNormalsTree`` / ``CGALClosestPointTree`` keep the reference's dtype coercions
(search.py:24,29,35-36,76,95); ``ClosestPointTree`` replaces the per-query scipy KDTree loop
(search.py:59-61) with the GPU point LBVH (nearest vertex = lexicographic min of (distance, index)).
"""
import numpy as np

from . import _native as N

__all__ = ['AabbTree', 'AabbNormalsTree', 'ClosestPointTree', 'CGALClosestPointTree', 'AabbTreeBatch']


class AabbTree(object):
    """Encapsulates an AABB (Axis Aligned Bounding Box) Tree (search.py:19-49)."""

    def __init__(self, m):
        from . import spatialsearch
        self.cpp_handle = spatialsearch.aabbtree_compute(m.v.astype(np.float64).copy(order='C'),
                                                         m.f.astype(np.uint32).copy(order='C'))

    def nearest(self, v_samples, nearest_part=False):
        "nearest_part tells you whether the closest point in triangle abc is in the interior (0), on an edge (ab:1,bc:2,ca:3), or a vertex (a:4,b:5,c:6)"
        from . import spatialsearch
        f_idxs, f_part, v = spatialsearch.aabbtree_nearest(self.cpp_handle,
                                                           np.array(v_samples, dtype=np.float64, order='C'))
        return (f_idxs, f_part, v) if nearest_part else (f_idxs, v)

    def nearest_alongnormal(self, points, normals):
        from . import spatialsearch
        distances, f_idxs, v = spatialsearch.aabbtree_nearest_alongnormal(self.cpp_handle,
                                                                          points.astype(np.float64),
                                                                          normals.astype(np.float64))
        return (distances, f_idxs, v)

    def intersections_indices(self, q_v, q_f):
        '''
            Given a set of query vertices and faces, the function computes which intersect the mesh
            A list with the indices in q_f is returned
            @param q_v The query vertices (array of 3xN float values)
            @param q_f The query faces (array 3xF integer values)
        '''
        from . import spatialsearch  # the reference's absolute import (search.py:46) fails; fixed
        return spatialsearch.aabbtree_intersections_indices(self.cpp_handle,
                                                            np.ascontiguousarray(q_v, dtype=np.float64),
                                                            np.ascontiguousarray(q_f, dtype=np.uint32))


class ClosestPointTree(object):
    """Provides nearest neighbor search for a cloud of vertices (i.e. triangles are not used)"""

    def __init__(self, m):
        self.v = m.v
        self._h = N.build_points(np.ascontiguousarray(m.v, dtype=np.float64))

    def _query(self, v_samples):
        q = np.ascontiguousarray(v_samples, dtype=np.float64).reshape(-1, 3)
        S = q.shape[0]
        idx = np.empty(S, dtype=np.uint32)
        dist = np.empty(S, dtype=np.float64)
        N.check(N.lib().msh_points_nearest(self._h.ptr, N.dptr(q), S, N.uptr(idx), N.dptr(dist)))
        return idx.astype(np.intp), dist

    def nearest(self, v_samples):
        # reference: zip(*[kdtree.query(v) for v in v_samples]) -> (indices tuple, distances tuple)
        idx, dist = self._query(v_samples)
        return (tuple(idx), tuple(dist))

    def nearest_vertices(self, v_samples):
        # reference indexes v with the tuple of indices (search.py:63-65), which fails for >= 3 samples;
        # the intended row gather is used here
        idx, _ = self._query(v_samples)
        return self.v[idx]


class CGALClosestPointTree(object):
    """Vertex NN through the triangle tree over 1e-12 'vertex triangles' (search.py:68-86)."""

    def __init__(self, m):
        from . import spatialsearch
        self.v = m.v
        n = m.v.shape[0]
        faces = np.vstack([np.array(range(n)), np.array(range(n)) + n, np.array(range(n)) + 2 * n]).T
        eps = 0.000000000001
        self.cpp_handle = spatialsearch.aabbtree_compute(
            np.vstack([m.v + eps * np.array([1.0, 0.0, 0.0]), m.v + eps * np.array([0.0, 1.0, 0.0]),
                       m.v - eps * np.array([1.0, 1.0, 0.0])]).astype(np.float64).copy(order='C'),
            faces.astype(np.uint32).copy(order='C'))

    def nearest(self, v_samples):
        from . import spatialsearch
        f_idxs, f_part, v = spatialsearch.aabbtree_nearest(self.cpp_handle,
                                                           np.array(v_samples, dtype=np.float64, order='C'))
        return (f_idxs.flatten(), (np.sum(((self.v[f_idxs.flatten()] - v_samples) ** 2.0), axis=1) ** 0.5).flatten())

    def nearest_vertices(self, v_samples):
        from . import spatialsearch
        f_idxs, f_part, v = spatialsearch.aabbtree_nearest(self.cpp_handle,
                                                           np.array(v_samples, dtype=np.float64, order='C'))
        return self.v[f_idxs.flatten()]


class AabbNormalsTree(object):
    def __init__(self, m):
        # the weight of the normals cosine is proportional to the std of the vertices
        # the best point can be translated up to 2*eps because of the normals
        from . import aabb_normals
        eps = 0.1  # np.std(m.v)#0  (search.py:94)
        self.tree_handle = aabb_normals.aabbtree_n_compute(np.ascontiguousarray(m.v, dtype=np.float64),
                                                           m.f.astype(np.uint32).copy(), eps)

    def nearest(self, v_samples, n_samples):
        from . import aabb_normals
        closest_tri, closest_p = aabb_normals.aabbtree_n_nearest(self.tree_handle, v_samples, n_samples)
        return (closest_tri, closest_p)


class AabbTreeBatch(object):
    """Many meshes sharing one topology, searched together (scan-to-mesh registration, BASELINE C4).

    The reference answers this with one ``AabbTree`` per mesh (search.py:21-30); ``AabbTreeBatch(v, f)``
    builds all B trees in one batched GPU build and ``nearest(q)`` answers every mesh's queries in one
    launch.  ``nearest(q)[..., b]`` equals ``AabbTree(mesh_b).nearest(q[b])`` with mesh-local face
    indices; shapes gain a leading mesh axis: face (B,S) uint32, part (B,S) uint32, point (B,S,3).
    """

    def __init__(self, v, f):
        v = np.ascontiguousarray(v, dtype=np.float64)
        f = np.ascontiguousarray(f, dtype=np.uint32)
        if v.ndim != 3 or v.shape[2] != 3:
            raise ValueError("Vertices must be BxPx3")
        if f.ndim != 2 or f.shape[1] != 3:
            raise ValueError("Faces must be Tx3")
        self.n_meshes = v.shape[0]
        self.cpp_handle = N.build_batch(v, f)

    def nearest(self, v_samples, nearest_part=False):
        q = np.ascontiguousarray(v_samples, dtype=np.float64)
        if q.ndim != 3 or q.shape[0] != self.n_meshes or q.shape[2] != 3:
            raise ValueError("Queries must be BxSx3 with B = %d" % self.n_meshes)
        B, S = q.shape[0], q.shape[1]
        face = np.empty((B, S), dtype=np.uint32)
        part = np.empty((B, S), dtype=np.uint32)
        pt = np.empty((B, S, 3), dtype=np.float64)
        N.check(N.lib().msh_batch_nearest(self.cpp_handle.ptr, N.dptr(q), S, N.uptr(face), N.uptr(part),
                                          N.dptr(pt)))
        return (face, part, pt) if nearest_part else (face, pt)
