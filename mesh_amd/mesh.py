"""Minimal ``Mesh`` facade carrying the search / visibility methods of psbody-mesh's ``Mesh``
(mesh/mesh.py:48-80 for v/f coercion, :208-222, :282-302, :439-455).  Only the hot-path callers are
mirrored; I/O, topology, texture and viewing are out of scope.
"""
import numpy as np

from . import _native as N
from . import search


class Mesh(object):
    def __init__(self, v=None, f=None, vn=None):
        if v is not None:
            self.v = np.array(v, dtype=np.float64)
        if f is not None:
            self.f = np.require(f, dtype=np.uint32)
        if vn is not None:
            self.vn = np.array(vn, dtype=np.float64)

    # ---- geometry helpers used by the callers (mesh.py:208-222) ----
    def estimate_vertex_normals(self):
        """Area-weighted vertex normals on the GPU (mesh.py:208-216): every vertex sums the scaled
        normals of its faces in ascending face order (the reference's sparse face->vertex product over
        TriNormalsScaled), then divides by the row norm (0 -> 1)."""
        v = np.ascontiguousarray(self.v, dtype=np.float64).reshape(-1, 3)
        f = np.ascontiguousarray(self.f, dtype=np.uint32).reshape(-1, 3)
        if f.size and int(f.max()) >= v.shape[0]:
            raise ValueError("face index out of range")
        vn = np.empty_like(v)
        N.check(N.lib().msh_vertex_normals(N.dptr(v), v.shape[0], N.uptr(f), f.shape[0], N.dptr(vn)))
        return vn

    def barycentric_coordinates_for_points(self, points, face_indices):
        """(vertex indices, barycentric coordinates of the projection) — mesh.py:218-222."""
        vertex_indices = self.f[face_indices.flatten(), :]
        a = self.v[vertex_indices[:, 0]]
        u = self.v[vertex_indices[:, 1]] - a
        w = self.v[vertex_indices[:, 2]] - a
        p = np.asarray(points, dtype=np.float64).reshape(-1, 3)
        n = np.cross(u, w)
        s = np.sum(n * n, axis=1)
        s[s == 0] = 1e-16
        oneOver4ASquared = 1.0 / s
        wp = p - a
        b2 = np.sum(np.cross(u, wp) * n, axis=1) * oneOver4ASquared
        b1 = np.sum(np.cross(wp, w) * n, axis=1) * oneOver4ASquared
        return vertex_indices, np.array((1 - b1 - b2, b1, b2)).T

    # ---- visibility (mesh.py:282-302) ----
    def vertex_visibility(self, camera, normal_threshold=None, omni_directional_camera=False, binary_visiblity=True):
        vis, n_dot_cam = self.vertex_visibility_and_normals(camera, omni_directional_camera)
        if normal_threshold is not None:
            vis = np.logical_and(vis, n_dot_cam > normal_threshold)
        return np.squeeze(vis) if binary_visiblity else np.squeeze(vis * n_dot_cam)

    def vertex_visibility_and_normals(self, camera, omni_directional_camera=False):
        from .visibility import visibility_compute
        arguments = {'v': self.v, 'f': self.f, 'cams': np.array([camera.origin.flatten()])}
        if not omni_directional_camera:
            arguments['sensors'] = np.array([camera.sensor_axis.flatten()])
        arguments['n'] = self.vn if hasattr(self, 'vn') else self.estimate_vertex_normals()
        return visibility_compute(**arguments)

    # ---- search methods (mesh.py:439-455) ----
    def compute_aabb_tree(self):
        return search.AabbTree(self)

    def compute_aabb_normals_tree(self):
        return search.AabbNormalsTree(self)

    def compute_closest_point_tree(self, use_cgal=False):
        return search.CGALClosestPointTree(self) if use_cgal else search.ClosestPointTree(self)

    def closest_vertices(self, vertices, use_cgal=False):
        return self.compute_closest_point_tree(use_cgal).nearest(vertices)

    def closest_points(self, vertices):
        return self.closest_faces_and_points(vertices)[1]

    def closest_faces_and_points(self, vertices):
        return self.compute_aabb_tree().nearest(vertices)
