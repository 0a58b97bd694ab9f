"""Minimal ``Mesh`` facade carrying the search / visibility methods of psbody-mesh's ``Mesh``
(mesh/mesh.py:48-80 for v/f coercion, :208-248, :282-302, :439-455).  Only the hot-path callers are
mirrored; I/O, topology, texture and viewing are out of scope.
"""
import numpy as np

from . import _native as N
from . import search


class Mesh(object):
    def __init__(self, v=None, f=None, vn=None, filename=None):
        if filename is not None:
            self.load_from_file(filename)
        if v is not None:
            self.v = np.array(v, dtype=np.float64)
        if f is not None:
            self.f = np.require(f, dtype=np.uint32)
        if vn is not None:
            self.vn = np.array(vn, dtype=np.float64)

    # ---- mesh files (serialization.py:97-131, 410-445) through the native readers ----
    def load_from_file(self, filename):
        if filename.endswith(".ply"):
            self.load_from_ply(filename)
        elif filename.endswith(".obj"):
            self.load_from_obj(filename)
        else:
            raise NotImplementedError("Unknown mesh file format.")

    def load_from_obj(self, filename):
        """Geometry, groups and landmarks of load_from_obj_cpp (serialization.py:97-131); materials and
        textures are out of scope."""
        from collections import OrderedDict
        from .serialization.loadobj import loadobj
        v, vt, vn, f, ft, fn, mtl_path, landm, segm = loadobj(filename)
        for name, a in (("v", v), ("f", f), ("vn", vn), ("vt", vt), ("fn", fn), ("ft", ft)):
            if a.size != 0:
                setattr(self, name, a)
        if segm:
            self.segm = OrderedDict((k, x.tolist()) for k, x in segm.items())
        if landm:
            self.landm = landm
            self.landm_xyz = dict((k, self.v[i]) for k, i in landm.items())

    def load_from_ply(self, filename):
        """serialization.py:426-445: v, f, vertex colours / 255, normals."""
        from .serialization import plyutils
        v, tri, color, normals = plyutils.read_arrays(filename)
        self.v = v
        self.f = tri.copy()
        if color is not None:
            self.vc = color / 255
        if normals is not None:
            self.vn = normals

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
        s[s == 0] = np.spacing(1)  # barycentric_coordinates_of_projection.py:38-41
        oneOver4ASquared = 1.0 / s
        wp = p - a
        b2 = np.sum(np.cross(u, wp) * n, axis=1) * oneOver4ASquared
        b1 = np.sum(np.cross(wp, w) * n, axis=1) * oneOver4ASquared
        return vertex_indices, np.array((1 - b1 - b2, b1, b2)).T

    # ---- segmentation transfer (mesh.py:224-248), a caller of the closest-face query ----
    def parts_by_face(self):
        """Part name of every face ('' for a face in no part), mesh.py:243-248."""
        segments_by_face = [''] * len(self.f)
        for part in self.segm.keys():
            for face in self.segm[part]:
                segments_by_face[face] = part
        return segments_by_face

    def transfer_segm(self, mesh, exclude_empty_parts=True):
        """Give every face of this mesh the part of the face of `mesh` closest to its centre
        (mesh.py:224-237).  The centres are computed vectorised with the reference's operation order
        (a face's mean is (v0 + v1 + v2) / 3, as np.mean over its 3 rows), all centres go to the GPU in
        one closest-face query, and the faces are grouped per part with a stable sort (each part's
        list ascending, as the reference's sorted lists).  A face whose closest face of `mesh` is in no
        part belongs to the part named '' when `mesh` has one (parts_by_face maps such faces to ''), and
        raises KeyError('') otherwise, as the reference's segm[''] lookup does."""
        self.segm = {}
        if not hasattr(mesh, 'segm'):
            return
        v = np.asarray(self.v, dtype=np.float64)
        f = np.asarray(self.f).astype(np.int64)
        centres = (v[f[:, 0]] + v[f[:, 1]] + v[f[:, 2]]) / 3.0
        closest_faces, _ = mesh.closest_faces_and_points(centres)
        names = list(mesh.segm.keys())
        part_of = np.full(len(mesh.f), -1, dtype=np.int64)
        for k, part in enumerate(names):  # later parts win, as in parts_by_face
            part_of[np.asarray(mesh.segm[part], dtype=np.int64)] = k
        pid = part_of[np.asarray(closest_faces).ravel().astype(np.int64)]
        if (pid < 0).any():
            if '' not in names:
                raise KeyError('')
            pid[pid < 0] = names.index('')
        order = np.argsort(pid, kind='stable')
        bounds = np.searchsorted(pid[order], np.arange(len(names) + 1))
        self.segm = dict((part, order[bounds[k]:bounds[k + 1]].tolist()) for k, part in enumerate(names))
        if exclude_empty_parts:
            for part in list(self.segm.keys()):
                if not self.segm[part]:
                    del self.segm[part]

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
        # a tree built for one query batch, as the reference does (mesh.py:454-455).  Its entry cut (each cell
        # answered at build time) pays off only when the batch is large against it.  Round 4, about 8 grid cells per
        # face (at most 2^23): C2's 10M queries on 13,776 faces 25 -> 21 ms with it, C3's 100M on 1M faces 149 -> 198 ms
        # (profiles/r04_facade_cut_policy.json).  Round 5: the default grid (64 cells per face, at most 2^26) takes C2
        # to 18.7 ms (22.1 with the coarse one) and C3 to 235 ms (100 ms without a cut;
        # profiles/r05_bench_configs_c4_facade.jsonl).  So: the default grid for >= 8 queries per cell of it, else the
        # coarse grid for >= 32 queries per cell of that, else none
        tree = self.compute_aabb_tree()
        n_q = int(np.prod(np.shape(vertices)[:-1])) if np.ndim(vertices) > 1 else 0
        fine, coarse = min(64 * len(self.f), 1 << 26), min(8 * len(self.f), 1 << 23)
        if n_q >= 8 * fine:
            tree.cpp_handle.set_entry_cut(-1)
        elif n_q >= 32 * coarse:
            tree.cpp_handle.set_entry_cut(max(16, int(round(coarse ** (1.0 / 3.0)))))
        else:
            tree.cpp_handle.set_entry_cut(0)
        return tree.nearest(vertices)
