"""ORACLE — test infrastructure only (see oracle.cpp header).

ctypes wrapper around ``oracle/_build/liboracle.so``, the CPU restatement of CGAL 4.7's
AABB-tree algorithms used by psbody-mesh (``mesh/src/spatialsearchmodule.cpp``,
``aabb_normals.cpp``, ``visibility.cpp``).  Only ``tests/``, ``__graft_entry__.smoke()`` and
``bench.py``'s ``cpu_baseline`` leg import this module, and only as the checker / CPU baseline.
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("ORACLE_LIB", os.path.join(_HERE, "_build", "liboracle.so"))  # ORACLE_LIB: sanitizer build

_c_double_p = ctypes.POINTER(ctypes.c_double)
_c_u32_p = ctypes.POINTER(ctypes.c_uint32)
_c_u64_p = ctypes.POINTER(ctypes.c_uint64)
_lib = None


def build():
    import subprocess
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        sz, vp, i = ctypes.c_size_t, ctypes.c_void_p, ctypes.c_int
        L.ora_point_triangle.restype = ctypes.c_double
        L.ora_point_triangle.argtypes = [_c_double_p] * 5 + [_c_u32_p]
        L.ora_cgal_tree_build.restype = vp
        L.ora_cgal_tree_build.argtypes = [_c_double_p, sz, _c_u32_p, sz, i, ctypes.c_double]
        L.ora_cgal_tree_free.argtypes = [vp]
        L.ora_cgal_tree_free.restype = None
        L.ora_cgal_tree_nearest.argtypes = [vp, _c_double_p, sz, _c_u32_p, _c_u32_p, _c_double_p, i, _c_u64_p]
        L.ora_cgal_tree_nearest.restype = None
        L.ora_cgal_ntree_nearest.argtypes = [vp, _c_double_p, _c_double_p, sz, _c_u32_p, _c_double_p, i]
        L.ora_cgal_ntree_nearest.restype = None
        L.ora_cgal_tree_alongnormal.argtypes = [vp, _c_double_p, _c_double_p, sz, _c_double_p, _c_u32_p, _c_double_p,
                                                i, _c_u64_p]
        L.ora_cgal_tree_alongnormal.restype = None
        L.ora_cgal_tree_visibility.argtypes = [vp, _c_double_p, sz, _c_double_p, sz, _c_double_p, _c_double_p,
                                               ctypes.c_double, _c_u32_p, _c_double_p, i]
        L.ora_cgal_tree_visibility.restype = None
        L.ora_brute_nearest.argtypes = [_c_double_p, sz, _c_u32_p, sz, _c_double_p, sz, _c_u32_p, _c_u32_p,
                                        _c_double_p, _c_double_p, i]
        L.ora_brute_nearest.restype = None
        L.ora_brute_nnearest.argtypes = [_c_double_p, sz, _c_u32_p, sz, ctypes.c_double, _c_double_p, _c_double_p, sz,
                                         _c_u32_p, _c_double_p, _c_double_p, i]
        L.ora_brute_nnearest.restype = None
        L.ora_brute_alongnormal.argtypes = [_c_double_p, sz, _c_u32_p, sz, _c_double_p, _c_double_p, sz, _c_double_p,
                                            _c_u32_p, _c_double_p, i]
        L.ora_brute_alongnormal.restype = None
        L.ora_brute_visibility.argtypes = [_c_double_p, sz, _c_double_p, sz, _c_double_p, sz, _c_double_p, _c_double_p,
                                           ctypes.c_double, _c_u32_p, _c_double_p, i]
        L.ora_brute_visibility.restype = None
        L.ora_tri_tri_overlap.argtypes = [_c_double_p, _c_double_p]
        L.ora_tri_tri_overlap.restype = i
        L.ora_brute_intersections.argtypes = [_c_double_p, sz, _c_u32_p, sz, _c_double_p, sz, _c_u32_p, sz, _c_u32_p, i]
        L.ora_brute_intersections.restype = sz
        L.ora_brute_selfintersects.argtypes = [_c_double_p, sz, _c_u32_p, sz, i]
        L.ora_brute_selfintersects.restype = ctypes.c_long
        L.ora_brute_vertex_nn.argtypes = [_c_double_p, sz, _c_double_p, sz, _c_u32_p, _c_double_p, i]
        L.ora_brute_vertex_nn.restype = None
        _lib = L
    return _lib


def _d(a):
    return np.ascontiguousarray(a, dtype=np.float64)


def _u(a):
    return np.ascontiguousarray(a, dtype=np.uint32)


def _pd(a):
    return a.ctypes.data_as(_c_double_p) if a is not None else None


def _pu(a):
    return a.ctypes.data_as(_c_u32_p) if a is not None else None


def point_triangle(q, a, b, c):
    """Closest point of triangle abc to q with CGAL's construction -> (point, part, d2)."""
    q, a, b, c = _d(q), _d(a), _d(b), _d(c)
    pt = np.empty(3)
    part = np.zeros(1, np.uint32)
    d2 = lib().ora_point_triangle(_pd(q), _pd(a), _pd(b), _pd(c), _pd(pt), _pu(part))
    return pt, int(part[0]), d2


class CgalTree(object):
    """CGAL 4.7 AABB_tree restatement (median split, KD hint, left-first traversal)."""

    def __init__(self, v, f, hint=True, eps=0.0):
        self.v, self.f = _d(v), _u(f)
        self.h = lib().ora_cgal_tree_build(_pd(self.v), self.v.shape[0], _pu(self.f), self.f.shape[0],
                                           1 if hint else 0, float(eps))

    def __del__(self):
        if getattr(self, "h", None):
            lib().ora_cgal_tree_free(self.h)
            self.h = None

    def nearest(self, q, threads=0, count_visits=False):
        q = _d(q).reshape(-1, 3)
        S = q.shape[0]
        face = np.empty(S, np.uint32)
        part = np.empty(S, np.uint32)
        pt = np.empty((S, 3))
        visits = np.zeros(1, np.uint64)
        lib().ora_cgal_tree_nearest(self.h, _pd(q), S, _pu(face), _pu(part), _pd(pt), int(threads),
                                    visits.ctypes.data_as(_c_u64_p) if count_visits else None)
        if count_visits:
            return face, part, pt, int(visits[0])
        return face, part, pt

    def nnearest(self, q, n, threads=0):
        q, n = _d(q).reshape(-1, 3), _d(n).reshape(-1, 3)
        S = q.shape[0]
        face = np.empty(S, np.uint32)
        pt = np.empty((S, 3))
        lib().ora_cgal_ntree_nearest(self.h, _pd(q), _pd(n), S, _pu(face), _pd(pt), int(threads))
        return face, pt

    def alongnormal(self, p, n, threads=0, count_tests=False):
        """aabbtree_nearest_alongnormal through the tree (spatialsearchmodule.cpp:272-321):
        (dist, face, point); no hit -> 1e100, 0xFFFFFFFF, NaN."""
        p, n = _d(p).reshape(-1, 3), _d(n).reshape(-1, 3)
        S = p.shape[0]
        dist = np.empty(S)
        face = np.empty(S, np.uint32)
        pt = np.empty((S, 3))
        tests = np.zeros(1, np.uint64)
        lib().ora_cgal_tree_alongnormal(self.h, _pd(p), _pd(n), S, _pd(dist), _pu(face), _pd(pt), int(threads),
                                        tests.ctypes.data_as(_c_u64_p) if count_tests else None)
        if count_tests:
            return dist, face, pt, int(tests[0])
        return dist, face, pt


class CgalVisibilityTree(CgalTree):
    """visibility_compute's tree over main + extra triangles (py_visibility.cpp:140-163), no hint."""

    def __init__(self, v, f, extra_v=None, extra_f=None):
        v, f = _d(v), _u(f)
        self.main_v = v
        if extra_v is not None and extra_f is not None:
            ev, ef = _d(extra_v), _u(extra_f)
            f = np.vstack([f, ef + np.uint32(v.shape[0])])
            v = np.vstack([v, ev])
        super().__init__(v, f, hint=False)

    def visibility(self, cams, n=None, sensors=None, min_dist=1e-3, threads=0, src_idx=None):
        """(vis (C,P'), ndc (C,P')) cast from the main vertices (or v[src_idx])."""
        cams = _d(cams).reshape(-1, 3)
        v = self.main_v if src_idx is None else _d(self.main_v[np.asarray(src_idx)])
        if n is not None and src_idx is not None:
            n = np.asarray(n)[np.asarray(src_idx)]
        P, C = v.shape[0], cams.shape[0]
        vis = np.empty((C, P), np.uint32)
        ndc = np.empty((C, P))
        nn = _d(n) if n is not None else None
        ss = _d(sensors) if sensors is not None else None
        lib().ora_cgal_tree_visibility(self.h, _pd(v), P, _pd(cams), C, _pd(nn), _pd(ss), float(min_dist), _pu(vis),
                                       _pd(ndc), int(threads))
        return vis, ndc


def brute_nearest(v, f, q, threads=0):
    """Exhaustive closest point, lexicographic min (d2, face) -> (face, part, point, d2)."""
    v, f, q = _d(v), _u(f), _d(q).reshape(-1, 3)
    S = q.shape[0]
    face = np.empty(S, np.uint32)
    part = np.empty(S, np.uint32)
    pt = np.empty((S, 3))
    d2 = np.empty(S)
    lib().ora_brute_nearest(_pd(v), v.shape[0], _pu(f), f.shape[0], _pd(q), S, _pu(face), _pu(part), _pd(pt), _pd(d2),
                            int(threads))
    return face, part, pt, d2


def brute_nnearest(v, f, eps, q, n, threads=0):
    v, f, q, n = _d(v), _u(f), _d(q).reshape(-1, 3), _d(n).reshape(-1, 3)
    S = q.shape[0]
    face = np.empty(S, np.uint32)
    pt = np.empty((S, 3))
    met = np.empty(S)
    lib().ora_brute_nnearest(_pd(v), v.shape[0], _pu(f), f.shape[0], float(eps), _pd(q), _pd(n), S, _pu(face), _pd(pt),
                             _pd(met), int(threads))
    return face, pt, met


def brute_alongnormal(v, f, p, n, threads=0):
    v, f, p, n = _d(v), _u(f), _d(p).reshape(-1, 3), _d(n).reshape(-1, 3)
    S = p.shape[0]
    dist = np.empty(S)
    face = np.empty(S, np.uint32)
    pt = np.empty((S, 3))
    lib().ora_brute_alongnormal(_pd(v), v.shape[0], _pu(f), f.shape[0], _pd(p), _pd(n), S, _pd(dist), _pu(face),
                                _pd(pt), int(threads))
    return dist, face, pt


def brute_visibility(v, f, cams, n=None, sensors=None, extra_v=None, extra_f=None, min_dist=1e-3, threads=0,
                     src_idx=None):
    """(vis (C,P'), ndc (C,P')); with src_idx only the rays from vertices v[src_idx] are cast (against
    every triangle), n is then indexed like v."""
    v, f, cams = _d(v), _u(f), _d(cams).reshape(-1, 3)
    tris = v[f.astype(np.int64)].reshape(-1, 9)
    if src_idx is not None:
        v = _d(v[np.asarray(src_idx)])
        if n is not None:
            n = np.asarray(n)[np.asarray(src_idx)]
    if extra_v is not None and extra_f is not None:
        ev, ef = _d(extra_v), _u(extra_f)
        tris = np.vstack([tris, ev[ef.astype(np.int64)].reshape(-1, 9)])
    tris = _d(tris)
    P, C = v.shape[0], cams.shape[0]
    vis = np.empty((C, P), np.uint32)
    ndc = np.empty((C, P))
    nn = _d(n) if n is not None else None
    ss = _d(sensors) if sensors is not None else None
    lib().ora_brute_visibility(_pd(v), P, _pd(tris), tris.shape[0], _pd(cams), C, _pd(nn), _pd(ss), float(min_dist),
                               _pu(vis), _pd(ndc), int(threads))
    return vis, ndc


def tri_tri_overlap(t1, t2):
    t1, t2 = _d(t1).reshape(9), _d(t2).reshape(9)
    return bool(lib().ora_tri_tri_overlap(_pd(t1), _pd(t2)))


def brute_intersections(v, f, qv, qf, threads=0):
    v, f, qv, qf = _d(v), _u(f), _d(qv), _u(qf)
    out = np.empty(qf.shape[0], np.uint32)
    K = lib().ora_brute_intersections(_pd(v), v.shape[0], _pu(f), f.shape[0], _pd(qv), qv.shape[0], _pu(qf),
                                      qf.shape[0], _pu(out), int(threads))
    return out[:K].copy()


def brute_selfintersects(v, f, threads=0):
    v, f = _d(v), _u(f)
    return int(lib().ora_brute_selfintersects(_pd(v), v.shape[0], _pu(f), f.shape[0], int(threads)))


def brute_vertex_nn(v, q, threads=0):
    v, q = _d(v), _d(q).reshape(-1, 3)
    S = q.shape[0]
    idx = np.empty(S, np.uint32)
    dist = np.empty(S)
    lib().ora_brute_vertex_nn(_pd(v), v.shape[0], _pd(q), S, _pu(idx), _pd(dist), int(threads))
    return idx, dist


# ---- geometry feeding the path (numpy/scipy restatements, operation for operation) ----------------
def tri_normals_scaled(v, f):
    """TriNormalsScaled (geometry/tri_normals.py:23-24, :40-44 _edges_for): cross(v[f1]-v[f0], v[f2]-v[f0])
    with numpy's cross (geometry/cross_product.py delegates to the same component formulas)."""
    v = np.asarray(v, dtype=np.float64).reshape(-1, 3)
    f = np.asarray(f).astype(np.int64)
    e1 = v[f[:, 1]] - v[f[:, 0]]
    e2 = v[f[:, 2]] - v[f[:, 0]]
    return np.cross(e1, e2)


def estimate_vertex_normals(v, f):
    """Mesh.estimate_vertex_normals (mesh.py:208-216) with faces_by_vertex(as_sparse_matrix=True)
    (mesh.py:202-205): CSR (P,T) incidence times the scaled face normals, row norms via ``** 0.5``,
    zero norms -> 1."""
    import scipy.sparse as sp
    v = np.asarray(v, dtype=np.float64).reshape(-1, 3)
    f = np.asarray(f, dtype=np.uint32).reshape(-1, 3)
    fn = tri_normals_scaled(v, f).reshape(-1, 3)
    row = f.flatten()
    col = np.array([range(f.shape[0])] * 3).T.flatten()
    data = np.ones(len(col))
    ftov = sp.csr_matrix((data, (row, col)), shape=(v.shape[0], f.shape[0]))
    nsn = ftov * fn
    norms = (np.sum(nsn ** 2.0, axis=1) ** 0.5).T
    norms[norms == 0] = 1.0
    return (nsn.T / norms).T


def vert_normals(v, f):
    """geometry/vert_normals.py:19-35 VertNormals (CSC (3P,3T) incidence, NormalizedNx3); the reference's
    tests/test_geometry.py:61-68 requires estimate_vertex_normals to match it within 1e-15."""
    import scipy.sparse as sp
    v = np.asarray(v, dtype=np.float64).reshape(-1, 3)
    f = np.asarray(f, dtype=np.uint32).reshape(-1, 3)
    IS = f.flatten().astype(np.int64)
    JS = np.array([range(f.shape[0])] * 3).T.flatten()
    data = np.ones(len(JS))
    IS = np.concatenate((IS * 3, IS * 3 + 1, IS * 3 + 2))
    JS = np.concatenate((JS * 3, JS * 3 + 1, JS * 3 + 2))
    data = np.concatenate((data, data, data))
    m = sp.csc_matrix((data, (IS, JS)), shape=(v.size, f.size))
    x = m.dot(tri_normals_scaled(v, f).flatten().reshape(-1, 1)).flatten()
    x = x.reshape(-1, 3)
    ss = np.sum(x ** 2, axis=1)
    ss[ss == 0] = 1
    return x / np.sqrt(ss).reshape(-1, 1)


def barycentric_coordinates_of_projection(p, q, u, v):
    """geometry/barycentric_coordinates_of_projection.py:9-49 (Heidrich, JGT 2005), same operation order."""
    p, q, u, v = (np.asarray(a, dtype=np.float64).T for a in (p, q, u, v))
    n = np.cross(u, v, axis=0)
    s = np.sum(n * n, axis=0)
    if np.isscalar(s):
        s = s if s else np.spacing(1)
    else:
        s[s == 0] = np.spacing(1)
    one_over_4a2 = 1.0 / s
    w = p - q
    b2 = np.sum(np.cross(u, w, axis=0) * n, axis=0) * one_over_4a2
    b1 = np.sum(np.cross(w, v, axis=0) * n, axis=0) * one_over_4a2
    return np.vstack((1 - b1 - b2, b1, b2)).T


def barycentric_coordinates_for_points(v, f, points, face_indices):
    """Mesh.barycentric_coordinates_for_points (mesh.py:218-222)."""
    vi = np.asarray(f)[np.asarray(face_indices).flatten(), :]
    a, b, c = v[vi[:, 0]], v[vi[:, 1]], v[vi[:, 2]]
    return vi, barycentric_coordinates_of_projection(points, a, b - a, c - a)


def transfer_segm(v, f, mesh_segm, closest_faces, exclude_empty_parts=True):
    """Mesh.transfer_segm (mesh.py:224-237) as the reference writes it, with the closest faces supplied
    (the reference gets them from mesh.closest_faces_and_points(face_centres))."""
    n_mesh_faces = 1 + max((max(x) for x in mesh_segm.values() if len(x)), default=0)
    segments_by_face = [''] * max(n_mesh_faces, int(np.max(closest_faces)) + 1)
    for part in mesh_segm.keys():
        for face in mesh_segm[part]:
            segments_by_face[face] = part
    parts_by_face = [segments_by_face[face] for face in np.asarray(closest_faces).flatten()]
    segm = dict([(part, []) for part in mesh_segm.keys()])
    for face, part in enumerate(parts_by_face):
        segm[part].append(face)
    for part in list(segm.keys()):
        segm[part].sort()
        if exclude_empty_parts and not segm[part]:
            del segm[part]
    return segm


def face_centres(v, f):
    """np.array([v[face, :].mean(axis=0) for face in f]) (mesh.py:227)."""
    return np.array([np.asarray(v)[face, :].mean(axis=0) for face in np.asarray(f)])


# ---- mesh files (pure-Python restatements of the reference readers; small files only) -------------
def loadobj(path):
    """mesh/src/py_loadobj.cpp:62-243, line for line: returns (v, vt, vn, f, ft, fn, mtl_path, landm, segm)."""
    import re
    num = re.compile(r"[+-]?(\d+\.?\d*|\.\d+)([eE][+-]?\d+)?")

    def doubles(s):
        out = []
        for tok in s.split():
            m = num.match(tok)
            if not m:
                break
            if m.group(0) in ("+", "-"):
                break
            out.append(float(m.group(0)))
            if m.end() != len(tok):
                break
        return out

    def atoi(s):
        m = re.match(r"\s*([+-]?\d+)", s)
        return int(m.group(1)) if m else 0

    v, vt, vn, f, ft, fn = [], [], [], [], [], []
    segm, landm = {}, {}
    next_v_is_land, land_name, curr, mtl, len_vt = False, "", "", "", 3
    with open(path, "rb") as fh:
        data = fh.read().decode("latin-1")
    lines = data.split("\n")
    if lines and lines[-1] == "":
        lines.pop()
    for line in lines:
        if line[:6] == "mtllib":
            mtl = line[6:]
        if line[:1] == "g":
            curr = line[2:]
            segm.setdefault(curr, [])
        if line[:2] == "vt":
            x = doubles(line[2:])
            vt += x
            len_vt = len(x)
        elif line[:2] == "vn":
            vn += doubles(line[2:])
        elif line[:1] == "f":
            lf, lt, ln = [], [], []
            for tok in line[1:].split():
                parts = tok.split("/")
                if parts and parts[-1] == "" and len(parts) > 1:
                    parts = parts[:-1]  # getline yields no empty tail after a trailing '/'
                for counter, el in enumerate(parts):
                    if el and counter < 3:
                        (lf, lt, ln)[counter].append(atoi(el))
            for (loc, dst) in ((lf, f), (lt, ft), (ln, fn)):
                for i in range(1, len(loc) - 1):
                    dst += [(loc[0] - 1) & 0xFFFFFFFF, (loc[i] - 1) & 0xFFFFFFFF, (loc[i + 1] - 1) & 0xFFFFFFFF]
                    if dst is f and curr != "":
                        segm[curr].append(len(f) // 3 - 1)
        elif line[:1] == "v":
            v += doubles(line[1:])
            if next_v_is_land:
                next_v_is_land = False
                landm[land_name] = len(v) // 3 - 1
        elif line[:9] == "#landmark":
            next_v_is_land = True
            land_name = line[10:]
    nv, nvn = len(v) // 3, len(vn) // 3
    nvt = len(vt) // len_vt if len_vt else 0
    return (np.array(v[:3 * nv], dtype=np.float64).reshape(nv, 3),
            np.array(vt[:nvt * len_vt], dtype=np.float64).reshape(nvt, len_vt),
            np.array(vn[:3 * nvn], dtype=np.float64).reshape(nvn, 3),
            np.array(f, dtype=np.uint32).reshape(-1, 3), np.array(ft, dtype=np.uint32).reshape(-1, 3),
            np.array(fn, dtype=np.uint32).reshape(-1, 3), mtl, dict(sorted(landm.items())),
            dict((k, np.array(x, dtype=np.uint32)) for k, x in sorted(segm.items())))


def ply_read(path):
    """plyutils.read (mesh/src/plyutils.c:64-139) over rply's reader: dict of lists of floats, or raises
    ValueError with the reference's message."""
    import struct
    with open(path, "rb") as fh:
        data = fh.read()
    if data[:4] != b"ply\n":
        raise ValueError("Failed to open PLY file.")
    pos = 4
    mode, elems = None, []
    types = {"int8": "b", "char": "b", "uint8": "B", "uchar": "B", "int16": "h", "short": "h", "uint16": "H",
             "ushort": "H", "int32": "i", "int": "i", "uint32": "I", "uint": "I", "float32": "f", "float": "f",
             "float64": "d", "double": "d"}
    ok = False
    while True:
        nl = data.find(b"\n", pos)
        if nl < 0:
            break
        w = data[pos:nl].decode("latin-1").replace("\r", " ").split()
        pos = nl + 1
        if not w:
            continue
        if w[0] == "end_header":
            ok = True
            break
        if w[0] in ("comment", "obj_info"):
            continue
        if w[0] == "format" and len(w) >= 3 and w[2] == "1.0" and w[1] in ("ascii", "binary_little_endian",
                                                                          "binary_big_endian"):
            mode = w[1]
        elif w[0] == "element" and len(w) == 3:
            elems.append([w[1], int(w[2]), []])
        elif w[0] == "property" and elems and len(w) == 5 and w[1] == "list" and w[2] in types and w[3] in types:
            elems[-1][2].append((w[4], types[w[2]], types[w[3]]))
        elif w[0] == "property" and elems and len(w) == 3 and w[1] in types:
            elems[-1][2].append((w[2], None, types[w[1]]))
        else:
            break
    if not ok or mode is None:
        raise ValueError("plyread_mex: Bad raw header.")
    body = data[pos:]
    ascii_words = body.decode("latin-1").split() if mode == "ascii" else None
    wi = [0]
    bo = [0]
    end = "<" if mode == "binary_little_endian" else ">"
    lims = {"b": (-128, 127), "B": (0, 255), "h": (-32768, 32767), "H": (0, 65535),
            "i": (-2 ** 31, 2 ** 31 - 1), "I": (0, 2 ** 32 - 1), "f": (-3.4028234663852886e38, 3.4028234663852886e38),
            "d": (-np.inf, np.inf)}

    def val(t):
        if ascii_words is not None:
            if wi[0] >= len(ascii_words):
                raise ValueError("Read failed. " + path)
            s = ascii_words[wi[0]]
            wi[0] += 1
            try:
                x = float(s) if t in "fd" else float(int(s, 10))
            except ValueError:
                raise ValueError("Read failed. " + path)
            if not (lims[t][0] <= x <= lims[t][1]):
                raise ValueError("Read failed. " + path)
            return x
        n = struct.calcsize(t)
        if bo[0] + n > len(body):
            raise ValueError("Read failed. " + path)
        x = struct.unpack(end + t, body[bo[0]:bo[0] + n])[0]
        bo[0] += n
        return float(x)

    vert = next((e for e in elems if e[0] == "vertex"), None)
    face = next((e for e in elems if e[0] == "face"), None)
    names = [p[0] for p in vert[2]] if vert else []
    has_color = any(n in names for n in ("red", "green", "blue"))
    has_normals = any(n in names for n in ("nx", "ny", "nz"))
    fnames = [p[0] for p in face[2]] if face else []
    fprop = "vertex_indices" if ("vertex_indices" in fnames and face[1] > 0) else "vertex_index"
    nv = vert[1] if vert else 0
    nf = face[1] if (face and fprop in fnames) else 0
    cols = {k: [float("nan")] * nv for k in ("x", "y", "z", "red", "green", "blue", "nx", "ny", "nz")}
    tri = [[float("nan")] * nf for _ in range(3)]
    for e in elems:
        for i in range(e[1]):
            for (name, ct, it) in e[2]:
                if ct is None:
                    x = val(it)
                    if e is vert and name in cols:
                        cols[name][i] = x
                else:
                    c = int(val(ct))
                    for k in range(c):
                        x = val(it)
                        if e is face and name == fprop and k < 3:
                            tri[k][i] = x
    res = {"pts": [cols["x"], cols["y"], cols["z"]], "tri": tri}
    if has_color:
        res["color"] = [cols["red"], cols["green"], cols["blue"]]
    if has_normals:
        res["normals"] = [cols["nx"], cols["ny"], cols["nz"]]
    return res
