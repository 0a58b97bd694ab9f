"""The oracle (CPU restatement of CGAL 4.7's algorithms) pinned against the reference's own known
answers and against scipy (ClosestPointTree's third-party arithmetic).  CPU only."""
import os

import numpy as np
import pytest

import workloads as W


def test_aabb_tree_known_answer(oracle, ref_tests):
    # tests/test_mesh.py:89-109
    t = ref_tests["test_aabb_tree"]
    v, f, q = np.array(t["v"], float), np.array(t["f"]), np.array(t["q"], float)
    for face, part, pt in [oracle.CgalTree(v, f).nearest(q), oracle.brute_nearest(v, f, q)[:3]]:
        assert np.max(np.abs(face.astype(int) - np.array(t["f_expected"]))) < 1e-6
        assert np.max(np.abs(pt - np.array(t["v_expected"]))) < t["tol"]


@pytest.mark.parametrize("name", ["test_dist_classic", "test_dist_normals"])
def test_normals_known_answer(oracle, meshes, ref_tests, name):
    # tests/test_aabb_n_tree.py:29-52 — exact equality of fp64 points
    t = ref_tests[name]
    v, f = meshes[t["mesh"] + "_v"], meshes[t["mesh"] + "_f"]
    face, pt = oracle.CgalTree(v, f, hint=False, eps=t["eps"]).nnearest(t["q"], t["n"])
    assert (face[None, :] == np.array(t["f_expected"])).all()
    assert (pt == np.array(t["p_expected"])).all()
    bface, bpt, _ = oracle.brute_nnearest(v, f, t["eps"], t["q"], t["n"])
    assert (bface == face).all() and (bpt == pt).all()


def _tri_normals(v, f):
    a, b, c = v[f[:, 0]], v[f[:, 1]], v[f[:, 2]]
    n = np.cross(b - a, c - a)
    return n / np.linalg.norm(n, axis=1)[:, None]


def cylinder_query(meshes):
    tv, tf = meshes["cylinder_trans_v"], meshes["cylinder_trans_f"]
    tn = _tri_normals(tv, tf)
    qn = np.zeros(tv.shape)
    for i in range(tf.shape[0]):
        qn[tf[i]] += tn[i]
    return tv, qn / np.linalg.norm(qn, axis=1)[:, None]


def test_cylinders_known_answer(oracle, meshes, ref_tests):
    # tests/test_aabb_n_tree.py:54-76
    t = ref_tests["test_cylinders"]
    v, f = meshes["cylinder_v"], meshes["cylinder_f"]
    q, qn = cylinder_query(meshes)
    a, _ = oracle.CgalTree(v, f, hint=False, eps=t["eps_no"]).nnearest(q, qn)
    b, _ = oracle.CgalTree(v, f, hint=False, eps=t["eps_yes"]).nnearest(q, qn)
    assert np.unique(a).shape[0] <= t["max_unique_no"]
    assert np.unique(b).shape[0] >= f.shape[0] - t["min_unique_yes_slack"]


def test_selfintersects_known_answer(oracle, meshes, ref_tests):
    # tests/test_aabb_n_tree.py:78-89
    for name, want in ref_tests["test_selfintersects"].items():
        assert oracle.brute_selfintersects(meshes[name + "_v"], meshes[name + "_f"]) == want


def test_intersections_known_answer(oracle, meshes, ref_tests):
    # tests/test_intersections.py:27 (disabled in the reference)
    t = ref_tests["test_intersections"]
    v, f = meshes["icosphere_v"], meshes["icosphere_f"]
    qv = v * t["radius"] + np.array(t["q_center"], float)
    mv = v * t["radius"] + np.array(t["m_center"], float)
    assert oracle.brute_intersections(mv, f, qv, f).tolist() == t["expected"]


def visibility_cases(t):
    v = np.array(t["v"])
    f = np.array(t["f1"], dtype=np.uint32) - 1
    ve = np.array(t["vextra"])
    fe = np.array(t["fextra1"], dtype=np.uint32) - 1
    n = v / np.linalg.norm(v[0])
    return v, f, ve, fe, n


def check_visibility_box(vis_fn, t):
    """The five asserts of tests/test_visibility.py:13-53 against a visibility_compute-like callable."""
    v, f, ve, fe, n = visibility_cases(t)
    vis, _ = vis_fn(v=v, f=f, cams=np.array([[1.0, 0.0, 0.0]]))
    assert ((v.T[0] > 0) == vis).all()
    vis, ndc = vis_fn(v=v, f=f, n=n, cams=np.array([[1e10, 0.0, 0.0]]))
    assert ((v.T[0] > 0) == np.logical_and(vis, ndc > .5)).all()
    vis, _ = vis_fn(v=v, f=f, cams=np.array([[0.0, 1.0, 0.0], [0.0, 0.0, 1.0]]))
    assert ((v.T[1:3] > 0) == vis).all()
    vis, _ = vis_fn(v=v, f=f, cams=np.array([[0.0, 0.0, 10.0]]), extra_v=ve, extra_f=fe)
    assert (np.zeros_like(v.T[0]) == vis).all()
    vis, _ = vis_fn(v=v, f=f, cams=np.array([[0.0, 0.0, 10.0]]), extra_v=ve, extra_f=fe, min_dist=1.0)
    assert ((v.T[2] > 0) == vis).all()


def test_visibility_known_answer(oracle, ref_tests):
    t = ref_tests["test_visibility_box"]

    def fn(v, f, cams, n=None, extra_v=None, extra_f=None, min_dist=1e-3):
        return oracle.brute_visibility(v, f, cams, n=n, extra_v=extra_v, extra_f=extra_f, min_dist=min_dist)

    check_visibility_box(fn, t)


def _tie_tolerant(oracle, v, f, q, face_a, pt_a, face_b, pt_b):
    diag = float(np.linalg.norm(v.max(0) - v.min(0)))
    tri = v[f.astype(np.int64)]
    da = np.sum((pt_a - q) ** 2, axis=1) ** 0.5
    db = np.sum((pt_b - q) ** 2, axis=1) ** 0.5
    same = face_a == face_b
    # identical face: identical construction
    assert (pt_a[same] == pt_b[same]).all()
    # different face: must be an equidistant tie (north_star: |d| <= 1e-9 diag)
    assert np.all(np.abs(da[~same] - db[~same]) <= 1e-9 * diag)
    return int((~same).sum())


def test_cgal_tree_vs_brute_sphere(oracle, meshes):
    v, f = meshes["sphere_v"], meshes["sphere_f"]
    q = W.uniform_in_box(v.min(0), v.max(0), 20000, seed=5)
    cf, cp, cpt = oracle.CgalTree(v, f).nearest(q)
    bf, bp, bpt, _ = oracle.brute_nearest(v, f, q)
    _tie_tolerant(oracle, v, f, q, cf, cpt, bf, bpt)
    assert (cp[cf == bf] == bp[cf == bf]).all()


def test_cgal_tree_vs_brute_on_surface(oracle):
    # queries close to the surface (C2-like), plus exact vertices and edge midpoints (tie-heavy)
    v, f = W.c2_mesh()
    q, _ = W.surface_samples(v, f, 5000, seed=7, sigma=0.005)
    e = 0.5 * (v[f[:200, 0]] + v[f[:200, 1]])
    q = np.vstack([q, v[:300], e])
    cf, _, cpt = oracle.CgalTree(v, f).nearest(q)
    bf, _, bpt, _ = oracle.brute_nearest(v, f, q)
    ties = _tie_tolerant(oracle, v, f, q, cf, cpt, bf, bpt)
    assert ties > 0  # vertices / edge midpoints are shared by several faces


def test_kdtree_golden(oracle, meshes):
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "kdtree.npz"))
    idx, dist = oracle.brute_vertex_nn(meshes["sphere_v"], g["q"])
    assert (idx == g["idx"]).all()
    assert np.allclose(dist, g["dist"], rtol=1e-12, atol=0)


def test_part_codes(oracle):
    a, b, c = np.array([0., 0, 0]), np.array([1., 0, 0]), np.array([0., 1, 0])
    cases = {(0.2, 0.2, 1.0): 0, (0.5, -1.0, 0.3): 1, (1.0, 1.0, -2.0): 2, (-1.0, 0.5, 0.0): 3,
             (-1.0, -1.0, 0.5): 4, (2.0, -0.5, 0.0): 5, (-0.5, 2.0, 1.0): 6}
    for q, want in cases.items():
        pt, part, _ = oracle.point_triangle(q, a, b, c)
        assert part == want, (q, part, want)


def test_degenerate_triangle(oracle):
    # zero-area triangle: nearest point over its closed edges (deliberate; CGAL yields NaN)
    a, b, c = np.array([0., 0, 0]), np.array([1., 0, 0]), np.array([2., 0, 0])
    pt, part, d2 = oracle.point_triangle([0.5, 1.0, 0.0], a, b, c)
    assert np.allclose(pt, [0.5, 0, 0]) and d2 == 1.0 and part in (1, 3)
    pt, part, d2 = oracle.point_triangle([3.0, 0.0, 0.0], a, b, c)
    assert (pt == c).all() and part == 6


def test_tri_tri_symmetric(oracle):
    rng = np.random.default_rng(3)
    for _ in range(300):
        t1, t2 = rng.normal(size=9), rng.normal(size=9)
        assert oracle.tri_tri_overlap(t1, t2) == oracle.tri_tri_overlap(t2, t1)
    # shared vertex touches, coplanar overlap, disjoint
    assert oracle.tri_tri_overlap([0, 0, 0, 1, 0, 0, 0, 1, 0], [0, 0, 0, -1, 0, 0, 0, 0, 1])
    assert oracle.tri_tri_overlap([0, 0, 0, 2, 0, 0, 0, 2, 0], [0.5, 0.5, 0, 3, 0.5, 0, 0.5, 3, 0])
    assert not oracle.tri_tri_overlap([0, 0, 0, 1, 0, 0, 0, 1, 0], [0, 0, 1, 1, 0, 1, 0, 1, 1])


# ---- geometry restatements feeding the path ----
def test_barycentric_known_answer(oracle, ref_tests):
    # tests/test_geometry.py:70-104 (columns are points)
    t = ref_tests["test_barycentric"]
    p, q, u, v, b = (np.array(t[k], dtype=np.float64).T for k in ("p", "q", "u", "v", "b"))
    est = oracle.barycentric_coordinates_of_projection(p, q, u, v)
    assert np.max(np.abs(est.flatten('F') - b.flatten('F'))) < t["tol"]
    est1 = oracle.barycentric_coordinates_of_projection(p[0], q[0], u[0], v[0])
    assert np.max(np.abs(np.ravel(est1) - b[0])) < t["tol"]


def test_barycentric_reconstructs_projection(oracle):
    rng = np.random.default_rng(5)
    a, e1, e2, p = (rng.normal(size=(200, 3)) for _ in range(4))
    w = oracle.barycentric_coordinates_of_projection(p, a, e1, e2)
    proj = w[:, [0]] * a + w[:, [1]] * (a + e1) + w[:, [2]] * (a + e2)
    n = np.cross(e1, e2)
    # p - proj is along the normal: the weights are those of p's orthogonal projection
    assert np.allclose(np.cross(p - proj, n), 0, atol=1e-9)
    assert np.allclose(w.sum(1), 1.0)


def test_vertex_normals_known_answer(oracle, meshes, ref_tests):
    # tests/test_mesh.py:111-118 and tests/test_geometry.py:61-68
    t = ref_tests["test_estimate_vertex_normals"]
    v = meshes[t["mesh"] + "_v"].copy()
    f = meshes[t["mesh"] + "_f"]
    v -= np.mean(v, axis=0)
    rad = np.linalg.norm(v[0])
    vn = oracle.estimate_vertex_normals(v, f)
    assert np.mean(np.sqrt(np.sum((vn - v / rad) ** 2, axis=1))) < t["mse_max"]
    assert np.max(np.abs(oracle.vert_normals(v, f) - vn)) < ref_tests["test_vert_normals"]["tol"]


def test_alongnormal_point_is_cgal_plane_line(oracle):
    # the oracle's hit point on a proper hit is CGAL's Plane_3/Line_3 construction: it lies on the
    # face's plane and on the ray's line (to rounding), at distance |hit - p|
    v, f = W.geodesic_icosphere(6)
    p, fi = W.surface_samples(v, f, 400, seed=21, sigma=0.05)
    n = np.random.default_rng(22).normal(size=p.shape)
    d, face, pt = oracle.brute_alongnormal(v, f, p, n)
    hit = d < 1e100
    assert hit.mean() > 0.5
    tri = v[f[face[hit]].astype(np.int64)]
    nrm = np.cross(tri[:, 1] - tri[:, 0], tri[:, 2] - tri[:, 0])
    nrm /= np.linalg.norm(nrm, axis=1)[:, None]
    assert np.abs(np.sum((pt[hit] - tri[:, 0]) * nrm, axis=1)).max() < 1e-12
    assert np.allclose(d[hit], np.linalg.norm(pt[hit] - p[hit], axis=1), rtol=0, atol=0)
    off = np.cross(pt[hit] - p[hit], n[hit]) / np.linalg.norm(n[hit], axis=1)[:, None]
    assert np.abs(off).max() < 1e-12


def test_cgal_tree_alongnormal_vs_brute(oracle):
    # the tree traversal (all_intersections of both rays, first minimum) finds the same nearest hit
    # as the exhaustive scan: equal distance everywhere, equal face and point unless two faces tie
    v, f = W.geodesic_icosphere(8)
    p, _ = W.surface_samples(v, f, 3000, seed=23, sigma=0.05)
    n = np.random.default_rng(24).normal(size=p.shape)
    p = np.vstack([p, [[5.0, 5.0, 5.0]]])  # misses both ways
    n = np.vstack([n, [[1.0, 0.0, 0.0]]])
    td, tf, tpt = oracle.CgalTree(v, f, hint=False).alongnormal(p, n)
    bd, bf, bpt = oracle.brute_alongnormal(v, f, p, n)
    assert (td == bd).all()
    same = tf == bf
    assert same.mean() > 0.99
    assert np.array_equal(tpt[same], bpt[same], equal_nan=True)
    assert td[-1] == 1e100 and tf[-1] == 0xFFFFFFFF


def test_cgal_tree_visibility_vs_brute(oracle, ref_tests):
    # any-hit through the tree == exhaustive any-hit, bit for bit, with extra triangles and sensors
    v, f = W.geodesic_icosphere(8)
    v = v * (1.0 + 0.1 * np.sin(5 * v[:, :1]) * np.sin(4 * v[:, 1:2]))
    cams = W.fibonacci_cameras(5, 3.0)
    nrm = v / np.linalg.norm(v, axis=1)[:, None]
    ev = np.array([[1.5, -0.3, -0.3], [1.5, 0.3, -0.3], [1.5, 0.0, 0.4]])
    ef = np.array([[0, 1, 2]], np.uint32)
    sens = np.tile([0.5, 0, 0, 0, 0.5, 0, 0, 0, 1.0], (cams.shape[0], 1))
    for kw in ({}, dict(extra_v=ev, extra_f=ef), dict(sensors=sens, min_dist=0.01)):
        tree = oracle.CgalVisibilityTree(v, f, kw.get("extra_v"), kw.get("extra_f"))
        tv, tn = tree.visibility(cams, n=nrm, sensors=kw.get("sensors"), min_dist=kw.get("min_dist", 1e-3))
        bv, bn = oracle.brute_visibility(v, f, cams, n=nrm, **kw)
        assert (tv == bv).all() and (tn == bn).all()
        assert 0.01 < tv.mean() < 0.9

    t = ref_tests["test_visibility_box"]

    def fn(v, f, cams, n=None, extra_v=None, extra_f=None, min_dist=1e-3):
        return oracle.CgalVisibilityTree(v, f, extra_v, extra_f).visibility(cams, n=n, min_dist=min_dist)

    check_visibility_box(fn, t)


def test_facade_barycentric_spacing_constant(oracle):
    # Mesh.barycentric_coordinates_for_points (numpy facade) substitutes numpy.spacing(1) for s == 0, as
    # barycentric_coordinates_of_projection.py:38-41 does: a triangle with edges ~1e-85 has n != 0 but
    # n.n == 0, and its weights for an O(1) point depend on that constant
    from mesh_amd.mesh import Mesh
    v = np.array([[0, 0, 2.0], [1e-85, 0, 2.0], [0, 1e-85, 2.0], [1.0, 0, 0], [0, 1, 0], [0, 0, 1.0]])
    f = np.array([[0, 1, 2], [3, 4, 5]], np.uint32)
    pts = np.random.default_rng(36).normal(0, 1, (8, 3))
    faces = np.array([0, 1] * 4, np.uint32)
    vi, w = Mesh(v=v, f=f).barycentric_coordinates_for_points(pts, faces)
    bvi, bw = oracle.barycentric_coordinates_for_points(v, f, pts, faces)
    assert np.array_equal(vi, bvi) and np.array_equal(w, bw)
    assert np.abs(w[0::2, 1:]).max() > 0
