"""GPU parity of the geometry that feeds and consumes the search path.

* fused barycentrics: ``aabbtree_nearest_barycentric`` / ``AabbTreeBatch.nearest_barycentric`` return the
  closest face and point (bit-exact vs the exhaustive oracle) plus Heidrich weights that must equal the
  oracle's numpy restatement of ``Mesh.barycentric_coordinates_for_points`` (mesh.py:218-222,
  geometry/barycentric_coordinates_of_projection.py:9-49) applied to that face and point, bit for bit.
  The restatement itself is pinned by tests/test_geometry.py:70-104's known answers (test_oracle.py).
* vertex normals: ``Mesh.estimate_vertex_normals`` (GPU) must equal the scipy-sparse restatement of
  mesh.py:208-216 bit for bit, and meet tests/test_mesh.py:111-118 / test_geometry.py:61-68.
* transfer_segm: ``Mesh.transfer_segm`` (GPU closest faces of the face centres) must give the same part
  lists as the reference's loop (mesh.py:224-237, restated in the oracle) on exhaustive closest faces.
"""
import numpy as np
import pytest

import workloads as W

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _device():
    from mesh_amd import _native
    _native.set_device(0)


def _check_bary(oracle, v, f, q, skip_faces=()):
    from mesh_amd import spatialsearch
    t = spatialsearch.aabbtree_compute(np.ascontiguousarray(v, np.float64), np.ascontiguousarray(f, np.uint32))
    face, pt, w = spatialsearch.aabbtree_nearest_barycentric(t, q)
    assert face.shape == (q.shape[0],) and face.dtype == np.uint32
    assert pt.shape == w.shape == (q.shape[0], 3) and w.dtype == np.float64
    bf, _, bpt, _ = oracle.brute_nearest(v, f, q)
    assert np.array_equal(face, bf)
    assert np.array_equal(pt, bpt)
    vi, bw = oracle.barycentric_coordinates_for_points(v, f, pt, face)
    assert np.array_equal(w, bw), np.abs(w - bw).max()
    # the point lies in its triangle: weights reconstruct it and are (nearly) a convex combination
    # (not for zero-area faces, whose Heidrich weights are (1, 0, 0) for any point)
    keep = ~np.isin(face, np.asarray(skip_faces, np.uint32))
    rec = np.einsum("sk,skd->sd", w[keep], v[vi[keep].astype(np.int64)])
    diag = float(np.linalg.norm(v.max(0) - v.min(0)))
    assert np.abs(rec - pt[keep]).max() < 1e-9 * diag
    assert w[keep].min() > -1e-6 and abs(w[keep].sum(1) - 1).max() < 1e-9
    # the same faces/points as the plain nearest call
    f2, _, p2 = spatialsearch.aabbtree_nearest(t, q)
    assert np.array_equal(f2[0], face) and np.array_equal(p2, pt)
    return face, pt, w


def test_barycentric_sphere(oracle, meshes):
    v, f = meshes["sphere_v"], meshes["sphere_f"]
    _check_bary(oracle, v, f, W.c1_queries(20000))


def test_barycentric_near_surface(oracle):
    v, f = W.c2_mesh()
    q, _ = W.surface_samples(v, f, 20000, seed=31, sigma=0.01)
    _check_bary(oracle, v, f, q)


def test_barycentric_landmarks_flow(oracle, ref_tests):
    # landmarks.py:58-63: closest_faces_and_points then barycentric_coordinates_for_points
    from mesh_amd.mesh import Mesh
    t = ref_tests["test_aabb_tree"]
    v, f = np.array(t["v"], dtype=np.float64), np.array(t["f"], dtype=np.uint32)
    q = np.array(t["q"], dtype=np.float64)
    m = Mesh(v=v, f=f)
    faces, pts = m.closest_faces_and_points(q)
    vi, coeff = m.barycentric_coordinates_for_points(pts, faces)
    face, pt, w = _check_bary(oracle, v, f, q)
    assert np.array_equal(face, faces[0]) and np.array_equal(vi, f[face])
    assert np.array_equal(w, coeff)


def test_barycentric_device_and_nonfinite(oracle):
    import torch
    from mesh_amd import spatialsearch
    from mesh_amd.distributed import nearest_bary_device
    v, f = W.geodesic_icosphere(20)
    q = W.uniform_in_box([-1.1] * 3, [1.1] * 3, 50000, seed=32, margin=0)
    q[7] = [np.nan, 0, 0]
    t = spatialsearch.aabbtree_compute(v, f)
    face, pt, w = spatialsearch.aabbtree_nearest_barycentric(t, q)
    assert face[7] == 0xFFFFFFFF and np.isnan(pt[7]).all() and np.isnan(w[7]).all()
    dq = torch.from_numpy(q).cuda()
    dface = torch.empty(q.shape[0], dtype=torch.int32, device="cuda")
    dpt = torch.empty_like(dq)
    dw = torch.empty_like(dq)
    nearest_bary_device(t, dq, dface, dpt, dw)
    torch.cuda.synchronize()
    assert np.array_equal(dface.cpu().numpy().view(np.uint32), face)
    assert np.array_equal(dpt.cpu().numpy(), pt, equal_nan=True)
    assert np.array_equal(dw.cpu().numpy(), w, equal_nan=True)


def test_batch_barycentric(oracle):
    from mesh_amd.search import AabbTreeBatch
    v, f, q = W.c4_batch(B=6, S=3000, seed=33)
    bt = AabbTreeBatch(v, f)
    face, pt, w = bt.nearest_barycentric(q)
    assert face.shape == (6, 3000) and pt.shape == w.shape == (6, 3000, 3)
    for b in range(6):
        bf, _, bpt, _ = oracle.brute_nearest(v[b], f, q[b])
        assert np.array_equal(face[b], bf) and np.array_equal(pt[b], bpt)
        _, bw = oracle.barycentric_coordinates_for_points(v[b], f, pt[b], face[b])
        assert np.array_equal(w[b], bw)


# ---------------------------------------------------------------- vertex normals
def test_vertex_normals_known_answer(meshes, ref_tests):
    from mesh_amd.mesh import Mesh
    t = ref_tests["test_estimate_vertex_normals"]
    m = Mesh(v=meshes[t["mesh"] + "_v"], f=meshes[t["mesh"] + "_f"])
    m.v -= np.mean(m.v, axis=0)
    rad = np.linalg.norm(m.v[0])
    vn = np.array(m.estimate_vertex_normals())
    assert np.mean(np.sqrt(np.sum((vn - m.v / rad) ** 2, axis=1))) < t["mse_max"]


@pytest.mark.parametrize("name", ["sphere", "c2", "bumpy", "degenerate"])
def test_vertex_normals_bit_exact(oracle, meshes, ref_tests, name):
    from mesh_amd.mesh import Mesh
    if name == "sphere":
        v, f = meshes["sphere_v"], meshes["sphere_f"]
    elif name == "c2":
        v, f = W.c2_mesh()
    elif name == "bumpy":
        v, f = W.geodesic_icosphere(60)
        v = v * (1 + 0.1 * np.sin(7 * v[:, [0]]) * np.cos(5 * v[:, [1]]))
    else:
        # an isolated vertex (zero norm -> 1 -> a zero normal) and a zero-area face
        v, f = W.geodesic_icosphere(3)
        v = np.vstack([v, [[5.0, 5.0, 5.0]]])
        f = np.vstack([f, [[0, 1, 1]]]).astype(np.uint32)
    vn = Mesh(v=v, f=f).estimate_vertex_normals()
    ref = oracle.estimate_vertex_normals(v, f)
    assert np.array_equal(vn, ref), np.abs(vn - ref).max()
    assert np.max(np.abs(oracle.vert_normals(v, f) - vn)) < ref_tests["test_vert_normals"]["tol"]


def test_vertex_normals_c5_size(oracle):
    # 5M faces / 2.5M vertices (the C5 mesh feeding visibility_compute): bit-exact on the whole mesh
    from mesh_amd.mesh import Mesh
    v, f = W.c5_mesh()
    vn = Mesh(v=v, f=f).estimate_vertex_normals()
    ref = oracle.estimate_vertex_normals(v, f)
    assert np.array_equal(vn, ref)


# ---------------------------------------------------------------- transfer_segm
@pytest.mark.parametrize("exclude", [True, False])
def test_transfer_segm(oracle, exclude):
    from mesh_amd.mesh import Mesh
    # source mesh: C2 stand-in with a segmentation by height band (one empty part); target: a finer
    # noisy sphere around it
    v, f = W.c2_mesh()
    src = Mesh(v=v, f=f)
    zc = (v[f[:, 0], 2] + v[f[:, 1], 2] + v[f[:, 2], 2]) / 3.0
    bands = np.digitize(zc, np.quantile(zc, [0.2, 0.5, 0.8]))
    src.segm = {"feet": np.nonzero(bands == 0)[0].tolist(), "legs": np.nonzero(bands == 1)[0].tolist(),
                "torso": np.nonzero(bands == 2)[0].tolist(), "head": np.nonzero(bands == 3)[0].tolist(),
                "nothing": []}
    tv, tf = W.geodesic_icosphere(30)
    tv = tv * np.array([0.6, 1.7, 0.3]) * 1.01
    tgt = Mesh(v=tv, f=tf)
    tgt.transfer_segm(src, exclude_empty_parts=exclude)
    centres = oracle.face_centres(tv, tf)
    bf, _, _, _ = oracle.brute_nearest(v, f, centres)
    want = oracle.transfer_segm(tv, tf, src.segm, bf, exclude_empty_parts=exclude)
    assert list(tgt.segm.keys()) == list(want.keys())
    for k in want:
        assert tgt.segm[k] == want[k], k
    assert ("nothing" in tgt.segm) == (not exclude)


def _degenerate_mesh():
    # an icosphere plus zero-area faces: collinear vertices, a repeated vertex, and a tiny triangle whose
    # n.n underflows to 0 although n != 0 (edges ~1e-85), so the s == 0 -> numpy.spacing(1) substitution
    # of barycentric_coordinates_of_projection.py:38-41 decides the weights
    v, f = W.geodesic_icosphere(6)
    P = v.shape[0]
    extra_v = np.array([[2.0, 0, 0], [2.5, 0, 0], [3.0, 0, 0],          # collinear
                        [0, 2.0, 0], [0, 2.5, 0.5],                     # repeated vertex
                        [0, 0, 2.0], [1e-85, 0, 2.0], [0, 1e-85, 2.0]])  # n.n underflows
    extra_f = np.array([[P, P + 1, P + 2], [P + 3, P + 3, P + 4], [P + 5, P + 6, P + 7]], np.uint32)
    return np.vstack([v, extra_v]), np.vstack([f, extra_f]).astype(np.uint32), P


def test_barycentric_zero_area_faces(oracle):
    from mesh_amd.mesh import Mesh
    v, f, P = _degenerate_mesh()
    T0 = f.shape[0] - 3
    rng = np.random.default_rng(34)
    q = np.vstack([rng.normal([2.5, 0, 0], 0.3, (3000, 3)), rng.normal([0, 2.2, 0.2], 0.2, (3000, 3)),
                   rng.normal([0, 0, 2.0], 0.05, (3000, 3)), W.uniform_in_box([-1.1] * 3, [1.1] * 3, 3000, 35, 0)])
    face, pt, w = _check_bary(oracle, v, f, q, skip_faces=[T0, T0 + 1, T0 + 2])
    assert np.isin(face, [T0, T0 + 1, T0 + 2]).sum() > 1000  # the zero-area faces are really hit
    # the facade (numpy) on the same faces and points, and on arbitrary points, where the tiny face's
    # underflowed s matters (w = p - a is O(1), so (u x w).n does not underflow)
    m = Mesh(v=v, f=f)
    vi, coeff = m.barycentric_coordinates_for_points(pt, face)
    assert np.array_equal(coeff, w)
    faces = np.array([T0, T0 + 1, T0 + 2] * 5, np.uint32)
    pts = rng.normal(0, 1, (faces.size, 3))
    vi, coeff = m.barycentric_coordinates_for_points(pts, faces)
    _, bw = oracle.barycentric_coordinates_for_points(v, f, pts, faces)
    assert np.array_equal(coeff, bw)
    assert np.abs(coeff[2::3, 1:]).max() > 0  # the tiny face's weights are not all zero


def test_transfer_segm_empty_named_part(oracle):
    # a part named '' (the OBJ reader makes one for a bare 'g' line): faces of `mesh` in no part map to it
    # (parts_by_face gives them ''), as in the reference's loop (mesh.py:224-237); without it, KeyError('')
    from mesh_amd.mesh import Mesh
    v, f = W.geodesic_icosphere(8)
    src = Mesh(v=v, f=f)
    src.segm = {"a": list(range(0, 300)), "": list(range(300, 400))}  # faces >= 400 in no part
    tv, tf = W.geodesic_icosphere(5)
    tgt = Mesh(v=tv * 1.02, f=tf)
    tgt.transfer_segm(src)
    bf, _, _, _ = oracle.brute_nearest(v, f, oracle.face_centres(tv * 1.02, tf))
    want = oracle.transfer_segm(tv * 1.02, tf, src.segm, bf)
    assert tgt.segm == want and len(want[""]) > 0
    del src.segm[""]
    with pytest.raises(KeyError):
        Mesh(v=tv * 1.02, f=tf).transfer_segm(src)


def test_vertex_normals_device_bad_index():
    # msh_vertex_normals_device gets device faces it cannot check on the host: an index >= P is found on the
    # device and reported as MSH_EINVAL (no out-of-bounds read of v, no write past the range buffer)
    import torch
    from mesh_amd import _native as N
    v, f = W.geodesic_icosphere(4)
    f = f.copy()
    f[5, 1] = v.shape[0] + 7
    dv = torch.from_numpy(v).cuda()
    df = torch.from_numpy(f.view(np.int32)).cuda()
    dn = torch.empty_like(dv)
    st = N.lib().msh_vertex_normals_device(dv.data_ptr(), v.shape[0], df.data_ptr(), f.shape[0], dn.data_ptr(),
                                           torch.cuda.current_stream().cuda_stream)
    assert st == N.MSH_EINVAL and b"out of range" in N.lib().msh_last_error()
    f[5, 1] = 0  # a valid mesh on the same buffers still works
    df.copy_(torch.from_numpy(f.view(np.int32)))
    st = N.lib().msh_vertex_normals_device(dv.data_ptr(), v.shape[0], df.data_ptr(), f.shape[0], dn.data_ptr(),
                                           torch.cuda.current_stream().cuda_stream)
    assert st == 0
