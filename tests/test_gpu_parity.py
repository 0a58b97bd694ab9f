"""Parity of the HIP path (through the C ABI) with the oracle and the reference's known answers.

Bar (BASELINE.json north_star): closest face identical except at equidistant ties
(|Δd| <= 1e-9 x bbox diagonal), closest point within 1e-6 x bbox diagonal.  Against the exhaustive
oracle with the same tie rule (lexicographic min of (d², face)) and the same CGAL construction, the
HIP results are required to be BIT-EXACT (face, part code and point); against the CGAL-tree
restatement (whose tie rule is traversal order) they are compared tie-tolerantly.
"""
import os

import numpy as np
import pytest

import workloads as W
from tests.test_oracle import check_visibility_box, cylinder_query

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _device():
    from mesh_amd import _native
    _native.set_device(0)


def _nearest(v, f, q):
    from mesh_amd import spatialsearch
    t = spatialsearch.aabbtree_compute(np.ascontiguousarray(v, np.float64), np.ascontiguousarray(f, np.uint32))
    face, part, pt = spatialsearch.aabbtree_nearest(t, np.ascontiguousarray(q, np.float64))
    assert face.shape == (1, q.shape[0]) and face.dtype == np.uint32
    assert part.shape == (1, q.shape[0]) and part.dtype == np.uint32
    assert pt.shape == (q.shape[0], 3) and pt.dtype == np.float64
    return face[0], part[0], pt


def _assert_bit_exact_vs_brute(oracle, v, f, q):
    face, part, pt = _nearest(v, f, q)
    bf, bp, bpt, _ = oracle.brute_nearest(v, f, q)
    assert np.array_equal(face, bf), "faces differ at %s" % np.nonzero(face != bf)[0][:10]
    assert np.array_equal(part, bp)
    assert np.array_equal(pt, bpt)
    return face, part, pt


# ---------------------------------------------------------------- reference known answers
def test_aabb_tree_known_answer(ref_tests):
    from mesh_amd.mesh import Mesh
    t = ref_tests["test_aabb_tree"]
    m = Mesh(v=np.array(t["v"]), f=np.array(t["f"]))
    f_est, v_est = m.compute_aabb_tree().nearest(np.array(t["q"]))
    assert max(abs(f_est - np.array(t["f_expected"])).flatten()) < 1e-6
    assert max(abs(v_est - np.array(t["v_expected"])).flatten()) < 1e-6


@pytest.mark.parametrize("name", ["test_dist_classic", "test_dist_normals"])
def test_normals_known_answer(meshes, ref_tests, name):
    from mesh_amd import aabb_normals
    t = ref_tests[name]
    v, f = meshes[t["mesh"] + "_v"], meshes[t["mesh"] + "_f"]
    h = aabb_normals.aabbtree_n_compute(v, f.astype(np.uint32).copy(), t["eps"])
    tri, p = aabb_normals.aabbtree_n_nearest(h, np.array(t["q"]), np.array(t["n"]))
    assert (tri == np.array(t["f_expected"])).all()
    assert (p == np.array(t["p_expected"])).all()


def test_cylinders_known_answer(meshes, ref_tests):
    from mesh_amd import aabb_normals
    t = ref_tests["test_cylinders"]
    v, f = meshes["cylinder_v"], meshes["cylinder_f"]
    q, qn = cylinder_query(meshes)
    a, _ = aabb_normals.aabbtree_n_nearest(aabb_normals.aabbtree_n_compute(v, f, t["eps_no"]), q, qn)
    b, _ = aabb_normals.aabbtree_n_nearest(aabb_normals.aabbtree_n_compute(v, f, t["eps_yes"]), q, qn)
    assert np.unique(a).shape[0] <= t["max_unique_no"]
    assert np.unique(b).shape[0] >= f.shape[0] - t["min_unique_yes_slack"]


def test_selfintersects_known_answer(meshes, ref_tests):
    from mesh_amd import aabb_normals
    for name, want in ref_tests["test_selfintersects"].items():
        h = aabb_normals.aabbtree_n_compute(meshes[name + "_v"], meshes[name + "_f"], 0.5)
        assert aabb_normals.aabbtree_n_selfintersects(h) == want


def test_visibility_known_answer(ref_tests):
    from mesh_amd.visibility import visibility_compute
    check_visibility_box(visibility_compute, ref_tests["test_visibility_box"])


def test_intersections_known_answer(meshes, ref_tests):
    from mesh_amd.mesh import Mesh
    t = ref_tests["test_intersections"]
    v, f = meshes["icosphere_v"], meshes["icosphere_f"]
    qm = Mesh(v=v * t["radius"] + np.array(t["q_center"], float), f=f)
    m = Mesh(v=v * t["radius"] + np.array(t["m_center"], float), f=f)
    got = m.compute_aabb_tree().intersections_indices(qm.v, qm.f)
    assert got.dtype == np.uint32 and got.tolist() == t["expected"]


def test_closest_point_tree_vs_scipy_golden(meshes):
    from mesh_amd.mesh import Mesh
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "kdtree.npz"))
    m = Mesh(v=meshes["sphere_v"], f=meshes["sphere_f"])
    idx, dist = m.closest_vertices(g["q"])
    assert isinstance(idx, tuple) and len(idx) == g["q"].shape[0]
    assert (np.array(idx) == g["idx"]).all()
    assert np.allclose(np.array(dist), g["dist"], rtol=1e-12, atol=0)
    nv = m.compute_closest_point_tree().nearest_vertices(g["q"][:10])
    assert (nv == meshes["sphere_v"][g["idx"][:10]]).all()


# ---------------------------------------------------------------- randomized parity
def test_c1_sphere_bit_exact(oracle, meshes):
    v, f = meshes["sphere_v"], meshes["sphere_f"]
    q = W.c1_queries(100000)
    face, part, pt = _assert_bit_exact_vs_brute(oracle, v, f, q)
    cf, cp, cpt = oracle.CgalTree(v, f).nearest(q)
    diag = float(np.linalg.norm(v.max(0) - v.min(0)))
    same = face == cf
    assert (pt[same] == cpt[same]).all() and (part[same] == cp[same]).all()
    dg = np.linalg.norm(pt - q, axis=1)
    dc = np.linalg.norm(cpt - q, axis=1)
    assert np.all(np.abs(dg - dc) <= 1e-9 * diag)


@pytest.mark.parametrize("leaf_list", ["1", "2", "0"])
def test_c2_near_surface_bit_exact(oracle, monkeypatch, leaf_list):
    # leaf_list 1: the wave leaf list with the LDS node prefetch (trees of <= 2^20 leaves); 2: the list without it
    # (larger trees); 0: the per-lane leaf queues that trees of >= 2^26 leaves use instead of the wave leaf list
    monkeypatch.setenv("MESH_AMD_LEAF_LIST", leaf_list)
    v, f = W.c2_mesh()
    q, _ = W.surface_samples(v, f, 20000, seed=9, sigma=0.01)
    q = np.vstack([q, v[:500], 0.5 * (v[f[:500, 0]] + v[f[:500, 1]])])  # vertex / edge ties
    _assert_bit_exact_vs_brute(oracle, v, f, q)


@pytest.mark.parametrize("leaf_list", ["1", "2", "0"])
def test_non_finite_queries(oracle, monkeypatch, leaf_list):
    # NaN / inf rows (documented deviation: the reference's CGAL call is undefined for them) answer NO_FACE,
    # part 0 and a NaN point; they sit among finite rows of a sorted launch with leader phases (C2 mesh: 13,776
    # faces, 20k queries), so some of them are leaders whose records followers must skip; every finite row
    # still matches brute force bit for bit
    monkeypatch.setenv("MESH_AMD_LEAF_LIST", leaf_list)
    v, f = W.c2_mesh()
    q, _ = W.surface_samples(v, f, 20000, seed=41, sigma=0.01)
    bad = np.random.default_rng(42).choice(q.shape[0], 800, replace=False)
    vals = np.array([np.nan, np.inf, -np.inf])
    q[bad, np.random.default_rng(43).integers(0, 3, bad.shape[0])] = vals[np.arange(bad.shape[0]) % 3]
    q[bad[:8] - bad[:8] % 8] = np.nan  # whole rows at leader slots of the caller's order too
    face, part, pt = _nearest(v, f, q)
    nf = ~np.isfinite(q).all(axis=1)
    assert nf.sum() >= 800
    assert (face[nf] == 0xFFFFFFFF).all() and (part[nf] == 0).all() and np.isnan(pt[nf]).all()
    bf, bp, bpt, _ = oracle.brute_nearest(v, f, q[~nf])
    assert np.array_equal(face[~nf], bf) and np.array_equal(part[~nf], bp) and np.array_equal(pt[~nf], bpt)


def test_c3_sample_both_leaf_paths(oracle, monkeypatch):
    # C3 mesh, 200k uniform queries (leader phases on): the wave leaf list with and without the LDS node prefetch
    # and the per-lane queues give the same arrays, and they match brute force on a 2000-row sample
    v, f = W.c3_mesh()
    q = np.random.default_rng(31).uniform(-1.1, 1.1, (200_000, 3))
    outs = []
    for leaf_list in ("1", "2", "0"):
        monkeypatch.setenv("MESH_AMD_LEAF_LIST", leaf_list)
        outs.append(_nearest(v, f, q))
    for other in outs[1:]:
        for a, b in zip(outs[0], other):
            assert np.array_equal(a, b)
    rows = np.random.default_rng(32).choice(q.shape[0], 2000, replace=False)
    bf, bp, bpt, _ = oracle.brute_nearest(v, f, q[rows])
    assert np.array_equal(outs[0][0][rows], bf) and np.array_equal(outs[0][1][rows], bp)
    assert np.array_equal(outs[0][2][rows], bpt)


def test_pass2_heavy_items_split(oracle):
    # Deferred queries near the sphere's centre, where nearly every face is equidistant, are pass 2's longest walks:
    # k_p2_plan lists those within 3 % of the largest deferred distance, pass 2 splits each over 8 waves that share
    # their bound, and k_knn_combine merges the parts.  30k such rows among 300k uniform ones give the arrays of the
    # same tree with the fine entry cut and without one (leader phases then), and 300 of them match brute force.
    from mesh_amd import spatialsearch
    v, f = W.c3_mesh()
    rng = np.random.default_rng(81)
    d = rng.normal(size=(30_000, 3))
    d /= np.linalg.norm(d, axis=1)[:, None]
    q = np.concatenate([rng.uniform(-1.1, 1.1, (300_000, 3)), d * rng.uniform(0.0, 0.05, (30_000, 1))])
    t = spatialsearch.aabbtree_compute(v, f)
    t.set_entry_cut(-1)
    with_cut = _nearest_tree(t, q)
    t.set_entry_cut(0)
    from_root = _nearest_tree(t, q)
    for a, b in zip(with_cut, from_root):
        assert np.array_equal(a, b)
    rows = 300_000 + rng.choice(30_000, 300, replace=False)
    bf, bp, bpt, _ = oracle.brute_nearest(v, f, q[rows])
    assert np.array_equal(with_cut[0][rows], bf) and np.array_equal(with_cut[1][rows], bp)
    assert np.array_equal(with_cut[2][rows], bpt)


def test_workspace_handoff_between_trees(oracle, meshes):
    # a freed triangle tree hands its query workspace to the next tree built on the device (api.cpp WsPool), as
    # a tree per call (Mesh.closest_faces_and_points) does: trees built and freed in turn on two meshes answer
    # the same arrays every round, and match brute force
    import gc
    vs, fs = meshes["sphere_v"], meshes["sphere_f"]
    v2, f2 = W.c2_mesh()
    qs = W.c1_queries(50000)
    q2, _ = W.surface_samples(v2, f2, 300000, seed=52, sigma=0.01)  # > kSortMin rows: the sorted path
    rounds = []
    for _ in range(2):
        a = _nearest(v2, f2, q2)
        gc.collect()
        b = _nearest(vs, fs, qs)
        gc.collect()
        rounds.append((a, b))
    for x, y in zip(rounds[0][0] + rounds[0][1], rounds[1][0] + rounds[1][1]):
        assert np.array_equal(x, y)
    bf, bp, bpt, _ = oracle.brute_nearest(vs, fs, qs)
    assert np.array_equal(rounds[1][1][0], bf) and np.array_equal(rounds[1][1][2], bpt)
    rows = np.random.default_rng(53).choice(q2.shape[0], 2000, replace=False)
    bf, bp, bpt, _ = oracle.brute_nearest(v2, f2, q2[rows])
    assert np.array_equal(rounds[1][0][0][rows], bf) and np.array_equal(rounds[1][0][2][rows], bpt)


def _nearest_tree(t, q):
    from mesh_amd import spatialsearch
    face, part, pt = spatialsearch.aabbtree_nearest(t, np.ascontiguousarray(q, np.float64))
    return face[0], part[0], pt


def test_entry_cut_bit_exact(oracle, monkeypatch):
    # C3 mesh: walks from the entry cut give the arrays of walks from the root (msh_tree_set_entry_cut(0)) -- the
    # fine automatic grid (G = 400, 32-B records of 4-B entries), a 64^3 and an 8^3 grid, and the fine grid read by
    # the list path without the node prefetch (8-B stack entries: MESH_AMD_LEAF_LIST=2) --
    # on uniform queries reaching past the grid (+-1.25 around the unit sphere), near-surface queries and queries on
    # cell faces of the default grid; 2000 rows match brute force
    from mesh_amd import spatialsearch
    v, f = W.c3_mesh()
    rng = np.random.default_rng(41)
    G = int(round(np.cbrt(min(64 * f.shape[0], 1 << 26))))  # api.cpp cut_grid: the fine automatic grid
    assert G == 400
    lo, w = -1.25, 2.5 / G  # scene box +-1 (icosphere vertices on the unit sphere), widened by 1/4
    on_faces = rng.uniform(-1.2, 1.2, (20_000, 3))
    on_faces[np.arange(20_000), rng.integers(0, 3, 20_000)] = lo + rng.integers(0, G + 1, 20_000) * w
    surf, _ = W.surface_samples(v, f, 50_000, seed=42, sigma=0.003)
    q = np.concatenate([rng.uniform(-1.4, 1.4, (150_000, 3)), surf, on_faces])
    t = spatialsearch.aabbtree_compute(v, f)
    outs = []
    for g in (0, -1, 64, 8):
        t.set_entry_cut(g)
        outs.append(_nearest_tree(t, q))
        info = t.entry_cut_info()
        assert info["state"] == ("off" if g == 0 else "built"), info
        assert info["G"] == (0 if g == 0 else (G if g < 0 else g))
        assert info["bytes"] == info["G"] ** 3 * 32
    t.set_entry_cut(-1)
    monkeypatch.setenv("MESH_AMD_LEAF_LIST", "2")
    outs.append(_nearest_tree(t, q))
    monkeypatch.delenv("MESH_AMD_LEAF_LIST")
    for o in outs[1:]:
        for a, b in zip(outs[0], o):
            assert np.array_equal(a, b)
    rows = rng.choice(q.shape[0], 2000, replace=False)
    bf, bp, bpt, _ = oracle.brute_nearest(v, f, q[rows])
    assert np.array_equal(outs[1][0][rows], bf) and np.array_equal(outs[1][1][rows], bp)
    assert np.array_equal(outs[1][2][rows], bpt)


def test_entry_cut_wide_records():
    # Trees of more than 2^20 leaves keep 64-B cut records of 8-B entries (the 4-B packing holds 21-bit refs): C5's
    # 5M-face mesh with 24^3 and 96^3 grids gives the arrays of walks from the root
    from mesh_amd import spatialsearch
    v, f = W.c5_mesh()
    rng = np.random.default_rng(43)
    surf, _ = W.surface_samples(v, f, 60_000, seed=44, sigma=0.01)
    q = np.concatenate([rng.uniform(-1.5, 1.5, (60_000, 3)), surf])
    t = spatialsearch.aabbtree_compute(v, f)
    t.set_entry_cut(0)
    ref = _nearest_tree(t, q)
    for g in (24, 96):
        t.set_entry_cut(g)
        got = _nearest_tree(t, q)
        info = t.entry_cut_info()
        assert info["state"] == "built" and info["G"] == g and info["bytes"] == g ** 3 * 64, info
        for a, b in zip(ref, got):
            assert np.array_equal(a, b)


def test_entry_cut_lazy_and_failure_fallback(oracle):
    # The automatic cut comes in two sizes: the coarse grid (8 cells per face: C2 48^3) is built by the closest-point
    # or alongnormal call that brings the handle's rows to one per 16 of its cells (6,888), never by the build, by
    # visibility or by the normals metric; the fine one (64 per face: 96^3) after 16 rows per fine cell, or at the next call after
    # set_entry_cut(-1) (a kept tree); a requested grid is built by the next call whatever its size; a cut that cannot
    # be built (here 4096^3 cells: more than one query call holds) is not an error: the handle records the failure and
    # its queries start at the root with the same answers.
    from mesh_amd import aabb_normals, spatialsearch
    v, f = W.c2_mesh()  # 13,776 faces: above the 4096-face floor
    q, _ = W.surface_samples(v, f, 40000, seed=51, sigma=0.02)
    tref = spatialsearch.aabbtree_compute(v, f)
    tref.set_entry_cut(0)
    ref = _nearest_tree(tref, q)  # walks from the root
    del tref
    t = spatialsearch.aabbtree_compute(v, f)
    assert t.entry_cut_info()["state"] == "pending"
    nrm = np.tile([[0.0, 0.0, 1.0]], (q.shape[0], 1))
    spatialsearch.aabbtree_nearest_alongnormal(t, q[:3000], nrm[:3000])  # alongnormal rows count too (round 6)
    assert t.entry_cut_info()["state"] == "pending" and t.entry_cut_info()["bytes"] == 0
    _nearest_tree(t, q[:3000])  # 6,000 rows: below the coarse grid's volume, walks from the root
    assert t.entry_cut_info()["state"] == "pending" and t.entry_cut_info()["bytes"] == 0
    again = _nearest_tree(t, q)  # 46,000 rows in all: the coarse grid is built by this call
    info = t.entry_cut_info()
    assert info["state"] == "built" and info["G"] == 48 and info["bytes"] == 48 ** 3 * 32 and info["build_ms"] > 0
    for a, b in zip(ref, again):
        assert np.array_equal(a, b)
    t.set_entry_cut(-1)  # a kept tree asks for the fine grid: built by the next call
    again = _nearest_tree(t, q)
    info = t.entry_cut_info()
    assert info["state"] == "built" and info["G"] == 96 and info["bytes"] == 96 ** 3 * 32
    for a, b in zip(ref, again):
        assert np.array_equal(a, b)
    t.set_entry_cut(4096)
    got = _nearest_tree(t, q)
    info = t.entry_cut_info()
    assert info["state"] == "failed" and info["bytes"] == 0 and info["G"] == 0
    for a, b in zip(ref, got):
        assert np.array_equal(a, b)
    bf, bp, bpt, _ = oracle.brute_nearest(v, f, q[:2000])
    assert np.array_equal(got[0][:2000], bf) and np.array_equal(got[1][:2000], bp) and np.array_equal(got[2][:2000], bpt)
    # back to the automatic grid: rebuilt by the next query (an explicit request: whatever its size)
    t.set_entry_cut(-1)
    assert t.entry_cut_info()["state"] == "pending"
    again = _nearest_tree(t, q[:1000])
    assert t.entry_cut_info()["state"] == "built" and t.entry_cut_info()["G"] == 96
    again = _nearest_tree(t, q)
    for a, b in zip(ref, again):
        assert np.array_equal(a, b)
    h = aabb_normals.aabbtree_n_compute(v, f, 0.1)
    aabb_normals.aabbtree_n_nearest(h, q, nrm)
    assert h.entry_cut_info()["state"] == "off" and h.entry_cut_info()["bytes"] == 0
    with pytest.raises(ValueError):
        t.set_entry_cut(5000)


def test_entry_cut_rebuild_memory_flat():
    # Rebuilding the entry cut (set_entry_cut(-1) then a query) frees its build temporaries (~420 MB of cell-centre
    # queries and answers on C3): device memory is flat across cycles.  msh_device_pool_trim then frees the idle
    # query workspace a freed tree leaves to the next one (api.cpp WsPool).
    import gc
    import torch
    from mesh_amd import _native as N, spatialsearch
    v, f = W.c3_mesh()
    q = W.uniform_in_box(v.min(0), v.max(0), 50_000, seed=61)
    t = spatialsearch.aabbtree_compute(v, f)
    ref = _nearest_tree(t, q)
    free = []
    for _ in range(4):
        t.set_entry_cut(-1)
        got = _nearest_tree(t, q)
        assert t.entry_cut_info()["state"] == "built"
        for a, b in zip(ref, got):
            assert np.array_equal(a, b)
        free.append(torch.cuda.mem_get_info(0)[0])
    assert max(free) - min(free) < (64 << 20), free
    del t
    gc.collect()
    ws, _, cached = N.device_pool_bytes()
    assert ws > 0  # the freed tree's workspace waits for the next tree
    before = torch.cuda.mem_get_info(0)[0]
    N.device_pool_trim()
    assert N.device_pool_bytes() == (0, 0, 0)
    assert torch.cuda.mem_get_info(0)[0] >= before + ws + cached - (16 << 20)


def test_c3_replication_roundtrip():
    # north_star's replication path on one GPU: the C3 tree packed into one device blob (what rank 0
    # broadcasts), unpacked on the same device (what every other rank does), answers the C3 stream bit for
    # bit like the source handle; the receiver builds its own entry cut on its first query (5M rows: above the
    # coarse automatic grid's volume, 1 row per 16 of its 8M cells)
    import torch
    from mesh_amd import _native, spatialsearch
    from mesh_amd.distributed import nearest_device
    v, f = W.c3_mesh()
    src = spatialsearch.aabbtree_compute(v, f)
    blob = torch.empty(_native.blob_size(src), dtype=torch.uint8, device="cuda:0")
    _native.blob_pack(src, blob.data_ptr())
    torch.cuda.synchronize()
    dst = _native.blob_unpack(blob.data_ptr(), blob.numel(), 0)
    del blob
    assert dst.entry_cut_info()["state"] == "pending"
    a, b = src.info(), dst.info()
    for k in ("n_points", "n_faces", "n_nodes", "bytes", "max_depth", "node_bytes", "leaf_bytes"):
        assert getattr(a, k) == getattr(b, k), k
    q = W.c3_stream(5_000_000, "cuda:0")
    outs = []
    for t in (src, dst):
        o = (torch.empty(q.shape[0], dtype=torch.int32, device="cuda:0"),
             torch.empty(q.shape[0], dtype=torch.int32, device="cuda:0"),
             torch.empty((q.shape[0], 3), dtype=torch.float64, device="cuda:0"))
        nearest_device(t, q, *o)
        outs.append(o)
    torch.cuda.synchronize()
    assert dst.entry_cut_info()["state"] == "built"
    assert dst.entry_cut_info()["G"] == src.entry_cut_info()["G"]
    for x, y in zip(*outs):
        assert torch.equal(x, y)


def test_query_order_equals_stable_argsort():
    # the closest-point path's query order (msh_tree_query_order: Hilbert indices of the 24-bit Morton cells + the
    # 3-pass LDS radix sort) equals numpy's stable argsort of the same keys (scripts/sort_debug.order_keys, the kernel's
    # fp32 arithmetic): on the C3 stream (100M rows), a ragged size, a size below one tile, rows with NaN / inf, and the
    # sizes around the scan forms (8192-key tiles: 131,073 rows = 2 chunk sums and 16,777,216 = 128, both scanned in
    # the scatter blocks; 16,777,217 = 129, the recursive scan)
    import torch
    from mesh_amd import _native, spatialsearch
    from scripts.sort_debug import order_keys, sort_box
    v, f = W.c3_mesh()
    t = spatialsearch.aabbtree_compute(v, f)
    lo, hi = sort_box(t.info())
    q = W.c3_stream(100_000_000, "cuda:0")
    bad = W.c3_stream(50_000, "cuda:0", seed=7)
    bad[::7, 0] = float("nan")
    bad[3::11, 2] = float("inf")
    for x in (q, q[:12_345_677], q[:1000], bad, q[:131_073], q[:16_777_216], q[:16_777_217]):
        p = torch.empty(x.shape[0], dtype=torch.int32, device="cuda:0")
        # on torch's stream: the rows come from torch's generator, whose kernels the tree's own (non-blocking)
        # stream would not wait for
        _native.check(_native.lib().msh_tree_query_order(t.ptr, x.data_ptr(), x.shape[0], p.data_ptr(),
                                                         torch.cuda.current_stream().cuda_stream))
        torch.cuda.synchronize()
        ref = np.argsort(order_keys(x.cpu().numpy(), lo, hi), kind="stable")
        assert np.array_equal(p.cpu().numpy().astype(np.int64), ref), "rows %d" % x.shape[0]


def test_c3_stream_shards_equal_whole():
    # BASELINE configs[2] sharded as bench.py does for N = 8, on one GPU: each of the 8 contiguous shards of the
    # 100M-query C3 stream answered by its own call (its own Morton sort, leader phases, entry cut walks and
    # pass 2 at 12.5M queries) gives exactly the rows of the answer of the whole stream
    import torch
    from mesh_amd import spatialsearch
    from mesh_amd.distributed import nearest_device
    v, f = W.c3_mesh()
    t = spatialsearch.aabbtree_compute(v, f)
    S = 100_000_000
    q = W.c3_stream(S, "cuda:0")

    def slab(n):
        return (torch.empty(n, dtype=torch.int32, device="cuda:0"), torch.empty(n, dtype=torch.int32, device="cuda:0"),
                torch.empty((n, 3), dtype=torch.float64, device="cuda:0"))

    whole, parts = slab(S), slab(S)
    nearest_device(t, q, *whole)
    for r in range(8):
        qs, (a, b) = W.c3_shard(q, r, 8)
        nearest_device(t, qs, parts[0][a:b], parts[1][a:b], parts[2][a:b])
    torch.cuda.synchronize()
    for x, y in zip(whole, parts):
        assert torch.equal(x, y)


def test_c3_full_size_properties(oracle):
    # BASELINE C3 mesh (1,003,520 faces) with 1M queries: size-independent properties on all queries,
    # tie-tolerant parity against the CGAL-tree restatement on a 3000-query sample.
    v, f = W.c3_mesh()
    q = np.random.default_rng(3).uniform(-1.1, 1.1, (1_000_000, 3))
    face, part, pt = _nearest(v, f, q)
    assert face.max() < f.shape[0] and part.max() <= 6
    tri = v[f[face].astype(np.int64)]
    # every returned point is the CGAL construction for its face
    for i in np.random.default_rng(1).choice(q.shape[0], 300, replace=False):
        p, pp, _ = oracle.point_triangle(q[i], tri[i, 0], tri[i, 1], tri[i, 2])
        assert (p == pt[i]).all() and pp == part[i]
    idx = np.random.default_rng(2).choice(q.shape[0], 3000, replace=False)
    cf, _, cpt = oracle.CgalTree(v, f).nearest(q[idx])
    diag = float(np.linalg.norm(v.max(0) - v.min(0)))
    dg = np.linalg.norm(pt[idx] - q[idx], axis=1)
    dc = np.linalg.norm(cpt - q[idx], axis=1)
    assert np.all(np.abs(dg - dc) <= 1e-9 * diag)
    same = face[idx] == cf
    # the icosphere is tie-heavy (queries outside project onto shared edges / vertices), so the CGAL tree's
    # traversal-order tie rule picks another face for some rows; where the faces agree the points are equal
    assert (pt[idx][same] == cpt[same]).all()
    assert np.all(np.abs(pt[idx] - cpt) <= 1e-6 * diag)
    # and with the same tie rule (lexicographic (d2, face)) the exhaustive oracle agrees bit for bit
    sub = idx[:1000]
    bf, bp, bpt, _ = oracle.brute_nearest(v, f, q[sub])
    assert np.array_equal(face[sub], bf) and np.array_equal(part[sub], bp) and np.array_equal(pt[sub], bpt)


def test_c3_headline_stream(oracle):
    # The exact stream bench.py times (100M uniform queries generated in HBM, seed 3, the device entry
    # point): shell bounds on every answer, and bit-exact against the exhaustive oracle on 2000 rows
    # (1500 at random + the 500 closest to the centre, where the deferred pass 2 answers).
    import torch
    from mesh_amd import spatialsearch
    from mesh_amd.distributed import nearest_device
    v, f = W.c3_mesh()
    S = 100_000_000
    dq = W.c3_stream(S, "cuda:0")
    t = spatialsearch.aabbtree_compute(v, f)
    df = torch.empty(S, dtype=torch.int32, device="cuda:0")
    dp = torch.empty(S, dtype=torch.int32, device="cuda:0")
    dpt = torch.empty((S, 3), dtype=torch.float64, device="cuda:0")
    nearest_device(t, dq, df, dp, dpt)
    torch.cuda.synchronize()
    q = dq.cpu().numpy()
    del dq
    face = df.cpu().numpy().view(np.uint32)
    part = dp.cpu().numpy().view(np.uint32)
    pt = dpt.cpu().numpy()
    del df, dp, dpt
    assert face.max() < f.shape[0] and part.max() <= 6 and np.isfinite(pt).all()
    # every vertex is on the unit sphere and every face plane at least r_in from the centre, so the
    # surface lies in the shell r_in <= |x| <= 1: d >= max(|q| - 1, r_in - |q|), and the face under the
    # radial projection of q is within one edge length: d <= ||q| - 1| + e_max
    tri = v[f.astype(np.int64)]
    nrm = np.cross(tri[:, 1] - tri[:, 0], tri[:, 2] - tri[:, 0])
    r_in = float(np.min(np.abs(np.einsum("ij,ij->i", nrm, tri[:, 0])) / np.linalg.norm(nrm, axis=1)))
    e_max = float(max(np.linalg.norm(tri[:, i] - tri[:, (i + 1) % 3], axis=1).max() for i in range(3)))
    d = np.sqrt(np.einsum("ij,ij->i", pt - q, pt - q))
    r = np.sqrt(np.einsum("ij,ij->i", q, q))
    tol = 1e-12
    assert np.all(d >= np.maximum(r - 1.0, r_in - r) - tol)
    assert np.all(d <= np.abs(r - 1.0) + e_max + tol)
    idx = np.concatenate([np.random.default_rng(5).choice(S, 1500, replace=False), np.argpartition(r, 500)[:500]])
    bf, bp, bpt, _ = oracle.brute_nearest(v, f, q[idx])
    assert np.array_equal(face[idx], bf), "faces differ at %s" % idx[np.nonzero(face[idx] != bf)[0][:10]]
    assert np.array_equal(part[idx], bp) and np.array_equal(pt[idx], bpt)


def test_normals_random_bit_exact(oracle):
    from mesh_amd import aabb_normals
    v, f = W.c2_mesh()
    q, fi = W.surface_samples(v, f, 5000, seed=11, sigma=0.02)
    n = np.random.default_rng(12).normal(size=q.shape)
    n /= np.linalg.norm(n, axis=1)[:, None]
    for eps in [0.0, 0.1, 2.0]:
        h = aabb_normals.aabbtree_n_compute(v, f, eps)
        face, pt = aabb_normals.aabbtree_n_nearest(h, q, n)
        bf, bpt, _ = oracle.brute_nnearest(v, f, eps, q, n)
        assert np.array_equal(face[0], bf), eps
        assert np.array_equal(pt, bpt), eps


def test_alongnormal_bit_exact(oracle):
    from mesh_amd.search import AabbTree
    from mesh_amd.mesh import Mesh
    v, f = W.c2_mesh()
    p, fi = W.surface_samples(v, f, 5000, seed=13, sigma=0.01)
    tri = v[f[fi].astype(np.int64)]
    n = np.cross(tri[:, 1] - tri[:, 0], tri[:, 2] - tri[:, 0])
    n /= np.linalg.norm(n, axis=1)[:, None]
    # add rays that miss everything
    p = np.vstack([p, [[5.0, 5.0, 5.0]] * 3])
    n = np.vstack([n, [[1.0, 0, 0]] * 3])
    d, face, pt = AabbTree(Mesh(v=v, f=f)).nearest_alongnormal(p, n)
    bd, bf, bpt = oracle.brute_alongnormal(v, f, p, n)
    assert d.shape == (p.shape[0],) and face.dtype == np.uint32
    assert np.array_equal(d, bd)
    assert np.array_equal(face, bf)
    hit = bd < 1e100
    assert np.array_equal(pt[hit], bpt[hit])
    assert (d[~hit] == 1e100).all() and (face[~hit] == 0xFFFFFFFF).all() and np.isnan(pt[~hit]).all()


def test_alongnormal_entry_cut_bit_exact(oracle):
    # alongnormal walks start from the closest-point entry cut's start list, the bound capped at the radius the list
    # covers around p, and walk again from the root when no hit lies that near (rays.hip traverse_along_pend): the
    # answers equal the walks from the root for the 48^3 (coarse), 96^3 (fine, built from the coarse one) and 8^3
    # grids, on near-surface rays (mostly answered from the list), far and random rays (mostly walked again), rays on
    # the grid's cell faces and outside it, and rays that miss; 6,000 of them against brute force
    from mesh_amd import spatialsearch
    v, f = W.c2_mesh()
    rng = np.random.default_rng(71)
    near, fi = W.surface_samples(v, f, 20_000, seed=72, sigma=0.01)
    tri = v[f[fi].astype(np.int64)]
    nn = np.cross(tri[:, 1] - tri[:, 0], tri[:, 2] - tri[:, 0])
    nn /= np.linalg.norm(nn, axis=1)[:, None]
    far, _ = W.surface_samples(v, f, 5_000, seed=73, sigma=0.3)
    lo, hi = v.min(0), v.max(0)
    box = rng.uniform(lo - 0.5 * (hi - lo), hi + 0.5 * (hi - lo), (10_000, 3))
    onf = rng.uniform(lo, hi, (3_000, 3))
    c, e = 0.5 * (lo + hi), 1.25 * 0.5 * (hi - lo)
    ax = rng.integers(0, 3, 3_000)
    onf[np.arange(3_000), ax] = (c - e)[ax] + rng.integers(0, 49, 3_000) * (2 * e / 48)[ax]
    rd = rng.normal(size=(18_000, 3))
    rd /= np.linalg.norm(rd, axis=1)[:, None]
    p = np.vstack([near, far, box, onf, [[50.0, 50.0, 50.0]] * 4])
    n = np.vstack([nn, rd[:5_000], rd[5_000:15_000], rd[15_000:18_000], [[1.0, 0.0, 0.0]] * 4])
    t = spatialsearch.aabbtree_compute(v, f)
    outs = []
    for g in (0, 48, -1, 8):
        t.set_entry_cut(g)
        outs.append(spatialsearch.aabbtree_nearest_alongnormal(t, p, n))
        info = t.entry_cut_info()
        assert info["state"] == ("off" if g == 0 else "built"), info
        assert info["G"] == (0 if g == 0 else (96 if g < 0 else g)), info
    for o in outs[1:]:
        assert np.array_equal(outs[0][0], o[0]) and np.array_equal(outs[0][1], o[1])
        assert np.array_equal(outs[0][2].view(np.int64), o[2].view(np.int64))  # NaN points of misses too
    rows = np.concatenate([rng.choice(20_000, 3_000, replace=False), 20_000 + rng.choice(18_004, 3_000, replace=False)])
    bd, bf, bpt = oracle.brute_alongnormal(v, f, p[rows], n[rows])
    d, face, pt = outs[2]
    assert np.array_equal(d[rows], bd) and np.array_equal(face[rows], bf)
    hit = bd < 1e100
    assert hit.sum() > 3_000
    assert np.array_equal(pt[rows][hit], bpt[hit])


def test_visibility_random_exact(oracle):
    from mesh_amd.visibility import visibility_compute
    v, f = W.geodesic_icosphere(12)
    th = np.arccos(np.clip(v[:, 2], -1, 1))
    ph = np.arctan2(v[:, 1], v[:, 0])
    v = v * (1 + 0.1 * np.sin(5 * th) * np.sin(4 * ph))[:, None]  # C5-style bumps: self-occlusion
    from mesh_amd.mesh import Mesh
    n = Mesh(v=v, f=f).estimate_vertex_normals()
    cams = W.uniform_in_box([-3, -3, -3], [3, 3, 3], 6, seed=14, margin=0)
    sens = np.random.default_rng(15).normal(size=(6, 9))
    for kw in [dict(), dict(n=n), dict(n=n, sensors=sens), dict(min_dist=0.05)]:
        vis, ndc = visibility_compute(cams=cams, v=v, f=f, **kw)
        bv, bn = oracle.brute_visibility(v, f, cams, **kw)
        assert np.array_equal(vis, bv), kw
        assert np.array_equal(ndc, bn), kw
        assert 0 < vis.mean() < 1


def test_visibility_borrowed_tree():
    from mesh_amd import spatialsearch
    from mesh_amd.visibility import visibility_compute
    v, f = W.geodesic_icosphere(4)
    t = spatialsearch.aabbtree_compute(v, f)
    a, _ = visibility_compute(cams=np.array([[0, 0, 3.0]]), tree=t)
    b, _ = visibility_compute(cams=np.array([[0, 0, 3.0]]), v=v, f=f)
    assert np.array_equal(a, b)
    # the borrowed handle is still usable (reference double-frees it, py_visibility.cpp:212)
    spatialsearch.aabbtree_nearest(t, np.zeros((2, 3)))


def test_intersections_random(oracle):
    from mesh_amd import spatialsearch
    v, f = W.geodesic_icosphere(6)
    rng = np.random.default_rng(16)
    for shift in [0.3, 1.0, 1.9, 3.0]:
        qv = v * 0.8 + np.array([shift, 0.1, -0.05])
        t = spatialsearch.aabbtree_compute(v, f)
        got = spatialsearch.aabbtree_intersections_indices(t, qv, f)
        want = oracle.brute_intersections(v, f, qv, f)
        assert np.array_equal(got, want), shift
    # random triangle soup
    qv = rng.normal(size=(300, 3))
    qf = np.arange(300, dtype=np.uint32).reshape(-1, 3)
    got = spatialsearch.aabbtree_intersections_indices(spatialsearch.aabbtree_compute(v, f), qv, qf)
    assert np.array_equal(got, oracle.brute_intersections(v, f, qv, qf))


def test_selfintersects_random(oracle):
    from mesh_amd import aabb_normals
    rng = np.random.default_rng(17)
    v = rng.normal(size=(600, 3))
    f = np.arange(600, dtype=np.uint32).reshape(-1, 3)
    f2 = np.vstack([f, np.array([[0, 1, 5], [3, 4, 200]], np.uint32)])  # shared-vertex pairs are skipped
    for ff in [f, f2]:
        h = aabb_normals.aabbtree_n_compute(v, ff, 0.1)
        assert aabb_normals.aabbtree_n_selfintersects(h) == oracle.brute_selfintersects(v, ff)


def test_points_random_exact(oracle):
    from mesh_amd.search import ClosestPointTree
    from mesh_amd.mesh import Mesh
    v, f = W.c2_mesh()
    q = W.uniform_in_box(v.min(0), v.max(0), 50000, seed=18)
    idx, dist = ClosestPointTree(Mesh(v=v, f=f)).nearest(q)
    bi, bd = oracle.brute_vertex_nn(v, q)
    assert np.array_equal(np.array(idx), bi)
    assert np.array_equal(np.array(dist), bd)


def test_cgal_closest_point_tree(meshes, oracle):
    from mesh_amd.mesh import Mesh
    v = meshes["sphere_v"]
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "kdtree.npz"))
    m = Mesh(v=v, f=meshes["sphere_f"])
    fi, d = m.closest_vertices(g["q"], use_cgal=True)
    assert np.array_equal(fi, g["idx"].astype(np.uint32))
    assert np.allclose(d, g["dist"], rtol=1e-9)


# ---------------------------------------------------------------- edge cases
def test_empty_queries():
    from mesh_amd import spatialsearch
    v, f = W.geodesic_icosphere(2)
    t = spatialsearch.aabbtree_compute(v, f)
    face, part, pt = spatialsearch.aabbtree_nearest(t, np.zeros((0, 3)))
    assert face.shape == (1, 0) and pt.shape == (0, 3)
    d, fc, p = spatialsearch.aabbtree_nearest_alongnormal(t, np.zeros((0, 3)), np.zeros((0, 3)))
    assert d.shape == (0,)


def test_empty_mesh_rejected():
    from mesh_amd import spatialsearch
    with pytest.raises(ValueError):
        spatialsearch.aabbtree_compute(np.zeros((3, 3)), np.zeros((0, 3), np.uint32))


@pytest.mark.parametrize("T", [1, 2, 3, 5])
def test_tiny_meshes(oracle, T):
    rng = np.random.default_rng(T)
    v = rng.normal(size=(3 * T, 3))
    f = np.arange(3 * T, dtype=np.uint32).reshape(-1, 3)
    _assert_bit_exact_vs_brute(oracle, v, f, rng.normal(size=(5000, 3)) * 2)


def test_duplicate_and_degenerate_triangles(oracle):
    # coincident centroids (duplicate Morton codes) and zero-area triangles
    v, f = W.geodesic_icosphere(5)
    f = np.vstack([f, f[:50], f[:50, [1, 2, 0]]])
    extra = np.array([[0.1, 0.1, 0.1], [0.2, 0.2, 0.2], [0.3, 0.3, 0.3]])  # collinear
    v2 = np.vstack([v, extra])
    P = v.shape[0]
    f = np.vstack([f, [[P, P + 1, P + 2], [P, P, P + 1]]]).astype(np.uint32)
    q = W.uniform_in_box([-1, -1, -1], [1, 1, 1], 20000, seed=19)
    _assert_bit_exact_vs_brute(oracle, v2, f, q)


def test_far_and_offset_queries(oracle):
    v, f = W.geodesic_icosphere(8)
    off = np.array([1e6, -2e6, 3e5])
    q = np.vstack([W.uniform_in_box([-1, -1, -1], [1, 1, 1], 5000, seed=20) * 1e4,
                   W.uniform_in_box([-1, -1, -1], [1, 1, 1], 5000, seed=21)])
    _assert_bit_exact_vs_brute(oracle, v, f, q)
    _assert_bit_exact_vs_brute(oracle, v + off, f, q + off)


def test_queries_on_vertices_and_edges(oracle):
    v, f = W.geodesic_icosphere(10)
    e = 0.5 * (v[f[:, 0]] + v[f[:, 1]])
    q = np.vstack([v, e, np.zeros((1, 3))])  # the centre is equidistant-ish from everything
    _assert_bit_exact_vs_brute(oracle, v, f, q)


def test_cooperative_pass_near_centre(oracle):
    # queries near the centre of a closed sphere exceed the pass-1 step budget and are finished by the
    # wave-cooperative pass 2 (bound shared across lanes); the result must still be the exact lexmin
    v, f = W.geodesic_icosphere(40)  # 32,000 faces
    rng = np.random.default_rng(25)
    q = np.vstack([rng.normal(size=(3000, 3)) * 0.02, rng.uniform(-1.1, 1.1, (3000, 3)), np.zeros((1, 3))])
    _assert_bit_exact_vs_brute(oracle, v, f, q)
    from mesh_amd import aabb_normals
    n = rng.normal(size=q.shape)
    n /= np.linalg.norm(n, axis=1)[:, None]
    face, pt = aabb_normals.aabbtree_n_nearest(aabb_normals.aabbtree_n_compute(v, f, 0.1), q, n)
    bf, bpt, _ = oracle.brute_nnearest(v, f, 0.1, q, n)
    assert np.array_equal(face[0], bf) and np.array_equal(pt, bpt)


def test_deep_tree_spill_path(oracle):
    # a mesh whose LBVH is deeper than the 16-entry LDS stack (clustered + spread triangles)
    rng = np.random.default_rng(22)
    pts = np.vstack([rng.normal(size=(3000, 3)) * 1e-4, rng.normal(size=(3000, 3)) * 100])
    v = np.repeat(pts, 3, axis=0) + rng.normal(size=(18000, 3)) * 1e-6
    f = np.arange(18000, dtype=np.uint32).reshape(-1, 3)
    from mesh_amd import spatialsearch
    t = spatialsearch.aabbtree_compute(v, f)
    q = rng.normal(size=(20000, 3)) * 50
    face, part, pt = spatialsearch.aabbtree_nearest(t, q)
    bf, bp, bpt, _ = oracle.brute_nearest(v, f, q)
    assert np.array_equal(face[0], bf) and np.array_equal(pt, bpt)


def test_build_deterministic_and_blob_roundtrip(oracle):
    import torch
    from mesh_amd import _native, spatialsearch
    v, f = W.c2_mesh()
    q = W.uniform_in_box(v.min(0), v.max(0), 30000, seed=23)
    t1 = spatialsearch.aabbtree_compute(v, f)
    t2 = spatialsearch.aabbtree_compute(v, f)
    r1 = spatialsearch.aabbtree_nearest(t1, q)
    r2 = spatialsearch.aabbtree_nearest(t2, q)
    assert all(np.array_equal(a, b) for a, b in zip(r1, r2))
    n = _native.blob_size(t1)
    blob = torch.empty(n, dtype=torch.uint8, device="cuda:0")
    _native.blob_pack(t1, blob.data_ptr())
    t3 = _native.blob_unpack(blob.data_ptr(), n, 0)
    r3 = spatialsearch.aabbtree_nearest(t3, q)
    assert all(np.array_equal(a, b) for a, b in zip(r1, r3))


def test_device_api_matches_host_api():
    import torch
    from mesh_amd import spatialsearch
    from mesh_amd.distributed import nearest_device
    v, f = W.c2_mesh()
    q = W.uniform_in_box(v.min(0), v.max(0), 100000, seed=24)
    t = spatialsearch.aabbtree_compute(v, f)
    face, part, pt = spatialsearch.aabbtree_nearest(t, q)
    dq = torch.from_numpy(q).cuda()
    df = torch.empty(q.shape[0], dtype=torch.int32, device="cuda")
    dp = torch.empty(q.shape[0], dtype=torch.int32, device="cuda")
    dpt = torch.empty((q.shape[0], 3), dtype=torch.float64, device="cuda")
    nearest_device(t, dq, df, dp, dpt)
    torch.cuda.synchronize()
    assert np.array_equal(df.cpu().numpy().view(np.uint32), face[0])
    assert np.array_equal(dp.cpu().numpy().view(np.uint32), part[0])
    assert np.array_equal(dpt.cpu().numpy(), pt)


def test_host_api_registered_and_staged_agree(monkeypatch):
    # calls above 16 MB of rows run chunked: the caller's arrays page-locked in place (hipHostRegister) or,
    # with MESH_AMD_HOST_REGISTER=0, through pinned staging slabs; both equal the device entry point's answer
    import torch
    from mesh_amd import spatialsearch
    from mesh_amd.distributed import nearest_device
    v, f = W.c2_mesh()
    q = W.uniform_in_box(v.min(0), v.max(0), 700000, seed=25)  # 39 MB of rows (56 B each): the chunked path
    monkeypatch.setenv("MESH_AMD_HOST_CHUNK", "262144")      # 3 chunks: both slabs reused
    t = spatialsearch.aabbtree_compute(v, f)
    monkeypatch.setenv("MESH_AMD_HOST_REGISTER", "1")
    reg = spatialsearch.aabbtree_nearest(t, q)
    monkeypatch.setenv("MESH_AMD_HOST_REGISTER", "0")
    stg = spatialsearch.aabbtree_nearest(t, q)
    for a, b in zip(reg, stg):
        assert np.array_equal(a, b)
    dq = torch.from_numpy(q).cuda()
    df = torch.empty(q.shape[0], dtype=torch.int32, device="cuda")
    dp = torch.empty(q.shape[0], dtype=torch.int32, device="cuda")
    dpt = torch.empty((q.shape[0], 3), dtype=torch.float64, device="cuda")
    nearest_device(t, dq, df, dp, dpt)
    torch.cuda.synchronize()
    assert np.array_equal(df.cpu().numpy().view(np.uint32), reg[0][0])
    assert np.array_equal(dpt.cpu().numpy(), reg[2])


def test_host_api_pinned_results(monkeypatch):
    # large host calls carve their results from the page-locked pool (msh_host_alloc) and download straight
    # into them; the arrays equal the pageable path's (pool disabled) for all three pipelined entry points, the
    # block returns to the pool when its arrays die and is reused by the next call, and an in-place
    # registration attempt on pool memory falls back to staging with the same answer
    from mesh_amd import _native as N, spatialsearch
    v, f = W.c2_mesh()
    q = W.uniform_in_box(v.min(0), v.max(0), 700000, seed=26)
    nrm = np.random.default_rng(27).normal(size=q.shape)
    monkeypatch.setenv("MESH_AMD_HOST_CHUNK", "262144")  # 3 chunks: both slabs reused
    monkeypatch.setattr(N, "PINNED_MIN_BYTES", 1 << 20)
    t = spatialsearch.aabbtree_compute(v, f)
    calls = [lambda: spatialsearch.aabbtree_nearest(t, q), lambda: spatialsearch.aabbtree_nearest_barycentric(t, q),
             lambda: spatialsearch.aabbtree_nearest_alongnormal(t, q, nrm)]
    monkeypatch.setenv("MESH_AMD_PINNED_POOL_MB", "0")
    ref = [c() for c in calls]
    assert all(r[0].base is None for r in ref)  # pool disabled: plain np.empty arrays
    monkeypatch.setenv("MESH_AMD_PINNED_POOL_MB", "1024")
    for c, r in zip(calls, ref):
        got = c()
        for a, b in zip(got, r):
            assert a.shape == b.shape and a.dtype == b.dtype and a.flags.c_contiguous
            assert np.array_equal(a, b, equal_nan=a.dtype.kind == "f")
        owner = got[0]
        while isinstance(owner, np.ndarray):
            owner = owner.base
        assert isinstance(owner, N._PinnedBlock)
        del got, owner
    held = N.lib().msh_host_pool_bytes()
    assert held > 0
    for _ in range(3):  # steady state: blocks come back and are reused
        out = spatialsearch.aabbtree_nearest(t, q)
        del out
    assert N.lib().msh_host_pool_bytes() == held
    monkeypatch.setenv("MESH_AMD_HOST_REGISTER", "1")
    for a, b in zip(spatialsearch.aabbtree_nearest(t, q), ref[0]):
        assert np.array_equal(a, b)
    monkeypatch.delenv("MESH_AMD_HOST_REGISTER")
    assert N.lib().msh_host_pool_trim() == 0
    # a pool too small for the block: the call falls back to pageable arrays with the same answer
    monkeypatch.setenv("MESH_AMD_PINNED_POOL_MB", "4")
    out = spatialsearch.aabbtree_nearest(t, q)  # 22 MB of results
    assert out[0].base is None
    for a, b in zip(out, ref[0]):
        assert np.array_equal(a, b)


def test_normals_and_points_host_chunked(oracle, monkeypatch):
    # aabb_normals.aabbtree_n_nearest and ClosestPointTree run through the chunked host pipeline (pinned result
    # arrays, several chunks) and give exactly the answers of small unchunked calls on the same rows; a sample
    # matches brute force
    from mesh_amd import _native as N, aabb_normals
    from mesh_amd.mesh import Mesh
    from mesh_amd.search import ClosestPointTree
    v, f = W.c2_mesh()
    q, fi = W.surface_samples(v, f, 400000, seed=51, sigma=0.01)
    tri = v[f[fi].astype(np.int64)]
    n = np.cross(tri[:, 1] - tri[:, 0], tri[:, 2] - tri[:, 0])
    n /= np.linalg.norm(n, axis=1)[:, None]
    n += np.random.default_rng(52).normal(scale=0.2, size=n.shape)
    monkeypatch.setattr(N, "PINNED_MIN_BYTES", 1 << 20)
    monkeypatch.setenv("MESH_AMD_HOST_CHUNK", "131072")  # 4 chunks: both slabs reused
    h = aabb_normals.aabbtree_n_compute(v, f, 0.1)
    face, pt = aabb_normals.aabbtree_n_nearest(h, q, n)
    owner = face
    while isinstance(owner, np.ndarray):
        owner = owner.base
    assert isinstance(owner, N._PinnedBlock)
    parts = [aabb_normals.aabbtree_n_nearest(h, q[k:k + 50000], n[k:k + 50000]) for k in range(0, q.shape[0], 50000)]
    assert np.array_equal(face, np.concatenate([p[0] for p in parts], axis=1))
    assert np.array_equal(pt, np.concatenate([p[1] for p in parts]))
    rows = np.random.default_rng(53).choice(q.shape[0], 3000, replace=False)
    bf, bpt = oracle.brute_nnearest(v, f, 0.1, q[rows], n[rows])[:2]
    assert np.array_equal(face[0][rows], np.asarray(bf).reshape(-1)) and np.array_equal(pt[rows], bpt)
    t = ClosestPointTree(Mesh(v=v, f=f))
    idx, dist = t._query(q)
    pidx = np.concatenate([t._query(q[k:k + 50000])[0] for k in range(0, q.shape[0], 50000)])
    assert np.array_equal(idx, pidx)
    bi, bd = oracle.brute_vertex_nn(v, q[rows])
    assert np.array_equal(idx[rows], np.asarray(bi).astype(idx.dtype)) and np.array_equal(dist[rows], bd)


@pytest.mark.parametrize("name", ["ico", "ico60", "c2", "offset"])
def test_tree_bounds_contain_primitives(name):
    # every child's quantised oriented box (frame n, t, n x t) contains all vertices below it
    from scripts.check_tree import check_mesh
    if name == "ico":
        v, f = W.geodesic_icosphere(20)
    elif name == "ico60":  # 72,000 faces: several levels of nodes over kObbBig leaves, up to 71 chunks each
        v, f = W.geodesic_icosphere(60)
    elif name == "c2":
        v, f = W.c2_mesh()
    else:
        v, f = W.geodesic_icosphere(10)
        v = v * 0.01 + np.array([1e5, -3e4, 2e5])
    r = check_mesh(v, f)
    assert r["obb_containment_violations"] == 0, r
    assert r["reached_nodes"] == f.shape[0] - 1
    # 8-bit codes: a bound moves outward by at most one code step, 2^e < 2/254 of the node's range along
    # that axis (plus the fp32 outward rounding)
    assert r["worst_relative_obb_looseness_first2000"] < 2.2 / 254, r


def test_many_tied_candidates(oracle):
    # Queries radially above / below icosphere vertices: the closest point is the vertex, shared by 5-6
    # faces at exactly equal distance, so more tied candidates than the pass-1 candidate list holds
    # (overflow -> exact on the spot) — the lexmin (d2, face) must still be bit-exact.
    v, f = W.geodesic_icosphere(40)
    q = np.vstack([v * 1.05, v * 0.95, v * 1.5])
    face, _, _ = _assert_bit_exact_vs_brute(oracle, v, f, q)
    assert face.shape[0] == q.shape[0]


def test_batch_bit_exact_per_mesh(oracle):
    # C4 shape at small B: the batched build + query must equal, mesh by mesh, the exhaustive answer
    from mesh_amd.search import AabbTreeBatch
    B = 6
    f = W.c4_mesh(0)[1]
    v = np.stack([W.c4_mesh(i)[0] for i in range(B)])
    rng = np.random.default_rng(41)
    q = np.empty((B, 3000, 3))
    for b in range(B):
        s, _ = W.surface_samples(v[b], f, 2000, seed=100 + b, sigma=0.003)
        lo, hi = v[b].min(0), v[b].max(0)
        q[b] = np.vstack([s, rng.uniform(lo - 0.05, hi + 0.05, (1000, 3))])
    face, part, pt = AabbTreeBatch(v, f).nearest(q, nearest_part=True)
    assert face.shape == (B, 3000) and part.shape == (B, 3000) and pt.shape == (B, 3000, 3)
    for b in range(B):
        bf, bp, bpt, _ = oracle.brute_nearest(v[b], f, q[b])
        assert np.array_equal(face[b], bf), b
        assert np.array_equal(part[b], bp), b
        assert np.array_equal(pt[b], bpt), b


def test_batch_matches_single_trees():
    from mesh_amd import spatialsearch
    from mesh_amd.search import AabbTreeBatch
    B = 3
    f = W.c4_mesh(0)[1]
    v = np.stack([W.c4_mesh(i)[0] + i for i in range(B)])  # different boxes / origins per mesh
    q = np.stack([W.uniform_in_box(v[b].min(0), v[b].max(0), 20000, seed=50 + b) for b in range(B)])
    face, part, pt = AabbTreeBatch(v, f).nearest(q, nearest_part=True)
    for b in range(B):
        t = spatialsearch.aabbtree_compute(np.ascontiguousarray(v[b]), f)
        sf, sp, spt = spatialsearch.aabbtree_nearest(t, q[b])
        assert np.array_equal(face[b], sf[0]) and np.array_equal(part[b], sp[0]) and np.array_equal(pt[b], spt)


def test_batch_of_one_off_origin_mesh(oracle):
    # a B == 1 batch is a batched handle (bounds relative to the per-mesh origin); it must answer
    # correctly through the batch entry points and be refused by the single-tree ones
    from mesh_amd import spatialsearch
    from mesh_amd.search import AabbTreeBatch
    v, f = W.c4_mesh(3)
    v = v + np.array([40.0, -25.0, 13.0])  # far from the scene origin
    q = W.uniform_in_box(v.min(0), v.max(0), 20000, seed=61)
    bt = AabbTreeBatch(v[None], f)
    face, part, pt = bt.nearest(q[None], nearest_part=True)
    bf, bp, bpt, _ = oracle.brute_nearest(v, f, q)
    assert np.array_equal(face[0], bf) and np.array_equal(part[0], bp) and np.array_equal(pt[0], bpt)
    with pytest.raises(ValueError):
        spatialsearch.aabbtree_nearest(bt.cpp_handle, q)


def test_c4_full_size(oracle):
    # BASELINE configs[3]: 4096 meshes x 10k scan points; exact vs brute force on 6 meshes, properties on all
    from mesh_amd.search import AabbTreeBatch
    v, f, q = W.c4_batch()
    face, part, pt = AabbTreeBatch(v, f).nearest(q, nearest_part=True)
    assert face.max() < f.shape[0] and part.max() <= 6 and np.isfinite(pt).all()
    for b in np.random.default_rng(7).choice(v.shape[0], 6, replace=False):
        bf, bp, bpt, _ = oracle.brute_nearest(v[b], f, q[b])
        assert np.array_equal(face[b], bf) and np.array_equal(part[b], bp) and np.array_equal(pt[b], bpt), b
    # every point is on its face's triangle (barycentric check, all 41M rows)
    tri = v[np.arange(v.shape[0])[:, None, None], f[face.astype(np.int64)]]  # (B,S,3,3)
    n = np.cross(tri[..., 1, :] - tri[..., 0, :], tri[..., 2, :] - tri[..., 0, :])
    off = np.abs(np.einsum("bsk,bsk->bs", pt - tri[..., 0, :], n)) / np.linalg.norm(n, axis=-1)
    assert off.max() < 1e-9


@pytest.mark.parametrize("chunk", [None, "7"])
def test_batch_host_pipelined_equals_device(monkeypatch, chunk):
    # AabbTreeBatch.nearest (numpy) runs pipelined over chunks of whole meshes (api.cpp batch_host): the answers equal
    # the device entry point's over the same rows, bit for bit, with the library's plan and with 7-mesh chunks (a
    # chunk that starts mid-batch: per-chunk sort, roots and origins of meshes mesh0...)
    import torch
    from mesh_amd import _native as N
    from mesh_amd.search import AabbTreeBatch
    if chunk:
        monkeypatch.setenv("MESH_AMD_HOST_CHUNK", chunk)
    B, S = 64, 10_000
    f = W.c4_mesh(0)[1]
    v = np.stack([W.c4_mesh(i)[0] + 0.1 * i for i in range(B)])
    rng = np.random.default_rng(71)
    q = np.stack([W.uniform_in_box(v[b].min(0), v[b].max(0), S, seed=int(rng.integers(1 << 30))) for b in range(B)])
    bt = AabbTreeBatch(v, f)
    face, part, pt = bt.nearest(q, nearest_part=True)
    bface, bpt, bw = bt.nearest_barycentric(q)
    dq = torch.from_numpy(q).cuda()
    df = torch.empty((B, S), dtype=torch.int32, device="cuda")
    dp = torch.empty((B, S), dtype=torch.int32, device="cuda")
    dpt = torch.empty((B, S, 3), dtype=torch.float64, device="cuda")
    dw = torch.empty((B, S, 3), dtype=torch.float64, device="cuda")
    N.check(N.lib().msh_batch_nearest_device(bt.cpp_handle.ptr, dq.data_ptr(), S, df.data_ptr(), dp.data_ptr(),
                                             dpt.data_ptr(), None))
    torch.cuda.synchronize()
    assert np.array_equal(face, df.cpu().numpy().view(np.uint32)) and np.array_equal(part, dp.cpu().numpy().view(np.uint32))
    assert np.array_equal(pt, dpt.cpu().numpy())
    N.check(N.lib().msh_batch_nearest_bary_device(bt.cpp_handle.ptr, dq.data_ptr(), S, df.data_ptr(), dpt.data_ptr(),
                                                  dw.data_ptr(), None))
    torch.cuda.synchronize()
    assert np.array_equal(bface, df.cpu().numpy().view(np.uint32)) and np.array_equal(bpt, dpt.cpu().numpy())
    assert np.array_equal(bw, dw.cpu().numpy())
    assert np.array_equal(bface, face)


@pytest.mark.parametrize("chunk", [None, "3"])
def test_visibility_host_pipelined_equals_device(monkeypatch, chunk):
    # visibility_compute (numpy) downloads its (C, P) outputs a few cameras at a time (api.cpp msh_visibility): equal
    # to msh_visibility_device over all vertices, with normals and sensors (offset per camera chunk), bit for bit
    import torch
    from mesh_amd import spatialsearch, visibility
    from mesh_amd.distributed import visibility_device
    from mesh_amd.mesh import Mesh
    if chunk:
        monkeypatch.setenv("MESH_AMD_HOST_CHUNK", chunk)
    v, f = W.geodesic_icosphere(100)
    v = v * (1.0 + 0.1 * np.sin(5 * v[:, :1]) * np.cos(4 * v[:, 1:2]))
    t = spatialsearch.aabbtree_compute(v, f)
    vn = Mesh(v=v, f=f).estimate_vertex_normals()
    C = 16
    cams = W.fibonacci_cameras(C, 3.0)
    sens = np.random.default_rng(72).normal(size=(C, 9)) * 4.0
    for kw in ({"n": vn}, {"n": vn, "sensors": sens}):
        vis, ndc = visibility.visibility_compute(cams=cams, tree=t, **kw)
        assert vis.shape == (C, v.shape[0]) and vis.dtype == np.uint32 and ndc.dtype == np.float64
        dv = torch.empty((C, v.shape[0]), dtype=torch.int32, device="cuda")
        dd = torch.empty((C, v.shape[0]), dtype=torch.float64, device="cuda")
        visibility_device(t, torch.from_numpy(cams).cuda(), dv, dd, torch.from_numpy(vn).cuda(),
                          torch.from_numpy(kw["sensors"]).cuda() if "sensors" in kw else None)
        torch.cuda.synchronize()
        assert np.array_equal(vis, dv.cpu().numpy().view(np.uint32)) and np.array_equal(ndc, dd.cpu().numpy())
        assert 0.05 < vis.mean() < 0.95


def test_multi_device_replicas_equal_one_device():
    # msh_set_device_list([0, 0, 0]): trees built next get two replicas (blob pack + copy + unpack, here on the one
    # GPU of the box), and host-buffer calls split their rows over the three handles from three host threads.  Every
    # entry point that fans out gives the one-device arrays bit for bit; G = 1 again afterwards.
    from mesh_amd import _native as N, aabb_normals, spatialsearch, visibility
    from mesh_amd.mesh import Mesh
    from mesh_amd.search import ClosestPointTree
    v, f = W.c2_mesh()
    q, _ = W.surface_samples(v, f, 1_500_000, seed=81, sigma=0.02)  # 84 MB of rows: above the fan-out floor
    nrm = np.random.default_rng(82).normal(size=q.shape)
    cams = W.fibonacci_cameras(16, 3.0)
    vb, fb = W.geodesic_icosphere(160)  # 256k vertices: 16 cameras x 256k x 12 B = 49 MB of outputs
    vn = Mesh(v=vb, f=fb).estimate_vertex_normals()

    def run():
        t = spatialsearch.aabbtree_compute(v, f)
        tb = spatialsearch.aabbtree_compute(vb, fb)
        h = aabb_normals.aabbtree_n_compute(v, f, 0.1)
        out = [spatialsearch.aabbtree_nearest(t, q), spatialsearch.aabbtree_nearest_barycentric(t, q),
               spatialsearch.aabbtree_nearest_alongnormal(t, q, nrm), aabb_normals.aabbtree_n_nearest(h, q, nrm),
               ClosestPointTree(Mesh(v=v, f=f))._query(q), visibility.visibility_compute(cams=cams, tree=tb, n=vn)]
        return out, N.tree_devices(t), N.tree_devices(h)

    one, d1, _ = run()
    assert d1 == [0]
    try:
        N.set_devices([0, 0, 0])
        many, d3, dh = run()
        assert d3 == [0, 0, 0] and dh == [0, 0, 0]
    finally:
        N.set_devices([0])
    for a, b in zip(one, many):
        for x, y in zip(a, b):
            assert np.array_equal(np.asarray(x), np.asarray(y), equal_nan=np.asarray(x).dtype.kind == "f")
    t = spatialsearch.aabbtree_compute(v, f)
    assert N.tree_devices(t) == [0]
    # msh_set_device drops the device list: no replica after set_devices([0, 0]) + set_device(0)
    try:
        N.set_devices([0, 0])
        assert N.tree_devices(spatialsearch.aabbtree_compute(v, f)) == [0, 0]
        N.set_device(0)
        assert N.tree_devices(spatialsearch.aabbtree_compute(v, f)) == [0]
    finally:
        N.set_devices([0])


def test_facade_entry_cut_policy():
    # Mesh.closest_faces_and_points builds a tree per call and picks its entry cut from the batch size (mesh.py): the
    # default grid for >= 8 queries per cell (C2 mesh, 7.5M queries), the coarse one for >= 32 per coarse cell, none
    # below; the answers equal a tree's without any cut, bit for bit
    from mesh_amd import spatialsearch
    from mesh_amd.mesh import Mesh
    v, f = W.c2_mesh()
    m = Mesh(v=v, f=f)
    t = spatialsearch.aabbtree_compute(v, f)
    t.set_entry_cut(0)
    for n in (7_500_000, 4_000_000, 200_000):
        q, _ = W.surface_samples(v, f, n, seed=90 + n % 7, sigma=0.01)
        face, pt = m.closest_faces_and_points(q)
        rf, _, rpt = spatialsearch.aabbtree_nearest(t, q)
        assert np.array_equal(face, rf) and np.array_equal(pt, rpt), n
