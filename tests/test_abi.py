"""C-ABI boundary checks that need no GPU: the library loads, exports every symbol the header declares,
the ctypes table matches the header, argument validation mirrors the reference's error surface, and
the product path fails loudly (no CPU fallback) when no HIP device is usable."""
import ctypes
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "meshsearch.h")


def header_symbols():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(msh_[a-z0-9_]+)\s*\(", txt)))


def test_library_exports_every_header_symbol():
    from mesh_amd import _native
    L = ctypes.CDLL(_native.LIB_PATH)
    syms = header_symbols()
    assert len(syms) >= 25
    missing = [s for s in syms if not hasattr(L, s)]
    assert not missing, missing


def test_ctypes_table_matches_header():
    from mesh_amd import _native
    assert sorted(n for n, _, _ in _native.SIGNATURES) == header_symbols()


def test_library_is_gfx950_hip():
    # the shared object carries an embedded gfx950 code object bundle
    blob = open(os.path.join(ROOT, "mesh_amd", "lib", "libmeshsearch.so"), "rb").read()
    assert b"gfx950" in blob
    assert b"k_knn" in blob and b"k_karras" in blob and b"k_scatter" in blob


def test_version_and_error_string():
    from mesh_amd import _native
    L = _native.lib()
    assert L.msh_version() == 2
    assert isinstance(L.msh_last_error(), bytes)


def _no_gpu():
    from mesh_amd import _native
    return _native.device_count() == 0


@pytest.mark.skipif(not _no_gpu(), reason="a HIP device is present")
def test_no_device_fails_loudly(meshes):
    from mesh_amd import spatialsearch
    with pytest.raises(RuntimeError):
        spatialsearch.aabbtree_compute(meshes["sphere_v"], meshes["sphere_f"])


def test_validation_mirrors_reference(meshes):
    from mesh_amd import _native, aabb_normals, spatialsearch, visibility
    v, f = meshes["sphere_v"], meshes["sphere_f"]
    with pytest.raises(ValueError, match="Vertices must be of type double, and 2 dimensional"):
        spatialsearch.aabbtree_compute(v.astype(np.float32), f)
    with pytest.raises(ValueError, match="Faces must be of type uint32, and 2 dimensional"):
        spatialsearch.aabbtree_compute(v, f.astype(np.int64))
    with pytest.raises(ValueError, match="Input must be Nx3"):
        spatialsearch.aabbtree_compute(v[:, :2].copy(), f)
    with pytest.raises(ValueError, match="Vertices must be of type double"):
        aabb_normals.aabbtree_n_compute(v.astype(np.float32), f, 0.1)
    fake = _native.Handle(1, "triangles")
    fake_n = _native.Handle(1, "normals")
    try:
        with pytest.raises(ValueError, match="Input must be Nx3"):
            spatialsearch.aabbtree_nearest(fake, np.zeros((4, 2)))
        with pytest.raises(ValueError, match="Points and normals must be Nx3"):
            spatialsearch.aabbtree_nearest_alongnormal(fake, np.zeros((4, 3)), np.zeros((5, 3)))
        with pytest.raises(ValueError, match="Query Faces must be of type uint32"):
            spatialsearch.aabbtree_intersections_indices(fake, np.zeros((3, 3)), np.zeros((1, 3), np.int32))
        with pytest.raises(ValueError, match="First argument must be a NumPy array"):
            aabb_normals.aabbtree_n_nearest(fake_n, [[0, 0, 0]], np.zeros((1, 3)))
        with pytest.raises(ValueError, match="Normals should have same dimensions as points"):
            aabb_normals.aabbtree_n_nearest(fake_n, np.zeros((2, 3)), np.zeros((3, 3)))
        with pytest.raises(ValueError, match="Array must be of a specific type"):
            visibility.visibility_compute(cams=np.zeros((1, 3)), v=v.astype(np.float32), f=f)
    finally:
        fake.ptr = None
        fake_n.ptr = None
    assert issubclass(spatialsearch.Mesh_IntersectionsError, Exception)
    assert issubclass(visibility.VisibilityError, Exception)


def test_null_handles_rejected():
    from mesh_amd import _native
    L = _native.lib()
    face = np.zeros(1, np.uint32)
    pt = np.zeros(3)
    q = np.zeros(3)
    assert L.msh_tree_nearest(None, _native.dptr(q), 1, _native.uptr(face), None, _native.dptr(pt)) == _native.MSH_EINVAL
    assert b"null" in L.msh_last_error()
    assert L.msh_tree_build(_native.dptr(q), 1, _native.uptr(face), 0, ctypes.byref(ctypes.c_void_p())) == \
        _native.MSH_EINVAL  # empty mesh


def test_bad_face_index_rejected_before_device():
    from mesh_amd import _native
    L = _native.lib()
    v = np.zeros((3, 3))
    f = np.array([[0, 1, 7]], np.uint32)
    out = ctypes.c_void_p()
    assert L.msh_tree_build(_native.dptr(v), 3, _native.uptr(f), 1, ctypes.byref(out)) == _native.MSH_EINVAL
    assert b"references vertex 7" in L.msh_last_error()


@pytest.mark.parametrize("mutation", [None, "MUTATE_TREE_TERM", "MUTATE_QUERY_MARGIN", "MUTATE_RAY_MARGIN",
                                      "MUTATE_LINE_DIST"])
def test_child_box_bound_is_conservative(tmp_path, mutation):
    """The traversal's fp32 child-box bound (common.h node_child_bounds with make_qf's margin) never exceeds
    the squared distance from the fp64 query to a point its box contains, and the ray kernels' fp32 slab
    test (make_rayf / ray_child_slabs) takes every child a ray passes a point of, and nearest_alongnormal's
    line test (ray_child_line_dist2) takes it with a key at most the squared distance along the line to that
    point: 300k random and adversarial nodes/queries/rays on a host build of the kernels' own header.  The
    mutated builds (one margin term dropped; the line key taken from the far end) must find violations, which
    shows the cases reach the margins."""
    import subprocess
    exe = str(tmp_path / "bound_check")
    cmd = ["/opt/rocm/bin/hipcc", "-O2", "-std=c++17", "-ffp-contract=off", "--offload-arch=gfx950", "-x", "hip",
           os.path.join(ROOT, "tests", "csrc", "bound_check.cpp"), "-I", os.path.join(ROOT, "mesh_amd", "csrc"),
           "-o", exe]
    if mutation:
        cmd.insert(1, "-D" + mutation)
    subprocess.check_call(cmd)
    out = subprocess.run([exe, "300000"], capture_output=True, text=True, timeout=300)
    line = [x for x in out.stdout.splitlines() if x.startswith("trials=")][-1]
    viol = int(line.split(" violations=")[1].split()[0])
    if mutation is None:
        assert out.returncode == 0 and viol == 0, out.stdout + out.stderr
    else:
        assert out.returncode == 1 and viol > 0, line


def test_batch_build_validation():
    # argument checks run on the host, before any device work
    from mesh_amd import _native
    L = _native.lib()
    v = np.zeros((2, 3, 3))
    f1 = np.array([[0, 1, 2]], np.uint32)
    out = ctypes.c_void_p()
    assert L.msh_batch_build(_native.dptr(v), 2, 3, _native.uptr(f1), 1, ctypes.byref(out)) == _native.MSH_EINVAL
    assert b"T >= 2" in L.msh_last_error()
    f2 = np.array([[0, 1, 2], [0, 2, 9]], np.uint32)
    assert L.msh_batch_build(_native.dptr(v), 2, 3, _native.uptr(f2), 2, ctypes.byref(out)) == _native.MSH_EINVAL
    assert b"references vertex 9" in L.msh_last_error()
    assert L.msh_batch_nearest(None, None, 0, None, None, None) == _native.MSH_EINVAL


def test_batch_python_validation():
    # shape checks of search.AabbTreeBatch happen before any device work
    from mesh_amd.search import AabbTreeBatch
    f = np.array([[0, 1, 2], [0, 2, 3]], np.uint32)
    with pytest.raises(ValueError, match="BxPx3"):
        AabbTreeBatch(np.zeros((4, 3)), f)
    with pytest.raises(ValueError, match="Tx3"):
        AabbTreeBatch(np.zeros((2, 4, 3)), np.zeros((2, 4), np.uint32))


def test_build_id_matches_sources():
    # the loaded library was built from the sources in the tree (profiles are keyed by this identity:
    # profiles/pmc_traffic.json's build_id must equal it for bench.py to report roofline.traffic)
    from mesh_amd import _native
    bid = _native.build_id()
    assert len(bid) == 16 and bid == _native.source_build_id()


@pytest.mark.parametrize("S,G", [(0, 1), (1, 3), (7, 3), (100, 8), (10**8, 8), (2**32 - 1, 7), (5, 8)])
def test_device_plan_matches_shard_range(S, G):
    # the row split of a host-buffer call over a handle's devices (msh_set_devices): contiguous, covering, balanced
    # and identical to the multi-process split (mesh_amd/distributed.py shard_range) — host only, no device
    from mesh_amd import _native
    from mesh_amd.distributed import shard_range
    b = _native.device_plan(S, G)
    assert len(b) == G + 1 and b[0] == 0 and b[-1] == S
    for g in range(G):
        assert (b[g], b[g + 1]) == shard_range(S, g, G)
    sizes = [b[g + 1] - b[g] for g in range(G)]
    assert max(sizes) - min(sizes) <= 1


def test_device_list_validation():
    from mesh_amd import _native
    with pytest.raises((ValueError, RuntimeError)):
        _native.set_devices([0, -1])
    with pytest.raises((ValueError, RuntimeError)):
        _native.device_plan(10, 0)
