"""Native OBJ / PLY readers (mesh_amd/csrc/loaders.cpp through the C ABI).

Host parsing only, so these run without a GPU.  Pinned by the reference's own fixtures and known answers
(tests/test_mesh.py:17-47 on data/unittest/test_box.{obj,ply} and test_box_le.ply; tests/golden/data holds
copies of the reference's mesh files), and compared field by field with the oracle's pure-Python
restatements of py_loadobj.cpp / plyutils.c + rply on every fixture and on synthetic files that exercise
the edge cases (polygons, v/vt/vn index forms, groups revisited, landmarks, mtllib, CRLF, comments,
big-endian binary, colours + normals, quads, vertex_index, bad magic / header / truncated body).
"""
import os
import struct

import numpy as np
import pytest

from mesh_amd.serialization import plyutils
from mesh_amd.serialization.loadobj import loadobj

HERE = os.path.dirname(os.path.abspath(__file__))
DATA = os.path.join(HERE, "golden", "data")


def _same_obj(a, b):
    for x, y in zip(a[:6], b[:6]):
        assert x.dtype == y.dtype and x.shape == y.shape and np.array_equal(x, y)
    assert a[6] == b[6]
    assert a[7] == b[7]
    assert list(a[8].keys()) == list(b[8].keys())
    for k in a[8]:
        assert a[8][k].dtype == np.uint32 and np.array_equal(a[8][k], b[8][k])


def test_load_box_known_answer(ref_tests):
    # tests/test_mesh.py:35-41
    t = ref_tests["test_load_box"]
    v, vt, vn, f, ft, fn, mtl, landm, segm = loadobj(os.path.join(DATA, "test_box.obj"))
    assert (v == np.array(t["v"])).all() and (f == np.array(t["f"])).all()
    assert f.dtype == np.uint32 and v.dtype == np.float64
    assert landm == t["landm"]
    assert set(segm) == set(t["segm"]) and all((segm[k] == np.array(t["segm"][k])).all() for k in segm)
    assert vn.shape == (8, 3) and (fn == f).all() and ft.shape == (0, 3) and vt.shape == (0, 3)


@pytest.mark.parametrize("name", ["test_box.ply", "test_box_le.ply"])
def test_load_ply_known_answer(ref_tests, name):
    # tests/test_mesh.py:43-47 (the ascii and the binary little-endian file hold the same box)
    t = ref_tests["test_load_box"]
    res = plyutils.read(os.path.join(DATA, name))
    assert sorted(res) == ["pts", "tri"]
    v = np.array(res["pts"]).T.copy()
    f = np.array(res["tri"]).T.copy()
    assert (v == np.array(t["v"])).all() and (f == np.array(t["f"])).all()


@pytest.mark.parametrize("name", sorted(n for n in os.listdir(DATA) if n.endswith(".obj")))
def test_obj_fixtures_vs_restatement(oracle, meshes, name):
    got = loadobj(os.path.join(DATA, name))
    _same_obj(got, oracle.loadobj(os.path.join(DATA, name)))
    key = name[:-4]
    if key + "_v" in meshes:  # the golden maker's parser of the same files
        assert np.array_equal(got[0], meshes[key + "_v"]) and np.array_equal(got[3], meshes[key + "_f"])


@pytest.mark.parametrize("name", sorted(n for n in os.listdir(DATA) if n.endswith(".ply")))
def test_ply_fixtures_vs_restatement(oracle, name):
    got = plyutils.read(os.path.join(DATA, name))
    want = oracle.ply_read(os.path.join(DATA, name))
    assert got == want


def test_sphere_obj_and_ply_agree():
    v, _, _, f, _, _, _, _, _ = loadobj(os.path.join(DATA, "sphere.obj"))
    pv, ptri, _, _ = plyutils.read_arrays(os.path.join(DATA, "sphere.ply"))
    assert np.array_equal(v, pv) and np.array_equal(f.astype(np.float64), ptri)


OBJ_EDGE = (
    "# comment\n"
    "mtllib  materials/skin.mtl\n"
    "v 1 2 3\n"
    "v 4.5e-1 -2.25 +3.0 1.0\n"          # 4 values: the 4th shifts the rows, as in the reference
    "v\t7 8 9 # trailing comment\n"
    "v 10 11 12abc 13\n"                  # stops at '12abc' after reading 12
    "v 0.1 0.2 0.3\r\n"                   # CRLF
    "v -1 -2 -3\n"
    "vp 1 2 3\n"                          # not a vertex: parsed as 'v' + 'p ...', no number
    "vt 0.5 0.25\n"
    "vt 0.75 1.0\n"
    "vn 0 0 1\n"
    "vn 0 1 0\n"
    "#landmark tip\n"
    "v 5 5 5\n"
    "#landmark tip\n"                     # same name again: the later vertex wins
    "v 6 6 6\n"
    "g first\n"
    "f 1/1/1 2/2/2 3/1/2 4/2/1\n"         # quad -> 2 triangles in f, ft, fn
    "f 2//1 3//2 5//1\n"
    "g second group\n"
    "f 1 2 3 4 5\n"                       # pentagon
    "g first\n"                           # revisited group
    "f 3/1 4/2 5/1\n"
    "f 0 1 2\n"                           # 0 wraps to 0xFFFFFFFF
    "g\n"                                 # short 'g' line: group ''
    "f 6 7 1\n"
    "usemtl skin\n"
)


def test_obj_edge_cases(oracle, tmp_path):
    p = tmp_path / "edge.obj"
    p.write_bytes(OBJ_EDGE.encode())
    got = loadobj(str(p))
    want = oracle.loadobj(str(p))
    _same_obj(got, want)
    v, vt, vn, f, ft, fn, mtl, landm, segm = got
    assert mtl == "  materials/skin.mtl"
    assert vt.shape == (2, 2) and fn.shape[0] == 3 and ft.shape[0] == 3
    assert f.shape == (9, 3) and (f == 0xFFFFFFFF).any()
    assert set(segm) == {"first", "second group", ""} and list(segm["first"]) == [0, 1, 2, 6, 7]
    assert set(landm) == {"tip"} and landm["tip"] == v.shape[0] - 1  # the later "tip" vertex wins


def test_obj_missing_file(tmp_path):
    with pytest.raises(ValueError, match="Could not load file"):
        loadobj(str(tmp_path / "nope.obj"))


def _ply_header(fmt, nv, nf, extra_v=(), face_prop="vertex_indices", ctype="uchar", itype="int"):
    h = ["ply", "format %s 1.0" % fmt, "comment made by a test", "element vertex %d" % nv,
         "property float x", "property float y", "property double z"]
    h += ["property %s %s" % (t, n) for t, n in extra_v]
    h += ["element face %d" % nf, "property list %s %s %s" % (ctype, itype, face_prop),
          "element edge 1", "property int a", "property int b", "end_header"]
    return ("\n".join(h) + "\n").encode()


def _ply_file(fmt, extra=True, face_prop="vertex_indices"):
    rng = np.random.default_rng(3)
    nv, nf = 7, 4
    v = rng.normal(size=(nv, 3)).astype(np.float32).astype(np.float64)
    col = rng.integers(0, 256, size=(nv, 3))
    nrm = rng.normal(size=(nv, 3)).astype(np.float32)
    faces = [[0, 1, 2], [2, 3, 4, 5], [5, 6, 0], [1, 3, 6]]  # one quad: its 4th index is ignored
    extra_v = [("uchar", "red"), ("uchar", "green"), ("uchar", "blue"), ("float", "nx"), ("float", "ny"),
               ("float", "nz")] if extra else []
    out = _ply_header(fmt, nv, nf, extra_v, face_prop)
    if fmt == "ascii":
        rows = []
        for i in range(nv):
            r = ["%r" % float(np.float32(v[i, 0])), "%r" % float(np.float32(v[i, 1])), "%r" % float(v[i, 2])]
            if extra:
                r += [str(int(c)) for c in col[i]] + ["%r" % float(x) for x in nrm[i]]
            rows.append(" ".join(r))
        rows += [" ".join(str(x) for x in [len(fc)] + fc) for fc in faces]
        rows += ["1 2"]
        return out + ("\n".join(rows) + "\n").encode()
    e = "<" if fmt == "binary_little_endian" else ">"
    body = b""
    for i in range(nv):
        body += struct.pack(e + "ffd", v[i, 0], v[i, 1], v[i, 2])
        if extra:
            body += struct.pack(e + "BBBfff", *[int(c) for c in col[i]], *nrm[i])
    for fc in faces:
        body += struct.pack(e + "B" + "i" * len(fc), len(fc), *fc)
    body += struct.pack(e + "ii", 1, 2)
    return out + body


@pytest.mark.parametrize("fmt", ["ascii", "binary_little_endian", "binary_big_endian"])
@pytest.mark.parametrize("extra", [False, True])
@pytest.mark.parametrize("face_prop", ["vertex_indices", "vertex_index"])
def test_ply_synthetic_vs_restatement(oracle, tmp_path, fmt, extra, face_prop):
    p = tmp_path / "t.ply"
    p.write_bytes(_ply_file(fmt, extra, face_prop))
    got = plyutils.read(str(p))
    want = oracle.ply_read(str(p))
    assert got == want
    assert ("color" in got) == extra and ("normals" in got) == extra
    assert got["tri"][0][1] == 2.0 and got["tri"][2][1] == 4.0  # the quad keeps its first three indices


def test_ply_all_formats_agree(tmp_path):
    res = []
    for fmt in ["ascii", "binary_little_endian", "binary_big_endian"]:
        p = tmp_path / (fmt + ".ply")
        p.write_bytes(_ply_file(fmt))
        res.append(plyutils.read(str(p)))
    assert res[0] == res[1] == res[2]


def test_ply_errors(tmp_path):
    bad_magic = tmp_path / "crlf.ply"
    bad_magic.write_bytes(b"ply\r\nformat ascii 1.0\r\nend_header\r\n")  # test_ascii_bad_endings.ply's failure
    with pytest.raises(plyutils.error, match=r"Failed to open PLY file\."):
        plyutils.read(str(bad_magic))
    with pytest.raises(plyutils.error, match=r"Failed to open PLY file\."):
        plyutils.read(str(tmp_path / "missing.ply"))
    bad_header = tmp_path / "hdr.ply"
    bad_header.write_bytes(b"ply\nformat ascii 2.0\nend_header\n")
    with pytest.raises(plyutils.error, match="Bad raw header"):
        plyutils.read(str(bad_header))
    trunc = tmp_path / "trunc.ply"
    trunc.write_bytes(_ply_file("binary_little_endian")[:-9])
    with pytest.raises(plyutils.error, match="Read failed"):
        plyutils.read(str(trunc))
    out_of_range = tmp_path / "range.ply"
    out_of_range.write_bytes(_ply_header("ascii", 1, 0, [("uchar", "red")]) + b"0 0 0 300\n1 2\n")
    with pytest.raises(plyutils.error, match="Read failed"):
        plyutils.read(str(out_of_range))


@pytest.mark.parametrize("count", [b"-1", b"99999999999", b"9223372036854775807", b"99999999999999999999", b"12x"])
@pytest.mark.parametrize("fmt", ["ascii", "binary_little_endian"])
def test_ply_bad_counts(tmp_path, fmt, count):
    # element counts that are negative, unparsable or larger than the bytes after end_header can hold are
    # refused with the module error before anything is allocated (no C++ exception escapes the C ABI)
    body = _ply_file(fmt)
    hdr, rest = body.split(b"end_header\n", 1)
    lines = hdr.split(b"\n")
    lines = [b"element vertex " + count if ln.startswith(b"element vertex") else ln for ln in lines]
    p = tmp_path / "count.ply"
    p.write_bytes(b"\n".join(lines) + b"end_header\n" + rest)
    with pytest.raises(plyutils.error, match="Read failed|Bad raw header"):
        plyutils.read(str(p))
    ok = tmp_path / "ok.ply"  # the unmodified file still reads
    ok.write_bytes(body)
    plyutils.read(str(ok))


@pytest.mark.parametrize("name", ["test_box.obj", "test_box.ply", "test_box_le.ply"])
def test_mesh_from_file(ref_tests, name):
    # tests/test_mesh.py:35-47 through Mesh(filename=...)
    from mesh_amd.mesh import Mesh
    t = ref_tests["test_load_box"]
    m = Mesh(filename=os.path.join(DATA, name))
    assert (m.v == np.array(t["v"])).all() and (m.f == np.array(t["f"])).all()
    if name.endswith(".obj"):
        assert m.landm == t["landm"]
        assert all((m.landm_xyz[k] == np.array(t["v"])[i]).all() for k, i in t["landm"].items())
        assert dict(m.segm) == t["segm"]
