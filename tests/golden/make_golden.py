"""Generate the committed golden fixtures under tests/golden/.

Run in the build container (the one that has /root/reference mounted):

    python tests/golden/make_golden.py

Outputs (data only — inputs and expected outputs, no reference source):
  meshes.npz       vertex/face arrays of the reference's own fixture meshes
                   (/root/reference/data/unittest/*.obj), parsed as the reference's OBJ loader does
                   (`v x y z`, `f a[/t][/n] ...`, 1-based indices)
  ref_tests.json   the literal known answers of the reference's hot-path tests:
                   tests/test_mesh.py:89-109, tests/test_aabb_n_tree.py:29-89,
                   tests/test_visibility.py:13-53, tests/test_intersections.py:27,
                   tests/test_geometry.py:61-104 and tests/test_mesh.py:111-118 (normals, barycentrics)
                   (the icosphere of mesh/sphere.py:19-57 is stored as data too)
  data/*.obj|ply   the reference's own mesh fixture files (native OBJ / PLY reader tests)
  kdtree.npz       scipy.spatial.KDTree answers for ClosestPointTree (search.py:52-65) on the
                   sphere fixture (scipy is the third-party arithmetic that path uses)
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF_DATA = "/root/reference/data/unittest"


def load_obj(path):
    v, f = [], []
    with open(path) as fh:
        for line in fh:
            tok = line.split()
            if not tok:
                continue
            if tok[0] == "v":
                v.append([float(x) for x in tok[1:4]])
            elif tok[0] == "f":
                idx = [int(t.split("/")[0]) - 1 for t in tok[1:]]
                for k in range(1, len(idx) - 1):  # fan-triangulate (all fixtures are triangles)
                    f.append([idx[0], idx[k], idx[k + 1]])
    return np.array(v, dtype=np.float64), np.array(f, dtype=np.uint32)


# mesh/sphere.py:19-57 — 42-vertex / 80-face icosphere used by tests/test_intersections.py
ICO_V = [[0.0000, -1.000, 0.0000], [0.7236, -0.447, 0.5257], [-0.278, -0.447, 0.8506], [-0.894, -0.447, 0.0000],
         [-0.278, -0.447, -0.850], [0.7236, -0.447, -0.525], [0.2765, 0.4472, 0.8506], [-0.723, 0.4472, 0.5257],
         [-0.720, 0.4472, -0.525], [0.2763, 0.4472, -0.850], [0.8945, 0.4472, 0.0000], [0.0000, 1.0000, 0.0000],
         [-0.165, -0.850, 0.4999], [0.4253, -0.850, 0.3090], [0.2629, -0.525, 0.8090], [0.4253, -0.850, -0.309],
         [0.8508, -0.525, 0.0000], [-0.525, -0.850, 0.0000], [-0.688, -0.525, 0.4999], [-0.162, -0.850, -0.499],
         [-0.688, -0.525, -0.499], [0.2628, -0.525, -0.809], [0.9518, 0.0000, -0.309], [0.9510, 0.0000, 0.3090],
         [0.5876, 0.0000, 0.8090], [0.0000, 0.0000, 1.0000], [-0.588, 0.0000, 0.8090], [-0.951, 0.0000, 0.3090],
         [-0.955, 0.0000, -0.309], [-0.587, 0.0000, -0.809], [0.0000, 0.0000, -1.000], [0.5877, 0.0000, -0.809],
         [0.6889, 0.5257, 0.4999], [-0.262, 0.5257, 0.8090], [-0.854, 0.5257, 0.0000], [-0.262, 0.5257, -0.809],
         [0.6889, 0.5257, -0.499], [0.5257, 0.8506, 0.0000], [0.1626, 0.8506, 0.4999], [-0.425, 0.8506, 0.3090],
         [-0.422, 0.8506, -0.309], [0.1624, 0.8506, -0.499]]
ICO_F = [[15, 3, 13], [13, 14, 15], [2, 15, 14], [13, 1, 14], [17, 2, 14], [14, 16, 17], [6, 17, 16], [14, 1, 16],
         [19, 4, 18], [18, 13, 19], [3, 19, 13], [18, 1, 13], [21, 5, 20], [20, 18, 21], [4, 21, 18], [20, 1, 18],
         [22, 6, 16], [16, 20, 22], [5, 22, 20], [16, 1, 20], [24, 2, 17], [17, 23, 24], [11, 24, 23], [23, 17, 6],
         [26, 3, 15], [15, 25, 26], [7, 26, 25], [25, 15, 2], [28, 4, 19], [19, 27, 28], [8, 28, 27], [27, 19, 3],
         [30, 5, 21], [21, 29, 30], [9, 30, 29], [29, 21, 4], [32, 6, 22], [22, 31, 32], [10, 32, 31], [31, 22, 5],
         [33, 7, 25], [25, 24, 33], [11, 33, 24], [24, 25, 2], [34, 8, 27], [27, 26, 34], [7, 34, 26], [26, 27, 3],
         [35, 9, 29], [29, 28, 35], [8, 35, 28], [28, 29, 4], [36, 10, 31], [31, 30, 36], [9, 36, 30], [30, 31, 5],
         [37, 11, 23], [23, 32, 37], [10, 37, 32], [32, 23, 6], [39, 7, 33], [33, 38, 39], [12, 39, 38], [38, 33, 11],
         [40, 8, 34], [34, 39, 40], [12, 40, 39], [39, 34, 7], [41, 9, 35], [35, 40, 41], [12, 41, 40], [40, 35, 8],
         [42, 10, 36], [36, 41, 42], [12, 42, 41], [41, 36, 9], [38, 11, 37], [37, 42, 38], [12, 38, 42], [42, 37, 10]]

REF_TESTS = {
    # tests/test_mesh.py:89-109 (tolerance 1e-6 absolute)
    "test_aabb_tree": {
        "v": [[-36, 37, 8], [5, -36, 35], [12, -15, 1], [-10, -42, -26], [-38, -32, -26], [-8, -45, 40], [44, -1, -1],
              [-16, 40, -13], [-39, 28, -11], [-26, -10, -40], [-37, 44, 46], [8, -44, -27], [-15, 32, -48],
              [-46, -33, 15], [23, 15, -5], [5, -20, 24], [-31, 19, -32], [-13, 13, 28], [-42, 43, 28], [-1, -6, -5]],
        "f": [[12, 16, 17], [5, 10, 1], [13, 19, 7], [13, 1, 5], [14, 8, 16], [9, 2, 8], [1, 19, 18], [4, 0, 3],
              [18, 15, 5], [3, 16, 2]],
        "q": [[-19, 1, 1], [32, 29, 14], [-12, 31, 3], [-15, 44, 38], [5, 12, 9]],
        "v_expected": [[-19.678178, 0.364208, -1.384218], [23.000000, 15.000000, -5.000000],
                       [-13.729523, 19.930467, 0.278131], [-31.869765, 34.228123, 44.656367],
                       [7.794764, 18.188195, -6.471474]],
        "f_expected": [2, 4, 0, 1, 4],
        "tol": 1e-6,
    },
    # tests/test_aabb_n_tree.py:29-52 on test_doublebox.obj (exact equality)
    "test_dist_classic": {"mesh": "test_doublebox", "eps": 0.0,
                          "q": [[0.5, 0.1, 0.25], [0.5, 0.1, 0.25]], "n": [[0.0, 1.0, 0.0], [1.0, 0.0, 0.0]],
                          "f_expected": [[0, 0]], "p_expected": [[0.5, 0.1, 0.25], [0.5, 0.1, 0.25]]},
    "test_dist_normals": {"mesh": "test_doublebox", "eps": 0.5,
                          "q": [[0.5, 0.1, 0.25], [0.5, 0.1, 0.25]], "n": [[0.0, 1.0, 0.0], [1.0, 0.0, 0.0]],
                          "f_expected": [[2, 0]], "p_expected": [[0.5, 0.5, 0.25], [0.5, 0.1, 0.25]]},
    # tests/test_aabb_n_tree.py:54-76: unique closest-face counts (cylinder.obj vs cylinder_trans.obj)
    "test_cylinders": {"eps_no": 0.0, "eps_yes": 10.0, "max_unique_no": 4, "min_unique_yes_slack": 4},
    # tests/test_aabb_n_tree.py:78-89
    "test_selfintersects": {"test_doublebox": 0, "self_intersecting_cyl": 16},
    # tests/test_visibility.py:13-53
    "test_visibility_box": {
        "v": [[0.50, 0.50, 0.50], [-0.5, 0.50, 0.50], [0.50, -0.5, 0.50], [-0.5, -0.5, 0.50], [0.50, 0.50, -0.5],
              [-0.5, 0.50, -0.5], [0.50, -0.5, -0.5], [-0.5, -0.5, -0.5]],
        "f1": [[1, 2, 3], [4, 3, 2], [1, 3, 5], [7, 5, 3], [1, 5, 2], [6, 2, 5], [8, 6, 7], [5, 7, 6], [8, 7, 4],
               [3, 4, 7], [8, 4, 6], [2, 6, 4]],
        "vextra": [[.9, .9, .9], [-.9, .9, .9], [.9, -.9, .9], [-.9, -.9, .9]],
        "fextra1": [[1, 2, 3], [4, 3, 2]],
    },
    # tests/test_geometry.py:70-104: barycentric_coordinates_of_projection vs the old matlab function
    # (columns are points; tolerance 1e-3), plus the single-point call on column 0
    "test_barycentric": {
        "p": [[-120, 48, -30, 88, -80], [71, 102, 29, -114, -291], [161, 72, -78, -106, 142]],
        "q": [[32, -169, 32, -3, 108], [-75, -10, 31, -16, 110], [136, -24, -86, 62, -86]],
        "u": [[8, -1, 37, -108, 109], [-120, 152, -22, 3, 153], [-110, -76, 111, 55, 9]],
        "v": [[-148, 233, -19, -139, -18], [-73, -61, 88, -141, -19], [-105, 74, -76, 48, 141]],
        "b": [[1.5266, -0.8601, 1.3245, 2.4450, 1.3452], [-1.5346, 0.8556, -0.1963, -2.1865, -2.0794],
              [1.0080, 1.0046, -0.1282, 0.7415, 1.7342]],
        "tol": 1e-3,
    },
    # tests/test_mesh.py:111-118: sphere.obj centred; mean |vn - v/rad| < 0.05
    "test_estimate_vertex_normals": {"mesh": "sphere", "mse_max": 0.05},
    # tests/test_geometry.py:61-68: estimate_vertex_normals == VertNormals within 1e-15 (sphere fixture)
    "test_vert_normals": {"mesh": "sphere", "tol": 1e-15},
    # tests/test_mesh.py:17-26,35-47: test_box.obj / test_box.ply loaded by the native readers
    "test_load_box": {
        "v": [[0.5, 0.5, 0.5], [-0.5, 0.5, 0.5], [0.5, -0.5, 0.5], [-0.5, -0.5, 0.5], [0.5, 0.5, -0.5],
              [-0.5, 0.5, -0.5], [0.5, -0.5, -0.5], [-0.5, -0.5, -0.5]],
        "f": [[0, 1, 2], [3, 2, 1], [0, 2, 4], [6, 4, 2], [0, 4, 1], [5, 1, 4], [7, 5, 6], [4, 6, 5], [7, 6, 3],
              [2, 3, 6], [7, 3, 5], [1, 5, 3]],
        "segm": {"a": [0, 1, 2, 3, 4, 5], "b": [6, 10, 11], "c": [7, 8, 9]},
        "landm": {"pospospos": 0, "negnegneg": 7},
    },
    # tests/test_intersections.py:27 (disabled in the reference; verified by brute force in SURVEY §4)
    "test_intersections": {"q_center": [-1, 0, 0], "m_center": [1, 0, 0], "radius": 2,
                           "expected": [2, 4, 5, 6, 16, 25, 26, 27, 36, 37, 38, 40, 58, 60, 61, 63, 76, 77, 79]},
}


def main():
    if not os.path.isdir(REF_DATA):
        sys.exit("reference data dir %s not present; fixtures are already committed" % REF_DATA)
    arrays = {}
    for name in ["sphere", "test_box", "test_doublebox", "cylinder", "cylinder_trans", "self_intersecting_cyl"]:
        v, f = load_obj(os.path.join(REF_DATA, name + ".obj"))
        arrays[name + "_v"] = v
        arrays[name + "_f"] = f
    arrays["icosphere_v"] = np.array(ICO_V, dtype=np.float64)
    arrays["icosphere_f"] = np.array(ICO_F, dtype=np.uint32) - 1
    np.savez_compressed(os.path.join(HERE, "meshes.npz"), **arrays)
    # the reference's mesh files themselves (inputs of the native-reader tests)
    os.makedirs(os.path.join(HERE, "data"), exist_ok=True)
    for name in sorted(os.listdir(REF_DATA)):
        if name.endswith((".obj", ".ply")):
            with open(os.path.join(REF_DATA, name), "rb") as src, open(os.path.join(HERE, "data", name), "wb") as dst:
                dst.write(src.read())
    with open(os.path.join(HERE, "ref_tests.json"), "w") as fh:
        json.dump(REF_TESTS, fh, indent=1)

    # ClosestPointTree goldens (search.py:55-61 uses scipy.spatial.KDTree.query per sample)
    from scipy.spatial import KDTree
    v = arrays["sphere_v"]
    lo, hi = v.min(0), v.max(0)
    ext = hi - lo
    q = np.random.default_rng(11).uniform(lo - 0.1 * ext, hi + 0.1 * ext, (2000, 3))
    d, i = KDTree(v).query(q)
    np.savez_compressed(os.path.join(HERE, "kdtree.npz"), q=q, dist=d, idx=i.astype(np.int64))
    print("wrote meshes.npz, ref_tests.json, kdtree.npz")


if __name__ == "__main__":
    main()
