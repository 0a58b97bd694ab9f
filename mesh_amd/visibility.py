"""Drop-in for the ``psbody.mesh.visibility`` extension (mesh/src/py_visibility.cpp, visibility.cpp).

``visibility_compute(cams, v=None, f=None, tree=None, n=None, sensors=None, extra_v=None,
extra_f=None, min_dist=1e-3) -> (vis (C,P) uint32, n_dot_cam (C,P) float64)`` — for every camera c and
main-mesh vertex v, vis = 1 iff the closed ray from v + min_dist*dir towards the camera misses every
triangle (main + extra mesh), optionally gated by the sensor-plane test (visibility.cpp:96-111).
Deliberate differences: a ``tree=`` handle is borrowed and never freed
(reference double-frees it, py_visibility.cpp:212); n_dot_cam is zero-filled when ``n`` is absent
(reference: uninitialised, visibility.cpp:94-95).
"""
import numpy as np

from . import _native as N


class VisibilityError(Exception):
    """Module error object (py_visibility.cpp:22,52-54)."""


def _parse(a, dtype):
    # parse_pyarray (py_visibility.cpp:64-79)
    if not isinstance(a, np.ndarray) or a.dtype != dtype or a.ndim != 2:
        raise ValueError("Array must be of a specific type, and 2 dimensional")
    if a.shape[1] != 3:
        raise ValueError("Array must be Nx3")
    return np.ascontiguousarray(a)


def visibility_compute(cams=None, v=None, f=None, tree=None, n=None, sensors=None, extra_v=None, extra_f=None,
                       min_dist=1e-3):
    if cams is None:
        raise TypeError("visibility_compute() missing required argument 'cams'")
    if not isinstance(cams, np.ndarray):
        raise TypeError("visibility_compute() argument 'cams' must be numpy.ndarray")
    if tree is not None:
        if not isinstance(tree, N.Handle) or tree.kind == "points" or tree.ptr is None:
            raise TypeError("visibility_compute: tree must be a handle from aabbtree_compute")
        handle = tree
    else:
        vv = _parse(v, np.float64)
        ff = _parse(f, np.uint32)
        if extra_v is not None and extra_f is not None:
            ev = _parse(extra_v, np.float64)
            ef = _parse(extra_f, np.uint32)
            handle = N.build_tree(vv, ff, ev, ef)
        else:
            handle = N.build_tree(vv, ff)
    if cams.dtype != np.float64 or cams.ndim != 2:
        raise ValueError("Camera positions must be of type double, and 2 dimensional")
    if cams.shape[1] != 3:
        raise ValueError("Cams must be Nx3")
    cams = np.ascontiguousarray(cams)
    P = int(handle.info().n_points)
    C = cams.shape[0]
    nn = None
    if n is not None:
        n = np.asarray(n)
        if n.ndim != 2 or n.shape[1] != 3 or n.shape[0] != P:
            raise ValueError("Normals should have same number of rows as vertices, and 3 columns")
        nn = np.ascontiguousarray(n, dtype=np.float64)
    ss = None
    if sensors is not None:
        sensors = np.asarray(sensors)
        if sensors.ndim != 2 or sensors.shape[1] != 9 or sensors.shape[0] != C:
            raise ValueError("Sensors should have same number of rows as cameras, 3x3 columns")
        ss = np.ascontiguousarray(sensors, dtype=np.float64)
    # large results come from the library's page-locked pool (downloaded straight into place, no page faults)
    vis, ndc = N.empty_results(((C, P), np.uint32), ((C, P), np.float64))
    N.check(N.lib().msh_visibility(handle.ptr, N.dptr(cams), C, N.dptr(nn), N.dptr(ss), float(min_dist), N.uptr(vis),
                                   N.dptr(ndc)), VisibilityError)
    return vis, ndc
