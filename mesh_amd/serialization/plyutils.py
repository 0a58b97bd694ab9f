"""``plyutils.read(filename)`` -> {'pts': [x, y, z], 'tri': [i0, i1, i2], ['color': [r, g, b]],
['normals': [nx, ny, nz]]}: lists of Python floats, as mesh/src/plyutils.c:64-139 returns them (the
caller, serialization.load_from_ply, transposes them into arrays).  ``read_arrays`` returns the same data
as float64 arrays (v (P,3), tri (F,3), colour / normals (P,3) or None) without building Python lists.
The parsing runs in libmeshsearch (msh_ply_*); see loaders.cpp."""
import ctypes

import numpy as np

from .. import _native as N


class error(Exception):
    """Module error object (plyutils.c:17,25)."""


def read_arrays(filename):
    if not isinstance(filename, str):
        raise error("plyutils.read doesn't know what to do without a filename.")
    L = N.lib()
    h = ctypes.c_void_p()
    st = L.msh_ply_load(filename.encode(), ctypes.byref(h))
    if st != N.MSH_OK:
        raise error(L.msh_last_error().decode("utf-8", "replace"))
    try:
        s = np.zeros(4, np.uint64)
        N.check(L.msh_ply_sizes(h, s.ctypes.data_as(N._c_u64_p)))
        nv, nf, has_color, has_normals = (int(x) for x in s)
        v = np.empty((nv, 3))
        tri = np.empty((nf, 3))
        color = np.empty((nv, 3)) if has_color else None
        normals = np.empty((nv, 3)) if has_normals else None
        N.check(L.msh_ply_arrays(h, N.dptr(v), N.dptr(tri), N.dptr(color), N.dptr(normals)))
        return v, tri, color, normals
    finally:
        L.msh_ply_free(h)


def read(filename):
    v, tri, color, normals = read_arrays(filename)
    res = {"pts": [list(c) for c in v.T.tolist()], "tri": [list(c) for c in tri.T.tolist()]}
    if color is not None:
        res["color"] = [list(c) for c in color.T.tolist()]
    if normals is not None:
        res["normals"] = [list(c) for c in normals.T.tolist()]
    return res
