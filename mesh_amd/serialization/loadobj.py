"""``loadobj(obj_path)`` -> (v, vt, vn, f, ft, fn, mtl_path, landm, segm), as mesh/src/py_loadobj.cpp:62-243
returns them: float64 (n,3) v / vn, (n, k) vt, uint32 (n,3) f / ft / fn, the mtllib path as written after
"mtllib" (leading space kept), landmark name -> vertex index, group name -> uint32 face indices.
The parsing runs in libmeshsearch (msh_obj_*); see loaders.cpp for the line semantics."""
import ctypes

import numpy as np

from .. import _native as N


class LoadObjError(Exception):
    """Module error object (py_loadobj.cpp:34,54)."""


def loadobj(obj_path):
    if not isinstance(obj_path, str):
        raise TypeError("loadobj() argument 'obj_path' must be str")
    L = N.lib()
    h = ctypes.c_void_p()
    N.check(L.msh_obj_load(obj_path.encode(), ctypes.byref(h)))
    try:
        s = np.zeros(9, np.uint64)
        N.check(L.msh_obj_sizes(h, s.ctypes.data_as(N._c_u64_p)))
        nv, nvt, lvt, nvn, nf, nft, nfn, ng, nl = (int(x) for x in s)
        v = np.empty((nv, 3))
        vt = np.empty((nvt, lvt))
        vn = np.empty((nvn, 3))
        f = np.empty((nf, 3), np.uint32)
        ft = np.empty((nft, 3), np.uint32)
        fn = np.empty((nfn, 3), np.uint32)
        N.check(L.msh_obj_arrays(h, N.dptr(v), N.dptr(vt), N.dptr(vn), N.uptr(f), N.uptr(ft), N.uptr(fn)))
        mtl_path = L.msh_obj_mtl_path(h).decode("utf-8", "surrogateescape")
        landm = {}
        name = ctypes.c_char_p()
        for k in range(nl):
            idx = ctypes.c_uint32(0)
            N.check(L.msh_obj_landmark(h, k, ctypes.byref(name), ctypes.byref(idx)))
            landm[name.value.decode("utf-8", "surrogateescape")] = int(idx.value)
        segm = {}
        for k in range(ng):
            n = ctypes.c_uint64(0)
            faces = N._c_u32_p()
            N.check(L.msh_obj_group(h, k, ctypes.byref(name), ctypes.byref(n), ctypes.byref(faces)))
            arr = np.ctypeslib.as_array(faces, shape=(int(n.value),)).copy() if n.value else np.empty(0, np.uint32)
            segm[name.value.decode("utf-8", "surrogateescape")] = arr
        return v, vt, vn, f, ft, fn, mtl_path, landm, segm
    finally:
        L.msh_obj_free(h)
