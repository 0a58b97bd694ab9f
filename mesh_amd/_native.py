"""ctypes binding of ``libmeshsearch.so`` (C ABI declared in ``include/meshsearch.h``).

This is the only place that touches the native library.  There is no CPU fallback: if the library is
missing, cannot be loaded, or no HIP device is usable, every call raises.
"""
import ctypes
import os
import threading

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("MESH_AMD_LIB", os.path.join(_HERE, "lib", "libmeshsearch.so"))

MSH_OK, MSH_EINVAL, MSH_EDEVICE, MSH_ENOMEM = 0, 1, 2, 3
NO_FACE = 0xFFFFFFFF

_c_double_p = ctypes.POINTER(ctypes.c_double)
_c_u32_p = ctypes.POINTER(ctypes.c_uint32)
_c_u64_p = ctypes.POINTER(ctypes.c_uint64)
_c_i64_p = ctypes.POINTER(ctypes.c_int64)
_vp = ctypes.c_void_p
_sz = ctypes.c_size_t
_i = ctypes.c_int

_lib = None
_lock = threading.Lock()

# (name, restype, argtypes) for every symbol of include/meshsearch.h
SIGNATURES = [
    ("msh_last_error", ctypes.c_char_p, []),
    ("msh_version", _i, []),
    ("msh_build_id", ctypes.c_char_p, []),
    ("msh_device_count", _i, [ctypes.POINTER(_i)]),
    ("msh_set_device", _i, [_i]),
    ("msh_set_devices", _i, [_i]),
    ("msh_set_device_list", _i, [ctypes.POINTER(_i), _i]),
    ("msh_tree_devices", _i, [_vp, ctypes.POINTER(_i), _i, ctypes.POINTER(_i)]),
    ("msh_device_plan", _i, [ctypes.c_uint64, _i, _c_u64_p]),
    ("msh_tree_build", _i, [_c_double_p, _sz, _c_u32_p, _sz, ctypes.POINTER(_vp)]),
    ("msh_tree_build_ex", _i, [_c_double_p, _sz, _c_u32_p, _sz, _c_double_p, _sz, _c_u32_p, _sz, ctypes.POINTER(_vp)]),
    ("msh_tree_free", None, [_vp]),
    ("msh_tree_get_info", _i, [_vp, _vp]),
    ("msh_tree_nearest", _i, [_vp, _c_double_p, _sz, _c_u32_p, _c_u32_p, _c_double_p]),
    ("msh_tree_nearest_device", _i, [_vp, _vp, _sz, _vp, _vp, _vp, _vp]),
    ("msh_tree_nearest_stats", _i, [_vp, _vp, _sz, _c_u64_p, _c_u64_p]),
    ("msh_tree_nearest_bary", _i, [_vp, _c_double_p, _sz, _c_u32_p, _c_double_p, _c_double_p]),
    ("msh_tree_nearest_bary_device", _i, [_vp, _vp, _sz, _vp, _vp, _vp, _vp]),
    ("msh_tree_points_from_faces_device", _i, [_vp, _vp, _sz, _vp, _vp, _vp, _vp]),
    ("msh_tree_set_entry_cut", _i, [_vp, _i]),
    ("msh_tree_query_order", _i, [_vp, _vp, _sz, _vp, _vp]),
    ("msh_tree_entry_cut_info", _i, [_vp, ctypes.POINTER(_i), ctypes.POINTER(_i), _c_u64_p, ctypes.POINTER(ctypes.c_double)]),
    ("msh_tree_nearest_alongnormal", _i, [_vp, _c_double_p, _c_double_p, _sz, _c_double_p, _c_u32_p, _c_double_p]),
    ("msh_tree_nearest_alongnormal_device", _i, [_vp, _vp, _vp, _sz, _vp, _vp, _vp, _vp]),
    ("msh_tree_nearest_alongnormal_stats", _i, [_vp, _vp, _vp, _sz, _c_u64_p, _c_u64_p]),
    ("msh_visibility_stats", _i, [_vp, _vp, _sz, ctypes.c_double, _c_u64_p, _c_u64_p]),
    ("msh_tree_intersections", _i, [_vp, _c_double_p, _sz, _c_u32_p, _sz, _c_u32_p, ctypes.POINTER(_sz)]),
    ("msh_ntree_build", _i, [_c_double_p, _sz, _c_u32_p, _sz, ctypes.c_double, ctypes.POINTER(_vp)]),
    ("msh_ntree_nearest", _i, [_vp, _c_double_p, _c_double_p, _sz, _c_u32_p, _c_double_p]),
    ("msh_ntree_selfintersects", _i, [_vp, _c_i64_p]),
    ("msh_visibility", _i, [_vp, _c_double_p, _sz, _c_double_p, _c_double_p, ctypes.c_double, _c_u32_p, _c_double_p]),
    ("msh_visibility_device", _i, [_vp, _vp, _sz, _vp, _vp, ctypes.c_double, _sz, _sz, _vp, _vp, _vp]),
    ("msh_vertex_normals", _i, [_c_double_p, _sz, _c_u32_p, _sz, _c_double_p]),
    ("msh_vertex_normals_device", _i, [_vp, _sz, _vp, _sz, _vp, _vp]),
    ("msh_points_build", _i, [_c_double_p, _sz, ctypes.POINTER(_vp)]),
    ("msh_points_nearest", _i, [_vp, _c_double_p, _sz, _c_u32_p, _c_double_p]),
    ("msh_tree_blob_size", _i, [_vp, ctypes.POINTER(_sz)]),
    ("msh_tree_blob_pack", _i, [_vp, _vp, _vp]),
    ("msh_tree_blob_unpack", _i, [_vp, _sz, _i, _vp, ctypes.POINTER(_vp)]),
    ("msh_batch_build", _i, [_c_double_p, _sz, _sz, _c_u32_p, _sz, ctypes.POINTER(_vp)]),
    ("msh_batch_nearest", _i, [_vp, _c_double_p, _sz, _c_u32_p, _c_u32_p, _c_double_p]),
    ("msh_batch_nearest_device", _i, [_vp, _vp, _sz, _vp, _vp, _vp, _vp]),
    ("msh_batch_nearest_bary", _i, [_vp, _c_double_p, _sz, _c_u32_p, _c_double_p, _c_double_p]),
    ("msh_batch_nearest_bary_device", _i, [_vp, _vp, _sz, _vp, _vp, _vp, _vp]),
    ("msh_blob_header_write", _i, [_i, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, _vp, _sz, _vp]),
    ("msh_blob_header_parse", _i, [_vp, _sz, _vp]),
    ("msh_obj_load", _i, [ctypes.c_char_p, ctypes.POINTER(_vp)]),
    ("msh_obj_sizes", _i, [_vp, _c_u64_p]),
    ("msh_obj_arrays", _i, [_vp, _c_double_p, _c_double_p, _c_double_p, _c_u32_p, _c_u32_p, _c_u32_p]),
    ("msh_obj_mtl_path", ctypes.c_char_p, [_vp]),
    ("msh_obj_group", _i, [_vp, _sz, ctypes.POINTER(ctypes.c_char_p), _c_u64_p, ctypes.POINTER(_c_u32_p)]),
    ("msh_obj_landmark", _i, [_vp, _sz, ctypes.POINTER(ctypes.c_char_p), _c_u32_p]),
    ("msh_obj_free", None, [_vp]),
    ("msh_ply_load", _i, [ctypes.c_char_p, ctypes.POINTER(_vp)]),
    ("msh_ply_sizes", _i, [_vp, _c_u64_p]),
    ("msh_ply_arrays", _i, [_vp, _c_double_p, _c_double_p, _c_double_p, _c_double_p]),
    ("msh_ply_free", None, [_vp]),
    ("msh_timing_enable", _i, [_i]),
    ("msh_timing_get", _i, [ctypes.c_char_p, ctypes.POINTER(ctypes.c_double), _c_i64_p]),
    ("msh_timing_reset", _i, []),
    ("msh_host_alloc", _i, [_sz, ctypes.POINTER(_vp)]),
    ("msh_host_free", None, [_vp]),
    ("msh_host_pool_trim", _i, []),
    ("msh_host_pool_bytes", _sz, []),
    ("msh_device_pool_trim", _i, []),
    ("msh_device_pool_bytes", _i, [_c_u64_p, _c_u64_p, _c_u64_p]),
]


class TreeInfo(ctypes.Structure):
    _fields_ = [("device", _i), ("kind", _i), ("n_points", ctypes.c_uint64), ("n_faces", ctypes.c_uint64),
                ("n_main_faces", ctypes.c_uint64), ("n_nodes", ctypes.c_uint64), ("bytes", ctypes.c_uint64),
                ("eps", ctypes.c_double), ("scene_lo", ctypes.c_float * 3), ("scene_hi", ctypes.c_float * 3),
                ("build_ms", ctypes.c_double), ("n_meshes", ctypes.c_uint64), ("node_bytes", ctypes.c_uint32),
                ("leaf_bytes", ctypes.c_uint32), ("max_depth", ctypes.c_int32)]


class BlobInfo(ctypes.Structure):
    """msh_blob_info (include/meshsearch.h): layout of a packed tree blob."""
    _fields_ = [("kind", ctypes.c_int32), ("max_depth", ctypes.c_int32), ("n_points", ctypes.c_uint64),
                ("n_faces", ctypes.c_uint64), ("n_main_faces", ctypes.c_uint64), ("off_vertices", ctypes.c_uint64),
                ("off_nodes", ctypes.c_uint64), ("off_leaves", ctypes.c_uint64), ("total", ctypes.c_uint64),
                ("node_bytes", ctypes.c_uint32), ("leaf_bytes", ctypes.c_uint32), ("origin", ctypes.c_double * 3)]


def _preload_single_hip_runtime():
    """Keep ONE HIP runtime per process.

    PyTorch-ROCm ships its own libamdhip64.so (SONAME libamdhip64.so.7, like /opt/rocm's).  If
    libmeshsearch pulled in /opt/rocm's copy first, a later `import torch` would load a second runtime
    that then fails to initialise ("No HIP GPUs are available").  Loading torch's copy first (without
    importing torch) makes our NEEDED libamdhip64.so.7 resolve to it, so torch and libmeshsearch share
    the runtime, streams and device memory whatever the import order.
    """
    if os.environ.get("MESH_AMD_SYSTEM_HIP"):
        return
    try:
        import importlib.util
        spec = importlib.util.find_spec("torch")
        if spec is None or not spec.submodule_search_locations:
            return
        for d in spec.submodule_search_locations:
            p = os.path.join(d, "lib", "libamdhip64.so")
            if os.path.exists(p):
                ctypes.CDLL(p, mode=ctypes.RTLD_GLOBAL)
                return
    except OSError:
        pass


def lib():
    """Load libmeshsearch.so (raises ImportError if it is missing — no fallback)."""
    global _lib
    if _lib is None:
        with _lock:
            if _lib is None:
                if not os.path.exists(LIB_PATH):
                    raise ImportError("libmeshsearch.so not built (%s): run `python -c 'import __graft_entry__ as g; "
                                      "g.build()'` or `make -C mesh_amd/csrc`" % LIB_PATH)
                _preload_single_hip_runtime()
                L = ctypes.CDLL(LIB_PATH)
                for name, res, args in SIGNATURES:
                    # an older build (MESH_AMD_LIB A/B variants) may lack newer entry points: they stay unbound
                    # (tests/test_abi.py checks that the in-tree library exports every header symbol)
                    fn = getattr(L, name, None)
                    if fn is None:
                        continue
                    fn.restype = res
                    fn.argtypes = args
                _lib = L
    return _lib


def check(status, exc_value=ValueError):
    if status == MSH_OK:
        return
    msg = lib().msh_last_error().decode("utf-8", "replace")
    if status == MSH_EINVAL:
        raise exc_value(msg)
    raise RuntimeError(msg)


def dptr(a):
    return a.ctypes.data_as(_c_double_p) if a is not None else None


def uptr(a):
    return a.ctypes.data_as(_c_u32_p) if a is not None else None


# Results of a host-buffer call of at least this many bytes are carved from the library's page-locked pool
PINNED_MIN_BYTES = 32 << 20


class _PinnedBlock(object):
    """One msh_host_alloc block seen as a uint8 buffer; numpy arrays over it keep it alive, and it goes back
    to the pool (msh_host_free) when the last of them dies."""

    def __init__(self, ptr, nbytes):
        self.ptr = ptr
        self.__array_interface__ = {"data": (ptr, False), "shape": (nbytes,), "typestr": "|u1", "version": 3}

    def __del__(self):
        try:
            if self.ptr and _lib is not None:
                _lib.msh_host_free(self.ptr)
        except Exception:
            pass
        self.ptr = None


def empty_results(*specs):
    """Result arrays of one host call, ``[(shape, dtype), ...]`` -> arrays as ``np.empty`` gives them.

    A call with >= PINNED_MIN_BYTES of results gets them from one block of the library's page-locked pool
    (msh_host_alloc), so the host-buffer entry point downloads from HBM straight into them instead of through
    a staging slab, and the first touch of fresh pages is paid once per pool block instead of once per call
    (C3: 3.2 GB of results per 100M queries).  When the pool is disabled (MESH_AMD_PINNED_POOL_MB=0) or full,
    the arrays are ordinary pageable ones."""
    sizes = [int(np.prod(shape, dtype=np.int64)) * np.dtype(dt).itemsize for shape, dt in specs]
    pads = [(s + 255) // 256 * 256 for s in sizes]
    total = sum(pads)
    if total >= PINNED_MIN_BYTES:
        p = _vp()
        if lib().msh_host_alloc(total, ctypes.byref(p)) == MSH_OK and p.value:
            raw = np.asarray(_PinnedBlock(p.value, total))
            out, off = [], 0
            for (shape, dt), s, pad in zip(specs, sizes, pads):
                out.append(raw[off:off + s].view(dt).reshape(shape))
                off += pad
            return out
    return [np.empty(shape, dt) for shape, dt in specs]


class Handle(object):
    """Owning reference to an ``msh_tree*`` (the reference's PyCapsule, spatialsearchmodule.cpp:125)."""

    __slots__ = ("ptr", "kind", "__weakref__")

    def __init__(self, ptr, kind):
        self.ptr = ptr
        self.kind = kind

    def info(self):
        inf = TreeInfo()
        check(lib().msh_tree_get_info(self.ptr, ctypes.byref(inf)))
        return inf

    def set_entry_cut(self, G=-1):
        """msh_tree_set_entry_cut: G < 0 the fine automatic grid (~64 cells per face), 0 none, > 0 G^3 cells; built by
        the next closest-point query whatever its size (without this call the handle gets the coarse automatic grid,
        ~8 cells per face, once its queries number 1/16 of its cells, and the fine one after 16 rows per fine cell)."""
        check(lib().msh_tree_set_entry_cut(self.ptr, int(G)))

    CUT_STATES = {0: "pending", 1: "built", 2: "off", 3: "failed"}

    def entry_cut_info(self):
        """msh_tree_entry_cut_info -> dict(state, G, bytes, build_ms)"""
        st, g, nb, ms = _i(0), _i(0), ctypes.c_uint64(0), ctypes.c_double(0)
        check(lib().msh_tree_entry_cut_info(self.ptr, ctypes.byref(st), ctypes.byref(g), ctypes.byref(nb),
                                            ctypes.byref(ms)))
        return {"state": self.CUT_STATES.get(st.value, st.value), "G": g.value, "bytes": nb.value,
                "build_ms": ms.value}

    def free(self):
        if self.ptr:
            lib().msh_tree_free(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass

    def __repr__(self):
        return "<meshsearch tree kind=%s at 0x%x>" % (self.kind, self.ptr or 0)


def build_id():
    """Identity of the loaded libmeshsearch.so's kernels (msh_build_id): SHA-256 prefix of its sources."""
    return lib().msh_build_id().decode()


def source_build_id(extra=""):
    """The build identity the current mesh_amd/csrc sources would get (the Makefile's SRC_HASH)."""
    import hashlib
    import os
    csrc = os.path.join(os.path.dirname(os.path.abspath(__file__)), "csrc")
    names = sorted(["sort.hip", "build.hip", "refine.hip", "nearest.hip", "rays.hip", "tritri.hip", "geometry.hip", "api.cpp",
                    "loaders.cpp", "common.h", "internal.h"])
    h = hashlib.sha256()
    for p in [os.path.join(csrc, n) for n in names] + [os.path.join(csrc, "..", "..", "include", "meshsearch.h")]:
        with open(p, "rb") as fh:
            h.update(fh.read())
    h.update(extra.encode())
    return h.hexdigest()[:16]


def device_count():
    n = ctypes.c_int(0)
    st = lib().msh_device_count(ctypes.byref(n))
    return n.value if st == MSH_OK else 0


def set_device(device):
    check(lib().msh_set_device(int(device)))


def set_devices(devices):
    """Devices of the trees built next on this thread: an int G (G devices from the current one,
    msh_set_devices) or a list of device ordinals (msh_set_device_list; entries may repeat).  Host-buffer calls
    on those trees split their rows over the devices."""
    if isinstance(devices, int):
        check(lib().msh_set_devices(devices))
        return
    arr = (ctypes.c_int * max(1, len(devices)))(*devices)
    check(lib().msh_set_device_list(arr, len(devices)))


def tree_devices(h):
    """msh_tree_devices -> the device ordinals of a handle and its replicas"""
    g = ctypes.c_int(0)
    check(lib().msh_tree_devices(h.ptr, None, 0, ctypes.byref(g)))
    arr = (ctypes.c_int * g.value)()
    check(lib().msh_tree_devices(h.ptr, arr, g.value, ctypes.byref(g)))
    return list(arr)


def device_plan(S, G):
    """msh_device_plan: row boundaries begins[0..G] of S rows split over G devices"""
    out = (ctypes.c_uint64 * (G + 1))()
    check(lib().msh_device_plan(int(S), int(G), out))
    return list(out)


def build_tree(v, f, extra_v=None, extra_f=None):
    out = _vp()
    if extra_v is not None and extra_f is not None:
        check(lib().msh_tree_build_ex(dptr(v), v.shape[0], uptr(f), f.shape[0], dptr(extra_v), extra_v.shape[0],
                                      uptr(extra_f), extra_f.shape[0], ctypes.byref(out)))
    else:
        check(lib().msh_tree_build(dptr(v), v.shape[0], uptr(f), f.shape[0], ctypes.byref(out)))
    return Handle(out.value, "triangles")


def build_ntree(v, f, eps):
    out = _vp()
    check(lib().msh_ntree_build(dptr(v), v.shape[0], uptr(f), f.shape[0], float(eps), ctypes.byref(out)))
    return Handle(out.value, "normals")


def build_batch(v, f):
    """B meshes sharing the faces f: v (B,P,3) float64 C-contiguous, f (T,3) uint32."""
    out = _vp()
    check(lib().msh_batch_build(dptr(v), v.shape[0], v.shape[1], uptr(f), f.shape[0], ctypes.byref(out)))
    return Handle(out.value, "batch")


def build_points(v):
    out = _vp()
    check(lib().msh_points_build(dptr(v), v.shape[0], ctypes.byref(out)))
    return Handle(out.value, "points")


def blob_size(h):
    n = _sz(0)
    check(lib().msh_tree_blob_size(h.ptr, ctypes.byref(n)))
    return n.value


def blob_pack(h, d_dst, stream=None):
    check(lib().msh_tree_blob_pack(h.ptr, _vp(d_dst), _vp(stream) if stream else None))


def blob_unpack(d_src, nbytes, device, stream=None, kind="triangles"):
    out = _vp()
    check(lib().msh_tree_blob_unpack(_vp(d_src), nbytes, int(device), _vp(stream) if stream else None,
                                     ctypes.byref(out)))
    return Handle(out.value, kind)


def device_pool_trim():
    """msh_device_pool_trim: free the idle query workspace and staging slabs kept between handles."""
    check(lib().msh_device_pool_trim())


def device_pool_bytes():
    """msh_device_pool_bytes -> (workspace, staging, cached block) bytes kept on the devices between handles."""
    w, s, c = ctypes.c_uint64(0), ctypes.c_uint64(0), ctypes.c_uint64(0)
    check(lib().msh_device_pool_bytes(ctypes.byref(w), ctypes.byref(s), ctypes.byref(c)))
    return w.value, s.value, c.value


def timing_enable(on=True):
    check(lib().msh_timing_enable(1 if on else 0))


def timing_get(name):
    ms = ctypes.c_double(0)
    n = ctypes.c_int64(0)
    check(lib().msh_timing_get(name.encode(), ctypes.byref(ms), ctypes.byref(n)))
    return ms.value, n.value


def timing_reset():
    check(lib().msh_timing_reset())


def as_f64_nx3(a, name="Input"):
    a = np.ascontiguousarray(a, dtype=np.float64)
    if a.ndim != 2 or a.shape[1] != 3:
        raise ValueError("%s must be Nx3" % name)
    return a
