"""Development check of the query order (msh_tree_query_order): both sorters against a numpy stable argsort of
the same 24-bit Morton keys (computed here with the kernels' fp32 arithmetic), on C3-stream prefixes.

    python scripts/sort_debug.py
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def keys24(q, lo, hi):
    f = np.float32
    out = np.zeros(q.shape[0], dtype=np.uint32)
    for k in range(3):
        e = f(hi[k]) - f(lo[k])
        n = (q[:, k].astype(f) - f(lo[k])) / e
        n = np.fmin(np.fmax(n * f(1024.0), f(0.0)), f(1023.0)).astype(np.uint32)  # C fminf / fmaxf: NaN -> 0
        v = n.copy()
        v = (v * np.uint32(0x00010001)) & np.uint32(0xFF0000FF)
        v = (v * np.uint32(0x00000101)) & np.uint32(0x0F00F00F)
        v = (v * np.uint32(0x00000011)) & np.uint32(0xC30C30C3)
        v = (v * np.uint32(0x00000005)) & np.uint32(0x49249249)
        out |= v << np.uint32(2 - k)
    return (out >> np.uint32(6)) & np.uint32(0xFFFFFF)


def main():
    import torch
    from mesh_amd import _native, spatialsearch
    import workloads as W
    v, f = W.c3_mesh()
    t = spatialsearch.aabbtree_compute(v, f)
    info = t.info()
    lo, hi = [], []
    for k in range(3):
        e = np.float32(info.scene_hi[k]) - np.float32(info.scene_lo[k])
        lo.append(np.float32(info.scene_lo[k]) - np.float32(0.1) * e)
        hi.append(np.float32(info.scene_hi[k]) + np.float32(0.1) * e)
    sizes = [int(x) for x in (sys.argv[1].split(",") if len(sys.argv) > 1 else
                              ["1000", "4096", "4097", "12345", "100000", "1000000", "4000000"])]
    qa = W.c3_stream(max(sizes), "cuda:0")
    for n in sizes:
        x = qa[:n].contiguous()
        perms = []
        for sorter in (0, 1):
            p = torch.empty(n, dtype=torch.int32, device="cuda:0")
            _native.check(_native.lib().msh_tree_query_order(t.ptr, x.data_ptr(), n, p.data_ptr(), sorter, None))
            torch.cuda.synchronize()
            perms.append(p.cpu().numpy().astype(np.int64))
        kk = keys24(x.cpu().numpy(), lo, hi)
        ref = np.argsort(kk, kind="stable")
        res = []
        for s, p in enumerate(perms):
            ok = np.array_equal(p, ref)
            isperm = np.array_equal(np.sort(p), np.arange(n))
            sorted_keys = bool(np.all(np.diff(kk[p].astype(np.int64)) >= 0)) if isperm else False
            first = int(np.argmax(p != ref)) if not ok else -1
            res.append(dict(sorter=s, equal_ref=ok, is_perm=isperm, keys_sorted=sorted_keys, first_diff=first))
        print(n, res, flush=True)


if __name__ == "__main__":
    main()
