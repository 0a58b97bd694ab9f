"""The closest-point path's query order (msh_tree_query_order) against numpy's stable argsort of the same 24-bit
Morton keys, computed here with the kernel's fp32 arithmetic (k_query_morton / common.h query_morton30), on prefixes
of the C3 stream.  tests/test_gpu_parity.py uses keys24 and sort_box.

    python scripts/sort_debug.py [n1,n2,...]
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


def hilbert24(keys):
    """24-bit Hilbert indices of the 256^3 cells whose 24-bit Morton codes are `keys` (sort.hip hilbert24: Skilling's
    axes-to-transpose, then the transposed bits interleaved, axis 0 first)"""
    keys = np.asarray(keys, dtype=np.uint32)

    def axis(m, k):
        v = (m >> np.uint32(k)) & np.uint32(0x00249249)
        v = (v | (v >> np.uint32(2))) & np.uint32(0x000C30C3)
        v = (v | (v >> np.uint32(4))) & np.uint32(0x0000F00F)
        v = (v | (v >> np.uint32(8))) & np.uint32(0x000000FF)
        return v

    X = [axis(keys, 2), axis(keys, 1), axis(keys, 0)]
    Q = 128
    while Q > 1:
        P = np.uint32(Q - 1)
        for i in range(3):
            m = (X[i] & np.uint32(Q)) != 0
            x0 = np.where(m, X[0] ^ P, X[0])
            t = np.where(m, np.uint32(0), (X[0] ^ X[i]) & P)
            if i == 0:
                X[0] = x0
            else:
                X[0] = x0 ^ t
                X[i] = X[i] ^ t
        Q >>= 1
    X[1] = X[1] ^ X[0]
    X[2] = X[2] ^ X[1]
    t = np.zeros_like(X[2])
    Q = 128
    while Q > 1:
        t = np.where((X[2] & np.uint32(Q)) != 0, t ^ np.uint32(Q - 1), t)
        Q >>= 1
    X = [x ^ t for x in X]

    def spread(v):
        v = (v | (v << np.uint32(8))) & np.uint32(0x0000F00F)
        v = (v | (v << np.uint32(4))) & np.uint32(0x000C30C3)
        v = (v | (v << np.uint32(2))) & np.uint32(0x00249249)
        return v

    return (spread(X[0]) << np.uint32(2)) | (spread(X[1]) << np.uint32(1)) | spread(X[2])


def order_keys(q, lo, hi):
    """the keys the query order sorts by (sort.hip k_qkeys): Hilbert indices of the 24-bit Morton cells"""
    return hilbert24(keys24(q, lo, hi))


def sort_box(info):
    """The cells of query_morton: the tree's scene box widened by 10 % of its extent per side, in fp32."""
    lo, hi = [], []
    for k in range(3):
        e = np.float32(info.scene_hi[k]) - np.float32(info.scene_lo[k])
        lo.append(np.float32(info.scene_lo[k]) - np.float32(0.1) * e)
        hi.append(np.float32(info.scene_hi[k]) + np.float32(0.1) * e)
    return lo, hi


def main():
    import torch
    from mesh_amd import _native, spatialsearch
    import workloads as W
    v, f = W.c3_mesh()
    t = spatialsearch.aabbtree_compute(v, f)
    lo, hi = sort_box(t.info())
    sizes = [int(x) for x in (sys.argv[1].split(",") if len(sys.argv) > 1 else
                              ["1000", "4096", "4097", "12345", "100000", "1000000", "4000000"])]
    qa = W.c3_stream(max(sizes), "cuda:0")
    for n in sizes:
        x = qa[:n].contiguous()
        p = torch.empty(n, dtype=torch.int32, device="cuda:0")
        _native.check(_native.lib().msh_tree_query_order(t.ptr, x.data_ptr(), n, p.data_ptr(),
                                                         torch.cuda.current_stream().cuda_stream))
        torch.cuda.synchronize()
        p = p.cpu().numpy().astype(np.int64)
        ref = np.argsort(order_keys(x.cpu().numpy(), lo, hi), kind="stable")
        print(n, "equal to the stable argsort:", bool(np.array_equal(p, ref)), flush=True)


if __name__ == "__main__":
    main()
