#!/usr/bin/env python3
"""Time the C3 replication path on one GPU (north_star: "mesh and BVH replicated via RCCL broadcast"):
pack the built tree into one device blob (what rank 0 broadcasts), unpack it on the same device (what every
receiving rank does) and let the receiver's first query build its entry cut.  Prints one JSON line.

    python scripts/replication_timing.py [--reps 5]
"""
import argparse
import json
import os
import sys
import time

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    import torch
    import workloads as W
    from mesh_amd import _native, spatialsearch
    from mesh_amd.distributed import nearest_device
    _native.set_device(0)
    v, f = W.c3_mesh()
    src = spatialsearch.aabbtree_compute(v, f)
    nbytes = _native.blob_size(src)
    q = W.c3_stream(1_000_000, "cuda:0")
    o = (torch.empty(q.shape[0], dtype=torch.int32, device="cuda:0"),
         torch.empty(q.shape[0], dtype=torch.int32, device="cuda:0"),
         torch.empty((q.shape[0], 3), dtype=torch.float64, device="cuda:0"))
    pack, unpack, first, cut = [], [], [], []
    for _ in range(args.reps):
        blob = torch.empty(nbytes, dtype=torch.uint8, device="cuda:0")
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        _native.blob_pack(src, blob.data_ptr())
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        dst = _native.blob_unpack(blob.data_ptr(), blob.numel(), 0)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        nearest_device(dst, q, *o)  # first query: builds the receiver's entry cut, then answers 1M queries
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        pack.append((t1 - t0) * 1e3)
        unpack.append((t2 - t1) * 1e3)
        first.append((t3 - t2) * 1e3)
        cut.append(dst.entry_cut_info()["build_ms"])
        del dst, blob
    med = lambda x: sorted(x)[len(x) // 2]
    print(json.dumps({"what": "C3 tree replication on one MI355X: blob pack (device copy), unpack on the same "
                              "device, receiver's first 1M-query call (entry cut build + queries)",
                      "build_id": _native.build_id(), "faces": int(f.shape[0]), "blob_bytes": nbytes,
                      "src_build_ms": src.info().build_ms,
                      "pack_ms": med(pack), "unpack_ms": med(unpack), "first_query_call_ms": med(first),
                      "entry_cut_build_ms": med(cut), "reps": args.reps,
                      "all": {"pack": pack, "unpack": unpack, "first": first, "cut": cut}}), flush=True)


if __name__ == "__main__":
    main()
