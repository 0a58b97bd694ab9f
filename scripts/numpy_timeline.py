"""Timeline of one C3 call through the numpy entry point (aabbtree_nearest: 100M host queries in, host arrays
out), for finding what serialises the host path: run it under

    rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/nptl -o run -- \
        python3 scripts/numpy_timeline.py

then `python scripts/numpy_timeline.py --parse gpurun_out/nptl` prints, for the last call, every copy and kernel
with its start / end relative to the call's first event, bytes and GB/s, and the busy time of each engine.
"""
import argparse
import csv
import glob
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(n, calls):
    from mesh_amd import _native, spatialsearch
    import workloads as W
    _native.set_device(0)
    v, f = W.c3_mesh()
    q = np.random.default_rng(3).uniform(-1.1, 1.1, (n, 3))
    tree = spatialsearch.aabbtree_compute(v, f)
    outs = []
    for k in range(calls):
        _native.timing_reset()
        _native.timing_enable(True)
        t0 = time.perf_counter()
        outs.append(spatialsearch.aabbtree_nearest(tree, q))
        outs = outs[-2:]  # a caller holding its previous result while it asks for the next
        wall = (time.perf_counter() - t0) * 1e3
        _native.timing_enable(False)
        parts = {name: _native.timing_get(name) for name in ("host_copy", "host_wait", "nearest", "sort")}
        print("call %d: %.1f ms  %s" % (k, wall, "  ".join("%s %.1f ms / %d" % (n, ms, c) for n, (ms, c) in
                                                              parts.items())), flush=True)


def parse(d):
    ev = []
    for path in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(path)):
            ev.append(("K", r["Kernel_Name"][:40], int(r["Start_Timestamp"]), int(r["End_Timestamp"]), 0))
    for path in glob.glob(os.path.join(d, "**", "*memory_copy_trace.csv"), recursive=True):
        for r in csv.DictReader(open(path)):
            ev.append(("C", r.get("Direction", "?"), int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                       int(r.get("Bytes") or 0)))
    ev.sort(key=lambda e: e[2])
    # the last call: events after the largest gap of > 20 ms between consecutive event starts
    starts = [e[2] for e in ev]
    cut = 0
    for i in range(1, len(starts)):
        if starts[i] - starts[i - 1] > 20_000_000:
            cut = i
    last = ev[cut:]
    t0 = last[0][2]
    busy = {}
    for kind, name, s, e, b in last:
        key = name if kind == "C" else "kernels"
        busy[key] = busy.get(key, 0) + (e - s)
        print("%s %-42s %9.2f %9.2f ms %8.1f MB %7.1f GB/s" % (kind, name, (s - t0) / 1e6, (e - t0) / 1e6, b / 1e6,
                                                               (b / (e - s)) if b and e > s else 0.0))
    print("span %.2f ms" % ((max(e[3] for e in last) - t0) / 1e6))
    for k, v in busy.items():
        print("busy %-30s %.2f ms" % (k, v / 1e6))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--parse", default=None)
    ap.add_argument("--queries", type=int, default=100_000_000)
    ap.add_argument("--calls", type=int, default=3)
    a = ap.parse_args()
    if a.parse:
        parse(a.parse)
    else:
        run(a.queries, a.calls)


if __name__ == "__main__":
    main()
