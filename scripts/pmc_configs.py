"""Summarise `TARGET=<cfg> scripts/profile_pmc.sh` (rocprofv3 passes over one scripts/bench_configs.py config)
into profiles/pmc_configs.json, which scripts/bench_configs.py reads to give that config's kernels measured
fabric bytes next to their byte-model figures.

Per kernel (every dispatch of the run, all launches of the config): mean FETCH_SIZE / WRITE_SIZE per dispatch,
HBM bytes per dispatch corrected as MI355X_MICROARCH.md §HBM prescribes for gfx950 ((2 * FETCH_SIZE +
WRITE_SIZE) * 1 KB), the L2 (TCC) hit rate, the mean duration from the --stats pass and the GB/s they imply.
The profiled library's build identity (gpurun_out/pmc_<cfg>/build_id.txt, written on the box) is stored with
them: bench_configs.py attaches a profile only to a library with that identity.

    python scripts/pmc_configs.py --target c5 --code $(git rev-parse --short HEAD)
    python scripts/pmc_configs.py --target c2 --skip 1 --code ...   (drops the entry cut's traversal)
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from scripts.pmc_summary import counters, kernel_stats  # noqa: E402


def summarise(pmc_dir, skip):
    allc = {}
    for p in sorted(os.listdir(pmc_dir)):
        d = os.path.join(pmc_dir, p)
        if os.path.isdir(d) and p != "stats":
            for k, cs in counters(d, skip).items():
                allc.setdefault(k, {}).update(cs)
    stats = kernel_stats(os.path.join(pmc_dir, "stats"), skip)
    out = {}
    for k, cs in allc.items():
        n = max(cs.get("_dispatches", 1), 1)
        per = {c: v / n for c, v in cs.items() if not c.startswith("_")}
        f, w = per.get("FETCH_SIZE"), per.get("WRITE_SIZE")
        hit, miss = per.get("TCC_HIT_sum"), per.get("TCC_MISS_sum")
        b = (2.0 * f + w) * 1024.0 if f is not None and w is not None else None
        calls, tot_ns = stats.get(k, (0, 0.0))
        ns = tot_ns / calls if calls else None
        out[k] = {"dispatches": n, "counters_per_dispatch": per, "hbm_bytes_per_dispatch": b,
                  "hbm_bytes_total": b * n if b is not None else None,
                  "l2_hit_rate": hit / (hit + miss) if hit is not None and miss and hit + miss > 0 else None,
                  "ms_per_dispatch": ns / 1e6 if ns else None,
                  "hbm_GBps": b / ns if b and ns else None}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--target", required=True)
    ap.add_argument("--code", required=True, help="commit whose kernels were profiled")
    ap.add_argument("--pmc", default=None, help="default gpurun_out/pmc_<target>")
    ap.add_argument("--skip", type=int, default=0,
                    help="closest-point traversals at the start of each run to drop (the entry cut's cell centres)")
    args = ap.parse_args()
    pmc = args.pmc or os.path.join(ROOT, "gpurun_out", "pmc_" + args.target)
    with open(os.path.join(pmc, "build_id.txt")) as fh:
        build_id = fh.read().strip()
    path = os.path.join(ROOT, "profiles", "pmc_configs.json")
    try:
        with open(path) as fh:
            allp = json.load(fh)
    except (OSError, ValueError):
        allp = {}
    allp[args.target] = {
        "code": args.code, "build_id": build_id,
        "units": "per dispatch; FETCH_SIZE / WRITE_SIZE in KB as rocprofv3 reports them; gfx950: bytes = "
                 "(2 * FETCH_SIZE + WRITE_SIZE) * 1024 (MI355X_MICROARCH.md §HBM); these count traffic leaving L2 "
                 "(Infinity Cache hits included), so DRAM traffic is at most this",
        "skipped_traversals": args.skip, "kernels": summarise(pmc, args.skip)}
    with open(path, "w") as fh:
        json.dump(allp, fh, indent=1)
    for k, v in allp[args.target]["kernels"].items():
        print(k, {x: v[x] for x in ("dispatches", "hbm_bytes_per_dispatch", "l2_hit_rate", "ms_per_dispatch",
                                    "hbm_GBps")})


if __name__ == "__main__":
    main()
