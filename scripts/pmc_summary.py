"""Summarise the rocprofv3 passes of scripts/profile_pmc.sh into profiles/.

Reads gpurun_out/pmc/<pass>/**/*counter_collection.csv (one --pmc pass per counter group) and
*kernel_stats.csv (the --stats pass), and writes:
  profiles/pmc_traffic.json  — what bench.py reads for roofline.traffic: HBM bytes per launch of the
                               closest-point traversal (k_knn<0,false> pass 1 + k_knn_coop<0,false> pass 2),
                               corrected as MI355X_MICROARCH.md §HBM prescribes (gfx950 FETCH_SIZE counts a
                               coalesced 128-B request as 64 B: bytes = 2 * FETCH_SIZE + WRITE_SIZE, KB units),
                               L2 hit rate, and per-kernel counter means;
  profiles/<tag>_pmc.json    — every counter mean per kernel (all passes), for the record.

    python scripts/pmc_summary.py --tag r03_c3_100M --code $(git rev-parse --short HEAD) [--queries 1e8]

The profiled library's build identity (msh_build_id, written to gpurun_out/pmc/build_id.txt on the box)
is stored as build_id: bench.py reports roofline.traffic only for a library with that identity.
"""
import argparse
import csv
import glob
import json
import os
import re
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TRAVERSAL = ("msh::k_knn<0, false, true, true>", "msh::k_knn_coop<0, false>")


def sys_path_root():
    import sys
    if ROOT not in sys.path:
        sys.path.insert(0, ROOT)


def short(name):
    m = re.search(r"(msh::[A-Za-z_0-9]+(<[^>]*>)?)", name)
    return m.group(1) if m else name


def skip_build(rows, skip):
    """Drop the traversal dispatches of the first `skip` traversals of a run (the tree build answers the entry
    cut's cell centres with the same kernels before the bench starts): every TRAVERSAL row whose dispatch id is
    <= that of the skip-th pass-2 dispatch."""
    if skip <= 0:
        return rows
    coop = sorted({int(r["Dispatch_Id"]) for r in rows if short(r.get("Kernel_Name", "")) == TRAVERSAL[1]})
    if len(coop) < skip:
        return rows
    last = coop[skip - 1]
    return [r for r in rows if not (short(r.get("Kernel_Name", "")) in TRAVERSAL and int(r["Dispatch_Id"]) <= last)]


def counters(pmc_dir, skip=0):
    """{kernel: {counter: total over dispatches, '_dispatches': n}} over every *counter_collection.csv
    under pmc_dir (per-dispatch rows of one counter are summed first)."""
    vals = defaultdict(lambda: defaultdict(lambda: defaultdict(float)))  # kernel -> counter -> dispatch -> sum
    vgpr = {}
    for path in glob.glob(os.path.join(pmc_dir, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as fh:
            rows = skip_build(list(csv.DictReader(fh)), skip)
            for row in rows:
                k = short(row.get("Kernel_Name", ""))
                c = row.get("Counter_Name")
                d = (path, row.get("Dispatch_Id") or row.get("Correlation_Id"))
                vals[k][c][d] += float(row.get("Counter_Value") or 0.0)
                if row.get("VGPR_Count"):
                    # raw rocprofv3 fields: on gfx950 its VGPR_Count decodes the kernel descriptor's granulated
                    # count with a granule of 4 where gfx950 allocates in granules of 8 (a 128-VGPR kernel reads
                    # 64), so the register figures of record come from the ISA (isa_of_build below)
                    vgpr[k] = {"VGPR_Count_rocprof_raw": int(float(row["VGPR_Count"])),
                               "Accum_VGPR_Count": int(float(row.get("Accum_VGPR_Count") or 0)),
                               "SGPR_Count": int(float(row.get("SGPR_Count") or 0)),
                               "LDS_Block_Size": int(float(row.get("LDS_Block_Size") or 0)),
                               "Scratch_Size_per_lane": int(float(row.get("Scratch_Size") or 0))}
    out = {}
    for k, cs in vals.items():
        out[k] = {c: sum(ds.values()) for c, ds in cs.items()}
        out[k]["_dispatches"] = max(len(ds) for ds in cs.values())
        if k in vgpr:
            out[k]["_launch_fields"] = vgpr[k]
    return out


def kernel_stats(stats_dir, skip=0):
    """{kernel: (calls, total ns)} from the --stats pass's kernel trace (build traversals dropped)."""
    out = {}
    for path in glob.glob(os.path.join(stats_dir, "**", "*kernel_trace.csv"), recursive=True):
        with open(path) as fh:
            for row in skip_build(list(csv.DictReader(fh)), skip):
                k = short(row["Kernel_Name"])
                c, ns = out.get(k, (0, 0.0))
                out[k] = (c + 1, ns + float(row["End_Timestamp"]) - float(row["Start_Timestamp"]))
    return out


def isa_of_build(build_id):
    """Register allocation of the pass-1 kernel from the gfx950 ISA of the current sources (scripts/isa_check.py:
    .vgpr_count, .vgpr_spill_count, scratch instructions), recorded only when those sources are the profiled build."""
    import sys
    sys.path.insert(0, ROOT)
    from mesh_amd import _native
    from scripts import isa_check
    if _native.source_build_id() != build_id:
        return {"note": "sources differ from the profiled build %s: ISA not recorded" % build_id}
    try:
        isa_check.LIST = True
        return dict(isa_check.report(isa_check.compile_asm([]), 0), kernel=TRAVERSAL[0])
    except Exception as e:  # hipcc missing: leave the field empty rather than fail the summary
        return {"note": "ISA check failed: %s" % e}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pmc", default=os.path.join(ROOT, "gpurun_out", "pmc"))
    ap.add_argument("--tag", required=True)
    ap.add_argument("--code", required=True, help="commit whose kernels were profiled")
    ap.add_argument("--build-id", default=None,
                    help="msh_build_id of the profiled library (default: gpurun_out/pmc/build_id.txt, written on "
                         "the box by profile_pmc.sh)")
    ap.add_argument("--queries", type=float, default=1e8)
    ap.add_argument("--freq", type=int, default=224)
    ap.add_argument("--build-traversals", type=int, default=2,
                    help="traversals per run that belong to the tree build (the entry cut's cell centres: since round 6 "
                         "the coarse grid's, then the fine grid's), dropped")
    args = ap.parse_args()
    S = int(args.queries)
    allc = {}
    for p in sorted(os.listdir(args.pmc)):
        d = os.path.join(args.pmc, p)
        if os.path.isdir(d) and p != "stats":
            for k, cs in counters(d, args.build_traversals).items():
                allc.setdefault(k, {}).update(cs)
    stats = kernel_stats(os.path.join(args.pmc, "stats"), args.build_traversals)
    T = 20 * args.freq ** 2
    sys_path_root()
    import workloads
    workload = workloads.c3_workload_name(args.freq, S)
    # one traversal = the pass-1 launches (leaders + followers) + one pass-2 launch: normalise every
    # figure per traversal by the number of pass-2 dispatches
    coop = TRAVERSAL[1]
    n_trav = allc.get(coop, {}).get("_dispatches", 1)
    n_trav_stats = stats.get(coop, (1, 0.0))[0]
    kern = {}
    tot_bytes, hit, miss, tot_ns = 0.0, 0.0, 0.0, 0.0
    for k in TRAVERSAL:
        c = allc.get(k, {})
        per = {n: (v / n_trav if not n.startswith("_") else v) for n, v in c.items()}
        fetch, write = per.get("FETCH_SIZE"), per.get("WRITE_SIZE")
        b = None
        if fetch is not None and write is not None:
            b = (2.0 * fetch + write) * 1024.0
            tot_bytes += b
        hit += per.get("TCC_HIT_sum", 0.0)
        miss += per.get("TCC_MISS_sum", 0.0)
        ns = stats.get(k, (0, 0.0))[1] / n_trav_stats
        tot_ns += ns
        kern[k] = {"counters_per_traversal": per, "hbm_bytes_per_traversal": b, "ms_per_traversal": ns / 1e6,
                   "hbm_GBps": (b / ns) if (b and ns) else None}
    build_id = args.build_id
    if build_id is None:
        with open(os.path.join(args.pmc, "build_id.txt")) as fh:
            build_id = fh.read().strip()
    k0 = allc.get(TRAVERSAL[0], {})
    per0 = {n: v / n_trav for n, v in k0.items() if not n.startswith("_")}

    def ratio(a, b):
        return per0[a] / per0[b] if per0.get(a) is not None and per0.get(b) else None

    lanes = per0.get("SQ_THREAD_CYCLES_VALU"), per0.get("SQ_ACTIVE_INST_VALU")
    res = {
        "workload": workload, "queries": S, "code": args.code, "build_id": build_id,
        # latency-side figures of the pass-1 kernel (k_knn<0,false>), same session
        "lanes_active_valu": lanes[0] / (64.0 * lanes[1]) if all(lanes) else None,
        "wave_cycles_waiting_frac": ratio("SQ_WAIT_ANY", "SQ_WAVE_CYCLES"),
        "wave_cycles_valu_frac": ratio("SQ_ACTIVE_INST_VALU", "SQ_WAVE_CYCLES"),
        "units": "FETCH_SIZE / WRITE_SIZE in KB as rocprofv3 reports them; gfx950: bytes = "
                 "(2 * FETCH_SIZE + WRITE_SIZE) * 1024 (MI355X_MICROARCH.md §HBM); TCC_HIT/MISS summed over "
                 "channels; every figure per traversal = pass-1 launches (leaders + followers) + pass 2; the "
                 "first %d traversal(s) of each run (the tree build's entry-cut centres) excluded" % args.build_traversals,
        "kernels": kern,
        "bytes_per_launch": tot_bytes or None,
        "bytes_per_query": (tot_bytes / S) if tot_bytes else None,
        "l2_hit_rate": hit / (hit + miss) if hit + miss > 0 else None,
        "traversal_ms": tot_ns / 1e6,
        "hbm_GBps": (tot_bytes / tot_ns) if (tot_bytes and tot_ns) else None,
    }
    res["isa"] = isa_of_build(build_id)
    os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
    with open(os.path.join(ROOT, "profiles", "pmc_traffic.json"), "w") as fh:
        json.dump(res, fh, indent=1)
    with open(os.path.join(ROOT, "profiles", "%s_pmc_%s.json" % (args.tag, args.code)), "w") as fh:
        json.dump({"code": args.code, "workload": workload, "kernel_stats_calls_total_ns": stats, "counters": allc}, fh,
                  indent=1)
    print(json.dumps({k: v for k, v in res.items() if k != "kernels"}, indent=1))


if __name__ == "__main__":
    main()
