"""Kernel statistics (name, calls, total/average us, share) from a rocprofv3 rocpd database -> CSV.
    python scripts/prof_stats.py gpurun_out/prof_c5/run_results.db profiles/r02_c5_kernel_stats_<code>.csv
The closest-point traversal kernels also get a row over the bench's own launches only: a tree with an entry
cut answers its cell centres with the same kernels at build time, before the bench (the first traversal, up
to the first pass-2 dispatch, is left out of those rows)."""
import csv
import sqlite3
import sys

TRAVERSAL = ("k_knn<0, false, true, true>", "k_knn_coop<0, false>")

con = sqlite3.connect(sys.argv[1])
with open(sys.argv[2], "w", newline="") as fh:
    w = csv.writer(fh)
    w.writerow(["name", "calls", "total_us", "average_us", "percentage"])  # rocpd top_kernels durations are in us
    for row in con.execute("select name, total_calls, total_duration, average, percentage from top_kernels"):
        w.writerow(row)
    rows = con.execute("select name, dispatch_id, duration from kernels order by dispatch_id").fetchall()
    coop = [d for n, d, _ in rows if TRAVERSAL[1] in n]
    if coop:
        first = coop[0]
        for k in TRAVERSAL:
            ds = [dur for n, d, dur in rows if k in n and d > first]
            if ds:  # rocpd kernels.duration is in ns
                w.writerow(["%s [bench launches: build-time cell-centre traversal excluded]" % k, len(ds),
                            sum(ds) / 1e3, sum(ds) / len(ds) / 1e3, ""])
