"""Kernel statistics (name, calls, total/average ns, share) from a rocprofv3 rocpd database -> CSV.
    python scripts/prof_stats.py gpurun_out/prof_c5/run_results.db profiles/r02_c5_kernel_stats_<code>.csv"""
import csv
import sqlite3
import sys

con = sqlite3.connect(sys.argv[1])
with open(sys.argv[2], "w", newline="") as fh:
    w = csv.writer(fh)
    w.writerow(["name", "calls", "total_us", "average_us", "percentage"])  # rocpd top_kernels durations are in us
    for row in con.execute("select name, total_calls, total_duration, average, percentage from top_kernels"):
        w.writerow(row)
