"""Development helper: one line per bench.py JSON log (value, step time, pass breakdown, node/leaf counts).
    python scripts/summarize_bench.py gpurun_out/var_*.log"""
import json
import sys

for path in sys.argv[1:]:
    try:
        with open(path) as fh:
            line = [ln for ln in fh.read().splitlines() if ln.startswith("{")][-1]
        d = json.loads(line)
    except (OSError, IndexError, ValueError) as e:
        print("%-40s (no bench line: %s)" % (path, type(e).__name__))
        continue
    b = d["breakdown_ms_per_step"]
    r = d["roofline"]
    print("%-34s %7.1f M q/s %6.2f ms  p1 %6.2f (sl %4.2f lead %5.2f fol %6.2f) p2 %4.2f sort %4.2f  nodes %5.1f leaves %5.2f"
          % (path, d["value"] / 1e6, d["ms_per_step"], b["pass1"], b["pass1_superleaders"], b["pass1_leaders"],
             b["pass1_followers"], b["pass2"], b["sort"], r["nodes_per_query"], r["leaves_per_query"]))
