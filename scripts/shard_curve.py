"""C3 strong-scaling shards measured on one GPU: bench.py on 12.5M / 25M / 50M / 100M uniform C3 queries (one rank's
contiguous shard of the 100M stream at N = 8 / 4 / 2 / 1; a shard of the uniform stream is itself a uniform stream
of that size), per-phase times from the library's HIP-event timers.  Writes one JSON record with the whole curve.

    python scripts/shard_curve.py [--steps 8] [--out gpurun_out/shard_curve.json]
"""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "shard_curve.json"))
    args = ap.parse_args()
    rows = []
    for n_gpu, q in ((8, 12_500_000), (4, 25_000_000), (2, 50_000_000), (1, 100_000_000)):
        out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--queries", str(q), "--steps",
                              str(args.steps), "--warmup", "2", "--no-cpu"], check=True, capture_output=True,
                             text=True, timeout=600).stdout
        d = json.loads(out.strip().splitlines()[-1])
        rows.append({"shard_of_N": n_gpu, "queries": q, "ms_per_step": d["ms_per_step"],
                     "queries_per_s": d["value"], "ns_per_query": d["ms_per_step"] * 1e6 / q,
                     "breakdown_ms_per_step": d["breakdown_ms_per_step"],
                     "nodes_per_query": d["roofline"]["nodes_per_query"],
                     "leaves_per_query": d["roofline"]["leaves_per_query"], "build_id": d["build_id"]})
        print(json.dumps(rows[-1]), flush=True)
    base = rows[-1]["ms_per_step"]
    for r in rows:
        # compute-only strong-scaling efficiency of the shard (no all-gather): whole-stream time / (N x shard time)
        r["compute_scaling_eff"] = base / (r["shard_of_N"] * r["ms_per_step"])
    rec = {"what": "one rank's share of the C3 100M stream at N = 8/4/2/1, each measured alone on one MI355X through "
                   "bench.py (device-resident, no all-gather); compute_scaling_eff = t(100M) / (N x t(shard))",
           "steps": args.steps, "curve": rows}
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    with open(args.out, "w") as fh:
        json.dump(rec, fh, indent=1)


if __name__ == "__main__":
    main()
