"""Calibration of rocprofv3's FETCH_SIZE / WRITE_SIZE on gfx950 against kernels whose bytes are known exactly.

MI355X_MICROARCH.md calibrates the two counters only for 16-B-per-lane streams (FETCH_SIZE reports half of the bytes
read, WRITE_SIZE the bytes written) and says other access widths are uncalibrated.  The query sort's kernels move a
known number of bytes with 4- and 8-B-per-lane accesses, so one PMC run of bench.py (scripts/profile_pmc.sh, summarised
by scripts/pmc_summary.py into profiles/<tag>_pmc.json) calibrates those widths:
  k_qkeys      reads the rows (3 x 8-B loads per lane, 24 B per row), writes one u32 key per row (4-B stores);
  k_qscatter2  <false,true> reads u32 keys, writes u32 keys + u32 rows; <true,true> reads and writes both;
               <true,false> reads both, writes the rows (4-B loads and stores, stores in digit runs of ~32 rows).
Prints, per kernel, the counter bytes over the known bytes for reads (raw FETCH_SIZE, i.e. before the guide's x2)
and writes.

    python scripts/pmc_calibration.py profiles/r05_c3_100M_pmc_1d3fa38.json [--rows 100000000]
"""
import argparse
import json

KNOWN = {  # kernel name prefix: (bytes read per row, bytes written per row)
    "msh::k_qkeys<": (24, 4),
    "msh::k_qscatter2<512, 16, false, true>": (4, 8),
    "msh::k_qscatter2<512, 16, true, true>": (8, 8),
    "msh::k_qscatter2<512, 16, true, false>": (8, 4),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("pmc")
    ap.add_argument("--rows", type=float, default=1e8)
    a = ap.parse_args()
    c = json.load(open(a.pmc))["counters"]
    out = {}
    for name, v in c.items():
        for pre, (rd, wr) in KNOWN.items():
            if name.startswith(pre):
                n = v.get("_dispatches", 1)  # the record holds totals over the run's dispatches
                out[name] = {"dispatches": n, "fetch_raw_over_read": v["FETCH_SIZE"] / n * 1024 / (rd * a.rows),
                             "write_over_written": v["WRITE_SIZE"] / n * 1024 / (wr * a.rows)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
