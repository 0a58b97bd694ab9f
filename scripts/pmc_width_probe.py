"""Counter bytes over moved bytes for tools/pmc_width_probe.hip's kernels (scripts/pmc_width_probe.sh).
    python scripts/pmc_width_probe.py gpurun_out/pmc_width"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from scripts.pmc_summary import counters  # noqa: E402

MB512 = 512 << 20
MOVED = {"k_ld<4>": ("read", MB512), "k_ld<8>": ("read", MB512), "k_ld<16>": ("read", MB512),
         "k_st<4>": ("write", MB512), "k_st<8>": ("write", MB512), "k_st<16>": ("write", MB512),
         "k_st_scatter<4>": ("write", 4 * (64 << 20)), "k_st_scatter<8>": ("write", 8 * (64 << 20))}


def main():
    d = sys.argv[1]
    f, w = counters(os.path.join(d, "fetch")), counters(os.path.join(d, "write"))
    out = {}
    for name, (kind, nbytes) in MOVED.items():
        kf = next((v for k, v in f.items() if name + "(" in k), {})
        kw = next((v for k, v in w.items() if name + "(" in k), {})
        out[name] = {"moves": kind, "bytes": nbytes,
                     "FETCH_SIZE_bytes_over_moved": kf.get("FETCH_SIZE", 0.0) * 1024 / nbytes,
                     "WRITE_SIZE_bytes_over_moved": kw.get("WRITE_SIZE", 0.0) * 1024 / nbytes}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
