"""Host <-> device copy rates on the GPU box, alone and concurrent: the bound of the numpy entry points, which
move 24 B per query in and 32 B out (C3: 2.4 GB up and 3.2 GB down per 100M queries).

    python scripts/pcie_probe.py [--gb 2]

Prints one JSON line: GB/s of a pinned H2D copy alone, a pinned D2H copy alone, and both at once on two
streams (each direction's rate and the combined rate).
"""
import argparse
import json
import time

import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gb", type=float, default=2.0)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    n = int(a.gb * (1 << 30))
    hu = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    hd = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    du = torch.empty(n, dtype=torch.uint8, device="cuda")
    dd = torch.empty(n, dtype=torch.uint8, device="cuda")
    hu.fill_(1)
    dd.fill_(2)
    su, sd = torch.cuda.Stream(), torch.cuda.Stream()

    def timed(fn):
        best = []
        for _ in range(a.reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            best.append(time.perf_counter() - t0)
        return sorted(best)[len(best) // 2]

    def up():
        with torch.cuda.stream(su):
            du.copy_(hu, non_blocking=True)

    def down():
        with torch.cuda.stream(sd):
            hd.copy_(dd, non_blocking=True)

    def both():
        up()
        down()

    t_up, t_down, t_both = timed(up), timed(down), timed(both)
    gb = n / 1e9
    print(json.dumps({"bytes_per_copy": n, "h2d_GBps": gb / t_up, "d2h_GBps": gb / t_down,
                      "concurrent_s": t_both, "concurrent_combined_GBps": 2 * gb / t_both,
                      "concurrent_vs_serial": t_both / (t_up + t_down)}), flush=True)


if __name__ == "__main__":
    main()
