#!/bin/bash
# FETCH_SIZE / WRITE_SIZE of tools/pmc_width_probe.hip's kernels (build/pmc_width_probe, built in the CPU container by
# `hipcc -O3 --offload-arch=gfx950 tools/pmc_width_probe.hip -o build/pmc_width_probe`): one --pmc pass per counter,
# then the counter bytes over the bytes each kernel moves (scripts/pmc_width_probe.py).
set -u
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=$R/gpurun_out/pmc_width
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- "$R/build/pmc_width_probe" > "$OUT/fetch.log" 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- "$R/build/pmc_width_probe" > "$OUT/write.log" 2>&1 || exit 2
cd "$R" && python3 scripts/pmc_width_probe.py "$OUT" > "$OUT/summary.json"
