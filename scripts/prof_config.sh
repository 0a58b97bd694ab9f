#!/bin/bash
# rocprofv3 kernel stats of one scripts/bench_configs.py config: bash scripts/prof_config.sh c4
# -> gpurun_out/prof_<cfg>/ (rocpd database; scripts/prof_stats.py turns it into a CSV)
set -u
R=$(cd "$(dirname "$0")/.." && pwd)
cfg=${1:?config}
mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_$cfg" -o run -- python3 "$R/scripts/bench_configs.py" --configs "$cfg" --reps 2 > "$R/gpurun_out/prof_$cfg.log" 2>&1
