#!/bin/bash
# Round-5 final-build records (each step under its own limit; the first failure ends it): the C3 shard curve,
# every bench_configs config, the parity sweeps, then the sort-variant A/B (build/variants fm0 fm128 fm512 nt512).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python scripts/shard_curve.py --out gpurun_out/shard_curve.json > gpurun_out/shard_curve.log 2>&1 || exit 1
STEPS="configs sweep" CFGS=c1,c2,c3np,c4,c5,facade SWEEP=c3,c2,c5,c5v bash scripts/r05_session.sh || exit 2
rm -f gpurun_out/abs_*
VARIANTS="${AB:-fm0 fm128 fm512 nt512}" QS="100000000 12500000" ROUNDS=2 VSTEPS=8 bash scripts/ab_shard.sh > gpurun_out/ab.log 2>&1 || exit 3
