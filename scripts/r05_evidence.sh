#!/bin/bash
# Round-5 evidence at one build, in one box session: smoke, the GPU suite, bench.py, its rocprof kernel stats, the
# PMC passes (C3, then C5 and C2), the C3 shard curve, every bench_configs config and the parity sweeps.  Each step
# under its own limit; the first failure ends the session.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
STAGES="smoke pytest bench prof pmc pmc_cfg" bash scripts/gpu_check.sh || exit 1
grep -q "rc=[1-9]" gpurun_out/status.txt && exit 1
timeout -k 10 400 python scripts/shard_curve.py --out gpurun_out/shard_curve.json > gpurun_out/shard_curve.log 2>&1 || exit 2
STEPS="configs sweep" CFGS=c1,c2,c3np,c4,c5,facade SWEEP=c3,c2,c5,c5v bash scripts/r05_session.sh || exit 3
