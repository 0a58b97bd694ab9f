#!/bin/bash
# Round-6 evidence at one build, in box sessions (each step under its own limit; the first failure ends a session).
#   PART=a: smoke, the GPU suite, bench.py (20 steps), its rocprof kernel stats, the C3 PMC passes
#   PART=b: bench.py --dist under torch.distributed.run (the collective path at N = 1), PMC of C5 and C2 (with SQ)
#   PART=c: the C3 shard curve, every bench_configs config, the parity sweeps
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
case ${PART:?set PART} in
  a) STAGES="smoke pytest bench20 prof pmc" bash scripts/gpu_check.sh || exit 1 ;;
  b) DSTEPS=20 STAGES="bench_dist" bash scripts/gpu_check.sh || exit 1
     PMC_CFGS="c5 c2" PMC_CFG_PASSES="stats fetch write tcc sq" STAGES="pmc_cfg" bash scripts/gpu_check.sh || exit 1 ;;
  c) timeout -k 10 500 python scripts/shard_curve.py --out gpurun_out/shard_curve.json > gpurun_out/shard_curve.log 2>&1 || exit 2
     STEPS="configs sweep" CFGS=c1,c2,c3np,c4,c5,facade SWEEP=c3,c2,c5,c5v bash scripts/r05_session.sh || exit 3 ;;
esac
grep -q "rc=[1-9]" gpurun_out/status.txt && exit 1
exit 0
