#!/bin/bash
# Round-5 measurement session on the GPU box (each step under its own time limit; the first failure ends it):
# query-order parity, sort A/B (build/variants sp / pk), C4 + C5 configs through bench_configs (numpy paths),
# C5 parity sweep (alongnormal rays + visibility pairs vs brute force).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for st in ${STEPS:-parity ab configs sweep}; do
  case $st in
    parity) timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -v -m gpu -p no:cacheprovider \
              -k "query_order or c3_headline or c3_stream_shards" --timeout 300 --timeout-method thread > gpurun_out/s_parity.log 2>&1 ;;
    ab) rm -f gpurun_out/abs_*; VSTEPS=8 VARIANTS="${AB:-sp pk}" QS="${ABQ:-100000000}" ROUNDS=2 bash scripts/ab_shard.sh ;;
    configs) timeout -k 10 900 python -u scripts/bench_configs.py --configs ${CFGS:-c4,c5} --reps 3 > gpurun_out/bench_configs_r05.jsonl 2> gpurun_out/bench_configs_r05.err ;;
    sweep) timeout -k 10 900 python -u scripts/parity_sweep.py --configs ${SWEEP:-c5,c5v} > gpurun_out/parity_sweep_r05.jsonl 2> gpurun_out/parity_sweep_r05.err ;;
  esac
  rc=$?
  echo "$st rc=$rc" | tee -a gpurun_out/session_status.txt
  [ $rc -eq 0 ] || exit $rc
done
echo done | tee -a gpurun_out/session_status.txt
