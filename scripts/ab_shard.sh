#!/bin/bash
# A/B of build/variants/*.so on C3 streams of several sizes (the N = 8/4/2/1 shard sizes of the 100M stream), interleaved
# over ROUNDS, one JSON line per run into gpurun_out/abs_<variant>_<queries>.log.  No parity gate: run
# scripts/ab_variants.sh (or the suite) on the variant that is kept.
#   VARIANTS="base klead1" QS="12500000 100000000" ROUNDS=2 bash scripts/ab_shard.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
VS=${VARIANTS:-$(ls build/variants | sed 's/\.so$//')}
RVS=$(echo $VS | tr ' ' '\n' | tac | tr '\n' ' ')
for r in $(seq 1 ${ROUNDS:-2}); do
  # odd rounds in the given order, even rounds reversed (ABBA: no variant always follows the same one)
  ORDER=$VS; [ $((r % 2)) -eq 0 ] && ORDER=$RVS
  for qn in ${QS:-12500000 100000000}; do
    for v in $ORDER; do
      MESH_AMD_LIB=$PWD/build/variants/$v.so timeout -k 10 300 python bench.py --queries $qn --steps ${VSTEPS:-10} \
        --warmup 2 --no-cpu >> gpurun_out/abs_${v}_$qn.log 2>&1
      rc=$?
      echo "abs_$v $qn round $r rc=$rc" | tee -a gpurun_out/abs_status.txt
      [ $rc -eq 0 ] || exit $rc
    done
  done
done
echo done | tee -a gpurun_out/abs_status.txt
