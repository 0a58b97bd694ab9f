#!/bin/bash
# Parity-gated A/B of build/variants/*.so on the GPU box: every variant first passes the closest-point parity tests
# (any failure ends the run before a variant is benched), then the C3 bench runs ROUNDS times over all variants,
# interleaved, into gpurun_out/ab_<name>.log (one JSON line per run).
#   VARIANTS="a_base d_asm" ROUNDS=2 VQ=100000000 bash scripts/ab_variants.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
VS=${VARIANTS:-$(ls build/variants | sed 's/\.so$//')}
for v in $VS; do
  MESH_AMD_LIB=$PWD/build/variants/$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu \
    -p no:cacheprovider --timeout 300 --timeout-method thread \
    -k "c1 or c2 or non_finite or c3_sample or entry_cut or c3_stream_shards or c3_headline or tiny or degenerate or far_and or on_vertices or cooperative or deep_tree or tied or batch_bit or barycentric or device_api" \
    > gpurun_out/abchk_$v.log 2>&1
  rc=$?
  echo "abchk_$v rc=$rc" | tee -a gpurun_out/ab_status.txt
  [ $rc -eq 0 ] || exit $rc
done
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in $VS; do
    MESH_AMD_LIB=$PWD/build/variants/$v.so timeout -k 10 300 python bench.py --queries ${VQ:-100000000} --steps ${VSTEPS:-10} \
      --warmup 2 --no-cpu >> gpurun_out/ab_$v.log 2>&1
    rc=$?
    echo "ab_$v round $r rc=$rc" | tee -a gpurun_out/ab_status.txt
    [ $rc -eq 0 ] || exit $rc
  done
done
echo done | tee -a gpurun_out/ab_status.txt
