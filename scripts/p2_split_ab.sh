#!/bin/bash
# Pass-2 split A/B (round 6): the GPU suite on the in-tree library, then bench.py on the 12.5M shard and on 100M over
# build/variants/<ORDER12 / ORDER100 names>.so; lines into gpurun_out/p2ab.jsonl.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
if [ -z "${NOTEST:-}" ]; then
  timeout -k 10 900 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_p2.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_p2.log
  [ $rc -eq 0 ] || exit $rc
fi
: > gpurun_out/p2ab.jsonl
for n in ${ORDER12:-}; do
  MESH_AMD_LIB=$PWD/build/variants/$n.so timeout -k 10 300 python bench.py --queries 12500000 --steps 10 --warmup 2 --no-cpu --no-one-shot 2> gpurun_out/p2ab_$n.err | tail -1 >> gpurun_out/p2ab.jsonl || exit 3
done
for n in ${ORDER100:-}; do
  MESH_AMD_LIB=$PWD/build/variants/$n.so timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu --no-one-shot 2> gpurun_out/p2ab_$n.err | tail -1 >> gpurun_out/p2ab.jsonl || exit 3
done
echo done
