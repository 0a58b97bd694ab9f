# A/B of visibility_compute's camera-chunk plan (build/variants v*): C5 through bench_configs, CPU legs off, ABBA order
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
VS=${VARIANTS:-v16_16 v5_16 v8_8 v5_10}
RVS=$(echo $VS | tr ' ' '\n' | tac | tr '\n' ' ')
for r in 1 2; do
  ORDER=$VS; [ $r -eq 2 ] && ORDER=$RVS
  for v in $ORDER; do
    MESH_AMD_LIB=$PWD/build/variants/$v.so MESH_AMD_NO_CPU=1 timeout -k 10 300 python scripts/bench_configs.py --configs c5 --reps 3 >> gpurun_out/vis_$v.jsonl 2>> gpurun_out/vis_ab.err || exit 1
    echo "$v round $r" >> gpurun_out/vis_ab_status.txt
  done
done
