# round-5 tile-tail hand-off A/B (build/variants t*): parity of two variants, the C3 shard A/B, one stats dump
set -u
mkdir -p gpurun_out
for v in ${CHK:-t8i40 t16i48}; do
  MESH_AMD_LIB=$PWD/build/variants/$v.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread -k "tail_handoff or c3_stream_shards or c3_headline or c3_sample or entry_cut or c2 or cooperative or tied or far_and" > gpurun_out/varchk_$v.log 2>&1 || exit 2
done
VARIANTS="${AB:-t0 t4i48 t8i40 t8i56 t16i48}" QS="100000000 12500000" ROUNDS=2 VSTEPS=8 bash scripts/ab_shard.sh > gpurun_out/ab.log 2>&1 || exit 3
MESH_AMD_LIB=$PWD/build/variants/${DUMP:-t8i40}.so MESH_AMD_STATS_DUMP=1 timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu > gpurun_out/tail_stats_dump.log 2>&1
